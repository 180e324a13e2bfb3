// service_kernels.hpp — resident message service for single GCM messages from host memory
// (gfx950).  The per-message EVP path (EVP_AEAD_CTX_seal / _open once per MPI message,
// send.c:294-315, recv.c:322) pays a kernel launch, the table staging and the host's completion
// wait on every message; this kernel is launched once, keeps the flow kernel's tables in LDS and
// serves messages posted in a page-locked host ring until it has been idle for `idle_ticks`
// (or has lived `life_ticks`): then it exits and the host relaunches it on the next message.
//
// Protocol (one message in flight per context; service_host.hpp is the host side):
//   host:   the ring is three 16-byte chunks {seq, three descriptor words} (op, len, in, out,
//           nonce: 9 words); the host writes the descriptor words, then seq into every chunk.
//   leader (workgroup 0, one lane): polls the three chunks with one 16-byte system-scope load each
//           (a 16-byte read is one snapshot of its chunk, so a chunk showing the new seq shows its
//           new words: the descriptor arrives with the seq, no second round trip); on a new seq in
//           all three it publishes the descriptor for the other workgroups as 13 self-tagged
//           8-byte units {seq, word} (the 12 descriptor words and the generation) in device memory
//           (agent-scope stores, none waited: a unit is one snapshot, so no seqlock — round 5: the
//           seqlock's three drains and the readers' two-phase reads took 1.7 + 1.5 us of each
//           64 KiB message, tools/svc_timeline.py);
//           on idle / lifetime / op STOP / a kick (the host word kick == gen: another context's
//           service takes this stream slot) it publishes a STOP descriptor, writes the exit word
//           (= gen) and exits.  A message whose chunks fit one workgroup is served by the leader's
//           workgroup alone and not published.
//   others: poll the 13 units (agent-scope loads, all in flight together) until every unit
//           carries one seq != the last one seen and the generation unit names theirs; run their
//           share, exit on STOP.
//   message: the flow decomposition (gcm_flow_kernel's unit code) over the DATA blocks: chunks of
//           C = 64·S blocks, S the smallest power of two <= 8 with at most 64 chunks, one wavefront
//           per chunk, 8 chunks per workgroup; every chunk's partial is weighted by
//           H^(2 + (nch-1-i)C) (host precomputed for the four S), and a ninth wave of workgroup 0
//           adds E_K(J0) ^ L·H (the length block), so the tag is the XOR of the partials and a
//           chunk of 64·S blocks is S steps (round 5: with the length block and J0 in chunk 0 it
//           ran a near-empty extra step, ~2.5 us of every message of a multiple of 1 KiB).
//           Every workgroup XORs its waves' partials and, after a system-scope release of its
//           record bytes, posts its own completion slot: four 8-byte {seq, word} pairs (the
//           partial) in two 16-byte system-scope stores — no cross-workgroup arrival (round 5:
//           the agent-scope counter, the last arriver's partial reads and its second release were
//           2.5 us of each multi-workgroup message).  The host takes a pair only with the new seq
//           in it (a pair cannot tear), waits for the message's workgroups' slots, and XORs the
//           partials into the tag: it writes a seal's tag into out + len and checks an open's
//           (a forged message's plaintext is zero-filled, aead.h:276-278).
//   counter-mode ops (CTR contexts: the 702 / 700 small-message XORs, send.c:1273-1465,
//           recv.c:954-1023, :1187-1220): kSvcXor out = in ^ mask, kSvcCtr out = in ^ E_K(ctr + j),
//           kSvcEcb out = E_K(in) per 16-byte block (the 602 sub-key K' = AES_K(V), send.c:583)
//           (in null: the keystream), at most kSvcMaxStreamLen bytes, served by the leader's
//           workgroup alone and completed like a one-workgroup seal (partial 0).
// Every wave's wait loop is bounded by the wall clock: the grid drains even if the host vanishes.
#pragma once
#include "ctr_kernels.hpp"
#include "gcm_kernels.hpp"

namespace cmpi {
namespace dev {

// Workgroups of the resident grid (8 = one per XCD when the chip is free, 8 CUs held while
// resident).  16 workgroups of 4 chunk waves (-DCMPI_SVC_GROUPS=16) served 64 KiB seal / open
// 0.5-1 us faster and 1 KiB 0.4 us faster on the same box, pageable 64 KiB 1 us slower
// (profiles/r05ac_*), at 16 CUs held between messages: not the default.
#ifndef CMPI_SVC_GROUPS
#define CMPI_SVC_GROUPS 8
#endif
constexpr uint32_t kSvcGroups = CMPI_SVC_GROUPS;         // workgroups (8: one per XCD when the chip is free)
constexpr uint32_t kSvcMaxChunks = 64u;                  // kSvcGroups x kSvcChunkWaves
constexpr uint32_t kSvcChunkWaves = kSvcMaxChunks / kSvcGroups;  // chunk waves per workgroup
constexpr uint32_t kSvcThreads = 64u * (kSvcChunkWaves + 1u);    // + the J0 wave (svc_j0_wave; idle in workgroups > 0)
constexpr uint32_t kSvcStage = kSvcChunkWaves >= 8u ? 512u : 256u;  // threads that stage the tables
constexpr uint32_t kSvcSeal = 0u, kSvcOpen = 1u, kSvcStop = 2u, kSvcXor = 3u, kSvcCtr = 4u, kSvcEcb = 5u;
// descriptor words: op, len, in lo/hi, out lo/hi, then the op's own: GCM nonce[3] at 6..8, XOR
// mask lo/hi at 6..7, CTR counter block as big-endian halves hi lo/hi, lo lo/hi at 8..11
constexpr uint32_t kSvcDesc = 12u;
constexpr uint32_t kSvcChunks = kSvcDesc / 3u;  // ring chunks {seq, three descriptor words}
constexpr uint32_t kSvcPubWords = 64u;          // go[64 + 2u .. 2u + 1]: published unit u = {seq, word}
constexpr uint32_t kSvcGoBytes = 512u;          // the device control area (host: hipMalloc)
constexpr uint32_t kSvcMaxStreamLen = 65536u;   // counter-mode ops: the 702 ring's small messages

struct SvcArgs {
  const uint32_t* ring;  // page-locked host words (device address): chunks [4c] = seq, [4c+1..4c+3] = desc[3c..3c+2]
  const uint32_t* kick;  // page-locked host word: == gen asks this generation to exit (its stream slot is wanted)
  uint32_t* done;        // page-locked host words: workgroup w's completion slot [8w .. 8w+7], four {seq, partial word} pairs
  uint32_t* exited;      // page-locked host word: the generation that exited
  uint32_t* go;          // device: [64..89] 13 published units {seq, word}
  const u32x4* wts;      // device: 4 x 64 x 4; wts[256s + 4k + 3] = H^(2 + (63-k)·64·2^s)
  const uint32_t* te0;
  const u32x4* wtab;     // the ten flow nibble tables (DevTables::fnib); null for CTR / ECB contexts
  uint32_t seq0;         // last seq consumed before this launch
  uint32_t ls_min;       // smallest chunk-step exponent (test hook cmpi_debug_set_svc_ls_min; 0)
  uint32_t gen;
  uint64_t idle_ticks, life_ticks, cap_ticks;  // 100 MHz wall clock
#if CMPI_TOOLS
  uint64_t* probe;  // diagnostics build: per-message phase stamps (cmpi_debug_set_svc_probe), or null
#endif
  RoundKeys rk;
};

// Diagnostics build only (-DCMPI_TOOLS=1, tools/svc_timeline.py): 100 MHz wall-clock stamps of a
// message's phases into probe[32 * (seq % 8) + slot]: 0 the leader sees the seq in the host ring,
// 1 the descriptor is in the leader workgroup's LDS (and published), 2 + wg a workgroup starts
// the message, 10 + wg its waves' record stores are performed, 18 + wg its completion slot is
// issued; 28..31 workgroup 0's first unit: first keystream, first step consumed, steps done,
// tree + weight.
#if CMPI_TOOLS
#define SVC_STAMP(s, seq, slot)                                                                       \
  do {                                                                                                \
    if ((s).probe) /* write-through: other XCDs' stamps reach memory while the kernel stays resident */  \
      __hip_atomic_store((s).probe + 32u * ((seq) & 7u) + (slot), wall_clock64(), __ATOMIC_RELAXED,   \
                         __HIP_MEMORY_SCOPE_AGENT);                                                   \
  } while (0)
#else
#define SVC_STAMP(s, seq, slot) \
  do {                          \
  } while (0)
#endif

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// one 16-byte system-scope read (sc0 sc1: past every cache) of a host chunk; p wave-uniform
__device__ __forceinline__ u32x4 sys_load16(const uint32_t* p) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(p), 0, 16, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 17);
}
// one 16-byte system-scope write (sc0 sc1) into a page-locked host chunk; p 16-byte aligned
__device__ __forceinline__ void sys_store16(uint32_t* p, u32x4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, 16, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, 0, 0, 17);
}
// The leader's descriptor for the other workgroups: units 0..11 = {seq, d[j]}, unit 12 = {seq, gen}.
__device__ __forceinline__ void svc_publish(uint32_t* go, uint32_t seq, uint32_t gen, const uint32_t (&d)[kSvcDesc]) {
  uint64_t* u = reinterpret_cast<uint64_t*>(go + kSvcPubWords);
#pragma unroll
  for (uint32_t j = 0; j < kSvcDesc; ++j)
    __hip_atomic_store(u + j, (uint64_t)seq | ((uint64_t)d[j] << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(u + kSvcDesc, (uint64_t)seq | ((uint64_t)gen << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A reader's poll: true with (seq, d) when all 13 units carry one seq != cur and the generation
// unit names `gen`.
__device__ __forceinline__ bool svc_take(const uint32_t* go, uint32_t cur, uint32_t gen, uint32_t& seq,
                                         uint32_t (&d)[kSvcDesc]) {
  const uint64_t* u = reinterpret_cast<const uint64_t*>(go + kSvcPubWords);
  uint64_t v[kSvcDesc + 1];
#pragma unroll
  for (uint32_t j = 0; j <= kSvcDesc; ++j) v[j] = __hip_atomic_load(u + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t q = (uint32_t)v[kSvcDesc];
  if (q == cur || (uint32_t)(v[kSvcDesc] >> 32) != gen) return false;
#pragma unroll
  for (uint32_t j = 0; j < kSvcDesc; ++j) {
    if ((uint32_t)v[j] != q) return false;
    d[j] = (uint32_t)(v[j] >> 32);
  }
  seq = q;
  return true;
}

// Completion slot of a workgroup: four {seq, word} pairs (its partial) in two 16-byte system-scope
// stores, neither waiting for the other's PCIe acknowledgement.
__device__ __forceinline__ void svc_post(uint32_t* slot, uint32_t seq, u32x4 x) {
  sys_store16(slot, u32x4{seq, x[0], seq, x[1]});
  sys_store16(slot + 4, u32x4{seq, x[2], seq, x[3]});
}

// LDS words shared by the workgroup (inside the flow aggregation area)
constexpr uint32_t kSvcX = kFlowAgg + 256u;  // [0] exit, [1] seq, [2..13] descriptor

// A 64-bit address from two LDS words (lo, hi), wave-uniform.  readfirstlane returns int: each
// word is taken as uint32_t before widening (a sign-extended low word with bit 31 set would put
// 0xFFFFFFFF in the high half).
__device__ __forceinline__ uint64_t lds_ptr64(uint32_t off) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane(lds32(off));
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane(lds32(off + 4u));
  return ((uint64_t)hi << 32) | lo;
}

// Chunk plan of a message of `len` bytes: C = 64·2^ls data blocks per chunk (the smallest of at
// most 64 chunks), nch = ceil(blocks / C) chunks, chunk 0 taking the remainder (1..C blocks), so
// no chunk runs more than S = C/64 steps (round 5: chunk 0 took C..2C-1 blocks, two steps for
// e.g. 65 000 B where one suffices); ngrp workgroups of kSvcChunkWaves chunks.  service_host.hpp
// svc_groups mirrors it.
__device__ __forceinline__ uint32_t svc_plan(uint32_t len, uint32_t& ls, uint32_t& nch, uint32_t ls_min = 0u) {
  const uint32_t nx = (len + 15u) >> 4;
  ls = ls_min;
  while (ls < 3u && nx > kSvcMaxChunks * (64u << ls)) ++ls;
  const uint32_t C = 64u << ls;
  nch = nx ? (nx + C - 1u) / C : 1u;
  return (nch + kSvcChunkWaves - 1u) / kSvcChunkWaves;
}

// E_K(J0) ^ L·H: the length block's GHASH term (weight H^1) and the tag mask, the part of the tag
// no chunk holds (flow_unit<.., SEP>).  Every lane computes it; lane 0's copy is used.
__device__ __forceinline__ u32x4 svc_j0_wave(const GcmArgs& a, const RoundKeys& rk, const RowLanes& rl, u32x4 lenblk) {
  uint32_t w0 = a.nfix[0], w1 = a.nfix[1], w2 = a.nfix[2], w3 = __builtin_bswap32(1u);
  aes128_enc(rk, rl, w0, w1, w2, w3);
  return u32x4{w0, w1, w2, w3} ^ gmul_nib(lenblk, flow_tab(0u));
}

template <bool DECRYPT>
__device__ __forceinline__ void svc_message(const SvcArgs& s, const RowLanes& rl, uint32_t seq) {
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u, wg = blockIdx.x;
  constexpr uint32_t wpb = kSvcChunkWaves;
  const uint32_t len = __builtin_amdgcn_readfirstlane(lds32(kSvcX + 12u));
  uint8_t* inp = reinterpret_cast<uint8_t*>(lds_ptr64(kSvcX + 16u));
  uint8_t* outp = reinterpret_cast<uint8_t*>(lds_ptr64(kSvcX + 24u));
  GcmArgs a{};
  a.in = inp;
  a.out = outp;
  a.len = len;
  a.nb = (len + 15u) >> 4;
  a.nrec = 1u;
  a.nmode = 3u;
  a.nfix[0] = __builtin_amdgcn_readfirstlane(lds32(kSvcX + 32u));
  a.nfix[1] = __builtin_amdgcn_readfirstlane(lds32(kSvcX + 36u));
  a.nfix[2] = __builtin_amdgcn_readfirstlane(lds32(kSvcX + 40u));
  const uint32_t nx = a.nb;  // data blocks (the X-sequence less its length block)
  uint32_t ls, nch;  // chunk 0: 1 <= r0 <= C blocks (0 for an empty message)
  const uint32_t ngrp = svc_plan(len, ls, nch, s.ls_min);  // workgroups with chunks
  const uint32_t C = 64u << ls;
  a.S = 1u << ls;
  a.nch = nch;
  a.r0 = nx - (nch - 1u) * C;
  a.chw = s.wts + 256u * ls + 4u * (kSvcMaxChunks - nch);  // a.chw[4i + 3] = H^(2 + (nch-1-i)C)
#if CMPI_TOOLS
  a.unit_stamps = s.probe ? s.probe + 32u * (seq & 7u) : nullptr;
#endif
  if (wg >= ngrp) return;
  const uint64_t cbits = (uint64_t)len * 8u;
  const u32x4 lenblk = {0u, 0u, __builtin_bswap32((uint32_t)(cbits >> 32)), __builtin_bswap32((uint32_t)cbits)};
  const uint32_t u = wg * wpb + wv;
  if (threadIdx.x == 0u && wg < 8u) SVC_STAMP(s, seq, 2u + wg);  // (stamps of workgroups 0..7)
  u32x4 pw = {0u, 0u, 0u, 0u};
  if (wv == wpb) {  // the J0 wave (workgroup 0's)
    if (wg == 0u) pw = svc_j0_wave(a, s.rk, rl, lenblk);
  } else if (u < nch) {
    uint32_t r;
    pw = flow_unit<DECRYPT, false, true>(a, s.rk, rl, lenblk, u, false, pw, pw, r);
  }
  if (lane == 0u) lds_st128(kFlowAgg + 16u * wv, pw);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's record stores are performed
  __syncthreads();
  if (threadIdx.x == 0u) {
    if (wg < 8u) SVC_STAMP(s, seq, 10u + wg);
    u32x4 x = lds128(kFlowAgg);
    for (uint32_t j = 1; j <= wpb; ++j) x ^= lds128(kFlowAgg + 16u * j);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // this workgroup's record bytes reach the host first
    svc_post(s.done + 8u * wg, seq, x);
    if (wg < 8u) SVC_STAMP(s, seq, 18u + wg);
  }
}

// Counter-mode op (leader workgroup): 16 bytes per lane and step, the last block's bytes only;
// kSvcCtr counts blocks like ctr_kernel (a 128-bit big-endian increment).  Every wave waits for
// its stores, then one system-scope release (the output reaches memory before the completion).
__device__ __forceinline__ void svc_stream_op(const SvcArgs& s, const RowLanes& rl, uint32_t op, uint32_t seq) {
  const uint32_t len = __builtin_amdgcn_readfirstlane(lds32(kSvcX + 12u));
  const uint8_t* inp = reinterpret_cast<const uint8_t*>(lds_ptr64(kSvcX + 16u));
  uint8_t* outp = reinterpret_cast<uint8_t*>(lds_ptr64(kSvcX + 24u));
  const uint8_t* mask = reinterpret_cast<const uint8_t*>(lds_ptr64(kSvcX + 32u));
  const uint64_t chi = lds_ptr64(kSvcX + 40u), clo = lds_ptr64(kSvcX + 48u);
  // kSvcCtr: word 6 = keystream bytes skipped before the message (cmpi_ctr_xor_host's `skip`)
  const uint32_t skip = op == kSvcCtr ? __builtin_amdgcn_readfirstlane(lds32(kSvcX + 32u)) : 0u;
  if (skip) {  // byte-granular: keystream block j covers message bytes [16j - skip, 16j + 16 - skip)
    for (uint32_t j = threadIdx.x; j < (skip + len + 15u) >> 4; j += kSvcThreads) {
      uint32_t w0, w1, w2, w3;
      ctr_words(chi, clo, j, w0, w1, w2, w3);
      aes128_enc(s.rk, rl, w0, w1, w2, w3);
      const uint32_t ks[4] = {w0, w1, w2, w3};
#pragma unroll
      for (uint32_t b = 0; b < 16u; ++b) {
        const int32_t i = (int32_t)(16u * j + b) - (int32_t)skip;
        if (i >= 0 && i < (int32_t)len)
          outp[i] = (uint8_t)((inp ? inp[i] : 0u) ^ (uint8_t)(ks[b >> 2] >> (8u * (b & 3u))));
      }
    }
  }
  const uint32_t nblk = skip ? 0u : (len + 15u) >> 4;
  // whole blocks stored write-through (sc1, as the flow kernel's records): the release before the
  // completion then has no dirty output lines to write back
  const __amdgpu_buffer_rsrc_t orsrc = wt_rsrc(outp);
  for (uint32_t j = threadIdx.x; j < nblk; j += kSvcThreads) {
    const uint32_t off = 16u * j, rem = len - off < 16u ? len - off : 16u;
    u32x4 ks;
    if (op == kSvcEcb) {  // whole blocks (the host sends multiples of 16)
      const u32x4 b = ld_blk(inp + off);
      uint32_t w0 = b[0], w1 = b[1], w2 = b[2], w3 = b[3];
      aes128_enc(s.rk, rl, w0, w1, w2, w3);
      st_wt(orsrc, off, u32x4{w0, w1, w2, w3});
      continue;
    }
    if (op == kSvcXor) {
      ks = rem == 16u ? ld_blk(mask + off) : load_partial(mask + off, rem);
    } else {
      uint32_t w0, w1, w2, w3;
      ctr_words(chi, clo, j, w0, w1, w2, w3);
      aes128_enc(s.rk, rl, w0, w1, w2, w3);
      ks = u32x4{w0, w1, w2, w3};
    }
    u32x4 v = {0u, 0u, 0u, 0u};
    if (inp) v = rem == 16u ? ld_blk(inp + off) : load_partial(inp + off, rem);
    if (rem == 16u) st_wt(orsrc, off, v ^ ks);
    else store_partial(outp + off, v ^ ks, rem);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0u) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    svc_post(s.done, seq, u32x4{0u, 0u, 0u, 0u});
  }
}

__global__ __launch_bounds__(kSvcThreads) void gcm_service_kernel(SvcArgs s) {
  if (s.wtab) {  // GCM: the AES rows and the flow kernel's ten GHASH tables
    GcmArgs t{};
    t.te0 = s.te0;
    t.wtab = s.wtab;
    if (threadIdx.x < kSvcStage) stage_flow_tables<kSvcStage>(t);
    __syncthreads();
  } else {  // CTR / ECB contexts: the AES rows only
    stage_rows(s.te0, kGcmRows);
    __syncthreads();
  }
  const RowLanes rl = row_lanes(kGcmRows);
  const bool leader = blockIdx.x == 0u;
  const uint64_t t0 = wall_clock64();
  uint64_t t_last = t0;
  uint32_t cur = s.seq0;
  for (;;) {
    if (threadIdx.x == 0u) {
      uint32_t ex = 0u, q = cur;
      uint32_t d[kSvcDesc] = {};
      if (leader) {
        for (;;) {
          asm volatile("" ::: "memory");  // a fresh read every pass
          u32x4 c0 = sys_load16(s.ring), c1 = sys_load16(s.ring + 4), c2 = sys_load16(s.ring + 8),
                c3 = sys_load16(s.ring + 12), ck = sys_load16(s.kick);
          asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(ck));  // all five reads in flight together
          q = c0[0];
          if (q != cur) {
            if (c1[0] != q || c2[0] != q || c3[0] != q) continue;  // the host is between chunks: read again
            d[0] = c0[1], d[1] = c0[2], d[2] = c0[3];
            d[3] = c1[1], d[4] = c1[2], d[5] = c1[3];
            d[6] = c2[1], d[7] = c2[2], d[8] = c2[3];
            d[9] = c3[1], d[10] = c3[2], d[11] = c3[3];
            if (d[0] == kSvcStop) ex = 1u;
            SVC_STAMP(s, q, 0u);
            break;
          }
          const uint64_t now = wall_clock64();
          // a posted message is always taken first (above); then a kick (another context's
          // service wants this stream slot), idle or lifetime ends the generation
          if (ck[0] == s.gen || now - t_last > s.idle_ticks || now - t0 > s.life_ticks) {
            ex = 1u;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        uint32_t ls_, nch_;
        if (!ex && d[0] <= kSvcOpen && svc_plan(d[1], ls_, nch_, s.ls_min) > 1u) {
          svc_publish(s.go, q, s.gen, d);
        } else if (ex) {  // a STOP descriptor under a seq no message uses
          uint32_t st[kSvcDesc] = {};
          st[0] = kSvcStop;
          svc_publish(s.go, cur ^ 0x80000000u, s.gen, st);
        }  // a message of one workgroup's chunks is the leader's alone: nothing to publish
      } else {
        for (;;) {
          if (svc_take(s.go, cur, s.gen, q, d)) {
            if (d[0] == kSvcStop) ex = 1u;
            break;
          }
          q = cur;
          if (wall_clock64() - t0 > s.cap_ticks) {  // bound: the leader exits long before this
            ex = 1u;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (leader && !ex) SVC_STAMP(s, q, 1u);
      lds_st32(kSvcX, ex);
      lds_st32(kSvcX + 4u, q);
#pragma unroll
      for (uint32_t j = 0; j < kSvcDesc; ++j) lds_st32(kSvcX + 8u + 4u * j, d[j]);
      if (!ex) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // this CU / XCD sees the host's fresh bytes
    }
    __syncthreads();
    if (lds32(kSvcX)) break;
    const uint32_t q = __builtin_amdgcn_readfirstlane(lds32(kSvcX + 4u));
    const uint32_t op = __builtin_amdgcn_readfirstlane(lds32(kSvcX + 8u));
    if (op == kSvcOpen) svc_message<true>(s, rl, q);
    else if (op == kSvcSeal) svc_message<false>(s, rl, q);
    else if (leader) svc_stream_op(s, rl, op, q);  // counter-mode ops are never published
    __syncthreads();  // LDS words reused by the next message
    cur = q;
    t_last = wall_clock64();
  }
  if (leader && threadIdx.x == 0u) __hip_atomic_store(s.exited, s.gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace dev
}  // namespace cmpi
