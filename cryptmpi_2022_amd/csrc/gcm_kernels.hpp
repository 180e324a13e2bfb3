// gcm_kernels.hpp — AES-128-GCM batched seal/open for uniform record batches (gfx950).
//
// Work decomposition (DESIGN.md §"GCM kernel"):
//   record r (len bytes, nb = ceil(len/16) data blocks) has the GHASH input sequence
//   X_0..X_nb-1 = ciphertext blocks, X_nb = length block.  That sequence is cut into nseg
//   segments from the END (every segment but the first has exactly G X-blocks), and every
//   (record, segment) is one "group" of L lanes (L in {1,2,4}) inside one wavefront.  Lane q of
//   a group owns segment slots u = q, q+L, q+2L, ...: it runs AES-CTR on those data blocks,
//   writes ct/pt, and folds its X-blocks into a private Horner accumulator with multiplier H^L
//   (byte table in LDS).  The L partial sums are then weighted by H^w (w = slots after the
//   lane's last one, nibble tables in LDS), XOR-reduced with wavefront shuffles, and the tag is
//   finished in-kernel when the record is one segment; otherwise partials go to HBM and
//   gcm_combine_kernel multiplies them by H^{k·G} and finishes the tag.  Segment 0 also owns the
//   extra slot that computes E_K(J0).
// The arithmetic it implements is BoringSSL's aead_aes_gcm seal/open behind
// EVP_AEAD_CTX_seal/open (aead.h:256-285) — SP 800-38D with a 96-bit IV, no AAD.
#pragma once
#include <type_traits>

#include "aes_device.hpp"
#include "keysetup_kernels.hpp"

namespace cmpi {
namespace dev {

struct GcmArgs {
  const uint8_t* in;
  uint8_t* out;
  const uint8_t* nonces;
  uint64_t in_stride, out_stride, nonce_stride;
  uint32_t len;     // plaintext bytes per record
  uint32_t nb;      // data blocks per record
  uint32_t nrec;
  uint32_t nseg;    // segments per record
  uint32_t G;       // X-blocks per segment (all but the first)
  uint32_t r0;      // X-blocks in the first segment
  uint32_t ngroups; // nrec * nseg
  const u32x4* htab;   // [v][p] byte table of H^L (global), 4096 entries (wide kernel: H^64)
  const u32x4* ntab;   // nibble tables of H^1..H^L (global), L*512 entries (L > 1)
  const uint32_t* te0; // Te0 (global), 256 words
  u32x4* partial;      // nrec*nseg segment partials (nseg > 1)
  u32x4* ekj0;         // nrec E_K(J0) (nseg > 1)
  int32_t* status;     // open: per-record result (may be null)
  const uint32_t* rkp; // device-keyed context: round keys in HBM (keysetup_kernels.hpp), else null
  // Nonce source (CryptMPI framings, DESIGN.md §"602 framing"):
  //  0: 12 bytes at nonces + r*nonce_stride
  //  1: "0000000" || the 5-byte segment prefix at nonces + r*nonce_stride   (602 receiver,
  //     recv.c:594-609 / :749-764 rebuilds the nonce from the wire)
  //  2: "0000000" || flag || BE32(nctr0 + r), flag = nflag (records r < nflag2_from) or
  //     nflag2 (r >= nflag2_from: the last outer message's segments); seal also writes that 5-byte prefix at
  //     nonces + r*nonce_stride                                              (602 sender,
  //     send.c:651-670 / :779-799)
  //  3: the 12 bytes nfix[] for every record; seal also writes them at nonces + r*nonce_stride
  //     when nonces != null                                                  (600 sender, one
  //     RAND_bytes nonce per message, send.c:294-311)
  //  4: fresh nonces, nfix[0] (4 random bytes of the context) || BE64(nfix[1]:nfix[2] + r); seal
  //     writes them at nonces + r*nonce_stride   (RAND_bytes + seal of the naive collectives,
  //     alltoall.c:797-801; cmpi_gcm_seal_batch_fresh)
  uint32_t nmode, nctr0, nflag, nflag2, nflag2_from;
  uint32_t nfix[3];
  // wide decomposition (gcm_flow_kernel): S steps per chunk, nch chunks per record, and the
  // kernel's ten nibble tables H^1,2,3,4,8,12,16,32,48,64 (DevTables::fnib)
  const u32x4* wtab;
  uint32_t S, nch;
  // host-keyed contexts: chunk weights chw[4i + 3] = H^(1 + (nch-1-i)·64S) of chunk i (chunk 0
  // adds E_K(J0): the combine only XORs); null for device-keyed contexts (gcm_combine_kernel
  // weighs the partials, E_K(J0) goes to ekj0)
  const u32x4* chw;
  // the whole batch is one workgroup's units (every record's chunks together): the workgroup's
  // LDS aggregation finishes the tags, no second launch (host-keyed only)
  uint32_t one_wg;
#if CMPI_TOOLS
  uint64_t* probe;  // per-WG phase timestamps (cmpi_debug_set_wide_probe), or null
  uint64_t* unit_stamps;  // service messages: wave 0 of workgroup 0's unit phases (slots 28..31)
#endif
  RoundKeys rk;
};

// Round keys: from the kernel arguments, or (device-derived sub-key contexts) loaded once from
// HBM at kernel entry — uniform address before any store, so they land in SGPRs like args.
__device__ __forceinline__ RoundKeys load_round_keys(const RoundKeys& arg, const uint32_t* rkp) {
  if (!rkp) return arg;
  RoundKeys k;
#pragma unroll
  for (int i = 0; i < 44; ++i) k.w[i] = __builtin_amdgcn_readfirstlane(rkp[i]);
  return k;
}

__device__ __forceinline__ u32x4 ld_blk(const uint8_t* p) { return *reinterpret_cast<const u32x4a*>(p); }
__device__ __forceinline__ void st_blk(uint8_t* p, u32x4 v) { *reinterpret_cast<u32x4a*>(p) = v; }
// Write-through (sc1) 16-byte store: the line leaves this XCD's L2 clean, so the end-of-kernel
// write-back has nothing to write.  The FLOW kernel's record stores (few long records: the
// launch boundary to the combine kernel is on the critical path) — 8 x 1 MiB seal 347 -> 362,
// open 343 -> 355 GiB/s; on the lane kernel it measured neutral (1 KiB) to mixed (4 KiB seal
// -5 %, open +3 %) and is not used there (profiles/r03j_ab_wt_stores.json).
// A buffer store through the builtin (aux 16 = sc1): the compiler counts it and pads its hazards.
// (It was an inline-asm global_store_dwordx4, which hipcc schedules as an opaque instruction: in
// a build whose schedule put a v_xor on the store's data registers right behind it, the open
// kernel stored corrupted plaintext.)  `rec` is wave-uniform (the unit's record), off < 4 GiB.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const uint8_t* rec) {
  const uint64_t b = (uint64_t)rec;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, -1, 0x00020000);
}
__device__ __forceinline__ void st_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
// record data streamed once (MEM bit 0: loads, bit 1: stores) with the non-temporal policy
template <int MEM>
__device__ __forceinline__ u32x4 ld_rec(const uint8_t* p) {
  if constexpr (MEM & 1) return __builtin_nontemporal_load(reinterpret_cast<const u32x4a*>(p));
  else return ld_blk(p);
}
template <int MEM>
__device__ __forceinline__ void st_rec(uint8_t* p, u32x4 v) {
  if constexpr (MEM & 2) __builtin_nontemporal_store(v, reinterpret_cast<u32x4a*>(p));
  else st_blk(p, v);
}

// Record r's 96-bit nonce as three LE words (see GcmArgs::nmode); `writer` (one lane of the
// record, seal only) also writes the nonce / 5-byte prefix the framing puts on the wire.
__device__ __forceinline__ void gcm_nonce(const GcmArgs& a, uint32_t r, bool writer, uint32_t& n0, uint32_t& n1,
                                          uint32_t& n2) {
  uint8_t* nb8 = const_cast<uint8_t*>(a.nonces) + (uint64_t)r * a.nonce_stride;
  if (a.nmode == 0u) {
    const u32a* np = reinterpret_cast<const u32a*>(nb8);
    n0 = np[0];
    n1 = np[1];
    n2 = np[2];
  } else if (a.nmode >= 3u) {
    n0 = a.nfix[0];
    n1 = a.nfix[1];
    n2 = a.nfix[2];
    if (a.nmode == 4u) {  // 64-bit counter in nfix[1]:nfix[2] (host order) + r, stored big-endian
      const uint32_t lo = n2 + r;
      n1 = __builtin_bswap32(n1 + (lo < r ? 1u : 0u));
      n2 = __builtin_bswap32(lo);
    }
    if (writer && nb8) {
      u32a* np = reinterpret_cast<u32a*>(nb8);
      np[0] = n0;
      np[1] = n1;
      np[2] = n2;
    }
  } else {
    uint32_t f, c;
    if (a.nmode == 1u) {
      f = nb8[0];
      c = ((uint32_t)nb8[1] << 24) | ((uint32_t)nb8[2] << 16) | ((uint32_t)nb8[3] << 8) | nb8[4];
    } else {
      f = r >= a.nflag2_from ? a.nflag2 : a.nflag;
      c = a.nctr0 + r;
      if (writer) {
        nb8[0] = (uint8_t)f;
        nb8[1] = (uint8_t)(c >> 24);
        nb8[2] = (uint8_t)(c >> 16);
        nb8[3] = (uint8_t)(c >> 8);
        nb8[4] = (uint8_t)c;
      }
    }
    n0 = 0x30303030u;              // "0000"
    n1 = 0x00303030u | (f << 24);  // "000" || flag
    n2 = __builtin_bswap32(c);     // BE32 counter
  }
}

// LDS: GHASH byte table [v][p] @0 (64 KiB), AES row image @64K (64 KiB), nibble tables of
// H^1..H^(L-1) @128K ((L-1) x 8 KiB; a lane whose weight is H^L multiplies by the byte table),
// then the workgroup's progress counter (16 B, gcm_progress_prio).
// The byte table is built in place from its 128 single-bit entries, staged first into a 2 KiB
// basis area after the progress counter (build_byte_table).
constexpr uint32_t kGcmRows = 65536u;
constexpr uint32_t kGcmNib = 131072u;
__host__ __device__ constexpr uint32_t gcm_prog_off(int L) { return kGcmNib + (uint32_t)(L - 1) * 8192u; }
__host__ __device__ constexpr uint32_t gcm_basis_off(int L) { return gcm_prog_off(L) + 16u; }
__host__ __device__ constexpr uint32_t gcm_lds_bytes(int L) { return gcm_basis_off(L) + 2048u; }

// GHASH byte table [v][p] (entry (v, p) at dst + v*256 + p*16, the layout of gf128_host.hpp
// build_byte_table) built in LDS from the global copy's 128 single-bit entries (v = 2^k):
// entry (v, p) = XOR of the entries (2^k, p) over the set bits k of v (the table is linear in v).
// 2 KiB leave L2 per workgroup instead of 64 KiB: with every CU staging at once the copy was
// bound by L2 bandwidth (256 workgroups x 64 KiB).  Thread t builds position p = t & 15, values
// 4m .. 4m+3 (m = t >> 4).  Ends with a barrier.
__device__ __forceinline__ void build_byte_table(const u32x4* __restrict__ src, uint32_t dst, uint32_t basis) {
  for (uint32_t i = threadIdx.x; i < 128u; i += blockDim.x) {  // basis[k][p] = entry (2^k, p)
    const uint32_t k = i >> 4, p = i & 15u;
    lds_st128(basis + i * 16u, src[(1u << k) * 16u + p]);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < 1024u; t += blockDim.x) {
    const uint32_t p = t & 15u, m = t >> 4;
    u32x4 e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = lds128(basis + ((uint32_t)k * 16u + p) * 16u);
    u32x4 b = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 2; k < 8; ++k)
      if ((m >> (k - 2)) & 1u) b ^= e[k];
    const uint32_t o = dst + 4u * m * 256u + p * 16u;
    lds_st128(o, b);
    lds_st128(o + 256u, b ^ e[0]);
    lds_st128(o + 512u, b ^ e[1]);
    lds_st128(o + 768u, b ^ e[0] ^ e[1]);
  }
}

// Diagnostics build only (tools/Makefile, -DCMPI_TOOLS=1): per-workgroup wall-clock stamps of
// the kernel phases (tools/probe_lane.py, tools/probe_flow.py).  The product library has none.
#if CMPI_TOOLS
#define CMPI_PROBE(a, slot)                                                                    \
  do {                                                                                         \
    if ((a).probe && threadIdx.x == 0u) (a).probe[blockIdx.x * 8u + (slot)] = wall_clock64(); \
  } while (0)
#else
#define CMPI_PROBE(a, slot) \
  do {                      \
  } while (0)
#endif

// Lane groups (many records): see the file header.  Waves take wave priority by progress
// (progress_prio: a workgroup counter in LDS; behind the average -> priority 3), so waves of
// equal work finish together.
// PAIR (L = 4): the record stores are grouped by 128-byte output line — a group's lanes hold their
// outputs of the last two steps and store a line's 8 blocks together in the step that completes
// it, so each line reaches the L2 whole instead of as two halves a step apart; the computation's
// schedule is unchanged.
// Diagnostics builds only (tools/ab_build.sh ... -DCMPI_ABLATE=<bits>): parts of the lane kernel's
// main loop switched off to measure what each costs (wrong output; never in the product build):
// 1 progress_prio, 2 the GHASH multiply (acc ^= x), 4 the AES (keystream = counter block).
#ifndef CMPI_ABLATE
#define CMPI_ABLATE 0
#endif
// Input blocks in flight per lane in the lane kernel's main loop (loaded this many steps ahead).
#ifndef CMPI_LANE_PREFETCH
#define CMPI_LANE_PREFETCH 1
#endif
#ifndef CMPI_LANE_UNROLL
#define CMPI_LANE_UNROLL 1
#endif
// progress_prio every CMPI_PRIO_EVERY steps of the line-store loop.  (Measured, not taken: the
// priority taken from the previous step's counter value so the add's round trip overlaps a step
// instead of draining the wave's LDS queue — seal 59.92 -> 60.89 us, profiles/r05ah_prio_late_ab.txt.)
#ifndef CMPI_PRIO_EVERY
#define CMPI_PRIO_EVERY 1
#endif
// record loads / stores of the full-block loop: MEM bit 0 non-temporal loads, bit 1 stores
#ifndef CMPI_LANE_MEM
#define CMPI_LANE_MEM 0
#endif
template <int L, bool DECRYPT, int PAIR>
__global__ __launch_bounds__(1024) void gcm_lane_kernel(GcmArgs a) {
  CMPI_PROBE(a, 0u);
  stage_rows(a.te0, kGcmRows);
  if (L > 1) stage_copy(a.ntab, kGcmNib, (uint32_t)(L - 1) * 512u);
  if (threadIdx.x == 0u) lds_st32(gcm_prog_off(L), 0u);
  build_byte_table(a.htab, 0u, gcm_basis_off(L));
  __syncthreads();
  CMPI_PROBE(a, 1u);

  const RoundKeys rk = load_round_keys(a.rk, a.rkp);  // folded (host / keysetup kernel)
  const uint32_t lane = threadIdx.x & 63u;
  const RowLanes rl = row_lanes(kGcmRows);
  const GhashLane gl = ghash_lane();
  const uint32_t q = threadIdx.x & (uint32_t)(L - 1);
  const uint32_t nb = a.nb;
  const uint32_t rem = a.len - 16u * (nb ? nb - 1u : 0u);       // bytes in the last data block
  const uint32_t nbf = nb == 0u ? 0u : (rem == 16u ? nb : nb - 1u);  // full data blocks
  const uint64_t cbits = (uint64_t)a.len * 8u;
  const u32x4 lenblk = {0u, 0u, __builtin_bswap32((uint32_t)(cbits >> 32)), __builtin_bswap32((uint32_t)cbits)};

  uint32_t done = 0;  // slots this wave has started (progress_prio)
  const uint32_t groups_per_iter = (gridDim.x * blockDim.x) / (uint32_t)L;
  for (uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) / (uint32_t)L; g < a.ngroups; g += groups_per_iter) {
    const uint32_t r = (a.nseg == 1) ? g : g / a.nseg;
    const uint32_t s = g - r * a.nseg;
    const uint32_t x0 = (s == 0) ? 0u : a.r0 + (s - 1u) * a.G;
    const uint32_t x1 = a.r0 + s * a.G;
    const uint32_t nxs = x1 - x0;                      // X-blocks in this segment
    const uint32_t nslots = nxs + (s == 0 ? 1u : 0u);  // + the J0 slot
    const uint32_t xf = x1 < nbf ? x1 : nbf;
    const uint32_t nfull = xf > x0 ? xf - x0 : 0u;     // full data-block slots [0, nfull)
    const uint8_t* in_rec = a.in + (uint64_t)r * a.in_stride;
    uint8_t* out_rec = a.out + (uint64_t)r * a.out_stride;
    uint32_t n0, n1, n2;
    gcm_nonce(a, r, !DECRYPT && s == 0u && q == 0u, n0, n1, n2);

    CtrCache cc;
    uint32_t cc_win = 0xffffffffu;
    auto keystream = [&](uint32_t ctr) -> u32x4 {  // E_K(nonce || ctr)
      const uint32_t w3 = __builtin_bswap32(ctr);
      if ((ctr >> 8) != cc_win) {
        ctr_cache_fill(rk, rl, n0, n1, n2, w3, cc);
        cc_win = ctr >> 8;
      }
      uint32_t s0 = n0, s1 = n1, s2 = n2, s3 = w3;
      if constexpr (!(CMPI_ABLATE & 4)) aes128_enc_ctr(rk, rl, cc, w3, s0, s1, s2, s3);
      return u32x4{s0, s1, s2, s3};
    };
    u32x4 acc = {0u, 0u, 0u, 0u};
    u32x4 ekj0 = {0u, 0u, 0u, 0u};

    // ---- full data blocks: slot u = X position x0 + u, counter 2 + x0 + u.  Branch-free main
    // loop, one input block in flight per lane (loaded a whole slot ahead: 97 VGPRs, no spills).
    // Loads past the full blocks are clamped to the segment's LAST full block (value unused): its
    // line was just read, so the clamped load hits L2 (clamped to the first block it re-read a line
    // fetched ~60 us earlier — +23 MB HBM reads per config-2 launch).
    const uint8_t* ip = in_rec + 16u * x0;
    uint8_t* op = out_rec + 16u * x0;
    if (nfull > 0u) {
      auto ld = [&](uint32_t uu) { return ld_rec<CMPI_LANE_MEM>(ip + 16u * (uu < nfull ? uu : nfull - 1u)); };
      if constexpr (PAIR != 0 && L == 4) {
        // Line-aligned stores: a 128-byte line of the output holds 8 blocks, two group steps.  The
        // group's blocks are computed in order as always; each lane keeps its outputs of the last
        // two steps (h1, h2) and the lanes store a line's 8 blocks together in the step that
        // completes it (every other step), so each line reaches the L2 whole.  s0 = position of
        // block 0 in its line (16-byte units, absolute address); steps run for all four lanes.
        const int32_t s0 = (int32_t)(((uint64_t)(uintptr_t)op >> 4) & 7u);
        const int32_t nf = (int32_t)nfull;
        const uint32_t nsteps = (nfull + 3u) >> 2;
        u32x4 v = ld(q), h1 = {0u, 0u, 0u, 0u}, h2 = {0u, 0u, 0u, 0u};
        u32x4 vn = CMPI_LANE_PREFETCH >= 2 ? ld(q + 4u) : u32x4{0u, 0u, 0u, 0u};
        u32x4 vnn = CMPI_LANE_PREFETCH >= 3 ? ld(q + 8u) : u32x4{0u, 0u, 0u, 0u};
        auto put = [&](int32_t b, u32x4 x) {
          if (b >= 0 && b < nf) st_rec<CMPI_LANE_MEM>(op + 16u * (uint32_t)b, x);
        };
#pragma unroll CMPI_LANE_UNROLL
        for (uint32_t k = 0; k < nsteps; ++k) {
          const int32_t u = 4 * (int32_t)k + (int32_t)q;
          if constexpr (!(CMPI_ABLATE & 1)) {
            if (CMPI_PRIO_EVERY == 1 || k % CMPI_PRIO_EVERY == 0u) progress_prio(gcm_prog_off(L), ++done);
          }
          const u32x4 o = v ^ keystream(2u + x0 + (uint32_t)u);
          const int32_t j = (s0 + 4 * (int32_t)k) & 7;
          if constexpr (PAIR == 1) {
            if (j >= 4) {  // this step ends the line of blocks [4k - j, 4k + 7 - j]
              if ((int32_t)q + j <= 7) {
                put(u - 4, h1);
                put(u, o);
              } else {
                put(u - 8, h2);
                put(u - 4, h1);
              }
            }
          } else {  // the same stores as selects: two predicated stores per step, no branches
            const bool cur = (int32_t)q + j <= 7;
            const int32_t ba = cur ? u - 4 : u - 8;
            const u32x4 xa = cur ? h1 : h2, xb = cur ? o : h1;
            if (j >= 4 && ba >= 0) st_rec<CMPI_LANE_MEM>(op + 16u * (uint32_t)ba, xa);
            if (j >= 4 && ba + 4 >= 0 && ba + 4 < nf) st_rec<CMPI_LANE_MEM>(op + 16u * (uint32_t)(ba + 4), xb);
          }
          h2 = h1;
          h1 = o;
          if constexpr (CMPI_ABLATE & 2) {
            if (u < nf) acc ^= DECRYPT ? v : o;
          } else {
            if (u < nf) acc = gmul_byte(acc, gl, DECRYPT ? v : o);
          }
          if constexpr (CMPI_LANE_PREFETCH >= 3) {
            v = vn;
            vn = vnn;
            vnn = ld((uint32_t)u + 12u);
          } else if constexpr (CMPI_LANE_PREFETCH == 2) {
            v = vn;
            vn = ld((uint32_t)u + 8u);
          } else {
            v = ld((uint32_t)u + 4u);
          }
        }
        // the blocks after the last completed line
        const int32_t kl = (int32_t)nsteps - 1, jl = (s0 + 4 * kl) & 7;
        const int32_t F = jl >= 4 ? 4 * kl + 7 - jl : 4 * kl - 1 - jl;
        const int32_t b1 = 4 * kl + (int32_t)q, b2 = b1 - 4;
        if (b2 > F) put(b2, h2);
        if (b1 > F) put(b1, h1);
      } else {
        u32x4 v = ld(q);
        for (uint32_t u = q; u < nfull; u += (uint32_t)L) {
          progress_prio(gcm_prog_off(L), ++done);
          const u32x4 o = v ^ keystream(2u + x0 + u);
          st_rec<CMPI_LANE_MEM>(op + 16u * u, o);
          acc = gmul_byte(acc, gl, DECRYPT ? v : o);
          v = ld(u + (uint32_t)L);
        }
      }
    }
    // ---- special slots: partial last block, length block, J0 (the lane's slots >= nfull)
    for (uint32_t ut = nfull <= q ? q : q + (uint32_t)L * ((nfull - q + (uint32_t)L - 1u) / (uint32_t)L); ut < nslots;
         ut += (uint32_t)L) {
      const uint32_t j = x0 + ut;
      const bool j0 = ut >= nxs;
      u32x4 ks = {0u, 0u, 0u, 0u};
      if (j0 || j < nb) ks = keystream(j0 ? 1u : 2u + j);
      if (j0) {
        ekj0 = ks;
        continue;
      }
      u32x4 x = lenblk;
      if (j < nb) {  // the partial last block (rem < 16)
        const u32x4 p = load_partial(in_rec + 16u * j, rem);
        const u32x4 o = mask_bytes(p ^ ks, rem);
        store_partial(out_rec + 16u * j, o, rem);
        x = DECRYPT ? p : o;
      }
      acc = gmul_byte(acc, gl, x);
    }

    // ---- weight the lane's Horner sum by H^w, w = nxs - (lane's last X slot)
    u32x4 f = {0u, 0u, 0u, 0u};
    if (L == 1) {
      f = gmul_byte(acc, gl);  // L = 1: byte table holds H, w = 1
    } else if (q < nxs) {
      const uint32_t ulast = q + (uint32_t)L * ((nxs - 1u - q) / (uint32_t)L);
      const uint32_t w = nxs - ulast;  // 1..L: H^L is the Horner byte table, H^1..H^(L-1) nibble tables
      if (w == (uint32_t)L) f = gmul_byte(acc, gl);
      else f = gmul_nib(acc, kGcmNib + (w - 1u) * 8192u);
    }
    if (a.nseg == 1) f ^= ekj0;
    if (L > 1) f = xq1(f);
    if (L > 2) f = xq2(f);

    if (a.nseg > 1) {
      if (q == 0) a.partial[g] = f;
      if (s == 0 && (nxs % (uint32_t)L) == q) a.ekj0[r] = ekj0;  // lane that owned slot nxs
      continue;
    }
    // single-segment record: finish the tag here
    if (!DECRYPT) {
      if (q == 0) st_blk(out_rec + a.len, f);
    } else {
      int ok = 1;
      if (q == 0) {
        const u32x4 d = ld_blk(in_rec + a.len) ^ f;
        ok = ((d[0] | d[1] | d[2] | d[3]) == 0u) ? 1 : 0;
        if (a.status) a.status[r] = ok;
      }
      if (L > 1) ok = __shfl(ok, (int)(lane & ~(uint32_t)(L - 1)));
      if (!ok) {  // zero-fill this record's plaintext (aead.h:276-278)
        for (uint32_t v = q; v < nxs; v += (uint32_t)L) {
          const uint32_t j = x0 + v;
          if (j >= nb) continue;
          if (j + 1u < nb || rem == 16u) st_blk(out_rec + 16u * j, u32x4{0u, 0u, 0u, 0u});
          else store_partial(out_rec + 16u * j, u32x4{0u, 0u, 0u, 0u}, rem);
        }
      }
    }
  }
#if CMPI_TOOLS
  if (a.probe) {
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0u && w < 6u) a.probe[blockIdx.x * 8u + 2u + w] = wall_clock64();
  }
#endif
}

// ---------------------------------------------------------------- FLOW wide kernel
// Few long records (the naive Alltoall's p peer blocks of 1 MiB, alltoall.c:795-834; 602
// segments; single EVP messages): a record's X-sequence is cut from the END into chunks of
// C = 64*S X-blocks (chunk 0 takes the remainder: C <= its length < 2C), every (record, chunk) is
// ONE wavefront.  At step k lane q owns X position base + 64k + q, so each wave-instruction moves
// 1 KiB of contiguous record data; the lane folds its blocks by Horner in H^64 (nibble table).
// The 64 lane accumulators are combined by a radix-4 tree — three levels, each ONE nibble
// multiply per active lane by a lane-chosen table (H^1..3, H^4..12, H^16..48), lanes packed low so
// a level touches 3, 1, 1 LDS lane groups — into V = XOR_q acc_q · H^(63-q).  NT threads per
// workgroup (512 or 1024), every table load issued before any LDS store.
//  * Host-keyed contexts: the chunk weight H^(1 + (nch-1-i)C) (host-built, chw) by one
//    wave-cooperative product (gmul_wave), E_K(J0) folded into chunk 0, so the tag is the XOR of
//    the chunk partials: gcm_xor_combine_kernel, or — every chunk of the batch in one workgroup —
//    the workgroup's own LDS aggregation in the same launch (one_wg).
//  * Device-keyed contexts (602 sub-keys: H exists only in HBM; chw == null): partial = V · H
//    (nibble table H^1), E_K(J0) to ekj0[r], and gcm_combine_kernel applies H^((nch-1-i)C) as
//    products of the key-setup kernel's H^(2^i) (C is a power of two for these contexts).
constexpr uint32_t kFlowAgg = 147456u;         // aggregation slots, 16 x 16 B partials + 16 x 4 B records
constexpr uint32_t kFlowLds = kFlowAgg + 512u;
constexpr uint32_t kFlowFail = kFlowAgg + 448u;  // one-workgroup open: per-slot failed record + 1

__device__ __forceinline__ uint32_t flow_tab(uint32_t f) {  // nibble table f (keysetup_kernels.hpp flow_nib_exp)
  return f < 8u ? f * 8192u : 131072u + (f - 8u) * 8192u;
}

// Tables of the FLOW kernel: the AES row image from Te0 (1 KiB) and the ten nibble tables
// (80 KiB), all loads issued before any LDS store (one L2 round trip).  (Measured, not taken:
// building the nibble tables in LDS from their ten multipliers with nib_row_to_lds — 160 B fetched
// instead of 80 KiB — staged at 5.4 us instead of 2.6 on 8 x 1 MiB: the 320 rows' VALU + 80 KiB
// of ds_write_b128 cost more than the L2 round trip.  Nor staging only the Horner's tables first
// and the tree's 64 KiB from registers behind a barrier after the Horner: 8 x 1 MiB seal 19.67 ->
// 20.15 us, profiles/r05aq_late_*.)
// (stage_flow_tables: the loads and stores only, by threads 0..NT-1 — the resident service runs
// more threads than it stages with; stage_flow adds the workgroup barrier.)
template <int NT>
__device__ __forceinline__ void stage_flow_tables(const GcmArgs& a) {
  constexpr int kR = 1024 / NT, kW = 5120 / NT;  // loads per thread
  uint32_t rv[kR];
  u32x4 wv[kW];
  const uint32_t t = threadIdx.x;
#pragma unroll
  for (int j = 0; j < kR; ++j) rv[j] = a.te0[(t + j * NT) >> 2];
#pragma unroll
  for (int j = 0; j < kW; ++j) wv[j] = a.wtab[t + j * NT];
#pragma unroll
  for (int j = 0; j < kR; ++j) {  // row image: entry e -> 64 words (Te0 x32 | Te1 x32), 4 threads
    const uint32_t i = t + j * NT, e = i >> 2, q = i & 3u;
    const uint32_t v = q >= 2u ? rotl8(rv[j]) : rv[j];
    const u32x4 w = {v, v, v, v};
    const uint32_t o = kGcmRows + e * 256u + q * 64u;
    lds_st128(o, w);
    lds_st128(o + 16u, w);
    lds_st128(o + 32u, w);
    lds_st128(o + 48u, w);
  }
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    const uint32_t e = t + j * NT;
    lds_st128(flow_tab(e >> 9) + (e & 511u) * 16u, wv[j]);
  }
}
template <int NT>
__device__ __forceinline__ void stage_flow(const GcmArgs& a) {
  stage_flow_tables<NT>(a);
  __syncthreads();
}

__device__ __forceinline__ u32x4 shfl4(u32x4 v, uint32_t src) {
  u32x4 r;
  r[0] = __shfl((int)v[0], (int)src);
  r[1] = __shfl((int)v[1], (int)src);
  r[2] = __shfl((int)v[2], (int)src);
  r[3] = __shfl((int)v[3], (int)src);
  return r;
}

// Radix-4 lane tree: returns (lane 0) V = XOR_q acc_q · H^(63-q).  Level l combines groups of
// four: lanes 16p+g (level 0), 4p+h (level 1), p (level 2) hold the p-th member, multiply by
// H^((3-p)·4^l) (tables 2-p, 5-p, 8-p), and XOR across p by two butterflies.
__device__ __forceinline__ u32x4 flow_tree_r4(u32x4 acc, uint32_t lane) {
  // the lane-chosen table offsets are made opaque where they are used: left visible, the compiler
  // hoists the 32 per-lookup addresses of each level out of the unit loop and spills them
  u32x4 x = shfl4(acc, 4u * (lane & 15u) + (lane >> 4));
  if (lane < 48u) {
    uint32_t tb = flow_tab(2u - (lane >> 4));
    asm volatile("" : "+v"(tb)::"memory");
    x = gmul_nib(x, tb);
  }
  x = x32(x16(x));  // every lane t: A_(t & 15)
  x = shfl4(x, 4u * (lane & 3u) + ((lane >> 2) & 3u));
  if (lane < 12u) {
    uint32_t tb = flow_tab(5u - (lane >> 2));
    asm volatile("" : "+v"(tb)::"memory");
    x = gmul_nib(x, tb);
  }
  x = xr8(xr4(x));  // lanes t < 16: B_(t & 3)
  if (lane < 3u) {
    uint32_t tb = flow_tab(8u - lane);
    asm volatile("" : "+v"(tb)::"memory");
    x = gmul_nib(x, tb);
  }
  x = xq2(xq1(x));  // lane 0: V
  return x;
}

// DK: device-keyed context (round keys loaded from HBM, partials weighted by the combine launch);
// its own instantiation so the host-keyed form keeps its round keys as kernel arguments (the
// runtime choice cost the host-keyed kernel 53 VGPRs and SGPR spills).
// (Measured, not taken: finishing multi-workgroup batches in the same launch — chunk partials
// published write-through, per-group arrival counters, the last workgroup XORs every record's
// partials and zero-fills forged records, plaintext stored write-through — 8 x 1 MiB seal 30.8 vs
// 20.8 us, 1 x 64 KiB 19.4 vs 13.4 us with the XOR-combine launch: profiles/r03d_flow_fused_ab.txt.
// A second form — no fences: each wave's partial stored write-through, one agent-scope add per
// record and round, the record's last arriving workgroup XORs that record's partials, per-stream
// zeroed counters — was also slower: 8 x 1 MiB 23.5 vs 21.1 us, 1 x 64 KiB 14.6 vs 13.4, 1 x 8 MiB
// 24.5 vs 21.9 (profiles/r03f_flow_fused_ab.txt): store drain + add round trip + partial loads on
// the last workgroup's path cost more than the launch boundary.  Round 5 re-measured a one-counter
// form (grid's last arriver finishes every record, counter zeroed by hipStreamWriteValue32): 29.8
// vs 19.3 us, of which the stream write alone costs 7.7 us per call (profiles/r05j_*, r05k_*).)
// Unit u = (record r, chunk i) of a flow decomposition: chunk 0 absorbs the remainder (r0 X-blocks,
// ceil(r0/64) steps), the others are C = 64·S X-blocks; returns the base X position of lane 0's
// first step.  sep: the X-sequence is the data blocks only (the resident service: the length
// block and E_K(J0) are another wave's, flow_unit<.., SEP>).
__device__ __forceinline__ int32_t flow_unit_base(const GcmArgs& a, uint32_t u, uint32_t& r, uint32_t& i,
                                                  uint32_t& steps, bool sep = false) {
  const int32_t nx = (int32_t)a.nb + (sep ? 0 : 1), C = 64 * (int32_t)a.S;
  r = u / a.nch;
  i = u - r * a.nch;
  steps = i == 0u ? (a.r0 + 63u) >> 6 : a.S;
  return i == 0u ? (int32_t)a.r0 - 64 * (int32_t)steps : nx - (int32_t)(a.nch - i) * C;
}
__device__ __forceinline__ bool flow_full_blk(const GcmArgs& a, int32_t p, uint32_t rem) {
  return p >= 0 && p < (int32_t)a.nb && (p + 1 < (int32_t)a.nb || rem == 16u);
}
// X block of step k for this lane (full data blocks only; others load a harmless block 0)
__device__ __forceinline__ u32x4 flow_load_x(const GcmArgs& a, const uint8_t* in_rec, int32_t base, uint32_t k,
                                             uint32_t rem) {
  const int32_t p = base + 64 * (int32_t)k + (int32_t)(threadIdx.x & 63u);
  return ld_blk(in_rec + 16u * (uint32_t)(flow_full_blk(a, p, rem) ? p : 0));
}

// One wavefront's unit: AES-CTR of its X positions (ciphertext / plaintext stored), Horner in
// H^64 per lane, the radix-4 lane tree, and the chunk weight (host-keyed: H^(1 + (nch-1-i)C) from
// a.chw, E_K(J0) folded into chunk 0) or V·H (device-keyed: E_K(J0) to a.ekj0).  va, vb: the
// unit's first two input rows when `pre` (requested before the table staging).  Returns the
// weighted partial (every lane), r = the unit's record.
// SEP (the resident service, host-keyed): the chunks cover the data blocks only, chunk weights
// H^(2 + (nch-1-i)C); the length block (L·H) and E_K(J0) are added by another wave (svc_j0_wave),
// so a chunk of 64·S blocks is exactly S steps — chunk 0 no longer runs a near-empty extra step.
// OWN: load only the unit's own input rows (records in host memory, read over PCIe).
template <bool DECRYPT, bool DK, bool SEP = false, bool OWN = SEP>
__device__ __forceinline__ u32x4 flow_unit(const GcmArgs& a, const RoundKeys& rk, const RowLanes& rl, u32x4 lenblk,
                                           uint32_t u, bool pre, u32x4 va, u32x4 vb, uint32_t& r) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nb = a.nb;
  const int32_t nx = (int32_t)nb + (SEP ? 0 : 1);
  const uint32_t rem = a.len - 16u * (nb ? nb - 1u : 0u);
  uint32_t i, steps;
  const int32_t base = flow_unit_base(a, u, r, i, steps, SEP);
  const uint8_t* in_rec = a.in + (uint64_t)r * a.in_stride;
  uint8_t* out_rec = a.out + (uint64_t)r * a.out_stride;
  uint32_t n0, n1, n2;
  gcm_nonce(a, r, !DECRYPT && i == 0u && lane == 0u, n0, n1, n2);
  // OWN (records in host memory: the service's messages, direct host paths): input rows of steps
  // beyond the unit's own are not loaded (wave-uniform) — they are the next chunk's blocks, a
  // second PCIe read of them (64 KiB served seal 13.9 -> 11.8 us).  On device records the same
  // skip made the flow kernel slower (8 x 1 MiB seal 19.7 -> 20.4 us, open 20.2 -> 21.9: the
  // over-read rows are L2 hits that warm the next chunk, profiles/r05w_flow_prefetch_ab.txt), so
  // there they are still loaded.
  auto prefetch = [&](uint32_t k) -> u32x4 {
    return (!OWN || k < steps) ? flow_load_x(a, in_rec, base, k, rem) : u32x4{0u, 0u, 0u, 0u};
  };
  CtrCache cc;
  uint32_t cc_win = 0xffffffffu;
  auto keystream = [&](uint32_t ctr) -> u32x4 {
    const uint32_t w3 = __builtin_bswap32(ctr);
    if ((ctr >> 8) != cc_win) {
      ctr_cache_fill(rk, rl, n0, n1, n2, w3, cc);
      cc_win = ctr >> 8;
    }
    uint32_t s0, s1, s2, s3;
    aes128_enc_ctr(rk, rl, cc, w3, s0, s1, s2, s3);
    return u32x4{s0, s1, s2, s3};
  };
  u32x4 acc = {0u, 0u, 0u, 0u};
  const __amdgpu_buffer_rsrc_t orsrc = wt_rsrc(out_rec);
  auto consume_ks = [&](uint32_t k, u32x4 v, u32x4 ks) {
    const int32_t p = base + 64 * (int32_t)k + (int32_t)lane;
    u32x4 x = {0u, 0u, 0u, 0u};
    if (p >= 0 && p < (int32_t)nb) {
      uint8_t* op = out_rec + 16u * (uint32_t)p;
      if (flow_full_blk(a, p, rem)) {
        const u32x4 o = v ^ ks;
        st_wt(orsrc, 16u * (uint32_t)p, o);
        x = DECRYPT ? v : o;
      } else {
        const u32x4 pp = load_partial(in_rec + 16u * (uint32_t)p, rem);
        const u32x4 o = mask_bytes(pp ^ ks, rem);
        store_partial(op, o, rem);
        x = DECRYPT ? pp : o;
      }
    } else if (!SEP && p == nx - 1) {
      x = lenblk;
    }
    if (k == 0u) acc = x;  // wave-uniform; acc was 0
    else acc = gmul_nib(acc, flow_tab(9u)) ^ x;
  };
  auto ctr_of = [&](uint32_t k) { return 2u + (uint32_t)(base + 64 * (int32_t)k + (int32_t)lane); };
  if (!pre) {
    va = prefetch(0);
    vb = prefetch(1);
  }
#if CMPI_TOOLS
  auto ustamp = [&](uint32_t slot) {
    if (a.unit_stamps && blockIdx.x == 0u && threadIdx.x == 0u) a.unit_stamps[slot] = wall_clock64();
  };
#else
  auto ustamp = [](uint32_t) {};
#endif
  uint32_t it = 0;
  // E_K(J0), folded into chunk 0's partial (only lane 0's copy is used).  Chunk 0 holds the
  // r0 = G..2G-1 leading positions, so its first step is partial whenever 64 does not divide
  // r0 (1 MiB: 257 positions, lane 63 alone): lane 0 is idle there and encrypts J0 in that
  // step instead of the wave paying a whole AES pass for it afterwards.
  const bool j0_step0 = !SEP && i == 0u && base < 0;
  u32x4 ekj = {0u, 0u, 0u, 0u};
  for (uint32_t k = 0; k < steps; k += 2u) {
    rotate_prio(it++);  // (progress_prio here — the lane kernel's — was slower: 8 x 1 MiB seal
                        // 19.43 -> 20.36 us, profiles/r05ao_flow_pprio_*.txt)
    const u32x4 ks = keystream(k == 0u && j0_step0 && lane == 0u ? 1u : ctr_of(k));
    if (k == 0u) ekj = ks;
    if (k == 0u) ustamp(28u);  // first keystream done (cache fill + one AES pass)
    consume_ks(k, va, ks);
    if (k == 0u) ustamp(29u);  // its input block arrived, ct stored, Horner step
    va = prefetch(k + 2u);
    if (k + 1u < steps) consume_ks(k + 1u, vb, keystream(ctr_of(k + 1u)));
    vb = prefetch(k + 3u);
  }
  if (SEP) ekj = u32x4{0u, 0u, 0u, 0u};
  else if (!j0_step0) ekj = i == 0u ? keystream(1u) : u32x4{0u, 0u, 0u, 0u};
  if (pre) CMPI_PROBE(a, 2u);
  ustamp(30u);  // all steps done
  u32x4 V = flow_tree_r4(acc, lane);
#pragma unroll
  for (int c = 0; c < 4; ++c) V[c] = (uint32_t)__builtin_amdgcn_readfirstlane(V[c]);
  u32x4 pw;
  if constexpr (!DK) {
    pw = gmul_wave(V, a.chw[4u * i + 3u]) ^ ekj;  // H^(1 + (nch-1-i)C) · V, E_K(J0) in chunk 0
  } else {  // device-keyed: V · H here, H^((nch-1-i)C) and E_K(J0) in gcm_combine_kernel
    pw = gmul_nib(V, flow_tab(0u));
    if (i == 0u && lane == 0u) a.ekj0[r] = ekj;
  }
  if (pre) CMPI_PROBE(a, 5u);
  ustamp(31u);  // lane tree + chunk weight done
  return pw;
}

// HOSTIN: the records are in host memory (device addresses of page-locked pages): each unit reads
// only its own input rows (flow_unit<.., OWN>).
template <bool DECRYPT, int NT, bool DK, bool HOSTIN = false>
__global__ __launch_bounds__(NT) void gcm_flow_kernel(GcmArgs a) {
  CMPI_PROBE(a, 0u);
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t nb = a.nb;
  const uint32_t rem = a.len - 16u * (nb ? nb - 1u : 0u);
  constexpr uint32_t wpb = NT / 64;
  const uint32_t units = a.nrec * a.nch;
  // the first unit's first two input rows are requested before the table staging: their HBM
  // latency overlaps it
  u32x4 va0 = {0u, 0u, 0u, 0u}, vb0 = {0u, 0u, 0u, 0u};
  {
    const uint32_t u = blockIdx.x * wpb + wv;
    if (u < units) {
      uint32_t r, i, steps;
      const int32_t base = flow_unit_base(a, u, r, i, steps);
      va0 = flow_load_x(a, a.in + (uint64_t)r * a.in_stride, base, 0u, rem);
      if (!HOSTIN || steps > 1u) vb0 = flow_load_x(a, a.in + (uint64_t)r * a.in_stride, base, 1u, rem);
    }
  }
  stage_flow<NT>(a);
  CMPI_PROBE(a, 1u);
  const RoundKeys rk = DK ? load_round_keys(a.rk, a.rkp) : a.rk;  // folded (keysetup kernel / host args)
  const RowLanes rl = row_lanes(kGcmRows);
  const uint64_t cbits = (uint64_t)a.len * 8u;
  const u32x4 lenblk = {0u, 0u, __builtin_bswap32((uint32_t)(cbits >> 32)), __builtin_bswap32((uint32_t)cbits)};
  for (uint32_t ub = blockIdx.x * wpb; ub < units; ub += gridDim.x * wpb) {  // workgroup-uniform
    const uint32_t u = ub + wv;
    u32x4 pw = {0u, 0u, 0u, 0u};
    uint32_t r = 0xffffffffu;
    if (u < units)  // wave-uniform
      pw = flow_unit<DECRYPT, DK, false, HOSTIN>(a, rk, rl, lenblk, u, ub == blockIdx.x * wpb, va0, vb0, r);
    if (DK || !a.one_wg) {  // partials for the combine launch, stored write-through like the records
      if (u < units && lane == 0u) st_wt(wt_rsrc(reinterpret_cast<const uint8_t*>(a.partial)), 16u * u, pw);
      continue;
    }
    // one-workgroup batch (host-keyed): every chunk of every record is in this workgroup, so the
    // XOR of a record's partials here is its tag
    if (lane == 0u) {
      lds_st128(kFlowAgg + 16u * wv, pw);
      lds_st32(kFlowAgg + 256u + 4u * wv, r);
      lds_st32(kFlowFail + 4u * wv, 0u);
    }
    // open: this wave's plaintext stores are performed before the barrier, so a zero-fill after it
    // lands behind them in the same L2
    if (DECRYPT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t l = threadIdx.x;
    const uint32_t rr = l < wpb ? lds32(kFlowAgg + 256u + 4u * l) : 0xffffffffu;
    if (rr != 0xffffffffu && (l == 0u || lds32(kFlowAgg + 256u + 4u * (l - 1u)) != rr)) {  // first slot of rr
      u32x4 x = {0u, 0u, 0u, 0u};
      for (uint32_t j = l; j < wpb && lds32(kFlowAgg + 256u + 4u * j) == rr; ++j) x ^= lds128(kFlowAgg + 16u * j);
      if (!DECRYPT) {
        st_blk(a.out + (uint64_t)rr * a.out_stride + a.len, x);
      } else {
        const u32x4 d = ld_blk(a.in + (uint64_t)rr * a.in_stride + a.len) ^ x;
        const bool ok = (d[0] | d[1] | d[2] | d[3]) == 0u;
        a.status[rr] = ok ? 1 : 0;
        if (!ok) lds_st32(kFlowFail + 4u * l, rr + 1u);
      }
    }
    __syncthreads();  // slots reused by the next round
    if (DECRYPT) {  // zero-fill the failed records (aead.h:276-278), whole workgroup
      for (uint32_t j = 0; j < wpb; ++j) {
        const uint32_t f = lds32(kFlowFail + 4u * j);  // rr + 1 of a failed record, else 0
        if (!f) continue;
        uint8_t* o = a.out + (uint64_t)(f - 1u) * a.out_stride;
        const uint32_t full4 = a.len & ~3u;
        for (uint32_t i = threadIdx.x * 4u; i < full4; i += NT * 4u) *reinterpret_cast<u32a*>(o + i) = 0u;
        for (uint32_t i = full4 + threadIdx.x; i < a.len; i += NT) o[i] = 0u;
      }
    }
  }
#if CMPI_TOOLS
  if (a.probe) {
    __syncthreads();
    CMPI_PROBE(a, 6u);
  }
#endif
}

struct GcmCombineArgs {
  const uint8_t* in;   // open: ct||tag records (for the received tag)
  uint8_t* out;        // seal: ct||tag records (tag written); open: pt records (zeroed on failure)
  uint64_t in_stride, out_stride;
  uint32_t len, nb, nrec, nseg;
  const u32x4* partial;  // nrec*nseg
  const u32x4* ekj0;     // nrec
  int32_t* status;
  const u32x4* mjp;      // device-keyed: M_j = H^{G·2^j} = H^(2^(log2 G + j)) in HBM, j < 7; or null:
  u32x4 mjv[7];          // host-keyed: M_j by value
  uint32_t prew;         // partials already weighted, E_K(J0) included (wide plan, chw): XOR only
};

// One wave per record: Y = XOR_s partial[s] · H^{(nseg-1-s)·G}; tag = Y ^ E_K(J0).
// With k = nseg-1-s = lane + 64m, lane `lane` folds its partials by Horner in M_6 = H^{64G}
// (m descending; a lane with fewer partials folds zeros) and multiplies the result by
// M^lane = product of M_j over the set bits j of lane: at most ceil(nseg/64) - 1 + 6
// multiplies in sequence, each by an LDS nibble table of one M_j (gmul_nib) — the block builds
// those tables once (one row per thread, nib_row_to_lds) for every record it handles.
// (Replaced a bit-serial 128-step generic multiply per partial: ~4 us each in sequence.)
constexpr uint32_t kCombineThreads = 256u;
constexpr size_t kCombineLds = 7u * 8192u;
template <bool DECRYPT>
__global__ __launch_bounds__(256) void gcm_combine_kernel(GcmCombineArgs a) {
  const uint32_t nseg = a.nseg;
  const uint32_t nt = a.prew ? 0u : nseg > 64u ? 7u : nseg > 1u ? 32u - __builtin_clz(nseg - 1u) : 0u;
  const uint32_t t = threadIdx.x, lane = t & 63u;
  if (t < nt * 32u) {
    const uint32_t j = t >> 5;
    u32x4 P = a.mjv[0];
#pragma unroll
    for (uint32_t q = 1; q < 7u; ++q)
      if (q == j) P = a.mjv[q];
    if (a.mjp) P = a.mjp[j];
    nib_row_to_lds(P, t & 31u, j * 8192u);
  }
  __syncthreads();
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t mmax = (nseg + 63u) >> 6;  // Horner steps (wave-uniform)
  for (uint32_t r = blockIdx.x * wpb + (t >> 6); r < a.nrec; r += gridDim.x * wpb) {
    const u32x4* part = a.partial + (uint64_t)r * nseg;
    u32x4 y = {0u, 0u, 0u, 0u};
    if (a.prew) {
      for (uint32_t k = lane; k < nseg; k += 64u) y ^= part[k];
    } else {
      for (uint32_t m = mmax; m-- > 0u;) {
        if (m + 1u < mmax) y = gmul_nib(y, 6u * 8192u);
        const uint32_t k = lane + 64u * m;
        if (k < nseg) y ^= part[nseg - 1u - k];
      }
#pragma unroll
      for (uint32_t j = 0; j < 6u; ++j) {
        if ((1u << j) >= nseg) break;  // wave-uniform: lane < nseg needs only bits j < nt
        const u32x4 q = gmul_nib(y, j * 8192u);
        if ((lane >> j) & 1u) y = q;
      }
    }
    y = xor_all_lanes(y);
    if (a.ekj0) y ^= a.ekj0[r];  // null: E_K(J0) already inside the partials
    if (!DECRYPT) {
      if (lane == 0u) st_blk(a.out + (uint64_t)r * a.out_stride + a.len, y);
      continue;
    }
    int ok = 1;
    if (lane == 0u) {
      const u32x4 d = ld_blk(a.in + (uint64_t)r * a.in_stride + a.len) ^ y;
      ok = ((d[0] | d[1] | d[2] | d[3]) == 0u) ? 1 : 0;
      if (a.status) a.status[r] = ok;
    }
    ok = __shfl(ok, 0);
    if (!ok) {
      uint8_t* o = a.out + (uint64_t)r * a.out_stride;
      const uint32_t full = a.len & ~3u;
      for (uint32_t i = lane * 4u; i < full; i += 64u * 4u) *reinterpret_cast<u32a*>(o + i) = 0u;
      for (uint32_t i = full + lane; i < a.len; i += 64u) o[i] = 0u;
    }
  }
}

// Combine of already-weighted partials (wide plan with chunk weights: tag = E_K(J0) folded into
// chunk 0, so tag = XOR of the record's partials): one 256-thread block per record, every
// partial load in flight at once (the generic combine's lane loop paid one load latency per 64
// partials: 8 in sequence for a 1 MiB record), a wave shuffle and an LDS step reduce.
constexpr uint32_t kXorCombineThreads = 256u;
template <bool DECRYPT>
__global__ __launch_bounds__(256) void gcm_xor_combine_kernel(GcmCombineArgs a) {
  const uint32_t r = blockIdx.x, t = threadIdx.x, lane = t & 63u;
  const u32x4* part = a.partial + (uint64_t)r * a.nseg;
  // open: the received tag's load is issued with the partials' (its latency off the chain)
  u32x4 tag = {0u, 0u, 0u, 0u};
  if (DECRYPT && t == 0u) tag = ld_blk(a.in + (uint64_t)r * a.in_stride + a.len);
  u32x4 y[4] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
  uint32_t k = t;
  for (; k + 3u * 256u < a.nseg; k += 4u * 256u) {
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] ^= part[k + (uint32_t)j * 256u];
  }
  for (; k < a.nseg; k += 256u) y[0] ^= part[k];
  u32x4 v = y[0] ^ y[1] ^ y[2] ^ y[3];
  v = xor_all_lanes(v);
  if (lane == 0u) lds_st128((t >> 6) * 16u, v);
  __syncthreads();
  if (t == 0u) {
    v = lds128(0u) ^ lds128(16u) ^ lds128(32u) ^ lds128(48u);
    if (!DECRYPT) {
      st_blk(a.out + (uint64_t)r * a.out_stride + a.len, v);
    } else {
      const u32x4 d = tag ^ v;
      const uint32_t ok = ((d[0] | d[1] | d[2] | d[3]) == 0u) ? 1u : 0u;
      if (a.status) a.status[r] = (int32_t)ok;
      lds_st32(64u, ok);
    }
  }
  if (!DECRYPT) return;
  __syncthreads();
  if (lds32(64u)) return;
  uint8_t* o = a.out + (uint64_t)r * a.out_stride;  // zero-fill (aead.h:276-278)
  const uint32_t full = a.len & ~3u;
  for (uint32_t i = t * 4u; i < full; i += 256u * 4u) *reinterpret_cast<u32a*>(o + i) = 0u;
  for (uint32_t i = full + t; i < a.len; i += 256u) o[i] = 0u;
}

}  // namespace dev
}  // namespace cmpi
