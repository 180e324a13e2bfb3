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
  uint32_t sched;      // bit 0: rotate wave priority per slot pair (rotate_prio)
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
  uint32_t nmode, nctr0, nflag, nflag2, nflag2_from;
  uint32_t nfix[3];
  // wide decomposition (gcm_wide_kernel): S steps per chunk, nch chunks per record, and the
  // nibble tables of H^(2^b), b = 0..6 (lane weights)
  const u32x4* wtab;
  uint32_t S, nch;
  // host-keyed contexts (FLOW wide kernel): chunk weights chw[4i + j] = H^(49 - 16j + (nch-1-i)·64S)
  // for the four quarter-wave sums of chunk i (chunk 0 adds E_K(J0): the combine only XORs)
  const u32x4* chw;
  uint64_t* probe;  // diagnostics (cmpi_debug_set_wide_probe): per-WG phase timestamps, or null
  // FLOW kernel, fused combine: per-record arrival counters (context memory, zero between
  // launches) and, for open, the received tags / status; null = partials for gcm_combine_kernel
  uint32_t* wcnt;
  // FLOW kernel: the whole batch is one workgroup's units (every record's chunks together): the
  // workgroup's LDS aggregation finishes the tags, no accumulators, no second launch
  uint32_t one_wg;
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
  } else if (a.nmode == 3u) {
    n0 = a.nfix[0];
    n1 = a.nfix[1];
    n2 = a.nfix[2];
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
constexpr uint32_t kGcmRows = 65536u;
constexpr uint32_t kGcmNib = 131072u;
__host__ __device__ constexpr uint32_t gcm_prog_off(int L) { return kGcmNib + (uint32_t)(L - 1) * 8192u; }
__host__ __device__ constexpr uint32_t gcm_lds_bytes(int L) { return gcm_prog_off(L) + 16u; }

// ABL (timing ablation, wrong results): bit 0 = GHASH multiply skipped, bit 1 = AES skipped
// (keystream = counter block), bit 2 = record data addressed as one coalesced stream per wave
// (same bytes moved, dense layouts only).
template <int L, bool DECRYPT, int ABL = 0, int PF = 2, int MEM = 0>
__global__ __launch_bounds__(1024) void gcm_batch_kernel(GcmArgs a) {
  const bool prb = a.probe && threadIdx.x == 0u;  // diagnostics: workgroup start / staged / end
  if (prb) a.probe[blockIdx.x * 8u + 0u] = wall_clock64();
  stage_copy(a.htab, 0u, 4096u);
  stage_rows(a.te0, kGcmRows);
  if (L > 1) stage_copy(a.ntab, kGcmNib, (uint32_t)(L - 1) * 512u);
  if (threadIdx.x == 0u) lds_st32(gcm_prog_off(L), 0u);
  __syncthreads();
  if (prb) a.probe[blockIdx.x * 8u + 1u] = wall_clock64();
  if (ABL & 8) {  // prologue only (table staging cost)
    if (threadIdx.x == 0 && a.nrec == 0xFFFFFFFFu) a.out[0] = (uint8_t)lds32(0u);
    return;
  }

  const RoundKeys rk = load_round_keys(a.rk, a.rkp);  // folded (host / keysetup kernel)
  const uint32_t lane = threadIdx.x & 63u;
  const RowLanes rl = row_lanes(kGcmRows);
  const GhashLane gl = ghash_lane();
  const uint32_t q = threadIdx.x & (uint32_t)(L - 1);
  const uint32_t nb = a.nb;
  const uint32_t rem = a.len - 16u * (nb ? nb - 1u : 0u);  // bytes in the last data block (1..16)
  // length block [len(A)]_64 || [len(C)]_64 in memory order
  const uint64_t cbits = (uint64_t)a.len * 8u;
  const u32x4 lenblk = {0u, 0u, __builtin_bswap32((uint32_t)(cbits >> 32)), __builtin_bswap32((uint32_t)cbits)};

  const uint32_t groups_per_iter = (gridDim.x * blockDim.x) / (uint32_t)L;
  uint32_t done = 0;  // slots this wave has started (progress_prio)
  for (uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) / (uint32_t)L; g < a.ngroups; g += groups_per_iter) {
    const uint32_t r = (a.nseg == 1) ? g : g / a.nseg;
    const uint32_t s = g - r * a.nseg;
    const uint32_t x0 = (s == 0) ? 0u : a.r0 + (s - 1u) * a.G;
    const uint32_t x1 = a.r0 + s * a.G;
    const uint32_t nxs = x1 - x0;                   // X-blocks in this segment
    const uint32_t nslots = nxs + (s == 0 ? 1u : 0u);  // + the J0 slot
    const uint8_t* in_rec = a.in + (uint64_t)r * a.in_stride;
    uint8_t* out_rec = a.out + (uint64_t)r * a.out_stride;
    uint32_t n0, n1, n2;
    gcm_nonce(a, r, !DECRYPT && s == 0u && q == 0u, n0, n1, n2);

    u32x4 acc = {0u, 0u, 0u, 0u};
    u32x4 ekj0 = {0u, 0u, 0u, 0u};
    // Output-aligned windows (a.sched & 8192): at loop step i the group's L lanes own slots
    // [L*i - phi, L*i - phi + L - 1], phi putting every window's 16L output bytes on a 16L-byte
    // boundary (dense ct||tag records are n+16 apart: without it each step's stores straddle two
    // 64-B sectors, written back twice).  Lane q then owns the slots u = qs (mod L).  Seal of a
    // one-segment record with a whole last block also holds back the data blocks of the window
    // that holds the tag and stores them with the tag in one instruction.
    const bool aligned = (a.sched & 8192u) != 0u;
    const uint32_t phi = aligned ? ((uint32_t)(reinterpret_cast<uintptr_t>(out_rec) >> 4) + x0) & (uint32_t)(L - 1) : 0u;
    const uint32_t qs = (q + (uint32_t)L - phi) & (uint32_t)(L - 1);
    const bool defer = !DECRYPT && aligned && L > 1 && a.nseg == 1 && rem == 16u && nb > 0u;
    const uint32_t tslot = nxs - 1u;  // the length block's slot: the tag's position
    const uint32_t wlast = ((tslot + phi) & ~(uint32_t)(L - 1)) - phi;  // first slot of its window (>= 0 or wraps)
    u32x4 pend = {0u, 0u, 0u, 0u};
    uint8_t* pend_at = nullptr;
    // Input blocks are software-prefetched two slots ahead: loads and stores share vmcnt, so a
    // load consumed right after issue would also wait for the previous slot's store to retire.
    auto full_blk = [&](uint32_t u) { return u < nxs && x0 + u < nb && (x0 + u + 1u < nb || rem == 16u); };
    const uint64_t wave_gid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t ablk_total = (uint64_t)a.nrec * nb;
    auto abl_off = [&](uint32_t u) -> uint64_t {  // ABL & 4: coalesced stand-in for block (r, x0+u)
      const uint64_t p = (wave_gid * ((nslots + L - 1) / L) + u / (uint32_t)L) * 64u + lane;
      return 16u * (p % ablk_total);
    };
    // Unconditional load of slot u's block, clamped to a block of this record when slot u has
    // no full input block (the value is then ignored): no exec-mask branch, no zero-init.
    // (Records without a full block may have no input at all: read the Te0 table instead.)
    const bool any_full = nb > 1u || (nb == 1u && rem == 16u);
    const uint8_t* pf_base = any_full ? in_rec : reinterpret_cast<const uint8_t*>(a.te0);
    auto prefetch = [&](uint32_t u) -> u32x4 {
      if (ABL & 4) return full_blk(u) ? ld_blk(a.in + abl_off(u)) : u32x4{0u, 0u, 0u, 0u};
      const uint32_t j = full_blk(u) ? x0 + u : 0u;
      return ld_rec<MEM>(pf_base + 16u * j);
    };
    // slot u with keystream ks and its prefetched input block v
    auto consume = [&](uint32_t u, u32x4 ks, u32x4 v) {
      if (u >= nxs) {  // J0 slot
        ekj0 = ks;
        return;
      }
      const uint32_t j = x0 + u;
      u32x4 x;
      if (j < nb) {
        uint8_t* op = (ABL & 4) ? a.out + abl_off(u) : out_rec + 16u * j;
        if (full_blk(u)) {
          const u32x4 o = v ^ ks;
          if (defer && u + phi >= wlast + phi && u < tslot) {  // held for the tag's store
            pend = o;
            pend_at = op;
          } else {
            st_rec<MEM>(op, o);
          }
          x = DECRYPT ? v : o;
        } else {
          const u32x4 p = load_partial(in_rec + 16u * j, rem);
          const u32x4 o = mask_bytes(p ^ ks, rem);
          store_partial(op, o, rem);
          x = DECRYPT ? p : o;
        }
      } else {
        x = lenblk;
      }
      if (ABL & 1) acc ^= x;
      else acc = gmul_byte(acc, gl) ^ x;
    };

    // counter blocks of a record share the nonce; windows of 256 counters share bytes 0..14
    CtrCache cc;
    uint32_t cc_win = 0xffffffffu;
    auto keystream = [&](uint32_t u) -> u32x4 {
      const uint32_t ctr = (u >= nxs) ? 1u : 2u + x0 + u;  // J0 = nonce || 1, block j = nonce || 2 + j
      const uint32_t w3 = __builtin_bswap32(ctr);
      if (!(ABL & 2) && (ctr >> 8) != cc_win) {
        ctr_cache_fill(rk, rl, n0, n1, n2, w3, cc);
        cc_win = ctr >> 8;
      }
      uint32_t s0 = n0, s1 = n1, s2 = n2, s3 = w3;
      if (!(ABL & 2)) aes128_enc_ctr(rk, rl, cc, w3, s0, s1, s2, s3);
      return u32x4{s0, s1, s2, s3};
    };
    // PF input buffers: slot u's block is reloaded with slot u+PF*L's as soon as u is consumed,
    // so each load has PF-1 slots of AES in front of its use and no register copies.
    const int32_t u0 = (int32_t)q - (int32_t)phi;  // negative: the lane sits out step 0
    u32x4 v[PF];
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      const int32_t uu = u0 + d * L;
      v[d] = prefetch(uu < 0 ? 0u : (uint32_t)uu);
    }
    uint32_t it = 0;
    const uint32_t prio_mode = a.sched & (1u | 4096u | 16384u);
    for (int32_t u = u0; u < (int32_t)nslots; u += PF * L) {
      if (prio_mode == 1u) rotate_prio(it++);
#pragma unroll
      for (int d = 0; d < PF; ++d) {
        const int32_t uu = u + d * L;
        if (prio_mode & 16384u) progress_prio(gcm_prog_off(L), ++done);  // behind the workgroup -> first
        else if (prio_mode & 4096u) rotate_prio(it++);  // per slot: finer interleaving of equal-work waves
        if (uu >= 0 && uu < (int32_t)nslots) consume((uint32_t)uu, keystream((uint32_t)uu), v[d]);
        v[d] = prefetch((uint32_t)(uu + PF * L));
      }
    }

    // ---- weight the lane's Horner sum by H^w, w = nxs - (lane's last X slot)
    u32x4 f;
    if (L == 1) {
      f = gmul_byte(acc, gl);  // L = 1: byte table holds H, w = 1
    } else {
      f = u32x4{0u, 0u, 0u, 0u};
      if (qs < nxs) {
        const uint32_t ulast = qs + (uint32_t)L * ((nxs - 1u - qs) / (uint32_t)L);
        const uint32_t w = nxs - ulast;  // 1..L: H^L is the Horner byte table, H^1..H^(L-1) nibble tables
        if (w == (uint32_t)L) f = gmul_byte(acc, gl);
        else f = gmul_nib(acc, kGcmNib + (w - 1u) * 8192u);
      }
    }
    if (a.nseg == 1) f ^= ekj0;
#pragma unroll
    for (int m = 1; m < L; m <<= 1) f ^= shfl_xor4(f, m);

    if (a.nseg > 1) {
      if (q == 0) a.partial[g] = f;
      if (s == 0 && (nxs % (uint32_t)L) == qs) a.ekj0[r] = ekj0;  // lane that owned slot nxs
      continue;
    }
    // single-segment record: finish the tag here
    if (!DECRYPT) {
      if (defer) {  // the tag's window in one store instruction: held data blocks + the tag
        uint8_t* at = pend_at;
        u32x4 val = pend;
        if (qs == (tslot & (uint32_t)(L - 1))) {
          at = out_rec + a.len;
          val = f;
        }
        if (at) st_blk(at, val);
      } else if (q == 0) {
        uint8_t* tp = out_rec + a.len;
        st_blk(tp, f);
      }
    } else {
      int ok = 1;
      if (q == 0) {
        const uint8_t* tp = in_rec + a.len;
        const u32x4 t = ld_blk(tp);
        const u32x4 d = t ^ f;
        ok = ((d[0] | d[1] | d[2] | d[3]) == 0u) ? 1 : 0;
        if (a.status) a.status[r] = ok;
      }
      if (L > 1) ok = __shfl(ok, (int)(lane & ~(uint32_t)(L - 1)));
      if (!ok) {  // zero-fill this record's plaintext (aead.h:276-278)
        for (uint32_t v = q; v < nxs; v += (uint32_t)L) {
          const uint32_t j = x0 + v;
          if (j >= nb) continue;
          uint8_t* op = out_rec + 16u * j;
          if (j + 1u < nb || rem == 16u) st_blk(op, u32x4{0u, 0u, 0u, 0u});
          else store_partial(op, u32x4{0u, 0u, 0u, 0u}, rem);
        }
      }
    }
  }
  if (a.probe) {
    // per-wave end times (lane 0 of each wave): slot 2 + wave index, up to 6 waves sampled
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0u && w < 6u) a.probe[blockIdx.x * 8u + 2u + w] = wall_clock64();
  }
}

// Lane-group kernel, round-2 form (the default lane plan): the same decomposition and LDS
// layout as gcm_batch_kernel, but a segment's slots are split into
//   * the FULL data blocks [0, nfull): a branch-free main loop — keystream, XOR with the block
//     prefetched PF slots ahead, 16-B store, Horner step — with no partial-block path, no J0 or
//     length-block case and no held-back stores inside, so the waitcnt pass sees one load, one
//     store and LDS traffic per slot and waits only for the load a slot consumes (the first form
//     also waited, through its conditional store / partial-block paths, for the load issued one
//     slot earlier and for the previous store, and carried ~70 SGPR-spill lane moves and ~90
//     register copies per two slots);
//   * the <= 3 special slots at the segment's end (a partial last block, the length block, the
//     E_K(J0) slot of segment 0): a tail step, AES only where one is needed.
// Every segment's special slots are its last ones, so Horner order is unchanged.
// ABL (timing ablation, wrong results): bit 0 = main-loop record loads/stores skipped (the
// keystream is folded into the Horner input instead), bit 1 = AES skipped (keystream = counter),
// bit 2 = main-loop GHASH multiply skipped (the Horner step is an XOR).
// PF = 1 (one input block in flight per lane, loaded a whole slot ahead) is the default: with PF = 2
// the kernel needed 128 VGPRs and spilled 19 to scratch (per-record scratch traffic measured as
// +13 MB reads / +16 MB writes per config-2 launch); at PF = 1 it has 97 VGPRs, no spills.
// AW (L = 4, one segment per record, 16-B-aligned records, nrec % 64 == 0 — the host checks):
// sector-aligned windows on both sides.  Dense ct||tag records (n + 16 apart) start at every
// 16-B phase, so with lane q owning slots q, q+4, .. each store instruction split every record's
// 64 bytes over two half-written 64-B output sectors, and the L2 wrote many of them back
// before the other half arrived (config-2 seal: 97 MB written per launch vs 68 MB algorithmic;
// the same kernel sealing into 64-B-aligned records wrote 81 MB).  With AW, store window i of a
// record covers slots 4i - phi .. 4i - phi + 3 (phi = the output's 16-B phase: whole sectors),
// load window k covers 4k - psi .. (psi = the input's phase: whole sectors), and the quad
// rotates the loaded blocks into place with DPP quad permutes (lane q <- lane (q + psi - phi) & 3
// of load window i or i + 1).  The rotation must be wave-uniform, so records are dealt to waves
// by residue mod 4 (the phases of equal-stride records repeat with period 4): wave w of a
// 64-record block takes records base + 4k + w.
template <int M>
__device__ __forceinline__ uint32_t qrot(uint32_t x) {  // lane q <- lane (q + M) & 3 of its quad
  constexpr int pat = (M & 3) | (((1 + M) & 3) << 2) | (((2 + M) & 3) << 4) | (((3 + M) & 3) << 6);
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, pat, 0xF, 0xF, false);
}
template <int M>
__device__ __forceinline__ u32x4 qsel(u32x4 x, u32x4 y, bool hi) {
  u32x4 r;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint32_t a = M ? qrot<M>(x[c]) : x[c], b = M ? qrot<M>(y[c]) : y[c];
    r[c] = hi ? b : a;
  }
  return r;
}

template <int L, bool DECRYPT, int PF = 1, int ABL = 0, bool AW = false>
__global__ __launch_bounds__(1024) void gcm_lane_kernel(GcmArgs a) {
  const bool prb = a.probe && threadIdx.x == 0u;
  if (prb) a.probe[blockIdx.x * 8u + 0u] = wall_clock64();
  stage_copy(a.htab, 0u, 4096u);
  stage_rows(a.te0, kGcmRows);
  if (L > 1) stage_copy(a.ntab, kGcmNib, (uint32_t)(L - 1) * 512u);
  if (threadIdx.x == 0u) lds_st32(gcm_prog_off(L), 0u);
  __syncthreads();
  if (prb) a.probe[blockIdx.x * 8u + 1u] = wall_clock64();

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
  const bool pprio = (a.sched & 16384u) != 0u;
  const bool rprio = !pprio && (a.sched & 1u) != 0u;

  uint32_t done = 0;  // slots this wave has started (progress_prio)
  const uint32_t groups_per_iter = (gridDim.x * blockDim.x) / (uint32_t)L;
  for (uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) / (uint32_t)L; g < a.ngroups; g += groups_per_iter) {
    // AW: records dealt to waves by residue mod 4 (one segment per record)
    const uint32_t r = AW ? ((g & ~63u) | ((g & 15u) << 2) | ((g >> 4) & 3u)) : (a.nseg == 1) ? g : g / a.nseg;
    const uint32_t s = AW ? 0u : g - r * a.nseg;
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
      if (!(ABL & 2)) aes128_enc_ctr(rk, rl, cc, w3, s0, s1, s2, s3);
      return u32x4{s0, s1, s2, s3};
    };
    u32x4 acc = {0u, 0u, 0u, 0u};
    u32x4 ekj0 = {0u, 0u, 0u, 0u};

    // ---- full data blocks: slot u = X position x0 + u, counter 2 + x0 + u
    const uint8_t* ip = in_rec + 16u * x0;
    uint8_t* op = out_rec + 16u * x0;
    auto full = [&](uint32_t u, u32x4 v) {
      if (pprio) progress_prio(gcm_prog_off(L), ++done);
      else if (rprio) rotate_prio(done++);
      const u32x4 o = v ^ keystream(2u + x0 + u);
      if (!(ABL & 1)) st_blk(op + 16u * u, o);
      acc = (ABL & 4) ? acc ^ (DECRYPT ? v : o) : gmul_byte(acc, gl, DECRYPT ? v : o);
    };
    uint32_t u = q;
    uint32_t qs = q;  // the lane's slot residue: it owns the slots u = qs (mod L)
    if constexpr (AW) {
      const bool ph = !(a.sched & 32768u);  // A/B: bit 15 keeps the record mapping, drops the phases
      const uint32_t phi = ph ? (uint32_t)(reinterpret_cast<uintptr_t>(out_rec) >> 4) & 3u : 0u;  // wave-uniform
      const uint32_t psi = ph ? (uint32_t)(reinterpret_cast<uintptr_t>(in_rec) >> 4) & 3u : 0u;
      qs = (q - phi) & 3u;
      // slot 4i - phi + q sits in load window i + e, lane (q + psi - phi) & 3, e = floor((q + psi - phi) / 4)
      const int32_t emin = psi >= phi ? 0 : -1;
      const bool hi = (((int32_t)q + (int32_t)psi - (int32_t)phi) >> 2) != emin;  // takes window i + emin + 1
      const uint32_t m = __builtin_amdgcn_readfirstlane((psi - phi) & 3u);
      auto ldw = [&](int32_t k) -> u32x4 {  // load window k: slot 4k - psi + q, clamped to a full block
        if (ABL & 1) return u32x4{(uint32_t)k, x0, lane, 0u};
        const int32_t t = 4 * k - (int32_t)psi + (int32_t)q;
        return ld_blk(ip + 16u * ((t >= 0 && (uint32_t)t < nfull) ? (uint32_t)t : nfull - 1u));
      };
      // one copy of the window loop per rotation (the rotation is a DPP immediate)
      auto windows = [&](auto mc) {
        constexpr int M = decltype(mc)::value;
        const uint32_t nwin = (nfull + phi + 3u) >> 2;
        u32x4 X = ldw(emin), Y = ldw(emin + 1);
        for (uint32_t i = 0; i < nwin; ++i) {
          const u32x4 v = qsel<M>(X, Y, hi);
          X = Y;
          Y = ldw((int32_t)i + emin + 2);
          const int32_t us = 4 * (int32_t)i - (int32_t)phi + (int32_t)q;
          if (us >= 0 && (uint32_t)us < nfull) full((uint32_t)us, v);
        }
      };
      if (nfull > 0u) {
        switch (m) {
          case 0: windows(std::integral_constant<int, 0>{}); break;
          case 1: windows(std::integral_constant<int, 1>{}); break;
          case 2: windows(std::integral_constant<int, 2>{}); break;
          default: windows(std::integral_constant<int, 3>{}); break;
        }
      }
    } else if (nfull > 0u) {
      // PF input buffers: slot u's block is reloaded with slot u + PF*L's once u is consumed;
      // loads past the full blocks are clamped to the segment's LAST full block (value unused):
      // its line was just read, so the clamped load hits L2 (clamped to the first block it
      // re-read a line fetched ~60 us earlier — +23 MB HBM reads per config-2 launch, and the
      // extra L2 traffic evicted partially written output lines early: +17 MB writes)
      auto ld = [&](uint32_t uu) {
        if (ABL & 1) return u32x4{uu, x0, lane, 0u};
        return ld_blk(ip + 16u * (uu < nfull ? uu : nfull - 1u));
      };
      u32x4 v[PF];
#pragma unroll
      for (int d = 0; d < PF; ++d) v[d] = ld(u + (uint32_t)(d * L));
      for (; u + (uint32_t)((PF - 1) * L) < nfull; u += (uint32_t)(PF * L)) {
#pragma unroll
        for (int d = 0; d < PF; ++d) {
          const uint32_t uu = u + (uint32_t)(d * L);
          full(uu, v[d]);
          v[d] = ld(uu + (uint32_t)(PF * L));
        }
      }
#pragma unroll
      for (int d = 0; d < PF - 1; ++d) {
        const uint32_t uu = u + (uint32_t)(d * L);
        if (uu < nfull) full(uu, v[d]);
      }
    }
    // ---- special slots: partial last block, length block, J0 (the lane's slots >= nfull)
    for (uint32_t ut = nfull <= qs ? qs : qs + (uint32_t)L * ((nfull - qs + (uint32_t)L - 1u) / (uint32_t)L); ut < nslots;
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
    } else if (qs < nxs) {
      const uint32_t ulast = qs + (uint32_t)L * ((nxs - 1u - qs) / (uint32_t)L);
      const uint32_t w = nxs - ulast;  // 1..L: H^L is the Horner byte table, H^1..H^(L-1) nibble tables
      if (w == (uint32_t)L) f = gmul_byte(acc, gl);
      else f = gmul_nib(acc, kGcmNib + (w - 1u) * 8192u);
    }
    if (a.nseg == 1) f ^= ekj0;
#pragma unroll
    for (int m = 1; m < L; m <<= 1) f ^= shfl_xor4(f, m);

    if (a.nseg > 1) {
      if (q == 0) a.partial[g] = f;
      if (s == 0 && (nxs % (uint32_t)L) == qs) a.ekj0[r] = ekj0;  // lane that owned slot nxs
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
  if (a.probe) {
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0u && w < 6u) a.probe[blockIdx.x * 8u + 2u + w] = wall_clock64();
  }
}

// ---------------------------------------------------------------- wide decomposition
// Few long records (the naive Alltoall's p peer blocks of 1 MiB, alltoall.c:795-834): a record's
// X-sequence is cut from the END into chunks of C = 64*S X-blocks (chunk 0 takes the remainder:
// C <= its length < 2C, ceil(len/64) steps) and
// every (record, chunk) is ONE wavefront.  At step k lane q owns X position base + 64k + q, so
// each wave-instruction moves 1 KiB of contiguous record data, and the lane folds its blocks
// into a Horner accumulator with multiplier H^64 (byte table of H^64 in LDS).  Lane q's last
// block sits at end - 64 + q in every chunk, so its sum carries the weight H^{64-q}: applied
// as H^(2^b) for the set bits b of 64 - q (7 nibble-table multiplies, the same for every lane,
// selected per lane), then XOR-reduced over the wave into the chunk partial.  The chunk weight
// H^{(nch-1-i)·C} and E_K(J0) are applied by gcm_combine_kernel exactly as for segments.
// LDS: [0, 64K) holds the byte table of H^64 while the waves run their chunks, then the seven
// nibble tables of H^1..H^64, restaged between two workgroup barriers; AES rows at 64K.
// (Measured, 8 x 1 MiB: this replaced one generic multiply per lane, 176 -> 202 GiB/s seal;
// seven restaged conflict-free byte tables instead of the nibble tables were slower, 184.)
// FLOW (host-keyed contexts): all tables staged once — H^64 byte table [0, 64K), AES rows
// [64K, 128K), nibble tables of H, H^2, H^4, H^8 [128K, 160K) — and no workgroup barrier after
// that: a wave goes from its Horner loop straight to its weights.  The lane tree stops after
// four levels (lanes 0, 16, 32, 48 hold the sums T_q of their 16 lanes, weights H^(15-t)); the
// remaining weights H^(49-q) and the chunk weight are one wave-cooperative product per quarter
// (gmul_wave4 with the host table chw), E_K(J0) is folded into chunk 0, the combine only XORs.
template <bool DECRYPT, bool FLOW = false>
__global__ __launch_bounds__(1024) void gcm_wide_kernel(GcmArgs a) {
  const bool prb = a.probe && threadIdx.x == 0u;
  if (prb) a.probe[blockIdx.x * 8u + 0u] = wall_clock64();
  stage_rows(a.te0, kGcmRows);
  if constexpr (FLOW) {
    stage_copy(a.htab, 0u, 4096u);             // byte table of H^64
    stage_copy(a.wtab, kGcmNib, 4u * 512u);     // nibble tables of H^(2^b), b = 0..3
    __syncthreads();
  }

  const RoundKeys rk = load_round_keys(a.rk, a.rkp);  // folded (host / keysetup kernel)
  const uint32_t lane = threadIdx.x & 63u;
  const RowLanes rl = row_lanes(kGcmRows);
  const GhashLane gl = ghash_lane();
  const uint32_t nb = a.nb;
  const int32_t nx = (int32_t)nb + 1;
  const uint32_t rem = a.len - 16u * (nb ? nb - 1u : 0u);
  const uint64_t cbits = (uint64_t)a.len * 8u;
  const u32x4 lenblk = {0u, 0u, __builtin_bswap32((uint32_t)(cbits >> 32)), __builtin_bswap32((uint32_t)cbits)};
  const int32_t C = 64 * (int32_t)a.S;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t units = a.nrec * a.nch;
  const uint32_t per_round = gridDim.x * wpb;
  const uint32_t rounds = (units + per_round - 1u) / per_round;  // uniform over the grid
  const uint32_t wexp = 64u - lane;                              // lane weight H^(64 - q)

  for (uint32_t rd = 0; rd < rounds; ++rd) {
    const uint32_t u = rd * per_round + blockIdx.x * wpb + (threadIdx.x >> 6);
    const bool active = u < units;  // wave-uniform
    if constexpr (!FLOW) {
      __syncthreads();                // [0, 64K) is free: the previous round's weights are done
      stage_copy(a.htab, 0u, 4096u);  // byte table of H^64
      __syncthreads();
    }
    if (prb && rd == 0u) a.probe[blockIdx.x * 8u + 1u] = wall_clock64();
    u32x4 acc = {0u, 0u, 0u, 0u};
    u32x4 ekj = {0u, 0u, 0u, 0u};
    if (active) {
      const uint32_t r = u / a.nch;
      const uint32_t i = u - r * a.nch;
      // chunk 0 runs ceil(r0/64) steps over [0, r0) (G <= r0 < 2G); chunk i > 0 runs S steps
      const uint32_t steps = i == 0u ? (a.r0 + 63u) >> 6 : a.S;
      const int32_t base = i == 0u ? (int32_t)a.r0 - 64 * (int32_t)steps  // step 0, lane 0 (may be < 0)
                                   : nx - (int32_t)(a.nch - i) * C;
      const uint8_t* in_rec = a.in + (uint64_t)r * a.in_stride;
      uint8_t* out_rec = a.out + (uint64_t)r * a.out_stride;
      uint32_t n0, n1, n2;
      gcm_nonce(a, r, !DECRYPT && i == 0u && lane == 0u, n0, n1, n2);

      // (records of a wide batch always have full blocks: nb >= 64)
      auto full_blk = [&](int32_t p) { return p >= 0 && p < (int32_t)nb && (p + 1 < (int32_t)nb || rem == 16u); };
      auto prefetch = [&](uint32_t k) -> u32x4 {
        const int32_t p = base + 64 * (int32_t)k + (int32_t)lane;
        return ld_blk(in_rec + 16u * (uint32_t)(full_blk(p) ? p : 0));
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
      auto consume = [&](uint32_t k, u32x4 v) {
        const int32_t p = base + 64 * (int32_t)k + (int32_t)lane;
        const u32x4 ks = keystream(2u + (uint32_t)p);  // block j = nonce || 2 + j
        u32x4 x = {0u, 0u, 0u, 0u};
        if (p >= 0 && p < (int32_t)nb) {
          uint8_t* op = out_rec + 16u * (uint32_t)p;
          if (full_blk(p)) {
            const u32x4 o = v ^ ks;
            st_blk(op, o);
            x = DECRYPT ? v : o;
          } else {
            const u32x4 pp = load_partial(in_rec + 16u * (uint32_t)p, rem);
            const u32x4 o = mask_bytes(pp ^ ks, rem);
            store_partial(op, o, rem);
            x = DECRYPT ? pp : o;
          }
        } else if (p == nx - 1) {
          x = lenblk;
        }
        acc = gmul_byte(acc, gl) ^ x;
      };
      u32x4 va = prefetch(0), vb = prefetch(1);
      uint32_t it = 0;
      for (uint32_t k = 0; k < steps; k += 2u) {
        if (a.sched & 1u) rotate_prio(it++);
        consume(k, va);
        va = prefetch(k + 2u);
        if (k + 1u < steps) consume(k + 1u, vb);
        vb = prefetch(k + 3u);
      }
      if (i == 0u) {  // E_K(J0): into chunk 0's partial (FLOW), or for the combine kernel
        const u32x4 e = keystream(1u);
        if (FLOW) ekj = e;
        else if (lane == 0u) a.ekj0[r] = e;
      }
    }
    if (prb && rd == 0u) a.probe[blockIdx.x * 8u + 2u] = wall_clock64();
    if constexpr (FLOW) {
      if (active) {
#pragma unroll
        for (uint32_t b = 0; b < 4u; ++b) {  // tree levels 0..3 (as below)
          const u32x4 up = shfl_down4(acc, 1u << b);
          if ((lane & ((2u << b) - 1u)) == 0u) {
            asm volatile("" ::: "memory");
            acc = gmul_nib(acc, kGcmNib + b * 8192u) ^ up;
          }
        }
        u32x4 T[4], M[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int c = 0; c < 4; ++c) T[j][c] = (uint32_t)__builtin_amdgcn_readlane(acc[c], 16 * j);
          M[j] = a.chw[4u * (u % a.nch) + (uint32_t)j];
        }
        const u32x4 pw = gmul_wave4(T, M) ^ ekj;
        if (lane == 0u) a.partial[u] = pw;
      }
      if (prb && rd == 0u) a.probe[blockIdx.x * 8u + 5u] = wall_clock64();
      continue;
    }
    __syncthreads();  // every wave is past its Horner loop: [0, 64K) takes the weight tables
    if (prb && rd == 0u) a.probe[blockIdx.x * 8u + 3u] = wall_clock64();
    stage_copy(a.wtab, 0u, 7u * 512u);  // nibble tables of H^(2^b), b = 0..6, 8 KiB apart
    __syncthreads();
    if (prb && rd == 0u) a.probe[blockIdx.x * 8u + 4u] = wall_clock64();
    if (active && (a.sched & 8u)) {  // A/B: per-lane weights (previous scheme)
#pragma unroll
      for (uint32_t b = 0; b < 7u; ++b) {
        const u32x4 m = gmul_nib(acc, b * 8192u);
        if ((wexp >> b) & 1u) acc = m;
      }
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) acc ^= shfl_xor4(acc, m);
      if (lane == 0u) a.partial[u] = acc;
    } else if (active) {
      // binary tree over the lanes: level b folds lane q + 2^b into lane q (q = 0 mod 2^(b+1))
      // with weight H^(2^b), so lane 0 ends with XOR_q acc_q · H^(63-q); one more H gives
      // H^(64-q).  Only the folding lanes multiply: 64 lane-multiplies per wave instead of 448.
#pragma unroll
      for (uint32_t b = 0; b < 6u; ++b) {
        const u32x4 up = shfl_down4(acc, 1u << b);
        if ((lane & ((2u << b) - 1u)) == 0u) {
          asm volatile("" ::: "memory");  // keep the branch: only the folding lanes read LDS
          acc = gmul_nib(acc, b * 8192u) ^ up;
        }
      }
      if (lane == 0u) a.partial[u] = gmul_nib(acc, 0u);
    }
    if (prb && rd == 0u) a.probe[blockIdx.x * 8u + 5u] = wall_clock64();
  }
  if (a.probe) {
    __syncthreads();
    if (prb) a.probe[blockIdx.x * 8u + 6u] = wall_clock64();
  }
}

// ---------------------------------------------------------------- FLOW wide kernel
// The host-keyed wide decomposition as its own kernel (gcm_wide_kernel<.., FLOW> below is the
// round-1 form, kept for the A/B knob): NT threads per workgroup (512 or 1024), every table load
// issued before any LDS store (one global round trip for the tables).  Two forms:
//  - R4 (default): the chunk's X blocks are folded per lane by Horner in H^64 (nibble table),
//    the 64 lane accumulators by a radix-4 tree — three levels, each ONE nibble multiply per
//    active lane by a lane-chosen table (H^1..3, H^4..12, H^16..48), lanes packed low so a level
//    touches 3, 1, 1 LDS lane groups — and the chunk weight H^(1 + (nch-1-i)C) by one
//    wave-cooperative product (gmul_wave).  Tables: 10 nibble tables (80 KiB) + AES rows.
//  - !R4 (round-2 first form): Horner in H^64 by its byte table (64 KiB), a 4-level radix-2 tree,
//    four products by the host weights M_j (gmul_wave4).
// Combine fused in (a.wcnt != null): R4 XORs its workgroup's partials per record in LDS and one
// lane per record XORs them into the record's accumulator (two 8-B agent atomics), waits, and
// adds the number of chunks to the record's counter; the adder that completes the count loads
// the accumulator (8-B agent atomic loads) and writes the tag / verdict, then zeroes both for
// the next launch — MI355X_MICROARCH.md "Valid forms" ({8-B agent atomics both sides}, row 1:
// one lane per storing workgroup, the last adder told by its add's return).  !R4 publishes each
// wave's partial write-through and counts per wave (one add per chunk: contended).
constexpr uint32_t kFlowAgg = 147456u;         // R4: aggregation slots, 16 x 16 B partials + 16 x 4 B records
constexpr uint32_t kFlowLdsR4 = kFlowAgg + 512u;
constexpr uint32_t kFlowFail = kFlowAgg + 448u;  // one-workgroup open: per-slot failed record + 1
__device__ __forceinline__ uint32_t flow_tab(uint32_t f) {  // R4 nibble table f (keysetup_kernels.hpp flow_nib_exp)
  return f < 8u ? f * 8192u : 131072u + (f - 8u) * 8192u;
}

template <int NT, bool R4>
__device__ __forceinline__ void stage_flow(const GcmArgs& a) {
  constexpr int kR = 1024 / NT, kH = R4 ? 0 : 4096 / NT, kW = (R4 ? 5120 : 2048) / NT;  // loads per thread
  uint32_t rv[kR];
  u32x4 hv[kH > 0 ? kH : 1], wv[kW];
  const uint32_t t = threadIdx.x;
#pragma unroll
  for (int j = 0; j < kR; ++j) rv[j] = a.te0[(t + j * NT) >> 2];
#pragma unroll
  for (int j = 0; j < kH; ++j) hv[j] = a.htab[t + j * NT];
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
  for (int j = 0; j < kH; ++j) lds_st128((t + j * NT) * 16u, hv[j]);
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    const uint32_t e = t + j * NT;
    lds_st128(R4 ? flow_tab(e >> 9) + (e & 511u) * 16u : kGcmNib + e * 16u, wv[j]);
  }
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
  x ^= shfl_xor4(x, 16);
  x ^= shfl_xor4(x, 32);  // every lane t: A_(t & 15)
  x = shfl4(x, 4u * (lane & 3u) + ((lane >> 2) & 3u));
  if (lane < 12u) {
    uint32_t tb = flow_tab(5u - (lane >> 2));
    asm volatile("" : "+v"(tb)::"memory");
    x = gmul_nib(x, tb);
  }
  x ^= shfl_xor4(x, 4);
  x ^= shfl_xor4(x, 8);  // lanes t < 16: B_(t & 3)
  if (lane < 3u) {
    uint32_t tb = flow_tab(8u - lane);
    asm volatile("" : "+v"(tb)::"memory");
    x = gmul_nib(x, tb);
  }
  x ^= shfl_xor4(x, 1);
  x ^= shfl_xor4(x, 2);  // lane 0: V
  return x;
}

template <bool DECRYPT, int NT, bool R4>
__global__ __launch_bounds__(NT) void gcm_flow_kernel(GcmArgs a) {
  const bool prb = a.probe && threadIdx.x == 0u;
  if (prb) a.probe[blockIdx.x * 8u + 0u] = wall_clock64();
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t nb = a.nb;
  const int32_t nx = (int32_t)nb + 1;
  const uint32_t rem = a.len - 16u * (nb ? nb - 1u : 0u);
  const int32_t C = 64 * (int32_t)a.S;
  constexpr uint32_t wpb = NT / 64;
  const uint32_t units = a.nrec * a.nch;
  // unit u = (record r, chunk i): chunk 0 absorbs the remainder, the others are C X-blocks
  auto unit_base = [&](uint32_t u, uint32_t& r, uint32_t& i, uint32_t& steps) -> int32_t {
    r = u / a.nch;
    i = u - r * a.nch;
    steps = i == 0u ? (a.r0 + 63u) >> 6 : a.S;
    return i == 0u ? (int32_t)a.r0 - 64 * (int32_t)steps : nx - (int32_t)(a.nch - i) * C;
  };
  auto full_blk = [&](int32_t p) { return p >= 0 && p < (int32_t)nb && (p + 1 < (int32_t)nb || rem == 16u); };
  auto load_x = [&](const uint8_t* in_rec, int32_t base, uint32_t k) -> u32x4 {
    const int32_t p = base + 64 * (int32_t)k + (int32_t)lane;
    if (a.sched & 4096u) return u32x4{(uint32_t)p, k, lane, 0u};  // timing ablation: no loads
    return ld_blk(in_rec + 16u * (uint32_t)(full_blk(p) ? p : 0));
  };
  // the first unit's first two input rows are requested before the table staging: their HBM
  // latency overlaps it
  u32x4 va0 = {0u, 0u, 0u, 0u}, vb0 = {0u, 0u, 0u, 0u};
  {
    const uint32_t u = blockIdx.x * wpb + wv;
    if (u < units) {
      uint32_t r, i, steps;
      const int32_t base = unit_base(u, r, i, steps);
      va0 = load_x(a.in + (uint64_t)r * a.in_stride, base, 0u);
      vb0 = load_x(a.in + (uint64_t)r * a.in_stride, base, 1u);
    }
  }
  stage_flow<NT, R4>(a);
  if (prb) a.probe[blockIdx.x * 8u + 1u] = wall_clock64();
  const RoundKeys rk = a.rk;  // host-keyed: folded round keys in the arguments
  const RowLanes rl = row_lanes(kGcmRows);
  const GhashLane gl = ghash_lane();
  const uint64_t cbits = (uint64_t)a.len * 8u;
  const u32x4 lenblk = {0u, 0u, __builtin_bswap32((uint32_t)(cbits >> 32)), __builtin_bswap32((uint32_t)cbits)};
  for (uint32_t ub = blockIdx.x * wpb; ub < units; ub += gridDim.x * wpb) {  // workgroup-uniform
    const uint32_t u = ub + wv;
    u32x4 pw = {0u, 0u, 0u, 0u};
    uint32_t r = 0xffffffffu;
    if (u < units) {  // wave-uniform
      uint32_t i, steps;
      const int32_t base = unit_base(u, r, i, steps);
      const uint8_t* in_rec = a.in + (uint64_t)r * a.in_stride;
      uint8_t* out_rec = a.out + (uint64_t)r * a.out_stride;
      uint32_t n0, n1, n2;
      gcm_nonce(a, r, !DECRYPT && i == 0u && lane == 0u, n0, n1, n2);
      auto prefetch = [&](uint32_t k) -> u32x4 { return load_x(in_rec, base, k); };
      CtrCache cc;
      uint32_t cc_win = 0xffffffffu;
      auto keystream = [&](uint32_t ctr) -> u32x4 {
        const uint32_t w3 = __builtin_bswap32(ctr);
        if (a.sched & 1024u) return u32x4{w3, n0, n1, n2};  // timing ablation: no AES
        if ((ctr >> 8) != cc_win) {
          ctr_cache_fill(rk, rl, n0, n1, n2, w3, cc);
          cc_win = ctr >> 8;
        }
        uint32_t s0, s1, s2, s3;
        aes128_enc_ctr(rk, rl, cc, w3, s0, s1, s2, s3);
        return u32x4{s0, s1, s2, s3};
      };
      u32x4 acc = {0u, 0u, 0u, 0u};
      auto consume_ks = [&](uint32_t k, u32x4 v, u32x4 ks) {
        const int32_t p = base + 64 * (int32_t)k + (int32_t)lane;
        u32x4 x = {0u, 0u, 0u, 0u};
        if (p >= 0 && p < (int32_t)nb) {
          uint8_t* op = out_rec + 16u * (uint32_t)p;
          if (full_blk(p)) {
            const u32x4 o = v ^ ks;
            if (!(a.sched & 2048u)) st_blk(op, o);  // timing ablation (2048): no stores
            x = DECRYPT ? v : o;
          } else {
            const u32x4 pp = load_partial(in_rec + 16u * (uint32_t)p, rem);
            const u32x4 o = mask_bytes(pp ^ ks, rem);
            store_partial(op, o, rem);
            x = DECRYPT ? pp : o;
          }
        } else if (p == nx - 1) {
          x = lenblk;
        }
        if constexpr (R4) {
          if (k == 0u) acc = x;  // wave-uniform; acc was 0
          else acc = gmul_nib(acc, flow_tab(9u)) ^ x;
        } else {
          acc = gmul_byte(acc, gl) ^ x;
        }
      };
      auto ctr_of = [&](uint32_t k) { return 2u + (uint32_t)(base + 64 * (int32_t)k + (int32_t)lane); };
      const bool first = ub == blockIdx.x * wpb;
      u32x4 va = first ? va0 : prefetch(0), vb = first ? vb0 : prefetch(1);
      uint32_t it = 0;
      // E_K(J0), folded into chunk 0's partial (only lane 0's copy is used).  Chunk 0 holds the
      // r0 = G..2G-1 leading positions, so its first step is partial whenever 64 does not divide
      // r0 (1 MiB: 257 positions, lane 63 alone): lane 0 is idle there and encrypts J0 in that
      // step instead of the wave paying a whole AES pass for it afterwards.
      const bool j0_step0 = i == 0u && base < 0;
      u32x4 ekj = {0u, 0u, 0u, 0u};
      for (uint32_t k = 0; k < steps; k += 2u) {
        if (a.sched & 1u) rotate_prio(it++);
        const u32x4 ks = keystream(k == 0u && j0_step0 && lane == 0u ? 1u : ctr_of(k));
        if (k == 0u) ekj = ks;
        consume_ks(k, va, ks);
        va = prefetch(k + 2u);
        if (k + 1u < steps) consume_ks(k + 1u, vb, keystream(ctr_of(k + 1u)));
        vb = prefetch(k + 3u);
      }
      if (!j0_step0) ekj = i == 0u ? keystream(1u) : u32x4{0u, 0u, 0u, 0u};
      if (prb && u == blockIdx.x * wpb) a.probe[blockIdx.x * 8u + 2u] = wall_clock64();
      if constexpr (R4) {
        const u32x4 M = a.chw[4u * i + 3u];  // H^(1 + (nch-1-i)C), requested before the tree
        u32x4 V = (a.sched & 256u) ? acc : flow_tree_r4(acc, lane);
#pragma unroll
        for (int c = 0; c < 4; ++c) V[c] = (uint32_t)__builtin_amdgcn_readfirstlane(V[c]);
        pw = ((a.sched & 512u) ? V ^ M : gmul_wave(V, M)) ^ ekj;
      } else {
#pragma unroll
        for (uint32_t b = 0; b < 4u; ++b) {  // lane tree levels 0..3 (as in gcm_wide_kernel)
          const u32x4 up = shfl_down4(acc, 1u << b);
          if ((lane & ((2u << b) - 1u)) == 0u && !(a.sched & 256u)) {
            asm volatile("" ::: "memory");
            acc = gmul_nib(acc, kGcmNib + b * 8192u) ^ up;
          }
        }
        u32x4 T[4], M[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int c = 0; c < 4; ++c) T[j][c] = (uint32_t)__builtin_amdgcn_readlane(acc[c], 16 * j);
          M[j] = a.chw[4u * i + (uint32_t)j];
        }
        pw = ((a.sched & 512u) ? T[0] ^ T[1] ^ T[2] ^ T[3] ^ M[0] : gmul_wave4(T, M)) ^ ekj;
      }
      if (prb && u == blockIdx.x * wpb) a.probe[blockIdx.x * 8u + 5u] = wall_clock64();
    }
    if (!a.wcnt && !a.one_wg) {  // partials for gcm_xor_combine_kernel
      if (u < units && lane == 0u) a.partial[u] = pw;
      continue;
    }
    if constexpr (R4) {
      if (lane == 0u) {
        lds_st128(kFlowAgg + 16u * wv, pw);
        lds_st32(kFlowAgg + 256u + 4u * wv, r);
        lds_st32(kFlowFail + 4u * wv, 0u);
      }
      // one workgroup, open: this wave's plaintext stores are performed before the barrier, so
      // a zero-fill after it lands behind them in the same L2
      if (DECRYPT && a.one_wg) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const uint32_t l = threadIdx.x;
      const uint32_t rr = l < wpb ? lds32(kFlowAgg + 256u + 4u * l) : 0xffffffffu;
      if (rr != 0xffffffffu && (l == 0u || lds32(kFlowAgg + 256u + 4u * (l - 1u)) != rr)) {  // first slot of rr
        u32x4 x = {0u, 0u, 0u, 0u};
        uint32_t cnt = 0;
        for (uint32_t j = l; j < wpb && lds32(kFlowAgg + 256u + 4u * j) == rr; ++j, ++cnt) x ^= lds128(kFlowAgg + 16u * j);
        if (a.one_wg) {  // every chunk of record rr is in this workgroup: x is the tag
          if (!DECRYPT) {
            st_blk(a.out + (uint64_t)rr * a.out_stride + a.len, x);
          } else {
            const u32x4 d = ld_blk(a.in + (uint64_t)rr * a.in_stride + a.len) ^ x;
            const bool ok = (d[0] | d[1] | d[2] | d[3]) == 0u;
            a.status[rr] = ok ? 1 : 0;
            if (!ok) lds_st32(kFlowFail + 4u * l, rr + 1u);
          }
        } else {
          uint64_t* ta = reinterpret_cast<uint64_t*>(a.wcnt + 8u * rr + 4u);
          __hip_atomic_fetch_xor(ta, (uint64_t)x[0] | ((uint64_t)x[1] << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_xor(ta + 1, (uint64_t)x[2] | ((uint64_t)x[3] << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          const uint32_t old = __hip_atomic_fetch_add(a.wcnt + 8u * rr, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (old + cnt == a.nch) {  // every chunk of record rr is in the accumulator
            const uint64_t lo = __hip_atomic_load(ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t hi = __hip_atomic_load(ta + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ta, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ta + 1, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.wcnt + 8u * rr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const u32x4 y = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
            if (!DECRYPT) {
              st_blk(a.out + (uint64_t)rr * a.out_stride + a.len, y);
            } else {  // verdict only: the zero-fill of a failed record is zero_failed_kernel's
              const u32x4 d = ld_blk(a.in + (uint64_t)rr * a.in_stride + a.len) ^ y;
              a.status[rr] = ((d[0] | d[1] | d[2] | d[3]) == 0u) ? 1 : 0;
            }
          }
        }
      }
      __syncthreads();  // slots reused by the next round
      if (DECRYPT && a.one_wg) {  // zero-fill the failed records (aead.h:276-278), whole workgroup
        for (uint32_t j = 0; j < wpb; ++j) {
          const uint32_t f = lds32(kFlowFail + 4u * j);  // rr + 1 of a failed record, else 0
          if (!f) continue;
          uint8_t* o = a.out + (uint64_t)(f - 1u) * a.out_stride;
          const uint32_t full4 = a.len & ~3u;
          for (uint32_t i = threadIdx.x * 4u; i < full4; i += NT * 4u) *reinterpret_cast<u32a*>(o + i) = 0u;
          for (uint32_t i = full4 + threadIdx.x; i < a.len; i += NT) o[i] = 0u;
        }
      }
    } else {
      if (u >= units) continue;
      // publish the partial write-through, count the arrival
      uint32_t old = 0;
      if (lane == 0u) {
        uint64_t* pp = reinterpret_cast<uint64_t*>(a.partial + u);
        __hip_atomic_store(pp, (uint64_t)pw[0] | ((uint64_t)pw[1] << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pp + 1, (uint64_t)pw[2] | ((uint64_t)pw[3] << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        old = __hip_atomic_fetch_add(a.wcnt + 8u * r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      old = __shfl(old, 0);
      if (old != a.nch - 1u) continue;  // wave-uniform: not the last chunk of record r to arrive
      if (lane == 0u) __hip_atomic_store(a.wcnt + 8u * r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      u32x4 y = {0u, 0u, 0u, 0u};
      const uint64_t* rp = reinterpret_cast<const uint64_t*>(a.partial + (uint64_t)r * a.nch);
      for (uint32_t k = lane; k < a.nch; k += 64u) {
        const uint64_t lo = __hip_atomic_load(rp + 2u * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t hi = __hip_atomic_load(rp + 2u * k + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        y ^= u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
      }
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) y ^= shfl_xor4(y, m);
      if (lane == 0u) {
        uint8_t* out_rec = a.out + (uint64_t)r * a.out_stride;
        if (!DECRYPT) {
          st_blk(out_rec + a.len, y);
        } else {
          const u32x4 d = ld_blk(a.in + (uint64_t)r * a.in_stride + a.len) ^ y;
          a.status[r] = ((d[0] | d[1] | d[2] | d[3]) == 0u) ? 1 : 0;
        }
      }
    }
  }
  if (a.probe) {
    __syncthreads();
    if (prb) a.probe[blockIdx.x * 8u + 6u] = wall_clock64();
  }
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
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) y ^= shfl_xor4(y, m);
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
  u32x4 y[4] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
  uint32_t k = t;
  for (; k + 3u * 256u < a.nseg; k += 4u * 256u) {
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] ^= part[k + (uint32_t)j * 256u];
  }
  for (; k < a.nseg; k += 256u) y[0] ^= part[k];
  u32x4 v = y[0] ^ y[1] ^ y[2] ^ y[3];
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v ^= shfl_xor4(v, m);
  if (lane == 0u) lds_st128((t >> 6) * 16u, v);
  __syncthreads();
  if (t == 0u) {
    v = lds128(0u) ^ lds128(16u) ^ lds128(32u) ^ lds128(48u);
    if (!DECRYPT) {
      st_blk(a.out + (uint64_t)r * a.out_stride + a.len, v);
    } else {
      const u32x4 d = ld_blk(a.in + (uint64_t)r * a.in_stride + a.len) ^ v;
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
