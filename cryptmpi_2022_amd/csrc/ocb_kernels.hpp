// ocb_kernels.hpp — AES-128-OCB3 (RFC 7253, TAGLEN 128, 96-bit nonce, no AAD) batched
// seal/open for uniform record batches (gfx950).  The reference advertises OCB
// (MV2_SECURITY_APPROACH=402, README.md:128-129) but ships none (OPENSSL_NO_OCB); this follows
// RFC 7253 and is pinned against its Appendix A and OpenSSL 3.
//
// Offsets in closed form: Offset_i = Offset_0 ^ XOR{ L_k : bit k of gray(i) }, gray(i) = i^(i>>1).
// A wavefront owns a "chunk" of S consecutive 64-block steps of one record; at step k lane l
// handles RFC block index i = 64k + l, so loads are 1 KiB coalesced, and
//   gray(64k + l) = ((k<<6) ^ (k<<5)) ^ gray(l)
// splits the offset into a lane constant D_l = XOR L over gray(l) and a wave-uniform U_k with
// U_{k+1} = U_k ^ L_5 ^ L_{6+ntz(k+1)}: two XORs of broadcast LDS values per step.
// The checksum (XOR of plaintext blocks) is reduced per wave with shuffles, written per chunk,
// and ocb_final_kernel XORs the chunk partials, handles the trailing partial block and
// computes Tag = E_K(Checksum ^ Offset ^ L_$) — open: the verdict, and it zero-fills forged
// records itself.  Offset_0 (one AES of the nonce block per record) is computed by each
// workgroup for the records of its waves, one lane per wave, at the start of every round; the
// chunk-0 wave stores it for the final kernel.  Two launches per call.
#pragma once
#include "aes_device.hpp"

namespace cmpi {
namespace dev {

struct OcbArgs {
  const uint8_t* in;
  uint8_t* out;
  const uint8_t* nonces;
  uint64_t in_stride, out_stride, nonce_stride;
  uint32_t len, m;        // bytes, full blocks per record
  uint32_t nrec, S;       // records, 64-block steps per chunk
  uint32_t nchunks;       // chunks per record
  uint32_t nitems;        // nrec * nchunks
  const uint32_t* te0;
  const uint32_t* td0;
  const uint32_t* isb;    // inverse S-box as words
  const u32x4* ltab;      // [0] = L_*, [1] = L_$, [2 + i] = L_i (i < 64)
  u32x4* off0;            // per-record Offset_0 (written by the chunk-0 wave, read by the final kernel)
  u32x4* partial;         // nitems checksum partials
  uint32_t sched;         // bit 2: rotate wave priority per step
  RoundKeys rk;           // encryption keys
  RoundKeys drk;          // equivalent-inverse-cipher keys
};

// LDS layouts.  seal / offset / final: Te row image @0 (64 KiB), L table @64K.
// open: Td row image @0 (64 KiB), inverse S-box image @64K (32 KiB), L table @96K.
constexpr uint32_t kOcbLSeal = 65536u;
constexpr uint32_t kOcbLOpen = 98304u;
constexpr uint32_t kOcbLdsSeal = kOcbLSeal + 66u * 16u;
constexpr uint32_t kOcbLdsOpen = kOcbLOpen + 66u * 16u;
// ocb_batch_kernel: the Offset_0 of each wave's record of the round, after the L table
constexpr uint32_t kOcbOffSlots = 16u * 16u;
// open only: plain Te0 (1 KiB) after the slots, for the Offset_0 encryptions (the open kernel's
// row image is the inverse cipher's)
constexpr uint32_t kOcbBatchLdsSeal = kOcbLdsSeal + kOcbOffSlots;
constexpr uint32_t kOcbBatchLdsOpen = kOcbLdsOpen + kOcbOffSlots + 1024u;
constexpr uint32_t kOcbFinalLds = kOcbLdsSeal + 16u;

// AES-128 encryption with a plain 1 KiB Te0 in LDS at tb (a few lanes: bank conflicts do not
// matter); k folded like every kernel's keys (rounds 1-9 stored as rotl16).
__device__ __forceinline__ void aes128_enc_plain(const RoundKeys& k, uint32_t tb, uint32_t& s0, uint32_t& s1,
                                                 uint32_t& s2, uint32_t& s3) {
  auto T = [&](uint32_t x) { return lds32(tb + 4u * (x & 0xffu)); };
  s0 ^= k.w[0];
  s1 ^= k.w[1];
  s2 ^= k.w[2];
  s3 ^= k.w[3];
  for (int r = 1; r < 10; ++r) {
    const uint32_t t0 = T(s0) ^ rotl8(T(s1 >> 8)) ^ rotl16(T(s2 >> 16)) ^ rotl8(rotl16(T(s3 >> 24))) ^ srot16(k.w[4 * r]);
    const uint32_t t1 = T(s1) ^ rotl8(T(s2 >> 8)) ^ rotl16(T(s3 >> 16)) ^ rotl8(rotl16(T(s0 >> 24))) ^ srot16(k.w[4 * r + 1]);
    const uint32_t t2 = T(s2) ^ rotl8(T(s3 >> 8)) ^ rotl16(T(s0 >> 16)) ^ rotl8(rotl16(T(s1 >> 24))) ^ srot16(k.w[4 * r + 2]);
    const uint32_t t3 = T(s3) ^ rotl8(T(s0 >> 8)) ^ rotl16(T(s1 >> 16)) ^ rotl8(rotl16(T(s2 >> 24))) ^ srot16(k.w[4 * r + 3]);
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  auto S = [&](uint32_t x) { return (T(x) >> 8) & 0xffu; };  // S[x] = byte 1 of Te0[x]
  const uint32_t t0 = S(s0) | (S(s1 >> 8) << 8) | (S(s2 >> 16) << 16) | (S(s3 >> 24) << 24);
  const uint32_t t1 = S(s1) | (S(s2 >> 8) << 8) | (S(s3 >> 16) << 16) | (S(s0 >> 24) << 24);
  const uint32_t t2 = S(s2) | (S(s3 >> 8) << 8) | (S(s0 >> 16) << 16) | (S(s1 >> 24) << 24);
  const uint32_t t3 = S(s3) | (S(s0 >> 8) << 8) | (S(s1 >> 16) << 16) | (S(s2 >> 24) << 24);
  s0 = t0 ^ k.w[40];
  s1 = t1 ^ k.w[41];
  s2 = t2 ^ k.w[42];
  s3 = t3 ^ k.w[43];
}

__device__ __forceinline__ u32x4 ocb_l(uint32_t base, uint32_t idx) { return lds128(base + idx * 16u); }

// Offset_0 from the 96-bit nonce (RFC 7253 §4.2): Nonce block = 0^31 || 1 || N.  Ktop by the
// row image (lb) or, PLAIN, by the plain Te0 at tb.
template <bool PLAIN = false>
__device__ __forceinline__ u32x4 ocb_offset0(const RoundKeys& rk, const RowLanes& lb, uint32_t n0, uint32_t n1,
                                             uint32_t n2, uint32_t tb = 0u) {
  const uint32_t bottom = (n2 >> 24) & 0x3fu;
  uint32_t s0 = 0x01000000u, s1 = n0, s2 = n1, s3 = n2 & 0xc0ffffffu;
  if (PLAIN) aes128_enc_plain(rk, tb, s0, s1, s2, s3);  // Ktop
  else aes128_enc(rk, lb, s0, s1, s2, s3);
  const uint64_t k0 = ((uint64_t)__builtin_bswap32(s0) << 32) | __builtin_bswap32(s1);
  const uint64_t k1 = ((uint64_t)__builtin_bswap32(s2) << 32) | __builtin_bswap32(s3);
  const uint64_t k2 = k0 ^ ((k0 << 8) | (k1 >> 56));  // Stretch bits 128..191
  uint64_t o0 = k0, o1 = k1;
  if (bottom) {
    o0 = (k0 << bottom) | (k1 >> (64u - bottom));
    o1 = (k1 << bottom) | (k2 >> (64u - bottom));
  }
  return u32x4{__builtin_bswap32((uint32_t)(o0 >> 32)), __builtin_bswap32((uint32_t)o0),
               __builtin_bswap32((uint32_t)(o1 >> 32)), __builtin_bswap32((uint32_t)o1)};
}

__device__ __forceinline__ u32x4 ocb_lsum(uint32_t base, uint64_t bits) {  // XOR of L_k over set bits
  u32x4 r = {0u, 0u, 0u, 0u};
  while (bits) {
    const uint32_t k = (uint32_t)__builtin_ctzll(bits);
    r ^= ocb_l(base, 2u + k);
    bits &= bits - 1u;
  }
  return r;
}

// seal: 65 KiB LDS -> two 1024-thread blocks per CU if VGPRs <= 64 (8 waves per SIMD)
template <bool DECRYPT>
__global__ __launch_bounds__(1024, DECRYPT ? 4 : 8) void ocb_batch_kernel(OcbArgs a) {
  constexpr uint32_t LB = DECRYPT ? kOcbLOpen : kOcbLSeal;
  if (DECRYPT) {
    stage_rows(a.td0, 0u);
    stage_rep32(a.isb, 65536u);
    for (uint32_t x = threadIdx.x; x < 256u; x += blockDim.x) lds_st32(kOcbLdsOpen + kOcbOffSlots + 4u * x, a.te0[x]);
  } else {
    stage_rows(a.te0, 0u);
  }
  stage_copy(a.ltab, LB, 66u);
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t OS = LB + 66u * 16u;  // Offset_0 slots
  const RowLanes rl = row_lanes(0u);
  const RoundKeys& ek = DECRYPT ? a.drk : a.rk;  // folded by the host
  const uint32_t lbs = 65536u | ((lane & 31u) << 2);
  const uint32_t waves_per_block = blockDim.x >> 6;
  const uint32_t total_waves = gridDim.x * waves_per_block;
  const uint32_t ksteps = a.m / 64u + 1u;  // steps covering i in [0, m]
  const u32x4 L5 = ocb_l(LB, 2u + 5u);
  const uint32_t gl = lane ^ (lane >> 1);
  u32x4 Dl = {0u, 0u, 0u, 0u};
  for (uint32_t b = 0; b < 6u; ++b)
    if (gl & (1u << b)) Dl ^= ocb_l(LB, 2u + b);

  for (uint32_t base = blockIdx.x * waves_per_block; base < a.nitems; base += total_waves) {  // workgroup-uniform
    // Offset_0 of the round's records: lane w of wave 0 computes it for wave w (RFC 7253 §4.2)
    if (threadIdx.x < waves_per_block) {
      const uint32_t it = base + threadIdx.x;
      u32x4 o = {0u, 0u, 0u, 0u};
      if (it < a.nitems) {
        const uint32_t rr = it / a.nchunks;
        const u32a* np = reinterpret_cast<const u32a*>(a.nonces + (uint64_t)rr * a.nonce_stride);
        o = DECRYPT ? ocb_offset0<true>(a.rk, rl, np[0], np[1], np[2], kOcbLdsOpen + kOcbOffSlots)
                    : ocb_offset0(a.rk, rl, np[0], np[1], np[2]);
        if (it - rr * a.nchunks == 0u) a.off0[rr] = o;  // for ocb_final_kernel
      }
      lds_st128(OS + 16u * threadIdx.x, o);
    }
    __syncthreads();
    const uint32_t item = base + wv;
    if (item >= a.nitems) {  // this wave idles the round; the workgroup stays together for the barriers
      __syncthreads();
      continue;
    }
    const uint32_t r = item / a.nchunks;
    const uint32_t c = item - r * a.nchunks;
    const uint32_t k0 = c * a.S;
    const uint32_t k1 = min(k0 + a.S, ksteps);
    const uint8_t* in_rec = a.in + (uint64_t)r * a.in_stride;
    uint8_t* out_rec = a.out + (uint64_t)r * a.out_stride;
    const u32x4 B = lds128(OS + 16u * wv) ^ Dl;
    u32x4 U = ocb_lsum(LB, ((uint64_t)k0 << 6) ^ ((uint64_t)k0 << 5));
    u32x4 csum = {0u, 0u, 0u, 0u};
    // The next step's block is loaded before this step's AES (loads and stores share vmcnt);
    // unconditional and clamped to block 1 (m == 0: the L table), so no branch.
    const uint8_t* ld_base = a.m ? in_rec : reinterpret_cast<const uint8_t*>(a.ltab);
    auto ld = [&](uint32_t k) -> u32x4 {
      const uint32_t i = 64u * k + lane;
      return *reinterpret_cast<const u32x4a*>(ld_base + 16ull * ((i >= 1u && i <= a.m) ? i - 1u : 0u));
    };
    u32x4 vcur = ld(k0);
    for (uint32_t k = k0; k < k1; ++k) {
      if (a.sched & 4u) rotate_prio(k);
      const uint32_t i = 64u * k + lane;  // RFC block index (1-based)
      const u32x4 vnext = ld(k + 1u);
      const u32x4 off = B ^ U;
      if (i >= 1u && i <= a.m) {
        const uint64_t boff = 16ull * (i - 1u);
        const u32x4 v = vcur;
        u32x4 x = v ^ off;
        uint32_t s0 = x[0], s1 = x[1], s2 = x[2], s3 = x[3];
        if (DECRYPT) aes128_dec(ek, rl, lbs, s0, s1, s2, s3);
        else aes128_enc(ek, rl, s0, s1, s2, s3);
        const u32x4 y = u32x4{s0, s1, s2, s3} ^ off;
        *reinterpret_cast<u32x4a*>(out_rec + boff) = y;
        csum ^= DECRYPT ? y : v;
      }
      U ^= L5 ^ ocb_l(LB, 2u + 6u + (uint32_t)__builtin_ctz(k + 1u));
      vcur = vnext;
    }
    csum = xor_all_lanes(csum);
    if (lane == 0) a.partial[item] = csum;
    __syncthreads();  // the Offset_0 slots are rewritten by the next round
  }
}

struct OcbFinalArgs {
  const uint8_t* in;
  uint8_t* out;
  const uint8_t* nonces;
  uint64_t in_stride, out_stride, nonce_stride;
  uint32_t len, m, nrec, nchunks;
  const uint32_t* te0;
  const u32x4* ltab;
  const u32x4* partial;
  const u32x4* off0;
  int32_t* status;   // open: per-record result (internal scratch if the caller passed none)
  RoundKeys rk;
};

template <bool DECRYPT>
__device__ __forceinline__ void ocb_final_record(const OcbFinalArgs& a, uint32_t r) {
  if (r >= a.nrec) return;
  const RowLanes lb = row_lanes(0u);
  const RoundKeys& rk = a.rk;  // folded by the host
  const uint8_t* in_rec = a.in + (uint64_t)r * a.in_stride;
  uint8_t* out_rec = a.out + (uint64_t)r * a.out_stride;
  u32x4 csum = {0u, 0u, 0u, 0u};
  for (uint32_t c = 0; c < a.nchunks; ++c) csum ^= a.partial[(uint64_t)r * a.nchunks + c];
  u32x4 off = a.off0[r] ^ ocb_lsum(kOcbLSeal, (uint64_t)a.m ^ ((uint64_t)a.m >> 1));  // Offset_m
  const uint32_t rem = a.len - 16u * a.m;
  if (rem) {
    off ^= ocb_l(kOcbLSeal, 0u);  // Offset_* = Offset_m ^ L_*
    uint32_t p0 = off[0], p1 = off[1], p2 = off[2], p3 = off[3];
    aes128_enc(rk, lb, p0, p1, p2, p3);  // Pad
    const u32x4 pad = {p0, p1, p2, p3};
    const u32x4 v = load_partial(in_rec + 16u * a.m, rem);
    const u32x4 o = mask_bytes(v ^ pad, rem);
    store_partial(out_rec + 16u * a.m, o, rem);
    u32x4 pst = DECRYPT ? o : v;  // P_* || 1 || 0*
    pst[rem >> 2] |= 0x80u << (8u * (rem & 3u));
    csum ^= pst;
  }
  u32x4 t = csum ^ off ^ ocb_l(kOcbLSeal, 1u);
  uint32_t t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3];
  aes128_enc(rk, lb, t0, t1, t2, t3);
  const u32x4 tag = {t0, t1, t2, t3};
  if (!DECRYPT) {
    uint8_t* tp = out_rec + a.len;
    *reinterpret_cast<u32x4a*>(tp) = tag;
  } else {
    const uint8_t* tp = in_rec + a.len;
    const u32x4 rt = *reinterpret_cast<const u32x4a*>(tp);
    const u32x4 d = rt ^ tag;
    const bool ok = (d[0] | d[1] | d[2] | d[3]) == 0u;
    a.status[r] = ok ? 1 : 0;
    if (!ok) lds_st32(kOcbLdsSeal, 1u);
  }
}

// One thread per record: checksum reduction, trailing partial block, tag.  Open: the verdict;
// then the block zero-fills its forged records (aead.h:276-278) — their plaintext was stored by
// the previous launch, so no other XCD's L2 can write it back over the zeros.
template <bool DECRYPT>
__global__ __launch_bounds__(256) void ocb_final_kernel(OcbFinalArgs a) {
  stage_rows(a.te0, 0u);
  stage_copy(a.ltab, kOcbLSeal, 66u);
  if (DECRYPT && threadIdx.x == 0u) lds_st32(kOcbLdsSeal, 0u);  // failed records of this block
  __syncthreads();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  ocb_final_record<DECRYPT>(a, r);
  if constexpr (DECRYPT) {
    __syncthreads();
    if (!lds32(kOcbLdsSeal)) return;  // block-uniform
    const uint32_t r1 = min(blockIdx.x * blockDim.x + blockDim.x, a.nrec);
    for (uint32_t q = blockIdx.x * blockDim.x; q < r1; ++q) {
      if (a.status[q] != 0) continue;  // block-uniform
      uint8_t* o = a.out + (uint64_t)q * a.out_stride;
      const uint32_t full = a.len & ~3u;
      for (uint32_t i = threadIdx.x * 4u; i < full; i += blockDim.x * 4u) *reinterpret_cast<u32a*>(o + i) = 0u;
      for (uint32_t i = full + threadIdx.x; i < a.len; i += blockDim.x) o[i] = 0u;
    }
  }
}

}  // namespace dev
}  // namespace cmpi
