// aes_device.hpp — CDNA4 (gfx950) device primitives: LDS-staged AES-128 T-table rounds and
// table-driven GF(2^128) multiplication, all in the little-endian word convention of
// aes_tables.hpp (a block = 4 LE words, word c = AES state column c, row r at bits 8r..8r+7).
//
// LDS images (byte offsets inside the kernel's dynamic LDS; dynamic LDS starts at address 0):
//  * AES "row image" (64 KiB, base a multiple of 64 KiB): row x at base + x*256 holds
//    [ Te0[x] x32 replicas | Te1[x] x32 replicas ], Te1 = rotl8(Te0).  Lane l reads replica
//    (l & 31), so in a ds_read_b32 (two 32-lane halves, bank = (addr/4) mod 32) every lane of a
//    half sits on its own bank whatever x is: conflict free.  Because rows are 256 B apart the
//    lookup address is   byte0 = (l&31)*4 (+128 for Te1), byte1 = x, byte2..3 = base >> 16
//    — ONE v_perm_b32 gathers it from the state word and a lane constant (no shift/mask pair).
//    With Te2 = rotl16(Te0), Te3 = rotl16(Te1) a column is Te0[a]^Te1[b]^rotl16(Te0[c]^Te1[d]):
//    8 VALU ops per column instead of 13.  The decryption image is the same with Td0/Td1.
//  * Inverse S-box image (32 KiB, old style): Si[x] (byte 0 of a word) at base + x*128 + (l&31)*4.
//  * GHASH byte table (multiplier P, 64 KiB at LDS 0): entry (v, p) = (byte p := v)·P at
//    v*256 + p*16.  Lane l visits the 16 byte positions in the rotated order p = (t + l) mod 16,
//    so at every step the 16 lanes of a ds_read_b128 group (whose l mod 16 are all distinct)
//    hit 16 different 16-byte slots: conflict free.  The address is again one v_perm_b32
//    (byte0 = p*16 from a packed lane constant, byte1 = v).
//  * GHASH nibble tables (8 KiB each, rarely used): entry (2p+h, v) at base + p*512 + h*256 + v*16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmpi {
namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Byte-aligned 16-byte / 4-byte views of record data: records may start at any byte offset
// (the nonce(12)||ct||tag wire layout with odd n, the 602 5-byte segment prefix).  On gfx950
// under amdhsa the backend runs in unaligned-access mode and still emits one
// global_load/store_dwordx4 (resp. _dword) for these.
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32a __attribute__((aligned(1)));

// LDS accesses by raw byte offset: all kernels here use only dynamic LDS (no static
// __shared__), so an offset IS the LDS address and ds_read uses it directly.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
__device__ __forceinline__ uint32_t lds32(uint32_t off) { return *(const lds_u32*)(size_t)off; }
__device__ __forceinline__ u32x4 lds128(uint32_t off) { return *(const lds_u32x4*)(size_t)off; }
__device__ __forceinline__ void lds_st32(uint32_t off, uint32_t v) { *(lds_u32*)(size_t)off = v; }
__device__ __forceinline__ void lds_st128(uint32_t off, u32x4 v) { *(lds_u32x4*)(size_t)off = v; }

__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
// gfx950 v_bitop3_b32 with LUT 0x96 = a ^ b ^ c in one VALU op (no v_xor3 on CDNA).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// v_perm_b32: result byte i = byte sel.byte[i] of {a (bytes 4..7), b (bytes 0..3)}, 0x0c -> 0x00.
__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t sel) { return __builtin_amdgcn_perm(a, b, sel); }

// Row-image address of (byte r of s): byte0/2/3 from the lane constant lb, byte1 = s.byte[r].
// Measured on gfx950 (tools/probe/valu_rate.hip, 8 waves/SIMD): v_perm / v_alignbit / shifts
// issue at ~4.2 cycles per wave-instruction, v_bitop3 with VGPR operands at ~2.9 — so byte 1,
// already in place, is masked in with one fast bitop3 ((s & 0xff00) | lb, mask in a VGPR).
__device__ __forceinline__ uint32_t byte1_mask() {
  uint32_t m;
  asm("v_mov_b32 %0, 0xff00" : "=v"(m));  // a VGPR operand: SGPR / literal operands issue slower
  return m;
}
template <int R>
__device__ __forceinline__ uint32_t ra(uint32_t s, uint32_t lb, uint32_t m = 0u) {
  if constexpr (R == 1) return __builtin_amdgcn_bitop3_b32(s, m, lb, 0xEA);  // (s & m) | lb, m = byte1_mask()
  return perm(s, lb, 0x03020400u | ((uint32_t)R << 8));
}

struct RoundKeys {
  uint32_t w[44];
};

// Issue grouping of LDS lookups (CMPI_LDS_BATCH): a scheduling fence after a round's 16
// independent table reads keeps hipcc from interleaving them with the XORs that consume them
// (its register-pressure schedule waited for the LDS after every second read, i.e. ~70 serial
// LDS round trips per AES block).
#ifndef CMPI_LDS_BATCH
#define CMPI_LDS_BATCH 0
#endif
__device__ __forceinline__ void lds_batch_fence() {
  if constexpr (CMPI_LDS_BATCH & 1) __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void ghash_batch_fence() {
  if constexpr (CMPI_LDS_BATCH & 2) __builtin_amdgcn_sched_barrier(0);
}

// Folded round keys.  A round column is T0[a] ^ T1[b] ^ K ^ rotl16(T0[c] ^ T1[d]); written as
// xor3(T0[a], T1[b], rotl16(xor3(T0[c], T1[d], rotl16(K)))) it is 3 VALU instead of 4 (rotl16
// is an involution).  The wave-uniform rotl16(K) of rounds 1..9 (words 4..39) is computed once
// by the host (kernel arguments) or the keysetup kernel: every AES routine below takes keys folded; words
// 0..3 (whitening) and 40..43 (last round) stay as they are.
__device__ __forceinline__ uint32_t srot16(uint32_t x) { return (x << 16) | (x >> 16); }
__device__ __forceinline__ RoundKeys fold_keys(const RoundKeys& k) {
  RoundKeys f = k;
#pragma unroll
  for (int i = 4; i < 40; ++i) f.w[i] = srot16(k.w[i]);
  return f;
}

// Lane constants of a row image at `base` (multiple of 64 KiB): Te0/Td0 half and Te1/Td1 half.
// m: the byte-1 mask in a VGPR, materialised once per kernel (per use it cost a v_mov per round).
struct RowLanes {
  uint32_t l0, l1, m;
};
__device__ __forceinline__ RowLanes row_lanes(uint32_t base) {
  const uint32_t l = ((threadIdx.x & 31u) << 2) | base;
  return RowLanes{l, l | 128u, byte1_mask()};
}

// One AES-128 encryption round (rounds 1..9) on state s, encryption row image; k* folded.
__device__ __forceinline__ void enc_round(const RowLanes& L, uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                          uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  const uint32_t a0 = lds32(ra<0>(s0, L.l0)), a1 = lds32(ra<1>(s1, L.l1, L.m)), a2 = lds32(ra<2>(s2, L.l0)), a3 = lds32(ra<3>(s3, L.l1));
  const uint32_t b0 = lds32(ra<0>(s1, L.l0)), b1 = lds32(ra<1>(s2, L.l1, L.m)), b2 = lds32(ra<2>(s3, L.l0)), b3 = lds32(ra<3>(s0, L.l1));
  const uint32_t c0 = lds32(ra<0>(s2, L.l0)), c1 = lds32(ra<1>(s3, L.l1, L.m)), c2 = lds32(ra<2>(s0, L.l0)), c3 = lds32(ra<3>(s1, L.l1));
  const uint32_t d0 = lds32(ra<0>(s3, L.l0)), d1 = lds32(ra<1>(s0, L.l1, L.m)), d2 = lds32(ra<2>(s1, L.l0)), d3 = lds32(ra<3>(s2, L.l1));
  lds_batch_fence();
  s0 = xor3(a0, a1, rotl16(xor3(a2, a3, k0)));
  s1 = xor3(b0, b1, rotl16(xor3(b2, b3, k1)));
  s2 = xor3(c0, c1, rotl16(xor3(c2, c3, k2)));
  s3 = xor3(d0, d1, rotl16(xor3(d2, d3, k3)));
}

// Last encryption round: S[x] = byte 1 of Te0[x]; gather byte 1 of the four lookups per column.
__device__ __forceinline__ void enc_last(const RowLanes& L, uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                         uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  const uint32_t a0 = lds32(ra<0>(s0, L.l0)), a1 = lds32(ra<1>(s1, L.l0, L.m)), a2 = lds32(ra<2>(s2, L.l0)), a3 = lds32(ra<3>(s3, L.l0));
  const uint32_t b0 = lds32(ra<0>(s1, L.l0)), b1 = lds32(ra<1>(s2, L.l0, L.m)), b2 = lds32(ra<2>(s3, L.l0)), b3 = lds32(ra<3>(s0, L.l0));
  const uint32_t c0 = lds32(ra<0>(s2, L.l0)), c1 = lds32(ra<1>(s3, L.l0, L.m)), c2 = lds32(ra<2>(s0, L.l0)), c3 = lds32(ra<3>(s1, L.l0));
  const uint32_t d0 = lds32(ra<0>(s3, L.l0)), d1 = lds32(ra<1>(s0, L.l0, L.m)), d2 = lds32(ra<2>(s1, L.l0)), d3 = lds32(ra<3>(s2, L.l0));
  lds_batch_fence();
  s0 = xor3(perm(a1, a0, 0x0c0c0501u), perm(a3, a2, 0x05010c0cu), k0);
  s1 = xor3(perm(b1, b0, 0x0c0c0501u), perm(b3, b2, 0x05010c0cu), k1);
  s2 = xor3(perm(c1, c0, 0x0c0c0501u), perm(c3, c2, 0x05010c0cu), k2);
  s3 = xor3(perm(d1, d0, 0x0c0c0501u), perm(d3, d2, 0x05010c0cu), k3);
}

// Full AES-128 encryption of (s0..s3); round keys folded, wave-uniform (kernarg -> SGPRs).
__device__ __forceinline__ void aes128_enc(const RoundKeys& k, const RowLanes& L, uint32_t& s0, uint32_t& s1,
                                           uint32_t& s2, uint32_t& s3) {
  s0 ^= k.w[0];
  s1 ^= k.w[1];
  s2 ^= k.w[2];
  s3 ^= k.w[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) enc_round(L, s0, s1, s2, s3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3]);
  enc_last(L, s0, s1, s2, s3, k.w[40], k.w[41], k.w[42], k.w[43]);
}

// Two independent blocks, rounds interleaved (more LDS requests in flight per wave).
__device__ __forceinline__ void aes128_enc2(const RoundKeys& k, const RowLanes& L, uint32_t& s0, uint32_t& s1,
                                            uint32_t& s2, uint32_t& s3, uint32_t& t0, uint32_t& t1, uint32_t& t2,
                                            uint32_t& t3) {
  s0 ^= k.w[0]; s1 ^= k.w[1]; s2 ^= k.w[2]; s3 ^= k.w[3];
  t0 ^= k.w[0]; t1 ^= k.w[1]; t2 ^= k.w[2]; t3 ^= k.w[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    enc_round(L, s0, s1, s2, s3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3]);
    enc_round(L, t0, t1, t2, t3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3]);
  }
  enc_last(L, s0, s1, s2, s3, k.w[40], k.w[41], k.w[42], k.w[43]);
  enc_last(L, t0, t1, t2, t3, k.w[40], k.w[41], k.w[42], k.w[43]);
}

// ---------------------------------------------------------------- counter-mode caching
// For counter blocks that differ only in their last byte (block byte 15 = byte 3 of word 3),
// round 1 has one varying lookup (Te1[b3(t3)] into column 0) and round 2 one varying lookup per
// column (the four bytes of round-1 column 0).  Everything else is a per-window constant:
// rounds 1+2 cost 5 lookups instead of 32 (Bernstein & Schwabe, "New AES software speed
// records", counter-mode caching).  A window = 256 consecutive counters sharing bytes 0..14.
struct CtrCache {
  uint32_t k0;              // round-1 column 0 without its varying term
  uint32_t q0, q1, q2, q3;  // round-2 columns without the term fed by round-1 column 0
};

// w0..w3: any counter block of the window (byte 3 of w3 is ignored).  k folded (fold_keys):
// the round-1/2 keys are unfolded here (once per window).
__device__ __forceinline__ void ctr_cache_fill(const RoundKeys& k, const RowLanes& L, uint32_t w0, uint32_t w1,
                                               uint32_t w2, uint32_t w3, CtrCache& c) {
  const uint32_t t0 = w0 ^ k.w[0], t1 = w1 ^ k.w[1], t2 = w2 ^ k.w[2], t3 = w3 ^ k.w[3];
  c.k0 = xor3(lds32(ra<0>(t0, L.l0)), lds32(ra<1>(t1, L.l1, L.m)), srot16(k.w[4])) ^ rotl16(lds32(ra<2>(t2, L.l0)));
  const uint32_t r1 = xor3(lds32(ra<0>(t1, L.l0)), lds32(ra<1>(t2, L.l1, L.m)), srot16(k.w[5])) ^
                      rotl16(lds32(ra<2>(t3, L.l0)) ^ lds32(ra<3>(t0, L.l1)));
  const uint32_t r2 = xor3(lds32(ra<0>(t2, L.l0)), lds32(ra<1>(t3, L.l1, L.m)), srot16(k.w[6])) ^
                      rotl16(lds32(ra<2>(t0, L.l0)) ^ lds32(ra<3>(t1, L.l1)));
  const uint32_t r3 = xor3(lds32(ra<0>(t3, L.l0)), lds32(ra<1>(t0, L.l1, L.m)), srot16(k.w[7])) ^
                      rotl16(lds32(ra<2>(t1, L.l0)) ^ lds32(ra<3>(t2, L.l1)));
  c.q0 = xor3(lds32(ra<1>(r1, L.l1, L.m)), srot16(k.w[8]), rotl16(lds32(ra<2>(r2, L.l0)) ^ lds32(ra<3>(r3, L.l1))));
  c.q1 = xor3(lds32(ra<0>(r1, L.l0)), lds32(ra<1>(r2, L.l1, L.m)), srot16(k.w[9])) ^ rotl16(lds32(ra<2>(r3, L.l0)));
  c.q2 = xor3(lds32(ra<0>(r2, L.l0)), lds32(ra<1>(r3, L.l1, L.m)), srot16(k.w[10])) ^ rotl16(lds32(ra<3>(r1, L.l1)));
  c.q3 = xor3(lds32(ra<0>(r3, L.l0)), srot16(k.w[11]), rotl16(lds32(ra<2>(r1, L.l0)) ^ lds32(ra<3>(r2, L.l1))));
}

// E_K(counter block) for a block of the cached window; w3 = its last word.
__device__ __forceinline__ void aes128_enc_ctr(const RoundKeys& k, const RowLanes& L, const CtrCache& c, uint32_t w3,
                                               uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3) {
  const uint32_t t3 = w3 ^ k.w[3];
  const uint32_t r0 = c.k0 ^ rotl16(lds32(ra<3>(t3, L.l1)));
  s0 = c.q0 ^ lds32(ra<0>(r0, L.l0));
  s3 = c.q3 ^ lds32(ra<1>(r0, L.l1, L.m));
  s2 = c.q2 ^ rotl16(lds32(ra<2>(r0, L.l0)));
  s1 = c.q1 ^ rotl16(lds32(ra<3>(r0, L.l1)));
#pragma unroll
  for (int r = 3; r < 10; ++r) enc_round(L, s0, s1, s2, s3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3]);
  enc_last(L, s0, s1, s2, s3, k.w[40], k.w[41], k.w[42], k.w[43]);
}

// AES-128 decryption (FIPS-197 §5.3.5 equivalent inverse cipher) with the Td0/Td1 row image
// (lanes LD) and the inverse S-box image at lbs = sbase | (lane&31)*4 for the last round.
__device__ __forceinline__ uint32_t sb0(uint32_t w) { return (w << 7) & 0x7f80u; }
__device__ __forceinline__ uint32_t sb1(uint32_t w) { return (w >> 1) & 0x7f80u; }
__device__ __forceinline__ uint32_t sb2(uint32_t w) { return (w >> 9) & 0x7f80u; }
__device__ __forceinline__ uint32_t sb3(uint32_t w) { return (w >> 17) & 0x7f80u; }

// (k: the decryption key schedule, folded by fold_keys like the encryption one.)
__device__ __forceinline__ void aes128_dec(const RoundKeys& k, const RowLanes& LD, uint32_t lbs, uint32_t& s0,
                                           uint32_t& s1, uint32_t& s2, uint32_t& s3) {
  s0 ^= k.w[0];
  s1 ^= k.w[1];
  s2 ^= k.w[2];
  s3 ^= k.w[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    // InvShiftRows: output column c takes row r from column c - r
    const uint32_t a0 = lds32(ra<0>(s0, LD.l0)), a1 = lds32(ra<1>(s3, LD.l1, LD.m)), a2 = lds32(ra<2>(s2, LD.l0)), a3 = lds32(ra<3>(s1, LD.l1));
    const uint32_t b0 = lds32(ra<0>(s1, LD.l0)), b1 = lds32(ra<1>(s0, LD.l1, LD.m)), b2 = lds32(ra<2>(s3, LD.l0)), b3 = lds32(ra<3>(s2, LD.l1));
    const uint32_t c0 = lds32(ra<0>(s2, LD.l0)), c1 = lds32(ra<1>(s1, LD.l1, LD.m)), c2 = lds32(ra<2>(s0, LD.l0)), c3 = lds32(ra<3>(s3, LD.l1));
    const uint32_t d0 = lds32(ra<0>(s3, LD.l0)), d1 = lds32(ra<1>(s2, LD.l1, LD.m)), d2 = lds32(ra<2>(s1, LD.l0)), d3 = lds32(ra<3>(s0, LD.l1));
    s0 = xor3(a0, a1, rotl16(xor3(a2, a3, k.w[4 * r + 0])));  // k folded
    s1 = xor3(b0, b1, rotl16(xor3(b2, b3, k.w[4 * r + 1])));
    s2 = xor3(c0, c1, rotl16(xor3(c2, c3, k.w[4 * r + 2])));
    s3 = xor3(d0, d1, rotl16(xor3(d2, d3, k.w[4 * r + 3])));
  }
  const uint32_t a0 = lds32(sb0(s0) | lbs), a1 = lds32(sb1(s3) | lbs), a2 = lds32(sb2(s2) | lbs), a3 = lds32(sb3(s1) | lbs);
  const uint32_t b0 = lds32(sb0(s1) | lbs), b1 = lds32(sb1(s0) | lbs), b2 = lds32(sb2(s3) | lbs), b3 = lds32(sb3(s2) | lbs);
  const uint32_t c0 = lds32(sb0(s2) | lbs), c1 = lds32(sb1(s1) | lbs), c2 = lds32(sb2(s0) | lbs), c3 = lds32(sb3(s3) | lbs);
  const uint32_t d0 = lds32(sb0(s3) | lbs), d1 = lds32(sb1(s2) | lbs), d2 = lds32(sb2(s1) | lbs), d3 = lds32(sb3(s0) | lbs);
  s0 = xor3(perm(a1, a0, 0x0c0c0400u), perm(a3, a2, 0x04000c0cu), k.w[40]);
  s1 = xor3(perm(b1, b0, 0x0c0c0400u), perm(b3, b2, 0x04000c0cu), k.w[41]);
  s2 = xor3(perm(c1, c0, 0x0c0c0400u), perm(c3, c2, 0x04000c0cu), k.w[42]);
  s3 = xor3(perm(d1, d0, 0x0c0c0400u), perm(d3, d2, 0x04000c0cu), k.w[43]);
}

// ---------------------------------------------------------------- table staging
// Row image from a 256-word T0 (Te0 or Td0): row x = [T0[x] x32 | rotl8(T0[x]) x32].
__device__ __forceinline__ void stage_rows(const uint32_t* __restrict__ t0, uint32_t base) {
  // entry e fills 64 words at base + 256e: 32 copies of Te0[e], then 32 of rotl8 (Te1[e]).
  // Four threads per entry, one global load and four 16-byte LDS stores each; the loads of up to
  // four passes (workgroups of >= 256 threads) are issued before any store, so a small workgroup
  // pays one global-load latency, not four (a word-per-iteration loop paid it 16 times).
  auto put = [&](uint32_t i, uint32_t v) {
    const uint32_t e = i >> 2, s = i & 3u;
    if (s >= 2u) v = rotl8(v);
    const u32x4 q = {v, v, v, v};
    const uint32_t o = base + e * 256u + s * 64u;
    lds_st128(o, q);
    lds_st128(o + 16u, q);
    lds_st128(o + 32u, q);
    lds_st128(o + 48u, q);
  };
  const uint32_t nt = blockDim.x;
  uint32_t v[4];
#pragma unroll
  for (uint32_t j = 0; j < 4u; ++j) {
    const uint32_t i = threadIdx.x + j * nt;
    v[j] = i < 1024u ? t0[i >> 2] : 0u;
  }
#pragma unroll
  for (uint32_t j = 0; j < 4u; ++j) {
    const uint32_t i = threadIdx.x + j * nt;
    if (i < 1024u) put(i, v[j]);
  }
  for (uint32_t i = threadIdx.x + 4u * nt; i < 1024u; i += nt) put(i, t0[i >> 2]);
}
// 32-way replicated 256-word table with 128-B rows (the inverse S-box image).
__device__ __forceinline__ void stage_rep32(const uint32_t* __restrict__ t, uint32_t base) {
  for (uint32_t i = threadIdx.x; i < 256u * 32u; i += blockDim.x) lds_st32(base + i * 4u, t[i >> 5]);
}
__device__ __forceinline__ void stage_copy(const u32x4* __restrict__ src, uint32_t dst_off, uint32_t n16) {
  const uint32_t step = blockDim.x;
  uint32_t i = threadIdx.x;
  for (; i + 3u * step < n16; i += 4u * step) {  // four loads in flight per thread
    const u32x4 a0 = src[i], a1 = src[i + step], a2 = src[i + 2u * step], a3 = src[i + 3u * step];
    lds_st128(dst_off + i * 16u, a0);
    lds_st128(dst_off + (i + step) * 16u, a1);
    lds_st128(dst_off + (i + 2u * step) * 16u, a2);
    lds_st128(dst_off + (i + 3u * step) * 16u, a3);
  }
  for (; i < n16; i += step) lds_st128(dst_off + i * 16u, src[i]);
}

// ---------------------------------------------------------------- GHASH
// Lane constants for the conflict-free byte-table multiply.
#ifndef CMPI_GHASH_B1
#define CMPI_GHASH_B1 0
#endif
struct GhashLane {
  uint32_t sh;        // 8 * (k & 3), k = lane & 15
  bool q1, q2;        // bits of k >> 2
  uint32_t po[4];     // po[j].byte[i] = ((4j + i + k) & 15) * 16
  uint32_t p1[4];     // CMPI_GHASH_B1: ((4j + 1 + k) & 15) * 16 in byte 0 (byte-1 positions by bitop3)
  uint32_t m;         // 0xff00 in a VGPR
};
__device__ __forceinline__ GhashLane ghash_lane() {
  GhashLane g;
  const uint32_t k = threadIdx.x & 15u;
  g.sh = 8u * (k & 3u);
  g.q1 = (k >> 2) & 1u;
  g.q2 = (k >> 3) & 1u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) w |= (((4u * j + i + k) & 15u) << 4) << (8 * i);
    g.po[j] = w;
    g.p1[j] = ((4u * j + 1u + k) & 15u) << 4;
  }
  g.m = byte1_mask();
  return g;
}

// X · P (+ Y) with the [v][p] byte table of P at LDS 0: rotate X by k bytes (X'.byte t =
// X.byte (t+k)), then 16 conflict-free ds_read_b128 at (X'.byte t) * 256 + ((t + k) & 15) * 16.
// The addend Y seeds the XOR chain (a Horner step's next block: no separate XOR).
__device__ __forceinline__ u32x4 gmul_byte(u32x4 x, const GhashLane& g, u32x4 y = u32x4{0u, 0u, 0u, 0u}) {
  const uint32_t y0 = __builtin_amdgcn_alignbit(x[1], x[0], g.sh);
  const uint32_t y1 = __builtin_amdgcn_alignbit(x[2], x[1], g.sh);
  const uint32_t y2 = __builtin_amdgcn_alignbit(x[3], x[2], g.sh);
  const uint32_t y3 = __builtin_amdgcn_alignbit(x[0], x[3], g.sh);
  const uint32_t z0 = g.q1 ? y1 : y0, z1 = g.q1 ? y2 : y1, z2 = g.q1 ? y3 : y2, z3 = g.q1 ? y0 : y3;
  const uint32_t w[4] = {g.q2 ? z2 : z0, g.q2 ? z3 : z1, g.q2 ? z0 : z2, g.q2 ? z1 : z3};
  u32x4 r = y;
  if constexpr (CMPI_LDS_BATCH & 2) {  // four reads in flight per wait
#pragma unroll
    for (int t = 0; t < 16; t += 4) {
      u32x4 e[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = t + i;
        const uint32_t sel = 0x0c0c0000u | ((4u + (p & 3)) << 8) | (uint32_t)(p & 3);
        e[i] = lds128(perm(w[p >> 2], g.po[p >> 2], sel));
      }
      ghash_batch_fence();
#pragma unroll
      for (int c = 0; c < 4; ++c) r[c] = xor3(r[c], e[0][c], e[1][c]) ^ (e[2][c] ^ e[3][c]);
    }
    return r;
  }
  auto gaddr = [&](int p) -> uint32_t {
    if constexpr (CMPI_GHASH_B1 != 0) {
      if ((p & 3) == 1) return __builtin_amdgcn_bitop3_b32(w[p >> 2], g.m, g.p1[p >> 2], 0xEA);  // (w & 0xff00) | p1
    }
    const uint32_t sel = 0x0c0c0000u | ((4u + (p & 3)) << 8) | (uint32_t)(p & 3);
    return perm(w[p >> 2], g.po[p >> 2], sel);
  };
#pragma unroll
  for (int t = 0; t < 16; t += 2) {
    const u32x4 e1 = lds128(gaddr(t));
    const u32x4 e2 = lds128(gaddr(t + 1));
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = xor3(r[c], e1[c], e2[c]);
  }
  return r;
}

// X · P with an 8 KiB nibble table of P at LDS byte offset `tb` (multiple of 8 KiB).
// The 32 lookups go out in batches of 8 (one s_waitcnt per batch): written as one loop the
// compiler, short of registers in the wide kernel, paired them with a wait after every two
// reads — 16 LDS round trips (~1 us) per multiply.
__device__ __forceinline__ u32x4 gmul_nib(u32x4 x, uint32_t tb) {
  u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int q = 0; q < 16; q += 4) {
    u32x4 e[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int p = q + t;
      const uint32_t w = x[p >> 2];
      const int sh = 8 * (p & 3);
      const uint32_t hi = (w >> sh) & 0xf0u;                              // (v >> 4) * 16
      const uint32_t lo = (sh == 0 ? (w << 4) : (w >> (sh - 4))) & 0xf0u;  // (v & 15) * 16
      e[2 * t] = lds128((hi | tb) + (uint32_t)p * 512u);
      e[2 * t + 1] = lds128((lo | tb) + (uint32_t)p * 512u + 256u);
    }
#pragma unroll
    for (int t = 0; t < 8; t += 2)
#pragma unroll
      for (int c = 0; c < 4; ++c) r[c] = xor3(r[c], e[t][c], e[t + 1][c]);
  }
  return r;
}

// GCM-order field element as (hi, lo) big-endian halves of its 16 memory bytes.
__device__ __forceinline__ void gf_split(u32x4 x, uint64_t& h, uint64_t& l) {
  h = ((uint64_t)__builtin_bswap32(x[0]) << 32) | __builtin_bswap32(x[1]);
  l = ((uint64_t)__builtin_bswap32(x[2]) << 32) | __builtin_bswap32(x[3]);
}
__device__ __forceinline__ u32x4 gf_join(uint64_t h, uint64_t l) {
  return u32x4{__builtin_bswap32((uint32_t)(h >> 32)), __builtin_bswap32((uint32_t)h),
               __builtin_bswap32((uint32_t)(l >> 32)), __builtin_bswap32((uint32_t)l)};
}

// X · x^s (0 <= s < 128) on (hi, lo) halves: the 128-bit right shift by s, whose shifted-out
// coefficients (x^128 ..) fold back through x^128 = 1 + x + x^2 + x^7 — twice, the second fold
// for the at most 7 bits the first one pushes past x^127.  Straight-line (no bit-serial loop).
__device__ __forceinline__ void gf_mulx_pow(uint64_t& h, uint64_t& l, uint32_t s) {
  uint64_t w0 = h, w1 = l, w2 = 0, w3 = 0;
  if (s & 64u) {
    w2 = w1;
    w1 = w0;
    w0 = 0;
  }
  const uint32_t q = s & 63u;
  if (q) {
    w3 = w2 << (64u - q);
    w2 = (w2 >> q) | (w1 << (64u - q));
    w1 = (w1 >> q) | (w0 << (64u - q));
    w0 >>= q;
  }
  const uint64_t sp = (w3 << 63) ^ (w3 << 62) ^ (w3 << 57);
  h = w0 ^ w2 ^ (w2 >> 1) ^ (w2 >> 2) ^ (w2 >> 7);
  l = w1 ^ w3 ^ ((w3 >> 1) | (w2 << 63)) ^ ((w3 >> 2) | (w2 << 62)) ^ ((w3 >> 7) | (w2 << 57));
  h ^= sp ^ (sp >> 1) ^ (sp >> 2) ^ (sp >> 7);
}

// Nibble-table row `row` (0..31) of P, built in LDS at tb + row*256 (the layout gmul_nib reads,
// gf128_host.hpp build_nibble_table): entry v = XOR over set bits k of v of P · x^(c - k),
// c = 8(row/2) + (row odd ? 7 : 3).  One variable shift, then three single shifts.
__device__ __forceinline__ void nib_row_to_lds(u32x4 P, uint32_t row, uint32_t tb) {
  uint64_t h, l;
  gf_split(P, h, l);
  gf_mulx_pow(h, l, 8u * (row >> 1) + ((row & 1u) ? 4u : 0u));  // P · x^(c - 3)
  u32x4 u[4];
#pragma unroll
  for (int k = 3; k >= 0; --k) {
    u[k] = gf_join(h, l);
    const uint64_t lsb = 0 - (l & 1u);
    l = (l >> 1) | (h << 63);
    h = (h >> 1) ^ (0xE100000000000000ULL & lsb);
  }
#pragma unroll
  for (uint32_t v = 0; v < 16u; ++v) {
    u32x4 e = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (v & (1u << k)) e ^= u[k];
    lds_st128(tb + row * 256u + v * 16u, e);
  }
}

// Generic X · Y (both arbitrary, memory-order words), bit-serial SP 800-38D Algorithm 1.
// Used only outside the hot loop (segment combination).
__device__ __forceinline__ u32x4 gmul_generic(u32x4 x, u32x4 y) {
  uint64_t xh = ((uint64_t)__builtin_bswap32(x[0]) << 32) | __builtin_bswap32(x[1]);
  uint64_t xl = ((uint64_t)__builtin_bswap32(x[2]) << 32) | __builtin_bswap32(x[3]);
  uint64_t vh = ((uint64_t)__builtin_bswap32(y[0]) << 32) | __builtin_bswap32(y[1]);
  uint64_t vl = ((uint64_t)__builtin_bswap32(y[2]) << 32) | __builtin_bswap32(y[3]);
  uint64_t zh = 0, zl = 0;
  for (int i = 0; i < 128; ++i) {
    const uint64_t bit = (i < 64) ? (xh >> (63 - i)) & 1 : (xl >> (127 - i)) & 1;
    const uint64_t m = 0 - bit;
    zh ^= vh & m;
    zl ^= vl & m;
    const uint64_t lsb = 0 - (vl & 1);
    vl = (vl >> 1) | (vh << 63);
    vh = (vh >> 1) ^ (0xE100000000000000ULL & lsb);
  }
  u32x4 z;
  z[0] = __builtin_bswap32((uint32_t)(zh >> 32));
  z[1] = __builtin_bswap32((uint32_t)zh);
  z[2] = __builtin_bswap32((uint32_t)(zl >> 32));
  z[3] = __builtin_bswap32((uint32_t)zl);
  return z;
}

// Generic X · Y on 32-bit big-endian words (same result as gmul_generic): per bit of X one
// sign-extended mask, four masked XORs (v_bitop3) and a 1-bit right shift of V across the
// words (3 v_alignbit + the reduction by 0xE1 || 0^120) — ~1.4 k VALU, a short dependency chain.
__device__ __forceinline__ u32x4 gmul_generic32(u32x4 x, u32x4 y) {
  uint32_t v0 = __builtin_bswap32(y[0]), v1 = __builtin_bswap32(y[1]), v2 = __builtin_bswap32(y[2]),
           v3 = __builtin_bswap32(y[3]);
  uint32_t z0 = 0u, z1 = 0u, z2 = 0u, z3 = 0u;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t xw = __builtin_bswap32(x[w]);
#pragma unroll
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t m = (uint32_t)((int32_t)(xw << (31 - bit)) >> 31);
      z0 ^= v0 & m;
      z1 ^= v1 & m;
      z2 ^= v2 & m;
      z3 ^= v3 & m;
      const uint32_t lsb = (uint32_t)((int32_t)(v3 << 31) >> 31);
      v3 = __builtin_amdgcn_alignbit(v2, v3, 1);
      v2 = __builtin_amdgcn_alignbit(v1, v2, 1);
      v1 = __builtin_amdgcn_alignbit(v0, v1, 1);
      v0 = (v0 >> 1) ^ (0xE1000000u & lsb);
    }
  }
  return u32x4{__builtin_bswap32(z0), __builtin_bswap32(z1), __builtin_bswap32(z2), __builtin_bswap32(z3)};
}

// Wave-issue fairness.  The SQ arbitrates VALU/LDS issue by priority, then age, so waves of a
// workgroup that carry EQUAL work finish far apart (measured with tools/probe/lds_probe.hip:
// lifetimes 190K..418K cycles for identical AES loops) and the CU idles through the tail.
// Rotating each wave's priority every loop iteration ((t + wave) mod 4, t wave-uniform)
// spreads issue fairly: -11 % time on the probe at one 1024-thread block per CU.
__device__ __forceinline__ void rotate_prio(uint32_t t) {
  switch ((__builtin_amdgcn_readfirstlane(t) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) & 3u) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}

// Progress-based priority: every wave adds one to a workgroup counter in LDS per unit of work it
// starts and takes priority 3..0 by how far it is behind / ahead of the workgroup average (the
// counter holds the sum of all waves' progress).  Waves of equal work then finish together
// instead of spread by issue arbitration (tools/probe/lds_probe.hip, 4 waves/SIMD: 2.71 -> 2.48
// CU-ns per block against rotate_prio, wave lifetimes 288K..375K -> 347K..362K cycles).
// Measured, not taken: a bounded s_sleep back-off of waves more than 4/8/16 slots ahead of the
// average (to hand the CU's LDS to slower SIMDs) left config 2 at 57.5-57.9 us per seal (warm
// clocks, tools/lane_ab.py, profiles/r03e_lane_backoff_ab.log).
__device__ __forceinline__ void progress_prio(uint32_t cnt_off, uint32_t done) {
  uint32_t tot = 0;
  if ((threadIdx.x & 63u) == 0u)
    tot = __hip_atomic_fetch_add((lds_u32*)(size_t)cnt_off, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  tot = __builtin_amdgcn_readfirstlane(tot) + 1u;
  const uint32_t nw = blockDim.x >> 6, mine = done * nw;
  const uint32_t p = mine + nw <= tot ? 3u : (mine <= tot ? 2u : (mine <= tot + nw ? 1u : 0u));
  switch (p) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}

__device__ __forceinline__ u32x4 shfl_down4(u32x4 v, uint32_t d) {
  u32x4 r;
  r[0] = __shfl_down((int)v[0], d);
  r[1] = __shfl_down((int)v[1], d);
  r[2] = __shfl_down((int)v[2], d);
  r[3] = __shfl_down((int)v[3], d);
  return r;
}

__device__ __forceinline__ u32x4 shfl_xor4(u32x4 v, int m) {
  u32x4 r;
  r[0] = __shfl_xor((int)v[0], m);
  r[1] = __shfl_xor((int)v[1], m);
  r[2] = __shfl_xor((int)v[2], m);
  r[3] = __shfl_xor((int)v[3], m);
  return r;
}

// XOR exchanges across lanes without the LDS crossbar (all 64 lanes active).  __shfl_xor
// compiles to ds_bpermute_b32: an LDS round trip per dword and step, which made the flow
// kernel's lane tree and chunk weight (56 of them in sequence-dependent groups) a latency chain.
// DPP row ops and gfx950's v_permlane16/32_swap are plain VALU:
//   xq1 / xq2   x ^ x[l ^ 1] / x ^ x[l ^ 2]        (quad_perm)
//   xr4 / xr8   x ^ x[l - 4] / x ^ x[l - 8] within a row of 16 (row_ror; applied in turn they sum
//               the four lanes l mod 4 of a row, as xor 4 then xor 8 do)
//   x16 / x32   x ^ x[l ^ 16] / x ^ x[l ^ 32]      (permlane16 / permlane32 swap, the pair XORed)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ u32x4 xq1(u32x4 v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] ^= dpp_mov<0xB1>(v[c]);  // quad_perm [1,0,3,2]
  return v;
}
__device__ __forceinline__ u32x4 xq2(u32x4 v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] ^= dpp_mov<0x4E>(v[c]);  // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ u32x4 xr4(u32x4 v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] ^= dpp_mov<0x124>(v[c]);  // row_ror:4
  return v;
}
__device__ __forceinline__ u32x4 xr8(u32x4 v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] ^= dpp_mov<0x128>(v[c]);  // row_ror:8 (= lane ^ 8 in a row)
  return v;
}
__device__ __forceinline__ u32x4 x16(u32x4 v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const auto r = __builtin_amdgcn_permlane16_swap(v[c], v[c], false, false);
    v[c] = r[0] ^ r[1];
  }
  return v;
}
__device__ __forceinline__ u32x4 x32(u32x4 v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const auto r = __builtin_amdgcn_permlane32_swap(v[c], v[c], false, false);
    v[c] = r[0] ^ r[1];
  }
  return v;
}
// XOR of all 64 lanes, in every lane.
__device__ __forceinline__ u32x4 xor_all_lanes(u32x4 v) { return x32(x16(xr8(xr4(xq2(xq1(v)))))); }

// Y · M for wave-uniform Y and M, computed by the whole wavefront (all 64 lanes active):
// Y·M = XOR_k m_k · (Y·x^k); lane l takes the coefficients k = 2l, 2l+1 of M (one variable
// shift gf_mulx_pow and one single shift), and the 64 lane terms are XOR-reduced with
// shuffles.  ~70 VALU per lane — one generic product where a single lane would need ~1.4 k.
// Every lane returns the product.
__device__ __forceinline__ u32x4 gmul_wave(u32x4 y, u32x4 m) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t yh, yl, mh, ml;
  gf_split(y, yh, yl);
  gf_split(m, mh, ml);
  const uint32_t k = 2u * lane;  // coefficient of x^k sits at bit 127 - k of (mh:ml)
  const uint64_t mw = lane < 32u ? mh : ml;
  const uint32_t kk = k & 63u;
  const uint64_t b0 = 0 - ((mw >> (63u - kk)) & 1u), b1 = 0 - ((mw >> (62u - kk)) & 1u);
  gf_mulx_pow(yh, yl, k);
  uint64_t zh = yh & b0, zl = yl & b0;
  const uint64_t lsb = 0 - (yl & 1u);
  yl = (yl >> 1) | (yh << 63);
  yh = (yh >> 1) ^ (0xE100000000000000ULL & lsb);
  zh ^= yh & b1;
  zl ^= yl & b1;
  u32x4 z = gf_join(zh, zl);
  z = xor_all_lanes(z);
  return z;
}

// XOR of four products Y_j · M_j (all wave-uniform), by the whole wavefront as gmul_wave with one
// shared shuffle reduction.  Every lane returns the sum.
__device__ __forceinline__ u32x4 gmul_wave4(const u32x4 (&y)[4], const u32x4 (&m)[4]) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t k = 2u * lane, kk = k & 63u;
  uint64_t zh = 0, zl = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint64_t yh, yl, mh, ml;
    gf_split(y[j], yh, yl);
    gf_split(m[j], mh, ml);
    const uint64_t mw = lane < 32u ? mh : ml;
    const uint64_t b0 = 0 - ((mw >> (63u - kk)) & 1u), b1 = 0 - ((mw >> (62u - kk)) & 1u);
    gf_mulx_pow(yh, yl, k);
    zh ^= yh & b0;
    zl ^= yl & b0;
    const uint64_t lsb = 0 - (yl & 1u);
    yl = (yl >> 1) | (yh << 63);
    yh = (yh >> 1) ^ (0xE100000000000000ULL & lsb);
    zh ^= yh & b1;
    zl ^= yl & b1;
  }
  u32x4 z = gf_join(zh, zl);
  z = xor_all_lanes(z);
  return z;
}

// Partial-block helpers (bytes [0, n) of a 16-byte block at an arbitrary address).
__device__ __forceinline__ u32x4 mask_bytes(u32x4 v, uint32_t n) {  // keep bytes [0, n)
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int lo = 4 * c;
    uint32_t m = (n >= (uint32_t)(lo + 4)) ? 0xffffffffu : (n <= (uint32_t)lo ? 0u : (0xffffffffu >> (8 * (lo + 4 - n))));
    v[c] &= m;
  }
  return v;
}
// Bytes [0, n) of a block that ends a record (n <= 16), zero above.  Every byte is read from a
// clamped address (nothing past p[n-1]) with no branch, so the 16 loads are in flight together:
// a per-byte conditional load had the compiler wait for each one in turn (about ten memory
// latencies in sequence per ragged record; over PCIe, for a host-memory message, ten round trips).
__device__ __forceinline__ u32x4 load_partial(const uint8_t* p, uint32_t n) {
  if (n == 0u) return u32x4{0u, 0u, 0u, 0u};
  const uint32_t last = n - 1u;
  uint32_t b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = p[min((uint32_t)i, last)];
  u32x4 r;
#pragma unroll
  for (int c = 0; c < 4; ++c) r[c] = b[4 * c] | (b[4 * c + 1] << 8) | (b[4 * c + 2] << 16) | (b[4 * c + 3] << 24);
  return mask_bytes(r, n);
}
__device__ __forceinline__ void store_partial(uint8_t* p, u32x4 v, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) p[i] = (uint8_t)(v[i >> 2] >> (8 * (i & 3)));
}

}  // namespace dev
}  // namespace cmpi
