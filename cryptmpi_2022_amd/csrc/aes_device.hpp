// aes_device.hpp — CDNA4 (gfx950) device primitives: LDS-staged AES-128 T-table rounds and
// table-driven GF(2^128) multiplication, all in the little-endian word convention of
// aes_tables.hpp.
//
// LDS images (byte offsets inside the kernel's dynamic LDS):
//  * Te0, 32-way replicated: entry x of replica k at tbase + x*128 + k*4.  Lane l reads replica
//    (l & 31): in a ds_read_b32 (two 32-lane halves, bank = (addr/4) mod 32) every lane of a half
//    hits its own bank whatever x is, so AES lookups are bank-conflict free.  tbase must be a
//    multiple of 32 KiB so the lane term ORs in (x*128 < 32 KiB).
//  * GHASH byte table (multiplier P): entry (p, v) = (byte p := v)·P at p*4096 + v*16, 64 KiB
//    at LDS offset 0 so p*4096 folds into the ds_read_b128 immediate offset.
//  * GHASH nibble tables: 8 KiB each, entry (2p+h, v) at base + p*512 + h*256 + v*16, bases
//    multiples of 8 KiB so the (p, h) part folds into the immediate and the value term ORs in.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmpi {
namespace dev {

extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Byte-aligned 16-byte / 4-byte views of record data: records may start at any byte offset
// (the nonce(12)||ct||tag wire layout with odd n, the 602 5-byte segment prefix).  On gfx950
// under amdhsa the backend runs in unaligned-access mode and still emits one
// global_load/store_dwordx4 (resp. _dword) for these.
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32a __attribute__((aligned(1)));

// LDS accesses by raw byte offset.  All kernels here use only dynamic LDS (no static
// __shared__), so the dynamic region starts at LDS address 0 and an offset IS the address:
// building address_space(3) pointers from the offset lets ds_read use it directly (going
// through `smem + off` costs an extra v_add per lookup).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
__device__ __forceinline__ uint32_t lds32(uint32_t off) { return *(const lds_u32*)(size_t)off; }
__device__ __forceinline__ u32x4 lds128(uint32_t off) { return *(const lds_u32x4*)(size_t)off; }
__device__ __forceinline__ void lds_st32(uint32_t off, uint32_t v) { *(lds_u32*)(size_t)off = v; }
__device__ __forceinline__ void lds_st128(uint32_t off, u32x4 v) { *(lds_u32x4*)(size_t)off = v; }

__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t rotl24(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 8); }
// gfx950 v_bitop3_b32 with LUT 0x96 = a ^ b ^ c in one VALU op (no v_xor3 on CDNA).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// (byte r of w) * 128, the Te0 row offset
__device__ __forceinline__ uint32_t tb0(uint32_t w) { return (w << 7) & 0x7f80u; }
__device__ __forceinline__ uint32_t tb1(uint32_t w) { return (w >> 1) & 0x7f80u; }
__device__ __forceinline__ uint32_t tb2(uint32_t w) { return (w >> 9) & 0x7f80u; }
__device__ __forceinline__ uint32_t tb3(uint32_t w) { return (w >> 17) & 0x7f80u; }

struct RoundKeys {
  uint32_t w[44];
};

// One full AES-128 encryption of the block (s0..s3), round keys wave-uniform (kernarg → SGPRs),
// lb = tbase | (lane & 31) * 4.
__device__ __forceinline__ void aes128_enc(const RoundKeys& k, uint32_t lb, uint32_t& s0, uint32_t& s1,
                                           uint32_t& s2, uint32_t& s3) {
  s0 ^= k.w[0];
  s1 ^= k.w[1];
  s2 ^= k.w[2];
  s3 ^= k.w[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    uint32_t a0 = lds32(tb0(s0) | lb), a1 = lds32(tb1(s1) | lb), a2 = lds32(tb2(s2) | lb), a3 = lds32(tb3(s3) | lb);
    uint32_t b0 = lds32(tb0(s1) | lb), b1 = lds32(tb1(s2) | lb), b2 = lds32(tb2(s3) | lb), b3 = lds32(tb3(s0) | lb);
    uint32_t c0 = lds32(tb0(s2) | lb), c1 = lds32(tb1(s3) | lb), c2 = lds32(tb2(s0) | lb), c3 = lds32(tb3(s1) | lb);
    uint32_t d0 = lds32(tb0(s3) | lb), d1 = lds32(tb1(s0) | lb), d2 = lds32(tb2(s1) | lb), d3 = lds32(tb3(s2) | lb);
    s0 = xor3(xor3(a0, rotl8(a1), rotl16(a2)), rotl24(a3), k.w[4 * r + 0]);
    s1 = xor3(xor3(b0, rotl8(b1), rotl16(b2)), rotl24(b3), k.w[4 * r + 1]);
    s2 = xor3(xor3(c0, rotl8(c1), rotl16(c2)), rotl24(c3), k.w[4 * r + 2]);
    s3 = xor3(xor3(d0, rotl8(d1), rotl16(d2)), rotl24(d3), k.w[4 * r + 3]);
  }
  // last round: S[x] = byte 1 of Te0[x]; gather byte 1 of the four lookups per column
  uint32_t a0 = lds32(tb0(s0) | lb), a1 = lds32(tb1(s1) | lb), a2 = lds32(tb2(s2) | lb), a3 = lds32(tb3(s3) | lb);
  uint32_t b0 = lds32(tb0(s1) | lb), b1 = lds32(tb1(s2) | lb), b2 = lds32(tb2(s3) | lb), b3 = lds32(tb3(s0) | lb);
  uint32_t c0 = lds32(tb0(s2) | lb), c1 = lds32(tb1(s3) | lb), c2 = lds32(tb2(s0) | lb), c3 = lds32(tb3(s1) | lb);
  uint32_t d0 = lds32(tb0(s3) | lb), d1 = lds32(tb1(s0) | lb), d2 = lds32(tb2(s1) | lb), d3 = lds32(tb3(s2) | lb);
  s0 = xor3(__builtin_amdgcn_perm(a1, a0, 0x0c0c0501u), __builtin_amdgcn_perm(a3, a2, 0x05010c0cu), k.w[40]);
  s1 = xor3(__builtin_amdgcn_perm(b1, b0, 0x0c0c0501u), __builtin_amdgcn_perm(b3, b2, 0x05010c0cu), k.w[41]);
  s2 = xor3(__builtin_amdgcn_perm(c1, c0, 0x0c0c0501u), __builtin_amdgcn_perm(c3, c2, 0x05010c0cu), k.w[42]);
  s3 = xor3(__builtin_amdgcn_perm(d1, d0, 0x0c0c0501u), __builtin_amdgcn_perm(d3, d2, 0x05010c0cu), k.w[43]);
}

// Two independent blocks interleaved (ILP for the LDS pipe).
__device__ __forceinline__ void aes128_enc2(const RoundKeys& k, uint32_t lb, uint32_t& s0, uint32_t& s1,
                                            uint32_t& s2, uint32_t& s3, uint32_t& t0, uint32_t& t1,
                                            uint32_t& t2, uint32_t& t3) {
  s0 ^= k.w[0]; s1 ^= k.w[1]; s2 ^= k.w[2]; s3 ^= k.w[3];
  t0 ^= k.w[0]; t1 ^= k.w[1]; t2 ^= k.w[2]; t3 ^= k.w[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    uint32_t a0 = lds32(tb0(s0) | lb), a1 = lds32(tb1(s1) | lb), a2 = lds32(tb2(s2) | lb), a3 = lds32(tb3(s3) | lb);
    uint32_t b0 = lds32(tb0(s1) | lb), b1 = lds32(tb1(s2) | lb), b2 = lds32(tb2(s3) | lb), b3 = lds32(tb3(s0) | lb);
    uint32_t c0 = lds32(tb0(s2) | lb), c1 = lds32(tb1(s3) | lb), c2 = lds32(tb2(s0) | lb), c3 = lds32(tb3(s1) | lb);
    uint32_t d0 = lds32(tb0(s3) | lb), d1 = lds32(tb1(s0) | lb), d2 = lds32(tb2(s1) | lb), d3 = lds32(tb3(s2) | lb);
    uint32_t e0 = lds32(tb0(t0) | lb), e1 = lds32(tb1(t1) | lb), e2 = lds32(tb2(t2) | lb), e3 = lds32(tb3(t3) | lb);
    uint32_t f0 = lds32(tb0(t1) | lb), f1 = lds32(tb1(t2) | lb), f2 = lds32(tb2(t3) | lb), f3 = lds32(tb3(t0) | lb);
    uint32_t g0 = lds32(tb0(t2) | lb), g1 = lds32(tb1(t3) | lb), g2 = lds32(tb2(t0) | lb), g3 = lds32(tb3(t1) | lb);
    uint32_t h0 = lds32(tb0(t3) | lb), h1 = lds32(tb1(t0) | lb), h2 = lds32(tb2(t1) | lb), h3 = lds32(tb3(t2) | lb);
    s0 = xor3(xor3(a0, rotl8(a1), rotl16(a2)), rotl24(a3), k.w[4 * r + 0]);
    s1 = xor3(xor3(b0, rotl8(b1), rotl16(b2)), rotl24(b3), k.w[4 * r + 1]);
    s2 = xor3(xor3(c0, rotl8(c1), rotl16(c2)), rotl24(c3), k.w[4 * r + 2]);
    s3 = xor3(xor3(d0, rotl8(d1), rotl16(d2)), rotl24(d3), k.w[4 * r + 3]);
    t0 = xor3(xor3(e0, rotl8(e1), rotl16(e2)), rotl24(e3), k.w[4 * r + 0]);
    t1 = xor3(xor3(f0, rotl8(f1), rotl16(f2)), rotl24(f3), k.w[4 * r + 1]);
    t2 = xor3(xor3(g0, rotl8(g1), rotl16(g2)), rotl24(g3), k.w[4 * r + 2]);
    t3 = xor3(xor3(h0, rotl8(h1), rotl16(h2)), rotl24(h3), k.w[4 * r + 3]);
  }
  {
    uint32_t a0 = lds32(tb0(s0) | lb), a1 = lds32(tb1(s1) | lb), a2 = lds32(tb2(s2) | lb), a3 = lds32(tb3(s3) | lb);
    uint32_t b0 = lds32(tb0(s1) | lb), b1 = lds32(tb1(s2) | lb), b2 = lds32(tb2(s3) | lb), b3 = lds32(tb3(s0) | lb);
    uint32_t c0 = lds32(tb0(s2) | lb), c1 = lds32(tb1(s3) | lb), c2 = lds32(tb2(s0) | lb), c3 = lds32(tb3(s1) | lb);
    uint32_t d0 = lds32(tb0(s3) | lb), d1 = lds32(tb1(s0) | lb), d2 = lds32(tb2(s1) | lb), d3 = lds32(tb3(s2) | lb);
    s0 = xor3(__builtin_amdgcn_perm(a1, a0, 0x0c0c0501u), __builtin_amdgcn_perm(a3, a2, 0x05010c0cu), k.w[40]);
    s1 = xor3(__builtin_amdgcn_perm(b1, b0, 0x0c0c0501u), __builtin_amdgcn_perm(b3, b2, 0x05010c0cu), k.w[41]);
    s2 = xor3(__builtin_amdgcn_perm(c1, c0, 0x0c0c0501u), __builtin_amdgcn_perm(c3, c2, 0x05010c0cu), k.w[42]);
    s3 = xor3(__builtin_amdgcn_perm(d1, d0, 0x0c0c0501u), __builtin_amdgcn_perm(d3, d2, 0x05010c0cu), k.w[43]);
  }
  {
    uint32_t a0 = lds32(tb0(t0) | lb), a1 = lds32(tb1(t1) | lb), a2 = lds32(tb2(t2) | lb), a3 = lds32(tb3(t3) | lb);
    uint32_t b0 = lds32(tb0(t1) | lb), b1 = lds32(tb1(t2) | lb), b2 = lds32(tb2(t3) | lb), b3 = lds32(tb3(t0) | lb);
    uint32_t c0 = lds32(tb0(t2) | lb), c1 = lds32(tb1(t3) | lb), c2 = lds32(tb2(t0) | lb), c3 = lds32(tb3(t1) | lb);
    uint32_t d0 = lds32(tb0(t3) | lb), d1 = lds32(tb1(t0) | lb), d2 = lds32(tb2(t1) | lb), d3 = lds32(tb3(t2) | lb);
    t0 = xor3(__builtin_amdgcn_perm(a1, a0, 0x0c0c0501u), __builtin_amdgcn_perm(a3, a2, 0x05010c0cu), k.w[40]);
    t1 = xor3(__builtin_amdgcn_perm(b1, b0, 0x0c0c0501u), __builtin_amdgcn_perm(b3, b2, 0x05010c0cu), k.w[41]);
    t2 = xor3(__builtin_amdgcn_perm(c1, c0, 0x0c0c0501u), __builtin_amdgcn_perm(c3, c2, 0x05010c0cu), k.w[42]);
    t3 = xor3(__builtin_amdgcn_perm(d1, d0, 0x0c0c0501u), __builtin_amdgcn_perm(d3, d2, 0x05010c0cu), k.w[43]);
  }
}

// AES-128 decryption (FIPS-197 §5.3.5 equivalent inverse cipher).  Td0 replicated x32 at
// dbase, the inverse S-box (as words, Si[x] in byte 0) replicated x32 at sbase; both bases
// multiples of 32 KiB; lane term ld = (lane & 31) * 4 is OR-ed in by the caller's dbase|ld.
__device__ __forceinline__ void aes128_dec(const RoundKeys& k, uint32_t ldd, uint32_t lds_, uint32_t& s0,
                                           uint32_t& s1, uint32_t& s2, uint32_t& s3) {
  s0 ^= k.w[0];
  s1 ^= k.w[1];
  s2 ^= k.w[2];
  s3 ^= k.w[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    uint32_t a0 = lds32(tb0(s0) | ldd), a1 = lds32(tb1(s3) | ldd), a2 = lds32(tb2(s2) | ldd), a3 = lds32(tb3(s1) | ldd);
    uint32_t b0 = lds32(tb0(s1) | ldd), b1 = lds32(tb1(s0) | ldd), b2 = lds32(tb2(s3) | ldd), b3 = lds32(tb3(s2) | ldd);
    uint32_t c0 = lds32(tb0(s2) | ldd), c1 = lds32(tb1(s1) | ldd), c2 = lds32(tb2(s0) | ldd), c3 = lds32(tb3(s3) | ldd);
    uint32_t d0 = lds32(tb0(s3) | ldd), d1 = lds32(tb1(s2) | ldd), d2 = lds32(tb2(s1) | ldd), d3 = lds32(tb3(s0) | ldd);
    s0 = xor3(xor3(a0, rotl8(a1), rotl16(a2)), rotl24(a3), k.w[4 * r + 0]);
    s1 = xor3(xor3(b0, rotl8(b1), rotl16(b2)), rotl24(b3), k.w[4 * r + 1]);
    s2 = xor3(xor3(c0, rotl8(c1), rotl16(c2)), rotl24(c3), k.w[4 * r + 2]);
    s3 = xor3(xor3(d0, rotl8(d1), rotl16(d2)), rotl24(d3), k.w[4 * r + 3]);
  }
  uint32_t a0 = lds32(tb0(s0) | lds_), a1 = lds32(tb1(s3) | lds_), a2 = lds32(tb2(s2) | lds_), a3 = lds32(tb3(s1) | lds_);
  uint32_t b0 = lds32(tb0(s1) | lds_), b1 = lds32(tb1(s0) | lds_), b2 = lds32(tb2(s3) | lds_), b3 = lds32(tb3(s2) | lds_);
  uint32_t c0 = lds32(tb0(s2) | lds_), c1 = lds32(tb1(s1) | lds_), c2 = lds32(tb2(s0) | lds_), c3 = lds32(tb3(s3) | lds_);
  uint32_t d0 = lds32(tb0(s3) | lds_), d1 = lds32(tb1(s2) | lds_), d2 = lds32(tb2(s1) | lds_), d3 = lds32(tb3(s0) | lds_);
  s0 = xor3(__builtin_amdgcn_perm(a1, a0, 0x0c0c0400u), __builtin_amdgcn_perm(a3, a2, 0x04000c0cu), k.w[40]);
  s1 = xor3(__builtin_amdgcn_perm(b1, b0, 0x0c0c0400u), __builtin_amdgcn_perm(b3, b2, 0x04000c0cu), k.w[41]);
  s2 = xor3(__builtin_amdgcn_perm(c1, c0, 0x0c0c0400u), __builtin_amdgcn_perm(c3, c2, 0x04000c0cu), k.w[42]);
  s3 = xor3(__builtin_amdgcn_perm(d1, d0, 0x0c0c0400u), __builtin_amdgcn_perm(d3, d2, 0x04000c0cu), k.w[43]);
}

// Stage a 256-word table 32-way replicated at `base` (Td0 or the inverse S-box as words).
__device__ __forceinline__ void stage_rep32(const uint32_t* __restrict__ t, uint32_t base) {
  for (uint32_t i = threadIdx.x; i < 256u * 32u; i += blockDim.x)
    lds_st32(base + i * 4u, t[i >> 5]);
}

// X · P with the 64 KiB byte table of P at LDS offset 0 (16 ds_read_b128, XORs paired
// through v_bitop3).
__device__ __forceinline__ uint32_t gbyte_off(u32x4 x, int p) {
  const uint32_t w = x[p >> 2];
  const int sh = 8 * (p & 3);
  return ((sh == 0 ? (w << 4) : (w >> (sh - 4))) & 0xff0u) + (uint32_t)p * 4096u;
}
__device__ __forceinline__ u32x4 gmul_byte(u32x4 x) {
  u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int p = 0; p < 16; p += 2) {
    const u32x4 e1 = lds128(gbyte_off(x, p));
    const u32x4 e2 = lds128(gbyte_off(x, p + 1));
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = xor3(r[c], e1[c], e2[c]);
  }
  return r;
}

// X · P with an 8 KiB nibble table of P at LDS byte offset `tb` (multiple of 8 KiB).
__device__ __forceinline__ u32x4 gmul_nib(u32x4 x, uint32_t tb) {
  u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const uint32_t w = x[p >> 2];
    const int sh = 8 * (p & 3);
    const uint32_t hi = (w >> sh) & 0xf0u;                              // (v >> 4) * 16
    const uint32_t lo = (sh == 0 ? (w << 4) : (w >> (sh - 4))) & 0xf0u;  // (v & 15) * 16
    const u32x4 e1 = lds128((hi | tb) + (uint32_t)p * 512u);
    const u32x4 e2 = lds128((lo | tb) + (uint32_t)p * 512u + 256u);
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = xor3(r[c], e1[c], e2[c]);
  }
  return r;
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

__device__ __forceinline__ u32x4 shfl_xor4(u32x4 v, int m) {
  u32x4 r;
  r[0] = __shfl_xor((int)v[0], m);
  r[1] = __shfl_xor((int)v[1], m);
  r[2] = __shfl_xor((int)v[2], m);
  r[3] = __shfl_xor((int)v[3], m);
  return r;
}

// Stage the 32-way replicated Te0 image at LDS offset tbase (all threads of the block help).
__device__ __forceinline__ void stage_te0(const uint32_t* __restrict__ te0, uint32_t tbase) {
  for (uint32_t i = threadIdx.x; i < 256u * 32u; i += blockDim.x)
    lds_st32(tbase + i * 4u, te0[i >> 5]);
}

__device__ __forceinline__ void stage_copy(const u32x4* __restrict__ src, uint32_t dst_off, uint32_t n16) {
  for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x)
    lds_st128(dst_off + i * 16u, src[i]);
}

// Partial-block helpers (bytes [0, n) of a 16-byte block at an arbitrary address).
__device__ __forceinline__ u32x4 load_partial(const uint8_t* p, uint32_t n) {
  uint32_t b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = (uint32_t)i < n ? p[i] : 0u;
  u32x4 r;
#pragma unroll
  for (int c = 0; c < 4; ++c) r[c] = b[4 * c] | (b[4 * c + 1] << 8) | (b[4 * c + 2] << 16) | (b[4 * c + 3] << 24);
  return r;
}
__device__ __forceinline__ void store_partial(uint8_t* p, u32x4 v, uint32_t n) {
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((uint32_t)i < n) p[i] = (uint8_t)(v[i >> 2] >> (8 * (i & 3)));
}
__device__ __forceinline__ u32x4 mask_bytes(u32x4 v, uint32_t n) {  // keep bytes [0, n)
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int lo = 4 * c;
    uint32_t m = (n >= (uint32_t)(lo + 4)) ? 0xffffffffu : (n <= (uint32_t)lo ? 0u : (0xffffffffu >> (8 * (lo + 4 - n))));
    v[c] &= m;
  }
  return v;
}

}  // namespace dev
}  // namespace cmpi
