// keysetup_kernels.hpp — per-key setup on the device (gfx950): the work EVP_AEAD_CTX_new does
// inside BoringSSL (key schedule + GHASH precomputation), run as one small kernel so that a
// CryptMPI 602 per-message sub-key K' = AES_K(V) (send.c:572-600, recv.c:549-576) is derived,
// expanded and tabled without a host round trip, ordered on the caller's stream.
//
// Output layout = DevTables in cmpi_aead.hip: keys[0..43] round keys (folded), keys[48..51] H;
// byte tables of H, H^2, H^4 ([v][p], 4096 x 16 B each) and nibble tables of H^1..H^4
// (512 x 16 B each) — bit-identical to gf128_host.hpp's host builders.
#pragma once
#include "aes_device.hpp"

namespace cmpi {
namespace dev {

struct KeysetupArgs {
  RoundKeys base;       // mode 1: keys of K (the master key, folded) used to derive K' = AES_K(V)
  uint32_t v[4];        // mode 0: K' itself; mode 1: V
  uint32_t mode;
  const uint32_t* te0;  // Te0 (global)
  uint32_t* keys;       // out: [0..43] round keys of K', [48..51] H = E_K'(0)
  u32x4* htab;          // out: 3 byte tables (H, H^2, H^4)
  u32x4* ntab;          // out: 4 nibble tables (H^1..H^4)
};

// GCM-order field element as (hi, lo) big-endian halves of its 16 memory bytes.
__device__ __forceinline__ void gf_split(u32x4 x, uint64_t& h, uint64_t& l) {
  h = ((uint64_t)__builtin_bswap32(x[0]) << 32) | __builtin_bswap32(x[1]);
  l = ((uint64_t)__builtin_bswap32(x[2]) << 32) | __builtin_bswap32(x[3]);
}
__device__ __forceinline__ u32x4 gf_join(uint64_t h, uint64_t l) {
  return u32x4{__builtin_bswap32((uint32_t)(h >> 32)), __builtin_bswap32((uint32_t)h),
               __builtin_bswap32((uint32_t)(l >> 32)), __builtin_bswap32((uint32_t)l)};
}

// LDS: AES row image @0 (64 KiB), basis chains Q_j[i] = P_j · x^i (j = 0..3 for H^1..H^4,
// i = 0..127) @64K (8 KiB), S-box bytes @72K (256 words).
constexpr uint32_t kKsBasis = 65536u;
constexpr uint32_t kKsSbox = 73728u;
constexpr uint32_t kKsLds = 74752u;

__global__ __launch_bounds__(256) void gcm_keysetup_kernel(KeysetupArgs a) {
  stage_rows(a.te0, 0u);
  for (uint32_t x = threadIdx.x; x < 256u; x += blockDim.x) lds_st32(kKsSbox + 4u * x, (a.te0[x] >> 8) & 0xffu);
  __syncthreads();
  const RowLanes rl = row_lanes(0u);
  // every lane computes the (tiny) key schedule redundantly: no broadcast needed
  uint32_t k0 = a.v[0], k1 = a.v[1], k2 = a.v[2], k3 = a.v[3];
  if (a.mode == 1u) aes128_enc(a.base, rl, k0, k1, k2, k3);  // K' = AES_K(V)
  RoundKeys rk;
  rk.w[0] = k0;
  rk.w[1] = k1;
  rk.w[2] = k2;
  rk.w[3] = k3;
  uint32_t rcon = 1u;
#pragma unroll
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk.w[i - 1];
    if ((i & 3) == 0) {
      t = (t >> 8) | (t << 24);  // RotWord on little-endian words
      t = lds32(kKsSbox + 4u * (t & 0xffu)) | (lds32(kKsSbox + 4u * ((t >> 8) & 0xffu)) << 8) |
          (lds32(kKsSbox + 4u * ((t >> 16) & 0xffu)) << 16) | (lds32(kKsSbox + 4u * (t >> 24)) << 24);
      t ^= rcon;
      rcon = (rcon << 1) ^ ((rcon & 0x80u) ? 0x11bu : 0u);
    }
    rk.w[i] = rk.w[i - 4] ^ t;
  }
  const RoundKeys fk = fold_keys(rk);  // stored folded: the GCM kernels load them as they are
  uint32_t h0 = 0u, h1 = 0u, h2 = 0u, h3 = 0u;
  aes128_enc(fk, rl, h0, h1, h2, h3);  // H = E_K'(0^128)
  const u32x4 H = u32x4{h0, h1, h2, h3};
  if (threadIdx.x < 44u) a.keys[threadIdx.x] = fk.w[threadIdx.x];
  if (threadIdx.x == 0) {
    a.keys[48] = h0;
    a.keys[49] = h1;
    a.keys[50] = h2;
    a.keys[51] = h3;
  }
  // basis chains: lane j < 4 walks P_j = H^(j+1) through P_j · x^i, i = 0..127
  if (threadIdx.x < 4u) {
    u32x4 P = H;
    for (uint32_t j = 0; j < threadIdx.x; ++j) P = gmul_generic(P, H);
    uint64_t ph, pl;
    gf_split(P, ph, pl);
    for (uint32_t i = 0; i < 128u; ++i) {
      lds_st128(kKsBasis + (threadIdx.x * 128u + i) * 16u, gf_join(ph, pl));
      const uint64_t lsb = 0 - (pl & 1u);
      pl = (pl >> 1) | (ph << 63);
      ph = (ph >> 1) ^ (0xE100000000000000ULL & lsb);
    }
  }
  __syncthreads();
  // byte tables: entry (v, p) of P = XOR over set bits k of v of P · x^(8p + 7 - k)
  const uint32_t bsel[3] = {0u, 1u, 3u};  // H, H^2, H^4
  for (uint32_t e = threadIdx.x; e < 3u * 4096u; e += blockDim.x) {
    const uint32_t t = e >> 12, v = (e >> 4) & 255u, p = e & 15u;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; k < 8u; ++k)
      if (v & (1u << k)) acc ^= lds128(kKsBasis + (bsel[t] * 128u + 8u * p + 7u - k) * 16u);
    a.htab[e] = acc;
  }
  // nibble tables: entry (2p + half, v): half 0 = byte p holds v << 4, half 1 = byte p holds v
  for (uint32_t e = threadIdx.x; e < 4u * 512u; e += blockDim.x) {
    const uint32_t t = e >> 9, row = (e >> 4) & 31u, v = e & 15u;
    const uint32_t p = row >> 1, shift = (row & 1u) ? 0u : 4u;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; k < 4u; ++k)
      if (v & (1u << k)) acc ^= lds128(kKsBasis + (t * 128u + 8u * p + 7u - (k + shift)) * 16u);
    a.ntab[e] = acc;
  }
}

// pw[k] = H^(k*G), k < n (multi-segment GCM combine weights) for a device-keyed context.
__global__ __launch_bounds__(64) void gcm_powers_kernel(const uint32_t* keys, uint32_t G, uint32_t n, u32x4* pw) {
  const u32x4 H = u32x4{keys[48], keys[49], keys[50], keys[51]};
  for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
    // square-and-multiply over the exponent k*G
    uint64_t e = (uint64_t)k * G;
    u32x4 r = {0x80u, 0u, 0u, 0u};  // 1 = x^0 (byte 0 bit 7)
    u32x4 b = H;
    while (e) {
      if (e & 1u) r = gmul_generic(r, b);
      b = gmul_generic(b, b);
      e >>= 1;
    }
    pw[k] = r;
  }
}

}  // namespace dev
}  // namespace cmpi
