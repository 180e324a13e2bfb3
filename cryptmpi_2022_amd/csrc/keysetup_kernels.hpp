// keysetup_kernels.hpp — per-key setup on the device (gfx950): the work EVP_AEAD_CTX_new does
// inside BoringSSL (key schedule + GHASH precomputation), run as one small kernel so that a
// CryptMPI 602 per-message sub-key K' = AES_K(V) (send.c:572-600, recv.c:549-576) is derived,
// expanded and tabled without a host round trip, ordered on the caller's stream.
//
// Output layout = DevTables in cmpi_aead.hip: keys[0..43] round keys (folded), keys[48..51] H,
// H^(2^i), basis chains; then gcm_tables_kernel expands byte tables of H, H^2, H^4 ([v][p],
// 4096 x 16 B each) and the nibble tables of H^1,2,3,4,8,12,16,32,48,64 (512 x 16 B each) —
// bit-identical to gf128_host.hpp's host builders.  Two launches.
#pragma once
#include "aes_device.hpp"

namespace cmpi {
namespace dev {

struct KeysetupArgs {
  RoundKeys base;       // mode 1: keys of K (the master key, folded) used to derive K' = AES_K(V)
  uint32_t v[4];        // mode 0: K' itself; mode 1: V
  uint32_t mode;
  const uint32_t* te0;  // Te0 (global)
  const u32x4* sqmat;   // [i-1][k] = (x^k)^(2^i), i = 1..31, k < 128: columns of the linear maps
                        // X -> X^(2^i) (key independent, host-built once per process)
  uint32_t* keys;       // out: [0..43] round keys of K' (folded), [48..51] H = E_K'(0)
  u32x4* h2pow;         // out: H^(2^i), i < 32
  u32x4* chains;        // out: basis chains P·x^i (i < 128) of P = H, H^2, H^3, H^4, H^8, H^16, H^32, H^64,
                        //      H^12, H^48
};

// The 10 chained multipliers: index -> exponent of H.
constexpr uint32_t kKsChains = 10;
__host__ __device__ constexpr uint32_t ks_chain_exp(uint32_t j) {
  return j == 0 ? 1u : j == 1 ? 2u : j == 2 ? 3u : j == 3 ? 4u : j == 4 ? 8u : j == 5 ? 16u : j == 6 ? 32u
       : j == 7 ? 64u : j == 8 ? 12u : 48u;
}

// LDS (dynamic only: offsets are addresses): AES row image @0 (64 KiB), S-box bytes @64K
// (256 words), then 10 slots: H^(2^i) for i < 7, H^3 (slot 7), H^12 (slot 8), H^48 (slot 9).
constexpr uint32_t kKsRows = 0u;
constexpr uint32_t kKsSbox = 65536u;
constexpr uint32_t kKsPow = kKsSbox + 1024u;
constexpr uint32_t kKsLds = kKsPow + 10u * 16u;

// bit k (coefficient of x^k) of a memory-order element
__device__ __forceinline__ uint32_t gf_bit(u32x4 x, uint32_t k) {
  return (x[k >> 5] >> (8u * ((k >> 3) & 3u) + 7u - (k & 7u))) & 1u;
}

// One workgroup of 256: key schedule of K' (= AES_K(V) in mode 1), H = E_K'(0); then, with no
// serial chain longer than one step: H^(2^i), i = 1..31, as XORs of the columns of the squaring
// maps (8 threads per i, 16 columns each); H^3 = H^2 · H by one wave (lane q holds H·x^q and
// H·x^(q+64)); and the basis chains P · x^i of the 8 multipliers, one gf_mulx_pow per entry.
__global__ __launch_bounds__(256) void gcm_keysetup_kernel(KeysetupArgs a) {
  const uint32_t t = threadIdx.x;
  // the 16 squaring-map columns this thread XORs for H^(2^i) depend on the key only through which
  // of them are selected: they are requested first, so their latency overlaps the staging and
  // the two AES encryptions below
  u32x4 cols[16];
  const uint32_t sq_i = 1u + (t >> 3), sq_k0 = 16u * (t & 7u);
  if (t < 248u) {
    const u32x4* col = a.sqmat + (sq_i - 1u) * 128u + sq_k0;
#pragma unroll
    for (uint32_t c = 0; c < 16u; ++c) cols[c] = col[c];
  }
  stage_rows(a.te0, kKsRows);
  for (uint32_t x = threadIdx.x; x < 256u; x += blockDim.x) lds_st32(kKsSbox + 4u * x, (a.te0[x] >> 8) & 0xffu);
  __syncthreads();
  const RowLanes rl = row_lanes(kKsRows);
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
  if (t < 44u) a.keys[t] = fk.w[t];
  if (t == 0u) {
    a.keys[48] = h0;
    a.keys[49] = h1;
    a.keys[50] = h2;
    a.keys[51] = h3;
    a.h2pow[0] = H;
    lds_st128(kKsPow, H);
  }
  // H^(2^i) = Sq^i(H) = XOR over the set bits k of H of column k of Sq^i
  if (t < 248u) {
    const uint32_t i = sq_i, k0c = sq_k0;
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t c = 0; c < 16u; ++c)
      if (gf_bit(H, k0c + c)) acc ^= cols[c];
    acc ^= shfl_xor4(acc, 1);
    acc ^= shfl_xor4(acc, 2);
    acc ^= shfl_xor4(acc, 4);
    if ((t & 7u) == 0u) {
      a.h2pow[i] = acc;
      if (i < 7u) lds_st128(kKsPow + 16u * i, acc);
    }
  }
  __syncthreads();
  // products by one wave each, lane q contributing A·x^q [bit q of B] and A·x^(q+64) [bit q+64]:
  // wave 0 H^3 = H^2 · H, wave 1 H^12 = H^8 · H^4, wave 2 H^48 = H^32 · H^16
  if (t < 192u) {
    const uint32_t w = t >> 6, q = t & 63u;
    const u32x4 A = lds128(kKsPow + 16u * (w == 0u ? 0u : w == 1u ? 2u : 4u));
    const u32x4 B = lds128(kKsPow + 16u * (w == 0u ? 1u : w == 1u ? 3u : 5u));
    uint64_t ah, al, bh, bl;
    gf_split(A, ah, al);
    bh = ah;
    bl = al;
    gf_mulx_pow(ah, al, q);
    gf_mulx_pow(bh, bl, q + 64u);
    u32x4 acc = {0u, 0u, 0u, 0u};
    if (gf_bit(B, q)) acc ^= gf_join(ah, al);
    if (gf_bit(B, q + 64u)) acc ^= gf_join(bh, bl);
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) acc ^= shfl_xor4(acc, m);
    if (q == 0u) lds_st128(kKsPow + 16u * (7u + w), acc);
  }
  __syncthreads();
  // basis chains: entry (j, i) = P_j · x^i, P_j = H, H^2, H^3, H^4, H^8, H^16, H^32, H^64, H^12, H^48
  for (uint32_t e = t; e < kKsChains * 128u; e += blockDim.x) {
    const uint32_t j = e >> 7, i = e & 127u;
    const uint32_t slot = j == 2u ? 7u : j >= 8u ? j : (j < 2u ? j : j - 1u);
    uint64_t ph, pl;
    gf_split(lds128(kKsPow + 16u * slot), ph, pl);
    gf_mulx_pow(ph, pl, i);
    a.chains[e] = gf_join(ph, pl);
  }
}

// Table expansion, one entry per thread (grid over every entry): entry (v, p) of a byte table
// of P = XOR over set bits k of v of P · x^(8p + 7 - k); nibble entry (2p + h, v) likewise over
// the 4 bits of v at x^(8p + 7 - k - (h ? 0 : 4)).  Outputs: byte tables of H, H^2, H^4 (GCM
// lane groups' Horner multipliers) and the ten nibble tables of H^1,2,3,4,8,12,16,32,48,64
// (gcm_flow_kernel; the lane groups' weights H^1..H^3 are the first three).
struct TablesArgs {
  const u32x4* chains;  // 10 x 128 (ks_chain_exp order)
  u32x4* htab;          // 3 x 4096: H, H^2, H^4
  u32x4* fnib;          // 10 x 512: H^1, 2, 3, 4, 8, 12, 16, 32, 48, 64
};
constexpr uint32_t kFlowNib = 10;
constexpr uint32_t kTabEntries = 3u * 4096u + kFlowNib * 512u;
// exponent of H of nibble table f, and its basis chain
__host__ __device__ constexpr uint32_t flow_nib_exp(uint32_t f) {
  return f == 0 ? 1u : f == 1 ? 2u : f == 2 ? 3u : f == 3 ? 4u : f == 4 ? 8u : f == 5 ? 12u : f == 6 ? 16u
       : f == 7 ? 32u : f == 8 ? 48u : 64u;
}
__host__ __device__ constexpr uint32_t flow_nib_chain(uint32_t f) {
  return f < 5u ? f : f == 5u ? 8u : f == 6u ? 5u : f == 7u ? 6u : f == 8u ? 9u : 7u;
}

__global__ __launch_bounds__(256) void gcm_tables_kernel(TablesArgs a) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kTabEntries) return;
  // byte tables: 0..2 -> chain 0 (H), 1 (H^2), 3 (H^4)
  if (e < 3u * 4096u) {
    const uint32_t t = e >> 12, v = (e >> 4) & 255u, p = e & 15u;
    const uint32_t ch = t == 0 ? 0u : t == 1 ? 1u : 3u;
    const u32x4* c = a.chains + ch * 128u + 8u * p + 7u;
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (v & (1u << k)) acc ^= *(c - k);
    a.htab[e] = acc;
    return;
  }
  const uint32_t f = e - 3u * 4096u;
  const uint32_t t = f >> 9, row = (f >> 4) & 31u, v = f & 15u, p = row >> 1, sh = (row & 1u) ? 0u : 4u;
  const u32x4* c = a.chains + flow_nib_chain(t) * 128u + 8u * p + 7u - sh;
  u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (v & (1u << k)) acc ^= *(c - k);
  a.fnib[f] = acc;
}

}  // namespace dev
}  // namespace cmpi
