// ctr_kernels.hpp — AES-128-CTR keystream (+XOR) and AES-128-ECB over device buffers (gfx950).
//
// CTR: block j uses counter (ctr_hi:ctr_lo) + j as a 128-bit big-endian integer — the
// EVP_aes_128_ctr increment behind EVP_EncryptUpdate in CryptMPI's 700/702 paths
// (MV/src/mpi/pt2pt/send.c:985-1008, :1716-1727, :1805-1808; recv.c:869-937, :1187-1220).
// The keystream-only variant is generateCommonEncMask's E_K(IV_A + c) over zeros
// (send.c:1162-1266).  ECB: EVP_EncryptUpdate(ctx_enc, …) for the 602 sub-key (send.c:583).
// Each thread owns two 16-byte blocks per iteration (ILP for the LDS pipe), consecutive lanes
// own consecutive blocks (1 KiB coalesced per wave-instruction).
#pragma once
#include "aes_device.hpp"

namespace cmpi {
namespace dev {

struct CtrArgs {
  const uint8_t* in;  // null for keystream-only
  uint8_t* out;
  uint64_t n;         // bytes (keystream: nblocks*16)
  uint64_t nblk;      // ceil(n/16)
  uint64_t ctr_hi, ctr_lo;  // counter block as two big-endian halves
  const uint32_t* te0;
  uint32_t sched;  // bit 1: rotate wave priority per step
  RoundKeys rk;
};

__device__ __forceinline__ void ctr_words(uint64_t hi, uint64_t lo, uint64_t j, uint32_t& w0, uint32_t& w1,
                                          uint32_t& w2, uint32_t& w3) {
  const uint64_t l2 = lo + j;
  const uint64_t h2 = hi + (l2 < lo ? 1u : 0u);
  w0 = __builtin_bswap32((uint32_t)(h2 >> 32));
  w1 = __builtin_bswap32((uint32_t)h2);
  w2 = __builtin_bswap32((uint32_t)(l2 >> 32));
  w3 = __builtin_bswap32((uint32_t)l2);
}

// full input block j (prefetched before the AES of its step), zeros otherwise
// Unconditional, clamped: blocks outside [0, nfull) read block 0 (value ignored by ctr_emit);
// nfull == 0 (no full block at all) reads the Te0 table.
template <bool XOR_IN>
__device__ __forceinline__ u32x4 ctr_load(const CtrArgs& a, uint64_t v, uint64_t phase, uint64_t nfull) {
  if (!XOR_IN) return u32x4{0u, 0u, 0u, 0u};
  const uint64_t j = v - phase;  // wraps for v < phase
  const uint8_t* base = nfull ? a.in : reinterpret_cast<const uint8_t*>(a.te0);
  return *reinterpret_cast<const u32x4a*>(base + (j < nfull ? j : 0u) * 16u);
}

template <bool XOR_IN>
__device__ __forceinline__ void ctr_emit(const CtrArgs& a, uint64_t j, u32x4 ks, u32x4 v) {
  const uint64_t off = j * 16u;
  if (off + 16u <= a.n) {
    *reinterpret_cast<u32x4a*>(a.out + off) = XOR_IN ? v ^ ks : ks;
  } else {  // the last block of a length that is not a multiple of 16: its bytes only
    const uint32_t rem = (uint32_t)(a.n - off);
    store_partial(a.out + off, XOR_IN ? load_partial(a.in + off, rem) ^ ks : ks, rem);
  }
}

// LDS: AES row image @0 (64 KiB) -> two 1024-thread blocks per CU.
// Wave step = 64 consecutive counters in one 64-aligned counter window (lane = offset), so each
// step's counters share bytes 0..14 and the round-1/2 cache is refilled wave-uniformly once
// every 4 steps.  Each wave owns a contiguous run of steps; loads/stores are 1 KiB coalesced.
#ifndef CMPI_CTR_PREFETCH
#define CMPI_CTR_PREFETCH 1
#endif
template <bool XOR_IN>
__global__ __launch_bounds__(1024, 8) void ctr_kernel(CtrArgs a) {
  stage_rows(a.te0, 0u);
  __syncthreads();
  const RoundKeys& rk = a.rk;  // folded by the host
  const RowLanes rl = row_lanes(0u);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t phase = a.ctr_lo & 63u;        // counter(v) = (ctr & ~63) + v, j = v - phase
  const uint64_t lo_base = a.ctr_lo & ~63ull;
  const uint64_t nsteps = (a.nblk + phase + 63u) / 64u;
  const uint64_t wpb = blockDim.x >> 6;
  const uint64_t waves = (uint64_t)gridDim.x * wpb;
  const uint64_t wave = (uint64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
  const uint64_t per = (nsteps + waves - 1u) / waves;
  const uint64_t st0 = wave * per;
  const uint64_t st1 = min(st0 + per, nsteps);
  CtrCache cc;
  uint64_t win = ~0ull;
  const uint64_t nfull = a.n / 16u;
  // the next step's block is loaded right after this step's store: a whole step of AES covers it
  // (CMPI_CTR_PREFETCH 2: two steps ahead, so a step's XOR never waits on the previous store)
  u32x4 in_cur = ctr_load<XOR_IN>(a, st0 * 64u + lane, phase, nfull);
  u32x4 in_nxt = CMPI_CTR_PREFETCH >= 2 ? ctr_load<XOR_IN>(a, st0 * 64u + 64u + lane, phase, nfull) : u32x4{0u, 0u, 0u, 0u};
  for (uint64_t st = st0; st < st1; ++st) {
    if (a.sched & 2u) rotate_prio((uint32_t)st);
    const uint64_t v = st * 64u + lane;
    uint32_t w0, w1, w2, w3;
    ctr_words(a.ctr_hi, lo_base, v, w0, w1, w2, w3);
    const uint64_t key = ((a.ctr_lo & 0xc0u) + st * 64u) >> 8;  // wave-uniform
    if (key != win) {
      ctr_cache_fill(rk, rl, w0, w1, w2, w3, cc);
      win = key;
    }
    uint32_t s0, s1, s2, s3;
    aes128_enc_ctr(rk, rl, cc, w3, s0, s1, s2, s3);
    if (v >= phase && v - phase < a.nblk) ctr_emit<XOR_IN>(a, v - phase, u32x4{s0, s1, s2, s3}, in_cur);
    if constexpr (CMPI_CTR_PREFETCH >= 2) {
      in_cur = in_nxt;
      in_nxt = ctr_load<XOR_IN>(a, v + 128u, phase, nfull);
    } else {
      in_cur = ctr_load<XOR_IN>(a, v + 64u, phase, nfull);
    }
  }
}

struct EcbArgs {
  const uint8_t* in;
  uint8_t* out;
  uint64_t nblk;
  const uint32_t* te0;
  RoundKeys rk;
};

__global__ __launch_bounds__(1024) void ecb_kernel(EcbArgs a) {
  stage_rows(a.te0, 0u);
  __syncthreads();
  const RowLanes lb = row_lanes(0u);
  const RoundKeys& rk = a.rk;  // folded by the host
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.nblk; j += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = *reinterpret_cast<const u32x4a*>(a.in + 16u * j);
    uint32_t s0 = v[0], s1 = v[1], s2 = v[2], s3 = v[3];
    aes128_enc(rk, lb, s0, s1, s2, s3);
    *reinterpret_cast<u32x4a*>(a.out + 16u * j) = u32x4{s0, s1, s2, s3};
  }
}

}  // namespace dev
}  // namespace cmpi

namespace cmpi {
namespace dev {

// out = a ^ b over n bytes, any byte alignment (mask-ring consumption, send.c:1300-1330 /
// recv.c:975-1002).  HBM-bound: 16 B per lane per step, grid-stride; the last n % 16 bytes
// are done bytewise by the lanes that own them.
__global__ __launch_bounds__(256) void xor_bytes_kernel(uint8_t* out, const uint8_t* a, const uint8_t* b, uint64_t n) {
  const uint64_t nv = n / 16u;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const u32x4 x = *reinterpret_cast<const u32x4a*>(a + 16u * i);
    const u32x4 y = *reinterpret_cast<const u32x4a*>(b + 16u * i);
    *reinterpret_cast<u32x4a*>(out + 16u * i) = x ^ y;
  }
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n - 16u * nv) out[16u * nv + t] = a[16u * nv + t] ^ b[16u * nv + t];
}

// Streaming device copy (the measured HBM peak of bench.py's roofline, cmpi_debug_copy): 16 B
// per lane, one load in flight per lane, plain loads and stores, a grid-stride loop run by 1 024
// workgroups of 256 threads (4 per CU).  The fastest of 80 forms measured on 1 GiB
// (tools/probe/copy_probe*.hip, profiles/r05e_copy_probe.jsonl, r05u_copy_probe2.jsonl: 5.71 TB/s
// read + write; 2 loads in flight, non-temporal stores, per-workgroup chunks, 512 / 1 024-thread
// workgroups and 256 - 16 384 workgroups all 1-15 % slower — the round's first form, four
// non-temporal loads per lane over 4 096 workgroups, ran 4.3 TB/s).
__global__ __launch_bounds__(256) void copy16_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src, uint64_t nv) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) dst[i] = src[i];
}

}  // namespace dev
}  // namespace cmpi
