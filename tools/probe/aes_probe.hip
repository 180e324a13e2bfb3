// aes_probe.hip — cost of the T-table AES-128 block on gfx950 in isolation (no HBM, no GHASH):
// SIMD cycles per block, from the in-kernel clock, for the forms the engine could use:
//   0  the engine's rounds (csrc/aes_device.hpp: [Te0|Te1] row image, Te2/Te3 by rotl16)
//   1  four tables: a second [Te2|Te3] row image (128 KiB of rows), no rotates
//   2  the engine's rounds, two independent blocks per lane (aes128_enc2)
// at 4 waves per SIMD (one 1024-thread workgroup per CU) and, where the LDS allows, 8.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../cryptmpi_2022_amd/csrc -o aes_probe aes_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "aes_device.hpp"
#include "aes_tables.hpp"

using namespace cmpi::dev;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int kBlocks = 256;  // blocks per lane

__device__ __forceinline__ void enc_round4(uint32_t la, uint32_t lb, uint32_t m, uint32_t& s0, uint32_t& s1,
                                           uint32_t& s2, uint32_t& s3, uint32_t k0, uint32_t k1, uint32_t k2,
                                           uint32_t k3) {
  // image A (@64K) = [Te0|Te1], image B (@0) = [Te2|Te3]: la = A lanes (Te0 half), lb = B lanes (Te2 half)
  const uint32_t la1 = la | 128u, lb1 = lb | 128u;
  const uint32_t a0 = lds32(ra<0>(s0, la)), a1 = lds32(ra<1>(s1, la1, m)), a2 = lds32(ra<2>(s2, lb)), a3 = lds32(ra<3>(s3, lb1));
  const uint32_t b0 = lds32(ra<0>(s1, la)), b1 = lds32(ra<1>(s2, la1, m)), b2 = lds32(ra<2>(s3, lb)), b3 = lds32(ra<3>(s0, lb1));
  const uint32_t c0 = lds32(ra<0>(s2, la)), c1 = lds32(ra<1>(s3, la1, m)), c2 = lds32(ra<2>(s0, lb)), c3 = lds32(ra<3>(s1, lb1));
  const uint32_t d0 = lds32(ra<0>(s3, la)), d1 = lds32(ra<1>(s0, la1, m)), d2 = lds32(ra<2>(s1, lb)), d3 = lds32(ra<3>(s2, lb1));
  s0 = xor3(a0, a1, xor3(a2, a3, k0));
  s1 = xor3(b0, b1, xor3(b2, b3, k1));
  s2 = xor3(c0, c1, xor3(c2, c3, k2));
  s3 = xor3(d0, d1, xor3(d2, d3, k3));
}

// SDWA lookup address: the lane constant lc (bytes 0, 2, 3) stays in A; byte 1 <- byte R of s
template <int R>
__device__ __forceinline__ uint32_t sdwa_addr(uint32_t& A, uint32_t s) {
  if constexpr (R == 0) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(A) : "v"(s));
  if constexpr (R == 1) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(A) : "v"(s));
  if constexpr (R == 2) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(A) : "v"(s));
  if constexpr (R == 3) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(A) : "v"(s));
  return A;
}
struct SdwaRegs {
  uint32_t a[16];
};
__device__ __forceinline__ void enc_round_sdwa(SdwaRegs& A, uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                               uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  // A.a[4c + r]: lane constant of the lookup of row r of column c (Te0 half for r even, Te1 odd)
  const uint32_t a0 = lds32(sdwa_addr<0>(A.a[0], s0)), a1 = lds32(sdwa_addr<1>(A.a[1], s1)), a2 = lds32(sdwa_addr<2>(A.a[2], s2)), a3 = lds32(sdwa_addr<3>(A.a[3], s3));
  const uint32_t b0 = lds32(sdwa_addr<0>(A.a[4], s1)), b1 = lds32(sdwa_addr<1>(A.a[5], s2)), b2 = lds32(sdwa_addr<2>(A.a[6], s3)), b3 = lds32(sdwa_addr<3>(A.a[7], s0));
  const uint32_t c0 = lds32(sdwa_addr<0>(A.a[8], s2)), c1 = lds32(sdwa_addr<1>(A.a[9], s3)), c2 = lds32(sdwa_addr<2>(A.a[10], s0)), c3 = lds32(sdwa_addr<3>(A.a[11], s1));
  const uint32_t d0 = lds32(sdwa_addr<0>(A.a[12], s3)), d1 = lds32(sdwa_addr<1>(A.a[13], s0)), d2 = lds32(sdwa_addr<2>(A.a[14], s1)), d3 = lds32(sdwa_addr<3>(A.a[15], s2));
  s0 = xor3(a0, a1, rotl16(xor3(a2, a3, k0)));
  s1 = xor3(b0, b1, rotl16(xor3(b2, b3, k1)));
  s2 = xor3(c0, c1, rotl16(xor3(c2, c3, k2)));
  s3 = xor3(d0, d1, rotl16(xor3(d2, d3, k3)));
}

template <int VAR>
__global__ void probe(const uint32_t* te0, RoundKeys k, uint32_t* out, unsigned long long* cyc) {
  stage_rows(te0, 65536u);
  if constexpr (VAR == 1) {  // [Te2|Te3] rows at 0: row x = [rotl16 Te0 x32 | rotl24 Te0 x32]
    for (uint32_t i = threadIdx.x; i < 256u * 64u; i += blockDim.x) {
      const uint32_t x = i >> 6, j = i & 63u;
      const uint32_t t = te0[x];
      lds_st32(x * 256u + j * 4u, j < 32u ? rotl16(t) : __builtin_amdgcn_alignbit(t, t, 8));
    }
  }
  __syncthreads();
  const RowLanes L = row_lanes(65536u);
  const uint32_t lbB = (threadIdx.x & 31u) << 2;
  SdwaRegs SA;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    SA.a[i] = (i & 1) ? L.l1 : L.l0;
    asm volatile("" : "+v"(SA.a[i]));
  }
  uint32_t s0 = threadIdx.x * 0x9e3779b9u, s1 = blockIdx.x, s2 = s0 ^ 0x1234567u, s3 = ~s0;
  uint32_t t0 = s0 ^ 1u, t1 = s1 ^ 2u, t2 = s2 ^ 3u, t3 = s3 ^ 4u;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int b = 0; b < kBlocks; ++b) {
    if constexpr (VAR == 0) {
      aes128_enc(k, L, s0, s1, s2, s3);
    } else if constexpr (VAR == 1) {
      s0 ^= k.w[0];
      s1 ^= k.w[1];
      s2 ^= k.w[2];
      s3 ^= k.w[3];
#pragma unroll
      for (int r = 1; r < 10; ++r) enc_round4(L.l0, lbB, L.m, s0, s1, s2, s3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3]);
      enc_last(L, s0, s1, s2, s3, k.w[40], k.w[41], k.w[42], k.w[43]);
    } else if constexpr (VAR == 3) {
      s0 ^= k.w[0];
      s1 ^= k.w[1];
      s2 ^= k.w[2];
      s3 ^= k.w[3];
#pragma unroll
      for (int r = 1; r < 10; ++r) enc_round_sdwa(SA, s0, s1, s2, s3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3]);
      enc_last(L, s0, s1, s2, s3, k.w[40], k.w[41], k.w[42], k.w[43]);
    } else {
      if (b & 1) continue;
      aes128_enc2(k, L, s0, s1, s2, s3, t0, t1, t2, t3);
    }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ t0 ^ t1 ^ t2 ^ t3;
  if ((threadIdx.x & 63u) == 0u) {
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    cyc[2 * w] = c1 - c0;
    cyc[2 * w + 1] = r1 - r0;
  }
}

template <int VAR>
int run(const char* name, int wps, const uint32_t* te0, const RoundKeys& k, uint32_t* out, unsigned long long* cyc,
        int ncu) {
  const int threads = 1024;
  const int blocks = ncu * (wps / 4);
  const size_t lds = VAR == 1 ? 131072 : 65536;
  CK(hipFuncSetAttribute((const void*)probe<VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<VAR>, dim3(blocks), dim3(threads), lds, 0, te0, k, out, cyc);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(probe<VAR>, dim3(blocks), dim3(threads), lds, 0, te0, k, out, cyc);
  CK(hipEventRecord(e1));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const int nw = blocks * threads / 64;
  static unsigned long long h[2 * 16384];
  CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * 2 * nw, hipMemcpyDeviceToHost));
  double sc = 0, rt = 0;
  for (int i = 0; i < nw; ++i) {
    sc += (double)h[2 * i];
    rt += (double)h[2 * i + 1];
  }
  sc /= nw;
  rt /= nw;
  const double ghz = sc / rt * 0.1;
  const double cyc_per_block_simd = sc / ((double)kBlocks * wps);  // SIMD cycles per block
  const double blocks_total = (double)blocks * threads * kBlocks;
  // a "wave-block" = one block in each of a wave's 64 lanes (one pass of the round code)
  printf("{\"var\": \"%s\", \"waves_per_simd\": %d, \"ghz\": %.3f, \"simd_cycles_per_wave_block\": %.1f, "
         "\"cu_cycles_per_block\": %.3f, \"kernel_ms\": %.3f, \"GBlocks_per_s\": %.1f}\n",
         name, wps, ghz, cyc_per_block_simd, cyc_per_block_simd / 256.0, ms, blocks_total / (ms * 1e-3) / 1e9);
  return 0;
}

int main() {
  int ncu = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
  uint32_t *out, *te0;
  unsigned long long* cyc;
  CK(hipMalloc(&out, 4u * ncu * 2048));
  CK(hipMalloc(&cyc, 16u * ncu * 32));
  CK(hipMalloc(&te0, 1024));
  CK(hipMemcpy(te0, cmpi::kAes.te0, 1024, hipMemcpyHostToDevice));
  RoundKeys k;
  for (int i = 0; i < 44; ++i) k.w[i] = 0x01234567u * (i + 1);
  run<0>("rows_te01_rotl16", 4, te0, k, out, cyc, ncu);
  run<0>("rows_te01_rotl16", 8, te0, k, out, cyc, ncu);
  run<2>("rows_te01_rotl16_two_blocks", 4, te0, k, out, cyc, ncu);
  run<1>("rows_te0123_norot", 4, te0, k, out, cyc, ncu);
  run<3>("rows_te01_sdwa_addr", 4, te0, k, out, cyc, ncu);
  run<3>("rows_te01_sdwa_addr", 8, te0, k, out, cyc, ncu);
  return 0;
}
