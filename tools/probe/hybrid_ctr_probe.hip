// hybrid_ctr_probe.hip — can a bitsliced AES kernel (VALU) run beside the T-table CTR kernel (LDS)
// and add throughput?  1 GiB CTR XOR, timed with HIP events:
//   ttab2     the library's cmpi_ctr_xor (2 workgroups of 1 024 per CU: every VGPR of the CU)
//   ttab1     the same with 1 workgroup per CU (cmpi_debug_set_ctr_wg_per_cu(1): half the VGPRs free)
//   bs        a bitsliced CTR kernel alone (tools/gen_bitslice.py network; counter blocks
//             transposed in, keystream transposed out, XORed into the data; 256 VGPRs, no LDS)
//   mix_f     ttab1 on the first 1-f of the stream and bs on the last f, on two streams at once
// TIMING ONLY: the bitsliced kernel's round keys are arbitrary planes (its output is not AES-CTR
// under the context's key); the question is throughput when the two share the CUs.
// Build (from tools/probe): hipcc -O3 --offload-arch=gfx950 -std=c++17 -o hybrid_ctr_probe hybrid_ctr_probe.hip
//   -L../../cryptmpi_2022_amd -lcmpi_aead -Wl,-rpath,'$ORIGIN/../../cryptmpi_2022_amd'
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/cmpi_aead.h"
#include "../../include/cmpi_debug.h"
#include "aes_bitslice_gen.hpp"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// in-place transpose of a 32x32 bit matrix held as a[0..31] (row i = a[i], bit j = column j)
__device__ __forceinline__ void transpose32(uint32_t* a) {
  uint32_t m = 0x0000ffffu;
#pragma unroll
  for (int j = 16; j != 0; j >>= 1, m ^= m << j) {
#pragma unroll
    for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
      const uint32_t t = (a[k] ^ (a[k + j] >> j)) & m;
      a[k] ^= t;
      a[k + j] ^= t << j;
    }
  }
}

// One wave-chunk = 2 048 blocks: lane L holds blocks c + L + 64 j (j < 32), so load / store
// instruction j of the wave touches 1 KiB of contiguous stream.
__global__ __launch_bounds__(256) void bs_ctr_xor(u32x4* __restrict__ out, const u32x4* __restrict__ in,
                                                  const uint32_t* __restrict__ kp, uint64_t blk0, uint64_t nchunks,
                                                  uint64_t ctr_lo) {
  const uint32_t lane = threadIdx.x & 63u, wave = (blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint32_t nwaves = gridDim.x * 4u;
  for (uint64_t ch = wave; ch < nchunks; ch += nwaves) {
    const uint64_t b0 = blk0 + ch * 2048u + lane;
    uint32_t s[128];
    // counter blocks (big-endian 128-bit, low 64 bits counted here) -> planes
#pragma unroll
    for (int w = 0; w < 4; ++w) {
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const uint64_t c = ctr_lo + b0 + 64u * (uint64_t)j;
        s[32 * w + j] = w == 3 ? __builtin_bswap32((uint32_t)c) : w == 2 ? __builtin_bswap32((uint32_t)(c >> 32)) : 0x12345678u * (w + 1);
      }
      transpose32(s + 32 * w);
    }
#pragma unroll
    for (int p = 0; p < 128; ++p) s[p] ^= kp[p];
#pragma unroll 1
    for (int r = 1; r < 10; ++r) cmpi::bs::round_mid(s, kp + 128 * r);
    cmpi::bs::round_last(s, kp + 128 * 10);
#pragma unroll
    for (int w = 0; w < 4; ++w) transpose32(s + 32 * w);  // s[32 w + j] = word w of block j
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const uint64_t b = b0 + 64u * (uint64_t)j;
      const u32x4 v = in[b];
      out[b] = v ^ u32x4{s[j], s[32 + j], s[64 + j], s[96 + j]};
    }
  }
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                          \
    }                                                                    \
  } while (0)

int main() {
  const size_t n = (size_t)1 << 30, nblk = n / 16;
  uint8_t *in, *out;
  uint32_t* kp;
  CK(hipMalloc(&in, n));
  CK(hipMalloc(&out, n));
  CK(hipMalloc(&kp, 11 * 128 * 4));
  CK(hipMemset(in, 3, n));
  uint32_t hk[11 * 128];
  for (int i = 0; i < 11 * 128; ++i) hk[i] = (i * 2654435761u) >> 31 ? 0xffffffffu : 0u;
  CK(hipMemcpy(kp, hk, sizeof hk, hipMemcpyHostToDevice));
  uint8_t key[16] = {1, 2, 3};
  cmpi_ctx* c = cmpi_ctx_new(CMPI_AES_128_CTR, key, 16, 0, 0);
  if (!c) return 1;
  const uint8_t ctr[16] = {0xf0, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa, 0xfb, 0xfc, 0xfd, 0xfe, 0xff};
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t e0, e1, ej;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&ej));
  int ncu = 256;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  // f: fraction of the stream (in 2 048-block chunks) given to the bitsliced kernel; wg_bs:
  // its 256-thread workgroups per CU (0: not launched); wpc: ctr_kernel workgroups per CU
  auto run = [&](const char* name, double f, int wpc, int wg_bs) -> int {
    const uint64_t nch = (uint64_t)(f * (double)(nblk / 2048));
    const uint64_t bs_blk = nch * 2048, t_blk = nblk - bs_blk;
    cmpi_debug_set_ctr_wg_per_cu(wpc);
    float best = 1e9;
    for (int r = 0; r < 6; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, sa));
      CK(hipStreamWaitEvent(sb, e0, 0));
      if (t_blk && cmpi_ctr_xor(c, out, in, t_blk * 16, ctr, sa) != CMPI_OK) return 1;
      if (nch) hipLaunchKernelGGL(bs_ctr_xor, dim3(ncu * wg_bs), dim3(256), 0, sb, (u32x4*)out, (const u32x4*)in, kp,
                                  (uint64_t)t_blk, nch, (uint64_t)0);
      CK(hipEventRecord(ej, sb));
      CK(hipStreamWaitEvent(sa, ej, 0));
      CK(hipEventRecord(e1, sa));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    printf("{\"form\": \"%s\", \"bs_fraction\": %.3f, \"ctr_wg_per_cu\": %d, \"bs_wg_per_cu\": %d, \"ms\": %.3f, \"GiBps\": %.1f}\n",
           name, (double)bs_blk / nblk, wpc, wg_bs, best, n / (best * 1e-3) / (1u << 30));
    fflush(stdout);
    return 0;
  };
  if (run("ttab2", 0, 2, 0) || run("ttab1", 0, 1, 0) || run("bs_1wg", 1.0, 1, 1) || run("bs_2wg", 1.0, 1, 2)) return 1;
  for (double f : {0.15, 0.25, 0.35, 0.45})
    if (run("mix", f, 1, 1)) return 1;
  for (double f : {0.15, 0.25})
    if (run("mix_ttab2", f, 2, 1)) return 1;
  return 0;
}
