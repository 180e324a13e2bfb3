// issue_probe.hip — issue cost of the VALU / LDS instruction forms the AES and GHASH loops use,
// measured with the in-kernel clock (s_memtime ticks over s_memrealtime's 100 MHz, so no clock
// assumption): SIMD cycles per wave-instruction with W waves per SIMD, 16 independent chains per
// wave (no dependency stall), and mixes of ds_read_b32 with VALU in the AES kernel's ratio.
// One JSON line per case.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o issue_probe issue_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

constexpr int kIters = 2048;
constexpr int kC = 16;  // independent chains per wave

// OP: 0 xor, 1 and, 2 bitop3 vvv, 3 bitop3 with an SGPR operand, 4 perm vvv, 5 alignbit (const
// shift), 6 cndmask e64 (SGPR-pair mask), 7 cndmask vcc, 8 lshlrev const, 9 add_u32, 10 mov,
// 11 or3, 12 lshl_or, 13 and_or, 14 bfe_u32, 15 xor with SGPR,
// 20 ds_read_b32 (conflict free, <= 8 in flight) + its address (and_or) + a xor, 21 the same with
// 2 bitop3, 22 with 2 perm (throughput only: the read results are not waited for exactly)
template <int OP>
__global__ void probe(uint32_t* out, uint32_t seed, unsigned long long* cyc) {
  extern __shared__ uint32_t lds[];
  for (uint32_t i = threadIdx.x; i < 16384u; i += blockDim.x) lds[i] = i * 2654435761u;
  __syncthreads();
  uint32_t v[kC];
#pragma unroll
  for (int i = 0; i < kC; ++i) v[i] = seed * (threadIdx.x + 1u) + 977u * i;
  uint32_t sk = __builtin_amdgcn_readfirstlane(seed ^ 0x5bd1e995u);
  uint64_t sm = __builtin_amdgcn_read_exec() & (seed ? 0x5555555555555555ull : 0ull);
  const uint32_t lb = (threadIdx.x & 31u) << 2;
  uint32_t kv = seed ^ threadIdx.x;
  asm volatile("" : "+v"(kv), "+s"(sk), "+s"(sm));
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < kC; ++i) {
      uint32_t& x = v[i];
      const uint32_t y = v[(i + 5) % kC];
      const uint32_t z = v[(i + 11) % kC];
      if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
      if constexpr (OP == 1) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(y));
      if constexpr (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "v"(z));
      if constexpr (OP == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "s"(sk));
      if constexpr (OP == 4) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
      if constexpr (OP == 5) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(x) : "v"(y));
      if constexpr (OP == 6) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(sm));
      if constexpr (OP == 7) asm volatile("s_mov_b64 vcc, %2\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(y), "s"(sm) : "vcc");
      if constexpr (OP == 8) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x));
      if constexpr (OP == 9) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y));
      if constexpr (OP == 10) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(y));
      if constexpr (OP == 11) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
      if constexpr (OP == 12) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(y));
      if constexpr (OP == 13) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
      if constexpr (OP == 14) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(x));
      if constexpr (OP == 15) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "s"(sk));
      if constexpr (OP == 30) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(x) : "v"(y));
      if constexpr (OP == 31) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(x) : "v"(y));
      if constexpr (OP == 32) asm volatile("v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD" : "=v"(x) : "v"(y), "v"(z));
      if constexpr (OP == 33) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
      if constexpr (OP == 34) asm volatile("v_and_b32 %0, 0xff00, %0" : "+v"(x));
      if constexpr (OP == 35) asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(x) : "v"(y));
      if constexpr (OP == 36) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(x) : "v"(y));
      if constexpr (OP == 37) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x) : "v"(y));
      if constexpr (OP == 39) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
      if constexpr (OP >= 20 && OP < 30) {
        if constexpr (OP == 20 || OP == 21 || OP == 22) {
          const uint32_t a = ((x & 0xff00u) | lb);
          uint32_t t;
          asm volatile("ds_read_b32 %0, %1" : "=v"(t) : "v"(a));
          asm volatile("s_waitcnt lgkmcnt(8)" ::);
          if constexpr (OP == 21) {
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(t), "v"(z));
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "v"(z));
          } else if constexpr (OP == 22) {
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(t), "v"(z));
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
          } else {
            x ^= t;
          }
        }
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < kC; ++i) acc ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63u) == 0u) {
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    cyc[2 * w] = t1 - t0;
    cyc[2 * w + 1] = r1 - r0;
  }
}

template <int OP>
int run(const char* name, int wps, int per_iter_valu, int per_iter_ds, uint32_t* out, unsigned long long* cyc, int ncu) {
  const int threads = 256 * (wps > 4 ? 4 : wps);
  const int blocks = ncu * (wps > 4 ? wps / 4 : 1);
  const size_t lds = 65536;
  CK(hipFuncSetAttribute((const void*)probe<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), lds, 0, out, 7u, cyc);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), lds, 0, out, 9u, cyc);
  CK(hipDeviceSynchronize());
  const int nw = blocks * threads / 64;
  static unsigned long long h[2 * 8192];
  CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * 2 * nw, hipMemcpyDeviceToHost));
  double sc = 0, rt = 0;
  for (int i = 0; i < nw; ++i) {
    sc += (double)h[2 * i];
    rt += (double)h[2 * i + 1];
  }
  sc /= nw;
  rt /= nw;
  const double ghz = sc / rt * 0.1;  // s_memtime ticks per 10 ns
  const double per_wave_slots = (double)kIters * kC;  // loop bodies per wave
  // SIMD cycles per loop body (all waves of the SIMD share it)
  const double cyc_per_body = sc / (per_wave_slots * wps);
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ghz\": %.3f, \"simd_cycles_per_body\": %.3f, "
         "\"valu_per_body\": %d, \"ds_per_body\": %d}\n",
         name, wps, ghz, cyc_per_body, per_iter_valu, per_iter_ds);
  return 0;
}

int main() {
  int ncu = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
  uint32_t* out;
  unsigned long long* cyc;
  CK(hipMalloc(&out, 4u * ncu * 2048));
  CK(hipMalloc(&cyc, 16u * ncu * 32));
  for (int wps : {4}) {
    run<30>("v_mov_b32_sdwa_byte1_preserve_from_byte0", wps, 1, 0, out, cyc, ncu);
    run<31>("v_mov_b32_sdwa_byte1_preserve_from_byte2", wps, 1, 0, out, cyc, ncu);
    run<32>("v_or_b32_sdwa_src0_byte2", wps, 1, 0, out, cyc, ncu);
    run<33>("v_bfi_b32_vvv", wps, 1, 0, out, cyc, ncu);
    run<34>("v_and_b32_literal", wps, 1, 0, out, cyc, ncu);
    run<35>("v_alignbyte_b32", wps, 1, 0, out, cyc, ncu);
    run<36>("v_xor_b32_sdwa_word1", wps, 1, 0, out, cyc, ncu);
    run<37>("v_lshlrev_b32_vgpr", wps, 1, 0, out, cyc, ncu);
    run<39>("v_add3_u32", wps, 1, 0, out, cyc, ncu);
  }
  if (getenv("PROBE_SDWA_ONLY")) return 0;
  for (int wps : {2, 4}) {
    run<0>("v_xor_b32", wps, 1, 0, out, cyc, ncu);
    run<1>("v_and_b32", wps, 1, 0, out, cyc, ncu);
    run<2>("v_bitop3_b32_vvv", wps, 1, 0, out, cyc, ncu);
    run<3>("v_bitop3_b32_vvs", wps, 1, 0, out, cyc, ncu);
    run<4>("v_perm_b32_vvv", wps, 1, 0, out, cyc, ncu);
    run<5>("v_alignbit_b32_const", wps, 1, 0, out, cyc, ncu);
    run<6>("v_cndmask_b32_e64_sgpr", wps, 1, 0, out, cyc, ncu);
    run<7>("s_mov_vcc+v_cndmask_b32_vcc", wps, 1, 0, out, cyc, ncu);
    run<8>("v_lshlrev_b32_const", wps, 1, 0, out, cyc, ncu);
    run<9>("v_add_u32", wps, 1, 0, out, cyc, ncu);
    run<10>("v_mov_b32", wps, 1, 0, out, cyc, ncu);
    run<11>("v_or3_b32", wps, 1, 0, out, cyc, ncu);
    run<12>("v_lshl_or_b32", wps, 1, 0, out, cyc, ncu);
    run<13>("v_and_or_b32", wps, 1, 0, out, cyc, ncu);
    run<14>("v_bfe_u32", wps, 1, 0, out, cyc, ncu);
    run<15>("v_xor_b32_sgpr", wps, 1, 0, out, cyc, ncu);
    run<20>("ds_read_b32+and_or+xor", wps, 2, 1, out, cyc, ncu);
    run<21>("ds_read_b32+and_or+2bitop3", wps, 3, 1, out, cyc, ncu);
    run<22>("ds_read_b32+and_or+2perm", wps, 3, 1, out, cyc, ncu);
  }
  return 0;
}
