// valu_rate.hip — issue rate of the VALU instruction forms the AES/GHASH kernels use on gfx950:
// cycles per wave64 instruction per SIMD for v_xor_b32 (VOP2), v_bitop3_b32 / v_perm_b32 /
// v_alignbit_b32 (VOP3), v_add_u32, v_fma_f32, with 8 independent chains per lane and 1, 2, 4
// or 8 waves per SIMD.  One JSON line per (op, waves/SIMD).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

constexpr int kIters = 4096;
constexpr int kChains = 8;

template <int OP>
__global__ void probe(uint32_t* out, uint32_t seed, unsigned long long* cyc) {
  uint32_t v[kChains];
  float f[kChains];
#pragma unroll
  for (int i = 0; i < kChains; ++i) {
    v[i] = seed * (threadIdx.x + 1u) + i;
    f[i] = (float)v[i];
  }
  const uint32_t k = seed ^ 0x9e3779b9u;
  uint32_t kv = k ^ threadIdx.x, sh = 16u + (threadIdx.x >> 10);  // per-lane VGPR operands
  asm volatile("" : "+v"(kv), "+v"(sh));
  const uint64_t t0 = clock64();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int i = 0; i < kChains; ++i) {
        if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]), "v"(v[(i + 2) % kChains]));
        if constexpr (OP == 2) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]), "s"(k));
        if constexpr (OP == 3) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 4) asm volatile("v_add_u32 %0, %1, %0" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 5) asm volatile("v_fma_f32 %0, %1, %0, %0" : "+v"(f[i]) : "v"(f[(i + 1) % kChains]));
        if constexpr (OP == 6) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]), "s"(k));
        if constexpr (OP == 7) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 8) asm volatile("v_lshlrev_b32 %0, 8, %0" : "+v"(v[i]));
        if constexpr (OP == 9) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(v[i]));
        if constexpr (OP == 10) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 11) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xec" : "+v"(v[i]) : "s"(k), "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 12) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 14) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]), "v"(kv));
        if constexpr (OP == 15) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]), "v"(sh));
        if constexpr (OP == 16) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "s"(k));
        if constexpr (OP == 17) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(v[i]) : "v"(sh));
        if constexpr (OP == 18) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(kv), "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 19) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]), "v"(v[(i + 2) % kChains]));
        if constexpr (OP == 20) asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(v[i]));
        if constexpr (OP == 21) asm volatile("v_pk_add_u16 %0, %1, %0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 22) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 23) asm volatile("v_and_b32 %0, %1, %0" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 24) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(v[(i + 1) % kChains]), "v"(v[(i + 2) % kChains]));
        if constexpr (OP == 25) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xec" : "+v"(v[i]) : "v"(kv), "v"(v[(i + 1) % kChains]));
        if constexpr (OP == 13) asm volatile("v_pk_mov_b32 %0, %1, %0 op_sel:[1,0]" : "+v"(f[i]) : "v"(f[(i + 1) % kChains]));
      }
    }
  }
  const uint64_t t1 = clock64();
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < kChains; ++i) acc ^= v[i] ^ __float_as_uint(f[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}

template <int OP>
int run(const char* name, int wps, uint32_t* out, unsigned long long* cyc, int ncu) {
  const int threads = 256 * (wps > 4 ? 4 : wps);  // 4 SIMDs x wps waves (8: two blocks per CU)
  const int blocks = ncu * (wps > 4 ? 2 : 1);
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), 0, 0, out, 7u, cyc);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(threads), 0, 0, out, 9u, cyc);
  CK(hipEventRecord(e1));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[1024];
  const int nw = blocks * threads / 64;
  CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * (nw < 1024 ? nw : 1024), hipMemcpyDeviceToHost));
  double avg = 0;
  const int m = nw < 1024 ? nw : 1024;
  for (int i = 0; i < m; ++i) avg += (double)h[i];
  avg /= m;
  const double insts = (double)kIters * 4 * kChains;       // per wave
  const double simd_cyc_per_inst = avg / (insts * wps);     // wave-clock cycles / (instrs of all waves on the SIMD)
  // wall-clock view at 2.4 GHz: SIMD-cycles per wave-instruction = ms * 2.4e6 / (instrs per SIMD)
  const double wall_cyc = ms * 2.4e6 / (insts * wps);
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cyc_per_inst_wall_2p4GHz\": %.3f, \"cyc_per_inst_clock64\": %.3f}\n",
         name, wps, ms, wall_cyc, simd_cyc_per_inst);
  return 0;
}

int main() {
  int ncu = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
  uint32_t* out;
  unsigned long long* cyc;
  CK(hipMalloc(&out, 4u * ncu * 2048));
  CK(hipMalloc(&cyc, 8u * ncu * 32));
  for (int wps : {8}) {
    run<20>("v_pk_add_u16_swap_self", wps, out, cyc, ncu);
    run<21>("v_pk_add_u16_swap_add", wps, out, cyc, ncu);
    run<22>("v_cndmask_b32", wps, out, cyc, ncu);
    run<23>("v_and_b32", wps, out, cyc, ncu);
    run<24>("v_or3_b32", wps, out, cyc, ncu);
    run<25>("v_bitop3_and_or_vgpr", wps, out, cyc, ncu);
    run<14>("v_perm_b32_vgpr_sel", wps, out, cyc, ncu);
    run<15>("v_alignbit_b32_vgpr_sh", wps, out, cyc, ncu);
    run<16>("v_xor_b32_sgpr", wps, out, cyc, ncu);
    run<17>("v_lshlrev_b32_vgpr", wps, out, cyc, ncu);
    run<18>("v_bitop3_b32_vgpr_const", wps, out, cyc, ncu);
    run<19>("v_perm_b32_all_vgpr_varying", wps, out, cyc, ncu);
    run<0>("v_xor_b32", wps, out, cyc, ncu);
    if (wps == 8) continue;
    run<1>("v_bitop3_b32", wps, out, cyc, ncu);
    run<2>("v_perm_b32", wps, out, cyc, ncu);
    run<3>("v_alignbit_b32", wps, out, cyc, ncu);
    run<4>("v_add_u32", wps, out, cyc, ncu);
    run<5>("v_fma_f32", wps, out, cyc, ncu);
    run<6>("v_and_or_b32", wps, out, cyc, ncu);
    run<7>("v_mov_b32_sdwa_byte_preserve", wps, out, cyc, ncu);
    run<8>("v_lshlrev_b32", wps, out, cyc, ncu);
    run<9>("v_bfe_u32", wps, out, cyc, ncu);
    run<10>("v_lshl_or_b32", wps, out, cyc, ncu);
    run<11>("v_bitop3_and_or_sgpr", wps, out, cyc, ncu);
    run<12>("v_xor_b32_sdwa_word1", wps, out, cyc, ncu);
  }
  return 0;
}
