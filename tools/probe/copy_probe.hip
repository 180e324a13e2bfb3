// copy_probe.hip — which device-copy form reaches the HBM peak on this box (bench.py's measured
// roofline peak, cmpi_debug_copy): 1 GiB copied, read + write bytes / time, best of 10, for
// plain / non-temporal accesses, 1 / 2 / 4 loads in flight per lane, and grid sizes.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o copy_probe copy_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copyk(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t nv) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < nv; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = NT ? __builtin_nontemporal_load(s + i + k * stride) : s[i + k * stride];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NT) __builtin_nontemporal_store(v[k], d + i + k * stride);
      else d[i + k * stride] = v[k];
    }
  }
  for (; i < nv; i += stride) d[i] = s[i];
}

template <int U, bool NT>
void run(const char* name, u32x4* d, const u32x4* s, uint64_t nv, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((copyk<U, NT>), dim3(blocks), dim3(256), 0, 0, d, s, nv);
  (void)hipDeviceSynchronize();
  float best = 1e9;
  for (int r = 0; r < 10; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((copyk<U, NT>), dim3(blocks), dim3(256), 0, 0, d, s, nv);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  printf("{\"form\": \"%s\", \"blocks\": %d, \"GBps\": %.1f}\n", name, blocks, 2.0 * nv * 16 / (best * 1e-3) / 1e9);
}

int main() {
  const uint64_t n = 1ull << 30, nv = n / 16;
  u32x4 *s, *d;
  if (hipMalloc(&s, n) != hipSuccess || hipMalloc(&d, n) != hipSuccess) return 1;
  (void)hipMemset(s, 1, n);
  (void)hipMemset(d, 0, n);
  for (int blocks : {1024, 2048, 4096, 8192, 16384}) {
    run<1, false>("plain_u1", d, s, nv, blocks);
    run<2, false>("plain_u2", d, s, nv, blocks);
    run<4, false>("plain_u4", d, s, nv, blocks);
    run<1, true>("nt_u1", d, s, nv, blocks);
    run<4, true>("nt_u4", d, s, nv, blocks);
  }
  return 0;
}
