// copy_probe2.hip — second sweep for the device copy peak (bench.py's measured roofline peak):
// 1 GiB copied (read + write bytes / time, best of 20) for grid-stride and per-block-chunk forms,
// 256 / 512 / 1024 threads per block, 1 / 2 16-byte loads in flight per lane, plain / nt stores.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o copy_probe2 copy_probe2.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int TPB, int U, bool NT>
__global__ __launch_bounds__(TPB) void stride_k(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t nv) {
  const uint64_t stride = (uint64_t)gridDim.x * TPB;
  uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
  for (; i + (U - 1) * stride < nv; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = s[i + k * stride];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NT) __builtin_nontemporal_store(v[k], d + i + k * stride);
      else d[i + k * stride] = v[k];
    }
  }
  for (; i < nv; i += stride) d[i] = s[i];
}

// block b copies the contiguous chunk [b * per, (b + 1) * per) (per a multiple of TPB * U)
template <int TPB, int U, bool NT>
__global__ __launch_bounds__(TPB) void chunk_k(u32x4* __restrict__ d, const u32x4* __restrict__ s, uint64_t per) {
  const uint64_t b0 = (uint64_t)blockIdx.x * per;
  for (uint64_t i = threadIdx.x; i < per; i += (uint64_t)TPB * U) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = s[b0 + i + k * TPB];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NT) __builtin_nontemporal_store(v[k], d + b0 + i + k * TPB);
      else d[b0 + i + k * TPB] = v[k];
    }
  }
}

template <class F>
void timeit(const char* form, int tpb, int u, bool nt, int blocks, uint64_t nv, F launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipDeviceSynchronize();
  float best = 1e9;
  for (int r = 0; r < 20; ++r) {
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  printf("{\"form\": \"%s\", \"tpb\": %d, \"loads_in_flight\": %d, \"nt_store\": %d, \"blocks\": %d, \"GBps\": %.1f}\n", form, tpb,
         u, nt ? 1 : 0, blocks, 2.0 * nv * 16 / (best * 1e-3) / 1e9);
  fflush(stdout);
}

template <int TPB, int U, bool NT>
void sweep(u32x4* d, const u32x4* s, uint64_t nv) {
  for (int blocks : {256, 512, 1024, 2048}) {
    timeit("stride", TPB, U, NT, blocks, nv, [&] { hipLaunchKernelGGL((stride_k<TPB, U, NT>), dim3(blocks), dim3(TPB), 0, 0, d, s, nv); });
    const uint64_t per = nv / blocks;  // nv / blocks is a multiple of TPB * U for these sizes
    timeit("chunk", TPB, U, NT, blocks, nv, [&] { hipLaunchKernelGGL((chunk_k<TPB, U, NT>), dim3(blocks), dim3(TPB), 0, 0, d, s, per); });
  }
}

int main() {
  const uint64_t n = 1ull << 30, nv = n / 16;
  u32x4 *s, *d;
  if (hipMalloc(&s, n) != hipSuccess || hipMalloc(&d, n) != hipSuccess) return 1;
  (void)hipMemset(s, 1, n);
  (void)hipMemset(d, 0, n);
  sweep<256, 1, false>(d, s, nv);
  sweep<256, 2, false>(d, s, nv);
  sweep<512, 1, false>(d, s, nv);
  sweep<512, 2, false>(d, s, nv);
  sweep<1024, 1, false>(d, s, nv);
  sweep<256, 1, true>(d, s, nv);
  sweep<512, 2, true>(d, s, nv);
  return 0;
}
