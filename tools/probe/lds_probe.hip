// lds_probe.hip — microbenchmark: does the LDS lookup pipe overlap with VALU work on gfx950?
// Runs AES-shaped round loops entirely out of registers + the 64 KiB row image in LDS, in
// variants that change only the VALU count, only the LDS count, the ILP (blocks per lane) and
// the occupancy (1 or 2 workgroups of 1024 per CU).  Prints one JSON line per variant with the
// measured CU cycles per block (s_memtime-free: wall time × reported clock is done offline;
// here we report ns and the per-wave clock64 cycles).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o lds_probe lds_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../cryptmpi_2022_amd/csrc/aes_device.hpp"

using namespace cmpi::dev;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

// MODE 0: real round (16 perm + 16 ds_read + 16 combine VALU)
// MODE 1: 16 perm + 16 ds_read + 8 combine (2 x xor3 per column)
// MODE 2: MODE 0 + 16 extra independent VALU per round (dummy chain)
// MODE 3: VALU only: the 16 ds_read replaced by a v_perm (48 VALU, no LDS)
// MODE 4: MODE 0 + 16 extra VALU on the critical path (no extra lookups)
template <int MODE>
__device__ __forceinline__ uint32_t look(uint32_t a) {
  if constexpr (MODE == 3) return perm(a, a, 0x01000302u);
  else return lds32(a);
}

template <int MODE>
__device__ __forceinline__ void round_(const RowLanes& L, uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                       uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t& dummy) {
  const uint32_t a0 = look<MODE>(ra<0>(s0, L.l0)), a1 = look<MODE>(ra<1>(s1, L.l1)), a2 = look<MODE>(ra<2>(s2, L.l0)), a3 = look<MODE>(ra<3>(s3, L.l1));
  const uint32_t b0 = look<MODE>(ra<0>(s1, L.l0)), b1 = look<MODE>(ra<1>(s2, L.l1)), b2 = look<MODE>(ra<2>(s3, L.l0)), b3 = look<MODE>(ra<3>(s0, L.l1));
  const uint32_t c0 = look<MODE>(ra<0>(s2, L.l0)), c1 = look<MODE>(ra<1>(s3, L.l1)), c2 = look<MODE>(ra<2>(s0, L.l0)), c3 = look<MODE>(ra<3>(s1, L.l1));
  const uint32_t d0 = look<MODE>(ra<0>(s3, L.l0)), d1 = look<MODE>(ra<1>(s0, L.l1)), d2 = look<MODE>(ra<2>(s1, L.l0)), d3 = look<MODE>(ra<3>(s2, L.l1));
  if constexpr (MODE == 1) {
    s0 = xor3(xor3(a0, a1, k0), a2, a3);
    s1 = xor3(xor3(b0, b1, k1), b2, b3);
    s2 = xor3(xor3(c0, c1, k2), c2, c3);
    s3 = xor3(xor3(d0, d1, k3), d2, d3);
  } else {
    s0 = xor3(a0, a1, k0) ^ rotl16(a2 ^ a3);
    s1 = xor3(b0, b1, k1) ^ rotl16(b2 ^ b3);
    s2 = xor3(c0, c1, k2) ^ rotl16(c2 ^ c3);
    s3 = xor3(d0, d1, k3) ^ rotl16(d2 ^ d3);
  }
  if constexpr (MODE == 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dummy = __builtin_amdgcn_alignbit(dummy, dummy, 7) ^ (dummy >> 3);
  }
  if constexpr (MODE == 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s0 = __builtin_amdgcn_alignbit(s0, s0, 8 + i) ^ k1;
      s1 = __builtin_amdgcn_alignbit(s1, s1, 8 + i) ^ k2;
    }
  }
}

struct Look16 {
  uint32_t a0, a1, a2, a3, b0, b1, b2, b3, c0, c1, c2, c3, d0, d1, d2, d3;
};
__device__ __forceinline__ Look16 issue16(const RowLanes& L, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3) {
  Look16 t;
  t.a0 = lds32(ra<0>(s0, L.l0)); t.a1 = lds32(ra<1>(s1, L.l1)); t.a2 = lds32(ra<2>(s2, L.l0)); t.a3 = lds32(ra<3>(s3, L.l1));
  t.b0 = lds32(ra<0>(s1, L.l0)); t.b1 = lds32(ra<1>(s2, L.l1)); t.b2 = lds32(ra<2>(s3, L.l0)); t.b3 = lds32(ra<3>(s0, L.l1));
  t.c0 = lds32(ra<0>(s2, L.l0)); t.c1 = lds32(ra<1>(s3, L.l1)); t.c2 = lds32(ra<2>(s0, L.l0)); t.c3 = lds32(ra<3>(s1, L.l1));
  t.d0 = lds32(ra<0>(s3, L.l0)); t.d1 = lds32(ra<1>(s0, L.l1)); t.d2 = lds32(ra<2>(s1, L.l0)); t.d3 = lds32(ra<3>(s2, L.l1));
  return t;
}
__device__ __forceinline__ void combine16(const Look16& t, uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                          uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  s0 = xor3(t.a0, t.a1, k0) ^ rotl16(t.a2 ^ t.a3);
  s1 = xor3(t.b0, t.b1, k1) ^ rotl16(t.b2 ^ t.b3);
  s2 = xor3(t.c0, t.c1, k2) ^ rotl16(t.c2 ^ t.c3);
  s3 = xor3(t.d0, t.d1, k3) ^ rotl16(t.d2 ^ t.d3);
}
#define FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ void setprio_dyn(uint32_t p);
// two blocks per lane, staggered by half a round: B's combine runs while A's lookups are in flight
template <bool PRIO>
__global__ __launch_bounds__(1024, 8) void probe_stagger(uint32_t* out, const uint32_t* table, int iters, RoundKeys k,
                                                         unsigned long long* cyc) {
  for (uint32_t i = threadIdx.x; i < 16384u; i += blockDim.x) lds_st32(i * 4u, table[i]);
  __syncthreads();
  const RowLanes L = row_lanes(0u);
  const uint64_t t0 = clock64();
  uint32_t a0 = threadIdx.x * 0x9E3779B1u + blockIdx.x, a1 = a0 + 0x1234567u, a2 = a0 + 0x2468ace, a3 = a0 + 0x369d035;
  uint32_t b0 = a0 ^ 0x55555555u, b1 = a1 ^ 0x55555555u, b2 = a2 ^ 0x55555555u, b3 = a3 ^ 0x55555555u;
  for (int it = 0; it < iters; ++it) {
    if (PRIO) setprio_dyn((uint32_t)it + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
    Look16 tb = issue16(L, b0, b1, b2, b3);
    FENCE();
#pragma unroll
    for (int r = 1; r < 11; ++r) {
      Look16 ta = issue16(L, a0, a1, a2, a3);
      FENCE();
      combine16(tb, b0, b1, b2, b3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3]);
      if (r < 10) {
        tb = issue16(L, b0, b1, b2, b3);
        FENCE();
      }
      combine16(ta, a0, a1, a2, a3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3]);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ b0 ^ b1 ^ b2 ^ b3;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = clock64() - t0;
}

__device__ __forceinline__ void setprio_dyn(uint32_t p) {
  switch (p & 3u) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}
// VARIANT 0: rotating priority per iteration; 1: dynamic distribution of iterations via an LDS counter
template <int VARIANT>
__global__ __launch_bounds__(1024, 8) void probe_fair(uint32_t* out, const uint32_t* table, int iters, RoundKeys k,
                                                      unsigned long long* cyc) {
  for (uint32_t i = threadIdx.x; i < 16384u; i += blockDim.x) lds_st32(i * 4u, table[i]);
  if (threadIdx.x == 0) lds_st32(65536u, 0u);
  __syncthreads();
  const RowLanes L = row_lanes(0u);
  const uint64_t t0 = clock64();
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t s0 = threadIdx.x * 0x9E3779B1u + blockIdx.x * 77u, s1 = s0 + 0x1234567u, s2 = s0 + 0x2468ace, s3 = s0 + 0x369d035;
  uint32_t dummy = 0;
  const uint32_t total = (uint32_t)iters * (blockDim.x >> 6);
  uint32_t it = 0;
  for (;;) {
    if (VARIANT == 0) {
      if (it >= (uint32_t)iters) break;
      setprio_dyn(it + wid);
      ++it;
    } else if (VARIANT == 2) {  // progress-based: behind the workgroup average -> higher priority
      if (it >= (uint32_t)iters) break;
      typedef __attribute__((address_space(3))) uint32_t lds_u;
      uint32_t tot = 0;
      if ((threadIdx.x & 63u) == 0) {
        __hip_atomic_fetch_add((lds_u*)(size_t)65536u, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tot = *(volatile lds_u*)(size_t)65536u;
      }
      tot = __builtin_amdgcn_readfirstlane(tot);
      const uint32_t avg16 = tot;             // 16 x average iterations done
      const uint32_t mine16 = (it + 1) * 16u;
      setprio_dyn(mine16 + 16u <= avg16 ? 3u : (mine16 <= avg16 ? 2u : (mine16 <= avg16 + 16u ? 1u : 0u)));
      ++it;
    } else {
      uint32_t got = 0;
      if ((threadIdx.x & 63u) == 0) got = __hip_atomic_fetch_add((__attribute__((address_space(3))) uint32_t*)(size_t)65536u, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      got = __builtin_amdgcn_readfirstlane(got);
      if (got >= total) break;
      ++it;
    }
#pragma unroll
    for (int r = 1; r < 11; ++r)
      round_<0>(L, s0, s1, s2, s3, k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2], k.w[4 * r + 3], dummy);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ it;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = clock64() - t0;
}

template <int MODE, int ILP>
__global__ __launch_bounds__(1024, 8) void probe(uint32_t* out, const uint32_t* table, int iters, RoundKeys k,
                                                  unsigned long long* cyc) {
  for (uint32_t i = threadIdx.x; i < 16384u; i += blockDim.x) lds_st32(i * 4u, table[i]);
  __syncthreads();
  const RowLanes L = row_lanes(0u);
  const uint64_t t0 = clock64();
  uint32_t s[ILP][4];
#pragma unroll
  for (int j = 0; j < ILP; ++j)
    for (int c = 0; c < 4; ++c) s[j][c] = threadIdx.x * 0x9E3779B1u + blockIdx.x * 77u + c * 0x1234567u + j;
  uint32_t dummy = threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 1; r < 11; ++r) {
#pragma unroll
      for (int j = 0; j < ILP; ++j)
        round_<MODE>(L, s[j][0], s[j][1], s[j][2], s[j][3], k.w[4 * r], k.w[4 * r + 1], k.w[4 * r + 2],
                     k.w[4 * r + 3], dummy);
    }
  }
  uint32_t acc = dummy;
#pragma unroll
  for (int j = 0; j < ILP; ++j) acc ^= s[j][0] ^ s[j][1] ^ s[j][2] ^ s[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = clock64() - t0;
}

template <int MODE, int ILP>
void run(const char* name, int lds_bytes, int ncu, uint32_t* out, uint32_t* table, unsigned long long* cyc,
         RoundKeys k);
template <int MODE, int ILP>
void run_fn(void (*fn)(uint32_t*, const uint32_t*, int, RoundKeys, unsigned long long*), const char* name, int lds_bytes, int ncu, uint32_t* out, uint32_t* table, unsigned long long* cyc,
         RoundKeys k);
template <int MODE, int ILP>
void run(const char* name, int lds_bytes, int ncu, uint32_t* out, uint32_t* table, unsigned long long* cyc,
         RoundKeys k) {
  run_fn<MODE, ILP>(probe<MODE, ILP>, name, lds_bytes, ncu, out, table, cyc, k);
}
template <int MODE, int ILP>
void run_fn(void (*fn)(uint32_t*, const uint32_t*, int, RoundKeys, unsigned long long*), const char* name, int lds_bytes, int ncu, uint32_t* out, uint32_t* table, unsigned long long* cyc,
         RoundKeys k) {
  CK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
  const int wg_per_cu = lds_bytes > 81920 ? 1 : 2;
  const int grid = ncu * wg_per_cu * 4;  // 4 waves of workgroups
  const int iters = 64 / ILP;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  fn<<<grid, 1024, lds_bytes>>>(out, table, iters, k, cyc);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(e0));
    fn<<<grid, 1024, lds_bytes>>>(out, table, iters, k, cyc);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double blocks = (double)grid * 1024 * 64;  // 10-round "blocks"
  unsigned long long* h = (unsigned long long*)malloc(sizeof(unsigned long long) * grid * 16);
  CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * grid * 16, hipMemcpyDeviceToHost));
  double avg = 0, mn = 1e300, mx = 0;
  for (int i = 0; i < grid * 16; ++i) {
    avg += h[i];
    mn = h[i] < mn ? h[i] : mn;
    mx = h[i] > mx ? h[i] : mx;
  }
  avg /= grid * 16;
  free(h);
  // CU cycles per block at clock f: best_ms*1e-3*f*ncu/blocks; report ns/block*ncu (=CU-ns per block)
  printf("{\"variant\": \"%s\", \"ilp\": %d, \"wg_per_cu\": %d, \"ms\": %.4f, \"cu_ns_per_block\": %.4f, "
         "\"wave_clock64_avg\": %.0f, \"min\": %.0f, \"max\": %.0f}\n",
         name, ILP, wg_per_cu, best, best * 1e6 * ncu / blocks, avg, mn, mx);
  fflush(stdout);
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  uint32_t *out, *table;
  unsigned long long* cyc;
  CK(hipMalloc(&out, (size_t)ncu * 8 * 1024 * 4));
  CK(hipMalloc(&table, 65536));
  CK(hipMalloc(&cyc, (size_t)ncu * 8 * 16 * 8));
  uint32_t* ht = (uint32_t*)malloc(65536);
  uint32_t x = 12345;
  for (int i = 0; i < 16384; ++i) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    ht[i] = x;
  }
  CK(hipMemcpy(table, ht, 65536, hipMemcpyHostToDevice));
  RoundKeys k;
  for (int i = 0; i < 44; ++i) k.w[i] = 0x01010101u * i + 0x5a;
  for (int lds : {163840 - 256, 65536 + 256}) {
    run<0, 1>("real", lds, ncu, out, table, cyc, k);
    run<0, 2>("real", lds, ncu, out, table, cyc, k);
    run_fn<0, 2>(probe_stagger<false>, "stagger2", lds, ncu, out, table, cyc, k);
    run_fn<0, 2>(probe_stagger<true>, "stagger2_rotprio", lds, ncu, out, table, cyc, k);
    run_fn<0, 1>(probe_fair<0>, "rotprio", lds, ncu, out, table, cyc, k);
    run_fn<0, 1>(probe_fair<1>, "dynamic", lds, ncu, out, table, cyc, k);
    run_fn<0, 1>(probe_fair<2>, "progress_prio", lds, ncu, out, table, cyc, k);
    run<1, 1>("combine8", lds, ncu, out, table, cyc, k);
    run<1, 2>("combine8", lds, ncu, out, table, cyc, k);
    run<2, 1>("extra16_indep", lds, ncu, out, table, cyc, k);
    run<4, 1>("extra16_crit", lds, ncu, out, table, cyc, k);
    run<3, 1>("valu_only", lds, ncu, out, table, cyc, k);
    run<3, 2>("valu_only", lds, ncu, out, table, cyc, k);
  }
  return 0;
}
