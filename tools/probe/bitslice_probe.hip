// bitslice_probe.hip — throughput of the bitsliced AES-128 network (tools/gen_bitslice.py ->
// csrc/aes_bitslice_gen.hpp) as a CTR keystream generator on gfx950: each lane encrypts 32
// counter blocks held as 128 bit-planes (bit j of plane p = bit p of block j), ten rounds, the
// planes folded into one word per lane (keeps every plane live; no output transpose).  Round keys
// are 11 x 128 key planes (0 / ~0) in a kernel-argument buffer (scalar operands).  Timing only:
// G blocks/s at the occupancy the register count allows, vs the T-table AES probe
// (profiles/r05c_aes_probe.jsonl: 91 G blocks/s at 4 waves per SIMD, 101 at 8).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o bitslice_probe bitslice_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "aes_bitslice_gen.hpp"

template <int TPB>
__global__ __launch_bounds__(TPB) void bs_ctr(const uint32_t* __restrict__ kp, uint32_t* __restrict__ out, uint32_t nonce0,
                                              uint32_t iters) {
  const uint32_t gid = blockIdx.x * TPB + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t s[128];
    // counter blocks c0 + j, j = 0..31 (c0 a multiple of 32): bytes 0..11 the nonce (constant per
    // lane: planes 0 / ~0), bytes 12..15 the big-endian counter (plane of bit b of a counter byte)
    const uint32_t c0 = (gid * iters + it) << 5;
#pragma unroll
    for (int p = 0; p < 96; ++p) s[p] = ((nonce0 ^ gid) >> (p & 31)) & 1u ? 0xffffffffu : 0u;
#pragma unroll
    for (int p = 96; p < 128; ++p) {
      const int byte = p >> 3, bit = p & 7, sh = 8 * (15 - byte) + bit;  // bit of the counter value
      uint32_t w;
      if (sh < 5) w = sh == 0 ? 0xaaaaaaaau : sh == 1 ? 0xccccccccu : sh == 2 ? 0xf0f0f0f0u : sh == 3 ? 0xff00ff00u : 0xffff0000u;
      else w = (c0 >> sh) & 1u ? 0xffffffffu : 0u;
      s[p] = w;
    }
#pragma unroll
    for (int p = 0; p < 128; ++p) s[p] ^= kp[p];
#pragma unroll 1
    for (int r = 1; r < 10; ++r) cmpi::bs::round_mid(s, kp + 128 * r);
    cmpi::bs::round_last(s, kp + 128 * 10);
#pragma unroll
    for (int p = 0; p < 128; ++p) acc ^= s[p] << (p & 7);
  }
  out[gid] = acc;
}

template <int TPB>
void run(const uint32_t* kp, uint32_t* out, int blocks, uint32_t iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((bs_ctr<TPB>), dim3(blocks), dim3(TPB), 0, 0, kp, out, 7u, iters);
  (void)hipDeviceSynchronize();
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((bs_ctr<TPB>), dim3(blocks), dim3(TPB), 0, 0, kp, out, 7u, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double blks = (double)blocks * TPB * iters * 32.0;
  printf("{\"tpb\": %d, \"workgroups\": %d, \"blocks_per_lane\": %u, \"kernel_ms\": %.3f, \"GBlocks_per_s\": %.1f}\n", TPB, blocks,
         32u * iters, best, blks / (best * 1e-3) / 1e9);
  fflush(stdout);
}

int main() {
  uint32_t* kp;
  uint32_t* out;
  if (hipMalloc(&kp, 11 * 128 * 4) != hipSuccess || hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  uint32_t hk[11 * 128];
  for (int i = 0; i < 11 * 128; ++i) hk[i] = (i * 2654435761u) >> 31 ? 0xffffffffu : 0u;
  (void)hipMemcpy(kp, hk, sizeof hk, hipMemcpyHostToDevice);
  int ncu = 256;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  for (int wpc : {4, 8, 12, 16}) run<256>(kp, out, ncu * wpc / 4, 16);  // 4..16 waves per CU
  for (int wpc : {8, 16}) run<512>(kp, out, ncu * wpc / 8, 16);
  return 0;
}
