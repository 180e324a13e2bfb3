// gcm_bs_probe.hip — config 2 (65 536 x 1 KiB AES-128-GCM seal) with the keystream from the
// bitsliced VALU AES network instead of the LDS T-tables: timing only.
//
// One lane per half record: lane (r, h) encrypts the 32 counter blocks 2 + 32h + j (j < 32) of
// record r as one bitsliced batch (128 state planes, the nonce words constant per lane, the
// counter word transposed in; tools/gen_bitslice.py's network, tools/probe/aes_bitslice_gen.hpp),
// transposes the keystream out (four 32 x 32 bit transposes), then runs its 32 Horner steps over
// the half record: load the plaintext block, XOR, store the ciphertext, acc = (acc ^ ct) · H from
// the 64 KiB GHASH byte table in LDS (gmul_byte, the lane kernel's multiply).  The two halves'
// partials, the length block and E_K(J0) are not combined (the tag written is not the GCM tag):
// what is measured is everything that scales with the data — keystream, transposes, loads, stores,
// GHASH — on 512-thread workgroups of 2 waves per SIMD (the state needs ~256 VGPRs).
// Compare with the T-table lane kernel's seal launch of the same shape (bench.py kernel_ms).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o gcm_bs_probe gcm_bs_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../cryptmpi_2022_amd/csrc/aes_device.hpp"
#include "aes_bitslice_gen.hpp"
namespace cmpi {
namespace dev {
#include "ctr_bs_kernel.hpp"  // bs_transpose32 (the generated network is included above, at namespace scope)
}  // namespace dev
}  // namespace cmpi

using cmpi::dev::u32x4;

__global__ __launch_bounds__(512, 1) void gcm_bs_probe(const uint32_t* __restrict__ kp, const u32x4* __restrict__ tab,
                                                       const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                       const uint32_t* __restrict__ nonces, uint32_t nrec) {
  using namespace cmpi::dev;
  for (uint32_t i = threadIdx.x; i < 4096u; i += 512u) lds_st128(16u * i, tab[i]);  // byte table of "H"
  __syncthreads();
  const uint32_t gid = blockIdx.x * 512u + threadIdx.x, r = gid >> 1, h = gid & 1u;
  if (r >= nrec) return;
  const uint32_t n0 = nonces[3u * r], n1 = nonces[3u * r + 1u], n2 = nonces[3u * r + 2u];
  uint32_t s[128];
#pragma unroll
  for (int b = 0; b < 32; ++b) {
    s[b] = (n0 >> b) & 1u ? 0xffffffffu : 0u;
    s[32 + b] = (n1 >> b) & 1u ? 0xffffffffu : 0u;
    s[64 + b] = (n2 >> b) & 1u ? 0xffffffffu : 0u;
  }
#pragma unroll
  for (int j = 0; j < 32; ++j) s[96 + j] = __builtin_bswap32(2u + 32u * h + (uint32_t)j);
  bs_transpose32(s + 96);
#pragma unroll
  for (int p = 0; p < 128; ++p) s[p] ^= kp[p];
#pragma unroll 1
  for (int rr = 1; rr < 10; ++rr) cmpi::bs::round_mid(s, kp + 128 * rr);
  cmpi::bs::round_last(s, kp + 128 * 10);
#pragma unroll
  for (int w = 0; w < 4; ++w) bs_transpose32(s + 32 * w);
  const GhashLane gl = ghash_lane();
  const u32x4* ip = in + (uint64_t)r * 64u + 32u * h;  // 1 KiB records, 16-byte blocks
  u32x4* op = reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(out) + (uint64_t)r * 1040u) + 32u * h;
  u32x4 acc = {0u, 0u, 0u, 0u};
  u32x4 v = ip[0];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const u32x4 vn = ip[j < 31 ? j + 1 : 31];
    const u32x4 o = v ^ u32x4{s[j], s[32 + j], s[64 + j], s[96 + j]};
    op[j] = o;
    acc = gmul_byte(acc ^ o, gl);
    v = vn;
  }
  if (h) op[32] = acc;  // a 16-byte "tag" slot (not the GCM tag)
}

int main() {
  const uint32_t nrec = 65536;
  uint32_t *kp, *nonces;
  u32x4 *tab, *in, *out;
  (void)hipMalloc(&kp, 11 * 128 * 4);
  (void)hipMalloc(&tab, 4096 * 16);
  (void)hipMalloc(&in, (size_t)nrec * 1024);
  (void)hipMalloc(&out, (size_t)nrec * 1040);
  (void)hipMalloc(&nonces, (size_t)nrec * 12);
  (void)hipMemset(kp, 0x5a, 11 * 128 * 4);
  (void)hipMemset(tab, 0x3c, 4096 * 16);
  (void)hipMemset(in, 0x11, (size_t)nrec * 1024);
  (void)hipMemset(nonces, 0x77, (size_t)nrec * 12);
  const uint32_t blocks = (2 * nrec + 511) / 512;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 200; ++w)  // warm-up (clocks)
    hipLaunchKernelGGL(gcm_bs_probe, dim3(blocks), dim3(512), 65536, 0, kp, tab, in, out, nonces, nrec);
  (void)hipDeviceSynchronize();
  float best = 1e9, sum = 0;
  const int reps = 100;
  for (int i = 0; i < reps; ++i) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(gcm_bs_probe, dim3(blocks), dim3(512), 65536, 0, kp, tab, in, out, nonces, nrec);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
    sum += ms;
  }
  const hipError_t err = hipGetLastError();
  const double gib = (double)nrec * 1024 / (1 << 30);
  printf("{\"probe\": \"gcm_bs_probe\", \"shape\": \"65536 x 1 KiB seal (no tag combine)\", \"us_mean\": %.2f, "
         "\"us_best\": %.2f, \"GiBps_mean\": %.1f, \"err\": \"%s\"}\n",
         sum / reps * 1e3, best * 1e3, gib / (sum / reps * 1e-3), hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
