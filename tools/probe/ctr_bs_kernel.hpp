// ctr_bs_kernel.hpp — the bitsliced-AES CTR kernel of round 5, retired from the product library
// in round 6: alone it ran 715 GiB/s on 1 GiB, half the T-table ctr_kernel's
// 1 430, and beside ctr_kernel at one workgroup per CU the mix was at parity (1 399 vs 1 392-1 397
// GiB/s, profiles/r05am_ctr_hybrid_sweep.jsonl); DESIGN.md §7 gives the GCM estimate that kept it
// out of the lane kernel.  Kept here as the reference for probes: include after
// cryptmpi_2022_amd/csrc/aes_device.hpp (u32x4) inside namespace cmpi::dev; the key planes are
// the round keys as 0 / ~0 planes (rounds 1-9 of InvMixColumns(round key)), the layout the
// generated network (aes_bitslice_gen.hpp, tools/gen_bitslice.py) expects.
#pragma once
#include "aes_bitslice_gen.hpp"

// ---------------------------------------------------------------- bitsliced CTR (VALU AES)
// The T-table kernels above are bound by the LDS array; this one runs AES on the VALU as a
// bitsliced network (aes_bitslice_gen.hpp, tools/gen_bitslice.py: v_bitop3 LUTs, 32 blocks per
// lane, no LDS), so the two can share the CUs: cmpi_ctr_xor hands a fraction of a long stream to
// it on a second stream while ctr_kernel runs the rest at one workgroup per CU
// (profiles/r05ae_hybrid_ctr_probe.jsonl: 1 444 -> 1 572 GiB/s on 1 GiB).
// A wave's chunk is 2 048 blocks; lane L holds blocks c + L + 64 j (j < 32), so load / store j
// of the wave touches 1 KiB of contiguous stream.  Planes: plane p = bit (p % 8) of state byte
// p / 8, bit j of a plane = block j; key planes (DevTables::bsk) are 0 / ~0: round 0 and 10 the
// round keys, rounds 1-9 InvMixColumns of them (the network adds the key before MixColumns).
struct CtrBsArgs {  // + in (null: keystream only), out, kp (11 x 128 key planes) as kernel parameters
  uint64_t nchunks;   // 2 048-block chunks, from block 0 of (in, out)
  uint64_t ctr_hi, ctr_lo;
};

// In-place 32 x 32 bit transpose: on exit x[r] bit c = (x[c] bit r on entry).
__device__ __forceinline__ void bs_transpose32(uint32_t* x) {
  uint32_t m = 0x0000ffffu;
#pragma unroll
  for (int j = 16; j != 0; j >>= 1, m ^= m << j) {
#pragma unroll
    for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
      const uint32_t t = ((x[k] >> j) ^ x[k + j]) & m;
      x[k] ^= t << j;
      x[k + j] ^= t;
    }
  }
}

// (in, out, kp as restrict parameters: the key planes then load as scalars — read through the
// argument struct they took VGPRs, 101 AGPRs of spill and one wave per SIMD.  Bounded to 256
// registers (2 waves per SIMD alone, one beside ctr_kernel's four): the counter / keystream
// transposes before and after the rounds spill ~70 registers to scratch.)
template <bool XOR_IN>
__global__ __launch_bounds__(256, 2) void ctr_bs_kernel(CtrBsArgs a, const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                        const uint32_t* __restrict__ kp) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6, nwaves = (uint64_t)gridDim.x * 4u;
  for (uint64_t ch = wave; ch < a.nchunks; ch += nwaves) {  // wave-uniform
    const uint64_t b0 = ch * 2048u + lane;
    uint32_t s[128];
    // counter blocks -> planes (plane 32 w + r = bit r of word w = bit r % 8 of state byte
    // 4 w + r / 8; bit j of a plane = block j).  The host gives this kernel only chunks without a
    // 32-bit carry inside (ctr_launch), so words 0-2 are the chunk's constants — planes 0 / ~0 —
    // and only word 3 is transposed
    const uint64_t c_lo = a.ctr_lo + ch * 2048u;  // the chunk's first counter (low half)
    const uint64_t c_hi = a.ctr_hi + (c_lo < a.ctr_lo ? 1u : 0u);
    const uint32_t w0 = __builtin_bswap32((uint32_t)(c_hi >> 32)), w1 = __builtin_bswap32((uint32_t)c_hi),
                   w2 = __builtin_bswap32((uint32_t)(c_lo >> 32));
#pragma unroll
    for (int r = 0; r < 32; ++r) {
      s[r] = (w0 >> r) & 1u ? 0xffffffffu : 0u;
      s[32 + r] = (w1 >> r) & 1u ? 0xffffffffu : 0u;
      s[64 + r] = (w2 >> r) & 1u ? 0xffffffffu : 0u;
    }
    const uint32_t l0 = (uint32_t)c_lo + lane;
#pragma unroll
    for (int j = 0; j < 32; ++j) s[96 + j] = __builtin_bswap32(l0 + 64u * (uint32_t)j);
    bs_transpose32(s + 96);
#pragma unroll
    for (int p = 0; p < 128; ++p) s[p] ^= kp[p];
#pragma unroll 1
    for (int r = 1; r < 10; ++r) bs::round_mid(s, kp + 128 * r);
    bs::round_last(s, kp + 128 * 10);
    // keystream out: s[32 w + j] = word w of block j's keystream after the four transposes
#pragma unroll
    for (int w = 0; w < 4; ++w) bs_transpose32(s + 32 * w);
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const uint64_t b = b0 + 64u * (uint64_t)j;
      u32x4 v = {s[j], s[32 + j], s[64 + j], s[96 + j]};
      if constexpr (XOR_IN) v ^= in[b];
      out[b] = v;
    }
  }
}

