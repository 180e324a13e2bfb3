/*
 * ctr_ref.c — AES-128-CTR keystream+XOR and CryptMPI's IV_Count helpers.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CTR: EVP_aes_128_ctr with a fresh EVP_EncryptInit_ex(ctx, NULL, NULL, NULL, iv) before each
 * EVP_EncryptUpdate (MV/src/mpi/pt2pt/send.c:985-1008 (700), :1716-1727 and :1805-1808 (702),
 * MV/src/mpi/pt2pt/recv.c:869-937, :1187-1220).  The EVP CTR mode increments the whole 16-byte
 * counter block as a 128-bit big-endian integer (SP 800-38A §B.1 standard incrementing).
 * IV_Count/IV_Count_out: MV/src/mpi/pt2pt/send.c:1019-1041, restated byte for byte.
 */
#include "oracle.h"

#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static void inc128(uint8_t cb[16]) {
  for (int i = 15; i >= 0; --i)
    if (++cb[i]) break;
}

/* cb += k (128-bit big-endian, k < 2^64) */
static void add128(uint8_t cb[16], uint64_t k) {
  unsigned carry = 0;
  for (int i = 15; i >= 0; --i) {
    unsigned s = (unsigned)cb[i] + (unsigned)(k & 0xff) + carry;
    cb[i] = (uint8_t)s;
    carry = s >> 8;
    k >>= 8;
  }
}

void orc_ctr128_xor(const uint8_t key[16], const uint8_t ctr0[16], const uint8_t *in, uint8_t *out,
                    size_t n) {
  uint8_t rk[176], cb[16], ks[16];
  orc_aes128_expand(key, rk);
  memcpy(cb, ctr0, 16);
  for (size_t off = 0; off < n; off += 16) {
    orc_aes128_encrypt(rk, cb, ks);
    size_t m = n - off < 16 ? n - off : 16;
    for (size_t i = 0; i < m; ++i) out[off + i] = (uint8_t)(in[off + i] ^ ks[i]);
    inc128(cb);
  }
}

void orc_ctr128_xor_mt(const uint8_t key[16], const uint8_t ctr0[16], const uint8_t *in,
                       uint8_t *out, size_t n, int nthreads) {
  size_t nblk = (n + 15) / 16;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_num_procs();
#else
  nthreads = 1;
#endif
  size_t per = (nblk + (size_t)nthreads - 1) / (size_t)nthreads;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
  for (int t = 0; t < nthreads; ++t) {
    size_t b0 = (size_t)t * per;
    if (b0 >= nblk) continue;
    size_t b1 = b0 + per < nblk ? b0 + per : nblk;
    size_t off = b0 * 16, end = b1 * 16 < n ? b1 * 16 : n;
    uint8_t cb[16];
    memcpy(cb, ctr0, 16);
    add128(cb, b0);
    orc_ctr128_xor(key, cb, in + off, out + off, end - off);
  }
}

void orc_iv_count(uint8_t iv[16], unsigned long cter) {
  uint32_t n = 16, c = (uint32_t)cter;
  do {
    --n;
    c += iv[n];
    iv[n] = (uint8_t)c;
    c >>= 8;
  } while (n);
}

void orc_iv_count_out(uint8_t iv[16], unsigned long cter, const uint8_t in[16]) {
  uint32_t n = 16, c = (uint32_t)cter;
  do {
    --n;
    c += in[n];
    iv[n] = (uint8_t)c;
    c >>= 8;
  } while (n);
}
