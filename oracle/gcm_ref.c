/*
 * gcm_ref.c — AES-128-GCM AEAD, restatement of NIST SP 800-38D (Algorithms 1-5) with the
 * EVP_AEAD_CTX_seal/open contract of MV/boringssl-master/include/openssl/aead.h:236-285.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Reference call sites this mirrors: seal MV/src/mpi/pt2pt/send.c:311 (600), :689 / :812 (602),
 * MV/src/mpi/coll/alltoall.c:801 (naive 1002); open MV/src/mpi/pt2pt/recv.c:322,
 * MV/src/mpi/coll/alltoall.c:826.  All pass a 12-byte nonce, no AAD, tag_len 0 (= 16).
 */
#include "oracle.h"

#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static uint64_t load_be64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}
static void store_be64(uint8_t *p, uint64_t v) {
  for (int i = 7; i >= 0; --i) {
    p[i] = (uint8_t)v;
    v >>= 8;
  }
}

/* SP 800-38D Algorithm 1: bit 0 of a block is the MSB of byte 0. */
void orc_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t z[16]) {
  uint64_t zh = 0, zl = 0;
  uint64_t vh = load_be64(y), vl = load_be64(y + 8);
  for (int i = 0; i < 128; ++i) {
    int bit = (x[i >> 3] >> (7 - (i & 7))) & 1;
    if (bit) {
      zh ^= vh;
      zl ^= vl;
    }
    int lsb = (int)(vl & 1);
    vl = (vl >> 1) | (vh << 63);
    vh >>= 1;
    if (lsb) vh ^= 0xE100000000000000ULL; /* R = 11100001 || 0^120 */
  }
  store_be64(z, zh);
  store_be64(z + 8, zl);
}

static void ghash_update(const uint8_t h[16], uint8_t y[16], const uint8_t *data, size_t len) {
  uint8_t blk[16];
  while (len) {
    size_t n = len < 16 ? len : 16;
    memset(blk, 0, 16);
    memcpy(blk, data, n);
    for (int i = 0; i < 16; ++i) y[i] ^= blk[i];
    orc_gf128_mul(y, h, y);
    data += n;
    len -= n;
  }
}

/* GHASH_H(A || 0^v || C || 0^u || [len(A)]_64 || [len(C)]_64) — SP 800-38D Algorithm 2/4. */
void orc_ghash(const uint8_t h[16], const uint8_t *aad, size_t aad_len, const uint8_t *c,
               size_t c_len, uint8_t out[16]) {
  uint8_t y[16] = {0}, lb[16];
  ghash_update(h, y, aad, aad_len);
  ghash_update(h, y, c, c_len);
  store_be64(lb, (uint64_t)aad_len * 8);
  store_be64(lb + 8, (uint64_t)c_len * 8);
  ghash_update(h, y, lb, 16);
  memcpy(out, y, 16);
}

static void inc32(uint8_t cb[16]) {
  for (int i = 15; i >= 12; --i)
    if (++cb[i]) break;
}

static void gcm_j0(const uint8_t h[16], const uint8_t *nonce, size_t nonce_len, uint8_t j0[16]) {
  if (nonce_len == 12) {
    memcpy(j0, nonce, 12);
    j0[12] = j0[13] = j0[14] = 0;
    j0[15] = 1;
  } else {
    orc_ghash(h, NULL, 0, nonce, nonce_len, j0); /* s = 128*ceil(len/128) - len; [0]_64 || [len]_64 */
  }
}

/* GCTR_K(icb, x) with inc32 (SP 800-38D Algorithm 3). */
static void gctr(const uint8_t rk[176], const uint8_t icb[16], const uint8_t *in, uint8_t *out,
                 size_t n) {
  uint8_t cb[16], ks[16];
  memcpy(cb, icb, 16);
  for (size_t off = 0; off < n; off += 16) {
    orc_aes128_encrypt(rk, cb, ks);
    size_t m = n - off < 16 ? n - off : 16;
    for (size_t i = 0; i < m; ++i) out[off + i] = (uint8_t)(in[off + i] ^ ks[i]);
    inc32(cb);
  }
}

int orc_gcm_seal(const uint8_t key[16], const uint8_t *nonce, size_t nonce_len, const uint8_t *ad,
                 size_t ad_len, const uint8_t *in, size_t in_len, uint8_t *out) {
  uint8_t rk[176], h[16] = {0}, j0[16], cb[16], s[16], ekj0[16];
  if (nonce_len == 0) return 0;
  orc_aes128_expand(key, rk);
  orc_aes128_encrypt(rk, h, h);
  gcm_j0(h, nonce, nonce_len, j0);
  memcpy(cb, j0, 16);
  inc32(cb);
  gctr(rk, cb, in, out, in_len);
  orc_ghash(h, ad, ad_len, out, in_len, s);
  orc_aes128_encrypt(rk, j0, ekj0);
  for (int i = 0; i < 16; ++i) out[in_len + i] = (uint8_t)(s[i] ^ ekj0[i]);
  return 1;
}

int orc_gcm_open(const uint8_t key[16], const uint8_t *nonce, size_t nonce_len, const uint8_t *ad,
                 size_t ad_len, const uint8_t *in, size_t in_len, uint8_t *out) {
  uint8_t rk[176], h[16] = {0}, j0[16], cb[16], s[16], ekj0[16];
  if (nonce_len == 0 || in_len < 16) return 0;
  size_t n = in_len - 16;
  orc_aes128_expand(key, rk);
  orc_aes128_encrypt(rk, h, h);
  gcm_j0(h, nonce, nonce_len, j0);
  orc_ghash(h, ad, ad_len, in, n, s);
  orc_aes128_encrypt(rk, j0, ekj0);
  uint8_t diff = 0;
  for (int i = 0; i < 16; ++i) diff |= (uint8_t)(s[i] ^ ekj0[i] ^ in[n + i]);
  if (diff) {
    memset(out, 0, n);
    return 0;
  }
  memcpy(cb, j0, 16);
  inc32(cb);
  gctr(rk, cb, in, out, n);
  return 1;
}

void orc_gcm_seal_batch(const uint8_t key[16], const uint8_t *nonces, size_t nonce_stride,
                        const uint8_t *in, size_t in_stride, uint8_t *out, size_t out_stride,
                        size_t len, size_t nrec, int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_num_procs();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
  for (long i = 0; i < (long)nrec; ++i)
    orc_gcm_seal(key, nonces + (size_t)i * nonce_stride, 12, NULL, 0, in + (size_t)i * in_stride,
                 len, out + (size_t)i * out_stride);
  (void)nthreads;
}

void orc_gcm_open_batch(const uint8_t key[16], const uint8_t *nonces, size_t nonce_stride,
                        const uint8_t *in, size_t in_stride, uint8_t *out, size_t out_stride,
                        size_t len, size_t nrec, int32_t *status, int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_num_procs();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
  for (long i = 0; i < (long)nrec; ++i) {
    int ok = orc_gcm_open(key, nonces + (size_t)i * nonce_stride, 12, NULL, 0,
                          in + (size_t)i * in_stride, len + 16, out + (size_t)i * out_stride);
    if (status) status[i] = ok;
  }
  (void)nthreads;
}
