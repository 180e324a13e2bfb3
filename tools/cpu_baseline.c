/*
 * cpu_baseline.c — CPU baseline harness for bench.py (NOT the oracle, NOT the product).
 *
 * Times the reference's CPU path as closely as this image allows: the reference seals with
 * BoringSSL's AES-NI/PCLMUL asm through EVP_AEAD_CTX_seal (send.c:311, alltoall.c:801); BoringSSL
 * cannot be built here (crypto/ sources absent), so this uses the system
 * OpenSSL 3 libcrypto EVP_aes_128_gcm / _ocb / _ctr (same CRYPTOGAMS AES-NI asm lineage),
 * with an OpenMP static partition over records exactly like send.c:292.
 */
#include <omp.h>
#include <openssl/evp.h>
#include <stdint.h>
#include <string.h>

/* Key schedule once per thread (like one EVP_AEAD_CTX shared by the OpenMP team, send.c:292),
 * then per record only the nonce is reset. */
static int aead_setup(EVP_CIPHER_CTX *c, const EVP_CIPHER *ci, int dec, const uint8_t *key) {
  int ok = 1;
  if (dec) {
    ok &= EVP_DecryptInit_ex(c, ci, NULL, NULL, NULL);
    ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL);
    ok &= EVP_DecryptInit_ex(c, NULL, NULL, key, NULL);
  } else {
    ok &= EVP_EncryptInit_ex(c, ci, NULL, NULL, NULL);
    ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL);
    if (ci == EVP_aes_128_ocb()) ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, NULL);
    ok &= EVP_EncryptInit_ex(c, NULL, NULL, key, NULL);
  }
  return ok;
}

static int aead_one(EVP_CIPHER_CTX *c, int dec, const uint8_t *nonce, const uint8_t *in, int n,
                    uint8_t *out) {
  int l = 0, ok = 1;
  if (dec) {
    ok &= EVP_DecryptInit_ex(c, NULL, NULL, NULL, nonce);
    ok &= EVP_DecryptUpdate(c, out, &l, in, n);
    ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, (void *)(in + n));
    ok &= EVP_DecryptFinal_ex(c, out + l, &l) > 0;
  } else {
    ok &= EVP_EncryptInit_ex(c, NULL, NULL, NULL, nonce);
    ok &= EVP_EncryptUpdate(c, out, &l, in, n);
    ok &= EVP_EncryptFinal_ex(c, out + l, &l);
    ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, out + n);
  }
  return ok;
}

/* alg 1 = GCM, 2 = OCB. Records: in + i*in_stride, out + i*out_stride, nonce + 12*i.
 * Returns the number of failed records. */
int cb_aead_batch(int alg, int dec, const uint8_t *key, const uint8_t *nonces, const uint8_t *in,
                  size_t in_stride, uint8_t *out, size_t out_stride, int n, long nrec, int nthreads) {
  const EVP_CIPHER *ci = alg == 2 ? EVP_aes_128_ocb() : EVP_aes_128_gcm();
  long bad = 0;
#pragma omp parallel num_threads(nthreads) reduction(+ : bad)
  {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    bad += !aead_setup(c, ci, dec, key);
#pragma omp for schedule(static)
    for (long i = 0; i < nrec; ++i)
      bad += !aead_one(c, dec, nonces + 12 * i, in + i * in_stride, n, out + i * out_stride);
    EVP_CIPHER_CTX_free(c);
  }
  return (int)bad;
}

/* CTR stream split on 16-byte boundaries, 128-bit BE counter advanced per thread. */
int cb_ctr(const uint8_t *key, const uint8_t ctr0[16], const uint8_t *in, uint8_t *out, size_t n,
           int nthreads) {
  size_t nblk = (n + 15) / 16, per = (nblk + nthreads - 1) / nthreads;
  int bad = 0;
#pragma omp parallel num_threads(nthreads) reduction(+ : bad)
  {
    int t = omp_get_thread_num();
    size_t b0 = per * t;
    if (b0 < nblk) {
      size_t b1 = b0 + per < nblk ? b0 + per : nblk, off = b0 * 16, end = b1 * 16 < n ? b1 * 16 : n;
      uint8_t cb[16];
      memcpy(cb, ctr0, 16);
      unsigned carry = 0;
      uint64_t k = b0;
      for (int i = 15; i >= 0; --i) {
        unsigned s = cb[i] + (unsigned)(k & 0xff) + carry;
        cb[i] = (uint8_t)s;
        carry = s >> 8;
        k >>= 8;
      }
      EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
      int l = 0;
      bad += !EVP_EncryptInit_ex(c, EVP_aes_128_ctr(), NULL, key, cb);
      bad += !EVP_EncryptUpdate(c, out + off, &l, in + off, (int)(end - off));
      EVP_CIPHER_CTX_free(c);
    }
  }
  return bad;
}
