/*
 * ocb_ref.c — AES-128-OCB3, restatement of RFC 7253 §4 (TAGLEN = 128).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The reference advertises "Naive OCB" / "OCB 2/4 unrolling" (MV2_SECURITY_APPROACH=402 etc.,
 * /root/reference/README.md:128-129, :188-197) but ships no OCB code and builds BoringSSL with
 * OPENSSL_NO_OCB (MV/boringssl-master/include/openssl/opensslconf.h:49).  Parity vs the
 * reference is therefore UNPINNED; this restatement is pinned to RFC 7253 Appendix A and to
 * the system OpenSSL 3 EVP_aes_128_ocb (tests/golden/gen_openssl_vectors.py).
 */
#include "oracle.h"

#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static void dbl(const uint8_t in[16], uint8_t out[16]) {
  uint8_t carry = (uint8_t)(in[0] >> 7);
  for (int i = 0; i < 15; ++i) out[i] = (uint8_t)((in[i] << 1) | (in[i + 1] >> 7));
  out[15] = (uint8_t)((in[15] << 1) ^ (carry ? 0x87 : 0x00));
}

static void xor16(uint8_t *d, const uint8_t *a) {
  for (int i = 0; i < 16; ++i) d[i] ^= a[i];
}

static unsigned ntz(size_t i) {
  unsigned n = 0;
  while (!(i & 1)) {
    i >>= 1;
    ++n;
  }
  return n;
}

typedef struct {
  uint8_t rk[176];
  uint8_t lstar[16], ldollar[16], l[64][16];
} ocb_keys;

static void ocb_setup(const uint8_t key[16], ocb_keys *k) {
  uint8_t z[16] = {0};
  orc_aes128_expand(key, k->rk);
  orc_aes128_encrypt(k->rk, z, k->lstar);
  dbl(k->lstar, k->ldollar);
  dbl(k->ldollar, k->l[0]);
  for (int i = 1; i < 64; ++i) dbl(k->l[i - 1], k->l[i]);
}

static void ocb_hash(const ocb_keys *k, const uint8_t *a, size_t alen, uint8_t sum[16]) {
  uint8_t off[16] = {0}, t[16];
  memset(sum, 0, 16);
  size_t m = alen / 16;
  for (size_t i = 1; i <= m; ++i) {
    xor16(off, k->l[ntz(i)]);
    memcpy(t, a + 16 * (i - 1), 16);
    xor16(t, off);
    orc_aes128_encrypt(k->rk, t, t);
    xor16(sum, t);
  }
  size_t r = alen % 16;
  if (r) {
    xor16(off, k->lstar);
    memset(t, 0, 16);
    memcpy(t, a + 16 * m, r);
    t[r] = 0x80;
    xor16(t, off);
    orc_aes128_encrypt(k->rk, t, t);
    xor16(sum, t);
  }
}

/* Offset_0 from the nonce (RFC 7253 §4.2). nonce_len in 1..15. */
static void ocb_offset0(const ocb_keys *k, const uint8_t *nonce, size_t nonce_len, uint8_t off[16]) {
  uint8_t nb[16] = {0}, ktop[16], stretch[24];
  /* Nonce = num2str(TAGLEN mod 128, 7) || zeros(120 - bitlen(N)) || 1 || N ; TAGLEN = 128 */
  memcpy(nb + 16 - nonce_len, nonce, nonce_len);
  nb[15 - nonce_len] |= 0x01;
  unsigned bottom = nb[15] & 0x3f;
  nb[15] &= 0xc0;
  orc_aes128_encrypt(k->rk, nb, ktop);
  memcpy(stretch, ktop, 16);
  for (int i = 0; i < 8; ++i) stretch[16 + i] = (uint8_t)(ktop[i] ^ ktop[i + 1]);
  unsigned byte = bottom / 8, bit = bottom % 8;
  for (int i = 0; i < 16; ++i) {
    unsigned v = (unsigned)stretch[i + byte] << 8 | (i + byte + 1 < 24 ? stretch[i + byte + 1] : 0);
    off[i] = (uint8_t)(v >> (8 - bit));
  }
}

static void ocb_crypt(const ocb_keys *k, const uint8_t *nonce, size_t nonce_len, const uint8_t *in,
                      size_t n, uint8_t *out, int decrypt, uint8_t tag_pre[16]) {
  uint8_t off[16], sum[16] = {0}, t[16];
  ocb_offset0(k, nonce, nonce_len, off);
  size_t m = n / 16;
  for (size_t i = 1; i <= m; ++i) {
    xor16(off, k->l[ntz(i)]);
    memcpy(t, in + 16 * (i - 1), 16);
    if (!decrypt) xor16(sum, t);
    xor16(t, off);
    if (decrypt)
      orc_aes128_decrypt(k->rk, t, t);
    else
      orc_aes128_encrypt(k->rk, t, t);
    xor16(t, off);
    memcpy(out + 16 * (i - 1), t, 16);
    if (decrypt) xor16(sum, t);
  }
  size_t r = n % 16;
  if (r) {
    uint8_t pad[16], pst[16] = {0};
    xor16(off, k->lstar);
    orc_aes128_encrypt(k->rk, off, pad);
    for (size_t j = 0; j < r; ++j) out[16 * m + j] = (uint8_t)(in[16 * m + j] ^ pad[j]);
    memcpy(pst, decrypt ? out + 16 * m : in + 16 * m, r);
    pst[r] = 0x80;
    xor16(sum, pst);
  }
  /* Tag = E(Checksum xor Offset xor L_$) xor HASH(K, A) — caller XORs the HASH */
  memcpy(t, sum, 16);
  xor16(t, off);
  xor16(t, k->ldollar);
  orc_aes128_encrypt(k->rk, t, tag_pre);
}

int orc_ocb_seal(const uint8_t key[16], const uint8_t *nonce, size_t nonce_len, const uint8_t *ad,
                 size_t ad_len, const uint8_t *in, size_t in_len, uint8_t *out) {
  ocb_keys k;
  uint8_t tag[16], h[16];
  if (nonce_len < 1 || nonce_len > 15) return 0;
  ocb_setup(key, &k);
  ocb_crypt(&k, nonce, nonce_len, in, in_len, out, 0, tag);
  ocb_hash(&k, ad, ad_len, h);
  xor16(tag, h);
  memcpy(out + in_len, tag, 16);
  return 1;
}

int orc_ocb_open(const uint8_t key[16], const uint8_t *nonce, size_t nonce_len, const uint8_t *ad,
                 size_t ad_len, const uint8_t *in, size_t in_len, uint8_t *out) {
  ocb_keys k;
  uint8_t tag[16], h[16];
  if (nonce_len < 1 || nonce_len > 15 || in_len < 16) return 0;
  size_t n = in_len - 16;
  ocb_setup(key, &k);
  ocb_crypt(&k, nonce, nonce_len, in, n, out, 1, tag);
  ocb_hash(&k, ad, ad_len, h);
  xor16(tag, h);
  uint8_t diff = 0;
  for (int i = 0; i < 16; ++i) diff |= (uint8_t)(tag[i] ^ in[n + i]);
  if (diff) {
    memset(out, 0, n);
    return 0;
  }
  return 1;
}

void orc_ocb_seal_batch(const uint8_t key[16], const uint8_t *nonces, size_t nonce_stride,
                        const uint8_t *in, size_t in_stride, uint8_t *out, size_t out_stride,
                        size_t len, size_t nrec, int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_num_procs();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
  for (long i = 0; i < (long)nrec; ++i)
    orc_ocb_seal(key, nonces + (size_t)i * nonce_stride, 12, NULL, 0, in + (size_t)i * in_stride,
                 len, out + (size_t)i * out_stride);
  (void)nthreads;
}
