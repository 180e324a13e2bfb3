/* evp_mt_client.c — CryptMPI's threaded use of the EVP surface, linked against libcmpi_evp.so
 * ahead of libcrypto (tests/test_gpu_evp_shim.py):
 *  1. an OpenMP-style team of T pthreads sealing its segments on ONE shared EVP_AEAD_CTX, then
 *     opening them (send.c:292-315 / :646-706, recv.c:305-330): ciphertexts go to the out file
 *     for a bit-exact check, every open must succeed;
 *  2. the 602 per-message context pattern (send.c:588-599): per message, T EVP_AEAD_CTX_new of
 *     one fresh key, one seal each, T frees — timed;
 *  3. EVP_aes_256_ecb (init.c:848 with SYMMETRIC_KEY_SIZE 32) through the shim's
 *     EVP_EncryptInit_ex/Update: forwarded to libcrypto, compared with libcrypto called directly.
 * usage: evp_mt_client T M n in.bin out.bin   (in = key(16) || nonces(T*M*12) || pt(T*M*n)) */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/cmpi_evp.h"

/* libcrypto's own; EVP_aes_256_ecb is not exported by the shim, so it resolves to libcrypto */
const EVP_CIPHER *EVP_aes_256_ecb(void);

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static int T, M;
static size_t n;
static uint8_t key[16], *nonces, *pt, *ct, *back;
static EVP_AEAD_CTX *shared;
static pthread_barrier_t bar;
static int failures;

static void *worker(void *arg) {
  const int t = (int)(long)arg;
  size_t ol;
  pthread_barrier_wait(&bar);
  for (int m = 0; m < M; ++m) {
    const size_t i = (size_t)t * M + m;
    if (!EVP_AEAD_CTX_seal(shared, ct + i * (n + 16), &ol, n + 16, nonces + 12 * i, 12, pt + i * n, n, NULL, 0) ||
        ol != n + 16)
      __sync_fetch_and_add(&failures, 1);
  }
  pthread_barrier_wait(&bar);
  for (int m = 0; m < M; ++m) {
    const size_t i = (size_t)t * M + m;
    if (!EVP_AEAD_CTX_open(shared, back + i * n, &ol, n, nonces + 12 * i, 12, ct + i * (n + 16), n + 16, NULL, 0) ||
        ol != n)
      __sync_fetch_and_add(&failures, 1);
  }
  return NULL;
}

int main(int argc, char **argv) {
  if (argc != 6) return 2;
  T = atoi(argv[1]);
  M = atoi(argv[2]);
  n = strtoul(argv[3], 0, 10);
  const size_t R = (size_t)T * M;
  FILE *f = fopen(argv[4], "rb");
  if (!f) return 3;
  nonces = malloc(12 * R);
  pt = malloc(n * R + 1);
  ct = malloc((n + 16) * R);
  back = malloc(n * R + 17);
  if (fread(key, 1, 16, f) != 16 || fread(nonces, 1, 12 * R, f) != 12 * R || fread(pt, 1, n * R, f) != n * R) return 4;
  fclose(f);

  /* 1. team on one shared context */
  shared = EVP_AEAD_CTX_new(EVP_aead_aes_128_gcm(), key, 16, 0);
  if (!shared) return 5;
  pthread_t th[256];
  pthread_barrier_init(&bar, NULL, (unsigned)T);
  const double t0 = now();
  for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, worker, (void *)(long)t);
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  const double team_s = now() - t0;
  if (failures || memcmp(back, pt, n * R)) return 6;
  EVP_AEAD_CTX_free(shared);

  /* 2. per-message contexts of a fresh key (602), T per message */
  const int msgs = 50;
  double t1 = now();
  for (int m = 0; m < msgs; ++m) {
    uint8_t k2[16];
    memcpy(k2, key, 16);
    k2[0] ^= (uint8_t)(m + 1);
    k2[1] ^= (uint8_t)(m >> 8);
    EVP_AEAD_CTX *cs[256];
    for (int t = 0; t < T; ++t)
      if (!(cs[t] = EVP_AEAD_CTX_new(EVP_aead_aes_128_gcm(), k2, 16, 0))) return 7;
    size_t ol;
    if (!EVP_AEAD_CTX_seal(cs[0], back, &ol, n + 16, nonces, 12, pt, n, NULL, 0)) return 8;
    for (int t = 0; t < T; ++t) EVP_AEAD_CTX_free(cs[t]);
  }
  const double newfree_us = (now() - t1) / msgs * 1e6;

  /* 3. a cipher the engine does not serve is forwarded to libcrypto */
  void *h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_NOLOAD);
  int fwd_ok = -1;
  if (h) {
    void *(*rnew)(void) = (void *(*)(void))dlsym(h, "EVP_CIPHER_CTX_new");
    int (*rinit)(void *, const void *, void *, const uint8_t *, const uint8_t *) =
        (int (*)(void *, const void *, void *, const uint8_t *, const uint8_t *))dlsym(h, "EVP_EncryptInit_ex");
    int (*rupd)(void *, uint8_t *, int *, const uint8_t *, int) =
        (int (*)(void *, uint8_t *, int *, const uint8_t *, int))dlsym(h, "EVP_EncryptUpdate");
    uint8_t k32[32], in[32], a[32], b[32];
    for (int i = 0; i < 32; ++i) k32[i] = (uint8_t)(3 * i + 1), in[i] = (uint8_t)(7 * i);
    int la = 0, lb = 0;
    void *rc = rnew();
    rinit(rc, EVP_aes_256_ecb(), NULL, k32, NULL);
    rupd(rc, a, &la, in, 32);
    EVP_CIPHER_CTX *sc = EVP_CIPHER_CTX_new();
    fwd_ok = EVP_EncryptInit_ex(sc, EVP_aes_256_ecb(), NULL, k32, NULL) == 1 && EVP_EncryptUpdate(sc, b, &lb, in, 32) == 1 &&
             la == 32 && lb == 32 && !memcmp(a, b, 32);
    /* the same shim context switches back to an engine cipher */
    uint8_t e1[16];
    int l1 = 0;
    fwd_ok = fwd_ok && EVP_EncryptInit_ex(sc, EVP_aes_128_ecb(), NULL, key, NULL) == 1 &&
             EVP_EncryptUpdate(sc, e1, &l1, in, 16) == 1 && l1 == 16;
    EVP_CIPHER_CTX_free(sc);
    FILE *g = fopen(argv[5], "wb");
    fwrite(ct, 1, (n + 16) * R, g);
    fwrite(e1, 1, 16, g);
    fclose(g);
  }
  printf("{\"threads\": %d, \"msgs_per_thread\": %d, \"n\": %zu, \"team_seal_open_s\": %.6f, "
         "\"team_msgs_per_s\": %.1f, \"ctx_new_free_us_per_msg\": %.2f, \"forwarded_aes256_ok\": %d}\n",
         T, M, n, team_s, 2.0 * R / team_s, newfree_us, fwd_ok);
  if (fwd_ok != 1) {  /* the engine's last error, for the test's failure message */
    const char *(*lerr)(void) = (const char *(*)(void))dlsym(RTLD_DEFAULT, "cmpi_last_error");
    fprintf(stderr, "engine: %s\n", lerr ? lerr() : "?");
  }
  return fwd_ok == 1 ? 0 : 9;
}
