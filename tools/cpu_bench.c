/*
 * cpu_bench.c — CPU baseline for bench.py (NOT the oracle, NOT the product).
 *
 * The reference seals on the host with BoringSSL's AES-NI/PCLMUL code through EVP_AEAD_CTX_seal,
 * one context shared lock-free by an OpenMP team (MV/src/mpi/pt2pt/send.c:292-315; naive
 * collectives alltoall.c:795-834).  BoringSSL cannot be built here (its crypto/ sources are
 * absent), so the stand-in is the system OpenSSL 3 EVP AES-128-GCM/OCB/CTR (same
 * CRYPTOGAMS AES-NI lineage).  OpenSSL 3.0 serialises EVP calls of threads in ONE process on
 * internal locks (measured on the GPU box: 16 threads 6.3 GiB/s, 16 processes ~55 GiB/s, one
 * thread 3.6 GiB/s for 1 KiB GCM seals), which BoringSSL's AEAD path does not do — so the
 * workers here are PROCESSES (fork), each with its own libcrypto state, static partition over
 * records like `#pragma omp for schedule(static)`.
 *
 * Inputs are deterministic (splitmix64, the same streams as cryptmpi_2022_amd/synth.py):
 * plaintext = splitmix64_bytes(seed_pt, N*n) row-major, nonces = splitmix64_bytes(seed_n, 12*N).
 * Timing: a process-shared barrier releases every worker for a pass; the parent times from the
 * release to the last worker's arrival.  `warmup` untimed passes, then `reps` timed ones; the
 * median is reported.  Output: one JSON line (rates in GiB/s of plaintext) plus the tags of the
 * first 16 records (hex) so bench.py can check them against the GPU's tags for the same inputs.
 *
 *   cpu_bench <gcm|ocb|ctr> <n> <nrec> <procs> <warmup> <reps> <seed_pt> <seed_nonce>
 */
#define _GNU_SOURCE
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static void splitmix_fill(uint64_t seed, uint8_t *out, size_t nbytes) {
  uint64_t z0 = seed;
  size_t nw = (nbytes + 7) / 8;
  for (size_t i = 0; i < nw; ++i) {
    uint64_t z = z0 + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    size_t rem = nbytes - 8 * i;
    memcpy(out + 8 * i, &z, rem < 8 ? rem : 8);
  }
}

struct shared {
  pthread_barrier_t start, done;
  int bad;
};

static const uint8_t kKey[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};

/* one AEAD record with a context whose key schedule is set once (aead_setup) */
static int aead_setup(EVP_CIPHER_CTX *c, const EVP_CIPHER *ci, int dec, int ocb) {
  int ok = 1;
  if (dec) {
    ok &= EVP_DecryptInit_ex(c, ci, NULL, NULL, NULL);
    ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL);
    ok &= EVP_DecryptInit_ex(c, NULL, NULL, kKey, NULL);
  } else {
    ok &= EVP_EncryptInit_ex(c, ci, NULL, NULL, NULL);
    ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL);
    if (ocb) ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, NULL);
    ok &= EVP_EncryptInit_ex(c, NULL, NULL, kKey, NULL);
  }
  return ok;
}

static int aead_one(EVP_CIPHER_CTX *c, int dec, const uint8_t *nonce, const uint8_t *in, int n, uint8_t *out) {
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

static void add128(uint8_t cb[16], uint64_t k) {
  unsigned carry = 0;
  for (int i = 15; i >= 0; --i) {
    unsigned s = (unsigned)cb[i] + (unsigned)(k & 0xff) + carry;
    cb[i] = (uint8_t)s;
    carry = s >> 8;
    k >>= 8;
  }
}

static int cmp_dbl(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
  if (argc != 9) {
    fprintf(stderr, "usage: %s <gcm|ocb|ctr> <n> <nrec> <procs> <warmup> <reps> <seed_pt> <seed_nonce>\n", argv[0]);
    return 2;
  }
  const char *alg = argv[1];
  const int is_ctr = !strcmp(alg, "ctr"), is_ocb = !strcmp(alg, "ocb");
  if (!is_ctr && !is_ocb && strcmp(alg, "gcm")) return 2;
  const size_t n = strtoull(argv[2], 0, 0), N = strtoull(argv[3], 0, 0);
  const int P = atoi(argv[4]), W = atoi(argv[5]), R = atoi(argv[6]);
  const uint64_t seed_pt = strtoull(argv[7], 0, 0), seed_n = strtoull(argv[8], 0, 0);
  if (P < 1 || P > 1024 || R < 1 || W < 0 || !N || (n > 0x7fffffff)) return 2;
  const size_t in_b = N * n, ct_b = is_ctr ? N * n : N * (n + 16);
  uint8_t *pt = mmap(0, in_b, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  uint8_t *ct = mmap(0, ct_b, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  uint8_t *bk = mmap(0, in_b, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  uint8_t *nn = mmap(0, 12 * N, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  struct shared *sh = mmap(0, sizeof *sh, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (pt == MAP_FAILED || ct == MAP_FAILED || bk == MAP_FAILED || nn == MAP_FAILED || sh == MAP_FAILED) return 3;
  splitmix_fill(seed_pt, pt, in_b);
  splitmix_fill(seed_n, nn, 12 * N);
  memset(ct, 0, ct_b);
  memset(bk, 0, in_b);
  pthread_barrierattr_t ba;
  pthread_barrierattr_init(&ba);
  pthread_barrierattr_setpshared(&ba, PTHREAD_PROCESS_SHARED);
  pthread_barrier_init(&sh->start, &ba, (unsigned)P + 1);
  pthread_barrier_init(&sh->done, &ba, (unsigned)P + 1);
  sh->bad = 0;
  const int passes = W + R;
  fflush(stdout);
  for (int w = 0; w < P; ++w) {
    pid_t pid = fork();
    if (pid < 0) return 4;
    if (pid) continue;
    /* worker w: records [a, b) (CTR: 16-byte blocks [a, b) of the stream) */
    const size_t units = is_ctr ? (in_b + 15) / 16 : N;
    const size_t a = units * (size_t)w / (size_t)P, b = units * (size_t)(w + 1) / (size_t)P;
    int bad = 0;
    for (int dec = 0; dec < 2; ++dec) {
      EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
      const EVP_CIPHER *ci = is_ctr ? EVP_aes_128_ctr() : is_ocb ? EVP_aes_128_ocb() : EVP_aes_128_gcm();
      if (!is_ctr) bad += !aead_setup(c, ci, dec, is_ocb);
      for (int p = 0; p < passes; ++p) {
        pthread_barrier_wait(&sh->start);
        if (is_ctr) {
          uint8_t cb[16] = {0};
          add128(cb, a);
          int l = 0;
          const size_t off = a * 16, end = b * 16 < in_b ? b * 16 : in_b;
          bad += !EVP_EncryptInit_ex(c, ci, NULL, kKey, cb);
          if (end > off) bad += !EVP_EncryptUpdate(c, (dec ? bk : ct) + off, &l, (dec ? ct : pt) + off, (int)(end - off));
        } else {
          for (size_t i = a; i < b; ++i) {
            if (dec)
              bad += !aead_one(c, 1, nn + 12 * i, ct + i * (n + 16), (int)n, bk + i * n);
            else
              bad += !aead_one(c, 0, nn + 12 * i, pt + i * n, (int)n, ct + i * (n + 16));
          }
        }
        pthread_barrier_wait(&sh->done);
      }
      EVP_CIPHER_CTX_free(c);
    }
    if (bad) __atomic_add_fetch(&sh->bad, bad, __ATOMIC_SEQ_CST);
    _exit(0);
  }
  double *ts = calloc((size_t)R, sizeof(double)), *to = calloc((size_t)R, sizeof(double));
  for (int dec = 0; dec < 2; ++dec)
    for (int p = 0; p < passes; ++p) {
      pthread_barrier_wait(&sh->start);
      const double t0 = now();
      pthread_barrier_wait(&sh->done);
      const double dt = now() - t0;
      if (p >= W) (dec ? to : ts)[p - W] = dt;
    }
  for (int w = 0; w < P; ++w) wait(NULL);
  const int round_trip = memcmp(bk, pt, in_b) == 0;
  qsort(ts, (size_t)R, sizeof(double), cmp_dbl);
  qsort(to, (size_t)R, sizeof(double), cmp_dbl);
  const double ms = ts[R / 2], mo = to[R / 2], G = 1073741824.0;
  printf("{\"alg\": \"%s\", \"n\": %zu, \"nrec\": %zu, \"procs\": %d, \"warmup\": %d, \"reps\": %d, "
         "\"seal_median_s\": %.6g, \"open_median_s\": %.6g, \"seal_GiBps\": %.4f, \"open_GiBps\": %.4f, "
         "\"seal_open_GiBps\": %.4f, \"round_trip\": %s, \"failed\": %d, \"tags16\": [",
         alg, n, N, P, W, R, ms, mo, in_b / ms / G, in_b / mo / G, in_b / (ms + mo) / G, round_trip ? "true" : "false",
         sh->bad);
  const size_t k = is_ctr ? 0 : (N < 16 ? N : 16);
  for (size_t i = 0; i < k; ++i) {
    printf("%s\"", i ? ", " : "");
    for (int j = 0; j < 16; ++j) printf("%02x", ct[i * (n + 16) + n + (size_t)j]);
    printf("\"");
  }
  printf("]");
  if (is_ctr) {
    printf(", \"ct_head\": \"");
    for (size_t j = 0; j < 32 && j < in_b; ++j) printf("%02x", ct[j]);
    printf("\"");
  }
  printf("}\n");
  return sh->bad ? 1 : 0;
}
