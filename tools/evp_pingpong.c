/*
 * evp_pingpong.c — CryptMPI's per-message 600 exchange between two processes, in C, through the
 * BoringSSL ABI.
 *
 * Two processes (fork, before any GPU call) exchange messages over a shared-memory mailbox — the
 * intra-node eager path of an MPI library: a send copies the bytes into the mailbox, a receive
 * copies them out.  Per message, exactly what MPI_SEC_Multi_Thread_Send_OpenMP /
 * MPI_SEC_Multi_Thread_Recv_OpenMP do (MV/src/mpi/pt2pt/send.c:221-337, recv.c:219-341):
 *   sender:   25-byte header into large_send_buffer ([0..3] BE32 n, [20] '1', [21..24] BE32 n),
 *             MPI_Isend(header) — issued before the seal (send.c:288);
 *             RAND_bytes(nonce, 12) into large_send_buffer + 25;
 *             EVP_AEAD_CTX_seal(ctx, large_send_buffer + 37, &len, n + 16, nonce, 12, buf, n, NULL, 0)
 *             (send.c:311); MPI_Isend(large_send_buffer + 25, n + 28); wait both;
 *   receiver: MPI_Recv(large_recv_buffer, 25); MPI_Recv(large_recv_buffer, n + 28) (recv.c:288);
 *             EVP_AEAD_CTX_open(ctx, buf, &count, n, large_recv_buffer, 12,
 *                               large_recv_buffer + 12, n + 16, NULL, 0) (recv.c:322).
 * large_send_buffer / large_recv_buffer are static arrays, as CryptMPI's are (mpiimpl.h:292-293);
 * the user buffers are malloc'd (pageable).  The plaintext mode is the same exchange as a plain
 * MPI_Send / MPI_Recv of n bytes, so secure - plain = what the crypto adds per one-way message.
 *
 * Crypto provider, chosen at build time (one source, identical call sites):
 *   default           the drop-in: link against cryptmpi_2022_amd/libcmpi_evp.so
 *   -DPROVIDER_OPENSSL the CPU path: the same EVP_AEAD_CTX_* calls served by OpenSSL 3's
 *                      EVP_aes_128_gcm on the calling core (BoringSSL's AES-NI/PCLMUL stand-in)
 *
 * usage: evp_pingpong <plain|secure> <bytes> <iters> [warmup_seconds]
 * Prints one JSON line: one-way latency (round trip / 2) median / mean / p90 in us.  Each side
 * checks every received plaintext against what its peer sent (the message carries its index).
 * Both processes bind to the CPUs of the GPU's NUMA node (CMPI_NUMA_BIND=0: no binding).
 * PINGPONG_REGISTER_USER=1 page-locks the user buffers as well (attribution of the bounce copies);
 * PINGPONG_DUMP=<path> writes rank 1's last received wire record and its plaintext (parity tests).
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <dlfcn.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/random.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#define MSG_HEADER_SIZE 25
#define MAX_MSG (4u << 20)
#define BUF_SIZE (MAX_MSG + 4096)

/* ------------------------------------------------------------------ crypto provider */
#ifdef PROVIDER_OPENSSL
#include <openssl/evp.h>
typedef EVP_CIPHER_CTX PCTX;
static PCTX *aead_new(const uint8_t key[16]) {
  EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
  if (!c || !EVP_CipherInit_ex(c, EVP_aes_128_gcm(), NULL, key, NULL, 1)) return NULL;
  return c;
}
static int aead_seal(PCTX *c, uint8_t *out, size_t *out_len, size_t max_out, const uint8_t *nonce, const uint8_t *in,
                     size_t n) {
  int l = 0, ok = max_out >= n + 16;
  ok = ok && EVP_CipherInit_ex(c, NULL, NULL, NULL, nonce, 1) && EVP_CipherUpdate(c, out, &l, in, (int)n) &&
       EVP_CipherFinal_ex(c, out + l, &l) && EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, out + n);
  *out_len = ok ? n + 16 : 0;
  return ok;
}
static int aead_open(PCTX *c, uint8_t *out, size_t *out_len, size_t max_out, const uint8_t *nonce, const uint8_t *in,
                     size_t in_len) {
  int l = 0;
  const size_t n = in_len - 16;
  int ok = in_len >= 16 && max_out >= n;
  ok = ok && EVP_CipherInit_ex(c, NULL, NULL, NULL, nonce, 0) && EVP_CipherUpdate(c, out, &l, in, (int)n) &&
       EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, (void *)(in + n)) && EVP_CipherFinal_ex(c, out + l, &l) > 0;
  *out_len = ok ? n : 0;
  return ok;
}
static const char *provider = "openssl3-cpu";
#else
#include "../include/cmpi_evp.h"
typedef EVP_AEAD_CTX PCTX;
static PCTX *aead_new(const uint8_t key[16]) { return EVP_AEAD_CTX_new(EVP_aead_aes_128_gcm(), key, 16, 0); }
static int aead_seal(PCTX *c, uint8_t *out, size_t *out_len, size_t max_out, const uint8_t *nonce, const uint8_t *in,
                     size_t n) {
  return EVP_AEAD_CTX_seal(c, out, out_len, max_out, nonce, 12, in, n, NULL, 0);
}
static int aead_open(PCTX *c, uint8_t *out, size_t *out_len, size_t max_out, const uint8_t *nonce, const uint8_t *in,
                     size_t in_len) {
  return EVP_AEAD_CTX_open(c, out, out_len, max_out, nonce, 12, in, in_len, NULL, 0);
}
static const char *provider = "libcmpi_evp.so";
#endif

/* CryptMPI's per-process message buffers: static storage (mpiimpl.h:292-293) */
static unsigned char large_send_buffer[BUF_SIZE];
static unsigned char large_recv_buffer[BUF_SIZE];

/* ------------------------------------------------------------------ shared-memory transport */
#define SLOTS 4
typedef struct {
  _Atomic uint64_t posted; /* messages written into the ring */
  char pad0[56];
  _Atomic uint64_t taken; /* messages copied out */
  char pad1[56];
  uint64_t len[SLOTS];
  unsigned char data[SLOTS][BUF_SIZE];
} Chan;

static void chan_send(Chan *ch, const void *buf, size_t len) { /* MPI_Send: copy in, publish */
  const uint64_t k = atomic_load_explicit(&ch->posted, memory_order_relaxed);
  while (k - atomic_load_explicit(&ch->taken, memory_order_acquire) >= SLOTS) {
  }
  memcpy(ch->data[k % SLOTS], buf, len);
  ch->len[k % SLOTS] = len;
  atomic_store_explicit(&ch->posted, k + 1, memory_order_release);
}

static size_t chan_recv(Chan *ch, void *buf) { /* MPI_Recv: wait, copy out, release the slot */
  const uint64_t k = atomic_load_explicit(&ch->taken, memory_order_relaxed);
  while (atomic_load_explicit(&ch->posted, memory_order_acquire) <= k) {
  }
  const size_t len = ch->len[k % SLOTS];
  memcpy(buf, ch->data[k % SLOTS], len);
  atomic_store_explicit(&ch->taken, k + 1, memory_order_release);
  return len;
}

/* ------------------------------------------------------------------ 600 framing */
static int secure_send(PCTX *ctx, Chan *ch, const uint8_t *buf, size_t n) {
  unsigned char *h = large_send_buffer;
  const uint32_t t = (uint32_t)n;
  h[0] = t >> 24, h[1] = t >> 16, h[2] = t >> 8, h[3] = t;
  h[20] = '1';
  h[21] = t >> 24, h[22] = t >> 16, h[23] = t >> 8, h[24] = t;
  chan_send(ch, h, MSG_HEADER_SIZE); /* MPI_Isend of the header, before the seal (send.c:288) */
  if (getrandom(h + MSG_HEADER_SIZE, 12, 0) != 12) return 0; /* RAND_bytes (send.c:294) */
  size_t clen = 0;
  if (!aead_seal(ctx, h + MSG_HEADER_SIZE + 12, &clen, n + 16, h + MSG_HEADER_SIZE, buf, n)) return 0;
  chan_send(ch, h + MSG_HEADER_SIZE, n + 28);
  return clen == n + 16;
}

static int secure_recv(PCTX *ctx, Chan *ch, uint8_t *buf, size_t *n_out) {
  chan_recv(ch, large_recv_buffer);
  const unsigned char *h = large_recv_buffer;
  const size_t n = ((size_t)h[0] << 24) | ((size_t)h[1] << 16) | ((size_t)h[2] << 8) | h[3];
  if (chan_recv(ch, large_recv_buffer) != n + 28) return 0;
  size_t count = 0;
  const int ok = aead_open(ctx, buf, &count, n, large_recv_buffer, large_recv_buffer + 12, n + 16);
  *n_out = count;
  return ok && count == n;
}

/* ------------------------------------------------------------------ placement, timing */
static int bind_gpu_node(int *bound) { /* as tools/msg_latency.hip: the CPUs of the GPU's node */
  *bound = 0;
  const char *env = getenv("CMPI_NUMA_BIND");
  if (env && atoi(env) == 0) return -1;
  void *hip = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
  if (!hip) return -1;
  int (*busid)(char *, int, int) = (int (*)(char *, int, int))dlsym(hip, "hipDeviceGetPCIBusId");
  char bus[64] = {0}, path[160], list[4096] = {0};
  if (!busid || busid(bus, sizeof bus, 0) != 0) return -1;
  for (char *q = bus; *q; ++q) *q = (char)tolower(*q);
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE *f = fopen(path, "r");
  int node = -1;
  if (!f) return -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  if (node < 0) return node;
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  if (!(f = fopen(path, "r"))) return node;
  const int ok = fgets(list, sizeof list, f) != NULL;
  fclose(f);
  if (!ok) return node;
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return node;
  for (char *tok = strtok(list, ",\n"); tok; tok = strtok(NULL, ",\n")) {
    int a = -1, b = -1;
    if (sscanf(tok, "%d-%d", &a, &b) < 2) b = a;
    for (int c = a; c >= 0 && c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) CPU_SET(c, &want);
  }
  const int n = CPU_COUNT(&want);
  if (n > 0 && sched_setaffinity(0, sizeof want, &want) == 0) *bound = n;
  return node;
}

static double now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmp_d(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

static void fill(uint8_t *b, size_t n, uint64_t seed) { /* splitmix64 */
  for (size_t i = 0; i < n; i += 8) {
    uint64_t z = (seed += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    memcpy(b + i, &z, n - i < 8 ? n - i : 8);
  }
}

/* One side of the ping-pong: rank 0 sends then receives, rank 1 receives then sends.  Message i
 * from rank r carries seed (r << 32 | i), so each receiver checks every plaintext. */
static int run_side(int rank, int secure, size_t n, long iters, double warm_s, Chan *tx, Chan *rx, double *rtt) {
  int bound = 0;
  const int node = bind_gpu_node(&bound);
  uint8_t key[16];
  for (int i = 0; i < 16; ++i) key[i] = (uint8_t)(0x30 + i);
  PCTX *ctx = secure ? aead_new(key) : NULL;
  if (secure && !ctx) return 2;
  uint8_t *sbuf = NULL, *rbuf = NULL, *want = malloc(n + 64);
  const size_t ucap = (n + 64 + 4095) & ~(size_t)4095;
  if (posix_memalign((void **)&sbuf, 4096, ucap) || posix_memalign((void **)&rbuf, 4096, ucap) || !want) return 2;
  /* PINGPONG_REGISTER_USER=1: the user buffers page-locked too (cmpi_host_register, what an MPI
   * library's registration cache would do) — attributes the pageable bounce copies */
  const char *ru = getenv("PINGPONG_REGISTER_USER");
  if (secure && ru && atoi(ru)) {
    int (*reg)(void *, size_t) = (int (*)(void *, size_t))dlsym(RTLD_DEFAULT, "cmpi_host_register");
    if (!reg || reg(sbuf, ucap) != 0 || reg(rbuf, ucap) != 0) return 2;
  }
  int bad = 0;
  long total = -1; /* warm-up messages until warm_s has passed, then `iters` timed round trips */
  const double t_warm = now_us() + warm_s * 1e6;
  for (long i = 0;; ++i) {
    int stop = 0;
    if (total < 0 && rank == 0 && now_us() >= t_warm) total = i + iters;
    /* rank 0 tells rank 1 when the run ends: the message's first byte is 1 on the last one */
    fill(sbuf, n, ((uint64_t)rank << 32) | (uint64_t)i);
    const double t0 = now_us();
    for (int phase = 0; phase < 2; ++phase) {
      if (phase == rank) { /* send */
        if (n) sbuf[0] = rank == 0 ? (uint8_t)(total >= 0 && i + 1 == total) : 0;
        if (secure) bad |= !secure_send(ctx, tx, sbuf, n);
        else chan_send(tx, sbuf, n);
      } else { /* receive and check */
        size_t got = n;
        if (secure) bad |= !secure_recv(ctx, rx, rbuf, &got);
        else got = chan_recv(rx, rbuf);
        fill(want, n, ((uint64_t)(1 - rank) << 32) | (uint64_t)i);
        if (n && rank == 1) stop = rbuf[0], want[0] = rbuf[0];
        if (n && rank == 0) want[0] = 0;
        bad |= got != n || memcmp(rbuf, want, n) != 0;
      }
    }
    if (rank == 0 && total >= 0 && i >= total - iters) rtt[i - (total - iters)] = now_us() - t0;
    /* PINGPONG_DUMP=<path>: rank 1 writes the last wire record it received (nonce || ct || tag, as
     * large_recv_buffer holds it) and the plaintext it opened, for a parity check against an oracle */
    const char *dump = getenv("PINGPONG_DUMP");
    if (dump && secure && rank == 1 && stop) {
      FILE *f = fopen(dump, "wb");
      if (!f || fwrite(large_recv_buffer, 1, n + 28, f) != n + 28 || fwrite(rbuf, 1, n, f) != n) bad = 1;
      if (f) fclose(f);
    }
    if ((rank == 0 && total >= 0 && i + 1 == total) || (rank == 1 && stop)) break;
  }
  if (rank == 0) fprintf(stderr, "numa_node=%d bound_cpus=%d\n", node, bound);
  free(sbuf);
  free(rbuf);
  free(want);
  return bad ? 3 : 0;
}

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <plain|secure> <bytes> <iters> [warmup_seconds]\n", argv[0]);
    return 1;
  }
  const int secure = strcmp(argv[1], "secure") == 0;
  const size_t n = strtoull(argv[2], NULL, 10);
  const long iters = atol(argv[3]);
  const double warm = argc > 4 ? atof(argv[4]) : 0.3;
  if (n == 0 || n > MAX_MSG || iters < 1) return 1;
  Chan *ch = mmap(NULL, 2 * sizeof(Chan), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  double *rtt = mmap(NULL, sizeof(double) * iters, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (ch == MAP_FAILED || rtt == MAP_FAILED) return 2;
  const pid_t pid = fork(); /* before anything touches the GPU */
  if (pid < 0) return 2;
  if (pid == 0) _exit(run_side(1, secure, n, iters, warm, &ch[1], &ch[0], rtt));
  const int rc0 = run_side(0, secure, n, iters, warm, &ch[0], &ch[1], rtt);
  int st = 0;
  waitpid(pid, &st, 0);
  const int rc1 = WIFEXITED(st) ? WEXITSTATUS(st) : 4;
  qsort(rtt, iters, sizeof(double), cmp_d);
  double sum = 0;
  for (long i = 0; i < iters; ++i) sum += rtt[i];
  printf("{\"provider\": \"%s\", \"mode\": \"%s\", \"bytes\": %zu, \"iters\": %ld, \"oneway_us_median\": %.3f, "
         "\"oneway_us_mean\": %.3f, \"oneway_us_p90\": %.3f, \"verified\": %s}\n",
         provider, secure ? "secure" : "plain", n, iters, rtt[iters / 2] / 2, sum / iters / 2,
         rtt[iters * 9 / 10] / 2, rc0 == 0 && rc1 == 0 ? "true" : "false");
  return rc0 ? rc0 : rc1;
}
