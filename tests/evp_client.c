/* evp_client.c — a C caller of the BoringSSL EVP API written exactly like CryptMPI's naive
 * secure Alltoall (MV/src/mpi/coll/alltoall.c:764-836) and its CTR / sub-key calls
 * (send.c:583, :1722-1723), linked against libcmpi_evp.so (the drop-in) instead of libcrypto.
 * Reads key || nonces || plaintext blocks from argv files, writes the wire buffer and the
 * decrypted blocks.  Used by tests/test_gpu_evp_shim.py. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <dlfcn.h>

#include "../include/cmpi_evp.h"

/* CMPI_TEST_PROVOKE_HIP_ERROR (tests/test_gpu_errors.py): a HIP error of the caller's own is left
 * pending in this thread before the first EVP call; after the last one it must still be pending
 * (the drop-in reports only errors its own calls cause, and never clears the caller's). */
typedef int (*hip_int_fn)(int);
typedef int (*hip_void_fn)(void);
static int provoked = 0;
static hip_void_fn peek_last = 0;

int main(int argc, char **argv) {
  if (argc != 5) return 2;
  if (getenv("CMPI_TEST_PROVOKE_HIP_ERROR")) {
    void *h = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return 13;
    hip_int_fn set_device = (hip_int_fn)dlsym(h, "hipSetDevice");
    peek_last = (hip_void_fn)dlsym(h, "hipPeekAtLastError");
    if (!set_device || !peek_last) return 13;
    provoked = set_device(9999);
    if (provoked == 0 || peek_last() != provoked) return 13;
  }
  int p = atoi(argv[1]);          /* peers */
  unsigned long n = strtoul(argv[2], 0, 10); /* bytes per peer block */
  FILE *f = fopen(argv[3], "rb");
  if (!f) return 3;
  uint8_t key[16];
  uint8_t *nonces = malloc(12 * p), *sendbuf = malloc(n * p), *recvbuf = malloc(n * p + 16);
  uint8_t *ciphertext_sendbuf = malloc((n + 28) * p);
  if (fread(key, 1, 16, f) != 16 || fread(nonces, 1, 12 * p, f) != (size_t)(12 * p) ||
      fread(sendbuf, 1, n * p, f) != n * p)
    return 4;
  fclose(f);
  EVP_AEAD_CTX *ctx = EVP_AEAD_CTX_new(EVP_aead_aes_128_gcm(), key, 16, 0);
  if (!ctx) return 5;
  unsigned long ciphertext_sendbuf_len = 0, count = 0, max_out_len = 16 + n;
  for (int i = 0; i < p; i++) { /* alltoall.c:795-811 */
    unsigned long next = (unsigned long)i * (n + 16 + 12), src = (unsigned long)i * n;
    memcpy(ciphertext_sendbuf + next, nonces + 12 * i, 12); /* stands in for RAND_bytes */
    if (!EVP_AEAD_CTX_seal(ctx, ciphertext_sendbuf + next + 12, &ciphertext_sendbuf_len, max_out_len,
                           ciphertext_sendbuf + next, 12, sendbuf + src, n, NULL, 0))
      return 6;
  }
  /* (MPIR_Alltoall_impl would exchange ciphertext_sendbuf here; loop back to ourselves) */
  for (int i = 0; i < p; i++) { /* alltoall.c:821-834 */
    unsigned long next = (unsigned long)i * (n + 16 + 12), dest = (unsigned long)i * n;
    if (!EVP_AEAD_CTX_open(ctx, recvbuf + dest, &count, n + 16, ciphertext_sendbuf + next, 12,
                           ciphertext_sendbuf + next + 12, n + 16, NULL, 0))
      return 7;
  }
  /* a forged block must fail and zero the output */
  ciphertext_sendbuf[12] ^= 1;
  if (EVP_AEAD_CTX_open(ctx, recvbuf + n * p, &count, 16, ciphertext_sendbuf, 12, ciphertext_sendbuf + 12, 16, NULL, 0) &&
      n == 0)
    return 8;
  ciphertext_sendbuf[12] ^= 1;
  /* 602 sub-key (send.c:572-600) and CTR (send.c:1722-1723) through the same EVP surface */
  EVP_CIPHER_CTX *ctx_enc = EVP_CIPHER_CTX_new();
  EVP_EncryptInit_ex(ctx_enc, EVP_aes_128_ecb(), NULL, key, NULL);
  uint8_t V[16], newkey[16];
  int len = 0;
  memcpy(V, nonces, 12);
  memcpy(V + 12, nonces, 4);
  if (1 != EVP_EncryptUpdate(ctx_enc, newkey, &len, V, 16) || len != 16) return 9;
  EVP_CIPHER_CTX *cctx = EVP_CIPHER_CTX_new();
  EVP_EncryptInit_ex(cctx, EVP_aes_128_ctr(), NULL, key, NULL);
  uint8_t iv[16];
  memcpy(iv, nonces, 12);
  memset(iv + 12, 0xff, 4);
  uint8_t *ctr_out = malloc(n * p + 1);
  EVP_EncryptInit_ex(cctx, NULL, NULL, NULL, iv);
  unsigned long half = n * p / 3;
  if (1 != EVP_EncryptUpdate(cctx, ctr_out, &len, sendbuf, (int)half)) return 10;
  if (1 != EVP_EncryptUpdate(cctx, ctr_out + half, &len, sendbuf + half, (int)(n * p - half))) return 11;
  FILE *o = fopen(argv[4], "wb");
  fwrite(ciphertext_sendbuf, 1, (n + 28) * p, o);
  fwrite(recvbuf, 1, n * p, o);
  fwrite(newkey, 1, 16, o);
  fwrite(ctr_out, 1, n * p, o);
  fclose(o);
  EVP_AEAD_CTX_free(ctx);
  EVP_CIPHER_CTX_free(ctx_enc);
  EVP_CIPHER_CTX_free(cctx);
  if (provoked) {
    const int now = peek_last();
    if (now != provoked) {
      fprintf(stderr, "caller HIP error %d replaced by %d\n", provoked, now);
      return 12;
    }
    fprintf(stderr, "caller error preserved (%d)\n", now);
  }
  return 0;
}
