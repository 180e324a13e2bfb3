/*
 * cmpi_evp.h — the BoringSSL entry points CryptMPI imports, re-exported by libcmpi_evp.so so the
 * engine drops in where CryptMPI calls BoringSSL today.  Link CryptMPI's
 * libmpi against libcmpi_evp.so ahead of libcrypto (or LD_PRELOAD it): every symbol below is
 * then served by the MI355X engine, everything else (RAND_bytes, RSA_*, BN_*) still resolves
 * to the real libcrypto.
 *
 * Prototypes are exactly those of MV/boringssl-master/include/openssl/aead.h and cipher.h
 * (API version 9); the structs are opaque here exactly as CryptMPI treats them.
 *   EVP_aead_aes_128_gcm   aead.h:100      EVP_AEAD_CTX_new    aead.h:210-212
 *   EVP_AEAD_CTX_free      aead.h:216      EVP_AEAD_CTX_seal   aead.h:256-260
 *   EVP_AEAD_CTX_open      aead.h:281-285  EVP_AEAD_nonce_length / max_overhead aead.h:159/:163
 *   EVP_aes_128_ecb/ctr    cipher.h:84/:86 EVP_CIPHER_CTX_new/free cipher.h:123/:131
 *   EVP_EncryptInit_ex     cipher.h:158    EVP_DecryptInit_ex  cipher.h:163
 *   EVP_EncryptUpdate      cipher.h:174    EVP_DecryptUpdate   cipher.h:191
 *
 * Semantics kept: return 1 / 0; on any seal/open error `out` is zero-filled for max_out_len
 * bytes and *out_len = 0 (aead.h:251-253, :276-278); concurrent use of one ctx from several
 * threads is allowed (calls are serialised per ctx inside the engine).  Limits of the drop-in:
 * AES-128 only (EVP_aes_256_* are not exported, so libcrypto keeps serving them), GCM nonce
 * length 12 and no AAD — exactly what every CryptMPI call site passes.
 * Device selection: env CMPI_DEVICE, else the MPI local rank (MV2_COMM_WORLD_LOCAL_RANK,
 * MPI_LOCALRANKID, OMPI_COMM_WORLD_LOCAL_RANK, LOCAL_RANK) modulo the GPU count.
 */
#ifndef CMPI_EVP_H
#define CMPI_EVP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct evp_aead_st EVP_AEAD;
typedef struct evp_aead_ctx_st EVP_AEAD_CTX;
typedef struct evp_cipher_st EVP_CIPHER;
typedef struct evp_cipher_ctx_st EVP_CIPHER_CTX;
typedef struct engine_st ENGINE;

const EVP_AEAD *EVP_aead_aes_128_gcm(void);
size_t EVP_AEAD_nonce_length(const EVP_AEAD *aead);
size_t EVP_AEAD_max_overhead(const EVP_AEAD *aead);
EVP_AEAD_CTX *EVP_AEAD_CTX_new(const EVP_AEAD *aead, const uint8_t *key, size_t key_len, size_t tag_len);
void EVP_AEAD_CTX_free(EVP_AEAD_CTX *ctx);
int EVP_AEAD_CTX_seal(const EVP_AEAD_CTX *ctx, uint8_t *out, size_t *out_len, size_t max_out_len,
                      const uint8_t *nonce, size_t nonce_len, const uint8_t *in, size_t in_len,
                      const uint8_t *ad, size_t ad_len);
int EVP_AEAD_CTX_open(const EVP_AEAD_CTX *ctx, uint8_t *out, size_t *out_len, size_t max_out_len,
                      const uint8_t *nonce, size_t nonce_len, const uint8_t *in, size_t in_len,
                      const uint8_t *ad, size_t ad_len);

const EVP_CIPHER *EVP_aes_128_ecb(void);
const EVP_CIPHER *EVP_aes_128_ctr(void);
EVP_CIPHER_CTX *EVP_CIPHER_CTX_new(void);
void EVP_CIPHER_CTX_free(EVP_CIPHER_CTX *ctx);
int EVP_EncryptInit_ex(EVP_CIPHER_CTX *ctx, const EVP_CIPHER *cipher, ENGINE *engine, const uint8_t *key,
                       const uint8_t *iv);
int EVP_DecryptInit_ex(EVP_CIPHER_CTX *ctx, const EVP_CIPHER *cipher, ENGINE *engine, const uint8_t *key,
                       const uint8_t *iv);
int EVP_EncryptUpdate(EVP_CIPHER_CTX *ctx, uint8_t *out, int *out_len, const uint8_t *in, int in_len);
int EVP_DecryptUpdate(EVP_CIPHER_CTX *ctx, uint8_t *out, int *out_len, const uint8_t *in, int in_len);

#ifdef __cplusplus
}
#endif
#endif /* CMPI_EVP_H */
