/*
 * cmpi_aead.h — C ABI of the MI355X-native AEAD seal/open engine (libcmpi_aead.so).
 *
 * This is the batched replacement for the BoringSSL calls CryptMPI makes on its per-message
 * hot path.  Plain pointers and sizes only; `stream` is a hipStream_t
 * passed as void* (NULL = the legacy default stream).  Device-resident entry points take
 * DEVICE pointers and are asynchronous on `stream`; the *_host entry points take HOST
 * pointers (pinned for full PCIe rate) and are synchronous (include/cmpi_async.h: the
 * non-blocking begin / wait form).
 *
 * Reference interfaces each entry point replaces (file:line):
 *   cmpi_ctx_new(CMPI_AES_128_GCM,…)  EVP_AEAD_CTX_new(EVP_aead_aes_128_gcm(), key, 16, 0)
 *                         MV/boringssl-master/include/openssl/aead.h:208-212; callers
 *                         MV/src/mpi/init/init.c:587-612, MV/src/mpi/pt2pt/send.c:588-599
 *   cmpi_ctx_new(CMPI_AES_128_CTR/ECB) EVP_CIPHER_CTX_new + EVP_EncryptInit_ex(…, EVP_aes_128_ctr|ecb,
 *                         NULL, key, NULL)  cipher.h:84-86, :123, :158; init.c:619, :716, :842-849
 *   cmpi_ctx_free         EVP_AEAD_CTX_free aead.h:216 / EVP_CIPHER_CTX_free cipher.h:131
 *   cmpi_gcm_seal_batch   a batch of EVP_AEAD_CTX_seal, aead.h:256-260; the loops at
 *                         MV/src/mpi/pt2pt/send.c:292-327 (600), :646-706 / :754-831 (602),
 *                         MV/src/mpi/coll/alltoall.c:795-811 (naive 1002)
 *   cmpi_gcm_open_batch   a batch of EVP_AEAD_CTX_open, aead.h:281-285; recv.c:322, :583-613,
 *                         :745-775, alltoall.c:821-834
 *   cmpi_ctr_xor          EVP_EncryptInit_ex(ctx,NULL,NULL,NULL,iv)+EVP_EncryptUpdate (CTR),
 *                         cipher.h:158/:174; send.c:985-1008, :1716-1727, :1805-1808
 *   cmpi_ctr_keystream    generateCommonEncMask (E_K(IV+i) over zeros), send.c:1162-1266
 *   cmpi_ecb_encrypt      EVP_EncryptUpdate(ctx_enc, newkey, &len, V, 16), send.c:583
 *   cmpi_ctx_new_subkey / derive_subkey / rekey_subkey
 *                         the 602 sub-key: K' = AES-ECB_K(V) then EVP_AEAD_CTX_new(K'),
 *                         send.c:572-600, recv.c:549-576 (derived and tabled on the device)
 *   cmpi_iv_count         IV_Count, send.c:1019-1030
 *   cmpi_ocb_seal/open_batch  AES-128-OCB (RFC 7253) — README-only "Naive OCB" (402); no
 *                         reference code exists (OPENSSL_NO_OCB, opensslconf.h:49)
 *
 * Conventions (EVP_AEAD_CTX_seal/open, aead.h:236-285): 12-byte nonce, no AAD, 16-byte tag
 * appended after the ciphertext.  open verifies in constant-time-free batch form: a record
 * whose tag mismatches gets status 0 and its plaintext output zero-filled (aead.h:276-278).
 * Contexts are immutable after creation and may be used concurrently from several threads /
 * streams (aead.h:240-241).  A call with workspace == NULL borrows the context's internal
 * scratch: the library orders such calls (the launch stream waits for the scratch's previous
 * user), so they serialise on the device; pass a `workspace` per stream to run concurrently.
 * The *_host calls use staging and scratch of their own.  Nothing is retained after a call
 * returns; device-resident work must be complete (or ordered before it) when the caller frees
 * a context or its buffers.
 *
 * Stream order: a device-resident call reads its inputs and writes its outputs, tags and
 * per-record statuses in the order of `stream` ONLY.  Work the caller queued on another stream
 * (e.g. a fill of the status array or the output buffer) is not ordered before the call unless
 * the caller makes `stream` wait for it (an event), and results are visible to other streams
 * only after they wait for `stream`.
 *
 * Errors: every call reports only failures its own HIP calls caused (a launch's own return
 * code, never the thread's hipGetLastError state), and it neither clears nor replaces a HIP
 * error the caller left pending in the calling thread (tests/test_gpu_errors.py).
 */
#ifndef CMPI_AEAD_H
#define CMPI_AEAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMPI_OK 0
#define CMPI_EINVAL (-1)  /* bad argument: size, alignment, NULL, wrong algorithm   */
#define CMPI_EHIP (-2)    /* HIP runtime error (message via cmpi_last_error)         */
#define CMPI_ENOMEM (-3)  /* device allocation failed                               */
#define CMPI_EAUTH (-4)   /* *_host open: at least one record failed authentication */
#define CMPI_ENODEV (-5)  /* no usable GPU                                          */

enum cmpi_alg {
  CMPI_AES_128_GCM = 1,
  CMPI_AES_128_OCB = 2,
  CMPI_AES_128_CTR = 3,
  CMPI_AES_128_ECB = 4
};

typedef struct cmpi_ctx cmpi_ctx;

/* Library info / errors. */
const char *cmpi_version(void);
const char *cmpi_last_error(void); /* thread-local; "" when none */
int cmpi_device_count(void);

/* Key context: expands the key schedule and the GHASH / OCB tables on the host once and
 * uploads them to `device` (HIP ordinal).  key_len must be 16.  tag_len 0 or 16.
 * Returns NULL on failure (see cmpi_last_error). */
cmpi_ctx *cmpi_ctx_new(int alg, const uint8_t *key, size_t key_len, size_t tag_len, int device);
/* 602 sub-key (send.c:572-600, recv.c:549-576): a GCM context for K' = AES-128_K(V), where
 * `base` is any context holding the master key K.  K' never leaves the device: one key-setup
 * kernel derives K', expands it, computes H = E_K'(0) and builds the GHASH tables.
 *   cmpi_ctx_derive_subkey  enqueues that kernel on `stream` and returns at once; use the
 *                           context on the same stream (or after synchronising it).
 *   cmpi_ctx_rekey_subkey   the same into an existing GCM context `dst` (no allocation: one
 *                           context per sender/receiver thread reused across messages).
 *   cmpi_ctx_new_subkey     derive + synchronise (blocking convenience).
 * A device-keyed context serves the GCM calls only (CTR/ECB on it return CMPI_EINVAL). */
cmpi_ctx *cmpi_ctx_derive_subkey(const cmpi_ctx *base, const uint8_t v[16], void *stream);
int cmpi_ctx_rekey_subkey(cmpi_ctx *dst, const cmpi_ctx *base, const uint8_t v[16], void *stream);
cmpi_ctx *cmpi_ctx_new_subkey(const cmpi_ctx *base, const uint8_t v[16]);
/* Re-key an existing context in place to a new host-known key (what a fresh cmpi_ctx_new would
 * hold, without its allocation and table upload): the device tables are rebuilt by a key-setup
 * kernel enqueued on `stream`; use the context on that stream or after synchronising it
 * (stream NULL: returns when the tables are built).
 * Replaces EVP_AEAD_CTX_new for the per-message 602 contexts (send.c:588-599, recv.c:562-575)
 * in the drop-in's context pool. */
int cmpi_ctx_rekey(cmpi_ctx *ctx, const uint8_t *key, size_t key_len, void *stream);
void cmpi_ctx_free(cmpi_ctx *ctx);
int cmpi_ctx_device(const cmpi_ctx *ctx);
/* Pin (page-lock) a host buffer for DMA, e.g. MPI send/receive buffers reused across calls, so
 * the *_host calls move it at PCIe rate; unregister before freeing it. */
int cmpi_host_register(void *ptr, size_t bytes);
int cmpi_host_unregister(void *ptr);

/* ---------------- AES-128-GCM, uniform batches (device pointers) ----------------
 * Record i (0 <= i < nrec):
 *   seal: reads  len bytes  of plaintext at in  + i*in_stride,
 *         writes len+16 bytes ct||tag     at out + i*out_stride,
 *         nonce  12 bytes                 at nonces + i*nonce_stride.
 *   open: reads  len+16 bytes ct||tag at in, writes len bytes plaintext at out,
 *         status[i] = 1 ok / 0 authentication failure (plaintext zero-filled); status may be NULL.
 * Pointers and strides may have any byte alignment; len is any value >= 0.  Records must
 * not overlap each other; out may equal in (in-place) but must not partially overlap it.
 * The naive-collective wire layout nonce(12)||ct(n)||tag(16) is expressed as
 *   out = wire + 12, nonces = wire, out_stride = nonce_stride = n + 28.
 * workspace: NULL (the context's internal scratch; the library orders such calls across
 * streams) or a device buffer of cmpi_gcm_workspace_size(len, nrec) bytes. */
size_t cmpi_gcm_workspace_size(const cmpi_ctx *ctx, size_t len, size_t nrec);
int cmpi_gcm_seal_batch(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                        size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                        size_t nrec, void *workspace, void *stream);
int cmpi_gcm_open_batch(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                        size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                        size_t nrec, int32_t *status, void *workspace, void *stream);

/* Host-memory variants, synchronous.  Up to 2 MiB of input + output records the kernel reads
 * and writes page-locked buffers directly (pageable ones through a pinned bounce buffer);
 * larger calls pipeline H2D -> kernel -> D2H in chunks over internal streams.  Returns CMPI_OK,
 * CMPI_EAUTH (open: some record failed; status[] on the host says which, may be NULL) or another
 * error.  Records of length 0 may pass NULL data pointers. */
int cmpi_gcm_seal_host(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                       size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                       size_t nrec);
int cmpi_gcm_open_host(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                       size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                       size_t nrec, int32_t *status);

/* ---------------- AES-128-OCB3 (RFC 7253), uniform batches (device pointers) ----------------
 * Same record layout and status semantics as the GCM batch calls (+ host-memory variants). */
size_t cmpi_ocb_workspace_size(const cmpi_ctx *ctx, size_t len, size_t nrec);
int cmpi_ocb_seal_batch(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                        size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                        size_t nrec, void *workspace, void *stream);
int cmpi_ocb_open_batch(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                        size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                        size_t nrec, int32_t *status, void *workspace, void *stream);
int cmpi_ocb_seal_host(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                       size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                       size_t nrec);
int cmpi_ocb_open_host(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                       size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                       size_t nrec, int32_t *status);

/* ---------------- AES-128-CTR ----------------
 * out[j] = in[j] XOR E_K(ctr_block + floor(j/16)) for 0 <= j < n, 128-bit big-endian counter
 * increment (EVP_aes_128_ctr).  ctr_block is a 16-byte HOST array (usually cmpi_iv_count()
 * of the common IV).  in/out device pointers, 4-byte aligned; in == out allowed. */
int cmpi_ctr_xor(const cmpi_ctx *ctx, uint8_t *out, const uint8_t *in, size_t n,
                 const uint8_t ctr_block[16], void *stream);
/* Materialised keystream: out = E_K(ctr_block + i) for i < nblocks (the mask ring of
 * generateCommonEncMask). */
int cmpi_ctr_keystream(const cmpi_ctx *ctx, uint8_t *out, size_t nblocks, const uint8_t ctr_block[16],
                       void *stream);
/* Host-memory CTR (synchronous): like cmpi_ctr_xor, but the first `skip` (0..15) bytes of the
 * first keystream block are discarded — the continuation state an EVP CTR context keeps
 * between EVP_EncryptUpdate calls. */
int cmpi_ctr_xor_host(const cmpi_ctx *ctx, uint8_t *out, const uint8_t *in, size_t n,
                      const uint8_t ctr_block[16], unsigned skip);
/* IV_Count (send.c:1019-1030), host helper: iv += (uint32_t)cter with CryptMPI's exact carry
 * behaviour (the carry out of the first byte add is dropped when cter + iv[15] >= 2^32). */
void cmpi_iv_count(uint8_t iv[16], unsigned long cter);
void cmpi_iv_count_out(uint8_t iv[16], unsigned long cter, const uint8_t in[16]);

/* ---------------- AES-128-ECB ----------------
 * out = E_K(in) over nblocks 16-byte blocks (device pointers). */
int cmpi_ecb_encrypt(const cmpi_ctx *ctx, uint8_t *out, const uint8_t *in, size_t nblocks, void *stream);
int cmpi_ecb_encrypt_host(const cmpi_ctx *ctx, uint8_t *out, const uint8_t *in, size_t nblocks);

#ifdef __cplusplus
}
#endif
#endif /* CMPI_AEAD_H */
