/*
 * cmpi_coll.h — the naive secure collectives of CryptMPI as one batch call per side
 * (SURVEY.md §8(a) row a9, §8(f) row 2).  Every naive wrapper of the reference seals blocks as
 * RAND_bytes(nonce, 12) + EVP_AEAD_CTX_seal into the wire block  nonce(12) || ct(n) || tag(16)
 * (stride n + 28), runs the stock collective on the ciphertext, and opens blocks the same way:
 *
 *   collective (reference)                         seal blocks            open blocks
 *   MPIR_Naive_Sec_Alltoall  alltoall.c:764-836    p (sendbuf[i*n])       p
 *   MPIR_Naive_Sec_Allgather allgather.c:839-899   1                      p
 *   gather 301               gather.c:1508-1606    1                      p (root)
 *   MPIR_Naive_Sec_Scatter   scatter.c:659-730     p (root)               1
 *   MPI_Naive_Sec_Bcast      bcast.c:1510-1580     1 (root)               1 (non-root)
 *
 * so two calls cover them all; the stock collective in between is untouched (host MPI, or
 * RCCL over xGMI when the buffers live in HBM).  Buffers are device memory; stream-ordered.
 */
#ifndef CMPI_COLL_H
#define CMPI_COLL_H

#include <stddef.h>
#include <stdint.h>

#include "cmpi_aead.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Seal with fresh nonces, the RAND_bytes + seal pair fused into the seal kernel itself:
 * nonce_r = P || BE64(c + r), P 4 bytes and the counter's start value 8 bytes drawn from the OS
 * CSPRNG when the context was created, c advanced by nrec per call — the deterministic
 * construction of SP 800-38D §8.2.1 with a random fixed field: a context never repeats a nonce
 * (its counter is 64 bits wide and advances under an atomic).  Across contexts under one key (ranks
 * sharing CryptMPI's global key) uniqueness is probabilistic, not assigned: two contexts repeat a
 * nonce only if their random 4-byte fields are equal (2^-32 per pair) AND their counter ranges
 * overlap (about (N1 + N2) / 2^64 for N1, N2 nonces drawn from random 64-bit starts) — below 2^-80
 * per pair for any realistic N, so for p ranks below p^2 · 2^-81.  This matches what CryptMPI's
 * RAND_bytes(nonce, 12) per message gives (send.c:294; a birthday bound over 96 random bits).
 * Nonces are written at nonce_out + r*nonce_stride. */
int cmpi_gcm_seal_batch_fresh(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                              size_t in_stride, uint8_t *nonce_out, size_t nonce_stride, size_t len, size_t nrec,
                              void *workspace, void *stream);
/* nblk blocks of n bytes (in + i*n) -> wire + i*(n+28) = nonce || ct || tag. */
int cmpi_naive_seal_blocks(const cmpi_ctx *ctx, uint8_t *wire, const uint8_t *in, size_t n, size_t nblk,
                           void *workspace, void *stream);
/* wire blocks -> out + i*n; status[i] 1 ok / 0 forged (zero-filled), may be NULL. */
int cmpi_naive_open_blocks(const cmpi_ctx *ctx, uint8_t *out, const uint8_t *wire, size_t n, size_t nblk,
                           int32_t *status, void *workspace, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CMPI_COLL_H */
