/*
 * cmpi_async.h — asynchronous host-memory batches for CryptMPI's non-blocking pair (SURVEY.md
 * §8(f) row 4).  The reference's MPI_Isend encrypts eagerly and returns a request; MPI_Wait /
 * MPI_Waitall complete it, decrypting received messages (MV/src/mpi/pt2pt/isend.c:187-1260,
 * wait.c:244-1780, waitall.c:438-2389; 64 requests in nonblock_req_handler[], isend.c:310-321).
 *
 *   *_host_begin   enqueue the seal/open of a host-memory batch (the record layout and status
 *                  semantics of the synchronous *_host calls, cmpi_aead.h) on a pooled stream
 *                  and return at once with a request: up to 2 MiB of records the kernel reads
 *                  and writes page-locked buffers itself, larger ones go H2D -> kernel -> D2H;
 *   cmpi_test      MPI_Test: *done = 1 and the request completed (and freed) when it finished;
 *   cmpi_wait      MPI_Wait: block until done; returns CMPI_OK, CMPI_EAUTH (open: a record
 *                  failed, status[] says which, its plaintext zero-filled) or another error;
 *   cmpi_waitall   MPI_Waitall over n requests (NULL entries skipped, every entry cleared).
 *
 * Input buffers may be reused when *_begin returns if pageable (they are packed into pinned
 * staging inside it); page-locked ones are read later by DMA or by the kernel — keep those
 * until completion, as MPI does.  Output and status buffers must stay valid until the request completes.  Requests are
 * independent: any number may be outstanding on one context, from any thread.
 */
#ifndef CMPI_ASYNC_H
#define CMPI_ASYNC_H

#include <stddef.h>
#include <stdint.h>

#include "cmpi_aead.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cmpi_req cmpi_req;

int cmpi_gcm_seal_host_begin(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                             size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                             size_t nrec, cmpi_req **req);
int cmpi_gcm_open_host_begin(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                             size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                             size_t nrec, int32_t *status, cmpi_req **req);
int cmpi_ocb_seal_host_begin(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                             size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                             size_t nrec, cmpi_req **req);
int cmpi_ocb_open_host_begin(const cmpi_ctx *ctx, uint8_t *out, size_t out_stride, const uint8_t *in,
                             size_t in_stride, const uint8_t *nonces, size_t nonce_stride, size_t len,
                             size_t nrec, int32_t *status, cmpi_req **req);
int cmpi_test(cmpi_req *req, int *done);
int cmpi_wait(cmpi_req *req);
int cmpi_waitall(cmpi_req **reqs, size_t n);

#ifdef __cplusplus
}
#endif
#endif /* CMPI_ASYNC_H */
