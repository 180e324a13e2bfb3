/*
 * cmpi_frame.h — CryptMPI's on-the-wire framings built on the device (SURVEY.md §8(a) rows
 * a4/a5, §8(f) row 1).  The byte layouts are those of the reference senders/receivers:
 *
 *   600 (MPI_SEC_Multi_Thread_Send_OpenMP, MV/src/mpi/pt2pt/send.c:221-337; recv.c:219-341):
 *     header[25]: [0..3] BE32 n, [20] '1' (send) / '2' (isend), [21..24] BE32 n
 *     payload   : nonce(12, RAND_bytes) || ct(n) || tag(16)
 *
 *   602 (MPI_SEC_MThreads_PipeLine_OpenMP_Send__largeSegment_3, send.c:339-884;
 *        MPI_SEC_MThreads_Pipelined_OpenMP_Recv_largeSegment_3, recv.c:343-809):
 *     header[25]: [0..3] BE32 n, [4..19] V (n > 65535: K' = AES-ECB_K(V)) or [4..15] nonce
 *                 (n <= 65535: small-message key), [20] mode '4' | '1', [21..24] BE32 chop
 *     wire      : per segment  prefix(5) || ct || tag(16)   with prefix = flag || BE32(ctr)
 *                 and nonce = "0000000" || prefix  (n >= 65536); a small message has one
 *                 segment whose nonce is header[4..15] and whose prefix bytes are not written.
 *     mode '4'  : segments of chop bytes (last one shorter), ctr = segment index, flag '0'.
 *     mode '1'  : 512 KiB outer messages, each cut into chop-byte segments; ctr counts all
 *                 segments of the message, flag '1' on the segments of the last outer message.
 *
 * All buffers passed to the seal/open calls are device memory; headers are host memory (the
 * 25-byte header travels as its own MPI message).  Calls are asynchronous on `stream`.  The
 * segment context must be keyed by the caller exactly as the reference does: for n > 65535
 * cmpi_ctx_rekey_subkey(seg_ctx, master, header + 4, stream) (K' derived on the device), else
 * the small-message context.
 */
#ifndef CMPI_FRAME_H
#define CMPI_FRAME_H

#include <stddef.h>
#include <stdint.h>

#include "cmpi_aead.h"
#include "cmpi_async.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cmpi_602_plan {
  uint32_t total;      /* n (plaintext bytes of the message) */
  uint32_t chop;       /* choping_sz: segment bytes (header[21..24]) */
  uint32_t outer;      /* MPI messages after the header: 1 in mode '4' */
  uint32_t nseg;       /* segments (GCM records) in the message */
  uint8_t mode;        /* '4' or '1' (header[20]) */
  uint8_t subkey;      /* 1 when n > 65535 (K' = AES_K(V)) */
  uint8_t pad_[2];
  uint64_t wire_bytes; /* bytes after the header: n + 21 * nseg */
} cmpi_602_plan;

/* The sender's decisions of send.c:392-549 for a message of n bytes: series_threads is
 * cyptmpi_series_thread (thread cap), pending_isends is pendingIsendRequestCount[dest]. */
int cmpi_602_plan_make(uint32_t n, int series_threads, int pending_isends, cmpi_602_plan *plan);
/* The receiver's view (recv.c:395-420): n, mode and chop from a received header. */
int cmpi_602_plan_from_header(const uint8_t header[25], cmpi_602_plan *plan);
/* header[25] of a message: rand16 = the RAND_bytes output (16 bytes used when n > 65535,
 * else bytes 0..11 are the nonce and 12..15 fill header[16..19]). */
int cmpi_602_header(const cmpi_602_plan *plan, const uint8_t rand16[16], uint8_t header[25]);
/* Byte span of outer message o (0 <= o < plan->outer) in the wire and in the plaintext:
 * what one MPI_Isend of the pipelined sender carries (send.c:833-835). */
int cmpi_602_outer_span(const cmpi_602_plan *plan, uint32_t o, uint64_t *wire_off, uint64_t *wire_len,
                        uint64_t *pt_off, uint64_t *pt_len);
/* Seal outer messages [first, first+count) of the message into `wire` (device, wire_bytes),
 * prefixes included; in = the whole plaintext (device, n bytes). */
int cmpi_602_seal_outer(const cmpi_ctx *seg_ctx, const cmpi_602_plan *plan, const uint8_t header[25],
                        uint8_t *wire, const uint8_t *in, uint32_t first, uint32_t count, void *stream);
int cmpi_602_seal(const cmpi_ctx *seg_ctx, const cmpi_602_plan *plan, const uint8_t header[25], uint8_t *wire,
                  const uint8_t *in, void *stream);
/* Open a received message: nonces rebuilt from the wire prefixes like recv.c; out = n bytes
 * (device); status = per-segment 1 ok / 0 forged (device int32[nseg], may be NULL).  Failed
 * segments are zero-filled (aead.h:276-278). */
int cmpi_602_open(const cmpi_ctx *seg_ctx, const uint8_t header[25], uint8_t *out, const uint8_t *wire,
                  int32_t *status, void *stream);

/* ---- 602 from and to host memory (MPI user buffers) ----
 * A request per call (cmpi_async.h: cmpi_test / cmpi_wait / cmpi_waitall), on the library's
 * pooled streams: H2D of the call's host span, the device seal/open above, D2H of its result.
 * Page-locked buffers move by DMA from / to the caller's pages; pageable ones through pinned
 * staging (inputs packed inside *_begin, outputs copied out at completion).  The pipelined sender
 * of send.c:729-850 is one seal_host_begin per outer message o (count 1) followed, in order, by
 * cmpi_wait(req[o]) and MPI_Isend of cmpi_602_outer_span(o): outer o+1 is being sealed on the
 * GPU while o is on the wire.  The receiver of recv.c:679-809 begins the open of each outer message
 * as it lands.  A segment context re-keyed on a caller stream (cmpi_ctx_rekey_subkey) is ordered
 * before these requests by the library.  Outputs must stay valid until the request completes. */
int cmpi_602_seal_host_begin(const cmpi_ctx *seg_ctx, const cmpi_602_plan *plan, const uint8_t header[25],
                             uint8_t *wire, const uint8_t *in, uint32_t first, uint32_t count, cmpi_req **req);
/* every outer message begun, then all waited (the whole pipelined send) */
int cmpi_602_seal_host(const cmpi_ctx *seg_ctx, const cmpi_602_plan *plan, const uint8_t header[25], uint8_t *wire,
                       const uint8_t *in);
/* open outer messages [first, first+count) of a received message: wire = the whole message's wire
 * buffer (host), out = the whole plaintext (host, n bytes); status (host int32[plan nseg], may be
 * NULL) gets the segments of those outers.  The wait returns CMPI_EAUTH when a segment failed (its
 * plaintext zero-filled). */
int cmpi_602_open_host_begin(const cmpi_ctx *seg_ctx, const uint8_t header[25], uint8_t *out, const uint8_t *wire,
                             uint32_t first, uint32_t count, int32_t *status, cmpi_req **req);
int cmpi_602_open_host(const cmpi_ctx *seg_ctx, const uint8_t header[25], uint8_t *out, const uint8_t *wire,
                       int32_t *status);

/* 600: header and payload of MPI_SEC_Multi_Thread_Send_OpenMP (kind '1') / isend (kind '2'). */
int cmpi_600_header(uint32_t n, uint8_t kind, uint8_t header[25]);
/* payload (device, n + 28 bytes) = nonce || ct || tag; the nonce comes from the host. */
int cmpi_600_seal(const cmpi_ctx *ctx, const uint8_t nonce[12], uint8_t *payload, const uint8_t *in, size_t n,
                  void *stream);
int cmpi_600_open(const cmpi_ctx *ctx, uint8_t *out, const uint8_t *payload, size_t n, int32_t *status,
                  void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CMPI_FRAME_H */
