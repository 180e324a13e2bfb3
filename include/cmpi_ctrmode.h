/*
 * cmpi_ctrmode.h — CryptMPI's counter-mode message paths as engine calls (SURVEY.md §8(a) rows
 * a6-a8, §8(f) row 3).  One call per side of a message; every keystream byte is made by a HIP
 * kernel on `stream`, the reference's counter / ring bookkeeping is kept on the host exactly.
 *
 *   700  MPI_SEC_BaseCounter_Pipeline_Send / _Recv   MV/src/mpi/pt2pt/send.c:886-1017,
 *        recv.c:812-940: ct = CTR(IV_Count(Send_common_IV, base_global_counter)) ^ pt.
 *   702  MPI_SEC_PreComputeCounter_Send_v4 / _Recv_v4 send.c:1502-1987, recv.c:1025-1403:
 *        two streams per rank, Send_common_IV[0..16) = stream A behind the 8 MiB mask ring
 *        (enc_common_buffer, generateCommonEncMask), [16..32) = stream B for long messages;
 *        messages < 64 KiB XOR from the ring when it holds enough (header[4] '0'), else stream B
 *        directly ('1'); messages >= 64 KiB are stream-B slices of choping_sz bytes at IV_Count
 *        offsets.  The receiver makes its decryption mask while the payload is in flight
 *        (cmpi_702_recv_premask, recv.c:1107-1196) and XORs when it lands.
 *
 * Header (COUNTER_HEADER_SIZE = 26, mpiimpl.h:385): [0..3] BE32 n, [4] stream '0'/'1' (702,
 * n < 64 KiB), [5..8] BE32 counter, [20] '1'/'4' (702), [21..24] BE32 choping_sz.  Bytes the
 * reference never writes (it sends whatever its static buffer held) are zero here.
 * Data pointers are device memory, headers and IVs host memory.  Calls on one sender (send,
 * precompute) may come from several threads: the ring lock is held from the stream choice of a
 * send to the XOR that consumes the ring; they are stream-ordered among themselves.
 * With a message service started on the CTR context (cmpi_service.h), the ops of messages up to
 * 64 KiB (ring XOR, direct CTR, premask, mask XOR) run on the resident kernel: the call waits
 * for the work already queued on `stream`, and returns with its output written.
 */
#ifndef CMPI_CTRMODE_H
#define CMPI_CTRMODE_H

#include <stddef.h>
#include <stdint.h>

#include "cmpi_aead.h"
#include "cmpi_async.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CMPI_CTR_HEADER 26

/* ---- 700 (base counter) ---- */
/* send.c:886-1017: header + ct of n bytes; *counter (base_global_counter) advances by
 * (unsigned long)(n - 1) / 16 + 1 exactly as the reference's expression. */
int cmpi_700_send(const cmpi_ctx *ctx, const uint8_t send_iv[16], uint64_t *counter, const uint8_t *in, size_t n,
                  uint8_t header[26], uint8_t *out, void *stream);
/* recv.c:812-940: recv_iv = Recv_common_IV[source*16 .. +16).  out holds out_cap bytes: a header
 * announcing more is refused (CMPI_EINVAL) — the reference trusts the wire. */
int cmpi_700_recv(const cmpi_ctx *ctx, const uint8_t recv_iv[16], const uint8_t header[26], uint8_t *out,
                  size_t out_cap, const uint8_t *in, void *stream);

/* ---- 702 (pre-computed counter) ---- */
typedef struct cmpi_702_sender cmpi_702_sender;
/* init_counter_mode_keys (init.c:766-792): ring of ring_bytes (8388608 in CryptMPI) with the
 * initial 4 KiB of stream A generated on `stream`; series_threads = cyptmpi_series_thread. */
cmpi_702_sender *cmpi_702_sender_new(const cmpi_ctx *ctx, const uint8_t send_iv[32], size_t ring_bytes,
                                     int series_threads, void *stream);
void cmpi_702_sender_free(cmpi_702_sender *s);
/* {ring start, end, compute_size, enc_common_counter, counter_needto_send,
 *  enc_common_counter_long_msg, counter_needto_send_large_msg} */
int cmpi_702_sender_state(const cmpi_702_sender *s, uint64_t state[7]);
/* send.c:1537-1860: header + ct (device, n bytes); pending_isends = pendingIsendRequestCount[dest].
 * Returns the number of MPI_Isend segments the reference posts (>= 1), < 0 on error. */
int cmpi_702_send(cmpi_702_sender *s, int pending_isends, const uint8_t *in, size_t n, uint8_t header[26],
                  uint8_t *out, void *stream);
/* send.c:1862-1983: the pre-computation the reference runs while its sends are pending, for a
 * message of n bytes, `rounds` iterations (one per failed MPI_Test in the reference).  Returns
 * the iterations that generated keystream. */
int cmpi_702_precompute(cmpi_702_sender *s, size_t n, int rounds, void *stream);
/* recv.c:1107-1196 (n < 64 KiB): the decryption mask of the message announced by `header`,
 * generated before the payload lands; *mask_len = bytes made (0 for n >= 64 KiB: no mask). */
int cmpi_702_recv_premask(const cmpi_ctx *ctx, const uint8_t recv_iv[32], const uint8_t header[26], uint8_t *mask,
                          size_t mask_cap, size_t *mask_len, void *stream);
/* recv.c:1198-1403: plaintext (device, n bytes, out_cap >= n) from the payload; mask/mask_len from
 * cmpi_702_recv_premask, or NULL/0 when the payload arrived first (direct CTR).  A header whose n
 * exceeds out_cap, or whose choping_sz is not a multiple of 16 in [16, n rounded up to 16], is
 * refused (CMPI_EINVAL). */
int cmpi_702_recv(const cmpi_ctx *ctx, const uint8_t recv_iv[32], const uint8_t header[26], uint8_t *out,
                  size_t out_cap, const uint8_t *in, const uint8_t *mask, size_t mask_len, void *stream);

/* ---- host-memory forms (MPI user buffers, send.c:1716-1727 / :1768-1816):
 * the same calls on host in/out buffers as requests on the library's pooled streams (cmpi_async.h),
 * and their synchronous forms (begin + wait).  Headers, IVs and counters are updated when *_begin
 * returns, exactly as by the device calls; page-locked buffers move by DMA, pageable ones through
 * pinned staging.  702 receive: the mask stays device memory (cmpi_702_recv_premask on
 * mask_stream while the payload is in flight); the request orders itself after mask_stream. */
int cmpi_700_send_host_begin(const cmpi_ctx *ctx, const uint8_t send_iv[16], uint64_t *counter, const uint8_t *in,
                             size_t n, uint8_t header[26], uint8_t *out, cmpi_req **req);
int cmpi_700_send_host(const cmpi_ctx *ctx, const uint8_t send_iv[16], uint64_t *counter, const uint8_t *in, size_t n,
                       uint8_t header[26], uint8_t *out);
int cmpi_700_recv_host_begin(const cmpi_ctx *ctx, const uint8_t recv_iv[16], const uint8_t header[26], uint8_t *out,
                             size_t out_cap, const uint8_t *in, cmpi_req **req);
int cmpi_700_recv_host(const cmpi_ctx *ctx, const uint8_t recv_iv[16], const uint8_t header[26], uint8_t *out,
                       size_t out_cap, const uint8_t *in);
/* *segments = what cmpi_702_send returns (MPI_Isend segments); the sync form returns it. */
int cmpi_702_send_host_begin(cmpi_702_sender *s, int pending_isends, const uint8_t *in, size_t n, uint8_t header[26],
                             uint8_t *out, int *segments, cmpi_req **req);
int cmpi_702_send_host(cmpi_702_sender *s, int pending_isends, const uint8_t *in, size_t n, uint8_t header[26],
                       uint8_t *out);
int cmpi_702_recv_host_begin(const cmpi_ctx *ctx, const uint8_t recv_iv[32], const uint8_t header[26], uint8_t *out,
                             size_t out_cap, const uint8_t *in, const uint8_t *mask, size_t mask_len,
                             void *mask_stream, cmpi_req **req);
int cmpi_702_recv_host(const cmpi_ctx *ctx, const uint8_t recv_iv[32], const uint8_t header[26], uint8_t *out,
                       size_t out_cap, const uint8_t *in, const uint8_t *mask, size_t mask_len, void *mask_stream);

#ifdef __cplusplus
}
#endif
#endif /* CMPI_CTRMODE_H */
