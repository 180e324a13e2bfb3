/*
 * cmpi_ring.h — CryptMPI's precomputed CTR mask ring on the device (SURVEY.md §8(a) row a8,
 * §8(f) row 3).  The reference keeps an 8 MiB ring enc_common_buffer (mpiimpl.h:397) of AES-CTR
 * keystream for the next counters of the sender's common stream and fills it while it spins in
 * MPI_Test; a send then XORs from the ring and runs direct CTR for whatever the ring lacks:
 *   generateCommonEncMask      send.c:1162-1266  -> cmpi_ctr_ring_generate
 *   encryption_common_counter  send.c:1273-1465  -> cmpi_ctr_ring_encrypt
 *   decryption_common_counter_ivflag recv.c:954-1023 -> cmpi_ctr_mask_decrypt
 * Here the ring lives in HBM and its fills are kernels on a stream (typically a low-priority
 * side stream, so they overlap the sends instead of MPI_Test spinning); the host keeps the
 * reference's bookkeeping exactly (start / end / compute_size / counter / counter_needto_send,
 * 16-byte rounding, the -1024 head-room guard), so the bytes produced equal the reference's for
 * the same call sequence.  Counter block of counter c = IV_Count(iv, c) (send.c:1019-1030).
 * Calls on one ring must be stream-ordered by the caller (generate and encrypt touch the ring).
 * Calls on different streams are ordered by the library (an event recorded on the previous
 * call's stream when the stream changes); the stream of a ring's (or 702 sender's) last call must
 * stay valid until its next call on another stream, or until the ring / sender is freed.
 */
#ifndef CMPI_RING_H
#define CMPI_RING_H

#include <stddef.h>
#include <stdint.h>

#include "cmpi_aead.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cmpi_ctr_ring cmpi_ctr_ring;

/* ctx: a CTR (or ECB/GCM) context holding the key; iv: the stream IV (Send_common_IV);
 * ring_bytes: multiple of 16, >= 2048 (8388608 in CryptMPI). */
cmpi_ctr_ring *cmpi_ctr_ring_new(const cmpi_ctx *ctx, const uint8_t iv[16], size_t ring_bytes);
void cmpi_ctr_ring_free(cmpi_ctr_ring *ring);
/* Keystream for the next ceil(gen_bytes/16) counters into the ring.  Returns 1 when generated,
 * 0 when the head-room guard skipped it (as the reference does), < 0 on error. */
int cmpi_ctr_ring_generate(cmpi_ctr_ring *ring, size_t gen_bytes, void *stream);
/* out[0..n) = in XOR keystream: first from the ring, then direct CTR from the next counter. */
int cmpi_ctr_ring_encrypt(cmpi_ctr_ring *ring, uint8_t *out, const uint8_t *in, size_t n, void *stream);
/* {start, end, compute_size, counter, counter_needto_send} */
int cmpi_ctr_ring_state(const cmpi_ctr_ring *ring, uint64_t state[5]);
/* Receiver: out = in XOR (mask[0..min(n, mask_len)), then CTR from IV_Count(iv, counter)). */
int cmpi_ctr_mask_decrypt(const cmpi_ctx *ctx, uint8_t *out, const uint8_t *in, size_t n, const uint8_t *mask,
                          size_t mask_len, const uint8_t iv[16], uint64_t counter, void *stream);
/* out = a XOR b (device, n bytes): the mask-consumption pass on its own. */
int cmpi_xor_bytes(uint8_t *out, const uint8_t *a, const uint8_t *b, size_t n, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CMPI_RING_H */
