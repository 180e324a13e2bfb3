/*
 * ctr_ring_ref.c — CryptMPI's precomputed-counter mask ring.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates, statement by statement, MV/src/mpi/pt2pt/send.c:
 *   generateCommonEncMask      :1162-1266  (keystream for the next counters into the ring)
 *   encryption_common_counter  :1273-1465  (XOR from the ring, then direct CTR for the rest)
 * and recv.c decryption_common_counter_ivflag :954-1023 (mask prefix XOR, then direct CTR).
 * The ring size is a parameter (MAX_COMMON_COUNTER_SZ = 8 MiB in mpiimpl.h:397) so tests can
 * exercise wrap-around with small rings; the -1024 head-room guard of :1167 is kept.
 * Counter blocks are IV_Count(IV, counter) (send.c:1019-1030, with its 32-bit accumulator).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static void ring_ctr(const orc_ring_t *r, unsigned long counter, const uint8_t *in, uint8_t *out, size_t n) {
  uint8_t iv[16];
  memcpy(iv, r->iv, 16);
  orc_iv_count(iv, counter);
  orc_ctr128_xor(r->key, iv, in, out, n);
}

void orc_ring_init(orc_ring_t *r, const uint8_t key[16], const uint8_t iv[16], uint8_t *ring, int max) {
  memset(r, 0, sizeof *r);
  memcpy(r->key, key, 16);
  memcpy(r->iv, iv, 16);
  r->buf = ring;
  r->max = max;
}

/* send.c:1162-1266 */
int orc_ring_generate(orc_ring_t *r, int common_counter_gen_sz) {
  int blockamount, tempamount;
  uint8_t *zeros;
  if (!(r->compute_size <= (r->max - common_counter_gen_sz - 1024))) return 0;
  blockamount = ((common_counter_gen_sz - 1) / 16) * 16 + 16;
  zeros = calloc((size_t)blockamount + 16, 1);
  if (r->end > r->start && r->end + blockamount <= r->max) {
    ring_ctr(r, r->counter, zeros, r->buf + r->end, (size_t)blockamount);
    r->compute_size += blockamount;
    r->end += blockamount;
    r->counter += (unsigned long)(blockamount / 16);
  } else if ((r->end > r->start && r->end + blockamount > r->max) || (r->end == r->start && r->compute_size == 0)) {
    tempamount = r->max - r->end;
    if (blockamount > tempamount) {
      if (tempamount) {
        ring_ctr(r, r->counter, zeros, r->buf + r->end, (size_t)tempamount);
        r->compute_size += tempamount;
        r->end += tempamount;
        r->counter += (unsigned long)(tempamount / 16);
      }
      blockamount = blockamount - tempamount;
      r->end = 0;
    }
    ring_ctr(r, r->counter, zeros, r->buf + r->end, (size_t)blockamount);
    r->compute_size += blockamount;
    r->end += blockamount;
    r->counter += (unsigned long)(blockamount / 16);
  } else if (r->end < r->start && blockamount + r->end < r->start) {
    ring_ctr(r, r->counter, zeros, r->buf + r->end, (size_t)blockamount);
    r->compute_size += blockamount;
    r->end += blockamount;
    r->counter += (unsigned long)(blockamount / 16);
  } else {
    free(zeros);
    return -1; /* the reference prints ___ERROR___ and exits (send.c:1253-1262) */
  }
  free(zeros);
  return 1;
}

static void xor_into(uint8_t *out, const uint8_t *a, const uint8_t *b, size_t n) {
  for (size_t i = 0; i < n; i++) out[i] = a[i] ^ b[i];
}

/* send.c:1273-1465: out[0..enc_datasize) = buf ^ keystream */
void orc_ring_encrypt(orc_ring_t *r, const uint8_t *buf, int enc_datasize, uint8_t *out) {
  int how_much_generate, temporary_datasize, datasize, tempamount, tempnext;
  if (enc_datasize > r->compute_size) {
    how_much_generate = enc_datasize - r->compute_size;
    datasize = temporary_datasize = r->compute_size;
  } else {
    how_much_generate = 0;
    temporary_datasize = datasize = enc_datasize;
  }
  if (r->compute_size > 0) {
    if (r->end > r->start) {
      if (r->start + datasize <= r->end) tempamount = datasize;
      else tempamount = r->end - r->start;
      xor_into(out, r->buf + r->start, buf, (size_t)tempamount);
      r->start += ((tempamount - 1) / 16) * 16 + 16;
      if (r->start >= r->max) r->start = 0;
      r->compute_size -= (((tempamount - 1) / 16) * 16 + 16);
      r->counter_needto_send += (unsigned long)(((tempamount - 1) / 16) + 1);
    } else if (r->end < r->start) {
      tempamount = r->max - r->start;
      tempnext = 0;
      if (datasize > tempamount) {
        if (tempamount) {
          xor_into(out, r->buf + r->start, buf, (size_t)tempamount);
          tempnext = tempamount;
        }
        r->start = 0;
        datasize = datasize - tempamount;
      }
      xor_into(out + tempnext, r->buf + r->start, buf + tempnext, (size_t)datasize);
      if (datasize > 0) r->start += ((datasize - 1) / 16) * 16 + 16;
      if (r->start >= r->max) r->start = 0;
      r->compute_size -= (((temporary_datasize - 1) / 16) * 16 + 16);
      r->counter_needto_send += (unsigned long)(((temporary_datasize - 1) / 16) + 1);
    }
  }
  if (how_much_generate) {
    ring_ctr(r, r->counter, buf + temporary_datasize, out + temporary_datasize, (size_t)how_much_generate);
    r->counter += (unsigned long)((how_much_generate - 1) / 16 + 1);
    r->counter_needto_send += (unsigned long)(((how_much_generate - 1) / 16) + 1);
  }
}

/* recv.c:954-1023: out = in ^ (mask[0..min(n, mask_len)) then CTR(IV_Count(iv, counter))) */
void orc_mask_decrypt(const uint8_t key[16], const uint8_t iv[16], unsigned long counter, const uint8_t *mask,
                      int mask_len, const uint8_t *in, int n, uint8_t *out) {
  int len = n > mask_len ? mask_len : n;
  xor_into(out, mask, in, (size_t)len);
  if (n > len) {
    uint8_t cb[16];
    memcpy(cb, iv, 16);
    orc_iv_count(cb, counter);
    orc_ctr128_xor(key, cb, in + len, out + len, (size_t)(n - len));
  }
}
