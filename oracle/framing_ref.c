/*
 * framing_ref.c — CryptMPI wire-framing helpers (nonce / header byte layouts).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * orc_nonce602: MV/src/mpi/pt2pt/send.c:651-670 (flag '4' path: local_nonce[0..7] = '0',
 *   [8..11] = BE32 segment) and :781-804 (pipeline path: [7] = '1' on the last segment);
 *   receiver rebuilds it from the 5-byte segment prefix, recv.c:594-607, :749-762.
 * orc_header600: MV/src/mpi/pt2pt/send.c:241-266 (MSG_HEADER_SIZE = 25).
 */
#include "oracle.h"

#include <string.h>

void orc_nonce602(uint8_t nonce[12], uint8_t flag, uint32_t seg) {
  memset(nonce, '0', 7);
  nonce[7] = flag;
  nonce[8] = (uint8_t)(seg >> 24);
  nonce[9] = (uint8_t)(seg >> 16);
  nonce[10] = (uint8_t)(seg >> 8);
  nonce[11] = (uint8_t)seg;
}

void orc_header600(uint8_t hdr[25], uint32_t total, uint8_t kind, uint32_t chunk) {
  hdr[0] = (uint8_t)(total >> 24);
  hdr[1] = (uint8_t)(total >> 16);
  hdr[2] = (uint8_t)(total >> 8);
  hdr[3] = (uint8_t)total;
  hdr[20] = kind;
  hdr[21] = (uint8_t)(chunk >> 24);
  hdr[22] = (uint8_t)(chunk >> 16);
  hdr[23] = (uint8_t)(chunk >> 8);
  hdr[24] = (uint8_t)chunk;
}

/* ---------------------------------------------------------------------------------------------
 * 602 sender (MPI_SEC_MThreads_PipeLine_OpenMP_Send__largeSegment_3, MV/src/mpi/pt2pt/
 * send.c:339-884) as compiled with MV/src/include/mpiimpl.h:254-350: OMP_DYNAMIC_THREADS_PIPELINE
 * = 1, CRYPTMPI_ADAPTIVE_CHOPP = 1, PSC_BRIDGE_TUNE = ONLY_ONE_THREAD_PIPELINE = 0,
 * PIPELINE_SIZE = 524288, LARGE_SEGMENT_SIZE = 1048575, SUBKEY_GEN_START = 65535,
 * MAX_PENDING_ISEND_LIMIT = 64, MSG_HEADER_SIZE = 25, NONCE_HEADER = 5, tag 16.
 * Restated statement by statement; `int` arithmetic as in the reference (n < 2^31).
 */
#define R602_PIPE 524288
#define R602_LARGE 1048575
#define R602_SUBKEY 65535

void orc_602_plan(uint32_t totaldata_u, int series_threads, int pending, orc_602_plan_t *p) {
  const int totaldata = (int)totaldata_u;
  int segments_no, my_thread_no, choping_sz;
  uint8_t mode;
  /* send.c:392-400 */
  if ((totaldata > R602_PIPE) && totaldata > R602_LARGE) {
    segments_no = 1;
    segments_no += (int)(totaldata - (R602_PIPE)-1) / (R602_PIPE) + 1;
  } else {
    segments_no = 1;
  }
  /* send.c:420-427 (OMP_DYNAMIC_THREADS_PIPELINE table), :433-436 (cap) */
  if (totaldata < 65536) my_thread_no = 1;
  else if (totaldata < 131072) my_thread_no = 2;
  else if (totaldata < 524288) my_thread_no = 4;
  else my_thread_no = 8;
  if (my_thread_no > series_threads) my_thread_no = series_threads;
  /* send.c:470-530 */
  if ((pending + segments_no > 64 && segments_no > 1) || (totaldata >= 65536 && totaldata <= R602_LARGE)) {
    mode = '4';
    choping_sz = (totaldata - 1) / my_thread_no + 1;
  } else {
    mode = '1';
    if (totaldata > R602_LARGE) {
      int temp_thread = 8; /* PIPELINE_SIZE >= FIVE_ONE_2K */
      if (temp_thread > series_threads) temp_thread = series_threads;
      my_thread_no = temp_thread;
    }
    choping_sz = (R602_PIPE - 1) / my_thread_no + 1;
  }
  p->total = totaldata_u;
  p->mode = mode;
  p->chop = (uint32_t)choping_sz;
  p->subkey = totaldata > R602_SUBKEY;
  p->outer = mode == '4' ? 1u : (uint32_t)segments_no;
  p->nseg = 0;
  if (mode == '4') {
    p->nseg = (uint32_t)((totaldata - 1) / choping_sz + 1); /* send.c:672 */
  } else {
    for (int s = 0; s < segments_no; s++) { /* send.c:751-763 */
      int inner_totaldata = (s == segments_no - 1) ? totaldata - (R602_PIPE * (segments_no - 1)) : R602_PIPE;
      p->nseg += (uint32_t)((inner_totaldata - 1) / choping_sz + 1);
    }
  }
  p->wire_bytes = (uint64_t)totaldata_u + (uint64_t)p->nseg * 21u;
}

/* Header + wire of one 602 message.  key = K (master), small_key = the small-message key
 * (global_small_msg_ctx), rand16 = the RAND_bytes output (send.c:566 / :596: 16 bytes when
 * n > 65535, else 12; header[16..19] then keep rand16[12..15] as the stale bytes).  Wire bytes
 * the reference leaves unwritten (the 5-byte prefix of a small message, send.c:800-803) are
 * left as the caller's buffer had them. */
void orc_602_seal(const uint8_t key[16], const uint8_t small_key[16], const orc_602_plan_t *p,
                  const uint8_t rand16[16], const uint8_t *buf, uint8_t header[25], uint8_t *wire) {
  const int totaldata = (int)p->total;
  uint8_t kprime[16];
  memset(header, 0, 25);
  header[0] = (uint8_t)(p->total >> 24); /* send.c:371-374 */
  header[1] = (uint8_t)(p->total >> 16);
  header[2] = (uint8_t)(p->total >> 8);
  header[3] = (uint8_t)p->total;
  memcpy(header + 4, rand16, 16);
  header[20] = p->mode;
  header[21] = (uint8_t)(p->chop >> 24); /* send.c:545-549 */
  header[22] = (uint8_t)(p->chop >> 16);
  header[23] = (uint8_t)(p->chop >> 8);
  header[24] = (uint8_t)p->chop;
  const uint8_t *seg_key = small_key;
  if (p->subkey) { /* send.c:553-572: K' = AES-ECB_K(V) */
    orc_aes128_ecb(key, rand16, kprime, 1);
    seg_key = kprime;
  }
  const int th_data = (int)p->chop;
  uint8_t nonce[12];
  if (p->mode == '4') { /* send.c:646-706 */
    const int segs = (int)p->nseg;
    for (int i = 0; i < segs; i++) {
      const size_t base = (size_t)i * (th_data + 16 + 5) + 5; /* relative to wire = buffer + 25 */
      orc_nonce602(nonce, '0', (uint32_t)i);
      wire[base - 5] = '0';
      wire[base - 4] = (uint8_t)(i >> 24);
      wire[base - 3] = (uint8_t)(i >> 16);
      wire[base - 2] = (uint8_t)(i >> 8);
      wire[base - 1] = (uint8_t)i;
      int enc_data = th_data;
      if (i == segs - 1) enc_data = totaldata - th_data * (segs - 1);
      orc_gcm_seal(seg_key, nonce, 12, NULL, 0, buf + (size_t)th_data * i, (size_t)enc_data, wire + base);
    }
    return;
  }
  int prsd_segment = 0, send_loc = 0, enc_loc = 0; /* send.c:734-850 */
  const int segments_no = (int)p->outer;
  for (int s = 0; s < segments_no; s++) {
    int inner_totaldata, ii;
    if (s == segments_no - 1) {
      inner_totaldata = totaldata - (R602_PIPE * (segments_no - 1));
      ii = (inner_totaldata - 1) / th_data + 1;
    } else {
      inner_totaldata = R602_PIPE;
      ii = (R602_PIPE - 1) / th_data + 1;
    }
    for (int m = 0; m < ii; m++) {
      int enc_data = th_data;
      if (m == ii - 1) enc_data = inner_totaldata - th_data * (ii - 1);
      const size_t base = (size_t)send_loc + (size_t)m * (th_data + 16 + 5) + 5;
      if (totaldata >= 65536) {
        const uint32_t nc = (uint32_t)(prsd_segment + m);
        orc_nonce602(nonce, (s == segments_no - 1) ? '1' : '0', nc);
        wire[base - 5] = nonce[7];
        wire[base - 4] = (uint8_t)(nc >> 24);
        wire[base - 3] = (uint8_t)(nc >> 16);
        wire[base - 2] = (uint8_t)(nc >> 8);
        wire[base - 1] = (uint8_t)nc;
      } else {
        memcpy(nonce, header + 4, 12);
      }
      orc_gcm_seal(seg_key, nonce, 12, NULL, 0, buf + enc_loc + (size_t)m * th_data, (size_t)enc_data, wire + base);
    }
    prsd_segment += ii;
    send_loc += inner_totaldata + ii * (16 + 5);
    enc_loc += inner_totaldata;
  }
}
