/*
 * ctrmode_ref.c — CryptMPI's counter-mode message paths.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates, statement by statement:
 *   700 sender  MPI_SEC_BaseCounter_Pipeline_Send      MV/src/mpi/pt2pt/send.c:886-1017
 *   700 receiver MPI_SEC_BaseCounter_Pipeline_Recv     MV/src/mpi/pt2pt/recv.c:812-940
 *   702 sender  MPI_SEC_PreComputeCounter_Send_v4      send.c:1502-1987 (incl. the "dynamic
 *               pre-computation" loop :1862-1983 and multithreaded_generateCommonEncMask
 *               :1052-1156), on the ring of ctr_ring_ref.c (generateCommonEncMask /
 *               encryption_common_counter)
 *   702 receiver MPI_SEC_PreComputeCounter_Recv_v4     recv.c:1025-1403 (mask generation while
 *               the payload is in flight :1107-1196, decryption_common_counter_ivflag :954-1023)
 *   702 keys    init_counter_mode_keys                 MV/src/mpi/init/init.c:766-792 (initial
 *               4 KiB mask of stream A)
 * with the reference's constants (mpiimpl.h:319-399): PIPELINE_SIZE 512 KiB, LARGE_SEGMENT_SIZE
 * 1 MiB - 1, PRE_COM_DATA_RANGE 64 KiB, COUNTER_HEADER_SIZE 26, DYNAMIC_PIPELINE 1,
 * PSC_BRIDGE_TUNE 0, BASE_COUNTER_NO_PIPELINE 1, BASE_COUNTER_LIBRARY_NONCE 0.  Integer
 * expressions keep the reference's types, including `(unsigned long)(n - 1) / 16 + 1` (which is
 * 2^60 for n = 0) where the reference writes it.  Header bytes the reference never writes (they
 * keep whatever the static large_send_buffer held) are zero here.  Timing-dependent loops (how
 * often MPI_Test fails) are parameters: `rounds` generation iterations, `premask` = the payload
 * had not arrived when the receiver started generating its mask.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define PIPELINE_SIZE 524288
#define LARGE_SEGMENT_SIZE 1048575
#define PRE_COM_DATA_RANGE 65536
#define SIXTY_4K 65536
#define TWO_FIVE_6K 262144
#define THIRTY_2K 32768
#define ONE_M 1048576

static void put_be32(uint8_t *p, unsigned int v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}
static unsigned int get_be32(const uint8_t *p) {
  return ((unsigned int)p[0] << 24) | ((unsigned int)p[1] << 16) | ((unsigned int)p[2] << 8) | p[3];
}

/* ------------------------------------------------------------------------- 700 (base counter) */
/* send.c:886-1017: header [0..3] BE32 n, [5..8] BE32 base_global_counter, [21..24] BE32
 * PIPELINE_SIZE; ct = CTR(IV_Count(Send_common_IV, base_global_counter)) ^ buf (one segment:
 * BASE_COUNTER_NO_PIPELINE). */
void orc_700_send(const uint8_t key[16], const uint8_t send_iv[16], unsigned long *base_global_counter,
                  const uint8_t *buf, int totaldata, uint8_t hdr[26], uint8_t *out) {
  uint8_t iv_buffer[20];
  memset(hdr, 0, 26);
  put_be32(hdr + 21, (unsigned int)PIPELINE_SIZE);
  put_be32(hdr, (unsigned int)totaldata);
  memcpy(iv_buffer, send_iv, 16);
  put_be32(hdr + 5, (unsigned int)*base_global_counter);
  orc_iv_count(iv_buffer, *base_global_counter);
  orc_ctr128_xor(key, iv_buffer, buf, out, (size_t)totaldata);
  *base_global_counter += (unsigned long)(totaldata - 1) / 16 + 1;
}

/* recv.c:812-940 (segments_no = 1) */
void orc_700_recv(const uint8_t key[16], const uint8_t recv_iv[16], const uint8_t hdr[26], const uint8_t *in,
                  uint8_t *out) {
  uint8_t iv_buffer[20];
  unsigned int totaldata = get_be32(hdr);
  unsigned long recv_counter = get_be32(hdr + 5);
  memcpy(iv_buffer, recv_iv, 16);
  orc_iv_count(iv_buffer, recv_counter);
  orc_ctr128_xor(key, iv_buffer, in, out, totaldata);
}

/* ------------------------------------------------------------------------- 702 (precomputed) */
void orc_702_init(orc_702_t *s, const uint8_t key[16], const uint8_t send_iv[32], uint8_t *ring, int max,
                  int series) {
  uint8_t *zeros;
  memset(s, 0, sizeof *s);
  orc_ring_init(&s->ring, key, send_iv, ring, max);
  memcpy(s->ivb, send_iv + 16, 16);
  s->series = series;
  /* init.c:772-781: INITIAL_COMMON_COUNTER_SZ of stream A from Send_common_IV */
  zeros = calloc(4096, 1);
  orc_ctr128_xor(key, send_iv, zeros, ring, 4096);
  free(zeros);
  s->ring.counter = 4096 / 16;
  s->ring.compute_size = 4096;
  s->ring.start = 0;
  s->ring.end = 4096;
  s->ring.counter_needto_send = 0;
}

/* send.c:1502-1860 (everything up to the pre-computation loop) */
int orc_702_send(orc_702_t *s, int pending, const uint8_t *buf, int totaldata, uint8_t hdr[26], uint8_t *out) {
  int segments_no, my_thread_no, choping_sz, th_data, inner_totaldata, ii, segment_counter;
  int inner_segment_counter, enc_data, base, send_loc, t_counter_data;
  unsigned long t_counter, temp_counter_to_send;
  uint8_t iv_buffer[50];
  memset(hdr, 0, 26);
  put_be32(hdr, (unsigned int)totaldata);
  choping_sz = PIPELINE_SIZE;
  if (totaldata > PIPELINE_SIZE && totaldata > LARGE_SEGMENT_SIZE) {
    segments_no = 1;
    segments_no += (totaldata - (PIPELINE_SIZE)-1) / (PIPELINE_SIZE) + 1;
  } else {
    segments_no = 1;
  }
  if (totaldata < SIXTY_4K) my_thread_no = 1;
  else if (totaldata < TWO_FIVE_6K) my_thread_no = 8;
  else my_thread_no = 12;
  if (my_thread_no > s->series) my_thread_no = s->series;
  if ((pending + segments_no > 64 && segments_no > 1) || (totaldata >= SIXTY_4K && totaldata <= LARGE_SEGMENT_SIZE)) {
    hdr[20] = '4';
    choping_sz = (totaldata - 1) / my_thread_no + 1;
    choping_sz = (choping_sz - 1) / 16 * 16 + 16;
    segments_no = 1;
  } else {
    hdr[20] = '1';
    if (totaldata > LARGE_SEGMENT_SIZE) {
      int temp_thread = 12; /* PIPELINE_SIZE > TWO_FIVE_6K */
      if (temp_thread > s->series) temp_thread = s->series;
      my_thread_no = temp_thread;
    }
    choping_sz = (PIPELINE_SIZE - 1) / my_thread_no + 1;
    choping_sz = (choping_sz - 1) / 16 * 16 + 16;
  }
  put_be32(hdr + 21, (unsigned int)choping_sz);
  if (totaldata < PRE_COM_DATA_RANGE) {
    if (s->ring.compute_size < totaldata) {
      hdr[4] = '1';
      temp_counter_to_send = s->counter_needto_send_large_msg;
    } else {
      hdr[4] = '0';
      temp_counter_to_send = s->ring.counter_needto_send;
    }
  } else {
    temp_counter_to_send = s->counter_needto_send_large_msg;
  }
  put_be32(hdr + 5, (unsigned int)temp_counter_to_send);
  if (totaldata < PRE_COM_DATA_RANGE) {
    if (s->ring.compute_size >= totaldata) {
      orc_ring_encrypt(&s->ring, buf, totaldata, out);
    } else {
      memcpy(iv_buffer, s->ivb, 16);
      orc_iv_count(iv_buffer, s->enc_common_counter_long_msg);
      orc_ctr128_xor(s->ring.key, iv_buffer, buf, out, (size_t)totaldata);
      s->enc_common_counter_long_msg += (unsigned long)(totaldata - 1) / 16 + 1;
      s->counter_needto_send_large_msg += ((totaldata - 1) / 16) + 1;
    }
    return 1;
  }
  send_loc = 0;
  for (segment_counter = 0; segment_counter < segments_no; segment_counter++) {
    th_data = choping_sz;
    if (segment_counter == segments_no - 1) {
      inner_totaldata = totaldata - (PIPELINE_SIZE * (segments_no - 1));
      ii = (inner_totaldata - 1) / th_data + 1;
    } else {
      inner_totaldata = PIPELINE_SIZE;
      ii = (PIPELINE_SIZE - 1) / th_data + 1;
    }
    for (inner_segment_counter = 0; inner_segment_counter < ii; inner_segment_counter++) {
      enc_data = th_data;
      if (inner_segment_counter == ii - 1) enc_data = inner_totaldata - th_data * (ii - 1);
      base = send_loc + inner_segment_counter * th_data;
      t_counter_data = th_data * inner_segment_counter;
      if (t_counter_data < 1) t_counter = s->enc_common_counter_long_msg;
      else t_counter = s->enc_common_counter_long_msg + (unsigned long)((t_counter_data - 1) / 16 + 1);
      memcpy(iv_buffer, s->ivb, 16);
      orc_iv_count(iv_buffer, t_counter);
      orc_ctr128_xor(s->ring.key, iv_buffer, buf + base, out + base, (size_t)enc_data);
    }
    s->enc_common_counter_long_msg += (unsigned long)(inner_totaldata - 1) / 16 + 1;
    send_loc += inner_totaldata;
  }
  s->counter_needto_send_large_msg += ((totaldata - 1) / 16) + 1;
  return segments_no;
}

/* send.c:1052-1156; returns 0, or -1 where the reference prints ___ERROR___ and exits */
static int mt_generate(orc_702_t *s, int common_counter_gen_sz, int t_common_start, int t_common_end,
                       int t_compute_size, unsigned long t_common_counter) {
  const int MAX = s->ring.max;
  int blockamount, tempamount;
  uint8_t iv_buffer[20], *zeros;
  if (!(t_compute_size <= (MAX - common_counter_gen_sz - 32))) return 0;
  blockamount = ((common_counter_gen_sz - 1) / 16) * 16 + 16;
  zeros = calloc((size_t)blockamount + 16, 1);
  if (t_common_end > t_common_start && t_common_end + blockamount <= MAX) {
    memcpy(iv_buffer, s->ring.iv, 16);
    orc_iv_count(iv_buffer, t_common_counter);
    orc_ctr128_xor(s->ring.key, iv_buffer, zeros, s->ring.buf + t_common_end, (size_t)blockamount);
  } else if (t_common_end > t_common_start && t_common_end + blockamount > MAX) {
    tempamount = MAX - t_common_end;
    if (blockamount > tempamount) {
      if (tempamount) {
        memcpy(iv_buffer, s->ring.iv, 16);
        orc_iv_count(iv_buffer, t_common_counter);
        orc_ctr128_xor(s->ring.key, iv_buffer, zeros, s->ring.buf + t_common_end, (size_t)tempamount);
        t_compute_size += tempamount;
        t_common_end += tempamount;
        t_common_counter += (unsigned long)(tempamount / 16);
      }
      blockamount = blockamount - tempamount;
      t_common_end = 0;
    }
    memcpy(iv_buffer, s->ring.iv, 16);
    orc_iv_count(iv_buffer, t_common_counter);
    orc_ctr128_xor(s->ring.key, iv_buffer, zeros, s->ring.buf + t_common_end, (size_t)blockamount);
  } else if (t_common_end < t_common_start && blockamount + t_common_end < t_common_start) {
    memcpy(iv_buffer, s->ring.iv, 16);
    orc_iv_count(iv_buffer, t_common_counter);
    orc_ctr128_xor(s->ring.key, iv_buffer, zeros, s->ring.buf + t_common_end, (size_t)blockamount);
  } else if (t_common_end == t_common_start && t_compute_size == 0) {
    tempamount = MAX - t_common_end;
    if (blockamount > tempamount) {
      if (tempamount) {
        memcpy(iv_buffer, s->ring.iv, 16);
        orc_iv_count(iv_buffer, t_common_counter);
        orc_ctr128_xor(s->ring.key, iv_buffer, zeros, s->ring.buf + t_common_end, (size_t)tempamount);
        t_compute_size += tempamount;
        t_common_end += tempamount;
        t_common_counter += (unsigned long)(tempamount / 16);
      }
      blockamount = blockamount - tempamount;
      t_common_end = 0;
    }
    memcpy(iv_buffer, s->ring.iv, 16);
    orc_iv_count(iv_buffer, t_common_counter);
    orc_ctr128_xor(s->ring.key, iv_buffer, zeros, s->ring.buf + t_common_end, (size_t)blockamount);
  } else {
    free(zeros);
    return -1;
  }
  free(zeros);
  return 0;
}

/* send.c:1862-1983 with `rounds` generation iterations (the reference runs one per failed
 * MPI_Test).  Returns the iterations that generated, or -1 on the reference's error exit. */
int orc_702_precompute(orc_702_t *s, int totaldata, int rounds) {
  int common_counter_gen_sz, my_thread_no, th_data, segments_no, pre_com_data = 0, done = 0, r, j;
  if (totaldata <= 16) common_counter_gen_sz = 16;
  else if (totaldata < 1024) common_counter_gen_sz = totaldata;
  else if (totaldata < 4096) common_counter_gen_sz = 1024;
  else common_counter_gen_sz = 4096;
  if (totaldata < SIXTY_4K) {
    for (r = 0; r < rounds; r++) {
      int g = orc_ring_generate(&s->ring, totaldata);
      if (g < 0) return -1;
      done += g;
    }
    return done;
  }
  if (common_counter_gen_sz < THIRTY_2K) my_thread_no = 1;
  else if (common_counter_gen_sz < SIXTY_4K) my_thread_no = 4;
  else if (common_counter_gen_sz <= TWO_FIVE_6K) my_thread_no = 8;
  else my_thread_no = 16;
  if (my_thread_no > s->series) my_thread_no = s->series;
  th_data = common_counter_gen_sz / my_thread_no;
  th_data = ((th_data - 1) / 16) * 16 + 16;
  segments_no = my_thread_no;
  if (totaldata > ONE_M) totaldata = totaldata / 2;
  for (r = 0; r < rounds; r++) {
    if ((s->ring.compute_size + th_data * segments_no) <= (s->ring.max - 16) &&
        (pre_com_data + th_data * segments_no <= totaldata)) {
      for (j = 0; j < segments_no; j++) {
        int t_end_pos = s->ring.end + th_data * j;
        unsigned long t_counter;
        if (t_end_pos >= s->ring.max) t_end_pos = t_end_pos - s->ring.max;
        if (j > 0) t_counter = s->ring.counter + (unsigned long)(((th_data * j) - 1) / 16 + 1);
        else t_counter = s->ring.counter;
        if (mt_generate(s, th_data, s->ring.start, t_end_pos, s->ring.compute_size, t_counter)) return -1;
      }
      s->ring.end += (th_data * segments_no);
      if (s->ring.end >= s->ring.max) s->ring.end = s->ring.end - s->ring.max;
      s->ring.counter += (unsigned long)(((th_data * segments_no) - 1) / 16 + 1);
      s->ring.compute_size += (th_data * segments_no);
      pre_com_data += (th_data * segments_no);
      done++;
    } else {
      break; /* MPI_Wait_original: no more generation for this request */
    }
  }
  return done;
}

/* recv.c:1025-1403.  recv_iv = Recv_common_IV[source*32 .. +32).  premask: the payload had not
 * arrived at the first MPI_Test, so the mask is generated first (and the generation loop ran to
 * completion); otherwise the direct-CTR path.  Returns the mask bytes generated. */
int orc_702_recv(const uint8_t key[16], const uint8_t recv_iv[32], const uint8_t hdr[26], const uint8_t *in,
                 uint8_t *out, int premask) {
  int totaldata = (int)get_be32(hdr);
  int choping_sz = (int)get_be32(hdr + 21);
  unsigned long common_recv_counter = get_be32(hdr + 5);
  unsigned int temp_recv_counter = (unsigned int)common_recv_counter;
  uint8_t iv_buffer[20];
  if (totaldata < PRE_COM_DATA_RANGE) {
    const uint8_t preCTRflag = hdr[4];
    const uint8_t *ivs = preCTRflag == '0' ? recv_iv : recv_iv + 16;
    if (premask) {
      int decryption_mask = 0, mask_cap = totaldata + 1024;
      uint8_t *dec_common_buffer = calloc((size_t)mask_cap, 1), *zeros = calloc((size_t)mask_cap, 1);
      if (totaldata > 1024) {
        const int common_counter_gen_sz = 512;
        for (;;) {
          orc_iv_count_out(iv_buffer, common_recv_counter, ivs);
          orc_ctr128_xor(key, iv_buffer, zeros, &dec_common_buffer[decryption_mask], (size_t)common_counter_gen_sz);
          decryption_mask += common_counter_gen_sz;
          common_recv_counter += (unsigned long)((common_counter_gen_sz - 1) / 16 + 1);
          if (decryption_mask >= totaldata) break;
        }
      } else {
        memcpy(iv_buffer, ivs, 16);
        orc_iv_count(iv_buffer, common_recv_counter);
        orc_ctr128_xor(key, iv_buffer, zeros, dec_common_buffer, (size_t)totaldata);
        decryption_mask = totaldata;
      }
      if (decryption_mask < totaldata) {
        decryption_mask = 0;
        common_recv_counter = temp_recv_counter;
      }
      /* decryption_common_counter_ivflag (recv.c:954-1023): mask prefix, then direct CTR */
      orc_mask_decrypt(key, ivs, common_recv_counter, dec_common_buffer, decryption_mask, in, totaldata, out);
      free(zeros);
      free(dec_common_buffer);
      return decryption_mask;
    }
    memcpy(iv_buffer, ivs, 16);
    orc_iv_count(iv_buffer, common_recv_counter);
    orc_ctr128_xor(key, iv_buffer, in, out, (size_t)totaldata);
    return 0;
  }
  {
    int segments_no, segment_counter, th_data, inner_totaldata, ii, m, recv_pos = 0;
    if (totaldata > PIPELINE_SIZE && totaldata > LARGE_SEGMENT_SIZE) {
      segments_no = 1;
      segments_no += (int)(totaldata - (PIPELINE_SIZE)-1) / (PIPELINE_SIZE) + 1;
    } else {
      segments_no = 1;
    }
    if (hdr[20] == '3' || hdr[20] == '4') segments_no = 1;
    for (segment_counter = 0; segment_counter < segments_no; segment_counter++) {
      th_data = choping_sz;
      if (segment_counter == segments_no - 1) {
        inner_totaldata = totaldata - (PIPELINE_SIZE * (segments_no - 1));
        ii = (inner_totaldata - 1) / th_data + 1;
      } else {
        inner_totaldata = PIPELINE_SIZE;
        ii = (PIPELINE_SIZE - 1) / th_data + 1;
      }
      for (m = 0; m < ii; m++) {
        int enc_data = th_data, pos, t_counter_data;
        unsigned long t_counter;
        if (m == ii - 1) enc_data = inner_totaldata - th_data * (ii - 1);
        pos = recv_pos + m * th_data;
        t_counter_data = th_data * m;
        if (t_counter_data < 1) t_counter = common_recv_counter;
        else t_counter = common_recv_counter + (unsigned long)((t_counter_data - 1) / 16 + 1);
        orc_iv_count_out(iv_buffer, t_counter, recv_iv + 16);
        orc_ctr128_xor(key, iv_buffer, in + pos, out + pos, (size_t)enc_data);
      }
      common_recv_counter += (unsigned long)(inner_totaldata - 1) / 16 + 1;
      recv_pos += inner_totaldata;
    }
  }
  return 0;
}
