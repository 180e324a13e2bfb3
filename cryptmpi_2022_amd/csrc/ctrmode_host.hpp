// ctrmode_host.hpp — include/cmpi_ctrmode.h: CryptMPI's 700 / 702 counter-mode messages as
// engine calls.  Included at the end of cmpi_aead.hip after ring_host.hpp (one translation
// unit: uses ctr_launch, xor_launch, the ring's bookkeeping).  The host code follows the
// reference statement by statement (oracle/ctrmode_ref.c is the CPU restatement the tests
// compare against); every keystream byte is a kernel's.
//
// Slices: the reference encrypts a long message as per-thread slices, each from its own
// IV_Count(IV, counter) block (send.c:1805-1808, recv.c:1378-1380).  A slice whose counter block
// equals the previous slice's last block + 1 continues one CTR stream, so such runs are merged
// into one launch; IV_Count's 32-bit accumulator (a dropped carry, send.c:1021) breaks a run
// exactly where the reference's blocks stop being consecutive.
#pragma once
#include "../../include/cmpi_ctrmode.h"

struct cmpi_702_sender {
  const cmpi_ctx* ctx = nullptr;
  cmpi_ctr_ring* ring = nullptr;  // stream A: enc_common_buffer (Send_common_IV[0..16))
  uint8_t ivb[16];                // stream B: Send_common_IV[16..32)
  unsigned long enc_common_counter_long_msg = 0, counter_needto_send_large_msg = 0;
  int series = 1;
};

namespace {

constexpr int kPipe = 524288;       // PIPELINE_SIZE, mpiimpl.h:333
constexpr int kLarge = 1048575;     // LARGE_SEGMENT_SIZE, mpiimpl.h:334
constexpr int kPreCom = 65536;      // PRE_COM_DATA_RANGE, mpiimpl.h:399

struct CtrSlice {
  size_t off, len;
  unsigned long counter;  // IV_Count(iv, counter) is the slice's first counter block
};

void add128_host(uint8_t cb[16], uint64_t k) {
  unsigned carry = 0;
  for (int i = 15; i >= 0; --i) {
    const unsigned s = (unsigned)cb[i] + (unsigned)(k & 0xff) + carry;
    cb[i] = (uint8_t)s;
    carry = s >> 8;
    k >>= 8;
  }
}

// out[off..off+len) = in ^ keystream (in == nullptr: keystream) per slice, consecutive counter
// blocks merged into one launch (or one served op: sv, begun).
int ctr_slices(const cmpi_ctx* c, const uint8_t iv[16], const std::vector<CtrSlice>& v, uint8_t* out,
               const uint8_t* in, void* stream, Served* sv = nullptr) {
  size_t i = 0;
  while (i < v.size()) {
    uint8_t cb[16], next[16];
    memcpy(cb, iv, 16);
    cmpi_iv_count(cb, v[i].counter);
    size_t j = i, len = v[i].len;
    while (j + 1 < v.size() && v[j].len % 16 == 0 && v[j + 1].off == v[j].off + v[j].len) {
      memcpy(next, cb, 16);
      add128_host(next, (len) / 16);  // block after the run so far
      uint8_t nb[16];
      memcpy(nb, iv, 16);
      cmpi_iv_count(nb, v[j + 1].counter);
      if (memcmp(nb, next, 16)) break;
      ++j;
      len += v[j].len;
    }
    const int rc = sv ? sv->ctr(out + v[i].off, in ? in + v[i].off : nullptr, len, cb)
                      : ctr_launch(c, out + v[i].off, in ? in + v[i].off : nullptr, len, cb, stream);
    if (rc) return rc;
    i = j + 1;
  }
  return CMPI_OK;
}

uint32_t be32h(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
void put_be32h(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

// multithreaded_generateCommonEncMask (send.c:1052-1156) on the engine ring: one thread's chunk
// at t_common_end; the caller updates the ring state afterwards.  0, or < 0 where the reference
// prints ___ERROR___ and exits.
int mt_generate_dev(cmpi_ctr_ring* r, int gen, int t_common_start, int t_common_end, int t_compute_size,
                    unsigned long t_common_counter, void* stream) {
  const int MAX = r->max;
  if (!(t_compute_size <= (MAX - gen - 32))) return CMPI_OK;
  int blockamount = ((gen - 1) / 16) * 16 + 16;
  auto fill = [&](int at, int amount, unsigned long ctr) { return ring_ctr(r, ctr, r->dring + at, nullptr, (size_t)amount, stream); };
  auto wrap_fill = [&]() {  // the bodies of the second and fourth branches
    const int tempamount = MAX - t_common_end;
    if (blockamount > tempamount) {
      if (tempamount) {
        const int e = fill(t_common_end, tempamount, t_common_counter);
        if (e) return e;
        t_common_counter += (unsigned long)(tempamount / 16);
      }
      blockamount -= tempamount;
      t_common_end = 0;
    }
    return fill(t_common_end, blockamount, t_common_counter);
  };
  if (t_common_end > t_common_start && t_common_end + blockamount <= MAX) return fill(t_common_end, blockamount, t_common_counter);
  if (t_common_end > t_common_start && t_common_end + blockamount > MAX) return wrap_fill();
  if (t_common_end < t_common_start && blockamount + t_common_end < t_common_start)
    return fill(t_common_end, blockamount, t_common_counter);
  if (t_common_end == t_common_start && t_compute_size == 0) return wrap_fill();
  return fail(CMPI_EINVAL, "702 mask ring inconsistent (send.c:1145-1153 error branch)");
}

}  // namespace

extern "C" {

int cmpi_700_send(const cmpi_ctx* c, const uint8_t send_iv[16], uint64_t* counter, const uint8_t* in, size_t n,
                  uint8_t header[26], uint8_t* out, void* stream) {
  if (!c || !send_iv || !counter || !header) return fail(CMPI_EINVAL, "null argument");
  if (n > 0x7FFFFFFFu) return fail(CMPI_EINVAL, "message larger than INT_MAX");
  if (n && (!in || !out)) return fail(CMPI_EINVAL, "null buffer");
  const int totaldata = (int)n;
  memset(header, 0, 26);
  put_be32h(header + 21, (uint32_t)kPipe);          // send.c:918-922
  put_be32h(header, (uint32_t)totaldata);           // :925-929
  put_be32h(header + 5, (uint32_t)*counter);        // :941-945
  uint8_t iv[16];
  memcpy(iv, send_iv, 16);
  cmpi_iv_count(iv, (unsigned long)*counter);       // :983-986 (one segment)
  int rc = CMPI_OK;
  if (n) {
    Served sv(c, n);
    if (sv) {
      if (!(rc = sv.begin(stream))) rc = sv.ctr(out, in, n, iv);
    } else {
      rc = ctr_launch(c, out, in, n, iv, stream);
    }
  }
  if (rc) return rc;
  *counter += (unsigned long)(totaldata - 1) / 16 + 1;  // :1005
  return CMPI_OK;
}

int cmpi_700_recv(const cmpi_ctx* c, const uint8_t recv_iv[16], const uint8_t header[26], uint8_t* out,
                  size_t out_cap, const uint8_t* in, void* stream) {
  if (!c || !recv_iv || !header) return fail(CMPI_EINVAL, "null argument");
  const uint32_t totaldata = be32h(header);
  if (totaldata && (!in || !out)) return fail(CMPI_EINVAL, "null buffer");
  // the length comes from the wire: bounded by the caller's buffer (the reference trusts it)
  if (totaldata > out_cap) return fail(CMPI_EINVAL, "header announces %u bytes, out holds %zu", totaldata, out_cap);
  uint8_t iv[16];
  memcpy(iv, recv_iv, 16);
  cmpi_iv_count(iv, be32h(header + 5));  // recv.c:867-871
  if (!totaldata) return CMPI_OK;
  Served sv(c, totaldata);
  if (!sv) return ctr_launch(c, out, in, totaldata, iv, stream);
  if (int rc = sv.begin(stream)) return rc;
  return sv.ctr(out, in, totaldata, iv);
}

cmpi_702_sender* cmpi_702_sender_new(const cmpi_ctx* c, const uint8_t send_iv[32], size_t ring_bytes,
                                     int series_threads, void* stream) {
  if (!c || !send_iv || series_threads < 1) {
    fail(CMPI_EINVAL, "null argument or series_threads < 1");
    return nullptr;
  }
  auto* s = new cmpi_702_sender();
  s->ctx = c;
  memcpy(s->ivb, send_iv + 16, 16);
  s->series = series_threads;
  s->ring = cmpi_ctr_ring_new(c, send_iv, ring_bytes);
  if (!s->ring) {
    delete s;
    return nullptr;
  }
  // init.c:772-781: INITIAL_COMMON_COUNTER_SZ (4 KiB) of stream A; on an empty ring this is
  // exactly generateCommonEncMask(4096)'s empty-ring branch (start 0, end 4096, counter 256)
  if (cmpi_ctr_ring_generate(s->ring, 4096, stream) != 1) {
    cmpi_ctr_ring_free(s->ring);
    delete s;
    return nullptr;
  }
  return s;
}

void cmpi_702_sender_free(cmpi_702_sender* s) {
  if (!s) return;
  cmpi_ctr_ring_free(s->ring);
  delete s;
}

int cmpi_702_sender_state(const cmpi_702_sender* s, uint64_t st[7]) {
  if (!s || !st) return fail(CMPI_EINVAL, "null argument");
  const cmpi_ctr_ring* r = s->ring;
  st[0] = (uint64_t)r->start;
  st[1] = (uint64_t)r->end;
  st[2] = (uint64_t)r->compute_size;
  st[3] = r->counter;
  st[4] = r->counter_needto_send;
  st[5] = s->enc_common_counter_long_msg;
  st[6] = s->counter_needto_send_large_msg;
  return CMPI_OK;
}

int cmpi_702_send(cmpi_702_sender* s, int pending, const uint8_t* in, size_t n, uint8_t header[26], uint8_t* out,
                  void* stream) {
  if (!s || !header) return fail(CMPI_EINVAL, "null argument");
  if (n > 0x7FFFFFFFu) return fail(CMPI_EINVAL, "message larger than INT_MAX");
  if (n && (!in || !out)) return fail(CMPI_EINVAL, "null buffer");
  const int totaldata = (int)n;
  memset(header, 0, 26);
  put_be32h(header, (uint32_t)totaldata);  // send.c:1537-1541
  int segments_no = (totaldata > kPipe && totaldata > kLarge) ? 1 + (totaldata - kPipe - 1) / kPipe + 1 : 1;
  int my_thread_no = totaldata < 65536 ? 1 : totaldata < 262144 ? 8 : 12;  // :1579-1586
  if (my_thread_no > s->series) my_thread_no = s->series;                  // :1588-1591
  int choping_sz;
  if ((pending + segments_no > 64 && segments_no > 1) || (totaldata >= 65536 && totaldata <= kLarge)) {
    header[20] = '4';  // :1595-1601
    choping_sz = (totaldata - 1) / my_thread_no + 1;
    choping_sz = (choping_sz - 1) / 16 * 16 + 16;
    segments_no = 1;
  } else {
    header[20] = '1';  // :1604-1637
    if (totaldata > kLarge) my_thread_no = std::min(12, s->series);
    choping_sz = (kPipe - 1) / my_thread_no + 1;
    choping_sz = (choping_sz - 1) / 16 * 16 + 16;
  }
  put_be32h(header + 21, (uint32_t)choping_sz);  // :1643-1647
  cmpi_ctr_ring* r = s->ring;
  std::unique_lock<std::mutex> lk(r->mu);
  unsigned long temp_counter_to_send;  // :1649-1672
  if (totaldata < kPreCom) {
    if (r->compute_size < totaldata) {
      header[4] = '1';
      temp_counter_to_send = s->counter_needto_send_large_msg;
    } else {
      header[4] = '0';
      temp_counter_to_send = r->counter_needto_send;
    }
  } else {
    temp_counter_to_send = s->counter_needto_send_large_msg;
  }
  put_be32h(header + 5, (uint32_t)temp_counter_to_send);
  DeviceGuard dg(s->ctx->device);
  int rc;
  if (totaldata < kPreCom) {  // :1689-1731
    Served sv(s->ctx, n);  // the context's message service, if started (ring_host.hpp)
    if (sv && (rc = sv.begin(stream))) return rc;
    if (r->compute_size >= totaldata) {  // encryption_common_counter (ring_host.hpp), stream A,
      rc = ring_encrypt_locked(r, out, in, n, stream, sv ? &sv : nullptr);  // under the lock that chose it
      return rc ? rc : 1;
    }
    uint8_t iv[16];
    memcpy(iv, s->ivb, 16);
    cmpi_iv_count(iv, s->enc_common_counter_long_msg);
    if (n && (rc = sv ? sv.ctr(out, in, n, iv) : ctr_launch(s->ctx, out, in, n, iv, stream))) return rc;
    s->enc_common_counter_long_msg += (unsigned long)(totaldata - 1) / 16 + 1;
    s->counter_needto_send_large_msg += ((totaldata - 1) / 16) + 1;
    return 1;
  }
  std::vector<CtrSlice> slices;  // :1741-1849
  int send_loc = 0;
  unsigned long ecclm = s->enc_common_counter_long_msg;
  for (int seg = 0; seg < segments_no; ++seg) {
    const int th_data = choping_sz;
    const int inner = seg == segments_no - 1 ? totaldata - kPipe * (segments_no - 1) : kPipe;
    const int ii = (inner - 1) / th_data + 1;
    for (int m = 0; m < ii; ++m) {
      const int enc_data = m == ii - 1 ? inner - th_data * (ii - 1) : th_data;
      const int base = send_loc + m * th_data;
      const int tcd = th_data * m;
      const unsigned long t_counter = tcd < 1 ? ecclm : ecclm + (unsigned long)((tcd - 1) / 16 + 1);
      slices.push_back({(size_t)base, (size_t)enc_data, t_counter});
    }
    ecclm += (unsigned long)(inner - 1) / 16 + 1;
    send_loc += inner;
  }
  if ((rc = ctr_slices(s->ctx, s->ivb, slices, out, in, stream))) return rc;
  s->enc_common_counter_long_msg = ecclm;
  s->counter_needto_send_large_msg += ((totaldata - 1) / 16) + 1;  // :1852
  return segments_no;
}

int cmpi_702_precompute(cmpi_702_sender* s, size_t n, int rounds, void* stream) {
  if (!s) return fail(CMPI_EINVAL, "null sender");
  if (n > 0x7FFFFFFFu || rounds < 0) return fail(CMPI_EINVAL, "bad size or rounds");
  int totaldata = (int)n;
  int gen = totaldata <= 16 ? 16 : totaldata < 1024 ? totaldata : totaldata < 4096 ? 1024 : 4096;  // send.c:1864-1871
  int done = 0;
  if (totaldata < 65536) {  // :1876-1891: generateCommonEncMask(totaldata) per failed MPI_Test
    for (int i = 0; i < rounds; ++i) {
      const int g = cmpi_ctr_ring_generate(s->ring, (size_t)totaldata, stream);
      if (g < 0) return g;
      done += g;
    }
    return done;
  }
  int my_thread_no = gen < 32768 ? 1 : gen < 65536 ? 4 : gen <= 262144 ? 8 : 16;  // :1895-1905
  if (my_thread_no > s->series) my_thread_no = s->series;
  int th_data = gen / my_thread_no;
  th_data = ((th_data - 1) / 16) * 16 + 16;
  const int segments_no = my_thread_no;
  int pre_com_data = 0;
  if (totaldata > 1048576) totaldata = totaldata / 2;
  cmpi_ctr_ring* r = s->ring;
  std::lock_guard<std::mutex> lk(r->mu);
  DeviceGuard dg(s->ctx->device);
  RingOrder ord{r, (hipStream_t)stream};  // ring fills chain after the ring's previous use
  if (int e = ord.begin()) return e;
  for (int i = 0; i < rounds; ++i) {  // :1919-1979
    if (!((r->compute_size + th_data * segments_no) <= (r->max - 16) && (pre_com_data + th_data * segments_no <= totaldata)))
      break;
    for (int j = 0; j < segments_no; ++j) {
      int t_end_pos = r->end + th_data * j;
      if (t_end_pos >= r->max) t_end_pos -= r->max;
      const unsigned long t_counter = j > 0 ? r->counter + (unsigned long)(((th_data * j) - 1) / 16 + 1) : r->counter;
      const int rc = mt_generate_dev(r, th_data, r->start, t_end_pos, r->compute_size, t_counter, stream);
      if (rc) return rc;
    }
    r->end += th_data * segments_no;
    if (r->end >= r->max) r->end -= r->max;
    r->counter += (unsigned long)(((th_data * segments_no) - 1) / 16 + 1);
    r->compute_size += th_data * segments_no;
    pre_com_data += th_data * segments_no;
    ++done;
  }
  return done;
}

int cmpi_702_recv_premask(const cmpi_ctx* c, const uint8_t recv_iv[32], const uint8_t header[26], uint8_t* mask,
                          size_t mask_cap, size_t* mask_len, void* stream) {
  if (!c || !recv_iv || !header || !mask_len) return fail(CMPI_EINVAL, "null argument");
  *mask_len = 0;
  const int totaldata = (int)be32h(header);
  if (totaldata < 0) return fail(CMPI_EINVAL, "malformed header");
  if (totaldata >= kPreCom) return CMPI_OK;  // the reference makes no mask for long messages
  const uint8_t* ivs = header[4] == '0' ? recv_iv : recv_iv + 16;
  const unsigned long c0 = be32h(header + 5);
  DeviceGuard dg(c->device);
  Served sv(c, ((size_t)totaldata + 511) / 512 * 512);
  if (sv)
    if (int rc = sv.begin(stream)) return rc;
  if (totaldata > 1024) {  // recv.c:1111-1139: 512-byte chunks at IV_Count_out(counter + 32k)
    const size_t need = ((size_t)totaldata + 511) / 512 * 512;
    if (!mask || mask_cap < need) return fail(CMPI_EINVAL, "mask buffer smaller than %zu bytes", need);
    std::vector<CtrSlice> v;
    unsigned long ctr = c0;
    for (size_t off = 0; off < need; off += 512) {
      v.push_back({off, 512, ctr});
      ctr += (unsigned long)((512 - 1) / 16 + 1);
    }
    const int rc = ctr_slices(c, ivs, v, mask, nullptr, stream, sv ? &sv : nullptr);
    if (rc) return rc;
    *mask_len = need;
    return CMPI_OK;
  }
  if (totaldata == 0) return CMPI_OK;
  if (!mask || mask_cap < (size_t)totaldata) return fail(CMPI_EINVAL, "mask buffer too small");
  uint8_t iv[16];  // recv.c:1187-1194: the whole (<= 1 KiB) mask from IV_Count(iv, counter)
  memcpy(iv, ivs, 16);
  cmpi_iv_count(iv, c0);
  const int rc = sv ? sv.ctr(mask, nullptr, (size_t)totaldata, iv) : ctr_launch(c, mask, nullptr, (size_t)totaldata, iv, stream);
  if (rc) return rc;
  *mask_len = (size_t)totaldata;
  return CMPI_OK;
}

int cmpi_702_recv(const cmpi_ctx* c, const uint8_t recv_iv[32], const uint8_t header[26], uint8_t* out,
                  size_t out_cap, const uint8_t* in, const uint8_t* mask, size_t mask_len, void* stream) {
  if (!c || !recv_iv || !header) return fail(CMPI_EINVAL, "null argument");
  const int totaldata = (int)be32h(header);
  if (totaldata < 0) return fail(CMPI_EINVAL, "malformed header");
  if (totaldata == 0) return CMPI_OK;
  if ((size_t)totaldata > out_cap) return fail(CMPI_EINVAL, "header announces %d bytes, out holds %zu", totaldata, out_cap);
  if (!out || !in) return fail(CMPI_EINVAL, "null buffer");
  const unsigned long c0 = be32h(header + 5);
  DeviceGuard dg(c->device);
  if (totaldata < kPreCom) {
    const uint8_t* ivs = header[4] == '0' ? recv_iv : recv_iv + 16;
    Served sv(c, (size_t)totaldata);  // the context's message service, if started (ring_host.hpp)
    if (sv)
      if (int rc = sv.begin(stream)) return rc;
    if (mask && mask_len >= (size_t)totaldata)  // decryption_common_counter_ivflag, mask covers it all
      return sv ? sv.xor_(out, mask, in, (size_t)totaldata) : xor_launch(out, mask, in, (size_t)totaldata, (hipStream_t)stream);
    uint8_t iv[16];  // recv.c:1203-1220: no (complete) mask -> direct CTR from the header counter
    memcpy(iv, ivs, 16);
    cmpi_iv_count(iv, c0);
    return sv ? sv.ctr(out, in, (size_t)totaldata, iv) : ctr_launch(c, out, in, (size_t)totaldata, iv, stream);
  }
  const int chop = (int)be32h(header + 21);
  // a sender's choping_sz is a multiple of 16 in [16, totaldata rounded up to 16] (send.c:1595-1637);
  // anything else would size the slice list from untrusted bytes
  if (chop < 16 || chop % 16 || (int64_t)chop > ((int64_t)totaldata + 15) / 16 * 16)
    return fail(CMPI_EINVAL, "malformed header (choping_sz %d for %d bytes)", chop, totaldata);
  int segments_no = (totaldata > kPipe && totaldata > kLarge) ? 1 + (totaldata - kPipe - 1) / kPipe + 1 : 1;
  if (header[20] == '3' || header[20] == '4') segments_no = 1;  // recv.c:1237-1238
  std::vector<CtrSlice> v;  // recv.c:1328-1399
  int recv_pos = 0;
  unsigned long crc = c0;
  for (int seg = 0; seg < segments_no; ++seg) {
    const int th_data = chop;
    const int inner = seg == segments_no - 1 ? totaldata - kPipe * (segments_no - 1) : kPipe;
    const int ii = (inner - 1) / th_data + 1;
    for (int m = 0; m < ii; ++m) {
      const int enc_data = m == ii - 1 ? inner - th_data * (ii - 1) : th_data;
      const int tcd = th_data * m;
      const unsigned long t_counter = tcd < 1 ? crc : crc + (unsigned long)((tcd - 1) / 16 + 1);
      v.push_back({(size_t)(recv_pos + m * th_data), (size_t)enc_data, t_counter});
    }
    crc += (unsigned long)(inner - 1) / 16 + 1;
    recv_pos += inner;
  }
  return ctr_slices(c, recv_iv + 16, v, out, in, stream);
}

}  // extern "C"
