// frame_host.hpp — include/cmpi_frame.h: CryptMPI 600/602 framings driven on the device.
// Included at the end of cmpi_aead.hip (one translation unit; uses gcm_batch / NonceSpec).
//
// A 602 message is a list of segments (plaintext offset, prefix offset in the wire, length,
// counter, flag) enumerated exactly as send.c:646-835 / recv.c:583-800 walk them.  Consecutive
// segments with equal length and flag, consecutive counters and constant strides form one
// uniform GCM batch (one launch): with the reference's thread counts (powers of two dividing
// 512 KiB) a whole message is one or two launches.  Nonces and the 5-byte prefixes are produced
// inside the GCM kernel (GcmArgs::nmode), so no host bytes move except the 25-byte header.
#pragma once
#include "../../include/cmpi_frame.h"

namespace {

constexpr uint32_t k602Pipe = 524288u;     // PIPELINE_SIZE, mpiimpl.h:333
constexpr uint32_t k602Large = 1048575u;   // LARGE_SEGMENT_SIZE, mpiimpl.h:334
constexpr uint32_t k602Subkey = 65535u;    // SUBKEY_GEN_START, mpiimpl.h:336

struct Seg602 {
  uint64_t pt_off, wire_off;  // wire_off = start of the 5-byte prefix
  uint32_t len, ctr;
  uint8_t flag;
};

uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

// Segments of outer messages [first, first + count): the walk of send.c:734-850 (mode '1')
// or :646-706 (mode '4', one outer message).
std::vector<Seg602> segments_602(const cmpi_602_plan& p, uint32_t first, uint32_t count) {
  std::vector<Seg602> v;
  const int64_t n = p.total, th = p.chop;
  if (p.mode == '4') {
    if (first > 0 || count == 0) return v;
    for (uint32_t i = 0; i < p.nseg; ++i) {
      const int64_t len = (i + 1 == p.nseg) ? n - th * (int64_t)(p.nseg - 1) : th;
      v.push_back({(uint64_t)(th * i), (uint64_t)i * (uint64_t)(th + 21), (uint32_t)len, i, (uint8_t)'0'});
    }
    return v;
  }
  uint64_t send_loc = 0, enc_loc = 0;
  uint32_t prsd = 0;
  for (uint32_t s = 0; s < p.outer && s < first + count; ++s) {
    const int64_t inner = (s + 1 == p.outer) ? n - (int64_t)k602Pipe * (p.outer - 1) : (int64_t)k602Pipe;
    const uint32_t ii = (uint32_t)((inner - 1) / th + 1);
    if (s >= first) {
      for (uint32_t m = 0; m < ii; ++m) {
        const int64_t len = (m + 1 == ii) ? inner - th * (int64_t)(ii - 1) : th;
        v.push_back({enc_loc + (uint64_t)(th * m), send_loc + (uint64_t)m * (uint64_t)(th + 21), (uint32_t)len,
                     prsd + m, (uint8_t)((s + 1 == p.outer) ? '1' : '0')});
      }
    }
    prsd += ii;
    send_loc += (uint64_t)inner + 21ull * ii;
    enc_loc += (uint64_t)inner;
  }
  return v;
}

// Run the segments as uniform batches.  nmode: seal 2 (prefix written), open 1 (prefix read).
// small (n <= 65535, mode '1'): one segment keyed by the header nonce (nmode 3).  The wire and
// plaintext pointers address byte pt_base / w_base of the message (the host paths stage one outer
// message's span at a time); status[k] is segment segs[0] + k.
template <bool DEC>
int run_602(const cmpi_ctx* c, const cmpi_602_plan& p, const uint8_t header[25], uint8_t* wire_out,
            const uint8_t* wire_in, uint8_t* pt_out, const uint8_t* pt_in, const std::vector<Seg602>& segs,
            int32_t* status, void* stream, uint64_t pt_base = 0, uint64_t w_base = 0, void* ws = nullptr,
            size_t* ws_need = nullptr) {
  // small message (recv.c:401-440 / send.c:800-803): one segment under the header nonce
  const bool small = p.mode == '1' && p.total <= k602Pipe;
  size_t i = 0;
  while (i < segs.size()) {
    // one batch per run of equal-length segments at uniform pitches; the sender's flag byte may
    // change once inside a run (the last outer message's segments carry '1', send.c:779-799),
    // the receiver reads it from the wire
    size_t j = i + 1, split = 0;
    if (!small && j < segs.size()) {
      const uint64_t dp = segs[j].pt_off - segs[i].pt_off, dw = segs[j].wire_off - segs[i].wire_off;
      while (j < segs.size() && segs[j].len == segs[i].len && segs[j].ctr == segs[i].ctr + (j - i) &&
             segs[j].pt_off == segs[i].pt_off + dp * (j - i) && segs[j].wire_off == segs[i].wire_off + dw * (j - i)) {
        if (!DEC && segs[j].flag != segs[j - 1].flag) {
          if (split) break;
          split = j - i;
        }
        ++j;
      }
    }
    const Seg602& s0 = segs[i];
    const size_t nrec = j - i;
    const size_t pt_stride = nrec > 1 ? segs[i + 1].pt_off - s0.pt_off : s0.len;
    const size_t w_stride = nrec > 1 ? segs[i + 1].wire_off - s0.wire_off : s0.len + 21;
    NonceSpec ns;
    if (small) {
      ns.mode = 3;
      memcpy(ns.fix, header + 4, 12);
    } else {
      ns.mode = DEC ? 1 : 2;
      ns.ctr0 = s0.ctr;
      ns.flag = s0.flag;
      if (split) {
        ns.flag2 = segs[i + split].flag;
        ns.flag2_from = (uint32_t)split;
      }
    }
    if (ws_need) {  // sizing pass: the largest workspace one of the batches needs (they run in turn)
      *ws_need = std::max(*ws_need, gcm_ws_bytes(c, plan_gcm(c, s0.len, nrec), nrec));
      i = j;
      continue;
    }
    int rc;
    const uint64_t po = s0.pt_off - pt_base, wo = s0.wire_off - w_base;
    if (!DEC) {
      rc = gcm_batch<false>(c, wire_out + wo + 5, w_stride, pt_in + po, pt_stride, small ? nullptr : wire_out + wo,
                            w_stride, s0.len, nrec, nullptr, ws, stream, ns);
    } else {
      rc = gcm_batch<true>(c, pt_out + po, pt_stride, wire_in + wo + 5, w_stride, small ? nullptr : wire_in + wo,
                           w_stride, s0.len, nrec, status ? status + s0.ctr - segs[0].ctr : nullptr, ws,
                           stream, ns);
    }
    if (rc) return rc;
    i = j;
  }
  return CMPI_OK;
}

int check_602(const cmpi_602_plan* p) {
  if (!p) return fail(CMPI_EINVAL, "null plan");
  if (p->mode != '4' && p->mode != '1') return fail(CMPI_EINVAL, "602 mode must be '4' or '1'");
  if (p->chop == 0) return fail(CMPI_EINVAL, "602 chop is 0");
  return CMPI_OK;
}

}  // namespace

extern "C" {

int cmpi_602_plan_make(uint32_t n, int series_threads, int pending_isends, cmpi_602_plan* plan) {
  if (!plan) return fail(CMPI_EINVAL, "null plan");
  if (n > 0x7FFFFFFFu) return fail(CMPI_EINVAL, "602 message larger than INT_MAX");
  if (series_threads < 1) return fail(CMPI_EINVAL, "series_threads must be >= 1");
  const int64_t total = n;
  // send.c:392-400
  int64_t segments_no = 1;
  if (total > k602Pipe && total > k602Large) segments_no = 1 + (total - k602Pipe - 1) / k602Pipe + 1;
  // send.c:420-436
  int t = total < 65536 ? 1 : total < 131072 ? 2 : total < 524288 ? 4 : 8;
  if (t > series_threads) t = series_threads;
  cmpi_602_plan p{};
  p.total = n;
  // send.c:470-530
  if (((int64_t)pending_isends + segments_no > 64 && segments_no > 1) || (total >= 65536 && total <= k602Large)) {
    p.mode = '4';
    p.chop = (uint32_t)((total - 1) / t + 1);
  } else {
    p.mode = '1';
    if (total > k602Large) t = std::min(8, series_threads);
    p.chop = (uint32_t)((int64_t)(k602Pipe - 1) / t + 1);
  }
  p.subkey = total > k602Subkey;
  p.outer = p.mode == '4' ? 1u : (uint32_t)segments_no;
  if (p.mode == '4') {
    p.nseg = (uint32_t)((total - 1) / p.chop + 1);
  } else {
    p.nseg = 0;
    for (int64_t s = 0; s < segments_no; ++s) {
      const int64_t inner = (s == segments_no - 1) ? total - (int64_t)k602Pipe * (segments_no - 1) : (int64_t)k602Pipe;
      p.nseg += (uint32_t)((inner - 1) / p.chop + 1);
    }
  }
  p.wire_bytes = (uint64_t)n + 21ull * p.nseg;
  *plan = p;
  return CMPI_OK;
}

int cmpi_602_plan_from_header(const uint8_t header[25], cmpi_602_plan* plan) {
  if (!header || !plan) return fail(CMPI_EINVAL, "null argument");
  cmpi_602_plan p{};
  p.total = be32(header);
  p.chop = be32(header + 21);
  p.subkey = p.total > k602Subkey;
  const uint8_t m = header[20];
  if (p.total > 0x7FFFFFFFu || p.chop == 0) return fail(CMPI_EINVAL, "malformed 602 header");
  const int64_t total = p.total;
  if (m == '3' || m == '4') {  // recv.c:537-540
    p.mode = '4';
    p.outer = 1;
    p.nseg = (uint32_t)((total - 1) / p.chop + 1);
  } else if (total <= k602Pipe) {  // recv.c:401-440: one segment of n bytes, header nonce
    p.mode = '1';
    p.chop = k602Pipe;  // one segment whatever the header says (the reference ignores it here)
    p.outer = 1;
    p.nseg = 1;
  } else {  // recv.c:444-452, :712-726
    p.mode = '1';
    int64_t segments_no = 1;
    if (total > k602Pipe && total > k602Large) segments_no = 1 + (total - k602Pipe - 1) / k602Pipe + 1;
    p.outer = (uint32_t)segments_no;
    p.nseg = 0;
    for (int64_t s = 0; s < segments_no; ++s) {
      const int64_t inner = (s == segments_no - 1) ? total - (int64_t)k602Pipe * (segments_no - 1) : (int64_t)k602Pipe;
      p.nseg += (uint32_t)((inner - 1) / p.chop + 1);
    }
  }
  p.wire_bytes = (uint64_t)p.total + 21ull * p.nseg;
  *plan = p;
  return CMPI_OK;
}

int cmpi_602_header(const cmpi_602_plan* plan, const uint8_t rand16[16], uint8_t header[25]) {
  int rc = check_602(plan);
  if (rc) return rc;
  if (!rand16 || !header) return fail(CMPI_EINVAL, "null argument");
  memset(header, 0, 25);
  put_be32(header, plan->total);      // send.c:371-374
  memcpy(header + 4, rand16, 16);      // send.c:553-566 (V) / :593-596 (nonce)
  header[20] = plan->mode;             // send.c:471 / :477
  put_be32(header + 21, plan->chop);   // send.c:545-549
  return CMPI_OK;
}

int cmpi_602_outer_span(const cmpi_602_plan* plan, uint32_t o, uint64_t* wire_off, uint64_t* wire_len,
                        uint64_t* pt_off, uint64_t* pt_len) {
  int rc = check_602(plan);
  if (rc) return rc;
  if (o >= plan->outer) return fail(CMPI_EINVAL, "outer index out of range");
  const std::vector<Seg602> s = segments_602(*plan, o, 1);
  if (s.empty()) return fail(CMPI_EINVAL, "empty outer message");
  const Seg602& last = s.back();
  if (wire_off) *wire_off = s.front().wire_off;
  if (wire_len) *wire_len = last.wire_off + last.len + 21 - s.front().wire_off;
  if (pt_off) *pt_off = s.front().pt_off;
  if (pt_len) *pt_len = last.pt_off + last.len - s.front().pt_off;
  return CMPI_OK;
}

int cmpi_602_seal_outer(const cmpi_ctx* c, const cmpi_602_plan* plan, const uint8_t header[25], uint8_t* wire,
                        const uint8_t* in, uint32_t first, uint32_t count, void* stream) {
  int rc = check_602(plan);
  if (rc) return rc;
  if (!c || !header || !wire || (!in && plan->total)) return fail(CMPI_EINVAL, "null argument");
  if (first > plan->outer || count > plan->outer - first) return fail(CMPI_EINVAL, "outer range out of bounds");
  const std::vector<Seg602> segs = segments_602(*plan, first, count);
  return run_602<false>(c, *plan, header, wire, nullptr, nullptr, in ? in : wire, segs, nullptr, stream);
}

int cmpi_602_seal(const cmpi_ctx* c, const cmpi_602_plan* plan, const uint8_t header[25], uint8_t* wire,
                  const uint8_t* in, void* stream) {
  int rc = check_602(plan);
  if (rc) return rc;
  return cmpi_602_seal_outer(c, plan, header, wire, in, 0, plan->outer, stream);
}

int cmpi_602_open(const cmpi_ctx* c, const uint8_t header[25], uint8_t* out, const uint8_t* wire, int32_t* status,
                  void* stream) {
  if (!c || !header || !wire || !out) return fail(CMPI_EINVAL, "null argument");
  cmpi_602_plan p;
  int rc = cmpi_602_plan_from_header(header, &p);
  if (rc) return rc;
  const std::vector<Seg602> segs = segments_602(p, 0, p.outer);
  return run_602<true>(c, p, header, nullptr, wire, out, nullptr, segs, status, stream);
}

int cmpi_600_header(uint32_t n, uint8_t kind, uint8_t header[25]) {
  if (!header) return fail(CMPI_EINVAL, "null header");
  if (kind != '1' && kind != '2') return fail(CMPI_EINVAL, "600 kind must be '1' (send) or '2' (isend)");
  memset(header, 0, 25);
  put_be32(header, n);         // send.c:238-241
  header[20] = kind;           // send.c:245 ('1'); isend.c ('2')
  put_be32(header + 21, n);    // send.c:258-262: one thread, chunk = n
  return CMPI_OK;
}

int cmpi_600_seal(const cmpi_ctx* c, const uint8_t nonce[12], uint8_t* payload, const uint8_t* in, size_t n,
                  void* stream) {
  if (!c || !nonce || !payload) return fail(CMPI_EINVAL, "null argument");
  NonceSpec ns;
  ns.mode = 3;
  memcpy(ns.fix, nonce, 12);
  // send.c:294-311: nonce at payload[0..11], ct||tag at payload + 12
  return gcm_batch<false>(c, payload + 12, n + 16, in, n, payload, 12, n, 1, nullptr, nullptr, stream, ns);
}

int cmpi_600_open(const cmpi_ctx* c, uint8_t* out, const uint8_t* payload, size_t n, int32_t* status, void* stream) {
  if (!c || !payload) return fail(CMPI_EINVAL, "null argument");
  return gcm_batch<true>(c, out, n, payload + 12, n + 16, payload, 12, n, 1, status, nullptr, stream);
}

}  // extern "C"
