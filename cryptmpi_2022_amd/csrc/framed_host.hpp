// framed_host.hpp — CryptMPI's framed message paths on host memory:
// the 602 pipelined sender / receiver (MV/src/mpi/pt2pt/send.c:729-850, recv.c:679-809), the
// 602 non-blocking pair (isend.c:550, wait.c:889) and the 700 / 702 counter-mode messages straight
// from MPI user buffers (send.c:886-1017, :1716-1727, :1768-1816; recv.c:812-940, :1025-1403).
// Included at the end of cmpi_aead.hip after async_host.hpp (one translation unit: the request
// pool, run_602, the 700/702 device calls).
//
// Every call is a request (cmpi_req, include/cmpi_async.h) on a pooled stream: the host spans it
// reads are copied H2D (page-locked ones by DMA straight from the user's pages, pageable ones
// packed into pinned staging first), the device form of the call runs on the staged bytes, and
// the spans it writes come back D2H (page-locked: into the user's pages; pageable: into pinned
// staging, copied out when the request completes).  The synchronous forms are begin + wait.
//
// The 602 sender's pipeline is the request sequence itself: one *_begin per outer 512 KiB message
// (send.c:754-835 seals outer message k+1 while MPI_Isend of k is in flight); requests go to
// different pooled streams, so outer k+1's H2D / seal / D2H overlap outer k's.  The caller waits
// outer k's request and posts its MPI_Isend, exactly where the reference does.
#pragma once
#include "../../include/cmpi_ctrmode.h"
#include "../../include/cmpi_frame.h"

namespace {

// Flat host copy split over host threads (one outer message is 512 KiB).
void par_copy_span(uint8_t* dst, const uint8_t* src, size_t len) {
  constexpr size_t kPiece = (size_t)256 << 10;
  const size_t n = len / kPiece;
  if (n) par_copy_records(dst, kPiece, src, kPiece, kPiece, n);
  if (len > n * kPiece) memcpy(dst + n * kPiece, src + n * kPiece, len - n * kPiece);
}

struct SpanIn {
  const uint8_t* host;
  size_t dev_off, len;
};
struct SpanOut {
  uint8_t* host;
  size_t dev_off, len;
};

// One framed request: every framed call has one input span (host bytes the device form reads)
// and one output span (host bytes it writes).  launch(din, dout, dstatus, ws, stream) enqueues the
// device form with din / dout the device addresses of the two spans and dstatus the segment
// statuses (open), which land in status[0..nst), ws the request's workspace.  order_after: the request first waits for the
// work enqueued so far on stream `after` (may be the null stream).
// Two forms:
//  * direct (in + out bytes <= g_span_direct): the kernels read and write the caller's
//    page-locked spans themselves over PCIe (device addresses of the pinned pages); pageable spans
//    are packed into / unpacked from the request's pinned staging, which the kernels access the
//    same way.  No DMA command and no device staging: one launch sequence and an event per call,
//    so the 602 sender's per-outer-message requests cost their launches, not copy submissions.
//  * DMA (larger calls): the spans are copied H2D into device staging, the device form runs on
//    it, the output span is copied back D2H (page-locked: straight into the user's pages).
std::atomic<size_t> g_span_direct{(size_t)16 << 20};

// ws_bytes: device workspace of the request's own (the 602 batches' partials): requests of one
// context then run concurrently on their pooled streams instead of queueing on the context's
// scratch lease one after the other.
template <class Launch>
int span_begin(const cmpi_ctx* c, size_t dev_bytes, const SpanIn& in, const SpanOut& out, int32_t* status, size_t nst,
               bool dec, bool order_after, hipStream_t after, Launch launch, cmpi_req** req, size_t ws_bytes = 0) {
  if (!req) return fail(CMPI_EINVAL, "null request");
  *req = nullptr;
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  DeviceGuard dg(c->device);
  StagePool& P = stage_pool(c->device);
  auto* r = new cmpi_req();
  r->device = c->device;
  r->dec = dec;
  r->nst = dec ? nst : 0;
  r->user_status = status;
  auto bail = [&](int rc) {
    if (r->st && r->done) (void)hipStreamSynchronize(r->st);
    req_release(r);
    return rc;
  };
  // every HIP failure after the request exists goes through bail (the request, its
  // pooled stream's work and its staging are released, not leaked)
#define SPAN_TRY(expr)                                                                        \
  do {                                                                                        \
    const hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return bail(fail(CMPI_EHIP, "%s: %s", #expr, hipGetErrorString(e_))); \
  } while (0)
  int rc = pool_stream(P, &r->st);
  if (rc) return bail(rc);
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (!P.events.empty()) {
      r->done = P.events.back();
      P.events.pop_back();
    }
  }
  if (!r->done && hipEventCreateWithFlags(&r->done, hipEventDisableTiming) != hipSuccess)
    return bail(fail(CMPI_EHIP, "event create failed"));
  hipStream_t st = r->st;
  if ((rc = wait_keys(c, st))) return bail(rc);
  if (order_after) {  // device work the call depends on, enqueued by the caller on its own stream
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, kOrderEvent) != hipSuccess) return bail(fail(CMPI_EHIP, "event create failed"));
    const bool ok = hipEventRecord(e, after) == hipSuccess && hipStreamWaitEvent(st, e, 0) == hipSuccess;
    (void)hipEventDestroy(e);  // released once the wait is satisfied
    if (!ok) return bail(fail(CMPI_EHIP, "ordering after the caller's stream failed"));
  }
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const bool direct = in.len + out.len <= g_span_direct.load();
  const uint8_t* in_pin = in.len && direct ? (const uint8_t*)pinned_dev_ptr(in.host) : nullptr;
  uint8_t* out_pin = out.len && direct ? (uint8_t*)pinned_dev_ptr(out.host) : nullptr;
  const bool in_pg = in.len && (direct ? !in_pin : !is_pinned(in.host));
  const bool out_pg = out.len && (direct ? !out_pin : !is_pinned(out.host));
  // pinned staging: pageable input, pageable output, statuses
  const size_t h_in = 0, h_out = in_pg ? up16(in.len) : 0, h_st = h_out + (out_pg ? up16(out.len) : 0);
  const size_t h_total = h_st + up16(4 * nst) + 16;
  if ((rc = pool_take(P, true, h_total, &r->hbuf, &r->hcap))) return bail(rc);
  uint8_t* H = (uint8_t*)r->hbuf;
  if (in_pg) par_copy_span(H + h_in, in.host, in.len);
  if (out_pg) {
    r->span_dst.emplace_back(out.host, H + h_out);
    r->span_len.push_back(out.len);
  }
  r->h_status = (int32_t*)(H + h_st);
  if (direct) {
    uint8_t* dH = (uint8_t*)pinned_dev_ptr(H);
    if (!dH) return bail(fail(CMPI_EHIP, "staging buffer has no device address"));
    if (ws_bytes && (rc = pool_take(P, false, ws_bytes, &r->dbuf, &r->dcap))) return bail(rc);
    // an empty span still gets a valid device address (never accessed), as in the DMA form
    const uint8_t* din = !in.len || in_pg ? dH + h_in : in_pin;
    uint8_t* dout = !out.len || out_pg ? dH + h_out : out_pin;
    if ((rc = launch(din, dout, dec ? (int32_t*)(dH + h_st) : nullptr, ws_bytes ? r->dbuf : nullptr, st)))
      return bail(rc);
  } else {
    const size_t d_st = up16(dev_bytes), d_ws = (d_st + 4 * nst + 255) & ~(size_t)255, d_total = d_ws + ws_bytes + 16;
    if ((rc = pool_take(P, false, d_total, &r->dbuf, &r->dcap))) return bail(rc);
    uint8_t* D = (uint8_t*)r->dbuf;
    if (in.len) SPAN_TRY(hipMemcpyAsync(D + in.dev_off, in_pg ? H + h_in : in.host, in.len, hipMemcpyHostToDevice, st));
    if ((rc = launch(D + in.dev_off, D + out.dev_off, dec ? (int32_t*)(D + d_st) : nullptr, ws_bytes ? D + d_ws : nullptr,
                     st)))
      return bail(rc);
    if (out.len) SPAN_TRY(hipMemcpyAsync(out_pg ? H + h_out : out.host, D + out.dev_off, out.len, hipMemcpyDeviceToHost, st));
    if (dec && nst) SPAN_TRY(hipMemcpyAsync(H + h_st, D + d_st, 4 * nst, hipMemcpyDeviceToHost, st));
  }
  SPAN_TRY(hipEventRecord(r->done, st));
#undef SPAN_TRY
  *req = r;
  return CMPI_OK;
}

// The byte spans of outer messages [first, first + count) of a 602 message.
struct Spans602 {
  std::vector<Seg602> segs;
  uint64_t pt_off = 0, pt_len = 0, w_off = 0, w_len = 0;
};
int spans_602(const cmpi_602_plan& p, uint32_t first, uint32_t count, Spans602& s) {
  if (first > p.outer || count > p.outer - first) return fail(CMPI_EINVAL, "outer range out of bounds");
  s.segs = segments_602(p, first, count);
  if (s.segs.empty()) return CMPI_OK;
  const Seg602 &a = s.segs.front(), &b = s.segs.back();
  s.pt_off = a.pt_off;
  s.pt_len = b.pt_off + b.len - a.pt_off;
  s.w_off = a.wire_off;
  s.w_len = b.wire_off + 5 + b.len + 16 - a.wire_off;
  return CMPI_OK;
}

int sync_req(int rc, cmpi_req* r) { return rc ? rc : cmpi_wait(r); }

constexpr uint32_t k602HostGroup = 4;  // outer messages per request of the synchronous 602 host calls

}  // namespace

extern "C" {

// ---- 602 (send.c:339-884 / recv.c:343-809) from and to host memory
int cmpi_602_seal_host_begin(const cmpi_ctx* c, const cmpi_602_plan* plan, const uint8_t header[25], uint8_t* wire,
                             const uint8_t* in, uint32_t first, uint32_t count, cmpi_req** req) {
  int rc = check_602(plan);
  if (rc) return rc;
  if (!c || !header || !wire || (!in && plan->total)) return fail(CMPI_EINVAL, "null argument");
  Spans602 s;
  if ((rc = spans_602(*plan, first, count, s))) return rc;
  const size_t d_pt = 0, d_w = (s.pt_len + 255) & ~(size_t)255;
  const cmpi_602_plan p = *plan;
  uint8_t hdr[25];
  memcpy(hdr, header, 25);
  // a small message (one segment under the header nonce) has no prefix on the wire: its 5 bytes are
  // not written (as by cmpi_602_seal), so they are not part of the output span either
  const size_t skip = p.mode == '1' && p.total <= k602Pipe ? 5 : 0;
  auto launch = [&](const uint8_t* din, uint8_t* dout, int32_t*, void* ws, hipStream_t st) -> int {
    if (s.segs.empty()) return CMPI_OK;
    return run_602<false>(c, p, hdr, dout - skip, nullptr, nullptr, din, s.segs, nullptr, st, s.pt_off, s.w_off, ws);
  };
  size_t ws = 0;
  if (!s.segs.empty() &&
      (rc = run_602<false>(c, p, hdr, nullptr, nullptr, nullptr, nullptr, s.segs, nullptr, nullptr, 0, 0, nullptr, &ws)))
    return rc;
  return span_begin(c, d_w + s.w_len, {in ? in + s.pt_off : nullptr, d_pt, s.pt_len},
                    {wire + s.w_off + skip, d_w + skip, s.w_len - skip}, nullptr, 0, false, false, nullptr, launch, req,
                    ws);
}

int cmpi_602_seal_host(const cmpi_ctx* c, const cmpi_602_plan* plan, const uint8_t header[25], uint8_t* wire,
                       const uint8_t* in) {
  int rc = check_602(plan);
  if (rc) return rc;
  // requests of k602HostGroup outer messages, all enqueued before the first wait: the pipeline of
  // send.c:754-835 with fewer, larger requests (the caller of the whole message has no MPI_Isend
  // to post between outer messages)
  std::vector<cmpi_req*> reqs;
  for (uint32_t o = 0; o < plan->outer && !rc; o += k602HostGroup) {
    reqs.push_back(nullptr);
    rc = cmpi_602_seal_host_begin(c, plan, header, wire, in, o, std::min(k602HostGroup, plan->outer - o), &reqs.back());
  }
  const int w = cmpi_waitall(reqs.data(), reqs.size());
  return rc ? rc : w;
}

int cmpi_602_open_host_begin(const cmpi_ctx* c, const uint8_t header[25], uint8_t* out, const uint8_t* wire,
                             uint32_t first, uint32_t count, int32_t* status, cmpi_req** req) {
  if (!c || !header || !wire || !out) return fail(CMPI_EINVAL, "null argument");
  cmpi_602_plan p;
  int rc = cmpi_602_plan_from_header(header, &p);
  if (rc) return rc;
  Spans602 s;
  if ((rc = spans_602(p, first, count, s))) return rc;
  const size_t d_w = 0, d_pt = (s.w_len + 255) & ~(size_t)255;
  uint8_t hdr[25];
  memcpy(hdr, header, 25);
  auto launch = [&](const uint8_t* din, uint8_t* dout, int32_t* dst, void* ws, hipStream_t st) -> int {
    if (s.segs.empty()) return CMPI_OK;
    return run_602<true>(c, p, hdr, nullptr, din, dout, nullptr, s.segs, dst, st, s.pt_off, s.w_off, ws);
  };
  size_t ws = 0;
  if (!s.segs.empty() &&
      (rc = run_602<true>(c, p, hdr, nullptr, nullptr, nullptr, nullptr, s.segs, nullptr, nullptr, 0, 0, nullptr, &ws)))
    return rc;
  const size_t first_seg = s.segs.empty() ? 0 : s.segs.front().ctr;
  return span_begin(c, d_pt + s.pt_len, {wire + s.w_off, d_w, s.w_len}, {out + s.pt_off, d_pt, s.pt_len},
                    status ? status + first_seg : nullptr, s.segs.size(), true, false, nullptr, launch, req, ws);
}

int cmpi_602_open_host(const cmpi_ctx* c, const uint8_t header[25], uint8_t* out, const uint8_t* wire,
                       int32_t* status) {
  cmpi_602_plan p;
  int rc = cmpi_602_plan_from_header(header, &p);
  if (rc) return rc;
  std::vector<cmpi_req*> reqs;
  for (uint32_t o = 0; o < p.outer && !rc; o += k602HostGroup) {
    reqs.push_back(nullptr);
    rc = cmpi_602_open_host_begin(c, header, out, wire, o, std::min(k602HostGroup, p.outer - o), status, &reqs.back());
  }
  const int w = cmpi_waitall(reqs.data(), reqs.size());
  return rc ? rc : w;
}

// ---- 700 (send.c:886-1017 / recv.c:812-940) from and to host memory
int cmpi_700_send_host_begin(const cmpi_ctx* c, const uint8_t send_iv[16], uint64_t* counter, const uint8_t* in,
                             size_t n, uint8_t header[26], uint8_t* out, cmpi_req** req) {
  if (!c || !send_iv || !counter || !header) return fail(CMPI_EINVAL, "null argument");
  if (n && (!in || !out)) return fail(CMPI_EINVAL, "null buffer");
  const size_t d_out = (n + 255) & ~(size_t)255;
  auto launch = [&](const uint8_t* din, uint8_t* dout, int32_t*, void*, hipStream_t st) -> int {
    return cmpi_700_send(c, send_iv, counter, din, n, header, dout, st);
  };
  return span_begin(c, d_out + n, {in, 0, n}, {out, d_out, n}, nullptr, 0, false, false, nullptr, launch, req);
}

int cmpi_700_send_host(const cmpi_ctx* c, const uint8_t send_iv[16], uint64_t* counter, const uint8_t* in, size_t n,
                       uint8_t header[26], uint8_t* out) {
  cmpi_req* r = nullptr;
  return sync_req(cmpi_700_send_host_begin(c, send_iv, counter, in, n, header, out, &r), r);
}

int cmpi_700_recv_host_begin(const cmpi_ctx* c, const uint8_t recv_iv[16], const uint8_t header[26], uint8_t* out,
                             size_t out_cap, const uint8_t* in, cmpi_req** req) {
  if (!c || !recv_iv || !header) return fail(CMPI_EINVAL, "null argument");
  const size_t n = be32h(header);
  if (n > out_cap) return fail(CMPI_EINVAL, "header announces %zu bytes, out holds %zu", n, out_cap);
  if (n && (!in || !out)) return fail(CMPI_EINVAL, "null buffer");
  const size_t d_out = (n + 255) & ~(size_t)255;
  auto launch = [&](const uint8_t* din, uint8_t* dout, int32_t*, void*, hipStream_t st) -> int {
    return cmpi_700_recv(c, recv_iv, header, dout, n, din, st);
  };
  return span_begin(c, d_out + n, {in, 0, n}, {out, d_out, n}, nullptr, 0, false, false, nullptr, launch, req);
}

int cmpi_700_recv_host(const cmpi_ctx* c, const uint8_t recv_iv[16], const uint8_t header[26], uint8_t* out,
                       size_t out_cap, const uint8_t* in) {
  cmpi_req* r = nullptr;
  return sync_req(cmpi_700_recv_host_begin(c, recv_iv, header, out, out_cap, in, &r), r);
}

// ---- 702 (send.c:1502-1987 / recv.c:1025-1403) from and to host memory
int cmpi_702_send_host_begin(cmpi_702_sender* s, int pending_isends, const uint8_t* in, size_t n, uint8_t header[26],
                             uint8_t* out, int* segments, cmpi_req** req) {
  if (!s || !header) return fail(CMPI_EINVAL, "null argument");
  if (n && (!in || !out)) return fail(CMPI_EINVAL, "null buffer");
  const size_t d_out = (n + 255) & ~(size_t)255;
  int segs = 0;
  auto launch = [&](const uint8_t* din, uint8_t* dout, int32_t*, void*, hipStream_t st) -> int {
    segs = cmpi_702_send(s, pending_isends, din, n, header, dout, st);
    return segs < 0 ? segs : CMPI_OK;
  };
  const int rc = span_begin(s->ctx, d_out + n, {in, 0, n}, {out, d_out, n}, nullptr, 0, false, false, nullptr, launch, req);
  if (!rc && segments) *segments = segs;
  return rc;
}

int cmpi_702_send_host(cmpi_702_sender* s, int pending_isends, const uint8_t* in, size_t n, uint8_t header[26],
                       uint8_t* out) {
  cmpi_req* r = nullptr;
  int segs = 0;
  const int rc = sync_req(cmpi_702_send_host_begin(s, pending_isends, in, n, header, out, &segs, &r), r);
  return rc ? rc : segs;
}

int cmpi_702_recv_host_begin(const cmpi_ctx* c, const uint8_t recv_iv[32], const uint8_t header[26], uint8_t* out,
                             size_t out_cap, const uint8_t* in, const uint8_t* mask, size_t mask_len,
                             void* mask_stream, cmpi_req** req) {
  if (!c || !recv_iv || !header) return fail(CMPI_EINVAL, "null argument");
  const size_t n = be32h(header);
  if (n > 0x7FFFFFFFu) return fail(CMPI_EINVAL, "malformed header");
  if (n > out_cap) return fail(CMPI_EINVAL, "header announces %zu bytes, out holds %zu", n, out_cap);
  if (n && (!in || !out)) return fail(CMPI_EINVAL, "null buffer");
  const size_t d_out = (n + 255) & ~(size_t)255;
  auto launch = [&](const uint8_t* din, uint8_t* dout, int32_t*, void*, hipStream_t st) -> int {
    return cmpi_702_recv(c, recv_iv, header, dout, n, din, mask, mask_len, st);
  };
  // the mask (device) was made on mask_stream while the payload was in flight: order after it
  return span_begin(c, d_out + n, {in, 0, n}, {out, d_out, n}, nullptr, 0, false, mask != nullptr,
                    (hipStream_t)mask_stream, launch, req);
}

int cmpi_702_recv_host(const cmpi_ctx* c, const uint8_t recv_iv[32], const uint8_t header[26], uint8_t* out,
                       size_t out_cap, const uint8_t* in, const uint8_t* mask, size_t mask_len, void* mask_stream) {
  cmpi_req* r = nullptr;
  return sync_req(cmpi_702_recv_host_begin(c, recv_iv, header, out, out_cap, in, mask, mask_len, mask_stream, &r), r);
}

void cmpi_debug_set_span_direct(size_t bytes) { g_span_direct.store(bytes); }

}  // extern "C"
