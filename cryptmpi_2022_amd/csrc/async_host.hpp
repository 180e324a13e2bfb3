// async_host.hpp — include/cmpi_async.h: asynchronous host-memory batches for CryptMPI's
// non-blocking pair.  MPI_Isend encrypts eagerly and returns; MPI_Wait / MPI_Waitall decrypt
// (MV/src/mpi/pt2pt/isend.c:187-1260, wait.c:244-1780, waitall.c:438-2389), with up to 64
// requests outstanding in nonblock_req_handler[] (isend.c:310-321).  Here *_begin enqueues
// H2D -> kernel -> D2H on a pooled stream and returns a request; cmpi_test / cmpi_wait complete
// it.  Included at the end of cmpi_aead.hip (one translation unit: gcm_batch, ocb_batch,
// is_pinned, par_copy_records).
//
// Staging (device buffers and pinned host bounce buffers) comes from per-device free lists and
// goes back at completion, so a steady stream of requests allocates nothing.  Pinned user
// buffers move by DMA straight to / from the device; pageable inputs are packed into pinned
// staging inside *_begin (the caller may reuse its buffer as soon as begin returns, MPI_Isend's
// contract is stricter), pageable outputs are unpacked at completion.
#pragma once
#include "../../include/cmpi_async.h"

namespace {

struct StagePool {
  std::mutex mu;
  std::multimap<size_t, void*> dev_free, host_free;
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> events;  // completion events of finished requests, reused
  size_t next = 0;
};
StagePool& stage_pool(int device) {
  static std::mutex m;
  static std::map<int, StagePool*> pools;
  std::lock_guard<std::mutex> lk(m);
  auto& p = pools[device];
  if (!p) p = new StagePool();  // process lifetime
  return *p;
}
size_t size_class(size_t b) {
  size_t c = (size_t)2 << 20;
  while (c < b) c <<= 1;
  return c;
}
int pool_take(StagePool& P, bool host, size_t need, void** out, size_t* cap) {
  const size_t c = size_class(need);
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto& fl = host ? P.host_free : P.dev_free;
    auto it = fl.lower_bound(c);
    if (it != fl.end() && it->first <= 4 * c) {
      *out = it->second;
      *cap = it->first;
      fl.erase(it);
      return CMPI_OK;
    }
  }
  if (host) {
    if (hipHostMalloc(out, c, hipHostMallocDefault) != hipSuccess) return fail(CMPI_ENOMEM, "hipHostMalloc(%zu) failed", c);
  } else if (hipMalloc(out, c) != hipSuccess) {
    return fail(CMPI_ENOMEM, "hipMalloc(%zu) failed", c);
  }
  *cap = c;
  return CMPI_OK;
}
void pool_give(StagePool& P, bool host, void* p, size_t cap) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(P.mu);
  (host ? P.host_free : P.dev_free).emplace(cap, p);
}
constexpr size_t kAsyncStreams = 8;
int pool_stream(StagePool& P, hipStream_t* st) {
  std::lock_guard<std::mutex> lk(P.mu);
  if (P.streams.empty()) {
    for (size_t i = 0; i < kAsyncStreams; ++i) {
      hipStream_t s;
      HIP_TRY(lib_stream(&s));
      P.streams.push_back(s);
    }
  }
  *st = P.streams[P.next++ % P.streams.size()];
  return CMPI_OK;
}

}  // namespace

struct cmpi_req {
  int device = 0;
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  void* dbuf = nullptr;
  size_t dcap = 0;
  void* hbuf = nullptr;  // pinned: packed inputs / outputs to unpack / statuses
  size_t hcap = 0;
  bool dec = false, unpack = false;
  uint8_t* user_out = nullptr;
  size_t out_stride = 0, out_rec = 0, op = 0, nrec = 0;
  uint8_t* h_out = nullptr;
  int32_t* h_status = nullptr;
  int32_t* user_status = nullptr;
  size_t nst = 0;  // statuses to report (open): nrec for record batches, segments for framed messages
  // framed requests (framed_host.hpp): pageable output spans copied from pinned staging at completion
  std::vector<std::pair<uint8_t*, const uint8_t*>> span_dst;
  std::vector<size_t> span_len;
  int error = CMPI_OK;
};

namespace {

void req_release(cmpi_req* r) {
  StagePool& P = stage_pool(r->device);
  pool_give(P, false, r->dbuf, r->dcap);
  pool_give(P, true, r->hbuf, r->hcap);
  if (r->done) {
    std::lock_guard<std::mutex> lk(P.mu);
    P.events.push_back(r->done);
  }
  delete r;
}

// Small requests (<= g_host_direct bytes in + out, cmpi_aead.hip): the kernel reads and writes
// page-locked user buffers itself, pageable ones go through the request's pinned buffer, nonces
// and statuses live there too; device memory only for the kernel workspace.  No DMA launches.
template <bool DEC, bool OCB, class Bail>
int direct_begin(const cmpi_ctx* c, StagePool& P, cmpi_req* r, uint8_t* out, size_t out_stride, const uint8_t* in,
                 size_t in_stride, const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, cmpi_req** req,
                 Bail& bail) {
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t in_rec = len + (DEC ? 16 : 0), out_rec = len + (DEC ? 0 : 16);
  void* din = in_rec ? pinned_dev_ptr(in) : nullptr;
  void* dout = out_rec ? pinned_dev_ptr(out) : nullptr;
  size_t ws = 0;
  if (OCB) {
    const OcbPlan pl = plan_ocb(c, len, nrec);
    ws = (size_t)nrec * pl.nchunks * 16 + nrec * 16 + nrec * 4;
  } else {
    ws = gcm_ws_bytes(c, plan_gcm(c, len, nrec), nrec);
  }
  int rc;
  if (ws && (rc = pool_take(P, false, up16(ws) + 16, &r->dbuf, &r->dcap))) return bail(rc);
  const size_t bi = !din ? up16(in_rec * nrec) : 0, bo = !dout ? up16(out_rec * nrec) : 0;
  const size_t h_in = 0, h_out = bi, h_n = bi + bo, h_st = h_n + up16(16 * nrec), h_total = h_st + up16(4 * nrec) + 16;
  if ((rc = pool_take(P, true, h_total, &r->hbuf, &r->hcap))) return bail(rc);
  uint8_t* H = (uint8_t*)r->hbuf;
  uint8_t* dH = (uint8_t*)pinned_dev_ptr(H);
  if (!dH) return bail(fail(CMPI_EHIP, "staging buffer has no device address"));
  size_t istr = in_stride, ostr = out_stride;
  if (!din) {
    if (in_rec) par_copy_records(H + h_in, in_rec, in, in_stride, in_rec, nrec);
    din = dH + h_in;
    istr = std::max<size_t>(in_rec, 1);
  }
  const bool unpack = !dout && out_rec;
  if (!dout) {
    dout = dH + h_out;
    ostr = std::max<size_t>(out_rec, 1);
  }
  for (size_t i = 0; i < nrec; ++i) memcpy(H + h_n + 16 * i, nonces + i * nonce_stride, 12);
  int32_t* dst = DEC ? (int32_t*)(dH + h_st) : nullptr;
  void* wsp = ws ? r->dbuf : nullptr;
  rc = OCB ? ocb_batch<DEC>(c, (uint8_t*)dout, ostr, (const uint8_t*)din, istr, dH + h_n, 16, len, nrec, dst, wsp, r->st)
           : gcm_batch<DEC>(c, (uint8_t*)dout, ostr, (const uint8_t*)din, istr, dH + h_n, 16, len, nrec, dst, wsp, r->st);
  if (rc) return bail(rc);
  HIP_TRY(hipEventRecord(r->done, r->st));
  r->unpack = unpack;
  r->user_out = out;
  r->out_stride = out_stride;
  r->out_rec = out_rec;
  r->op = ostr;
  r->h_out = H + h_out;
  r->h_status = (int32_t*)(H + h_st);
  *req = r;
  return CMPI_OK;
}

template <bool DEC, bool OCB>
int host_begin(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
               const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status, cmpi_req** req) {
  if (!req) return fail(CMPI_EINVAL, "null request");
  *req = nullptr;
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  if (OCB ? c->alg != CMPI_AES_128_OCB : c->alg != CMPI_AES_128_GCM) return fail(CMPI_EINVAL, "ctx algorithm mismatch");
  if (nrec && (!out || !in || !nonces)) return fail(CMPI_EINVAL, "null buffer");
  const size_t in_rec = len + (DEC ? 16 : 0), out_rec = len + (DEC ? 0 : 16);
  if (nrec > 1 && (in_stride < in_rec || out_stride < out_rec || nonce_stride < 12))
    return fail(CMPI_EINVAL, "stride smaller than record");
  if (nrec == 1) in_stride = in_rec, out_stride = out_rec, nonce_stride = 12;
  DeviceGuard dg(c->device);
  StagePool& P = stage_pool(c->device);
  auto* r = new cmpi_req();
  r->device = c->device;
  r->dec = DEC;
  r->nrec = nrec;
  r->nst = DEC ? nrec : 0;
  r->user_status = status;
  auto bail = [&](int rc) {
    if (r->st && r->done) (void)hipStreamSynchronize(r->st);
    req_release(r);
    return rc;
  };
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
  if ((rc = wait_keys(c, r->st))) return bail(rc);
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  if (nrec && nrec * (in_rec + out_rec) <= g_host_direct.load())
    return direct_begin<DEC, OCB>(c, P, r, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, req, bail);
  const bool in_pinned = in_rec && is_pinned(in), out_pinned = out_rec && is_pinned(out);
  const bool in_flat = in_pinned && (nrec == 1 || in_stride <= in_rec + 64);
  const bool out_flat = out_pinned && (nrec == 1 || out_stride == out_rec);
  const size_t ip = in_flat ? in_stride : up16(in_rec), op = out_flat ? out_stride : up16(out_rec);
  size_t ws = 0;
  if (nrec) {
    if (OCB) {
      const OcbPlan pl = plan_ocb(c, len, nrec);
      ws = (size_t)nrec * pl.nchunks * 16 + nrec * 16 + nrec * 4;
    } else {
      ws = gcm_ws_bytes(c, plan_gcm(c, len, nrec), nrec);
    }
  }
  // device layout: in | out | nonces | status | workspace (16-B aligned regions)
  const size_t d_in = 0, d_out = up16(ip * nrec), d_n = d_out + up16(op * nrec), d_st = d_n + up16(16 * nrec),
               d_ws = d_st + up16(4 * nrec), d_total = d_ws + up16(ws) + 16;
  if ((rc = pool_take(P, false, d_total, &r->dbuf, &r->dcap))) return bail(rc);
  uint8_t* D = (uint8_t*)r->dbuf;
  // host (pinned) layout: packed inputs | outputs to unpack | nonces | statuses
  const bool pack_in = in_rec && !in_flat, unpack = out_rec && !out_flat;
  const size_t h_in = 0, h_out = pack_in ? up16(ip * nrec) : 0, h_n = h_out + (unpack ? up16(op * nrec) : 0),
               h_st = h_n + up16(16 * nrec), h_total = h_st + up16(4 * nrec) + 16;
  if ((rc = pool_take(P, true, h_total, &r->hbuf, &r->hcap))) return bail(rc);
  uint8_t* H = (uint8_t*)r->hbuf;
  hipStream_t st = r->st;
  if (nrec) {
    if (pack_in) {
      par_copy_records(H + h_in, ip, in, in_stride, in_rec, nrec);
      HIP_TRY(hipMemcpyAsync(D + d_in, H + h_in, ip * nrec, hipMemcpyHostToDevice, st));
    } else if (in_rec) {
      HIP_TRY(hipMemcpyAsync(D + d_in, in, (nrec - 1) * ip + in_rec, hipMemcpyHostToDevice, st));
    }
    int32_t* dst = DEC ? (int32_t*)(D + d_st) : nullptr;
    void* wsp = ws ? (void*)(D + d_ws) : nullptr;
    if (!OCB && nrec == 1) {  // one message (an MPI_Isend): the nonce travels in the kernel arguments
      NonceSpec ns;
      ns.mode = 3;
      memcpy(ns.fix, nonces, 12);
      rc = gcm_batch<DEC>(c, D + d_out, op, D + d_in, ip, nullptr, 12, len, 1, dst, wsp, st, ns);
    } else {
      for (size_t i = 0; i < nrec; ++i) memcpy(H + h_n + 16 * i, nonces + i * nonce_stride, 12);
      HIP_TRY(hipMemcpyAsync(D + d_n, H + h_n, 16 * nrec, hipMemcpyHostToDevice, st));
      rc = OCB ? ocb_batch<DEC>(c, D + d_out, op, D + d_in, ip, D + d_n, 16, len, nrec, dst, wsp, st)
               : gcm_batch<DEC>(c, D + d_out, op, D + d_in, ip, D + d_n, 16, len, nrec, dst, wsp, st);
    }
    if (rc) return bail(rc);
    if (out_rec) {
      if (unpack)
        HIP_TRY(hipMemcpyAsync(H + h_out, D + d_out, op * nrec, hipMemcpyDeviceToHost, st));
      else
        HIP_TRY(hipMemcpyAsync(out, D + d_out, (nrec - 1) * op + out_rec, hipMemcpyDeviceToHost, st));
    }
    if (DEC) HIP_TRY(hipMemcpyAsync(H + h_st, D + d_st, 4 * nrec, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipEventRecord(r->done, st));
  r->unpack = unpack;
  r->user_out = out;
  r->out_stride = out_stride;
  r->out_rec = out_rec;
  r->op = op;
  r->h_out = H + h_out;
  r->h_status = (int32_t*)(H + h_st);
  *req = r;
  return CMPI_OK;
}

// the request's work is done on the device: unpack, statuses, release
int req_finish(cmpi_req* r) {
  DeviceGuard dg(r->device);
  int rc = r->error;
  if (!rc && r->unpack && r->nrec) par_copy_records(r->user_out, r->out_stride, r->h_out, r->op, r->out_rec, r->nrec);
  for (size_t i = 0; !rc && i < r->span_dst.size(); ++i)
    par_copy_records(r->span_dst[i].first, r->span_len[i], r->span_dst[i].second, r->span_len[i], r->span_len[i], 1);
  if (!rc && r->dec && r->nst) {
    size_t bad = 0;
    for (size_t i = 0; i < r->nst; ++i) bad += r->h_status[i] != 1;
    if (r->user_status) memcpy(r->user_status, r->h_status, 4 * r->nst);
    if (bad) rc = fail(CMPI_EAUTH, "%zu of %zu records failed authentication", bad, r->nst);
  }
  req_release(r);
  return rc;
}

}  // namespace

extern "C" {

int cmpi_gcm_seal_host_begin(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                             const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, cmpi_req** req) {
  return host_begin<false, false>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, nullptr, req);
}
int cmpi_gcm_open_host_begin(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                             const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status,
                             cmpi_req** req) {
  return host_begin<true, false>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, status, req);
}
int cmpi_ocb_seal_host_begin(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                             const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, cmpi_req** req) {
  return host_begin<false, true>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, nullptr, req);
}
int cmpi_ocb_open_host_begin(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                             const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status,
                             cmpi_req** req) {
  return host_begin<true, true>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, status, req);
}

int cmpi_test(cmpi_req* r, int* done) {
  if (!r || !done) return fail(CMPI_EINVAL, "null argument");
  *done = 0;
  DeviceGuard dg(r->device);
  const hipError_t e = hipEventQuery(r->done);
  if (e == hipErrorNotReady) return CMPI_OK;
  if (e != hipSuccess) r->error = fail(CMPI_EHIP, "request failed: %s", hipGetErrorString(e));
  *done = 1;
  return req_finish(r);
}

int cmpi_wait(cmpi_req* r) {
  if (!r) return fail(CMPI_EINVAL, "null request");
  {
    DeviceGuard dg(r->device);
    const hipError_t e = hipEventSynchronize(r->done);
    if (e != hipSuccess) r->error = fail(CMPI_EHIP, "request failed: %s", hipGetErrorString(e));
  }
  return req_finish(r);
}

int cmpi_waitall(cmpi_req** reqs, size_t n) {
  if (n && !reqs) return fail(CMPI_EINVAL, "null request array");
  int first = CMPI_OK;
  for (size_t i = 0; i < n; ++i) {
    if (!reqs[i]) continue;
    const int rc = cmpi_wait(reqs[i]);
    reqs[i] = nullptr;
    if (rc && !first) first = rc;
  }
  return first;
}

}  // extern "C"
