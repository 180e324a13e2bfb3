// ring_host.hpp — include/cmpi_ring.h: the CTR mask ring of send.c:1162-1465 with the ring in
// HBM.  Included at the end of cmpi_aead.hip (one translation unit; uses ctr_launch).
// The bookkeeping below follows the reference statement by statement (oracle/ctr_ring_ref.c
// is the CPU restatement the tests compare against); every byte moved is moved by a kernel.
#pragma once
#include "../../include/cmpi_ring.h"

struct cmpi_ctr_ring {
  const cmpi_ctx* ctx = nullptr;
  uint8_t iv[16];
  uint8_t* dring = nullptr;  // device ring
  int max = 0, start = 0, end = 0, compute_size = 0;
  unsigned long counter = 0, counter_needto_send = 0;
  std::mutex mu;
  // every ring operation is ordered after the previous one (a fill on one stream, the XOR that
  // consumes it on another): the event is recorded on the last operation's stream when an
  // operation on another stream needs it (or at the ring's free), not after every operation —
  // that record cost ~0.7 us of host time and ~1.6 us of stream time per 702 message.  The
  // stream of the ring's last operation must therefore stay valid until the ring's next operation
  // on another stream or its free (cmpi_ring.h).
  hipEvent_t last = nullptr;
  hipStream_t last_stream = nullptr;
  bool used = false;
  bool pending = false;  // the last operation is not yet captured by `last`
};

namespace {

int xor_launch(uint8_t* out, const uint8_t* a, const uint8_t* b, size_t n, hipStream_t st) {
  if (n == 0) return CMPI_OK;
  const uint64_t nv = n / 16;
  const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((nv + 255) / 256, 4096));
  HIP_TRY(launch_k(cmpi::dev::xor_bytes_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, out, a, b, (uint64_t)n));
  return CMPI_OK;
}

// keystream (in == nullptr) or in ^ keystream of the counters starting at IV_Count(iv, counter)
int ring_ctr(const cmpi_ctr_ring* r, unsigned long counter, uint8_t* out, const uint8_t* in, size_t n, void* stream) {
  uint8_t cb[16];
  memcpy(cb, r->iv, 16);
  cmpi_iv_count(cb, counter);
  return ctr_launch(r->ctx, out, in, n, cb, stream);
}

// Served counter-mode ops (service_host.hpp): when the context runs a message service
// (cmpi_service_start on the CTR context), the ring XORs and keystreams of messages up to
// kSvcMaxStreamLen bytes run on it — one ring post and a completion word instead of a launch and
// a stream wait.  A served op runs now, not in stream order: begin() waits for the work already
// queued on the caller's stream (the input's producer), and the ring's last operation is drained
// before a served ring op (ring_drain).  Holds hmu (after r->mu where a ring is involved).
struct Served {
  const cmpi_ctx* c;
  std::unique_lock<std::mutex> lk;
  Svc* S = nullptr;
  Served(const cmpi_ctx* c_, size_t n) : c(c_), lk(c_->hmu) {
    if (c->svc && n <= cmpi::dev::kSvcMaxStreamLen) S = c->svc;
    else lk.unlock();
  }
  explicit operator bool() const { return S != nullptr; }
  int begin(void* stream) {
    const hipError_t e = hipStreamQuery((hipStream_t)stream);
    if (e == hipSuccess) return CMPI_OK;
    if (e != hipErrorNotReady) return fail(CMPI_EHIP, "stream: %s", hipGetErrorString(e));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return CMPI_OK;
  }
  int xor_(uint8_t* out, const uint8_t* mask, const uint8_t* in, size_t n) {
    return svc_stream(c, *S, cmpi::dev::kSvcXor, out, in, mask, nullptr, n);
  }
  int ctr(uint8_t* out, const uint8_t* in, size_t n, const uint8_t cb[16]) {
    return svc_stream(c, *S, cmpi::dev::kSvcCtr, out, in, nullptr, cb, n);
  }
};

// Ring operations chain on r->last (called with r->mu held): the launch stream waits for the
// previous operation when it ran on another stream, and records the new last use after.
// Constructed in place and never copied (a copied temporary's destructor marked the
// new stream as the ring's last one before begin() ran, so the cross-stream wait was skipped);
// the ring's last use moves to `st` only once begin() has ordered the stream.
struct RingOrder {
  cmpi_ctr_ring* r;
  hipStream_t st;
  bool armed = false;
  RingOrder(cmpi_ctr_ring* r_, hipStream_t st_) : r(r_), st(st_) {}
  RingOrder(const RingOrder&) = delete;
  RingOrder& operator=(const RingOrder&) = delete;
  int begin() {
    if (r->used && r->last_stream != st) {
      if (r->pending) {
        HIP_TRY(hipEventRecord(r->last, r->last_stream));
        r->pending = false;
      }
      HIP_TRY(hipStreamWaitEvent(st, r->last, 0));
    }
    armed = true;
    return CMPI_OK;
  }
  ~RingOrder() {
    if (!armed) return;
    r->used = true;
    r->last_stream = st;
    r->pending = true;
  }
};

// Before a served ring op: the ring's last stream operation is complete (then nothing is left to
// order after: the served op completes before the call returns).
int ring_drain(cmpi_ctr_ring* r) {
  if (!r->used) return CMPI_OK;
  if (r->pending) {
    HIP_TRY(hipStreamSynchronize(r->last_stream));
  } else {
    HIP_TRY(hipEventSynchronize(r->last));
  }
  r->used = false;
  r->pending = false;
  return CMPI_OK;
}

}  // namespace

extern "C" {

cmpi_ctr_ring* cmpi_ctr_ring_new(const cmpi_ctx* ctx, const uint8_t iv[16], size_t ring_bytes) {
  if (!ctx || !iv) {
    fail(CMPI_EINVAL, "null argument");
    return nullptr;
  }
  if (ctx->dev_keys) {
    fail(CMPI_EINVAL, "device-derived sub-key context supports GCM only");
    return nullptr;
  }
  if (ring_bytes < 2048 || ring_bytes % 16 || ring_bytes > 0x40000000u) {
    fail(CMPI_EINVAL, "ring_bytes must be a multiple of 16 in [2048, 1 GiB]");
    return nullptr;
  }
  DeviceGuard dg(ctx->device);
  auto* r = new cmpi_ctr_ring();
  r->ctx = ctx;
  memcpy(r->iv, iv, 16);
  r->max = (int)ring_bytes;
  if (hipMalloc(&r->dring, ring_bytes) != hipSuccess) {
    fail(CMPI_ENOMEM, "hipMalloc ring failed");
    delete r;
    return nullptr;
  }
  if (hipEventCreateWithFlags(&r->last, kOrderEvent) != hipSuccess) {
    fail(CMPI_EHIP, "hipEventCreate failed");
    (void)hipFree(r->dring);
    delete r;
    return nullptr;
  }
  return r;
}

void cmpi_ctr_ring_free(cmpi_ctr_ring* r) {
  if (!r) return;
  DeviceGuard dg(r->ctx->device);
  if (r->used) {  // the ring's last fill / consumption
    bool drained = false;
    if (r->pending) {
      // if the record fails (the last op's stream is gone), the ring must still not be
      // freed under its last use — drain the device instead (free is rare; no error is left behind
      // unless the caller already had one pending)
      const hipError_t prior = hipPeekAtLastError();
      if (hipEventRecord(r->last, r->last_stream) != hipSuccess) {
        if (prior == hipSuccess) (void)hipGetLastError();
        (void)hipDeviceSynchronize();
        drained = true;
      }
    }
    if (!drained) (void)hipEventSynchronize(r->last);
  }
  if (r->last) (void)hipEventDestroy(r->last);
  if (r->dring) (void)hipFree(r->dring);
  delete r;
}

int cmpi_ctr_ring_state(const cmpi_ctr_ring* r, uint64_t st[5]) {
  if (!r || !st) return fail(CMPI_EINVAL, "null argument");
  st[0] = (uint64_t)r->start;
  st[1] = (uint64_t)r->end;
  st[2] = (uint64_t)r->compute_size;
  st[3] = r->counter;
  st[4] = r->counter_needto_send;
  return CMPI_OK;
}

// send.c:1162-1266
int cmpi_ctr_ring_generate(cmpi_ctr_ring* r, size_t gen_bytes, void* stream) {
  if (!r) return fail(CMPI_EINVAL, "null ring");
  // gen_bytes 0 is legal: like the reference it still makes one 16-byte block (send.c:1170);
  // more than the ring holds is refused by the head-room guard below (returns 0), as there
  if (gen_bytes > 0x7FFFFFFFu) return fail(CMPI_EINVAL, "gen_bytes out of range");
  std::lock_guard<std::mutex> lk(r->mu);
  DeviceGuard dg(r->ctx->device);
  const int gen = (int)gen_bytes;
  if (!(r->compute_size <= (r->max - gen - 1024))) return 0;
  RingOrder ord(r, (hipStream_t)stream);
  if (int e = ord.begin()) return e;
  int blockamount = ((gen - 1) / 16) * 16 + 16;
  int rc;
  auto fill = [&](int amount) {
    int e = ring_ctr(r, r->counter, r->dring + r->end, nullptr, (size_t)amount, stream);
    r->compute_size += amount;
    r->end += amount;
    r->counter += (unsigned long)(amount / 16);
    return e;
  };
  if (r->end > r->start && r->end + blockamount <= r->max) {
    rc = fill(blockamount);
  } else if ((r->end > r->start && r->end + blockamount > r->max) || (r->end == r->start && r->compute_size == 0)) {
    const int tempamount = r->max - r->end;
    if (blockamount > tempamount) {
      if (tempamount && (rc = fill(tempamount))) return rc;
      blockamount -= tempamount;
      r->end = 0;
    }
    rc = fill(blockamount);
  } else if (r->end < r->start && blockamount + r->end < r->start) {
    rc = fill(blockamount);
  } else {  // the reference prints ___ERROR___ in generation and exits (send.c:1253-1262)
    return fail(CMPI_EINVAL, "mask ring state inconsistent (start %d end %d size %d)", r->start, r->end,
                r->compute_size);
  }
  return rc ? rc : 1;
}

}  // extern "C"

namespace {
// send.c:1273-1465, with r->mu held by the caller (cmpi_ctr_ring_encrypt, and cmpi_702_send, whose
// stream choice and header counter must see the same ring state as the XOR that follows).
// sv: the XORs and the keystream tail run on the context's message service (Served, begun).
int ring_encrypt_locked(cmpi_ctr_ring* r, uint8_t* out, const uint8_t* in, size_t n, void* stream,
                        Served* sv = nullptr) {
  // n == 0 is not a no-op: like the reference, it retires one 16-byte ring block
  // (((0 - 1) / 16) * 16 + 16 == 16, send.c:1331-1335).
  if (n && (!out || !in)) return fail(CMPI_EINVAL, "null buffer");
  if (n > 0x7FFFFFFFu) return fail(CMPI_EINVAL, "message larger than INT_MAX");
  DeviceGuard dg(r->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  std::optional<RingOrder> ord;
  if (sv) {
    if (int e = ring_drain(r)) return e;
  } else {
    ord.emplace(r, st);
    if (int e = ord->begin()) return e;
  }
  auto xor_op = [&](uint8_t* o, const uint8_t* m, const uint8_t* i, size_t len) {
    return sv ? sv->xor_(o, m, i, len) : xor_launch(o, m, i, len, st);
  };
  const int enc_datasize = (int)n;
  int how_much_generate, temporary_datasize, datasize;
  if (enc_datasize > r->compute_size) {
    how_much_generate = enc_datasize - r->compute_size;
    datasize = temporary_datasize = r->compute_size;
  } else {
    how_much_generate = 0;
    temporary_datasize = datasize = enc_datasize;
  }
  int rc;
  if (r->compute_size > 0) {
    if (r->end > r->start) {
      const int tempamount = (r->start + datasize <= r->end) ? datasize : r->end - r->start;
      if ((rc = xor_op(out, r->dring + r->start, in, (size_t)tempamount))) return rc;
      r->start += ((tempamount - 1) / 16) * 16 + 16;
      if (r->start >= r->max) r->start = 0;
      r->compute_size -= ((tempamount - 1) / 16) * 16 + 16;
      r->counter_needto_send += (unsigned long)(((tempamount - 1) / 16) + 1);
    } else if (r->end < r->start) {
      const int tempamount = r->max - r->start;
      int tempnext = 0;
      if (datasize > tempamount) {
        if (tempamount) {
          if ((rc = xor_op(out, r->dring + r->start, in, (size_t)tempamount))) return rc;
          tempnext = tempamount;
        }
        r->start = 0;
        datasize -= tempamount;
      }
      if ((rc = xor_op(out + tempnext, r->dring + r->start, in + tempnext, (size_t)datasize))) return rc;
      if (datasize > 0) r->start += ((datasize - 1) / 16) * 16 + 16;
      if (r->start >= r->max) r->start = 0;
      r->compute_size -= ((temporary_datasize - 1) / 16) * 16 + 16;
      r->counter_needto_send += (unsigned long)(((temporary_datasize - 1) / 16) + 1);
    }
  }
  if (how_much_generate) {
    if (sv) {
      uint8_t cb[16];
      memcpy(cb, r->iv, 16);
      cmpi_iv_count(cb, r->counter);
      rc = sv->ctr(out + temporary_datasize, in + temporary_datasize, (size_t)how_much_generate, cb);
    } else {
      rc = ring_ctr(r, r->counter, out + temporary_datasize, in + temporary_datasize, (size_t)how_much_generate, stream);
    }
    if (rc) return rc;
    r->counter += (unsigned long)((how_much_generate - 1) / 16 + 1);
    r->counter_needto_send += (unsigned long)(((how_much_generate - 1) / 16) + 1);
  }
  return CMPI_OK;
}
}  // namespace

extern "C" {

int cmpi_ctr_ring_encrypt(cmpi_ctr_ring* r, uint8_t* out, const uint8_t* in, size_t n, void* stream) {
  if (!r) return fail(CMPI_EINVAL, "null ring");
  std::lock_guard<std::mutex> lk(r->mu);
  Served sv(r->ctx, n);
  if (sv)
    if (int e = sv.begin(stream)) return e;
  return ring_encrypt_locked(r, out, in, n, stream, sv ? &sv : nullptr);
}

// recv.c:954-1023
int cmpi_ctr_mask_decrypt(const cmpi_ctx* ctx, uint8_t* out, const uint8_t* in, size_t n, const uint8_t* mask,
                          size_t mask_len, const uint8_t iv[16], uint64_t counter, void* stream) {
  if (!ctx || !iv) return fail(CMPI_EINVAL, "null argument");
  if (n == 0) return CMPI_OK;
  if (!out || !in || (!mask && mask_len)) return fail(CMPI_EINVAL, "null buffer");
  DeviceGuard dg(ctx->device);
  const size_t len = std::min(n, mask_len);
  Served sv(ctx, n);
  if (sv)
    if (int e = sv.begin(stream)) return e;
  int rc = sv ? sv.xor_(out, mask, in, len) : xor_launch(out, mask, in, len, (hipStream_t)stream);
  if (rc || n == len) return rc;
  uint8_t cb[16];
  memcpy(cb, iv, 16);
  cmpi_iv_count(cb, (unsigned long)counter);
  return sv ? sv.ctr(out + len, in + len, n - len, cb) : ctr_launch(ctx, out + len, in + len, n - len, cb, stream);
}

int cmpi_xor_bytes(uint8_t* out, const uint8_t* a, const uint8_t* b, size_t n, void* stream) {
  if (n && (!out || !a || !b)) return fail(CMPI_EINVAL, "null buffer");
  return xor_launch(out, a, b, n, (hipStream_t)stream);
}

}  // extern "C"
