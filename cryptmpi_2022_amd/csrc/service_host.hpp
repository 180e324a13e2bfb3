// service_host.hpp — host side of the resident message service (service_kernels.hpp), included by
// cmpi_aead.hip.  Opt-in per context (cmpi_service_start): single GCM messages from host memory
// (cmpi_gcm_seal_host / _open_host with nrec = 1, len <= kSvcMaxLen) are posted to the running
// service kernel instead of launching the direct path's kernel; the host spins on a page-locked
// word the kernel writes.  On CTR contexts the service serves the 702 small-message XORs and
// keystreams (ctrmode_host.hpp: svc_stream), synchronously and outside stream order.  The kernel exits after `idle_us` without messages (the CUs are
// returned) and is relaunched by the next message.  No CPU cipher on any path: a service that
// cannot start fails the call.

#include "../../include/cmpi_service.h"
#include "service_kernels.hpp"

namespace {

constexpr size_t kSvcMaxLen = (size_t)512 << 10;  // 64 chunks of 8 steps
constexpr uint64_t kSvcLifeUs = 100000;           // relaunched at least every 100 ms

// Stream slots of a device's services.  HIP maps the streams of one priority onto at most
// GPU_MAX_HW_QUEUES (4) hardware queues, and a resident kernel holds its queue: with a stream per
// service, the fifth context's service shared a queue with another's resident kernel and waited
// for it to idle out (20 ms at the EVP shim's cap, tools/svc_many_probe.py).  So the services of
// a device share kSvcSlots greatest-priority streams, one resident generation per slot: a
// context whose service launches on a slot held by another's kicks that generation (the kick
// word its leader polls; a posted message is always served first) and queues behind it.
constexpr int kSvcSlots = 4;
constexpr int kSvcMaxDevices = 16;
struct Svc;
struct SvcSlot {
  std::mutex m;
  hipStream_t st = nullptr;
  Svc* owner = nullptr;     // the service whose generation was launched last on this slot
  uint32_t owner_gen = 0;   // that generation (the owner may since have moved to another slot)
};
SvcSlot& svc_slot(int dev, int i) {
  static SvcSlot slots[kSvcMaxDevices][kSvcSlots];
  return slots[dev][i];
}
std::atomic<uint32_t> g_svc_next_slot[kSvcMaxDevices];
std::atomic<int> g_svc_ls_min{0};  // cmpi_debug_set_svc_ls_min (A/B of the service's chunk length)
// cmpi_debug_set_svc_fake_stuck (test): the next shutdowns treat the stop as failed and the
// generation as still resident, exercising the path that leaks the Svc
std::atomic<int> g_svc_fake_stuck{0};

struct Svc {
  hipStream_t st = nullptr;    // the slot's stream (shared; not owned)
  int dev = 0, slot = 0;
  hipEvent_t ev = nullptr;     // recorded after this service's last launch
  bool launched = false;
  uint32_t* hw = nullptr;      // page-locked coherent (kSvcHostBytes): ring [0..15] (four 16-B chunks), kick [16],
                               // exit word [20], completion slots [64 + 8w .. 64 + 8w + 7] of workgroups w < 8
  uint32_t* dw = nullptr;      // its device address
  uint32_t* go = nullptr;      // device control area: published units (at +256)
  cmpi::dev::u32x4* wts = nullptr;  // device chunk weights (4 x 64 x 4 blocks)
  bool wts_ok = false;
  uint8_t* bounce = nullptr;   // page-locked: pageable messages
  size_t bcap = 0;
  uint32_t seq = 0;            // last seq posted
  uint32_t gen = 0;            // generation of the last launch
  bool running = false;
  uint32_t idle_us = 2000;
  uint32_t ls_min = 0;         // the running generation's chunk-plan floor (SvcArgs::ls_min)
  uint32_t* ring() { return hw; }
  uint32_t* kick() { return hw + 16; }
  uint32_t* exited() { return hw + 20; }
  uint32_t* done() { return hw + 64; }
};
constexpr size_t kSvcHostBytes = 1024;

// Workgroups that serve a message of `len` bytes (service_kernels.hpp svc_plan; each posts a
// completion slot): GCM messages by the chunk plan, counter-mode ops by the leader alone.
uint32_t svc_groups(uint32_t op, size_t len, uint32_t ls_min) {
  if (op != cmpi::dev::kSvcSeal && op != cmpi::dev::kSvcOpen) return 1;
  const uint32_t nx = (uint32_t)((len + 15) >> 4);
  uint32_t ls = ls_min;
  while (ls < 3u && nx > cmpi::dev::kSvcMaxChunks * (64u << ls)) ++ls;
  const uint32_t C = 64u << ls, nch = nx ? (nx + C - 1u) / C : 1u;
  return (nch + cmpi::dev::kSvcChunkWaves - 1u) / cmpi::dev::kSvcChunkWaves;
}

// This service's last generation has left the device (its stream slot may already run another
// context's generation behind it).
int svc_drain(Svc& S) {
  if (S.launched) HIP_TRY(hipEventSynchronize(S.ev));
  return CMPI_OK;
}

// Post descriptor d[0..11] under `seq`: chunk c = {seq, d[3c..3c+2]} at ring[4c]; the words first,
// then seq into every chunk (the kernel takes a chunk's words only with the new seq in all four).
void svc_post(Svc& S, const uint32_t (&d)[cmpi::dev::kSvcDesc], uint32_t seq) {
  uint32_t* r = S.ring();
  for (uint32_t c = 0; c < cmpi::dev::kSvcChunks; ++c)
    for (uint32_t j = 0; j < 3; ++j) r[4 * c + 1 + j] = d[3 * c + j];
  for (uint32_t c = 0; c < cmpi::dev::kSvcChunks; ++c) __atomic_store_n(r + 4 * c, seq, __ATOMIC_RELEASE);
}

constexpr size_t kSvcWtsBytes = 4 * 64 * 4 * 16;

// Key-derived and message bytes the service keeps between messages: the chunk weights (powers of
// H), the workgroup partials, the bounce buffer's last message.  Stream drained.
void svc_wipe(Svc& S) {
  wipe_dev(S.wts, kSvcWtsBytes);
  wipe_dev(S.go, cmpi::dev::kSvcGoBytes);
  if (S.hw) memset(S.done(), 0, 4 * 8 * cmpi::dev::kSvcGroups);  // the last message's partials
  if (S.bounce) memset(S.bounce, 0, S.bcap);
  S.wts_ok = false;
  wipe_sync();  // svc_weights' next upload must land after the wipe
}

void svc_release(Svc& S) {
  svc_wipe(S);
  wipe_sync();  // the memsets before the frees
  for (int i = 0; i < kSvcSlots; ++i) {  // every slot that still names this service (it moves between slots)
    SvcSlot& sl = svc_slot(S.dev, i);
    std::lock_guard<std::mutex> g(sl.m);
    if (sl.owner == &S) sl.owner = nullptr;
  }
  if (S.ev) (void)hipEventDestroy(S.ev);
  if (S.hw) (void)hipHostFree(S.hw);
  if (S.go) (void)hipFree(S.go);
  if (S.wts) (void)hipFree(S.wts);
  if (S.bounce) (void)hipHostFree(S.bounce);
  S.hw = nullptr;  // (the Svc is deleted by its caller)
  S.go = nullptr;
  S.wts = nullptr;
  S.bounce = nullptr;
  S.ev = nullptr;
}

// H^(2 + (63-k)·64·2^s) at wts[256s + 4k + 3] (the flow kernel's chunk-weight slot layout; the
// service's chunks cover the data blocks only, the length block is the J0 wave's L·H)
int svc_weights(const cmpi_ctx* c, Svc& S) {
  if (c->alg != CMPI_AES_128_GCM) {  // counter-mode service: no GHASH
    S.wts_ok = true;
    return CMPI_OK;
  }
  std::vector<Blk> w(4 * 64 * 4);
  for (uint32_t s = 0; s < 4; ++s) {
    const Blk P = cmpi::gf_pow(c->H, 64u << s);
    Blk wi = cmpi::gf_mul(c->H, c->H);  // k = 63 down to 0
    for (uint32_t k = 64; k-- > 0;) {
      w[256 * s + 4 * k + 3] = wi;
      wi = cmpi::gf_mul(wi, P);
    }
  }
  HIP_TRY(hipMemcpy(S.wts, w.data(), w.size() * sizeof(Blk), hipMemcpyHostToDevice));
  S.wts_ok = true;
  return CMPI_OK;
}

int svc_launch(const cmpi_ctx* c, Svc& S, uint32_t seq0) {
  if (!S.wts_ok)
    if (int rc = svc_weights(c, S)) return rc;
  int rc = set_lds_attr(reinterpret_cast<const void*>(cmpi::dev::gcm_service_kernel), c->device, cmpi::dev::kFlowLds);
  if (rc) return rc;
  // a slot that is free (no holder, or its holder's generation has exited), starting from this
  // service's last; else this service's own slot, whose holder is kicked
  std::unique_lock<std::mutex> g;
  for (int k = 0; k < kSvcSlots; ++k) {
    const int i = (S.slot + k) % kSvcSlots;
    std::unique_lock<std::mutex> t(svc_slot(S.dev, i).m);
    const SvcSlot& c_sl = svc_slot(S.dev, i);
    Svc* o = c_sl.owner;
    if (!o || o == &S || __atomic_load_n(o->exited(), __ATOMIC_ACQUIRE) == c_sl.owner_gen) {
      S.slot = i;
      g = std::move(t);
      break;
    }
  }
  if (!g.owns_lock()) g = std::unique_lock<std::mutex>(svc_slot(S.dev, S.slot).m);
  SvcSlot& sl = svc_slot(S.dev, S.slot);
  DeviceGuard dg(S.dev);
  if (!sl.st && lib_stream(&sl.st, true) != hipSuccess) return fail(CMPI_EHIP, "service stream creation failed");
  S.st = sl.st;
  if (sl.owner && sl.owner != &S)  // the slot's generation (if still resident) leaves at its next poll
    __atomic_store_n(sl.owner->kick(), sl.owner_gen, __ATOMIC_RELEASE);
  if ((rc = wait_keys(c, S.st))) return rc;  // tables of a re-key still in flight on the caller's stream
  cmpi::dev::SvcArgs a{};
  a.ring = S.dw;
  a.kick = S.dw + 16;
  a.exited = S.dw + 20;
  a.done = S.dw + 64;
  a.go = S.go;
  a.wts = S.wts;
  a.te0 = c->dt->te0;
  a.wtab = c->alg == CMPI_AES_128_GCM ? reinterpret_cast<const cmpi::dev::u32x4*>(c->dt->fnib[0]) : nullptr;
  a.seq0 = seq0;
  a.ls_min = S.ls_min = (uint32_t)g_svc_ls_min.load();
  a.gen = ++S.gen;
  a.idle_ticks = (uint64_t)S.idle_us * 100u;
  a.life_ticks = kSvcLifeUs * 100u;
  a.cap_ticks = (kSvcLifeUs + 100000u) * 100u;
  a.rk = folded(c->rk);
#if CMPI_TOOLS
  a.probe = g_svc_probe.load();
#endif
  void* kargs[] = {&a};
  HIP_TRY(hipLaunchKernel(reinterpret_cast<const void*>(cmpi::dev::gcm_service_kernel), dim3(cmpi::dev::kSvcGroups),
                          dim3(cmpi::dev::kSvcThreads), kargs, cmpi::dev::kFlowLds, S.st));
  HIP_TRY(hipEventRecord(S.ev, S.st));
  sl.owner = &S;
  sl.owner_gen = S.gen;
  S.launched = true;
  S.running = true;
  return CMPI_OK;
}

// The current generation has exited (idle, lifetime, stop): its exit word is written.
bool svc_exited(Svc& S) { return __atomic_load_n(S.exited(), __ATOMIC_ACQUIRE) == S.gen; }

// Completion of message `seq`: the slots of its ngrp workgroups carry it in all four {seq, word}
// pairs (each read as one 8-byte load, so its word belongs to its seq); x = the XOR of their
// partials (a GCM message's tag).
bool svc_done(Svc& S, uint32_t seq, uint32_t ngrp, uint32_t (&x)[4]) {
  const uint64_t* p = reinterpret_cast<const uint64_t*>(S.done());
  uint32_t t[4] = {0, 0, 0, 0};
  for (uint32_t w = 0; w < ngrp; ++w)
    for (int i = 0; i < 4; ++i) {
      const uint64_t v = __atomic_load_n(p + 4 * w + i, __ATOMIC_ACQUIRE);
      if ((uint32_t)v != seq) return false;
      t[i] ^= (uint32_t)(v >> 32);
    }
  memcpy(x, t, sizeof t);
  return true;
}

// Stop a running service and wait until its generation has left (ctx free, re-key,
// cmpi_service_stop).  hmu held.
int svc_stop_locked(Svc& S) {
  if (!S.launched) return CMPI_OK;
  if (S.running && !svc_exited(S)) {
    const uint32_t d[cmpi::dev::kSvcDesc] = {cmpi::dev::kSvcStop};
    svc_post(S, d, ++S.seq);
  }
  if (int rc = svc_drain(S)) return rc;  // the kernel exits at its next poll
  S.running = false;
  return CMPI_OK;
}

// Stop and free the context's service (hmu held).  If the stop failed (its launch event could not
// be waited), the generation may still be resident: its memory is freed only once its exit word
// shows it left (200 ms bound).  Otherwise the whole Svc is left allocated — its
// device words, and the object itself, which a stream slot may still name as its owner: the next
// svc_launch on that slot reads the owner's exit word and writes its kick word, so neither may be
// freed (a leak, never a kernel or a host thread touching freed memory).
int svc_shutdown_locked(cmpi_ctx* c) {
  if (!c->svc) return CMPI_OK;
  Svc& S = *c->svc;
  const bool fake = g_svc_fake_stuck.load() != 0;
  const int rc = fake ? fail(CMPI_EHIP, "message service stop failed (test hook)") : svc_stop_locked(S);
  bool gone = !fake && (!rc || !S.launched || svc_exited(S));
  for (const auto t0 = std::chrono::steady_clock::now();
       !fake && !gone && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(200);)
    gone = svc_exited(S);
  if (gone) {
    svc_release(S);  // clears every slot that names it
    delete c->svc;
  }
  c->svc = nullptr;
  return rc;
}

// Post descriptor d as the next message (the service launched first if it is not running) and
// wait for its workgroups' completion slots; w = the XOR of their partials.  hmu held.
int svc_exec(const cmpi_ctx* c, Svc& S, const uint32_t (&d)[cmpi::dev::kSvcDesc], uint32_t (&w)[4]) {
  if (S.running && svc_exited(S)) {  // idled out (or kicked) since the last message
    if (int rc = svc_drain(S)) return rc;
    S.running = false;
  }
  if (!S.running)
    if (int rc = svc_launch(c, S, S.seq)) return rc;
  const uint32_t seq = ++S.seq;
  svc_post(S, d, seq);
  uint32_t ngrp = svc_groups(d[0], d[1], S.ls_min);
  const auto t0 = std::chrono::steady_clock::now();
  int relaunches = 0;
  for (uint32_t i = 1;; ++i) {
    if (svc_done(S, seq, ngrp, w)) break;
    if (svc_exited(S)) {  // the generation ended (lifetime, kick): let every workgroup finish first
      if (int rc = svc_drain(S)) return rc;
      S.running = false;
      if (svc_done(S, seq, ngrp, w)) break;
      if (++relaunches > 2) return fail(CMPI_EHIP, "message service did not complete message %u", seq);
      if (int rc = svc_launch(c, S, seq - 1)) return rc;  // it never saw the message
      ngrp = svc_groups(d[0], d[1], S.ls_min);  // the new generation's chunk plan
      continue;
    }
    if ((i & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) {
      const hipError_t e = hipEventQuery(S.ev);  // this generation (the slot's stream may hold others)
      if (e != hipSuccess && e != hipErrorNotReady) return fail(CMPI_EHIP, "service kernel: %s", hipGetErrorString(e));
      if (e == hipSuccess && !svc_done(S, seq, ngrp, w) && !svc_exited(S))
        return fail(CMPI_EHIP, "service kernel ended without completing message %u", seq);
    }
  }
  return CMPI_OK;
}

// The page-locked bounce buffer of pageable messages, at least `need` bytes.  hmu held.
int svc_bounce(Svc& S, size_t need) {
  if (S.bcap >= need) return CMPI_OK;
  if (S.bounce) {
    memset(S.bounce, 0, S.bcap);  // its last message
    (void)hipHostFree(S.bounce);
  }
  S.bounce = nullptr;
  S.bcap = 0;
  const size_t cap = std::max<size_t>(need, (size_t)1 << 20);
  if (hipHostMalloc((void**)&S.bounce, cap, hipHostMallocDefault) != hipSuccess)
    return fail(CMPI_ENOMEM, "hipHostMalloc service bounce failed");
  S.bcap = cap;
  return CMPI_OK;
}

// One message through the service.  hmu held; pageable buffers go through the bounce.
template <bool DEC>
int svc_call(const cmpi_ctx* c, Svc& S, uint8_t* out, const uint8_t* in, const uint8_t* nonce, size_t len,
             int32_t* status) {
  const size_t in_rec = len + (DEC ? 16 : 0), out_rec = len + (DEC ? 0 : 16);
  void* din = in_rec ? pinned_dev_ptr(in) : nullptr;
  void* dout = pinned_dev_ptr(out);
  uint8_t* hout = nullptr;
  const size_t bi = (in_rec + 255) & ~(size_t)255, need = bi + out_rec + 256;
  if (!din || !dout)
    if (int rc = svc_bounce(S, need)) return rc;
  if (!din) {
    if (in_rec) memcpy(S.bounce, in, in_rec);
    din = pinned_dev_ptr(S.bounce);
  }
  if (!dout) {
    hout = S.bounce + bi;
    dout = pinned_dev_ptr(hout);
  }
  if (!din || !dout) return fail(CMPI_EHIP, "service buffers have no device address");
  uint32_t d[cmpi::dev::kSvcDesc] = {DEC ? cmpi::dev::kSvcOpen : cmpi::dev::kSvcSeal,
                                     (uint32_t)len,
                                     (uint32_t)(uintptr_t)din,
                                     (uint32_t)((uintptr_t)din >> 32),
                                     (uint32_t)(uintptr_t)dout,
                                     (uint32_t)((uintptr_t)dout >> 32)};
  memcpy(d + 6, nonce, 12);
  uint32_t tag[4];
  if (int rc = svc_exec(c, S, d, tag)) return rc;  // the tag: the XOR of the workgroups' partials
  if (!DEC) {
    if (hout) memcpy(out, hout, len);
    memcpy(out + len, tag, 16);
    return CMPI_OK;
  }
  uint8_t diff = 0;  // the received tag vs the computed one, every byte compared
  for (int i = 0; i < 16; ++i) diff |= in[len + i] ^ reinterpret_cast<const uint8_t*>(tag)[i];
  const int32_t ok = diff == 0 ? 1 : 0;
  if (status) *status = ok;
  if (!ok) {  // a forged message's plaintext is zero-filled (aead.h:276-278)
    memset(out, 0, len);
    return fail(CMPI_EAUTH, "1 of 1 records failed authentication");
  }
  if (hout) memcpy(out, hout, len);
  return CMPI_OK;
}

// One counter-mode op through a CTR context's service (ctrmode_host.hpp, ring_host.hpp): kSvcXor
// out = in ^ mask, kSvcCtr out = in ^ E_K(ctr + j) (in null: the keystream); device (or page-locked)
// buffers, len <= kSvcMaxStreamLen.  Synchronous: the bytes are in `out` when it returns.  hmu held.
int svc_stream(const cmpi_ctx* c, Svc& S, uint32_t op, uint8_t* out, const uint8_t* in, const uint8_t* mask,
               const uint8_t ctr[16], size_t len, unsigned skip = 0) {
  if (len == 0) return CMPI_OK;
  if (len + skip > cmpi::dev::kSvcMaxStreamLen) return fail(CMPI_EINVAL, "served counter-mode op over 64 KiB");
  const uint64_t pi = (uint64_t)(uintptr_t)in, po = (uint64_t)(uintptr_t)out;
  uint32_t d[cmpi::dev::kSvcDesc] = {op, (uint32_t)len, (uint32_t)pi, (uint32_t)(pi >> 32), (uint32_t)po,
                                     (uint32_t)(po >> 32)};
  if (op == cmpi::dev::kSvcXor) {
    const uint64_t pm = (uint64_t)(uintptr_t)mask;
    d[6] = (uint32_t)pm;
    d[7] = (uint32_t)(pm >> 32);
  } else if (op == cmpi::dev::kSvcCtr) {
    const uint64_t h = cmpi::be64(ctr), l = cmpi::be64(ctr + 8);
    d[6] = skip;  // keystream bytes skipped before the message's first byte (0..15)
    d[8] = (uint32_t)h;
    d[9] = (uint32_t)(h >> 32);
    d[10] = (uint32_t)l;
    d[11] = (uint32_t)(l >> 32);
  }
  uint32_t w[4];
  return svc_exec(c, S, d, w);
}

// cmpi_ctr_xor_host (op kSvcCtr) / cmpi_ecb_encrypt_host (kSvcEcb, cb unused) through the context's
// service: page-locked buffers in place, pageable ones through the service's bounce buffer.  hmu
// held.
int svc_ctr_host(const cmpi_ctx* c, Svc& S, uint8_t* out, const uint8_t* in, size_t n, const uint8_t cb[16],
                 unsigned skip, uint32_t op = cmpi::dev::kSvcCtr) {
  void* din = pinned_dev_ptr(in);
  void* dout = pinned_dev_ptr(out);
  uint8_t* hout = nullptr;
  const size_t bi = (n + 255) & ~(size_t)255;
  if (!din || !dout)
    if (int rc = svc_bounce(S, bi + n + 256)) return rc;
  if (!din) {
    memcpy(S.bounce, in, n);
    din = pinned_dev_ptr(S.bounce);
  }
  if (!dout) {
    hout = S.bounce + bi;
    dout = pinned_dev_ptr(hout);
  }
  if (!din || !dout) return fail(CMPI_EHIP, "service buffers have no device address");
  const int rc = svc_stream(c, S, op, static_cast<uint8_t*>(dout), static_cast<const uint8_t*>(din), nullptr, cb, n,
                            skip);
  if (!rc && hout) memcpy(out, hout, n);
  return rc;
}

}  // namespace

extern "C" {

int cmpi_service_start(cmpi_ctx* c, uint32_t idle_us) {
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  if (c->alg != CMPI_AES_128_GCM && c->alg != CMPI_AES_128_CTR && c->alg != CMPI_AES_128_ECB)
    return fail(CMPI_EINVAL, "the message service serves AES-128-GCM, -CTR and -ECB contexts");
  if (c->dev_keys) return fail(CMPI_EINVAL, "the message service needs a host-keyed context");
  DeviceGuard dg(c->device);
  std::lock_guard<std::mutex> lk(c->hmu);
  if (c->device < 0 || c->device >= kSvcMaxDevices) return fail(CMPI_EINVAL, "device index beyond the service slots");
  if (!c->svc) c->svc = new Svc();
  Svc& S = *c->svc;
  S.idle_us = idle_us ? std::min<uint32_t>(idle_us, 1000000u) : 2000u;
  if (S.hw) return CMPI_OK;
  S.dev = c->device;
  S.slot = (int)(g_svc_next_slot[c->device].fetch_add(1) % kSvcSlots);
  if (hipEventCreateWithFlags(&S.ev, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc((void**)&S.hw, kSvcHostBytes, hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&S.dw, S.hw, 0) != hipSuccess || hipMalloc((void**)&S.go, cmpi::dev::kSvcGoBytes) != hipSuccess ||
      hipMalloc((void**)&S.wts, kSvcWtsBytes) != hipSuccess || hipMemset(S.go, 0, cmpi::dev::kSvcGoBytes) != hipSuccess) {
    svc_release(S);
    delete c->svc;
    c->svc = nullptr;
    return fail(CMPI_EHIP, "message service allocation failed");
  }
  memset(S.hw, 0, kSvcHostBytes);
  return CMPI_OK;
}

int cmpi_service_stop(cmpi_ctx* c) {
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  DeviceGuard dg(c->device);
  std::lock_guard<std::mutex> lk(c->hmu);
  if (!c->svc) return CMPI_OK;
  return svc_shutdown_locked(c);
}

int cmpi_service_running(const cmpi_ctx* c) {
  if (!c) return 0;
  std::lock_guard<std::mutex> lk(c->hmu);
  return c->svc && c->svc->running && !svc_exited(*c->svc) ? 1 : 0;
}

}  // extern "C"
