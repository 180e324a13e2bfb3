// cmpi_evp_shim.cpp — libcmpi_evp.so: BoringSSL-ABI drop-in (include/cmpi_evp.h) forwarding
// CryptMPI's EVP calls to the MI355X engine (include/cmpi_aead.h).  This is the literal boundary
// CryptMPI's libmpi links against; three things make it more than one GPU round
// trip per call:
//  * Context pool.  EVP_AEAD_CTX_new with a key the pool already holds shares that engine
//    context; a new key re-keys an idle pooled context on the device (cmpi_ctx_rekey: key
//    schedule + tables in one key-setup kernel) instead of allocating and uploading ~450 KB.
//    CryptMPI creates `my_thread_no` contexts of one sub-key per 602 message (send.c:588-599,
//    recv.c:562-575).  CMPI_EVP_CTX_CACHE = idle contexts kept (default 16, 0 = none).
//  * Call coalescing.  An OpenMP team sealing on one shared context (send.c:292, :646, :754)
//    calls EVP_AEAD_CTX_seal from every thread at once.  Concurrent calls on one engine context
//    are combined: the first caller becomes the leader and runs every request pending at that
//    moment as ONE batch launch per record length (packed through pinned staging); callers that
//    arrive meanwhile form the next batch.  After a multi-caller batch the leader waits up to
//    CMPI_EVP_COALESCE_US (default 30) for as many callers as last time.
//  * Foreign ciphers.  EVP_EncryptInit_ex with an EVP_CIPHER this library did not issue (e.g.
//    libcrypto's EVP_aes_256_ecb() at init.c:848 when SYMMETRIC_KEY_SIZE is 32) is forwarded to
//    the next libcrypto in the link order (dlsym RTLD_NEXT) on a real EVP_CIPHER_CTX the shim
//    keeps inside its own; without one the call fails (returns 0) instead of misreading it.
#include <sys/random.h>
#include <dlfcn.h>
#include <link.h>
#include <unistd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <list>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/cmpi_aead.h"
#include "../../include/cmpi_evp.h"
#include "../../include/cmpi_service.h"

struct evp_aead_st {
  int id;
};
struct evp_cipher_st {
  int alg;
};

namespace {

// ---------------------------------------------------------------- pooled, coalescing contexts
struct Req {
  uint8_t* out;
  const uint8_t* nonce;
  const uint8_t* in;
  size_t len;  // plaintext bytes
  int ok = 0;
  bool done = false;
};

struct Combiner {
  std::mutex m;
  std::condition_variable done, arrive;
  std::vector<Req*> pending;
  bool busy = false;
  size_t last = 2;  // callers in the previous batch (2: the first batch opens a gathering window)
};

using Key = std::array<uint8_t, 16>;

struct Shared {
  cmpi_ctx* c = nullptr;
  Key key{};
  int refs = 0;
  Combiner seal, open;
  std::mutex stage_mu;  // pinned staging of coalesced batches (used by one leader at a time)
  uint8_t* stage = nullptr;
  size_t stage_cap = 0;
  std::vector<int32_t> status;
};

size_t env_size(const char* name, size_t dflt) {
  const char* s = getenv(name);
  return (s && *s) ? (size_t)strtoull(s, nullptr, 10) : dflt;
}
const size_t kIdleCap = env_size("CMPI_EVP_CTX_CACHE", 16);
const long kWindowUs = (long)env_size("CMPI_EVP_COALESCE_US", 30);
// CMPI_EVP_SERVICE_US = n > 0 (default 2000): every context serves its single messages from the
// resident message service (include/cmpi_service.h), which returns its CUs after n us without
// messages — the AEAD contexts' seal / open and the CTR / ECB cipher contexts' EVP_EncryptUpdate of
// up to 64 KiB (the 700 / 702 per-message calls, the 602 sub-key derivation).  0: one kernel launch
// per EVP call.  On by default since round 6: a launch per call costs a 64 KiB seal + open 57.6 us
// against 24 served, more than one CPU core's 25; while idle the kernel holds
// 8 CUs for at most n us (capped at 20 ms) and then leaves.
const size_t kServiceUs = env_size("CMPI_EVP_SERVICE_US", 2000);
// idle limit of the drop-in's services: a resident kernel delays device-wide synchronisation
// (hipDeviceSynchronize) of the whole process until it idles out (cmpi_service.h)
constexpr size_t kServiceCapUs = 20000;

int pick_device() {
  const char* vars[] = {"CMPI_DEVICE", "MV2_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK",
                        "LOCAL_RANK"};
  int n = cmpi_device_count();
  if (n <= 0) return 0;
  for (const char* v : vars) {
    const char* s = getenv(v);
    if (s && *s) return atoi(s) % n;
  }
  return 0;
}

// Live contexts are shared by key (CryptMPI's OpenMP team seals on one global context); a freed
// context keeps no key material: its key is wiped and the engine context re-keyed to a random key
// (device schedule and tables overwritten) before it joins the idle list, from which the next
// EVP_AEAD_CTX_new re-keys it (BoringSSL wipes key material on free).
struct Pool {
  std::mutex m;
  std::map<Key, Shared*> by_key;  // live contexts (refs > 0)
  std::list<Shared*> idle;        // refs == 0, scrubbed, oldest first
};
Pool& pool() {
  static Pool* p = new Pool();  // never destroyed: contexts may be freed from atexit handlers
  return *p;
}

void destroy(Shared* s) {
  cmpi_ctx_free(s->c);  // wipes the engine's host copy of the key
  if (s->stage) {
    (void)cmpi_host_unregister(s->stage);
    free(s->stage);
  }
  explicit_bzero(s->key.data(), s->key.size());
  delete s;
}

// Idle context: no key material left behind (host key wiped, device schedule re-keyed at random).
bool scrub(Shared* s) {
  explicit_bzero(s->key.data(), s->key.size());
  uint8_t rnd[16];
  size_t got = 0;
  while (got < sizeof rnd) {
    const ssize_t r = getrandom(rnd + got, sizeof rnd - got, 0);
    if (r <= 0) return false;
    got += (size_t)r;
  }
  const bool ok = cmpi_ctx_rekey(s->c, rnd, 16, nullptr) == CMPI_OK;
  explicit_bzero(rnd, sizeof rnd);
  return ok;
}

// A live context with this key is shared; otherwise the oldest idle context is re-keyed on the
// device (or a new one made) with the pool lock released, and published under the lock — if
// another thread published the same key meanwhile, that one is shared and ours is destroyed.
Shared* acquire(const uint8_t* key) {
  Key k;
  memcpy(k.data(), key, 16);
  Pool& P = pool();
  Shared* s = nullptr;
  {
    std::lock_guard<std::mutex> lk(P.m);
    auto it = P.by_key.find(k);
    if (it != P.by_key.end()) {  // same key as a live context: share it
      Shared* live = it->second;
      ++live->refs;
      explicit_bzero(k.data(), k.size());
      return live;
    }
    if (!P.idle.empty()) {
      s = P.idle.front();
      P.idle.pop_front();
    }
  }
  if (s && cmpi_ctx_rekey(s->c, key, 16, nullptr) != CMPI_OK) {
    destroy(s);
    s = nullptr;
  }
  if (!s) {
    cmpi_ctx* c = cmpi_ctx_new(CMPI_AES_128_GCM, key, 16, 0, pick_device());
    if (!c) {
      explicit_bzero(k.data(), k.size());
      return nullptr;
    }
    s = new Shared();
    s->c = c;
    if (kServiceUs && cmpi_service_start(c, (uint32_t)std::min<size_t>(kServiceUs, kServiceCapUs)) != CMPI_OK) {
      destroy(s);
      explicit_bzero(k.data(), k.size());
      return nullptr;
    }
  }
  Shared* other = nullptr;
  {
    std::lock_guard<std::mutex> lk(P.m);
    auto it = P.by_key.find(k);
    if (it != P.by_key.end()) {
      other = it->second;
      ++other->refs;
    } else {
      s->key = k;
      s->refs = 1;
      P.by_key[k] = s;
    }
  }
  explicit_bzero(k.data(), k.size());
  if (other) {
    destroy(s);
    return other;
  }
  return s;
}

// The last reference: the context leaves by_key under the pool lock, is scrubbed (a device re-key
// that drains the context's own streams) with the lock released — EVP_AEAD_CTX_new / _free on
// other OpenMP threads do not wait behind it — and joins the idle list under the lock
// again.  Contexts beyond the idle cap are destroyed outside the lock as well.
void release(Shared* s) {
  Pool& P = pool();
  {
    std::lock_guard<std::mutex> lk(P.m);
    if (--s->refs > 0) return;
    P.by_key.erase(s->key);
  }
  if (kIdleCap == 0 || !scrub(s)) {
    destroy(s);
    return;
  }
  std::vector<Shared*> evict;
  {
    std::lock_guard<std::mutex> lk(P.m);
    P.idle.push_back(s);
    while (P.idle.size() > kIdleCap) {
      evict.push_back(P.idle.front());
      P.idle.pop_front();
    }
  }
  for (Shared* o : evict) destroy(o);
}

// ---------------------------------------------------------------- static message buffers
// CryptMPI seals into and opens from its own static arrays (large_send_buffer / large_recv_buffer,
// mpiimpl.h:292-293, 64 MiB each in libmpi's .bss; send.c:311, recv.c:322).  Page-locked, the
// engine's kernels read and write them in place over PCIe; pageable, every byte goes through the
// service's bounce buffer (a memcpy each way).  Static storage of an object loaded at program start
// is never unmapped, so the shim page-locks such a segment, whole and once, the first time a
// message touches it — the registration can never outlive the memory (what makes a general
// pin-down cache of user buffers unsafe without allocator hooks: freed and re-mapped pages).
// CMPI_EVP_REGISTER_STATIC = 0 turns it off; segments above CMPI_EVP_REGISTER_STATIC_MAX bytes
// (default 1 GiB) are left pageable.
struct StaticSeg {
  uintptr_t lo, hi;  // whole pages inside one writable PT_LOAD segment
  std::once_flag once;
  bool ok = false;
};
struct StaticSegs {
  std::vector<StaticSeg*> v;
};
// (function-local statics: the snapshot below runs from a constructor, which may run before this
// translation unit's namespace-scope initialisers)
size_t reg_static_on() {
  static const size_t v = env_size("CMPI_EVP_REGISTER_STATIC", 1);
  return v;
}
size_t reg_static_max() {
  static const size_t v = env_size("CMPI_EVP_REGISTER_STATIC_MAX", (size_t)1 << 30);
  return v;
}

int collect_seg(struct dl_phdr_info* info, size_t, void* arg) {
  auto* segs = static_cast<StaticSegs*>(arg);
  const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
  uintptr_t relro_end = 0;  // the start of a writable segment turns read-only after relocation
  for (int i = 0; i < info->dlpi_phnum; ++i)
    if (info->dlpi_phdr[i].p_type == PT_GNU_RELRO)
      relro_end = info->dlpi_addr + info->dlpi_phdr[i].p_vaddr + info->dlpi_phdr[i].p_memsz;
  for (int i = 0; i < info->dlpi_phnum; ++i) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[i];
    if (ph.p_type != PT_LOAD || !(ph.p_flags & PF_W)) continue;
    uintptr_t a = info->dlpi_addr + ph.p_vaddr;
    const uintptr_t b = a + ph.p_memsz;
    if (relro_end > a && relro_end < b) a = relro_end;
    // whole writable pages only: the first may share a page with the RELRO (read-only) part
    const uintptr_t lo = (a + pg - 1) & ~(pg - 1), hi = (b + pg - 1) & ~(pg - 1);
    if (hi > lo && hi - lo <= reg_static_max()) {
      auto* s = new StaticSeg();
      s->lo = lo;
      s->hi = hi;
      segs->v.push_back(s);
    }
  }
  return 0;
}

// The writable segments of the objects loaded when the shim was (program start for a DT_NEEDED
// libmpi); never freed.
const StaticSegs& static_segs() {
  static const StaticSegs* s = [] {
    auto* x = new StaticSegs();
    if (reg_static_on()) dl_iterate_phdr(collect_seg, x);
    return x;
  }();
  return *s;
}
__attribute__((constructor)) void snapshot_static_segs() { (void)static_segs(); }

// [p, p + n) inside a static segment: page-lock that segment (once; a failure leaves it pageable).
void register_static(const void* p, size_t n) {
  if (!reg_static_on() || !p || n < 4096) return;  // small messages: the bounce copy is cheaper
  const uintptr_t a = (uintptr_t)p, b = a + n;
  for (StaticSeg* s : static_segs().v)
    if (a >= s->lo && b <= s->hi) {
      std::call_once(s->once, [s] {
        s->ok = cmpi_host_register((void*)s->lo, s->hi - s->lo) == CMPI_OK;
        if (getenv("CMPI_EVP_DEBUG"))
          fprintf(stderr, "cmpi_evp: static segment [%#lx, %#lx) %zu bytes page-locked: %s\n", (unsigned long)s->lo,
                  (unsigned long)s->hi, (size_t)(s->hi - s->lo), s->ok ? "yes" : "no");
      });
      return;
    }
}

bool ensure_stage(Shared* s, size_t need) {
  if (need <= s->stage_cap) return true;
  if (s->stage) {
    (void)cmpi_host_unregister(s->stage);
    free(s->stage);
    s->stage = nullptr;
    s->stage_cap = 0;
  }
  size_t cap = std::max(need, (size_t)1 << 20);
  cap = (cap + 4095) & ~(size_t)4095;
  void* p = nullptr;
  if (posix_memalign(&p, 4096, cap)) return false;
  (void)cmpi_host_register(p, cap);  // pinned: DMA at PCIe rate (pageable still works if this fails)
  s->stage = (uint8_t*)p;
  s->stage_cap = cap;
  return true;
}

// One batch of k equal-length requests through the engine's host-memory batch call.
void run_group(Shared* s, Req** r, size_t k, bool open) {
  const size_t n = r[0]->len;
  if (k == 1) {
    int32_t st = 0;
    register_static(r[0]->in, open ? n + 16 : n);
    register_static(r[0]->out, open ? n : n + 16);
    if (!open)
      r[0]->ok = cmpi_gcm_seal_host(s->c, r[0]->out, 0, r[0]->in ? r[0]->in : r[0]->out, 0, r[0]->nonce, 12, n, 1) == CMPI_OK;
    else
      r[0]->ok = cmpi_gcm_open_host(s->c, r[0]->out, 0, r[0]->in, 0, r[0]->nonce, 12, n, 1, &st) == CMPI_OK && st == 1;
    return;
  }
  const size_t in_rec = open ? n + 16 : n, out_rec = open ? n : n + 16;
  std::lock_guard<std::mutex> lk(s->stage_mu);
  if (!ensure_stage(s, k * (12 + in_rec + out_rec) + 64)) {
    for (size_t i = 0; i < k; ++i) r[i]->ok = 0;
    return;
  }
  uint8_t* nn = s->stage;
  uint8_t* in = nn + 12 * k;
  uint8_t* out = in + in_rec * k;
  for (size_t i = 0; i < k; ++i) {
    memcpy(nn + 12 * i, r[i]->nonce, 12);
    if (in_rec) memcpy(in + in_rec * i, r[i]->in, in_rec);
  }
  int rc;
  if (!open) {
    rc = cmpi_gcm_seal_host(s->c, out, out_rec, in, in_rec, nn, 12, n, k);
    for (size_t i = 0; i < k; ++i) {
      r[i]->ok = rc == CMPI_OK;
      if (rc == CMPI_OK) memcpy(r[i]->out, out + out_rec * i, out_rec);
    }
  } else {
    s->status.assign(k, 0);
    rc = cmpi_gcm_open_host(s->c, out, out_rec, in, in_rec, nn, 12, n, k, s->status.data());
    for (size_t i = 0; i < k; ++i) {
      r[i]->ok = (rc == CMPI_OK || rc == CMPI_EAUTH) && s->status[i] == 1;
      if (r[i]->ok && out_rec) memcpy(r[i]->out, out + out_rec * i, out_rec);
    }
  }
}

void run_batch(Shared* s, std::vector<Req*>& b, bool open) {
  std::stable_sort(b.begin(), b.end(), [](const Req* x, const Req* y) { return x->len < y->len; });
  for (size_t i = 0; i < b.size();) {
    size_t j = i + 1;
    while (j < b.size() && b[j]->len == b[i]->len) ++j;
    run_group(s, b.data() + i, j - i, open);
    i = j;
  }
}

int submit(Shared* s, Req& r, bool open) {
  Combiner& cb = open ? s->open : s->seal;
  std::unique_lock<std::mutex> lk(cb.m);
  cb.pending.push_back(&r);
  cb.arrive.notify_one();
  if (cb.busy) {
    cb.done.wait(lk, [&] { return r.done; });
    return r.ok;
  }
  cb.busy = true;
  if (cb.last > 1 && kWindowUs > 0)
    cb.arrive.wait_for(lk, std::chrono::microseconds(kWindowUs), [&] { return cb.pending.size() >= cb.last; });
  while (!cb.pending.empty()) {
    std::vector<Req*> batch;
    batch.swap(cb.pending);
    lk.unlock();
    run_batch(s, batch, open);
    lk.lock();
    for (Req* q : batch) q->done = true;
    cb.last = batch.size();
    cb.done.notify_all();
  }
  cb.busy = false;
  return r.ok;
}

// ---------------------------------------------------------------- CTR / ECB (+ forwarding)
const evp_aead_st kGcm{1};
const evp_cipher_st kCtr{CMPI_AES_128_CTR};
const evp_cipher_st kEcb{CMPI_AES_128_ECB};

struct Real {  // the next libcrypto in the link order, for ciphers the engine does not serve
  void* (*ctx_new)();
  void (*ctx_free)(void*);
  int (*enc_init)(void*, const void*, void*, const uint8_t*, const uint8_t*);
  int (*dec_init)(void*, const void*, void*, const uint8_t*, const uint8_t*);
  int (*enc_update)(void*, uint8_t*, int*, const uint8_t*, int);
  int (*dec_update)(void*, uint8_t*, int*, const uint8_t*, int);
  bool ok;
};
const Real& real() {
  static const Real r = [] {
    Real x{};
    x.ctx_new = (void* (*)())dlsym(RTLD_NEXT, "EVP_CIPHER_CTX_new");
    x.ctx_free = (void (*)(void*))dlsym(RTLD_NEXT, "EVP_CIPHER_CTX_free");
    x.enc_init = (int (*)(void*, const void*, void*, const uint8_t*, const uint8_t*))dlsym(RTLD_NEXT, "EVP_EncryptInit_ex");
    x.dec_init = (int (*)(void*, const void*, void*, const uint8_t*, const uint8_t*))dlsym(RTLD_NEXT, "EVP_DecryptInit_ex");
    x.enc_update = (int (*)(void*, uint8_t*, int*, const uint8_t*, int))dlsym(RTLD_NEXT, "EVP_EncryptUpdate");
    x.dec_update = (int (*)(void*, uint8_t*, int*, const uint8_t*, int))dlsym(RTLD_NEXT, "EVP_DecryptUpdate");
    x.ok = x.ctx_new && x.ctx_free && x.enc_init && x.dec_init && x.enc_update && x.dec_update;
    return x;
  }();
  return r;
}

bool ours(const EVP_CIPHER* c) { return c == &kCtr || c == &kEcb; }

void add128(uint8_t cb[16], uint64_t k) {
  unsigned carry = 0;
  for (int i = 15; i >= 0; --i) {
    unsigned s = (unsigned)cb[i] + (unsigned)(k & 0xff) + carry;
    cb[i] = (uint8_t)s;
    carry = s >> 8;
    k >>= 8;
  }
}

}  // namespace

struct evp_aead_ctx_st {
  Shared* s;
};
struct evp_cipher_ctx_st {
  int alg = 0;             // CMPI_AES_128_CTR / _ECB, -1 = forwarded to libcrypto, 0 = unset
  cmpi_ctx* c = nullptr;
  void* fwd = nullptr;     // libcrypto EVP_CIPHER_CTX of a forwarded cipher
  uint8_t iv[16] = {0};    // counter block at the start of the current stream
  uint64_t pos = 0;        // CTR bytes consumed since the last IV (EVP keeps `num` state)
  uint8_t partial[16];     // ECB: buffered bytes of an incomplete block
  int npartial = 0;
};

namespace {

int cipher_init(EVP_CIPHER_CTX* ctx, const EVP_CIPHER* cipher, ENGINE* engine, const uint8_t* key,
                const uint8_t* iv, bool dec) {
  if (!ctx) return 0;
  if ((cipher && !ours(cipher)) || (!cipher && ctx->alg == -1)) {  // forwarded cipher
    const Real& R = real();
    if (!R.ok) return 0;
    if (ctx->c) {
      cmpi_ctx_free(ctx->c);
      ctx->c = nullptr;
    }
    if (!ctx->fwd && !(ctx->fwd = R.ctx_new())) return 0;
    ctx->alg = -1;
    return (dec ? R.dec_init : R.enc_init)(ctx->fwd, cipher, engine, key, iv);
  }
  if (cipher) {
    if (dec && cipher->alg == CMPI_AES_128_ECB) return 0;  // ECB decryption: never used by CryptMPI
    if (ctx->fwd) {
      real().ctx_free(ctx->fwd);
      ctx->fwd = nullptr;
    }
    if (ctx->c && ctx->alg != cipher->alg) {
      cmpi_ctx_free(ctx->c);
      ctx->c = nullptr;
    }
    ctx->alg = cipher->alg;
  }
  if (ctx->alg <= 0) return 0;
  if (dec && ctx->alg == CMPI_AES_128_ECB) return 0;
  if (key) {
    if (ctx->c) {
      if (cmpi_ctx_rekey(ctx->c, key, 16, nullptr) != CMPI_OK) return 0;
    } else if (!(ctx->c = cmpi_ctx_new(ctx->alg, key, 16, 0, pick_device()))) {
      return 0;
    } else if (kServiceUs && (ctx->alg == CMPI_AES_128_CTR || ctx->alg == CMPI_AES_128_ECB) &&
               cmpi_service_start(ctx->c, (uint32_t)std::min<size_t>(kServiceUs, kServiceCapUs)) != CMPI_OK) {
      cmpi_ctx_free(ctx->c);
      ctx->c = nullptr;
      return 0;
    }
  }
  if (iv) memcpy(ctx->iv, iv, 16);
  if (iv || key) {
    ctx->pos = 0;
    ctx->npartial = 0;
  }
  return 1;
}

int cipher_update(EVP_CIPHER_CTX* ctx, uint8_t* out, int* out_len, const uint8_t* in, int in_len, bool dec) {
  if (!ctx || in_len < 0 || !out_len) return 0;
  if (ctx->alg == -1) return (dec ? real().dec_update : real().enc_update)(ctx->fwd, out, out_len, in, in_len);
  if (!ctx->c) return 0;
  *out_len = 0;
  if (in_len == 0) return 1;
  if (ctx->alg == CMPI_AES_128_CTR) {
    uint8_t cb[16];
    memcpy(cb, ctx->iv, 16);
    add128(cb, ctx->pos / 16);
    if (cmpi_ctr_xor_host(ctx->c, out, in, (size_t)in_len, cb, (unsigned)(ctx->pos % 16)) != CMPI_OK) return 0;
    ctx->pos += (uint64_t)in_len;
    *out_len = in_len;
    return 1;
  }
  if (dec) return 0;
  // ECB, no padding on Update: emit whole blocks, keep the remainder
  int total = ctx->npartial + in_len;
  int full = total / 16 * 16;
  if (full == 0) {
    memcpy(ctx->partial + ctx->npartial, in, (size_t)in_len);
    ctx->npartial = total;
    return 1;
  }
  std::vector<uint8_t> buf((size_t)full);
  memcpy(buf.data(), ctx->partial, (size_t)ctx->npartial);
  memcpy(buf.data() + ctx->npartial, in, (size_t)(full - ctx->npartial));
  int rest = total - full;
  uint8_t tail[16];
  memcpy(tail, in + (in_len - rest), (size_t)rest);
  if (cmpi_ecb_encrypt_host(ctx->c, out, buf.data(), (size_t)full / 16) != CMPI_OK) return 0;
  memcpy(ctx->partial, tail, (size_t)rest);
  ctx->npartial = rest;
  *out_len = full;
  return 1;
}

}  // namespace

extern "C" {

const EVP_AEAD* EVP_aead_aes_128_gcm(void) { return &kGcm; }
size_t EVP_AEAD_nonce_length(const EVP_AEAD*) { return 12; }
size_t EVP_AEAD_max_overhead(const EVP_AEAD*) { return 16; }

EVP_AEAD_CTX* EVP_AEAD_CTX_new(const EVP_AEAD* aead, const uint8_t* key, size_t key_len, size_t tag_len) {
  if (aead != &kGcm || !key || key_len != 16 || !(tag_len == 0 || tag_len == 16)) return nullptr;
  Shared* s = acquire(key);
  if (!s) return nullptr;
  return new evp_aead_ctx_st{s};
}

void EVP_AEAD_CTX_free(EVP_AEAD_CTX* ctx) {
  if (!ctx) return;
  release(ctx->s);
  delete ctx;
}

int EVP_AEAD_CTX_seal(const EVP_AEAD_CTX* ctx, uint8_t* out, size_t* out_len, size_t max_out_len,
                      const uint8_t* nonce, size_t nonce_len, const uint8_t* in, size_t in_len,
                      const uint8_t* ad, size_t ad_len) {
  (void)ad;
  if (ctx && out && out_len && nonce && nonce_len == 12 && ad_len == 0 && max_out_len >= in_len + 16 &&
      (in || in_len == 0)) {
    Req r{out, nonce, in, in_len};
    if (submit(ctx->s, r, false)) {
      *out_len = in_len + 16;
      return 1;
    }
  }
  if (out) memset(out, 0, max_out_len);  // aead.h:251-253
  if (out_len) *out_len = 0;
  return 0;
}

int EVP_AEAD_CTX_open(const EVP_AEAD_CTX* ctx, uint8_t* out, size_t* out_len, size_t max_out_len,
                      const uint8_t* nonce, size_t nonce_len, const uint8_t* in, size_t in_len,
                      const uint8_t* ad, size_t ad_len) {
  (void)ad;
  if (ctx && out && out_len && nonce && in && nonce_len == 12 && ad_len == 0 && in_len >= 16 &&
      max_out_len >= in_len - 16) {
    Req r{out, nonce, in, in_len - 16};
    if (submit(ctx->s, r, true)) {
      *out_len = in_len - 16;
      return 1;
    }
  }
  if (out) memset(out, 0, max_out_len);  // aead.h:276-278
  if (out_len) *out_len = 0;
  return 0;
}

const EVP_CIPHER* EVP_aes_128_ecb(void) { return &kEcb; }
const EVP_CIPHER* EVP_aes_128_ctr(void) { return &kCtr; }

EVP_CIPHER_CTX* EVP_CIPHER_CTX_new(void) { return new evp_cipher_ctx_st; }

void EVP_CIPHER_CTX_free(EVP_CIPHER_CTX* ctx) {
  if (!ctx) return;
  if (ctx->c) cmpi_ctx_free(ctx->c);
  if (ctx->fwd) real().ctx_free(ctx->fwd);
  delete ctx;
}

int EVP_EncryptInit_ex(EVP_CIPHER_CTX* ctx, const EVP_CIPHER* cipher, ENGINE* engine, const uint8_t* key,
                       const uint8_t* iv) {
  return cipher_init(ctx, cipher, engine, key, iv, false);
}

int EVP_DecryptInit_ex(EVP_CIPHER_CTX* ctx, const EVP_CIPHER* cipher, ENGINE* engine, const uint8_t* key,
                       const uint8_t* iv) {
  return cipher_init(ctx, cipher, engine, key, iv, true);
}

int EVP_EncryptUpdate(EVP_CIPHER_CTX* ctx, uint8_t* out, int* out_len, const uint8_t* in, int in_len) {
  return cipher_update(ctx, out, out_len, in, in_len, false);
}

int EVP_DecryptUpdate(EVP_CIPHER_CTX* ctx, uint8_t* out, int* out_len, const uint8_t* in, int in_len) {
  return cipher_update(ctx, out, out_len, in, in_len, true);
}

}  // extern "C"
