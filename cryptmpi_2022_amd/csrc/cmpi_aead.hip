// cmpi_aead.hip — libcmpi_aead.so: the C ABI of include/cmpi_aead.h (host side) + kernel
// instantiations.  One translation unit so every kernel lives in one code object for gfx950.
//
// Host responsibilities: key schedule and GHASH/OCB tables once per key (what
// EVP_AEAD_CTX_new does inside BoringSSL), launch planning (lanes per record, segmentation),
// argument validation, and the staging path of the *_host entry points.  No cipher arithmetic
// runs on the host on any data path: every byte of ciphertext, plaintext or tag is produced by
// a HIP kernel.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <array>
#include <map>
#include <memory>
#include <optional>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <type_traits>
#include <vector>

#include <sys/random.h>
#include <cstdlib>

#include "../../include/cmpi_aead.h"
#include "../../include/cmpi_coll.h"
#include "../../include/cmpi_debug.h"
#include "../../include/cmpi_ring.h"
#include "aes_tables.hpp"
#include "ctr_kernels.hpp"
#include "gcm_kernels.hpp"
#include "gf128_host.hpp"
#include "keysetup_kernels.hpp"
#include "ocb_kernels.hpp"
#include "hsa_copy.hpp"

using cmpi::Blk;
using cmpi::dev::u32x4;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) return fail(CMPI_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// Kernel launch that reports its own status: hipGetLastError() after a triple-chevron
// or hipLaunchKernelGGL launch returns the thread's last error from ANY earlier HIP call — the
// caller's included — and clears it, so an unrelated earlier failure would fail the seal (and the
// EVP shim put zeros on the wire) while the caller lost its own error.  hipLaunchKernel returns
// the launch's status and leaves a pending error of the caller's alone.
// Kernel timing for bench.py's roofline (cmpi_debug_time_next_launch): the kernels this thread
// launches go through hipExtLaunchKernel — the first with the start event, every one with the stop
// event (a two-launch call, flow kernel + combine, is timed from the first kernel's start to the
// last one's end) — until the hook is cleared.  These events time the kernels themselves rather
// than the stream between two event records (a record bracket also holds the dependent launch's
// dispatch gap after the previous kernel).
thread_local hipEvent_t t_time_start = nullptr, t_time_stop = nullptr;

hipError_t launch_raw(const void* fn, dim3 grid, dim3 block, void** args, size_t lds, hipStream_t st) {
  if (t_time_start || t_time_stop) {
    const hipEvent_t e0 = t_time_start;
    t_time_start = nullptr;
    return hipExtLaunchKernel(fn, grid, block, args, lds, st, e0, t_time_stop, 0);
  }
  return hipLaunchKernel(fn, grid, block, args, lds, st);
}

template <class... P, class... A>
hipError_t launch_k(void (*fn)(P...), dim3 grid, dim3 block, size_t lds, hipStream_t st, A&&... a) {
  static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
  std::tuple<std::decay_t<P>...> t(std::forward<A>(a)...);
  return std::apply(
      [&](auto&... x) {
        void* args[] = {static_cast<void*>(&x)...};
        return launch_raw(reinterpret_cast<const void*>(fn), grid, block, args, lds, st);
      },
      t);
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

constexpr uint32_t kGcmThreads = 1024;
constexpr size_t kByteTab = 4096 * 16;
constexpr size_t kNibTab = 512 * 16;

// Device table block of a context (one allocation).
struct DevTables {
  uint32_t te0[256];
  uint32_t td0[256];
  uint32_t isb[256];
  uint32_t keys[256];            // [0..43] round keys, [48..51] H (device-keyed contexts read these)
  uint8_t htab[3][kByteTab];     // byte tables for H^1, H^2, H^4 (lane groups' Horner multipliers)
  uint8_t ltab[66][16];          // OCB: L_*, L_$, L_0..L_63
  // device-keyed (602 sub-key) contexts: written by gcm_keysetup_kernel / gcm_tables_kernel
  uint8_t sqmat[31][128][16];    // columns of X -> X^(2^i), i = 1..31 (key independent, host)
  uint8_t h2pow[32][16];         // H^(2^i)
  uint8_t chains[10][128][16];   // basis chains of H, H^2, H^3, H^4, H^8, H^16, H^32, H^64, H^12, H^48
  // nibble tables of H^1,2,3,4,8,12,16,32,48,64: gcm_flow_kernel (all ten), lane-group weights
  // H^1..H^3 (the first three)
  uint8_t fnib[10][kNibTab];
};

// Columns of the squaring maps X -> X^(2^i) (key setup of device-derived keys), once per process.
const std::vector<Blk>& sq_columns() {
  static const std::vector<Blk> v = [] {
    std::vector<Blk> m(31 * 128);
    cmpi::build_sq_columns(m.data());
    return m;
  }();
  return v;
}

}  // namespace

// Host-path pipeline state of a context (aead_host): three streams, g_host_slots staging slots.
struct HostPipe {
  hipStream_t s[3] = {nullptr, nullptr, nullptr};  // H2D, kernel, D2H
  hipEvent_t in_ready[4], k_done[4], slot_free[4];  // per staging slot (g_host_slots <= 4 in use)
  uint8_t* buf = nullptr;   // device staging, 2 slots
  uint8_t* hbuf = nullptr;  // pinned host staging, 2 slots (pageable user buffers)
  uint8_t* dnon = nullptr;  // device: the whole batch's nonces, one H2D per call (page-locked nonces)
  size_t dnon_cap = 0;
  size_t cap = 0;           // bytes per slot
  size_t ns = 0;            // slots allocated
  int32_t* hst = nullptr;   // pinned per-record open status of the whole batch
  size_t hst_cap = 0;
  uint8_t* dbounce = nullptr;  // pinned: direct path's packed pageable records, nonces, statuses
  size_t dcap = 0;
  uint32_t* hflag = nullptr;  // pinned coherent word: the direct path's completion sequence number
  uint32_t* dflag = nullptr;  // its device address
  uint32_t seq = 0;
  hsa_signal_t dsig[4] = {};  // output modes 4-5: completion of each slot's SDMA D2H (value 0 = done)
  hsa_signal_t hsig[4] = {};  // output mode 5: completion of each slot's SDMA H2D (records + nonces)
  bool dsig_init = false;
  bool init = false;
};

namespace {
struct Svc;  // resident message service (service_host.hpp)
}

struct cmpi_ctx {
  int alg = 0;
  int device = 0;
  int ncu = 256;
  uint8_t key[16];
  std::atomic<bool> dev_keys{false};  // key, rk, drk and H exist only on the device (derived 602 sub-key)
  uint32_t nprefix = 0;              // fresh nonces (cmpi_gcm_seal_batch_fresh): 4 random bytes
  std::atomic<uint64_t> nctr{0};     // and a 64-bit counter that starts at a random value
  cmpi::dev::RoundKeys rk{};
  cmpi::dev::RoundKeys drk{};
  Blk H{};
  DevTables* dt = nullptr;  // device
  // per-G combine multipliers H^{G·2^j}, j < 7 (host-keyed contexts; passed by value)
  mutable std::mutex mu;
  mutable std::map<uint32_t, std::array<Blk, 7>> mj;
  // wide-plan chunk weights H^(1 + (nch-1-i)·C) in HBM, per (C, nch) (host-keyed contexts)
  mutable std::map<std::pair<uint32_t, uint32_t>, void*> chw;
  // internal scratch (partials, status) of device-resident calls that pass no workspace, and
  // the event of its last user: the next user's stream waits on it, so NULL-workspace calls on
  // one ctx from different streams are ordered (the host pipeline has scratch of its own)
  mutable void* scratch = nullptr;
  mutable size_t scratch_cap = 0;
  mutable hipEvent_t scratch_ev = nullptr;
  mutable bool scratch_used = false;

  mutable std::mutex smu;  // scratch lease (held through the launches of one call)
  mutable uint8_t* stage = nullptr;
  mutable size_t stage_cap = 0;
  mutable hipStream_t hstream = nullptr;
  mutable std::mutex hmu;                 // host-path pipeline (aead_host)
  std::unique_ptr<HostPipe> pipe{new HostPipe()};
  // the last device re-key (cmpi_ctx_rekey / _rekey_subkey) on the caller's stream: the library's
  // own streams (host paths, async requests) order their launches after it (wait_keys)
  mutable hipEvent_t key_ev = nullptr;
  mutable std::atomic<bool> key_pending{false};
  Svc* svc = nullptr;  // cmpi_service_start (guarded by hmu)
};

namespace {

// Kernel-argument round keys are passed folded (aes_device.hpp fold_keys): rounds 1..9 as
// rotl16(K), so each AES column costs 3 VALU and the kernels keep them as plain kernargs.
cmpi::dev::RoundKeys folded(const cmpi::dev::RoundKeys& k) {
  cmpi::dev::RoundKeys f = k;
  for (int i = 4; i < 40; ++i) f.w[i] = (k.w[i] << 16) | (k.w[i] >> 16);
  return f;
}

// Events that only order device work after device work (hipStreamWaitEvent: a re-key before the
// launches that read its tables, a scratch buffer's previous user, ring fills before the XOR that
// consumes them, H2D before the kernel): a device-scope release, not the default system-scope
// fence, whose cache writeback / invalidate left a ~5 us bubble before the next kernel of the
// stream (702 send: ring XOR + event ~5.5 us over the launch floor, profiles/r04e_msg_latency.json).
// Events the host waits on before reading host memory keep the default.
constexpr unsigned kOrderEvent = hipEventDisableTiming | hipEventReleaseToDevice;

// Order a launch on one of the library's streams after the context's last device re-key.
int wait_keys(const cmpi_ctx* c, hipStream_t st) {
  if (!c->key_pending.load()) return CMPI_OK;
  const hipError_t q = hipEventQuery(c->key_ev);
  if (q == hipSuccess) {
    c->key_pending.store(false);
    return CMPI_OK;
  }
  if (q != hipErrorNotReady) return fail(CMPI_EHIP, "key setup failed: %s", hipGetErrorString(q));
  HIP_TRY(hipStreamWaitEvent(st, c->key_ev, 0));
  return CMPI_OK;
}

// After a re-key launched on `stream`: publish its completion event for wait_keys.
int record_keys(const cmpi_ctx* c, hipStream_t stream) {
  if (!c->key_ev) HIP_TRY(hipEventCreateWithFlags(&c->key_ev, kOrderEvent));
  HIP_TRY(hipEventRecord(c->key_ev, stream));
  c->key_pending.store(true);
  return CMPI_OK;
}

// The library's own streams (host pipeline, async request pool, message service, staging stream)
// are made here.  g_stream_mode (test hook cmpi_debug_set_stream_mode) picks the form:
//   0  hipStreamCreateWithFlags(non-blocking)
//   1  non-blocking at the greatest priority (its own pool of hardware queues)
//   2  hipExtStreamCreateWithCUMask over every CU (a hardware queue of its own; blocking)
// `own_pool`: the resident message service's stream.  A persistent kernel holds its hardware
// queue, and streams that HIP maps onto the same queue (at most GPU_MAX_HW_QUEUES = 4 per priority
// on the test box) wait behind it for up to its lifetime; at the greatest priority it sits in the
// high-priority pool, away from the caller's and torch's normal-priority streams
// (tools/queue_probe.py, profiles/r04a_queue_probe.jsonl: a kernel on another stream waited up to
// 98 ms behind the service at normal priority, <= 0.6 ms once its streams were warm at high).
std::atomic<int> g_stream_mode{0};
// A stream with a CU mask over every CU: a hardware queue of its own (blocking)
hipError_t cu_stream(hipStream_t* s) {
  int dev = 0, ncu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  std::vector<uint32_t> m((size_t)(ncu + 31) / 32, ~0u);
  if (ncu % 32) m.back() = (1u << (ncu % 32)) - 1u;
  return hipExtStreamCreateWithCUMask(s, (uint32_t)m.size(), m.data());
}
hipError_t lib_stream(hipStream_t* s, bool own_pool = false) {
  const int mode = own_pool ? 1 : g_stream_mode.load();
  if (mode == 1) {
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return e;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
  }
  if (mode == 2) return cu_stream(s);
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// Device memory that held key-derived values (chunk weights H^k, GHASH partials, tables) is
// zeroed before it is released or reused for another key (powers of H are enough to
// forge tags under the old key).  Callers have drained the streams that used it.  The memsets run
// on a library stream of the current device and wipe_sync() waits for them alone (no device-wide
// synchronise: the per-message 602 path frees contexts at message rate).
hipStream_t wipe_stream() {
  static std::mutex m;
  static std::map<int, hipStream_t> ws;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(m);
  auto it = ws.find(dev);
  if (it != ws.end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  ws[dev] = s;  // process lifetime
  return s;
}
void wipe_dev(void* d, size_t bytes) {
  if (!d || !bytes) return;
  hipStream_t s = wipe_stream();
  if (!s || hipMemsetAsync(d, 0, bytes, s) != hipSuccess) (void)hipMemset(d, 0, bytes);
}
void wipe_sync() {
  if (hipStream_t s = wipe_stream()) (void)hipStreamSynchronize(s);
}
void wipe_chw(std::map<std::pair<uint32_t, uint32_t>, void*>& chw) {
  for (auto& kv : chw) wipe_dev(kv.second, (size_t)kv.first.second * 64);  // nch x 4 weights of 16 B
  wipe_sync();
  for (auto& kv : chw) (void)hipFree(kv.second);
  chw.clear();
}

// host-side key-derived values (the combine's powers of H) zeroed before their map entries are released
template <class M>
void wipe_map(M& m) {
  for (auto& kv : m) memset(&kv.second, 0, sizeof kv.second);
  m.clear();
}

int ensure_buf(void** p, size_t* cap, size_t need) {
  if (need <= *cap) return CMPI_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  size_t sz = std::max(need, (size_t)1 << 20);
  if (hipMalloc(p, sz) != hipSuccess) return fail(CMPI_ENOMEM, "hipMalloc(%zu) failed", sz);
  *cap = sz;
  return CMPI_OK;
}

// Workspace of one batch call: the caller's buffer, or the context's scratch under a lease that
// holds the ctx lock through the launches, makes the launch stream wait for the scratch's previous
// user and records the new last use when it ends (NULL-workspace calls from two
// streams used to overwrite each other's partials).
struct ScratchLease {
  const cmpi_ctx* c;
  hipStream_t st;
  std::unique_lock<std::mutex> lk;
  uint8_t* ptr = nullptr;
  bool internal = false;
  ScratchLease(const cmpi_ctx* c_, void* workspace, hipStream_t st_) : c(c_), st(st_) {
    ptr = (uint8_t*)workspace;
  }
  // order this call after the previous user of the context's scratch / counters
  int order() {
    if (internal) return CMPI_OK;
    lk = std::unique_lock<std::mutex>(c->smu);
    internal = true;
    if (!c->scratch_ev) HIP_TRY(hipEventCreateWithFlags(&c->scratch_ev, kOrderEvent));
    if (c->scratch_used) HIP_TRY(hipStreamWaitEvent(st, c->scratch_ev, 0));
    return CMPI_OK;
  }
  int acquire(size_t need) {
    if (ptr || !need) return CMPI_OK;
    int rc = order();
    if (rc) return rc;
    rc = ensure_buf(&c->scratch, &c->scratch_cap, need);
    if (rc) return rc;
    ptr = (uint8_t*)c->scratch;
    return CMPI_OK;
  }
  ~ScratchLease() {
    if (internal && hipEventRecord(c->scratch_ev, st) == hipSuccess) c->scratch_used = true;
  }
};

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device).
std::mutex g_attr_mu;
std::map<std::pair<const void*, int>, int> g_attr_done;
int set_lds_attr(const void* fn, int device, size_t lds) {
  std::lock_guard<std::mutex> lk(g_attr_mu);
  auto key = std::make_pair(fn, device);
  auto it = g_attr_done.find(key);
  if (it != g_attr_done.end() && it->second >= (int)lds) return CMPI_OK;
  HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  g_attr_done[key] = (int)lds;
  return CMPI_OK;
}

// ---------------------------------------------------------------- GCM launch planning
// wide plan: a wave's fixed cost (table staging, lane weights) in units of one 64-block step
constexpr uint64_t kWideFixedSteps = 4;
struct GcmPlan {
  int L;
  uint32_t nb, nseg, G, r0;
  bool wide = false;  // gcm_flow_kernel: nseg = chunks per record, G = 64*S X-blocks per chunk
  uint32_t S = 0;
  uint32_t nt = 1024; // FLOW kernel threads per workgroup
};

// test hooks (include/cmpi_debug.h): they pick among correct decompositions, never change output
std::atomic<int> g_force_L{0};          // lanes per record, 0 = automatic
std::atomic<uint32_t> g_force_nseg{0};  // segments per record, 0 = automatic
std::atomic<int> g_force_wide{0};       // wide decomposition: 0 automatic, 1 always (when legal), -1 never
std::atomic<uint32_t> g_force_S{0};     // wide steps per chunk, 0 = automatic
std::atomic<int> g_flow_nt{0};          // FLOW kernel threads per workgroup: 0 automatic, 512 / 1024 forced
std::atomic<int> g_flow_one_wg{1};      // FLOW kernel: one-workgroup batches finish their tags in-kernel
#if CMPI_TOOLS
std::atomic<uint64_t*> g_wide_probe{nullptr};  // diagnostics build: per-workgroup phase timestamps
std::atomic<uint64_t*> g_svc_probe{nullptr};   // diagnostics build: service message phase stamps
#endif
// wave priority: bit 1 CTR, bit 2 OCB rotate per step (the GCM kernels: progress / rotation, fixed)
constexpr uint32_t kSched = 7u;

GcmPlan plan_gcm(const cmpi_ctx* c, size_t len, size_t nrec) {
  GcmPlan p{};
  p.nb = (uint32_t)((len + 15) / 16);
  const uint64_t nx = (uint64_t)p.nb + 1;
  const uint64_t target = (uint64_t)c->ncu * kGcmThreads;  // lanes that fill the chip once
  p.L = 4;
  if ((uint64_t)nrec * 1 >= target && nx >= 1) p.L = 1;
  else if ((uint64_t)nrec * 2 >= target) p.L = 2;
  if (nx < 8) p.L = 1;  // tiny records: one lane each
  uint64_t nseg = 1;
  const uint64_t lanes = (uint64_t)nrec * p.L;
  if (lanes < target) {
    const uint64_t want = (target + lanes - 1) / lanes;
    const uint64_t maxseg = std::max<uint64_t>(1, nx / (uint64_t)(p.L * 32));  // >= 32 X-blocks per lane
    nseg = std::min(want, maxseg);
  }
  if (g_force_L.load()) p.L = g_force_L.load();
  if (g_force_nseg.load()) nseg = std::min<uint64_t>(g_force_nseg.load(), nx);
  // Wide decomposition (gcm_flow_kernel) when the lane-group plan leaves most of the chip idle
  // (few long records: the naive collectives' p peer blocks, 602 segments, single messages);
  // records need >= 64 data blocks (short ones: below).
  // Short records (under 64 data blocks), at most one round of flow waves of them: one partial
  // step + the lane tree per record instead of a lane's nx / L serial steps (1 x 1000 B seal
  // 32.3 -> 11.2 us, 2048 x 1000 B 52.8 -> 18.5 us, 2048 x 300 B 25.9 -> 17.4 us:
  // profiles/r03l_flow_short_ab.json, r03l_flow_short16_ab.json).  Below 16 blocks only batches
  // one workgroup finishes in-launch (16 x 100 B: 11.2 us on the lane kernel, 14.8 with the flow
  // kernel's combine launch).
  const int fw = g_force_wide.load();
  const bool short_few = p.nb >= 1 && p.nb < 64 && (p.nb >= 16 || nrec <= 8) &&
                         (uint64_t)nrec <= (uint64_t)c->ncu * 8 && !g_force_L.load();
  const bool wide_ok = p.nb >= 64 || short_few;
  if (wide_ok && (fw > 0 || (fw == 0 && (short_few || (p.L == 4 && (uint64_t)nrec * p.L * nseg * 2 < target &&
                                                        (nx >= 256 || (uint64_t)nrec * p.L * nseg * 8 <= target)))))) {
    // A round = one wave per (record, chunk) on every CU (W waves); a wave's time ~ (fixed
    // staging/weight phases) + S steps.  Chunks are cut from the end with chunk 0 absorbing the
    // remainder (G <= its length < 2G), so 1 MiB records (nx = 2^16 + 1) split into exactly
    // 2^16 / G chunks instead of one extra 1-block chunk that would start a second round.
    // 512-thread workgroups, one per CU (228 VGPRs, no spills; 8 x 1 MiB at S = 4: 22.6 us vs
    // 30.9 at 1024 threads): a round is 8 waves per CU
    const int fnt = g_flow_nt.load();
    const uint64_t W = (uint64_t)c->ncu * (fnt ? (uint64_t)fnt / 64 : 8);
    const uint64_t smax = std::max<uint64_t>(1, nx / 64);
    uint64_t S = g_force_S.load();
    if (!S) {
      double best = 1e300;
      for (uint64_t s = 1; s <= smax; s = c->dev_keys ? 2 * s : s + 1) {
        const uint64_t units = (uint64_t)nrec * std::max<uint64_t>(1, nx / (64 * s));
        const double est = (double)((units + W - 1) / W) * (double)(kWideFixedSteps + s);
        if (est < best) best = est, S = s;
        if (units <= W / 2) break;  // one round already: longer chunks only lengthen it
      }
    }
    S = std::min<uint64_t>(std::max<uint64_t>(S, 1), smax);
    if (c->dev_keys) S = (uint64_t)1 << (63 - __builtin_clzll(S));  // combine weights from H^(2^i)
    p.wide = true;
    p.S = (uint32_t)S;
    p.L = 64;
    p.G = (uint32_t)(64 * S);
    p.nseg = (uint32_t)std::max<uint64_t>(1, nx / p.G);
    p.r0 = (uint32_t)(nx - (uint64_t)(p.nseg - 1) * p.G);
    // 512-thread workgroups: few waves (single messages, the 600/EVP regime; the naive
    // alltoall's 8 x 1 MiB: 1 x 64 KiB seal 21.0 -> 15.7 us at S = 2) and several rounds alike
    // (the 1024-thread form is capped at 128 VGPRs and spills: 3000 / 4096 / 6000 x 1 KiB seal
    // 25.0 / 25.8 / 38.4 -> 23.7 / 24.2 / 32.3 us, profiles/r04zzb_nt_ab.txt)
    p.nt = 512;
    if (fnt) p.nt = (uint32_t)fnt;
    return p;
  }
  uint64_t G = (nx + nseg - 1) / nseg;
  // device-keyed contexts weight segment partials by products of H^(2^i) (no host H): G = 2^g
  if (c->dev_keys && nseg > 1 && G > 1) G = (uint64_t)1 << (64 - __builtin_clzll(G - 1));
  nseg = (nx + G - 1) / G;
  p.G = (uint32_t)G;
  p.nseg = (uint32_t)nseg;
  p.r0 = (uint32_t)(nx - (nseg - 1) * G);
  return p;
}

// workspace: partials [nrec][nseg], E_K(J0) [nrec], and for device-keyed contexts H^{kG} [nseg]
size_t gcm_ws_bytes(const cmpi_ctx* c, const GcmPlan& p, size_t nrec) {
  if (p.wide) return (size_t)nrec * p.nseg * 16 + nrec * 16;  // (E_K(J0) slots double as statuses)
  if (p.nseg <= 1) return 0;
  return (size_t)nrec * p.nseg * 16 + nrec * 16;
}

// Combine multipliers M_j = H^{G·2^j}, j < 7 (gcm_combine_kernel).  Host-keyed contexts: computed
// here once per segment length G and passed in the kernel arguments (no allocation or copy on
// the launch path, which also runs inside the multi-stream host pipeline); device-keyed:
// H^(2^(log2 G + j)) in the context's device tables (written by the key-setup kernel).
int get_mj(const cmpi_ctx* c, uint32_t G, cmpi::dev::GcmCombineArgs& ca) {
  if (c->dev_keys) {
    if (G & (G - 1u) || __builtin_ctz(G) + 7 > 32) return fail(CMPI_EINVAL, "device-keyed segment length");
    ca.mjp = reinterpret_cast<const u32x4*>(c->dt->h2pow[__builtin_ctz(G)]);
    return CMPI_OK;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  auto it = c->mj.find(G);
  if (it == c->mj.end()) {
    std::array<Blk, 7> m;
    m[0] = cmpi::gf_pow(c->H, G);
    for (int j = 1; j < 7; ++j) m[j] = cmpi::gf_mul(m[j - 1], m[j - 1]);
    it = c->mj.emplace(G, m).first;
  }
  ca.mjp = nullptr;
  static_assert(sizeof(Blk) == sizeof(u32x4), "field element layout");
  memcpy(ca.mjv, it->second.data(), sizeof(ca.mjv));
  return CMPI_OK;
}

// Chunk weights of the FLOW wide kernel, chw[4i + j] = H^(49 - 16j + (nch-1-i)·C), i < nch,
// j < 4 (the weights of chunk i's four quarter-wave sums, so the combine only XORs): built on
// the host from H once per (C, nch) and kept in HBM for the context's lifetime.  Device-keyed
// contexts (no host H) return null and keep the barrier-phased kernel + combine weighting.
// At most kChwCache entries per context (record lengths vary in the per-message regimes).  A
// cached entry is uploaded with a blocking copy before it is published, so a call on another
// stream that finds it can never launch before its bytes are in HBM, and cached entries are freed
// only with the context (or at a re-key, which the caller orders after all use).  Past the cap,
// the weights of one call go to a stream-ordered allocation on the launch stream that the caller
// releases with hipFreeAsync after its launches (*transient = true) — ADVICE r2.
constexpr size_t kChwCache = 32;
int get_chw(const cmpi_ctx* c, uint32_t C, uint32_t nch, const u32x4** out, hipStream_t st, bool* transient) {
  *out = nullptr;
  *transient = false;
  if (c->dev_keys) return CMPI_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  auto key = std::make_pair(C, nch);
  auto it = c->chw.find(key);
  if (it == c->chw.end()) {
    std::vector<Blk> w((size_t)nch * 4);
    const Blk P = cmpi::gf_pow(c->H, C), H16 = cmpi::gf_pow(c->H, 16);
    Blk wi = c->H;  // H^(1 + (nch-1-i)·C), i = nch-1 down to 0
    for (uint32_t i = nch; i-- > 0;) {
      Blk q = wi;
      for (int j = 3; j >= 0; --j) {  // j = 3: H^1·W, j = 2: H^17·W, ...
        w[(size_t)4 * i + j] = q;
        q = cmpi::gf_mul(q, H16);
      }
      wi = cmpi::gf_mul(wi, P);
    }
    void* d = nullptr;
    if (c->chw.size() >= kChwCache) {  // transient: stream-ordered, freed by the caller after its launches
      if (hipMallocAsync(&d, (size_t)nch * 64, st) != hipSuccess) return fail(CMPI_ENOMEM, "hipMallocAsync chunk weights failed");
      if (hipMemcpyAsync(d, w.data(), (size_t)nch * 64, hipMemcpyHostToDevice, st) != hipSuccess) {
        (void)hipFreeAsync(d, st);
        return fail(CMPI_EHIP, "chunk weights copy failed");
      }
      *out = reinterpret_cast<const u32x4*>(d);
      *transient = true;
      return CMPI_OK;
    }
    if (hipMalloc(&d, (size_t)nch * 64) != hipSuccess) return fail(CMPI_ENOMEM, "hipMalloc chunk weights failed");
    if (hipMemcpy(d, w.data(), (size_t)nch * 64, hipMemcpyHostToDevice) != hipSuccess) {  // complete before publishing
      (void)hipFree(d);
      return fail(CMPI_EHIP, "chunk weights copy failed");
    }
    it = c->chw.emplace(key, d).first;
  }
  *out = reinterpret_cast<const u32x4*>(it->second);
  return CMPI_OK;
}

template <bool DEC>
int launch_gcm_combine(const cmpi_ctx* c, cmpi::dev::GcmCombineArgs& ca, uint32_t G, hipStream_t st) {
  if (ca.prew && !ca.ekj0) {  // partials already weighted, E_K(J0) inside: XOR only
    HIP_TRY(launch_k(cmpi::dev::gcm_xor_combine_kernel<DEC>, dim3(ca.nrec), dim3(cmpi::dev::kXorCombineThreads), 128,
                       st, ca));
    return CMPI_OK;
  }
  int rc = get_mj(c, G, ca);
  if (rc) return rc;
  const uint32_t wpb = cmpi::dev::kCombineThreads / 64u;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((ca.nrec + wpb - 1u) / wpb, 2u * (uint32_t)c->ncu));
  HIP_TRY(launch_k(cmpi::dev::gcm_combine_kernel<DEC>, dim3(grid), dim3(cmpi::dev::kCombineThreads),
                     cmpi::dev::kCombineLds, st, ca));
  return CMPI_OK;
}

// lane kernel (L = 4) record stores grouped by 128-byte output line (gcm_lane_kernel PAIR): 2 =
// predicated selects (default; HBM writes per 65 536 x 1 KiB seal 97 -> 70 MB, open 90 -> 67 MB,
// headline neutral to +1 %: profiles/r04u_*, r04w_*), 1 = branches, 0 = a store per step
std::atomic<int> g_lane_pair{2};
template <int L, bool DEC>
int launch_gcm_main(const cmpi::dev::GcmArgs& a, int device, uint32_t grid, size_t lds, hipStream_t st) {
  // the line-aligned store forms exist for L = 4 and pay off on batches that stream HBM; a small
  // batch's single round of waves ran ~1 us longer with them (16 x 100 B: 9.9 -> 11.1 us)
  // (hook values 3 / 4: the select / branch form on every batch, for the parity tests)
  const bool big = (uint64_t)a.ngroups * (uint64_t)L >= (uint64_t)grid * kGcmThreads;
  const int h = g_lane_pair.load();
  const int pr = L != 4 ? 0 : h >= 3 ? (h == 3 ? 2 : 1) : big ? h : 0;
  auto fn = pr == 2   ? cmpi::dev::gcm_lane_kernel<L, DEC, (L == 4 ? 2 : 0)>
            : pr == 1 ? cmpi::dev::gcm_lane_kernel<L, DEC, (L == 4 ? 1 : 0)>
                      : cmpi::dev::gcm_lane_kernel<L, DEC, 0>;
  int rc = set_lds_attr(reinterpret_cast<const void*>(fn), device, lds);
  if (rc) return rc;
  HIP_TRY(launch_k(fn, dim3(grid), dim3(kGcmThreads), lds, st, a));
  return CMPI_OK;
}

// Where a batch's nonces come from (GcmArgs::nmode): 0 = memory, 1 = "0000000"||wire prefix,
// 2 = "0000000"||flag||BE32(ctr0 + r) with the prefix written, 3 = fixed 12 bytes.
struct NonceSpec {
  uint32_t mode = 0, ctr0 = 0, flag = 0;
  uint32_t flag2 = 0, flag2_from = 0xFFFFFFFFu;  // mode 2: records >= flag2_from carry flag2
  uint32_t fix[3] = {0, 0, 0};
};

bool is_pinned(const void* p);  // page-locked host memory (below)

template <bool DEC>
int gcm_batch(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
              const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status,
              void* workspace, void* stream, const NonceSpec& ns = NonceSpec()) {
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  if (c->alg != CMPI_AES_128_GCM) return fail(CMPI_EINVAL, "ctx is not AES-128-GCM");
  if (nrec == 0) return CMPI_OK;
  if (!out || (!nonces && ns.mode != 3) || (!in && (DEC || len))) return fail(CMPI_EINVAL, "null buffer");
  if (!in) in = out;  // seal of empty records reads nothing
  if (len > 0xFFFFFFF0ull || nrec > 0x7FFFFFFFull) return fail(CMPI_EINVAL, "len/nrec out of range");
  const size_t in_rec = len + (DEC ? 16 : 0), out_rec = len + (DEC ? 0 : 16);
  if (nrec > 1 && (in_stride < in_rec || out_stride < out_rec || (ns.mode == 0 && nonce_stride < 12)))
    return fail(CMPI_EINVAL, "stride smaller than record");
  DeviceGuard dg(c->device);
  hipStream_t st = (hipStream_t)stream;
  const GcmPlan p = plan_gcm(c, len, nrec);
  if ((uint64_t)nrec * p.nseg > 0xFFFFFFFFull) return fail(CMPI_EINVAL, "too many segments");

  cmpi::dev::GcmArgs a{};
  a.in = in;
  a.out = out;
  a.nonces = nonces;
  a.in_stride = in_stride;
  a.out_stride = out_stride;
  a.nonce_stride = nonce_stride;
  a.len = (uint32_t)len;
  a.nb = p.nb;
  a.nrec = (uint32_t)nrec;
  a.nseg = p.nseg;
  a.G = p.G;
  a.r0 = p.r0;
  a.ngroups = (uint32_t)(nrec * p.nseg);
  a.htab = reinterpret_cast<const u32x4*>(c->dt->htab[p.L == 1 ? 0 : (p.L == 2 ? 1 : 2)]);
  a.ntab = reinterpret_cast<const u32x4*>(c->dt->fnib[0]);  // H^1..H^3
  a.te0 = c->dt->te0;
  a.status = status;
  a.rk = folded(c->rk);
  a.rkp = c->dev_keys ? c->dt->keys : nullptr;
  a.nmode = ns.mode;
  a.nctr0 = ns.ctr0;
  a.nflag = ns.flag;
  a.nflag2 = ns.flag2;
  a.nflag2_from = ns.flag2_from;
  memcpy(a.nfix, ns.fix, sizeof a.nfix);
#if CMPI_TOOLS
  a.probe = g_wide_probe.load();
#endif
  ScratchLease lease(c, workspace, st);
  if (p.wide) {
    if ((uint64_t)nrec * p.nseg * 16 > 0xFFFFFFFFull) return fail(CMPI_EINVAL, "too many chunks");
    int rc0 = lease.acquire(gcm_ws_bytes(c, p, nrec));
    if (rc0) return rc0;
    uint8_t* ws = lease.ptr;
    a.partial = reinterpret_cast<u32x4*>(ws);
    a.ekj0 = reinterpret_cast<u32x4*>(ws + (size_t)nrec * p.nseg * 16);
    a.S = p.S;
    a.nch = p.nseg;
    a.wtab = reinterpret_cast<const u32x4*>(c->dt->fnib[0]);
    bool chw_transient = false;
    int rc = get_chw(c, p.G, p.nseg, &a.chw, st, &chw_transient);  // null for device-keyed contexts
    if (rc) return rc;
    // a transient weights buffer is released in stream order after this call's launches
    struct FreeAsync {
      const void* p;
      hipStream_t s;
      ~FreeAsync() {
        if (p) (void)hipFreeAsync(const_cast<void*>(p), s);
      }
    } chw_guard{chw_transient ? (const void*)a.chw : nullptr, st};
    const uint64_t waves = (uint64_t)nrec * p.nseg;
    const int NT = (int)p.nt;
    // every chunk of the batch in one workgroup (single small messages, host-keyed): the tags are
    // finished from the workgroup's LDS aggregation in the same launch
    const bool one_wg = a.chw && g_flow_one_wg.load() && waves <= (uint64_t)(NT / 64);
    a.one_wg = one_wg ? 1u : 0u;
    if (one_wg && DEC && !status) a.status = reinterpret_cast<int32_t*>(ws + (size_t)nrec * p.nseg * 16);
    const bool dk = !a.chw;  // device-keyed context
    // records in host memory (the direct host paths: 602 outer messages, single messages without
    // the service): units read only their own rows over PCIe
    const bool hostin = NT == 512 && is_pinned(in);
    using namespace cmpi::dev;
    const void* fn = hostin ? (dk ? reinterpret_cast<const void*>(gcm_flow_kernel<DEC, 512, true, true>)
                                  : reinterpret_cast<const void*>(gcm_flow_kernel<DEC, 512, false, true>))
                   : NT == 512 ? (dk ? reinterpret_cast<const void*>(gcm_flow_kernel<DEC, 512, true>)
                                     : reinterpret_cast<const void*>(gcm_flow_kernel<DEC, 512, false>))
                               : (dk ? reinterpret_cast<const void*>(gcm_flow_kernel<DEC, 1024, true>)
                                     : reinterpret_cast<const void*>(gcm_flow_kernel<DEC, 1024, false>));
    const size_t lds = (size_t)cmpi::dev::kFlowLds;
    if ((rc = set_lds_attr(fn, c->device, lds))) return rc;
    const uint32_t wpb = (uint32_t)NT / 64u;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((waves + wpb - 1) / wpb, (uint64_t)c->ncu));
    void* kargs[] = {&a};
    HIP_TRY(launch_raw(fn, dim3(grid), dim3(NT), kargs, lds, st));
    if (one_wg) return CMPI_OK;
    cmpi::dev::GcmCombineArgs ca{};
    ca.in = in;
    ca.out = out;
    ca.in_stride = in_stride;
    ca.out_stride = out_stride;
    ca.len = (uint32_t)len;
    ca.nb = p.nb;
    ca.nrec = (uint32_t)nrec;
    ca.nseg = p.nseg;
    ca.partial = a.partial;
    ca.ekj0 = a.chw ? nullptr : a.ekj0;  // device-keyed: E_K(J0) and the chunk weights applied here
    ca.status = status;
    ca.prew = a.chw ? 1u : 0u;
    return launch_gcm_combine<DEC>(c, ca, p.G, st);  // chunk i weighted by H^{(nch-1-i)·64S}, as segments
  }
  if (p.nseg > 1) {
    int rc0 = lease.acquire(gcm_ws_bytes(c, p, nrec));
    if (rc0) return rc0;
    uint8_t* ws = lease.ptr;
    a.partial = reinterpret_cast<u32x4*>(ws);
    a.ekj0 = reinterpret_cast<u32x4*>(ws + (size_t)nrec * p.nseg * 16);
  }
  const size_t lds = cmpi::dev::gcm_lds_bytes(p.L);
  const uint64_t want = ((uint64_t)a.ngroups * p.L + kGcmThreads - 1) / kGcmThreads;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->ncu));
  int rc;
  switch (p.L) {
    case 1: rc = launch_gcm_main<1, DEC>(a, c->device, grid, lds, st); break;
    case 2: rc = launch_gcm_main<2, DEC>(a, c->device, grid, lds, st); break;
    default: rc = launch_gcm_main<4, DEC>(a, c->device, grid, lds, st); break;
  }
  if (rc) return rc;
  if (p.nseg > 1) {
    cmpi::dev::GcmCombineArgs ca{};
    ca.in = in;
    ca.out = out;
    ca.in_stride = in_stride;
    ca.out_stride = out_stride;
    ca.len = (uint32_t)len;
    ca.nb = p.nb;
    ca.nrec = (uint32_t)nrec;
    ca.nseg = p.nseg;
    ca.partial = a.partial;
    ca.ekj0 = a.ekj0;
    ca.status = status;
    rc = launch_gcm_combine<DEC>(c, ca, p.G, st);
    if (rc) return rc;
  }
  return CMPI_OK;
}

// ---------------------------------------------------------------- OCB
struct OcbPlan {
  uint32_t m, S, nchunks;
};

OcbPlan plan_ocb(const cmpi_ctx* c, size_t len, size_t nrec) {
  OcbPlan p{};
  p.m = (uint32_t)(len / 16);
  const uint32_t ksteps = p.m / 64 + 1;
  // aim for >= 8 waves per CU over the whole batch, >= 4 steps per chunk
  const uint64_t target_waves = (uint64_t)c->ncu * 32;
  uint64_t chunks = std::max<uint64_t>(1, (target_waves + nrec - 1) / std::max<size_t>(nrec, 1));
  chunks = std::min<uint64_t>(chunks, std::max<uint32_t>(1, ksteps / 4));
  p.S = (uint32_t)((ksteps + chunks - 1) / chunks);
  p.nchunks = (ksteps + p.S - 1) / p.S;
  return p;
}

template <bool DEC>
int ocb_batch(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
              const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status,
              void* workspace, void* stream) {
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  if (c->alg != CMPI_AES_128_OCB) return fail(CMPI_EINVAL, "ctx is not AES-128-OCB");
  if (nrec == 0) return CMPI_OK;
  if (!out || !nonces || (!in && (DEC || len))) return fail(CMPI_EINVAL, "null buffer");
  if (!in) in = out;  // seal of empty records reads nothing
  if (len > 0xFFFFFFF0ull || nrec > 0x7FFFFFFFull) return fail(CMPI_EINVAL, "len/nrec out of range");
  const size_t in_rec = len + (DEC ? 16 : 0), out_rec = len + (DEC ? 0 : 16);
  if (nrec > 1 && (in_stride < in_rec || out_stride < out_rec || nonce_stride < 12))
    return fail(CMPI_EINVAL, "stride smaller than record");
  DeviceGuard dg(c->device);
  hipStream_t st = (hipStream_t)stream;
  const OcbPlan p = plan_ocb(c, len, nrec);
  const size_t part_bytes = (size_t)nrec * p.nchunks * 16;
  const size_t off_bytes = (size_t)nrec * 16;
  const size_t need = part_bytes + off_bytes + (size_t)nrec * 4;
  ScratchLease lease(c, workspace, st);
  {
    int rc0 = lease.acquire(need);
    if (rc0) return rc0;
  }
  uint8_t* ws = lease.ptr;
  u32x4* d_part = reinterpret_cast<u32x4*>(ws);
  u32x4* d_off0 = reinterpret_cast<u32x4*>(ws + part_bytes);
  int32_t* st_arr = status ? status : reinterpret_cast<int32_t*>(ws + part_bytes + off_bytes);

  cmpi::dev::OcbArgs a{};
  a.in = in;
  a.out = out;
  a.nonces = nonces;
  a.in_stride = in_stride;
  a.out_stride = out_stride;
  a.nonce_stride = nonce_stride;
  a.len = (uint32_t)len;
  a.m = p.m;
  a.nrec = (uint32_t)nrec;
  a.S = p.S;
  a.nchunks = p.nchunks;
  a.nitems = (uint32_t)(nrec * p.nchunks);
  a.te0 = c->dt->te0;
  a.td0 = c->dt->td0;
  a.isb = c->dt->isb;
  a.ltab = reinterpret_cast<const u32x4*>(c->dt->ltab);
  a.off0 = d_off0;
  a.partial = d_part;
  a.rk = folded(c->rk);
  a.sched = kSched;
  a.drk = folded(c->drk);
  const size_t lds = DEC ? cmpi::dev::kOcbBatchLdsOpen : cmpi::dev::kOcbBatchLdsSeal;
  const uint32_t per_cu = DEC ? 1u : 2u;  // LDS-limited 1024-thread blocks per CU
  auto fn = cmpi::dev::ocb_batch_kernel<DEC>;
  int rc = set_lds_attr(reinterpret_cast<const void*>(fn), c->device, lds);
  if (rc) return rc;
  const uint64_t waves = a.nitems;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((waves + 15) / 16, (uint64_t)c->ncu * per_cu));
  HIP_TRY(launch_k(fn, dim3(grid), dim3(1024), lds, st, a));

  cmpi::dev::OcbFinalArgs f{};
  f.in = in;
  f.out = out;
  f.nonces = nonces;
  f.in_stride = in_stride;
  f.out_stride = out_stride;
  f.nonce_stride = nonce_stride;
  f.len = (uint32_t)len;
  f.m = p.m;
  f.nrec = (uint32_t)nrec;
  f.nchunks = p.nchunks;
  f.te0 = c->dt->te0;
  f.ltab = a.ltab;
  f.partial = d_part;
  f.off0 = d_off0;
  f.status = st_arr;
  f.rk = folded(c->rk);
  {
    int rc1 = set_lds_attr(reinterpret_cast<const void*>(cmpi::dev::ocb_final_kernel<DEC>), c->device, cmpi::dev::kOcbFinalLds);
    if (rc1) return rc1;
  }
  HIP_TRY(launch_k(cmpi::dev::ocb_final_kernel<DEC>, dim3((uint32_t)((nrec + 255) / 256)), dim3(256),
                     cmpi::dev::kOcbFinalLds, st, f));  // open: verdicts and the zero-fill of forged records
  return CMPI_OK;
}

// ---------------------------------------------------------------- host staging
// Host-memory batches (the *_host entry points: CryptMPI's buffers are host memory bound for a
// NIC).  The batch is cut into chunks of ~g_host_chunk bytes pipelined over
// three streams with NS staging slots (3):  H2D(i+1) | kernel(i) | D2H(i-1)  overlap, the slot of
// chunk i is reused by chunk i+NS once D2H(i) completed.  Pinned host buffers (hipHostMalloc /
// cmpi_host_register) move by DMA at PCIe rate; pageable ones are staged by the HIP runtime.
std::atomic<size_t> g_host_slots{3};  // staging slots, 2..4 (cmpi_debug_set_host_slots)
// 0 = automatic: 8 MiB when records, outputs and nonces are all page-locked (mode 5: 4 / 8 / 16 MiB
// ran 37.3-37.6 / 37.2-37.5 / 35.6-36.1 GiB/s, tools/host_pipe_sweep.py r06ak), else 16 MiB (the
// pageable path packs each chunk on the CPU: 8 MiB chunks ran it at 15.2 instead of 18-20)
std::atomic<size_t> g_host_chunk{0};
// Host pipeline copy modes (cmpi_debug_set_host_out_direct), page-locked dense outputs:
//   0  hipMemcpyAsync both ways (HIP runs a D2H into page-locked memory as a blit kernel, and
//      while one runs no other command of the pipeline starts: kernel and D2H of each chunk in
//      series, 34.8 GiB/s — profiles/r06_hostpath_timelines.txt);
//   1  the kernel writes the outputs (and open's statuses) over PCIe itself (32.9: the kernel's
//      scattered 16-byte stores reach 49 GB/s where a copy reaches 57);
//   4  hipMemcpyAsync H2D, D2H on an SDMA engine through HSA (hsa_copy.hpp), issued by this thread
//      when the chunk's kernel is done (37.0);
//   5  both ways on SDMA through HSA, this thread launching each chunk's kernel when its input
//      landed — no HIP event between copies and kernels (the marker after each H2D held the next
//      H2D and the kernel ~23 us) (37.4) — needs page-locked inputs, outputs and nonces and more
//      than one chunk; otherwise mode 4's D2H, otherwise mode 0.
std::atomic<int> g_host_out_direct{5};

// true when p lies in page-locked host memory (hipHostMalloc / hipHostRegister): it can be the
// direct source/target of an asynchronous DMA.  Pageable memory is never handed to async copies
// (the runtime's pageable path under concurrent streams faulted in testing, round 1): it goes
// through our pinned staging slots with a CPU pack/unpack overlapped with the other chunks.
//
// hipPointerGetAttributes fails (hipErrorInvalidValue) on pageable memory and records that as the
// thread's last error; ptr_attrs clears the failure it caused only when no error of the caller's
// was pending before the query, so a caller's error stays readable.
bool ptr_attrs(const void* p, hipPointerAttribute_t* at) {
  const hipError_t prior = hipPeekAtLastError();
  if (hipPointerGetAttributes(at, p) == hipSuccess) return true;
  if (prior == hipSuccess) (void)hipGetLastError();
  return false;
}

bool is_pinned(const void* p) {
  hipPointerAttribute_t at;
  if (!ptr_attrs(p, &at)) return false;
  return at.type == hipMemoryTypeHost;
}

// Record-wise copy between a caller's pageable buffer and a pinned staging slot (the CPU side of
// the pageable host path), split over host threads: one thread packs ~8-10 GB/s, so 16 MiB
// chunks otherwise bound the pageable path near 8 GiB/s.  Threads: CMPI_HOST_THREADS (default
// 8, at most the hardware's), one part on the calling thread.
void par_copy_records(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t rec, size_t n) {
  static const unsigned kThreads = [] {
    unsigned t = 8;
    if (const char* e = getenv("CMPI_HOST_THREADS")) t = (unsigned)std::max(1, atoi(e));
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    return std::min(t, hw);
  }();
  auto part = [&](size_t a, size_t b) {
    if (dpitch == rec && spitch == rec) {
      memcpy(dst + a * rec, src + a * rec, (b - a) * rec);
      return;
    }
    for (size_t i = a; i < b; ++i) memcpy(dst + i * dpitch, src + i * spitch, rec);
  };
  const size_t T = std::min<size_t>(kThreads, std::max<size_t>(1, n * rec / ((size_t)1 << 20)));  // >= 1 MiB each
  if (T <= 1) {
    part(0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (size_t t = 1; t < T; ++t) th.emplace_back(part, n * t / T, n * (t + 1) / T);
  part(0, n / T);
  for (auto& x : th) x.join();
}

// Device address of page-locked host memory (the kernel reads / writes it over PCIe), or null.
void* pinned_dev_ptr(const void* p) {
  hipPointerAttribute_t at;
  if (!ptr_attrs(p, &at)) return nullptr;
  if (at.type != hipMemoryTypeHost || !at.devicePointer) return nullptr;
  const uintptr_t off = at.hostPointer ? (uintptr_t)p - (uintptr_t)at.hostPointer : 0;
  return (uint8_t*)at.devicePointer + off;
}

// Completion of a direct-path call (an MPI progress loop's busy wait).  g_host_spin selects how
// the host learns that the call's kernels are done:
//   0  blocking hipStreamSynchronize;
//   1  the stream writes the call's sequence number into a page-locked coherent host word after
//      the kernels (hipStreamWriteValue32) and the host spins on that word;
//   2  the same word written by a one-wave kernel launched after the call's kernels;
//   3  polling hipStreamQuery (the round-2 form).
// In modes 1 and 2 the loop also asks the stream after 200 us, so a failed kernel returns its
// error instead of spinning.
std::atomic<int> g_host_spin{0};
__global__ void done_flag_kernel(uint32_t* flag, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
hipError_t flag_wait(HostPipe& P, hipStream_t st) {
  const int mode = g_host_spin.load();
  if (mode == 0) return hipStreamSynchronize(st);
  if (mode == 3) {
    for (;;) {
      const hipError_t e = hipStreamQuery(st);
      if (e != hipErrorNotReady) return e;
    }
  }
  if (!P.hflag) {
    hipError_t e = hipHostMalloc((void**)&P.hflag, 64, hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    *P.hflag = P.seq;
    if ((e = hipHostGetDevicePointer((void**)&P.dflag, P.hflag, 0)) != hipSuccess) {
      (void)hipHostFree(P.hflag);
      P.hflag = nullptr;
      return e;
    }
  }
  const uint32_t seq = ++P.seq;
  hipError_t e = hipSuccess;
  if (mode == 1) {
    e = hipStreamWriteValue32(st, P.dflag, seq, 0);
  } else {
    e = launch_k(done_flag_kernel, dim3(1), dim3(64), 0, st, P.dflag, seq);
  }
  if (e != hipSuccess) return e;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1;; ++i) {
    if (__atomic_load_n(P.hflag, __ATOMIC_ACQUIRE) == seq) return hipSuccess;
    if ((i & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) {
      e = hipStreamQuery(st);
      if (e == hipSuccess) return __atomic_load_n(P.hflag, __ATOMIC_ACQUIRE) == seq ? hipSuccess : hipErrorUnknown;
      if (e != hipErrorNotReady) return e;
    }
  }
}

// Direct host path for small batches (a single MPI message, an EVP call): no DMA launches and no
// cross-stream events — the kernel reads the records from and writes them to page-locked host
// memory itself (zero-copy over PCIe), nonces and statuses in a pinned bounce buffer, pageable
// records packed / unpacked through it on the CPU.  One launch (+ the combine) and one stream
// synchronisation per call, where the pipeline pays H2D + kernel + D2H + 3 stream joins.
std::atomic<size_t> g_host_direct{((size_t)2 << 20) + 64};  // largest in+out bytes taken direct (0 = never)

template <bool DEC, bool OCB>
int host_direct(const cmpi_ctx* c, HostPipe& P, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status) {
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t in_rec = len + (DEC ? 16 : 0), out_rec = len + (DEC ? 0 : 16);
  void* din = in_rec ? pinned_dev_ptr(in) : nullptr;
  void* dout = out_rec ? pinned_dev_ptr(out) : nullptr;
  const size_t bi = in_rec && !din ? up16(in_rec * nrec) : 0, bo = out_rec && !dout ? up16(out_rec * nrec) : 0;
  const size_t need = bi + bo + up16(16 * nrec) + up16(4 * nrec) + 64;
  if (P.dcap < need) {
    HIP_TRY(hipStreamSynchronize(P.s[1]));
    if (P.dbounce) (void)hipHostFree(P.dbounce);
    P.dbounce = nullptr;
    P.dcap = 0;
    const size_t cap = std::max<size_t>(need, (size_t)1 << 20);
    if (hipHostMalloc((void**)&P.dbounce, cap, hipHostMallocDefault) != hipSuccess)
      return fail(CMPI_ENOMEM, "hipHostMalloc bounce failed");
    P.dcap = cap;
  }
  uint8_t* B = P.dbounce;
  uint8_t* dB = (uint8_t*)pinned_dev_ptr(B);
  if (!dB) return fail(CMPI_EHIP, "bounce buffer has no device address");
  size_t istr = in_stride, ostr = out_stride;
  if (!din) {  // pageable (or empty) input records: packed into the bounce buffer
    if (in_rec) par_copy_records(B, in_rec, in, in_stride, in_rec, nrec);
    din = dB;
    istr = std::max<size_t>(in_rec, 1);
  }
  uint8_t* hout = nullptr;
  if (!dout) {
    hout = B + bi;
    dout = dB + bi;
    ostr = std::max<size_t>(out_rec, 1);
  }
  uint8_t* hn = B + bi + bo;
  for (size_t i = 0; i < nrec; ++i) memcpy(hn + 16 * i, nonces + i * nonce_stride, 12);
  int32_t* hst = reinterpret_cast<int32_t*>(hn + up16(16 * nrec));
  int32_t* dst = reinterpret_cast<int32_t*>(dB + (bi + bo + up16(16 * nrec)));
  int rc = OCB ? ocb_batch<DEC>(c, (uint8_t*)dout, ostr, (const uint8_t*)din, istr, dB + bi + bo, 16, len, nrec,
                               DEC ? dst : nullptr, nullptr, P.s[1])
               : gcm_batch<DEC>(c, (uint8_t*)dout, ostr, (const uint8_t*)din, istr, dB + bi + bo, 16, len, nrec,
                               DEC ? dst : nullptr, nullptr, P.s[1]);
  if (rc) return rc;
  HIP_TRY(flag_wait(P, P.s[1]));
  if (hout && out_rec) par_copy_records(out, out_stride, hout, out_rec, out_rec, nrec);
  if (DEC) {
    size_t bad = 0;
    for (size_t i = 0; i < nrec; ++i) bad += hst[i] != 1;
    if (status) memcpy(status, hst, 4 * nrec);
    if (bad) return fail(CMPI_EAUTH, "%zu of %zu records failed authentication", bad, nrec);
  }
  return CMPI_OK;
}

}  // namespace
#include "service_host.hpp"
namespace {

template <bool DEC, bool OCB>
int aead_host(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
              const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status) {
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  if (nrec == 0) return CMPI_OK;
  const size_t in_rec = len + (DEC ? 16 : 0), out_rec = len + (DEC ? 0 : 16);
  if ((!out && out_rec) || (!in && in_rec) || !nonces) return fail(CMPI_EINVAL, "null buffer");
  if (nrec > 1 && (in_stride < in_rec || out_stride < out_rec || nonce_stride < 12))
    return fail(CMPI_EINVAL, "stride smaller than record");
  if (nrec == 1) in_stride = in_rec, out_stride = out_rec, nonce_stride = 12;
  DeviceGuard dg(c->device);
  std::unique_lock<std::mutex> lk(c->hmu);  // the pipeline and its staging are per ctx
  HostPipe& P = *c->pipe;
  if (!P.init) {
    // The H2D stream on a hardware queue of its own (a CU-masked stream): HIP maps the other
    // streams onto at most GPU_MAX_HW_QUEUES queues per priority, and when the H2D and the D2H
    // stream landed on one queue (it depends on what streams the process made before — in round
    // 6's bench sequence they did) each chunk's input copy waited for the previous chunk's D2H blit
    // kernel: 24.5 GiB/s instead of 31.8-34.7 (profiles/r06jkmn_stream_queue_ab.jsonl: the H2D
    // stream at the least priority instead gave 34.3-34.7 but cost the 602 outer-message requests
    // on the normal-priority pool 20-25 %; every library stream at the greatest priority gave 34.3
    // and kept them, but shares the resident services' queues).  A CU-masked stream is blocking: a host-path call also
    // waits for work queued before it on the legacy null stream (it is synchronous anyway).
    // (the hardware has a finite number of queues: when a dedicated one cannot be had, an ordinary
    // library stream still works, only without the guarantee)
    const hipError_t prior = hipPeekAtLastError();
    if (cu_stream(&P.s[0]) != hipSuccess) {
      if (prior == hipSuccess) (void)hipGetLastError();  // clear our own error, never the caller's
      HIP_TRY(lib_stream(&P.s[0]));
    }
    HIP_TRY(lib_stream(&P.s[1]));
    HIP_TRY(lib_stream(&P.s[2]));
    for (int i = 0; i < 4; ++i) {
      HIP_TRY(hipEventCreateWithFlags(&P.in_ready[i], kOrderEvent));
      HIP_TRY(hipEventCreateWithFlags(&P.k_done[i], kOrderEvent));
      HIP_TRY(hipEventCreateWithFlags(&P.slot_free[i], hipEventDisableTiming));
    }
    P.init = true;
  }
  if (int e = wait_keys(c, P.s[1])) return e;
  if (!OCB && c->svc && nrec == 1 && len <= kSvcMaxLen)  // the resident service (opt-in)
    return svc_call<DEC>(c, *c->svc, out, in, nonces, len, status);
  if (nrec * (in_rec + out_rec) <= g_host_direct.load())
    return host_direct<DEC, OCB>(c, P, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, status);
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const bool in_pinned = in_rec && is_pinned(in), out_pinned = out_rec && is_pinned(out);
  // Device pitch = the user's stride when one flat DMA can move the chunk: inputs may carry
  // small gaps (read and ignored), outputs only when they are dense (a flat D2H would overwrite
  // the caller's bytes between records, e.g. the next record's nonce in the wire layout).
  // hipMemcpy2DAsync on host memory runs far below the flat-copy PCIe rate (measured round 1).
  const bool in_flat = in_pinned && (nrec == 1 || in_stride <= in_rec + 64);
  const bool out_flat = out_pinned && (nrec == 1 || out_stride == out_rec);
  const size_t ip = in_flat ? in_stride : up16(in_rec), op = out_flat ? out_stride : up16(out_rec);
  const bool n_flat = (nrec == 1 || nonce_stride <= 64) && is_pinned(nonces);
  const size_t npitch = n_flat ? nonce_stride : 16;
  const size_t NS = (size_t)g_host_slots.load();  // staging slots (chunks in flight)
  size_t chunk_b = g_host_chunk.load();
  if (!chunk_b) chunk_b = in_flat && out_flat && n_flat ? ((size_t)8 << 20) : ((size_t)16 << 20);
  const size_t per = std::max<size_t>(1, chunk_b / std::max<size_t>(std::max(ip, op), 16));
  // records per chunk: at most `per`, and the chunks of a batch equal — a short last chunk (e.g.
  // 1 012 of 65 536 x 1 KiB after four of 16 131) took the FLOW plan, whose one-workgroup-per-CU
  // kernel then waited for the CUs of the previous chunk's D2H, a blit kernel: 314 us for 1 MiB
  // (rocprofv3 --kernel-trace --memory-copy-trace, profiles/r06e_hostpipe_timeline.txt)
  const size_t K = (nrec + (nrec + per - 1) / per - 1) / ((nrec + per - 1) / per);
  // every region and slot 2 MiB aligned (DMA into regions that straddle 2 MiB boundaries ran
  // 20.6 instead of 33 GiB/s in some allocation histories, tools/host_calls.py)
  auto up2m = [](size_t x) { return (x + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1); };
  // kernel workspace of its own per slot (never the context's scratch, which device-resident
  // calls on caller streams may hold): the larger of a full chunk's and the last chunk's
  auto ws_for = [&](size_t nr) -> size_t {
    if (!nr) return 0;
    if (OCB) {
      const OcbPlan op_ = plan_ocb(c, len, nr);
      return (size_t)nr * op_.nchunks * 16 + nr * 16 + nr * 4;
    }
    return gcm_ws_bytes(c, plan_gcm(c, len, nr), nr);
  };
  // (Measured, not taken, round 6: chunks ramping K/8, K/4, K/2 up and back down around the 16 MiB
  // ones, to shorten the pipeline's fill and drain — 33.0-33.7 GiB/s with or without, two
  // alternated rounds on one box, profiles/r06c_host_ramp.jsonl.)
  const size_t ws_b = up16(std::max(ws_for(K), ws_for(nrec - (nrec - 1) / K * K)));
  const size_t in_b = up2m(ip * K), out_b = up2m(op * K), n_b = up16(npitch * K), st_b = up16(4 * K);
  const size_t slot_b = up2m(in_b + out_b + n_b + st_b + ws_b);
  if (P.cap < slot_b || P.ns < NS) {
    for (auto& st : P.s) HIP_TRY(hipStreamSynchronize(st));
    if (P.dsig_init)  // (calls return with no copy in flight; this only guards the free below)
      for (int i = 0; i < 4; ++i) (void)sig_wait_done(P.dsig[i]), (void)sig_wait_done(P.hsig[i]);
    if (P.buf) (void)hipFree(P.buf);
    if (P.hbuf) (void)hipHostFree(P.hbuf);
    P.buf = P.hbuf = nullptr;
    P.cap = 0;
    if (hipMalloc(&P.buf, NS * slot_b + ((size_t)2 << 20)) != hipSuccess) return fail(CMPI_ENOMEM, "hipMalloc staging failed");
    if (hipHostMalloc(&P.hbuf, NS * slot_b, hipHostMallocDefault) != hipSuccess) {
      (void)hipFree(P.buf);
      P.buf = nullptr;
      return fail(CMPI_ENOMEM, "hipHostMalloc staging failed");
    }
    P.cap = slot_b;
    P.ns = NS;
  }
  // page-locked nonces at a small stride: one H2D of the whole batch's nonces up front instead of
  // one small copy per chunk on the H2D stream (each ~10 us of latency plus its gap in front of
  // the next chunk's input copy, the stream that bounds the pipeline)
  const bool n_once = n_flat && nrec > K;
  if (n_once && P.dnon_cap < nrec * npitch) {
    for (auto& st : P.s) HIP_TRY(hipStreamSynchronize(st));
    if (P.dnon) (void)hipFree(P.dnon);
    P.dnon = nullptr;
    P.dnon_cap = 0;
    if (hipMalloc(&P.dnon, nrec * npitch) != hipSuccess) return fail(CMPI_ENOMEM, "hipMalloc nonces failed");
    P.dnon_cap = nrec * npitch;
  }
  if (DEC && P.hst_cap < nrec) {  // statuses land here by DMA, chunk by chunk
    for (auto& st : P.s) HIP_TRY(hipStreamSynchronize(st));
    if (P.hst) (void)hipHostFree(P.hst);
    P.hst = nullptr;
    P.hst_cap = 0;
    const size_t n = std::max<size_t>(nrec, 4096);
    if (hipHostMalloc((void**)&P.hst, 4 * n, hipHostMallocDefault) != hipSuccess)
      return fail(CMPI_ENOMEM, "hipHostMalloc status failed");
    P.hst_cap = n;
  }
  // Host-side waits only where the CPU touches a staging slot: packing pageable inputs (or
  // non-flat nonces) into it, unpacking pageable outputs from it.  With pinned buffers the
  // whole batch is enqueued at once and the three streams pipeline on events alone.
  const bool cpu_pack = (in_rec && !in_pinned) || !n_flat;
  const bool cpu_unpack = out_rec && !out_pinned;
  const size_t nchunks = (nrec + K - 1) / K;
  // the device addresses of the caller's page-locked outputs (and of the status array) for the
  // copy modes that write them without hipMemcpyAsync (g_host_out_direct)
  const int omode = g_host_out_direct.load();
  uint8_t* dout_all = out_rec && out_flat && omode ? (uint8_t*)pinned_dev_ptr(out) : nullptr;
  int32_t* dst_all = DEC && dout_all ? (int32_t*)pinned_dev_ptr(P.hst) : nullptr;
  if (DEC && !dst_all) dout_all = nullptr;
  static const bool dbg_sync = getenv("CMPI_DEBUG_SYNC") != nullptr;  // diagnose: sync + check each step
  auto step = [&](const char* what, size_t ci) -> int {
    if (!dbg_sync) return CMPI_OK;
    for (auto& st : P.s) {
      const hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) return fail(CMPI_EHIP, "%s (chunk %zu): %s", what, ci, hipGetErrorString(e));
    }
    return CMPI_OK;
  };
  auto layout = [&](int sl, uint8_t* base) {
    struct L {
      uint8_t *in, *out, *n, *ws;
      int32_t* st;
    } l;
    if (base == P.buf) base = reinterpret_cast<uint8_t*>(up2m(reinterpret_cast<uintptr_t>(base)));
    l.in = base + sl * slot_b;
    l.out = l.in + in_b;
    l.n = l.out + out_b;
    l.st = reinterpret_cast<int32_t*>(l.n + n_b);
    l.ws = l.n + n_b + st_b;
    return l;
  };
  // copy chunk ci's outputs from the pinned slot to the user's buffers (after its D2H)
  auto unpack = [&](size_t ci) -> int {
    const int sl = (int)(ci % NS);
    const size_t r0 = ci * K, nr = std::min(K, nrec - r0);
    HIP_TRY(hipEventSynchronize(P.slot_free[sl]));
    const auto h = layout(sl, P.hbuf);
    par_copy_records(out + r0 * out_stride, out_stride, h.out, op, out_rec, nr);
    return CMPI_OK;
  };
  // modes 4-5: D2H on an SDMA engine through HSA, issued by this thread once the chunk's kernel is
  // done; a slot is reused after its copy's signal reached 0
  const HsaAgents* ha = nullptr;
  uint8_t* sd_out = nullptr;
  int32_t* sd_st = nullptr;
  if (omode >= 4 && dout_all) {
    const HsaAgents& a = hsa_agents(c->device);
    if (a.ok) {
      if (!P.dsig_init) {
        for (int i = 0; i < 8; ++i)
          if (hsa_signal_create(0, 0, nullptr, i < 4 ? &P.dsig[i] : &P.hsig[i - 4]) != HSA_STATUS_SUCCESS) {
            for (int j = 0; j < i; ++j) (void)hsa_signal_destroy(j < 4 ? P.dsig[j] : P.hsig[j - 4]);
            return fail(CMPI_EHIP, "hsa_signal_create failed");
          }
        P.dsig_init = true;
      }
      ha = &a;
      sd_out = dout_all;
      sd_st = dst_all;
    }
  }
  if (omode != 1) dout_all = nullptr, dst_all = nullptr;  // mode 1 alone: the kernel writes them
  auto sdma_wait = [&](int sl) { return sig_wait_done(P.dsig[sl]) == 0; };
  // D2H of chunk ci by SDMA: wait (spinning) for its kernel, then one copy (open's statuses the
  // kernel wrote into the page-locked status array itself: a second copy per chunk cost ~10 us)
  auto sdma_d2h = [&](size_t ci, size_t r0, size_t nr) -> int {
    const int sl = (int)(ci % NS);
    const auto d = layout(sl, P.buf);
    hipError_t q;
    while ((q = hipEventQuery(P.k_done[sl])) == hipErrorNotReady) {
    }
    if (q != hipSuccess) return fail(CMPI_EHIP, "chunk %zu kernel: %s", ci, hipGetErrorString(q));
    hsa_signal_store_relaxed(P.dsig[sl], 1);
    if (sdma_copy(sd_out + r0 * out_stride, ha->cpu, d.out, ha->gpu, (nr - 1) * op + out_rec, 0, nullptr, P.dsig[sl],
                  ha->eng_d2h) != HSA_STATUS_SUCCESS) {
      hsa_signal_store_relaxed(P.dsig[sl], 0);  // nothing in flight on this slot
      return fail(CMPI_EHIP, "hsa_amd_memory_async_copy (chunk %zu) failed", ci);
    }
    return CMPI_OK;
  };
  // mode 5: both directions on SDMA engines through HSA, the host launching each chunk's kernel
  // when its input copy's signal reached 0 — no HIP event between the copies and the kernels (the
  // marker after each input copy held both the next copy and the kernel ~23 us, r06ag)
  uint8_t* in_d = ha && omode == 5 && in_flat && n_once ? (uint8_t*)pinned_dev_ptr(in) : nullptr;
  uint8_t* non_d = in_d ? (uint8_t*)pinned_dev_ptr(nonces) : nullptr;
  if (in_d && non_d) {
    auto sig_ok = [&](hsa_signal_t sg) { return sig_wait_done(sg) == 0; };
    // chunks of K records, the last one the remainder (measured and not taken, round 6: a ramp of
    // K/8, K/4, K/2 first to shorten the fill, and each chunk's nonces copied with it instead of
    // the batch's once — 33.9-37.4 against 37.1-37.5 GiB/s; each output copy split in 2 or 4
    // copies — 35.9 / 33.2 against 37.4; profiles/r06_hostpath_sweeps.jsonl)
    std::vector<size_t> cs{0};
    while (cs.back() < nrec) cs.push_back(std::min(nrec, cs.back() + K));
    const size_t nch = cs.size() - 1;
    auto issue_in = [&](size_t ci) -> int {
      const int sl = (int)(ci % NS);
      const size_t r0 = cs[ci], nr = cs[ci + 1] - cs[ci];
      const auto d = layout(sl, P.buf);
      const uint32_t ndep = ci >= NS ? 1u : 0u;  // chunk ci-NS's output copy has read the slot
      hsa_signal_store_relaxed(P.hsig[sl], ci == 0 ? 2 : 1);  // chunk 0: the batch's nonces too
      if (ci == 0 && sdma_copy(P.dnon, ha->gpu, non_d, ha->cpu, (nrec - 1) * npitch + 12, 0, nullptr, P.hsig[sl],
                               ha->eng_h2d) != HSA_STATUS_SUCCESS) {
        hsa_signal_store_relaxed(P.hsig[sl], 0);
        return fail(CMPI_EHIP, "hsa_amd_memory_async_copy (nonces) failed");
      }
      if (sdma_copy(d.in, ha->gpu, in_d + r0 * in_stride, ha->cpu, (nr - 1) * ip + in_rec, ndep, ndep ? &P.dsig[sl] : nullptr,
                    P.hsig[sl], ha->eng_h2d) != HSA_STATUS_SUCCESS) {
        hsa_signal_subtract_relaxed(P.hsig[sl], 1);
        return fail(CMPI_EHIP, "hsa_amd_memory_async_copy (chunk %zu input) failed", ci);
      }
      return CMPI_OK;
    };
    int rc = CMPI_OK;
    size_t ni = 0;  // chunks whose input copy has been issued
    for (; ni < std::min(NS, nch) && !rc; ++ni) rc = issue_in(ni);
    // one polling loop over both events that move the pipeline: a chunk's input landed (launch
    // its kernel) and a chunk's kernel finished (its output copy, then the input copy of the chunk
    // that takes the slot next, behind that output copy on the device)
    size_t kl = 0, dl = 0;  // next kernel to launch, next output copy to issue
    while (dl < nch && !rc) {
      if (kl < ni) {
        const int sl = (int)(kl % NS);
        const hsa_signal_value_t v = hsa_signal_load_scacquire(P.hsig[sl]);
        if (v < 0) {
          rc = fail(CMPI_EHIP, "chunk %zu input copy failed (signal %ld)", kl, (long)v);
          break;
        }
        if (v == 0) {
          const size_t r0 = cs[kl], nr = cs[kl + 1] - cs[kl];
          const auto d = layout(sl, P.buf);
          void* wsp = ws_b ? (void*)d.ws : nullptr;
          int32_t* ks = DEC ? sd_st + r0 : nullptr;  // open's statuses: the kernel writes them to the page-locked array
          rc = OCB ? ocb_batch<DEC>(c, d.out, op, d.in, ip, P.dnon + r0 * npitch, npitch, len, nr, ks, wsp, P.s[1])
                   : gcm_batch<DEC>(c, d.out, op, d.in, ip, P.dnon + r0 * npitch, npitch, len, nr, ks, wsp, P.s[1]);
          if (rc) break;
          HIP_TRY(hipEventRecord(P.k_done[sl], P.s[1]));
          ++kl;
        }
      }
      if (dl < kl) {
        const hipError_t q = hipEventQuery(P.k_done[dl % NS]);
        if (q == hipSuccess) {
          if ((rc = sdma_d2h(dl, cs[dl], cs[dl + 1] - cs[dl]))) break;
          if (dl + NS < nch) {
            if ((rc = issue_in(dl + NS))) break;
            ++ni;
          }
          ++dl;
        } else if (q != hipErrorNotReady) {
          rc = fail(CMPI_EHIP, "chunk %zu kernel: %s", dl, hipGetErrorString(q));
        }
      }
    }
    for (size_t i = 0; i < NS; ++i) {  // nothing of this call in flight on return (also after an error)
      if (!sig_ok(P.hsig[i]) && !rc) rc = fail(CMPI_EHIP, "input copy failed");
      if (!sig_ok(P.dsig[i]) && !rc) rc = fail(CMPI_EHIP, "output copy failed");
    }
    HIP_TRY(hipStreamSynchronize(P.s[1]));
    if (rc) return rc;
    if (DEC) {
      size_t bad = 0;
      for (size_t i = 0; i < nrec; ++i) bad += P.hst[i] == 0;
      if (status) memcpy(status, P.hst, 4 * nrec);
      if (bad) return fail(CMPI_EAUTH, "%zu of %zu records failed authentication", bad, nrec);
    }
    return CMPI_OK;
  }
  int rc = CMPI_OK;
  // (Measured and not taken, round 6: the H2D on the kernel's stream, 33.0 GiB/s; the D2H on it,
  // 30.6; all on one, 21.9; each stream on a hardware queue of its own, or the D2H confined to 16
  // CUs beside the kernel: unchanged — the blit D2H still held the next kernel.)
  hipStream_t sH = P.s[0], sK = P.s[1], sD = P.s[2];
  for (size_t ci = 0; ci < nchunks && !rc; ++ci) {
    const int sl = (int)(ci % NS);
    const size_t r0 = ci * K, nr = std::min(K, nrec - r0);
    const auto d = layout(sl, P.buf);
    const auto h = layout(sl, P.hbuf);
    // slot sl was last used by chunk ci-2: its H2D must have read the pinned inputs and its
    // outputs must have been unpacked (done at iteration ci-1) before we overwrite them
    if (ci >= NS && cpu_pack) HIP_TRY(hipEventSynchronize(P.in_ready[sl]));
    if (in_rec && !in_pinned) par_copy_records(h.in, ip, in + r0 * in_stride, in_stride, in_rec, nr);
    if (!n_flat)
      for (size_t i = 0; i < nr; ++i) memcpy(h.n + 16 * i, nonces + (r0 + i) * nonce_stride, 12);
    if (ci >= NS && ha) {  // chunk ci-NS's SDMA copy has read the slot
      if (!sdma_wait(sl)) {
        rc = fail(CMPI_EHIP, "chunk %zu output copy failed", ci - NS);
        break;
      }
    } else if (ci >= NS)
      HIP_TRY(hipStreamWaitEvent(sH, P.slot_free[sl], 0));
    // the batch's nonces ahead of chunk 0's records: the first kernel then starts when they land
    if (n_once && ci == 0) HIP_TRY(hipMemcpyAsync(P.dnon, nonces, (nrec - 1) * npitch + 12, hipMemcpyHostToDevice, sH));
    if (in_rec) {
      if (in_flat)
        HIP_TRY(hipMemcpyAsync(d.in, in + r0 * in_stride, (nr - 1) * ip + in_rec, hipMemcpyHostToDevice, sH));
      else if (in_pinned)
        HIP_TRY(hipMemcpy2DAsync(d.in, ip, in + r0 * in_stride, in_stride, in_rec, nr, hipMemcpyHostToDevice, sH));
      else
        HIP_TRY(hipMemcpyAsync(d.in, h.in, ip * nr, hipMemcpyHostToDevice, sH));
    }
    if (n_once) {
    } else if (n_flat)
      HIP_TRY(hipMemcpyAsync(d.n, nonces + r0 * nonce_stride, (nr - 1) * npitch + 12, hipMemcpyHostToDevice, sH));
    else
      HIP_TRY(hipMemcpyAsync(d.n, h.n, 16 * nr, hipMemcpyHostToDevice, sH));
    if ((rc = step("H2D", ci))) break;
    HIP_TRY(hipEventRecord(P.in_ready[sl], sH));
    HIP_TRY(hipStreamWaitEvent(sK, P.in_ready[sl], 0));
    void* wsp = ws_b ? (void*)d.ws : nullptr;
    const uint8_t* dn = n_once ? P.dnon + r0 * npitch : d.n;
    uint8_t* ko = dout_all ? dout_all + r0 * out_stride : d.out;
    int32_t* ks = DEC ? (dout_all ? dst_all + r0 : ha ? sd_st + r0 : d.st) : nullptr;
    if (OCB)
      rc = ocb_batch<DEC>(c, ko, op, d.in, ip, dn, npitch, len, nr, ks, wsp, sK);
    else
      rc = gcm_batch<DEC>(c, ko, op, d.in, ip, dn, npitch, len, nr, ks, wsp, sK);
    if (rc) break;
    if ((rc = step("kernel", ci))) break;
    if (dout_all) {  // nothing to copy back: the slot is free once the kernel has read it
      HIP_TRY(hipEventRecord(P.slot_free[sl], sK));
      continue;
    }
    HIP_TRY(hipEventRecord(P.k_done[sl], sK));
    if (ha) {  // the previous chunk's output by SDMA (its kernel ran while this chunk's input copied)
      if (ci >= 1 && (rc = sdma_d2h(ci - 1, (ci - 1) * K, K))) break;
      continue;
    }
    HIP_TRY(hipStreamWaitEvent(sD, P.k_done[sl], 0));
    if (out_rec) {
      if (out_flat)
        HIP_TRY(hipMemcpyAsync(out + r0 * out_stride, d.out, (nr - 1) * op + out_rec, hipMemcpyDeviceToHost, sD));
      else if (out_pinned)
        HIP_TRY(hipMemcpy2DAsync(out + r0 * out_stride, out_stride, d.out, op, out_rec, nr, hipMemcpyDeviceToHost, sD));
      else
        HIP_TRY(hipMemcpyAsync(h.out, d.out, op * nr, hipMemcpyDeviceToHost, sD));
    }
    if (DEC)
      HIP_TRY(hipMemcpyAsync(P.hst + r0, d.st, 4 * nr, hipMemcpyDeviceToHost, sD));
    if ((rc = step("D2H", ci))) break;
    HIP_TRY(hipEventRecord(P.slot_free[sl], sD));
    if (cpu_unpack && ci >= 1 && (rc = unpack(ci - 1))) break;  // overlaps the GPU work of chunk ci
  }
  if (ha) {
    if (!rc) rc = sdma_d2h(nchunks - 1, (nchunks - 1) * K, nrec - (nchunks - 1) * K);
    for (size_t i = 0; i < NS; ++i)  // every issued copy done (also after an error)
      if (!sdma_wait((int)i) && !rc) rc = fail(CMPI_EHIP, "output copy failed");
  }
  if (!rc && cpu_unpack) rc = unpack(nchunks - 1);
  for (auto& st : P.s) HIP_TRY(hipStreamSynchronize(st));
  if (rc) return rc;
  if (DEC) {
    size_t bad = 0;
    for (size_t i = 0; i < nrec; ++i) bad += P.hst[i] == 0;
    if (status) memcpy(status, P.hst, 4 * nrec);
    if (bad) return fail(CMPI_EAUTH, "%zu of %zu records failed authentication", bad, nrec);
  }
  return CMPI_OK;
}

std::atomic<int> g_ctr_wg_per_cu{2};  // cmpi_debug_set_ctr_wg_per_cu (co-residence experiments)

int ctr_launch(const cmpi_ctx* c, uint8_t* out, const uint8_t* in, size_t n, const uint8_t ctr[16],
                      void* stream) {
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  if (c->alg != CMPI_AES_128_CTR && c->alg != CMPI_AES_128_GCM && c->alg != CMPI_AES_128_ECB)
    return fail(CMPI_EINVAL, "ctx algorithm cannot run CTR");
  if (c->dev_keys) return fail(CMPI_EINVAL, "device-derived sub-key context supports GCM only");
  if (!ctr || !out) return fail(CMPI_EINVAL, "null argument");
  if (n == 0) return CMPI_OK;
  DeviceGuard dg(c->device);
  hipStream_t st = (hipStream_t)stream;
  cmpi::dev::CtrArgs a{};
  a.in = in;
  a.out = out;
  a.n = n;
  a.ctr_hi = cmpi::be64(ctr);
  a.ctr_lo = cmpi::be64(ctr + 8);
  a.te0 = c->dt->te0;
  a.rk = folded(c->rk);
  a.sched = kSched;
  const int wg_per_cu = g_ctr_wg_per_cu.load();
  a.nblk = (a.n + 15) / 16;
  const uint64_t blocks = (a.nblk + 1023) / 1024;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)c->ncu * (uint64_t)wg_per_cu));
  auto fn = in ? cmpi::dev::ctr_kernel<true> : cmpi::dev::ctr_kernel<false>;
  const int lds = 65536;
  int rc = set_lds_attr(reinterpret_cast<const void*>(fn), c->device, lds);
  if (rc) return rc;
  HIP_TRY(launch_k(fn, dim3(grid), dim3(1024), lds, st, a));
  return CMPI_OK;
}

// Stage host bytes into the ctx's device buffer at byte offset `pad`, run `fn(dev_in, dev_out)`
// on the internal stream, copy [pad, pad+n) back.  Serialised per ctx.
template <typename F>
int host_stream_op(const cmpi_ctx* c, uint8_t* out, const uint8_t* in, size_t n, unsigned pad, F fn) {
  DeviceGuard dg(c->device);
  std::unique_lock<std::mutex> lk(c->mu);
  if (!c->hstream) HIP_TRY(lib_stream(&c->hstream));
  const size_t span = ((size_t)pad + n + 15) & ~(size_t)15;
  int rc = ensure_buf((void**)&c->stage, &c->stage_cap, 2 * span);
  if (rc) return rc;
  uint8_t* d_in = c->stage;
  uint8_t* d_out = c->stage + span;
  HIP_TRY(hipMemcpyAsync(d_in + pad, in, n, hipMemcpyHostToDevice, c->hstream));
  rc = fn(d_in, d_out, span, c->hstream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, d_out + pad, n, hipMemcpyDeviceToHost, c->hstream));
  HIP_TRY(hipStreamSynchronize(c->hstream));
  return CMPI_OK;
}

}  // namespace

// ================================================================= exported C ABI
extern "C" {

const char* cmpi_version(void) { return "cmpi_aead 0.1 (gfx950)"; }
const char* cmpi_last_error(void) { return g_err.c_str(); }

int cmpi_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

cmpi_ctx* cmpi_ctx_new(int alg, const uint8_t* key, size_t key_len, size_t tag_len, int device) {
  if (!key || key_len != 16) {
    fail(CMPI_EINVAL, "key_len must be 16 (AES-128)");
    return nullptr;
  }
  if (!(tag_len == 0 || tag_len == 16)) {
    fail(CMPI_EINVAL, "tag_len must be 0 or 16");
    return nullptr;
  }
  if (alg < CMPI_AES_128_GCM || alg > CMPI_AES_128_ECB) {
    fail(CMPI_EINVAL, "unknown algorithm %d", alg);
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    fail(CMPI_ENODEV, "no HIP device %d (count %d)", device, ndev);
    return nullptr;
  }
  DeviceGuard dg(device);
  auto* c = new cmpi_ctx();
  c->alg = alg;
  c->device = device;
  memcpy(c->key, key, 16);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) c->ncu = prop.multiProcessorCount;
  cmpi::aes128_expand_words(key, c->rk.w);
  cmpi::aes128_dec_words(c->rk.w, c->drk.w);
  {
    uint8_t kn[16];
    size_t got = 0;
    while (got < sizeof kn) {
      const ssize_t r = getrandom(kn + got, sizeof kn - got, 0);
      if (r <= 0) {
        fail(CMPI_EHIP, "getrandom failed");
        delete c;
        return nullptr;
      }
      got += (size_t)r;
    }
    uint64_t c0;
    memcpy(&c->nprefix, kn, 4);
    memcpy(&c0, kn + 4, 8);
    c->nctr.store(c0);
    memset(kn, 0, sizeof kn);
  }
  uint32_t z[4] = {0, 0, 0, 0}, h[4];
  cmpi::aes128_encrypt_words_host(c->rk.w, z, h);  // H = E_K(0^128), L_* for OCB
  memcpy(c->H.b, h, 16);

  auto* ht = new DevTables();
  memcpy(ht->te0, cmpi::kAes.te0, sizeof ht->te0);
  memcpy(ht->td0, cmpi::kAes.td0, sizeof ht->td0);
  for (int x = 0; x < 256; ++x) ht->isb[x] = cmpi::kAes.inv_sbox[x];
  {
    const cmpi::dev::RoundKeys fk = folded(c->rk);  // same convention as the keysetup kernel
    memcpy(ht->keys, fk.w, sizeof fk.w);
  }
  memcpy(ht->keys + 48, c->H.b, 16);
  memcpy(ht->sqmat, sq_columns().data(), sizeof ht->sqmat);
  {
    Blk p = c->H;
    for (int i = 0; i < 32; ++i) {
      memcpy(ht->h2pow[i], p.b, 16);
      p = cmpi::gf_mul(p, p);
    }
  }
  if (alg == CMPI_AES_128_GCM) {
    const Blk H2 = cmpi::gf_mul(c->H, c->H), H4 = cmpi::gf_mul(H2, H2);
    cmpi::build_byte_table(c->H, reinterpret_cast<Blk*>(ht->htab[0]));
    cmpi::build_byte_table(H2, reinterpret_cast<Blk*>(ht->htab[1]));
    cmpi::build_byte_table(H4, reinterpret_cast<Blk*>(ht->htab[2]));
    for (uint32_t f = 0; f < cmpi::dev::kFlowNib; ++f)
      cmpi::build_nibble_table(cmpi::gf_pow(c->H, cmpi::dev::flow_nib_exp(f)), reinterpret_cast<Blk*>(ht->fnib[f]));
  }
  if (alg == CMPI_AES_128_OCB) {
    // RFC 7253 §4.1: L_* = E_K(0), L_$ = double(L_*), L_0 = double(L_$), L_i = double(L_{i-1})
    auto dbl = [](const uint8_t* in, uint8_t* o) {
      const uint8_t carry = in[0] >> 7;
      for (int i = 0; i < 15; ++i) o[i] = (uint8_t)((in[i] << 1) | (in[i + 1] >> 7));
      o[15] = (uint8_t)((in[15] << 1) ^ (carry ? 0x87 : 0));
    };
    memcpy(ht->ltab[0], c->H.b, 16);
    for (int i = 1; i < 66; ++i) dbl(ht->ltab[i - 1], ht->ltab[i]);
  }
  if (hipMalloc(&c->dt, sizeof(DevTables)) != hipSuccess) {
    fail(CMPI_ENOMEM, "hipMalloc tables failed");
    delete ht;
    delete c;
    return nullptr;
  }
  hipError_t e = hipMemcpy(c->dt, ht, sizeof(DevTables), hipMemcpyHostToDevice);
  delete ht;
  if (e != hipSuccess) {
    fail(CMPI_EHIP, "hipMemcpy tables: %s", hipGetErrorString(e));
    (void)hipFree(c->dt);
    delete c;
    return nullptr;
  }
  return c;
}

void cmpi_ctx_free(cmpi_ctx* c) {
  if (!c) return;
  DeviceGuard dg(c->device);
  {
    std::lock_guard<std::mutex> hl(c->hmu);
    (void)svc_shutdown_locked(c);
  }
  // Drain the context's own streams and its scratch's last user (not the whole device: the
  // per-message 602 path frees contexts at message rate).  Device-resident calls the caller
  // enqueued on its own streams must be complete or ordered before the free, as for any buffer
  // the caller releases (cmpi_aead.h); hipFree itself does not return memory still in use.
  if (c->pipe && c->pipe->init)
    for (auto& ps : c->pipe->s) (void)hipStreamSynchronize(ps);
  if (c->hstream) (void)hipStreamSynchronize(c->hstream);
  if (c->scratch_used) (void)hipEventSynchronize(c->scratch_ev);
  if (c->scratch_ev) (void)hipEventDestroy(c->scratch_ev);
  if (c->key_ev) {
    (void)hipEventSynchronize(c->key_ev);
    (void)hipEventDestroy(c->key_ev);
  }
  wipe_dev(c->scratch, c->scratch_cap);  // segment / chunk partials
  wipe_dev(c->stage, c->stage_cap);
  wipe_dev(c->dt, sizeof(DevTables));  // round keys, H, GHASH tables
  wipe_chw(c->chw);                     // (waits for the memsets above too)
  wipe_map(c->mj);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->stage) (void)hipFree(c->stage);
  if (c->hstream) (void)hipStreamDestroy(c->hstream);
  if (c->pipe) {
    HostPipe& P = *c->pipe;
    if (P.init) {
      for (auto& st : P.s) (void)hipStreamDestroy(st);
      for (int i = 0; i < 4; ++i) {
        (void)hipEventDestroy(P.in_ready[i]);
        (void)hipEventDestroy(P.k_done[i]);
        (void)hipEventDestroy(P.slot_free[i]);
      }
    }
    if (P.buf) (void)hipFree(P.buf);
    if (P.dnon) (void)hipFree(P.dnon);
    if (P.hbuf) (void)hipHostFree(P.hbuf);
    if (P.hst) (void)hipHostFree(P.hst);
    if (P.dbounce) (void)hipHostFree(P.dbounce);
    if (P.hflag) (void)hipHostFree(P.hflag);
    if (P.dsig_init) {  // (every call waits for its copies; a copy is never left to outlive the staging)
      for (auto& sg : P.dsig) (void)sig_wait_done(sg), (void)hsa_signal_destroy(sg);
      for (auto& sg : P.hsig) (void)sig_wait_done(sg), (void)hsa_signal_destroy(sg);
    }
  }
  if (c->dt) (void)hipFree(c->dt);
  memset(c->key, 0, 16);
  memset(&c->rk, 0, sizeof c->rk);
  memset(&c->drk, 0, sizeof c->drk);
  memset(&c->H, 0, sizeof c->H);
  delete c;
}

int cmpi_ctx_device(const cmpi_ctx* c) { return c ? c->device : -1; }

int cmpi_host_register(void* ptr, size_t bytes) {
  if (!ptr || !bytes) return fail(CMPI_EINVAL, "null/empty buffer");
  HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
  return CMPI_OK;
}

int cmpi_host_unregister(void* ptr) {
  if (!ptr) return fail(CMPI_EINVAL, "null buffer");
  HIP_TRY(hipHostUnregister(ptr));
  return CMPI_OK;
}

void cmpi_debug_set_host_chunk(size_t bytes) { g_host_chunk.store(bytes); }

void cmpi_debug_force_plan(int lanes_per_record, uint32_t segments) {
  g_force_L.store(lanes_per_record == 1 || lanes_per_record == 2 || lanes_per_record == 4 ? lanes_per_record : 0);
  g_force_nseg.store(segments);
}

void cmpi_debug_set_host_direct(size_t bytes) { g_host_direct.store(bytes); }
void cmpi_debug_set_host_out_direct(int mode) { g_host_out_direct.store(mode == 0 || mode == 1 || mode == 4 || mode == 5 ? mode : 5); }
void cmpi_debug_set_host_slots(int slots) { g_host_slots.store(slots >= 2 && slots <= 4 ? (size_t)slots : 3); }
void cmpi_debug_set_stream_mode(int mode) { g_stream_mode.store(mode >= 0 && mode <= 2 ? mode : 0); }
void cmpi_debug_set_host_spin(int mode) { g_host_spin.store(mode >= 0 && mode <= 3 ? mode : 0); }

void cmpi_debug_set_flow_one_wg(int on) { g_flow_one_wg.store(on ? 1 : 0); }
void cmpi_debug_set_svc_ls_min(int ls) { g_svc_ls_min.store(ls >= 0 && ls <= 3 ? ls : 0); }
void cmpi_debug_set_svc_fake_stuck(int on) { g_svc_fake_stuck.store(on ? 1 : 0); }
void cmpi_debug_set_lane_pair(int on) { g_lane_pair.store(on >= 1 && on <= 4 ? on : 0); }
void cmpi_debug_set_flow_threads(int threads) { g_flow_nt.store(threads == 512 || threads == 1024 ? threads : 0); }
void cmpi_debug_set_ctr_wg_per_cu(int n) { g_ctr_wg_per_cu.store(n >= 1 && n <= 2 ? n : 2); }

// Timing events without the system-scope release fence (hipEventDisableSystemFence): a default
// event's fence writes back and invalidates the caches and leaves a ~6 us bubble before the
// next launch — the bench times kernels with these instead.
int cmpi_debug_copy(void* dst, const void* src, size_t n, void* stream) {
  if (!dst || !src || n % 16 || ((uintptr_t)dst | (uintptr_t)src) % 16) return fail(CMPI_EINVAL, "copy: n % 16 / alignment");
  if (n == 0) return CMPI_OK;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  int ncu = 256;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
  const uint64_t nv = n / 16u;
  const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((nv + 255u) / 256u, (uint64_t)ncu * 4u));
  HIP_TRY(launch_k(cmpi::dev::copy16_kernel, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream,
                   reinterpret_cast<u32x4*>(dst), reinterpret_cast<const u32x4*>(src), nv));
  return CMPI_OK;
}

void* cmpi_debug_event_new(void) {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}
int cmpi_debug_event_record(void* ev, void* stream) {
  return hipEventRecord((hipEvent_t)ev, (hipStream_t)stream) == hipSuccess ? CMPI_OK : CMPI_EHIP;
}
float cmpi_debug_event_ms(void* a, void* b) {
  float ms = -1.0f;
  if (hipEventElapsedTime(&ms, (hipEvent_t)a, (hipEvent_t)b) != hipSuccess) return -1.0f;
  return ms;
}
void cmpi_debug_event_free(void* ev) {
  if (ev) (void)hipEventDestroy((hipEvent_t)ev);
}
void cmpi_debug_time_next_launch(void* start_ev, void* stop_ev) {
  t_time_start = (hipEvent_t)start_ev;
  t_time_stop = (hipEvent_t)stop_ev;
}
#if CMPI_TOOLS
void cmpi_debug_set_wide_probe(void* buf) { g_wide_probe.store(reinterpret_cast<uint64_t*>(buf)); }
// device buffer of 8 x 32 uint64 (service_kernels.hpp SVC_STAMP); taken by the next service launch
void cmpi_debug_set_svc_probe(void* buf) { g_svc_probe.store(reinterpret_cast<uint64_t*>(buf)); }
#endif

void cmpi_debug_force_wide(int mode, uint32_t steps) {
  g_force_wide.store(mode > 0 ? 1 : (mode < 0 ? -1 : 0));
  g_force_S.store(steps);
}

int cmpi_debug_gcm_plan(const cmpi_ctx* c, size_t len, size_t nrec, uint32_t out[4]) {
  if (!c || !out) return fail(CMPI_EINVAL, "null argument");
  const GcmPlan p = plan_gcm(c, len, nrec);
  out[0] = (uint32_t)p.L;
  out[1] = p.nseg;
  out[2] = p.G;
  out[3] = p.r0;
  return CMPI_OK;
}

size_t cmpi_gcm_workspace_size(const cmpi_ctx* c, size_t len, size_t nrec) {
  if (!c) return 0;
  return gcm_ws_bytes(c, plan_gcm(c, len, nrec), nrec);
}

int cmpi_gcm_seal_batch(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                        const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, void* workspace,
                        void* stream) {
  return gcm_batch<false>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, nullptr, workspace,
                          stream);
}

int cmpi_gcm_open_batch(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                        const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status,
                        void* workspace, void* stream) {
  return gcm_batch<true>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, status, workspace,
                         stream);
}

int cmpi_gcm_seal_batch_fresh(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in,
                              size_t in_stride, uint8_t* nonce_out, size_t nonce_stride, size_t len, size_t nrec,
                              void* workspace, void* stream) {
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  if (nrec == 0) return CMPI_OK;
  if (!nonce_out) return fail(CMPI_EINVAL, "null nonce_out");
  if (nrec > 1 && nonce_stride < 12) return fail(CMPI_EINVAL, "nonce_stride < 12");
  // nonce_r = prefix || BE64(base + r): the seal kernel makes and writes them itself (one launch,
  // where round 4 ran a DRBG kernel first: 4.6 us per naive-collective seal)
  const uint64_t base = const_cast<cmpi_ctx*>(c)->nctr.fetch_add(nrec);
  NonceSpec ns;
  ns.mode = 4;
  ns.fix[0] = c->nprefix;
  ns.fix[1] = (uint32_t)(base >> 32);
  ns.fix[2] = (uint32_t)base;
  return gcm_batch<false>(c, out, out_stride, in, in_stride, nonce_out, nonce_stride, len, nrec, nullptr, workspace,
                          stream, ns);
}

int cmpi_naive_seal_blocks(const cmpi_ctx* c, uint8_t* wire, const uint8_t* in, size_t n, size_t nblk,
                           void* workspace, void* stream) {
  if (!wire) return fail(CMPI_EINVAL, "null wire");
  return cmpi_gcm_seal_batch_fresh(c, wire + 12, n + 28, in, n, wire, n + 28, n, nblk, workspace, stream);
}

int cmpi_naive_open_blocks(const cmpi_ctx* c, uint8_t* out, const uint8_t* wire, size_t n, size_t nblk,
                           int32_t* status, void* workspace, void* stream) {
  if (!wire) return fail(CMPI_EINVAL, "null wire");
  return gcm_batch<true>(c, out, n, wire + 12, n + 28, wire, n + 28, n, nblk, status, workspace, stream);
}

int cmpi_gcm_seal_host(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                       const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec) {
  return aead_host<false, false>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, nullptr);
}

int cmpi_gcm_open_host(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                       const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status) {
  return aead_host<true, false>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, status);
}

size_t cmpi_ocb_workspace_size(const cmpi_ctx* c, size_t len, size_t nrec) {
  if (!c) return 0;
  const OcbPlan p = plan_ocb(c, len, nrec);
  return (size_t)nrec * p.nchunks * 16 + nrec * 16 + nrec * 4;
}

int cmpi_ocb_seal_batch(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                        const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, void* workspace,
                        void* stream) {
  return ocb_batch<false>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, nullptr, workspace,
                          stream);
}

int cmpi_ocb_open_batch(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                        const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status,
                        void* workspace, void* stream) {
  return ocb_batch<true>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, status, workspace,
                         stream);
}

int cmpi_ocb_seal_host(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                       const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec) {
  return aead_host<false, true>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, nullptr);
}

int cmpi_ocb_open_host(const cmpi_ctx* c, uint8_t* out, size_t out_stride, const uint8_t* in, size_t in_stride,
                       const uint8_t* nonces, size_t nonce_stride, size_t len, size_t nrec, int32_t* status) {
  return aead_host<true, true>(c, out, out_stride, in, in_stride, nonces, nonce_stride, len, nrec, status);
}

int cmpi_ctr_xor(const cmpi_ctx* c, uint8_t* out, const uint8_t* in, size_t n, const uint8_t ctr_block[16],
                 void* stream) {
  if (!in) return fail(CMPI_EINVAL, "null input");
  return ctr_launch(c, out, in, n, ctr_block, stream);
}

int cmpi_ctr_keystream(const cmpi_ctx* c, uint8_t* out, size_t nblocks, const uint8_t ctr_block[16], void* stream) {
  return ctr_launch(c, out, nullptr, nblocks * 16, ctr_block, stream);
}

int cmpi_ctr_xor_host(const cmpi_ctx* c, uint8_t* out, const uint8_t* in, size_t n, const uint8_t ctr_block[16],
                      unsigned skip) {
  if (!c || !out || !in || !ctr_block) return fail(CMPI_EINVAL, "null argument");
  if (skip > 15) return fail(CMPI_EINVAL, "skip must be 0..15");
  if (n == 0) return CMPI_OK;
  if (n + skip <= cmpi::dev::kSvcMaxStreamLen) {  // the context's message service, when started
    DeviceGuard dg(c->device);
    std::unique_lock<std::mutex> lk(c->hmu);
    if (c->svc) return svc_ctr_host(c, *c->svc, out, in, n, ctr_block, skip);
  }
  return host_stream_op(c, out, in, n, skip, [&](uint8_t* di, uint8_t* dout, size_t span, hipStream_t s) {
    return ctr_launch(c, dout, di, (size_t)skip + n, ctr_block, s);
  });
}

int cmpi_ecb_encrypt_host(const cmpi_ctx* c, uint8_t* out, const uint8_t* in, size_t nblocks) {
  if (!c || !out || !in) return fail(CMPI_EINVAL, "null argument");
  if (nblocks == 0) return CMPI_OK;
  if (nblocks * 16 <= cmpi::dev::kSvcMaxStreamLen && c->alg == CMPI_AES_128_ECB) {  // served, when started
    DeviceGuard dg(c->device);
    std::unique_lock<std::mutex> lk(c->hmu);
    if (c->svc) return svc_ctr_host(c, *c->svc, out, in, nblocks * 16, nullptr, 0, cmpi::dev::kSvcEcb);
  }
  return host_stream_op(c, out, in, nblocks * 16, 0, [&](uint8_t* di, uint8_t* dout, size_t span, hipStream_t s) {
    return cmpi_ecb_encrypt(c, dout, di, nblocks, s);
  });
}

void cmpi_iv_count(uint8_t iv[16], unsigned long cter) {
  uint32_t n = 16, c = (uint32_t)cter;  // uint32 accumulator exactly as send.c:1021-1029
  do {
    --n;
    c += iv[n];
    iv[n] = (uint8_t)c;
    c >>= 8;
  } while (n);
}

void cmpi_iv_count_out(uint8_t iv[16], unsigned long cter, const uint8_t in[16]) {
  uint32_t n = 16, c = (uint32_t)cter;  // send.c:1032-1041
  do {
    --n;
    c += in[n];
    iv[n] = (uint8_t)c;
    c >>= 8;
  } while (n);
}

int cmpi_ecb_encrypt(const cmpi_ctx* c, uint8_t* out, const uint8_t* in, size_t nblocks, void* stream) {
  if (!c) return fail(CMPI_EINVAL, "null ctx");
  if (c->dev_keys) return fail(CMPI_EINVAL, "device-derived sub-key context supports GCM only");
  if (!out || !in) return fail(CMPI_EINVAL, "null buffer");
  if (nblocks == 0) return CMPI_OK;
  DeviceGuard dg(c->device);
  cmpi::dev::EcbArgs a{};
  a.in = in;
  a.out = out;
  a.nblk = nblocks;
  a.te0 = c->dt->te0;
  a.rk = folded(c->rk);
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nblocks + 1023) / 1024, (uint64_t)c->ncu * 2));
  int rc = set_lds_attr(reinterpret_cast<const void*>(cmpi::dev::ecb_kernel), c->device, 65536);
  if (rc) return rc;
  HIP_TRY(launch_k(cmpi::dev::ecb_kernel, dim3(grid), dim3(1024), 65536, (hipStream_t)stream, a));
  return CMPI_OK;
}

int cmpi_ctx_rekey_subkey(cmpi_ctx* dst, const cmpi_ctx* base, const uint8_t v[16], void* stream) {
  if (!dst || !base || !v) return fail(CMPI_EINVAL, "null argument");
  if (dst->alg != CMPI_AES_128_GCM) return fail(CMPI_EINVAL, "destination ctx is not AES-128-GCM");
  if (base->dev_keys) return fail(CMPI_EINVAL, "base ctx must hold a host-known master key");
  if (dst->device != base->device) return fail(CMPI_EINVAL, "contexts on different devices");
  DeviceGuard dg(dst->device);
  cmpi::dev::KeysetupArgs a{};
  a.base = folded(base->rk);
  memcpy(a.v, v, 16);
  a.mode = 1;
  a.te0 = dst->dt->te0;
  a.sqmat = reinterpret_cast<const u32x4*>(dst->dt->sqmat[0]);
  a.keys = dst->dt->keys;
  a.h2pow = reinterpret_cast<u32x4*>(dst->dt->h2pow[0]);
  a.chains = reinterpret_cast<u32x4*>(dst->dt->chains[0]);
  cmpi::dev::TablesArgs ta{};
  ta.chains = a.chains;
  ta.htab = reinterpret_cast<u32x4*>(dst->dt->htab[0]);
  ta.fnib = reinterpret_cast<u32x4*>(dst->dt->fnib[0]);
  int rc = set_lds_attr(reinterpret_cast<const void*>(cmpi::dev::gcm_keysetup_kernel), dst->device, cmpi::dev::kKsLds);
  if (rc) return rc;
  {
    // The context's own streams (host pipeline, host-memory CTR/ECB) may still read the old
    // tables: drain them first.  Work the caller enqueued on other streams of its own must be
    // ordered before `stream` by the caller (cmpi_aead.h: derived contexts are stream-ordered).
    std::lock_guard<std::mutex> hl(dst->hmu);
    if (int e = svc_shutdown_locked(dst)) return e;  // a device-keyed context has no service
    if (dst->pipe && dst->pipe->init)
      for (auto& ps : dst->pipe->s) HIP_TRY(hipStreamSynchronize(ps));
    if (dst->hstream) HIP_TRY(hipStreamSynchronize(dst->hstream));
    if (dst->scratch_used) HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, dst->scratch_ev, 0));
  }
  {
    std::lock_guard<std::mutex> lk(dst->mu);
    wipe_chw(dst->chw);
    wipe_map(dst->mj);
    dst->dev_keys = true;
    memset(dst->key, 0, 16);
    memset(&dst->rk, 0, sizeof dst->rk);
    memset(&dst->drk, 0, sizeof dst->drk);
    memset(&dst->H, 0, sizeof dst->H);
  }
  HIP_TRY(launch_k(cmpi::dev::gcm_keysetup_kernel, dim3(1), dim3(256), cmpi::dev::kKsLds, (hipStream_t)stream, a));
  HIP_TRY(launch_k(cmpi::dev::gcm_tables_kernel, dim3((cmpi::dev::kTabEntries + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, ta));
  return record_keys(dst, (hipStream_t)stream);
}

// Re-key a context in place to a host-known key (no allocation, no host table build): the host
// expands the key and computes H = E_K(0) (what the kernel arguments and the host-built weights
// need), the key-setup kernel in mode 0 rebuilds every device table from K on `stream`.  The
// drop-in's context pool (cmpi_evp_shim.cpp) turns CryptMPI's per-message EVP_AEAD_CTX_new
// (send.c:588-599, recv.c:562-575) into this instead of an allocation + 450 KB upload.
int cmpi_ctx_rekey(cmpi_ctx* c, const uint8_t* key, size_t key_len, void* stream) {
  if (!c || !key) return fail(CMPI_EINVAL, "null argument");
  if (key_len != 16) return fail(CMPI_EINVAL, "key_len must be 16 (AES-128)");
  DeviceGuard dg(c->device);
  cmpi::dev::KeysetupArgs a{};
  memcpy(a.v, key, 16);
  a.mode = 0;
  a.te0 = c->dt->te0;
  a.sqmat = reinterpret_cast<const u32x4*>(c->dt->sqmat[0]);
  a.keys = c->dt->keys;
  a.h2pow = reinterpret_cast<u32x4*>(c->dt->h2pow[0]);
  a.chains = reinterpret_cast<u32x4*>(c->dt->chains[0]);
  cmpi::dev::TablesArgs ta{};
  ta.chains = a.chains;
  ta.htab = reinterpret_cast<u32x4*>(c->dt->htab[0]);
  ta.fnib = reinterpret_cast<u32x4*>(c->dt->fnib[0]);
  int rc = set_lds_attr(reinterpret_cast<const void*>(cmpi::dev::gcm_keysetup_kernel), c->device, cmpi::dev::kKsLds);
  if (rc) return rc;
  {
    std::lock_guard<std::mutex> hl(c->hmu);
    if (c->svc) {  // the service holds the old key and tables: the next message relaunches it
      if (int e = svc_stop_locked(*c->svc)) return e;
      svc_wipe(*c->svc);  // its chunk weights (powers of the old H), partials, last message
    }
    if (c->pipe && c->pipe->init)
      for (auto& ps : c->pipe->s) HIP_TRY(hipStreamSynchronize(ps));
    if (c->hstream) HIP_TRY(hipStreamSynchronize(c->hstream));
    if (c->scratch_used) HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, c->scratch_ev, 0));
  }
  std::lock_guard<std::mutex> lk(c->mu);
  wipe_chw(c->chw);
  wipe_map(c->mj);
  memcpy(c->key, key, 16);
  cmpi::aes128_expand_words(key, c->rk.w);
  cmpi::aes128_dec_words(c->rk.w, c->drk.w);
  uint32_t z[4] = {0, 0, 0, 0}, h[4];
  cmpi::aes128_encrypt_words_host(c->rk.w, z, h);
  memcpy(c->H.b, h, 16);
  c->dev_keys = false;
  HIP_TRY(launch_k(cmpi::dev::gcm_keysetup_kernel, dim3(1), dim3(256), cmpi::dev::kKsLds, (hipStream_t)stream, a));
  HIP_TRY(launch_k(cmpi::dev::gcm_tables_kernel, dim3((cmpi::dev::kTabEntries + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, ta));
  if (c->alg == CMPI_AES_128_OCB) {  // RFC 7253 L table from L_* = E_K(0) (host, 1 KiB)
    uint8_t lt[66][16];
    memcpy(lt[0], c->H.b, 16);
    for (int i = 1; i < 66; ++i) {
      const uint8_t carry = lt[i - 1][0] >> 7;
      for (int j = 0; j < 15; ++j) lt[i][j] = (uint8_t)((lt[i - 1][j] << 1) | (lt[i - 1][j + 1] >> 7));
      lt[i][15] = (uint8_t)((lt[i - 1][15] << 1) ^ (carry ? 0x87 : 0));
    }
    HIP_TRY(hipMemcpyAsync(c->dt->ltab, lt, sizeof lt, hipMemcpyHostToDevice, (hipStream_t)stream));
  }
  if (!stream) {
    HIP_TRY(hipStreamSynchronize(nullptr));  // NULL stream: synchronous re-key
    return CMPI_OK;
  }
  return record_keys(c, (hipStream_t)stream);
}

cmpi_ctx* cmpi_ctx_derive_subkey(const cmpi_ctx* base, const uint8_t v[16], void* stream) {
  if (!base || !v) {
    fail(CMPI_EINVAL, "null argument");
    return nullptr;
  }
  // a GCM context with placeholder keys (all-zero key), re-keyed on the device in stream order
  static const uint8_t zero[16] = {0};
  cmpi_ctx* c = cmpi_ctx_new(CMPI_AES_128_GCM, zero, 16, 0, base->device);
  if (!c) return nullptr;
  if (cmpi_ctx_rekey_subkey(c, base, v, stream) != CMPI_OK) {
    std::string e = g_err;
    cmpi_ctx_free(c);
    g_err = e;
    return nullptr;
  }
  return c;
}

cmpi_ctx* cmpi_ctx_new_subkey(const cmpi_ctx* base, const uint8_t v[16]) {
  cmpi_ctx* c = cmpi_ctx_derive_subkey(base, v, nullptr);
  if (!c) return nullptr;
  DeviceGuard dg(c->device);
  if (const hipError_t e = hipStreamSynchronize(nullptr); e != hipSuccess) {
    fail(CMPI_EHIP, "key setup failed: %s", hipGetErrorString(e));
    cmpi_ctx_free(c);
    return nullptr;
  }
  return c;
}

}  // extern "C"

#include "frame_host.hpp"
#include "ring_host.hpp"
#include "ctrmode_host.hpp"
#include "async_host.hpp"
#include "framed_host.hpp"
