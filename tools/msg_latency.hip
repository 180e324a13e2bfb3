// Per-message latency breakdown at the EVP / 600 boundary, from C (no Python on the path):
// launch floor (empty kernel + blocking sync / stream polling / kernel-written host flag), the
// CPU cost of a launch and of the pointer queries, and the engine's single-message calls on device
// buffers and through the host API (pinned and pageable).  Medians over `iters` calls.
// Build: make -C tools msg_latency    Run: tools/msg_latency [iters]   (prints one JSON line)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <sched.h>

#include "../include/cmpi_aead.h"
#include "../include/cmpi_debug.h"
#include "../include/cmpi_ctrmode.h"
#include "../include/cmpi_ring.h"
#include "../include/cmpi_frame.h"
#include "../include/cmpi_async.h"
#include "../include/cmpi_service.h"

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)
#define CM(x)                                                                                  \
  do {                                                                                         \
    int r_ = (x);                                                                              \
    if (r_) {                                                                                  \
      fprintf(stderr, "%s:%d %s = %d (%s)\n", __FILE__, __LINE__, #x, r_, cmpi_last_error()); \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

__global__ void empty_kernel() {}

// Writes `seq` to a page-locked host word after a system-scope release (vector store).
__global__ void flag_kernel(unsigned* flag, unsigned seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Spins ~`us` microseconds on the 100 MHz wall clock, then optionally writes the host flag.
__global__ void busy_kernel(unsigned us, unsigned* flag, unsigned seq) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(1);
  __syncthreads();
  if (flag && threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Bind this process to the CPUs of the GPU's NUMA node that it may run on (as
// an MPI launcher's --bind-to numa does), before any page-locked allocation (first touch): from
// the far socket every served message pays ≈ 0.9 µs more per PCIe round trip (DESIGN.md §5 "Host
// NUMA placement").  CMPI_NUMA_BIND=0 keeps the inherited placement.  Returns the GPU's node
// (-1 unknown) and sets *bound to the number of CPUs bound (0: not bound).
static int bind_gpu_node(int dev, int* bound) {
  *bound = 0;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) != hipSuccess) return -1;
  for (char* q = bus; *q; ++q) *q = (char)tolower(*q);
  char path[160];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  int node = -1;
  if (!f) return -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  const char* env = getenv("CMPI_NUMA_BIND");
  if (node < 0 || (env && atoi(env) == 0)) return node;
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  if (!(f = fopen(path, "r"))) return node;
  char list[4096] = {0};
  const bool ok = fgets(list, sizeof list, f) != nullptr;
  fclose(f);
  if (!ok) return node;
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return node;
  for (char* tok = strtok(list, ",\n"); tok; tok = strtok(nullptr, ",\n")) {  // "a-b,c,..."
    int a = -1, b = -1;
    if (sscanf(tok, "%d-%d", &a, &b) < 2) b = a;
    for (int c = a; c >= 0 && c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) CPU_SET(c, &want);
  }
  const int n = CPU_COUNT(&want);
  if (n > 0 && sched_setaffinity(0, sizeof want, &want) == 0) *bound = n;
  return node;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median_us(int iters, const std::function<void()>& fn) {
  for (int i = 0; i < std::max(20, iters / 10); ++i) fn();
  std::vector<double> t(iters);
  for (int i = 0; i < iters; ++i) {
    const double a = now_us();
    fn();
    t[i] = now_us() - a;
  }
  std::nth_element(t.begin(), t.begin() + iters / 2, t.end());
  return t[iters / 2];
}

static void spin(hipStream_t s) {
  for (;;) {
    hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) CK(e);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  int numa_cpus = 0;
  const int numa_node = bind_gpu_node(0, &numa_cpus);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::string js = "{";
  auto put = [&](const char* k, double v) {
    char b[96];
    snprintf(b, sizeof b, "%s\"%s\": %.2f", js.size() > 1 ? ", " : "", k, v);
    js += b;
  };
  put("numa_gpu_node", numa_node);
  put("numa_bound_cpus", numa_cpus);  // 0: the inherited placement (not bound)
  put("empty_launch_sync_us", median_us(iters, [&] {
        empty_kernel<<<1, 64, 0, s>>>();
        CK(hipStreamSynchronize(s));
      }));
  put("empty_launch_query_spin_us", median_us(iters, [&] {
        empty_kernel<<<1, 64, 0, s>>>();
        spin(s);
      }));
  put("launch_cpu_us", median_us(iters, [&] { empty_kernel<<<1, 64, 0, s>>>(); }));
  CK(hipStreamSynchronize(s));
  unsigned* hflag;
  CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocDefault));
  *hflag = 0;
  unsigned* dflag;
  CK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
  unsigned seq = 0;
  put("flag_kernel_host_spin_us", median_us(iters, [&] {
        ++seq;
        flag_kernel<<<1, 64, 0, s>>>(dflag, seq);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) {
        }
      }));
  CK(hipStreamSynchronize(s));
  put("empty_launch_writevalue_host_spin_us", median_us(iters, [&] {
        ++seq;
        empty_kernel<<<1, 64, 0, s>>>();
        CK(hipStreamWriteValue32(s, dflag, seq, 0));
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) {
        }
      }));
  CK(hipStreamSynchronize(s));
  put("empty_then_flag_kernel_host_spin_us", median_us(iters, [&] {
        ++seq;
        empty_kernel<<<1, 64, 0, s>>>();
        flag_kernel<<<1, 64, 0, s>>>(dflag, seq);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) {
        }
      }));
  CK(hipStreamSynchronize(s));
  // a kernel that runs ~5 us (a single small message's seal), then each way of waiting for it
  put("busy5_sync_us", median_us(iters, [&] {
        busy_kernel<<<4, 256, 0, s>>>(5, nullptr, 0);
        CK(hipStreamSynchronize(s));
      }));
  put("busy5_query_spin_us", median_us(iters, [&] {
        busy_kernel<<<4, 256, 0, s>>>(5, nullptr, 0);
        spin(s);
      }));
  put("busy5_inkernel_flag_us", median_us(iters, [&] {
        ++seq;
        busy_kernel<<<1, 256, 0, s>>>(5, dflag, seq);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) {
        }
      }));
  CK(hipStreamSynchronize(s));
  put("busy5_writevalue_us", median_us(iters, [&] {
        ++seq;
        busy_kernel<<<4, 256, 0, s>>>(5, nullptr, 0);
        CK(hipStreamWriteValue32(s, dflag, seq, 0));
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) {
        }
      }));
  CK(hipStreamSynchronize(s));
  put("busy5_flag_kernel_us", median_us(iters, [&] {
        ++seq;
        busy_kernel<<<4, 256, 0, s>>>(5, nullptr, 0);
        flag_kernel<<<1, 64, 0, s>>>(dflag, seq);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) {
        }
      }));
  CK(hipStreamSynchronize(s));
  {  // the same two flag forms on a coherent (fine-grained) host word
    unsigned *hc_flag, *dc_flag;
    CK(hipHostMalloc((void**)&hc_flag, 64, hipHostMallocCoherent));
    *hc_flag = 0;
    CK(hipHostGetDevicePointer((void**)&dc_flag, hc_flag, 0));
    put("busy5_inkernel_flag_coherent_us", median_us(iters, [&] {
          ++seq;
          busy_kernel<<<1, 256, 0, s>>>(5, dc_flag, seq);
          while (__atomic_load_n(hc_flag, __ATOMIC_ACQUIRE) != seq) {
          }
        }));
    CK(hipStreamSynchronize(s));
    put("busy5_writevalue_coherent_us", median_us(iters, [&] {
          ++seq;
          busy_kernel<<<4, 256, 0, s>>>(5, nullptr, 0);
          CK(hipStreamWriteValue32(s, dc_flag, seq, 0));
          while (__atomic_load_n(hc_flag, __ATOMIC_ACQUIRE) != seq) {
          }
        }));
    CK(hipStreamSynchronize(s));
    CK(hipHostFree(hc_flag));
  }
  {
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    put("empty_launch_event_query_spin_us", median_us(iters, [&] {
          empty_kernel<<<1, 64, 0, s>>>();
          CK(hipEventRecord(ev, s));
          for (;;) {
            hipError_t e = hipEventQuery(ev);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) CK(e);
          }
        }));
    CK(hipEventDestroy(ev));
  }
  {
    hipPointerAttribute_t at;
    put("pointer_attributes_us", median_us(iters, [&] { (void)hipPointerGetAttributes(&at, hflag); }));
  }

  uint8_t key[16];
  for (int i = 0; i < 16; ++i) key[i] = (uint8_t)i;
  cmpi_ctx* c = cmpi_ctx_new(CMPI_AES_128_GCM, key, 16, 16, 0);
  if (!c) {
    fprintf(stderr, "cmpi_ctx_new: %s\n", cmpi_last_error());
    return 1;
  }
  // 1000 and 65000 B: ragged lengths (a partial last block)
  const size_t sizes[] = {1024, 4096, 65536, 1000, 65000};
  const char* names[] = {"1k", "4k", "64k", "1000b", "65000b"};
  uint8_t nonce[12] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12};
  for (int si = 0; si < 5; ++si) {
    const size_t n = sizes[si];
    uint8_t *dp, *dc, *db, *hp, *hc, *hb;
    CK(hipMalloc((void**)&dp, n));
    CK(hipMalloc((void**)&dc, n + 16));
    CK(hipMalloc((void**)&db, n));
    CK(hipMemset(dp, 7, n));
    CK(hipHostMalloc((void**)&hp, n, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&hc, n + 16, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&hb, n, hipHostMallocDefault));
    std::vector<uint8_t> pp(n), pc(n + 16), pb(n);
    for (size_t i = 0; i < n; ++i) hp[i] = pp[i] = (uint8_t)(i * 31 + 5);
    uint8_t* dn;
    CK(hipMalloc((void**)&dn, 16));
    CK(hipMemcpy(dn, nonce, 12, hipMemcpyHostToDevice));
    int32_t* dst;
    CK(hipMalloc((void**)&dst, 4));
    char k[96];
    snprintf(k, sizeof k, "dev_seal_%s_us", names[si]);
    put(k, median_us(iters, [&] {
          CM(cmpi_gcm_seal_batch(c, dc, n + 16, dp, n, dn, 12, n, 1, nullptr, s));
          spin(s);
        }));
    snprintf(k, sizeof k, "dev_open_%s_us", names[si]);
    put(k, median_us(iters, [&] {
          CM(cmpi_gcm_open_batch(c, db, n, dc, n + 16, dn, 12, n, 1, dst, nullptr, s));
          spin(s);
        }));
    const char* modes[] = {"sync", "writevalue", "flagkernel", "query"};
    for (int m = 0; m < 4; ++m) {
      cmpi_debug_set_host_spin(m);
      snprintf(k, sizeof k, "host_pinned_seal_%s_%s_us", names[si], modes[m]);
      put(k, median_us(iters, [&] { CM(cmpi_gcm_seal_host(c, hc, n + 16, hp, n, nonce, 12, n, 1)); }));
    }
    cmpi_debug_set_host_spin(0);
    snprintf(k, sizeof k, "host_pinned_open_%s_us", names[si]);
    int32_t st = 0;
    put(k, median_us(iters, [&] { CM(cmpi_gcm_open_host(c, hb, n, hc, n + 16, nonce, 12, n, 1, &st)); }));
    if (memcmp(hb, hp, n) || st != 1) {
      fprintf(stderr, "pinned round trip failed (%zu)\n", n);
      return 1;
    }
    snprintf(k, sizeof k, "host_pageable_seal_open_%s_us", names[si]);
    put(k, median_us(iters, [&] {
          CM(cmpi_gcm_seal_host(c, pc.data(), n + 16, pp.data(), n, nonce, 12, n, 1));
          CM(cmpi_gcm_open_host(c, pb.data(), n, pc.data(), n + 16, nonce, 12, n, 1, &st));
        }));
    if (memcmp(pb.data(), pp.data(), n) || memcmp(pc.data(), hc, n + 16)) {
      fprintf(stderr, "pageable round trip failed (%zu)\n", n);
      return 1;
    }
    // the same calls through the resident message service (include/cmpi_service.h)
    CM(cmpi_service_start(c, 0));
    snprintf(k, sizeof k, "svc_pinned_seal_%s_us", names[si]);
    put(k, median_us(iters, [&] { CM(cmpi_gcm_seal_host(c, hc, n + 16, hp, n, nonce, 12, n, 1)); }));
    snprintf(k, sizeof k, "svc_pinned_open_%s_us", names[si]);
    put(k, median_us(iters, [&] { CM(cmpi_gcm_open_host(c, hb, n, hc, n + 16, nonce, 12, n, 1, &st)); }));
    if (memcmp(hb, hp, n) || st != 1) {
      fprintf(stderr, "service pinned round trip failed (%zu)\n", n);
      return 1;
    }
    snprintf(k, sizeof k, "svc_pageable_seal_open_%s_us", names[si]);
    put(k, median_us(iters, [&] {
          CM(cmpi_gcm_seal_host(c, pc.data(), n + 16, pp.data(), n, nonce, 12, n, 1));
          CM(cmpi_gcm_open_host(c, pb.data(), n, pc.data(), n + 16, nonce, 12, n, 1, &st));
        }));
    if (memcmp(pb.data(), pp.data(), n) || memcmp(pc.data(), hc, n + 16)) {
      fprintf(stderr, "service pageable round trip failed (%zu)\n", n);
      return 1;
    }
    CM(cmpi_service_stop(c));
    CK(hipFree(dp));
    CK(hipFree(dc));
    CK(hipFree(db));
    CK(hipFree(dn));
    CK(hipFree(dst));
    CK(hipHostFree(hp));
    CK(hipHostFree(hc));
    CK(hipHostFree(hb));
  }
  cmpi_ctx_free(c);
  {  // 702 messages (send.c:1537-1731, recv.c:1107-1220), device-resident, 4 KiB and 1 KiB:
     // stream A from the mask ring (the sender's precompute refills it), receiver premask + XOR
    uint8_t key2[16];
    for (int i = 0; i < 16; ++i) key2[i] = (uint8_t)(i + 100);
    cmpi_ctx* cc = cmpi_ctx_new(CMPI_AES_128_CTR, key2, 16, 0, 0);
    if (!cc) {
      fprintf(stderr, "cmpi_ctx_new ctr: %s\n", cmpi_last_error());
      return 1;
    }
    uint8_t iv[32];
    for (int i = 0; i < 32; ++i) iv[i] = (uint8_t)(3 * i + 1);
    cmpi_702_sender* snd = cmpi_702_sender_new(cc, iv, (size_t)8 << 20, 8, s);
    if (!snd) {
      fprintf(stderr, "cmpi_702_sender_new: %s\n", cmpi_last_error());
      return 1;
    }
    for (size_t n : {(size_t)4096, (size_t)1024}) {
      uint8_t *dpt, *dct, *dbk, *dmask;
      CK(hipMalloc((void**)&dpt, n));
      CK(hipMalloc((void**)&dct, n));
      CK(hipMalloc((void**)&dbk, n));
      CK(hipMalloc((void**)&dmask, n + 1024));
      CK(hipMemset(dpt, 0x5a, n));
      uint8_t hdr[26];
      size_t ml = 0;
      auto msg = [&](bool precompute) {
        if (cmpi_702_send(snd, 0, dpt, n, hdr, dct, s) < 1) CM(-1);
        if (precompute) CM(cmpi_702_precompute(snd, n, 2, s) < 0);
        CM(cmpi_702_recv_premask(cc, iv, hdr, dmask, n + 1024, &ml, s));
        CM(cmpi_702_recv(cc, iv, hdr, dbk, n, dct, dmask, ml, s));
      };
      char k[96];
      const char* nm = n == 4096 ? "4k" : "1k";
      snprintf(k, sizeof k, "c702_%s_send_precompute_recv_spin_us", nm);
      put(k, median_us(iters, [&] {
            msg(true);
            spin(s);
          }));
      snprintf(k, sizeof k, "c702_%s_send_recv_spin_us", nm);
      int cnt = 0;
      put(k, median_us(iters, [&] {
            msg(false);
            // the ring is refilled every 256th message (outside the median: the ring never drains)
            if (++cnt % 256 == 0 && cmpi_702_precompute(snd, 65535, 512, s) < 0) CM(-1);
            spin(s);
          }));
      // the same with the host spinning on a page-locked word a one-wave kernel writes after the
      // message's kernels (the completion floor is 6 us there, 13 us with hipStreamQuery polling)
      auto flag_wait = [&] {
        ++seq;
        flag_kernel<<<1, 64, 0, s>>>(dflag, seq);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) {
        }
      };
      cnt = 0;
      snprintf(k, sizeof k, "c702_%s_send_premask_recv_flag_us", nm);
      put(k, median_us(iters, [&] {
            msg(false);
            if (++cnt % 256 == 0 && cmpi_702_precompute(snd, 65535, 512, s) < 0) CM(-1);
            flag_wait();
          }));
      cnt = 0;
      snprintf(k, sizeof k, "c702_%s_send_recv_nomask_flag_us", nm);  // payload landed first: direct CTR
      put(k, median_us(iters, [&] {
            if (cmpi_702_send(snd, 0, dpt, n, hdr, dct, s) < 1) CM(-1);
            CM(cmpi_702_recv(cc, iv, hdr, dbk, n, dct, nullptr, 0, s));
            if (++cnt % 256 == 0 && cmpi_702_precompute(snd, 65535, 512, s) < 0) CM(-1);
            flag_wait();
          }));
      cnt = 0;
      snprintf(k, sizeof k, "c702_%s_send_only_flag_us", nm);
      put(k, median_us(iters, [&] {
            if (cmpi_702_send(snd, 0, dpt, n, hdr, dct, s) < 1) CM(-1);
            if (++cnt % 256 == 0 && cmpi_702_precompute(snd, 65535, 512, s) < 0) CM(-1);
            flag_wait();
          }));
      // the kernels alone, each followed by the flag kernel: a 4 KiB XOR (cmpi_xor_bytes), a 4 KiB
      // CTR keystream XOR (cmpi_ctr_xor), and an event record between two flag kernels
      snprintf(k, sizeof k, "c702_%s_xor_kernel_flag_us", nm);
      put(k, median_us(iters, [&] {
            CM(cmpi_xor_bytes(dbk, dct, dpt, n, s));
            flag_wait();
          }));
      uint8_t ctr0[16] = {0};
      snprintf(k, sizeof k, "c702_%s_ctr_kernel_flag_us", nm);
      put(k, median_us(iters, [&] {
            CM(cmpi_ctr_xor(cc, dbk, dct, n, ctr0, s));
            flag_wait();
          }));
      snprintf(k, sizeof k, "c702_%s_two_ctr_kernels_flag_us", nm);
      put(k, median_us(iters, [&] {
            CM(cmpi_ctr_xor(cc, dbk, dct, n, ctr0, s));
            CM(cmpi_ctr_xor(cc, dmask, dct, n, ctr0, s));
            flag_wait();
          }));
      {
        hipEvent_t e1;
        CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming | hipEventReleaseToDevice));
        snprintf(k, sizeof k, "c702_%s_xor_event_flag_us", nm);
        put(k, median_us(iters, [&] {
              CM(cmpi_xor_bytes(dbk, dct, dpt, n, s));
              CK(hipEventRecord(e1, s));
              flag_wait();
            }));
        snprintf(k, sizeof k, "event_record_cpu_us");
        put(k, median_us(iters, [&] { CK(hipEventRecord(e1, s)); }));
        spin(s);
        CK(hipEventDestroy(e1));
      }
      // host CPU time of the calls alone (the stream drained every 64 calls, outside the median)
      cnt = 0;
      snprintf(k, sizeof k, "c702_%s_send_call_cpu_us", nm);
      put(k, median_us(iters, [&] {
            if (++cnt % 64 == 0) {
              if (cmpi_702_precompute(snd, 65535, 512, s) < 0) CM(-1);
              spin(s);
              return;
            }
            if (cmpi_702_send(snd, 0, dpt, n, hdr, dct, s) < 1) CM(-1);
          }));
      spin(s);
      cnt = 0;
      snprintf(k, sizeof k, "c702_%s_recv_direct_call_cpu_us", nm);
      put(k, median_us(iters, [&] {
            if (++cnt % 64 == 0) {
              spin(s);
              return;
            }
            CM(cmpi_702_recv(cc, iv, hdr, dbk, n, dct, nullptr, 0, s));
          }));
      spin(s);
      // throughput: 200 messages back to back, one wait at the end
      snprintf(k, sizeof k, "c702_%s_send_precompute_recv_pipelined_us", nm);
      put(k, median_us(std::max(20, iters / 50), [&] {
            for (int i = 0; i < 200; ++i) msg(true);
            spin(s);
          }) / 200.0);
      // the same messages through the CTR context's message service (cmpi_service_start on cc:
      // every op of <= 64 KiB runs on the resident kernel and is complete when the call returns,
      // so no flag kernel is needed)
      CM(cmpi_service_start(cc, 20000));
      cnt = 0;
      snprintf(k, sizeof k, "c702_%s_served_send_premask_recv_us", nm);
      put(k, median_us(iters, [&] {
            msg(false);
            if (++cnt % 256 == 0 && cmpi_702_precompute(snd, 65535, 512, s) < 0) CM(-1);
          }));
      cnt = 0;
      snprintf(k, sizeof k, "c702_%s_served_send_recv_nomask_us", nm);  // payload landed first: direct CTR
      put(k, median_us(iters, [&] {
            if (cmpi_702_send(snd, 0, dpt, n, hdr, dct, s) < 1) CM(-1);
            CM(cmpi_702_recv(cc, iv, hdr, dbk, n, dct, nullptr, 0, s));
            if (++cnt % 256 == 0 && cmpi_702_precompute(snd, 65535, 512, s) < 0) CM(-1);
          }));
      cnt = 0;
      snprintf(k, sizeof k, "c702_%s_served_send_only_us", nm);
      put(k, median_us(iters, [&] {
            if (cmpi_702_send(snd, 0, dpt, n, hdr, dct, s) < 1) CM(-1);
            if (++cnt % 256 == 0 && cmpi_702_precompute(snd, 65535, 512, s) < 0) CM(-1);
          }));
      // the receiver's path once the payload has landed: the XOR with the premade mask
      if (cmpi_702_send(snd, 0, dpt, n, hdr, dct, s) < 1) CM(-1);
      CM(cmpi_702_recv_premask(cc, iv, hdr, dmask, n + 1024, &ml, s));
      snprintf(k, sizeof k, "c702_%s_served_recv_mask_us", nm);
      put(k, median_us(iters, [&] { CM(cmpi_702_recv(cc, iv, hdr, dbk, n, dct, dmask, ml, s)); }));
      CM(cmpi_service_stop(cc));
      std::vector<uint8_t> a(n), b(n);
      CK(hipMemcpy(a.data(), dpt, n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), dbk, n, hipMemcpyDeviceToHost));
      if (memcmp(a.data(), b.data(), n) || hdr[4] != '0') {
        fprintf(stderr, "702 round trip failed (%zu, stream %c)\n", n, hdr[4]);
        return 1;
      }
      CK(hipFree(dpt));
      CK(hipFree(dct));
      CK(hipFree(dbk));
      CK(hipFree(dmask));
    }
    {  // EVP_EncryptUpdate on a CTR context through the shim = cmpi_ctr_xor_host on the MPI user
       // buffer: 4 KiB page-locked, a launch per call vs the context's resident service
      uint8_t *hin, *hout;
      CK(hipHostMalloc((void**)&hin, 4096, hipHostMallocDefault));
      CK(hipHostMalloc((void**)&hout, 4096, hipHostMallocDefault));
      memset(hin, 0x3c, 4096);
      uint8_t cb[16];
      for (int i = 0; i < 16; ++i) cb[i] = (uint8_t)(i * 5);
      put("ctr_host_4k_launch_us", median_us(iters, [&] { CM(cmpi_ctr_xor_host(cc, hout, hin, 4096, cb, 0)); }));
      CM(cmpi_service_start(cc, 20000));
      put("ctr_host_4k_served_us", median_us(iters, [&] { CM(cmpi_ctr_xor_host(cc, hout, hin, 4096, cb, 0)); }));
      std::vector<uint8_t> pg_in(4096, 0x3c), pg_out(4096);
      put("ctr_pageable_4k_served_us",
          median_us(iters, [&] { CM(cmpi_ctr_xor_host(cc, pg_out.data(), pg_in.data(), 4096, cb, 0)); }));
      CM(cmpi_service_stop(cc));
      put("ctr_pageable_4k_launch_us",
          median_us(iters, [&] { CM(cmpi_ctr_xor_host(cc, pg_out.data(), pg_in.data(), 4096, cb, 0)); }));
      if (memcmp(pg_out.data(), hout, 4096)) {
        fprintf(stderr, "ctr host served / launched outputs differ\n");
        return 1;
      }
      CK(hipHostFree(hin));
      CK(hipHostFree(hout));
      // the 602 sub-key derivation, EVP_EncryptUpdate(ctx_enc, K', V, 16) on an ECB context
      // (send.c:583), pageable 16 bytes: a launch per call vs the ECB context's service
      cmpi_ctx* ce = cmpi_ctx_new(CMPI_AES_128_ECB, key2, 16, 0, 0);
      uint8_t v16[16] = {1, 2, 3}, k16[16], k16b[16];
      put("ecb_16b_launch_us", median_us(iters, [&] { CM(cmpi_ecb_encrypt_host(ce, k16, v16, 1)); }));
      CM(cmpi_service_start(ce, 20000));
      put("ecb_16b_served_us", median_us(iters, [&] { CM(cmpi_ecb_encrypt_host(ce, k16b, v16, 1)); }));
      CM(cmpi_service_stop(ce));
      cmpi_ctx_free(ce);
      if (memcmp(k16, k16b, 16)) {
        fprintf(stderr, "ecb served / launched outputs differ\n");
        return 1;
      }
    }
    cmpi_702_sender_free(snd);
    cmpi_ctx_free(cc);
  }
  {  // 602: an 8 MiB message from / into page-locked memory, one request per outer message
     // (send.c:729-850, recv.c:679-809): CPU time of the 16 *_begin calls and the whole message
    uint8_t mkey[16];
    for (int i = 0; i < 16; ++i) mkey[i] = (uint8_t)(7 * i);
    cmpi_ctx* master = cmpi_ctx_new(CMPI_AES_128_GCM, mkey, 16, 16, 0);
    const uint32_t n = 8u << 20;
    cmpi_602_plan plan;
    CM(cmpi_602_plan_make(n, 8, 0, &plan));
    uint8_t rnd[16], hdr[25];
    for (int i = 0; i < 16; ++i) rnd[i] = (uint8_t)(i + 16);
    CM(cmpi_602_header(&plan, rnd, hdr));
    cmpi_ctx* seg = cmpi_ctx_derive_subkey(master, hdr + 4, s);
    if (!master || !seg) {
      fprintf(stderr, "602 contexts: %s\n", cmpi_last_error());
      return 1;
    }
    CK(hipStreamSynchronize(s));
    uint8_t *src, *wire, *back;
    CK(hipHostMalloc((void**)&src, n, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&wire, plan.wire_bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&back, n, hipHostMallocDefault));
    for (uint32_t i = 0; i < n; ++i) src[i] = (uint8_t)(i * 13 + 1);
    std::vector<cmpi_req*> rq(plan.outer);
    double begin_us = 0;
    auto seal_outer = [&] {
      const double a = now_us();
      for (uint32_t o = 0; o < plan.outer; ++o) CM(cmpi_602_seal_host_begin(seg, &plan, hdr, wire, src, o, 1, &rq[o]));
      begin_us = now_us() - a;
      CM(cmpi_waitall(rq.data(), rq.size()));
    };
    const int it602 = std::max(20, iters / 50);
    put("c602_8m_seal_per_outer_us", median_us(it602, seal_outer));
    put("c602_8m_seal_16_begins_cpu_us", begin_us);
    put("c602_8m_open_per_outer_us", median_us(it602, [&] {
          for (uint32_t o = 0; o < plan.outer; ++o) CM(cmpi_602_open_host_begin(seg, hdr, back, wire, o, 1, nullptr, &rq[o]));
          CM(cmpi_waitall(rq.data(), rq.size()));
        }));
    put("c602_8m_seal_whole_us", median_us(it602, [&] { CM(cmpi_602_seal_host(seg, &plan, hdr, wire, src)); }));
    if (memcmp(src, back, n)) {
      fprintf(stderr, "602 round trip failed\n");
      return 1;
    }
    CK(hipHostFree(src));
    CK(hipHostFree(wire));
    CK(hipHostFree(back));
    cmpi_ctx_free(seg);
    cmpi_ctx_free(master);
  }
  CK(hipHostFree(hflag));
  CK(hipStreamDestroy(s));
  printf("%s}\n", js.c_str());
  return 0;
}
