// Doorbell probe (round 3): can the host post a message word into DEVICE memory that a resident
// kernel polls locally, and what does the host -> GPU -> host round trip cost against the
// page-locked host ring the message service polls over PCIe today?
//   mode 0: doorbell in page-locked host memory (hipHostMalloc), GPU polls it over PCIe
//   mode 1: doorbell in fine-grained device memory (hipExtMallocWithFlags finegrained), written
//           by the host through its mapping (if the runtime gives the host one)
// The kernel (one wave) spins on the doorbell word for seq = 1..N and answers each by writing
// seq into a page-locked host word; the host times post -> answer.  Every spin is bounded.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(3);                                                                 \
    }                                                                          \
  } while (0)

__global__ void pong(const uint32_t* bell, uint32_t* answer, uint32_t n, uint32_t* err) {
  if (threadIdx.x != 0) return;
  for (uint32_t s = 1; s <= n; ++s) {
    uint64_t spins = 0;
    while (__hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != s) {
      if (++spins > (1ull << 22)) {  // bounded: ~seconds
        err[0] = s;
        return;
      }
    }
    __hip_atomic_store(answer, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double run(int mode, uint32_t n) {
  uint32_t* bell = nullptr;
  if (mode == 0) CK(hipHostMalloc((void**)&bell, 4096, hipHostMallocCoherent));
  else CK(hipExtMallocWithFlags((void**)&bell, 4096, hipDeviceMallocFinegrained));
  uint32_t *answer = nullptr, *err = nullptr;
  CK(hipHostMalloc((void**)&answer, 4096, hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&err, 4096, hipHostMallocCoherent));
  CK(hipMemset(bell, 0, 4096));
  CK(hipDeviceSynchronize());
  uint32_t* hbell = bell;  // the host's address of the doorbell
  if (mode == 1) {
    hipPointerAttribute_t at{};
    CK(hipPointerGetAttributes(&at, bell));
    printf("{\"mode\": 1, \"device_ptr\": \"%p\", \"host_ptr\": \"%p\"}\n", (void*)bell, at.hostPointer);
    fflush(stdout);
    if (!at.hostPointer) {
      CK(hipFree(bell));
      return -1.0;
    }
    hbell = static_cast<uint32_t*>(at.hostPointer);
  }
  *answer = 0;
  *err = 0;
  hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, 0, bell, answer, n, err);
  CK(hipGetLastError());
  std::vector<double> us;
  volatile uint32_t* vb = hbell;
  volatile uint32_t* va = answer;
  for (uint32_t s = 1; s <= n; ++s) {
    auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(const_cast<uint32_t*>(vb), s, __ATOMIC_RELEASE);  // host store into the mapping
    __builtin_ia32_sfence();
    uint64_t spins = 0;
    while (*va != s && *err == 0 && ++spins < (1ull << 26)) {
    }
    auto t1 = std::chrono::steady_clock::now();
    if (*va != s) {
      fprintf(stderr, "mode %d: no answer at seq %u (err %u)\n", mode, s, *err);
      break;
    }
    us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  CK(hipDeviceSynchronize());
  std::sort(us.begin(), us.end());
  const double med = us.empty() ? -1.0 : us[us.size() / 2];
  printf("{\"mode\": %d, \"bell\": \"%s\", \"n\": %zu, \"round_trip_us_median\": %.3f, \"p10\": %.3f, \"p90\": %.3f}\n",
         mode, mode == 0 ? "page-locked host" : "fine-grained device", us.size(), med,
         us.empty() ? -1.0 : us[us.size() / 10], us.empty() ? -1.0 : us[us.size() * 9 / 10]);
  if (mode == 0) CK(hipHostFree(bell));
  else CK(hipFree(bell));
  CK(hipHostFree(answer));
  CK(hipHostFree(err));
  return med;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
  run(0, n);
  run(1, n);
  return 0;
}
