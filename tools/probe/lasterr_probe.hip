// lasterr_probe.hip — how HIP's per-thread "last error" behaves on this ROCm (what the C ABI's
// error reporting may assume): does a later successful call clear a pending error, does a failed
// query overwrite it, what does hipLaunchKernel return with an error pending, and which pointer
// queries fail (and so set the last error) on pageable host memory.  One JSON object on stdout.
// Build: hipcc -O2 --offload-arch=gfx950 -o lasterr_probe lasterr_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 0) p[0] = 1;
}

__global__ void k_spin(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}

static const char* nm(hipError_t e) { return hipGetErrorName(e); }

int main() {
  printf("{");
  hipError_t r;
  (void)hipGetLastError();
  // 1. a caller-side error, then a successful call: is it still pending?
  r = hipSetDevice(9999);
  printf("\"setdevice_9999\": \"%s\", \"peek_after\": \"%s\"", nm(r), nm(hipPeekAtLastError()));
  int* d = nullptr;
  r = hipMalloc(&d, 64);
  printf(", \"malloc_ok\": \"%s\", \"peek_after_success\": \"%s\"", nm(r), nm(hipPeekAtLastError()));
  // 2. a launch with the error pending: its own return, and the pending state
  void* args[] = {&d};
  r = hipLaunchKernel((const void*)k_empty, dim3(1), dim3(64), args, 0, 0);
  printf(", \"launch_ret_with_pending\": \"%s\", \"peek_after_launch\": \"%s\"", nm(r), nm(hipPeekAtLastError()));
  // 3. a failing pointer query with the error pending: does it overwrite?
  char* pageable = (char*)malloc(4096);
  hipPointerAttribute_t at;
  r = hipPointerGetAttributes(&at, pageable);
  printf(", \"ptrattrs_pageable\": \"%s\", \"peek_after_query\": \"%s\"", nm(r), nm(hipPeekAtLastError()));
  r = hipGetLastError();
  printf(", \"getlast\": \"%s\", \"peek_after_get\": \"%s\"", nm(r), nm(hipPeekAtLastError()));
  // 4. clean state: which queries leave an error behind on pageable memory
  r = hipPointerGetAttributes(&at, pageable);
  printf(", \"clean_ptrattrs\": \"%s\", \"clean_peek1\": \"%s\"", nm(r), nm(hipGetLastError()));
  unsigned int mt = 12345;
  r = hipPointerGetAttribute(&mt, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE, (hipDeviceptr_t)pageable);
  printf(", \"clean_ptrattr_memtype\": \"%s\", \"memtype\": %u, \"clean_peek2\": \"%s\"", nm(r), mt,
         nm(hipGetLastError()));
  void* dp = nullptr;
  r = hipHostGetDevicePointer(&dp, pageable, 0);
  printf(", \"clean_hostgetdevptr\": \"%s\", \"clean_peek3\": \"%s\"", nm(r), nm(hipGetLastError()));
  unsigned int fl = 0;
  r = hipHostGetFlags(&fl, pageable);
  printf(", \"clean_hostgetflags\": \"%s\", \"clean_peek4\": \"%s\"", nm(r), nm(hipGetLastError()));
  // 5. pinned memory: the same queries
  char* pinned = nullptr;
  (void)hipHostMalloc((void**)&pinned, 4096, 0);
  r = hipPointerGetAttribute(&mt, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE, (hipDeviceptr_t)pinned);
  printf(", \"pinned_ptrattr_memtype\": \"%s\", \"pinned_memtype\": %u", nm(r), mt);
  r = hipPointerGetAttributes(&at, pinned);
  printf(", \"pinned_ptrattrs\": \"%s\", \"pinned_type\": %d", nm(r), (int)at.type);
  // 6. stream query on busy stream: does NotReady become the last error?
  hipStream_t s;
  (void)hipStreamCreate(&s);
  (void)hipGetLastError();
  r = hipStreamQuery(s);
  printf(", \"streamquery_idle\": \"%s\"", nm(r));
  void* sargs[] = {nullptr};
  long long cyc = 200000000LL;
  sargs[0] = &cyc;
  (void)hipLaunchKernel((const void*)k_spin, dim3(1), dim3(64), sargs, 0, s);
  r = hipStreamQuery(s);
  printf(", \"streamquery_busy\": \"%s\", \"peek_after_busy_query\": \"%s\"", nm(r), nm(hipPeekAtLastError()));
  (void)hipStreamSynchronize(s);
  (void)hipGetLastError();
  r = hipEventQuery(nullptr);
  printf(", \"eventquery_null\": \"%s\", \"peek_after_eventquery\": \"%s\"", nm(r), nm(hipGetLastError()));
  // 7. out-of-memory as the pending error, then a failing query: which one is reported?
  void* big = nullptr;
  r = hipMalloc(&big, (size_t)1 << 50);
  printf(", \"malloc_1PB\": \"%s\"", nm(r));
  r = hipPointerGetAttributes(&at, pageable);
  printf(", \"peek_oom_then_query\": \"%s\"", nm(hipPeekAtLastError()));
  (void)hipGetLastError();
  (void)hipDeviceSynchronize();
  printf(", \"final_peek\": \"%s\"}\n", nm(hipGetLastError()));
  return 0;
}
