// Environment probe (not product code): what each HIP host call on ncclAllReduce's per-call path
// costs on this box -- pointer queries for the send / recv buffers, the capture check, the event
// record -- so the per-call host overhead can be budgeted before it is optimised.
// Build: hipcc -O2 -o tools/probe_host_calls tools/probe_host_calls.cpp
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

template <typename F>
static double per_call_us(F f, int n = 20000) {
  for (int i = 0; i < 100; ++i) f();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
}

int main() {
  CK(hipSetDevice(0));
  char* buf = nullptr;
  CK(hipMalloc((void**)&buf, 64 << 20));
  // a few more allocations so the runtime's pointer map is not trivially small
  void* others[64];
  for (auto& o : others) CK(hipMalloc(&o, 1 << 20));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  char* p = buf + 4096;
  printf("hipPointerGetAttributes      %.3f us\n", per_call_us([&] {
           hipPointerAttribute_t a;
           CK(hipPointerGetAttributes(&a, p));
         }));
  printf("hipMemGetAddressRange        %.3f us\n", per_call_us([&] {
           hipDeviceptr_t b = 0;
           size_t sz = 0;
           CK(hipMemGetAddressRange(&b, &sz, (hipDeviceptr_t)p));
         }));
  printf("hipPointerGetAttribute(ID)   %.3f us\n", per_call_us([&] {
           unsigned long long id = 0;
           CK(hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p));
         }));
  printf("hipStreamIsCapturing         %.3f us\n", per_call_us([&] {
           hipStreamCaptureStatus c;
           CK(hipStreamIsCapturing(st, &c));
         }));
  printf("hipGetDevice                 %.3f us\n", per_call_us([&] {
           int d;
           CK(hipGetDevice(&d));
         }));
  printf("hipEventRecord               %.3f us\n", per_call_us([&] { CK(hipEventRecord(ev, st)); }));
  printf("hipEventQuery (done)         %.3f us\n", per_call_us([&] { (void)hipEventQuery(ev); }));
  CK(hipStreamSynchronize(st));
  for (auto& o : others) CK(hipFree(o));
  CK(hipFree(buf));
  return 0;
}
