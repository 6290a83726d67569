// Environment probe (not product code): HBM rate of a pure stream with R read streams and W
// write streams of 16-byte vectors (the shape of the all-reduce kernels without their
// protocol): local reduce = 2R:1W, push-form read kernel at n ranks = nR:nW (n = 2: 2R:2W),
// the ring's fused kernel ~ (3n-2)R:(3n-2)W.  One wave per workgroup, one vector per lane and
// stream (local_reduce_vec's exact grid).  Loads non-temporal; stores non-temporal or sc0 sc1.
//
// Usage: mix_probe [MiB per stream] [case]  -> one line per (R, W, store form); case = e.g. "22s"
// (R=2, W=2, sc0 sc1 stores) runs that one only (for counter passes), default all
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

struct Streams {
  const v4u* src[4];
  v4u* dst[4];
};

// buffer stores (32-bit offsets: streams < 4 GiB); the store form is the aux bits
template <int R, int W, int AUX>
__global__ void __launch_bounds__(64) mix2(Streams s, unsigned long long nvec) {
  const unsigned long long i = (unsigned long long)blockIdx.x * 64 + threadIdx.x;
  if (i >= nvec) return;
  v4u v = __builtin_nontemporal_load(s.src[0] + i);
#pragma unroll
  for (int r = 1; r < R; ++r) v += __builtin_nontemporal_load(s.src[r] + i);
#pragma unroll
  for (int w = 0; w < W; ++w) {
    auto rs = __builtin_amdgcn_make_buffer_rsrc(s.dst[w], (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (unsigned)(i * 16), 0, AUX);
  }
}

static const char* g_case = nullptr;

template <int R, int W, int AUX>
void run(Streams s, unsigned long long nvec, const char* form) {
  if (g_case) {
    char c[8];
    snprintf(c, sizeof c, "%d%d%c", R, W, AUX == 2 ? 'n' : 's');
    if (strcmp(c, g_case)) return;
  }
  const dim3 g((unsigned)((nvec + 63) / 64)), b(64);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((mix2<R, W, AUX>), g, b, 0, 0, s, nvec);
  CK(hipEventRecord(e0, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((mix2<R, W, AUX>), g, b, 0, 0, s, nvec);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)nvec * 16 * (R + W);
  printf("R=%d W=%d stores %-8s: %.3f ms per launch, %.0f GB/s = %.1f %% of 8 TB/s\n", R, W, form, ms / it,
         bytes / (ms / it * 1e-3) / 1e9, bytes / (ms / it * 1e-3) / 8e12 * 100);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const unsigned long long mib = argc > 1 ? strtoull(argv[1], nullptr, 0) : 512;
  const unsigned long long bytes = mib << 20, nvec = bytes / 16;
  if (argc > 2) g_case = argv[2];
  CK(hipSetDevice(0));
  Streams s;
  for (int k = 0; k < 4; ++k) {
    v4u* p = nullptr;
    CK(hipMalloc((void**)&p, bytes));
    CK(hipMemset(p, k + 1, bytes));
    s.src[k] = p;
    CK(hipMalloc((void**)&s.dst[k], bytes));
    CK(hipMemset(s.dst[k], 0, bytes));
  }
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 2; ++rep) {
    run<1, 1, 2>(s, nvec, "nt");
    run<1, 1, 17>(s, nvec, "sc0 sc1");
    run<2, 1, 2>(s, nvec, "nt");
    run<2, 1, 17>(s, nvec, "sc0 sc1");
    run<2, 2, 2>(s, nvec, "nt");
    run<2, 2, 17>(s, nvec, "sc0 sc1");
    run<4, 4, 2>(s, nvec, "nt");
    run<4, 4, 17>(s, nvec, "sc0 sc1");
    run<3, 1, 2>(s, nvec, "nt");
    run<1, 2, 17>(s, nvec, "sc0 sc1");
  }
  return 0;
}
