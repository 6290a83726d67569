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

// The read kernel's structure without its protocol (read_fold_all at n = 2: one peer stream and
// the local stream read, the result stored twice, V vectors per lane per batch, the next batch's
// loads issued before this one is stored): P persistent one-wave workgroups; BLOCKED = each wave
// walks its own contiguous 1/P of the streams (as a read pipeline walks its own slices), else the
// waves take batches round robin (batch k*P + w: all waves inside one window of memory).
template <int V, bool BLOCKED>
__global__ void __launch_bounds__(64) persist(Streams s, unsigned long long nvec) {
  const int lane = threadIdx.x, w = blockIdx.x, P = gridDim.x;
  const unsigned long long B = 64ull * V, nb = nvec / B, per = nb / P;
  auto rs = [&](const void* p) { return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000); };
  const auto r0 = rs(s.src[0]), r1 = rs(s.src[1]), w0 = rs(s.dst[0]), w1 = rs(s.dst[1]);
  auto bidx = [&](unsigned long long k) { return BLOCKED ? per * w + k : k * P + w; };
  v4u xa[V], ya[V], xb[V], yb[V];
  auto load = [&](v4u(&x)[V], v4u(&y)[V], unsigned long long k) {
    const unsigned base = (unsigned)(bidx(k) * B * 16);
#pragma unroll
    for (int u = 0; u < V; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b128(r1, base + (u * 64 + lane) * 16, 0, 17);
#pragma unroll
    for (int u = 0; u < V; ++u) y[u] = __builtin_amdgcn_raw_buffer_load_b128(r0, base + (u * 64 + lane) * 16, 0, 2);
  };
  auto store = [&](v4u(&x)[V], v4u(&y)[V], unsigned long long k) {
    const unsigned base = (unsigned)(bidx(k) * B * 16);
#pragma unroll
    for (int u = 0; u < V; ++u) y[u] += x[u];
#pragma unroll
    for (int u = 0; u < V; ++u) __builtin_amdgcn_raw_buffer_store_b128(y[u], w0, base + (u * 64 + lane) * 16, 0, 17);
#pragma unroll
    for (int u = 0; u < V; ++u) __builtin_amdgcn_raw_buffer_store_b128(y[u], w1, base + (u * 64 + lane) * 16, 0, 17);
  };
  if (per == 0) return;
  load(xa, ya, 0);
  for (unsigned long long k = 0;;) {
    if (k + 1 < per) load(xb, yb, k + 1);
    store(xa, ya, k);
    if (++k >= per) break;
    if (k + 1 < per) load(xa, ya, k + 1);
    store(xb, yb, k);
    if (++k >= per) break;
  }
}

template <int V, bool BLOCKED>
void run_persist(Streams s, unsigned long long nvec, int P) {
  if (g_case && strcmp(g_case, BLOCKED ? "pb" : "pi")) return;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((persist<V, BLOCKED>), dim3(P), dim3(64), 0, 0, s, nvec);
  CK(hipEventRecord(e0, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((persist<V, BLOCKED>), dim3(P), dim3(64), 0, 0, s, nvec);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const unsigned long long done = nvec / (64ull * V) / P * P * 64ull * V;  // whole batches per wave
  const double bytes = (double)done * 16 * 4;
  printf("persistent %s, %d waves, V=%d, 2R:2W (read kernel at n = 2): %.3f ms per launch, %.0f GB/s = %.1f %% of 8 TB/s\n",
         BLOCKED ? "blocked (each wave its own 1/P)" : "interleaved (batch k*P + w)", P, V, ms / it,
         bytes / (ms / it * 1e-3) / 1e9, bytes / (ms / it * 1e-3) / 8e12 * 100);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

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
    for (int P : {512, 1024, 2048}) {
      run_persist<12, true>(s, nvec, P);
      run_persist<12, false>(s, nvec, P);
    }
    run_persist<4, true>(s, nvec, 2048);
    run_persist<4, false>(s, nvec, 2048);
  }
  return 0;
}
