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
static bool g_mode_geo = false;  // "allocgeo": the alloc rounds with the persistent geometry sweep

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

// The persistent structure's knobs (interleaved batches): V vectors per lane per batch, DB = the
// next batch's loads issued before this one is stored (else one batch in flight per wave: the
// wave count hides the latency), PAUX = the peer stream's load bits (17 = sc0 sc1 as the read
// kernel's peer loads, 2 = nt).
template <int V, bool DB, int PAUX>
__global__ void __launch_bounds__(64) persist2(Streams s, unsigned long long nvec) {
  const int lane = threadIdx.x, w = blockIdx.x, P = gridDim.x;
  const unsigned long long B = 64ull * V, nb = nvec / B;
  auto rs = [&](const void* p) { return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000); };
  const auto r0 = rs(s.src[0]), r1 = rs(s.src[1]), w0 = rs(s.dst[0]), w1 = rs(s.dst[1]);
  v4u xa[V], ya[V], xb[V], yb[V];
  auto load = [&](v4u(&x)[V], v4u(&y)[V], unsigned long long k) {
    const unsigned base = (unsigned)(k * B * 16);
#pragma unroll
    for (int u = 0; u < V; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b128(r1, base + (u * 64 + lane) * 16, 0, PAUX);
#pragma unroll
    for (int u = 0; u < V; ++u) y[u] = __builtin_amdgcn_raw_buffer_load_b128(r0, base + (u * 64 + lane) * 16, 0, 2);
  };
  auto store = [&](v4u(&x)[V], v4u(&y)[V], unsigned long long k) {
    const unsigned base = (unsigned)(k * B * 16);
#pragma unroll
    for (int u = 0; u < V; ++u) y[u] += x[u];
#pragma unroll
    for (int u = 0; u < V; ++u) __builtin_amdgcn_raw_buffer_store_b128(y[u], w0, base + (u * 64 + lane) * 16, 0, 17);
#pragma unroll
    for (int u = 0; u < V; ++u) __builtin_amdgcn_raw_buffer_store_b128(y[u], w1, base + (u * 64 + lane) * 16, 0, 17);
  };
  unsigned long long k = w;
  if (k >= nb) return;
  if (!DB) {
    for (; k < nb; k += P) {
      load(xa, ya, k);
      store(xa, ya, k);
    }
    return;
  }
  // unconditional prefetch (the last batch again past the end), as split's loader: what remains
  // of the wait is the stores' share of vmcnt
  auto nxt = [&](unsigned long long kk) { return kk + P < nb ? kk + P : nb - 1; };
  load(xa, ya, k);
  for (;;) {
    load(xb, yb, nxt(k));
    store(xa, ya, k);
    if ((k += P) >= nb) break;
    load(xa, ya, nxt(k));
    store(xb, yb, k);
    if ((k += P) >= nb) break;
  }
}

// Between the grid and the persistent forms: each one-wave workgroup walks G consecutive batches
// of one vector per lane (one batch in flight) and exits (G = 1: mix2's grid); TICKET = P
// persistent waves that take groups of G batches in order from a device-scope counter (the
// dispatcher's order without the dispatcher).
template <int G, bool TICKET>
__global__ void __launch_bounds__(64) grouped(Streams s, unsigned long long nvec, unsigned* ticket) {
  const int lane = threadIdx.x;
  const unsigned long long nb = nvec / 64, ng = nb / G;
  auto rs = [&](const void* p) { return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000); };
  const auto r0 = rs(s.src[0]), r1 = rs(s.src[1]), w0 = rs(s.dst[0]), w1 = rs(s.dst[1]);
  auto group = [&](unsigned long long g) {
    for (int i = 0; i < G; ++i) {
      const unsigned off = (unsigned)(((g * G + i) * 64 + lane) * 16);
      v4u x = __builtin_amdgcn_raw_buffer_load_b128(r1, off, 0, 17);
      v4u y = __builtin_amdgcn_raw_buffer_load_b128(r0, off, 0, 2);
      y += x;
      __builtin_amdgcn_raw_buffer_store_b128(y, w0, off, 0, 17);
      __builtin_amdgcn_raw_buffer_store_b128(y, w1, off, 0, 17);
    }
  };
  if (!TICKET) {
    if (blockIdx.x < ng) group(blockIdx.x);
    return;
  }
  for (;;) {
    unsigned g = 0;
    if (lane == 0) g = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g = __shfl(g, 0);
    if (g >= ng) return;
    group(g);
  }
}

// Loads and stores in different waves: on gfx9 a wave's loads and stores share one counter
// (vmcnt), so a wave that stores and then waits for a later load also waits for its stores'
// acknowledgements (hipcc: vmcnt(0) in every loop that mixes them).  Here wave 0 of each
// two-wave workgroup only loads (next batch in flight while it folds this one) and hands the
// folded batch to wave 1 through a double-buffered LDS slot; wave 1 only stores, never waiting.
template <int V>
__global__ void __launch_bounds__(128) split(Streams s, unsigned long long nvec) {
  __shared__ v4u buf[2][V * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, P = gridDim.x;
  const unsigned long long B = 64ull * V, nb = nvec / B;
  auto rs = [&](const void* p) { return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000); };
  unsigned long long k = blockIdx.x;
  if (k >= nb) return;
  if (wave == 0) {
    const auto r0 = rs(s.src[0]), r1 = rs(s.src[1]);
    v4u xa[V], ya[V], xb[V], yb[V];
    auto load = [&](v4u(&x)[V], v4u(&y)[V], unsigned long long kk) {
      const unsigned base = (unsigned)(kk * B * 16);
#pragma unroll
      for (int u = 0; u < V; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b128(r1, base + (u * 64 + lane) * 16, 0, 17);
#pragma unroll
      for (int u = 0; u < V; ++u) y[u] = __builtin_amdgcn_raw_buffer_load_b128(r0, base + (u * 64 + lane) * 16, 0, 2);
    };
    auto hand = [&](v4u(&x)[V], v4u(&y)[V], int slot) {
#pragma unroll
      for (int u = 0; u < V; ++u) buf[slot][u * 64 + lane] = x[u] + y[u];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    // the prefetch is unconditional (the last batch again past the end): a conditional load
    // makes hipcc wait vmcnt(0) where the two paths join
    auto nxt = [&](unsigned long long kk) { return kk + P < nb ? kk + P : nb - 1; };
    load(xa, ya, k);
    for (int slot = 0;;) {
      load(xb, yb, nxt(k));
      hand(xa, ya, slot);
      slot ^= 1;
      if ((k += P) >= nb) break;
      load(xa, ya, nxt(k));
      hand(xb, yb, slot);
      slot ^= 1;
      if ((k += P) >= nb) break;
    }
  } else {
    const auto w0 = rs(s.dst[0]), w1 = rs(s.dst[1]);
    for (int slot = 0; k < nb; k += P, slot ^= 1) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const unsigned base = (unsigned)(k * B * 16);
      v4u y[V];
#pragma unroll
      for (int u = 0; u < V; ++u) y[u] = buf[slot][u * 64 + lane];
#pragma unroll
      for (int u = 0; u < V; ++u) __builtin_amdgcn_raw_buffer_store_b128(y[u], w0, base + (u * 64 + lane) * 16, 0, 17);
#pragma unroll
      for (int u = 0; u < V; ++u) __builtin_amdgcn_raw_buffer_store_b128(y[u], w1, base + (u * 64 + lane) * 16, 0, 17);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
}

template <int V>
void run_split(Streams s, unsigned long long nvec, int P) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((split<V>), dim3(P), dim3(128), 0, 0, s, nvec);
  CK(hipEventRecord(e0, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((split<V>), dim3(P), dim3(128), 0, 0, s, nvec);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)(nvec / (64ull * V) * 64ull * V) * 16 * 4;
  printf("split: %d workgroups of a load wave + a store wave (LDS hand-off), V=%d, 2R:2W: %.3f ms per launch, %.0f GB/s = %.1f %% of 8 TB/s\n",
         P, V, ms / it, bytes / (ms / it * 1e-3) / 1e9, bytes / (ms / it * 1e-3) / 8e12 * 100);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int G, bool TICKET>
void run_grouped(Streams s, unsigned long long nvec, int P, unsigned* ticket) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned grid = TICKET ? (unsigned)P : (unsigned)(nvec / 64 / G);
  auto launch = [&] {
    if (TICKET) CK(hipMemsetAsync(ticket, 0, 4, 0));
    hipLaunchKernelGGL((grouped<G, TICKET>), dim3(grid), dim3(64), 0, 0, s, nvec, ticket);
  };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(e0, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)(nvec / 64 / G * G * 64) * 16 * 4;
  if (TICKET)
    printf("ticket: %d persistent waves take groups of %d batches in order, 2R:2W: %.3f ms per launch, %.0f GB/s = %.1f %% of 8 TB/s\n",
           P, G, ms / it, bytes / (ms / it * 1e-3) / 1e9, bytes / (ms / it * 1e-3) / 8e12 * 100);
  else
    printf("grouped: %u one-wave workgroups of %d batches each, 2R:2W: %.3f ms per launch, %.0f GB/s = %.1f %% of 8 TB/s\n",
           grid, G, ms / it, bytes / (ms / it * 1e-3) / 1e9, bytes / (ms / it * 1e-3) / 8e12 * 100);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int V, bool DB, int PAUX>
void run_persist2(Streams s, unsigned long long nvec, int P) {
  if (g_case && strcmp(g_case, "p2") && strcmp(g_case, "g") && strcmp(g_case, "s")) return;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((persist2<V, DB, PAUX>), dim3(P), dim3(64), 0, 0, s, nvec);
  CK(hipEventRecord(e0, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((persist2<V, DB, PAUX>), dim3(P), dim3(64), 0, 0, s, nvec);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)(nvec / (64ull * V) * 64ull * V) * 16 * 4;
  printf("persistent interleaved, %d waves, V=%d, %s, peer loads %s, 2R:2W: %.3f ms per launch, %.0f GB/s = %.1f %% of 8 TB/s\n",
         P, V, DB ? "next batch prefetched" : "one batch in flight", PAUX == 17 ? "sc0 sc1" : "nt", ms / it,
         bytes / (ms / it * 1e-3) / 1e9, bytes / (ms / it * 1e-3) / 8e12 * 100);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
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
  if (g_case && !strcmp(g_case, "allocgeo")) {
    g_case = "alloc";
    g_mode_geo = true;
  }
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
  unsigned* ticket = nullptr;
  CK(hipMalloc((void**)&ticket, 4));
  CK(hipDeviceSynchronize());
  if (g_case && !strcmp(g_case, "offset")) {
    // one allocation; stream k (src0, src1, dst0, dst1) at k x (bytes + delta): the same physical
    // pages for every delta, only the streams' relative offsets change -- does the persistent
    // form's rate follow the relative placement of its streams?
    for (int k = 0; k < 4; ++k) {
      CK(hipFree((void*)s.src[k]));
      CK(hipFree(s.dst[k]));
    }
    char* big = nullptr;
    const size_t slack = 64ull << 20;
    CK(hipMalloc((void**)&big, 4 * (bytes + slack)));
    CK(hipMemset(big, 1, 4 * (bytes + slack)));
    const size_t deltas[] = {0, 4096, 65536, 256 << 10, 1 << 20, (2 << 20) + 65536, 8 << 20, (32 << 20) + 4096};
    for (size_t d : deltas) {
      Streams t;
      t.src[0] = (const v4u*)(big + 0 * (bytes + d));
      t.src[1] = (const v4u*)(big + 1 * (bytes + d));
      t.dst[0] = (v4u*)(big + 2 * (bytes + d));
      t.dst[1] = (v4u*)(big + 3 * (bytes + d));
      t.src[2] = t.src[3] = t.src[0];
      t.dst[2] = t.dst[3] = t.dst[0];
      printf("== delta %zu B\n", d);
      g_case = "22s";
      run<2, 2, 17>(t, nvec, "sc0 sc1");
      g_case = "p2";
      run_persist2<4, false, 17>(t, nvec, 512);
      run_persist2<12, true, 17>(t, nvec, 512);
    }
    return 0;
  }
  if (g_case && !strcmp(g_case, "alloc")) {
    // the same kernels on 8 fresh sets of allocations, each placed behind a spacer of another
    // size: does the rate depend on where the buffers landed (the 2-rank read kernel's bimodal
    // 740 / 900 us at 1 GiB)?
    for (int round = 0; round < 8; ++round) {
      for (int k = 0; k < 4; ++k) {
        CK(hipFree((void*)s.src[k]));
        CK(hipFree(s.dst[k]));
      }
      void* spacer = nullptr;
      const size_t sp = (size_t)((round * 37) % 251 + 1) << 20;
      CK(hipMalloc(&spacer, sp));
      for (int k = 0; k < 4; ++k) {
        v4u* p = nullptr;
        CK(hipMalloc((void**)&p, bytes));
        CK(hipMemset(p, k + 1, bytes));
        s.src[k] = p;
        CK(hipMalloc((void**)&s.dst[k], bytes));
        CK(hipMemset(s.dst[k], 0, bytes));
      }
      CK(hipDeviceSynchronize());
      printf("== allocation round %d (spacer %zu MiB, src0 %p dst0 %p)\n", round, sp >> 20, (void*)s.src[0], (void*)s.dst[0]);
      g_case = "22s";
      run<2, 2, 17>(s, nvec, "sc0 sc1");
      g_case = "p2";
      run_persist2<4, false, 17>(s, nvec, 512);
      run_persist2<4, true, 17>(s, nvec, 512);
      if (g_mode_geo) {  // which persistent geometry holds its rate on every placement?
        run_persist2<1, false, 17>(s, nvec, 1024);
        run_persist2<1, false, 17>(s, nvec, 2048);
        run_persist2<2, false, 17>(s, nvec, 512);
        run_persist2<2, false, 17>(s, nvec, 1024);
        run_persist2<4, false, 17>(s, nvec, 256);
        run_persist2<4, false, 17>(s, nvec, 1024);
        run_persist2<12, true, 17>(s, nvec, 512);
      }
      g_case = "alloc";
      CK(hipFree(spacer));
    }
    return 0;
  }
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
    if (g_case && (!strcmp(g_case, "pb") || !strcmp(g_case, "pi"))) {  // round-4 runs: profiles/r4_mix_probe.txt
      for (int P : {512, 1024, 2048}) {
        run_persist<12, true>(s, nvec, P);
        run_persist<12, false>(s, nvec, P);
      }
      run_persist<4, true>(s, nvec, 2048);
      run_persist<4, false>(s, nvec, 2048);
    }
    if (g_case && !strcmp(g_case, "s")) {
      for (int P : {512, 1024, 2048, 4096}) {
        run_split<2>(s, nvec, P);
        run_split<4>(s, nvec, P);
        run_split<8>(s, nvec, P);
      }
      run_persist2<4, false, 17>(s, nvec, 512);
      run_persist2<1, false, 17>(s, nvec, 2048);
      run_persist2<4, true, 17>(s, nvec, 1024);
      run_persist2<4, true, 17>(s, nvec, 2048);
      continue;
    }
    if (g_case && !strcmp(g_case, "g")) {
      run_grouped<1, false>(s, nvec, 0, ticket);
      run_grouped<4, false>(s, nvec, 0, ticket);
      run_grouped<16, false>(s, nvec, 0, ticket);
      run_grouped<64, false>(s, nvec, 0, ticket);
      run_grouped<256, false>(s, nvec, 0, ticket);
      for (int P : {1024, 2048, 4096}) {
        run_grouped<1, true>(s, nvec, P, ticket);
        run_grouped<4, true>(s, nvec, P, ticket);
        run_grouped<16, true>(s, nvec, P, ticket);
      }
      for (int P : {256, 512, 1024}) {
        run_persist2<1, false, 17>(s, nvec, P);
        run_persist2<4, false, 17>(s, nvec, P);
        run_persist2<8, false, 17>(s, nvec, P);
      }
      continue;
    }
    for (int P : {2048, 4096, 8192}) {
      run_persist2<1, false, 17>(s, nvec, P);
      run_persist2<2, false, 17>(s, nvec, P);
      run_persist2<4, false, 17>(s, nvec, P);
      run_persist2<1, true, 17>(s, nvec, P);
      run_persist2<2, true, 17>(s, nvec, P);
      run_persist2<4, true, 17>(s, nvec, P);
      run_persist2<2, true, 2>(s, nvec, P);
    }
  }
  return 0;
}
