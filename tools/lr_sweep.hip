// Tuning sweep for the local-reduce (scatter-reduce element-wise) kernel: out = a + b over
// 1 GiB fp32, variants timed with hipEvents, interleaved rounds in one process
// (cdna_hip_programming.md s5.4 rule 24).  Not product code; the winner goes to kernels.hip.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

template <int U, int NTL, int NTS>
__global__ void gs(v4f* out, const v4f* a, const v4f* b, size_t nvec) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < nvec; base += stride * U) {
    v4f x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + (size_t)u * blockDim.x;
      if (i < nvec) {
        if (NTL) { x[u] = __builtin_nontemporal_load(a + i); y[u] = __builtin_nontemporal_load(b + i); }
        else { x[u] = a[i]; y[u] = b[i]; }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + (size_t)u * blockDim.x;
      if (i < nvec) {
        if (NTS) __builtin_nontemporal_store(x[u] + y[u], out + i);
        else out[i] = x[u] + y[u];
      }
    }
  }
}

// full tiles without bounds checks (nvec multiple of blockDim*U*grid handled by caller)
template <int U, int NTL, int NTS>
__global__ void gs_nochk(v4f* out, const v4f* a, const v4f* b, size_t nvec) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < nvec; base += stride) {
    v4f x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + (size_t)u * blockDim.x;
      if (NTL) { x[u] = __builtin_nontemporal_load(a + i); y[u] = __builtin_nontemporal_load(b + i); }
      else { x[u] = a[i]; y[u] = b[i]; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + (size_t)u * blockDim.x;
      if (NTS) __builtin_nontemporal_store(x[u] + y[u], out + i);
      else out[i] = x[u] + y[u];
    }
  }
}

template <int U>
__global__ void contig(v4f* out, const v4f* a, const v4f* b, size_t nvec) {
  const size_t base = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * U;
  v4f x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u < nvec) { x[u] = __builtin_nontemporal_load(a + base + u); y[u] = __builtin_nontemporal_load(b + base + u); }
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u < nvec) __builtin_nontemporal_store(x[u] + y[u], out + base + u);
}

// the north star's "LDS staging of the arriving peer slice", measured: (1) through registers,
// (2) by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip) -- incoming b lands in LDS first
__global__ void __launch_bounds__(64) lds_reg(v4f* out, const v4f* a, const v4f* b, size_t nvec) {
  __shared__ v4f tile[64];
  const size_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= nvec) return;
  tile[threadIdx.x] = __builtin_nontemporal_load(b + i);
  const v4f x = __builtin_nontemporal_load(a + i);
  __syncthreads();
  __builtin_nontemporal_store(x + tile[threadIdx.x], out + i);
}
__global__ void __launch_bounds__(64) lds_dma(v4f* out, const v4f* a, const v4f* b, size_t nvec) {
  __shared__ v4f tile[64];
  const size_t i = blockIdx.x * 64 + threadIdx.x;
  __builtin_amdgcn_global_load_lds((const void*)(b + i), (__attribute__((address_space(3))) void*)tile, 16, 0, 2);
  const v4f x = __builtin_nontemporal_load(a + i);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  __builtin_nontemporal_store(x + tile[threadIdx.x], out + i);
}

struct Var { const char* name; void (*launch)(v4f*, const v4f*, const v4f*, size_t); };

template <int U, int NTL, int NTS, int NT, int GRID>
void L(v4f* o, const v4f* a, const v4f* b, size_t n) { gs<U, NTL, NTS><<<GRID, NT>>>(o, a, b, n); }
template <int U, int NTL, int NTS, int NT>
void Lexact(v4f* o, const v4f* a, const v4f* b, size_t n) { gs<U, NTL, NTS><<<(unsigned)((n + (size_t)NT * U - 1) / ((size_t)NT * U)), NT>>>(o, a, b, n); }
template <int U, int NT>
void Lcontig(v4f* o, const v4f* a, const v4f* b, size_t n) { contig<U><<<(unsigned)((n + (size_t)NT * U - 1) / ((size_t)NT * U)), NT>>>(o, a, b, n); }
void Llds_reg(v4f* o, const v4f* a, const v4f* b, size_t n) { lds_reg<<<(unsigned)((n + 63) / 64), 64>>>(o, a, b, n); }
void Llds_dma(v4f* o, const v4f* a, const v4f* b, size_t n) { lds_dma<<<(unsigned)(n / 64), 64>>>(o, a, b, n); }
template <int U, int NTL, int NTS, int NT, int GRID>
void Lnc(v4f* o, const v4f* a, const v4f* b, size_t n) { gs_nochk<U, NTL, NTS><<<GRID, NT>>>(o, a, b, n); }

int main() {
  const size_t count = 268435456, nvec = count / 4;
  v4f *a, *b;
  CK(hipMalloc(&a, count * 4));
  CK(hipMalloc(&b, count * 4));
  CK(hipMemset(a, 0, count * 4));
  CK(hipMemset(b, 0, count * 4));
  std::vector<Var> vs = {
    {"U4 nt/nt 256x4096 grid-stride", L<4, 1, 1, 256, 4096>},
    {"U4 pl/pl 256x4096 grid-stride", L<4, 0, 0, 256, 4096>},
    {"U1 nt/nt 64 exact (shipped)", Lexact<1, 1, 1, 64>},
    {"U1 nt/nt 128 exact", Lexact<1, 1, 1, 128>},
    {"U1 nt/nt 256 exact", Lexact<1, 1, 1, 256>},
    {"U2 nt/nt 64 exact", Lexact<2, 1, 1, 64>},
    {"U1 pl/pl 64 exact", Lexact<1, 0, 0, 64>},
    {"LDS-staged b (registers) 64", Llds_reg},
    {"LDS-staged b (LDS-DMA) 64", Llds_dma},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int rounds = 7, reps = 10;
  std::vector<std::vector<float>> t(vs.size());
  for (int rnd = 0; rnd < rounds; ++rnd)
    for (size_t v = 0; v < vs.size(); ++v) {
      vs[v].launch(a, a, b, nvec);
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) vs[v].launch(a, a, b, nvec);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms / reps);
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(t[v].begin(), t[v].end());
    const double med = t[v][t[v].size() / 2], mn = t[v][0];
    printf("%-32s median %.4f ms min %.4f ms -> %.0f GB/s (%.1f%% of 8 TB/s)\n", vs[v].name, med, mn,
           3.0 * count * 4 / (med * 1e-3) / 1e9, 3.0 * count * 4 / (med * 1e-3) / 8e12 * 100);
  }
  return 0;
}
