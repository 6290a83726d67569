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

// XCD-aware block order: workgroups are dealt round-robin to the 8 XCDs (b % 8); remap so
// XCD x walks contiguous runs of G KiB-blocks instead of every 8th KiB
template <int G>
__global__ void __launch_bounds__(64) xcd_remap(v4f* out, const v4f* a, const v4f* b, size_t nvec) {
  const size_t nblk = gridDim.x;  // multiple of 8 * G (caller)
  const size_t bx = blockIdx.x, x = bx & 7, k = bx >> 3;  // k-th block of XCD x
  const size_t per = nblk / 8;
  const size_t lb = (G == 0) ? x * per + k : ((k / G) * 8 + x) * G + (k % G);
  const size_t i = lb * 64 + threadIdx.x;
  const v4f p = __builtin_nontemporal_load(a + i);
  const v4f q = __builtin_nontemporal_load(b + i);
  __builtin_nontemporal_store(p + q, out + i);
}
// cache-policy bits on buffer ops (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
template <int LA, int SA>
__global__ void __launch_bounds__(64) pol(v4f* out, const v4f* a, const v4f* b, size_t nvec) {
  const size_t i = blockIdx.x * 64 + threadIdx.x;
  const size_t base = (size_t)blockIdx.x * 1024;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)((char*)a + base), (short)0, 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)((char*)b + base), (short)0, 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)((char*)out + base), (short)0, 1024, 0x00020000);
  (void)i;
  v4u p = __builtin_amdgcn_raw_buffer_load_b128(ra, threadIdx.x * 16, 0, LA);
  v4u q = __builtin_amdgcn_raw_buffer_load_b128(rb, threadIdx.x * 16, 0, LA);
  v4f r = __builtin_bit_cast(v4f, p) + __builtin_bit_cast(v4f, q);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, r), ro, threadIdx.x * 16, 0, SA);
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
template <int G>
void Lxcd(v4f* o, const v4f* a, const v4f* b, size_t n) { xcd_remap<G><<<(unsigned)(n / 64), 64>>>(o, a, b, n); }
template <int LA, int SA>
void Lpol(v4f* o, const v4f* a, const v4f* b, size_t n) { pol<LA, SA><<<(unsigned)(n / 64), 64>>>(o, a, b, n); }
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
    {"U1 nt/nt 64 exact (shipped)", Lexact<1, 1, 1, 64>},
    {"XCD remap: 8 contiguous regions", Lxcd<0>},
    {"XCD remap: runs of 4 KiB", Lxcd<4>},
    {"XCD remap: runs of 64 KiB", Lxcd<64>},
    {"XCD remap: runs of 1 MiB", Lxcd<1024>},
    {"buffer ld nt / st nt", Lpol<2, 2>},
    {"buffer ld nt / st nt|sc1", Lpol<2, 18>},
    {"buffer ld nt / st sc0|sc1", Lpol<2, 17>},
    {"buffer ld 0 / st nt", Lpol<0, 2>},
    {"buffer ld nt|sc1 / st nt", Lpol<18, 2>},
    {"U1 nt/nt 128 exact", Lexact<1, 1, 1, 128>},
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
