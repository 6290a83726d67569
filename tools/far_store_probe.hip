// far_store_probe.hip -- how many bytes of far-memory stores (and loads) one wave keeps in flight.
// gfx950 counts loads and stores in one in-order vmcnt, so a copy loop "U loads, U stores"
// can only use batch k+1's loads after batch k's stores are acknowledged.  For a store into
// far memory (a peer's HBM over xGMI; here: pinned host memory over PCIe, the far target one
// GPU has) that is a round trip, so a wave's rate should be ~ U KiB / RTT.  This times a
// device -> far copy with W one-wave workgroups and U 16-byte vectors per lane per batch,
// with the all-reduce kernels' store form (sc0 sc1 buffer stores).  Not product code.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e = (x);                                                                          \
    if (e != hipSuccess) {                                                                       \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));                            \
      return 1;                                                                                  \
    }                                                                                            \
  } while (0)

// wave w copies bytes [w * per, (w + 1) * per) of src to dst; per is a multiple of U KiB
template <int U>
__global__ void __launch_bounds__(64) copy_far(const v4u* __restrict__ src, char* dst, size_t per) {
  const int lane = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * per;
  const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(dst + base, (short)0, (int)per, 0x00020000);
  const v4u* in = src + base / 16;
  for (size_t b = 0; b < per / 16; b += 64 * U) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(in + b + u * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], out, (uint32_t)((b + u * 64 + lane) * 16), 0, 17);
  }
}

// the other direction, as the read schedule moves bytes: sc0 sc1 buffer loads FROM far memory
// (U per lane in flight), plain stores into local memory
template <int U>
__global__ void __launch_bounds__(64) load_far(const char* src, v4u* dst, size_t per) {
  const int lane = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * per;
  const __amdgpu_buffer_rsrc_t in =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src) + base, (short)0, (int)per, 0x00020000);
  v4u* out = dst + base / 16;
  for (size_t b = 0; b < per / 16; b += 64 * U) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(in, (uint32_t)((b + u * 64 + lane) * 16), 0, 17);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], out + b + u * 64 + lane);
  }
}

template <int U>
static float run(const v4u* src, char* dst, int waves, size_t per, hipEvent_t e0, hipEvent_t e1, bool load) {
  auto go = [&] {
    if (load) load_far<U><<<waves, 64>>>(dst, const_cast<v4u*>(src), per);
    else copy_far<U><<<waves, 64>>>(src, dst, per);
  };
  go();
  hipEventRecord(e0);
  const int reps = 5;
  for (int i = 0; i < reps; ++i) go();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const size_t total = 256ull << 20;
  v4u* src;
  char *dev_dst, *host_dst;
  CK(hipMalloc(&src, total));
  CK(hipMemset(src, 1, total));
  CK(hipMalloc(&dev_dst, total));
  CK(hipHostMalloc(&host_dst, total, hipHostMallocMapped));
  char* host_dev = nullptr;
  CK(hipHostGetDevicePointer((void**)&host_dev, host_dst, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int wave_counts[] = {1, 4, 16, 64, 256};
  printf("%-20s %6s %4s %12s %14s\n", "target", "waves", "U", "GB/s", "GB/s per wave");
  for (int load = 0; load < 2; ++load)
    for (int t = 0; t < 2; ++t) {
      char* dst = t ? host_dev : dev_dst;
      for (int w : wave_counts) {
        // bytes per wave: enough for a steady state, bounded so 1 wave stays quick
        size_t per = (w >= 64 ? total / w : (4ull << 20));
        per &= ~((size_t)(64 * 16 * 16) - 1);
        for (int U : {4, 8, 16}) {
          float ms = U == 4   ? run<4>(src, dst, w, per, e0, e1, load)
                     : U == 8 ? run<8>(src, dst, w, per, e0, e1, load)
                              : run<16>(src, dst, w, per, e0, e1, load);
          const double gbs = (double)per * w / (ms * 1e-3) / 1e9;
          printf("%-20s %6d %4d %12.2f %14.3f\n",
                 load ? (t ? "load from host(PCIe)" : "load from device") : (t ? "store to host(PCIe)" : "store to device"),
                 w, U, gbs, gbs / w);
        }
      }
    }
  CK(hipGetLastError());
  return 0;
}
