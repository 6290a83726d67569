// testkern.hip -- TEST INFRASTRUCTURE (tests/lib/libmnccl_testkern.so), never linked by the
// product.  Position-coded fill / check for buffers too large for host-side checking
// (tests/test_gpu.py::test_chunks_beyond_4gib), and the "ordinary consumer" kernels of the
// cross-device-shaped GPU test
// (tests/test_gpu.py::test_read_push_visible_to_cached_consumers): plain global loads and stores,
// cached in this GPU's L2 like any framework kernel's, so a stale L2 line of a buffer that a peer
// pushed into during an all-reduce would be read back by them (kernels.hip header, "Coherence of
// the pushes" in DESIGN.md).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

// every 4-byte word of p read with plain loads (the lines end up in this GPU's L2); the xor of the
// words lands in *out so the loads cannot be dropped
__global__ void __launch_bounds__(256) touch_kernel(const uint32_t* __restrict__ p, uint64_t nwords,
                                                    uint32_t* __restrict__ out) {
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x)
    x ^= p[i];
  if (x == 0x9e3779b9u) out[0] = x;  // almost never taken; keeps the loads live
}

// dst = src with plain loads and stores
__global__ void __launch_bounds__(256) copy_kernel(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                   uint64_t nwords) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// p[i] = uint32(i) * mult (wrapping): every word names its position modulo 2^32 elements, so a
// 32-bit wrap of a byte offset (4 GiB) in the kernel under test reads a different value
__global__ void __launch_bounds__(256) iota_kernel(uint32_t* __restrict__ p, uint64_t nwords, uint32_t mult) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i * mult;
}

// p[i] == uint32(i) * (i < body ? mult_body : mult_tail)?  Mismatches counted in res[0], the
// lowest mismatching index in res[1] (a vector atomic per mismatching lane: rare by design)
__global__ void __launch_bounds__(256) check_iota_kernel(const uint32_t* __restrict__ p, uint64_t nwords,
                                                         uint64_t body, uint32_t mult_body, uint32_t mult_tail,
                                                         unsigned long long* __restrict__ res) {
  unsigned long long bad = 0, first = ~0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x)
    if (p[i] != (uint32_t)i * (i < body ? mult_body : mult_tail)) {
      ++bad;
      if (first == ~0ull) first = i;
    }
  if (bad) {
    atomicAdd(&res[0], bad);
    atomicMin(&res[1], first);
  }
}

unsigned grid_for(uint64_t nwords) {
  const uint64_t b = (nwords + 255) / 256;
  return (unsigned)(b < 4096 ? (b ? b : 1) : 4096);
}

}  // namespace

extern "C" {

int mnccl_test_touch(const void* p, uint64_t bytes, void* scratch_word, hipStream_t st) {
  hipLaunchKernelGGL(touch_kernel, dim3(grid_for(bytes / 4)), dim3(256), 0, st, (const uint32_t*)p, bytes / 4,
                     (uint32_t*)scratch_word);
  return (int)hipGetLastError();
}

int mnccl_test_copy(void* dst, const void* src, uint64_t bytes, hipStream_t st) {
  hipLaunchKernelGGL(copy_kernel, dim3(grid_for(bytes / 4)), dim3(256), 0, st, (uint32_t*)dst, (const uint32_t*)src,
                     bytes / 4);
  return (int)hipGetLastError();
}

int mnccl_test_iota(void* p, uint64_t nwords, uint32_t mult, hipStream_t st) {
  hipLaunchKernelGGL(iota_kernel, dim3(grid_for(nwords)), dim3(256), 0, st, (uint32_t*)p, nwords, mult);
  return (int)hipGetLastError();
}

// res: 2 device words, set here to {0, ~0}
int mnccl_test_check_iota(const void* p, uint64_t nwords, uint64_t body, uint32_t mult_body, uint32_t mult_tail,
                          void* res, hipStream_t st) {
  const unsigned long long init[2] = {0ull, ~0ull};
  hipError_t e = hipMemcpyAsync(res, init, sizeof init, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(check_iota_kernel, dim3(grid_for(nwords)), dim3(256), 0, st, (const uint32_t*)p, nwords, body,
                     mult_body, mult_tail, (unsigned long long*)res);
  return (int)hipGetLastError();
}

}  // extern "C"
