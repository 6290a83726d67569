// testkern.hip -- TEST INFRASTRUCTURE (tests/lib/libmnccl_testkern.so), never linked by the
// product.  The "ordinary consumer" kernels of the cross-device-shaped GPU test
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

}  // extern "C"
