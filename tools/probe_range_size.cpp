// Environment probe (not product code): HIP_POINTER_ATTRIBUTE_RANGE_SIZE vs hipMemGetAddressRange
// for allocations around and above 4 GiB (peerbuf.cpp's describe() uses the latter).
#include <hip/hip_runtime.h>

#include <cstdio>

int main() {
  for (size_t gib : {1, 3, 4, 5}) {
    void* p = nullptr;
    const size_t bytes = gib << 30;
    if (hipMalloc(&p, bytes) != hipSuccess) return 1;
    size_t a = 0, c = 0;
    hipDeviceptr_t b = 0;
    hipPointer_attribute attr = HIP_POINTER_ATTRIBUTE_RANGE_SIZE;
    void* vals[1] = {&a};
    const hipError_t e1 = hipDrvPointerGetAttributes(1, &attr, vals, (hipDeviceptr_t)p);
    const hipError_t e2 = hipMemGetAddressRange(&b, &c, (hipDeviceptr_t)p);
    printf("%zu GiB: RANGE_SIZE attribute %zu (%s), hipMemGetAddressRange %zu (%s)\n", gib, a, hipGetErrorString(e1), c,
           hipGetErrorString(e2));
    (void)hipFree(p);
  }
  return 0;
}
