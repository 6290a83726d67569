// Probe (not product code): are 16-byte global loads/stores at 4-byte-aligned (not 16-byte)
// addresses correct on gfx950, plain and non-temporal?  Checks every byte.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__global__ void copy16(const char* src, char* dst, int n16, int nt) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n16) return;
  const v4u* s = reinterpret_cast<const v4u*>(src + (size_t)i * 16);
  v4u* d = reinterpret_cast<v4u*>(dst + (size_t)i * 16);
  if (nt) __builtin_nontemporal_store(__builtin_nontemporal_load(s), d);
  else *d = *s;
}
int main() {
  const int n16 = 1 << 20;
  const size_t bytes = (size_t)n16 * 16 + 64;
  std::vector<unsigned char> h(bytes), o(bytes);
  for (size_t i = 0; i < bytes; ++i) h[i] = (unsigned char)(i * 131 + 7);
  char *s, *d;
  hipMalloc(&s, bytes); hipMalloc(&d, bytes);
  hipMemcpy(s, h.data(), bytes, hipMemcpyHostToDevice);
  int bad_total = 0;
  for (int nt = 0; nt < 2; ++nt)
    for (int so = 0; so < 16; so += 4)
      for (int dof = 0; dof < 16; dof += 4) {
        hipMemset(d, 0, bytes);
        copy16<<<n16 / 256, 256>>>(s + so, d + dof, n16, nt);
        hipError_t e = hipDeviceSynchronize();
        hipMemcpy(o.data(), d, bytes, hipMemcpyDeviceToHost);
        int bad = 0;
        for (size_t i = 0; i < (size_t)n16 * 16; ++i) bad += o[dof + i] != h[so + i];
        bad_total += bad;
        printf("nt=%d src+%2d dst+%2d: %s, %d bad bytes\n", nt, so, dof, hipGetErrorString(e), bad);
      }
  // timing: aligned vs misaligned
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int off = 0; off < 16; off += 4) {
    hipEventRecord(a);
    for (int k = 0; k < 20; ++k) copy16<<<n16 / 256, 256>>>(s + off, d + off, n16, 1);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("offset %2d: %.1f GB/s copy\n", off, 2.0 * n16 * 16 * 20 / (ms * 1e-3) / 1e9);
  }
  printf("TOTAL_BAD %d\n", bad_total);
  return 0;
}
