// Environment probe (not product code): checks, on one GPU, that
//  (1) HIP IPC handles of hipMalloc and of hipDeviceMallocUncached memory can
//      be exported by one process and opened by another on the SAME device,
//  (2) two processes' spinning kernels run concurrently (flag ping-pong through
//      an IPC-mapped uncached word),
//  (3) pinned host-mapped memory is visible to a spinning kernel (abort word).
// Every spin is bounded by s_memrealtime so nothing can hang the box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <sys/wait.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "[pid %d] %s:%d %s -> %s\n", getpid(), __FILE__, __LINE__, #x, hipGetErrorString(e)); exit(2);} } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ u64 ld_sys(u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(u64* p, u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ping-pong: role 0 writes peer[0] = i+1 then waits mine[0] == i+1 ... iters rounds
__global__ void pingpong(u64* mine, u64* peer, int role, int iters, u64* result, u64 timeout_ticks) {
  if (threadIdx.x != 0) return;
  u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    if (role == 0) {
      st_sys(peer, (u64)i + 1);
      while (ld_sys(mine) < (u64)i + 1) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) { result[0] = 0xdead; result[1] = i; return; }
      }
    } else {
      while (ld_sys(mine) < (u64)i + 1) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) { result[0] = 0xdead; result[1] = i; return; }
      }
      st_sys(peer, (u64)i + 1);
    }
  }
  result[0] = 1;
  result[1] = __builtin_amdgcn_s_memrealtime() - t0;
}

__global__ void fill(float* p, size_t n, float v) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

struct Msg { hipIpcMemHandle_t h_plain, h_unc; };

int main() {
  int p2c[2], c2p[2];
  if (pipe(p2c) || pipe(c2p)) return 1;
  pid_t pid = fork();
  int role = pid == 0 ? 1 : 0;
  int rd = role ? p2c[0] : c2p[0];
  int wr = role ? c2p[1] : p2c[1];
  CK(hipSetDevice(0));
  const size_t N = 1 << 20;
  float* plain; u64* unc;
  CK(hipMalloc(&plain, N * sizeof(float)));
  CK(hipExtMallocWithFlags((void**)&unc, 4096, hipDeviceMallocUncached));
  CK(hipMemset(unc, 0, 4096));
  fill<<<N / 256, 256>>>(plain, N, role ? 2.0f : 1.0f);
  CK(hipDeviceSynchronize());
  Msg mine, theirs;
  CK(hipIpcGetMemHandle(&mine.h_plain, plain));
  CK(hipIpcGetMemHandle(&mine.h_unc, unc));
  if (write(wr, &mine, sizeof mine) != sizeof mine) return 3;
  if (read(rd, &theirs, sizeof theirs) != sizeof theirs) return 3;
  float* peer_plain; u64* peer_unc;
  CK(hipIpcOpenMemHandle((void**)&peer_plain, theirs.h_plain, hipIpcMemLazyEnablePeerAccess));
  CK(hipIpcOpenMemHandle((void**)&peer_unc, theirs.h_unc, hipIpcMemLazyEnablePeerAccess));
  float host[4];
  CK(hipMemcpy(host, peer_plain, sizeof host, hipMemcpyDeviceToHost));
  printf("[role %d] peer plain[0] = %.1f (expect %.1f)\n", role, host[0], role ? 1.0f : 2.0f);
  // sync both sides before ping-pong
  char c = 'x';
  if (write(wr, &c, 1) != 1 || read(rd, &c, 1) != 1) return 3;
  u64* res; CK(hipHostMalloc((void**)&res, 16, hipHostMallocMapped));
  res[0] = res[1] = 0;
  const int iters = 10000;
  pingpong<<<1, 64>>>(unc, peer_unc, role, iters, res, 100000000ull * 5);
  CK(hipDeviceSynchronize());
  if (res[0] == 1)
    printf("[role %d] pingpong ok: %d round trips in %.3f ms -> %.2f us/rt\n", role, iters, res[1] / 1e5, res[1] / 100.0 / iters);
  else
    printf("[role %d] pingpong TIMEOUT at iter %llu\n", role, res[1]);
  if (write(wr, &c, 1) != 1 || read(rd, &c, 1) != 1) return 3;
  CK(hipIpcCloseMemHandle(peer_plain));
  CK(hipIpcCloseMemHandle(peer_unc));
  if (pid) { int st; waitpid(pid, &st, 0); printf("child exit %d\n", WEXITSTATUS(st)); }
  return 0;
}
