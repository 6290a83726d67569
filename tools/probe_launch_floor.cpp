// Environment probe (not product code): the floor of a blocking call when N processes share one
// GPU -- what any schedule's small call at N co-located ranks pays before it moves a byte.
// Each of N forked processes (forked before any HIP call) repeats ITERS times, timing rank 0:
//   empty     launch an empty one-wave kernel, hipStreamSynchronize
//   barrier   a process-shared host barrier, then `empty` (the negotiated call's host rendezvous)
//   meet      a one-wave kernel that stores its call number into a flag in host shared memory
//             (registered with the GPU) and waits until every process's flag reaches it (the
//             device-side rendezvous of a registered-window call), hipStreamSynchronize
//   *-poll    the same three, waiting as the library's blocking calls do (comm.cpp wait_for: an
//             event recorded after the kernel, hipEventQuery + sched_yield until it completes)
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/bin/probe_launch_floor tools/probe_launch_floor.cpp
// Run:   tools/bin/probe_launch_floor <N> [ITERS]   (prints one line per mode, rank 0's us/call)
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <new>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      _exit(2);                                                                           \
    }                                                                                     \
  } while (0)

struct Shared {
  pthread_barrier_t bar;
  alignas(64) unsigned flags[64 * 16];  // one 64-byte line per process
};

constexpr size_t kMapBytes = 1 << 16;

__global__ void empty_kernel() {}

// every lane < n polls process `lane`'s flag (system scope: host memory written by other
// processes' kernels); bounded, so a wave always exits
__global__ void meet_kernel(unsigned* flags, int n, int me, unsigned call, unsigned* timeouts) {
  const int lane = threadIdx.x;
  if (lane == 0) __hip_atomic_store(&flags[me * 16], call, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (lane < n) {
    long spins = 0;
    while (__hip_atomic_load(&flags[lane * 16], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < call) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1L << 22)) {
        __hip_atomic_fetch_add(timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
}

static int run(Shared* sh, int n, int me, int iters) {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Shared* dsh = nullptr;  // the whole page-aligned mapping, registered in every process
  CK(hipHostRegister(sh, kMapBytes, hipHostRegisterMapped));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dsh), sh, 0));
  unsigned* dflags = dsh->flags;
  unsigned* timeouts = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&timeouts), sizeof(unsigned), hipHostMallocMapped));
  *timeouts = 0;
  unsigned call = 0;
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const char* names[6] = {"empty", "barrier", "meet", "empty-poll", "barrier-poll", "meet-poll"};
  for (int m6 = 0; m6 < 6; ++m6) {
    const int mode = m6 % 3;
    const bool poll = m6 >= 3;
    double us = 0;
    for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms up
      pthread_barrier_wait(&sh->bar);
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; ++i) {
        if (mode == 1) pthread_barrier_wait(&sh->bar);
        if (mode == 2) {
          meet_kernel<<<1, 64, 0, s>>>(dflags, n, me, ++call, timeouts);
        } else {
          empty_kernel<<<1, 64, 0, s>>>();
        }
        if (poll) {
          CK(hipEventRecord(ev, s));
          hipError_t q;
          while ((q = hipEventQuery(ev)) == hipErrorNotReady) sched_yield();
          CK(q);
        } else {
          CK(hipStreamSynchronize(s));
        }
      }
      us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    }
    if (me == 0) printf("n=%d mode=%-12s %8.2f us/call  (%d calls)\n", n, names[m6], us, iters);
    fflush(stdout);
  }
  pthread_barrier_wait(&sh->bar);
  if (*timeouts) fprintf(stderr, "rank %d: %u meet waits timed out\n", me, *timeouts);
  const int rc = *timeouts ? 3 : 0;
  CK(hipHostUnregister(sh));
  return rc;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2;
  const int iters = argc > 2 ? atoi(argv[2]) : 500;
  if (n < 1 || n > 64) return 1;
  // page-aligned shared mapping (hipHostRegister wants whole pages)
  void* mem = mmap(nullptr, kMapBytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (mem == MAP_FAILED) return 1;
  Shared* sh = new (mem) Shared();
  pthread_barrierattr_t a;
  pthread_barrierattr_init(&a);
  pthread_barrierattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_barrier_init(&sh->bar, &a, n);
  for (int r = 1; r < n; ++r) {
    if (fork() == 0) _exit(run(sh, n, r, iters));  // children fork before any HIP call
  }
  int rc = run(sh, n, 0, iters);
  for (int r = 1; r < n; ++r) {
    int st = 0;
    wait(&st);
    if (!WIFEXITED(st) || WEXITSTATUS(st)) rc = 4;
  }
  return rc;
}
