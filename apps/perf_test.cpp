// perf_test -- the reference's measurement harness (tests/perf_test.cpp:34-158) for the
// MI355X build, written against the same C ABI (include/mini_nccl_api.h).
//
//   perf_test <rank> <n_ranks> [master_ip] [--mode device|host|staged] [--sizes MiB,MiB,...] [--window]
//
// Same protocol as the reference: sizes 1/16/64/128 MiB fp32, every rank sends 1.0, 5
// warm-up and 20 timed all-reduces between CLOCK_MONOTONIC reads, an AVX2 compare scan
// that every element equals nRanks, and the algbw / busbw table
// (algbw = bytes / time, busbw = algbw * 2(n-1)/n; perf_test.cpp:140-143).
//   --mode device  (default) buffers resident in HBM: the headline measurement;
//   --mode host    the reference's own usage: pinned host buffers (cudaHostAlloc,
//                  perf_test.cpp:78-79) handed straight to ncclAllReduce; the kernel reads
//                  and writes them through their device mapping, i.e. the end-to-end rate
//                  including PCIe;
//   --mode staged  pinned host -> explicit H2D -> all-reduce -> D2H per call.
//   --window       (device mode) register send and recv with mncclCommRegister first: the calls
//                  then run with no host rendezvous (the Schedule column reads "read/win").
// Device: rank % device_count (the reference pinned every rank to GPU 0, :46;
// MINI_NCCL_PERF_DEVICE overrides).
#include <hip/hip_runtime.h>

#include "mini_nccl_ext.h"  // mncclCommGetInfoV: which schedule each size ran (diagnostic column)

// weak: the program also runs against a library without it (an older build, or another
// implementation of the ABI), and prints "?" there
extern "C" ncclResult_t mncclCommGetInfoV(ncclComm_t comm, void* info, size_t size) __attribute__((weak));
extern "C" ncclResult_t mncclCommRegister(ncclComm_t comm, void* buff, size_t size, void** handle) __attribute__((weak));
extern "C" ncclResult_t mncclCommDeregister(ncclComm_t comm, void* handle) __attribute__((weak));
#include <immintrin.h>
#include <time.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mini_nccl_api.h"

#define HIP_OK(cmd)                                                                             \
  do {                                                                                          \
    hipError_t e_ = (cmd);                                                                      \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "HIP error %s:%d '%s'\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(EXIT_FAILURE);                                                                       \
    }                                                                                           \
  } while (0)

#define NCCL_OK(cmd)                                                                            \
  do {                                                                                          \
    ncclResult_t r_ = (cmd);                                                                    \
    if (r_ != ncclSuccess) {                                                                    \
      fprintf(stderr, "mini-nccl error %s:%d '%s'\n", __FILE__, __LINE__, ncclGetErrorString(r_)); \
      exit(EXIT_FAILURE);                                                                       \
    }                                                                                           \
  } while (0)

static double now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

// AVX2 scan: index of the first element != expected, or -1 (perf_test.cpp:105-134)
static long first_mismatch(const float* p, size_t n, float expected) {
  const __m256 want = _mm256_set1_ps(expected);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    const int m = _mm256_movemask_ps(_mm256_cmp_ps(_mm256_loadu_ps(p + i), want, _CMP_NEQ_OQ));
    if (m) return (long)(i + (size_t)__builtin_ctz((unsigned)m));
  }
  for (; i < n; ++i)
    if (std::fabs(p[i] - expected) > 1e-5f) return (long)i;
  return -1;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "Usage: %s <rank> <n_ranks> [master_ip] [--mode device|host|staged] [--sizes 1,16,64,128 (MiB; 64k = KiB)]\n", argv[0]);
    return 1;
  }
  const int rank = atoi(argv[1]);
  const int nranks = atoi(argv[2]);
  const char* ip = "127.0.0.1";
  std::string mode = "device";
  std::vector<size_t> sizes = {1u << 20, 16u << 20, 64u << 20, 128u << 20};  // bytes
  int iters = 20, warmup = 5;
  bool window = false;
  for (int a = 3; a < argc; ++a) {
    std::string s = argv[a];
    if (s == "--mode" && a + 1 < argc) mode = argv[++a];
    else if (s == "--sizes" && a + 1 < argc) {
      sizes.clear();  // MiB, or KiB with a "k" suffix ("4k,64k,1")
      for (char* t = strtok(argv[++a], ","); t; t = strtok(nullptr, ",")) {
        char* end = nullptr;
        const size_t v = strtoul(t, &end, 10);
        sizes.push_back(end && (*end == 'k' || *end == 'K') ? v << 10 : v << 20);
      }
    } else if (s == "--iters" && a + 1 < argc) iters = atoi(argv[++a]);
    else if (s == "--warmup" && a + 1 < argc) warmup = atoi(argv[++a]);
    else if (s == "--window") window = true;
    else ip = argv[a];
  }
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  const char* dv = getenv("MINI_NCCL_PERF_DEVICE");
  HIP_OK(hipSetDevice(dv ? atoi(dv) : rank % (ndev > 0 ? ndev : 1)));

  ncclComm_t comm;
  NCCL_OK(ncclCommInitRank(&comm, nranks, rank, ip));
  hipStream_t stream;
  HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));

  if (rank == 0) {
    printf("\n=== Mini-NCCL (MI355X) Performance Benchmark, %d ranks, %s buffers ===\n", nranks,
           mode == "device" ? "HBM-resident" : mode == "host" ? "pinned host buffers passed to ncclAllReduce" : "host-staged (H2D + all-reduce + D2H)");
    printf("%15s %15s %15s %15s %9s\n", "Size(B)", "Time(us)", "AlgBW(GB/s)", "BusBW(GB/s)", "Schedule");
  }
  int failures = 0;
  for (size_t bytes : sizes) {
    const size_t count = bytes / sizeof(float);
    float *h_send = nullptr, *h_recv = nullptr, *d_send = nullptr, *d_recv = nullptr;
    HIP_OK(hipHostMalloc((void**)&h_send, bytes, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&h_recv, bytes, hipHostMallocDefault));
    HIP_OK(hipMalloc((void**)&d_send, bytes));
    HIP_OK(hipMalloc((void**)&d_recv, bytes));
    for (size_t i = 0; i < count; ++i) h_send[i] = 1.0f;  // perf_test.cpp:82
    memset(h_recv, 0, bytes);
    HIP_OK(hipMemcpy(d_send, h_send, bytes, hipMemcpyHostToDevice));
    void *w_send = nullptr, *w_recv = nullptr;
    if (window && mode == "device") {
      if (!mncclCommRegister) {
        fprintf(stderr, "--window: this library has no mncclCommRegister\n");
        return 1;
      }
      NCCL_OK(mncclCommRegister(comm, d_send, bytes, &w_send));
      NCCL_OK(mncclCommRegister(comm, d_recv, bytes, &w_recv));
    }

    auto one = [&]() {
      if (mode == "staged") HIP_OK(hipMemcpyAsync(d_send, h_send, bytes, hipMemcpyHostToDevice, stream));
      if (mode == "host") NCCL_OK(ncclAllReduce(h_send, h_recv, count, ncclFloat, ncclSum, comm, stream));
      else NCCL_OK(ncclAllReduce(d_send, d_recv, count, ncclFloat, ncclSum, comm, stream));
      if (mode == "staged") HIP_OK(hipMemcpyAsync(h_recv, d_recv, bytes, hipMemcpyDeviceToHost, stream));
    };
    for (int i = 0; i < warmup; ++i) one();
    HIP_OK(hipStreamSynchronize(stream));
    const double t0 = now_us();
    for (int i = 0; i < iters; ++i) one();
    HIP_OK(hipStreamSynchronize(stream));
    const double t1 = now_us();
    if (mode == "device") HIP_OK(hipMemcpy(h_recv, d_recv, bytes, hipMemcpyDeviceToHost));

    // every element of the n * (count / n) body is the sum; the count % n tail keeps this
    // rank's own input (1.0): the reference never reduces it (mini_nccl.cu:69), so its own
    // check would flag these sizes for nRanks that do not divide the element count
    const size_t body = (count / (size_t)nranks) * (size_t)nranks;
    long bad = first_mismatch(h_recv, body, (float)nranks);
    if (bad < 0) {
      const long t = first_mismatch(h_recv + body, count - body, 1.0f);
      if (t >= 0) bad = (long)body + t;
    }
    if (bad >= 0) {
      printf("[Rank %d] Verification FAILED for size %zu at %ld: %f\n", rank, bytes, bad, h_recv[bad]);
      ++failures;
    }
    const double us = (t1 - t0) / iters;
    const double alg = (double)bytes / us / 1e3;
    const double bus = alg * 2.0 * (nranks - 1) / nranks;
    mncclCommInfo_t info;
    memset(&info, 0, sizeof info);
    const char* sched = !mncclCommGetInfoV || mncclCommGetInfoV(comm, &info, sizeof info) != ncclSuccess ? "?"
                        : info.last_algo == 0 ? "ring" : info.last_algo == 2 ? (w_send ? "read/win" : "read")
                        : info.last_algo == 3 ? "oneshot" : "-";
    if (rank == 0) printf("%15zu %15.2f %15.2f %15.2f %9s %s\n", bytes, us, alg, bus, sched, bad >= 0 ? "(FAIL)" : "");
    fflush(stdout);
    if (w_send) NCCL_OK(mncclCommDeregister(comm, w_send));
    if (w_recv) NCCL_OK(mncclCommDeregister(comm, w_recv));
    HIP_OK(hipFree(d_send));
    HIP_OK(hipFree(d_recv));
    HIP_OK(hipHostFree(h_send));
    HIP_OK(hipHostFree(h_recv));
  }
  HIP_OK(hipStreamDestroy(stream));
  NCCL_OK(ncclCommDestroy(comm));
  return failures ? 2 : 0;
}
