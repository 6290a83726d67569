// The C ABI and the communicator's host code (api.cpp, comm.cpp, bootstrap.cpp, config.cpp)
// under AddressSanitizer + UBSan, linked with the normal (unsanitized) gfx950 kernels.
// Without a GPU: the argument checks and error paths (init fails cleanly).  With a GPU: two
// ranks as threads of this process run in- and out-of-place all-reduces through the ABI
// and compare with a host sum in ring order.  Built and run by tests/test_host_sanitizers.py.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <thread>
#include <vector>

#include "mini_nccl_api.h"

static int arg_checks() {
  int bad = 0;
  ncclComm_t c = nullptr;
  void* fake = (void*)0x1000;
  bad += ncclCommInitRank(nullptr, 2, 0, "127.0.0.1") != ncclInvalidArgument;
  bad += ncclCommInitRank(&c, 2, 2, nullptr) != ncclInvalidArgument;
  bad += ncclCommInitRank(&c, 2, -1, nullptr) != ncclInvalidUsage;
  bad += ncclCommDestroy(nullptr) != ncclInvalidArgument;
  bad += ncclAllReduce(nullptr, fake, 4, ncclFloat, ncclSum, (ncclComm_t)fake, nullptr) != ncclInvalidArgument;
  bad += ncclAllReduce(fake, fake, 0, ncclFloat, ncclSum, (ncclComm_t)fake, nullptr) != ncclSuccess;
  bad += ncclAllReduce(fake, fake, 4, ncclInt8, ncclSum, (ncclComm_t)fake, nullptr) != ncclInternalError;
  bad += strcmp(ncclGetErrorString(ncclInvalidUsage), "invalid usage") != 0;
  return bad;
}

static int two_rank_allreduce() {
  const size_t count = (1 << 20) + 3;
  int bad = 0;
  std::vector<std::vector<float>> host(2, std::vector<float>(count)), out(2, std::vector<float>(count));
  for (int r = 0; r < 2; ++r)
    for (size_t i = 0; i < count; ++i) host[(size_t)r][i] = (float)((i * 7 + (size_t)r * 13) % 1021) * 0.25f;
  std::vector<int> rcs(2, -1);
  auto rank = [&](int r) {
    hipSetDevice(0);
    ncclComm_t comm;
    if (ncclCommInitRank(&comm, 2, r, "127.0.0.1") != ncclSuccess) return;
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    float *s = nullptr, *d = nullptr;
    hipMalloc((void**)&s, count * 4);
    hipMalloc((void**)&d, count * 4);
    hipMemcpyAsync(s, host[(size_t)r].data(), count * 4, hipMemcpyHostToDevice, st);
    hipStreamSynchronize(st);
    int rc = ncclAllReduce(s, d, count, ncclFloat, ncclSum, comm, st);      // out of place
    rc |= ncclAllReduce(d, d, count, ncclFloat, ncclMax, comm, st);        // in place
    hipMemcpyAsync(out[(size_t)r].data(), d, count * 4, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    hipFree(s);
    hipFree(d);
    hipStreamDestroy(st);
    rc |= ncclCommDestroy(comm);
    rcs[(size_t)r] = rc;
  };
  std::thread t0(rank, 0), t1(rank, 1);
  t0.join();
  t1.join();
  const size_t body = count / 2 * 2;
  for (int r = 0; r < 2; ++r) {
    bad += rcs[(size_t)r] != 0;
    for (size_t i = 0; i < count; ++i) {
      // integer-valued quarters: sums are exact in any order; max of equal values is itself
      const float want = i < body ? host[0][i] + host[1][i] : host[(size_t)r][i];
      if (out[(size_t)r][i] != want) {
        ++bad;
        break;
      }
    }
  }
  return bad;
}

int main() {
  int fails = arg_checks();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  if (ndev > 0) {
    fails += two_rank_allreduce();
    printf("abi selftest (GPU): %s\n", fails ? "FAILED" : "ok");
  } else {
    ncclComm_t c = nullptr;
    const ncclResult_t rc = ncclCommInitRank(&c, 1, 0, nullptr);  // no device: clean failure
    fails += !(rc == ncclSystemError || rc == ncclSuccess);
    printf("abi selftest (no GPU): %s\n", fails ? "FAILED" : "ok");
  }
  return fails ? 1 : 0;
}
