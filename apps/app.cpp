// app -- the reference's minimal application (src/main.cpp:1-70) against this build's ABI:
// 2 ranks, 1 Mi floats, in-place all-reduce, rank 0 contributes 1.0 and rank 1 2.0, every
// element must come back as exactly 3.0.
//   app <rank> [server_ip]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mini_nccl_api.h"

#define NCCL_OK(cmd)                                                          \
  do {                                                                        \
    ncclResult_t r_ = (cmd);                                                  \
    if (r_ != ncclSuccess) {                                                  \
      fprintf(stderr, "NCCL Error: %s\n", ncclGetErrorString(r_));            \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "Usage: ./app <rank> [server_ip]\n");
    return 1;
  }
  const int rank = atoi(argv[1]);
  const char* ip = argc > 2 ? argv[2] : "127.0.0.1";
  const int nranks = 2;
  int ndev = 1;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) ndev = 1;
  if (hipSetDevice(rank % ndev) != hipSuccess) return 1;
  printf("[App] Rank %d starting...\n", rank);

  ncclComm_t comm;
  NCCL_OK(ncclCommInitRank(&comm, nranks, rank, ip));

  const int count = 1024 * 1024;
  std::vector<float> host((size_t)count, rank == 0 ? 1.0f : 2.0f);
  float* data = nullptr;
  if (hipMalloc((void**)&data, count * sizeof(float)) != hipSuccess) return 1;
  if (hipMemcpy(data, host.data(), count * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipStream_t stream;
  if (hipStreamCreate(&stream) != hipSuccess) return 1;

  printf("[App] Calling ncclAllReduce...\n");
  NCCL_OK(ncclAllReduce(data, data, count, ncclFloat, ncclSum, comm, stream));  // in place
  if (hipStreamSynchronize(stream) != hipSuccess) return 1;
  if (hipMemcpy(host.data(), data, count * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return 1;

  int bad = 0;
  for (int i = 0; i < count; ++i)
    if (host[(size_t)i] != 3.0f) {
      if (bad < 5) fprintf(stderr, "Mismatch at %d expected 3.0 got %f\n", i, host[(size_t)i]);
      ++bad;
    }
  printf(bad ? "Result: [FAIL]\n" : "Result: [PASS] All values are 3.0!\n");
  NCCL_OK(ncclCommDestroy(comm));
  hipStreamDestroy(stream);
  hipFree(data);
  return bad ? 2 : 0;
}
