// app -- the reference's minimal application (src/main.cpp:1-70) against this build's ABI, as
// written: 2 ranks, 1 Mi floats in PINNED host memory (cudaHostAlloc -> hipHostMalloc,
// main.cpp:35), filled on the host (rank 0: 1.0, rank 1: 2.0), one in-place all-reduce on a
// fresh stream, stream sync, and every element checked on the host to be exactly 3.0.  Like
// the reference it never selects a device (every rank on device 0).
//   app <rank> [server_ip] [--device-buffer]   (--device-buffer: hipMalloc'd buffer instead)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
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
    fprintf(stderr, "Usage: ./app <rank> [server_ip] [--device-buffer]\n");
    return 1;
  }
  const int rank = atoi(argv[1]);
  const char* ip = "127.0.0.1";
  bool device_buffer = false;
  for (int a = 2; a < argc; ++a) {
    if (!strcmp(argv[a], "--device-buffer")) device_buffer = true;
    else ip = argv[a];
  }
  const int nranks = 2;
  printf("[App] Rank %d starting...\n", rank);
  fflush(stdout);

  ncclComm_t comm;
  NCCL_OK(ncclCommInitRank(&comm, nranks, rank, ip));

  const int count = 1024 * 1024;
  const size_t bytes = (size_t)count * sizeof(float);
  float* data = nullptr;     // what ncclAllReduce gets
  float* host = nullptr;     // what the host fills and checks
  std::vector<float> staging;
  if (device_buffer) {
    if (hipMalloc((void**)&data, bytes) != hipSuccess) return 1;
    staging.assign((size_t)count, 0.0f);
    host = staging.data();
  } else {
    if (hipHostMalloc((void**)&data, bytes, hipHostMallocDefault) != hipSuccess) return 1;  // pinned
    host = data;
  }
  for (int i = 0; i < count; ++i) host[i] = (rank == 0) ? 1.0f : 2.0f;
  if (device_buffer && hipMemcpy(data, host, bytes, hipMemcpyHostToDevice) != hipSuccess) return 1;

  hipStream_t stream;
  if (hipStreamCreate(&stream) != hipSuccess) return 1;

  printf("[App] Calling ncclAllReduce...\n");
  fflush(stdout);
  NCCL_OK(ncclAllReduce(data, data, count, ncclFloat, ncclSum, comm, stream));  // in place
  if (hipStreamSynchronize(stream) != hipSuccess) return 1;
  if (device_buffer && hipMemcpy(host, data, bytes, hipMemcpyDeviceToHost) != hipSuccess) return 1;

  int bad = 0;
  for (int i = 0; i < count; ++i)
    if (host[i] != 3.0f) {
      if (bad < 5) fprintf(stderr, "Mismatch at %d expected 3.0 got %f\n", i, host[i]);
      ++bad;
    }
  printf(bad ? "Result: [FAIL]\n" : "Result: [PASS] All values are 3.0!\n");
  NCCL_OK(ncclCommDestroy(comm));
  hipStreamDestroy(stream);
  if (device_buffer) hipFree(data);
  else hipHostFree(data);
  return bad ? 2 : 0;
}
