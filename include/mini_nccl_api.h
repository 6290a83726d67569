/*
 * mini_nccl_api.h -- the drop-in C ABI of libmini_nccl.so (MI355X / gfx950 build).
 *
 * Same names, enum values and argument meaning as the reference's public header
 * (XuDongGong/Mini-NCCL include/mini_nccl_api.h:1-75), with the one substitution
 * the platform needs: the stream argument is a hipStream_t instead of cudaStream_t.
 * A caller that compiled against the reference re-compiles against this header
 * (cudaStream_t -> hipStream_t) and links -lmini_nccl unchanged.
 *
 * Entry points (each replaces the reference symbol of the same name):
 *   ncclGetErrorString  <- src/api.cpp:14-26
 *   ncclCommInitRank    <- src/api.cpp:28-66   (mini_nccl_api.h:61)
 *   ncclCommDestroy     <- src/api.cpp:68-77   (mini_nccl_api.h:63)
 *   ncclCommUserRank    <- src/api.cpp:79-88   (mini_nccl_api.h:66)
 *   ncclCommCount       <- src/api.cpp:90-99   (mini_nccl_api.h:69)
 *   ncclAllReduce       <- src/api.cpp:136-190 (mini_nccl_api.h:71-73)
 *
 * Error convention (reference api.cpp): NULL comm/buffer -> ncclInvalidArgument;
 * rank out of range -> ncclInvalidArgument; count == 0 -> ncclSuccess; failure
 * during init -> ncclSystemError; unsupported dtype/op or a watchdog timeout during
 * the all-reduce -> ncclInternalError.  No C++ exception crosses this boundary.
 */
#ifndef MINI_NCCL_API_H_
#define MINI_NCCL_API_H_

#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1, /* kept for source compatibility: an unhandled HIP runtime error */
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
  ncclRemoteError = 6,
  ncclInProgress = 7
} ncclResult_t;

/* opaque communicator handle */
typedef struct ncclComm* ncclComm_t;

/* element types; numbering identical to the reference (and to RCCL's rccl.h) */
typedef enum {
  ncclInt8 = 0,
  ncclUint8 = 1,
  ncclInt32 = 2,
  ncclUint32 = 3,
  ncclInt64 = 4,
  ncclUint64 = 5,
  ncclFloat16 = 6,
  ncclFloat = 7,
  ncclDouble = 8,
  ncclBfloat16 = 9
} ncclDataType_t;

typedef enum {
  ncclSum = 0,
  ncclProd = 1,
  ncclMax = 2,
  ncclMin = 3,
  ncclAvg = 4
} ncclRedOp_t;

const char* ncclGetErrorString(ncclResult_t result);

/* nRanks processes, one per GPU (the current HIP device of the calling thread);
 * rank 0 listens on `ip`:MINI_NCCL_PORT (default 8888, as the reference) and the
 * others connect to it.  ip == NULL means "127.0.0.1".  rank == -1 (the reference's
 * Hera auto-rank mode, api.cpp:38-51) is not supported: ncclInvalidUsage. */
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nRanks, int rank, const char* ip);

ncclResult_t ncclCommDestroy(ncclComm_t comm);

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank);

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count);

/* All-reduce of `count` elements; sendbuff/recvbuff are device pointers on the
 * communicator's GPU (send == recv means in place).  Elements [n*(count/n), count)
 * are not reduced (reference mini_nccl.cu:69): recv keeps this rank's own input
 * there.  Supported: ncclFloat, ncclDouble, ncclInt32 (the reference's set) plus
 * ncclFloat16 and ncclBfloat16, with ncclSum/ncclProd/ncclMax/ncclMin.
 * Blocks the calling thread until the stream has drained, as the reference does
 * (mini_nccl.cu:200-214), unless MINI_NCCL_BLOCKING=0 or the stream is capturing. */
ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count,
                           ncclDataType_t datatype, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MINI_NCCL_API_H_ */
