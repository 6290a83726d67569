// api.cpp -- the C ABI (include/mini_nccl_api.h, include/mini_nccl_ext.h).
//
// Thin bridge, as the reference's src/api.cpp: argument checks in the reference's order
// and with its error codes, an exception firewall (no C++ exception crosses the ABI),
// dtype/op validation, one roctx range per all-reduce (the reference's NVTX range,
// api.cpp:142-151), then the communicator's hot path.
#include <hip/hip_runtime_api.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstddef>
#include <cstdio>
#include <exception>
#include <new>
#include <stdexcept>
#include <string>

#include <cstring>

#include "comm.h"
#include "ipcreg.h"
#include "kernels.h"
#include "mini_nccl_api.h"
#include "mini_nccl_ext.h"

using mnccl::Comm;

namespace {

// reference api.cpp:101-128: Float/Int32/Double x Sum/Prod/Max/Min; this build adds
// Float16/Bfloat16 (build-defined parity).  Anything else -> error.
bool dtype_ok(ncclDataType_t t) {
  return t == ncclFloat || t == ncclDouble || t == ncclInt32 || t == ncclFloat16 || t == ncclBfloat16;
}
bool op_ok(ncclRedOp_t op) { return op == ncclSum || op == ncclProd || op == ncclMax || op == ncclMin; }

struct RoctxRange {
  explicit RoctxRange(const char* m) { roctxRangePushA(m); }
  ~RoctxRange() { roctxRangePop(); }
};

}  // namespace

extern "C" {

const char* ncclGetErrorString(ncclResult_t result) {
  switch (result) {
    case ncclSuccess: return "no error";
    case ncclUnhandledCudaError: return "unhandled hip error";
    case ncclSystemError: return "system error";
    case ncclInternalError: return "internal error";
    case ncclInvalidArgument: return "invalid argument";
    case ncclInvalidUsage: return "invalid usage";
    case ncclRemoteError: return "remote error";
    case ncclInProgress: return "in progress";
    default: return "unknown error";
  }
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nRanks, int rank, const char* ip) {
  if (!comm) return ncclInvalidArgument;
  if (rank == -1) {
    fprintf(stderr, "[Mini-NCCL] Hera auto-rank mode (rank == -1) is not supported by this build\n");
    return ncclInvalidUsage;
  }
  if (nRanks < 1 || rank < 0 || rank >= nRanks) return ncclInvalidArgument;
  try {
    Comm* c = new Comm(nRanks, rank, ip ? std::string(ip) : std::string("127.0.0.1"));
    *comm = reinterpret_cast<ncclComm_t>(c);
    return ncclSuccess;
  } catch (const std::exception& e) {
    // every init failure is ncclSystemError, as in the reference (api.cpp:62-65): also a
    // configuration that differs between ranks, an unparsable MINI_NCCL_* value, nRanks > 16
    fprintf(stderr, "[Mini-NCCL] Init Failed: %s\n", e.what());
    return ncclSystemError;
  } catch (...) {
    return ncclSystemError;
  }
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  try {
    delete reinterpret_cast<Comm*>(comm);
    return ncclSuccess;
  } catch (...) {
    return ncclSystemError;
  }
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  if (!comm || !rank) return ncclInvalidArgument;
  *rank = reinterpret_cast<const Comm*>(comm)->rank();
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  if (!comm || !count) return ncclInvalidArgument;
  *count = reinterpret_cast<const Comm*>(comm)->nranks();
  return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
  if (!comm || !sendbuff || !recvbuff) return ncclInvalidArgument;  // api.cpp:139
  if (count == 0) return ncclSuccess;                               // api.cpp:140
  RoctxRange range("mini_ncclAllReduce");
  if (!dtype_ok(datatype) || !op_ok(op)) {
    // the reference throws inside get_type_size / to_internal_op -> ncclInternalError (:182-185)
    fprintf(stderr, "[Mini-NCCL] AllReduce Internal Error: unsupported %s\n", dtype_ok(datatype) ? "RedOp" : "DataType");
    return ncclInternalError;
  }
  try {
    return reinterpret_cast<Comm*>(comm)->allreduce(sendbuff, recvbuff, count, (int)datatype, (int)op, stream);
  } catch (const std::exception& e) {
    fprintf(stderr, "[Mini-NCCL] AllReduce Internal Error: %s\n", e.what());
    return ncclInternalError;
  } catch (...) {
    return ncclSystemError;
  }
}

// ------------------------------------------------------------------ extensions
ncclResult_t mncclLocalReduce(void* out, const void* local, const void* incoming, size_t count,
                              ncclDataType_t datatype, ncclRedOp_t op, hipStream_t stream) {
  if (!out || !local || !incoming) return ncclInvalidArgument;
  if (count == 0) return ncclSuccess;
  if (!dtype_ok(datatype) || !op_ok(op)) return ncclInternalError;
  try {
    return mnccl::local_reduce(out, local, incoming, count, (int)datatype, (int)op, stream);
  } catch (const std::exception& e) {
    fprintf(stderr, "[Mini-NCCL] LocalReduce Internal Error: %s\n", e.what());
    return ncclInternalError;
  } catch (...) {
    return ncclSystemError;
  }
}

ncclResult_t mncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError) {
  if (!comm || !asyncError) return ncclInvalidArgument;
  *asyncError = reinterpret_cast<Comm*>(comm)->async_error();
  return ncclSuccess;
}

// The legacy entry point writes the layout it was published with (before 300): a caller built
// against an older header is never written past the end of its struct; mncclCommGetInfoV gives
// the rest.
ncclResult_t mncclCommGetInfo(ncclComm_t comm, mncclCommInfo_t* info) {
  return mncclCommGetInfoV(comm, info, offsetof(mncclCommInfo_t, ipc_open_failures));
}

ncclResult_t mncclCommGetInfoV(ncclComm_t comm, void* out, size_t size) {
  if (!comm || !out) return ncclInvalidArgument;
  const Comm* c = reinterpret_cast<const Comm*>(comm);
  const mnccl::Config& k = c->config();
  mncclCommInfo_t full;
  memset(&full, 0, sizeof full);
  mncclCommInfo_t* info = &full;
  info->rank = c->rank();
  info->nranks = c->nranks();
  info->device = c->device();
  info->slice_bytes = k.slice_size;
  info->window = k.window_size;
  info->signal_batch = k.signal_batch;
  info->slots = k.slots;
  info->threads = k.threads;
  info->algo = c->algo();
  info->blocking = k.blocking;
  info->sys_fence = k.sys_fence;
  info->timeout_s = k.timeout_ms / 1000.0;
  info->scratch_bytes = c->scratch_bytes();
  info->tune_ms[0] = info->tune_ms[1] = 0.0;  // round 1's init-time calibration, removed in 0.3.1
  info->channels = c->workgroups();
  info->pipelines = c->wave_channels();
  info->ranks_on_device = c->ranks_on_device();
  info->slot_bytes = c->wave_slice();
  info->last_algo = c->last_algo();
  info->peer_mappings = c->peer_mappings();
  info->scratch_algo = mncclAlgoRing;  // the read schedule's fallback
  info->calib_choice = -1;              // MINI_NCCL_CALIBRATE was removed in 400
  info->calib_ms[0] = info->calib_ms[1] = 0.0;
  info->ipc_open_failures = mnccl::ipc::open_failures();
  info->read_map_failures = c->peer_buffers().map_failures();
  info->read_rounds = c->peer_buffers().agreements();
  info->closed_freed = c->peer_buffers().closed_freed();
  info->live_exports = mnccl::ipc::live_exports();
  info->cap_refusals = mnccl::ipc::cap_refusals();
  info->liveness_queries = mnccl::ipc::liveness_queries();
  info->read_push = 1;  // since 6.0 the read schedule has only its push form
  info->auto_read = c->topology_allows_read() ? 1 : 0;
  for (int q = 0; q < 16; ++q) {
    info->peer_link[q] = q < c->nranks() ? c->peer_link(q) : -1;
    info->peer_hops[q] = q < c->nranks() ? c->peer_hops(q) : 0;
  }
  snprintf(info->auto_reason, sizeof info->auto_reason, "%s", c->topology_reason().c_str());
  info->read_grid_calls = c->read_grid_calls();
  info->window_calls = c->window_calls();
  info->windows = (int)c->windows();
  info->auto_grid = c->auto_grid() ? 1 : 0;
  info->retired_imports = (int)mnccl::ipc::retired_imports();
  info->retired_bytes = mnccl::ipc::retired_bytes();
  info->retired_budget = mnccl::ipc::retired_budget();
  info->budget_refusals = mnccl::ipc::budget_refusals();
  info->window_fast = c->window_fast() ? 1 : 0;
  info->run_pipelines = c->run_pipes();
  memcpy(out, &full, size < sizeof full ? size : sizeof full);
  return ncclSuccess;
}

// Collective in effect: every rank must select the same schedule before its next call (the
// schedules' messages share mailboxes and slots), as with any other communicator setting.
ncclResult_t mncclCommSetAlgo(ncclComm_t comm, int algo) {
  if (!comm) return ncclInvalidArgument;
  // mncclAlgoDirect (1) was removed in 400: it never beat the ring on any measured setup
  if (algo != mncclAlgoRing && algo != mncclAlgoRead && algo != mncclAlgoOneShot && algo != mncclAlgoReadGrid &&
      algo != mncclAlgoAuto)
    return ncclInvalidArgument;
  reinterpret_cast<Comm*>(comm)->set_algo(algo);
  return ncclSuccess;
}

ncclResult_t mncclCommLinkProbe(ncclComm_t comm, int allPeers, size_t bytes, int iters, double* gbps) {
  if (!comm || !gbps) return ncclInvalidArgument;
  try {
    return reinterpret_cast<Comm*>(comm)->link_probe(allPeers, bytes, iters, gbps);
  } catch (const std::exception& e) {
    fprintf(stderr, "[Mini-NCCL] LinkProbe Error: %s\n", e.what());
    return ncclInternalError;
  } catch (...) {
    return ncclSystemError;
  }
}

ncclResult_t mncclCommRegister(ncclComm_t comm, void* buff, size_t size, void** handle) {
  if (!comm || !buff || !handle || size == 0) return ncclInvalidArgument;
  try {
    return reinterpret_cast<Comm*>(comm)->register_window(buff, size, handle);
  } catch (const std::exception& e) {
    fprintf(stderr, "[Mini-NCCL] CommRegister Error: %s\n", e.what());
    return ncclInternalError;
  } catch (...) {
    return ncclSystemError;
  }
}

ncclResult_t mncclCommDeregister(ncclComm_t comm, void* handle) {
  if (!comm || !handle) return ncclInvalidArgument;
  return reinterpret_cast<Comm*>(comm)->deregister_window(handle);
}

int mncclVersion(void) { return MNCCL_VERSION; }

}  // extern "C"
