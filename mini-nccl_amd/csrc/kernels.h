// kernels.h -- host-side view of the HIP kernels in kernels.hip (launch wrappers only).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace mnccl {

// Element types the kernels are instantiated for (subset of ncclDataType_t values).
enum DType : int { kI32 = 2, kF16 = 6, kF32 = 7, kF64 = 8, kBF16 = 9 };
enum RedOp : int { kSum = 0, kProd = 1, kMax = 2, kMin = 3 };

// Everything a ring / read kernel needs; passed by value as the kernel argument.
struct CollParams {
  const char* send;        // this rank's input (device)
  char* recv;              // this rank's output (device; may equal send)
  uint64_t chunk_bytes;    // (count / n) * elem_size
  uint64_t slice_bytes;    // payload bytes per channel message (<= slot_bytes)
  uint64_t slot_bytes;     // scratch slot stride (fixed per communicator: the configured slice)
  uint64_t nslices;        // ceil(chunk_bytes / slice_bytes)
  uint32_t iters;          // ceil(nslices / A): slices per pipeline of this call
  int32_t n, rank, nslots;
  char* scratch;           // this rank's scratch (regions per source rank)
  uint64_t* mbox;          // this rank's mailbox
  uint64_t* tx_seq;        // [peer][channel] messages sent so far (device, private)
  uint64_t* rx_seq;        // [peer][channel] messages received so far (device, private)
  char* peer_scratch[16];  // peers' scratch bases (IPC-mapped), indexed by rank
  uint64_t* peer_mbox[16]; // peers' mailboxes (IPC-mapped), indexed by rank
  uint32_t* status;        // host-mapped status word (kStatus* bits)
  const uint32_t* host_abort;  // host-mapped abort request
  uint32_t* started;       // host-mapped start word: the kernel writes call_seq when it begins
  uint32_t call_seq;       // this launch's sequence number (Comm::wait_for's deadline starts here)
  uint64_t timeout_ticks;  // s_memrealtime ticks (100 MHz)
  int32_t sys_fence;       // system-scope release fence before each ready flag
  int32_t pipes;           // the communicator's pipelines (mailbox / scratch / counter layout);
                           // a call's grid may run fewer (schedule.h call_pipelines)
  const char* peer_send[16];  // read schedule: every rank's send buffer, mapped here (own at [rank])
  const char* peer_recv[16];  // read schedule: every rank's recv buffer, mapped here
  uint64_t tail_bytes;        // bytes past n * chunk_bytes that the kernel copies send -> recv
                              // (the reference leaves them as its copy made them, api.cpp:173-175)
  uint32_t* claim;            // device word, 0 until the communicator's first give-up claims it:
                              // only that lane writes the status and its diagnostic
  uint32_t* go;               // device word: the read schedule's grid form -- call_seq once START
                              // is through (read_start_kernel), checked by the grid and DONE launches
  uint64_t sig;               // registered-window call (no host rendezvous): this call's signature,
                              // sent with START and compared with every peer's before any peer
                              // buffer is touched (0: a negotiated call, nothing to check)
};

constexpr int kMaxRanks = 16;
// The persistent collective kernels are built for at least this many resident waves per SIMD
// (__launch_bounds__: <= 256 registers per wave): a GPU keeps CUs x 4 SIMDs x this many of their
// waves resident at once, and every rank's pipeline w waits for its peers' pipeline w.
constexpr int kMinWavesPerSimd = 2;

// Launchers return hipSuccess or the launch error; dtype/op must be supported
// (checked by the caller).  vec = 16-byte path (all offsets 16-byte aligned).
hipError_t launch_ring(int dtype, int op, bool vec, int channels, int threads,
                       const CollParams& p, hipStream_t stream);
hipError_t launch_read(int dtype, int op, bool vec, int channels, int threads,
                       const CollParams& p, hipStream_t stream);
hipError_t launch_oneshot(int dtype, int op, bool vec, int channels, int threads,
                          const CollParams& p, hipStream_t stream);
// the read schedule's push form for large calls as three launches (start, grid fold, done):
// schedule.h read_grid_fits(p.chunk_bytes, p.n, kReadGridFloor) (2 <= n <= 8, whole 16-byte vectors), p.go set
// vectors: 0 = schedule.h read_grid_vectors; 1 / 2 / 4 (MINI_NCCL_GRID_VECTORS) for fp32 Sum only
hipError_t launch_read_grid(int dtype, int op, const CollParams& p, hipStream_t stream, int vectors = 0);
// out[i] = op(local[i], incoming[i]) for i < count
hipError_t launch_local_reduce(int dtype, int op, void* out, const void* local,
                               const void* incoming, uint64_t count, hipStream_t stream);

// Link probe: blocks spread over the `nremote` peers move `bytes` between `local` and each
// remote[d]: pushes (pull = false, the schedules' direction) or loads over the link (pull =
// true), with the remote side's cache policy `form`: kProbeSys = the hot path's 16-byte
// sc0 sc1 accesses, kProbeNt = non-temporal, kProbePlain = default policy.  Used to measure
// the xGMI bandwidth the schedules are bound by, and what other access forms would get.
enum : int { kProbeSys = 0, kProbeNt = 1, kProbePlain = 2 };
hipError_t launch_link_probe(char* local, char* const* remote, int nremote, uint64_t bytes, int form, bool pull,
                             hipStream_t stream);

bool dtype_supported(int dtype);
int dtype_size(int dtype);

}  // namespace mnccl
