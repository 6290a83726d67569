/*
 * mini_nccl_ext.h -- MI355X-build extensions next to the drop-in ABI.
 *
 * Nothing here is needed to use the library as a drop-in for the reference; these
 * entry points expose the hot path's pieces for measurement and diagnostics:
 *
 *   mncclLocalReduce     the ★ scatter-reduce element-wise kernel on its own
 *                        (reference elementwise_reduce_kernel, mini_nccl.cu:43-47):
 *                        out[i] = op(local[i], incoming[i]); the 1-GPU "local reduce"
 *                        workload of BASELINE.md and bench.py at N = 1.
 *   mncclCommGetAsyncError  sticky error of a communicator (a timed-out or aborted
 *                        all-reduce leaves the ring state inconsistent; every later
 *                        call returns this error), like NCCL's ncclCommGetAsyncError.
 *   mncclCommGetInfo     resolved configuration of a communicator (mncclCommGetInfoV: the
 *                        caller states its struct's size, so an older caller is never
 *                        written past its end; mncclCommGetInfo writes the pre-300 prefix).
 *   mncclCommSetAlgo     choose the schedule for later calls (same association order).
 *   mncclCommLinkProbe   measure the xGMI write bandwidth the schedules are bound by.
 */
#ifndef MINI_NCCL_EXT_H_
#define MINI_NCCL_EXT_H_

#include "mini_nccl_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* mncclVersion() of the library this header describes, 10000*major + 100*minor + patch:
   300 mncclCommInfo_t grew (mncclCommGetInfoV); 301 user buffers shared as dma-bufs,
   MINI_NCCL_TUNE removed; 400 the direct schedule and MINI_NCCL_PULL / DIRECT_OVERLAP /
   CALIBRATE / PIPE_DEPTH / MIN_SLICE / STAGE_HOST removed, MINI_NCCL_READ_PUSH added, the ring
   runs only the pipelines a call's slices need, mncclCommInfo_t grew again (same prefix);
   401 the one-shot schedule (mncclAlgoOneShot; auto's small calls that would run the ring);
   500 auto runs the read schedule only where every pair of GPUs is one xGMI hop apart (or
   shares a GPU), mncclCommInfo_t grew (same prefix: auto_read, peer_link / peer_hops,
   auto_reason, read_grid_calls, window_calls, windows, auto_grid), mncclAlgoReadGrid, registered windows
   (mncclCommRegister / mncclCommDeregister: read calls with no host rendezvous);
   501 imports of a same-GPU peer's memory are never unmapped while the process lives (the GPU
   driver's handle loss), mncclCommInfo_t grew (same prefix: retired_imports), auto's
   large read calls take the grid form wherever it fits (co-located ranks too);
   600 the read schedule's load form and MINI_NCCL_READ_PUSH removed (read_push is always 1), a
   byte budget on retired same-GPU imports (MINI_NCCL_RETIRED_MB; mncclCommInfo_t grew, same
   prefix: retired_bytes, retired_budget, budget_refusals, window_fast, run_pipelines), window calls carry the
   schedule choice in their signature and skip the host rendezvous only when no two ranks share a
   GPU (MINI_NCCL_WINDOW_RENDEZVOUS) */
#define MNCCL_VERSION 600

/* schedules; all produce bit-identical results (same fold order per element) */
typedef enum {
  mncclAlgoAuto = -1,  /* the library's default: read for device buffers every rank can share
                          when every pair of GPUs is one xGMI hop apart (or shares a GPU: see
                          mncclCommInfo_t.auto_read) -- its large calls in the grid form (since 501
                          wherever they fit it, co-located ranks too; 500: only when every rank had
                          a GPU of its own), the rest persistent; every other call one-shot when at
                          most 64 KiB, else the ring */
  mncclAlgoRing = 0,   /* the reference's ring: neighbour r -> r+1, 2(n-1) steps */
  mncclAlgoDirect = 1, /* removed in 400 (never faster than the ring); mncclCommSetAlgo and
                          MINI_NCCL_ALGO reject it */
  mncclAlgoRead = 2    /* no scratch: rank c loads the peers' slices of chunk c straight from
                          their send buffers (mapped per allocation, negotiated per call) and
                          folds them in the same order, then stores the result into its own
                          recv AND into every peer's recv -- the peers write chunk c of YOUR
                          recv during the call, and those writes are visible to your stream's
                          work after the call.  A call whose buffers some rank
                          cannot share (host memory, a full export table) runs the ring
                          instead, on every rank alike */,
  mncclAlgoOneShot = 3 /* since 401, small calls: every rank stores its whole input into every
                          peer's scratch in one message per pipeline and folds all n chunks
                          itself in the same order -- one hand-off instead of the ring's
                          2(n-1).  mncclAlgoAuto takes it for calls of at most 64 KiB that the
                          read schedule cannot take (host buffers, a full export table); forced,
                          every call whose pieces fit one round of the pipelines (the others run
                          as with mncclAlgoAuto) */,
  mncclAlgoReadGrid = 4 /* since 500: mncclAlgoRead with its large calls (chunks of >= 4 MiB, whole
                           16-byte vectors, up to 8 ranks, push form) launched as a one-wave START,
                           a grid of one-batch fold workgroups and a one-wave DONE instead of the
                           persistent kernel; the same bits.  A runtime form for the node to
                           measure beside the default (mncclCommInfo_t.read_grid_calls) */
} mncclAlgo_t;

typedef struct {
  int rank, nranks, device;
  size_t slice_bytes;     /* MINI_NCCL_SLICE_SIZE: bytes per channel message */
  int window;             /* MINI_NCCL_WINDOW_SIZE \ pipelines x slots <= WINDOW x SIGNAL_BATCH: the  */
  int signal_batch;       /* MINI_NCCL_SIGNAL_BATCH / reference's bound on messages in flight per link */
  int channels;           /* workgroups of the persistent kernel; each wave is one pipeline */
  int slots;              /* scratch slots per channel (2 = the reference's double buffer) */
  int threads;            /* threads per workgroup */
  int algo;               /* mncclAlgo_t used by ncclAllReduce */
  int blocking;           /* MINI_NCCL_BLOCKING */
  int sys_fence;          /* MINI_NCCL_SYS_FENCE: system-scope release fence before each flag */
  double timeout_s;       /* MINI_NCCL_TIMEOUT_MS / 1000 */
  size_t scratch_bytes;   /* device scratch owned by this rank */
  double tune_ms[2];      /* always 0 since 301 (MINI_NCCL_TUNE was removed); kept for the
                             layout */
  int pipelines;          /* channels x threads / 64 */
  int ranks_on_device;    /* ranks of this communicator on this rank's GPU (itself included) */
  size_t slot_bytes;      /* largest payload per message (MINI_NCCL_SLICE_SIZE unless the
                             scratch cap MINI_NCCL_SCRATCH_MB shrank it) */
  int last_algo;          /* schedule the last all-reduce ran (mncclAlgo_t; -1: no kernel
                             yet): mncclAlgoRead falls back to the scratch schedule for a
                             call some rank's buffers cannot take part in */
  size_t peer_mappings;   /* peers' user allocations mapped into this process for the read
                             schedule (dma-buf imports of every communicator; csrc/ipcreg.h) */
  int scratch_algo;       /* the read schedule's fallback for calls whose buffers cannot be
                             shared: always the ring (mncclAlgoRing) */
  int calib_choice;       /* -1 since 400 (MINI_NCCL_CALIBRATE was removed); kept for the layout */
  double calib_ms[2];     /* 0 since 400; kept for the layout */
  /* since 300 */
  unsigned long long ipc_open_failures;  /* user-buffer imports that failed in this process */
  unsigned long long read_map_failures;  /* read calls this rank could not map (call fell back) */
  unsigned long long read_rounds;        /* read calls that needed the mapping round */
  unsigned long long closed_freed;       /* imports closed because their owner freed them */
  size_t live_exports;                   /* this process's user allocations exported and alive */
  /* since 400 */
  unsigned long long cap_refusals;       /* exports / imports refused because this process holds
                                            512 exports / 1024 imports already: each such call
                                            ran the ring (warned once per process) */
  unsigned long long liveness_queries;   /* pointer queries this process made to find freed
                                            exports (per call: the call's own buffers + at most
                                            4 others) */
  int read_push;                         /* always 1 since 600 (the load form and MINI_NCCL_READ_PUSH
                                            were removed); kept for the layout */
  /* since 500 */
  int auto_read;                         /* 1: the topology lets auto run the read schedule (every pair
                                            of ranks shares a GPU or is one xGMI hop apart; the
                                            same on every rank); 0: auto runs the ring */
  int peer_link[16];                     /* how this rank's GPU reaches rank q's: -1 the same GPU,
                                            -2 unknown (not visible here), else the runtime's link
                                            type (hipExtGetLinkTypeAndHopCount: 2 PCIe, 4 xGMI) */
  int peer_hops[16];                     /* hop count of that link (0 for the same GPU) */
  char auto_reason[160];                 /* the rule's verdict in words (NUL-terminated) */
  unsigned long long read_grid_calls;    /* calls this communicator ran in the read schedule's grid
                                            form (mncclAlgoReadGrid) */
  unsigned long long window_calls;       /* calls launched on registered windows: no host rendezvous */
  int windows;                           /* windows registered on this communicator */
  int auto_grid;                         /* 1: auto launches large read calls in the grid form
                                            (mncclAlgoReadGrid's; since 501 whenever auto runs the
                                            read schedule in its push form) */
  /* since 501 */
  int retired_imports;                   /* process-wide: peers' freed allocations on this GPU still
                                            mapped here (same-GPU ranks only; held until the process
                                            exits -- DESIGN.md, Same-GPU handle loss) */
  /* since 600 */
  unsigned long long retired_bytes;      /* process-wide: bytes those retired imports keep mapped */
  unsigned long long retired_budget;     /* MINI_NCCL_RETIRED_MB in bytes (default: 1/8 of this GPU's
                                            memory / the ranks on it): once retired_bytes reaches it, a call that would
                                            map a new buffer of a same-GPU peer runs the ring instead
                                            (on every rank alike) */
  unsigned long long budget_refusals;    /* process-wide: same-GPU imports refused by that budget (each
                                            such call ran the ring; warned once per process) */
  int window_fast;                       /* 1: calls on registered windows launch with no host
                                            rendezvous (MINI_NCCL_WINDOW_RENDEZVOUS=0, or auto when
                                            no two ranks share a GPU); 0: they are negotiated like
                                            other calls (co-located ranks meet faster on the host) */
  int run_pipelines;                     /* the pipelines a call may launch: `pipelines`, capped so
                                            that the waves of every rank sharing a GPU stay resident
                                            together (CUs x 4 SIMDs x 2 waves / ranks on the most
                                            crowded GPU) */
} mncclCommInfo_t;

ncclResult_t mncclLocalReduce(void* out, const void* local, const void* incoming, size_t count,
                              ncclDataType_t datatype, ncclRedOp_t op, hipStream_t stream);

ncclResult_t mncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError);

ncclResult_t mncclCommGetInfo(ncclComm_t comm, mncclCommInfo_t* info);
/* mncclCommGetInfo writes the pre-300 prefix only (up to ipc_open_failures), so a caller built
   against an older header is never overrun; mncclCommGetInfoV writes min(size,
   sizeof(mncclCommInfo_t)) bytes: callers pass their struct's size */
ncclResult_t mncclCommGetInfoV(ncclComm_t comm, void* info, size_t size);

/* every rank must make the same choice before its next all-reduce; mncclAlgoAuto restores the
   default; mncclAlgoDirect -> ncclInvalidArgument (removed in 400) */
ncclResult_t mncclCommSetAlgo(ncclComm_t comm, int algo);

/* Collective diagnostic: every rank streams `bytes` (0 = its whole scratch region) into the
 * next rank's scratch (allPeers bit 0 = 0: one xGMI link per rank, the ring's) or into every
 * peer's at once (bit 0 = 1: the mesh, the read schedule's), `iters` times, with the hot
 * path's store form; *gbps = bytes per second per destination link.  Further bits of allPeers
 * select variants for comparison: bits 1-2 = the remote accesses' cache policy (0 = the hot
 * path's sc0 sc1, 1 = non-temporal, 2 = default), bit 3 = pull (load from the peers' scratch
 * over the link instead of storing into it), bit 4 = the peers' ordinary device memory (a
 * hipMalloc buffer each rank exports for the probe -- what the read schedule loads from)
 * instead of their uncached scratch.  Call only when no all-reduce is in flight on any rank (it
 * overwrites scratch slots). */
ncclResult_t mncclCommLinkProbe(ncclComm_t comm, int allPeers, size_t bytes, int iters, double* gbps);

/* Registered windows (since 500; NCCL's collective buffer registration; since 600 the no-rendezvous
 * launch below applies when no two ranks share a GPU or with MINI_NCCL_WINDOW_RENDEZVOUS=0 --
 * otherwise window calls are negotiated like any other, same results).  COLLECTIVE: every rank
 * calls mncclCommRegister with its buffer of the window -- device memory of its own GPU, the same
 * `size` on every rank -- in the same order (the window's number is the registration's).  After
 * it, an ncclAllReduce whose send and recv lie in registered windows -- the SAME windows at the
 * SAME byte offsets on every rank, with the same count / datatype / op (the symmetric layout of a
 * data-parallel gradient buffer) -- runs the read schedule with no host rendezvous: the call only
 * publishes its record and launches, so with MINI_NCCL_BLOCKING=0 a rank returns without waiting
 * for its peers.  The promise is checked on the device before any peer buffer is touched; a call
 * that breaks it (other windows or offsets on some rank, or an unregistered buffer where a peer
 * passed a registered one) fails with ncclInvalidUsage on every rank and the communicator is no
 * longer usable.  The buffer must stay allocated until mncclCommDeregister (also collective, same
 * order); calls on buffers outside any window are negotiated per call as before.  *handle
 * identifies the window; a communicator of one rank accepts and ignores windows. */
ncclResult_t mncclCommRegister(ncclComm_t comm, void* buff, size_t size, void** handle);
ncclResult_t mncclCommDeregister(ncclComm_t comm, void* handle);

/* library version, 10000*major + 100*minor + patch */
int mncclVersion(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MINI_NCCL_EXT_H_ */
