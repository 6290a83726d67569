// schedule.h -- the per-channel message schedules, shared verbatim by the HIP kernels
// (kernels.hip) and by the host-side schedule simulator (sim.cpp, run by the CPU test
// suite), so the index math the GPU executes is the index math the CPU tests check.
//
// Ring (reference mini_nccl.cu:108-194).  The reference walks step-major: for each step,
// every slice of the chunk.  Each element's arithmetic depends only on which chunk it
// is in, so we walk slice-major per channel instead (for each slice owned by the
// channel, all 2(n-1) steps), which keeps every link busy with a 2-slot FIFO and gives
// per element exactly the reference's sequence of ops:
//   op 0         : send the raw chunk r                         (SR step 0 send, :128-131)
//   op 1..n-1    : SR step i = op-1 receives chunk (r-i-1) mod n (:110) and reduces
//                  op(local, incoming) (:126); i < n-2 forwards the partial (the next
//                  step's send of the same chunk, :109), i == n-2 is the final value of
//                  chunk r+1: stored to recv AND forwarded (all-gather step 0, :160)
//   op n..2n-2   : AG step j = op-n receives chunk (r-j) mod n (:172, the sender's
//                  send_idx (r-1)-j+1), stores it to recv, forwards unless j == n-2.
// Messages per channel iteration: 2(n-1) sent to r+1, 2(n-1) received from r-1.
//
// Read (the default for device buffers, same fold order, every link): rank r folds slice s of
// its own chunk r straight from the peers' send buffers in ring order r, r+1, ..., r-1
// (acc = op(x_q, acc): the visited rank's value is the LEFT/local operand exactly as at rank q
// of the ring) and pushes the result into every peer's recv (kernels.hip read_kernel).
//
// One-shot (small calls the read schedule cannot take): every rank stores its pieces into every
// peer's scratch and folds each piece of the result from all n ranks in that same order
// (kernels.hip oneshot_kernel; geometry below).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MNCCL_HD __host__ __device__ __forceinline__
#else
#define MNCCL_HD inline
#endif

namespace mnccl {

enum RingKind : int {
  kSend = 0,            // out <- local
  kReduceSend = 1,      // out <- op(local, in)
  kReduceCopySend = 2,  // v = op(local, in); recv <- v; out <- v
  kCopySend = 3,        // recv <- in; out <- in
  kCopy = 4             // recv <- in
};

struct RingOp {
  int kind;
  int chunk;     // chunk index the op touches
  int send_msg;  // message index (within the iteration) sent to r+1, or -1
  int recv_msg;  // message index received from r-1, or -1
};

// Threads per workgroup of the persistent kernels (MINI_NCCL_THREADS is clamped to it): the
// launch bound lets the compiler give a pipeline's wave up to 512 VGPRs instead of the 128 a
// 1024-thread bound allows (the direct fold spilled at 128); one wave per workgroup is the default.
constexpr int kMaxThreads = 256;
// Largest message payload / slot stride (MINI_NCCL_SLICE_SIZE is clamped to it): message
// lengths and slot offsets are 32-bit in the kernels' buffer resources.
constexpr uint64_t kMaxSlice = 256ull << 20;
// Default pipelines of the persistent kernels: one per CU of the 256.
constexpr int kDefaultPipelines = 256;

MNCCL_HD int mod_n(int a, int n) { return ((a % n) + n) % n; }

MNCCL_HD int ring_num_ops(int n) { return 2 * n - 1; }
MNCCL_HD int ring_msgs_per_iter(int n) { return 2 * (n - 1); }

MNCCL_HD RingOp ring_op(int n, int r, int k) {
  RingOp o;
  if (k == 0) {
    o.kind = kSend; o.chunk = r; o.send_msg = 0; o.recv_msg = -1;
  } else if (k < n) {
    const int i = k - 1;
    o.kind = (i < n - 2) ? kReduceSend : kReduceCopySend;
    o.chunk = mod_n(r - i - 1, n);
    o.send_msg = k; o.recv_msg = k - 1;
  } else {
    const int j = k - n;
    o.kind = (j < n - 2) ? kCopySend : kCopy;
    o.chunk = mod_n(r - j, n);
    o.send_msg = (j < n - 2) ? k : -1;
    o.recv_msg = k - 1;
  }
  return o;
}

// Peer order of the read schedule's fold (ring order from r + 1) and of its pushes.
MNCCL_HD int direct_peer(int n, int r, int k) { return mod_n(r + k, n); }  // k = 1..n-1

// Read schedule (MINI_NCCL_ALGO=read): no scratch; rank r loads the peers' raw slices of chunk
// r straight from their send buffers and stores the result into every rank's recv.  Messages per
// (pair, pipeline) and call, all on the READY word: START and DONE; the count advances by
// iters + 2 (the 4.0-5.x load form also sent one READY per iteration; every rank counts alike).
MNCCL_HD uint64_t read_msgs_per_call(uint32_t iters) { return (uint64_t)iters + 2; }

// Pipelines a call runs (ring and read alike): one per slice, up to all C of them, rounded up to
// whole workgroups of `waves` pipelines.  The others sit the call out on every rank alike (a
// pure function of the call's size and the rank-uniform geometry), so their per-pair counters
// stay in step; a small call then dispatches, handshakes and drains a few waves, not C (the
// reference moves only the slices that exist, mini_nccl.cu:112-115).  Slice s of a call goes
// to pipeline s mod A (iteration s / A).
MNCCL_HD int call_pipelines(uint64_t nslices, int C, int waves) {
  uint64_t a = nslices < (uint64_t)C ? nslices : (uint64_t)C;
  if (a == 0) a = 1;
  a = (a + (uint64_t)waves - 1) / (uint64_t)waves * (uint64_t)waves;
  return a < (uint64_t)C ? (int)a : C;
}

// Slice geometry shared by both schedules: pipeline w of a call running A pipelines owns slices
// w, w+A, w+2A, ... of every chunk; message bytes of slice s (0 for the padding slices past the end, which
// still move flags so every channel sends the same number of messages).
MNCCL_HD uint64_t slice_len(uint64_t chunk_bytes, uint64_t slice_bytes, uint64_t s) {
  const uint64_t off = s * slice_bytes;
  if (off >= chunk_bytes) return 0;
  const uint64_t rest = chunk_bytes - off;
  return rest < slice_bytes ? rest : slice_bytes;
}

// Payload bytes per message for one call: the configured slice for large chunks; for chunks
// too small to give every channel `depth` slices of it, ceil(chunk / (C * depth)) rounded up
// to whole waves of 16-byte vectors (1 KiB) and at least `min_slice` (kMinSlice), so small all-reduces
// still spread over every pipeline instead of queueing on a few.  A pure function of the
// call's size and the (rank-uniform) config: every rank picks the same value.  Scratch slot
// addresses keep the configured stride whatever the payload (scratch_slot_off), so calls of
// different sizes never alias each other's slots.  Slicing never changes results.
constexpr uint64_t kMinSlice = 1024;  // one 16-byte vector per lane of a wave
MNCCL_HD uint64_t effective_slice(uint64_t chunk_bytes, int C, uint64_t slice, uint64_t min_slice, int depth) {
  if (min_slice >= slice || depth < 1) return slice;
  const uint64_t per = (uint64_t)C * (uint64_t)depth;
  uint64_t want = (chunk_bytes + per - 1) / per;
  want = (want + 1023) & ~(uint64_t)1023;
  if (want < min_slice) want = min_slice;
  return want < slice ? want : slice;
}

// Read schedule payload: no scratch slot bounds it, so it aims for kReadDepth iterations per
// pipeline (a pipeline's first fold and last copy do not overlap anything: more, smaller
// iterations shrink that fill and drain) while slices stay >= kReadMinSlice; below that, fewer
// iterations of kReadMinSlice, down to the adaptive one-slice-per-pipeline payload of small
// calls.  Measured on the one-GPU proxy, 1 GiB per rank (profiles/r2_read_depth_sweep.txt):
// 4 ranks 508 -> 615 GB/s, 8 ranks 262 -> 301 GB/s, 2 ranks unchanged.  A pure function of the
// call's size and the rank-uniform config, like effective_slice.
constexpr int kReadDepth = 16;
constexpr uint64_t kReadMinSlice = 16u << 10;
MNCCL_HD uint64_t read_slice(uint64_t chunk_bytes, int C, uint64_t slice, uint64_t min_slice, int depth) {
  uint64_t s = effective_slice(chunk_bytes, C, slice, min_slice, depth);
  if (s < kReadMinSlice) {
    const uint64_t one = effective_slice(chunk_bytes, C, slice, min_slice, 1);
    s = one < kReadMinSlice ? one : kReadMinSlice;
  }
  return s;
}

// One-shot (kernels.hip oneshot_kernel): pipeline w = s * n + c carries slice s of chunk c --
// its message to every peer is that piece of this rank's send, and it folds that piece of the
// result from all n ranks' pieces.  A call takes it when its n x nslices pipelines fit one round
// (n x nslices <= C) and its bytes (n chunks) are at most kOneShotMaxBytes -- or at any size that
// fits when forced (MINI_NCCL_ALGO=oneshot).  Each rank sends (n - 1) x the call's bytes: a
// latency path, not a bandwidth one.  Under auto it replaces the ring for small calls whose
// buffers the read schedule cannot take (host memory, a full export table).
constexpr uint64_t kOneShotMaxBytes = 64u << 10;
MNCCL_HD uint64_t oneshot_slice(uint64_t chunk_bytes, int n, int C, uint64_t slot_bytes) {
  const int per = n > 0 && C / n > 0 ? C / n : 1;
  return effective_slice(chunk_bytes, per, slot_bytes, kMinSlice, 1);
}
MNCCL_HD bool oneshot_fits(uint64_t chunk_bytes, int n, int C, uint64_t slot_bytes, bool forced) {
  if (n < 2 || chunk_bytes == 0 || (!forced && chunk_bytes * (uint64_t)n > kOneShotMaxBytes)) return false;
  const uint64_t sl = oneshot_slice(chunk_bytes, n, C, slot_bytes);
  return sl <= slot_bytes && (chunk_bytes + sl - 1) / sl * (uint64_t)n <= (uint64_t)C;
}

// The read schedule's grid form (mncclAlgoReadGrid; kernels.hip read_grid_kernel): three launches
// instead of the persistent kernel -- a one-wave START, a grid of one-batch workgroups that only
// fold and push, a one-wave DONE -- with the protocol of a one-slice read call on pipeline 0.
// Chunks of at least kReadGridMin bytes (MINI_NCCL_GRID_MIN: a tuning knob, rank-uniform), whole
// 16-byte vectors, up to 8 ranks (the fold's peer groups); smaller or ragged calls run the
// persistent read kernel.  Measured in profiles/r4_read_grid_ab.txt and r5_grid_min_ab.txt (on the
// one-GPU proxy the grid form below 4 MiB chunks was slower or equal).
constexpr uint64_t kReadGridMin = 4ull << 20;
constexpr uint64_t kReadGridFloor = 64ull << 10;  // the smallest MINI_NCCL_GRID_MIN
MNCCL_HD bool read_grid_fits(uint64_t chunk_bytes, int n, uint64_t min_bytes = kReadGridMin) {
  return n >= 2 && n <= 8 && chunk_bytes >= min_bytes && chunk_bytes % 16 == 0;
}
// 16-byte vectors per lane in one grid workgroup (V KiB of the chunk, from every peer): one up to
// 4 ranks, two from 5 (profiles/r5_grid_v_ab.txt, 1 GiB per rank on the one-GPU proxy: 8 ranks
// 3.07 vs 4.72 ms per call with V = 2 vs 1 -- as fast as the persistent kernel -- while 2 and 4
// ranks are 7 % and 3 % faster with V = 1)
MNCCL_HD int read_grid_vectors(int n) { return n <= 4 ? 1 : 2; }

// Scratch layout: one region per PEER rank (n - 1 of them: the owner never sends to itself),
// [C][slots][slice_bytes] each.  region_index maps a peer rank q != owner to its region.
MNCCL_HD uint64_t scratch_region_bytes(int C, int slots, uint64_t slice_bytes) { return (uint64_t)C * slots * slice_bytes; }
MNCCL_HD int region_index(int owner, int q) { return q < owner ? q : q - 1; }
MNCCL_HD uint64_t scratch_slot_off(int C, int slots, uint64_t slice_bytes, int region, int w, uint64_t seq) {
  return (uint64_t)region * scratch_region_bytes(C, slots, slice_bytes) +
         ((uint64_t)w * slots + (seq % (uint64_t)slots)) * slice_bytes;
}

// Kernel geometry of one communicator (Comm, and the CPU tests through the simulator library):
// a pure function of the rank-uniform config and n, so every rank computes the same.
//  * workgroups: MINI_NCCL_CHANNELS if set; otherwise one pipeline per CU (256), bounded by the
//    reference's in-flight bound: WINDOW pending signalled requests, each covering SIGNAL_BATCH
//    messages (mini_nccl.cu:119,144,167), i.e. pipelines x slots <= WINDOW x SIGNAL_BATCH
//    messages in flight per link (64 x 16 = 1024 >= 256 x 2 at the defaults);
//  * then the scratch cap: (n-1) regions x pipelines x slots x slot <= cap (fewer pipelines, the
//    payload per message stays MINI_NCCL_SLICE_SIZE; only if one workgroup cannot fit does the
//    slot shrink, to whole KiB).
struct Geometry {
  int workgroups;
  int waves;             // per workgroup (threads / 64): pipelines = workgroups x waves
  uint64_t slot_bytes;   // slot stride and largest payload per message
  uint64_t scratch_bytes;
};
MNCCL_HD Geometry pipeline_geometry(int n, int channels, int threads, int window, int signal_batch, int slots,
                                    uint64_t slice, uint64_t cap) {
  Geometry g;
  g.waves = threads / 64 > 0 ? threads / 64 : 1;
  if (slots < 1) slots = 1;
  if (channels > 0) {
    g.workgroups = channels;
  } else {
    uint64_t inflight = (uint64_t)(window > 0 ? window : 1) * (uint64_t)(signal_batch > 0 ? signal_batch : 1);
    uint64_t P = inflight / (uint64_t)slots;
    if (P > (uint64_t)kDefaultPipelines) P = kDefaultPipelines;
    uint64_t wg = P / (uint64_t)g.waves;
    g.workgroups = wg < 1 ? 1 : (int)wg;
  }
  g.slot_bytes = slice;
  const uint64_t regions = n > 1 ? (uint64_t)(n - 1) : 0;
  if (regions) {
    const uint64_t per_wg = (uint64_t)g.waves * (uint64_t)slots * slice * regions;
    const uint64_t max_wg = cap / per_wg;
    if (max_wg < 1) {
      g.workgroups = 1;
      uint64_t s = (cap / ((uint64_t)g.waves * (uint64_t)slots * regions)) & ~(uint64_t)1023;
      g.slot_bytes = s < 1024 ? 1024 : s;
    } else if ((uint64_t)g.workgroups > max_wg) {
      g.workgroups = (int)max_wg;
    }
  }
  g.scratch_bytes = regions * scratch_region_bytes(g.workgroups * g.waves, slots, g.slot_bytes);
  return g;
}

// Mailbox layout (uint64 words, one 128-byte line per flag):
//   READY(src, w)  : written by rank src when its message for this rank landed
//   CREDIT(dst, w) : written by rank dst when it has consumed a message from this rank
//   ABORT          : written by any rank that gives up (timeout / host abort)
constexpr int kFlagStride = 16;  // uint64 words per flag line
MNCCL_HD uint64_t mbox_ready(int C, int src, int w) { return ((uint64_t)src * C + w) * kFlagStride; }
MNCCL_HD uint64_t mbox_credit(int n, int C, int dst, int w) { return ((uint64_t)n * C + (uint64_t)dst * C + w) * kFlagStride; }
MNCCL_HD uint64_t mbox_abort(int n, int C) { return (uint64_t)2 * n * C * kFlagStride; }
MNCCL_HD uint64_t mbox_words(int n, int C) { return mbox_abort(n, C) + kFlagStride; }

// Where message `seq` from rank `src` to rank `dst` (pipeline w) lives: in the receiver's
// scratch, region src -- the sender's stores cross the link.
MNCCL_HD uint64_t msg_slot_off(int C, int slots, uint64_t slot_bytes, int src, int dst, int w, uint64_t seq) {
  return scratch_slot_off(C, slots, slot_bytes, region_index(dst, src), w, seq);
}

// Topology rule of the default schedule (MINI_NCCL_ALGO=auto).  The read schedule loads from and
// pushes into every peer's memory directly, so it is only the fast path when every pair of GPUs
// is one xGMI hop apart -- an MI355X node's full mesh; over PCIe (or a multi-hop route) every
// byte would cross the host fabric and the ring, which moves 2(n-1)/n of the buffer through one
// neighbour link, is the safer choice.  Ranks sharing a GPU (the reference's perf_test topology)
// reach each other through that GPU's own memory: allowed.  A peer whose GPU this process cannot
// see cannot be classified: not allowed (the runtime could not tell us the link).  The reference
// decides per peer whether its same-host IPC path applies (RDMATransport.h:109-111,583-590);
// here every rank applies this to its own row and the communicator takes the AND over ranks
// (Comm::exchange_and_map), so every rank decides alike.  link[q * n + p] / hops[q * n + p]: how
// rank q's GPU reaches rank p's (kPeerSameGpu, kPeerUnknown, or the HSA link type: 2 PCIe, 4 xGMI).
enum : int { kPeerSameGpu = -1, kPeerUnknown = -2, kLinkPcie = 2, kLinkXgmi = 4 };
// 0: the read schedule may be the default; otherwise 1 + the first offending pair's index q * n + p
MNCCL_HD int topology_blocks_read(int n, const int* link, const int* hops) {
  for (int q = 0; q < n; ++q)
    for (int p = 0; p < n; ++p) {
      if (p == q) continue;
      const int l = link[q * n + p];
      if (l == kPeerSameGpu) continue;
      if (l != kLinkXgmi || hops[q * n + p] != 1) return 1 + q * n + p;
    }
  return 0;
}

// The pipelines a call may launch (Comm::run_pipes): pipeline w of every rank waits for pipeline w
// of its peers, so the waves a call launches on the most crowded GPU -- `most` ranks on a GPU of
// `cus` CUs, each CU's 4 SIMDs keeping `waves_per_simd` of the kernels' waves resident -- must all
// fit at once: min(P, cus x 4 x waves_per_simd / most), whole workgroups of `waves`, at least one.
MNCCL_HD int resident_pipes(int P, int waves, int cus, int most, int waves_per_simd) {
  if (most < 1) most = 1;
  if (waves < 1) waves = 1;
  int cap = cus * 4 * waves_per_simd / most / waves * waves;
  if (cap < waves) cap = waves;
  return P < cap ? P : cap;
}

// Whether a read-schedule call launches in the grid form (kernels.hip read_start / read_grid /
// read_done) rather than the persistent read_kernel: forced (mncclAlgoReadGrid) or under auto,
// for the push form's calls that fit it.  Auto took the grid only with every rank on a GPU of its
// own until the grid's workgroup size followed the rank count (read_grid_vectors); since then it
// measured at least the persistent kernel's rate with co-located ranks too: 2 ranks 1.20x (the
// persistent kernel's bimodal placement), 4 ranks 1.04x, 8 ranks 0.99-1.02x
// (profiles/r5_read_vs_grid_forms.txt, r5_bench_n{2,8}_auto_grid.json).  Uniform across ranks:
// every input is.
MNCCL_HD bool read_grid_form(bool forced, bool auto_mode, bool vec, uint64_t chunk_bytes, int n,
                             uint64_t min_bytes = kReadGridMin) {
  return (forced || auto_mode) && vec && read_grid_fits(chunk_bytes, n, min_bytes);
}

// Kernel status bits (host-mapped status word)
// kStatusMismatch: a registered-window call whose ranks passed different windows / offsets / count /
// dtype / op (the START signatures differ, read_kernel): no data was touched, the call fails with
// ncclInvalidUsage on every rank.
enum : uint32_t { kStatusTimeout = 1u, kStatusHostAbort = 2u, kStatusRemoteAbort = 4u, kStatusMismatch = 8u };

// Word of a READY line (mbox_ready, 16 words per line) that carries the sender's call signature
// with its START of a registered-window call (0 = none).
constexpr int kSigWord = 1;

}  // namespace mnccl
