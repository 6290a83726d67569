// sim.cpp -- host-side simulator of the ring / read / one-shot kernels' protocol, for the CPU test
// suite (no GPU).  Each (rank, channel) runs the same op sequence as kernels.hip, using the
// same schedule.h index math, scratch layout and mailbox layout; a wait that is not
// satisfied yields, and the scheduler round-robins over all programs.  It checks:
//   * the data each rank ends with (compared by the tests against oracle/ring_oracle.c),
//   * deadlock freedom for the given (n, channels, slots, sizes): no progress => -1,
//   * that the per-channel sequence bases carried across calls keep flags consistent.
// fp32 only (the schedule does not depend on the element type); ops as reference
// mini_nccl.cu:38-41 with a = local, b = incoming.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "schedule.h"

using namespace mnccl;

namespace {

float apply(int op, float a, float b) {
  switch (op) {
    case 0: return a + b;
    case 1: return a * b;
    case 2: return (a > b) ? a : b;
    default: return (a < b) ? a : b;
  }
}

struct World {
  int n, C, K, op, algo;
  int A = 0;  // pipelines the current call runs (schedule.h call_pipelines)
  uint64_t slice, slot_bytes, chunk_bytes, nslices;  // payload per message, slot stride
  uint32_t iters;
  std::vector<const float*> send;
  std::vector<float*> recv;
  std::vector<std::vector<char>> scratch;     // per rank
  std::vector<std::vector<uint64_t>> mbox;    // per rank
  std::vector<std::vector<uint64_t>> tx_seq, rx_seq;  // per rank: [peer * C + w]
  std::vector<uint64_t> sig;           // registered-window call: each rank's START signature (empty: none)
  std::vector<int> mismatch;           // per rank: pipelines that saw a differing signature

  // message `seq` from src to dst on pipeline w (schedule.h msg_slot_off: the receiver's scratch)
  char* slot(int src, int dst, int w, uint64_t seq) {
    return scratch[dst].data() + msg_slot_off(C, K, slot_bytes, src, dst, w, seq);
  }
  uint64_t& ready(int owner, int src, int w) { return mbox[owner][mbox_ready(C, src, w)]; }
  uint64_t& credit(int owner, int dst, int w) { return mbox[owner][mbox_credit(n, C, dst, w)]; }
};

// copy / reduce over `bytes` bytes of floats
void do_move(int kind, int op, const float* local, const float* in, float* recv, float* out, uint64_t bytes) {
  const uint64_t ne = bytes / 4;
  for (uint64_t i = 0; i < ne; ++i) {
    float v;
    switch (kind) {
      case kSend: v = local[i]; break;
      case kReduceSend:
      case kReduceCopySend: v = apply(op, local[i], in[i]); break;
      default: v = in[i]; break;
    }
    if (kind == kReduceCopySend || kind == kCopySend || kind == kCopy) recv[i] = v;
    if (kind != kCopy) out[i] = v;
  }
}

struct Prog {
  int r, w;
  uint32_t it = 0;
  int k = 0;      // ring: op index within the iteration
  uint32_t j = 0; // read: stage
  bool done = false;
};

// One ring op (kernels.hip ring_kernel body); returns false if a wait is unsatisfied.
bool ring_step(World& W, Prog& P) {
  const int n = W.n, r = P.r, w = P.w, K = W.K;
  const int prev = mod_n(r - 1, n), next = mod_n(r + 1, n);
  const uint64_t tx_base = W.tx_seq[r][(size_t)next * W.C + w], rx_base = W.rx_seq[r][(size_t)prev * W.C + w];
  const int mpi = ring_msgs_per_iter(n);
  const uint64_t s = (uint64_t)P.it * W.A + w;  // slice s on pipeline s mod A (kernels.hip ring_kernel)
  const uint64_t len = slice_len(W.chunk_bytes, W.slice, s);
  const uint64_t soff = s * W.slice;
  const uint64_t itoff = (uint64_t)P.it * mpi;
  const RingOp o = ring_op(n, r, P.k);
  const uint64_t rseq = rx_base + itoff + (uint64_t)o.recv_msg, sseq = tx_base + itoff + (uint64_t)o.send_msg;
  if (o.recv_msg >= 0 && W.ready(r, prev, w) < rseq + 1) return false;
  if (o.send_msg >= 0 && sseq + 1 > (uint64_t)K && W.credit(r, next, w) < sseq + 1 - K) return false;
  if (len) {
    const uint64_t coff = (uint64_t)o.chunk * W.chunk_bytes + soff;
    const float* local = (const float*)((const char*)W.send[r] + coff);
    float* recv = (float*)((char*)W.recv[r] + coff);
    const float* in = o.recv_msg >= 0 ? (const float*)W.slot(prev, r, w, rseq) : nullptr;
    float* out = o.send_msg >= 0 ? (float*)W.slot(r, next, w, sseq) : nullptr;
    do_move(o.kind, W.op, local, in, recv, out, len);
  }
  if (o.send_msg >= 0) W.ready(next, r, w) = sseq + 1;
  if (o.recv_msg >= 0) W.credit(prev, r, w) = rseq + 1;
  if (++P.k == ring_num_ops(n)) {
    P.k = 0;
    if (++P.it == W.iters) P.done = true;
  }
  return true;
}

// One step of the read schedule (kernels.hip read_kernel): stage 0 publishes START, 1 waits for
// every peer's START, 2 runs the iterations, 3 publishes DONE (+ credits), 4 waits for every
// peer's DONE.  One step per iteration -- the fold of slice it of chunk r from the peers' send
// buffers, stored into this rank's recv AND pushed into every peer's recv at the same offset, no
// READY.  Every peer access touches the peer's own buffers (W.send / W.recv of that rank), so an
// in-place call whose order were wrong would read overwritten data and fail the oracle comparison.
bool read_step(World& W, Prog& P) {
  const int n = W.n, r = P.r, w = P.w;
  auto tx = [&](int d) { return W.tx_seq[r][(size_t)d * W.C + w]; };
  auto rx = [&](int q) { return W.rx_seq[r][(size_t)q * W.C + w]; };
  const uint64_t mpc = read_msgs_per_call(W.iters);
  auto fold = [&](uint32_t it) {  // slice `it` of chunk r, stored and pushed
    const uint64_t s = (uint64_t)it * W.A + w;
    const uint64_t len = slice_len(W.chunk_bytes, W.slice, s);
    const uint64_t coff = (uint64_t)r * W.chunk_bytes + s * W.slice;
    const float* local = (const float*)((const char*)W.send[r] + coff);
    std::vector<float> res((size_t)(len / 4));
    for (uint64_t i = 0; i < len / 4; ++i) {
      float acc = local[i];
      for (int k = 1; k < n; ++k) {
        const int q = direct_peer(n, r, k);
        acc = apply(W.op, ((const float*)((const char*)W.send[q] + coff))[i], acc);
      }
      res[(size_t)i] = acc;
    }
    // every load of the slice came first (in place, recv chunk r of a peer is its send chunk r)
    if (len) {
      memcpy((char*)W.recv[r] + coff, res.data(), (size_t)len);
      for (int k = 1; k < n; ++k) memcpy((char*)W.recv[direct_peer(n, r, k)] + coff, res.data(), (size_t)len);
    }
  };
  switch (P.j) {
    case 0:
      // START (kernels.hip read_kernel).  A registered-window call's signature is stored with it but
      // not drained first, so it may land after the flag: modelled as a later step (stage 5)
      for (int k = 1; k < n; ++k) W.ready(direct_peer(n, r, k), r, w) = tx(direct_peer(n, r, k)) + 1;
      P.j = W.sig.empty() ? 1 : 5;
      return true;
    case 5:
      for (int k = 1; k < n; ++k) W.mbox[direct_peer(n, r, k)][mbox_ready(W.C, r, w) + kSigWord] = W.sig[r];
      P.j = 1;
      return true;
    case 1:
      for (int k = 1; k < n; ++k)
        if (W.ready(r, direct_peer(n, r, k), w) < rx(direct_peer(n, r, k)) + 1) return false;
      if (!W.sig.empty()) {  // kernels.hip starts_agree: wait for each signature, compare, clear
        for (int k = 1; k < n; ++k)
          if (W.mbox[r][mbox_ready(W.C, direct_peer(n, r, k), w) + kSigWord] == 0) return false;
        bool bad = false;
        for (int k = 1; k < n; ++k) {
          uint64_t& word = W.mbox[r][mbox_ready(W.C, direct_peer(n, r, k), w) + kSigWord];
          bad = bad || word != W.sig[r];
          word = 0;
        }
        if (bad) {
          ++W.mismatch[r];
          P.done = true;
          return true;
        }
      }
      P.j = 2;
      P.it = 0;
      P.k = 0;
      return true;
    case 2:
      if (P.it < W.iters) fold(P.it++);
      if (P.it >= W.iters) P.j = 3;
      return true;
    case 3:
      for (int k = 1; k < n; ++k) {
        const int q = direct_peer(n, r, k);
        W.credit(q, r, w) = rx(q) + mpc;
        W.ready(q, r, w) = tx(q) + mpc;
      }
      P.j = 4;
      return true;
    default:
      for (int k = 1; k < n; ++k)
        if (W.ready(r, direct_peer(n, r, k), w) < rx(direct_peer(n, r, k)) + mpc) return false;
      P.done = true;
      return true;
  }
}

// One step of the one-shot schedule (kernels.hip oneshot_kernel): pipeline w = s * n + c owns
// slice s of chunk c.  Stage 0 waits for every peer's credit, stores that piece of its send into
// every peer's slot and raises READY; stage 1 waits for every peer's READY, folds the piece in
// ring order from the slots (its own piece from its send) into recv and returns the credits.
bool oneshot_step(World& W, Prog& P) {
  const int n = W.n, r = P.r, w = P.w, K = W.K;
  auto tx = [&](int d) { return W.tx_seq[r][(size_t)d * W.C + w]; };
  auto rx = [&](int q) { return W.rx_seq[r][(size_t)q * W.C + w]; };
  const int c = w % n;
  const uint64_t s = (uint64_t)(w / n);
  const uint64_t len = slice_len(W.chunk_bytes, W.slice, s), coff = (uint64_t)c * W.chunk_bytes + s * W.slice;
  if (P.j == 0) {
    for (int k = 1; k < n; ++k) {
      const int q = direct_peer(n, r, k);
      if (tx(q) + 1 > (uint64_t)K && W.credit(r, q, w) < tx(q) + 1 - K) return false;
    }
    for (int k = 1; k < n; ++k) {
      const int q = direct_peer(n, r, k);
      if (len) memcpy(W.slot(r, q, w, tx(q)), (const char*)W.send[r] + coff, len);
      W.ready(q, r, w) = tx(q) + 1;
    }
    P.j = 1;
    return true;
  }
  for (int k = 1; k < n; ++k) {
    const int q = direct_peer(n, r, k);
    if (W.ready(r, q, w) < rx(q) + 1) return false;
  }
  auto piece = [&](int q) -> const float* {
    return (const float*)(q == r ? (const char*)W.send[r] + coff : W.slot(q, r, w, rx(q)));
  };
  if (len) {
    // every piece is read before recv's (in place: send's) piece is written
    std::vector<float> res((size_t)(len / 4));
    for (uint64_t i = 0; i < len / 4; ++i) {
      float acc = piece(c)[i];
      for (int k = 1; k < n; ++k) acc = apply(W.op, piece(direct_peer(n, c, k))[i], acc);
      res[(size_t)i] = acc;
    }
    memcpy((char*)W.recv[r] + coff, res.data(), (size_t)len);
  }
  for (int k = 1; k < n; ++k) {
    const int q = direct_peer(n, r, k);
    W.credit(q, r, w) = rx(q) + 1;
  }
  P.done = true;
  return true;
}

}  // namespace

extern "C" {

// csrc/schedule.h one-shot geometry, exported for the host-logic tests
uint64_t mnccl_oneshot_slice(uint64_t chunk_bytes, int n, int channels, uint64_t slot_bytes) {
  return oneshot_slice(chunk_bytes, n, channels, slot_bytes);
}
int mnccl_oneshot_fits(uint64_t chunk_bytes, int n, int channels, uint64_t slot_bytes, int forced) {
  return oneshot_fits(chunk_bytes, n, channels, slot_bytes, forced != 0) ? 1 : 0;
}

// csrc/schedule.h effective_slice, exported for the host-logic tests
uint64_t mnccl_effective_slice(uint64_t chunk_bytes, int channels, uint64_t slice, uint64_t min_slice, int depth) {
  return effective_slice(chunk_bytes, channels, slice, min_slice, depth);
}
// csrc/schedule.h pipeline_geometry (what Comm allocates and launches): out = {workgroups,
// waves, slot_bytes, scratch_bytes}
void mnccl_pipeline_geometry(int n, int channels, int threads, int window, int signal_batch, int slots,
                             uint64_t slice, uint64_t cap, uint64_t* out) {
  const Geometry g = pipeline_geometry(n, channels, threads, window, signal_batch, slots, slice, cap);
  out[0] = (uint64_t)g.workgroups;
  out[1] = (uint64_t)g.waves;
  out[2] = g.slot_bytes;
  out[3] = g.scratch_bytes;
}

uint64_t mnccl_read_slice(uint64_t chunk_bytes, int channels, uint64_t slice, uint64_t min_slice, int depth) {
  return read_slice(chunk_bytes, channels, slice, min_slice, depth);
}

int mnccl_call_pipelines(uint64_t nslices, int channels, int waves) { return call_pipelines(nslices, channels, waves); }
int mnccl_resident_pipes(int P, int waves, int cus, int most, int waves_per_simd) {
  return resident_pipes(P, waves, cus, most, waves_per_simd);
}

// schedule.h topology_blocks_read over an n x n matrix (rank q's row: how q's GPU reaches p's)
int mnccl_topology_blocks_read(int n, const int* link, const int* hops) { return topology_blocks_read(n, link, hops); }
int mnccl_read_grid_form(int forced, int auto_mode, int vec, uint64_t chunk_bytes, int n, uint64_t min_bytes) {
  return read_grid_form(forced != 0, auto_mode != 0, vec != 0, chunk_bytes, n, min_bytes) ? 1 : 0;
}

// Runs `calls` consecutive all-reduces (send -> recv, fp32; send == recv for in place) on n
// simulated ranks with the GPU kernels' protocol; call i uses schedule (algo >> 3i) & 7 (0 ring,
// 1 one-shot, 2 read (persistent kernel), 4 read's grid form (3, the 4.0-5.x load form, is gone) -- START and
// DONE on pipeline 0, the whole chunk folded and pushed between them, as kernels.hip
// read_start / read_grid / read_done do; schedules can alternate on one communicator state, as
// mncclCommSetAlgo allows; at most 21 calls).  A one-shot call's slice: oneshot_slice when
// min_slice != 0 (Comm::launch; -2 if the call does not fit), else the slot.  schedule_seed != 0 permutes the order programs are tried
// in (pseudo-random), exploring different interleavings.  min_slice: 0 = fixed payload (the
// configured slice), else the adaptive payload of Comm::launch.  Returns 0, -1 on deadlock,
// -2 on bad arguments.  *steps_out = ops executed.
int mnccl_sim_allreduce(uint64_t algo, const float* const* send, float* const* recv, int n, uint64_t count, int op,
                        uint64_t slice_bytes, uint64_t min_slice, int channels, int slots, int calls,
                        uint64_t schedule_seed, uint64_t* steps_out) {
  if (n < 1 || n > 16 || channels < 1 || slots < 1 || slice_bytes < 4 || slice_bytes % 4) return -2;
  World W;
  W.n = n; W.C = channels; W.K = slots; W.op = op; W.algo = (int)algo; W.slot_bytes = slice_bytes;
  const uint64_t chunk = count / (uint64_t)n;
  W.chunk_bytes = chunk * 4;
  W.send.assign(send, send + n);
  W.recv.assign(recv, recv + n);
  // n - 1 regions per rank, exactly as Comm allocates (schedule.h region_index)
  W.scratch.assign((size_t)n, std::vector<char>((size_t)(n > 1 ? n - 1 : 1) * scratch_region_bytes(channels, slots, slice_bytes)));
  W.mbox.assign((size_t)n, std::vector<uint64_t>((size_t)mbox_words(n, channels), 0));
  W.tx_seq.assign((size_t)n, std::vector<uint64_t>((size_t)n * channels, 0));
  W.rx_seq.assign((size_t)n, std::vector<uint64_t>((size_t)n * channels, 0));
  uint64_t steps = 0;
  uint64_t rng = schedule_seed * 6364136223846793005ull + 1442695040888963407ull;
  for (int call = 0; call < calls; ++call) {
    const int code = (int)((algo >> (3 * call)) & 7);
    if (code > 4 || code == 3) return -2;
    const int a = code >= 2 ? 2 : code;  // 0 ring, 1 one-shot, 2 read
    // as Comm::launch: adaptive payload (min_slice 0 = off; the read schedule's own rule), fixed
    // slot stride, one pipeline per slice up to all of them
    if (a == 1 && W.chunk_bytes) {
      if (min_slice && !oneshot_fits(W.chunk_bytes, n, channels, slice_bytes, true)) return -2;
      W.slice = min_slice ? oneshot_slice(W.chunk_bytes, n, channels, slice_bytes) : slice_bytes;
      if ((W.chunk_bytes + W.slice - 1) / W.slice * (uint64_t)n > (uint64_t)channels) return -2;
    } else if (!min_slice || a == 1) W.slice = slice_bytes;
    else if (a == 2) W.slice = read_slice(W.chunk_bytes, channels, slice_bytes, min_slice, kReadDepth);
    else W.slice = effective_slice(W.chunk_bytes, channels, slice_bytes, min_slice, 1);
    if (code == 4 && W.chunk_bytes) W.slice = W.chunk_bytes;  // grid form: one "slice", pipeline 0's protocol
    W.nslices = (W.chunk_bytes + W.slice - 1) / W.slice;
    W.A = call_pipelines(a == 1 ? W.nslices * (uint64_t)n : W.nslices, channels, 1);  // one-shot: per chunk too
    W.iters = (uint32_t)((W.nslices + (uint64_t)W.A - 1) / (uint64_t)W.A);
    for (int r = 0; r < n; ++r) {  // send -> recv copy of the tail (Comm::allreduce)
      if ((const void*)recv[r] == (const void*)send[r]) continue;  // in place
      const uint64_t body = W.chunk_bytes * (uint64_t)n;
      if (n == 1 || chunk == 0) memcpy(recv[r], send[r], count * 4);
      else if (count * 4 > body) memcpy((char*)recv[r] + body, (const char*)send[r] + body, count * 4 - body);
    }
    if (n == 1 || chunk == 0) continue;
    std::vector<Prog> progs;
    for (int r = 0; r < n; ++r)
      for (int w = 0; w < channels; ++w) {
        Prog p;
        p.r = r; p.w = w;
        p.done = W.iters == 0 || w >= W.A;  // pipelines past A sit the call out
        progs.push_back(p);
      }
    for (;;) {
      bool any = false, all_done = true;
      const size_t np = progs.size();
      const size_t start = schedule_seed ? (size_t)((rng >> 33) % np) : 0;
      for (size_t j = 0; j < np; ++j) {
        Prog& P = progs[(start + j) % np];
        if (P.done) continue;
        all_done = false;
        // a random number of ops per turn for this program when seeded
        int burst = 1;
        if (schedule_seed) {
          rng = rng * 6364136223846793005ull + 1442695040888963407ull;
          burst = 1 + (int)((rng >> 40) % 4);
        }
        for (int b = 0; b < burst && !P.done; ++b) {
          const bool ok = a == 2 ? read_step(W, P) : a == 1 ? oneshot_step(W, P) : ring_step(W, P);
          if (!ok) break;
          any = true;
          ++steps;
        }
      }
      if (schedule_seed) rng = rng * 6364136223846793005ull + 1442695040888963407ull;
      if (all_done) break;
      if (!any) return -1;  // deadlock
    }
    // the kernels' last action per pipeline that ran: advance the per-pair FIFO counters
    for (int r = 0; r < n; ++r)
      for (int w = 0; w < W.A; ++w) {
        if (a == 2 || a == 1) {
          const uint64_t m = a == 2 ? read_msgs_per_call(W.iters) : 1;  // one-shot: one message each way
          for (int q = 0; q < n; ++q) {
            if (q == r) continue;
            W.tx_seq[r][(size_t)q * channels + w] += m;
            W.rx_seq[r][(size_t)q * channels + w] += m;
          }
        } else {
          const uint64_t m = (uint64_t)W.iters * ring_msgs_per_iter(n);
          W.tx_seq[r][(size_t)mod_n(r + 1, n) * channels + w] += m;
          W.rx_seq[r][(size_t)mod_n(r - 1, n) * channels + w] += m;
        }
      }
  }
  if (steps_out) *steps_out = steps;
  return 0;
}

// One read call (push form) on registered windows: every rank's START carries sigs[r] and every
// pipeline compares its peers' with its own before touching data (kernels.hip starts_agree).
// mismatch_out[r] = pipelines of rank r that gave up.  0: every pipeline ran; 1: some gave up
// (then every pipeline must have, and no recv touched); -1 deadlock; -2 bad arguments.
int mnccl_sim_signed_read(const float* const* send, float* const* recv, int n, uint64_t count, int channels,
                          uint64_t slice_bytes, const uint64_t* sigs, uint64_t schedule_seed, int* mismatch_out) {
  if (n < 2 || n > 16 || channels < 1 || slice_bytes < 4 || slice_bytes % 4) return -2;
  World W;
  W.n = n; W.C = channels; W.K = 2; W.op = 0; W.algo = 2; W.slot_bytes = slice_bytes;
  W.chunk_bytes = count / (uint64_t)n * 4;
  W.send.assign(send, send + n);
  W.recv.assign(recv, recv + n);
  W.mbox.assign((size_t)n, std::vector<uint64_t>((size_t)mbox_words(n, channels), 0));
  W.tx_seq.assign((size_t)n, std::vector<uint64_t>((size_t)n * channels, 0));
  W.rx_seq.assign((size_t)n, std::vector<uint64_t>((size_t)n * channels, 0));
  W.sig.assign(sigs, sigs + n);
  W.mismatch.assign((size_t)n, 0);
  W.slice = slice_bytes;
  W.nslices = (W.chunk_bytes + W.slice - 1) / W.slice;
  W.A = call_pipelines(W.nslices, channels, 1);
  W.iters = (uint32_t)((W.nslices + (uint64_t)W.A - 1) / (uint64_t)W.A);
  if (W.chunk_bytes == 0) return -2;
  std::vector<Prog> progs;
  for (int r = 0; r < n; ++r)
    for (int w = 0; w < W.A; ++w) {
      Prog p;
      p.r = r; p.w = w;
      progs.push_back(p);
    }
  uint64_t rng = schedule_seed * 6364136223846793005ull + 1442695040888963407ull;
  for (;;) {
    bool any = false, all_done = true;
    const size_t np = progs.size();
    rng = rng * 6364136223846793005ull + 1442695040888963407ull;
    const size_t start = (size_t)((rng >> 33) % np);
    for (size_t j = 0; j < np; ++j) {
      Prog& P = progs[(start + j) % np];
      if (P.done) continue;
      all_done = false;
      rng = rng * 6364136223846793005ull + 1442695040888963407ull;
      const int burst = 1 + (int)((rng >> 40) % 4);
      for (int b = 0; b < burst && !P.done; ++b) {
        if (!read_step(W, P)) break;
        any = true;
      }
    }
    if (all_done) break;
    if (!any) return -1;
  }
  int total = 0;
  for (int r = 0; r < n; ++r) {
    mismatch_out[r] = W.mismatch[r];
    total += W.mismatch[r];
  }
  return total ? 1 : 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// Host-only hooks for the CPU test suite: the bootstrap (TCP star) and the env config,
// exercised without a GPU.  Not part of libmini_nccl.so.
#include <stdio.h>

#include <stdexcept>
#include <string>

#include <unistd.h>

#include "bootstrap.h"
#include "config.h"
#include "kernels.h"
#include "peerbuf.h"

extern "C" {

// connect, all-gather a 256-byte record per rank, barrier twice; 0 on success,
// -1 on exception, -2 if gathered contents are wrong.
int mnccl_bootstrap_selftest(int rank, int nranks, const char* ip, int port, int timeout_ms) {
  try {
    mnccl::Bootstrap b;
    b.connect(rank, nranks, ip ? ip : "127.0.0.1", port, timeout_ms / 1000.0);
    unsigned char mine[256];
    for (int i = 0; i < 256; ++i) mine[i] = (unsigned char)(rank * 31 + i);
    std::vector<unsigned char> all((size_t)nranks * 256);
    b.allgather(mine, all.data(), 256);
    b.barrier();
    for (int r = 0; r < nranks; ++r)
      for (int i = 0; i < 256; ++i)
        if (all[(size_t)r * 256 + i] != (unsigned char)(r * 31 + i)) return -2;
    b.barrier();
    return 0;
  } catch (const std::exception& e) {
    fprintf(stderr, "bootstrap selftest rank %d: %s\n", rank, e.what());
    return -1;
  }
}

// The read schedule's per-call rendezvous (csrc/peerbuf.cpp) across real processes, without a
// GPU: every call is negotiated with eligible = false (host buffers), so no HIP call is made
// and the decision must be kFallback on every rank -- except where the ranks disagree on the
// count (scenario 1: call calls/2 -> kMismatch everywhere) or one rank never calls (scenario 2:
// the others time out).  Scenario 3 adds random host delays per rank (the 16-record board
// wraps around many times).  decisions[i] = PeerBuffers::Decision of call i, -9 on timeout.
// Returns 0, -1 on an unexpected exception, -3 without shared memory.
int mnccl_board_selftest(int rank, int nranks, const char* ip, int port, int scenario, int calls,
                         double timeout_s, int* decisions) {
  try {
    mnccl::Bootstrap b;
    b.connect(rank, nranks, ip ? ip : "127.0.0.1", port, 20.0);
    std::vector<uint64_t> nonces((size_t)nranks);
    for (int q = 0; q < nranks; ++q) nonces[(size_t)q] = 1000u + (uint64_t)q;  // one process per rank
    mnccl::PeerBuffers pb;
    // scenario 7: the last rank's descriptor socket is out of its peers' reach (another network
    // namespace): init must turn the read schedule off on EVERY rank (-3), within seconds
    if (scenario == 7 && rank == nranks - 1) pb.set_test_unreachable(true);
    pb.init(b, rank, nranks, nonces, port);
    if (!pb.available()) return -3;
    // scenarios 4 / 5: every rank eligible with synthetic buffers (no HIP); 4: rank 1 cannot map
    // on call 3 (every rank must fall back on that call alone); 5: the same buffers every call
    // after the first (the mapping round runs once), except a fresh buffer on call calls/2
    // scenario 6: as 5, and at call calls/2 every rank reports its first buffers freed (its
    // peers close their mappings of them, every rank forgets them)
    std::vector<char> arena(1 << 20);
    const bool fake = scenario == 4 || scenario == 5 || scenario == 6;
    if (fake) pb.set_test_fake(true, scenario == 4 && rank == 1 ? 3u : 0u);
    uint64_t rng = 0x9E3779B97F4A7C15ull * (uint64_t)(rank + 1);
    for (int i = 0; i < calls; ++i) decisions[i] = 99;
    for (int i = 0; i < calls; ++i) {
      if (scenario == 2 && rank == nranks - 1) break;  // this rank never reaches the calls
      if (scenario == 3) {
        rng = rng * 6364136223846793005ull + 1442695040888963407ull;
        usleep((useconds_t)((rng >> 33) % 300));
      }
      const uint64_t count = (scenario == 1 && i == calls / 2) ? 1000u + (uint64_t)rank : 1000u;
      const char* ps[mnccl::kMaxRanks] = {};
      const char* pr[mnccl::kMaxRanks] = {};
      bool vec = false;
      try {
        const void* sb = nullptr;
        void* rb = nullptr;
        if (scenario == 4) {  // a new send / recv page every call
          sb = arena.data() + (size_t)(2 * i) * 4096 % arena.size();
          rb = arena.data() + (size_t)(2 * i + 1) * 4096 % arena.size();
        } else if (scenario == 5 || scenario == 6) {
          const int gen = scenario == 6 ? (i >= calls / 2 ? 1 : 0) : i == calls / 2 ? 1 : 0;
          if (scenario == 6 && i == calls / 2)
            for (int g = 0; g < 2; ++g) {
              const char* p = arena.data() + (size_t)g * 4096;
              pb.test_report_freed((uint64_t)(uintptr_t)p & ~(uint64_t)4095, (uint64_t)(uintptr_t)p);
            }
          sb = arena.data() + (size_t)(2 * gen) * 4096;
          rb = arena.data() + (size_t)(2 * gen + 1) * 4096;
        }
        decisions[i] = (int)pb.negotiate(sb, rb, fake, count, 7, 0, timeout_s, [] {}, ps, pr, &vec);
        if (fake) decisions[i] += 10 * (int)pb.agreements();  // decision + 10 x mapping rounds so far
        if (scenario == 6) decisions[i] += 1000 * (int)pb.closed_freed();  // + 1000 x mappings closed
      } catch (const std::runtime_error&) {
        decisions[i] = -9;
        break;
      }
    }
    b.barrier();
    return 0;
  } catch (const std::exception& e) {
    fprintf(stderr, "board selftest rank %d: %s\n", rank, e.what());
    return -1;
  }
}

// Config::from_env() rendered to text; -1 if the environment is invalid.
int mnccl_config_describe(char* buf, int len) {
  try {
    const std::string s = mnccl::Config::from_env().describe();
    snprintf(buf, (size_t)len, "%s", s.c_str());
    return 0;
  } catch (const std::exception& e) {
    snprintf(buf, (size_t)len, "%s", e.what());
    return -1;
  }
}

}  // extern "C"
