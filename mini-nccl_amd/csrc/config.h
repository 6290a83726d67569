// config.h -- environment knobs (reference include/Config.h:9-62), resolved once per
// communicator (the scratch ring is sized from them at init, as the reference sizes its
// scratch at Context construction, mini_nccl.cu:14-20).
#pragma once
#include <stddef.h>
#include <string>

namespace mnccl {

struct Config {
  // reference knobs, same names and defaults (Config.h:29-51)
  size_t slice_size = 128 * 1024;  // MINI_NCCL_SLICE_SIZE (bytes per channel message; 0 -> 1024)
  int window_size = 64;            // MINI_NCCL_WINDOW_SIZE \  messages in flight per link <=
  int signal_batch = 16;           // MINI_NCCL_SIGNAL_BATCH / WINDOW x SIGNAL_BATCH (see Comm::geometry)
  // this build's knobs
  int slots = 2;                   // MINI_NCCL_SLOTS   scratch slots per channel (>= 2; 2 = double buffer)
  int channels = 0;                // MINI_NCCL_CHANNELS workgroups (0 -> derived, Comm::geometry)
  size_t scratch_cap = 512u << 20; // MINI_NCCL_SCRATCH_MB cap on this rank's uncached scratch
  int threads = 64;                // MINI_NCCL_THREADS threads per workgroup (one pipeline per wave)
  int algo = -1;                   // MINI_NCCL_ALGO    auto (-1) | ring (0) | read (2) | oneshot (3)
  int blocking = 1;                // MINI_NCCL_BLOCKING host waits for the stream (reference behaviour)
  int sys_fence = 0;               // MINI_NCCL_SYS_FENCE 1: system release / acquire fences around each hand-off
  int grid_vectors = 0;            // MINI_NCCL_GRID_VECTORS 1 / 2 / 4: the grid form's 16-byte vectors per lane
                                   // for fp32 Sum (a tuning knob for the node's sweep); 0 = schedule.h's rule
  size_t grid_min = 4u << 20;      // MINI_NCCL_GRID_MIN: the smallest chunk (bytes) a read call takes the grid
                                   // form for (schedule.h kReadGridMin; >= 64 KiB, 16-byte multiple; rank-uniform)
  int window_rendezvous = -1;      // MINI_NCCL_WINDOW_RENDEZVOUS: calls on registered windows -- 0 launch with
                                   // no host rendezvous (the signature checked on the device), 1 negotiate
                                   // like other calls (the windows' buffers are mapped already), -1 auto:
                                   // 0 unless two ranks share a GPU (Comm::window_fast_; rank-uniform)
  long long retired_mb = -1;       // MINI_NCCL_RETIRED_MB: bytes of freed same-GPU peer allocations this process
                                   // may keep mapped (ipcreg.h close_import), in MiB; -1 = 1/8 of the GPU's
                                   // memory / the ranks on it (Comm resolves it); past it, calls bringing a new same-GPU peer
                                   // buffer run the ring (rank-uniform)
  double timeout_ms = 10000.0;     // MINI_NCCL_TIMEOUT_MS (reference watchdog: 10 s)
  int port = 8888;                 // MINI_NCCL_PORT   bootstrap port (reference: 8888)
  double bootstrap_timeout_ms = 60000.0;  // MINI_NCCL_BOOTSTRAP_TIMEOUT_MS
  int debug = 0;                   // MINI_NCCL_DEBUG

  static Config from_env();
  std::string describe() const;
};

}  // namespace mnccl
