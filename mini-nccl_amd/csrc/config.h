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
  int algo = -1;                   // MINI_NCCL_ALGO    auto (-1) | ring (0) | direct (1) | read (2)
  int blocking = 1;                // MINI_NCCL_BLOCKING host waits for the stream (reference behaviour)
  int sys_fence = 0;               // MINI_NCCL_SYS_FENCE 1: system release / acquire fences around each hand-off
  size_t min_slice = 1024;         // MINI_NCCL_MIN_SLICE smallest adaptive payload (>= SLICE_SIZE: adaptation off)
  int pipe_depth = 1;              // MINI_NCCL_PIPE_DEPTH slices per pipeline targeted for small calls
  int direct_overlap = 1;          // MINI_NCCL_DIRECT_OVERLAP next iteration's raw pushes before this one's results
  int pull = 0;                    // MINI_NCCL_PULL   1: slots in the sender's scratch, loaded over the link
  int stage_host = 0;              // MINI_NCCL_STAGE_HOST pinned host buffers: 0 = kernel maps them, 1 = staged copy
  int calibrate = 0;               // MINI_NCCL_CALIBRATE auto algo: time read vs the scratch schedule on the first
                                   //   large calls and keep the faster; 0 off (default: the scratch schedule has not
                                   //   yet run across GPUs), 1 on, "auto" = when the ranks span >1 GPU
  size_t calibrate_bytes = 64u << 20;  // MINI_NCCL_CALIBRATE_BYTES calls at least this large are timed / switched
  double timeout_ms = 10000.0;     // MINI_NCCL_TIMEOUT_MS (reference watchdog: 10 s)
  int port = 8888;                 // MINI_NCCL_PORT   bootstrap port (reference: 8888)
  double bootstrap_timeout_ms = 60000.0;  // MINI_NCCL_BOOTSTRAP_TIMEOUT_MS
  int debug = 0;                   // MINI_NCCL_DEBUG

  static Config from_env();
  std::string describe() const;
};

}  // namespace mnccl
