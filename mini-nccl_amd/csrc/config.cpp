// config.cpp -- see config.h.
#include "config.h"

#include "schedule.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

namespace mnccl {

namespace {

long long env_int(const char* name, long long dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  long long x = std::strtoll(v, &end, 0);
  if (end == v || *end) throw std::invalid_argument(std::string(name) + "=" + v + " is not an integer");
  return x;
}

// Knobs of earlier versions that are gone: set, they would otherwise be ignored silently (a 3.x
// deployment's STAGE_HOST=1 staged pinned buffers; now the kernel always maps them).  Warned once
// per process, naming what replaced each.
void warn_removed_knobs() {
  static bool warned = false;
  if (warned) return;
  warned = true;
  static const struct {
    const char* name;
    const char* now;
  } removed[] = {
      {"MINI_NCCL_PULL", "removed in 4.0 with the direct schedule"},
      {"MINI_NCCL_READ_PUSH", "removed in 6.0: the read schedule always pushes its results into the peers' recv "
                              "(the load form was 1.1-1.45x slower wherever it was measured)"},
      {"MINI_NCCL_DIRECT_OVERLAP", "removed in 4.0 with the direct schedule"},
      {"MINI_NCCL_CALIBRATE", "removed in 4.0: auto decides per call (and, since 5.0, from the topology)"},
      {"MINI_NCCL_CALIBRATE_BYTES", "removed in 4.0 with MINI_NCCL_CALIBRATE"},
      {"MINI_NCCL_PIPE_DEPTH", "removed in 4.0: one slice per pipeline per iteration, sized by the call"},
      {"MINI_NCCL_MIN_SLICE", "removed in 4.0: the adaptive payload's floor is 1 KiB"},
      {"MINI_NCCL_STAGE_HOST", "removed in 4.0: pinned host buffers are always mapped into the kernel, "
                               "pageable ones staged"},
      {"MINI_NCCL_TUNE", "removed in 3.0.1: no init-time calibration"},
  };
  for (const auto& k : removed) {
    const char* v = std::getenv(k.name);
    if (v && *v) fprintf(stderr, "[Mini-NCCL] warning: %s=%s is ignored (%s)\n", k.name, v, k.now);
  }
}

}  // namespace

Config Config::from_env() {
  warn_removed_knobs();
  Config c;
  long long slice = env_int("MINI_NCCL_SLICE_SIZE", 128 * 1024);
  if (slice <= 0) slice = 1024;  // Config.h:50 maps 0 -> 1024
  slice &= ~15LL;                // whole 16-byte vectors per message (slicing never changes results)
  if (slice < 16) slice = 16;
  // message lengths and slot offsets are 32-bit in the kernels (buffer resources): bound it
  if (slice > (long long)kMaxSlice) slice = (long long)kMaxSlice;
  c.slice_size = (size_t)slice;
  c.window_size = (int)env_int("MINI_NCCL_WINDOW_SIZE", 64);
  if (c.window_size <= 0) c.window_size = 1;  // Config.h:51
  c.signal_batch = (int)env_int("MINI_NCCL_SIGNAL_BATCH", 16);
  if (c.signal_batch <= 0) c.signal_batch = 1;
  c.slots = (int)env_int("MINI_NCCL_SLOTS", 2);
  // >= 2: with one slot, op k of a rank would wait for its neighbour's op k (the credit for
  // the message it is about to overwrite) -- a cycle; tests/test_schedule.py shows it
  if (c.slots < 2) c.slots = 2;
  if (c.slots > 64) c.slots = 64;
  // workgroups; each wave is one pipeline.  0 = derived per communicator (Comm::geometry: one
  // pipeline per CU, bounded by WINDOW x SIGNAL_BATCH messages in flight and the scratch cap)
  c.channels = (int)env_int("MINI_NCCL_CHANNELS", 0);
  if (c.channels < 0) c.channels = 0;
  if (c.channels > 1024) c.channels = 1024;
  long long cap_mb = env_int("MINI_NCCL_SCRATCH_MB", 512);
  if (cap_mb < 1) cap_mb = 1;
  if (cap_mb > (64LL << 10)) cap_mb = 64LL << 10;
  c.scratch_cap = (size_t)cap_mb << 20;
  c.threads = (int)env_int("MINI_NCCL_THREADS", 64);
  if (c.threads < 64) c.threads = 64;
  if (c.threads > kMaxThreads) c.threads = kMaxThreads;  // the kernels' launch bound (kernels.h)
  c.threads &= ~63;
  const char* a = std::getenv("MINI_NCCL_ALGO");
  if (a && *a) {
    if (!strcmp(a, "ring")) c.algo = 0;
    else if (!strcmp(a, "read")) c.algo = 2;
    else if (!strcmp(a, "oneshot")) c.algo = 3;
    else if (!strcmp(a, "read_grid")) c.algo = 4;
    else if (!strcmp(a, "auto")) c.algo = -1;
    else if (!strcmp(a, "direct"))  // round 1-3's third schedule: never faster than the ring, removed in 4.0
      throw std::invalid_argument("MINI_NCCL_ALGO=direct is no longer built (4.0): use auto, ring, read or oneshot");
    else throw std::invalid_argument(std::string("MINI_NCCL_ALGO=") + a + " (expected auto|ring|read|oneshot|read_grid)");
  }
  c.blocking = env_int("MINI_NCCL_BLOCKING", 1) != 0;
  c.sys_fence = env_int("MINI_NCCL_SYS_FENCE", 0) != 0;
  c.grid_vectors = (int)env_int("MINI_NCCL_GRID_VECTORS", 0);
  const long long gmin = env_int("MINI_NCCL_GRID_MIN", (long long)kReadGridMin);
  if (gmin < (long long)kReadGridFloor || gmin % 16)
    throw std::invalid_argument("MINI_NCCL_GRID_MIN=" + std::to_string(gmin) + " (expected a multiple of 16, >= " +
                                std::to_string(kReadGridFloor) + ")");
  c.grid_min = (size_t)gmin;
  if (c.grid_vectors != 0 && c.grid_vectors != 1 && c.grid_vectors != 2 && c.grid_vectors != 4)
    throw std::invalid_argument("MINI_NCCL_GRID_VECTORS=" + std::to_string(c.grid_vectors) + " (expected 0, 1, 2 or 4)");
  c.window_rendezvous = (int)env_int("MINI_NCCL_WINDOW_RENDEZVOUS", -1);
  if (c.window_rendezvous < -1 || c.window_rendezvous > 1)
    throw std::invalid_argument("MINI_NCCL_WINDOW_RENDEZVOUS=" + std::to_string(c.window_rendezvous) +
                                " (expected -1, 0 or 1)");
  c.retired_mb = env_int("MINI_NCCL_RETIRED_MB", -1);
  if (c.retired_mb < -1) c.retired_mb = -1;
  c.timeout_ms = (double)env_int("MINI_NCCL_TIMEOUT_MS", 10000);
  if (c.timeout_ms < 1) c.timeout_ms = 1;
  c.port = (int)env_int("MINI_NCCL_PORT", 8888);
  c.bootstrap_timeout_ms = (double)env_int("MINI_NCCL_BOOTSTRAP_TIMEOUT_MS", 60000);
  c.debug = (int)env_int("MINI_NCCL_DEBUG", 0);
  return c;
}

std::string Config::describe() const {
  char b[320];
  snprintf(b, sizeof b,
           "SLICE_SIZE=%zu B, WINDOW=%d, BATCH=%d, slots=%d, channels=%d, threads=%d, scratch_cap=%zu MiB, algo=%s, "
           "blocking=%d, sys_fence=%d, window_rendezvous=%d, grid_vectors=%d, grid_min=%zu B, timeout=%.0f ms, port=%d",
           slice_size, window_size, signal_batch, slots, channels, threads, scratch_cap >> 20,
           algo < 0 ? "auto" : algo == 2 ? "read" : algo == 3 ? "oneshot" : algo == 4 ? "read_grid" : "ring", blocking,
           sys_fence, window_rendezvous, grid_vectors, grid_min, timeout_ms, port);
  return b;
}

}  // namespace mnccl
