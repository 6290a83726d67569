// peerbuf.h -- the read schedule's per-call rendezvous (MINI_NCCL_ALGO=read).
//
// The read schedule loads its peers' send and recv buffers directly (kernels.hip read_kernel),
// so before each call every rank must know where its peers' buffers are mapped in its own
// address space.  The reference exchanged IPC handles of the user buffers through rank 0 on
// EVERY call over TCP and opened/closed them each time (RDMATransport.h:171-257).  Here:
//  * each rank publishes a small record per call -- (allocation base, allocation id, offset, HIP
//    IPC handle) of send and recv, count / dtype / op, and whether it can take part -- on a
//    board in host shared memory (one node: every rank is on this host), read by its peers
//    with no network round trip;
//  * a peer's allocation is opened once (hipIpcOpenMemHandle) and cached by (rank, base, id):
//    the id (HIP_POINTER_ATTRIBUTE_BUFFER_ID) is new for every allocation, so a freed and
//    re-allocated address is never served from a stale mapping ("key the IPC
//    cache by (base pointer, size) and tolerate address reuse");
//  * every rank reads the same records, so every rank takes the same decision: the read
//    schedule when all ranks can, the communicator's scratch schedule otherwise, an error when
//    the ranks disagree on count / dtype / op.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <deque>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "bootstrap.h"

namespace mnccl {

struct Board;  // shared-memory layout (peerbuf.cpp)

// A peer abandoned the communicator in an earlier rendezvous (its calls fail from now on).
struct PeerGaveUp : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class PeerBuffers {
 public:
  PeerBuffers() = default;
  ~PeerBuffers();
  PeerBuffers(const PeerBuffers&) = delete;
  PeerBuffers& operator=(const PeerBuffers&) = delete;

  // Collective (every rank of the communicator, after the scratch exchange).  nonces[q] is
  // rank q's process nonce: ranks with this process's nonce are addressed by raw pointers.
  // Never throws for a missing /dev/shm: the board is then unavailable on every rank alike.
  void init(Bootstrap& boot, int rank, int nranks, const std::vector<uint64_t>& nonces, int port);
  bool available() const { return board_ != nullptr; }

  enum Decision { kRead = 1, kFallback = 0, kMismatch = -1 };
  // One call's rendezvous.  `eligible`: this rank's buffers are device memory of this GPU.  On kRead, psend / precv[q] hold rank q's buffers mapped
  // here (this rank's own at [rank]) and *vec_all whether every rank's buffers are dword-aligned.
  // `sync_previous` waits for this communicator's last kernel (before a cached mapping is
  // closed).  Throws std::runtime_error when a peer does not arrive within timeout_s.
  // `pin`: the call is being captured into a graph whose replays will read through these
  // mappings: they are never evicted (closed only with the communicator).
  // my_t / max_t (optional): two timings this rank publishes with its record, and per timing
  // the max over every rank's published value, or 0 while some rank's is still unknown (0).
  Decision negotiate(const void* send, const void* recv, bool eligible, uint64_t count, int dtype, int op,
                     double timeout_s, const std::function<void()>& sync_previous, const char** psend,
                     const char** precv, bool* vec_all, bool pin = false, const float* my_t = nullptr,
                     float* max_t = nullptr);
  // Unmaps every peer allocation; call when no kernel of this communicator can still run.
  void close_all();

  // for tests / diagnostics
  size_t mapped_allocations() const { return peers_.size(); }
  uint64_t agreements() const { return agreements_; }  // calls that needed the mapping round
  // CPU self-test only (no GPU): describe() returns synthetic (base, id) from the pointer value,
  // map_peer() returns the owner's raw address, and map_peer() fails on call `fail_call` (0:
  // never), as a failed hipIpcOpenMemHandle would
  void set_test_fake(bool fake, uint64_t fail_call) {
    test_fake_ = fake;
    test_fail_call_ = fail_call;
  }

 private:
  struct Export {
    uint64_t base, id;
    hipIpcMemHandle_t h;
  };
  struct Mapping {
    int rank;
    uint64_t base, id;  // in the owner's process
    char* local;        // the allocation base mapped here
    uint64_t last_use;
    bool pinned;        // used by a captured graph: never evicted
  };
  template <typename Wait>
  Decision negotiate_body(uint64_t k, const void* send, const void* recv, bool eligible, uint64_t count, int dtype,
                          int op, const std::function<void()>& sync_previous, const char** psend, const char** precv,
                          bool* vec_all, bool pin, const float* my_t, float* max_t, const Wait& wait);
  bool describe(const void* p, uint64_t* base, uint64_t* id, hipIpcMemHandle_t* h);
  char* map_peer(int q, uint64_t base, uint64_t id, const hipIpcMemHandle_t& h,
                 const std::function<void()>& sync_previous, bool pin);

  Board* board_ = nullptr;
  size_t board_bytes_ = 0;
  int rank_ = 0, nranks_ = 0;
  std::vector<uint64_t> nonces_;
  uint64_t seq_ = 0;  // calls negotiated so far
  std::vector<Export> exports_;
  std::vector<Mapping> peers_;
  struct RecentKey {
    int rank;
    uint64_t base, id;
  };
  std::deque<std::vector<RecentKey>> recent_;  // buffers of the last read calls (every rank alike)
  uint64_t agreements_ = 0;
  bool test_fake_ = false;
  uint64_t test_fail_call_ = 0;
};

}  // namespace mnccl
