// peerbuf.h -- the read schedule's per-call rendezvous (MINI_NCCL_ALGO=read).
//
// The read schedule loads its peers' send buffers and stores into their recv buffers directly
// (kernels.hip read_kernel),
// so before each call every rank must know where its peers' buffers are mapped in its own
// address space.  The reference exchanged IPC handles of the user buffers through rank 0 on
// EVERY call over TCP and opened/closed them each time (RDMATransport.h:171-257).  Here:
//  * each rank publishes a small record per call -- (allocation base, allocation id, offset,
//    dma-buf inode and offset) of send and recv, count / dtype / op, whether it can take part, and
//    which of its earlier exported allocations it has freed since -- on a board in host shared
//    memory (one node: every rank is on this host), read by its peers with no network round trip;
//  * a call that brings an allocation new to the communicator carries its dma-buf descriptor to
//    every peer process over a Unix datagram socket (SCM_RIGHTS); the peer maps it once and keeps
//    the mapping until the owner reports the allocation freed (ipcreg.h: a dma-buf import keeps
//    its memory alive and can never show another allocation, unlike round 2's hipIpc handles);
//  * every rank reads the same records, so every rank takes the same decision: the read
//    schedule when all ranks can, the ring otherwise, an error when
//    the ranks disagree on count / dtype / op.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <deque>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <vector>

#include "bootstrap.h"
#include "ipcreg.h"

namespace mnccl {

struct Board;  // shared-memory layout (peerbuf.cpp)
struct FdMsg;  // a datagram of descriptors (peerbuf.cpp)

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

  // kWindowPeer: a peer ran this call on registered windows (publish_fast) while this rank's
  // buffers are not in them -- the caller broke the windows' contract
  enum Decision { kRead = 1, kFallback = 0, kMismatch = -1, kWindowPeer = -2 };
  // One call's rendezvous.  `eligible`: this rank's buffers are device memory (the rendezvous
  // also requires them to be memory of this rank's GPU, and shareable).  On kRead, psend /
  // precv[q] hold rank q's buffers mapped here (this rank's own at [rank]) and *vec_all whether
  // every rank's buffers are dword-aligned.  `sync_previous` waits for this communicator's last
  // kernel (before a freed peer allocation's mapping is closed).  `form`: the kernel form this
  // rank would launch for the call (Comm: its schedule choice, mncclCommSetAlgo) -- ranks that
  // differ in it get kMismatch, as for count / dtype / op (a grid-form rank's DONE could otherwise
  // be met by a persistent peer's pipeline 0 while the other pipelines never start).  Throws
  // std::runtime_error when a peer does not arrive within timeout_s.
  Decision negotiate(const void* send, const void* recv, bool eligible, uint64_t count, int dtype, int op,
                     double timeout_s, const std::function<void()>& sync_previous, const char** psend,
                     const char** precv, bool* vec_all, int form = 0);

  // A registered-window call (Comm::allreduce's fast path): this rank's record for the next call,
  // marked fast with the call's signature, published WITHOUT reading the peers' -- their kernels
  // check the signature on the device (kernels.hip starts_agree).  Waits only while the record
  // slot is still unread by some peer (kBoardDepth calls behind); throws as negotiate does.
  void publish_fast(uint64_t count, int dtype, int op, uint64_t sig, double timeout_s);

  // This rank's exported allocations freed since the last call are found and queued for its next
  // record: every export holding send or recv is checked (so known() below cannot name a freed
  // allocation's export), plus kReapBatch others (ipcreg.h).  Call before known() in each call.
  void reap(const void* send, const void* recv);
  // p lies in one of this rank's live exported allocations (no HIP call): device memory of
  // this GPU that the read schedule can share
  bool known(const void* p) const;

  // for tests / diagnostics
  size_t mapped_allocations() const;                    // peer allocations mapped in this process
  uint64_t agreements() const { return agreements_; }  // calls that needed the mapping round
  uint64_t map_failures() const { return map_failures_; }  // opens that failed (any rank's call fell back)
  uint64_t closed_freed() const { return closed_freed_; }  // imports closed because their owner freed them
  // CPU self-test only (no GPU): describe() returns synthetic (base, id) from the pointer value,
  // map_peer() returns the owner's raw address, and map_peer() fails on call `fail_call` (0:
  // never), as a failed hipIpcOpenMemHandle would
  void set_test_fake(bool fake, uint64_t fail_call) {
    test_fake_ = fake;
    test_fail_call_ = fail_call;
  }
  // CPU self-test (before init): bind this rank's socket under another name, as if it lived in
  // another network namespace (its peers' datagrams are refused)
  void set_test_unreachable(bool v) { test_unreachable_ = v; }
  // CPU self-test: report this rank's allocation (base, id) freed with its next record
  void test_report_freed(uint64_t base, uint64_t id) { freed_.emplace_back(base, id); }

 private:
  // descriptors of new allocations, from one rank of another process, for call k
  struct Pending {
    uint64_t k;
    int src, nfd;
    uint64_t base[2], id[2];
    int fd[2];
  };
  using WaitFn = std::function<void(const std::function<bool()>&, int, const char*)>;
  template <typename WaitFor>
  Decision negotiate_body(uint64_t k, const void* send, const void* recv, bool eligible, uint64_t count, int dtype,
                          int op, int form, const std::function<void()>& sync_previous, const char** psend,
                          const char** precv, bool* vec_all, const WaitFor& wait_for);
  bool describe(const void* p, uint64_t* base, uint64_t* id, ipc::Shared* d);
  char* map_peer(int q, uint64_t base, uint64_t id, int fd, const ipc::Shared& d, std::string* why);
  void sock_addr(int q, void* addr, unsigned* len) const;
  int try_send(int q, const FdMsg& m, const int* fds, int nfd);  // 1 sent, 0 queue full, -1 error
  bool drain();  // takes every datagram waiting on my socket into pending_; true if any
  bool hello(double timeout_s);  // init: every rank of another process reachable both ways
  void send_fds(int q, const FdMsg& m, const int* fds, const WaitFn& wait_for);
  Pending take_fds(int q, uint64_t k, const WaitFn& wait_for);

  Board* board_ = nullptr;
  size_t board_bytes_ = 0;
  int rank_ = 0, nranks_ = 0;
  int device_ = -1;
  std::vector<uint64_t> nonces_;
  uint64_t seq_ = 0;  // calls negotiated so far
  // allocations this rank exported and has since freed, not yet published
  std::deque<std::pair<uint64_t, uint64_t>> freed_;
  size_t freed_cursor_ = 0;  // next entry of the process's freed log (ipcreg.h) to publish
  // (rank, base, id) of every buffer a read call ran on and no owner has reported freed since:
  // every rank still maps them (imports stay open until then), so a call whose buffers are all
  // here needs no mapping round.  Derived from the records alone: the same on every rank.
  struct Known {
    int rank;
    uint64_t base, id;
    bool operator==(const Known& o) const { return rank == o.rank && base == o.base && id == o.id; }
  };
  struct KnownHash {
    size_t operator()(const Known& k) const { return std::hash<uint64_t>{}(k.base ^ (k.id << 20) ^ (uint64_t)k.rank); }
  };
  std::unordered_set<Known, KnownHash> known_;
  std::deque<Known> known_order_;  // insertion order, to bound known_
  std::vector<Known> fake_maps_;   // CPU self-test: the "imports"
  uint64_t agreements_ = 0, map_failures_ = 0, closed_freed_ = 0;
  uint64_t fallbacks_ = 0;  // calls that fell back because some rank could not map (warning rate)
  bool test_fake_ = false;
  bool test_unreachable_ = false;
  bool warned_export_ = false;
  int sock_ = -1;          // this rank's datagram socket (abstract namespace), for descriptors
  std::string sock_base_;  // the communicator's socket names: <base>-r<rank>
  std::vector<Pending> pending_;  // arrived, not yet taken
  std::map<std::pair<uint64_t, uint64_t>, int> fake_fds_;  // CPU self-test: a memfd per "allocation"
  uint64_t test_fail_call_ = 0;
};

}  // namespace mnccl
