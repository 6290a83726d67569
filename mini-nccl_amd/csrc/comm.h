// comm.h -- the communicator behind ncclComm_t (reference: Context + RDMATransport,
// include/mini_nccl.h:71-111 and src/transport/RDMATransport.h:99-637, re-designed for one
// MI355X node: HIP IPC over xGMI instead of verbs, device scratch instead of host-mapped).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "bootstrap.h"
#include "config.h"
#include "kernels.h"
#include "mini_nccl_api.h"
#include "peerbuf.h"
#include "schedule.h"

namespace mnccl {

class Comm {
 public:
  // Throws on failure; the API layer maps exceptions to ncclSystemError (api.cpp:62-65).
  Comm(int nranks, int rank, const std::string& ip);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  // The hot path: returns an ncclResult_t; throws only on HIP runtime errors.
  ncclResult_t allreduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t stream);

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int device() const { return device_; }
  const Config& config() const { return cfg_; }
  int algo() const { return auto_ ? -1 : algo_; }
  // a < 0: the default (read for buffers every rank can share; for the other calls the one-shot
  // when small, else the ring); 0 ring, 2 read, 3 one-shot wherever a call fits it, 4 read with
  // its large calls in the grid form (kernels.hip read_grid_kernel)
  void set_algo(int a) {
    auto_ = a < 0;
    algo_ = a < 0 ? 2 : a;
  }
  int last_algo() const { return last_algo_; }  // schedule of the last launched kernel, -1: none
  // Registered windows (mncclCommRegister / mncclCommDeregister, collective): a call whose send and
  // recv lie in windows -- the same windows at the same offsets on every rank -- runs the read
  // schedule with no host rendezvous (kernels.hip starts_agree checks the promise on the device)
  ncclResult_t register_window(void* buf, size_t bytes, void** handle);
  ncclResult_t deregister_window(void* handle);
  size_t windows() const { return windows_.size(); }
  unsigned long long window_calls() const { return window_calls_; }
  bool window_fast() const { return window_fast_; }  // window calls skip the host rendezvous
  unsigned long long read_grid_calls() const { return read_grid_calls_; }  // calls run in the grid form
  size_t peer_mappings() const { return pbuf_.mapped_allocations(); }
  const PeerBuffers& peer_buffers() const { return pbuf_; }
  // rank processes / communicators whose GPU is this rank's GPU (this rank included)
  int ranks_on_device() const { return ranks_on_device_; }
  // auto's topology rule (schedule.h topology_blocks_read), the same on every rank: whether the
  // default runs the read schedule, why, and how this rank's GPU reaches each peer's
  bool topology_allows_read() const { return topo_read_; }
  bool auto_grid() const { return auto_ && topo_read_; }  // auto's large read calls: grid form
  const std::string& topology_reason() const { return topo_why_; }
  int peer_link(int q) const { return peer_link_[q]; }
  int peer_hops(int q) const { return peer_hops_[q]; }
  ncclResult_t async_error();
  // Collective: every rank writes `bytes` into the next rank's scratch (all_peers = 0) or into
  // every peer's scratch at once (1), `iters` times; *gbps = bytes per second per link
  // direction (max over nothing: this rank's own time).  No all-reduce may be in flight.
  ncclResult_t link_probe(int all_peers, size_t bytes, int iters, double* gbps);
  size_t scratch_bytes() const { return scratch_bytes_; }
  // kernel geometry (schedule.h pipeline_geometry): one pipeline per wave, each moving up to
  // slot_bytes (MINI_NCCL_SLICE_SIZE unless the scratch cap shrank it) per message
  int workgroups() const { return geo_.workgroups; }
  int wave_channels() const { return geo_.workgroups * geo_.waves; }
  // the pipelines a call may launch: wave_channels(), capped so that every co-located rank's waves
  // fit the GPU at once (exchange_and_map)
  int run_pipes() const { return run_pipes_ > 0 ? run_pipes_ : wave_channels(); }
  uint64_t wave_slice() const { return geo_.slot_bytes; }

 private:
  void setup_device_resources();
  void release();
  void exchange_and_map();
  void classify_topology(const void* records);  // records: every rank's init record (comm.cpp)
  ncclResult_t wait_for(hipStream_t stream, uint32_t seq);
  enum class Reach { kDevice, kMapped, kStaged };
  Reach reach(const void* p, const void** kernel_ptr, bool* local) const;
  void ensure_stage(size_t bytes, hipStream_t stream);
  // algo: 0 ring, 2 read (psend / precv: every rank's buffers mapped here), 3 one-shot
  void launch(int algo, const void* send, void* recv, size_t chunk_bytes, int dtype, int op, hipStream_t stream,
              uint32_t seq, bool vec, const char* const* psend = nullptr, const char* const* precv = nullptr,
              size_t tail_bytes = 0, uint64_t sig = 0);
  // one rendezvous failure of the read schedule, reported like the kernel's (sticky, peers aborted)
  ncclResult_t rendezvous_failed(const std::exception& e, bool peer_gave_up, int cur_dev);
  struct Window {
    uint64_t id;                    // registration number, the same on every rank
    const char* base;               // this rank's buffer
    size_t bytes;
    const char* peer[kMaxRanks];    // every rank's buffer of this window, mapped here
    bool aligned;                   // every rank's base is dword-aligned
  };
  const Window* find_window(const void* p, size_t bytes) const;
  void wait_previous_call();
  ncclResult_t check_status();
  // a rank that gives up on a call outside its kernel (the read schedule's rendezvous) raises
  // every peer's ABORT word, as a timed-out kernel does, so the peers fail fast instead of
  // running into their own watchdog
  void abort_peers();

  int rank_, nranks_, device_ = 0;
  Config cfg_;
  Geometry geo_;
  int algo_ = 0;                 // 0 ring, 2 read (its calls fall back to the ring when some rank's
                                 // buffers cannot be shared), 3 one-shot (larger calls: as auto)
  bool auto_ = true;             // the default: as algo_ = 2, with the ring's small calls one-shot
  int last_algo_ = -1;
  unsigned long long read_grid_calls_ = 0;  // read calls launched as start / grid / done
  std::vector<Window> windows_;
  uint64_t next_window_ = 1;
  unsigned long long window_calls_ = 0;     // calls launched on registered windows (no rendezvous)
  bool window_fast_ = true;                 // window calls skip the host rendezvous (MINI_NCCL_WINDOW_RENDEZVOUS)
  int run_pipes_ = 0;                       // 0 until exchange_and_map: run_pipes()
  int ranks_on_device_ = 1;
  bool topo_read_ = true;        // auto may run the read schedule (every pair: same GPU or 1 xGMI hop)
  std::string topo_why_ = "read: one rank";
  int peer_link_[kMaxRanks] = {}, peer_hops_[kMaxRanks] = {};
  uint32_t call_seq_ = 0;        // kernel launches of this communicator (the kernel's start word)
  Bootstrap boot_;

  char* scratch_ = nullptr;      // uncached device memory, peers write into it
  size_t scratch_bytes_ = 0;
  uint64_t* mbox_ = nullptr;     // uncached device memory: READY / CREDIT / ABORT words
  size_t mbox_bytes_ = 0;
  uint64_t* pair_seq_ = nullptr; // [2][n][C]: per (peer, channel) tx / rx message counters (device)
  uint32_t* claim_ = nullptr;    // after them: the kernels' first-give-up word (kernels.h)
  uint32_t* go_ = nullptr;       // and the grid form's START-through word (kernels.h CollParams::go)
  uint32_t* h_ctl_ = nullptr;    // host-mapped: [0] status, [1] abort request, [2] last started call
  uint32_t* d_ctl_ = nullptr;    // device view of h_ctl_

  std::vector<char*> peer_scratch_;
  std::vector<uint64_t*> peer_mbox_;
  hipIpcMemHandle_t scratch_h_, mbox_h_;  // exported once (pool blocks, ipcreg.h)
  uint64_t scratch_id_ = 0, mbox_id_ = 0;
  PeerBuffers pbuf_;               // read schedule: per-call rendezvous + peers' buffer mappings
  std::vector<uint64_t> owners_;   // process nonces of the peers in other processes
  bool registered_ = false;        // ipc::comm_opened(owners_) done

  char* stage_ = nullptr;         // device staging copy for pageable host buffers (grown on demand)
  size_t stage_bytes_ = 0;

  hipEvent_t order_ev_ = nullptr;     // recorded after every call: cross-stream ordering, and the
                                      // blocking call's completion (wait_for)
  hipStream_t last_stream_ = nullptr;
  bool have_last_ = false;
  ncclResult_t sticky_ = ncclSuccess;
  bool warned_capture_ = false;
};

// 1-GPU local reduce (mini_nccl_ext.h): no communicator needed.
ncclResult_t local_reduce(void* out, const void* local, const void* incoming, size_t count, int dtype, int op,
                          hipStream_t stream);

}  // namespace mnccl
