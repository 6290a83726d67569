// comm.cpp -- see comm.h.
#include "comm.h"

#include <sched.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <stdexcept>

#include "ipcreg.h"
#include "schedule.h"

namespace mnccl {

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + what + " : " + hipGetErrorString(e));
}

double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

uint64_t host_hash() {
  char h[256] = {0};
  gethostname(h, sizeof h - 1);
  return (uint64_t)std::hash<std::string>{}(std::string(h));
}

// Identifies this process among the ranks (pids repeat across pid namespaces, e.g. containers
// of one pod sharing a hostname): random, drawn once per process.
uint64_t process_nonce() {
  static const uint64_t nonce = [] {
    std::random_device rd;
    uint64_t v = ((uint64_t)rd() << 32) ^ (uint64_t)rd();
    v ^= (uint64_t)getpid() * 0x9E3779B97F4A7C15ull ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    return v ? v : 1;
  }();
  return nonce;
}

// Physical identity of a device (PCI domain / bus / device): device ordinals differ between
// processes that see different device sets, the PCI location does not.
uint64_t pci_id(int dev) {
  int dom = 0, bus = 0, d = 0;
  if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev) != hipSuccess ||
      hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&d, hipDeviceAttributePciDeviceId, dev) != hipSuccess) {
    (void)hipGetLastError();
    return ~0ull - (uint64_t)dev;
  }
  return ((uint64_t)(uint32_t)dom << 32) | ((uint64_t)(bus & 0xffff) << 16) | (uint64_t)(d & 0xffff);
}

// This process's ordinal of the device at PCI location `id`, or -1 if it is not visible here.
int local_device_with_pci(uint64_t id) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (int d = 0; d < ndev; ++d)
    if (pci_id(d) == id) return d;
  return -1;
}

void enable_peer_access(int dev, int peer_dev, bool required) {
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, dev, peer_dev) != hipSuccess) (void)hipGetLastError();
  if (!can) {
    if (required)
      throw std::runtime_error("device " + std::to_string(dev) + " cannot access peer device " + std::to_string(peer_dev));
    return;
  }
  const hipError_t e = hipDeviceEnablePeerAccess(peer_dev, 0);
  if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    if (required) throw std::runtime_error(std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
  }
  (void)hipGetLastError();
}

// Record every rank publishes once at init (the reference's RdmaInfo/DynamicMemInfo,
// RDMATransport.h:25-48, reduced to what one node over HIP IPC needs).
struct PeerInfo {
  uint32_t magic;
  int32_t rank, nranks, pid, device, grid_min_kib;  // grid_min_kib: MINI_NCCL_GRID_MIN / 1024
  uint64_t host, nonce, pci;  // nonce: same process <=> same nonce; pci: the physical GPU
  uint64_t slice, scratch_bytes, mbox_bytes, scratch_cap;
  int32_t channels, slots, threads, abi;
  int32_t window, signal_batch, algo, pad0;
  hipIpcMemHandle_t scratch_h, mbox_h;
  uint64_t scratch_ptr, mbox_ptr;  // raw addresses (same-process ranks) / the allocations' bases
  uint64_t scratch_id, mbox_id;    // HIP allocation ids (the import registry's keys)
  int64_t retired_mb;              // MINI_NCCL_RETIRED_MB as configured (-1: the default)
  int32_t window_rendezvous, cus;  // MINI_NCCL_WINDOW_RENDEZVOUS as configured; the GPU's CUs
};
constexpr uint32_t kInfoMagic = 0x4d4e4934u;  // 'MNI4' (4.0's record: a 3.x rank fails the check)

}  // namespace

Comm::Comm(int nranks, int rank, const std::string& ip) : rank_(rank), nranks_(nranks) {
  cfg_ = Config::from_env();
  // auto: the read schedule (same bits; no scratch; each call falls back to the ring when some
  // rank's buffers cannot be shared)
  set_algo(cfg_.algo);
  if (nranks > kMaxRanks) throw std::invalid_argument("nRanks > 16 is not supported on one node");
  geo_ = pipeline_geometry(nranks, cfg_.channels, cfg_.threads, cfg_.window_size, cfg_.signal_batch, cfg_.slots,
                           cfg_.slice_size, cfg_.scratch_cap);
  hip_check(hipGetDevice(&device_), "hipGetDevice");
  if (cfg_.debug && rank == 0)
    fprintf(stderr, "[Config] Loaded: %s; geometry: %d workgroups x %d waves, slot %llu B, scratch %llu B\n",
            cfg_.describe().c_str(), geo_.workgroups, geo_.waves, (unsigned long long)geo_.slot_bytes,
            (unsigned long long)geo_.scratch_bytes);
  try {
    setup_device_resources();
    boot_.connect(rank, nranks, ip, cfg_.port, cfg_.bootstrap_timeout_ms / 1000.0);
    exchange_and_map();
  } catch (...) {
    release();
    throw;
  }
}

void Comm::setup_device_resources() {
  // one channel per wave: `channels` workgroups x threads/64 waves; the reference's slice
  // (bytes per channel step) is split across the workgroup's waves
  const int C = wave_channels();
  scratch_bytes_ = geo_.scratch_bytes;  // (n-1) peer regions, <= MINI_NCCL_SCRATCH_MB
  mbox_bytes_ = (size_t)mbox_words(nranks_, C) * sizeof(uint64_t);
  hip_check(hipHostMalloc((void**)&h_ctl_, 4096, hipHostMallocMapped | hipHostMallocCoherent), "alloc ctl");
  memset(h_ctl_, 0, 4096);
  hip_check(hipHostGetDevicePointer((void**)&d_ctl_, h_ctl_, 0), "ctl device pointer");
  hip_check(hipEventCreateWithFlags(&order_ev_, hipEventDisableTiming), "event");
  if (nranks_ > 1) {
    // from the process's pool (ipcreg.h): a communicator created after another one re-uses its
    // blocks and the peers' imports of them instead of exporting a re-used address
    scratch_ = (char*)ipc::pool_acquire(scratch_bytes_, hipDeviceMallocUncached, &scratch_h_, &scratch_id_);
    mbox_ = (uint64_t*)ipc::pool_acquire(mbox_bytes_, hipDeviceMallocUncached, &mbox_h_, &mbox_id_);
    const size_t seq_bytes = (size_t)2 * nranks_ * C * sizeof(uint64_t);  // C = wave channels
    // + the kernels' claim word (kernels.h CollParams::claim) in its own 256 bytes after them
    hip_check(hipMalloc((void**)&pair_seq_, seq_bytes + 256), "alloc pair_seq");
    claim_ = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(pair_seq_) + seq_bytes);
    go_ = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(pair_seq_) + seq_bytes + 128);
    // zeroed on a private stream: a device-wide sync (or the legacy null stream) would also wait
    // for other communicators' persistent kernels in this process, which may be waiting for us
    hipStream_t st = nullptr;
    hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "init stream");
    hipError_t e = hipMemsetAsync(scratch_, 0, scratch_bytes_, st);
    if (e == hipSuccess) e = hipMemsetAsync(mbox_, 0, mbox_bytes_, st);
    if (e == hipSuccess) e = hipMemsetAsync(pair_seq_, 0, seq_bytes + 256, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    hipStreamDestroy(st);
    hip_check(e, "zero scratch / mailbox / counters");
  }
}

void Comm::exchange_and_map() {
  peer_scratch_.assign((size_t)nranks_, nullptr);
  peer_mbox_.assign((size_t)nranks_, nullptr);
  if (nranks_ == 1) return;
  PeerInfo me;
  memset(&me, 0, sizeof me);
  me.magic = kInfoMagic;
  me.rank = rank_;
  me.nranks = nranks_;
  me.pid = (int32_t)getpid();
  me.device = device_;
  me.host = host_hash();
  me.nonce = process_nonce();
  me.pci = pci_id(device_);
  me.slice = cfg_.slice_size;
  me.scratch_bytes = scratch_bytes_;
  me.mbox_bytes = mbox_bytes_;
  me.scratch_cap = cfg_.scratch_cap;
  me.channels = cfg_.channels;
  me.slots = cfg_.slots;
  me.threads = cfg_.threads;
  me.abi = 6;  // 6.0: no load form, the retired-import budget in the record
  me.window = cfg_.window_size;
  me.signal_batch = cfg_.signal_batch;
  me.algo = cfg_.algo;
  me.grid_min_kib = (int32_t)(cfg_.grid_min >> 10);
  me.scratch_h = scratch_h_;
  me.mbox_h = mbox_h_;
  me.scratch_ptr = (uint64_t)(uintptr_t)scratch_;
  me.mbox_ptr = (uint64_t)(uintptr_t)mbox_;
  me.scratch_id = scratch_id_;
  me.mbox_id = mbox_id_;
  me.retired_mb = cfg_.retired_mb;
  me.window_rendezvous = cfg_.window_rendezvous;
  if (hipDeviceGetAttribute(&me.cus, hipDeviceAttributeMultiprocessorCount, device_) != hipSuccess) {
    (void)hipGetLastError();
    me.cus = 256;
  }

  std::vector<PeerInfo> all((size_t)nranks_);
  boot_.allgather(&me, all.data(), sizeof me);
  for (int q = 0; q < nranks_; ++q) {
    const PeerInfo& p = all[(size_t)q];
    if (p.magic != kInfoMagic || p.rank != q || p.nranks != nranks_)
      throw std::runtime_error("bootstrap: inconsistent rank records");
    if (p.host != me.host) throw std::runtime_error("rank " + std::to_string(q) + " is on another host: only one node is supported");
    // every knob that shapes the kernels' geometry, message protocol or init sequence must agree
    if (p.slice != me.slice || p.channels != me.channels || p.slots != me.slots || p.threads != me.threads ||
        p.window != me.window || p.signal_batch != me.signal_batch || p.scratch_cap != me.scratch_cap ||
        p.algo != me.algo || p.abi != me.abi || p.grid_min_kib != me.grid_min_kib ||
        p.retired_mb != me.retired_mb || p.window_rendezvous != me.window_rendezvous)
      throw std::invalid_argument(
          "MINI_NCCL_SLICE_SIZE / WINDOW_SIZE / SIGNAL_BATCH / SLOTS / CHANNELS / THREADS / SCRATCH_MB / ALGO / "
          "GRID_MIN / RETIRED_MB / WINDOW_RENDEZVOUS differ between ranks (or their library versions differ)");
  }
  ranks_on_device_ = 0;
  for (int q = 0; q < nranks_; ++q)
    if (all[(size_t)q].pci == me.pci) ++ranks_on_device_;
  // Residency: pipeline w of every rank waits for pipeline w of its peers, so the waves a call
  // launches on the most crowded GPU must all be resident at once -- CUs x 4 SIMDs x
  // kMinWavesPerSimd of them, shared by the ranks on that GPU.  A call launches at most run_pipes_
  // pipelines (the mailbox / scratch / counter layout keeps all P; the others sit the call out, on
  // every rank alike: the records are the same everywhere).  8 co-located ranks with
  // MINI_NCCL_CHANNELS=512 (8 x 512 waves for 2048 slots) timed out without it.
  {
    int cus = 1 << 30, most = 1;
    for (int q = 0; q < nranks_; ++q) {
      cus = std::min(cus, std::max(1, (int)all[(size_t)q].cus));
      int same = 0;
      for (int p = 0; p < nranks_; ++p) same += all[(size_t)p].pci == all[(size_t)q].pci;
      most = std::max(most, same);
    }
    run_pipes_ = resident_pipes(wave_channels(), geo_.waves, cus, most, kMinWavesPerSimd);
    if (run_pipes_ < wave_channels() && rank_ == 0)
      fprintf(stderr, "[Mini-NCCL] %d rank(s) share a GPU of %d CUs: calls launch at most %d of the communicator's %d "
              "pipelines, so every rank's waves stay resident together\n", most, cus, run_pipes_, wave_channels());
  }
  // Window calls without a host rendezvous: by default only when no two ranks share a GPU.  Ranks
  // sharing one GPU meet faster on the host than on the device -- 8 co-located ranks, 4 KiB blocking
  // calls: 88 us per window call launched at once vs 68-70 us negotiated, 4 ranks 25.7 vs 24.8-25.2
  // (profiles/r6_small_calls_windows.txt) -- since their kernels, launched out of step, spin for
  // each other while 8 processes' dispatches share one command processor.  The same answer on
  // every rank: every rank sees every PCI location.
  bool shared_gpu = false;
  for (int q = 0; q < nranks_; ++q)
    for (int p = q + 1; p < nranks_; ++p) shared_gpu = shared_gpu || all[(size_t)q].pci == all[(size_t)p].pci;
  window_fast_ = cfg_.window_rendezvous == 0 || (cfg_.window_rendezvous < 0 && !shared_gpu);
  // Rank PROCESSES sharing this GPU: a persistent kernel waits for its peers' kernels, so all of
  // them must be resident at once; the GPU's scheduler maps a bounded number of processes and
  // hardware queues together, beyond which it time-slices and every hand-off waits for a turn
  // (measured on MI355X: 8 processes x 2 queues each run at full rate, 8 x 4 -- HIP's default
  // GPU_MAX_HW_QUEUES -- are ~200x slower, and a 9th GPU process stalls them).
  {
    std::vector<uint64_t> procs;
    for (int q = 0; q < nranks_; ++q)
      if (all[(size_t)q].pci == me.pci && std::find(procs.begin(), procs.end(), all[(size_t)q].nonce) == procs.end())
        procs.push_back(all[(size_t)q].nonce);
    const char* hq = std::getenv("GPU_MAX_HW_QUEUES");
    const int queues = hq && *hq ? std::max(1, atoi(hq)) : 4;
    bool first_here = true;  // warn once per GPU: from its lowest rank
    for (int q = 0; q < rank_; ++q)
      if (all[(size_t)q].pci == me.pci) first_here = false;
    // 8 x 4 queues time-sliced every hand-off (profiles/r2_coloc8_*); 2 x 4 did as soon as each
    // process made one more stream (profiles/r5_bench_size_order.txt), 2 per process never did
    if (procs.size() > 1 && queues > 2 && first_here)
      fprintf(stderr,
              "[Mini-NCCL] warning: %zu rank processes share GPU %d with up to %d hardware queues each; the "
              "all-reduce needs every rank's kernel resident at once -- with more than 2 queues per process "
              "(GPU_MAX_HW_QUEUES) the GPU may time-slice the processes' queues once they hold more streams, "
              "and every call then stalls; set GPU_MAX_HW_QUEUES=2 (and keep other processes off this GPU)\n",
              procs.size(), device_, queues);
  }
  // the bytes of freed same-GPU peer allocations this process may keep mapped (ipcreg.h
  // close_import): MINI_NCCL_RETIRED_MB, by default 1/8 of this GPU's memory shared by the ranks on
  // it (36 GB on MI355X between them: each co-located process pins memory of the same GPU)
  if (ranks_on_device_ > 1) {
    uint64_t budget = (uint64_t)cfg_.retired_mb << 20;
    if (cfg_.retired_mb < 0) {
      size_t fr = 0, total = 0;
      if (hipMemGetInfo(&fr, &total) != hipSuccess) {
        (void)hipGetLastError();
        total = (size_t)288 << 30;
      }
      budget = (uint64_t)total / 8 / (uint64_t)ranks_on_device_;
    }
    ipc::set_retired_budget(budget);
  }
  classify_topology(all.data());
  for (int q = 0; q < nranks_; ++q) {
    if (q == rank_) {
      peer_scratch_[(size_t)q] = scratch_;
      peer_mbox_[(size_t)q] = mbox_;
      continue;
    }
    const PeerInfo& p = all[(size_t)q];
    if (p.nonce == me.nonce) {
      // same process (threads of one program, one rank each): plain pointers; another device's
      // memory needs peer access from this one
      if (p.device != device_) enable_peer_access(device_, p.device, true);
      peer_scratch_[(size_t)q] = (char*)(uintptr_t)p.scratch_ptr;
      peer_mbox_[(size_t)q] = (uint64_t*)(uintptr_t)p.mbox_ptr;
      continue;
    }
    // another process: its GPU by PCI location (ordinals differ between processes that see
    // different device sets); if it is visible here, enable peer access to it explicitly,
    // otherwise the IPC mapping's lazy peer access does it
    const int pd = local_device_with_pci(p.pci);
    if (pd >= 0 && pd != device_) enable_peer_access(device_, pd, false);
    // through the process's import registry: a peer block this process imported for an earlier
    // communicator is still mapped (imports of pool blocks are never closed, ipcreg.h)
    hipError_t e = hipSuccess;
    char* ps = ipc::open_block(p.nonce, p.scratch_ptr, p.scratch_id, p.scratch_h, &e);
    hip_check(ps ? hipSuccess : e, "ipc open scratch");
    char* pm = ipc::open_block(p.nonce, p.mbox_ptr, p.mbox_id, p.mbox_h, &e);
    hip_check(pm ? hipSuccess : e, "ipc open mailbox");
    peer_scratch_[(size_t)q] = ps;
    peer_mbox_[(size_t)q] = (uint64_t*)pm;
  }
  // every rank has mapped every peer and its own memory is zeroed before anyone writes
  boot_.barrier();
  // the read schedule's per-call board (collective; unavailable on every rank alike if shared
  // memory is)
  std::vector<uint64_t> nonces((size_t)nranks_);
  for (int q = 0; q < nranks_; ++q) nonces[(size_t)q] = all[(size_t)q].nonce;
  pbuf_.init(boot_, rank_, nranks_, nonces, cfg_.port);
  // the peers in other processes, for the import lifecycle (ipcreg.h comm_opened / comm_closed)
  for (int q = 0; q < nranks_; ++q)
    if (all[(size_t)q].nonce != me.nonce &&
        std::find(owners_.begin(), owners_.end(), all[(size_t)q].nonce) == owners_.end())
      owners_.push_back(all[(size_t)q].nonce);
  ipc::comm_opened(owners_);
  registered_ = true;
}

// How this rank's GPU reaches every peer's (the runtime's link type and hop count), gathered from
// every rank; auto runs the read schedule only if schedule.h topology_blocks_read allows it for
// every pair -- the same matrix, so the same decision, on every rank.  Collective (one allgather).
void Comm::classify_topology(const void* records) {
  const PeerInfo* all = static_cast<const PeerInfo*>(records);
  const int n = nranks_;
  struct Row {
    int32_t link[kMaxRanks], hops[kMaxRanks];
  } mine;
  for (int p = 0; p < kMaxRanks; ++p) {
    mine.link[p] = kPeerSameGpu;
    mine.hops[p] = 0;
  }
  for (int p = 0; p < n; ++p) {
    if (p == rank_ || all[p].pci == all[rank_].pci) continue;
    const int pd = local_device_with_pci(all[p].pci);
    uint32_t lt = 0, hc = 0;
    if (pd < 0 || hipExtGetLinkTypeAndHopCount(device_, pd, &lt, &hc) != hipSuccess) {
      (void)hipGetLastError();
      mine.link[p] = kPeerUnknown;
      mine.hops[p] = -1;
    } else {
      mine.link[p] = (int32_t)lt;
      mine.hops[p] = (int32_t)hc;
    }
  }
  std::vector<Row> rows((size_t)n);
  boot_.allgather(&mine, rows.data(), sizeof mine);
  std::vector<int> link((size_t)n * n), hops((size_t)n * n);
  for (int q = 0; q < n; ++q)
    for (int p = 0; p < n; ++p) {
      link[(size_t)q * n + p] = rows[(size_t)q].link[p];
      hops[(size_t)q * n + p] = rows[(size_t)q].hops[p];
    }
  for (int p = 0; p < kMaxRanks; ++p) {
    peer_link_[p] = p < n ? mine.link[p] : kPeerSameGpu;
    peer_hops_[p] = p < n ? mine.hops[p] : 0;
  }
  const int bad = topology_blocks_read(n, link.data(), hops.data());
  topo_read_ = bad == 0;
  char why[160];
  if (bad == 0) {
    snprintf(why, sizeof why, "read (grid form for large calls): every pair of ranks shares a GPU or is one xGMI hop "
             "apart");
  } else {
    const int q = (bad - 1) / n, p = (bad - 1) % n, l = link[(size_t)bad - 1];
    const char* name = l == kPeerUnknown ? "an unknown link (its GPU is not visible to that process)"
                       : l == kLinkPcie  ? "PCIe"
                       : l == kLinkXgmi  ? "xGMI"
                                         : "a non-xGMI link";
    snprintf(why, sizeof why, "ring: rank %d reaches rank %d over %s, %d hop(s)", q, p, name, hops[(size_t)bad - 1]);
    if (rank_ == 0 && auto_)
      fprintf(stderr, "[Mini-NCCL] auto: the read schedule is off for this communicator (%s); calls run the ring "
              "(MINI_NCCL_ALGO=read forces it)\n", why);
  }
  topo_why_ = why;
}

Comm::~Comm() {
  hipSetDevice(device_);
  // the last call may still run (stream-ordered mode): its kernel writes into the peers' scratch
  // and mailboxes, which they free after the barrier below -- wait for it first
  if (have_last_ && order_ev_) hipEventSynchronize(order_ev_);
  if (nranks_ > 1 && !peer_scratch_.empty()) {
    try {
      // nobody still writes into my memory: my scratch / mailbox may go to the next
      // communicator of this process (the peers' imports of them stay open, ipcreg.h)
      if (sticky_ == ncclSuccess) boot_.barrier();
    } catch (...) {
    }
  }
  // this communicator's kernels are done (waited above): its imports of peers no other live
  // communicator of this process talks to are closed, and the exports too if it was the last one.
  // Also after a failure (skipping this pinned every export of the process for good):
  // a peer whose kernel still runs reads and writes this process's buffers through ITS imports,
  // which hold their own reference on the memory -- closing this process's export descriptors or
  // its own (idle) imports cannot pull memory from under it.  What a failed peer may still write
  // into -- this communicator's scratch and mailbox -- stays out of the pool (release()).
  if (registered_) ipc::comm_closed(owners_);
  registered_ = false;
  release();
}

void Comm::release() {
  boot_.close_all();
  // a communicator that failed (sticky error) may still have peers writing into its blocks:
  // they are not handed to another communicator (the pool keeps them busy)
  if (sticky_ == ncclSuccess) {
    ipc::pool_release(scratch_);
    ipc::pool_release(mbox_);
  }
  if (pair_seq_) hipFree(pair_seq_);
  if (h_ctl_) hipHostFree(h_ctl_);
  if (stage_) hipFree(stage_);
  stage_ = nullptr;
  stage_bytes_ = 0;
  if (order_ev_) hipEventDestroy(order_ev_);
  order_ev_ = nullptr;
  have_last_ = false;
  scratch_ = nullptr;
  mbox_ = nullptr;
  pair_seq_ = nullptr;
  claim_ = nullptr;
  go_ = nullptr;
  h_ctl_ = nullptr;
  (void)hipGetLastError();
}

ncclResult_t Comm::check_status() {
  const uint32_t st = __atomic_load_n(&h_ctl_[0], __ATOMIC_ACQUIRE);
  if (st == 0) return ncclSuccess;
  if (sticky_ == ncclSuccess) {
    // a registered-window call whose ranks disagreed (kernels.hip starts_agree), seen here or
    // relayed by the peer that saw it: the caller's error, ncclInvalidUsage
    const uint64_t a0 = (st & kStatusRemoteAbort) ? reinterpret_cast<const volatile uint64_t*>(h_ctl_ + 4)[3] : 0;
    const bool mismatch = (st & kStatusMismatch) || ((uint32_t)(a0 >> 32) & kStatusMismatch);
    sticky_ = mismatch ? ncclInvalidUsage
              : (st & kStatusRemoteAbort) && !(st & kStatusTimeout) ? ncclRemoteError : ncclInternalError;
    fprintf(stderr, "[Mini-NCCL] rank %d: all-reduce %s (status 0x%x); communicator is no longer usable\n", rank_,
            mismatch ? "on registered windows: the ranks passed different windows / offsets / count / datatype / op"
            : (st & kStatusTimeout) ? "timed out (watchdog)" : (st & kStatusHostAbort) ? "aborted by host" : "aborted by a peer",
            st);
    if ((st & kStatusRemoteAbort) && !(st & (kStatusTimeout | kStatusHostAbort))) {
      // the ABORT word the first aborting peer wrote (kernels.hip abort_word; the host's
      // abort_peers writes rank + 1 only)
      const uint64_t a = reinterpret_cast<const volatile uint64_t*>(h_ctl_ + 4)[3];
      const uint32_t why = (uint32_t)(a >> 32);
      if (a)
        fprintf(stderr, "[Mini-NCCL] rank %d: first abort came from rank %d (%s)\n", rank_, (int)(a & 0xffffffffu) - 1,
                (why & kStatusTimeout) ? "its watchdog timed out" : (why & kStatusHostAbort) ? "its host aborted"
                : (why & kStatusMismatch) ? "its peers' call signatures differed from its own"
                : (why & kStatusRemoteAbort) ? "relaying an abort" : "it gave up outside its kernel");
    }
    if (st & kStatusTimeout) {
      // which mailbox word the first timed-out wait was stuck on (kernels.hip record_timeout)
      const volatile uint64_t* diag = reinterpret_cast<const volatile uint64_t*>(h_ctl_ + 4);
      const uint64_t word = diag[0], line = word / kFlagStride;
      const int P = wave_channels(), n = nranks_;
      const bool ready = line < (uint64_t)n * P;
      const uint64_t idx = ready ? line : line - (uint64_t)n * P;
      fprintf(stderr, "[Mini-NCCL] rank %d: stuck on %s word of peer %llu, pipeline %llu: waiting for >= %llu, saw %llu\n",
              rank_, ready ? "READY" : "CREDIT", (unsigned long long)(idx / P), (unsigned long long)(idx % P),
              (unsigned long long)diag[1], (unsigned long long)diag[2]);
    }
  }
  return sticky_;
}

ncclResult_t Comm::async_error() {
  if (sticky_ != ncclSuccess) return sticky_;
  if (h_ctl_) return check_status();
  return ncclSuccess;
}

// Host side of the reference's watchdog (mini_nccl.cu:200-214): wait for the stream; once this
// call's kernel has started (it writes its sequence number into the start word, so work the
// caller queued before it never counts), after the kernel's own timeout plus a grace period,
// raise the abort word the kernel polls.  Work ahead of the kernel on the stream is the caller's
// and is waited for without a deadline (the abort word could not reach it anyway).
ncclResult_t Comm::wait_for(hipStream_t stream, uint32_t seq) {
  // order_ev_ was recorded on `stream` right after this call's work (allreduce): it is the
  // completion event too (one event record per call, ~1.8 us each on MI355X)
  (void)stream;
  double t0 = -1.0;
  const double limit = cfg_.timeout_ms / 1000.0 + 2.0;
  bool aborted = false;
  for (int spins = 0;; ++spins) {
    hipError_t q = hipEventQuery(order_ev_);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) hip_check(q, "stream query");
    if (t0 < 0.0) {
      const uint32_t started = __atomic_load_n(&h_ctl_[2], __ATOMIC_ACQUIRE);
      if (seq != 0 && (int32_t)(started - seq) < 0) {
        if (spins < 2000) sched_yield();
        else usleep(100);
        continue;
      }
      t0 = now_s();
    }
    const double el = now_s() - t0;
    if (!aborted && el > limit) {
      fprintf(stderr, "[Watchdog] TIMEOUT DETECTED on rank %d! Aborting GPU kernels...\n", rank_);
      __atomic_store_n(&h_ctl_[1], 1u, __ATOMIC_RELEASE);
      aborted = true;
    }
    if (aborted && el > limit + 10.0) {
      sticky_ = ncclInternalError;
      return sticky_;
    }
    if (spins < 2000) sched_yield();
    else usleep(el < 0.01 ? 10 : 100);
  }
  return check_status();
}

// Which memory the kernel can address for a user buffer (see allreduce); *local: plain device
// memory of this rank's GPU (what the read schedule can share with the peers).
Comm::Reach Comm::reach(const void* p, const void** kernel_ptr, bool* local) const {
  hipPointerAttribute_t a;
  memset(&a, 0, sizeof a);
  *local = false;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return Reach::kStaged;  // not known to HIP: pageable host memory
  }
  if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.isManaged) {
    *local = a.type == hipMemoryTypeDevice && !a.isManaged && a.device == device_;
    return Reach::kDevice;
  }
  if (a.type == hipMemoryTypeHost && a.devicePointer) {
    // device address of p itself (devicePointer / hostPointer may name the allocation base)
    const char* hp = (const char*)(a.hostPointer ? a.hostPointer : p);
    *kernel_ptr = (const char*)a.devicePointer + ((const char*)p - hp);
    return Reach::kMapped;
  }
  return Reach::kStaged;
}

// Stream-ordered on the call's stream (which already waits for this communicator's previous
// call, see allreduce): no device-wide sync, which would also wait for other communicators'
// persistent kernels in this process.
void Comm::ensure_stage(size_t bytes, hipStream_t stream) {
  if (stage_bytes_ >= bytes) return;
  if (stage_) {
    hip_check(hipFreeAsync(stage_, stream), "free stage");
    stage_ = nullptr;
    stage_bytes_ = 0;
  }
  const size_t want = (bytes + ((size_t)1 << 20) - 1) & ~(((size_t)1 << 20) - 1);
  hip_check(hipMallocAsync((void**)&stage_, want, stream), "alloc stage");
  stage_bytes_ = want;
}

// Host wait for this communicator's last call (its kernel writes into the peers' memory)
void Comm::wait_previous_call() {
  if (have_last_) hip_check(hipEventSynchronize(order_ev_), "wait for the previous call");
}

void Comm::launch(int algo, const void* send, void* recv, size_t chunk_bytes, int dtype, int op, hipStream_t stream,
                  uint32_t seq, bool vec, const char* const* psend, const char* const* precv,
                  size_t tail_bytes, uint64_t sig) {
  const int n = nranks_;
  CollParams p;
  memset(&p, 0, sizeof p);
  p.send = (const char*)send;
  p.recv = (char*)recv;
  p.chunk_bytes = chunk_bytes;
  // C: the pipelines this call may launch (run_pipes_, <= the layout's wave_channels())
  const int C = run_pipes();
  p.slot_bytes = wave_slice();
  p.slice_bytes = algo == 2   ? read_slice(chunk_bytes, C, cfg_.slice_size, kMinSlice, kReadDepth)
                  : algo == 3 ? oneshot_slice(chunk_bytes, n, C, wave_slice())
                              : effective_slice(chunk_bytes, C, wave_slice(), kMinSlice, 1);
  p.nslices = (chunk_bytes + p.slice_bytes - 1) / p.slice_bytes;
  // every kernel runs one pipeline per slice up to C (schedule.h call_pipelines); the one-shot one
  // per slice of every chunk
  const int A = call_pipelines(algo == 3 ? p.nslices * (uint64_t)n : p.nslices, C, geo_.waves);
  p.iters = (uint32_t)((p.nslices + (uint64_t)A - 1) / (uint64_t)A);
  p.pipes = wave_channels();
  p.n = n;
  p.rank = rank_;
  p.nslots = cfg_.slots;
  p.scratch = scratch_;
  p.mbox = mbox_;
  p.tx_seq = pair_seq_;
  p.rx_seq = pair_seq_ + (size_t)n * wave_channels();
  for (int q = 0; q < n; ++q) {
    p.peer_scratch[q] = peer_scratch_[(size_t)q];
    p.peer_mbox[q] = peer_mbox_[(size_t)q];
    if (psend) p.peer_send[q] = psend[q];
    if (precv) p.peer_recv[q] = precv[q];
  }
  p.status = d_ctl_;
  p.host_abort = d_ctl_ + 1;
  p.started = d_ctl_ + 2;
  p.call_seq = seq;
  p.timeout_ticks = (uint64_t)(cfg_.timeout_ms * 1e5);  // s_memrealtime runs at 100 MHz
  p.sys_fence = cfg_.sys_fence;
  p.tail_bytes = tail_bytes;
  p.claim = claim_;
  p.go = go_;
  p.sig = algo == 2 ? sig : 0;
  const int nt = cfg_.threads, wg = A / geo_.waves;
  // mncclAlgoReadGrid: the push form's large calls as start / grid fold / done (the same on every
  // rank: the schedule, the push form, vec and the size are rank-uniform)
  // (and auto's: schedule.h read_grid_form)
  const bool grid = algo == 2 && read_grid_form(algo_ == 4, auto_, vec, chunk_bytes, n,
                                                 cfg_.grid_min);
  hipError_t e = grid        ? launch_read_grid(dtype, op, p, stream, cfg_.grid_vectors)
                 : algo == 2 ? launch_read(dtype, op, vec, wg, nt, p, stream)
                 : algo == 3 ? launch_oneshot(dtype, op, vec, wg, nt, p, stream)
                             : launch_ring(dtype, op, vec, wg, nt, p, stream);
  hip_check(e, "kernel launch");
  last_algo_ = algo;
  if (grid) ++read_grid_calls_;
}

ncclResult_t Comm::allreduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t stream) {
  if (sticky_ != ncclSuccess) return sticky_;
  if (check_status() != ncclSuccess) return sticky_;
  const int esz = dtype_size(dtype);
  const size_t bytes = count * (size_t)esz;
  int cur_dev = -1;
  hip_check(hipGetDevice(&cur_dev), "hipGetDevice");
  if (cur_dev != device_) hip_check(hipSetDevice(device_), "hipSetDevice");

  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) != hipSuccess) {
    (void)hipGetLastError();
    cap = hipStreamCaptureStatusNone;
  }
  if (cap == hipStreamCaptureStatusActive && !warned_capture_) {
    // the reference warns here too (api.cpp:153-166); this build needs no host polling,
    // so a captured all-reduce replays correctly (sequence state lives on the device)
    if (cfg_.debug) fprintf(stderr, "[Mini-NCCL] HIP graph capture detected: host-side wait skipped\n");
    warned_capture_ = true;
  }

  // One communicator, one sequence of calls: the persistent kernels read and advance the
  // per-pipeline FIFO counters, and the staging buffer is shared, so a call on another stream
  // waits for the previous call (NCCL's rule: calls on a communicator are ordered).  Graph
  // capture keeps its own order (the captured stream) and is left alone.
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (!capturing && have_last_ && stream != last_stream_)
    hip_check(hipStreamWaitEvent(stream, order_ev_, 0), "order after previous call");

  const int n = nranks_;
  uint32_t seq = 0;  // this call's kernel (0: the call launches none)
  const size_t chunk = n > 0 ? count / (size_t)n : 0;  // mini_nccl.cu:69
  const size_t chunk_bytes = chunk * (size_t)esz;
  if (n == 1 || chunk == 0) {
    // nRanks == 1 returns after the copy (mini_nccl.cu:66); chunk == 0 moves no slice
    if (send != recv) hip_check(hipMemcpyAsync(recv, send, bytes, hipMemcpyDefault, stream), "copy");
  } else {
    // Where the kernel reads and writes: device memory as is; pinned / registered host
    // memory through its device mapping (the kernel then streams it over PCIe itself,
    // pipelined slice by slice -- what the reference's kernels did with its
    // cudaHostAlloc'd perf_test buffers, perf_test.cpp:78-79); pageable host memory
    // through a device staging copy.  Every rank launches the same kernel either way.
    const void* ksend = send;
    void* krecv = recv;
    // buffers the read schedule already shares (live exports of this process, checked by reap())
    // need no pointer query: device memory of this GPU
    bool local_s = false, local_r = false;
    // forced one-shot wherever a call fits it; otherwise the read schedule where every rank can
    // share its buffers, and for the other calls the ring -- or, under auto, the one-shot for
    // small ones (its one hand-off against the ring's 2(n-1); on the proxy the read schedule
    // still wins at 8 ranks, profiles/r4_small_calls.txt, so auto keeps read first).  A pure
    // function of the call's size and the rank-uniform config up to the read rendezvous, which
    // all ranks decide alike.
    const bool oneshot = algo_ == 3 && oneshot_fits(chunk_bytes, n, run_pipes(), wave_slice(), true);
    const bool small = auto_ && oneshot_fits(chunk_bytes, n, run_pipes(), wave_slice(), false);
    // (auto, and a forced one-shot's larger calls, only where the topology allows the read
    // schedule: classify_topology; MINI_NCCL_ALGO=read forces it anywhere)
    const bool read_sched = !oneshot &&
                            (((algo_ == 2 || algo_ == 4) && (!auto_ || topo_read_)) || (algo_ == 3 && topo_read_)) &&
                            pbuf_.available();
    // registered windows: the read schedule with no host rendezvous (no record to wait for, no
    // pointer query) -- every rank promised the same windows and offsets, the kernel checks it
    const Window* win_s = read_sched && window_fast_ && !windows_.empty() ? find_window(send, bytes) : nullptr;
    const Window* win_r = win_s ? find_window(recv, bytes) : nullptr;
    if (win_s && win_r) {
      const uint64_t os = (uint64_t)((const char*)send - win_s->base), orv = (uint64_t)((char*)recv - win_r->base);
      const char* psend[kMaxRanks] = {};
      const char* precv[kMaxRanks] = {};
      for (int q = 0; q < n; ++q) {
        psend[q] = win_s->peer[q] + os;
        precv[q] = win_r->peer[q] + orv;
      }
      // the call's signature: windows, offsets, count, datatype, op and the schedule choice that
      // picks the kernel form (auto / mncclCommSetAlgo: a grid-form rank paired with a persistent
      // one could see its DONE met while the peer's other pipelines never start -- ADVICE r5)
      // (FNV-1a over the words)
      uint64_t sig = 1469598103934665603ull;
      const uint64_t mode = auto_ ? ~0ull : (uint64_t)algo_;
      for (uint64_t v : {win_s->id, os, win_r->id, orv, (uint64_t)count, (uint64_t)dtype, (uint64_t)op, mode})
        for (int b = 0; b < 8; ++b) sig = (sig ^ ((v >> (8 * b)) & 0xff)) * 1099511628211ull;
      sig |= 1;  // never 0 (0 = a negotiated call)
      try {
        pbuf_.publish_fast(count, dtype, op, sig, cfg_.timeout_ms / 1000.0 + 2.0);
      } catch (const PeerGaveUp& e) {
        return rendezvous_failed(e, true, cur_dev);
      } catch (const std::exception& e) {
        return rendezvous_failed(e, false, cur_dev);
      }
      const bool vec_w = win_s->aligned && win_r->aligned && os % 4 == 0 && orv % 4 == 0 && chunk_bytes % 4 == 0;
      const size_t body = chunk_bytes * (size_t)n;
      const size_t tail = send != recv && bytes > body ? bytes - body : 0;
      seq = ++call_seq_;
      if (seq == 0) seq = ++call_seq_;
      launch(2, send, recv, chunk_bytes, dtype, op, stream, seq, vec_w, psend, precv, tail, sig);
      ++window_calls_;
      if (!capturing) {
        hip_check(hipEventRecord(order_ev_, stream), "order event");
        last_stream_ = stream;
        have_last_ = true;
      }
      if (cur_dev != device_) hipSetDevice(cur_dev);
      if (cfg_.blocking && !capturing) return wait_for(stream, seq);
      return ncclSuccess;
    }
    if (read_sched) pbuf_.reap(send, recv);
    const Reach rs = read_sched && pbuf_.known(send) ? (local_s = true, Reach::kDevice) : reach(send, &ksend, &local_s);
    const Reach rr = read_sched && pbuf_.known(recv) ? (local_r = true, Reach::kDevice)
                                                     : reach(recv, (const void**)&krecv, &local_r);
    if (rs == Reach::kStaged || rr == Reach::kStaged) {
      if (cap != hipStreamCaptureStatusNone) {
        fprintf(stderr, "[Mini-NCCL] pageable host buffers cannot be captured into a HIP graph\n");
        if (cur_dev != device_) hipSetDevice(cur_dev);
        return ncclInvalidUsage;
      }
      ensure_stage(bytes, stream);
      if (rs == Reach::kStaged) {
        hip_check(hipMemcpyAsync(stage_, send, bytes, hipMemcpyDefault, stream), "stage in");
        ksend = stage_;
      }
      if (rr == Reach::kStaged) krecv = stage_;  // also in place when send is staged too
    }
    // elements past n*chunk keep this rank's own input (the reference copies the whole
    // buffer and never touches the tail, api.cpp:173-175 + mini_nccl.cu:69); the kernels
    // write every other element of recv and copy the tail themselves (kernels.hip copy_tail)
    const size_t body = chunk_bytes * (size_t)n;
    const size_t tail = ksend != krecv && bytes > body ? bytes - body : 0;
    // 16-byte vector path whenever every message's local base is dword-aligned (vectors may
    // straddle 16-byte boundaries on the local side; each message's last len % 16 bytes go
    // element by element); element-wise path otherwise (2-byte types with odd chunks)
    bool vec = (((uintptr_t)ksend | (uintptr_t)krecv) % 4 == 0) && (chunk_bytes % 4 == 0);
    int algo = oneshot ? 3 : 0;  // else the ring unless every rank can share its buffers
    const char* psend[kMaxRanks] = {};
    const char* precv[kMaxRanks] = {};
    if (read_sched) {
      // the read schedule: every rank takes part in the rendezvous, all decide alike (a captured
      // call reads through mappings its replays keep using: imports stay open until their owner
      // frees the allocation, which invalidates the graph anyway)
      const bool eligible = ksend == send && krecv == recv && local_s && local_r;
      bool vec_all = false;
      PeerBuffers::Decision d = PeerBuffers::kFallback;
      try {
        // a peer that does not reach the call within the watchdog's limit fails it, as the
        // kernel's own wait would (the reference's 10 s watchdog, mini_nccl.cu:200-214)
        // (the schedule choice rides along: ranks that differ in it -- mncclCommSetAlgo is per rank
        // -- would launch different kernel forms, so they fail the call as a mismatch)
        d = pbuf_.negotiate(send, recv, eligible, count, dtype, op, cfg_.timeout_ms / 1000.0 + 2.0,
                            [this] { wait_previous_call(); }, psend, precv, &vec_all, auto_ ? -1 : algo_);
      } catch (const PeerGaveUp& e) {
        return rendezvous_failed(e, true, cur_dev);
      } catch (const std::exception& e) {
        return rendezvous_failed(e, false, cur_dev);
      }
      if (d == PeerBuffers::kWindowPeer) {
        fprintf(stderr, "[Mini-NCCL] rank %d: a peer ran this all-reduce on registered windows, this rank's buffers "
                "are not in them (every rank must pass buffers of the same windows); communicator is no longer "
                "usable\n", rank_);
        sticky_ = ncclInvalidUsage;
        abort_peers();  // the peer's kernel waits for this rank's START: fail it now
        if (cur_dev != device_) hipSetDevice(cur_dev);
        return sticky_;
      }
      if (d == PeerBuffers::kMismatch) {
        fprintf(stderr, "[Mini-NCCL] rank %d: ranks called ncclAllReduce with different count / datatype / op / "
                "schedule (mncclCommSetAlgo)\n", rank_);
        if (cur_dev != device_) hipSetDevice(cur_dev);
        return ncclInvalidUsage;
      }
      if (d == PeerBuffers::kRead) {
        algo = 2;
        vec = vec_all && (chunk_bytes % 4 == 0);
      }
    }
    if (algo == 0 && small) algo = 3;
    seq = ++call_seq_;
    if (seq == 0) seq = ++call_seq_;  // 0 = "no kernel" (wait_for)
    launch(algo, ksend, krecv, chunk_bytes, dtype, op, stream, seq, vec, psend, precv, tail);
    if (rr == Reach::kStaged) hip_check(hipMemcpyAsync(recv, stage_, bytes, hipMemcpyDefault, stream), "stage out");
  }
  if (!capturing) {
    hip_check(hipEventRecord(order_ev_, stream), "order event");
    last_stream_ = stream;
    have_last_ = true;
  }
  if (cur_dev != device_) hipSetDevice(cur_dev);
  if (cfg_.blocking && cap == hipStreamCaptureStatusNone) return wait_for(stream, seq);
  return ncclSuccess;
}

ncclResult_t Comm::rendezvous_failed(const std::exception& e, bool peer_gave_up, int cur_dev) {
  fprintf(stderr, "[Mini-NCCL] rank %d: %s; communicator is no longer usable\n", rank_, e.what());
  if (peer_gave_up) {
    // a peer's communicator died in an earlier rendezvous: as a peer's ABORT in the kernel
    sticky_ = ncclRemoteError;
  } else {
    sticky_ = ncclInternalError;
    abort_peers();
  }
  if (cur_dev != device_) hipSetDevice(cur_dev);
  return sticky_;
}

const Comm::Window* Comm::find_window(const void* p, size_t bytes) const {
  const char* c = static_cast<const char*>(p);
  for (const Window& w : windows_)
    if (c >= w.base && (size_t)(c - w.base) <= w.bytes && bytes <= w.bytes - (size_t)(c - w.base)) return &w;
  return nullptr;
}

// Collective: every rank registers its buffer of the window (same size) in the same order.  One
// negotiated rendezvous of the read schedule maps every rank's buffer here (the same dma-buf
// imports the negotiated calls use, kept until the owner frees the allocation); the window's
// number is the registration's, the same on every rank.
ncclResult_t Comm::register_window(void* buf, size_t bytes, void** handle) {
  *handle = nullptr;
  if (sticky_ != ncclSuccess) return sticky_;
  if (check_status() != ncclSuccess) return sticky_;
  if (!buf || bytes == 0) return ncclInvalidArgument;
  int cur_dev = -1;
  hip_check(hipGetDevice(&cur_dev), "hipGetDevice");
  if (cur_dev != device_) hip_check(hipSetDevice(device_), "hipSetDevice");
  Window w;
  memset(&w, 0, sizeof w);
  w.base = static_cast<const char*>(buf);
  w.bytes = bytes;
  if (nranks_ == 1) {
    w.id = next_window_++;
    w.peer[0] = w.base;
    w.aligned = (uintptr_t)buf % 4 == 0;
    windows_.push_back(w);
    *handle = (void*)(uintptr_t)w.id;
    if (cur_dev != device_) hipSetDevice(cur_dev);
    return ncclSuccess;
  }
  if (!pbuf_.available()) {
    fprintf(stderr, "[Mini-NCCL] rank %d: registered windows need the read schedule's shared board, which is off\n",
            rank_);
    if (cur_dev != device_) hipSetDevice(cur_dev);
    return ncclInvalidUsage;  // the board is off on every rank alike: every rank returns this
  }
  pbuf_.reap(buf, buf);
  bool local = false;
  const void* kp = buf;
  const bool eligible = pbuf_.known(buf) || (reach(buf, &kp, &local) == Reach::kDevice && local);
  const char* psend[kMaxRanks] = {};
  const char* precv[kMaxRanks] = {};
  bool vec_all = false;
  PeerBuffers::Decision d = PeerBuffers::kFallback;
  constexpr int kRegisterDtype = 0x52;  // never an all-reduce's: a call cannot pair with a registration
  try {
    d = pbuf_.negotiate(buf, buf, eligible, bytes, kRegisterDtype, 0, cfg_.timeout_ms / 1000.0 + 2.0,
                        [this] { wait_previous_call(); }, psend, precv, &vec_all);
  } catch (const PeerGaveUp& e) {
    return rendezvous_failed(e, true, cur_dev);
  } catch (const std::exception& e) {
    return rendezvous_failed(e, false, cur_dev);
  }
  if (cur_dev != device_) hipSetDevice(cur_dev);
  if (d == PeerBuffers::kWindowPeer) {
    sticky_ = ncclInvalidUsage;
    abort_peers();
    return sticky_;
  }
  if (d == PeerBuffers::kMismatch) {
    fprintf(stderr, "[Mini-NCCL] rank %d: mncclCommRegister: the ranks registered windows of different sizes (or a "
            "rank called an all-reduce instead)\n", rank_);
    return ncclInvalidUsage;
  }
  if (d != PeerBuffers::kRead) {
    fprintf(stderr, "[Mini-NCCL] rank %d: mncclCommRegister: some rank's buffer is not device memory of its GPU "
            "that the peers can map\n", rank_);
    return ncclInvalidUsage;
  }
  w.id = next_window_++;
  for (int q = 0; q < nranks_; ++q) w.peer[q] = psend[q];
  w.aligned = vec_all;
  windows_.push_back(w);
  *handle = (void*)(uintptr_t)w.id;
  return ncclSuccess;
}

ncclResult_t Comm::deregister_window(void* handle) {
  const uint64_t id = (uint64_t)(uintptr_t)handle;
  for (size_t i = 0; i < windows_.size(); ++i)
    if (windows_[i].id == id) {
      windows_.erase(windows_.begin() + (long)i);
      return ncclSuccess;
    }
  return ncclInvalidArgument;
}

void Comm::abort_peers() {
  const uint64_t one = (uint64_t)(rank_ + 1);  // kernels.hip abort_word, with no kernel status
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  const uint64_t w = mbox_abort(nranks_, wave_channels());
  for (int q = 0; q < nranks_; ++q)
    if (q != rank_ && peer_mbox_[(size_t)q]) (void)hipMemcpyAsync(peer_mbox_[(size_t)q] + w, &one, sizeof one, hipMemcpyHostToDevice, st);
  (void)hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  (void)hipGetLastError();
}

ncclResult_t Comm::link_probe(int all_peers, size_t bytes, int iters, double* gbps) {
  if (nranks_ < 2 || iters < 1) return ncclInvalidArgument;
  // mode bits (mini_nccl_ext.h): 0 every peer, 1-2 access form, 3 pull instead of push, 4 the
  // peers' ordinary device memory instead of their scratch
  const int form = (all_peers >> 1) & 3;
  const bool pull = (all_peers >> 3) & 1;
  const bool user = (all_peers >> 4) & 1;
  if (form > kProbePlain || (all_peers & ~31)) return ncclInvalidArgument;
  all_peers &= 1;
  const size_t region = scratch_region_bytes(wave_channels(), cfg_.slots, wave_slice());
  if (bytes == 0 || bytes > region) bytes = region;  // the probe writes this rank's region at each peer
  int cur_dev = -1;
  hip_check(hipGetDevice(&cur_dev), "hipGetDevice");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  wait_previous_call();  // no all-reduce of this communicator may still be writing slots
  hipStream_t st;
  hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "probe stream");
  char* src = nullptr;
  hip_check(hipMalloc((void**)&src, bytes), "probe alloc");
  hip_check(hipMemsetAsync(src, 0x5a, bytes, st), "probe memset");
  std::vector<char*> dst;
  // user memory: every rank exports an ordinary (cached) device buffer of nranks x bytes; rank
  // d's slice [rank * bytes, +bytes) is this rank's target there (as the scratch region is).
  // From the process's pool and imported through its registry (ipcreg.h): repeated probes
  // re-use the buffers and the imports
  char* ub = nullptr;
  std::vector<char*> opened((size_t)nranks_, nullptr);
  if (user) {
    struct UserBuf {
      hipIpcMemHandle_t h;
      uint64_t nonce, base, id;
    } mine;
    ub = (char*)ipc::pool_acquire(bytes * (size_t)nranks_, 0, &mine.h, &mine.id);
    mine.nonce = process_nonce();
    mine.base = (uint64_t)(uintptr_t)ub;
    hip_check(hipMemsetAsync(ub, 0x3c, bytes * (size_t)nranks_, st), "probe memset");
    std::vector<UserBuf> all((size_t)nranks_);
    boot_.allgather(&mine, all.data(), sizeof mine);
    for (int q = 0; q < nranks_; ++q) {
      const UserBuf& u = all[(size_t)q];
      if (q == rank_ || u.nonce == mine.nonce) {
        opened[(size_t)q] = (char*)(uintptr_t)u.base;
        continue;
      }
      hipError_t e = hipSuccess;
      opened[(size_t)q] = ipc::open_block(u.nonce, u.base, u.id, u.h, &e);
      hip_check(opened[(size_t)q] ? hipSuccess : e, "probe ipc open");
    }
  }
  for (int k = 1; k < nranks_; ++k) {
    const int d = (rank_ + k) % nranks_;
    // in push mode this rank's region at d is where d receives from this rank
    dst.push_back(user ? opened[(size_t)d] + (size_t)rank_ * bytes
                       : peer_scratch_[(size_t)d] + (size_t)region_index(d, rank_) * region);
    if (!all_peers) break;
  }
  hipEvent_t e0, e1;
  hip_check(hipEventCreate(&e0), "event");
  hip_check(hipEventCreate(&e1), "event");
  hip_check(hipStreamSynchronize(st), "probe sync");
  boot_.barrier();  // every rank idle and launching together
  hip_check(launch_link_probe(src, dst.data(), (int)dst.size(), bytes, form, pull, st), "probe warm-up");
  hip_check(hipEventRecord(e0, st), "event");
  for (int i = 0; i < iters; ++i)
    hip_check(launch_link_probe(src, dst.data(), (int)dst.size(), bytes, form, pull, st), "probe");
  hip_check(hipEventRecord(e1, st), "event");
  hip_check(hipEventSynchronize(e1), "probe wait");
  float ms = 0;
  hip_check(hipEventElapsedTime(&ms, e0, e1), "event time");
  boot_.barrier();  // nobody starts an all-reduce while a peer still writes its slots
  *gbps = (double)bytes * iters / (ms * 1e-3) / 1e9;
  if (user) ipc::pool_release(ub);  // every peer is done with it (the barrier above)
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipStreamDestroy(st);
  hipFree(src);
  if (cur_dev != device_) hipSetDevice(cur_dev);
  return ncclSuccess;
}

ncclResult_t local_reduce(void* out, const void* local, const void* incoming, size_t count, int dtype, int op,
                          hipStream_t stream) {
  hip_check(launch_local_reduce(dtype, op, out, local, incoming, count, stream), "local reduce launch");
  return ncclSuccess;
}

}  // namespace mnccl
