// peerbuf.cpp -- see peerbuf.h.
#include "peerbuf.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "kernels.h"

namespace mnccl {

namespace {

constexpr uint32_t kBoardMagic = 0x4d4e4252u;  // 'MNBR'
constexpr int kBoardDepth = 16;                // records per rank in flight (calls ahead of the slowest peer)
constexpr size_t kMaxExports = 64, kMaxMappings = 64;

double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

void backoff(int spins) {
  if (spins < 2000) sched_yield();
  else usleep(20);
}

}  // namespace

struct BufDesc {
  uint64_t base, id, off;  // allocation base / id in the owner's process, buffer - base
  uint64_t raw;            // the buffer's address in the owner's process (same-process peers)
  hipIpcMemHandle_t h;     // of the allocation base
};

struct alignas(64) CallRec {
  std::atomic<uint64_t> seq;  // the call this record describes; stored last (release)
  uint64_t count;
  int32_t dtype, op, eligible, aligned;
  BufDesc send, recv;
};

struct alignas(64) Counter {
  std::atomic<uint64_t> v;
};

struct Board {
  uint32_t magic, nranks;
  Counter consumed[kMaxRanks];  // last call whose records rank q has read
  CallRec rec[kMaxRanks][kBoardDepth];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "the board needs address-free atomics");

PeerBuffers::~PeerBuffers() {
  close_all();
  if (board_) munmap(board_, board_bytes_);
  board_ = nullptr;
}

void PeerBuffers::init(Bootstrap& boot, int rank, int nranks, const std::vector<uint64_t>& nonces, int port) {
  rank_ = rank;
  nranks_ = nranks;
  nonces_ = nonces;
  board_bytes_ = (sizeof(Board) + 4095) & ~(size_t)4095;
  // rank 0 creates the segment under a name unique to this communicator and shares it; every
  // rank maps it; once all have, rank 0 unlinks it (nothing is left in /dev/shm, even if a
  // process dies later)
  char name[64];
  memset(name, 0, sizeof name);
  int fd = -1;
  if (rank == 0) {
    snprintf(name, sizeof name, "/mnccl-%d-%d-%016llx", (int)getpid(), port, (unsigned long long)nonces[0]);
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd >= 0 && ftruncate(fd, (off_t)board_bytes_) != 0) {
      close(fd);
      shm_unlink(name);
      fd = -1;
    }
    if (fd < 0) name[0] = 0;
  }
  std::vector<char> names((size_t)nranks * sizeof name);
  boot.allgather(name, names.data(), sizeof name);
  if (rank != 0 && names[0]) fd = shm_open(names.data(), O_RDWR, 0600);
  void* m = MAP_FAILED;
  if (fd >= 0) {
    m = mmap(nullptr, board_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
  }
  int ok = m != MAP_FAILED ? 1 : 0;
  std::vector<int> oks((size_t)nranks);
  boot.allgather(&ok, oks.data(), sizeof ok);
  if (rank == 0 && names[0]) shm_unlink(names.data());
  bool all = true;
  for (int v : oks) all = all && v;
  if (!all) {
    if (m != MAP_FAILED) munmap(m, board_bytes_);
    return;  // no board anywhere: the read schedule falls back on every rank
  }
  board_ = static_cast<Board*>(m);
  if (rank == 0) {
    board_->magic = kBoardMagic;
    board_->nranks = (uint32_t)nranks;
  }
  boot.barrier();  // the zeroed board is initialised before anyone negotiates
}

bool PeerBuffers::describe(const void* p, uint64_t* base, uint64_t* id, hipIpcMemHandle_t* h) {
  hipDeviceptr_t b = 0;
  size_t sz = 0;
  unsigned long long bid = 0;
  if (hipMemGetAddressRange(&b, &sz, (hipDeviceptr_t)p) != hipSuccess ||
      hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  *base = (uint64_t)(uintptr_t)b;
  *id = bid;
  for (const Export& e : exports_)
    if (e.base == *base && e.id == bid) {
      *h = e.h;
      return true;
    }
  if (hipIpcGetMemHandle(h, (void*)b) != hipSuccess) {  // e.g. a virtual-memory-managed allocation
    (void)hipGetLastError();
    return false;
  }
  if (exports_.size() >= kMaxExports) exports_.erase(exports_.begin());
  exports_.push_back(Export{*base, bid, *h});
  return true;
}

char* PeerBuffers::map_peer(int q, uint64_t base, uint64_t id, const hipIpcMemHandle_t& h,
                            const std::function<void()>& sync_previous, bool pin) {
  for (Mapping& m : peers_)
    if (m.rank == q && m.base == base && m.id == id) {
      m.last_use = seq_;
      m.pinned = m.pinned || pin;
      return m.local;
    }
  size_t unpinned = 0;
  for (const Mapping& m : peers_) unpinned += m.pinned ? 0 : 1;
  if (unpinned >= kMaxMappings) {
    // least recently used (unpinned) out; the last kernel may still read through it
    size_t lru = peers_.size();
    for (size_t i = 0; i < peers_.size(); ++i)
      if (!peers_[i].pinned && (lru == peers_.size() || peers_[i].last_use < peers_[lru].last_use)) lru = i;
    sync_previous();
    (void)hipIpcCloseMemHandle(peers_[lru].local);
    peers_.erase(peers_.begin() + (long)lru);
  }
  void* p = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  // an open can fail transiently while the runtime finishes a close; retry a few times before
  // failing the call (every failure and retry is reported)
  for (int attempt = 1; e != hipSuccess && attempt <= 5; ++attempt) {
    (void)hipGetLastError();
    char hx[129];
    for (int i = 0; i < 64; ++i) snprintf(hx + 2 * i, 3, "%02x", (unsigned char)h.reserved[i]);
    fprintf(stderr,
            "[Mini-NCCL] rank %d: hipIpcOpenMemHandle of rank %d's allocation (base 0x%llx, id %llu) failed: %s; "
            "%zu mappings open, handle %s; retry %d\n",
            rank_, q, (unsigned long long)base, (unsigned long long)id, hipGetErrorString(e), peers_.size(), hx, attempt);
    usleep(1000u << attempt);
    e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    throw std::runtime_error(std::string("read schedule: hipIpcOpenMemHandle of rank ") + std::to_string(q) +
                             "'s buffer: " + hipGetErrorString(e));
  }
  peers_.push_back(Mapping{q, base, id, (char*)p, seq_, pin});
  return (char*)p;
}

void PeerBuffers::close_all() {
  for (Mapping& m : peers_) (void)hipIpcCloseMemHandle(m.local);
  peers_.clear();
  (void)hipGetLastError();
}

PeerBuffers::Decision PeerBuffers::negotiate(const void* send, const void* recv, bool eligible, uint64_t count,
                                             int dtype, int op, double timeout_s,
                                             const std::function<void()>& sync_previous, const char** psend,
                                             const char** precv, bool* vec_all, bool pin) {
  const uint64_t k = ++seq_;
  const int slot = (int)(k % kBoardDepth);
  const double t0 = now_s();
  auto wait = [&](const std::atomic<uint64_t>& v, uint64_t want, int q, const char* what) {
    for (int spins = 0; v.load(std::memory_order_acquire) < want; ++spins) {
      if (now_s() - t0 > timeout_s)
        throw std::runtime_error("read schedule: rank " + std::to_string(q) + " did not " + what + " all-reduce #" +
                                 std::to_string(k) + " within " + std::to_string((int)timeout_s) + " s");
      backoff(spins);
    }
  };
  // my record slot is free once every peer has read the record kBoardDepth calls back
  if (k > (uint64_t)kBoardDepth)
    for (int q = 0; q < nranks_; ++q)
      if (q != rank_) wait(board_->consumed[q].v, k - kBoardDepth, q, "finish reading the records before");

  CallRec& me = board_->rec[rank_][slot];
  BufDesc sd, rd;
  memset(&sd, 0, sizeof sd);
  memset(&rd, 0, sizeof rd);
  bool ok = eligible && describe(send, &sd.base, &sd.id, &sd.h) && describe(recv, &rd.base, &rd.id, &rd.h);
  sd.raw = (uint64_t)(uintptr_t)send;
  rd.raw = (uint64_t)(uintptr_t)recv;
  sd.off = ok ? sd.raw - sd.base : 0;
  rd.off = ok ? rd.raw - rd.base : 0;
  me.count = count;
  me.dtype = dtype;
  me.op = op;
  me.eligible = ok ? 1 : 0;
  me.aligned = ((sd.raw | rd.raw) % 4 == 0) ? 1 : 0;
  me.send = sd;
  me.recv = rd;
  me.seq.store(k, std::memory_order_release);

  struct Seen {
    uint64_t count;
    int32_t dtype, op, eligible, aligned;
    BufDesc send, recv;
  };
  std::vector<Seen> recs((size_t)nranks_);
  for (int q = 0; q < nranks_; ++q) {
    const CallRec& c = board_->rec[q][slot];
    if (q != rank_) wait(c.seq, k, q, "reach");
    recs[(size_t)q] = Seen{c.count, c.dtype, c.op, c.eligible, c.aligned, c.send, c.recv};
  }
  board_->consumed[rank_].v.store(k, std::memory_order_release);  // my copies are taken
  bool all = true, mismatch = false, aligned = true;
  for (const Seen& c : recs) {
    all = all && c.eligible;
    aligned = aligned && c.aligned;
    mismatch = mismatch || c.count != count || c.dtype != dtype || c.op != op;
  }
  const Decision d = mismatch ? kMismatch : all ? kRead : kFallback;
  if (d != kRead) return d;
  for (int q = 0; q < nranks_; ++q) {
    const Seen& c = recs[(size_t)q];
    if (q == rank_ || nonces_[(size_t)q] == nonces_[(size_t)rank_]) {
      psend[q] = (const char*)(uintptr_t)c.send.raw;  // this process's address space
      precv[q] = (const char*)(uintptr_t)c.recv.raw;
      continue;
    }
    psend[q] = map_peer(q, c.send.base, c.send.id, c.send.h, sync_previous, pin) + c.send.off;
    precv[q] = map_peer(q, c.recv.base, c.recv.id, c.recv.h, sync_previous, pin) + c.recv.off;
  }
  *vec_all = aligned;
  return d;
}

}  // namespace mnccl
