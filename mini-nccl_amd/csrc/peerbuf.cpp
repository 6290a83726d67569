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
  float t[2];  // this rank's calibration timings so far (Comm: read, scratch schedule; 0 = unknown)
  // second round (only when some rank may have to open a new mapping): the call whose mapping
  // outcome map_ok reports, stored after it (release)
  alignas(64) std::atomic<uint64_t> mapped;
  int32_t map_ok;
};

struct alignas(64) Counter {
  std::atomic<uint64_t> v;
};

struct Board {
  uint32_t magic, nranks;
  Counter consumed[kMaxRanks];  // last call whose records rank q has read
  Counter gave_up[kMaxRanks];   // != 0: rank q abandoned a rendezvous (its communicator is dead)
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
  if (test_fake_) {  // CPU self-test: the pointer's page is its "allocation", the value its id
    *base = (uint64_t)(uintptr_t)p & ~(uint64_t)4095;
    *id = (uint64_t)(uintptr_t)p;
    memset(h, 0, sizeof *h);
    return true;
  }
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
  if (test_fake_) {  // CPU self-test: no HIP; fail on the chosen call
    if (seq_ == test_fail_call_) throw std::runtime_error("read schedule: injected mapping failure (self-test)");
    peers_.push_back(Mapping{q, base, id, (char*)(uintptr_t)base, seq_, pin});
    if (peers_.size() > kMaxMappings) peers_.erase(peers_.begin());
    return (char*)(uintptr_t)base;
  }
  void* p = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  // an open can fail transiently; retry a few times before failing the call (every failure
  // and retry is reported)
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
  // over the bound: the least recently used (unpinned) mapping goes, AFTER the new one is open
  // (a close immediately followed by an open could hand the new import the address range the
  // runtime is still releasing); the last kernel may still read through it, so wait for it
  size_t unpinned = 0;
  for (const Mapping& m : peers_) unpinned += m.pinned ? 0 : 1;
  if (unpinned > kMaxMappings) {
    size_t lru = peers_.size();
    for (size_t i = 0; i < peers_.size(); ++i)
      if (!peers_[i].pinned && (lru == peers_.size() || peers_[i].last_use < peers_[lru].last_use)) lru = i;
    sync_previous();
    (void)hipIpcCloseMemHandle(peers_[lru].local);
    (void)hipGetLastError();
    peers_.erase(peers_.begin() + (long)lru);
  }
  return (char*)p;
}

void PeerBuffers::close_all() {
  if (!test_fake_)
    for (Mapping& m : peers_) (void)hipIpcCloseMemHandle(m.local);
  peers_.clear();
  (void)hipGetLastError();
}

PeerBuffers::Decision PeerBuffers::negotiate(const void* send, const void* recv, bool eligible, uint64_t count,
                                             int dtype, int op, double timeout_s,
                                             const std::function<void()>& sync_previous, const char** psend,
                                             const char** precv, bool* vec_all, bool pin, const float* my_t,
                                             float* max_t) {
  const uint64_t k = ++seq_;
  const double t0 = now_s();
  auto wait = [&](const std::atomic<uint64_t>& v, uint64_t want, int q, const char* what) {
    for (int spins = 0; v.load(std::memory_order_acquire) < want; ++spins) {
      if (board_->gave_up[q].v.load(std::memory_order_acquire) != 0)
        throw PeerGaveUp("read schedule: rank " + std::to_string(q) + " abandoned the communicator before all-reduce #" +
                         std::to_string(k));
      if (now_s() - t0 > timeout_s)
        throw std::runtime_error("read schedule: rank " + std::to_string(q) + " did not " + what + " all-reduce #" +
                                 std::to_string(k) + " within " + std::to_string((int)timeout_s) + " s");
      backoff(spins);
    }
  };
  try {
    return negotiate_body(k, send, recv, eligible, count, dtype, op, sync_previous, psend, precv, vec_all, pin,
                          my_t, max_t, wait);
  } catch (...) {
    // this rank gives up (a peer that never came or gave up itself, a mapping that failed): say
    // so on the board, so every peer waiting in a rendezvous with it fails at once instead of at
    // its own limit (the abandonment cascades through the ranks)
    board_->gave_up[rank_].v.store(k, std::memory_order_release);
    throw;
  }
}

template <typename Wait>
PeerBuffers::Decision PeerBuffers::negotiate_body(uint64_t k, const void* send, const void* recv, bool eligible,
                                                  uint64_t count, int dtype, int op,
                                                  const std::function<void()>& sync_previous, const char** psend,
                                                  const char** precv, bool* vec_all, bool pin, const float* my_t,
                                                  float* max_t, const Wait& wait) {
  const int slot = (int)(k % kBoardDepth);
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
  me.t[0] = my_t ? my_t[0] : 0.f;
  me.t[1] = my_t ? my_t[1] : 0.f;
  me.seq.store(k, std::memory_order_release);

  struct Seen {
    uint64_t count;
    int32_t dtype, op, eligible, aligned;
    BufDesc send, recv;
  };
  std::vector<Seen> recs((size_t)nranks_);
  float tmax[2] = {0.f, 0.f};
  bool tall[2] = {true, true};
  for (int q = 0; q < nranks_; ++q) {
    const CallRec& c = board_->rec[q][slot];
    if (q != rank_) wait(c.seq, k, q, "reach");
    recs[(size_t)q] = Seen{c.count, c.dtype, c.op, c.eligible, c.aligned, c.send, c.recv};
    for (int i = 0; i < 2; ++i) {
      tall[i] = tall[i] && c.t[i] > 0.f;
      tmax[i] = c.t[i] > tmax[i] ? c.t[i] : tmax[i];
    }
  }
  if (max_t)  // every rank's timing known -> their max (what every rank reads alike), else 0
    for (int i = 0; i < 2; ++i) max_t[i] = tall[i] ? tmax[i] : 0.f;
  bool all = true, mismatch = false, aligned = true;
  for (const Seen& c : recs) {
    all = all && c.eligible;
    aligned = aligned && c.aligned;
    mismatch = mismatch || c.count != count || c.dtype != dtype || c.op != op;
  }
  const Decision d = mismatch ? kMismatch : all ? kRead : kFallback;
  if (d != kRead) {
    board_->consumed[rank_].v.store(k, std::memory_order_release);  // my copies are taken
    return d;
  }
  // Would any rank have to open a mapping?  Every buffer used by a read call in the last
  // `horizon` read calls is still mapped by every other rank (each keeps its kMaxMappings most
  // recently used; those calls used at most 2(n-1) per rank), so if every buffer of this call is
  // among them, no rank opens anything -- the common case of a caller reusing its buffers -- and
  // no second round is needed.  Computed from the records alone: every rank reaches the same
  // answer.
  const size_t horizon = kMaxMappings / (size_t)(2 * (nranks_ > 1 ? nranks_ - 1 : 1));
  auto recent = [&](int q, const BufDesc& b) {
    for (const auto& call : recent_)
      for (const RecentKey& x : call)
        if (x.rank == q && x.base == b.base && x.id == b.id) return true;
    return false;
  };
  bool need_agree = false;
  for (int q = 0; q < nranks_ && !need_agree; ++q)
    need_agree = !recent(q, recs[(size_t)q].send) || !recent(q, recs[(size_t)q].recv);
  bool mapped = true;
  std::string why;
  for (int q = 0; q < nranks_; ++q) {
    const Seen& c = recs[(size_t)q];
    if (q == rank_ || nonces_[(size_t)q] == nonces_[(size_t)rank_]) {
      psend[q] = (const char*)(uintptr_t)c.send.raw;  // this process's address space
      precv[q] = (const char*)(uintptr_t)c.recv.raw;
      continue;
    }
    if (!mapped) continue;
    try {
      psend[q] = map_peer(q, c.send.base, c.send.id, c.send.h, sync_previous, pin) + c.send.off;
      precv[q] = map_peer(q, c.recv.base, c.recv.id, c.recv.h, sync_previous, pin) + c.recv.off;
    } catch (const std::runtime_error& e) {
      if (!need_agree) throw;  // cannot happen (nothing new to open); fail loudly if it does
      mapped = false;
      why = e.what();
    }
  }
  Decision out = kRead;
  if (need_agree) {
    // second round: every rank's mapping outcome; one failure -> the scratch schedule for this
    // call on every rank (same bits, no buffer of a peer is read)
    ++agreements_;
    me.map_ok = mapped ? 1 : 0;
    me.mapped.store(k, std::memory_order_release);
    int failed = -1;
    for (int q = 0; q < nranks_; ++q) {
      const CallRec& c = board_->rec[q][slot];
      if (q != rank_) wait(c.mapped, k, q, "report its mappings for");
      if (!c.map_ok && failed < 0) failed = q;
    }
    if (failed >= 0) {
      fprintf(stderr, "[Mini-NCCL] rank %d: all-reduce #%llu falls back to the scratch schedule: rank %d could not map "
              "a peer's buffer%s%s\n", rank_, (unsigned long long)k, failed, why.empty() ? "" : ": ", why.c_str());
      out = kFallback;
    }
  }
  board_->consumed[rank_].v.store(k, std::memory_order_release);  // my copies are taken
  if (out == kRead) {
    std::vector<RecentKey> keys;
    for (int q = 0; q < nranks_; ++q) {
      keys.push_back(RecentKey{q, recs[(size_t)q].send.base, recs[(size_t)q].send.id});
      keys.push_back(RecentKey{q, recs[(size_t)q].recv.base, recs[(size_t)q].recv.id});
    }
    recent_.push_back(std::move(keys));
    while (recent_.size() > horizon) recent_.pop_front();
  }
  *vec_all = aligned;
  return out;
}

}  // namespace mnccl
