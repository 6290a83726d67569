// peerbuf.cpp -- see peerbuf.h.
#include "peerbuf.h"

#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "ipcreg.h"
#include "kernels.h"

namespace mnccl {

namespace {

constexpr uint32_t kBoardMagic = 0x4d4e4253u;  // 'MNBS'
constexpr int kBoardDepth = 16;                // records per rank in flight (calls ahead of the slowest peer)
constexpr int kMaxFreed = 8;                   // freed allocations one record reports (the rest: next calls)
constexpr size_t kMaxKnown = 4096;
constexpr size_t kReapBatch = 4;               // other live exports checked for a free per call

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
  ipc::Shared d;           // the allocation's dma-buf export (ipcreg.h)
};

struct alignas(64) CallRec {
  std::atomic<uint64_t> seq;  // the call this record describes; stored last (release)
  uint64_t count;
  int32_t dtype, op, eligible, aligned;
  int32_t form;  // the kernel form this rank launches for the call (negotiate's `form`)
  BufDesc send, recv;
  int32_t nfreed;
  uint64_t freed[kMaxFreed][2];  // (base, id) of this rank's exported allocations freed since its last record
  // a registered-window call (publish_fast): this rank did not wait for the others' records, its
  // kernel checks the call's signature on the device
  int32_t fast;
  uint64_t sig;
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

// A datagram carrying the descriptors of a rank's allocations that are new to the communicator
// (SCM_RIGHTS: nfd descriptors, in the order of base / id).
struct FdMsg {
  uint64_t k;  // the call
  int32_t src, nfd;
  uint64_t base[2], id[2];
};

PeerBuffers::~PeerBuffers() {
  // imports stay open (ipcreg.h): a later communicator of this process reuses them
  if (board_) munmap(board_, board_bytes_);
  board_ = nullptr;
  if (sock_ >= 0) close(sock_);
  for (Pending& p : pending_)
    for (int i = 0; i < p.nfd; ++i) close(p.fd[i]);
  for (auto& f : fake_fds_) close(f.second);
}

void PeerBuffers::sock_addr(int q, void* addr, unsigned* len) const {
  sockaddr_un* a = static_cast<sockaddr_un*>(addr);
  memset(a, 0, sizeof *a);
  a->sun_family = AF_UNIX;
  // abstract namespace (leading NUL): nothing on the file system, gone with the socket
  const int k = snprintf(a->sun_path + 1, sizeof a->sun_path - 1, "%s-r%d", sock_base_.c_str(), q);
  *len = (unsigned)(offsetof(sockaddr_un, sun_path) + 1 + (size_t)k);
}

void PeerBuffers::init(Bootstrap& boot, int rank, int nranks, const std::vector<uint64_t>& nonces, int port) {
  rank_ = rank;
  nranks_ = nranks;
  nonces_ = nonces;
  if (!test_fake_ && hipGetDevice(&device_) != hipSuccess) {
    (void)hipGetLastError();
    device_ = -1;
  }
  if (!test_fake_) freed_cursor_ = ipc::freed_log_size();  // earlier frees: earlier communicators' business
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
  if (ok && rank == 0) {
    Board* b = static_cast<Board*>(m);
    b->magic = kBoardMagic;
    b->nranks = (uint32_t)nranks;
  }
  // this rank's socket for the descriptors of new allocations (named after the board: unique
  // to the communicator)
  if (ok) {
    sock_base_ = std::string("mnccl") + (names.data() + 1);
    sock_ = socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    sockaddr_un a;
    unsigned len = 0;
    sock_addr(rank, &a, &len);
    if (test_unreachable_ && len + 2 <= sizeof a) {  // CPU self-test: a name no peer sends to
      a.sun_path[len - offsetof(sockaddr_un, sun_path)] = '-';
      a.sun_path[len - offsetof(sockaddr_un, sun_path) + 1] = 'x';
      len += 2;
    }
    const int one = 1;  // the sender's credentials come with every datagram (checked in drain)
    if (sock_ < 0 || bind(sock_, (const sockaddr*)&a, (socklen_t)len) != 0 ||
        setsockopt(sock_, SOL_SOCKET, SO_PASSCRED, &one, sizeof one) != 0)
      ok = 0;
  }
  std::vector<int> oks((size_t)nranks);
  boot.allgather(&ok, oks.data(), sizeof ok);  // also: rank 0's board is initialised
  if (rank == 0 && names[0]) shm_unlink(names.data());
  bool all = true;
  for (int v : oks) all = all && v;
  const char* off_why = "the ranks share no /dev/shm (per-call records)";
  if (all) {
    // every socket is bound: can every rank reach every rank of another process?  (Abstract
    // sockets live in a network namespace: ranks in separate containers that share /dev/shm
    // would otherwise fail their first call with new buffers instead of running the ring.)
    int reach = hello(10.0) ? 1 : 0;  // generous: a loaded host must not turn it off
    boot.allgather(&reach, oks.data(), sizeof reach);
    for (int v : oks) all = all && v;
    off_why = "a rank cannot reach its peers' descriptor sockets (separate network namespaces?)";
  }
  if (!all) {
    if (m != MAP_FAILED) munmap(m, board_bytes_);
    if (sock_ >= 0) close(sock_);
    sock_ = -1;
    for (Pending& p : pending_)
      for (int i = 0; i < p.nfd; ++i) close(p.fd[i]);
    pending_.clear();
    if (rank == 0)
      fprintf(stderr, "[Mini-NCCL] warning: %s: the read schedule is off and every call runs the ring\n", off_why);
    return;  // no board anywhere: the read schedule falls back on every rank
  }
  board_ = static_cast<Board*>(m);
  boot.barrier();  // the board is initialised before anyone negotiates
}

// Init: a datagram with no descriptors (call 0) to every rank of another process, and one from
// each of them, within timeout_s.  False as soon as a peer's socket refuses (it is not in this
// network namespace) or when the time is up.
bool PeerBuffers::hello(double timeout_s) {
  FdMsg m;
  memset(&m, 0, sizeof m);
  m.src = rank_;
  std::vector<char> sent((size_t)nranks_, 0), heard((size_t)nranks_, 0);
  for (int q = 0; q < nranks_; ++q)
    if (q == rank_ || nonces_[(size_t)q] == nonces_[(size_t)rank_]) sent[(size_t)q] = heard[(size_t)q] = 1;
  const double t0 = now_s();
  for (int spins = 0;; ++spins) {
    bool done = true;
    for (int q = 0; q < nranks_; ++q) {
      if (sent[(size_t)q]) continue;
      const int rc = try_send(q, m, nullptr, 0);
      if (rc < 0) return false;
      sent[(size_t)q] = rc > 0;
      done = done && rc > 0;
    }
    drain();
    for (size_t i = 0; i < pending_.size();) {
      if (pending_[i].k != 0) {
        ++i;
        continue;
      }
      heard[(size_t)pending_[i].src] = 1;
      for (int j = 0; j < pending_[i].nfd; ++j) close(pending_[i].fd[j]);
      pending_.erase(pending_.begin() + (long)i);
    }
    for (char h : heard) done = done && h;
    if (done) return true;
    if (now_s() - t0 > timeout_s) return false;
    backoff(spins);
  }
}

void PeerBuffers::reap(const void* send, const void* recv) {
  // allocations this process exported and has freed since my last call: my peers close their
  // imports (the process's log: another communicator of this process may have found them)
  if (test_fake_) return;
  const uint64_t addrs[2] = {(uint64_t)(uintptr_t)send, (uint64_t)(uintptr_t)recv};
  ipc::reap_freed_exports(addrs, 2, kReapBatch);
  for (const size_t end = ipc::freed_log_size(); freed_cursor_ < end; ++freed_cursor_)
    freed_.push_back(ipc::freed_log_at(freed_cursor_));
}

bool PeerBuffers::known(const void* p) const {
  uint64_t b = 0, i = 0;
  ipc::Shared d;
  return !test_fake_ && ipc::find_live_export((uint64_t)(uintptr_t)p, &b, &i, &d);
}

size_t PeerBuffers::mapped_allocations() const { return test_fake_ ? fake_maps_.size() : ipc::imports(); }

// (base, id, export) of the allocation holding p, exported once; false: it cannot be shared
// (not a plain device allocation, or its export failed)
bool PeerBuffers::describe(const void* p, uint64_t* base, uint64_t* id, ipc::Shared* d) {
  if (test_fake_) {  // CPU self-test: the pointer's page is its "allocation", the value its id,
                     // a memfd its "dma-buf" (the descriptors really travel)
    *base = (uint64_t)(uintptr_t)p & ~(uint64_t)4095;
    *id = (uint64_t)(uintptr_t)p;
    memset(d, 0, sizeof *d);
    auto it = fake_fds_.find(std::make_pair(*base, *id));
    if (it == fake_fds_.end())
      it = fake_fds_.emplace(std::make_pair(*base, *id), memfd_create("mnccl-selftest", MFD_CLOEXEC)).first;
    const int fd = it->second;
    struct stat sb;
    if (fd < 0 || fstat(fd, &sb) != 0) return false;
    d->fd = fd;
    d->ino = (uint64_t)sb.st_ino;
    return true;
  }
  if (ipc::find_live_export((uint64_t)(uintptr_t)p, base, id, d)) return true;  // checked alive by reap()
  // a new allocation (once per allocation): its range and id.  Not HIP_POINTER_ATTRIBUTE_RANGE_SIZE:
  // it comes back truncated to 32 bits (0 for a 4 GiB allocation on ROCm 7.2)
  hipDeviceptr_t b = 0;
  size_t sz = 0;
  unsigned long long bid = 0;
  if (hipMemGetAddressRange(&b, &sz, (hipDeviceptr_t)p) != hipSuccess || !b || !sz ||
      hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  *base = (uint64_t)(uintptr_t)b;
  *id = bid;
  std::string why;
  if (ipc::export_allocation(*base, bid, sz, d, &why)) return true;
  if (!warned_export_) {
    fprintf(stderr, "[Mini-NCCL] rank %d: a buffer cannot be shared with the peers (%s): its calls run the ring\n", rank_,
            why.c_str());
    warned_export_ = true;
  }
  return false;
}

// rank q's allocation (base, id) mapped here; nullptr (and *why) if it cannot be.  fd: a
// duplicate of the owner's descriptor if one arrived for it (-1 if none), always consumed.
char* PeerBuffers::map_peer(int q, uint64_t base, uint64_t id, int fd, const ipc::Shared& d, std::string* why) {
  if (test_fake_) {  // CPU self-test: no HIP; fail on the chosen call
    struct stat sb;
    const bool named = fd >= 0 && fstat(fd, &sb) == 0 && (uint64_t)sb.st_ino == d.ino;
    if (fd >= 0) close(fd);
    for (const Known& k : fake_maps_)
      if (k.rank == q && k.base == base && k.id == id) return (char*)(uintptr_t)base;
    if (seq_ == test_fail_call_) {
      *why = "injected mapping failure (self-test)";
      return nullptr;
    }
    if (!named) {
      *why = fd < 0 ? "no descriptor arrived from the owner (self-test)"
                    : "the received descriptor does not name the owner's (self-test)";
      return nullptr;
    }
    fake_maps_.push_back(Known{q, base, id});
    return (char*)(uintptr_t)base;
  }
  const uint64_t owner = nonces_[(size_t)q];
  if (char* p = ipc::find_import(owner, base, id)) {
    if (fd >= 0) close(fd);
    return p;
  }
  if (ipc::imports() + ipc::retired_imports() >= ipc::kMaxImports) {
    if (fd >= 0) close(fd);
    *why = "the process maps " + std::to_string(ipc::kMaxImports) + " peer allocations already";
    ipc::note_cap_refusal(*why);
    return nullptr;
  }
  std::string w;
  char* p = ipc::open_import(owner, base, id, fd, d, &w);
  if (!p) {
    char msg[160];
    snprintf(msg, sizeof msg, "import of rank %d's allocation (base 0x%llx, id %llu): ", q, (unsigned long long)base,
             (unsigned long long)id);
    *why = msg + w;
  }
  return p;
}

void PeerBuffers::publish_fast(uint64_t count, int dtype, int op, uint64_t sig, double timeout_s) {
  const uint64_t k = ++seq_;
  const double t0 = now_s();
  const int slot = (int)(k % kBoardDepth);
  try {
    // my record slot is free once every peer has read the record kBoardDepth calls back (a peer on
    // registered windows too marks its records read as it publishes them): a rank runs at most
    // kBoardDepth calls ahead of its slowest peer, the only host-side wait of a window call
    if (k > (uint64_t)kBoardDepth)
      for (int q = 0; q < nranks_; ++q) {
        if (q == rank_) continue;
        for (int spins = 0; board_->consumed[q].v.load(std::memory_order_acquire) < k - kBoardDepth; ++spins) {
          if (board_->gave_up[q].v.load(std::memory_order_acquire) != 0)
            throw PeerGaveUp("read schedule: rank " + std::to_string(q) + " abandoned the communicator before all-reduce #" +
                             std::to_string(k));
          if (now_s() - t0 > timeout_s)
            throw std::runtime_error("registered windows: rank " + std::to_string(q) + " stayed more than " +
                                     std::to_string(kBoardDepth) + " calls behind for " + std::to_string((int)timeout_s) +
                                     " s (all-reduce #" + std::to_string(k) + ")");
          backoff(spins);
        }
      }
  } catch (...) {
    board_->gave_up[rank_].v.store(k, std::memory_order_release);
    throw;
  }
  CallRec& me = board_->rec[rank_][slot];
  me.count = count;
  me.dtype = dtype;
  me.op = op;
  me.form = 0;
  me.eligible = 1;
  me.aligned = 1;
  memset(&me.send, 0, sizeof me.send);
  memset(&me.recv, 0, sizeof me.recv);
  me.nfreed = 0;  // frees wait for this rank's next negotiated record
  me.fast = 1;
  me.sig = sig;
  me.seq.store(k, std::memory_order_release);
  board_->consumed[rank_].v.store(k, std::memory_order_release);  // nothing of this call to read
}

PeerBuffers::Decision PeerBuffers::negotiate(const void* send, const void* recv, bool eligible, uint64_t count,
                                             int dtype, int op, double timeout_s,
                                             const std::function<void()>& sync_previous, const char** psend,
                                             const char** precv, bool* vec_all, int form) {
  const uint64_t k = ++seq_;
  const double t0 = now_s();
  // spins until ready() -- bounded by the peer q giving up and by the rendezvous limit
  auto wait_for = [&](const std::function<bool()>& ready, int q, const char* what) {
    for (int spins = 0; !ready(); ++spins) {
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
    return negotiate_body(k, send, recv, eligible, count, dtype, op, form, sync_previous, psend, precv, vec_all,
                          wait_for);
  } catch (...) {
    // this rank gives up (a peer that never came or gave up itself): say so on the board, so
    // every peer waiting in a rendezvous with it fails at once instead of at its own limit (the
    // abandonment cascades through the ranks)
    board_->gave_up[rank_].v.store(k, std::memory_order_release);
    throw;
  }
}

int PeerBuffers::try_send(int q, const FdMsg& m, const int* fds, int nfd) {
  sockaddr_un a;
  unsigned len = 0;
  sock_addr(q, &a, &len);
  iovec io{const_cast<FdMsg*>(&m), sizeof m};
  char cbuf[CMSG_SPACE(2 * sizeof(int))];
  memset(cbuf, 0, sizeof cbuf);
  msghdr h;
  memset(&h, 0, sizeof h);
  h.msg_name = &a;
  h.msg_namelen = (socklen_t)len;
  h.msg_iov = &io;
  h.msg_iovlen = 1;
  if (nfd > 0) {
    h.msg_control = cbuf;
    h.msg_controllen = CMSG_SPACE((size_t)nfd * sizeof(int));
    cmsghdr* c = CMSG_FIRSTHDR(&h);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN((size_t)nfd * sizeof(int));
    memcpy(CMSG_DATA(c), fds, (size_t)nfd * sizeof(int));
  }
  if (sendmsg(sock_, &h, MSG_DONTWAIT | MSG_NOSIGNAL) >= 0) return 1;
  return errno == EAGAIN || errno == EWOULDBLOCK ? 0 : -1;
}

bool PeerBuffers::drain() {
  bool any = false;
  for (;;) {
    FdMsg m;
    memset(&m, 0, sizeof m);
    iovec io{&m, sizeof m};
    alignas(cmsghdr) char cbuf[CMSG_SPACE(2 * sizeof(int)) + CMSG_SPACE(sizeof(ucred))];
    msghdr h;
    memset(&h, 0, sizeof h);
    h.msg_iov = &io;
    h.msg_iovlen = 1;
    h.msg_control = cbuf;
    h.msg_controllen = sizeof cbuf;
    const ssize_t r = recvmsg(sock_, &h, MSG_DONTWAIT | MSG_CMSG_CLOEXEC);
    if (r < 0) return any;
    any = true;
    Pending p;
    memset(&p, 0, sizeof p);
    p.fd[0] = p.fd[1] = -1;
    int nfd = 0;
    bool mine = false;  // sent by a process of this user (abstract sockets carry no permissions)
    for (cmsghdr* c = CMSG_FIRSTHDR(&h); c; c = CMSG_NXTHDR(&h, c)) {
      if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_CREDENTIALS) {
        ucred u;
        memcpy(&u, CMSG_DATA(c), sizeof u);
        mine = u.uid == getuid();
      }
      if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS) {
        const int k = (int)((c->cmsg_len - CMSG_LEN(0)) / sizeof(int));
        for (int i = 0; i < k; ++i) {
          int f = -1;
          memcpy(&f, CMSG_DATA(c) + (size_t)i * sizeof(int), sizeof f);
          if (nfd < 2) p.fd[nfd++] = f;
          else close(f);
        }
      }
    }
    if (!mine || r != (ssize_t)sizeof m || m.src < 0 || m.src >= nranks_ || m.nfd < 0 || m.nfd > 2) {
      for (int i = 0; i < nfd; ++i) close(p.fd[i]);
      continue;  // not ours
    }
    p.k = m.k;
    p.src = m.src;
    p.nfd = m.nfd < nfd ? m.nfd : nfd;  // a truncated message keeps only what arrived
    for (int i = p.nfd; i < nfd; ++i) close(p.fd[i]), p.fd[i] = -1;
    for (int i = 0; i < 2; ++i) p.base[i] = m.base[i], p.id[i] = m.id[i];
    pending_.push_back(p);
  }
}

void PeerBuffers::send_fds(int q, const FdMsg& m, const int* fds, const WaitFn& wait_for) {
  int rc = 0;
  // a peer's queue holds net.unix.max_dgram_qlen datagrams (10 by default) and every rank sends
  // before it takes: a full queue is waited out while taking my own arrivals
  wait_for([&] { return (rc = try_send(q, m, fds, m.nfd)) != 0 || (drain(), false); }, q, "take the descriptors of");
  if (rc > 0) return;
  // cannot pass the descriptors (e.g. the peer's descriptor table is full): the header alone, so
  // the peer's mapping fails and the call runs the ring on every rank
  FdMsg bare = m;
  bare.nfd = 0;
  wait_for([&] { return (rc = try_send(q, bare, nullptr, 0)) != 0 || (drain(), false); }, q, "take the descriptors of");
  if (rc < 0) throw std::runtime_error(std::string("read schedule: sending to rank ") + std::to_string(q) + ": " +
                                       strerror(errno));
}

PeerBuffers::Pending PeerBuffers::take_fds(int q, uint64_t k, const WaitFn& wait_for) {
  Pending out;
  memset(&out, 0, sizeof out);
  out.fd[0] = out.fd[1] = -1;
  bool found = false;
  auto look = [&] {
    for (size_t i = 0; i < pending_.size(); ++i) {
      if (pending_[i].k < k) {  // an abandoned call's (cannot happen in a live communicator)
        for (int j = 0; j < pending_[i].nfd; ++j) close(pending_[i].fd[j]);
        pending_.erase(pending_.begin() + (long)i--);
        continue;
      }
      if (pending_[i].src == q && pending_[i].k == k) {
        out = pending_[i];
        pending_.erase(pending_.begin() + (long)i);
        return found = true;
      }
    }
    return false;
  };
  wait_for([&] { return look() || (drain() && look()); }, q, "send the descriptors of");
  return out;
}

template <typename WaitFor>
PeerBuffers::Decision PeerBuffers::negotiate_body(uint64_t k, const void* send, const void* recv, bool eligible,
                                                  uint64_t count, int dtype, int op, int form,
                                                  const std::function<void()>& sync_previous, const char** psend,
                                                  const char** precv, bool* vec_all, const WaitFor& wait_for) {
  auto wait = [&](const std::atomic<uint64_t>& v, uint64_t want, int q, const char* what) {
    wait_for([&] { return v.load(std::memory_order_acquire) >= want; }, q, what);
  };
  const int slot = (int)(k % kBoardDepth);
  // my record slot is free once every peer has read the record kBoardDepth calls back
  if (k > (uint64_t)kBoardDepth)
    for (int q = 0; q < nranks_; ++q)
      if (q != rank_) wait(board_->consumed[q].v, k - kBoardDepth, q, "finish reading the records before");

  CallRec& me = board_->rec[rank_][slot];
  BufDesc sd, rd;
  memset(&sd, 0, sizeof sd);
  memset(&rd, 0, sizeof rd);
  bool ok = eligible && describe(send, &sd.base, &sd.id, &sd.d) && describe(recv, &rd.base, &rd.id, &rd.d);
  sd.raw = (uint64_t)(uintptr_t)send;
  rd.raw = (uint64_t)(uintptr_t)recv;
  sd.off = ok ? sd.raw - sd.base : 0;
  rd.off = ok ? rd.raw - rd.base : 0;
  me.count = count;
  me.dtype = dtype;
  me.op = op;
  me.form = form;
  me.fast = 0;
  me.sig = 0;
  me.eligible = ok ? 1 : 0;
  me.aligned = ((sd.raw | rd.raw) % 4 == 0) ? 1 : 0;
  me.send = sd;
  me.recv = rd;
  me.nfreed = 0;
  while (!freed_.empty() && me.nfreed < kMaxFreed) {
    me.freed[me.nfreed][0] = freed_.front().first;
    me.freed[me.nfreed][1] = freed_.front().second;
    ++me.nfreed;
    freed_.pop_front();
  }
  me.seq.store(k, std::memory_order_release);

  struct Seen {
    uint64_t count;
    int32_t dtype, op, eligible, aligned, fast, form;
    BufDesc send, recv;
    int32_t nfreed;
    uint64_t freed[kMaxFreed][2];
  };
  std::vector<Seen> recs((size_t)nranks_);
  for (int q = 0; q < nranks_; ++q) {
    const CallRec& c = board_->rec[q][slot];
    if (q != rank_) wait(c.seq, k, q, "reach");
    Seen& s = recs[(size_t)q];
    s.count = c.count;
    s.dtype = c.dtype;
    s.op = c.op;
    s.eligible = c.eligible;
    s.aligned = c.aligned;
    s.fast = c.fast;
    s.form = c.form;
    s.send = c.send;
    s.recv = c.recv;
    s.nfreed = c.nfreed < 0 ? 0 : c.nfreed > kMaxFreed ? kMaxFreed : c.nfreed;
    memcpy(s.freed, c.freed, sizeof s.freed);
  }
  board_->consumed[rank_].v.store(k, std::memory_order_release);  // my copies are taken
  // a peer launched this call on its registered windows without waiting for the records: it takes
  // for granted that every rank does, and this rank's buffers are not in them -- the caller broke
  // the windows' contract (Comm fails the call on every rank, the peer's kernel through its ABORT)
  for (const Seen& c : recs)
    if (c.fast) return kWindowPeer;

  // the peers' freed allocations: forget them (every rank alike) and close my imports of them.
  // The owner's call that used one last ended only after every peer's kernel was done with it
  // (read_kernel's DONE); my own last kernel is waited for all the same.
  bool synced = false;
  for (int q = 0; q < nranks_; ++q)
    for (int i = 0; i < recs[(size_t)q].nfreed; ++i) {
      const uint64_t fb = recs[(size_t)q].freed[i][0], fi = recs[(size_t)q].freed[i][1];
      known_.erase(Known{q, fb, fi});
      if (q == rank_ || nonces_[(size_t)q] == nonces_[(size_t)rank_]) continue;
      if (test_fake_) {
        for (size_t j = 0; j < fake_maps_.size(); ++j)
          if (fake_maps_[j] == Known{q, fb, fi}) {
            fake_maps_.erase(fake_maps_.begin() + (long)j);
            ++closed_freed_;
            break;
          }
        continue;
      }
      if (!ipc::find_import(nonces_[(size_t)q], fb, fi)) continue;
      if (!synced) {
        sync_previous();
        synced = true;
      }
      closed_freed_ += ipc::close_import(nonces_[(size_t)q], fb, fi) ? 1 : 0;
    }

  bool all = true, mismatch = false, aligned = true;
  for (const Seen& c : recs) {
    all = all && c.eligible;
    aligned = aligned && c.aligned;
    mismatch = mismatch || c.count != count || c.dtype != dtype || c.op != op || c.form != form;
  }
  const Decision d = mismatch ? kMismatch : all ? kRead : kFallback;
  *vec_all = aligned;
  if (d != kRead) return d;
  // Would any rank have to open a mapping?  A buffer some earlier read call ran on, and whose
  // owner has not reported it freed since, is still mapped by every rank (imports stay open), so
  // if every buffer of this call is one -- the common case of a caller reusing its buffers -- no
  // rank opens anything and no second round is needed.  Decided from the records alone: every
  // rank reaches the same answer.
  bool need_agree = false;
  for (int q = 0; q < nranks_ && !need_agree; ++q)
    need_agree = !known_.count(Known{q, recs[(size_t)q].send.base, recs[(size_t)q].send.id}) ||
                 !known_.count(Known{q, recs[(size_t)q].recv.base, recs[(size_t)q].recv.id});
  // The descriptors of the allocations new to this communicator travel first: every rank with a
  // new buffer sends one datagram with them to every rank of another process, and every rank
  // takes one from each such peer -- the same predicate on every rank, so nothing is left over.
  auto is_new = [&](int q, const BufDesc& b) { return !known_.count(Known{q, b.base, b.id}); };
  auto elsewhere = [&](int q) { return q != rank_ && nonces_[(size_t)q] != nonces_[(size_t)rank_]; };
  std::vector<Pending> got((size_t)nranks_);
  if (need_agree) {
    FdMsg m;
    memset(&m, 0, sizeof m);
    m.k = k;
    m.src = rank_;
    int fds[2] = {-1, -1};
    for (const BufDesc* b : {&recs[(size_t)rank_].send, &recs[(size_t)rank_].recv}) {
      if (!is_new(rank_, *b) || (m.nfd == 1 && m.base[0] == b->base && m.id[0] == b->id)) continue;
      m.base[m.nfd] = b->base;
      m.id[m.nfd] = b->id;
      fds[m.nfd++] = b->d.fd;
    }
    if (m.nfd)
      for (int q = 0; q < nranks_; ++q)
        if (elsewhere(q)) send_fds(q, m, fds, wait_for);
    for (int q = 0; q < nranks_; ++q)
      if (elsewhere(q) && (is_new(q, recs[(size_t)q].send) || is_new(q, recs[(size_t)q].recv)))
        got[(size_t)q] = take_fds(q, k, wait_for);
  }
  // the descriptor that arrived for (q, base, id), handed over (-1: none)
  auto fd_for = [&](int q, uint64_t base, uint64_t id) {
    Pending& g = got[(size_t)q];
    for (int i = 0; i < g.nfd; ++i)
      if (g.base[i] == base && g.id[i] == id && g.fd[i] >= 0) {
        const int f = g.fd[i];
        g.fd[i] = -1;
        return f;
      }
    return -1;
  };
  bool mapped = true;
  std::string why;
  for (int q = 0; q < nranks_; ++q) {
    const Seen& c = recs[(size_t)q];
    if (!elsewhere(q)) {
      psend[q] = (const char*)(uintptr_t)c.send.raw;  // this process's address space
      precv[q] = (const char*)(uintptr_t)c.recv.raw;
      continue;
    }
    const int fs = fd_for(q, c.send.base, c.send.id);
    const int fr = fd_for(q, c.recv.base, c.recv.id);  // -1 too when send and recv share an allocation
    const char* s = mapped ? map_peer(q, c.send.base, c.send.id, fs, c.send.d, &why) : nullptr;
    const char* r = s ? map_peer(q, c.recv.base, c.recv.id, fr, c.recv.d, &why) : nullptr;
    if (!s && fs >= 0 && !mapped) close(fs);  // map_peer consumes what it is given
    if (!s && fr >= 0) close(fr);
    if (!s || !r) {
      if (mapped) ++map_failures_;
      mapped = false;
      continue;  // every descriptor that arrived is still consumed
    }
    psend[q] = s + c.send.off;
    precv[q] = r + c.recv.off;
  }
  for (Pending& g : got)  // left over only after a failure
    for (int i = 0; i < g.nfd; ++i)
      if (g.fd[i] >= 0) close(g.fd[i]);
  if (!mapped && !need_agree)  // cannot happen (every buffer is mapped already); fail loudly if it does
    throw std::runtime_error("read schedule: a mapping of a known buffer is missing: " + why);
  Decision out = kRead;
  if (need_agree) {
    // second round: every rank's mapping outcome; one failure -> the ring for this
    // call on every rank (same bits, no buffer of a peer is read)
    ++agreements_;
    CallRec& mine = board_->rec[rank_][slot];
    mine.map_ok = mapped ? 1 : 0;
    mine.mapped.store(k, std::memory_order_release);
    int failed = -1;
    for (int q = 0; q < nranks_; ++q) {
      const CallRec& c = board_->rec[q][slot];
      if (q != rank_) wait(c.mapped, k, q, "report its mappings for");
      if (!c.map_ok && failed < 0) failed = q;
    }
    if (failed >= 0) {
      // a driver that cannot import the peers' memory fails every call alike: say so at the 1st,
      // 2nd, 4th, 8th ... fallback, not at every call
      ++fallbacks_;
      if ((fallbacks_ & (fallbacks_ - 1)) == 0)
        fprintf(stderr, "[Mini-NCCL] rank %d: all-reduce #%llu falls back to the ring (fallback %llu): rank "
                "%d could not map a peer's buffer%s%s\n", rank_, (unsigned long long)k,
                (unsigned long long)fallbacks_, failed, why.empty() ? "" : ": ", why.c_str());
      out = kFallback;
    }
  }
  if (out == kRead) {
    for (int q = 0; q < nranks_; ++q)
      for (const BufDesc* b : {&recs[(size_t)q].send, &recs[(size_t)q].recv})
        if (known_.insert(Known{q, b->base, b->id}).second) known_order_.push_back(Known{q, b->base, b->id});
    while (known_order_.size() > kMaxKnown) {  // forgetting only brings back a mapping round
      known_.erase(known_order_.front());
      known_order_.pop_front();
    }
  }
  return out;
}

}  // namespace mnccl
