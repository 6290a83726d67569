// Environment probe (not product code): can the read schedule share user buffers between rank
// processes through dma-buf file descriptors instead of hipIpc handles?
//
// Per round every process allocates a send and a recv buffer (the same size sequence in every
// process, so addresses coincide across processes and re-occur across rounds, as in the tests and
// in the reference's perf_test, which frees and re-allocates per size), writes a word that names
// (round, rank, buffer), exports each with hsa_amd_portable_export_dmabuf, and hands the fd to
// every peer; every peer imports it with hsa_amd_interop_map_buffer and loads the word with a
// kernel.  Imports are kept for KEEP rounds after their owner FREED the allocation, and re-checked
// every round: a dma-buf holds a reference on the memory, so an import must keep reading what it
// read when opened (or the owner's new data when the owner's new allocation is the same buffer
// object -- same dma-buf inode -- as HIP may re-use a freed block).
//
// mode 0: fds move by pidfd_getfd(pidfd_open(owner), owner's fd)   (owner keeps its fd until it frees)
// mode 1: fds move over abstract AF_UNIX datagram sockets (SCM_RIGHTS); the owner closes after sending
//
// Usage: probe_dmabuf <ranks> <rounds> <mode> [keep]   (spawns the ranks before any HIP call)
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <fcntl.h>
#include <sched.h>
#include <spawn.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

extern char** environ;

static std::atomic<int>* g_abort = nullptr;
#define CK(x)                                                                                                   \
  do {                                                                                                          \
    hipError_t e_ = (x);                                                                                        \
    if (e_ != hipSuccess) {                                                                                     \
      fprintf(stderr, "[pid %d] %s:%d %s -> %s\n", getpid(), __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      if (g_abort) g_abort->store(1);                                                                           \
      _exit(2);                                                                                                 \
    }                                                                                                           \
  } while (0)

namespace {

constexpr int kMaxR = 16;

struct Pub {
  int pid, fd, ok;
  uint64_t ino, off, bytes, base;
  unsigned value;
};
struct Stats {
  uint64_t exports, export_fails, getfd_fails, ino_mismatch, imports, map_fails, bad_fresh, bad_kept, kept_checks,
      same_bo_reuse, unmaps, unmap_fails, export_dup_fd_same_ino;
  double t_export, t_getfd, t_map, t_unmap;
  uint64_t max_map_bytes;
};
struct alignas(64) Shared {
  std::atomic<uint64_t> arrive;
  std::atomic<int> abort;
  Pub pub[kMaxR][2];
  Stats st[kMaxR];
  int first_err_printed;
};

__global__ void load_word(const unsigned* p, unsigned* out) { *out = __builtin_nontemporal_load(p); }

double now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

void barrier(Shared* s, int n, uint64_t k, const std::function<void()>& idle = nullptr) {
  s->arrive.fetch_add(1);
  for (int i = 0; s->arrive.load() < (uint64_t)n * k; ++i) {
    if (s->abort.load()) _exit(3);
    if (idle) idle();  // a rank still sending to me needs my queue drained
    if (i > 1000) sched_yield();
  }
}

size_t round_bytes(int r, int b) {
  static const size_t sizes[] = {16396, 4194304, 308, 32020, 16777252, 2560, 1048576, 493828, 2060, 8388608, 69632};
  return sizes[(size_t)(r * 2 + b) % (sizeof sizes / sizeof sizes[0])];
}

hsa_agent_t g_gpu{0};
hsa_status_t find_gpu(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle)
    g_gpu = a;
  return HSA_STATUS_SUCCESS;
}

void sock_name(sockaddr_un* a, socklen_t* len, int ppid, int rank) {
  memset(a, 0, sizeof *a);
  a->sun_family = AF_UNIX;
  int k = snprintf(a->sun_path + 1, sizeof a->sun_path - 1, "dmaprobe-%d-%d", ppid, rank);
  *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + k);
}

struct Msg {
  int src, b, round;
};

int child(const char* shm, int rank, int n, int rounds, int mode, int keep, int ppid) {
  int fd = shm_open(shm, O_RDWR, 0600);
  if (fd < 0) return 10;
  Shared* s = (Shared*)mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (s == MAP_FAILED) return 11;
  g_abort = &s->abort;
  Stats& st = s->st[rank];
  CK(hipSetDevice(0));
  if (hsa_init() != HSA_STATUS_SUCCESS) return 12;
  hsa_iterate_agents(find_gpu, nullptr);
  if (!g_gpu.handle) return 13;
  int sock = -1;
  if (mode == 1) {
    sock = socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0);
    sockaddr_un a;
    socklen_t len;
    sock_name(&a, &len, ppid, rank);
    if (sock < 0 || bind(sock, (sockaddr*)&a, len) != 0) {
      fprintf(stderr, "rank %d: bind: %s\n", rank, strerror(errno));
      return 14;
    }
  }
  std::vector<int> pidfd((size_t)n, -1);
  barrier(s, n, 1);  // every socket is bound, every pid published below is alive
  unsigned* dword = nullptr;
  CK(hipMalloc((void**)&dword, 4));
  struct Imp {
    int q, b, born;
    uint64_t ino;
    char* p;  // mapping base
    uint64_t off;
    unsigned want;
  };
  std::vector<Imp> imps;
  uint64_t bk = 1;
  auto load = [&](const char* p) {
    load_word<<<1, 1>>>((const unsigned*)p, dword);
    CK(hipGetLastError());
    unsigned v = 0;
    CK(hipMemcpy(&v, dword, 4, hipMemcpyDeviceToHost));
    return v;
  };
  int printed = 0;
  std::vector<std::pair<Msg, int>> stash;  // received (header, fd), this round's
  auto recv_one = [&](int flags) -> bool {
    Msg m{};
    iovec io{&m, sizeof m};
    char cbuf[CMSG_SPACE(sizeof(int))];
    msghdr h{};
    h.msg_iov = &io, h.msg_iovlen = 1, h.msg_control = cbuf, h.msg_controllen = sizeof cbuf;
    if (recvmsg(sock, &h, MSG_CMSG_CLOEXEC | flags) < 0) return false;
    cmsghdr* c = CMSG_FIRSTHDR(&h);
    int f = -1;
    if (c && c->cmsg_type == SCM_RIGHTS) memcpy(&f, CMSG_DATA(c), sizeof(int));
    stash.emplace_back(m, f);
    return true;
  };
  for (int r = 0; r < rounds; ++r) {
    char* mine[2];
    int myfd[2] = {-1, -1};
    for (int b = 0; b < 2; ++b) {
      const size_t bytes = round_bytes(r, b);
      CK(hipMalloc((void**)&mine[b], bytes));
      const unsigned v = (unsigned)(r * 64 + rank * 2 + b);
      CK(hipMemsetD32((hipDeviceptr_t)mine[b], v, 1));
      CK(hipDeviceSynchronize());
      Pub& d = s->pub[rank][b];
      d.ok = 0;
      int dfd = -1;
      uint64_t off = 0;
      const double t0 = now_us();
      hsa_status_t e = hsa_amd_portable_export_dmabuf(mine[b], bytes, &dfd, &off);
      st.t_export += now_us() - t0;
      ++st.exports;
      if (e != HSA_STATUS_SUCCESS) {
        if (st.export_fails++ < 2) fprintf(stderr, "rank %d round %d: export of %zu B failed: 0x%x\n", rank, r, bytes, e);
        continue;
      }
      struct stat sb;
      fstat(dfd, &sb);
      d.pid = getpid(), d.fd = dfd, d.ino = sb.st_ino, d.off = off, d.bytes = bytes, d.value = v;
      d.base = (uint64_t)(uintptr_t)mine[b];
      // a kept import of my own earlier allocation with the same inode: HIP handed back the same
      // buffer object; the peers' kept mappings then legitimately show the new word
      myfd[b] = dfd;
      d.ok = 1;
    }
    if (mode == 1) {
      for (int b = 0; b < 2; ++b) {
        if (!s->pub[rank][b].ok) continue;
        for (int k = 1; k < n; ++k) {
          const int q = (rank + k) % n;
          sockaddr_un a;
          socklen_t len;
          sock_name(&a, &len, ppid, q);
          Msg m{rank, b, r};
          iovec io{&m, sizeof m};
          char cbuf[CMSG_SPACE(sizeof(int))];
          memset(cbuf, 0, sizeof cbuf);
          msghdr h{};
          h.msg_name = &a, h.msg_namelen = len, h.msg_iov = &io, h.msg_iovlen = 1;
          h.msg_control = cbuf, h.msg_controllen = sizeof cbuf;
          cmsghdr* c = CMSG_FIRSTHDR(&h);
          c->cmsg_level = SOL_SOCKET, c->cmsg_type = SCM_RIGHTS, c->cmsg_len = CMSG_LEN(sizeof(int));
          memcpy(CMSG_DATA(c), &myfd[b], sizeof(int));
          // non-blocking: a peer's queue holds net.unix.max_dgram_qlen (10) datagrams, and every
          // rank sends before it receives -- on EAGAIN take what is waiting for me, then retry
          while (sendmsg(sock, &h, MSG_DONTWAIT) < 0) {
            if (errno != EAGAIN && errno != EWOULDBLOCK) {
              fprintf(stderr, "rank %d: sendmsg to %d: %s\n", rank, q, strerror(errno));
              s->abort.store(1);
              return 15;
            }
            while (recv_one(MSG_DONTWAIT)) {
            }
            if (s->abort.load()) return 16;
            sched_yield();
          }
        }
        close(myfd[b]);
        myfd[b] = -1;
      }
    }
    barrier(s, n, ++bk, [&] {
      if (mode == 1)
        while (recv_one(MSG_DONTWAIT)) {
        }
    });
    // collect the peers' fds
    int got[kMaxR][2];
    for (int q = 0; q < n; ++q) got[q][0] = got[q][1] = -1;
    const double tg = now_us();
    if (mode == 1) {
      int expect = 0;
      for (int q = 0; q < n; ++q)
        if (q != rank) expect += s->pub[q][0].ok + s->pub[q][1].ok;
      while ((int)stash.size() < expect && recv_one(0)) {
      }
      for (size_t i = 0; i < stash.size(); ++i) {
        const Msg m = stash[i].first;
        const int f = stash[i].second;
        if (m.round != r || f < 0) {
          ++st.getfd_fails;
          if (f >= 0) close(f);
          continue;
        }
        got[m.src][m.b] = f;
      }
      if ((int)stash.size() != expect) st.getfd_fails += (uint64_t)(expect - (int)stash.size());
      stash.clear();
    } else {
      for (int k = 1; k < n; ++k) {
        const int q = (rank + k) % n;
        for (int b = 0; b < 2; ++b) {
          const Pub d = s->pub[q][b];
          if (!d.ok) continue;
          if (pidfd[(size_t)q] < 0) pidfd[(size_t)q] = (int)syscall(SYS_pidfd_open, d.pid, 0);
          int f = pidfd[(size_t)q] < 0 ? -1 : (int)syscall(SYS_pidfd_getfd, pidfd[(size_t)q], d.fd, 0);
          if (f < 0) {
            if (st.getfd_fails++ < 2)
              fprintf(stderr, "rank %d: pidfd_%s(%d, fd %d): %s\n", rank, pidfd[(size_t)q] < 0 ? "open" : "getfd", d.pid,
                      d.fd, strerror(errno));
            continue;
          }
          got[q][b] = f;
        }
      }
    }
    st.t_getfd += now_us() - tg;
    // import, check fresh
    for (int k = 1; k < n; ++k) {
      const int q = (rank + k) % n;
      for (int b = 0; b < 2; ++b) {
        const Pub d = s->pub[q][b];
        const int f = got[q][b];
        if (!d.ok || f < 0) continue;
        struct stat sb;
        fstat(f, &sb);
        if ((uint64_t)sb.st_ino != d.ino) ++st.ino_mismatch;
        // a kept import of the same buffer object: its word is the owner's new one now
        for (Imp& m : imps)
          if (m.q == q && m.ino == (uint64_t)sb.st_ino) {
            ++st.same_bo_reuse;
            m.want = d.value;
            m.off = d.off;
          }
        size_t sz = 0;
        void* p = nullptr;
        hsa_handle_t hh = (hsa_handle_t)f;
        const double t0 = now_us();
        hsa_status_t e = hsa_amd_interop_map_buffer(1, &g_gpu, hh, 0, &sz, &p, nullptr, nullptr);
        st.t_map += now_us() - t0;
        ++st.imports;
        close(f);
        if (e != HSA_STATUS_SUCCESS) {
          if (st.map_fails++ < 3)
            fprintf(stderr, "rank %d round %d: interop map of rank %d's %s (%llu B, off %llu) failed: 0x%x\n", rank, r, q,
                    b ? "recv" : "send", (unsigned long long)d.bytes, (unsigned long long)d.off, e);
          continue;
        }
        if (sz > st.max_map_bytes) st.max_map_bytes = sz;
        const unsigned v = load((char*)p + d.off);
        if (v != d.value && printed++ < 4)
          fprintf(stderr, "rank %d round %d: fresh import of rank %d's %s read %u (round %u rank %u buf %u) want %u\n", rank,
                  r, q, b ? "recv" : "send", v, v / 64, (v % 64) / 2, v % 2, d.value);
        st.bad_fresh += v != d.value;
        imps.push_back(Imp{q, b, r, (uint64_t)sb.st_ino, (char*)p, d.off, d.value});
      }
    }
    // kept imports of allocations their owners freed in earlier rounds still read what they read (or the
    // same object's new word); expired ones are unmapped while other processes are still importing
    for (size_t i = 0; i < imps.size();) {
      const unsigned v = load(imps[i].p + imps[i].off);
      ++st.kept_checks;
      if (v != imps[i].want) {
        if (printed++ < 8)
          fprintf(stderr, "rank %d round %d: kept import (round %d, rank %d's %s) read %u (round %u rank %u buf %u) want %u\n",
                  rank, r, imps[i].born, imps[i].q, imps[i].b ? "recv" : "send", v, v / 64, (v % 64) / 2, v % 2,
                  imps[i].want);
        ++st.bad_kept;
      }
      if (r - imps[i].born >= keep) {
        const double t0 = now_us();
        if (hsa_amd_interop_unmap_buffer(imps[i].p) != HSA_STATUS_SUCCESS) ++st.unmap_fails;
        st.t_unmap += now_us() - t0;
        ++st.unmaps;
        imps.erase(imps.begin() + (long)i);
      } else {
        ++i;
      }
    }
    barrier(s, n, ++bk);
    // owners free while every peer still maps their buffers
    for (int b = 0; b < 2; ++b) {
      CK(hipFree(mine[b]));
      if (myfd[b] >= 0) close(myfd[b]);
    }
    CK(hipDeviceSynchronize());
    barrier(s, n, ++bk);
    barrier(s, n, ++bk);
  }
  for (Imp& m : imps) hsa_amd_interop_unmap_buffer(m.p);
  CK(hipFree(dword));
  hsa_shut_down();
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 8 && !strcmp(argv[1], "child"))
    return child(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]), atoi(argv[8]));
  if (argc < 4) {
    fprintf(stderr, "usage: %s <ranks> <rounds> <mode 0=pidfd 1=scm> [keep]\n", argv[0]);
    return 1;
  }
  const int n = atoi(argv[1]), rounds = atoi(argv[2]), mode = atoi(argv[3]);
  const int keep = argc > 4 ? atoi(argv[4]) : 3;
  if (n < 2 || n > kMaxR) return 1;
  char name[64];
  snprintf(name, sizeof name, "/dmaprobe-%d", (int)getpid());
  int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, sizeof(Shared)) != 0) return 2;
  Shared* s = (Shared*)mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  memset((void*)s, 0, sizeof(Shared));
  std::vector<pid_t> pids;
  const double t0 = now_us();
  for (int r = 0; r < n; ++r) {
    char a[6][16];
    snprintf(a[0], 16, "%d", r);
    snprintf(a[1], 16, "%d", n);
    snprintf(a[2], 16, "%d", rounds);
    snprintf(a[3], 16, "%d", mode);
    snprintf(a[4], 16, "%d", keep);
    snprintf(a[5], 16, "%d", (int)getpid());
    char* cargv[] = {argv[0], (char*)"child", name, a[0], a[1], a[2], a[3], a[4], a[5], nullptr};
    pid_t pid;
    if (posix_spawn(&pid, argv[0], nullptr, nullptr, cargv, environ)) return 3;
    pids.push_back(pid);
  }
  int bad_exit = 0;
  for (pid_t p : pids) {
    int stt = 0;
    waitpid(p, &stt, 0);
    if (!WIFEXITED(stt) || WEXITSTATUS(stt)) {
      ++bad_exit;
      fprintf(stderr, "child %d: status 0x%x\n", (int)p, stt);
    }
  }
  shm_unlink(name);
  Stats t;
  memset(&t, 0, sizeof t);
  for (int r = 0; r < n; ++r) {
    const Stats& x = s->st[r];
    t.exports += x.exports, t.export_fails += x.export_fails, t.getfd_fails += x.getfd_fails;
    t.ino_mismatch += x.ino_mismatch, t.imports += x.imports, t.map_fails += x.map_fails, t.bad_fresh += x.bad_fresh;
    t.bad_kept += x.bad_kept, t.kept_checks += x.kept_checks, t.same_bo_reuse += x.same_bo_reuse;
    t.unmaps += x.unmaps, t.unmap_fails += x.unmap_fails;
    t.t_export += x.t_export, t.t_getfd += x.t_getfd, t.t_map += x.t_map, t.t_unmap += x.t_unmap;
    if (x.max_map_bytes > t.max_map_bytes) t.max_map_bytes = x.max_map_bytes;
  }
  printf("dmabuf mode %s ranks %d rounds %d keep %d: %.1f s, bad exits %d\n", mode ? "scm" : "pidfd", n, rounds, keep,
         (now_us() - t0) * 1e-6, bad_exit);
  printf("  exports %llu (failed %llu, mean %.1f us), fd transfers failed %llu, inode mismatches %llu\n",
         (unsigned long long)t.exports, (unsigned long long)t.export_fails, t.t_export / (double)(t.exports ? t.exports : 1),
         (unsigned long long)t.getfd_fails, (unsigned long long)t.ino_mismatch);
  printf("  imports %llu (map failed %llu, mean %.1f us; largest mapping %llu B), fresh wrong values %llu\n",
         (unsigned long long)t.imports, (unsigned long long)t.map_fails, t.t_map / (double)(t.imports ? t.imports : 1),
         (unsigned long long)t.max_map_bytes, (unsigned long long)t.bad_fresh);
  printf("  kept-import checks after the owner freed %llu: wrong values %llu; same buffer object handed back by HIP %llu; "
         "unmaps %llu (failed %llu, mean %.1f us)\n",
         (unsigned long long)t.kept_checks, (unsigned long long)t.bad_kept, (unsigned long long)t.same_bo_reuse,
         (unsigned long long)t.unmaps, (unsigned long long)t.unmap_fails, t.t_unmap / (double)(t.unmaps ? t.unmaps : 1));
  munmap(s, sizeof(Shared));
  return bad_exit ? 4 : 0;
}
