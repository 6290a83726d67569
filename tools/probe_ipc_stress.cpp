// Environment probe (not product code): the read schedule's IPC pattern with N rank processes
// on one GPU, as the 8-rank GPU tests run it -- every process allocates a send and a recv buffer
// per round (the same size sequence on every rank, so addresses coincide across processes, as
// they do in the tests), exports them, opens every peer's, reads 4 bytes through each mapping,
// then frees its own.  Open failures are counted with what surrounded them.
//
// Policy = sum of flags (0 = the library's round-2 behaviour: cache by (rank, base, id), at most
// K open, least recently used closed AFTER the new open; owners free while peers still hold
// their imports):
//   1 stale   a mapping of the same (rank, base) with an older id -- a freed allocation whose
//             address came back -- is closed before the new one is opened
//   2 percall every import closed at the end of its round, before the owner frees (the
//             reference's per-call lifecycle, RDMATransport.h:231-255)
//   4 serial  every open / close in every process serialised by one lock
//   8 nofree  owners never free (no import ever outlives its allocation)
//  16 big     every buffer >= 4 MiB (no sub-allocated fragments)
//  32 fresh   an owner never exports an address it exported before for another allocation
//             (such a buffer is skipped, as a call on it would fall back to the scratch schedule)
//
// Usage: probe_ipc_stress <ranks> <rounds> <policy> [K]   (spawns the ranks before any HIP call)
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sched.h>
#include <spawn.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern char** environ;

static std::atomic<int>* g_abort = nullptr;  // shared: a rank that fails stops every rank
#define CK(x)                                                                                               \
  do {                                                                                                      \
    hipError_t e_ = (x);                                                                                    \
    if (e_ != hipSuccess) {                                                                                 \
      fprintf(stderr, "[rank pid %d] %s:%d %s -> %s\n", getpid(), __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      if (g_abort) g_abort->store(1);                                                                       \
      _exit(2);                                                                                             \
    }                                                                                                       \
  } while (0)

namespace {

constexpr int kMaxR = 16;
enum State { kIdle = 0, kOpening, kClosing, kFreeing, kAllocating, kReading };
const char* state_name[] = {"idle", "opening", "closing", "freeing", "allocating", "reading"};

struct Buf {
  uint64_t base, id, off, size;
  hipIpcMemHandle_t h;
};
struct Stats {
  uint64_t opens, fails, fails_final, closes, stale_closes, bad_reads;
  uint64_t fail_peer_state[6];   // what the owner was doing when the open failed
  uint64_t fail_other_closing;   // some process (not the owner) was closing at that moment
  uint64_t fail_own_live;        // this process had a live range at the owner's base address
  uint64_t fail_stale_same_base; // this process still mapped an older allocation of (owner, base)
  uint64_t fail_same_block;      // ... or another allocation of the owner's 2 MiB block
  uint64_t fail_fragment;        // the handle describes a sub-allocated fragment
  uint64_t fail_after_close_us;  // sum of the time since this process's last close (us)
  uint64_t fail_retry_ok;        // the open succeeded on a retry
  uint64_t export_fails;         // hipIpcGetMemHandle failed (the buffer is skipped by the peers)
  uint64_t bad_kernel;           // wrong value loaded by a kernel through the mapping (what the library does)
  uint64_t bad_old_round;        // ... a value some earlier round wrote (a stale allocation's contents)
  uint64_t bad_fresh;            // ... through a mapping opened in this round
  uint64_t dup_handles;          // an owner's handle repeats bytes of one of its earlier handles
  uint64_t reused_va_exports;    // exports of an address this owner exported before (another allocation)
  uint64_t export_fails_reused;  // export failures on such an address
  uint64_t bad_reused_va;        // wrong values through a mapping of such an address
  uint64_t fails_reused_va;      // open failures of such an address
  uint64_t skipped_reused;       // policy 32: buffers not exported for that reason
};
struct Buf2 {
  uint32_t reused;  // the owner had exported this address before (for another allocation)
};
struct alignas(64) Shared {
  std::atomic<uint64_t> arrive;
  std::atomic<int> abort;
  std::atomic<int> lock;
  std::atomic<int> state[kMaxR];
  Buf buf[kMaxR][2];
  Buf2 buf2[kMaxR][2];
  Stats st[kMaxR];
};

__global__ void load_word(const unsigned* p, unsigned* out) { *out = __builtin_nontemporal_load(p); }

double now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

void barrier(Shared* s, int n, uint64_t k) {
  s->arrive.fetch_add(1);
  for (int i = 0; s->arrive.load() < (uint64_t)n * k; ++i) {
    if (s->abort.load()) _exit(3);
    if (i > 1000) sched_yield();
  }
}

size_t round_bytes(int policy, int r, int b) {
  static const size_t sizes[] = {16396, 4194304, 308, 32020, 16777252, 2560, 1048576, 493828, 2060, 8388608, 69632};
  size_t s = sizes[(size_t)(r * 2 + b) % (sizeof sizes / sizeof sizes[0])];
  if ((policy & 16) && s < ((size_t)4 << 20)) s = ((size_t)4 << 20) + s;
  return s;
}

int child(const char* shm, int rank, int n, int rounds, int policy, int K) {
  int fd = shm_open(shm, O_RDWR, 0600);
  if (fd < 0) return 10;
  Shared* s = (Shared*)mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (s == MAP_FAILED) return 11;
  g_abort = &s->abort;
  CK(hipSetDevice(0));
  Stats& st = s->st[rank];
  struct Map {
    int q;
    uint64_t base, id, size;
    char* p;
    int last;
  };
  std::vector<Map> maps;
  std::vector<char*> kept;
  std::vector<std::vector<hipIpcMemHandle_t>> seen((size_t)n);
  std::vector<uint64_t> exported;  // addresses this process exported
  unsigned* dword = nullptr;
  CK(hipMalloc((void**)&dword, 4));
  int printed_bad = 0;
  double last_close = 0;
  int printed = 0;
  uint64_t bk = 0;
  auto lock = [&] {
    if (!(policy & 4)) return;
    int z = 0;
    while (!s->lock.compare_exchange_weak(z, 1)) z = 0, sched_yield();
  };
  auto unlock = [&] {
    if (policy & 4) s->lock.store(0);
  };
  auto close_map = [&](size_t i) {
    lock();
    s->state[rank].store(kClosing);
    CK(hipIpcCloseMemHandle(maps[i].p));
    s->state[rank].store(kIdle);
    unlock();
    last_close = now_us();
    ++st.closes;
    maps.erase(maps.begin() + (long)i);
  };
  for (int r = 0; r < rounds; ++r) {
    char* mine[2];
    s->state[rank].store(kAllocating);
    for (int b = 0; b < 2; ++b) {
      const size_t bytes = round_bytes(policy, r, b);
      CK(hipMalloc((void**)&mine[b], bytes));
      CK(hipMemsetD32((hipDeviceptr_t)mine[b], (unsigned)(r * 64 + rank * 2 + b), 1));
      hipDeviceptr_t base = 0;
      size_t sz = 0;
      Buf& d = s->buf[rank][b];
      CK(hipMemGetAddressRange(&base, &sz, (hipDeviceptr_t)mine[b]));
      unsigned long long id = 0;
      CK(hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)mine[b]));
      d.id = 0;
      int prior = 0;
      for (uint64_t a : exported) prior += a == (uint64_t)(uintptr_t)base;
      s->buf2[rank][b].reused = prior > 0;
      if (prior && (policy & 32)) {
        ++st.skipped_reused;
        d.base = 0;
        continue;
      }
      st.reused_va_exports += prior > 0;
      if (hipIpcGetMemHandle(&d.h, (void*)base) != hipSuccess) {
        (void)hipGetLastError();
        st.export_fails_reused += prior > 0;
        exported.push_back((uint64_t)(uintptr_t)base);  // a failed export counts as one (policy 32)
        if (st.export_fails++ < 2)
          fprintf(stderr, "rank %d round %d: export of its %s (ptr %p, base 0x%llx, %zu B) failed; address exported %d "
                  "times before\n", rank, r, b ? "recv" : "send", (void*)mine[b], (unsigned long long)(uintptr_t)base,
                  sz, prior);
        d.base = 0;
        continue;
      }
      exported.push_back((uint64_t)(uintptr_t)base);
      d.base = (uint64_t)(uintptr_t)base;
      d.id = id;
      d.size = sz;
      d.off = (uint64_t)(mine[b] - (char*)base);
    }
    CK(hipDeviceSynchronize());
    s->state[rank].store(kIdle);
    barrier(s, n, ++bk);
    for (int k = 1; k < n; ++k) {
      const int q = (rank + k) % n;
      for (int b = 0; b < 2; ++b) {
        const Buf d = s->buf[q][b];
        if (!d.base) continue;  // the owner could not export it
        char* p = nullptr;
        for (Map& m : maps)
          if (m.q == q && m.base == d.base && m.id == d.id) p = m.p, m.last = r;
        const bool fresh = !p;
        if (!p) {
          for (const hipIpcMemHandle_t& o : seen[(size_t)q])
            if (!memcmp(&o, &d.h, sizeof o)) {
              ++st.dup_handles;
              break;
            }
          seen[(size_t)q].push_back(d.h);
          if (policy & 1)
            for (size_t i = 0; i < maps.size();) {
              if (maps[i].q == q && maps[i].base == d.base) {
                close_map(i);
                ++st.stale_closes;
              } else {
                ++i;
              }
            }
          const uint32_t w6 = ((const uint32_t*)d.h.reserved)[6];
          lock();
          s->state[rank].store(kOpening);
          void* v = nullptr;
          hipError_t e = hipIpcOpenMemHandle(&v, d.h, hipIpcMemLazyEnablePeerAccess);
          s->state[rank].store(kIdle);
          unlock();
          ++st.opens;
          if (e != hipSuccess) {
            (void)hipGetLastError();
            ++st.fails;
            st.fails_reused_va += s->buf2[q][b].reused;
            const int ps = s->state[q].load();
            ++st.fail_peer_state[ps];
            bool other_closing = false;
            for (int x = 0; x < n; ++x)
              if (x != q && x != rank && s->state[x].load() == kClosing) other_closing = true;
            st.fail_other_closing += other_closing;
            hipDeviceptr_t ob = 0;
            size_t osz = 0;
            const bool own_live = hipMemGetAddressRange(&ob, &osz, (hipDeviceptr_t)d.base) == hipSuccess;
            (void)hipGetLastError();
            st.fail_own_live += own_live;
            const uint64_t frag_off = (w6 & 0x80000000u) ? (uint64_t)(w6 & 0x1ffu) * 4096 : 0;
            int stale = 0, block = 0;
            for (const Map& m : maps) {
              if (m.q != q) continue;
              if (m.base == d.base) ++stale;
              if ((m.base & ~(uint64_t)0x1fffff) == ((d.base - frag_off) & ~(uint64_t)0x1fffff)) ++block;
            }
            st.fail_stale_same_base += stale > 0;
            st.fail_same_block += block > 0;
            st.fail_fragment += (w6 & 0x80000000u) ? 1 : 0;
            const double since = now_us() - last_close;
            st.fail_after_close_us += last_close > 0 ? (uint64_t)since : 0;
            if (printed++ < 4)
              fprintf(stderr,
                      "rank %d round %d: open of rank %d's %s (base 0x%llx, id %llu, %llu B, frag %s) failed: %s; "
                      "owner %s, other closing %d, own live range at that address %d (0x%llx + %zu), "
                      "older mapping of (owner, base) %d, of its block %d, maps %zu, %.0f us since my last close\n",
                      rank, r, q, b ? "recv" : "send", (unsigned long long)d.base, (unsigned long long)d.id,
                      (unsigned long long)d.size, (w6 & 0x80000000u) ? "yes" : "no", hipGetErrorString(e),
                      state_name[ps], (int)other_closing, (int)own_live, (unsigned long long)(uintptr_t)ob, osz, stale,
                      block, maps.size(), since);
            for (int a = 1; a <= 3 && e != hipSuccess; ++a) {
              usleep(1000u << a);
              e = hipIpcOpenMemHandle(&v, d.h, hipIpcMemLazyEnablePeerAccess);
              (void)hipGetLastError();
            }
            if (e != hipSuccess) {
              ++st.fails_final;
              continue;
            }
            ++st.fail_retry_ok;
          }
          maps.push_back(Map{q, d.base, d.id, d.size, (char*)v, r});
          p = (char*)v;
          if (!(policy & 2) && (int)maps.size() > K) {
            size_t lru = 0;
            for (size_t i = 1; i < maps.size(); ++i)
              if (maps[i].last < maps[lru].last) lru = i;
            close_map(lru);
          }
        }
        s->state[rank].store(kReading);
        unsigned v = 0, kv = 0;
        CK(hipMemcpy(&v, p + d.off, 4, hipMemcpyDeviceToHost));
        load_word<<<1, 1>>>((const unsigned*)(p + d.off), dword);
        CK(hipGetLastError());
        CK(hipMemcpy(&kv, dword, 4, hipMemcpyDeviceToHost));
        s->state[rank].store(kIdle);
        const unsigned want = (unsigned)(r * 64 + q * 2 + b);
        if (v != want) ++st.bad_reads;
        if (kv != want) {
          ++st.bad_kernel;
          st.bad_reused_va += s->buf2[q][b].reused;
          const bool old = kv % 64 == (unsigned)(q * 2 + b) && kv / 64 < (unsigned)r;
          st.bad_old_round += old;
          st.bad_fresh += fresh;
          if (printed_bad++ < 3)
            fprintf(stderr, "rank %d round %d: kernel load through the mapping of rank %d's %s (base 0x%llx, id %llu, "
                    "%llu B, %s mapping) read %u (round %u rank %u buf %u), want %u; hipMemcpy read %u\n",
                    rank, r, q, b ? "recv" : "send", (unsigned long long)d.base, (unsigned long long)d.id,
                    (unsigned long long)d.size, fresh ? "new" : "cached", kv, kv / 64, (kv % 64) / 2, kv % 2, want, v);
        }
      }
    }
    if (policy & 2)
      while (!maps.empty()) close_map(maps.size() - 1);
    barrier(s, n, ++bk);
    s->state[rank].store(kFreeing);
    for (int b = 0; b < 2; ++b) {
      if (policy & 8) kept.push_back(mine[b]);
      else CK(hipFree(mine[b]));
    }
    s->state[rank].store(kIdle);
  }
  while (!maps.empty()) close_map(maps.size() - 1);
  barrier(s, n, ++bk);
  for (char* p : kept) CK(hipFree(p));
  CK(hipFree(dword));
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 7 && !strcmp(argv[1], "child"))
    return child(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]));
  if (argc < 4) {
    fprintf(stderr, "usage: %s <ranks> <rounds> <policy> [K]\n", argv[0]);
    return 1;
  }
  const int n = atoi(argv[1]), rounds = atoi(argv[2]), policy = atoi(argv[3]);
  const int K = argc > 4 ? atoi(argv[4]) : 64;
  if (n < 2 || n > kMaxR) return 1;
  char name[64];
  snprintf(name, sizeof name, "/ipcstress-%d", (int)getpid());
  int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, sizeof(Shared)) != 0) return 2;
  Shared* s = (Shared*)mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  memset((void*)s, 0, sizeof(Shared));
  std::vector<pid_t> pids;
  const double t0 = now_us();
  for (int r = 0; r < n; ++r) {
    char a[5][16];
    snprintf(a[0], 16, "%d", r);
    snprintf(a[1], 16, "%d", n);
    snprintf(a[2], 16, "%d", rounds);
    snprintf(a[3], 16, "%d", policy);
    snprintf(a[4], 16, "%d", K);
    char* cargv[] = {argv[0], (char*)"child", name, a[0], a[1], a[2], a[3], a[4], nullptr};
    pid_t pid;
    if (posix_spawn(&pid, argv[0], nullptr, nullptr, cargv, environ)) return 3;
    pids.push_back(pid);
  }
  int bad_exit = 0;
  for (pid_t p : pids) {
    int stt = 0;
    waitpid(p, &stt, 0);
    if (!WIFEXITED(stt) || WEXITSTATUS(stt)) ++bad_exit;
  }
  shm_unlink(name);
  Stats t;
  memset(&t, 0, sizeof t);
  for (int r = 0; r < n; ++r) {
    const Stats& x = s->st[r];
    t.opens += x.opens, t.fails += x.fails, t.fails_final += x.fails_final, t.closes += x.closes;
    t.stale_closes += x.stale_closes, t.bad_reads += x.bad_reads, t.fail_other_closing += x.fail_other_closing;
    t.fail_own_live += x.fail_own_live, t.fail_stale_same_base += x.fail_stale_same_base;
    t.fail_same_block += x.fail_same_block, t.fail_fragment += x.fail_fragment;
    t.fail_after_close_us += x.fail_after_close_us, t.fail_retry_ok += x.fail_retry_ok;
    t.export_fails += x.export_fails;
    t.bad_kernel += x.bad_kernel, t.bad_old_round += x.bad_old_round, t.bad_fresh += x.bad_fresh;
    t.dup_handles += x.dup_handles;
    t.reused_va_exports += x.reused_va_exports, t.export_fails_reused += x.export_fails_reused;
    t.bad_reused_va += x.bad_reused_va, t.fails_reused_va += x.fails_reused_va, t.skipped_reused += x.skipped_reused;
    for (int i = 0; i < 6; ++i) t.fail_peer_state[i] += x.fail_peer_state[i];
  }
  char pn[96];
  snprintf(pn, sizeof pn, "%s%s%s%s%s%s", policy ? "" : "lru", (policy & 1) ? "+stale" : "", (policy & 2) ? "+percall" : "",
           (policy & 4) ? "+serial" : "", (policy & 8) ? "+nofree" : "", (policy & 16) ? "+big" : "");
  printf("policy %s ranks %d rounds %d K %d: %.1f s, opens %llu, FAILED %llu (retry ok %llu, final %llu), closes %llu "
         "(stale-first %llu), bad reads %llu, export failures %llu, bad exits %d\n",
         pn, n, rounds, K, (now_us() - t0) * 1e-6, (unsigned long long)t.opens, (unsigned long long)t.fails,
         (unsigned long long)t.fail_retry_ok, (unsigned long long)t.fails_final, (unsigned long long)t.closes,
         (unsigned long long)t.stale_closes, (unsigned long long)t.bad_reads, (unsigned long long)t.export_fails,
         bad_exit);
  printf("  wrong values loaded by a kernel %llu (an earlier round's value %llu, through a new mapping %llu); "
         "handles repeating an earlier handle's bytes %llu\n",
         (unsigned long long)t.bad_kernel, (unsigned long long)t.bad_old_round, (unsigned long long)t.bad_fresh,
         (unsigned long long)t.dup_handles);
  printf("  exports of a re-used address %llu (failed %llu; skipped by policy %llu); on such addresses: open failures "
         "%llu, wrong values %llu\n", (unsigned long long)t.reused_va_exports, (unsigned long long)t.export_fails_reused,
         (unsigned long long)t.skipped_reused, (unsigned long long)t.fails_reused_va, (unsigned long long)t.bad_reused_va);
  if (t.fails)
    printf("  failures: owner idle/opening/closing/freeing/allocating/reading %llu/%llu/%llu/%llu/%llu/%llu, another "
           "rank closing %llu, own live range at the address %llu, older mapping of (owner, base) %llu, of its block "
           "%llu, fragment %llu, mean %.0f us since the importer's last close\n",
           (unsigned long long)t.fail_peer_state[0], (unsigned long long)t.fail_peer_state[1],
           (unsigned long long)t.fail_peer_state[2], (unsigned long long)t.fail_peer_state[3],
           (unsigned long long)t.fail_peer_state[4], (unsigned long long)t.fail_peer_state[5],
           (unsigned long long)t.fail_other_closing, (unsigned long long)t.fail_own_live,
           (unsigned long long)t.fail_stale_same_base, (unsigned long long)t.fail_same_block,
           (unsigned long long)t.fail_fragment, (double)t.fail_after_close_us / (double)t.fails);
  munmap(s, sizeof(Shared));
  return bad_exit ? 4 : 0;
}
