// Environment probe (not product code): the read schedule's IPC pattern under allocation churn.
// The exporter allocates a send and a recv buffer per "call" (sizes like the GPU tests'), exports
// their handles (allocation base, as PeerBuffers::describe does), hands them to the importer,
// waits for its ack, frees both; the importer keeps at most K open mappings (least recently
// used closed first, as PeerBuffers::map_peer does), opens every new handle and checks the value
// the exporter wrote.  Reports: handles whose bytes repeat an earlier handle's, open failures
// (and whether they follow a close), stale reads.
// Usage: probe_ipc_churn <calls> <K> <min_kib> <max_kib>   (spawns itself as the importer)
#include <hip/hip_runtime.h>

#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern char** environ;

#define CK(x)                                                                                          \
  do {                                                                                                 \
    hipError_t e_ = (x);                                                                               \
    if (e_ != hipSuccess) {                                                                            \
      fprintf(stderr, "[pid %d] %s:%d %s -> %s\n", getpid(), __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                                         \
    }                                                                                                  \
  } while (0)

struct Msg {
  int call;
  unsigned long long id[2];
  size_t off[2];
  hipIpcMemHandle_t h[2];
};

static int importer(int K) {
  CK(hipSetDevice(0));
  struct Map {
    unsigned long long id;
    char* p;
    int last;
    hipIpcMemHandle_t h;
  };
  std::vector<Map> maps;
  std::vector<hipIpcMemHandle_t> seen;
  int fails = 0, stale = 0, closes = 0, fails_after_close = 0, repeats = 0;
  bool closed_this_call = false;
  Msg m;
  while (fread(&m, sizeof m, 1, stdin) == 1) {
    closed_this_call = false;
    char* p[2] = {nullptr, nullptr};
    for (int b = 0; b < 2; ++b) {
      for (auto& mp : maps)
        if (mp.id == m.id[b]) { p[b] = mp.p; mp.last = m.call; }
      if (p[b]) continue;
      for (auto& s : seen)
        if (!memcmp(&s, &m.h[b], sizeof s)) { ++repeats; break; }
      seen.push_back(m.h[b]);
      if ((int)maps.size() >= K) {
        size_t lru = 0;
        for (size_t i = 1; i < maps.size(); ++i)
          if (maps[i].last < maps[lru].last) lru = i;
        CK(hipIpcCloseMemHandle(maps[lru].p));
        maps.erase(maps.begin() + (long)lru);
        ++closes;
        closed_this_call = true;
      }
      void* q = nullptr;
      hipError_t e = hipIpcOpenMemHandle(&q, m.h[b], hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) {
        ++fails;
        if (closed_this_call) ++fails_after_close;
        if (fails <= 10)
          printf("importer: call %d buffer %d open failed: %s (after a close this call: %d, maps %zu)\n", m.call, b,
                 hipGetErrorString(e), closed_this_call, maps.size());
        (void)hipGetLastError();
        continue;
      }
      maps.push_back(Map{m.id[b], (char*)q, m.call, m.h[b]});
      p[b] = (char*)q;
    }
    if (p[0]) {
      int v = -1;
      CK(hipMemcpy(&v, p[0] + m.off[0], sizeof v, hipMemcpyDeviceToHost));
      if (v != m.call) {
        ++stale;
        if (stale <= 10) printf("importer: call %d read %d (stale)\n", m.call, v);
      }
    }
    char ack = 1;
    if (write(1, &ack, 1) != 1) return 3;
  }
  for (auto& mp : maps) (void)hipIpcCloseMemHandle(mp.p);
  fprintf(stderr, "importer: K=%d opens failed %d (%d right after a close), stale reads %d, closes %d, handle repeats %d\n",
          K, fails, fails_after_close, stale, closes, repeats);
  return fails || stale ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && !strcmp(argv[1], "import")) return importer(atoi(argv[2]));
  const int calls = argc > 1 ? atoi(argv[1]) : 200;
  const char* K = argc > 2 ? argv[2] : "64";
  const int lo = argc > 3 ? atoi(argv[3]) : 100, hi = argc > 4 ? atoi(argv[4]) : 400;
  int to_child[2], from_child[2];
  if (pipe(to_child) || pipe(from_child)) return 4;
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, to_child[0], 0);
  posix_spawn_file_actions_adddup2(&fa, from_child[1], 1);
  posix_spawn_file_actions_addclose(&fa, to_child[1]);
  posix_spawn_file_actions_addclose(&fa, from_child[0]);
  pid_t pid;
  char* cargv[] = {argv[0], (char*)"import", (char*)K, nullptr};
  if (posix_spawn(&pid, argv[0], &fa, nullptr, cargv, environ)) return 5;  // before any HIP call
  close(to_child[0]);
  close(from_child[1]);
  CK(hipSetDevice(0));
  std::vector<hipIpcMemHandle_t> seen;
  int repeats = 0;
  for (int c = 0; c < calls; ++c) {
    const size_t kib = (size_t)lo + (size_t)(c * 7919) % (size_t)(hi - lo + 1);
    char* buf[2];
    Msg m;
    memset(&m, 0, sizeof m);
    m.call = c;
    for (int b = 0; b < 2; ++b) {
      CK(hipMalloc((void**)&buf[b], kib << 10));
      hipDeviceptr_t base = 0;
      size_t sz = 0;
      CK(hipMemGetAddressRange(&base, &sz, (hipDeviceptr_t)buf[b]));
      CK(hipPointerGetAttribute(&m.id[b], HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)buf[b]));
      CK(hipIpcGetMemHandle(&m.h[b], (void*)base));
      m.off[b] = (size_t)(buf[b] - (char*)base);
      for (auto& s : seen)
        if (!memcmp(&s, &m.h[b], sizeof s)) { ++repeats; break; }
      seen.push_back(m.h[b]);
    }
    CK(hipMemcpy(buf[0], &c, sizeof c, hipMemcpyHostToDevice));
    if (write(to_child[1], &m, sizeof m) != (ssize_t)sizeof m) return 6;
    char ack;
    if (read(from_child[0], &ack, 1) != 1) return 7;
    CK(hipFree(buf[0]));
    CK(hipFree(buf[1]));
  }
  close(to_child[1]);
  int st = 0;
  waitpid(pid, &st, 0);
  printf("exporter: %d calls, %d-%d KiB, K=%s: handle bytes repeating an earlier handle: %d; importer exit %d\n", calls,
         lo, hi, K, repeats, WIFEXITED(st) ? WEXITSTATUS(st) : -1);
  return 0;
}
