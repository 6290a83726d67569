// Environment probe (not product code): can a rank map its PEERS' user buffers cheaply?
//  (1) hipIpcGetMemHandle on an allocation base: cost per call, are repeated handles the same
//      bytes, does it leak file descriptors;
//  (2) a pointer inside an allocation: hipMemGetAddressRange base/size, BUFFER_ID;
//  (3) another process opens the handle (cost) and reads the bytes at an offset;
//  (4) hipFree + hipMalloc at the same address: new handle / new BUFFER_ID?
// Host-side HIP calls only, no kernels.  Usage: probe_ub (spawns itself as the importer).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

extern char** environ;

#define CK(x)                                                                                          \
  do {                                                                                                 \
    hipError_t e_ = (x);                                                                               \
    if (e_ != hipSuccess) {                                                                            \
      fprintf(stderr, "[pid %d] %s:%d %s -> %s\n", getpid(), __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                                         \
    }                                                                                                  \
  } while (0)

static int nfds() {
  int n = 0;
  DIR* d = opendir("/proc/self/fd");
  if (!d) return -1;
  while (readdir(d)) ++n;
  closedir(d);
  return n;
}
static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void hex(const char* tag, const hipIpcMemHandle_t& h) {
  printf("%s ", tag);
  for (int i = 0; i < 64; ++i) printf("%02x", (unsigned char)h.reserved[i]);
  printf("\n");
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "import")) {
    // child: read the handle from stdin (hex), open it, read 16 floats at offset 4096
    hipIpcMemHandle_t h;
    for (int i = 0; i < 64; ++i) {
      unsigned v;
      if (scanf("%2x", &v) != 1) return 3;
      h.reserved[i] = (char)v;
    }
    CK(hipSetDevice(0));
    void* p = nullptr;
    double t0 = now();
    CK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    double t1 = now();
    float v[4];
    CK(hipMemcpy(v, (char*)p + 4096, sizeof v, hipMemcpyDeviceToHost));
    printf("child: open %.1f us, values at +4096: %g %g %g %g\n", (t1 - t0) * 1e6, v[0], v[1], v[2], v[3]);
    void* p2 = nullptr;
    hipError_t e2 = hipIpcOpenMemHandle(&p2, h, hipIpcMemLazyEnablePeerAccess);
    printf("child: second open of the same handle -> %s, same pointer %d\n", hipGetErrorString(e2), p2 == p);
    if (e2 == hipSuccess && p2 != p) hipIpcCloseMemHandle(p2);
    double t2 = now();
    CK(hipIpcCloseMemHandle(p));
    printf("child: close %.1f us\n", (now() - t2) * 1e6);
    return 0;
  }
  CK(hipSetDevice(0));
  const size_t bytes = (size_t)1 << 30;
  char* base = nullptr;
  CK(hipMalloc((void**)&base, bytes));
  float ones[1024];
  for (int i = 0; i < 1024; ++i) ones[i] = 1.0f + i;
  CK(hipMemcpy(base + 4096, ones, sizeof ones, hipMemcpyHostToDevice));
  char* inner = base + 4096;
  hipDeviceptr_t rb = 0;
  size_t rs = 0;
  CK(hipMemGetAddressRange(&rb, &rs, (hipDeviceptr_t)inner));
  unsigned long long bid = 0;
  hipError_t eb = hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)inner);
  printf("range of base+4096: base ok %d size %zu; BUFFER_ID -> %s %llu\n", (char*)rb == base, rs, hipGetErrorString(eb), bid);

  hipIpcMemHandle_t h0, h1, hi;
  int f0 = nfds();
  double t0 = now();
  CK(hipIpcGetMemHandle(&h0, base));
  double t1 = now();
  const int N = 200;
  for (int i = 0; i < N; ++i) CK(hipIpcGetMemHandle(&h1, base));
  double t2 = now();
  int f1 = nfds();
  printf("get handle: first %.1f us, then %.2f us per call; repeated handle identical %d; fds %d -> %d\n",
         (t1 - t0) * 1e6, (t2 - t1) / N * 1e6, !memcmp(&h0, &h1, sizeof h0), f0, f1);
  hex("h0", h0);
  hipError_t ei = hipIpcGetMemHandle(&hi, inner);
  printf("get handle on base+4096 -> %s; identical to base's %d\n", hipGetErrorString(ei),
         ei == hipSuccess && !memcmp(&hi, &h0, sizeof h0));
  if (ei == hipSuccess) hex("hi", hi);

  // importer process
  int pin[2];
  if (pipe(pin)) return 4;
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, pin[0], 0);
  posix_spawn_file_actions_addclose(&fa, pin[1]);
  pid_t pid;
  char* cargv[] = {argv[0], (char*)"import", nullptr};
  if (posix_spawn(&pid, argv[0], &fa, nullptr, cargv, environ)) return 5;
  close(pin[0]);
  FILE* w = fdopen(pin[1], "w");
  for (int i = 0; i < 64; ++i) fprintf(w, "%02x", (unsigned char)h0.reserved[i]);
  fclose(w);
  int st = 0;
  waitpid(pid, &st, 0);
  printf("importer exit %d\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1);

  // free + malloc: same address? new handle? new BUFFER_ID?
  CK(hipFree(base));
  char* b2 = nullptr;
  CK(hipMalloc((void**)&b2, bytes));
  unsigned long long bid2 = 0;
  hipPointerGetAttribute(&bid2, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)b2);
  hipIpcMemHandle_t h2;
  CK(hipIpcGetMemHandle(&h2, b2));
  printf("realloc: same address %d, BUFFER_ID %llu -> %llu, handle identical %d, fds %d\n", b2 == base, bid, bid2,
         !memcmp(&h2, &h0, sizeof h0), nfds());
  hex("h2", h2);
  CK(hipFree(b2));
  return 0;
}
