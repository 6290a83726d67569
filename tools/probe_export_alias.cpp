// Environment probe (not product code): after the same-GPU handle loss of probe_export_reuse.cpp,
// does a later export of the victim allocation fail -- or silently hand out ANOTHER buffer?
// Two forked processes on one GPU (forked before any HIP call); A exports, B imports:
//   1. A: hipMalloc X (20 MiB), export it; B imports it (same GPU)
//   2. A: hipFree X, close its export                      (X's handle deleted once)
//   3. A: hipMalloc Y (2 MiB), fill with 0x11              (the victim)
//   4. B: unmap its import of X                            (the same handle deleted again)
//   5. A: hipMalloc W (2 MiB), fill with 0x22
//   6. A: export Y (dma-buf) and hipIpcGetMemHandle(Y); B maps both and reads Y's first bytes:
//      0x11 = Y (correct), 0x22 = W (the export names another buffer), or the call fails
// Build: hipcc -O2 -o tools/bin/probe_export_alias tools/probe_export_alias.cpp -L/opt/rocm/lib -lhsa-runtime64
// Run:   tools/bin/probe_export_alias [ROUNDS]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      _exit(2);                                                                           \
    }                                                                                     \
  } while (0)

static void send_msg(int sock, int fd, const void* data, size_t n) {
  iovec io{const_cast<void*>(data), n};
  alignas(cmsghdr) char buf[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  if (fd >= 0) {
    m.msg_control = buf;
    m.msg_controllen = sizeof buf;
    cmsghdr* c0 = CMSG_FIRSTHDR(&m);
    c0->cmsg_level = SOL_SOCKET;
    c0->cmsg_type = SCM_RIGHTS;
    c0->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(c0), &fd, sizeof(int));
  }
  if (sendmsg(sock, &m, 0) != (ssize_t)n) _exit(5);
}

static int recv_msg(int sock, void* data, size_t n) {
  iovec io{data, n};
  alignas(cmsghdr) char buf[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = buf;
  m.msg_controllen = sizeof buf;
  if (recvmsg(sock, &m, MSG_WAITALL) != (ssize_t)n) _exit(6);
  cmsghdr* c0 = CMSG_FIRSTHDR(&m);
  int fd = -1;
  if (c0 && c0->cmsg_type == SCM_RIGHTS) memcpy(&fd, CMSG_DATA(c0), sizeof(int));
  return fd;
}

static hsa_status_t pick_gpu(hsa_agent_t a, void* out) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU) {
    *static_cast<hsa_agent_t*>(out) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// reads one byte of a mapped peer buffer on the GPU (the library's kernels read imports the same
// way; hipMemcpy does not know an interop mapping)
__global__ void peek(const unsigned char* p, unsigned char* out) {
  if (threadIdx.x == 0) out[0] = p[0];
}

static unsigned char read_byte(const void* p) {
  unsigned char* d = nullptr;
  unsigned char h = 0;
  CK(hipMalloc(reinterpret_cast<void**>(&d), 64));
  peek<<<1, 64>>>(static_cast<const unsigned char*>(p), d);
  CK(hipMemcpy(&h, d, 1, hipMemcpyDeviceToHost));
  CK(hipFree(d));
  return h;
}

struct Msg {
  int ok;  // 1: an fd rides along
  uint64_t off;
  hipIpcMemHandle_t ipc;
  int ipc_ok;
};

static int run(pthread_barrier_t* bar, int sock, int me, int rounds) {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  hsa_agent_t gpu{0};
  hsa_iterate_agents(pick_gpu, &gpu);
  int bad = 0;
  for (int r = 0; r < rounds; ++r) {
    const size_t big = 20u << 20, small = 2u << 20;
    void *x = nullptr, *y = nullptr, *w = nullptr, *imp = nullptr;
    int fd = -1;
    uint64_t off = 0;
    Msg m{};
    if (me == 0) {  // A
      CK(hipMalloc(&x, big));
      m.ok = hsa_amd_portable_export_dmabuf(x, big, &fd, &off) == HSA_STATUS_SUCCESS;
      send_msg(sock, m.ok ? fd : -1, &m, sizeof m);
    } else {  // B
      const int pfd = recv_msg(sock, &m, sizeof m);
      size_t sz = 0;
      if (m.ok && hsa_amd_interop_map_buffer(1, &gpu, (hsa_handle_t)pfd, 0, &sz, &imp, nullptr, nullptr) != HSA_STATUS_SUCCESS)
        imp = nullptr;
      if (pfd >= 0) close(pfd);
    }
    pthread_barrier_wait(bar);
    if (me == 0) {
      CK(hipFree(x));
      hsa_amd_portable_close_dmabuf(fd);
      CK(hipMalloc(&y, small));
      CK(hipMemset(y, 0x11, small));
      CK(hipDeviceSynchronize());
    }
    pthread_barrier_wait(bar);
    if (me == 1 && imp) hsa_amd_interop_unmap_buffer(imp);
    pthread_barrier_wait(bar);
    if (me == 0) {
      CK(hipMalloc(&w, small));
      CK(hipMemset(w, 0x22, small));
      CK(hipDeviceSynchronize());
      Msg e{};
      int yfd = -1;
      errno = 0;
      const hsa_status_t s = hsa_amd_portable_export_dmabuf(y, small, &yfd, &e.off);
      e.ok = s == HSA_STATUS_SUCCESS;
      const int err = errno;
      e.ipc_ok = hipIpcGetMemHandle(&e.ipc, y) == hipSuccess;
      if (!e.ipc_ok) (void)hipGetLastError();
      printf("round %d A: Y %p, W %p; export Y: %s (status 0x%x errno %d), hipIpcGetMemHandle(Y): %s\n", r, y, w,
             e.ok ? "ok" : "FAILED", (unsigned)s, err, e.ipc_ok ? "ok" : "FAILED");
      send_msg(sock, e.ok ? yfd : -1, &e, sizeof e);
      if (yfd >= 0) hsa_amd_portable_close_dmabuf(yfd);
    } else {
      Msg e{};
      const int yfd = recv_msg(sock, &e, sizeof e);
      unsigned char got[2] = {0, 0};
      const char* what[2] = {"-", "-"};
      void* ymap = nullptr;
      size_t sz = 0;
      printf("round %d B: received Y's export (%s)\n", r, e.ok ? "fd" : "none");
      if (e.ok && hsa_amd_interop_map_buffer(1, &gpu, (hsa_handle_t)yfd, 0, &sz, &ymap, nullptr, nullptr) == HSA_STATUS_SUCCESS) {
        got[0] = read_byte((char*)ymap + e.off);
        what[0] = got[0] == 0x11 ? "Y (correct)" : got[0] == 0x22 ? "W: ANOTHER BUFFER" : "unknown bytes";
      }
      void* ip = nullptr;
      if (e.ipc_ok && hipIpcOpenMemHandle(&ip, e.ipc, hipIpcMemLazyEnablePeerAccess) == hipSuccess) {
        got[1] = read_byte(ip);
        what[1] = got[1] == 0x11 ? "Y (correct)" : got[1] == 0x22 ? "W: ANOTHER BUFFER" : "unknown bytes";
      } else {
        (void)hipGetLastError();
      }
      printf("round %d B: dma-buf import of Y reads 0x%02x = %s; hipIpc open of Y reads 0x%02x = %s\n", r, got[0],
             what[0], got[1], what[1]);
      bad += (got[0] == 0x22) + (got[1] == 0x22);
      // left mapped: unmapping would delete more handles mid-probe
      if (yfd >= 0) close(yfd);
    }
    pthread_barrier_wait(bar);
  }
  fflush(stdout);
  return bad ? 1 : 0;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  void* mem = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (mem == MAP_FAILED) return 1;
  pthread_barrier_t* bar = new (mem) pthread_barrier_t;
  pthread_barrierattr_t a;
  pthread_barrierattr_init(&a);
  pthread_barrierattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_barrier_init(bar, &a, 2);
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 1;
  setvbuf(stdout, nullptr, _IOLBF, 0);
  if (fork() == 0) _exit(run(bar, sv[1], 1, rounds));  // before any HIP call
  int rc = run(bar, sv[0], 0, rounds);
  int st = 0;
  wait(&st);
  if (!WIFEXITED(st) || WEXITSTATUS(st)) rc |= 4;
  return rc;
}
