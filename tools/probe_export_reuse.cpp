// Environment probe (not product code): does a dma-buf export fail after an earlier exported
// buffer was freed, and what does it take?  Round 5's stress found hsa_amd_portable_export_dmabuf
// refusing (HSA_STATUS_ERROR_OUT_OF_RESOURCES, errno ENOENT) a new 2 MiB allocation on some ranks
// after a call on fresh 20 MiB buffers that the peers had imported and the owner had freed
// (tools/r5_export_bisect.py).  Two forked processes (forked before any HIP call), each:
//   1. hipMalloc X (20 MiB), export it, send the descriptor to the other process over a socket
//   2. (MODE & 1) import the other's X with hsa_amd_interop_map_buffer
//   3. (MODE & 4) hipFree X and close its export; barrier
//   4. (MODE & 2) unmap the import of the other's X; barrier
//   5. hipMalloc K buffers of 2 MiB, export each: prints which fail (status, errno)
//   (MODE & 8) allocate step 5's buffers between steps 3 and 4 (before the unmap), export after
// Build: hipcc -O2 -o tools/bin/probe_export_reuse tools/probe_export_reuse.cpp -L/opt/rocm/lib -lhsa-runtime64
// Run:   tools/bin/probe_export_reuse <MODE> [K]
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

static int send_fd(int sock, int fd) {
  char c = 0;
  iovec io{&c, 1};
  alignas(cmsghdr) char buf[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = buf;
  m.msg_controllen = sizeof buf;
  cmsghdr* c0 = CMSG_FIRSTHDR(&m);
  c0->cmsg_level = SOL_SOCKET;
  c0->cmsg_type = SCM_RIGHTS;
  c0->cmsg_len = CMSG_LEN(sizeof(int));
  memcpy(CMSG_DATA(c0), &fd, sizeof(int));
  return sendmsg(sock, &m, 0) == 1 ? 0 : -1;
}

static int recv_fd(int sock) {
  char c = 0;
  iovec io{&c, 1};
  alignas(cmsghdr) char buf[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = buf;
  m.msg_controllen = sizeof buf;
  if (recvmsg(sock, &m, 0) != 1) return -1;
  cmsghdr* c0 = CMSG_FIRSTHDR(&m);
  if (!c0 || c0->cmsg_type != SCM_RIGHTS) return -1;
  int fd = -1;
  memcpy(&fd, CMSG_DATA(c0), sizeof(int));
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

static int run(pthread_barrier_t* bar, int sock, int me, int mode, int k) {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  hsa_agent_t gpu{0};
  hsa_iterate_agents(pick_gpu, &gpu);
  const size_t big = 20u << 20;
  void* x = nullptr;
  CK(hipMalloc(&x, big));
  int fd = -1;
  uint64_t off = 0;
  hsa_status_t e = hsa_amd_portable_export_dmabuf(x, big, &fd, &off);
  printf("p%d: export X %p -> %s\n", me, x, e == HSA_STATUS_SUCCESS ? "ok" : "FAILED");
  if (e != HSA_STATUS_SUCCESS) return 3;
  int dup_fd = dup(fd);
  send_fd(sock, dup_fd);
  close(dup_fd);
  const int peer_fd = recv_fd(sock);
  void* peer = nullptr;
  if (mode & 1) {
    size_t sz = 0;
    e = hsa_amd_interop_map_buffer(1, &gpu, (hsa_handle_t)peer_fd, 0, &sz, &peer, nullptr, nullptr);
    printf("p%d: import peer X -> %s at %p (%zu bytes)\n", me, e == HSA_STATUS_SUCCESS ? "ok" : "FAILED", peer, sz);
  }
  close(peer_fd);
  pthread_barrier_wait(bar);
  if (mode & 4) {
    CK(hipFree(x));
    hsa_amd_portable_close_dmabuf(fd);
    printf("p%d: freed X, closed its export\n", me);
  }
  pthread_barrier_wait(bar);
  void* early[64] = {};
  if (mode & 8)
    for (int i = 0; i < k && i < 64; ++i) CK(hipMalloc(&early[i], 2u << 20));
  pthread_barrier_wait(bar);
  if ((mode & 2) && peer) {
    e = hsa_amd_interop_unmap_buffer(peer);
    printf("p%d: unmapped the import -> %s\n", me, e == HSA_STATUS_SUCCESS ? "ok" : "FAILED");
  }
  pthread_barrier_wait(bar);
  int fails = 0;
  for (int i = 0; i < k; ++i) {
    void* b = early[i < 64 ? i : 0];
    if (!(mode & 8) || i >= 64) CK(hipMalloc(&b, 2u << 20));
    int f = -1;
    errno = 0;
    e = hsa_amd_portable_export_dmabuf(b, 2u << 20, &f, &off);
    const int err = errno;
    const bool in_old = (char*)b >= (char*)x && (char*)b < (char*)x + big;
    const bool in_peer = peer && (char*)b >= (char*)peer && (char*)b < (char*)peer + big;
    printf("p%d: 2 MiB #%d at %p%s%s: export %s", me, i, b, in_old ? " (inside freed X)" : "",
           in_peer ? " (inside the peer import's range)" : "", e == HSA_STATUS_SUCCESS ? "ok\n" : "FAILED");
    if (e != HSA_STATUS_SUCCESS) {
      printf(" status 0x%x errno %d\n", (unsigned)e, err);
      ++fails;
    } else {
      hsa_amd_portable_close_dmabuf(f);
    }
  }
  fflush(stdout);
  return fails ? 1 : 0;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 7;
  const int k = argc > 2 ? atoi(argv[2]) : 8;
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
  printf("mode %d (import %d, unmap %d, free %d, allocate before the unmap %d), %d exports of 2 MiB\n", mode,
         mode & 1, (mode >> 1) & 1, (mode >> 2) & 1, (mode >> 3) & 1, k);
  if (fork() == 0) _exit(run(bar, sv[1], 1, mode, k));  // before any HIP call
  int rc = run(bar, sv[0], 0, mode, k);
  int st = 0;
  wait(&st);
  if (!WIFEXITED(st) || WEXITSTATUS(st)) rc |= 4;
  return rc;
}
