// Environment probe (not product code): if another process writes into this process's ordinary
// device memory through a dma-buf import, does this process's next kernel read the new data, or
// stale lines its L2s kept from an earlier kernel?  (DESIGN.md "Next": a read schedule that
// pushes each result slice into the peers' recv would rely on the answer.)
//
// The owner (this process) allocates X, fills it with A and reads all of it with default-policy
// loads (its L2s now hold lines of X); the writer (a child process, spawned before any HIP call)
// imports X and overwrites it with B using one store form -- default policy, non-temporal, or
// sc0 sc1 (system coherent, the schedules' remote stores) -- and synchronises; then the owner
// counts the words that are not B, once with default-policy loads on the same grid as the first
// read (same workgroup -> XCD deal, so the same L2s) and once with sc0 sc1 loads (the truth).
//
// Usage: probe_coherence [mib] [reps]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <spawn.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

extern char** environ;

#define CK(x)                                                                                               \
  do {                                                                                                      \
    hipError_t e_ = (x);                                                                                    \
    if (e_ != hipSuccess) {                                                                                 \
      fprintf(stderr, "[pid %d] %s:%d %s -> %s\n", getpid(), __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      _exit(2);                                                                                             \
    }                                                                                                       \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

constexpr int kGrid = 2048, kBlock = 256;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__global__ void fill(v4u* x, size_t nvec, unsigned v) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < nvec; i += (size_t)kGrid * kBlock)
    x[i] = v4u{v, v, v, v};
}

// default-policy loads; the sum keeps them alive
__global__ void touch(const v4u* x, size_t nvec, unsigned* sink) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < nvec; i += (size_t)kGrid * kBlock) {
    const v4u v = x[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) *sink = s;
}

// form 0: default policy, 1: non-temporal, 2: sc0 sc1 buffer stores
__global__ void overwrite(v4u* x, size_t nvec, unsigned v, int form) {
  const auto r = rsrc(x, (unsigned)(nvec * 16 > 0xffffffffull ? 0xffffffffu : nvec * 16));
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < nvec; i += (size_t)kGrid * kBlock) {
    const v4u w{v, v, v, v};
    if (form == 0) x[i] = w;
    else if (form == 1) __builtin_nontemporal_store(w, x + i);
    else __builtin_amdgcn_raw_buffer_store_b128(w, r, (unsigned)(i * 16), 0, 17);
  }
}

// words != v; sys: sc0 sc1 loads (bypass every cache), else default policy
__global__ void count_not(const v4u* x, size_t nvec, unsigned v, int sys, unsigned long long* bad) {
  const auto r = rsrc(x, (unsigned)(nvec * 16 > 0xffffffffull ? 0xffffffffu : nvec * 16));
  unsigned long long b = 0;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < nvec; i += (size_t)kGrid * kBlock) {
    const v4u w = sys ? __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(i * 16), 0, 17) : x[i];
    b += (w.x != v) + (w.y != v) + (w.z != v) + (w.w != v);
  }
  if (b) atomicAdd(bad, b);
}

struct Msg {
  int form;  // -1: quit
  unsigned value;
  unsigned long long off, bytes;
};

int send_msg(int s, const Msg& m, int fd) {
  iovec io{const_cast<Msg*>(&m), sizeof m};
  char cbuf[CMSG_SPACE(sizeof(int))];
  memset(cbuf, 0, sizeof cbuf);
  msghdr h{};
  h.msg_iov = &io, h.msg_iovlen = 1;
  if (fd >= 0) {
    h.msg_control = cbuf, h.msg_controllen = sizeof cbuf;
    cmsghdr* c = CMSG_FIRSTHDR(&h);
    c->cmsg_level = SOL_SOCKET, c->cmsg_type = SCM_RIGHTS, c->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(c), &fd, sizeof fd);
  }
  return sendmsg(s, &h, 0) == (ssize_t)sizeof m ? 0 : -1;
}

int recv_msg(int s, Msg* m, int* fd) {
  iovec io{m, sizeof *m};
  char cbuf[CMSG_SPACE(sizeof(int))];
  msghdr h{};
  h.msg_iov = &io, h.msg_iovlen = 1, h.msg_control = cbuf, h.msg_controllen = sizeof cbuf;
  if (recvmsg(s, &h, MSG_CMSG_CLOEXEC) != (ssize_t)sizeof *m) return -1;
  *fd = -1;
  cmsghdr* c = CMSG_FIRSTHDR(&h);
  if (c && c->cmsg_type == SCM_RIGHTS) memcpy(fd, CMSG_DATA(c), sizeof(int));
  return 0;
}

hsa_agent_t g_gpu{0};
hsa_status_t find_gpu(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle)
    g_gpu = a;
  return HSA_STATUS_SUCCESS;
}

int writer(int s) {
  CK(hipSetDevice(0));
  if (hsa_init() != HSA_STATUS_SUCCESS) return 12;
  hsa_iterate_agents(find_gpu, nullptr);
  for (;;) {
    Msg m;
    int fd = -1;
    if (recv_msg(s, &m, &fd) != 0) return 13;
    if (m.form < 0) break;
    size_t sz = 0;
    void* p = nullptr;
    if (hsa_amd_interop_map_buffer(1, &g_gpu, (hsa_handle_t)fd, 0, &sz, &p, nullptr, nullptr) != HSA_STATUS_SUCCESS) {
      fprintf(stderr, "writer: interop map failed\n");
      return 14;
    }
    close(fd);
    v4u* x = (v4u*)((char*)p + m.off);
    overwrite<<<kGrid, kBlock>>>(x, m.bytes / 16, m.value, m.form);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    hsa_amd_interop_unmap_buffer(p);
    Msg done{m.form, m.value, 0, 0};
    if (send_msg(s, done, -1) != 0) return 15;
  }
  hsa_shut_down();
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && !strcmp(argv[1], "writer")) return writer(atoi(argv[2]));
  const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 64;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const size_t bytes = mib << 20;
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) != 0) return 3;
  char a[16];
  snprintf(a, sizeof a, "%d", sv[1]);
  char* cargv[] = {argv[0], (char*)"writer", a, nullptr};
  pid_t pid;
  if (posix_spawn(&pid, argv[0], nullptr, nullptr, cargv, environ)) return 4;
  close(sv[1]);
  CK(hipSetDevice(0));
  unsigned* sink = nullptr;
  unsigned long long* bad = nullptr;
  CK(hipMalloc((void**)&sink, 4));
  CK(hipMalloc((void**)&bad, 16));
  const char* names[3] = {"default-policy stores", "non-temporal stores", "sc0 sc1 stores"};
  int rc = 0;
  for (int form = 0; form < 3 && !rc; ++form)
    for (int rep = 0; rep < reps && !rc; ++rep) {
      v4u* x = nullptr;
      CK(hipMalloc((void**)&x, bytes));
      const unsigned A = 0xa0000000u + (unsigned)(form * 16 + rep), B = 0xb0000000u + (unsigned)(form * 16 + rep);
      fill<<<kGrid, kBlock>>>(x, bytes / 16, A);
      touch<<<kGrid, kBlock>>>(x, bytes / 16, sink);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      int fd = -1;
      uint64_t off = 0;
      if (hsa_amd_portable_export_dmabuf(x, bytes, &fd, &off) != HSA_STATUS_SUCCESS) {
        fprintf(stderr, "owner: export failed\n");
        rc = 5;
        break;
      }
      Msg m{form, B, off, bytes};
      if (send_msg(sv[0], m, fd) != 0) rc = 6;
      hsa_amd_portable_close_dmabuf(fd);
      int nofd = -1;
      Msg done;
      if (!rc && recv_msg(sv[0], &done, &nofd) != 0) rc = 7;
      if (rc) break;
      unsigned long long h[2] = {0, 0};
      CK(hipMemset(bad, 0, 16));
      count_not<<<kGrid, kBlock>>>(x, bytes / 16, B, 0, bad);
      count_not<<<kGrid, kBlock>>>(x, bytes / 16, B, 1, bad + 1);
      CK(hipGetLastError());
      CK(hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost));
      printf("%-22s rep %d: %zu MiB, words not the writer's after this process's next kernel: default-policy loads %llu, "
             "sc0 sc1 loads %llu (of %zu)\n", names[form], rep, mib, h[0], h[1], bytes / 4);
      fflush(stdout);
      CK(hipFree(x));
    }
  Msg quit{-1, 0, 0, 0};
  send_msg(sv[0], quit, -1);
  int st = 0;
  waitpid(pid, &st, 0);
  if (!WIFEXITED(st) || WEXITSTATUS(st)) {
    fprintf(stderr, "writer exited with status 0x%x\n", st);
    if (!rc) rc = 8;
  }
  return rc;
}
