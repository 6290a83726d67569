// ipcreg.cpp -- see ipcreg.h.
#include "ipcreg.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace mnccl {
namespace ipc {

namespace {

constexpr size_t kMaxExports = 512;  // descriptors this process holds open for its peers

struct Export {
  uint64_t base, id, size;
  Shared d;
};
struct Import {
  uint64_t owner, base, id;
  void* map;      // the dma-buf's mapping (unmapped on close)
  char* local;    // map + the owner's bo_off: the owner's base
  bool same_gpu;  // the owner's memory is on this process's GPU (close_import retires it)
  bool retired;   // its owner freed it; kept mapped while the process lives (ipcreg.h close_import)
  uint64_t bytes; // the mapping's size (the dma-buf's)
};
struct BlockImport {
  uint64_t owner, base, id;
  char* local;
};
struct Block {
  void* p;
  size_t bytes;
  unsigned flags;
  uint64_t id;
  hipIpcMemHandle_t h;
  bool busy;
};

struct State {
  std::mutex mu;
  std::vector<Export> exports;                       // live exports
  std::vector<std::pair<uint64_t, uint64_t>> freed;  // exports found freed, in order
  std::vector<Import> imports;
  std::vector<BlockImport> blocks;
  std::vector<Block> pool;
  std::vector<std::pair<int, hsa_agent_t>> agents;  // HIP device ordinal -> its HSA agent
  uint64_t open_failures = 0;
  uint64_t liveness_queries = 0, cap_refusals = 0;
  uint64_t retired_bytes = 0, retired_budget = ~0ull, budget_refusals = 0;
  bool warned_retired = false, warned_budget = false;
  size_t reap_cursor = 0;                            // next export the round-robin batch checks
  std::vector<std::pair<uint64_t, int>> owner_refs;  // peer process nonce -> live communicators
  int live_comms = 0;
};

State& st() {
  static State* s = new State;  // never destroyed: imports / pool live until the process exits
  return *s;
}

std::string err_str(const char* what, hsa_status_t e) {
  const char* m = nullptr;
  if (hsa_status_string(e, &m) != HSA_STATUS_SUCCESS || !m) m = "unknown status";
  char b[256];
  snprintf(b, sizeof b, "%s: HSA status 0x%x (%.80s)", what, (unsigned)e, m);
  return b;
}

struct AgentMatch {
  uint32_t domain, bdf;
  hsa_agent_t found;
};

hsa_status_t match_agent(hsa_agent_t a, void* arg) {
  AgentMatch* m = static_cast<AgentMatch*>(arg);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS ||
      hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  // BDFID = bus << 8 | device << 3 | function; HIP reports bus and device
  if (dom == m->domain && (bdf >> 3) == (m->bdf >> 3)) {
    m->found = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// An agent's PCI location, as Shared::gpu carries it (0 if unknown)
uint32_t agent_location(hsa_agent_t a) {
  uint32_t bdf = 0, dom = 0;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS ||
      hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) != HSA_STATUS_SUCCESS)
    return 0;
  return (dom << 16) | (bdf & 0xfff8u);
}

// The HSA agent of this thread's current HIP device (HIP runs on the same runtime).  Caller holds
// s.mu.
bool current_agent(State& s, hsa_agent_t* out, std::string* why) {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    *why = "hipGetDevice failed";
    return false;
  }
  for (const auto& a : s.agents)
    if (a.first == dev) {
      *out = a.second;
      return true;
    }
  int dom = 0, bus = 0, devno = 0;
  if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev) != hipSuccess ||
      hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&devno, hipDeviceAttributePciDeviceId, dev) != hipSuccess) {
    (void)hipGetLastError();
    *why = "PCI location of the current device unknown";
    return false;
  }
  AgentMatch m{(uint32_t)dom, (uint32_t)((bus << 8) | (devno << 3)), hsa_agent_t{0}};
  // HIP has brought the runtime up (the device is in use); only if it has not, take a reference
  // of our own (never released: HIP's shutdown then leaves the runtime to the process exit)
  if (hsa_iterate_agents(match_agent, &m) == HSA_STATUS_ERROR_NOT_INITIALIZED) {
    const hsa_status_t e = hsa_init();
    if (e != HSA_STATUS_SUCCESS) {
      *why = err_str("hsa_init", e);
      return false;
    }
    hsa_iterate_agents(match_agent, &m);
  }
  if (!m.found.handle) {
    *why = "no HSA agent at the current device's PCI location";
    return false;
  }
  s.agents.emplace_back(dev, m.found);
  *out = m.found;
  return true;
}

}  // namespace

bool find_live_export(uint64_t p, uint64_t* base, uint64_t* id, Shared* d) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (const Export& e : s.exports)
    if (p >= e.base && p - e.base < e.size) {
      *base = e.base;
      *id = e.id;
      *d = e.d;
      return true;
    }
  return false;
}

bool export_allocation(uint64_t base, uint64_t id, uint64_t size, Shared* d, std::string* why) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (const Export& e : s.exports)
    if (e.base == base && e.id == id) {
      *d = e.d;
      return true;
    }
  std::string w;
  hsa_agent_t a;
  if (!current_agent(s, &a, &w)) {  // also brings HSA up
    if (why) *why = w;
    return false;
  }
  if (s.exports.size() >= kMaxExports) {
    if (why) *why = "this process holds " + std::to_string(kMaxExports) + " exports already";
    ++s.cap_refusals;
    static bool warned = false;  // once per process (under s.mu)
    if (!warned) {
      warned = true;
      fprintf(stderr, "[Mini-NCCL] warning: this process shares %zu buffers with its peers already (the cap): calls "
              "on buffers beyond it run the ring (counted in mncclCommInfo_t.cap_refusals)\n", kMaxExports);
    }
    return false;
  }
  int fd = -1;
  uint64_t off = 0;
  errno = 0;
  const hsa_status_t e = hsa_amd_portable_export_dmabuf((const void*)(uintptr_t)base, size, &fd, &off);
  if (e != HSA_STATUS_SUCCESS) {
    const int err = errno;  // the export ioctl's, when it failed there
    if (why)
      *why = err_str("hsa_amd_portable_export_dmabuf", e) + " (errno " + std::to_string(err) + ": " + strerror(err) +
             "; " + std::to_string(s.exports.size()) + " exports live, " + std::to_string(size) + " bytes)";
    return false;
  }
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    hsa_amd_portable_close_dmabuf(fd);
    if (why) *why = std::string("fstat of an exported dma-buf: ") + strerror(errno);
    return false;
  }
  // a dma-buf's size is its buffer object's: one too small to hold the allocation at `off` is not
  // this allocation's (the same-GPU handle reuse of profiles/r5_export_reuse.txt can hand the export
  // another object's handle) -- refused, the calls run the ring
  const off_t end = lseek(fd, 0, SEEK_END);
  if (end >= 0 && (uint64_t)end < off + size) {
    hsa_amd_portable_close_dmabuf(fd);
    if (why)
      *why = "the exported dma-buf (" + std::to_string((long long)end) + " bytes) cannot hold the allocation (" +
             std::to_string(size) + " bytes at offset " + std::to_string(off) + ")";
    return false;
  }
  d->fd = fd;
  d->gpu = agent_location(a);
  d->ino = (uint64_t)sb.st_ino;
  d->bo_off = off;
  s.exports.push_back(Export{base, id, size, *d});
  return true;
}

size_t freed_log_size() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.freed.size();
}

std::pair<uint64_t, uint64_t> freed_log_at(size_t i) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.freed.at(i);
}

void reap_freed_exports(const uint64_t* addrs, int naddrs, size_t batch) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  const size_t n = s.exports.size();
  if (!n) return;
  std::vector<char> check(n, 0);
  for (size_t i = 0; i < n; ++i)
    for (int a = 0; a < naddrs; ++a)
      if (addrs[a] >= s.exports[i].base && addrs[a] - s.exports[i].base < s.exports[i].size) check[i] = 1;
  for (size_t k = 0; k < batch && k < n; ++k) check[(s.reap_cursor + k) % n] = 1;
  s.reap_cursor = n ? (s.reap_cursor + batch) % n : 0;
  // is the allocation at the export's base still the one exported (same HIP buffer id)?
  std::vector<Export> keep;
  keep.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    const Export& x = s.exports[i];
    bool alive = true;
    if (check[i]) {
      unsigned long long id = 0;
      ++s.liveness_queries;
      const hipError_t e = hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)x.base);
      alive = e == hipSuccess && id == x.id;
      if (e != hipSuccess) (void)hipGetLastError();
    }
    if (alive) {
      keep.push_back(x);
    } else {
      // the peers' imports hold their own references: closing ours releases nothing they use
      hsa_amd_portable_close_dmabuf(x.d.fd);
      s.freed.emplace_back(x.base, x.id);
    }
  }
  s.exports.swap(keep);
  if (s.reap_cursor >= s.exports.size()) s.reap_cursor = 0;
}

uint64_t liveness_queries() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.liveness_queries;
}

size_t live_exports() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.exports.size();
}

char* find_import(uint64_t owner, uint64_t base, uint64_t id) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (const Import& m : s.imports)
    if (!m.retired && m.owner == owner && m.base == base && m.id == id) return m.local;
  return nullptr;
}

char* open_import(uint64_t owner, uint64_t base, uint64_t id, int fd, const Shared& d, std::string* why,
                  bool* budget_refused) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  if (budget_refused) *budget_refused = false;
  for (const Import& m : s.imports)
    if (!m.retired && m.owner == owner && m.base == base && m.id == id) {
      if (fd >= 0) close(fd);
      return m.local;
    }
  auto fail = [&](const std::string& w) -> char* {
    if (fd >= 0) close(fd);
    ++s.open_failures;
    *why = w;
    return nullptr;
  };
  if (fd < 0) return fail("no descriptor arrived from the owner");
  hsa_agent_t agent;
  std::string w;
  if (!current_agent(s, &agent, &w)) return fail(w);
  const uint32_t here = agent_location(agent);
  const bool same_gpu = here != 0 && here == d.gpu;
  if (same_gpu && s.retired_bytes >= s.retired_budget) {
    // one more same-GPU import would pin its memory too once its owner frees it (close_import)
    close(fd);
    ++s.budget_refusals;
    if (budget_refused) *budget_refused = true;
    char b[256];
    snprintf(b, sizeof b, "freed allocations of same-GPU peers already hold %llu MiB mapped here (MINI_NCCL_RETIRED_MB "
             "= %llu)", (unsigned long long)(s.retired_bytes >> 20), (unsigned long long)(s.retired_budget >> 20));
    *why = b;
    if (!s.warned_budget) {
      s.warned_budget = true;
      fprintf(stderr, "[Mini-NCCL] warning: %s: calls that bring a new buffer of a peer on this GPU run the ring from "
              "now on (counted in mncclCommInfo_t.budget_refusals)\n", b);
    }
    return nullptr;
  }
  struct stat sb;
  if (fstat(fd, &sb) != 0 || (uint64_t)sb.st_ino != d.ino)
    return fail("the received descriptor does not name the exported dma-buf");
  size_t sz = 0;
  void* p = nullptr;
  const hsa_status_t e = hsa_amd_interop_map_buffer(1, &agent, (hsa_handle_t)fd, 0, &sz, &p, nullptr, nullptr);
  if (e != HSA_STATUS_SUCCESS) return fail(err_str("hsa_amd_interop_map_buffer", e));
  close(fd);  // the mapping holds its own reference
  if (d.bo_off >= sz) {
    hsa_amd_interop_unmap_buffer(p);
    ++s.open_failures;
    *why = "an exported allocation lies outside its dma-buf";
    return nullptr;
  }
  char* local = (char*)p + d.bo_off;
  s.imports.push_back(Import{owner, base, id, p, local, same_gpu, false, (uint64_t)sz});
  return local;
}

bool close_import(uint64_t owner, uint64_t base, uint64_t id) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (size_t i = 0; i < s.imports.size(); ++i)
    if (!s.imports[i].retired && s.imports[i].owner == owner && s.imports[i].base == base && s.imports[i].id == id) {
      if (s.imports[i].same_gpu) {  // see ipcreg.h: kept mapped while the process lives
        s.imports[i].retired = true;
        s.retired_bytes += s.imports[i].bytes;
        const size_t nret = (size_t)std::count_if(s.imports.begin(), s.imports.end(),
                                                  [](const Import& m) { return m.retired; });
        if (!s.warned_retired && (nret * 4 >= kMaxImports * 3 ||
                                  (s.retired_budget != ~0ull && s.retired_bytes * 4 >= s.retired_budget * 3))) {
          s.warned_retired = true;
          fprintf(stderr, "[Mini-NCCL] warning: %zu freed allocations of peers on this GPU (%llu MiB) stay mapped in "
                  "this process (the GPU driver shares their handle, DESIGN.md); at %zu imports or MINI_NCCL_RETIRED_MB "
                  "= %llu MiB, calls on new peer buffers run the ring -- reuse buffers (a caching allocator) to avoid "
                  "it\n", nret, (unsigned long long)(s.retired_bytes >> 20), kMaxImports,
                  (unsigned long long)(s.retired_budget >> 20));
        }
        return true;
      }
      hsa_amd_interop_unmap_buffer(s.imports[i].map);
      s.imports.erase(s.imports.begin() + (long)i);
      return true;
    }
  return false;
}

size_t imports() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return (size_t)std::count_if(s.imports.begin(), s.imports.end(), [](const Import& m) { return !m.retired; });
}

size_t retired_imports() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return (size_t)std::count_if(s.imports.begin(), s.imports.end(), [](const Import& m) { return m.retired; });
}

uint64_t retired_bytes() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.retired_bytes;
}

void set_retired_budget(uint64_t bytes) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  s.retired_budget = bytes;
}

uint64_t retired_budget() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.retired_budget;
}

uint64_t budget_refusals() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.budget_refusals;
}

void note_cap_refusal(const std::string& what) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  ++s.cap_refusals;
  static bool warned = false;  // once per process (under s.mu)
  if (!warned) {
    warned = true;
    fprintf(stderr, "[Mini-NCCL] warning: %s: calls on further peer buffers run the ring (counted in "
            "mncclCommInfo_t.cap_refusals)\n", what.c_str());
  }
}

uint64_t cap_refusals() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.cap_refusals;
}

void comm_opened(const std::vector<uint64_t>& owners) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  ++s.live_comms;
  for (uint64_t o : owners) {
    bool found = false;
    for (auto& r : s.owner_refs)
      if (r.first == o) {
        ++r.second;
        found = true;
      }
    if (!found) s.owner_refs.emplace_back(o, 1);
  }
}

void comm_closed(const std::vector<uint64_t>& owners) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  if (s.live_comms > 0) --s.live_comms;
  for (uint64_t o : owners)
    for (size_t i = 0; i < s.owner_refs.size(); ++i) {
      if (s.owner_refs[i].first != o) continue;
      if (--s.owner_refs[i].second > 0) break;
      s.owner_refs.erase(s.owner_refs.begin() + (long)i);
      // no live communicator of this process talks to that owner any more: its imports go --
      // except imports of this GPU's memory, which stay mapped while the process lives (ipcreg.h
      // close_import: their unmap would be a second delete of the owner's handle, whoever went first)
      for (size_t j = 0; j < s.imports.size();) {
        if (s.imports[j].owner == o && !s.imports[j].same_gpu) {
          hsa_amd_interop_unmap_buffer(s.imports[j].map);
          s.imports.erase(s.imports.begin() + (long)j);
        } else {
          ++j;
        }
      }
      break;
    }
  if (s.live_comms == 0) {
    // no peer can import from this process any more (its communicators are gone with ours):
    // the descriptors go, so a later free of any exported allocation releases its memory
    for (const Export& x : s.exports) hsa_amd_portable_close_dmabuf(x.d.fd);
    s.exports.clear();
    s.reap_cursor = 0;
  }
}

uint64_t open_failures() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.open_failures;
}

void* pool_acquire(size_t bytes, unsigned flags, hipIpcMemHandle_t* h, uint64_t* id) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) throw std::runtime_error("hipGetDevice");
  for (Block& b : s.pool) {
    hipPointerAttribute_t a;
    if (b.busy || b.bytes != bytes || b.flags != flags) continue;
    if (hipPointerGetAttributes(&a, b.p) != hipSuccess || a.device != dev) {
      (void)hipGetLastError();
      continue;  // a block of another device
    }
    b.busy = true;
    *h = b.h;
    *id = b.id;
    return b.p;
  }
  void* p = nullptr;
  hipError_t e = flags ? hipExtMallocWithFlags(&p, bytes, flags) : hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    throw std::runtime_error(std::string("device allocation of ") + std::to_string(bytes) + " B: " +
                             hipGetErrorString(e));
  }
  unsigned long long bid = 0;
  e = hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p);
  if (e == hipSuccess) e = hipIpcGetMemHandle(h, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(p);
    throw std::runtime_error(std::string("IPC export of a communicator buffer: ") + hipGetErrorString(e));
  }
  s.pool.push_back(Block{p, bytes, flags, bid, *h, true});
  *id = bid;
  return p;
}

void pool_release(void* p) {
  if (!p) return;
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (Block& b : s.pool)
    if (b.p == p) b.busy = false;
}

char* open_block(uint64_t owner, uint64_t base, uint64_t id, const hipIpcMemHandle_t& h, hipError_t* err) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (const BlockImport& m : s.blocks)
    if (m.owner == owner && m.base == base && m.id == id) return m.local;
  void* p = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *err = e;
    return nullptr;
  }
  s.blocks.push_back(BlockImport{owner, base, id, (char*)p});
  return (char*)p;
}

}  // namespace ipc
}  // namespace mnccl
