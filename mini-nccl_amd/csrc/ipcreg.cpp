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
  void* map;    // the dma-buf's mapping (unmapped on close)
  char* local;  // map + the owner's bo_off: the owner's base
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
};

State& st() {
  static State* s = new State;  // never destroyed: imports / pool live until the process exits
  return *s;
}

std::string err_str(const char* what, hsa_status_t e) {
  const char* m = nullptr;
  if (hsa_status_string(e, &m) != HSA_STATUS_SUCCESS || !m) m = "unknown status";
  char b[256];
  snprintf(b, sizeof b, "%s: HSA status 0x%x (%s)", what, (unsigned)e, m);
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
    return false;
  }
  int fd = -1;
  uint64_t off = 0;
  const hsa_status_t e = hsa_amd_portable_export_dmabuf((const void*)(uintptr_t)base, size, &fd, &off);
  if (e != HSA_STATUS_SUCCESS) {
    if (why) *why = err_str("hsa_amd_portable_export_dmabuf", e);
    return false;
  }
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    hsa_amd_portable_close_dmabuf(fd);
    if (why) *why = std::string("fstat of an exported dma-buf: ") + strerror(errno);
    return false;
  }
  d->fd = fd;
  d->pad = 0;
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

void reap_freed_exports() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (size_t i = 0; i < s.exports.size();) {
    unsigned long long id = 0;
    const hipError_t e = hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)s.exports[i].base);
    if (e != hipSuccess || id != s.exports[i].id) {
      (void)hipGetLastError();
      // the peers' imports hold their own references: closing ours releases nothing they use
      hsa_amd_portable_close_dmabuf(s.exports[i].d.fd);
      s.freed.emplace_back(s.exports[i].base, s.exports[i].id);
      s.exports.erase(s.exports.begin() + (long)i);
    } else {
      ++i;
    }
  }
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
    if (m.owner == owner && m.base == base && m.id == id) return m.local;
  return nullptr;
}

char* open_import(uint64_t owner, uint64_t base, uint64_t id, int fd, const Shared& d, std::string* why) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (const Import& m : s.imports)
    if (m.owner == owner && m.base == base && m.id == id) {
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
  s.imports.push_back(Import{owner, base, id, p, local});
  return local;
}

bool close_import(uint64_t owner, uint64_t base, uint64_t id) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (size_t i = 0; i < s.imports.size(); ++i)
    if (s.imports[i].owner == owner && s.imports[i].base == base && s.imports[i].id == id) {
      hsa_amd_interop_unmap_buffer(s.imports[i].map);
      s.imports.erase(s.imports.begin() + (long)i);
      return true;
    }
  return false;
}

size_t imports() {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  return s.imports.size();
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
