// ipcreg.cpp -- see ipcreg.h.
#include "ipcreg.h"

#include <algorithm>
#include <cstdio>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_set>

namespace mnccl {
namespace ipc {

namespace {

struct Export {
  uint64_t base, id, size;
  hipIpcMemHandle_t h;
};
struct Import {
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
struct Key {
  uint64_t owner, base, id;
  bool operator==(const Key& o) const { return owner == o.owner && base == o.base && id == o.id; }
};
struct KeyHash {
  size_t operator()(const Key& k) const { return std::hash<uint64_t>{}(k.owner * 0x9E3779B97F4A7C15ull ^ k.base ^ (k.id << 17)); }
};

struct State {
  std::mutex mu;
  std::vector<Export> exports;            // live exports
  std::vector<std::pair<uint64_t, uint64_t>> freed;  // exports found freed, in order
  std::unordered_set<uint64_t> exported;  // every address ever exported or tried (never again for another id)
  std::vector<Import> imports;
  std::unordered_set<Key, KeyHash> closed;  // imports closed: never re-opened
  std::vector<Block> pool;
  uint64_t open_failures = 0;
};

State& st() {
  static State* s = new State;  // never destroyed: imports / pool live until the process exits
  return *s;
}

}  // namespace

bool find_live_export(uint64_t p, uint64_t* base, uint64_t* id, hipIpcMemHandle_t* h) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (const Export& e : s.exports)
    if (p >= e.base && p - e.base < e.size) {
      *base = e.base;
      *id = e.id;
      *h = e.h;
      return true;
    }
  return false;
}

bool export_allocation(uint64_t base, uint64_t id, uint64_t size, hipIpcMemHandle_t* h) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (const Export& e : s.exports)
    if (e.base == base && e.id == id) {
      *h = e.h;
      return true;
    }
  if (!s.exported.insert(base).second) return false;  // this address was exported before (another allocation)
  if (hipIpcGetMemHandle(h, (void*)(uintptr_t)base) != hipSuccess) {
    (void)hipGetLastError();
    return false;  // the address stays marked: never tried again
  }
  s.exports.push_back(Export{base, id, size, *h});
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

char* open_import(uint64_t owner, uint64_t base, uint64_t id, const hipIpcMemHandle_t& h, hipError_t* err) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (const Import& m : s.imports)
    if (m.owner == owner && m.base == base && m.id == id) return m.local;
  if (s.closed.count(Key{owner, base, id})) {
    *err = hipErrorInvalidValue;  // re-opening a closed import can map the wrong memory
    return nullptr;
  }
  void* p = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    ++s.open_failures;
    *err = e;
    return nullptr;
  }
  s.imports.push_back(Import{owner, base, id, (char*)p});
  return (char*)p;
}

bool close_import(uint64_t owner, uint64_t base, uint64_t id) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  for (size_t i = 0; i < s.imports.size(); ++i)
    if (s.imports[i].owner == owner && s.imports[i].base == base && s.imports[i].id == id) {
      (void)hipIpcCloseMemHandle(s.imports[i].local);
      (void)hipGetLastError();
      s.imports.erase(s.imports.begin() + (long)i);
      s.closed.insert(Key{owner, base, id});
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
  for (int attempt = 0;; ++attempt) {
    const hipError_t e = flags ? hipExtMallocWithFlags(&p, bytes, flags) : hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      throw std::runtime_error(std::string("device allocation of ") + std::to_string(bytes) + " B: " +
                               hipGetErrorString(e));
    }
    if (!s.exported.count((uint64_t)(uintptr_t)p)) break;
    // an address this process exported before (a freed user buffer's): never export it again;
    // keep the block out of use (freeing it would hand the same address back)
    s.pool.push_back(Block{p, bytes, flags, 0, hipIpcMemHandle_t{}, true});
    if (attempt == 3) throw std::runtime_error("device allocation: no address that was not exported before");
  }
  hipError_t e = hipSuccess;
  unsigned long long bid = 0;
  e = hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p);
  if (e == hipSuccess) e = hipIpcGetMemHandle(h, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(p);
    throw std::runtime_error(std::string("IPC export of a communicator buffer: ") + hipGetErrorString(e));
  }
  s.exported.insert((uint64_t)(uintptr_t)p);
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

}  // namespace ipc
}  // namespace mnccl
