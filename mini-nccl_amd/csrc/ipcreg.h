// ipcreg.h -- every export and import of device memory between this process and its peers.
//
// Two kinds, two mechanisms:
//
// * USER buffers (the read schedule loads its peers' send / recv): shared as dma-buf file
//   descriptors.  The owner exports an allocation once (hsa_amd_portable_export_dmabuf) and keeps
//   the descriptor while the allocation lives; it sends a duplicate to each peer process over a
//   Unix socket (SCM_RIGHTS, PeerBuffers), which maps it (hsa_amd_interop_map_buffer) and closes
//   the duplicate.  A dma-buf holds a reference on the memory, so an import stays valid -- and
//   keeps showing that allocation's memory -- even after the owner frees it, and a new allocation
//   at a re-used address is a new dma-buf.  Round 3's probe of hipIpc handles
//   (tools/probe_ipc_stress.cpp, profiles/r3_ipc_stress.txt) found the opposite for them: opens
//   that fail while another process closes, and re-opened imports or re-exported addresses that
//   map ANOTHER process's allocation; tools/probe_dmabuf.cpp runs the same pattern through
//   dma-bufs (profiles/r3_dmabuf_probe.txt).  (pidfd_getfd, which would need no socket, is
//   refused on the GPU boxes: EPERM.)  Imports are closed when the owner reports the allocation
//   freed (PeerBuffers), which releases its memory.
//
// * Communicator blocks (scratch, mailboxes, link-probe buffers): hipIpc handles, exported once
//   per block; blocks come from a pool that is never freed and their imports are never closed,
//   so re-creating a communicator re-uses them and no address is ever exported twice.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace mnccl {
namespace ipc {

// --- user buffers (dma-buf)
// One exported allocation, as its owner holds it (fd) and publishes it (ino, bo_off).
struct Shared {
  int32_t fd;       // the dma-buf descriptor in the owner's table, open while the allocation lives
  uint32_t gpu;     // the owner's GPU (PCI domain << 16 | bus << 8 | device << 3): see close_import
  uint64_t ino;     // the dma-buf's inode: what a received duplicate must name
  uint64_t bo_off;  // the allocation base's offset inside the dma-buf
};

// The export of allocation (base, id, size); created on first use.  False when it cannot be
// exported (not memory of a GPU, or this process holds too many exports): that call runs the ring.
bool export_allocation(uint64_t base, uint64_t id, uint64_t size, Shared* d, std::string* why = nullptr);
// A live export (as of the last reap_freed_exports) holding address p, with no HIP call.
bool find_live_export(uint64_t p, uint64_t* base, uint64_t* id, Shared* d);
// Finds exports whose allocation has been freed, closes their descriptors and appends them to
// the process's freed log.  Checked: every export holding one of `addrs` (a call's own buffers:
// a call must never publish the export of a freed allocation whose address a new one re-uses),
// then `batch` more in round-robin order -- so a call costs 2 + batch pointer queries whatever
// the number of live exports, and a freed allocation's export is found within
// live_exports / batch calls (its memory is pinned until then).
void reap_freed_exports(const uint64_t* addrs, int naddrs, size_t batch);
uint64_t liveness_queries();  // pointer queries made by reap_freed_exports, process-wide
// The freed log (base, id), append-only: every communicator reads it from its own cursor.
size_t freed_log_size();
std::pair<uint64_t, uint64_t> freed_log_at(size_t i);
size_t live_exports();

// Imports of peers' user allocations, keyed by the owner's process nonce and (base, id); the
// returned address corresponds to the owner's base.
char* find_import(uint64_t owner, uint64_t base, uint64_t id);
// Maps the owner's export from a received duplicate of its descriptor, fd, which this call
// always closes (a cached import is returned as is); nullptr on failure (*why set).  An import of
// memory of this process's own GPU is refused while the retired imports (close_import) already
// hold the retired budget's bytes: *budget_refused is then set (not an open failure: the call runs
// the ring on every rank, as for any mapping that does not happen).
char* open_import(uint64_t owner, uint64_t base, uint64_t id, int fd, const Shared& d, std::string* why,
                  bool* budget_refused = nullptr);
// Unmaps an import whose owner freed the allocation; the caller makes sure no kernel of this
// process still reads through it.  False if there was none.  An import of memory of this process's
// OWN GPU is retired instead -- never found again, kept mapped while the process lives (comm_closed
// keeps same-GPU imports too): the GPU driver gives a same-GPU import the exporter's buffer-object
// handle, so the owner's free and this unmap would delete that handle twice, and a buffer
// allocated in between loses it -- its later export fails or, worse, names another buffer
// (profiles/r5_export_alias.txt; DESIGN.md *Same-GPU handle loss*).  The second delete is left to
// the process's exit.  Retired mappings count against the import cap (kMaxImports) and their bytes
// against the retired budget (set_retired_budget): a co-located job whose peers keep freeing
// buffers the read schedule shared would otherwise pin that memory without bound.  A one-time
// warning comes at 3/4 of either bound.
bool close_import(uint64_t owner, uint64_t base, uint64_t id);
size_t imports();          // live imports
size_t retired_imports();  // same-GPU imports of freed allocations, held until the process exits
uint64_t retired_bytes();  // the bytes those keep mapped
// The retired budget (bytes; process-wide, the last communicator created sets it: Comm resolves
// MINI_NCCL_RETIRED_MB, by default 1/8 of the GPU's memory), and the same-GPU imports it refused.
void set_retired_budget(uint64_t bytes);
uint64_t retired_budget();
uint64_t budget_refusals();
uint64_t open_failures();  // user-buffer imports that failed in this process
// Exports (kMaxExports, 512) and imports (kMaxImports, live + retired) are capped per process; a
// refused one sends its call to the ring.  Counted here, warned about once per process.
constexpr size_t kMaxImports = 1024;
void note_cap_refusal(const std::string& what);
uint64_t cap_refusals();

// Communicator lifecycle.  Every live communicator registers the process nonces of its peers
// in other processes; comm_closed (once no kernel of the closing communicator runs) closes this
// process's imports of an owner no other live communicator shares (other GPUs' memory only, see
// close_import), and -- when it was the last
// live communicator of the process -- this process's exports too, so memory a caller frees
// after its last communicator is gone is released at once (the dma-bufs held it).
void comm_opened(const std::vector<uint64_t>& owners);
void comm_closed(const std::vector<uint64_t>& owners);

// --- communicator blocks (hipIpc), never freed while the process lives; a released block is
// handed to the next communicator asking for the same size and flags.  *h: the block's handle.
void* pool_acquire(size_t bytes, unsigned flags, hipIpcMemHandle_t* h, uint64_t* id);
void pool_release(void* p);
// A peer's block mapped here (opened once, never closed); nullptr on failure (*err set).
char* open_block(uint64_t owner, uint64_t base, uint64_t id, const hipIpcMemHandle_t& h, hipError_t* err);

}  // namespace ipc
}  // namespace mnccl
