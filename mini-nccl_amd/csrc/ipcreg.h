// ipcreg.h -- every HIP IPC export and import of this process, in one place.
//
// The reference exchanged and opened IPC handles of its buffers per call and closed them after
// (RDMATransport.h:231-255).  Measured on MI355X with 8 rank processes on one GPU
// (tools/probe_ipc_stress.cpp, profiles/r3_ipc_stress.txt), ROCm's IPC misbehaves in exactly the
// patterns that lifecycle produces:
//  * hipIpcOpenMemHandle fails ("invalid device pointer", HSA status 0x1001) while another
//    process closes an import at the same moment -- 0 failures in 56 000 opens once the opens
//    and closes of all processes are serialised;
//  * re-opening an allocation whose import was closed before, or exporting a new allocation at
//    an address this process exported before, can silently map ANOTHER process's allocation
//    (1 757 wrong values in 32 000 reads when imports are closed and re-opened per round);
//  * exporting a re-used address can fail, or produce a handle every importer rejects.
// So this process exports every allocation at most once and never exports an address it
// exported (or tried to export) before for another allocation; it keeps every import open until
// its owner reports the allocation freed (owners check their exports' liveness per call) and
// never re-opens an allocation it closed; communicator scratch and mailboxes come from a pool
// that is never freed, so re-creating a communicator re-uses allocations and imports instead of
// re-exporting addresses.  Callers serialise opens and closes across processes
// (PeerBuffers' board lock) where other processes may be closing.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <utility>
#include <vector>

namespace mnccl {
namespace ipc {

// --- exports (this process's allocations)
// The handle of allocation (base, id); exported on first use.  False (no handle) when the
// address was exported before for another allocation, or the export fails: such a buffer
// cannot be shared safely and its calls run a scratch schedule.
bool export_allocation(uint64_t base, uint64_t id, uint64_t size, hipIpcMemHandle_t* h);
// A live export (as of the last reap_freed_exports) holding address p: its base, id and handle,
// with no HIP call (a caller that reuses its buffers pays no pointer queries per call).
bool find_live_export(uint64_t p, uint64_t* base, uint64_t* id, hipIpcMemHandle_t* h);
// Finds the exports whose allocation has been freed (one pointer query per live export), moves
// them from the live list to the process's freed log; their addresses are never exported again.
void reap_freed_exports();
// The freed log (base, id), append-only: every communicator of the process reads it from its
// own cursor (any of them may have shared the allocation with its peers).
size_t freed_log_size();
std::pair<uint64_t, uint64_t> freed_log_at(size_t i);
size_t live_exports();

// --- imports (peers' allocations), keyed by the owner's process nonce and (base, id)
char* find_import(uint64_t owner, uint64_t base, uint64_t id);
// Opens and records the import (a cached one is returned as is); nullptr on failure (*err set).
// Never re-opens an import this process closed.  Caller holds the cross-process lock when
// other processes may be closing imports.
char* open_import(uint64_t owner, uint64_t base, uint64_t id, const hipIpcMemHandle_t& h, hipError_t* err);
// Closes an import whose owner freed the allocation; the caller makes sure no kernel still
// reads through it and holds the cross-process lock.  False if there was none.
bool close_import(uint64_t owner, uint64_t base, uint64_t id);
size_t imports();
uint64_t open_failures();  // hipIpcOpenMemHandle failures in this process

// --- device memory of communicators (scratch, mailboxes, probe buffers): never freed while the
// process lives; a released block is handed to the next communicator asking for the same size
// and flags, so its address is exported once and every peer's import of it stays valid.
// *h: the block's IPC handle (exported once).  Throws on allocation failure.
void* pool_acquire(size_t bytes, unsigned flags, hipIpcMemHandle_t* h, uint64_t* id);
void pool_release(void* p);

}  // namespace ipc
}  // namespace mnccl
