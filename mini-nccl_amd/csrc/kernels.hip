// kernels.hip -- the hot path, hand-written for CDNA4 (gfx950).
//
//  ring_kernel    persistent ring all-reduce (reference mini_nccl.cu:56-217 re-designed):
//                 one WAVE per pipeline (channel), each an independent slice pipeline; the
//                 reference's per-slice launches of wait_kernel (:22-30),
//                 elementwise_reduce_kernel (:43-47), the IPC memcpy (:131,:174) and
//                 set_flag_kernel (:32-36) become one launch per call in which every
//                 pipeline moves its slices through a `slots`-deep FIFO in the next
//                 rank's scratch with epoch-free monotone flags and explicit credits.
//                 Default geometry: 256 one-wave workgroups = one pipeline per CU.
//  read_kernel    the default: same association order, no scratch -- each rank loads its
//                 peers' send buffers over the links and pushes its results into their recv
//                 buffers (mapped by Comm per allocation).
//  read_start / read_grid / read_done   the read schedule's push form as three launches (the
//                 runtime form mncclAlgoReadGrid, for large calls): a grid of one-batch workgroups
//                 between a one-wave START and a one-wave DONE.
//  oneshot_kernel small calls the read schedule cannot take (host buffers): one hand-off -- every
//                 rank stores its pieces into every peer's scratch and folds the result itself,
//                 same association order.
//  local_reduce   the element-wise op alone: out = op(local, incoming), 16 B per lane.
//
// Memory-ordering protocol (cross-process, cross-device over xGMI):
//  * everything another rank writes in the ring lives in THIS rank's scratch / mailbox,
//    allocated hipDeviceMallocUncached: no cache of any agent keeps a copy of those lines;
//  * payload stores to a peer's slot are sc0 sc1 16-byte buffer stores (the instruction a
//    system-scope atomic store is; write-through, nothing left dirty in an L2); the wave
//    drains (s_waitcnt vmcnt(0) in asm, so the compiler cannot drop it) and lane 0 stores
//    the READY word with a system-scope atomic store;
//  * the consumer polls its own READY word with system-scope relaxed loads from lane 0
//    (s_sleep between polls) and reads the slot with sc0 sc1 loads (system-scope atomic
//    loads: they bypass L1/L2 whatever the mapping), so neither a release fence before
//    the flag nor an acquire fence after the poll is needed (cdna_hip_programming.md
//    Guideline 16's sc1 form); MINI_NCCL_SYS_FENCE=1 adds both (system scope);
//  * after the drain that follows the last load of a slot, lane 0 returns a CREDIT to
//    the sender; the sender reuses a slot only after the credit for the message that
//    last used it (seq - slots) arrived.
//  * flags are monotone 64-bit sequence numbers per (peer, pipeline) that continue across
//    calls (kept in device memory and advanced by the kernel itself, so graph replays stay
//    consistent); nothing is reset per call and stale flags cannot satisfy a wait.
//  * every spin is bounded (MINI_NCCL_TIMEOUT_MS via s_memrealtime) and also exits on
//    the host abort word or a peer's ABORT; the kernel always terminates.
//  * read_kernel loads the peers' send buffers with the same sc0 sc1 loads, after their START
//    (their send is in memory: every kernel before the call ended and wrote its data back),
//    and pushes its result slices into their recv with sc0 sc1 stores, drained before DONE.
//    Why the owner's later kernels then read the pushed bytes and not stale lines its L2 kept
//    of recv from before the call: a write that reaches memory from a CU under another L2
//    invalidates this L2's copy of the line, and an sc0 sc1 store is acknowledged only once it
//    has reached memory (measured across the eight L2s of one MI355X with no kernel boundary:
//    tools/probe_xcd_coherence.hip, profiles/r4_xcd_coherence.txt; DESIGN.md "Coherence of the
//    pushes").  Plain or non-temporal stores would NOT do: they are acknowledged from the
//    writer's L2 and the owner's stale line survives (same probe).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "kernels.h"
#include "schedule.h"

namespace mnccl {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef uint64_t u64;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int kAuxSys = 17;  // sc0 | sc1: system-coherent buffer access

struct bf16_t { uint16_t v; };

// ---------------------------------------------------------------- element ops
// c = op(a = local, b = incoming), reference mini_nccl.cu:38-41
template <typename T, int OPC> struct Op;
template <typename T> struct Op<T, kSum> { __device__ static T f(T a, T b) { return a + b; } };
template <typename T> struct Op<T, kProd> { __device__ static T f(T a, T b) { return a * b; } };
template <typename T> struct Op<T, kMax> { __device__ static T f(T a, T b) { return (a > b) ? a : b; } };
template <typename T> struct Op<T, kMin> { __device__ static T f(T a, T b) { return (a < b) ? a : b; } };
// int32 +,*: two's-complement wrap (no signed-overflow UB)
template <> struct Op<int32_t, kSum> {
  __device__ static int32_t f(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
};
template <> struct Op<int32_t, kProd> {
  __device__ static int32_t f(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
};
// bf16: widen (exact), op in f32, round to nearest even (correctly rounded: 24 >= 2*8+2) with
// the hardware's v_cvt_pk_bf16_f32 (gfx950; the compiler pairs two elements per instruction);
// NaN stays NaN (its payload is the hardware's, as IEEE leaves it to the implementation)
__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float((uint32_t)x.v << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  bf16_t r;
  r.v = __builtin_bit_cast(uint16_t, (__bf16)f);
  return r;
}
template <> struct Op<bf16_t, kSum> { __device__ static bf16_t f(bf16_t a, bf16_t b) { return f2bf(bf2f(a) + bf2f(b)); } };
template <> struct Op<bf16_t, kProd> { __device__ static bf16_t f(bf16_t a, bf16_t b) { return f2bf(bf2f(a) * bf2f(b)); } };
template <> struct Op<bf16_t, kMax> { __device__ static bf16_t f(bf16_t a, bf16_t b) { return (bf2f(a) > bf2f(b)) ? a : b; } };
template <> struct Op<bf16_t, kMin> { __device__ static bf16_t f(bf16_t a, bf16_t b) { return (bf2f(a) < bf2f(b)) ? a : b; } };

template <typename T> struct alignas(16) Pack16 { T x[16 / sizeof(T)]; };

template <typename T, int OPC>
__device__ __forceinline__ v4u reduce16(v4u a, v4u b) {
  Pack16<T> pa = __builtin_bit_cast(Pack16<T>, a);
  const Pack16<T> pb = __builtin_bit_cast(Pack16<T>, b);
#pragma unroll
  for (int i = 0; i < (int)(16 / sizeof(T)); ++i) pa.x[i] = Op<T, OPC>::f(pa.x[i], pb.x[i]);
  return __builtin_bit_cast(v4u, pa);
}

// ---------------------------------------------------------------- memory primitives
__device__ __forceinline__ u64 ld_sys(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(u64* p, u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ v4u ld_slot16(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSys);
}
__device__ __forceinline__ void st_slot16(rsrc_t r, uint32_t off, v4u v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSys);
}
// non-temporal buffer access (this rank's own bytes in the read kernel's short-slice forms:
// out-of-range lanes of a buffer access read 0 and write nothing, so those loops need no
// per-lane predicate)
constexpr int kAuxNt = 2;
__device__ __forceinline__ v4u ld_nt16(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxNt);
}
__device__ __forceinline__ void st_nt16(rsrc_t r, uint32_t off, v4u v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxNt);
}
// this rank's own send / recv bytes are touched once per call: non-temporal (see local reduce)
__device__ __forceinline__ v4u ld_g16(const char* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
}
__device__ __forceinline__ void st_g16(char* p, v4u v) { __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p)); }

// scalar (unaligned-count) path: one element per access
template <int SZ> struct Scal;
template <> struct Scal<2> {
  typedef uint16_t U;
  __device__ static U ld(rsrc_t r, uint32_t o) { return __builtin_amdgcn_raw_buffer_load_b16(r, o, 0, kAuxSys); }
  __device__ static void st(rsrc_t r, uint32_t o, U v) { __builtin_amdgcn_raw_buffer_store_b16(v, r, o, 0, kAuxSys); }
};
template <> struct Scal<4> {
  typedef uint32_t U;
  __device__ static U ld(rsrc_t r, uint32_t o) { return __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, kAuxSys); }
  __device__ static void st(rsrc_t r, uint32_t o, U v) { __builtin_amdgcn_raw_buffer_store_b32(v, r, o, 0, kAuxSys); }
};
template <> struct Scal<8> {
  typedef u64 U;
  __device__ static U ld(rsrc_t r, uint32_t o) {
    auto v = __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, kAuxSys);
    return __builtin_bit_cast(U, v);
  }
  __device__ static void st(rsrc_t r, uint32_t o, U v) {
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), r, o, 0, kAuxSys);
  }
};

// message `seq` from `src` to `dst` on pipeline w: in the receiver's scratch (schedule.h
// msg_slot_off); peer_scratch[rank] is this rank's own scratch
__device__ __forceinline__ char* msg_slot(const CollParams& p, int C, int src, int dst, int w, u64 seq) {
  return p.peer_scratch[dst] + msg_slot_off(C, p.nslots, p.slot_bytes, src, dst, w, seq);
}

// ---------------------------------------------------------------- bounded waits
struct Ctl {
  uint32_t* status;
  const uint32_t* host_abort;
  const u64* my_abort;
  uint64_t timeout_ticks;
  const u64* mbox;   // this rank's mailbox base (for the timeout diagnostic)
  uint32_t* claim;   // device word: the first give-up of the communicator takes it (claim_first)
};

// The first give-up -- a timeout, a peer's ABORT, the host's abort -- of any lane of any wave
// claims the status with one agent-scope compare-and-swap on a device word (the host-mapped
// status page itself takes no atomics: no PCIe atomics needed), so the cause and the diagnostic
// the host reports come from ONE lane: lanes of wave_wait_peers that give up in the same round,
// or a timeout racing a peer's ABORT, can no longer mix their words or overwrite the first cause
// (ADVICE r4).  The winner writes its words, then the status; the others just give up.
__device__ __forceinline__ bool claim_first(const Ctl& c) {
  uint32_t expected = 0;
  return __hip_atomic_compare_exchange_strong(c.claim, &expected, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
}

// a timed-out wait: which mailbox word, the target and the last value seen (host-mapped words
// 4..6 of the control page, plain system-scope stores), then the status
__device__ __forceinline__ void record_timeout(const Ctl& c, const u64* flag, u64 target, u64 seen) {
  if (!claim_first(c)) return;
  u64* diag = reinterpret_cast<u64*>(c.status + 4);
  __hip_atomic_store(diag + 0, (u64)(flag - c.mbox), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(diag + 1, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(diag + 2, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  st_sys32(c.status, kStatusTimeout);
}

// a peer's ABORT word seen: recorded only as the first cause (a peer's abort that echoes this
// rank's own timeout must not hide it); the word names the peer and its cause
__device__ __forceinline__ void note_remote_abort(const Ctl& c, u64 a) {
  if (!claim_first(c)) return;
  __hip_atomic_store(reinterpret_cast<u64*>(c.status + 4) + 3, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  st_sys32(c.status, kStatusRemoteAbort);
}

// lane-0 spin until *flag >= target; false on timeout / abort (status already set).  The
// spin is out of line (kept out of the message bodies' code and registers); Ctl goes by value
// so it travels in registers -- by reference it had to live in scratch memory.
#ifndef MNCCL_POLL_SLEEP
#define MNCCL_POLL_SLEEP 1  // s_sleep units (64 clocks each) between two polls of a flag
#endif
__device__ __noinline__ bool wait_ge_spin(const u64* flag, u64 target, const Ctl c) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t polls = 1;; ++polls) {
    __builtin_amdgcn_s_sleep(MNCCL_POLL_SLEEP);
    if (ld_sys(flag) >= target) return true;
    if ((polls & 63) == 0) {
      if (const u64 a = ld_sys(c.my_abort)) {
        note_remote_abort(c, a);
        return false;
      }
      if (ld_sys32(c.host_abort) != 0) {
        if (claim_first(c)) st_sys32(c.status, kStatusHostAbort);
        return false;
      }
      if (ld_sys32(c.status) != 0) return false;  // a sibling workgroup gave up
      if (__builtin_amdgcn_s_memrealtime() - t0 > c.timeout_ticks) {
        record_timeout(c, flag, target, ld_sys(flag));
        return false;
      }
    }
  }
}

// the common case (the flag is already there) costs one load and no call
__device__ __forceinline__ bool wait_ge(const u64* flag, u64 target, const Ctl& c) {
  if (ld_sys(flag) >= target) return true;
  return wait_ge_spin(flag, target, c);
}

// After a READY poll.  Every load of handed-off bytes is an sc0 sc1 buffer load of uncached
// scratch (never L1/L2 resident) and every producer stored them sc0 sc1 and drained before its
// flag (cdna_hip_programming.md G16 "sc1 loads replace the acquire"), so with
// MINI_NCCL_SYS_FENCE=0 the fence is only a compiler barrier; =1 keeps the system acquire.
__device__ __forceinline__ void acquire_sys(int sys_fence) {
  if (sys_fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// every storing wave: drain its stores (asm so the compiler cannot elide it)
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// lane 0, after its wave's drain
__device__ __forceinline__ void publish(u64* flag, u64 v, int sys_fence) {
  if (sys_fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  st_sys(flag, v);
}

// ---------------------------------------------------------------- wave-level sync
// A channel is ONE wave (64 lanes): lane 0 polls and signals, the wave's own s_waitcnt orders
// its memory operations, and no workgroup barrier is ever needed -- the waves of a
// workgroup (one by default) are independent pipelines.
__device__ __forceinline__ bool wave_wait_ge(const u64* flag, u64 target, const Ctl& c, int lane) {
  int ok = 1;
  if (lane == 0) ok = wait_ge(flag, target, c) ? 1 : 0;
  return __builtin_amdgcn_readfirstlane(ok) != 0;
}

// Lane l waits for its own word (the peers' READY / CREDIT / DONE words, one lane per peer):
// every peer's flag is polled in the same round instead of one peer after the other (n - 1
// uncached round trips in a row at every hand-off of the read and one-shot kernels).  True when
// every active lane's word arrived; a lane that gives up sets the status as wait_ge does.
// check_abort: lane 63 (never a peer's: at most 16 ranks) also reads this rank's ABORT word in
// the same round -- a wait whose flags are all there already never spins, so without it a rank
// that comes late to a call its peer gave up on (the peer raised its ABORT word, its messages
// already sent) would complete the call as if nothing had happened.
__device__ __forceinline__ bool wave_wait_peers(const u64* flag, u64 target, bool active, const Ctl& c, int lane,
                                                bool check_abort) {
  int bad = 0;
  if (active) {
    bad = wait_ge(flag, target, c) ? 0 : 1;
  } else if (check_abort && lane == 63) {
    if (const u64 a = ld_sys(c.my_abort)) {
      note_remote_abort(c, a);
      bad = 1;
    }
  }
  return __builtin_amdgcn_ballot_w64(bad != 0) == 0;
}

// Registered-window calls (Comm::allreduce's fast path) are launched without a host rendezvous: the
// peers' buffer addresses come from the windows every rank registered together, on the promise
// that every rank passes the same windows, offsets, count, dtype and op.  The promise is checked
// here, on the device, before any peer buffer is touched: START carries the caller's signature
// (a hash of those, never 0) in word kSigWord of the READY line, stored just before the flag (no
// drain between the two: the signature may land after the flag).  After every peer's START, lane
// q waits for peer q's signature word to be non-zero, compares it with this rank's and clears it
// (so a later call never meets a stale one: a peer writes its next signature only after this
// call's DONE).  Any difference -- seen by every rank alike, as every rank compares every pair it
// is part of -- gives up the call with kStatusMismatch (ncclInvalidUsage).
// The START of read_start_kernel; read_kernel writes the same stores inline, its flag value read
// inside the peer-lane branch (read outside it, from a clamped LDS index, the persistent kernel's
// fold spilled 36 registers to scratch at the 256-register bound).
__device__ __forceinline__ void send_start(const CollParams& p, int C, int lane, u64 v, int w) {
  const int n = p.n, r = p.rank;
  if (lane < n && lane != r && p.sig) st_sys(p.peer_mbox[lane] + mbox_ready(C, r, w) + kSigWord, p.sig);
  if (lane < n && lane != r) st_sys(p.peer_mbox[lane] + mbox_ready(C, r, w), v);
}

// lane q: does peer q's signature differ from mine?  Clears the word.  Out of line: kept out of
// the persistent kernel's register allocation, whose fold sits at the 256-register bound
__device__ __noinline__ bool sig_differs(u64* word, u64 sig) {
  const bool bad = ld_sys(word) != sig;
  st_sys(word, 0);
  return bad;
}

// after every peer's START: false (status claimed, nothing touched) if some peer's signature differs.
// *seen: kStatusMismatch when this wave saw the difference itself -- its ABORT word then carries
// that cause even if another wave won the claim and its status store has not landed yet (ADVICE
// r5: re-reading the shared status could send a bare abort, and the peer report ncclRemoteError)
__device__ __forceinline__ bool starts_agree(const CollParams& p, const Ctl& c, int C, int lane, int w,
                                             uint32_t* seen) {
  if (!p.sig) return true;
  const int n = p.n, r = p.rank;
  const bool peer = lane < n && lane != r;
  u64* word = p.mbox + mbox_ready(C, peer ? lane : 0, w) + kSigWord;
  if (!wave_wait_peers(word, 1, peer, c, lane, false)) return false;  // (status set: timeout / abort)
  bool bad = false;
  if (peer) bad = sig_differs(word, p.sig);
  if (__builtin_amdgcn_ballot_w64(bad) == 0) return true;
  *seen = kStatusMismatch;
  if (lane == 0 && claim_first(c)) st_sys32(c.status, kStatusMismatch);
  return false;
}

// ---------------------------------------------------------------- message bodies (one wave)
enum : int { kHasLocal = 1, kHasIn = 2, kWritesRecv = 4, kSends = 8, kReduces = 16 };
template <int KIND> struct KindBits;
template <> struct KindBits<kSend> { static constexpr int v = kHasLocal | kSends; };
template <> struct KindBits<kReduceSend> { static constexpr int v = kHasLocal | kHasIn | kSends | kReduces; };
template <> struct KindBits<kReduceCopySend> { static constexpr int v = kHasLocal | kHasIn | kSends | kReduces | kWritesRecv; };
template <> struct KindBits<kCopySend> { static constexpr int v = kHasIn | kSends | kWritesRecv; };
template <> struct KindBits<kCopy> { static constexpr int v = kHasIn | kWritesRecv; };

constexpr int kU = 8;  // 16-byte vectors per lane per batch: 8 KiB per wave in flight per stream

template <typename T, int OPC, int KIND>
__device__ __forceinline__ void vec_one(const char* lsrc, char* ldst, rsrc_t in, rsrc_t out, uint32_t i) {
  constexpr int B = KindBits<KIND>::v;
  v4u l, x, v;
  if (B & kHasLocal) l = ld_g16(lsrc + (size_t)i * 16);
  if (B & kHasIn) x = ld_slot16(in, i * 16);
  if (B & kReduces) v = reduce16<T, OPC>(l, x);
  else if (B & kHasIn) v = x;
  else v = l;
  if (B & kWritesRecv) st_g16(ldst + (size_t)i * 16, v);
  if (B & kSends) st_slot16(out, i * 16, v);
}

template <typename T, int OPC, int KIND>
__device__ __forceinline__ void move_scalar(const char* __restrict__ lsrc, char* __restrict__ ldst, rsrc_t in,
                                            rsrc_t out, uint32_t nbytes, int lane, uint32_t off0);

// 16-byte vectors over the message, then its last (nbytes % 16) bytes element by element.
// The local side (send / recv) may be element- but not 16-byte-aligned (4-byte-aligned
// dwordx4 accesses are valid on gfx950); the slot side is always 16-byte-aligned.
template <typename T, int OPC, int KIND, int UB = kU>
__device__ __forceinline__ void move_vec(const char* __restrict__ lsrc, char* __restrict__ ldst, rsrc_t in,
                                         rsrc_t out, uint32_t nbytes, int lane) {
  constexpr int B = KindBits<KIND>::v;
  const uint32_t nvec = nbytes >> 4;
  uint32_t b = 0;
  for (; b + 64 * UB <= nvec; b += 64 * UB) {  // full batches: every lane issues UB loads per stream
    v4u l[UB], x[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const uint32_t i = b + (uint32_t)(u * 64 + lane);
      if (B & kHasLocal) l[u] = ld_g16(lsrc + (size_t)i * 16);
      if (B & kHasIn) x[u] = ld_slot16(in, i * 16);
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const uint32_t i = b + (uint32_t)(u * 64 + lane);
      v4u v;
      if (B & kReduces) v = reduce16<T, OPC>(l[u], x[u]);
      else if (B & kHasIn) v = x[u];
      else v = l[u];
      if (B & kWritesRecv) st_g16(ldst + (size_t)i * 16, v);
      if (B & kSends) st_slot16(out, i * 16, v);
    }
  }
  for (uint32_t i = b + (uint32_t)lane; i < nvec; i += 64) vec_one<T, OPC, KIND>(lsrc, ldst, in, out, i);
  if (nbytes & 15u) move_scalar<T, OPC, KIND>(lsrc, ldst, in, out, nbytes, lane, nvec * 16);
}

// elements [off0 / sizeof(T), nbytes / sizeof(T)) of the message, one per lane
template <typename T, int OPC, int KIND>
__device__ __forceinline__ void move_scalar(const char* __restrict__ lsrc, char* __restrict__ ldst, rsrc_t in,
                                            rsrc_t out, uint32_t nbytes, int lane, uint32_t off0) {
  constexpr int B = KindBits<KIND>::v;
  typedef typename Scal<sizeof(T)>::U U;
  const uint32_t ne = nbytes / sizeof(T);
  for (uint32_t i = off0 / sizeof(T) + lane; i < ne; i += 64) {
    U l = 0, x = 0, v;
    if (B & kHasLocal) l = reinterpret_cast<const U*>(lsrc)[i];
    if (B & kHasIn) x = Scal<sizeof(T)>::ld(in, i * (uint32_t)sizeof(T));
    if (B & kReduces) v = __builtin_bit_cast(U, Op<T, OPC>::f(__builtin_bit_cast(T, l), __builtin_bit_cast(T, x)));
    else if (B & kHasIn) v = x;
    else v = l;
    if (B & kWritesRecv) reinterpret_cast<U*>(ldst)[i] = v;
    if (B & kSends) Scal<sizeof(T)>::st(out, i * (uint32_t)sizeof(T), v);
  }
}

template <typename T, int OPC, bool VEC, int KIND, int UB = kU>
__device__ __forceinline__ void move(const char* lsrc, char* ldst, rsrc_t in, rsrc_t out, uint32_t nbytes, int lane) {
  if (VEC) move_vec<T, OPC, KIND, UB>(lsrc, ldst, in, out, nbytes, lane);
  else move_scalar<T, OPC, KIND>(lsrc, ldst, in, out, nbytes, lane, 0);
}

// the ABORT word a giving-up rank writes into its peers' mailboxes: its rank + 1 (never 0) and
// its own status (why it gave up), plus the cause this wave saw itself (`seen`) -- the peers
// report both (Comm::check_status)
__device__ __forceinline__ u64 abort_word(const CollParams& p, uint32_t seen = 0) {
  return ((u64)(ld_sys32(p.status) | seen) << 32) | (u64)(p.rank + 1);
}

__device__ __forceinline__ void abort_peers(const CollParams& p, int C, int a, int b) {
  st_sys(p.peer_mbox[a] + mbox_abort(p.n, C), abort_word(p));
  st_sys(p.peer_mbox[b] + mbox_abort(p.n, C), abort_word(p));
}

// the host watchdog's deadline starts when the kernel does (Comm::wait_for): one posted write
__device__ __forceinline__ void signal_start(const CollParams& p) {
  if (blockIdx.x == 0 && threadIdx.x == 0) st_sys32(p.started, p.call_seq);
}

// The count % n elements past the chunks keep this rank's own input (api.cpp:173-175 copies the
// whole buffer, mini_nccl.cu:69 never touches the tail): pipeline 0 copies them, byte by byte
// (under 128 bytes), so a call is one launch.  Measured on the one-GPU box: a copy kernel queued
// in front of a persistent kernel can find no room left by the co-located ranks' persistent
// kernels, which then wait for this rank's forever (tools/dr_probe.py,
// profiles/r3_device_rendezvous.txt: 2 of 2 runs stalled with the copy, 4 of 4 clean without).
__device__ __forceinline__ void copy_tail(const CollParams& p, int w, int lane) {
  if (w != 0 || p.tail_bytes == 0) return;
  const uint64_t off = p.chunk_bytes * (uint64_t)p.n;
  for (uint64_t i = (uint64_t)lane; i < p.tail_bytes; i += 64) p.recv[off + i] = p.send[off + i];
}

// channel geometry: one channel per wave
struct WaveId {
  int lane, wv, w, C;
};
__device__ __forceinline__ WaveId wave_id() {
  WaveId id;
  id.lane = threadIdx.x & 63;
  const int W = blockDim.x >> 6;
  id.wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  id.w = __builtin_amdgcn_readfirstlane(blockIdx.x * W + id.wv);
  id.C = gridDim.x * W;
  return id;
}

// ---------------------------------------------------------------- ring kernel
// Every rank's persistent kernel waits for its peers' kernels, so on a GPU that several rank
// processes share (the reference's perf_test topology, the one-GPU test box) all of them must be
// resident at once: 8 ranks x 256 one-wave pipelines = 2 waves on each of the 1024 SIMDs.  The
// collective kernels therefore ask for >= 2 waves per SIMD (<= 256 VGPRs + AGPRs per wave; a
// read-kernel variant at 256 + 1 AGPR fitted only one, and 8 co-located ranks crawled until
// their watchdogs fired).  With one rank per GPU this costs nothing.  (kernels.h
// kMinWavesPerSimd; Comm caps a call's pipelines so that every rank's waves fit, Comm::run_pipes.)

template <typename T, int OPC, bool VEC>
__global__ void __launch_bounds__(kMaxThreads, kMinWavesPerSimd) ring_kernel(CollParams p) {
  signal_start(p);
  const WaveId id = wave_id();
  // C: the communicator's pipelines (mailbox, scratch and counter layout); A: the ones this call
  // runs (its grid, schedule.h call_pipelines), slice s on pipeline s mod A
  const int lane = id.lane, w = id.w, C = p.pipes, A = id.C;
  const int n = p.n, r = p.rank, K = p.nslots;
  copy_tail(p, w, lane);
  const int prev = mod_n(r - 1, n), next = mod_n(r + 1, n);
  const Ctl ctl{p.status, p.host_abort, p.mbox + mbox_abort(n, C), p.timeout_ticks, p.mbox, p.claim};
  // per-pair message counters: the FIFO to `next` and the FIFO from `prev` on this channel
  u64* tx_ctr = p.tx_seq + (u64)next * C + w;
  u64* rx_ctr = p.rx_seq + (u64)prev * C + w;
  const u64 tx_base = *tx_ctr, rx_base = *rx_ctr;
  const int mpi = ring_msgs_per_iter(n);
  const u64* my_ready = p.mbox + mbox_ready(C, prev, w);
  const u64* my_credit = p.mbox + mbox_credit(n, C, next, w);
  u64* out_ready = p.peer_mbox[next] + mbox_ready(C, r, w);
  u64* out_credit = p.peer_mbox[prev] + mbox_credit(n, C, r, w);
  const int nops = ring_num_ops(n);

  for (uint32_t it = 0; it < p.iters; ++it) {
    const u64 s = (u64)it * A + w;
    const uint32_t len = (uint32_t)slice_len(p.chunk_bytes, p.slice_bytes, s);
    const u64 soff = s * p.slice_bytes;
    const u64 itoff = (u64)it * mpi;
    for (int k = 0; k < nops; ++k) {
      const RingOp o = ring_op(n, r, k);
      const u64 rseq = rx_base + itoff + (u64)o.recv_msg, sseq = tx_base + itoff + (u64)o.send_msg;
      bool ok = true;
      if (o.recv_msg >= 0) ok = wave_wait_ge(my_ready, rseq + 1, ctl, lane);
      if (ok && o.send_msg >= 0 && sseq + 1 > (u64)K) ok = wave_wait_ge(my_credit, sseq + 1 - K, ctl, lane);
      if (!ok) {
        if (lane == 0) abort_peers(p, C, prev, next);
        return;
      }
      if (o.recv_msg >= 0) acquire_sys(p.sys_fence);
      if (len) {
        const u64 coff = (u64)o.chunk * p.chunk_bytes + soff;
        const rsrc_t in = make_rsrc(msg_slot(p, C, prev, r, w, rseq), len);
        const rsrc_t out = make_rsrc(msg_slot(p, C, r, next, w, sseq), len);
        const char* lsrc = p.send + coff;
        char* ldst = p.recv + coff;
        switch (o.kind) {
          case kSend: move<T, OPC, VEC, kSend>(lsrc, ldst, in, out, len, lane); break;
          case kReduceSend: move<T, OPC, VEC, kReduceSend>(lsrc, ldst, in, out, len, lane); break;
          case kReduceCopySend: move<T, OPC, VEC, kReduceCopySend>(lsrc, ldst, in, out, len, lane); break;
          case kCopySend: move<T, OPC, VEC, kCopySend>(lsrc, ldst, in, out, len, lane); break;
          default: move<T, OPC, VEC, kCopy>(lsrc, ldst, in, out, len, lane); break;
        }
      }
      drain_stores();  // every load of the slot has returned and every store has landed
      if (lane == 0) {
        if (o.send_msg >= 0) publish(out_ready, sseq + 1, p.sys_fence);
        if (o.recv_msg >= 0) st_sys(out_credit, rseq + 1);
      }
    }
  }
  if (lane == 0) {
    *tx_ctr = tx_base + (u64)p.iters * mpi;
    *rx_ctr = rx_base + (u64)p.iters * mpi;
  }
}

constexpr int kMaxWaves = kMaxThreads / 64;

// ---------------------------------------------------------------- read kernel
// MINI_NCCL_ALGO=read (schedule.h): no scratch.  Comm maps every peer's send and recv buffers
// (dma-buf imports, negotiated per call); rank r folds slice s of its own chunk r straight from
// the peers' send buffers (sc0 sc1 loads over the links, in ring order) and stores the result
// into its own recv and into every peer's recv with sc0 sc1 stores (the push form; 4.0-5.x also
// built a load form, every peer copying the result out of the owner's recv after a READY: 1.1-1.45x
// slower everywhere it was measured, removed in 6.0).
//
// Fold of slice `nbytes` at byte `coff` of chunk r: acc = op(x_q, acc) in ring order.
template <typename T, int OPC>
__device__ __forceinline__ void read_fold_scalar(const CollParams& p, uint64_t coff, uint32_t nbytes, int lane,
                                                 uint32_t off0) {
  const int n = p.n, r = p.rank;
  typedef typename Scal<sizeof(T)>::U Us;
  const rsrc_t out = make_rsrc(p.recv + coff, nbytes);
  const uint32_t ne = nbytes / sizeof(T);
  for (uint32_t i = off0 / sizeof(T) + lane; i < ne; i += 64) {
    T acc = reinterpret_cast<const T*>(p.send + coff)[i];
    for (int k = 1; k < n; ++k) {
      const rsrc_t in = make_rsrc(p.peer_send[direct_peer(n, r, k)] + coff, nbytes);
      acc = Op<T, OPC>::f(__builtin_bit_cast(T, Scal<sizeof(T)>::ld(in, i * (uint32_t)sizeof(T))), acc);
    }
    Scal<sizeof(T)>::st(out, i * (uint32_t)sizeof(T), __builtin_bit_cast(Us, acc));
  }
}

// Vectors per lane per batch of the read kernel's fold past 8 ranks: 16 (two peers' 16 KiB in
// flight per wave).  Latency insurance for loads that cross xGMI: a wave's rate is its bytes in
// flight over the load's round trip, so twice the scratch kernels' batches halve the pipelines a
// link needs to stay busy; measured free on the one-GPU proxy (profiles/r2_read_batch_variants.txt).
#ifndef MNCCL_READ_FOLD_U
#define MNCCL_READ_FOLD_U 16
#endif
constexpr int kReadFoldU = MNCCL_READ_FOLD_U;

// Short slices (below one full batch, and the part of a slice past its full batches): every
// peer's vectors of a step are loaded at once -- (n-1) x kWideV KiB in flight per wave -- so a
// step costs one load round trip, where a peer-by-peer loop of single vectors cost one per peer
// and vector (a 1 KiB slice over 7 peers: 1 round trip instead of 7 in the fold, and in the
// copy).  The buffer resources end at the slice's last whole vector: lanes past it load 0 and
// store nothing (no predicate, so no load waits on another); the last nbytes % 16 bytes go
// element by element as before.
constexpr int kWideV = 2;
constexpr int kWideG = 7;  // peers per group (a node's n - 1): their buffer descriptors stay in SGPRs

template <typename T, int OPC>
__device__ __forceinline__ void read_fold_wide(const CollParams& p, uint64_t coff, uint32_t vlo, uint32_t nvec,
                                               int lane) {
  const int n = p.n, r = p.rank;
  const uint32_t vb = nvec * 16;
  const rsrc_t loc = make_rsrc(p.send + coff, vb), out = make_rsrc(p.recv + coff, vb);
  for (uint32_t b = vlo; b < nvec; b += 64 * kWideV) {
    v4u acc[kWideV];
#pragma unroll
    for (int u = 0; u < kWideV; ++u) acc[u] = ld_nt16(loc, (b + (uint32_t)(u * 64 + lane)) * 16);
    for (int k0 = 1; k0 < n; k0 += kWideG) {  // ring order: groups in turn, peers in turn
      v4u x[kWideG][kWideV];
#pragma unroll
      for (int g = 0; g < kWideG; ++g)
        if (k0 + g < n) {
          const rsrc_t in = make_rsrc(p.peer_send[direct_peer(n, r, k0 + g)] + coff, vb);
#pragma unroll
          for (int u = 0; u < kWideV; ++u) x[g][u] = ld_slot16(in, (b + (uint32_t)(u * 64 + lane)) * 16);
        }
#pragma unroll
      for (int g = 0; g < kWideG; ++g)
        if (k0 + g < n) {
#pragma unroll
          for (int u = 0; u < kWideV; ++u) acc[u] = reduce16<T, OPC>(x[g][u], acc[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < kWideV; ++u) st_slot16(out, (b + (uint32_t)(u * 64 + lane)) * 16, acc[u]);
  }
}

// The fold of a slice from 4 to 8 ranks (a node): each batch loads V vectors per lane from EVERY
// peer at once, and the next batch's loads leave before this batch is folded (two register
// sets).  The fold's order is fixed (ring order), its load order is not: loaded one peer after
// the other, every wave of every rank would start its batches at peer r+1 and the ranks'
// incoming traffic would sit on one link at a time -- over xGMI, a seventh of a rank's links
// at 8 ranks; loaded together, every link carries its share all the time.  G peer slots, V
// vectors: (n-1) x V KiB per batch, two batches in flight per wave (2 ranks: 12 KiB, 3: 8 KiB
// per peer, 4-5: 4 KiB, 6-8: 3 KiB; all within 256 registers without spilling).  Measured on
// the one-GPU proxy against the one-peer-ahead batches below (used past 8 ranks): equal at 2
// and 3 ranks (profiles/r2_read_fold_all_n23_ab.txt), 0.94-1.05x at 4 and 8.
#ifndef MNCCL_READ_FOLD_ALL
#define MNCCL_READ_FOLD_ALL 1
#endif
#ifndef MNCCL_FOLD_ALL_MIN_N
#define MNCCL_FOLD_ALL_MIN_N 2
#endif
// The read schedule's second half: each rank pushes its result slices into every peer's recv
// (sc0 sc1 stores, straight from the fold's registers) -- no per-iteration READY, no copy phase,
// and each GPU's HBM moves 2n chunks per call (a load form, every peer reading the result back
// from the owner's recv, moved 3n-1 and was 1.1-1.45x slower: profiles/r3_read_push_ab.txt); DONE
// also means "my pushes into your recv have landed", and every rank waits for every peer's DONE
// before its kernel ends.  Only rank r ever writes chunk r of any recv (in place: after its own
// loads of that slice).  The pushes are sc0 sc1 stores: each is acknowledged once it reached the
// owner's memory, which drops any copy of the line the owner's L2 kept (file header), and this
// rank never reads the pushed ranges inside the call.

// The fold's store into this rank's OWN recv: no peer reads it inside the call (the pushes are the
// peers' copies), so it needs no system-scope write-through -- MNCCL_OWN_NT=1 stores it
// non-temporal, as the local reduce does (an A/B knob; the pushes stay sc0 sc1).
#ifndef MNCCL_OWN_NT
#define MNCCL_OWN_NT 0
#endif
__device__ __forceinline__ void st_own16(rsrc_t r, uint32_t off, v4u v) {
  if (MNCCL_OWN_NT) st_nt16(r, off, v);
  else st_slot16(r, off, v);
}

template <typename T, int OPC, int G, int V>
__device__ __forceinline__ void read_fold_all(const CollParams& p, uint64_t coff, uint32_t nvec, int lane) {
  constexpr uint32_t step = 64 * V;
  const int n = p.n, r = p.rank, w = wave_id().w;
  const uint32_t vb = nvec * 16;
  const rsrc_t loc = make_rsrc(p.send + coff, vb), out = make_rsrc(p.recv + coff, vb);
  rsrc_t in[G];
#pragma unroll
  for (int g = 0; g < G; ++g) in[g] = make_rsrc(p.peer_send[direct_peer(n, r, 1 + (g + 1 < n ? g : 0))] + coff, vb);
  // the result also goes to the same offset of every peer's recv (pipeline w starts at peer
  // w mod n-1, so a rank's pipelines spread their pushes over all links)
  rsrc_t pout[G];
#pragma unroll
  for (int g = 0; g < G; ++g)
    pout[g] = make_rsrc(p.peer_recv[direct_peer(n, r, 1 + (g + 1 < n ? (g + w) % (n - 1) : 0))] + coff, vb);
  v4u xa[G][V], aa[V], xb[G][V], ab[V];
  auto load = [&](v4u(&x)[G][V], v4u(&a)[V], uint32_t b) {
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (g + 1 < n) {
#pragma unroll
        for (int u = 0; u < V; ++u) x[g][u] = ld_slot16(in[g], (b + (uint32_t)(u * 64 + lane)) * 16);
      }
#pragma unroll
    for (int u = 0; u < V; ++u) a[u] = ld_nt16(loc, (b + (uint32_t)(u * 64 + lane)) * 16);
  };
  auto fold_store = [&](v4u(&x)[G][V], v4u(&a)[V], uint32_t b) {
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (g + 1 < n) {
#pragma unroll
        for (int u = 0; u < V; ++u) a[u] = reduce16<T, OPC>(x[g][u], a[u]);
      }
#pragma unroll
    for (int u = 0; u < V; ++u) st_own16(out, (b + (uint32_t)(u * 64 + lane)) * 16, a[u]);
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (g + 1 < n) {
#pragma unroll
        for (int u = 0; u < V; ++u) st_slot16(pout[g], (b + (uint32_t)(u * 64 + lane)) * 16, a[u]);
      }
  };
  // The next batch's loads are issued unconditionally: past the slice they fall outside the
  // buffer resources' range, return 0 and touch no memory.  A conditional prefetch made hipcc
  // wait vmcnt(0) where the two paths join -- for the prefetch itself and, as loads and stores
  // share vmcnt, for every store of the batch before: the double buffer then never overlapped
  // (tools/mix_probe.hip "persist2"; profiles/r4_vmcnt.txt).  A slice is at most kMaxSlice, so
  // the past-the-end offsets stay below 2^32.
  uint32_t b = 0;
  load(xa, aa, b);
  for (;;) {
    load(xb, ab, b + step);
    fold_store(xa, aa, b);
    if ((b += step) >= nvec) break;
    load(xa, aa, b + step);
    fold_store(xb, ab, b);
    if ((b += step) >= nvec) break;
  }
}

// Returns the leading bytes of the slice whose result it also pushed to the peers.
template <typename T, int OPC, bool VEC>
__device__ __forceinline__ uint32_t read_fold(const CollParams& p, uint64_t coff, uint32_t nbytes, int lane) {
  if (!VEC) {
    read_fold_scalar<T, OPC>(p, coff, nbytes, lane, 0);
    return 0;
  }
  const int n = p.n, r = p.rank;
  const uint32_t nvec = nbytes >> 4;
  if (MNCCL_READ_FOLD_ALL && n >= MNCCL_FOLD_ALL_MIN_N && n <= 8) {
    // (2-byte types widen to f32 in reduce16: fewer vectors per peer keep the bf16 / fp16
    // variants within 256 registers without spilling)
    constexpr int h = sizeof(T) == 2 ? 1 : 0;
    if (!nvec) {
    } else if (n == 2) read_fold_all<T, OPC, 1, 12 - 4 * h>(p, coff, nvec, lane);
    else if (n == 3) read_fold_all<T, OPC, 2, 8 - 2 * h>(p, coff, nvec, lane);
    else if (n <= 5) read_fold_all<T, OPC, 4, 4 - h>(p, coff, nvec, lane);
    else read_fold_all<T, OPC, 7, 3 - h>(p, coff, nvec, lane);
    if (nbytes & 15u) read_fold_scalar<T, OPC>(p, coff, nbytes, lane, nvec * 16);
    return nvec * 16;
  }
  constexpr int U = kReadFoldU;
  const rsrc_t out = make_rsrc(p.recv + coff, nbytes);
  const char* lsrc = p.send + coff;
  uint32_t b = 0;
  // full batches: the n-1 remote streams are issued back to back (one peer ahead of the fold)
  for (; b + 64 * U <= nvec; b += 64 * U) {
    v4u acc[U], cur[U], nxt[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = ld_g16(lsrc + (size_t)(b + (uint32_t)(u * 64 + lane)) * 16);
    {
      const rsrc_t in = make_rsrc(p.peer_send[direct_peer(n, r, 1)] + coff, nbytes);
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = ld_slot16(in, (b + (uint32_t)(u * 64 + lane)) * 16);
    }
    for (int k = 1; k < n; ++k) {
      if (k + 1 < n) {
        const rsrc_t in = make_rsrc(p.peer_send[direct_peer(n, r, k + 1)] + coff, nbytes);
#pragma unroll
        for (int u = 0; u < U; ++u) nxt[u] = ld_slot16(in, (b + (uint32_t)(u * 64 + lane)) * 16);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = reduce16<T, OPC>(cur[u], acc[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st_slot16(out, (b + (uint32_t)(u * 64 + lane)) * 16, acc[u]);
  }
  if (b < nvec) read_fold_wide<T, OPC>(p, coff, b, nvec, lane);
  if (nbytes & 15u) read_fold_scalar<T, OPC>(p, coff, nbytes, lane, nvec * 16);
  return 0;
}

// The folds that do not push as they fold (scalar, past 8 ranks): bytes [off0, nbytes) of my result
// slice, read back from my recv (stored and drained) into every peer's recv
template <typename T, bool VEC>
__device__ __forceinline__ void read_push_rest(const CollParams& p, uint64_t coff, uint32_t nbytes, uint32_t off0,
                                               int lane) {
  const int n = p.n, r = p.rank;
  const rsrc_t src = make_rsrc(p.recv + coff, nbytes);
  // 16-byte vectors only where the buffers are dword-aligned (VEC), element by element otherwise
  const uint32_t v0 = VEC ? (off0 + 15u) >> 4 : 0, v1 = VEC ? nbytes >> 4 : 0;
  for (int k = 1; k < n; ++k) {
    const rsrc_t dst = make_rsrc(p.peer_recv[direct_peer(n, r, k)] + coff, nbytes);
    for (uint32_t i = v0 + (uint32_t)lane; i < v1; i += 64) st_slot16(dst, i * 16, ld_slot16(src, i * 16));
    const uint32_t e0 = (v1 > v0 ? v1 * 16 : off0) / sizeof(T), ne = nbytes / sizeof(T);
    for (uint32_t i = e0 + (uint32_t)lane; i < ne; i += 64)
      Scal<sizeof(T)>::st(dst, i * (uint32_t)sizeof(T), Scal<sizeof(T)>::ld(src, i * (uint32_t)sizeof(T)));
  }
}

// Messages per (pair, pipeline) and call: START (my send is readable and my recv writable: the
// call began on my stream), DONE (I no longer read your buffers, my pushes into your recv have
// landed: your stream may go on).  Per pipeline: START, F0 F1 ... F(I-1), DONE.  The READY word
// counts iters + 2 messages per call (it jumps from START to DONE: the count the 4.0-5.x load
// form's per-iteration READYs kept, which the scratch schedules' slot counters still follow);
// DONE also returns credits for every message (the counters continue across calls, whatever the
// schedule).
template <typename T, int OPC, bool VEC>
__global__ void __launch_bounds__(kMaxThreads, kMinWavesPerSimd) read_kernel(CollParams p) {
  signal_start(p);
  const WaveId id = wave_id();
  // C: the communicator's pipelines (mailbox and counter layout); A: the ones this call runs
  // (its grid), slice s on pipeline s mod A
  const int lane = id.lane, w = id.w, C = p.pipes, A = id.C, wv = id.wv;
  const int n = p.n, r = p.rank;
  copy_tail(p, w, lane);
  __shared__ u64 s_tx[kMaxWaves][kMaxRanks], s_rx[kMaxWaves][kMaxRanks];
  u64* tx = s_tx[wv];
  u64* rx = s_rx[wv];
  const Ctl ctl{p.status, p.host_abort, p.mbox + mbox_abort(n, C), p.timeout_ticks, p.mbox, p.claim};
  const uint32_t iters = p.iters;
  const u64 mpc = read_msgs_per_call(iters);
  uint32_t seen = 0;  // a cause this wave saw itself (starts_agree), for its ABORT word
  if (lane < n) {
    tx[lane] = p.tx_seq[(u64)lane * C + w];
    rx[lane] = p.rx_seq[(u64)lane * C + w];
  }
  __builtin_amdgcn_wave_barrier();
  // START to every peer (with the call's signature on a registered-window call), then wait for theirs
  if (lane < n && lane != r) {
    if (p.sig) st_sys(p.peer_mbox[lane] + mbox_ready(C, r, w) + kSigWord, p.sig);
    st_sys(p.peer_mbox[lane] + mbox_ready(C, r, w), tx[lane] + 1);
  }
  if (!wave_wait_peers(p.mbox + mbox_ready(C, lane, w), rx[lane < n ? lane : 0] + 1, lane < n && lane != r, ctl, lane,
                       true))
    goto aborted;
  if (!starts_agree(p, ctl, C, lane, w, &seen)) goto aborted;
  acquire_sys(p.sys_fence);
  for (uint32_t j = 0; j < iters; ++j) {
    // F(j): fold my chunk's slice j from the peers' send buffers, store it and push it into every
    // peer's recv; no READY (the peers wait only for DONE, which drains every push), so no drain
    // per slice -- except before the part read back from my recv to be pushed
    const u64 s = (u64)j * A + w;
    const uint32_t len = (uint32_t)slice_len(p.chunk_bytes, p.slice_bytes, s);
    const u64 coff = (u64)r * p.chunk_bytes + s * p.slice_bytes;
    const uint32_t pushed = len ? read_fold<T, OPC, VEC>(p, coff, len, lane) : 0;
    if (pushed < len) {
      drain_stores();
      read_push_rest<T, VEC>(p, coff, len, pushed, lane);
    }
  }
  // DONE: every load of a peer's buffer has returned (and every push into the peers' recv has
  // landed); then wait until nobody reads mine (and every peer's pushes into mine have landed)
  drain_stores();
  if (p.sys_fence && lane == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane < n && lane != r) {
    st_sys(p.peer_mbox[lane] + mbox_credit(n, C, r, w), rx[lane] + mpc);
    st_sys(p.peer_mbox[lane] + mbox_ready(C, r, w), tx[lane] + mpc);
  }
  if (!wave_wait_peers(p.mbox + mbox_ready(C, lane, w), rx[lane < n ? lane : 0] + mpc, lane < n && lane != r, ctl, lane,
                       false))
    goto aborted;
  if (lane < n && lane != r) {
    p.tx_seq[(u64)lane * C + w] = tx[lane] + mpc;
    p.rx_seq[(u64)lane * C + w] = rx[lane] + mpc;
  }
  return;
aborted:
  if (lane == 0)
    for (int k = 1; k < n; ++k) st_sys(p.peer_mbox[direct_peer(n, r, k)] + mbox_abort(n, C), abort_word(p, seen));
}

// ---------------------------------------------------------------- read schedule, grid form
// mncclAlgoReadGrid / MINI_NCCL_ALGO=read_grid, and auto's large read calls since 5.1
// (schedule.h read_grid_form): the push form of a large call (read_grid_fits) as three launches on
// the call's stream --
// read_start_kernel (one wave, pipeline 0: START to every peer, wait for theirs, then the device
// word `go` = this call), read_grid_kernel (the fold with no flag in sight: one one-wave
// workgroup per 1 KiB of my chunk, dispatched in address order, gone when done) and
// read_done_kernel (one wave: DONE to every peer, wait for theirs).  Why: the persistent kernel's
// long-lived waves move a 1:1 read:write stream at 72-80 % of HBM depending on where the buffers
// landed physically, while the dispatcher's one-batch workgroups held 77-81 % on every placement
// (tools/mix_probe.hip, profiles/r4_mix_probe_alloc.txt); on the one-GPU proxy, with the
// workgroup size following the rank count (read_grid_vectors), 1.16-1.21x the persistent form at
// 2 / 4 ranks and equal at 3 / 5 / 6 / 8 (profiles/r5_read_vs_grid_forms*.txt,
// r5_bench_n{2,4,8}_auto_grid.json); the node's bench measures both (schedules.read_grid).  The
// protocol is the push form's with one pipeline and one iteration
// (START, DONE: read_msgs_per_call(1) messages on pipeline 0's counters), which the simulator
// checks for a one-slice read call.  Stream order does the rest: the grid starts after START is
// through (its workgroups still check `go`: after a failed START they must not touch a peer's
// buffers), and every wave drains its stores before it ends, so when DONE is raised every load of
// a peer's send has returned and every push has been acknowledged by the peer's memory.
__global__ void __launch_bounds__(64) read_start_kernel(CollParams p) {
  signal_start(p);
  const int lane = threadIdx.x, n = p.n, r = p.rank, C = p.pipes;
  copy_tail(p, 0, lane);
  const Ctl ctl{p.status, p.host_abort, p.mbox + mbox_abort(n, C), p.timeout_ticks, p.mbox, p.claim};
  const bool peer = lane < n && lane != r;
  const u64 tx = peer ? p.tx_seq[(u64)lane * C] : 0, rx = peer ? p.rx_seq[(u64)lane * C] : 0;
  send_start(p, C, lane, tx + 1, 0);
  uint32_t seen = 0;
  const bool ok = wave_wait_peers(p.mbox + mbox_ready(C, lane, 0), rx + 1, peer, ctl, lane, true) &&
                  starts_agree(p, ctl, C, lane, 0, &seen);
  // 0 after a failed START (a graph replay reuses call_seq: the word must not keep a stale "go")
  if (lane == 0) *p.go = ok ? p.call_seq : 0u;
  if (!ok && lane == 0)
    for (int k = 1; k < n; ++k) st_sys(p.peer_mbox[direct_peer(n, r, k)] + mbox_abort(n, C), abort_word(p, seen));
}

// one batch of V vectors per lane of my chunk: the peers' slices of it loaded together (G peer
// slots, as read_fold_all), folded in ring order, stored into my recv and pushed into every
// peer's recv (the push order rotated by workgroup so the workgroups' stores spread over the links)
// MNCCL_GRID_WAVES: one-wave batches per workgroup (an A/B knob: fewer, larger workgroups for the
// dispatcher; each wave still folds its own batch, wave w of workgroup b batch b * W + w)
#ifndef MNCCL_GRID_WAVES
#define MNCCL_GRID_WAVES 1
#endif
constexpr int kGridWaves = MNCCL_GRID_WAVES;

template <typename T, int OPC, int G, int V>
__global__ void __launch_bounds__(64 * kGridWaves) read_grid_kernel(CollParams p) {
  if (*p.go != p.call_seq) return;  // START failed: the peers' buffers are not ours to touch
  constexpr uint32_t B = 64u * 16u * V;
  const uint32_t batch = blockIdx.x * (uint32_t)kGridWaves + (kGridWaves > 1 ? threadIdx.x / 64u : 0u);
  const uint64_t off = (uint64_t)batch * B;
  if (off >= p.chunk_bytes) return;
  const int n = p.n, r = p.rank, lane = kGridWaves > 1 ? (int)(threadIdx.x % 64u) : (int)threadIdx.x;
  const uint32_t len = (uint32_t)(p.chunk_bytes - off < B ? p.chunk_bytes - off : B);
  const uint64_t coff = (uint64_t)r * p.chunk_bytes + off;
  const rsrc_t loc = make_rsrc(p.send + coff, len), out = make_rsrc(p.recv + coff, len);
  v4u x[G][V], a[V];
#pragma unroll
  for (int g = 0; g < G; ++g)
    if (g + 1 < n) {
      const rsrc_t in = make_rsrc(p.peer_send[direct_peer(n, r, 1 + g)] + coff, len);
#pragma unroll
      for (int u = 0; u < V; ++u) x[g][u] = ld_slot16(in, (uint32_t)(u * 64 + lane) * 16);
    }
#pragma unroll
  for (int u = 0; u < V; ++u) a[u] = ld_nt16(loc, (uint32_t)(u * 64 + lane) * 16);
#pragma unroll
  for (int g = 0; g < G; ++g)
    if (g + 1 < n) {
#pragma unroll
      for (int u = 0; u < V; ++u) a[u] = reduce16<T, OPC>(x[g][u], a[u]);
    }
#pragma unroll
  for (int u = 0; u < V; ++u) st_own16(out, (uint32_t)(u * 64 + lane) * 16, a[u]);
#pragma unroll
  for (int g = 0; g < G; ++g)
    if (g + 1 < n) {
      const int q = direct_peer(n, r, 1 + (int)((g + batch) % (unsigned)(n - 1)));
      const rsrc_t po = make_rsrc(p.peer_recv[q] + coff, len);
#pragma unroll
      for (int u = 0; u < V; ++u) st_slot16(po, (uint32_t)(u * 64 + lane) * 16, a[u]);
    }
  drain_stores();  // every push acknowledged by the peer's memory before this wave ends
}

__global__ void __launch_bounds__(64) read_done_kernel(CollParams p) {
  if (*p.go != p.call_seq) return;  // START failed and already raised the peers' ABORT words
  const int lane = threadIdx.x, n = p.n, r = p.rank, C = p.pipes;
  const Ctl ctl{p.status, p.host_abort, p.mbox + mbox_abort(n, C), p.timeout_ticks, p.mbox, p.claim};
  const bool peer = lane < n && lane != r;
  const u64 mpc = read_msgs_per_call(1);
  const u64 tx = peer ? p.tx_seq[(u64)lane * C] : 0, rx = peer ? p.rx_seq[(u64)lane * C] : 0;
  if (p.sys_fence && lane == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (peer) {
    st_sys(p.peer_mbox[lane] + mbox_credit(n, C, r, 0), rx + mpc);
    st_sys(p.peer_mbox[lane] + mbox_ready(C, r, 0), tx + mpc);
  }
  if (!wave_wait_peers(p.mbox + mbox_ready(C, lane, 0), rx + mpc, peer, ctl, lane, false)) {
    if (lane == 0)
      for (int k = 1; k < n; ++k) st_sys(p.peer_mbox[direct_peer(n, r, k)] + mbox_abort(n, C), abort_word(p));
    return;
  }
  if (peer) {
    p.tx_seq[(u64)lane * C] = tx + mpc;
    p.rx_seq[(u64)lane * C] = rx + mpc;
  }
}

// ---------------------------------------------------------------- one-shot kernel
// Small calls (schedule.h oneshot_fits): one hand-off instead of the ring's 2(n-1) dependent
// ones.  Pipeline w = s * n + c owns slice s of chunk c: it stores that piece of its send into
// every peer's scratch slot -- one message per (pair, pipeline) on the same FIFOs, READY words,
// credits and counters as the ring (calls of either schedule follow each other freely) -- and,
// once every peer's piece is in, folds the piece of the result itself in ring order: x_c, then
// acc = op(x_q, acc) for q = c+1, ..., c-1 (the read schedule's order, the reference ring's
// association), so every rank computes every element exactly as the ring does.  The n
// pipelines of a slice run side by side: a 4 KiB call at 8 ranks is 8 waves, each one piece
// out, one flag round, one fold.  Costs (n-1) x the call's bytes out per rank: small calls only.
template <typename T, int OPC, bool VEC>
__global__ void __launch_bounds__(kMaxThreads, kMinWavesPerSimd) oneshot_kernel(CollParams p) {
  signal_start(p);
  const WaveId id = wave_id();
  const int lane = id.lane, w = id.w, C = p.pipes, wv = id.wv;
  const int n = p.n, r = p.rank, K = p.nslots;
  copy_tail(p, w, lane);
  __shared__ u64 s_tx[kMaxWaves][kMaxRanks], s_rx[kMaxWaves][kMaxRanks];
  u64* tx = s_tx[wv];
  u64* rx = s_rx[wv];
  const Ctl ctl{p.status, p.host_abort, p.mbox + mbox_abort(n, C), p.timeout_ticks, p.mbox, p.claim};
  if (lane < n) {
    tx[lane] = p.tx_seq[(u64)lane * C + w];
    rx[lane] = p.rx_seq[(u64)lane * C + w];
  }
  __builtin_amdgcn_wave_barrier();
  const bool peer = lane < n && lane != r;  // lane q speaks for peer q
  const u64 mytx = tx[lane < n ? lane : 0], myrx = rx[lane < n ? lane : 0];
  const int c = w % n;
  const u64 s = (u64)(w / n);
  const uint32_t len = (uint32_t)slice_len(p.chunk_bytes, p.slice_bytes, s);
  const u64 coff = (u64)c * p.chunk_bytes + s * p.slice_bytes;
  const uint32_t nvec = VEC ? len >> 4 : 0;
  typedef typename Scal<sizeof(T)>::U U;
  const uint32_t ne = len / (uint32_t)sizeof(T), e0 = nvec * 16 / (uint32_t)sizeof(T);
  const rsrc_t mine = make_rsrc(p.send + coff, len);
  // my message's slot in every peer must be free (the peer consumed message tx - slots)
  if (!wave_wait_peers(p.mbox + mbox_credit(n, C, lane, w), mytx + 1 - (u64)K, peer && mytx + 1 > (u64)K, ctl, lane,
                       false))
    goto aborted;
  // my piece into every peer's slot
  for (uint32_t i = (uint32_t)lane; i < nvec; i += 64) {
    const v4u v = ld_slot16(mine, i * 16);
    for (int k = 1; k < n; ++k) {
      const int q = direct_peer(n, r, k);
      st_slot16(make_rsrc(msg_slot(p, C, r, q, w, tx[q]), len), i * 16, v);
    }
  }
  for (uint32_t e = e0 + (uint32_t)lane; e < ne; e += 64) {
    const U v = Scal<sizeof(T)>::ld(mine, e * (uint32_t)sizeof(T));
    for (int k = 1; k < n; ++k) {
      const int q = direct_peer(n, r, k);
      Scal<sizeof(T)>::st(make_rsrc(msg_slot(p, C, r, q, w, tx[q]), len), e * (uint32_t)sizeof(T), v);
    }
  }
  drain_stores();
  if (p.sys_fence && lane == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (peer) st_sys(p.peer_mbox[lane] + mbox_ready(C, r, w), mytx + 1);
  // every peer's piece, then the fold: in[k] = rank c + k's piece (my own send for me)
  if (!wave_wait_peers(p.mbox + mbox_ready(C, lane, w), myrx + 1, peer, ctl, lane, true)) goto aborted;
  acquire_sys(p.sys_fence);
  if (len) {
    rsrc_t in[kMaxRanks];
#pragma unroll
    for (int k = 0; k < kMaxRanks; ++k)
      if (k < n) {
        const int q = mod_n(c + k, n);
        in[k] = q == r ? mine : make_rsrc(msg_slot(p, C, q, r, w, rx[q]), len);
      }
    const rsrc_t out = make_rsrc(p.recv + coff, len);
    for (uint32_t i = (uint32_t)lane; i < nvec; i += 64) {
      v4u x[kMaxRanks];
#pragma unroll
      for (int k = 0; k < kMaxRanks; ++k)
        if (k < n) x[k] = ld_slot16(in[k], i * 16);
      v4u acc = x[0];
#pragma unroll
      for (int k = 1; k < kMaxRanks; ++k)
        if (k < n) acc = reduce16<T, OPC>(x[k], acc);
      st_nt16(out, i * 16, acc);
    }
    for (uint32_t e = e0 + (uint32_t)lane; e < ne; e += 64) {
      U x[kMaxRanks];
#pragma unroll
      for (int k = 0; k < kMaxRanks; ++k)
        if (k < n) x[k] = Scal<sizeof(T)>::ld(in[k], e * (uint32_t)sizeof(T));
      U acc = x[0];
#pragma unroll
      for (int k = 1; k < kMaxRanks; ++k)
        if (k < n) acc = __builtin_bit_cast(U, Op<T, OPC>::f(__builtin_bit_cast(T, x[k]), __builtin_bit_cast(T, acc)));
      Scal<sizeof(T)>::st(out, e * (uint32_t)sizeof(T), acc);
    }
  }
  drain_stores();  // every load of the peers' pieces has returned: their slots are free again
  if (peer) {
    st_sys(p.peer_mbox[lane] + mbox_credit(n, C, r, w), myrx + 1);
    p.tx_seq[(u64)lane * C + w] = mytx + 1;
    p.rx_seq[(u64)lane * C + w] = myrx + 1;
  }
  return;
aborted:
  if (lane == 0)
    for (int k = 1; k < n; ++k) st_sys(p.peer_mbox[direct_peer(n, r, k)] + mbox_abort(n, C), abort_word(p));
}

// ---------------------------------------------------------------- local reduce
// One 16-byte vector per lane, one wave per workgroup, one workgroup per 1 KiB of output,
// non-temporal loads and stores (the bytes are touched once).  Measured on MI355X for
// a <- a + b over 1 GiB fp32 (tools/lr_sweep.hip, interleaved rounds): 6.72 TB/s = 84 % of
// the 8 TB/s spec, vs 5.84 TB/s for a 4096-block grid-stride loop with 4 vectors per lane
// and 5.27 TB/s with plain (temporal) loads/stores.  Short-lived single-wave workgroups
// let the dispatcher keep every CU's memory pipeline full without a tail.
template <typename T, int OPC>
__global__ void __launch_bounds__(64) local_reduce_vec(char* __restrict__ out, const char* __restrict__ a,
                                                       const char* __restrict__ b, u64 nvec) {
  const u64 i = (u64)blockIdx.x * 64 + threadIdx.x;
  if (i < nvec) {
    const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a) + i);
    const v4u y = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(b) + i);
    __builtin_nontemporal_store(reduce16<T, OPC>(x, y), reinterpret_cast<v4u*>(out) + i);
  }
}

// grid-stride form for buffers beyond 2^32 threads of the exact grid (> 64 GiB)
template <typename T, int OPC>
__global__ void __launch_bounds__(256) local_reduce_vec_gs(char* __restrict__ out, const char* __restrict__ a,
                                                           const char* __restrict__ b, u64 nvec) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a) + i);
    const v4u y = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(b) + i);
    __builtin_nontemporal_store(reduce16<T, OPC>(x, y), reinterpret_cast<v4u*>(out) + i);
  }
}

template <typename T, int OPC>
__global__ void __launch_bounds__(256) local_reduce_scalar(T* __restrict__ out, const T* __restrict__ a,
                                                           const T* __restrict__ b, u64 n) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = Op<T, OPC>::f(a[i], b[i]);
}

// ---------------------------------------------------------------- link probe
struct ProbeArgs {
  char* local;
  char* remote[kMaxRanks];
  int nremote;
  uint64_t bytes;
};

// cache-policy bits of the probe's remote accesses (kProbe* in kernels.h): the hot path's
// sc0 sc1, non-temporal, or the default policy
template <int FORM> struct ProbeAux;
template <> struct ProbeAux<kProbeSys> { static constexpr int v = kAuxSys; };
template <> struct ProbeAux<kProbeNt> { static constexpr int v = 2; };
template <> struct ProbeAux<kProbePlain> { static constexpr int v = 0; };

// blocks [d * per, (d+1) * per) move `bytes` between `local` and remote d; 8 x 16 B per lane in
// flight.  PULL = false: local -> remote (the schedules' pushes); true: remote -> local (loads
// over the link, for comparison).
template <int FORM, bool PULL>
__global__ void __launch_bounds__(256) link_probe_kernel(ProbeArgs a) {
  constexpr int AUX = ProbeAux<FORM>::v;
  const int per = gridDim.x / a.nremote;
  const int d = blockIdx.x / per, b = blockIdx.x % per;
  if (d >= a.nremote) return;
  const uint64_t nvec = a.bytes / 16;
  const rsrc_t rem = make_rsrc(a.remote[d], (uint32_t)a.bytes);
  const rsrc_t loc = make_rsrc(a.local, (uint32_t)a.bytes);
  for (uint64_t base = (uint64_t)b * 256 * 8 + threadIdx.x; base < nvec; base += (uint64_t)per * 256 * 8) {
    v4u v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = base + (uint64_t)u * 256;
      if (i < nvec)
        v[u] = PULL ? __builtin_amdgcn_raw_buffer_load_b128(rem, (uint32_t)(i * 16), 0, AUX)
                    : __builtin_amdgcn_raw_buffer_load_b128(loc, (uint32_t)(i * 16), 0, 2);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = base + (uint64_t)u * 256;
      if (i < nvec) {
        if (PULL) __builtin_amdgcn_raw_buffer_store_b128(v[u], loc, (uint32_t)(i * 16), 0, 2);
        else __builtin_amdgcn_raw_buffer_store_b128(v[u], rem, (uint32_t)(i * 16), 0, AUX);
      }
    }
  }
}

hipError_t launch_link_probe(char* local, char* const* remote, int nremote, uint64_t bytes, int form, bool pull,
                             hipStream_t st) {
  if (nremote < 1 || nremote > kMaxRanks || bytes == 0 || bytes > 0xffffffffull) return hipErrorInvalidValue;
  ProbeArgs a;
  a.local = local;
  for (int i = 0; i < kMaxRanks; ++i) a.remote[i] = i < nremote ? remote[i] : nullptr;
  a.nremote = nremote;
  a.bytes = bytes;
  const int per = 256 / nremote > 0 ? 256 / nremote : 1;
  const dim3 g(per * nremote), blk(256);
#define PROBE_CASE(F)                                                        \
  case F:                                                                    \
    if (pull) hipLaunchKernelGGL((link_probe_kernel<F, true>), g, blk, 0, st, a); \
    else hipLaunchKernelGGL((link_probe_kernel<F, false>), g, blk, 0, st, a);     \
    break;
  switch (form) {
    PROBE_CASE(kProbeSys) PROBE_CASE(kProbeNt) PROBE_CASE(kProbePlain)
    default: return hipErrorInvalidValue;
  }
#undef PROBE_CASE
  return hipGetLastError();
}

// ---------------------------------------------------------------- dispatch
template <template <typename, int, bool> class K>
struct Unused {};

#define MNCCL_DISPATCH_T(dtype, MACRO)      \
  switch (dtype) {                          \
    case kF32: MACRO(float); break;         \
    case kF64: MACRO(double); break;        \
    case kI32: MACRO(int32_t); break;       \
    case kF16: MACRO(_Float16); break;      \
    case kBF16: MACRO(bf16_t); break;       \
    default: return hipErrorInvalidValue;   \
  }

template <typename T>
static hipError_t ring_for_t(int op, bool vec, int C, int nt, const CollParams& p, hipStream_t st) {
#define RING_CASE(OPC)                                                                           \
  case OPC:                                                                                      \
    if (vec) hipLaunchKernelGGL((ring_kernel<T, OPC, true>), dim3(C), dim3(nt), 0, st, p);      \
    else hipLaunchKernelGGL((ring_kernel<T, OPC, false>), dim3(C), dim3(nt), 0, st, p);         \
    break;
  switch (op) {
    RING_CASE(kSum) RING_CASE(kProd) RING_CASE(kMax) RING_CASE(kMin)
    default: return hipErrorInvalidValue;
  }
#undef RING_CASE
  return hipGetLastError();
}

template <typename T>
static hipError_t read_for_t(int op, bool vec, int C, int nt, const CollParams& p, hipStream_t st) {
#define READ_LAUNCH(OPC, V) hipLaunchKernelGGL((read_kernel<T, OPC, V>), dim3(C), dim3(nt), 0, st, p);
#define READ_CASE(OPC)           \
  case OPC:                      \
    if (vec) {                   \
      READ_LAUNCH(OPC, true)     \
    } else {                     \
      READ_LAUNCH(OPC, false)    \
    }                            \
    break;
  switch (op) {
    READ_CASE(kSum) READ_CASE(kProd) READ_CASE(kMax) READ_CASE(kMin)
    default: return hipErrorInvalidValue;
  }
#undef READ_CASE
#undef READ_LAUNCH
  return hipGetLastError();
}

template <typename T>
static hipError_t local_for_t(int op, void* out, const void* a, const void* b, u64 count, hipStream_t st) {
  // 16-byte vectors over the body whenever the three buffers are dword-aligned (4-byte-aligned
  // dwordx4 accesses are valid on gfx950), then the last (bytes % 16) bytes element-wise
  const bool vec = ((uintptr_t)out | (uintptr_t)a | (uintptr_t)b) % 4 == 0;
  const u64 nvec = vec ? count * sizeof(T) / 16 : 0;
  const u64 done = nvec * 16 / sizeof(T);
  const u64 kMaxExactBlocks = (1ull << 31) / 64;  // keep the exact grid under 2^31 threads
#define LOCAL_CASE(OPC)                                                                                         \
  case OPC:                                                                                                     \
    if (nvec && (nvec + 63) / 64 <= kMaxExactBlocks)                                                            \
      hipLaunchKernelGGL((local_reduce_vec<T, OPC>), dim3((unsigned)((nvec + 63) / 64)), dim3(64), 0, st,      \
                         (char*)out, (const char*)a, (const char*)b, nvec);                                     \
    else if (nvec)                                                                                              \
      hipLaunchKernelGGL((local_reduce_vec_gs<T, OPC>), dim3(16384), dim3(256), 0, st, (char*)out,             \
                         (const char*)a, (const char*)b, nvec);                                                 \
    if (count > done)                                                                                           \
      hipLaunchKernelGGL((local_reduce_scalar<T, OPC>),                                                         \
                         dim3((unsigned)std::min<u64>((count - done + 255) / 256, 16384)), dim3(256), 0, st,    \
                         (T*)out + done, (const T*)a + done, (const T*)b + done, count - done);                 \
    break;
  switch (op) {
    LOCAL_CASE(kSum) LOCAL_CASE(kProd) LOCAL_CASE(kMax) LOCAL_CASE(kMin)
    default: return hipErrorInvalidValue;
  }
#undef LOCAL_CASE
  return hipGetLastError();
}

hipError_t launch_ring(int dtype, int op, bool vec, int C, int nt, const CollParams& p, hipStream_t st) {
#define M(T) return ring_for_t<T>(op, vec, C, nt, p, st)
  MNCCL_DISPATCH_T(dtype, M)
#undef M
}

hipError_t launch_read(int dtype, int op, bool vec, int C, int nt, const CollParams& p, hipStream_t st) {
#define M(T) return read_for_t<T>(op, vec, C, nt, p, st)
  MNCCL_DISPATCH_T(dtype, M)
#undef M
}

template <typename T>
static hipError_t oneshot_for_t(int op, bool vec, int C, int nt, const CollParams& p, hipStream_t st) {
#define ONESHOT_CASE(OPC)                                                                           \
  case OPC:                                                                                         \
    if (vec) hipLaunchKernelGGL((oneshot_kernel<T, OPC, true>), dim3(C), dim3(nt), 0, st, p);      \
    else hipLaunchKernelGGL((oneshot_kernel<T, OPC, false>), dim3(C), dim3(nt), 0, st, p);         \
    break;
  switch (op) {
    ONESHOT_CASE(kSum) ONESHOT_CASE(kProd) ONESHOT_CASE(kMax) ONESHOT_CASE(kMin)
    default: return hipErrorInvalidValue;
  }
#undef ONESHOT_CASE
  return hipGetLastError();
}

template <typename T>
static hipError_t read_grid_for_t(int op, const CollParams& p, hipStream_t st, int vectors) {
  // V 16-byte vectors per lane per workgroup: V KiB of the chunk each (schedule.h read_grid_vectors)
  const int n = p.n;
  // MINI_NCCL_GRID_VECTORS: 1 / 2 / 4 vectors per lane for fp32 Sum (the bench's workload: the
  // node's sweep weighs them over xGMI); every other call follows the rule
  const bool tuned = vectors != 0 && std::is_same<T, float>::value && op == kSum;
  const int V = tuned ? vectors : read_grid_vectors(n);
  // the rule's instantiations below hard-code V per rank count; a rule they do not match is
  // refused rather than launched with a grid sized for another V
  if (!tuned && V != (n <= 4 ? 1 : 2)) return hipErrorInvalidValue;
  const uint64_t per_block = 1024ull * (uint64_t)V * kGridWaves;
  const unsigned blocks = (unsigned)((p.chunk_bytes + per_block - 1) / per_block);
#define GRID_G(OPC, G, VV) \
  hipLaunchKernelGGL((read_grid_kernel<T, OPC, G, VV>), dim3(blocks), dim3(64 * kGridWaves), 0, st, p)
  if constexpr (std::is_same<T, float>::value) {
    if (tuned) {
#define GRID_V(VV)                                    if (n == 2) GRID_G(kSum, 1, VV);                    else if (n == 3) GRID_G(kSum, 2, VV);               else if (n <= 5) GRID_G(kSum, 4, VV);               else GRID_G(kSum, 7, VV);
      if (V == 1) { GRID_V(1) }
      else if (V == 2) { GRID_V(2) }
      else { GRID_V(4) }
#undef GRID_V
      return hipGetLastError();
    }
  }
#define GRID_CASE(OPC)                    \
  case OPC:                               \
    if (n == 2) GRID_G(OPC, 1, 1);        \
    else if (n == 3) GRID_G(OPC, 2, 1);   \
    else if (n == 4) GRID_G(OPC, 4, 1);   \
    else if (n == 5) GRID_G(OPC, 4, 2);   \
    else GRID_G(OPC, 7, 2);               \
    break;
  switch (op) {
    GRID_CASE(kSum) GRID_CASE(kProd) GRID_CASE(kMax) GRID_CASE(kMin)
    default: return hipErrorInvalidValue;
  }
#undef GRID_CASE
#undef GRID_G
  return hipGetLastError();
}

hipError_t launch_read_grid(int dtype, int op, const CollParams& p, hipStream_t st, int vectors) {
  // the shapes the grid kernel assumes, checked before anything is launched
  if (p.n < 2 || p.n > 8 || p.chunk_bytes % 16 || !p.go || !read_grid_fits(p.chunk_bytes, p.n, kReadGridFloor) ||
      (p.chunk_bytes + 1023) / 1024 > 0x7fffffffull || (read_grid_vectors(p.n) != 1 && read_grid_vectors(p.n) != 2) ||
      (vectors != 0 && vectors != 1 && vectors != 2 && vectors != 4))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(read_start_kernel, dim3(1), dim3(64), 0, st, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
#define M(T) e = read_grid_for_t<T>(op, p, st, vectors)
  MNCCL_DISPATCH_T(dtype, M)
#undef M
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(read_done_kernel, dim3(1), dim3(64), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_oneshot(int dtype, int op, bool vec, int C, int nt, const CollParams& p, hipStream_t st) {
#define M(T) return oneshot_for_t<T>(op, vec, C, nt, p, st)
  MNCCL_DISPATCH_T(dtype, M)
#undef M
}

hipError_t launch_local_reduce(int dtype, int op, void* out, const void* local, const void* incoming, uint64_t count,
                               hipStream_t st) {
  if (count == 0) return hipSuccess;
#define M(T) return local_for_t<T>(op, out, local, incoming, count, st)
  MNCCL_DISPATCH_T(dtype, M)
#undef M
}

bool dtype_supported(int dtype) { return dtype_size(dtype) != 0; }

int dtype_size(int dtype) {
  switch (dtype) {
    case kF32: case kI32: return 4;
    case kF64: return 8;
    case kF16: case kBF16: return 2;
    default: return 0;
  }
}

}  // namespace mnccl
