// Environment probe (not product code): does a write from a CU under ANOTHER L2 invalidate the
// clean line this L2 holds of ordinary (coarse-grained hipMalloc) device memory, with no kernel
// boundary and no acquire in between?
//
// Why it matters: the read schedule's push form stores each rank's result into its peers' recv.
// On the node the owner's L2 may hold clean lines of recv from kernels that ran before the call;
// the peers' stores arrive from CUs under other L2s (another GPU's).  LLVM's AMDGPUUsage memory
// model for GFX942 (which gfx950 follows) states the rule the push form relies on: "Any local
// memory cache lines will be automatically invalidated by writes from CUs associated with other
// L2 caches, or writes from the CPU, due to the cache probe caused by the PTE C-bit" (local
// memory is mapped MTYPE RW, remote memory MTYPE NC with the C-bit).  One MI355X has eight L2s
// (one per XCD): a writer on another XCD is a CU "associated with another L2", so the rule can
// be exercised on one GPU.
//
// One launch, one-wave workgroups.  Block 0 is the reader; the first block found on another XCD
// (s_getreg HW_REG_XCC_ID) -- or on the SAME XCD for the control -- is the writer.  Per trial t
// (its own 4 KiB region, initially OLD):
//   reader: load the region (first form), load it again (timed: an L2 hit if the line stayed),
//           raise A[t];
//   writer: wait A[t], store NEW (store form), s_waitcnt vmcnt(0), raise B[t];
//   reader: wait B[t], re-load the region (re-read form, no fence), count words != NEW.
// Load forms: sc1 (agent scope: skips L1, served by this XCD's L2) or plain (may hit L1).  The
// plain/plain case is the negative control: L1 keeps stale lines (MI355X_MICROARCH.md:161),
// so the probe can see staleness when there is some.
//
// Usage: probe_xcd_coherence [trials]    (prints one line per case)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

constexpr int kRegionWords = 1024;    // 4 KiB per trial: 64 lanes x 16 B
constexpr int kFlagStride = 32;       // u32 words: one 128-B line per flag
constexpr u64 kTimeoutTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)

enum { kLoadSc1 = 0, kLoadPlain = 1 };
enum { kStPlain = 0, kStNt = 1, kStSys = 2 };

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_flag(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// lane-uniform bounded spin; false on timeout
__device__ bool wait_flag(const unsigned* p, unsigned v) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_flag(p) < v) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) return false;
  }
  return true;
}
__device__ __forceinline__ v4u load_form(__amdgpu_buffer_rsrc_t r, const v4u* p, unsigned off, int form) {
  (void)p;
  // (not a volatile pointer: LLVM gives volatile accesses sc0 sc1 on gfx94x/gfx950)
  if (form == kLoadSc1) return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);  // sc1
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);                          // plain
}

struct Args {
  unsigned* data;   // trials x kRegionWords
  unsigned* flags;  // trials x 2 flag lines
  unsigned* ctl;    // [0] reader xcc + 1, [1] writer block + 1, [2] writer xcc + 1, [3] error
  unsigned long long* stale;  // per trial: words != NEW at the re-read
  unsigned* cyc;    // per trial: cold, warm, re-read cycles (x3)
  int trials, same_xcd, first_form, reread_form, store_form;
  int writer_wait_us;  // writer: s_sleep this long after its vmcnt(0) wait, before the flag
  int writer_release;  // writer: agent-scope release (buffer_wbl2 sc1) before the flag
  int reader_acquire;  // reader: 0 none, 1 agent acquire (buffer_inv sc1), 2 system (sc0 sc1)
};

__global__ void __launch_bounds__(64) probe(Args a) {
  const int lane = threadIdx.x;
  const unsigned my_xcc = xcc_id();
  bool reader = blockIdx.x == 0, writer = false;
  if (reader) {
    if (lane == 0) st_flag(&a.ctl[0], my_xcc + 1);
  } else {
    unsigned rx = 0;
    if (lane == 0) {
      const u64 t0 = __builtin_amdgcn_s_memrealtime();
      while ((rx = ld_flag(&a.ctl[0])) == 0 && __builtin_amdgcn_s_memrealtime() - t0 < kTimeoutTicks)
        __builtin_amdgcn_s_sleep(1);
    }
    rx = __builtin_amdgcn_readfirstlane(rx);
    if (rx == 0) return;
    const bool eligible = a.same_xcd ? (my_xcc + 1 == rx) : (my_xcc + 1 != rx);
    int won = 0;
    if (eligible && lane == 0) won = atomicCAS(&a.ctl[1], 0u, blockIdx.x + 1) == 0;
    writer = __builtin_amdgcn_readfirstlane(won) != 0;
    if (!writer) return;
    if (lane == 0) st_flag(&a.ctl[2], my_xcc + 1);
  }
  const unsigned OLD = 0xa0000000u, NEW = 0xb0000000u;
  if (reader) {
    // wait for a writer to be chosen (bounded)
    int ok = 1;
    if (lane == 0) ok = wait_flag(&a.ctl[1], 1);
    if (!__builtin_amdgcn_readfirstlane(ok)) {
      if (lane == 0) st_flag(&a.ctl[3], 1);
      return;
    }
    for (int t = 0; t < a.trials; ++t) {
      unsigned* reg = a.data + (size_t)t * kRegionWords;
      const auto r = rsrc(reg, kRegionWords * 4);
      const unsigned off = (unsigned)lane * 16;
      u64 c0 = __builtin_readcyclecounter();
      v4u v = load_form(r, (const v4u*)reg, off, a.first_form);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u64 c1 = __builtin_readcyclecounter();
      v4u w = load_form(r, (const v4u*)reg, off, a.first_form);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u64 c2 = __builtin_readcyclecounter();
      unsigned bad_old = (v.x != OLD + t) + (v.y != OLD + t) + (v.z != OLD + t) + (v.w != OLD + t) +
                         (w.x != OLD + t) + (w.y != OLD + t) + (w.z != OLD + t) + (w.w != OLD + t);
      if (bad_old) atomicAdd(&a.ctl[3], 0x100u);  // the region was not OLD before the write
      if (lane == 0) st_flag(&a.flags[(size_t)t * 2 * kFlagStride], 1);
      ok = 1;
      if (lane == 0) ok = wait_flag(&a.flags[((size_t)t * 2 + 1) * kFlagStride], 1);
      if (!__builtin_amdgcn_readfirstlane(ok)) {
        if (lane == 0) st_flag(&a.ctl[3], 2);
        return;
      }
      if (a.reader_acquire == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      else if (a.reader_acquire == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u64 c3 = __builtin_readcyclecounter();
      v4u x = load_form(r, (const v4u*)reg, off, a.reread_form);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u64 c4 = __builtin_readcyclecounter();
      unsigned long long stale = (x.x != NEW + t) + (x.y != NEW + t) + (x.z != NEW + t) + (x.w != NEW + t);
      if (stale) atomicAdd(&a.stale[t], stale);
      if (lane == 0) {
        a.cyc[t * 3 + 0] = (unsigned)(c1 - c0);
        a.cyc[t * 3 + 1] = (unsigned)(c2 - c1);
        a.cyc[t * 3 + 2] = (unsigned)(c4 - c3);
      }
    }
  } else {
    for (int t = 0; t < a.trials; ++t) {
      int ok = 1;
      if (lane == 0) ok = wait_flag(&a.flags[(size_t)t * 2 * kFlagStride], 1);
      if (!__builtin_amdgcn_readfirstlane(ok)) {
        if (lane == 0) st_flag(&a.ctl[3], 4);
        return;
      }
      unsigned* reg = a.data + (size_t)t * kRegionWords;
      const auto r = rsrc(reg, kRegionWords * 4);
      const unsigned off = (unsigned)lane * 16;
      const v4u v{NEW + t, NEW + t, NEW + t, NEW + t};
      if (a.store_form == kStSys) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 17);
      else if (a.store_form == kStNt) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 2);
      else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (a.writer_release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (a.writer_wait_us) {
        const u64 t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (u64)a.writer_wait_us * 100) __builtin_amdgcn_s_sleep(2);
      }
      if (lane == 0) st_flag(&a.flags[((size_t)t * 2 + 1) * kFlagStride], 1);
    }
  }
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 512;
  CK(hipSetDevice(0));
  struct Case {
    const char* name;
    int same, first, reread, store, wait_us, release, acquire;
  } cases[] = {
      {"other XCD, sc1 loads, sc0 sc1 stores (push form)", 0, kLoadSc1, kLoadSc1, kStSys, 0, 0, 0},
      {"other XCD, sc1 loads, plain stores", 0, kLoadSc1, kLoadSc1, kStPlain, 0, 0, 0},
      {"other XCD, sc1 loads, nt stores", 0, kLoadSc1, kLoadSc1, kStNt, 0, 0, 0},
      {"other XCD, plain first load, sc1 re-read, sc0 sc1 stores", 0, kLoadPlain, kLoadSc1, kStSys, 0, 0, 0},
      {"same XCD, sc1 loads, sc0 sc1 stores (control)", 1, kLoadSc1, kLoadSc1, kStSys, 0, 0, 0},
      {"other XCD, plain loads (L1: negative control)", 0, kLoadPlain, kLoadPlain, kStSys, 0, 0, 0},
      {"other XCD, sc1 loads, nt stores, writer waits 20 us", 0, kLoadSc1, kLoadSc1, kStNt, 20, 0, 0},
      {"other XCD, sc1 loads, plain stores + writer agent release", 0, kLoadSc1, kLoadSc1, kStPlain, 0, 1, 0},
      {"other XCD, sc1 loads, nt stores + reader agent acquire", 0, kLoadSc1, kLoadSc1, kStNt, 0, 0, 1},
      {"other XCD, sc1 loads, nt stores + reader system acquire", 0, kLoadSc1, kLoadSc1, kStNt, 0, 0, 2},
  };
  const size_t dbytes = (size_t)trials * kRegionWords * 4;
  std::vector<unsigned> init((size_t)trials * kRegionWords);
  for (int t = 0; t < trials; ++t)
    for (int i = 0; i < kRegionWords; ++i) init[(size_t)t * kRegionWords + i] = 0xa0000000u + t;
  int rc = 0;
  for (const Case& c : cases) {
    for (int rep = 0; rep < 2; ++rep) {
      Args a{};
      CK(hipMalloc((void**)&a.data, dbytes));
      CK(hipMalloc((void**)&a.flags, (size_t)trials * 2 * kFlagStride * 4));
      CK(hipMalloc((void**)&a.ctl, 64));
      CK(hipMalloc((void**)&a.stale, (size_t)trials * 8));
      CK(hipMalloc((void**)&a.cyc, (size_t)trials * 3 * 4));
      CK(hipMemcpy(a.data, init.data(), dbytes, hipMemcpyHostToDevice));
      CK(hipMemset(a.flags, 0, (size_t)trials * 2 * kFlagStride * 4));
      CK(hipMemset(a.ctl, 0, 64));
      CK(hipMemset(a.stale, 0, (size_t)trials * 8));
      CK(hipMemset(a.cyc, 0, (size_t)trials * 3 * 4));
      CK(hipDeviceSynchronize());
      a.trials = trials;
      a.same_xcd = c.same;
      a.first_form = c.first;
      a.reread_form = c.reread;
      a.store_form = c.store;
      a.writer_wait_us = c.wait_us;
      a.writer_release = c.release;
      a.reader_acquire = c.acquire;
      hipLaunchKernelGGL(probe, dim3(64), dim3(64), 0, 0, a);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      unsigned ctl[4];
      std::vector<unsigned long long> stale(trials);
      std::vector<unsigned> cyc((size_t)trials * 3);
      CK(hipMemcpy(ctl, a.ctl, 16, hipMemcpyDeviceToHost));
      CK(hipMemcpy(stale.data(), a.stale, (size_t)trials * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(cyc.data(), a.cyc, (size_t)trials * 12, hipMemcpyDeviceToHost));
      unsigned long long tot = 0;
      int trials_stale = 0;
      for (int t = 0; t < trials; ++t) {
        tot += stale[t];
        trials_stale += stale[t] != 0;
      }
      auto med = [&](int k) {
        std::vector<unsigned> v;
        for (int t = 0; t < trials; ++t) v.push_back(cyc[(size_t)t * 3 + k]);
        std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
        return v[v.size() / 2];
      };
      printf("%-60s rep %d: reader XCD %u, writer XCD %d | stale words at re-read %llu of %llu (%d of %d trials) | "
             "median cycles: first load %u, second load %u, re-read %u | error 0x%x\n",
             c.name, rep, ctl[0] - 1, (int)ctl[2] - 1, tot, (unsigned long long)trials * kRegionWords, trials_stale,
             trials, med(0), med(1), med(2), ctl[3]);
      fflush(stdout);
      if (ctl[3] & 0xff) rc = 3;
      CK(hipFree(a.data));
      CK(hipFree(a.flags));
      CK(hipFree(a.ctl));
      CK(hipFree(a.stale));
      CK(hipFree(a.cyc));
    }
  }
  return rc;
}
