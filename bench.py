#!/usr/bin/env python3
"""bench.py -- the headline metric: all-reduce algbw (GB/s) on 1 GiB fp32, device-resident.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

One step = one pass of the hot path over one batch of synthetic fp32 input already
resident in HBM:
  N = 1  the 1-GPU local reduce of BASELINE.md (a <- a + b over 1 GiB): the scatter-reduce
         element-wise kernel alone (the reference's all-reduce is a no-op at one rank,
         mini_nccl.cu:66);
  N > 1  one ncclAllReduce(send, recv, 268435456, ncclFloat, ncclSum) per rank through the
         C ABI (one process per GPU, HIP IPC over xGMI), all-ones input as the reference's
         perf_test (tests/perf_test.cpp:82), result checked == N.
value = bytes / (time per step), time = max over ranks of K steps between barriers +
device synchronisation.  rank 0 prints ONE JSON line; diagnostics go to stderr.

roofline: algorithmic HBM bytes of the dominant kernel per launch (3*4 B per
reduced element; N=1: 3 * 1 GiB; N>1: 3*4*(n-1)*count/n) / its average launch duration,
measured here with HIP events on the stream the kernel runs on.  traffic: PMC bytes per
launch from the rocprofv3 pass committed under profiles/ (see profiles/README.md), or null.
cpu_baseline (rank 0, N = 1 only): the AVX2 host restatement (oracle/ring_oracle.c, the
reference has no CPU reduce; its AVX2 code is a verify scan) timed on this host.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mini-nccl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "all-reduce algbw (GB/s) on 1 GiB fp32, device-resident, at 1/2/4/8 MI355X"
COUNT = 268435456  # 1 GiB of fp32
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


_T0 = time.time()


def log(*a):
    print(f"[{time.time() - _T0:7.1f}s]", *a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------ CPU baseline (oracle)
def cpu_baseline(budget_s=18.0):
    """The host path, timed on this box's cores: AVX2 a += b over the same 1 GiB (the N=1
    workload), plus the reference's C1 config (2-rank 127.0.0.1 TCP ring, 4 MiB)."""
    import numpy as np

    import oracle_api as O
    L = O.load()
    threads = max(1, min(16, os.cpu_count() or 1))
    a = np.full(COUNT, 1.0, np.float32)
    b = np.full(COUNT, 2.0, np.float32)
    t_start = time.time()
    t_last = L.oracle_cpu_local_reduce_avx2(a.ctypes.data, b.ctypes.data, COUNT, threads, 1)  # first touch / warm
    # timed passes in ~0.5 s batches until the budget is spent: bounded by the clock, not by a
    # pass count extrapolated from the first pass (a busy host once stretched that to 71 s)
    iters, spent = 0, 0.0
    while spent < budget_s * 0.8 and iters < 2000:
        k = max(1, min(50, int(0.5 / max(t_last, 1e-3))))
        t_last = L.oracle_cpu_local_reduce_avx2(a.ctypes.data, b.ctypes.data, COUNT, threads, k)
        spent += t_last * k
        iters += k
    t_mt = spent / iters
    t_st = L.oracle_cpu_local_reduce_avx2(a.ctypes.data, b.ctypes.data, COUNT, 1, 1)
    # every core the lease allows (affinity, bounded by the cgroup's CPU quota), beside the
    # 16-thread figure: a few passes, same workload
    lease = lease_cores()
    t_all, all_iters = None, 0
    if lease > threads:
        t_all = L.oracle_cpu_local_reduce_avx2(a.ctypes.data, b.ctypes.data, COUNT, lease, 1)  # warm
        all_iters = max(1, min(200, int(3.0 / max(t_all, 1e-3))))
        t_all = L.oracle_cpu_local_reduce_avx2(a.ctypes.data, b.ctypes.data, COUNT, lease, all_iters)
    ok = L.oracle_verify_avx2(a.ctypes.data, COUNT,
                              float(1.0 + 2.0 * (2 + iters + (1 + all_iters if t_all else 0)))) == -1
    del a, b
    # C1: 2 ranks over loopback TCP, 4 MiB fp32, 128 KiB slices (BASELINE.json configs[0])
    c1 = None
    try:
        import ctypes
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        n_c1, cnt = 2, (4 << 20) // 4
        bufs = [np.ones(cnt, np.float32) for _ in range(n_c1)]
        secs = [ctypes.c_double() for _ in range(n_c1)]
        rcs = [None] * n_c1
        c1_iters = 20

        def rank(r):
            rcs[r] = L.oracle_cpu_ring_tcp(r, n_c1, b"127.0.0.1", port, bufs[r].ctypes.data, cnt, 131072, c1_iters,
                                           ctypes.byref(secs[r]))

        # daemon threads: a C1 ring that does not finish within the join limit must not hold the
        # process at exit (the JSON line is already out by then)
        th = [threading.Thread(target=rank, args=(r,), daemon=True) for r in range(n_c1)]
        for t in th:
            t.start()
        c1_deadline = time.time() + 30.0  # the whole C1 sample: ~10 ms of work when the host is idle
        for t in th:
            t.join(max(0.1, c1_deadline - time.time()))
        if not all(rc == 0 for rc in rcs):
            log(f"C1 TCP baseline did not complete within 30 s (rc {rcs}): reported as null")
        if all(rc == 0 for rc in rcs):
            t_c1 = max(x.value for x in secs)
            c1 = {"config": "2-rank 127.0.0.1 TCP ring, 4 MiB fp32, SLICE 128 KiB, AVX2 adds",
                  "algbw_GBps": round(cnt * 4 / t_c1 / 1e9, 3), "us_per_allreduce": round(t_c1 * 1e6, 1),
                  "iters": c1_iters, "threads": n_c1}
    except Exception as e:  # reported, never fatal
        log("C1 TCP baseline failed:", e)
    return {
        "value": round(COUNT * 4 / t_mt / 1e9, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"a += b over the full 1 GiB fp32 workload, {iters} timed passes after 1 warm pass "
                  f"(AVX2 _mm256_add_ps, {threads} threads); verify scan {'ok' if ok else 'FAILED'}",
        "single_thread_GBps": round(COUNT * 4 / t_st / 1e9, 3),
        "lease_cores": lease,
        "lease_GBps": round(COUNT * 4 / t_all / 1e9, 3) if t_all else None,
        "lease_note": (f"the same 1 GiB a += b on all {lease} cores the lease allows, {all_iters} passes"
                       if t_all else f"the lease allows {lease} cores: the {threads}-thread figure is all of them"),
        "nproc": os.cpu_count(),  # the whole machine's CPUs (the box's share is 16)
        "c1_tcp_ring": c1,
        "wall_s": round(time.time() - t_start, 1),
    }


def lease_cores():
    """CPUs this process may run on: its affinity, bounded by the cgroup's CPU quota (the GPU box
    gives a one-GPU lease 16 of the machine's cores)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_ring_baseline(n, budget_s=6.0):
    """N > 1 companion of cpu_baseline: the host ring, n threads of this box
    (one per rank), the reference's schedule and operand order with AVX2 adds, on the workload's
    own size (1 GiB fp32 per rank, as the GPU runs)."""
    import ctypes

    import numpy as np

    import oracle_api as O
    L = O.load()
    cnt = COUNT
    bufs = [np.ones(cnt, np.float32) for _ in range(n)]
    arr = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    t1 = L.oracle_cpu_ring_threads_avx2(arr, n, cnt, 131072, 1)  # also the first touch
    iters = max(1, min(10, int(budget_s / max(t1, 1e-3))))
    t = L.oracle_cpu_ring_threads_avx2(arr, n, cnt, 131072, iters)
    # the known answer (perf_test.cpp:81-134): one more call on fresh all-ones gives n everywhere
    for b in bufs:
        b.fill(1.0)
    L.oracle_cpu_ring_threads_avx2(arr, n, cnt, 131072, 1)
    ok = all(L.oracle_verify_avx2(b.ctypes.data, (cnt // n) * n, float(n)) == -1 for b in bufs)
    del bufs
    return {"value": round(cnt * 4 / t / 1e9, 3), "unit": "GB/s", "cores": n, "nproc": os.cpu_count(), "kind": "port",
            "sample": f"{n}-thread in-process host ring (reference schedule, AVX2 adds), 1 GiB fp32 per rank (the "
                      f"workload's size), {iters} timed all-reduces after 1; known answer {'ok' if ok else 'FAILED'}"}


# ------------------------------------------------------------------ N > 1 configuration sweeps
# (schedule, knob) points timed on a 256 MiB buffer, and the
# BASELINE.json configs[3] (C4) grid: ring, 4 GiB fp32, SLICE x WINDOW.  Each point builds its
# own communicator (the knobs are read at ncclCommInitRank, as the reference's Config).
SWEEP_POINTS = [
    # (algo, knobs over the library defaults: 256 one-wave workgroups, 128 KiB slices, 2 slots,
    #  no hand-off fences)
    ("read", {}),
    ("read", {"MINI_NCCL_SLICE_SIZE": 32768}), ("read", {"MINI_NCCL_SLICE_SIZE": 524288}),
    ("read", {"MINI_NCCL_CHANNELS": 128}), ("read", {"MINI_NCCL_CHANNELS": 512}),
    ("read", {"MINI_NCCL_THREADS": 128}), ("read", {"MINI_NCCL_SYS_FENCE": 1}),
    ("ring", {}), ("ring", {"MINI_NCCL_SLOTS": 4}), ("ring", {"MINI_NCCL_SLICE_SIZE": 524288}),
    ("ring", {"MINI_NCCL_SYS_FENCE": 1}),
    # the grid form's vectors per lane per workgroup (schedule.h read_grid_vectors: 1 up to 4 ranks,
    # 2 from 5, decided on the one-GPU proxy): on the node's links, where a remote load waits longer
    ("read_grid", {}), ("read_grid", {"MINI_NCCL_GRID_VECTORS": 1}), ("read_grid", {"MINI_NCCL_GRID_VECTORS": 2}),
    ("read_grid", {"MINI_NCCL_GRID_VECTORS": 4}),
]
# a DDP-bucket-sized call (25 MiB, torch's default bucket): at 8 ranks its chunks are ~3 MiB, just
# under the grid form's 4 MiB threshold -- the persistent kernel by default, the grid form with
# MINI_NCCL_GRID_MIN lowered; the node's links decide which is faster for such calls
MID_POINTS = [("auto", {}), ("auto", {"MINI_NCCL_GRID_MIN": 262144})]
MID_MIB = 25
ALGO_IDS = {"ring": 0, "read": 2, "read_grid": 4}  # mncclAlgo_t
RAN_AS = {"ring": 0, "read": 2, "read_grid": 2}    # mncclCommInfo_t.last_algo of each (the grid form is read)
ALGO_NAMES = {v: k for k, v in ALGO_IDS.items()}


def kernel_form(algo):
    """The kernel a schedule launches: ring_kernel, the persistent read_kernel or read's grid
    launches (read_grid_kernel): what a PMC entry must have profiled to describe this line's kernel
    ("read_push": the persistent read kernel's key since round 3, when it gained its push form)."""
    return {"read_grid": "read_grid", "ring": "ring"}.get(algo, "read_push")


def fused_bytes(form, esz, chunk, n):
    """Every byte one rank's fused kernel moves through its GPU's HBM per call (DESIGN.md,
    Kernels): the ring reads each chunk of the input and writes each of the output once, and
    2(n-1) chunks land in and are read back from scratch: (6n - 4) chunks; read has no scratch:
    every chunk of the input read once (n - 1 of them by the peers) and every chunk of the output
    written once (n - 1 of them by the peers' pushes): 2n."""
    k = {"ring": 6 * n - 4, "read_push": 2 * n, "read_grid": 2 * n}[form]
    return esz * chunk * k
C4_SLICES = [65536, 131072, 262144, 1048576]
C4_WINDOWS = [16, 32, 64]
# 4 GiB fp32 per rank; MNCCL_BENCH_C4_MIB / MNCCL_BENCH_C4=1 rehearse the grid smaller / at n < 8
C4_COUNT = int(os.environ.get("MNCCL_BENCH_C4_MIB", "4096")) * (1 << 20) // 4


def sweep_point(M, torch, dist, dev, n, rank, env, algo, count, reps, max_over_ranks, dtype="f32"):
    """one communicator with `env` knobs; returns algbw GB/s (max time over ranks) and check"""
    tdt, ndt, esz = {"f32": (torch.float32, M.ncclFloat, 4), "bf16": (torch.bfloat16, M.ncclBfloat16, 2),
                     "f16": (torch.float16, M.ncclFloat16, 2)}[dtype]
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    comm = None
    try:
        comm = M.Comm(n, rank, os.environ.get("MASTER_ADDR", "127.0.0.1"))
        comm.set_algo(M.ALGO_AUTO if algo == "auto" else ALGO_IDS[algo])
        grid0 = comm.info()["read_grid_calls"]
        st = torch.cuda.Stream(device=dev)
        send = torch.ones(count, device=dev, dtype=tdt)
        recv = torch.empty(count, device=dev, dtype=tdt)

        def call():
            rc = comm.all_reduce(send.data_ptr(), recv.data_ptr(), count, ndt, M.ncclSum, st.cuda_stream)
            if rc != 0:
                raise M.NcclError(rc, "ncclAllReduce")

        call()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            call()
        torch.cuda.synchronize()
        dt = max_over_ranks(time.perf_counter() - t0)
        ok = comm.async_error() == 0 and bool((recv == float(n)).all().item())
        ok = ok and verify_calls(M, torch, comm, dev, n, rank, send, recv, count, tdt, ndt, st, 1, dist.barrier)
        i = comm.info()
        # the point ran its own schedule (auto: read where the topology allows it, else the ring)
        want = (2 if i["auto_read"] else 0) if algo == "auto" else RAN_AS[algo]
        ok = ok and i["last_algo"] == want
        ok = max_over_ranks(0.0 if ok else 1.0) == 0.0
        return {"GBps": round(count * esz / (dt / reps) / 1e9, 2), "ok": ok, "workgroups": i["channels"],
                "pipelines": i["pipelines"], "run_pipelines": i["run_pipelines"], "slot_bytes": i["slot_bytes"], "scratch_MiB": i["scratch_bytes"] >> 20,
                "grid_calls": i["read_grid_calls"] - grid0}
    except Exception as e:
        return {"error": str(e)[:120]}
    finally:
        if comm is not None:
            comm.destroy()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        # no torch.cuda.empty_cache(): the next point's tensors come from the same cached segments,
        # so the read schedule shares allocations it shared before (a segment handed back to HIP
        # and re-allocated at the same address would not be shared again, csrc/ipcreg.h)


def verify_calls(M, torch, comm, dev, n, rank, send, recv, count, tdt, ndt, stream, calls=3, barrier=None):
    """Cross-rank result check that a protocol race cannot pass: every call gets new,
    rank- and position-dependent integer-valued inputs (sums exact in any order and in
    bf16/f16), so a stale or torn slot, a missed hand-off or a wrong chunk owner shows up
    as a wrong element.  True when every element of every call matches on this rank."""
    mod = 1021 if tdt == torch.float32 else 8
    chunk = count // n
    body = chunk * n
    piece = 1 << 26  # inputs and expected values built 64 Mi elements at a time: a 4 GiB C4 point
    ok = True        # needs no temporaries beyond send / recv (8 ranks may share one GPU's HBM)

    def vals(a, b, q, c):
        return (torch.arange(a, b, device=dev, dtype=torch.int64) + (7 * q + 31 * c)) % mod

    for c in range(calls):
        for a in range(0, count, piece):
            b = min(count, a + piece)
            send[a:b].copy_(vals(a, b, rank, c))
        recv.fill_(-1)
        torch.cuda.synchronize()
        if barrier is not None:
            barrier()  # every rank enters the call together: input preparation is not the call's skew
        rc = comm.all_reduce(send.data_ptr(), recv.data_ptr(), count, ndt, M.ncclSum, stream.cuda_stream)
        torch.cuda.synchronize()
        ok = ok and rc == 0 and comm.async_error() == 0
        for a in range(0, count, piece):
            if not ok:
                break
            b = min(count, a + piece)
            exp = torch.zeros(b - a, device=dev, dtype=torch.float32)
            for q in range(n):
                exp += vals(a, b, q, c).to(torch.float32)
            if b > body:  # the count % n tail keeps this rank's input
                exp[max(body, a) - a:] = send[max(body, a):b].float()
            ok = bool(torch.equal(recv[a:b].float(), exp))
            del exp
    return ok


def order_ranges(count, n, piece=1 << 24):
    """The pieces verify_order generates and checks, in increasing order: chunk by chunk (so a
    piece never straddles two chunks), then the count % n tail."""
    chunk = count // n
    for c in range(n):
        for a in range(c * chunk, (c + 1) * chunk, piece):
            yield c, a, min((c + 1) * chunk, a + piece)
    if chunk * n < count:
        yield -1, chunk * n, count


def verify_order(M, torch, comm, dev, n, rank, send, recv, count, tdt, ndt, stream, barrier, seed=1234):
    """one call on seeded uniform[-1, 1) inputs (rank q's from seed 1234 + q,
    SURVEY.md s8(d)), every element of the result compared bit for bit with the reference ring's
    association: the reduce of chunk c starts at rank c and visits c+1, ..., c-1, each adding its
    own value as the local operand (mini_nccl.cu:108-126), i.e. x[c-1] + (... + (x[c+1] + x[c])).
    Each rank regenerates every peer's input on its own GPU, piece by piece (the same generator
    stream the peer filled its send buffer with), and folds with torch's own adds -- torch, not the
    oracle, so the check is outside the timed path and the oracle rule.  Unlike verify_calls'
    integer-valued data, a wrong association changes bits here.  Returns "ok" or what differed."""
    chunk = count // n
    ity = torch.int32 if tdt == torch.float32 else torch.int16

    def gen(q):
        g = torch.Generator(device=dev)
        g.manual_seed(seed + q)
        return g

    def draw(g, m):
        return (torch.rand(m, generator=g, device=dev, dtype=torch.float32) * 2 - 1).to(tdt)

    g = gen(rank)
    for _, a, b in order_ranges(count, n):
        send[a:b].copy_(draw(g, b - a))
    recv.fill_(-1)
    torch.cuda.synchronize()
    barrier()
    rc = comm.all_reduce(send.data_ptr(), recv.data_ptr(), count, ndt, M.ncclSum, stream.cuda_stream)
    torch.cuda.synchronize()
    if rc != 0 or comm.async_error() != 0:
        return f"FAILED: ncclAllReduce returned {rc} (async {comm.async_error()})"
    gens = [gen(q) for q in range(n)]
    for c, a, b in order_ranges(count, n):
        xs = [draw(gens[q], b - a) for q in range(n)]
        if c < 0:  # the count % n tail keeps this rank's own input (mini_nccl.cu:69)
            want = xs[rank]
        else:
            want = xs[c]
            for k in range(1, n):
                want = xs[(c + k) % n] + want
        got = recv[a:b]
        if not torch.equal(got.view(ity), want.view(ity)):
            i = int(torch.nonzero(got.view(ity) != want.view(ity))[0].item())
            return (f"FAILED: element {a + i} (chunk {c}) is {got[i].item()!r}, the ring's association gives "
                    f"{want[i].item()!r}")
        del xs, want
    return "ok"


def run_sweeps(M, torch, dist, dev, n, rank, max_over_ranks, with_c4, out, on_point=lambda: None, deadline=None):
    """fills `out` point by point (on_point after each), so a guard that ends the run early or a
    crash still reports what ran.  BASELINE.json's own configs go first (C5, then the C4 grid),
    the exploratory (schedule, knob) points on 256 MiB after them.  Past `deadline` (time.time())
    every rank stops before its next point alike (the ranks agree through max_over_ranks)."""

    def go_on():
        if deadline is None or max_over_ranks(1.0 if time.time() > deadline else 0.0) == 0.0:
            return True
        out["stopped"] = "the sweep's time budget ran out: later points skipped (bench.py LINK_RESERVE_S)"
        return False

    if with_c4:
        # BASELINE.json configs[4] (C5): 1 GiB of bf16 / fp16 per rank, library defaults (auto:
        # read, its large calls in the grid form -- grid_calls says which ran); the check is exact
        # (integer-valued sums stay exact in 2-byte floats)
        c5 = out["c5_read_1GiB"] = {}
        for dt in ("bf16", "f16"):
            if not go_on():
                return out
            if rank == 0:
                log(f"C5: auto {dt}")
            c5[dt] = sweep_point(M, torch, dist, dev, n, rank, {}, "auto", (1 << 30) // 2, 5, max_over_ranks, dtype=dt)
            on_point()
        # BASELINE.json configs[3] (C4): ring, 4 GiB fp32, SLICE x WINDOW
        out["c4_buffer_MiB"] = C4_COUNT * 4 >> 20
        out["c4_knobs"] = ("SLICE_SIZE = payload bytes per message; WINDOW_SIZE x SIGNAL_BATCH (16) = messages in "
                           "flight per link, the reference's bound (mini_nccl.cu:119,144,167): pipelines x 2 slots <= "
                           "WINDOW x 16, at most 256 pipelines; scratch capped at MINI_NCCL_SCRATCH_MB (512): "
                           "(n-1) x pipelines x 2 x SLICE <= cap, so large slices run fewer pipelines "
                           "(csrc/schedule.h pipeline_geometry; each point reports its geometry)")
        # the same 4 GiB with the library defaults (auto: the read schedule, grid form)
        if not go_on():
            return out
        if rank == 0:
            log("C4: library defaults")
        out["c4_read_4GiB_defaults"] = sweep_point(M, torch, dist, dev, n, rank, {}, "auto", C4_COUNT, 3,
                                                   max_over_ranks)
        on_point()
        c4 = out["c4_ring_4GiB"] = []
        for w in C4_WINDOWS:
            for sl in C4_SLICES:
                env = {"MINI_NCCL_WINDOW_SIZE": w, "MINI_NCCL_SLICE_SIZE": sl}
                if not go_on():
                    return out
                if rank == 0:
                    log(f"C4: ring {env}")
                r = sweep_point(M, torch, dist, dev, n, rank, env, "ring", C4_COUNT, 3, max_over_ranks)
                c4.append({"window": w, "slice": sl, **r})
                on_point()
    out.update({"buffer": "256 MiB fp32", "points": []})
    for i, (algo, env) in enumerate(SWEEP_POINTS):
        if not go_on():
            return out
        if rank == 0:
            log(f"sweep {i + 1}/{len(SWEEP_POINTS)}: {algo} {env}")
        r = sweep_point(M, torch, dist, dev, n, rank, env, algo, 64 << 20, 5, max_over_ranks)
        out["points"].append({"algo": algo, "env": {k[len("MINI_NCCL_"):].lower(): v for k, v in env.items()}, **r})
        on_point()
    out["mid_points"] = []
    for algo, env in MID_POINTS:
        if not go_on():
            return out
        if rank == 0:
            log(f"sweep {MID_MIB} MiB: {algo} {env}")
        r = sweep_point(M, torch, dist, dev, n, rank, env, algo, (MID_MIB << 20) // 4, 20, max_over_ranks)
        out["mid_points"].append({"MiB": MID_MIB, "algo": algo,
                                  "env": {k[len("MINI_NCCL_"):].lower(): v for k, v in env.items()}, **r})
        on_point()
    return out


PERF_TEST_MIB = [1, 16, 64, 128]  # tests/perf_test.cpp:69


def size_curve(M, torch, dist, comm, pg, send, recv, stream, n, max_over_ranks, warm=5, reps=20, who=("mini_nccl", "rccl"),
               rows=None):
    """algbw of this library (default schedule) and of RCCL at the reference perf_test's sizes.
    who: the columns measured; rows: an earlier call's rows to add them to (bench.py measures its
    own column right after the schedules, RCCL's among the extras)"""
    rows = [] if rows is None else rows
    by_mib = {r["MiB"]: r for r in rows}
    for mib in PERF_TEST_MIB:
        k = (mib << 20) // 4
        if k > send.numel():
            break
        s_, r_ = send[:k], recv[:k]

        def ours():
            rc = comm.all_reduce(s_.data_ptr(), r_.data_ptr(), k, M.ncclFloat, M.ncclSum, stream.cuda_stream)
            if rc != 0:
                raise M.NcclError(rc, "ncclAllReduce")

        row = by_mib.get(mib) or {"MiB": mib}
        for name, fn in (("mini_nccl", ours), ("rccl", None if pg is None else
                                                  (lambda: torch.distributed.all_reduce(r_, group=pg)))):
            if fn is None or name not in who:
                continue
            try:
                for _ in range(warm):
                    fn()
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(reps):
                    fn()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                dt = max_over_ranks(time.perf_counter() - t0) / reps
                row[name + "_us"] = round(dt * 1e6, 1)
                row[name + "_host_us"] = round(max_over_ranks(t1 - t0) / reps * 1e6, 1)  # the enqueue loop alone
                row[name + "_algbw_GBps"] = round(k * 4 / dt / 1e9, 2)
            except Exception as e:
                if name == "mini_nccl":
                    raise
                pg = None  # RCCL refused (e.g. two ranks on one GPU): skip it from here on
                row["rccl_error"] = str(e)[:80]
                dist.barrier()
        if "mini_nccl" in who:
            ok = comm.async_error() == 0
            ours()
            torch.cuda.synchronize()
            row["schedule"] = {0: "ring", 2: "read", 3: "oneshot"}.get(comm.info()["last_algo"], "?")
            row["ok"] = max_over_ranks(0.0 if (ok and bool((r_ == float(n)).all().item())) else 1.0) == 0.0
        if mib not in by_mib:
            rows.append(row)
    return rows


def small_calls(M, torch, dist, comm, send, recv, stream, n, max_over_ranks, warm=10, reps=100):
    """us per blocking 4 KiB / 64 KiB fp32 call for each schedule (forced), all ranks in step:
    what auto's order for small calls (read first for shareable device buffers, the one-shot for
    the ring's small calls) should be decided from on this topology; read_window: the read
    schedule on registered windows (no host rendezvous)"""
    rows = []
    names = {"ring": M.ALGO_RING, "read": M.ALGO_READ, "oneshot": M.ALGO_ONESHOT, "read_window": M.ALGO_READ}
    wins = None
    try:
        for kib in (4, 64):
            k = (kib << 10) // 4
            s_, r_ = send[:k], recv[:k]
            row = {"KiB": kib}
            for name, a in names.items():
                comm.set_algo(a)
                if name == "read_window" and wins is None:
                    # send / recv registered as windows (mncclCommRegister, collective): the same
                    # calls with no host rendezvous
                    wins = (comm.register(send.data_ptr(), send.numel() * send.element_size()),
                            comm.register(recv.data_ptr(), recv.numel() * recv.element_size()))

                def call():
                    rc = comm.all_reduce(s_.data_ptr(), r_.data_ptr(), k, M.ncclFloat, M.ncclSum, stream.cuda_stream)
                    if rc != 0:
                        raise M.NcclError(rc, f"ncclAllReduce ({name}, {kib} KiB)")
                for _ in range(warm):
                    call()
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(reps):
                    call()
                    torch.cuda.synchronize()
                dt = max_over_ranks(time.perf_counter() - t0) / reps
                ci = comm.info()
                ran = ci["last_algo"]
                if name == "read_window":
                    # with no two ranks on one GPU window calls skip the host rendezvous; ranks sharing
                    # a GPU negotiate them (MINI_NCCL_WINDOW_RENDEZVOUS auto: they meet faster on the host)
                    row["read_window_path"] = "device" if ci["window_fast"] else "negotiated"
                    if ci["window_fast"] and ci["window_calls"] < warm + reps:
                        ran = -1  # not the window path: reported as a failed point
                row[name + "_us"] = round(dt * 1e6, 1)
                row[name + "_ok"] = max_over_ranks(0.0 if (ran == a and bool((r_ == float(n)).all().item()))
                                                   else 1.0) == 0.0
            rows.append(row)
    finally:
        comm.set_algo(M.ALGO_AUTO)
        if wins is not None:
            for h in wins:
                comm.deregister(h)
    return rows


def host_buffer_rate(M, torch, dist, comm, stream, n, max_over_ranks, mib=256, warm=2, reps=5):
    """algbw of ncclAllReduce on pinned host send/recv buffers (never the headline value)"""
    err = None
    try:
        k = (mib << 20) // 4
        hs = torch.ones(k, dtype=torch.float32).pin_memory()
        hr = torch.empty(k, dtype=torch.float32).pin_memory()

        def call():
            rc = comm.all_reduce(hs.data_ptr(), hr.data_ptr(), k, M.ncclFloat, M.ncclSum, stream.cuda_stream)
            if rc != 0:
                raise M.NcclError(rc, "ncclAllReduce (host buffers)")

        for _ in range(warm):
            call()
        torch.cuda.synchronize()
    except Exception as e:
        err = str(e)[:160]
    if max_over_ranks(1.0 if err else 0.0) != 0.0:  # every rank agrees before timing
        return {"error": err or "failed on another rank"}
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    torch.cuda.synchronize()
    dt = max_over_ranks(time.perf_counter() - t0) / reps
    ok = max_over_ranks(0.0 if bool((hr == float(n)).all().item()) else 1.0) == 0.0
    return {"buffer": f"{mib} MiB fp32 pinned host memory (send and recv), mapped into the kernel",
            "algbw_GBps": round(k * 4 / dt / 1e9, 2), "ms": round(dt * 1e3, 3), "ok": ok}


def host_inclusive_n1(M, torch, dev, count, tdt, ndt, reps=3, piece_mib=64):
    """N = 1, the path as the reference's callers use it (host memory in and out,
    perf_test.cpp:78-79): a <- a + b with a and b in pinned host memory, copied H2D, reduced
    by the same local_reduce kernel, the result copied D2H.  "serial": one copy in, one
    launch, one copy out per step; "pipelined": the same in `piece_mib` pieces on a copy-in,
    a compute and a copy-out stream (H2D of piece i+1 and D2H of piece i-1 overlap the
    reduce of piece i).  Never the headline value."""
    esz = torch.empty(0, dtype=tdt).element_size()
    ha = torch.rand(count, dtype=torch.float32).to(tdt).pin_memory()
    hb = torch.rand(count, dtype=torch.float32).to(tdt).pin_memory()
    ref = (ha[: 1 << 20].float() + hb[: 1 << 20].float()).to(tdt)  # one correctly rounded add
    a0 = ha[: 1 << 20].clone()
    da = torch.empty(count, device=dev, dtype=tdt)
    db = torch.empty(count, device=dev, dtype=tdt)
    s_in, s_k, s_out = (torch.cuda.Stream(device=dev) for _ in range(3))
    piece = (piece_mib << 20) // esz

    def reduce_on(s, lo, hi):
        rc = M.local_reduce(da[lo:].data_ptr(), da[lo:].data_ptr(), db[lo:].data_ptr(), hi - lo, ndt, M.ncclSum,
                            s.cuda_stream)
        if rc != 0:
            raise M.NcclError(rc, "mncclLocalReduce")

    def serial():
        with torch.cuda.stream(s_k):
            da.copy_(ha, non_blocking=True)
            db.copy_(hb, non_blocking=True)
            reduce_on(s_k, 0, count)
            ha.copy_(da, non_blocking=True)
        s_k.synchronize()

    def pipelined():
        for lo in range(0, count, piece):
            hi = min(count, lo + piece)
            e_in, e_k = torch.cuda.Event(), torch.cuda.Event()
            with torch.cuda.stream(s_in):
                da[lo:hi].copy_(ha[lo:hi], non_blocking=True)
                db[lo:hi].copy_(hb[lo:hi], non_blocking=True)
                e_in.record(s_in)
            s_k.wait_event(e_in)
            reduce_on(s_k, lo, hi)
            e_k.record(s_k)
            s_out.wait_event(e_k)
            with torch.cuda.stream(s_out):
                ha[lo:hi].copy_(da[lo:hi], non_blocking=True)
        s_out.synchronize()

    out = {"buffers": f"a, b: {count * esz >> 20} MiB {str(tdt).replace('torch.', '')} each in pinned host memory; "
                      "result back in a (host)", "piece_MiB": piece_mib}
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        ha[: 1 << 20].copy_(a0)
        fn()  # warm-up (also the correctness step: a was restored first)
        ok = bool(torch.equal(ha[: 1 << 20], ref))
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        dt = (time.perf_counter() - t0) / reps
        out[name] = {"GBps": round(count * esz / dt / 1e9, 3), "ms": round(dt * 1e3, 3), "first_step_exact": ok}
    del da, db
    return out


# ------------------------------------------------------------------ helpers
def reduce_max(dist, x):
    """max over ranks of a host scalar through the harness's (gloo) process group"""
    if dist is None:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def peer_topology(dev, n, same_device):
    """How this rank's GPU reaches every other rank's (device = rank on the node): the HIP
    runtime's link type and hop count (hipExtGetLinkTypeAndHopCount; 4 = xGMI, 2 = PCIe) and
    whether peer access is possible.  Diagnostics for tuning, never part of `value`."""
    import ctypes
    try:  # the HIP runtime torch (and libmini_nccl.so) already use, never a second copy
        hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_LAZY)
    except OSError:
        return {"error": "HIP runtime not loaded"}
    names = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}
    ndev = ctypes.c_int(0)
    hip.hipGetDeviceCount(ctypes.byref(ndev))
    out = {"visible_devices": ndev.value, "peers": []}
    if same_device:
        out["note"] = "every rank on one GPU (rehearsal)"
        return out
    for q in range(n):
        if q == dev or q >= ndev.value:
            continue
        lt, hc, can = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_int(0)
        rc = hip.hipExtGetLinkTypeAndHopCount(dev, q, ctypes.byref(lt), ctypes.byref(hc))
        hip.hipDeviceCanAccessPeer(ctypes.byref(can), dev, q)
        out["peers"].append({"device": q, "link": names.get(lt.value, lt.value) if rc == 0 else f"rc {rc}",
                             "hops": hc.value if rc == 0 else None, "peer_access": bool(can.value)})
    return out


def pmc_traffic(key, form=None, fused=None):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary (profiles/pmc_summary.json),
    keyed by kernel form.  An entry is used only if it profiled the kernel this line timed: its
    kernel_form must be `form` and its fused_algorithmic_bytes_per_launch must equal `fused` (the
    bytes of the form timed here) -- so a line can never pair one kernel's time with another
    kernel's bytes.  (traffic, source) or (None, why)."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        d = json.load(open(p))
    except Exception as e:
        return None, f"no PMC summary ({str(e)[:60]})"
    e = d.get(key)
    if not e:
        return None, None
    if form is not None and e.get("kernel_form") != form:
        return None, f"refused: {key} profiled kernel form {e.get('kernel_form')!r}, this line timed {form!r}"
    if fused is not None and e.get("fused_algorithmic_bytes_per_launch") != fused:
        return None, (f"refused: {key} describes {e.get('fused_algorithmic_bytes_per_launch')} fused bytes per launch, "
                      f"the kernel timed here moves {fused}")
    return e["hbm_bytes_per_launch"], e.get("source")


def trace_of(key, alg_bytes):
    """The committed kernel trace behind a pmc_summary.json entry (tools/pmc_summary.py writes
    trace_source / trace_mean_ns / head): kernel_source, the trace's mean launch and the roofline
    fraction it gives for `alg_bytes` per launch, or {} when there is none."""
    try:
        e = json.load(open(os.path.join(ROOT, "profiles", "pmc_summary.json"))).get(key) or {}
    except Exception:
        return {}
    if not e.get("trace_source") or not e.get("trace_mean_ns"):
        return {}
    ms = e["trace_mean_ns"] / 1e6
    return {"kernel_source": e["trace_source"], "trace_kernel_ms": round(ms, 4),
            "trace_frac": round(alg_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4), "trace_head": e.get("head"),
            "trace_line": e.get("paired_line")}


EXTRAS_LIMIT_S = float(os.environ.get("MNCCL_BENCH_EXTRAS_S", "300"))
LINK_RESERVE_S = 90.0  # of EXTRAS_LIMIT_S, kept for the link probes that run after the sweeps
_emitted = []


_json_fd = [1]


def quiet_stdout():
    """Native libraries (gloo's connection banner, RCCL's version banner) print to fd 1: send
    fd 1 to stderr for the whole run and keep the real stdout for the one JSON line."""
    sys.stdout.flush()
    _json_fd[0] = os.dup(1)
    os.dup2(2, 1)


_crash = []


def arm(result):
    """Insurance for the extras after the headline: if this process dies on a fatal signal (a
    GPU fault makes the HSA runtime abort), tools/libcrashline.so writes the line as it stands
    now to the real stdout.  Rank 0 only; a missing helper only loses the insurance."""
    if _emitted:
        return
    try:
        if not _crash:
            import ctypes
            lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libcrashline.so"))
            lib.crashline_arm.argtypes = [ctypes.c_int, ctypes.c_char_p]
            _crash.append(lib)
        if _crash[0] is not None:
            _crash[0].crashline_arm(_json_fd[0], json.dumps(result).encode())
    except OSError as e:
        _crash.append(None)
        log("crash-line insurance unavailable:", e)


def emit(result):
    """write THE one JSON line (at most once) to the real stdout; `result` is a dict, or a line a
    rank process already serialised (the self-launch forwards rank 0's)"""
    if not _emitted:
        _emitted.append(True)
        if _crash and _crash[0] is not None:
            _crash[0].crashline_disarm()
        sys.stdout.flush()
        for attempt in range(5):  # the guard thread may serialise while the main thread adds a point
            try:
                line = result if isinstance(result, str) else json.dumps(result)
                break
            except RuntimeError:
                time.sleep(0.05)
        else:
            line = json.dumps({k: v for k, v in list(result.items()) if k != "sweep"})
        os.write(_json_fd[0], (line.rstrip("\n") + "\n").encode())


# ------------------------------------------------------------------ rank processes
def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def die_with_parent():
    """In a rank process spawn_ranks started (MNCCL_BENCH_PARENT = the launcher's pid), before it
    touches the GPU: SIGTERM when the launcher dies (PR_SET_PDEATHSIG), so no rank outlives a killed
    bench.py; a launcher already gone by then ends the rank at once."""
    ppid = os.environ.get("MNCCL_BENCH_PARENT")
    if not ppid:
        return
    import ctypes
    import signal
    try:
        ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGTERM), 0, 0, 0)  # PR_SET_PDEATHSIG = 1
    except Exception:
        return
    if os.getppid() != int(ppid):
        os._exit(1)


def spawn_ranks(argv, n, env=None, timeout=None, grace=30.0):
    """Starts n rank processes of `argv`, one per GPU as the reference's perf_test runs one process
    per rank (tests/perf_test.cpp:34-49): RANK = LOCAL_RANK = r, WORLD_SIZE = n, MASTER_ADDR
    127.0.0.1 and a free MASTER_PORT -- the variables torch.distributed.run sets.  The caller must
    not have touched the GPU (the children are fresh programs, never an exec of this one).  Rank 0's
    stdout is collected, the other ranks' is dropped (bench.py prints its line from rank 0 only);
    stderr is shared.  When a rank fails, the rest get `grace` seconds, then SIGTERM (rank 0 then
    prints its armed line), then SIGKILL; likewise past `timeout`.
    Returns (exit status: the first rank's to fail, or 0; rank 0's last stdout line or None)."""
    import subprocess
    port = free_port()
    base = dict(os.environ if env is None else env)
    # the library's own bootstrap port (bench.py defaults it to MASTER_PORT + 7): a free one too
    base.setdefault("MINI_NCCL_PORT", str(free_port()))
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MNCCL_BENCH_PARENT=str(os.getpid()))
        procs.append(subprocess.Popen(argv, env=e, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    # a launcher that stops this process (SIGTERM at its time limit) stops the ranks too
    import signal

    def stop(signum, frame):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        raise SystemExit(128 + signum)
    old_term = signal.signal(signal.SIGTERM, stop) if threading.current_thread() is threading.main_thread() else None
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    t_end = None if timeout is None else time.time() + timeout
    first_fail, first_rc = None, 0
    while any(p.poll() is None for p in procs):
        if first_fail is None and any(p.poll() not in (None, 0) for p in procs):
            first_fail = time.time()
            first_rc = next(p.returncode for p in procs if p.returncode not in (None, 0))
        late = t_end is not None and time.time() > t_end
        if late or (first_fail is not None and time.time() - first_fail > grace):
            log(f"rank processes: {'time limit' if late else 'a rank failed'}: ending the rest")
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            t_kill = time.time() + 10
            while any(p.poll() is None for p in procs) and time.time() < t_kill:
                time.sleep(0.1)
            for p in procs:
                if p.poll() is None:
                    p.kill()
            for p in procs:
                p.wait()
            break
        time.sleep(0.1)
    reader.join(10)
    if old_term is not None:
        signal.signal(signal.SIGTERM, old_term)
    lines = [ln for ln in (out[0] if out else b"").decode(errors="replace").splitlines() if ln.strip()]
    rc = first_rc or next((p.returncode for p in procs if p.returncode != 0), 0)
    return rc, (lines[-1] if lines else None)


def launch_plan(gpus, world_env, visible, same_device):
    """How bench.py runs: "ranks" -- this process is one rank (a launcher set WORLD_SIZE, or one GPU);
    "spawn" -- start `gpus` rank processes itself (no launcher); ("error", why) -- more GPUs asked for
    than this process sees and not the one-GPU rehearsal (never a silent co-location or N = 1 run)."""
    if world_env is not None or gpus <= 1:
        return "ranks", None
    if not same_device and gpus > visible:
        return "error", (f"--gpus {gpus} but {visible} GPU(s) visible: one process per GPU needs {gpus} GPUs "
                         f"(--same-device rehearses every rank on GPU 0)")
    return "spawn", None


def summarize_proxy(d, n, rc):
    """proxy_allreduce's fields from the rank processes' line `d` (a --core-only N > 1 line): the
    default schedule (config.algo) and the ring, each with ms per call, kernel ms, its fractions and
    its checks; ok only if both ran, rank 0 exited 0 and every check passed."""
    out = {"rc": rc}
    if "error" in d or not d.get("schedules"):
        out["error"] = (d.get("error") or "no line from rank 0")[:300]
    algo = (d.get("config") or {}).get("algo")
    for name, p in (d.get("schedules") or {}).items():
        if "value" not in p:
            out[name] = {"error": p.get("error")}
            continue
        rf = p.get("roofline") or {}
        out["default" if name == algo else name] = {
            "schedule": name, "GBps": p["value"], "ms_per_call": p["ms_per_step"], "kernel_ms": p.get("kernel_ms"),
            "sum_frac": rf.get("frac"), "fused_frac": rf.get("fused_frac"),
            "fused_frac_all_ranks": round(n * rf["fused_frac"], 4) if rf.get("fused_frac") is not None else None,
            "result_check": p.get("result_check"),
            "order_sensitive": (p.get("verify") or {}).get("order_sensitive")}
    out["ok"] = bool(rc == 0 and "default" in out and "ring" in out and all(
        out[k].get("result_check") == "ok" and out[k].get("order_sensitive") == "ok" for k in ("default", "ring")))
    return out


def proxy_allreduce(budget_s=150.0):
    """VERDICT r5 #4, an extra of the N = 1 run (never `value`): BASELINE.json configs[1]'s shape,
    2 rank processes on GPU 0 (all ranks on one GPU, as the reference's perf_test, perf_test.cpp:46),
    256 MiB fp32 per rank, MINI_NCCL_SLICE_SIZE 128 KiB, GPU_MAX_HW_QUEUES=2, 5 warm-up + 20 timed
    calls (perf_test.cpp:86-99): the library's default schedule and the reference's ring, each
    checked bit for bit against the ring's association.  Started as fresh rank processes before this
    process touches the GPU."""
    t0 = time.time()
    n, count = 2, 67108864
    argv = [sys.executable, os.path.abspath(__file__), "--gpus", str(n), "--same-device", "--no-alt", "--no-sweep",
            "--no-cpu-baseline", "--core-only", "--count", str(count), "--steps", "20", "--warmup", "5"]
    env = dict(os.environ, MINI_NCCL_SLICE_SIZE="131072", GPU_MAX_HW_QUEUES="2", MNCCL_BENCH_SAME_DEVICE_QUEUES="2")
    env.pop("MINI_NCCL_ALGO", None)
    out = {"what": "labelled proxy, never `value`: 2 rank processes sharing GPU 0 (BASELINE.json configs[1]'s size; "
                   "every 'link' is this GPU's HBM), 256 MiB fp32 per rank, SLICE 128 KiB, GPU_MAX_HW_QUEUES=2, "
                   "5 + 20 stream-ordered calls per schedule, ms and GB/s = max over ranks of the wall clock between "
                   "barriers; fused_frac_all_ranks = both ranks' fused HBM bytes / rank kernel time / 8 TB/s"}
    try:
        rc, line = spawn_ranks(argv, n, env=env, timeout=budget_s)
        out.update(summarize_proxy(json.loads(line) if line else {}, n, rc))
    except Exception as e:
        out["error"] = str(e)[:200]
        return out
    out["wall_s"] = round(time.time() - t0, 1)
    return out


def main():
    die_with_parent()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)   # perf_test.cpp:93-99: 20 timed
    ap.add_argument("--warmup", type=int, default=5)   # perf_test.cpp:86-90: 5 warm-up
    ap.add_argument("--count", type=int, default=0, help="elements (default: 1 GiB of --dtype)")
    ap.add_argument("--dtype", choices=["f32", "bf16", "f16"], default="f32",
                    help="f32 = the headline; bf16/f16 = BASELINE.json configs[4] (C5)")
    ap.add_argument("--algo", choices=["auto", "ring", "read", "read_grid"],
                    default=os.environ.get("MINI_NCCL_ALGO", "auto"),
                    help="auto = the library default (read for device buffers; same bits whatever the schedule)")
    ap.add_argument("--no-alt", action="store_true", help="skip the extras: N>1 the second schedule and the RCCL reference, N=1 the host-inclusive rate")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true", help="N>1: skip the configuration sweeps")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on GPU 0 (as the reference's perf_test)")
    ap.add_argument("--core-only", action="store_true",
                    help="N>1: the schedules and their checks only (the N = 1 run's proxy_allreduce extra)")
    args = ap.parse_args()
    quiet_stdout()

    # no launcher (WORLD_SIZE unset) and --gpus N > 1: this process starts the N rank processes
    # itself and prints rank 0's line; it never touches the GPU (counting devices does not)
    plan, why = "ranks", None
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        visible = 0
        if not args.same_device:
            import torch
            visible = torch.cuda.device_count()
        plan, why = launch_plan(args.gpus, None, visible, args.same_device)
    if plan == "error":
        log(why)
        emit({"metric": METRIC, "value": 0.0, "unit": "GB/s", "n_gpus": args.gpus, "steps": args.steps,
              "warmup": args.warmup, "higher_is_better": True, "error": why})
        sys.exit(2)
    if plan == "spawn":
        log(f"no launcher: starting {args.gpus} rank processes")
        rc, line = spawn_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus)
        emit(line or json.dumps({"metric": METRIC, "value": 0.0, "unit": "GB/s", "n_gpus": args.gpus,
                                 "higher_is_better": True, "error": f"rank 0 printed no line (exit status {rc})"}))
        sys.exit(rc)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    n = world

    cpu = None
    if n == 1 and rank == 0 and not args.no_cpu_baseline and args.dtype == "f32":
        try:
            cpu = cpu_baseline()  # before the GPU is touched
            log("cpu baseline:", json.dumps(cpu))
        except Exception as e:
            log("cpu baseline failed:", e)

    proxy = None
    if n == 1 and rank == 0 and not args.no_alt and args.dtype == "f32" and args.count == 0:
        # before this process touches the GPU: the rank processes are fresh programs on GPU 0
        log("proxy_allreduce: 2 rank processes on GPU 0, 256 MiB fp32")
        try:
            proxy = proxy_allreduce()
        except Exception as e:
            proxy = {"error": str(e)[:200]}
        log("proxy_allreduce:", json.dumps(proxy))

    cpu_ring = None
    if n > 1 and rank == 0 and not args.no_cpu_baseline:
        try:
            cpu_ring = cpu_ring_baseline(n)  # before the GPU is touched; the other ranks wait
        except Exception as e:
            cpu_ring = {"error": str(e)[:200]}

    if args.same_device:
        # rehearsal with every rank on one GPU: each rank's persistent kernel waits for the
        # others', so all n processes' queues must be mapped at once; the GPU's scheduler maps
        # 16 hardware queues across processes at most (8 x 2 ran at full rate, 8 x 4 -- HIP's
        # default, which the GPU box also exports -- time-sliced ~200x slower:
        # profiles/r2_coloc8_*), and even 2 processes x 4 time-sliced as soon as one more stream
        # was created (every later call ~100 us slower; with 2 queues per process no change:
        # profiles/r5_bench_size_order.txt); set before HIP starts.  Only this rehearsal mode.
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MNCCL_BENCH_SAME_DEVICE_QUEUES", "2")
    import torch
    import mini_nccl as M
    M.load()
    if args.same_device:
        local_rank = 0
    ndev = torch.cuda.device_count()
    if 0 < ndev <= local_rank:  # a launcher that shows each rank only its own GPU(s)
        log(f"LOCAL_RANK {local_rank} but {ndev} visible device(s): using device {local_rank % ndev}")
        local_rank %= ndev
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    if n > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=n)
        os.environ.setdefault("MINI_NCCL_PORT", str(int(os.environ.get("MASTER_PORT", "29500")) + 7))
        os.environ.setdefault("MINI_NCCL_BLOCKING", "0")  # stream-ordered calls, errors checked after

    def barrier_sync():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        return reduce_max(dist, x)

    stream = torch.cuda.Stream(device=dev)
    tdt, ndt, esz = {"f32": (torch.float32, M.ncclFloat, 4), "bf16": (torch.bfloat16, M.ncclBfloat16, 2),
                     "f16": (torch.float16, M.ncclFloat16, 2)}[args.dtype]
    count = args.count or (COUNT * 4) // esz
    nbytes = count * esz
    metric = METRIC if args.dtype == "f32" else METRIC.replace("fp32", args.dtype)
    result = {"metric": metric, "unit": "GB/s", "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
              "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
              "data": "synthetic"}

    def timed(step_fn, k):
        """K steps between barrier+sync; returns (wall s, mean per-launch event ms).  The two HIP
        events bracket the K launches on the stream they run on (no event between launches: a
        marker between back-to-back kernels costs each step ~9 us on MI355X), so the mean is
        the launches' device time per step, inter-launch gaps included."""
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier_sync()
        t0 = time.perf_counter()
        e0.record(stream)
        for i in range(k):
            step_fn()
        e1.record(stream)
        barrier_sync()
        wall = time.perf_counter() - t0
        return wall, e0.elapsed_time(e1) / k

    if n == 1:
        g = torch.Generator(device=dev)
        g.manual_seed(1234)
        a = torch.rand(count, device=dev, generator=g, dtype=torch.float32).to(tdt)
        b = torch.rand(count, device=dev, generator=g, dtype=torch.float32).to(tdt)
        # parity: every step is one IEEE add per element (bf16/f16: correctly rounded), so torch's
        # own add over the FULL buffer, repeated as many times, must give the same bits
        a0 = a.clone()
        sh = stream.cuda_stream

        def step():
            rc = M.local_reduce(a.data_ptr(), a.data_ptr(), b.data_ptr(), count, ndt, M.ncclSum, sh)
            if rc != 0:
                raise M.NcclError(rc, "mncclLocalReduce")

        step()
        torch.cuda.synchronize()
        ref = a0 + b
        exact = bool(torch.equal(a, ref))  # first step, all `count` elements
        for _ in range(args.warmup):
            step()
        wall, ev_ms = timed(step, args.steps)
        # every step of the job (1 + warmup + timed), recomputed by torch, compared bit for bit;
        # the recompute is timed too (events on torch's current stream, where add_ runs): the
        # same bytes through PyTorch-ROCm's own element-wise kernel, for comparison
        torch.cuda.synchronize()
        t0e, t1e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0e.record()
        for _ in range(args.warmup + args.steps):
            ref.add_(b)
        t1e.record()
        torch.cuda.synchronize()
        torch_add_ms = t0e.elapsed_time(t1e) / (args.warmup + args.steps)
        exact_all = bool(torch.equal(a, ref))
        del ref, a0
        ms = wall / args.steps * 1e3
        alg_bytes = 3 * nbytes
        result.update({
            "value": round(nbytes / (ms / 1e3) / 1e9, 3),
            "ms_per_step": round(ms, 4),
            "config": {"workload": f"1-GPU local reduce a <- a + b, 1 GiB {args.dtype} (BASELINE.md row '1-GPU local reduce')",
                       "count": count, "bytes": nbytes, "kernel": f"local_reduce_vec<{args.dtype},Sum>",
                       "parity_step_exact": exact, "parity_all_steps_exact": exact_all,
                       "parity_check": "full buffer vs torch's own add repeated 1 + warmup + steps times",
                       "torch_add": {"ms": round(torch_add_ms, 4),
                                     "GBps": round(nbytes / (torch_add_ms / 1e3) / 1e9, 3),
                                     "what": "the parity recompute a.add_(b): same bytes through torch's own kernel"}},
        })
        traffic, tsrc = pmc_traffic(f"local_reduce_{args.dtype}_1GiB", "local_reduce", None)
        kern_key = "local_reduce_vec"
    else:
        comm = M.Comm(n, rank, os.environ.get("MASTER_ADDR", "127.0.0.1"))
        info = comm.info()
        # the headline runs the library's default for device buffers (MINI_NCCL_ALGO=auto: at the
        # bench's sizes the read schedule -- one-shot is for calls of <= 64 KiB);
        # --algo forces one schedule
        auto_mode = args.algo == "auto"
        if auto_mode:
            # auto: read where the topology rule allows it on every pair of ranks, else the ring
            # (schedule.h topology_blocks_read; the library decides, the line reports)
            args.algo = ("read" if info["auto_read"] else "ring") if info["algo"] < 0 else ALGO_NAMES[info["algo"]]
            # ... its large calls in the grid form (auto_grid; schedule.h read_grid_form: <= 8 ranks,
            # chunks of >= 4 MiB in whole 16-byte vectors)
            chunk_b = (count // n) * esz
            if (args.algo == "read" and info["auto_grid"] and n <= 8 and chunk_b >= (4 << 20)
                    and chunk_b % 16 == 0):
                args.algo = "read_grid"
        headline_algo = args.algo
        send = torch.ones(count, device=dev, dtype=tdt)
        recv = torch.empty(count, device=dev, dtype=tdt)
        sh = stream.cuda_stream
        sum_bytes = 3 * esz * (n - 1) * (count // n)  # the scatter-reduce sum's bytes

        def make_step():
            def step():
                rc = comm.all_reduce(send.data_ptr(), recv.data_ptr(), count, ndt, M.ncclSum, sh)
                if rc != 0:
                    raise M.NcclError(rc, "ncclAllReduce")
            return step

        def inject(where):
            """MNCCL_BENCH_INJECT=<where>: rehearses the failure paths below (a GPU fault aborts the
            process: the armed line must still come out).  Stages after the ring: run_read (the
            headline), sizes, small_calls, standalone, rccl, host_buffers, sweep, probe (last);
            <stage>_error raises
            an ncclInternalError there instead; verify_<algo> marks that schedule's results wrong on
            rank 0 (run_algo)"""
            if os.environ.get("MNCCL_BENCH_INJECT") == where and rank == 0:
                log(f"injected abort at {where}")
                os.abort()
            if os.environ.get("MNCCL_BENCH_INJECT") == where + "_error":
                raise M.NcclError(M.ncclInternalError, f"injected at {where} (MNCCL_BENCH_INJECT)")

        fallbacks = {}
        verifies = {}

        def run_algo(algo, auto=False):
            comm.set_algo(M.ALGO_AUTO if auto else ALGO_IDS[algo])
            inject(f"run_{algo}")
            grid0 = comm.info()["read_grid_calls"]
            step = make_step()
            recv.fill_(-1.0)
            for _ in range(max(1, args.warmup)):
                step()
            torch.cuda.synchronize()
            ok = bool((recv == float(n)).all().item())  # perf_test.cpp:101-134 known answer
            wall, ev_ms = timed(step, args.steps)
            ae = comm.async_error()
            ok = ok and ae == 0 and bool((recv == float(n)).all().item())
            # then 3 calls on varying data (outside the timed region), restoring the buffers
            ok = ok and verify_calls(M, torch, comm, dev, n, rank, send, recv, count, tdt, ndt, stream,
                                    barrier=dist.barrier)
            # and one call on seeded uniform data against the ring's association, every element
            order = verify_order(M, torch, comm, dev, n, rank, send, recv, count, tdt, ndt, stream, dist.barrier)
            bad_order = max_over_ranks(0.0 if order == "ok" else 1.0 + rank)
            verifies[algo] = {"order_sensitive": "ok" if bad_order == 0.0 else
                              (order if order != "ok" else f"FAILED on rank {int(bad_order) - 1}"),
                              "what": "seeded uniform[-1, 1) inputs (seed 1234 + rank), every element of every "
                                      "rank vs torch fp32 adds in the ring's association x[c-1] + (... + "
                                      "(x[c+1] + x[c])), bit for bit",
                              "integer_calls": "3 calls of rank- and position-dependent integer data, every "
                                               "element" + ("" if ok else ": FAILED")}
            ok = ok and order == "ok"
            i = comm.info()
            ran_ok = i["last_algo"] == RAN_AS[algo]  # the timed calls ran this schedule (no fallback)
            if algo == "read_grid":  # every call of the point (warm-up, timed, checks) in the grid form
                ran_ok = ran_ok and i["read_grid_calls"] - grid0 >= max(1, args.warmup) + args.steps
            if not ran_ok:
                # e.g. the read schedule could not map a peer's buffers on this node and the calls
                # ran the ring: on record in the line, not only as a FAILED check
                fallbacks[algo] = {"rank": rank, "ran": {0: "ring", 2: "read", 3: "oneshot"}.get(i["last_algo"], "?"),
                                   "grid_calls": i["read_grid_calls"] - grid0,
                                   "read_map_failures": i["read_map_failures"],
                                   "ipc_open_failures": i["ipc_open_failures"], "cap_refusals": i["cap_refusals"]}
                log(f"rank {rank}: {algo} calls ran {fallbacks[algo]['ran']}: {fallbacks[algo]}")
                result["config"]["fallbacks"] = dict(fallbacks)
            ok = ok and ran_ok
            if os.environ.get("MNCCL_BENCH_INJECT") == f"verify_{algo}" and rank == 0:
                ok = False  # rehearses a wrong-result schedule (the line must fall back to the ring's number)
                verifies.setdefault(algo, {})["order_sensitive"] = "FAILED: injected (MNCCL_BENCH_INJECT)"
            send.fill_(1.0)
            ok = max_over_ranks(0.0 if ok else 1.0) == 0.0
            return max_over_ranks(wall), max_over_ranks(ev_ms), ok

        def point(algo, wall, ev_ms, ok):
            """one schedule's measured line: algbw, its kernel's roofline fraction (SURVEY s8(d)
            sum bytes over the fused kernel's own time) and every byte it moves through HBM"""
            ms_ = wall / args.steps * 1e3
            fused = fused_bytes(kernel_form(algo), esz, count // n, n)
            return {"algo": algo, "kernel_form": kernel_form(algo),
                    "value": round(nbytes / (ms_ / 1e3) / 1e9, 3), "ms_per_step": round(ms_, 4),
                    "kernel_ms": round(ev_ms, 4), "result_check": "ok" if ok else "FAILED",
                    "verify": verifies.get(algo),
                    "roofline": {"frac": round(sum_bytes / (ev_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "fused_frac": round(fused / (ev_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "fused_alg_bytes_per_launch": fused}}

        def set_line(algo, wall, ev_ms, ok, note=None):
            """the line's headline fields from one schedule's measurement"""
            ms_ = wall / args.steps * 1e3
            bw = nbytes / (ms_ / 1e3) / 1e9
            fused = fused_bytes(kernel_form(algo), esz, count // n, n)
            fa = fused / (ev_ms / 1e3) / 1e9
            result.update({
                "value": round(bw, 3),
                "ms_per_step": round(ms_, 4),
                "busbw": round(bw * 2 * (n - 1) / n, 3),
                "config": {"workload": f"{n}-rank all-reduce (reference ring association), 1 GiB {args.dtype} per "
                                       f"rank, HIP IPC over xGMI, {algo} schedule",
                           "count": count, "bytes": nbytes, "algo": algo, "slice_bytes": info["slice_bytes"],
                           "channels": info["channels"], "slots": info["slots"], "threads": info["threads"],
                           "pipelines": info["pipelines"], "run_pipelines": info["run_pipelines"],
                           "scratch_bytes": info["scratch_bytes"],
                           "ranks_on_device": info["ranks_on_device"],
                           "parallelism": f"dp{n}", "result_check": "ok" if ok else "FAILED",
                           "headline_schedule": headline_why,
                           "auto_schedule": {"read": bool(info["auto_read"]), "reason": info["auto_reason"],
                                             "rank0_peer_link": info["peer_link"],
                                             "rank0_peer_hops": info["peer_hops"],
                                             "rule": "auto runs read only if every pair of ranks shares a GPU or "
                                                     "is one xGMI hop apart (csrc/schedule.h topology_blocks_read)"}},
                "roofline": {"bound": "hbm", "achieved": round(sum_bytes / (ev_ms / 1e3) / 1e9, 2),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(sum_bytes / (ev_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                             "traffic": None, "kernel": f"{algo}_kernel", "kernel_form": kernel_form(algo),
                             "kernel_ms": round(ev_ms, 4),
                             "alg_bytes_per_launch": sum_bytes, "fused_alg_bytes_per_launch": fused,
                             "fused_achieved": round(fa, 2), "fused_frac": round(fa / HBM_PEAK_GBS, 4)},
                # the host path beside every N: the CPU ring, timed before the GPU was
                # touched
                "cpu_baseline": cpu_ring,
            })
            if note:
                result["config"]["result_check"] = note
            if fallbacks:
                result["config"]["fallbacks"] = dict(fallbacks)
            return bw

        headline_why = ("the library default for device buffers (MINI_NCCL_ALGO=auto -> read: each rank folds its "
                        "chunk from the peers' send buffers over the links in the reference ring's association "
                        "order and pushes the result into every peer's recv -- the same bits as the ring, 2/n of the buffer per "
                        "link instead of 2(n-1)/n through one link); the north star's ring is measured first and "
                        "beside it in schedules.ring with its own roofline and link fractions; headline_check "
                        "states whether this line's own numbers uphold that default"
                        if headline_algo == "read" else
                        "the library default for device buffers (MINI_NCCL_ALGO="
                        "auto -> read, its large calls in the grid form: a one-wave START, a grid of one-batch workgroups that fold each "
                        "KiB of the rank's chunk from the peers' send buffers in the ring's association order and push "
                        "it into every peer's recv, a one-wave DONE); the persistent read kernel and the north star's "
                        "ring are measured beside it (schedules.read, schedules.ring), headline_check compares them"
                        if headline_algo == "read_grid" and auto_mode else
                        f"{headline_algo} ({'forced by --algo' if not auto_mode else 'auto'})")
        # 0. a line exists before anything runs on the GPU: if the process dies (a GPU fault
        # aborts it), the armed line is printed
        result.update({"value": 0.0, "cpu_baseline": cpu_ring,
                       "error": "the process died before any schedule was measured"})
        if rank == 0:
            arm(result)
        result.pop("error")
        result["schedules"] = {}
        # 1. the reference's ring first (the north star's schedule, C3's "8 MI355X ring"): measured
        # and armed before the default, so a fault in the default still leaves a measured line
        ring_meas = None
        if headline_algo != "ring":
            if rank == 0:
                log("schedule ring (armed first)")
            try:
                wr, er, okr = run_algo("ring")
                ring_meas = (wr, er, okr)
                result["schedules"]["ring"] = point("ring", wr, er, okr)
                set_line("ring", wr, er, okr, note=f"PROVISIONAL: the ring's line; the default schedule "
                                                   f"({headline_algo}) was being measured when the process ended")
                if rank == 0:
                    arm(result)
            except M.NcclError as e:
                result["schedules"]["ring"] = {"algo": "ring", "error": str(e)[:200]}
        # 2. the headline: the library default (or --algo)
        try:
            wall, ev_ms, ok = run_algo(headline_algo, auto=auto_mode)
            result["schedules"][headline_algo] = point(headline_algo, wall, ev_ms, ok)
            algbw = set_line(headline_algo, wall, ev_ms, ok)
            if not ok and ring_meas and ring_meas[2]:
                # the default's results were wrong on some rank (verify_calls / verify_order): a
                # number for wrong bits is no measurement -- the line carries the ring's (checked ok),
                # the default's failure on record in schedules.<algo> and result_check
                algbw = set_line("ring", *ring_meas,
                                 note=f"FAILED: the default schedule ({headline_algo}) gave wrong results on some "
                                      f"rank ({(result['schedules'][headline_algo].get('verify') or {}).get('order_sensitive')}); "
                                      "value is the ring's")
                result["config"]["headline_error"] = f"{headline_algo}: wrong results"
        except M.NcclError as e:
            # the default schedule failed (every rank's calls fail alike): the line says so
            # (result_check FAILED, headline_error) and carries the ring's number, measured on a
            # new communicator, so the failure is on record with a measured fallback beside it
            headline_error = f"{headline_algo}: {str(e)[:200]}"
            result["schedules"][headline_algo] = {"algo": headline_algo, "error": headline_error}
            log(f"headline failed ({e}); new communicator, ring schedule")
            try:
                comm.destroy()
            except Exception:
                pass
            torch.cuda.synchronize()
            dist.barrier()
            comm = M.Comm(n, rank, os.environ.get("MASTER_ADDR", "127.0.0.1"))
            auto_mode = False
            args.algo = "ring"
            wall, ev_ms, ok = run_algo("ring")
            algbw = set_line("ring", wall, ev_ms, False,
                             note=f"FAILED: the default schedule failed ({headline_error}); value is the ring's")
            result["config"]["headline_error"] = headline_error
        else:
            args.algo = headline_algo
        if rank == 0:
            arm(result)
        # 3. the other schedules on the same buffers (same bits), each its own labelled point
        if not args.no_alt:
            for other in ("ring", "read", "read_grid"):
                if other in result["schedules"]:
                    continue
                if rank == 0:
                    log(f"schedule {other}")
                try:
                    result["schedules"][other] = point(other, *run_algo(other))
                except Exception as e:
                    result["schedules"][other] = {"algo": other, "error": str(e)[:200]}
                if rank == 0:
                    arm(result)
            comm.set_algo(M.ALGO_AUTO if auto_mode else ALGO_IDS[args.algo])
        # the rule behind the default, checked against this line's own numbers: read stays the
        # library default while it moves the buffer at least as fast as the reference's ring
        rd, rg = result["schedules"].get("read", {}), result["schedules"].get("ring", {})
        gd = result["schedules"].get("read_grid", {})
        if "value" in rd and "value" in rg:
            # the default's form of read: the grid form where auto chose it (every rank alone on its GPU)
            dflt = gd if headline_algo == "read_grid" and "value" in gd else rd
            other = rd if dflt is gd else gd
            result["config"]["headline_check"] = {
                "rule": "read (in the form auto chose) is the default while its value >= schedules.ring.value (same "
                        "buffers, same bits); otherwise this node should run MINI_NCCL_ALGO=ring; the form auto chose "
                        "should also be >= the other read form",
                "default_form": "read_grid" if dflt is gd else "read",
                "read_GBps": rd["value"], "ring_GBps": rg["value"], "read_over_ring": round(rd["value"] / rg["value"], 3),
                "holds": dflt["value"] >= rg["value"]}
            if "value" in gd:
                result["config"]["headline_check"].update({
                    "read_grid_GBps": gd["value"], "read_grid_over_read": round(gd["value"] / rd["value"], 3),
                    "form_holds": dflt["value"] >= other["value"]})
        if rank == 0:
            arm(result)
        # 3b. this library at the reference perf_test's sizes and small calls by schedule, right
        # after the schedules (the link probes below left later small calls of co-located ranks
        # 5x slower on the one-GPU proxy, profiles/r5_bench_size_order.txt); RCCL's column of
        # `sizes` is added among the extras
        if args.dtype == "f32" and not args.core_only:
            if rank == 0:
                log("sizes, small calls")
            try:
                inject("sizes")
                result["sizes"] = size_curve(M, torch, dist, comm, None, send, recv, stream, n, max_over_ranks,
                                             who=("mini_nccl",))
            except Exception as e:
                result["sizes"] = {"error": str(e)[:200]}
            try:
                inject("small_calls")
                result["small_calls"] = small_calls(M, torch, dist, comm, send, recv, stream, n, max_over_ranks)
            except Exception as e:
                result["small_calls"] = {"error": str(e)[:200]}
            comm.set_algo(M.ALGO_AUTO if auto_mode else ALGO_IDS[args.algo])
            if rank == 0:
                arm(result)
        def measure_links():
            """the link probes (step 4), run LAST: after the first probe this process's later calls ran
            ~100 us slower each on the one-GPU proxy, new communicators included (cause not isolated,
            profiles/r5_bench_size_order.txt) -- so nothing measured after them, RCCL's number and the
            sweeps included, may run behind them"""
            # 4. the xGMI roofline the schedules are bound by, after the schedules themselves: bytes
            # per link with the hot path's access forms, one link per rank (the ring's) and every link
            # at once (read's loads and pushes)
            link = {}
            lc = None
            try:
                # a communicator of its own (the run's was destroyed before the sweeps), same knobs
                lc = M.Comm(n, rank, os.environ.get("MASTER_ADDR", "127.0.0.1"))
                torch.cuda.synchronize()
                dist.barrier()
                inject("probe")
                # min over ranks (the ceiling is set by the slowest link); max alongside for the spread
                pn = lc.link_probe(False, 0, 10)
                pm = lc.link_probe(True, 0, 10)
                link["probe_next_GBps"] = round(max_over_ranks(-pn) * -1, 2)
                link["probe_mesh_GBps_per_link"] = round(max_over_ranks(-pm) * -1, 2)
                link["probe_next_max_GBps"] = round(max_over_ranks(pn), 2)
                link["probe_mesh_max_GBps_per_link"] = round(max_over_ranks(pm), 2)
                var = {}
                # *_user: the peers' ordinary device memory (hipMalloc, what the read schedule loads
                # from) instead of their uncached scratch
                for name, form, pull, user in (("push_nt", "nt", False, False), ("push_plain", "plain", False, False),
                                               ("pull_sys", "sys", True, False), ("pull_plain", "plain", True, False),
                                               ("pull_sys_user", "sys", True, True), ("push_sys_user", "sys", False, True)):
                    for where, allp in (("next", False), ("mesh", True)):
                        g = lc.link_probe(allp, 0, 10, form=form, pull=pull, user=user)
                        var[f"{where}_{name}"] = round(max_over_ranks(-g) * -1, 2)
                link["probe_variants_GBps_per_link"] = var
            except Exception as e:
                link["error"] = str(e)[:200]
            finally:
                if lc is not None:
                    lc.destroy()
            if rank == 0:
                try:
                    link["topology_rank0"] = peer_topology(local_rank, n, args.same_device)
                except Exception as e:
                    link["topology_rank0"] = {"error": str(e)[:120]}
            # each schedule's ceiling from the probed links (min over ranks): the ring moves
            # 2(n-1)/n of the buffer through one link; read 2/n per link direction, half as loads (its
            # fold: the probe's mesh pull from user memory) and half as stores (its result pushes: the
            # mesh push into user memory) -> n / (1/pull + 1/push)
            if args.same_device:
                # every "link" of the one-GPU rehearsal is this GPU's HBM, shared with the other ranks'
                # kernels: a schedule's rate over that is no link fraction (round 2 printed 1.43)
                link["frac"] = None
                link["note"] = "ranks share one GPU: the probes measure its HBM, not xGMI; no link fractions"
            elif "probe_next_GBps" in link:
                pv = link.get("probe_variants_GBps_per_link", {})
                pull = pv.get("mesh_pull_sys_user") or pv.get("mesh_pull_sys")
                push = pv.get("mesh_push_sys_user") or link["probe_mesh_GBps_per_link"]
                ceil = {"ring": link["probe_next_GBps"] * n / (2 * (n - 1))}
                if pull and push:
                    ceil["read"] = n / (1.0 / pull + 1.0 / push)
                link.update({f"{a}_ceiling_GBps": round(c, 2) for a, c in ceil.items()})
                for a, ptn in result["schedules"].items():
                    if a in ceil and "value" in ptn:
                        ptn["link_frac"] = round(ptn["value"] / ceil[a], 4)
                if args.algo in ceil:
                    link["frac"] = round(algbw / ceil[args.algo], 4)
            result["link"] = link
            if rank == 0:
                arm(result)
        form = kernel_form(args.algo)
        traffic, tsrc = pmc_traffic(f"{form}_{args.dtype}_1GiB_n{n}" + ("_same_gpu" if args.same_device else ""),
                                    form, fused_bytes(form, esz, count // n, n))
        if traffic is not None:
            result["roofline"].update({"traffic": traffic, "traffic_source": tsrc})
        elif tsrc:
            result["roofline"]["traffic_note"] = tsrc
        kern_key = f"{args.algo}_kernel"
    if n == 1:
        achieved = alg_bytes / (ev_ms / 1e3) / 1e9
        result["roofline"] = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                              "kernel": kern_key, "kernel_ms": round(ev_ms, 4), "alg_bytes_per_launch": alg_bytes}
        if traffic is not None:
            result["roofline"]["traffic_source"] = tsrc
        # the committed rocprofv3 kernel trace of the same kernel: its mean launch and
        # the fraction it gives, beside the live HIP-event figure above
        tr = trace_of(f"local_reduce_{args.dtype}_1GiB", alg_bytes)
        if tr:
            result["roofline"].update(tr)
    if n > 1 and not args.core_only:
        # roofline.frac above is SURVEY §8(d)'s sum bytes over the FUSED all-reduce kernel's time.
        # For reference only: the same element-wise op as a standalone launch on THIS GPU over the
        # (n-1) * chunk elements a rank reduces per call (same bytes), HIP events around each
        # launch -- what the sum would cost if nothing else (links, hand-offs) bounded it
        m = (n - 1) * (count // n)
        sk_ms, sk_err = 0.0, None
        # on a real node every rank has its own GPU; ranks sharing one GPU take turns
        for turn in (range(n) if args.same_device else [rank]):
            if args.same_device:
                dist.barrier()
            if turn != rank:
                continue
            try:
                inject("standalone")
                sh_ = stream.cuda_stream
                ks = []
                for i in range(25):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    rc = M.local_reduce(recv.data_ptr(), recv.data_ptr(), send.data_ptr(), m, ndt, M.ncclSum, sh_)
                    e1.record(stream)
                    if rc != 0:
                        raise M.NcclError(rc, "mncclLocalReduce")
                    if i >= 5:
                        ks.append((e0, e1))
                torch.cuda.synchronize()
                sk_ms = sum(a.elapsed_time(b) for a, b in ks) / len(ks)
            except Exception as e:
                sk_ms, sk_err = float("inf"), str(e)[:200]
        sk_ms = max_over_ranks(sk_ms)  # every rank gets here, failed or not
        if sk_err is None and sk_ms != float("inf"):
            sk = 3 * esz * m / (sk_ms / 1e3) / 1e9
            result["roofline"]["standalone_sum_kernel_reference"] = {
                "kernel": "local_reduce_vec (separate launch, not the all-reduce)", "elements": m,
                "alg_bytes": 3 * esz * m, "kernel_ms": round(sk_ms, 4), "achieved": round(sk, 2),
                "frac": round(sk / HBM_PEAK_GBS, 4)}
        else:
            result["roofline"]["standalone_sum_kernel_reference"] = {"error": sk_err or "failed on another rank"}
    # the extras below (RCCL's number, the sweeps) must never cost the headline line: if they
    # have not finished in EXTRAS_LIMIT_S, every rank gives up and rank 0 prints what it has
    if n == 1 and not args.no_alt:
        # PCIe-inclusive end-to-end rate (host buffers in and out); never `value`
        arm(result)
        try:
            result["host_inclusive"] = host_inclusive_n1(M, torch, dev, count, tdt, ndt)
        except Exception as e:
            result["host_inclusive"] = {"error": str(e)[:200]}
    if n == 1:
        result["cpu_baseline"] = cpu
        if proxy is not None:
            result["proxy_allreduce"] = proxy
    elif cpu_ring is not None:
        result["cpu_ring_baseline"] = cpu_ring  # the same object as cpu_baseline (kept under its old name)
    if rank == 0:
        arm(result)
    guard = None
    if n > 1:
        import threading

        def bail():
            result["extras"] = (f"RCCL reference / sweeps unfinished after {EXTRAS_LIMIT_S} s: the rest skipped "
                                "(the points above ran)")
            if rank == 0:
                emit(result)
            os._exit(0)
        guard = threading.Timer(EXTRAS_LIMIT_S, bail)
        guard.daemon = True
        guard.start()
        t_guard = time.time()
    if n > 1 and not args.no_alt and not args.core_only:
        # the comparison ceiling: RCCL's all-reduce on the same buffer (torch.distributed nccl)
        pg = None
        if rank == 0:
            log("extras: RCCL reference")
        try:
            inject("rccl")
            if args.same_device:
                raise RuntimeError("skipped: every rank on one GPU (RCCL needs one GPU per rank)")
            import torch.distributed as dist_
            pg = dist_.new_group(backend="nccl")
            x = torch.ones(count, device=dev, dtype=tdt)
            for _ in range(max(1, args.warmup)):
                dist_.all_reduce(x, group=pg)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                dist_.all_reduce(x, group=pg)
            torch.cuda.synchronize()
            dist.barrier()
            w3 = max_over_ranks(time.perf_counter() - t0)
            result["rccl_reference"] = {"value": round(nbytes / (w3 / args.steps) / 1e9, 3),
                                        "ms_per_step": round(w3 / args.steps * 1e3, 4)}
            del x
        except Exception as e:
            result["rccl_reference"] = {"error": str(e)[:200]}
            pg = None
        if rank == 0:
            arm(result)
        # the reference's perf_test sizes (perf_test.cpp:69: 1/16/64/128 MiB): RCCL's all-reduce
        # beside this library's column (measured after the schedules), device-resident fp32
        if pg is not None and args.dtype == "f32" and isinstance(result.get("sizes"), list):
            if rank == 0:
                log("extras: RCCL at the perf_test sizes")
            try:
                size_curve(M, torch, dist, comm, pg, send, recv, stream, n, max_over_ranks, who=("rccl",),
                           rows=result["sizes"])
            except Exception as e:
                result["sizes_rccl_error"] = str(e)[:200]
            if rank == 0:
                arm(result)
        # the reference's own usage: host buffers in, host buffers out (perf_test.cpp:78-79);
        # pinned memory is mapped into the kernel, so this is the PCIe-inclusive end-to-end rate
        if args.dtype == "f32":
            if rank == 0:
                log("extras: host buffers")
            try:
                inject("host_buffers")
                result["host_buffers"] = host_buffer_rate(M, torch, dist, comm, stream, n, max_over_ranks)
            except M.NcclError as e:
                result["host_buffers"] = {"error": str(e)[:200]}
            if rank == 0:
                arm(result)
    if n > 1:
        comm.destroy()
        del send, recv  # back to torch's cache (not to HIP: see sweep_point)
        if not args.no_sweep and args.dtype == "f32":
            t_sw = time.time()
            result["sweep"] = {}
            inject("sweep")
            run_sweeps(M, torch, dist, dev, n, rank, max_over_ranks,
                       with_c4=(n == 8 or os.environ.get("MNCCL_BENCH_C4") == "1"), out=result["sweep"],
                       on_point=(lambda: arm(result)) if rank == 0 else (lambda: None),
                       deadline=t_guard + EXTRAS_LIMIT_S - LINK_RESERVE_S)
            result["sweep"]["wall_s"] = round(time.time() - t_sw, 1)
    if n > 1 and not args.core_only:
        if rank == 0:
            log("link probes (last)")
        measure_links()
    if guard is not None:
        guard.cancel()
    if rank == 0:
        emit(result)
    if n > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except Exception as e:  # still one JSON line from rank 0, so the failure is on record
        import traceback
        traceback.print_exc()
        if int(os.environ.get("RANK", "0")) == 0 and not _emitted:
            emit({"metric": METRIC, "value": 0.0, "unit": "GB/s", "n_gpus": int(os.environ.get("WORLD_SIZE", "1")),
                  "higher_is_better": True, "error": f"{type(e).__name__}: {e}"[:500]})
        sys.exit(1)
