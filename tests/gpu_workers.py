"""Rank processes for the multi-process GPU tests (spawned; one process = one rank).

Placement (rank_device): rank r runs on GPU r % ndev of the box -- one rank per GPU on a
multi-GPU box, as the node runs (so the suite, unedited, is a cross-device parity run over
xGMI there) -- and every rank on GPU 0 on a 1-GPU box or under MNCCL_TEST_COLOCATE=1 (the
reference's perf_test topology, tests/perf_test.cpp:46).  Co-located, every rank opens the
others' scratch / mailbox / buffers through IPC on the same device, so the whole cross-process
protocol (bootstrap, IPC mapping, flags, credits, sequence continuation, aborts) still runs
for real.  Every rank reports the device and the ranks_on_device its communicator saw, and the
tests check them against the placement they asked for.  The oracle each rank compares
against is computed in-process from the same seeded inputs.
"""
import os
import sys
import time
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "mini-nccl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def colocated(env=None):
    """MNCCL_TEST_COLOCATE=1: every rank on GPU 0 whatever the box (today's 1-GPU layout)."""
    v = (env if env is not None else os.environ).get("MNCCL_TEST_COLOCATE", "0")
    return v not in ("", "0")


def rank_device(rank, ndev, colocate=None):
    """The GPU rank `rank` runs on, given `ndev` visible GPUs: rank % ndev, or 0 when co-located."""
    if colocate is None:
        colocate = colocated()
    return 0 if colocate or ndev < 2 else rank % ndev


def ranks_sharing_device(rank, n, ndev, colocate=None):
    """Ranks of an n-rank communicator on `rank`'s GPU (itself included): the communicator's
    mncclCommInfo_t.ranks_on_device under this placement."""
    d = rank_device(rank, ndev, colocate)
    return sum(1 for q in range(n) if rank_device(q, ndev, colocate) == d)


def use_rank_device(rank):
    """In a rank process: select rank_device(rank) (TEST_DEVICE=<d> overrides) and return it."""
    import hip_rt
    d = os.environ.get("TEST_DEVICE")
    d = int(d) if d not in (None, "") else rank_device(rank, hip_rt.device_count())
    hip_rt.set_device(d)
    return d


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def compare(got, exp, dtype, arith):
    """Number of mismatching elements: bit-exact, except NaN payloads of arithmetic ops."""
    if dtype in ("f32", "f64", "f16") and arith:
        gn, en = np.isnan(got), np.isnan(exp)
        bad = (gn != en) | (~gn & (got.view(np.uint8).reshape(got.size, -1) != exp.view(np.uint8).reshape(exp.size, -1)).any(axis=1))
        return int(bad.sum()), (int(np.argmax(bad)) if bad.any() else -1)
    eq = (got.view(np.uint8).reshape(got.size, -1) == exp.view(np.uint8).reshape(exp.size, -1)).all(axis=1)
    return int((~eq).sum()), (int(np.argmin(eq)) if not eq.all() else -1)


def make_inputs(n, count, dtype, seed, special):
    import oracle_api as O
    xs = O.random_inputs(n, count, dtype, seed=seed)
    if special and dtype in ("f32", "f64"):
        vals = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40], dtype=xs[0].dtype)
        for r, x in enumerate(xs):
            g = np.random.default_rng(seed * 31 + r)
            k = g.choice(count, size=min(count, 64), replace=False)
            x[k] = vals[np.arange(k.size) % vals.size]
    return xs


def allreduce_rank(rank, n, port, cases, env, out_q, barrier=None):
    """Run `cases` on one communicator; report per-case mismatch counts.  With a barrier (a
    multiprocessing.Barrier shared by the rank processes), every rank finishes its host-side
    preparation (inputs, oracle, uploads) before any rank enters a call, so the watchdog
    measures the library, not the harness's per-process skew."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        stream = hip_rt.Stream()
        results = []
        for case in cases:
            dtype, op, count, inplace, algo, calls, seed = (case[k] for k in
                                                            ("dtype", "op", "count", "inplace", "algo", "calls", "seed"))
            comm.set_algo(algo)
            if case.get("known") == "ones":  # perf_test.cpp:81-84
                xs = [np.ones(count, dtype=np.float32) for _ in range(n)]
            else:
                xs = make_inputs(n, count, dtype, seed, case.get("special", False))
            exp = O.allreduce(xs, dtype, op, inplace=inplace)[rank]
            code, npd = O.DTYPES[dtype]
            nbytes = xs[rank].nbytes
            off = case.get("offset", 0)  # misaligned base (bytes) -> scalar path
            # where the buffers live: HBM (default), pinned host, or pageable host memory
            # (a list gives each rank its own placement)
            def placement(key, dflt):
                m = case.get(key, dflt)
                return m[rank % len(m)] if isinstance(m, (list, tuple)) else m
            fresh = case.get("fresh", False)  # own hipMalloc / hipFree (allocation churn), not the cache
            if case.get("one_alloc") and not inplace:
                # send and recv as two regions of ONE device allocation (one export serves both)
                whole = hip_rt.buffer("device", 2 * (nbytes + off) + 256, fresh)
                send = hip_rt.View(whole, 0, nbytes + off)
                recv = hip_rt.View(whole, (nbytes + off + 255) // 256 * 256, nbytes + off)
            else:
                send = hip_rt.buffer(placement("mem", "device"), nbytes + off, fresh)
                recv = send if inplace else hip_rt.buffer(placement("recv_mem", placement("mem", "device")),
                                                          nbytes + off, fresh)
            if not inplace:
                recv.fill_byte(0xAB)
            # "window": send / recv registered (mncclCommRegister, collective: every rank runs the
            # same cases in the same order) for this case, deregistered after it.  "window_optional"
            # (the mixed stress): a registration the library refuses -- on every rank alike, it is
            # collective -- is recorded and the case runs unregistered (co-located ranks: the GPU
            # driver can lose a buffer's export handle, profiles/r5_export_reuse.txt)
            wins, refused = [], 0
            if case.get("window") and case.get("window_optional"):
                for b in ([send] if inplace else [send, recv]):
                    wrc, h = comm.register_rc(b.ptr, nbytes + off)
                    if wrc != 0:
                        refused = wrc
                        break
                    wins.append(h)
            elif case.get("window"):
                wins.append(comm.register(send.ptr, nbytes + off))
                if not inplace:
                    wins.append(comm.register(recv.ptr, nbytes + off))
            rc = 0
            grid0 = comm.info()["read_grid_calls"]
            win0 = comm.info()["window_calls"]
            t0 = time.time()
            bad, first, detail = 0, -1, ""
            # "vary": new inputs every call, each call checked (a stale slot or flag from the
            # previous call cannot pass); "skew_ms": each rank sleeps a random time before
            # each call, so ranks enter every call out of step (injected-delay protocol test)
            vary, skew = case.get("vary", False), case.get("skew_ms", 0)
            rng = np.random.default_rng(seed * 97 + rank)
            for c in range(calls):
                if vary and c > 0:
                    xs = make_inputs(n, count, dtype, seed + 1000 * c, case.get("special", False))
                    exp = O.allreduce(xs, dtype, op, inplace=inplace)[rank]
                send.upload(xs[rank], off)
                if barrier is not None:
                    barrier.wait(120)
                if skew:
                    time.sleep(float(rng.uniform(0, skew)) / 1000.0)
                rc = comm.all_reduce(send.ptr + off, recv.ptr + off, count, code, O.OPS[op], stream.handle)
                if rc != 0:
                    break
                if vary:
                    stream.sync()
                    got = recv.download(npd, count, off)
                    b, f = compare(got, exp, dtype, op in ("sum", "prod"))
                    if b and not bad:
                        first, detail = f, f"call {c}: got {got[f]!r} expected {exp[f]!r}"
                    bad += b
            stream.sync()
            dt = time.time() - t0
            if not vary:
                got = recv.download(npd, count, off)
                bad, first = compare(got, exp, dtype, op in ("sum", "prod")) if rc == 0 else (-1, -1)
                detail = (f"got {got[first]!r} expected {exp[first]!r}" if bad and first >= 0 else "")
            elif rc != 0:
                bad, first = -1, -1
            ci = comm.info()
            results.append({"case": case, "rc": rc, "bad": bad, "first": first, "detail": detail, "secs": dt,
                            "async": comm.async_error(), "last_algo": ci["last_algo"],
                            "grid_calls": ci["read_grid_calls"] - grid0,
                            "window_calls": ci["window_calls"] - win0,
                            "peer_mappings": ci["peer_mappings"], "ipc_open_failures": ci["ipc_open_failures"],
                            "read_map_failures": ci["read_map_failures"], "closed_freed": ci["closed_freed"],
                            "live_exports": ci["live_exports"], "register_refused": refused,
                            "retired_imports": ci["retired_imports"]})
            for h in wins:
                comm.deregister(h)
            send.free()
            if not inplace:
                recv.free()
        stream.destroy()
        info = comm.info()
        rc = comm.destroy()
        out_q.put((rank, {"results": results, "destroy": rc, "info": info}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def many_buffers_rank(rank, n, port, env, pairs, out_q):
    """`pairs` distinct send / recv allocations, all alive until the end (a data-parallel caller's
    gradient buckets), one read call on each in turn: every call bit-exact; the process's export
    cap (512) sends the calls beyond it to the ring on every rank, counted in cap_refusals; the
    per-call liveness queries stay bounded (the call's own buffers + a batch of 4, ipcreg.h)."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        comm.set_algo(2)
        st = hip_rt.Stream()
        count = 4099
        bufs = [(hip_rt.DeviceBuffer(count * 4, fresh=True), hip_rt.DeviceBuffer(count * 4, fresh=True))
                for _ in range(pairs)]
        bad, rcs, algos, queries = 0, [], [], []
        for i, (s, r) in enumerate(bufs):
            xs = make_inputs(n, count, "f32", 2000 + i, False)
            s.upload(xs[rank])
            q0 = comm.info()["liveness_queries"]
            rc = comm.all_reduce(s.ptr, r.ptr, count, M.ncclFloat, M.ncclSum, st.handle)
            st.sync()
            ci = comm.info()
            queries.append(ci["liveness_queries"] - q0)
            rcs.append(rc)
            algos.append(ci["last_algo"])
            bad += compare(r.download(np.float32, count), O.allreduce(xs, "f32", "sum")[rank], "f32", True)[0]
        # the same buffers again: all of them are known now (no mapping round), still exact
        for i, (s, r) in enumerate(bufs[:64]):
            xs = make_inputs(n, count, "f32", 5000 + i, False)
            s.upload(xs[rank])
            rcs.append(comm.all_reduce(s.ptr, r.ptr, count, M.ncclFloat, M.ncclSum, st.handle))
            st.sync()
            bad += compare(r.download(np.float32, count), O.allreduce(xs, "f32", "sum")[rank], "f32", True)[0]
        info = comm.info()
        for s, r in bufs:
            s.free()
            r.free()
        st.destroy()
        out_q.put((rank, {"bad": bad, "rcs": rcs, "algos": algos, "queries": queries, "info": info,
                          "destroy": comm.destroy()}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def release_rank(rank, n, port, env, nbytes, out_q, barrier=None):
    """memory a caller frees after its last communicator is destroyed must come back.
    Every rank runs a read call on its own `nbytes` allocation (exported as a dma-buf, imported by
    the peers), destroys the communicator, then the ranks free their allocations one at a time
    and each measures the device's free memory around its own hipFree."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        comm.set_algo(2)
        count = nbytes // 4
        buf = hip_rt.DeviceBuffer(nbytes, fresh=True)
        buf.upload(np.ones(count, np.float32))
        hip_rt.sync()
        rc = comm.all_reduce(buf.ptr, buf.ptr, count, M.ncclFloat, M.ncclSum, 0)
        hip_rt.sync()
        got = buf.download(np.float32, 1024)
        info = comm.info()
        rc_destroy = comm.destroy()
        barrier.wait(120)  # every communicator is gone
        freed = 0
        for r in range(n):
            if r == rank:
                f0, _ = hip_rt.mem_get_info()
                buf.free()
                hip_rt.sync()
                f1, _ = hip_rt.mem_get_info()
                freed = f1 - f0
            barrier.wait(120)
        out_q.put((rank, {"rc": rc, "destroy": rc_destroy, "last_algo": info["last_algo"], "freed": freed,
                          "ok": bool((got == n).all()), "ranks_on_device": info["ranks_on_device"]}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def churn_rank(rank, n, port, env, calls, nbytes, out_q, barrier=None):
    """VERDICT r5 #3 / ADVICE r5: `calls` all-reduces, each on a FRESH in-place allocation of `nbytes`
    that is freed right after its call (no caching allocator: every call brings buffers new to the
    peers).  Co-located ranks retire their imports of each other's freed buffers (csrc/ipcreg.h),
    so the retired budget (MINI_NCCL_RETIRED_MB) or the import count cap must take the later calls
    to the ring.  Integer-valued data (sums exact in any order), every element checked; the
    device's free memory sampled after every call."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        st = hip_rt.Stream()
        count = nbytes // 4
        base = (np.arange(count, dtype=np.int64) % 1021).astype(np.float32)
        hip_rt.sync()
        barrier.wait(120)
        free0, _ = hip_rt.mem_get_info()
        min_free, rcs, algos, bad = free0, [], [], 0
        for i in range(calls):
            buf = hip_rt.DeviceBuffer(nbytes, fresh=True)
            buf.upload(base + np.float32(7 * rank + i % 13))
            rc = comm.all_reduce(buf.ptr, buf.ptr, count, M.ncclFloat, M.ncclSum, st.handle)
            st.sync()
            rcs.append(rc)
            algos.append(comm.info()["last_algo"])
            want = n * base + np.float32(sum(7 * q + i % 13 for q in range(n)))
            got = buf.download(np.float32, count)
            bad += int((got != want).sum())
            buf.free()
            hip_rt.sync()
            min_free = min(min_free, hip_rt.mem_get_info()[0])
        info = comm.info()
        st.destroy()
        out_q.put((rank, {"rcs": rcs, "algos": algos, "bad": bad, "free0": free0, "min_free": min_free,
                          "info": info, "destroy": comm.destroy()}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def two_comms_rank(rank, n, ports, env, rounds, out_q):
    """Two communicators in one process sharing the same send / recv buffers, calls alternating
    between them; every other round on fresh allocations (freed after it).  Each communicator
    brings the buffers as new the first time (the owner sends their dma-bufs again, the peer's
    import is found and the duplicate closed); frees reach both through the process's freed log."""
    try:
        os.environ.update(env)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comms = []
        for p in ports:
            os.environ["MINI_NCCL_PORT"] = str(p)
            comms.append(M.Comm(n, rank, "127.0.0.1"))
        for c in comms:
            c.set_algo(2)
        stream = hip_rt.Stream()
        code, npd = O.DTYPES["f32"]
        bad, rcs, algos = 0, [], []
        for i in range(rounds):
            count = 70001 + 3 * i
            fresh = i % 2 == 1
            send = hip_rt.buffer("device", count * 4, fresh)
            recv = hip_rt.buffer("device", count * 4, fresh)
            for j, c in enumerate(comms + comms):
                xs = make_inputs(n, count, "f32", 700 + 10 * i + j, False)
                exp = O.allreduce(xs, "f32", "sum")[rank]
                send.upload(xs[rank])
                rc = c.all_reduce(send.ptr, recv.ptr, count, code, O.OPS["sum"], stream.handle)
                stream.sync()
                rcs.append(rc)
                got = recv.download(npd, count)
                bad += compare(got, exp, "f32", True)[0]
                algos.append(c.info()["last_algo"])
            send.free()
            recv.free()
        infos = [c.info() for c in comms]
        stream.destroy()
        destroy = [c.destroy() for c in comms]
        out_q.put((rank, {"bad": bad, "rcs": rcs, "algos": algos, "destroy": destroy,
                          "ipc_open_failures": infos[0]["ipc_open_failures"],
                          "read_map_failures": [x["read_map_failures"] for x in infos],
                          "closed_freed": [x["closed_freed"] for x in infos]}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def fullsize_input(rank, count, dtype, seed=1234, piece=1 << 24):
    """Rank r's full-size buffer: seeded uniform[-1, 1) (seed = 1234 + r),
    generated piece by piece (the same stream as one call) so no float64 temporary of the whole
    buffer is needed.  The parent and the rank process build identical bytes independently."""
    import oracle_api as O
    code, npd = O.DTYPES[dtype]
    g = np.random.default_rng(seed + rank)
    out = np.empty(count, dtype=npd)
    f = np.empty(min(piece, count), dtype=np.float32)
    for a in range(0, count, piece):
        b = min(count, a + piece)
        v = f[:b - a]
        g.random(dtype=np.float32, out=v)  # [0, 1)
        v *= 2
        v -= 1
        if dtype == "bf16":  # truncated to bf16 (the top 16 bits: exact, no rounding step)
            out[a:b] = v.view(np.uint32) >> 16
        else:
            out[a:b] = v
    return out


def block_digests(arr, block_bytes=1 << 24):
    """sha1 of every 16 MiB block: a full-size result is compared by digest, and a mismatch is
    located to its block without shipping the buffer between processes."""
    import hashlib
    mv = memoryview(np.ascontiguousarray(arr).view(np.uint8))
    return [hashlib.sha1(mv[i:i + block_bytes]).hexdigest() for i in range(0, len(mv), block_bytes)]


def fullsize_rank(rank, n, port, env, dtype, count, algos, out_q, barrier=None):
    """One full-size all-reduce per schedule in `algos` (BASELINE C3 / C5 sizes) on this rank's
    seeded input, in place and out of place alternately; reports the block digests of recv."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        x = fullsize_input(rank, count, dtype)
        code, npd = O.DTYPES[dtype]
        comm = M.Comm(n, rank, "127.0.0.1")
        stream = hip_rt.Stream()
        send = hip_rt.DeviceBuffer(x.nbytes)
        recv = hip_rt.DeviceBuffer(x.nbytes)
        res = []
        for i, algo in enumerate(algos):
            inplace = i % 2 == 1
            comm.set_algo(algo)
            grid0 = comm.info()["read_grid_calls"]
            send.upload(x)
            dst = send if inplace else recv
            if not inplace:
                recv.fill_byte(0xAB)
            stream.sync()
            if barrier is not None:
                barrier.wait(300)
            t0 = time.time()
            rc = comm.all_reduce(send.ptr, dst.ptr, count, code, M.ncclSum, stream.handle)
            stream.sync()
            secs = time.time() - t0
            got = dst.download(npd, count)
            ci = comm.info()
            res.append({"algo": algo, "inplace": inplace, "rc": rc, "async": comm.async_error(), "secs": secs,
                        "last_algo": ci["last_algo"], "grid_calls": ci["read_grid_calls"] - grid0,
                        "digests": block_digests(got)})
            del got
        send.free()
        recv.free()
        stream.destroy()
        info = comm.info()
        out_q.put((rank, {"results": res, "info": info, "destroy": comm.destroy()}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def graph_rank(rank, n, port, env, replays, out_q):
    """Capture one ncclAllReduce into a HIP graph, replay it `replays` times with fresh input
    each time; the per-pair sequence counters live on the device, so replays stay in step."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        st = hip_rt.Stream()
        count = int(env.get("GRAPH_COUNT", (1 << 18) + 1))
        send, recv = hip_rt.DeviceBuffer(count * 4), hip_rt.DeviceBuffer(count * 4)
        if env.get("GRAPH_WINDOW") == "1":  # the captured call on registered windows (no rendezvous)
            comm.register(send.ptr, count * 4)
            comm.register(recv.ptr, count * 4)
        rcs = []
        g = hip_rt.Graph(st, lambda: rcs.append(comm.all_reduce(send.ptr, recv.ptr, count, M.ncclFloat, M.ncclSum,
                                                                st.handle)))
        captured_algo = comm.info()["last_algo"]  # the schedule baked into the graph
        captured_grid = comm.info()["read_grid_calls"]
        captured_window = comm.info()["window_calls"]
        bad = []
        for k in range(replays):
            xs = O.random_inputs(n, count, "f32", seed=500 + k)
            exp = O.allreduce(xs, "f32", "sum")[rank]
            send.upload(xs[rank])
            g.launch()
            st.sync()
            got = recv.download(np.float32, count)
            bad.append(int((got.view(np.uint32) != exp.view(np.uint32)).sum()))
        # an eager call after the replays still lines up with the peers
        xs = O.random_inputs(n, count, "f32", seed=999)
        send.upload(xs[rank])
        rc = comm.all_reduce(send.ptr, recv.ptr, count, M.ncclFloat, M.ncclSum, st.handle)
        st.sync()
        got = recv.download(np.float32, count)
        exp = O.allreduce(xs, "f32", "sum")[rank]
        g.destroy()
        out_q.put((rank, {"capture_rc": rcs, "bad": bad, "eager_rc": rc, "captured_algo": captured_algo,
                          "captured_grid": captured_grid, "captured_window": captured_window,
                          "eager_bad": int((got.view(np.uint32) != exp.view(np.uint32)).sum())}))
        send.free()
        recv.free()
        st.destroy()
        comm.destroy()
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def streams_rank(rank, n, port, env, calls, out_q):
    """Stream-ordered calls (MINI_NCCL_BLOCKING=0) that alternate between two streams with no
    host sync in between: the communicator orders call k+1 after call k whatever stream
    each is on (NCCL's rule; two persistent kernels of one communicator must never overlap)."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        sts = [hip_rt.Stream(), hip_rt.Stream()]
        count = (1 << 20) + 3
        bufs, exps, rcs = [], [], []
        for c in range(calls):
            xs = O.random_inputs(n, count, "f32", seed=700 + c)
            exps.append(O.allreduce(xs, "f32", "sum")[rank])
            s, r = hip_rt.DeviceBuffer(count * 4), hip_rt.DeviceBuffer(count * 4)
            s.upload(xs[rank])
            bufs.append((s, r))
        hip_rt.sync()
        for c in range(calls):
            s, r = bufs[c]
            rcs.append(comm.all_reduce(s.ptr, r.ptr, count, M.ncclFloat, M.ncclSum, sts[c % 2].handle))
        for st in sts:
            st.sync()
        bad = []
        for c in range(calls):
            got = bufs[c][1].download(np.float32, count)
            bad.append(int((got.view(np.uint32) != exps[c].view(np.uint32)).sum()))
            bufs[c][0].free()
            bufs[c][1].free()
        for st in sts:
            st.destroy()
        out_q.put((rank, {"rcs": rcs, "bad": bad, "async": comm.async_error(), "destroy": comm.destroy()}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def probe_rank(rank, n, port, env, out_q):
    """mncclCommLinkProbe is collective; afterwards an all-reduce must still be correct
    (the probe overwrote scratch slots while no message was in flight)."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        res = {"next": comm.link_probe(False, 8 << 20, 3), "mesh": comm.link_probe(True, 8 << 20, 3)}
        # the comparison forms (push nt / default policy, pull) on the same links
        res["variants"] = [comm.link_probe(allp, 4 << 20, 2, form=f, pull=pl, user=u)
                           for f, pl, u in (("nt", False, False), ("plain", False, False), ("sys", True, False),
                                            ("plain", True, False), ("sys", True, True), ("sys", False, True))
                           for allp in (False, True)]
        count = 100003
        xs = O.random_inputs(n, count, "f32", seed=3)
        send, recv = hip_rt.DeviceBuffer(count * 4), hip_rt.DeviceBuffer(count * 4)
        send.upload(xs[rank])
        res["rc"] = comm.all_reduce(send.ptr, recv.ptr, count, M.ncclFloat, M.ncclSum, 0)
        hip_rt.sync()
        got = recv.download(np.float32, count)
        res["exact"] = bool(np.array_equal(got.view(np.uint32), O.allreduce(xs)[rank].view(np.uint32)))
        send.free()
        recv.free()
        comm.destroy()
        out_q.put((rank, res))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def init_rank(rank, n, port, env, out_q):
    """ncclCommInitRank with per-rank environment (env[rank]); report the result code."""
    try:
        os.environ.update(env.get(rank, {}))
        os.environ["MINI_NCCL_PORT"] = str(port)
        import ctypes
        import hip_rt
        import mini_nccl as M
        use_rank_device(rank)
        h = ctypes.c_void_p()
        rc = M.load().ncclCommInitRank(ctypes.byref(h), n, rank, b"127.0.0.1")
        if rc == 0:
            M.load().ncclCommDestroy(h)
        out_q.put((rank, {"rc": rc}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def mismatch_rank(rank, n, port, env, out_q):
    """Read schedule: ranks pass different counts to one call (a caller bug the reference would
    hang or corrupt on) -> every rank gets ncclInvalidUsage from the per-call rendezvous, and the
    communicator stays usable: a matching call right after is bit-exact.  MISMATCH=algo: the
    counts agree but rank 0 chose auto and the others mncclAlgoRead (mncclCommSetAlgo is per rank:
    auto would launch the grid form, read the persistent kernel) -- the same ncclInvalidUsage."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        st = hip_rt.Stream()
        count = 40000
        xs = O.random_inputs(n, count, "f32", seed=321)
        send, recv = hip_rt.DeviceBuffer(count * 4), hip_rt.DeviceBuffer(count * 4)
        send.upload(xs[rank])
        if os.environ.get("MISMATCH") == "algo":
            comm.set_algo(M.ALGO_AUTO if rank == 0 else M.ALGO_READ)
            rc_bad = comm.all_reduce(send.ptr, recv.ptr, count, M.ncclFloat, M.ncclSum, st.handle)
            comm.set_algo(M.ALGO_READ)
        else:
            rc_bad = comm.all_reduce(send.ptr, recv.ptr, count - rank, M.ncclFloat, M.ncclSum, st.handle)
        rc_ok = comm.all_reduce(send.ptr, recv.ptr, count, M.ncclFloat, M.ncclSum, st.handle)
        st.sync()
        got = recv.download(np.float32, count)
        exp = O.allreduce(xs, "f32", "sum")[rank]
        info = comm.info()
        send.free()
        recv.free()
        st.destroy()
        out_q.put((rank, {"rc_bad": rc_bad, "rc_ok": rc_ok, "bad": int((got.view(np.uint32) != exp.view(np.uint32)).sum()),
                          "last_algo": info["last_algo"], "async": comm.async_error(), "destroy": comm.destroy()}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def info_rank(rank, n, port, env, out_q):
    """Create a communicator with `env`, report mncclCommGetInfo, destroy it."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        info = comm.info()
        out_q.put((rank, {"info": info, "destroy": comm.destroy()}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def huge_rank(rank, n, port, env, count, out_q):
    """64-bit element counts (the reference narrowed count to int, mini_nccl.h:113): bf16
    all-ones in place -> body == n, tail == 1 (size-independent known answer)."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        buf = hip_rt.DeviceBuffer(count * 2)
        chunk = 1 << 26
        ones = np.full(chunk, 0x3F80, np.uint16)  # bf16 1.0
        for off in range(0, count, chunk):
            m = min(chunk, count - off)
            buf.upload(ones[:m], off * 2)
        rc = comm.all_reduce(buf.ptr, buf.ptr, count, M.ncclBfloat16, M.ncclSum, 0)
        hip_rt.sync()
        body = (count // n) * n
        want = {2: 0x4000, 4: 0x4080}[n]
        bad = 0
        for off in range(0, count, chunk):
            m = min(chunk, count - off)
            got = buf.download(np.uint16, m, off * 2)
            idx = np.arange(off, off + m)
            bad += int((got != np.where(idx < body, want, 0x3F80)).sum())
        buf.free()
        comm.destroy()
        out_q.put((rank, {"rc": rc, "bad": bad}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def far_offsets_rank(rank, n, port, env, count, algos, out_q):
    """Chunks beyond 4 GiB (byte offsets past 2^32 in every kernel's addressing, 288 GB of HBM per
    GPU): int32 x_r[i] = uint32(i) * (r + 1), wrapping, so every element's value names its position
    up to 2^32 elements -- a 32-bit wrap of a byte offset reads another position's value.  Filled and
    checked on the device (testkern.hip: 8 GiB per rank is too much for a host-side check).  Out of
    place, one call per schedule, the whole recv checked each time: body = the sum over ranks
    (n(n+1)/2 * i, wrapping), tail = this rank's own input."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import ctypes
        import hip_rt
        import mini_nccl as M
        use_rank_device(rank)
        K = testkern()
        comm = M.Comm(n, rank, "127.0.0.1")
        send = hip_rt.DeviceBuffer(count * 4)
        recv = hip_rt.DeviceBuffer(count * 4)
        res_buf = hip_rt.DeviceBuffer(256)
        vp = ctypes.c_void_p
        hip_rt.check(K.mnccl_test_iota(vp(send.ptr), count, rank + 1, None), "iota")
        hip_rt.sync()
        body = (count // n) * n

        def check(buf, mult_body, mult_tail):
            hip_rt.check(K.mnccl_test_check_iota(vp(buf.ptr), count, body, mult_body, mult_tail, vp(res_buf.ptr),
                                                 None), "check")
            hip_rt.sync()
            bad, first = (int(v) for v in res_buf.download(np.uint64, 2))
            return bad, (first if bad else -1)

        # the checker itself: my input is not the sum, so it must flag the body from element 1 on
        checker = check(send, n * (n + 1) // 2, rank + 1)
        res = []
        for algo in algos:
            recv.fill_byte(0xA5)
            comm.set_algo(algo)
            rc = comm.all_reduce(send.ptr, recv.ptr, count, M.ncclInt32, M.ncclSum, 0)
            hip_rt.sync()
            bad, first = check(recv, n * (n + 1) // 2, rank + 1)
            ci = comm.info()
            res.append({"algo": algo, "rc": rc, "bad": bad, "first": first,
                        "last_algo": ci["last_algo"], "grid_calls": ci["read_grid_calls"]})
        send.free()
        recv.free()
        res_buf.free()
        out_q.put((rank, {"results": res, "checker": checker, "body": body, "destroy": comm.destroy()}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def threaded_ranks_proc(n, port, env, cases, out_q):
    """n ranks as threads of ONE process, all on this GPU: the library's same-process peer paths
    (comm.cpp exchange_and_map: raw pointers for scratch / mailbox; peerbuf.cpp: the peers' user
    buffers in this address space, no dma-buf) instead of IPC.  Each rank thread has its own
    non-blocking stream; every allocation, upload, memset and free happens between barriers while
    no all-reduce kernel runs (a device-wide synchronisation would otherwise wait for another
    thread's kernel, which waits for this thread's).  Each case is checked bit-exact against the
    oracle.  Reports {rank: results}."""
    import threading
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        bar = threading.Barrier(n)
        out = {}
        # inputs and the oracle's outputs once per case, shared by the rank threads
        prepared = []
        for case in cases:
            xs = make_inputs(n, case["count"], case["dtype"], case["seed"], False)
            prepared.append((xs, O.allreduce(xs, case["dtype"], "sum", inplace=case["inplace"])))

        def rank_main(r):
            try:
                hip_rt.set_device(0)
                comm = M.Comm(n, r, "127.0.0.1")
                st = hip_rt.Stream()
                res = []
                for case, (xs, outs) in zip(cases, prepared):
                    dtype, count, algo, inplace = case["dtype"], case["count"], case["algo"], case["inplace"]
                    exp = outs[r]
                    code, npd = O.DTYPES[dtype]
                    send = hip_rt.DeviceBuffer(xs[r].nbytes)
                    recv = send if inplace else hip_rt.DeviceBuffer(xs[r].nbytes)
                    send.upload(xs[r])
                    if not inplace:
                        recv.fill_byte(0xAB)
                    comm.set_algo(algo)
                    bar.wait(120)  # every thread prepared: no memset / copy / free from here on
                    rc = comm.all_reduce(send.ptr, recv.ptr, count, code, M.ncclSum, st.handle)
                    st.sync()
                    bar.wait(120)  # every thread's kernel done
                    bad, first = compare(recv.download(npd, count), exp, dtype, True)
                    res.append({"case": case, "rc": rc, "bad": bad, "first": first,
                                "last_algo": comm.info()["last_algo"]})
                    if recv is not send:
                        recv.free()
                    send.free()
                    bar.wait(120)  # frees done before anyone's next call
                info = comm.info()
                st.destroy()
                out[r] = {"results": res, "ranks_on_device": info["ranks_on_device"],
                          "ipc_open_failures": info["ipc_open_failures"], "destroy": comm.destroy()}
            except Exception:
                out[r] = {"error": traceback.format_exc()}
                bar.abort()

        ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        out_q.put((0, {"ranks": out}))
    except Exception:
        out_q.put((0, {"error": traceback.format_exc()}))


def destroy_inflight_rank(rank, n, port, env, out_q):
    """Stream-ordered calls still running when ncclCommDestroy is called: destroy waits for
    them (their kernels write into the peers' memory, which the peers free right after), and
    the results are complete once it returns."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        stream = hip_rt.Stream()
        count = (64 << 20) // 4
        buf = hip_rt.DeviceBuffer(count * 4)
        buf.upload(np.ones(count, np.float32))
        hip_rt.sync()
        rcs = [comm.all_reduce(buf.ptr, buf.ptr, count, M.ncclFloat, M.ncclSum, stream.handle) for _ in range(3)]
        rc_destroy = comm.destroy()  # no synchronisation before it
        got = buf.download(np.float32, count)
        stream.destroy()
        buf.free()
        body = (count // n) * n  # the count % n tail keeps this rank's input (mini_nccl.cu:69)
        want = np.where(np.arange(count) < body, float(n) ** 3, 1.0).astype(np.float32)
        out_q.put((rank, {"rcs": rcs, "destroy": rc_destroy, "bad": int((got != want).sum())}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def stall_rank(rank, n, port, env, call_allreduce, out_q):
    """Timeout test: rank 0 calls all-reduce, the other ranks never do."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        buf = hip_rt.DeviceBuffer(1 << 20)
        res = {}
        if call_allreduce:
            t0 = time.time()
            res["rc"] = comm.all_reduce(buf.ptr, buf.ptr, (1 << 20) // 4, M.ncclFloat, M.ncclSum, 0)
            res["secs"] = time.time() - t0
            res["rc2"] = comm.all_reduce(buf.ptr, buf.ptr, (1 << 20) // 4, M.ncclFloat, M.ncclSum, 0)
            res["async"] = comm.async_error()
            if env.get("LATE_CALL") == "1":  # keep the buffer and the memory alive for the late rank
                time.sleep(max(0.0, float(env.get("STALL_SECS", "4")) + 4.0 - (time.time() - t0)))
        else:
            time.sleep(float(env.get("STALL_SECS", "4")))
            if env.get("LATE_CALL") == "1":
                # arrives after rank 0 gave up: rank 0 raised this rank's ABORT word, so the
                # kernel fails at once (ncclRemoteError) instead of waiting out its watchdog
                t0 = time.time()
                res["rc"] = comm.all_reduce(buf.ptr, buf.ptr, (1 << 20) // 4, M.ncclFloat, M.ncclSum, 0)
                res["secs"] = time.time() - t0
        out_q.put((rank, res))
        buf.free()
        comm.destroy()
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def delayed_start_rank(rank, n, port, env, delay_s, out_q):
    """Work queued ahead of the all-reduce on its stream (a stream wait on a host word that a
    timer thread raises after delay_s) must not count against the watchdog: the host deadline
    starts when the kernel does.  Blocking call, MINI_NCCL_TIMEOUT_MS well below delay_s."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import threading
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        st = hip_rt.Stream()
        count = (1 << 20) + 3
        xs = O.random_inputs(n, count, "f32", seed=77)
        send, recv = hip_rt.DeviceBuffer(count * 4), hip_rt.DeviceBuffer(count * 4)
        send.upload(xs[rank])
        gate = hip_rt.HostBuffer(64)
        gate.fill_byte(0)
        st.wait_value32(gate.ptr, 1)
        t = threading.Timer(delay_s, lambda: gate.upload(np.array([1], np.uint32)))
        t.start()
        t0 = time.time()
        rc = comm.all_reduce(send.ptr, recv.ptr, count, M.ncclFloat, M.ncclSum, st.handle)
        secs = time.time() - t0
        t.join()
        st.sync()
        got = recv.download(np.float32, count)
        bad = int((got.view(np.uint32) != O.allreduce(xs)[rank].view(np.uint32)).sum())
        res = {"rc": rc, "secs": secs, "bad": bad, "async": comm.async_error()}
        send.free()
        recv.free()
        gate.free()
        st.destroy()
        res["destroy"] = comm.destroy()
        out_q.put((rank, res))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def local_reduce_case(dtype, op, count, offset):
    """mncclLocalReduce on seeded inputs vs the oracle's element-wise op (in the calling
    process); returns (mismatches, first index, got, expected) for the test's message."""
    import hip_rt
    import mini_nccl as M
    import oracle_api as O
    hip_rt.set_device(0)
    code, npd = O.DTYPES[dtype]
    a, b = make_inputs(2, count, dtype, seed=count + 7, special=op in ("max", "min"))
    exp = O.reduce(a, b, dtype, op)
    esz = np.dtype(npd).itemsize
    off = offset * esz if offset else 0
    da, db, dc = (hip_rt.DeviceBuffer(count * esz + off) for _ in range(3))
    try:
        da.upload(a, off)
        db.upload(b, off)
        rc = M.local_reduce(dc.ptr + off, da.ptr + off, db.ptr + off, count, code, O.OPS[op], 0)
        if rc != M.ncclSuccess:
            return (-1, -1, f"ncclResult {rc}", "")
        hip_rt.sync()
        got = dc.download(npd, count, off)
        bad, first = compare(got, exp, dtype, op in ("sum", "prod"))
        return (bad, first, repr(got[first]) if bad else "", repr(exp[first]) if bad else "")
    finally:
        for x in (da, db, dc):
            x.free()


def local_reduce_in_place_large():
    """256 MiB fp32 a <- a + b in place, bit-exact vs the oracle; returns mismatches."""
    import hip_rt
    import mini_nccl as M
    import oracle_api as O
    hip_rt.set_device(0)
    count = 64 << 20
    a, b = make_inputs(2, count, "f32", seed=5, special=False)
    exp = O.reduce(a, b, "f32", "sum")
    da, db = hip_rt.DeviceBuffer(a.nbytes), hip_rt.DeviceBuffer(b.nbytes)
    try:
        da.upload(a)
        db.upload(b)
        if M.local_reduce(da.ptr, da.ptr, db.ptr, count, M.ncclFloat, M.ncclSum, 0) != 0:
            return -1
        hip_rt.sync()
        return int((da.download(np.float32, count).view(np.uint32) != exp.view(np.uint32)).sum())
    finally:
        da.free()
        db.free()


def testkern():
    """tests/lib/libmnccl_testkern.so: plain-load consumer kernels and the position-coded fill /
    check (test infrastructure)."""
    import ctypes
    L = ctypes.CDLL(os.path.join(HERE, "lib", "libmnccl_testkern.so"))
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    L.mnccl_test_touch.argtypes = [vp, u64, vp, vp]
    L.mnccl_test_copy.argtypes = [vp, vp, u64, vp]
    L.mnccl_test_iota.argtypes = [vp, u64, ctypes.c_uint32, vp]
    L.mnccl_test_check_iota.argtypes = [vp, u64, u64, ctypes.c_uint32, ctypes.c_uint32, vp, vp]
    return L


def cached_consumer_rank(rank, n, port, env, count, calls, out_q, barrier=None):
    """VERDICT r4 #1, the push form's cross-device visibility in the shape the node gives it: recv
    is first read by an ordinary kernel (plain loads: its lines sit in this GPU's L2), then the
    read schedule's call -- the peers push their result chunks into this recv (from other GPUs over
    xGMI when the placement spreads the ranks, from other XCDs' L2s when they share a GPU) -- and an
    ordinary consumer kernel copies recv with plain loads right behind the call on the same stream
    (MINI_NCCL_BLOCKING=0: no host wait in between).  Seeded uniform[-1, 1) inputs, new every call
    (order-sensitive: a wrong association, a stale line or a torn push each change bits), compared
    bit for bit with the oracle's ring fold."""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import ctypes
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        K = testkern()
        comm = M.Comm(n, rank, "127.0.0.1")
        comm.set_algo(int(env.get("TEST_ALGO", "2")))
        st = hip_rt.Stream()
        nb = count * 4
        send, recv, seen = hip_rt.DeviceBuffer(nb), hip_rt.DeviceBuffer(nb), hip_rt.DeviceBuffer(nb)
        word = hip_rt.DeviceBuffer(256)
        bad, rcs, algos = [], [], []
        for c in range(calls):
            inplace = c % 3 == 2
            dst = send if inplace else recv
            xs = O.random_inputs(n, count, "f32", seed=4000 + 17 * c)
            exp = O.allreduce(xs, "f32", "sum", inplace=inplace)[rank]
            send.upload(xs[rank])
            hip_rt.sync()
            if barrier is not None:
                barrier.wait(120)
            # the previous call's result (or the fresh input, in place) into this GPU's L2 ...
            hip_rt.check(K.mnccl_test_touch(ctypes.c_void_p(dst.ptr), nb, ctypes.c_void_p(word.ptr),
                                            ctypes.c_void_p(st.handle)), "touch")
            rc = comm.all_reduce(send.ptr, dst.ptr, count, M.ncclFloat, M.ncclSum, st.handle)
            # ... and read by an ordinary kernel right after the call
            hip_rt.check(K.mnccl_test_copy(ctypes.c_void_p(seen.ptr), ctypes.c_void_p(dst.ptr), nb,
                                           ctypes.c_void_p(st.handle)), "copy")
            st.sync()
            rcs.append(rc)
            algos.append(comm.info()["last_algo"])
            got = seen.download(np.float32, count)
            bad.append(compare(got, exp, "f32", True)[0])
        info = comm.info()
        for b in (send, recv, seen, word):
            b.free()
        st.destroy()
        out_q.put((rank, {"rcs": rcs, "bad": bad, "algos": algos, "info": info, "async": comm.async_error(),
                          "destroy": comm.destroy()}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def window_rank(rank, n, port, env, scenario, out_q, barrier=None):
    """Registered windows (mncclCommRegister): calls whose send / recv lie in the windows at the same
    offsets on every rank run the read schedule with no host rendezvous.
      parity   -- calls on sub-ranges of two windows (and in place in one), several sizes / dtypes /
                  ops, varying data, interleaved with negotiated and ring calls: bit-exact, and
                  window_calls counts exactly the window calls
      async    -- MINI_NCCL_BLOCKING=0, rank 1 sleeps 50 ms before each call: rank 0's call returns
                  without waiting for it (host time reported), results bit-exact
      mismatch -- rank 0 passes another offset: every rank's call fails with ncclInvalidUsage
      mismatch_algo -- same windows and offsets, but rank 0 chose auto and the others mncclAlgoRead
                  (different kernel forms for a large call): the same ncclInvalidUsage
      unregistered -- rank 0 passes window buffers, the others buffers outside any window: every
                  rank fails fast (no watchdog wait)"""
    try:
        os.environ.update(env)
        os.environ["MINI_NCCL_PORT"] = str(port)
        import hip_rt
        import mini_nccl as M
        import oracle_api as O
        use_rank_device(rank)
        comm = M.Comm(n, rank, "127.0.0.1")
        st = hip_rt.Stream()
        wbytes = 16 << 20
        sbuf, rbuf = hip_rt.DeviceBuffer(wbytes, fresh=True), hip_rt.DeviceBuffer(wbytes, fresh=True)
        hs = comm.register(sbuf.ptr, wbytes)
        hr = comm.register(rbuf.ptr, wbytes)
        res = {"windows": comm.info()["windows"]}
        if scenario == "parity":
            # (dtype, op, count, send offset, recv offset or None = in place in the send window, algo)
            plan = [("f32", "sum", (1 << 20) + 5, 0, 0, -1), ("bf16", "sum", 300007, 4096, 8192, -1),
                    ("f32", "max", 77777, 1 << 20, None, -1), ("f64", "prod", 4099, 64, 128, 2),
                    ("f32", "sum", 1000, 256, 512, -1), ("i32", "min", n * 1024, 1 << 22, 1 << 22, 2),
                    ("f16", "sum", 9 * 4096 + 3, 12, 36, -1), ("f32", "sum", (2 << 20) + 1, 0, None, 4)]
            bad, rcs, kinds, wc = [], [], [], []
            for i, (dt, op, count, so, ro, algo) in enumerate(plan * 2):
                comm.set_algo(algo)
                code, npd = O.DTYPES[dt]
                inplace = ro is None
                xs = make_inputs(n, count, dt, 3000 + i, op in ("max", "min"))
                exp = O.allreduce(xs, dt, op, inplace=inplace)[rank]
                sp, rp = sbuf.ptr + so, sbuf.ptr + so if inplace else rbuf.ptr + ro
                sbuf.upload(xs[rank], so)
                hip_rt.sync()
                barrier.wait(120)
                w0 = comm.info()["window_calls"]
                rcs.append(comm.all_reduce(sp, rp, count, code, O.OPS[op], st.handle))
                st.sync()
                got = (sbuf if inplace else rbuf).download(npd, count, so if inplace else ro)
                bad.append(compare(got, exp, dt, op in ("sum", "prod"))[0])
                ci = comm.info()
                kinds.append(ci["last_algo"])
                wc.append(ci["window_calls"] - w0)
                if i % 3 == 2:  # a negotiated call (buffers outside the windows) and a ring call between
                    other = hip_rt.DeviceBuffer(4 * 5003)
                    ys = make_inputs(n, 5003, "f32", 3500 + i, False)
                    other.upload(ys[rank])
                    hip_rt.sync()
                    barrier.wait(120)
                    comm.set_algo(-1 if i % 2 else 0)
                    rcs.append(comm.all_reduce(other.ptr, other.ptr, 5003, M.ncclFloat, M.ncclSum, st.handle))
                    st.sync()
                    bad.append(compare(other.download(np.float32, 5003), O.allreduce(ys, inplace=True)[rank], "f32",
                                       True)[0])
                    other.free()
            res.update(bad=bad, rcs=rcs, kinds=kinds, wc=wc)
        elif scenario == "async":
            count = (1 << 20) + 3
            times, bad = [], []
            for c in range(4):
                xs = make_inputs(n, count, "f32", 3700 + c, False)
                sbuf.upload(xs[rank])
                hip_rt.sync()
                barrier.wait(120)
                if rank == 1:
                    time.sleep(0.05)
                t0 = time.perf_counter()
                rc = comm.all_reduce(sbuf.ptr, rbuf.ptr, count, M.ncclFloat, M.ncclSum, st.handle)
                times.append(time.perf_counter() - t0)
                st.sync()
                bad.append(-1 if rc else compare(rbuf.download(np.float32, count), O.allreduce(xs)[rank], "f32", True)[0])
            res.update(call_s=times, bad=bad, window_calls=comm.info()["window_calls"])
        elif scenario in ("mismatch", "mismatch_algo", "unregistered"):
            count = 100003
            other = hip_rt.DeviceBuffer(count * 4)
            barrier.wait(120)
            t0 = time.time()
            if scenario == "mismatch":
                off = 4096 if rank == 0 else 0
                rc = comm.all_reduce(sbuf.ptr + off, rbuf.ptr + off, count, M.ncclFloat, M.ncclSum, st.handle)
            elif scenario == "mismatch_algo":
                comm.set_algo(M.ALGO_AUTO if rank == 0 else M.ALGO_READ)
                rc = comm.all_reduce(sbuf.ptr, rbuf.ptr, n << 20, M.ncclFloat, M.ncclSum, st.handle)  # 4 MiB chunks: auto would take the grid form
            else:
                p = sbuf.ptr if rank == 0 else other.ptr
                rc = comm.all_reduce(p, p, count, M.ncclFloat, M.ncclSum, st.handle)
            res.update(rc=rc, secs=time.time() - t0, async_=comm.async_error(),
                       rc2=comm.all_reduce(sbuf.ptr, rbuf.ptr, count, M.ncclFloat, M.ncclSum, st.handle))
            other.free()
        res["info"] = comm.info()
        if scenario in ("parity", "async"):
            comm.deregister(hs)
            comm.deregister(hr)
            res["windows_after"] = comm.info()["windows"]
        st.destroy()
        res["destroy"] = comm.destroy()
        sbuf.free()
        rbuf.free()
        out_q.put((rank, res))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


def device_count_probe(out_q):
    import hip_rt
    out_q.put((0, {"count": hip_rt.device_count()}))


def _serve(conn):
    """Worker loop: (function name, args) in, ("ok", result) / ("error", traceback) out."""
    while True:
        msg = conn.recv()
        if msg is None:
            break
        name, args = msg
        try:
            conn.send(("ok", globals()[name](*args)))
        except Exception:
            conn.send(("error", traceback.format_exc()))
    conn.close()


class Worker:
    """A long-lived GPU process for single-process GPU tests.  The pytest process itself never
    touches the GPU: the GPU's scheduler maps at most 8 processes at once, and a 9th process
    holding queues (the test runner) makes 8 co-located rank processes time-slice, which stalls
    the persistent all-reduce kernels.  close() ends the process and frees its queues."""

    def __init__(self):
        import multiprocessing as mp
        ctx = mp.get_context("forkserver")
        self.conn, child = ctx.Pipe()
        self.proc = ctx.Process(target=_serve, args=(child,))
        self.proc.start()
        child.close()

    def call(self, name, *args, timeout=300):
        self.conn.send((name, args))
        if not self.conn.poll(timeout):
            raise TimeoutError(f"{name}{args} did not finish in {timeout} s")
        status, val = self.conn.recv()
        if status != "ok":
            raise RuntimeError(val)
        return val

    def close(self):
        try:
            self.conn.send(None)
        except Exception:
            pass
        self.proc.join(30)
        if self.proc.is_alive():
            self.proc.kill()
            self.proc.join(5)


def run_ranks(target, n, args_for_rank, timeout, barrier=False):
    """Spawn n rank processes, collect one result each; kill stragglers at the deadline.
    barrier=True passes a shared multiprocessing.Barrier(n) as the target's `barrier` kwarg."""
    import multiprocessing as mp
    # forkserver: children fork from a server started before this process touched the GPU
    # (conftest starts it), so no child is forked from a GPU-initialised process and
    # nothing exec()s after HIP init
    ctx = mp.get_context("forkserver")
    q = ctx.Queue()
    kw = {"barrier": ctx.Barrier(n)} if barrier else {}
    procs = [ctx.Process(target=target, args=args_for_rank(r) + (q,), kwargs=kw) for r in range(n)]
    for p in procs:
        p.start()
    out = {}
    deadline = time.time() + timeout
    try:
        while len(out) < n and time.time() < deadline:
            try:
                r, res = q.get(timeout=max(0.1, min(5.0, deadline - time.time())))
                out[r] = res
            except Exception:
                if all(not p.is_alive() for p in procs) and q.empty():
                    break
    finally:
        for p in procs:
            p.join(timeout=max(1.0, deadline - time.time()) if len(out) == n else 1.0)
            if p.is_alive():
                p.kill()
                p.join(5)
    return out


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port
