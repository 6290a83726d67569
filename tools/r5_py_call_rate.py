#!/usr/bin/env python3
"""Why does bench.py's `sizes` / `small_calls` show 50-140 us per small call at 2 co-located ranks
when perf_test's stream-ordered calls take 12-20 us (profiles/r5_async_ab.txt)?  N rank processes
on one GPU, stream-ordered calls (MINI_NCCL_BLOCKING=0), ITERS calls per size timed around a
stream synchronize, the same library, in three hosts:
  hiprt        ctypes HIP buffers and a non-blocking stream, no torch (the GPU tests' plumbing)
  torch        torch tensors, a torch.cuda.Stream (bench.py's plumbing)
  torch-dist   the same after torch.distributed (gloo) init, as bench.py runs
  benchlike    bench.py's size_curve: slices of 1 GiB tensors, 5 warm-up calls, dist.barrier, 20
               timed calls closed by torch.cuda.synchronize() -- and the same with 200 calls

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/r5_py_call_rate.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mini-nccl_amd")]
SIZES = [4 << 10, 64 << 10, 1 << 20, 16 << 20]


def main():
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mode = os.environ.get("MODE", "hiprt")
    iters = int(os.environ.get("ITERS", "200"))
    os.environ["MINI_NCCL_BLOCKING"] = "0"
    os.environ["MINI_NCCL_PORT"] = str(int(os.environ["MASTER_PORT"]) + 7)
    import mini_nccl as M
    if mode == "hiprt":
        import hip_rt
        hip_rt.lib().hipSetDevice(0)
        st = hip_rt.Stream()
        sh = st.handle
        bufs = {s: (hip_rt.DeviceBuffer(s), hip_rt.DeviceBuffer(s)) for s in SIZES}
        ptrs = {s: (b[0].ptr, b[1].ptr) for s, b in bufs.items()}
        sync = st.sync
    elif mode == "benchlike":
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=n)
        st = torch.cuda.Stream()
        send = torch.ones(1 << 28, device="cuda")
        recv = torch.empty(1 << 28, device="cuda")
        comm = M.Comm(n, rank, os.environ.get("MASTER_ADDR", "127.0.0.1"))
        # what bench.py runs before its size curve, one piece at a time (PRE=...): a 1 GiB call in
        # the grid form, the link probes (every variant bench.py measures), the ring on 1 GiB
        for pre in os.environ.get("PRE", "").split(","):
            if pre == "grid":
                comm.set_algo(M.ALGO_READ_GRID)
                comm.all_reduce(send.data_ptr(), recv.data_ptr(), 1 << 28, M.ncclFloat, M.ncclSum, st.cuda_stream)
                comm.set_algo(M.ALGO_AUTO)
            elif pre == "ring":
                comm.set_algo(M.ALGO_RING)
                comm.all_reduce(send.data_ptr(), recv.data_ptr(), 1 << 28, M.ncclFloat, M.ncclSum, st.cuda_stream)
                comm.set_algo(M.ALGO_AUTO)
            elif pre == "probe":
                for allp in (False, True):
                    for form in ("sys", "nt", "plain"):
                        comm.link_probe(allp, 0, 10, form=form)
                    comm.link_probe(allp, 0, 10, pull=True)
                    comm.link_probe(allp, 0, 10, pull=True, user=True)
            elif pre in ("bench3", "bench3v", "bench3o"):
                # bench.py's three schedules on the 1 GiB buffers: 5 + 20 calls each, then (bench3v)
                # its integer verify calls and (bench3o) its order-sensitive call too
                sys.path.insert(0, ROOT)
                import bench as B
                for algo in ("ring", "read", "read_grid"):
                    comm.set_algo({"ring": M.ALGO_RING, "read": M.ALGO_READ, "read_grid": M.ALGO_READ_GRID}[algo])
                    for _ in range(25):
                        comm.all_reduce(send.data_ptr(), recv.data_ptr(), 1 << 28, M.ncclFloat, M.ncclSum, st.cuda_stream)
                    torch.cuda.synchronize()
                    if pre in ("bench3v", "bench3o"):
                        B.verify_calls(M, torch, comm, torch.device("cuda", 0), n, rank, send, recv, 1 << 28,
                                       torch.float32, M.ncclFloat, st, barrier=dist.barrier)
                    if pre == "bench3o":
                        B.verify_order(M, torch, comm, torch.device("cuda", 0), n, rank, send, recv, 1 << 28,
                                       torch.float32, M.ncclFloat, st, dist.barrier)
                    send.fill_(1.0)
                comm.set_algo(M.ALGO_AUTO)
            elif pre.startswith("benchprobe"):
                # bench.py's probe sequence exactly; benchprobe:<i> stops after the i-th variant
                stop = int(pre.split(":")[1]) if ":" in pre else 99
                comm.link_probe(False, 0, 10)
                comm.link_probe(True, 0, 10)
                for i, (form, pull, user) in enumerate((("nt", False, False), ("plain", False, False),
                                                        ("sys", True, False), ("plain", True, False),
                                                        ("sys", True, True), ("sys", False, True))):
                    if i >= stop:
                        break
                    for allp in (False, True):
                        comm.link_probe(allp, 0, 10, form=form, pull=pull, user=user)
            elif pre == "pushuser":
                comm.link_probe(False, 0, 10, form="sys", pull=False, user=True)
                comm.link_probe(True, 0, 10, form="sys", pull=False, user=True)
            elif pre == "pulluser":
                comm.link_probe(False, 0, 10, form="sys", pull=True, user=True)
                comm.link_probe(True, 0, 10, form="sys", pull=True, user=True)
            elif pre == "standalone":
                m = (n - 1) * ((1 << 28) // n)
                for _ in range(25):
                    M.local_reduce(recv.data_ptr(), recv.data_ptr(), send.data_ptr(), m, M.ncclFloat, M.ncclSum,
                                   st.cuda_stream)
            torch.cuda.synchronize()
        if rank == 0:
            print(f"mode=benchlike PRE={os.environ.get('PRE', '')}", flush=True)
        for mib in (1, 16, 64, 1, 16):
            k = (mib << 20) // 4
            s_, r_ = send[:k], recv[:k]
            for reps in (20, 200):
                for _ in range(5):
                    comm.all_reduce(s_.data_ptr(), r_.data_ptr(), k, M.ncclFloat, M.ncclSum, st.cuda_stream)
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(reps):
                    comm.all_reduce(s_.data_ptr(), r_.data_ptr(), k, M.ncclFloat, M.ncclSum, st.cuda_stream)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                if rank == 0:
                    print(f"mode=benchlike n={n} {mib:>4d} MiB reps {reps:>3d}: {(t2 - t0) / reps * 1e6:8.2f} us/call "
                          f"(host loop {(t1 - t0) / reps * 1e6:6.2f}, final sync {(t2 - t1) * 1e6:7.1f} us)", flush=True)
        assert comm.async_error() == 0
        comm.destroy()
        return
    else:
        import torch
        torch.cuda.set_device(0)
        if mode == "torch-dist":
            import torch.distributed as dist
            dist.init_process_group("gloo", rank=rank, world_size=n)
        st = torch.cuda.Stream()
        sh = st.cuda_stream
        tens = {s: (torch.ones(s // 4, device="cuda"), torch.empty(s // 4, device="cuda")) for s in SIZES}
        ptrs = {s: (t[0].data_ptr(), t[1].data_ptr()) for s, t in tens.items()}
        sync = st.synchronize
    comm = M.Comm(n, rank, os.environ.get("MASTER_ADDR", "127.0.0.1"))
    for s in SIZES:
        snd, rcv = ptrs[s]
        k = s // 4
        for _ in range(10):
            assert comm.all_reduce(snd, rcv, k, M.ncclFloat, M.ncclSum, sh) == 0
        sync()
        t0 = time.perf_counter()
        for _ in range(iters):
            comm.all_reduce(snd, rcv, k, M.ncclFloat, M.ncclSum, sh)
        t1 = time.perf_counter()
        sync()
        t2 = time.perf_counter()
        if rank == 0:
            print(f"mode={mode:10s} n={n} {s:>9d} B  {(t2 - t0) / iters * 1e6:8.2f} us/call "
                  f"(host loop {(t1 - t0) / iters * 1e6:6.2f} us/call)", flush=True)
    assert comm.async_error() == 0
    comm.destroy()


if __name__ == "__main__":
    main()
