"""Multi-process paths on the CPU (world_size 2 and 4, gloo): the bench harness's barrier /
max-over-ranks, the TCP bootstrap across processes, and the reference's C1 configuration
(2-rank 127.0.0.1 TCP ring with AVX2 adds, oracle/ring_oracle.c) checked bit-exactly against
the oracle -- the N > 1 host-side plumbing without a GPU."""
import os
import sys
import time
import traceback

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _rank_main(rank, world, master_port, ring_port, boot_port, out_q):
    try:
        sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "mini-nccl_amd")]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master_port))
        import ctypes

        import torch.distributed as dist

        import bench
        import oracle_api as O
        import sim_api as S
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = {}
        # bench.py's harness: barrier, then max over ranks of a per-rank time
        dist.barrier()
        res["max"] = bench.reduce_max(dist, 10.0 + rank)
        # bootstrap star across processes (the communicator's init path, no GPU)
        res["boot"] = S.load().mnccl_bootstrap_selftest(rank, world, b"127.0.0.1", boot_port, 20000)
        # C1: the CPU ring over TCP, one process per rank, random fp32 -> bit-exact vs oracle
        count = (4 << 20) // 4 + 3
        xs = O.random_inputs(world, count, "f32", seed=42)
        exp = O.allreduce(xs, "f32", "sum", slice_bytes=131072)[rank]
        buf = xs[rank].copy()
        sec = ctypes.c_double()
        rc = O.load().oracle_cpu_ring_tcp(rank, world, b"127.0.0.1", ring_port, buf.ctypes.data, count, 131072, 1,
                                          ctypes.byref(sec))
        res["ring_rc"] = rc
        res["ring_exact"] = bool(np.array_equal(buf.view(np.uint32), exp.view(np.uint32)))
        dist.barrier()
        dist.destroy_process_group()
        out_q.put((rank, res))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_harness_bootstrap_and_host_ring(oracle_lib, sim_lib, world):
    import gpu_workers as GW
    ports = [GW.free_port() for _ in range(3)]
    out = GW.run_ranks(_rank_main, world, lambda r: (r, world, *ports), 120)
    assert sorted(out) == list(range(world)), out
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
        assert out[r]["max"] == 10.0 + world - 1
        assert out[r]["boot"] == 0
        assert out[r]["ring_rc"] == 0 and out[r]["ring_exact"], out[r]


def _board_rank(rank, world, port, scenario, calls, out_q):
    try:
        sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "mini-nccl_amd")]
        import sim_api as S
        t0 = time.time()
        rc, dec = S.board_selftest(rank, world, port, scenario, calls, timeout_s=2.0)
        out_q.put((rank, {"rc": rc, "dec": dec, "secs": time.time() - t0}))
    except Exception:
        out_q.put((rank, {"error": traceback.format_exc()}))


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("scenario", [0, 1, 2, 3], ids=["agree", "count-mismatch", "rank-missing", "jitter"])
def test_read_schedule_rendezvous_across_processes(sim_lib, world, scenario):
    # csrc/peerbuf.cpp, one process per rank, no GPU: every call's records on the shared-memory
    # board; host buffers everywhere -> the scratch fallback on every rank (PeerBuffers::kFallback
    # = 0); a count that differs on one call -> kMismatch (-1) on every rank for that call only;
    # a rank that never calls -> the others fail that call after the timeout (-9) instead of
    # hanging; random per-rank delays over 64 calls (the 16-record board wraps 4 times) -> same
    import gpu_workers as GW
    calls = 64 if scenario == 3 else 24
    port = GW.free_port()
    out = GW.run_ranks(_board_rank, world, lambda r: (r, world, port, scenario, calls), 120)
    assert sorted(out) == list(range(world)), out
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
        assert out[r]["rc"] == 0, out[r]
        dec = out[r]["dec"]
        if scenario == 2:
            if r == world - 1:
                assert dec == [99] * calls  # never called
            else:
                assert dec[0] == -9 and out[r]["secs"] < 30, out[r]
        else:
            exp = [0] * calls
            if scenario == 1:
                exp[calls // 2] = -1
            assert dec == exp, (r, dec)


@pytest.mark.parametrize("world", [2, 4])
def test_read_schedule_off_when_a_socket_is_unreachable(sim_lib, world):
    # csrc/peerbuf.cpp init: the ranks share the board but one rank's descriptor socket cannot be
    # reached (as from another network namespace) -> the read schedule is off on EVERY rank (the
    # self-test returns -3, "no board"), decided at init within the 10 s hello limit, instead of a
    # failed first call with new buffers
    import gpu_workers as GW
    port = GW.free_port()
    out = GW.run_ranks(_board_rank, world, lambda r: (r, world, port, 7, 4), 120)
    assert sorted(out) == list(range(world)), out
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
        assert out[r]["rc"] == -3 and out[r]["secs"] < 30, out[r]


@pytest.mark.parametrize("world", [2, 4, 8, 16])
@pytest.mark.parametrize("scenario", [4, 5, 6], ids=["map-failure", "reused-buffers", "freed-buffers"])
def test_read_schedule_mapping_round(sim_lib, world, scenario):
    # csrc/peerbuf.cpp's second round, one process per rank, no GPU (synthetic buffers): when a
    # call brings a buffer no read call used recently, every rank reports whether it could map
    # its peers' buffers before any launches; one failure (rank 1, call 3: an injected
    # import failure) -> the scratch schedule (0) for that call on EVERY rank and
    # the read schedule (1) on every other call; buffers reused call after call -> the round
    # runs only for the calls that bring a new buffer; buffers reported freed by their owners ->
    # every peer closes its mappings of them (1000 x closed).  dec[i] = decision + 10 x rounds so
    # far.  The new buffers' descriptors (memfds standing in for dma-bufs) really travel between
    # the rank processes over the communicator's sockets and are checked by inode on arrival; at
    # 16 ranks 15 senders overrun a socket's 10-datagram queue (net.unix.max_dgram_qlen).
    import gpu_workers as GW
    calls = 24
    port = GW.free_port()
    out = GW.run_ranks(_board_rank, world, lambda r: (r, world, port, scenario, calls), 120)
    assert sorted(out) == list(range(world)), out
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
        assert out[r]["rc"] == 0, out[r]
        dec = out[r]["dec"]
        if scenario == 4:
            exp = [(0 if i == 2 else 1) + 10 * (i + 1) for i in range(calls)]
        elif scenario == 5:
            exp = [1 + 10 * (1 if i < calls // 2 else 2) for i in range(calls)]
        else:  # the freed buffers' mappings closed on every peer (2 per peer), new ones mapped once
            exp = [1 + 10 if i < calls // 2 else 1 + 20 + 1000 * 2 * (world - 1) for i in range(calls)]
        assert dec == exp, (r, dec)
