"""GPU parity tests (-m gpu): the HIP path through the C ABI vs the CPU oracle.

* mncclLocalReduce (the scatter-reduce element-wise kernel alone) vs oracle_reduce,
  every dtype x op, vector and scalar (misaligned / odd-size) paths, bit-exact;
* ncclAllReduce with 2-10 rank processes, rank r on GPU r % ndev (one rank per GPU on a
  multi-GPU box: a cross-device run over xGMI) or all on GPU 0 on a 1-GPU box / under
  MNCCL_TEST_COLOCATE=1 (as the reference's perf_test does, tests/perf_test.cpp:46), every
  rank's device and co-located rank count checked against that placement; the ring, the
  read schedule (persistent and grid forms) and the one-shot, in/out of place, odd counts
  (tail), repeated calls, slices smaller than a chunk, bit-exact vs the oracle (NaN
  payloads of +/* excepted: NaN-ness must match);
* error paths: watchdog timeout -> ncclInternalError and a sticky error afterwards.
"""
import os
import time

import numpy as np
import pytest

import gpu_workers as GW
import oracle_api as O

pytestmark = pytest.mark.gpu

DTYPES = ["f32", "f64", "i32", "f16", "bf16"]
OPS = ["sum", "prod", "max", "min"]
# (schedule, extra environment): the ring, read (the default's persistent kernel)
SCHEDULES = [pytest.param((0, {}), id="ring"), pytest.param((2, {}), id="read")]


@pytest.fixture(scope="module")
def dev(nccl_lib, oracle_lib):
    # the device check runs in a child: this (pytest) process must hold no GPU queues, or the
    # 8-rank tests would put 9 processes on the GPU (see gpu_workers.Worker)
    out = GW.run_ranks(GW.device_count_probe, 1, lambda r: (), 120)
    if not out or out[0]["count"] < 1:
        pytest.fail("no HIP device visible: the -m gpu suite must run on the MI355X box")
    # placement (gpu_workers.rank_device): rank r on GPU r % ndev, every rank on GPU 0 on a 1-GPU
    # box or under MNCCL_TEST_COLOCATE=1
    NDEV[0] = out[0]["count"]
    print(f"\n[placement] {NDEV[0]} GPU(s) visible, co-located={GW.colocated()}: rank r on GPU "
          f"{'0' if GW.colocated() or NDEV[0] < 2 else 'r % ' + str(NDEV[0])}")
    return NDEV[0]


NDEV = [1]  # GPUs the rank processes see (set by the `dev` fixture)


def _check_placement(r, n, info, env=None):
    """rank r's communicator ran where the placement put it, with the right co-located ranks"""
    colo = GW.colocated(dict(os.environ, **(env or {})))
    want = GW.rank_device(r, NDEV[0], colo)
    if "TEST_DEVICE" in (env or {}):
        return
    assert info["device"] == want, f"rank {r}: device {info['device']}, placement asked for {want}"
    assert info["ranks_on_device"] == GW.ranks_sharing_device(r, n, NDEV[0], colo), (r, n, NDEV[0], info)


class TestLocalReduce:
    """mncclLocalReduce (the scatter-reduce element-wise kernel) in one worker process that ends
    with the class, before the multi-rank tests start."""

    @pytest.fixture(scope="class")
    def worker(self, dev):
        w = GW.Worker()
        yield w
        w.close()

    @pytest.mark.parametrize("dtype", DTYPES)
    @pytest.mark.parametrize("op", OPS)
    @pytest.mark.parametrize("count,offset", [(1 << 20, 0), (100003, 0), (4099, 4), (17, 2), (65539, 1), (1 << 16, 3)])
    def test_local_reduce_parity(self, worker, dtype, op, count, offset):
        bad, first, got, exp = worker.call("local_reduce_case", dtype, op, count, offset)
        assert bad == 0, f"{bad} mismatches, first at {first}: got {got} expected {exp}"

    def test_local_reduce_in_place_large(self, worker):
        assert worker.call("local_reduce_in_place_large") == 0


def _run_allreduce(n, cases, env=None, timeout=300, barrier=True):
    port = GW.free_port()
    # every case sets its schedule explicitly; the ranks line up before each call (barrier); window
    # cases launch with no host rendezvous wherever the ranks are (the device-checked path; auto
    # negotiates them when ranks share a GPU: test_registered_windows_auto_rendezvous)
    e = {"MINI_NCCL_TIMEOUT_MS": "30000", "MINI_NCCL_WINDOW_RENDEZVOUS": "0"}
    e.update(env or {})
    out = GW.run_ranks(GW.allreduce_rank, n, lambda r: (r, n, port, cases, e), timeout,
                       barrier=barrier)
    assert len(out) == n, f"only ranks {sorted(out)} reported (timeout?)"
    for r in range(n):
        assert "error" not in out[r], f"rank {r}:\n{out[r]['error']}"
        assert out[r]["destroy"] == 0
        _check_placement(r, n, out[r]["info"], env)
        for res in out[r]["results"]:
            c = res["case"]
            assert res["rc"] == 0, f"rank {r} case {c}: ncclResult {res['rc']}"
            assert res["bad"] == 0, f"rank {r} case {c}: {res['bad']} mismatches, first at {res['first']} {res.get('detail', '')}"
            assert res["async"] == 0
            # the read schedule ran (no fallback) whenever every rank's buffers are device memory,
            # fresh allocations at re-used addresses included (dma-buf exports, csrc/ipcreg.h)
            dev_bufs = all(c.get(k, "device") == "device" for k in ("mem", "recv_mem"))
            if c["algo"] in (2, 4) and dev_bufs and c["count"] >= n:
                assert res["last_algo"] == 2, f"rank {r} case {c}: ran schedule {res['last_algo']}"
            # forced one-shot: every case of the tests below fits it
            if c["algo"] == 3 and c["count"] >= n:
                assert res["last_algo"] == 3, f"rank {r} case {c}: ran schedule {res['last_algo']}"
            if "expect_algo" in c:
                assert res["last_algo"] == c["expect_algo"], f"rank {r} case {c}: ran schedule {res['last_algo']}"
            if c.get("window") and c["algo"] in (-1, 2, 4) and c["count"] >= n:  # no rendezvous, every call
                assert res["window_calls"] == c["calls"], (r, c, res["window_calls"])
            if "expect_grid" in c:  # the read schedule's grid form ran every call of the case (or none)
                assert res["grid_calls"] == (c["calls"] if c["expect_grid"] else 0), (r, c, res["grid_calls"])
            # no IPC open ever failed (nothing retries: a failure would send a call to the
            # ring, csrc/peerbuf.cpp), in this process or in any rank's mapping round
            assert res["ipc_open_failures"] == 0 and res["read_map_failures"] == 0, (r, c, res)
    return out


def _case(dtype="f32", op="sum", count=1 << 18, inplace=False, algo=0, calls=1, seed=1234, special=False, offset=0,
          **kw):
    return dict(dtype=dtype, op=op, count=count, inplace=inplace, algo=algo, calls=calls, seed=seed, special=special,
                offset=offset, **kw)


@pytest.mark.parametrize("sched", SCHEDULES)
@pytest.mark.parametrize("n", [2, 3, 4])
def test_allreduce_fp32_sum(dev, n, sched):
    algo, env = sched
    cases = [
        _case(count=1 << 20, algo=algo),                     # 4 MiB: C1's size
        _case(count=(1 << 18) + 3, algo=algo, inplace=True),  # tail of count % n
        _case(count=1000, algo=algo),                        # fewer slices than channels
        _case(count=n - 1, algo=algo),                       # count < n: copy only
        _case(count=123457, algo=algo, calls=3, seed=9),     # repeated calls, odd size
    ]
    _run_allreduce(n, cases, env)


@pytest.mark.parametrize("algo", [0, 2], ids=["ring", "read"])
def test_host_buffers(dev, algo):
    # the reference's perf_test hands cudaHostAlloc'd (pinned host) buffers straight to
    # ncclAllReduce (perf_test.cpp:78-79,88): pinned memory is read and written by the kernel
    # through its device mapping, pageable memory is staged through HBM; mixed placements and
    # ranks whose buffers differ must agree (a read call with host buffers runs the ring)
    cases = [
        _case(count=(1 << 20) + 3, algo=algo, mem="pinned"),
        _case(count=(1 << 18) + 1, algo=algo, mem="pinned", inplace=True, seed=5),
        _case(count=(1 << 19) + 5, algo=algo, mem="pageable", seed=6),
        _case(count=(1 << 18) + 2, algo=algo, mem="pageable", inplace=True, seed=7),
        _case(count=200003, algo=algo, mem="device", recv_mem="pinned", seed=8),
        _case(count=200005, algo=algo, mem="pageable", recv_mem="device", seed=9),
        _case(dtype="bf16", count=300001, algo=algo, mem="pinned", calls=2, seed=10),
        _case(count=(1 << 20) + 1, algo=algo, mem=("device", "pinned", "pageable"), seed=11),
    ]
    _run_allreduce(3, cases)


@pytest.mark.parametrize("sched", SCHEDULES + [pytest.param((3, {}), id="oneshot")])
@pytest.mark.parametrize("blocking", ["1", "0"], ids=["blocking", "async"])
def test_skewed_ranks_varying_data(dev, sched, blocking):
    algo, env = sched
    # injected delays (SURVEY.md §5 race detection): every rank sleeps 0-30 ms before each of
    # 4 calls, inputs change every call and every call is checked; sizes alternate so the
    # adaptive payload changes between calls while a peer may still drain the previous one
    cases = [_case(count=c, algo=algo, calls=4, seed=40 + i, vary=True, skew_ms=30)
             for i, c in enumerate(((1 << 20) + 3, 5000, (1 << 18) + 1))]
    cases += [_case(dtype="bf16", count=300007, algo=algo, calls=4, seed=50, vary=True, skew_ms=30, inplace=True)]
    _run_allreduce(4, cases, env={"MINI_NCCL_BLOCKING": blocking, **env})


def test_auto_schedule_no_init_allreduce(dev):
    # MINI_NCCL_ALGO=auto (default): the read schedule (push form), the ring as its fallback; no
    # all-reduce runs at init
    port = GW.free_port()
    out = GW.run_ranks(GW.info_rank, 3, lambda r: (r, 3, port, {}), 120)
    assert all("error" not in out[r] for r in range(3)), out
    for r in range(3):
        i = out[r]["info"]
        # auto (-1): the read schedule; its fallback for buffers that cannot be shared: the ring
        # here (the one-shot for small ones)
        assert i["tune_ms"] == [0.0, 0.0] and i["algo"] == -1 and i["scratch_algo"] == 0, i
        assert i["read_push"] == 1 and i["calib_choice"] == -1 and i["calib_ms"] == [0.0, 0.0], i
        _check_placement(r, 3, i)
        assert i["last_algo"] == -1, i
        assert i["channels"] == 256 and i["pipelines"] == 256 and i["slot_bytes"] == 128 << 10
        assert i["scratch_bytes"] == 2 * 256 * 2 * (128 << 10)  # (n-1) peer regions
    port = GW.free_port()
    out = GW.run_ranks(GW.info_rank, 3, lambda r: (r, 3, port, {"MINI_NCCL_ALGO": "ring", "MINI_NCCL_READ_PUSH": "0"}),
                       120)
    # (MINI_NCCL_READ_PUSH: the load form was removed in 6.0 -- the knob is warned about and ignored)
    assert out[0]["info"]["algo"] == 0 and out[0]["info"]["read_push"] == 1
    # MINI_NCCL_ALGO=direct (removed in 4.0) fails init instead of silently running another schedule
    import mini_nccl as M
    port = GW.free_port()
    out = GW.run_ranks(GW.init_rank, 2, lambda r: (r, 2, port, {0: {"MINI_NCCL_ALGO": "direct"},
                                                               1: {"MINI_NCCL_ALGO": "direct"}}), 120)
    assert out[0]["rc"] == M.ncclSystemError and out[1]["rc"] == M.ncclSystemError


@pytest.mark.parametrize("algo", [0, 2], ids=["ring", "read"])
def test_sys_fence_on(dev, algo):
    # MINI_NCCL_SYS_FENCE=1: system release / acquire fences around every hand-off (the
    # default relies on sc0 sc1 payload accesses of uncached scratch instead)
    cases = [_case(count=(1 << 20) + 1, algo=algo, seed=21), _case(dtype="bf16", count=77777, algo=algo, seed=22)]
    _run_allreduce(3, cases, env={"MINI_NCCL_SYS_FENCE": "1"})


@pytest.mark.parametrize("sched", SCHEDULES)
def test_allreduce_8_ranks(dev, sched):
    algo, env = sched
    # the 8-GPU node's rank count, all on GPU 0 at the library's default geometry (256
    # pipelines): every pair of the mesh exercised; BASELINE C3 (fp32) and C5 (fp16, bf16) on
    # order-sensitive seeded data, bit-exact vs the oracle
    cases = [_case(count=(1 << 20) + 5, algo=algo, seed=8),                              # C3 fp32
             _case(dtype="f16", count=(1 << 20) + 3, algo=algo, inplace=True, seed=9),  # C5 fp16
             _case(dtype="bf16", count=(1 << 19) + 3, algo=algo, inplace=True, seed=10),  # C5 bf16
             _case(count=8 * 4099 + 7, algo=algo, calls=2, seed=11)]
    _run_allreduce(8, cases, env, timeout=600)


@pytest.mark.parametrize("algo", [0, 2], ids=["ring", "read"])
def test_allreduce_10_ranks(dev, algo):
    # past a node's 8 ranks (up to 16 per communicator): the read kernel's one-peer-ahead fold and
    # its peer groups of 7 in the short-slice forms; 10 rank processes on the one GPU with 64
    # pipelines each and one hardware queue each (all resident at once), bit-exact vs the oracle
    cases = [_case(count=10 * 70001 + 3, algo=algo, seed=12),                        # 1-2 KiB slices
             _case(count=10 * (1 << 20), algo=algo, inplace=True, seed=13),          # full batches
             _case(dtype="bf16", count=10 * 50007, algo=algo, seed=14)]
    env = {"MINI_NCCL_CHANNELS": "64", "GPU_MAX_HW_QUEUES": "1"}
    _run_allreduce(10, cases, env, timeout=600)


def test_read_schedule_8_ranks_mixed_calls(dev):
    # the node's rank count through 20 read calls of changing size, placement and dtype on one
    # communicator: the 16-record board wraps, small calls run a few pipelines and large ones
    # all of them, fresh buffers bring the mapping round, reused ones skip it -- every call
    # bit-exact against the oracle
    sizes = [4099, 1 << 20, 77, 8 * 1000 + 5, (1 << 22) + 9, 640, 1 << 18, 123457, 8 * 64 + 3, 1 << 21]
    cases = [_case(dtype=("f32", "bf16")[i % 2], count=sizes[i % len(sizes)], algo=2, inplace=(i % 3 == 0),
                   seed=500 + i, vary=(i % 4 == 1), calls=1 + (i % 4 == 1)) for i in range(20)]
    _run_allreduce(8, cases, {"GPU_MAX_HW_QUEUES": "2"}, timeout=600)


def test_allreduce_8_ranks_c3_ring_128mib(dev):
    # C3's schedule (the reference's ring) in fp32 at 8 ranks on 128 MiB per rank: 16 MiB chunks,
    # every one of the 256 pipelines busy (64 KiB payloads), bit-exact vs the oracle
    cases = [_case(count=8 * (4 << 20) + 3, algo=0, seed=1234)]
    _run_allreduce(8, cases, timeout=600)


@pytest.mark.parametrize("algo", [0, 2], ids=["ring", "read"])
@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("slice_kib", [64, 256, 1024])
def test_allreduce_slice_points(dev, slice_kib, n, algo):
    # BASELINE C4's MINI_NCCL_SLICE_SIZE points (64K / 256K / 1M; 128K is the default everywhere
    # else) with full-size payloads: 16 workgroups so that each pipeline moves >= 3 full slices
    # per chunk plus a ragged one; fp32 and fp16, order-sensitive data, bit-exact vs the oracle
    sl = slice_kib << 10
    chunk_el = 16 * 3 * sl // 4 + 12345
    cases = [_case(count=n * chunk_el + 1, algo=algo, seed=60 + slice_kib),
             _case(dtype="f16", count=n * (chunk_el // 2) + 3, algo=algo, inplace=True, seed=61 + slice_kib)]
    _run_allreduce(n, cases, env={"MINI_NCCL_SLICE_SIZE": str(sl), "MINI_NCCL_CHANNELS": "16"}, timeout=600)


@pytest.mark.parametrize("sched", SCHEDULES)
def test_allreduce_dtypes_ops(dev, sched):
    algo, env = sched
    cases = [_case(dtype=d, op=o, count=50000 + 7 * i, algo=algo, seed=100 + i, special=o in ("max", "min"))
             for i, (d, o) in enumerate((d, o) for d in DTYPES for o in OPS)]
    _run_allreduce(3, cases, env)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_oneshot_parity(dev, n):
    # the one-shot schedule (small calls; forced here so larger calls that fit a slot per pipeline
    # take it too): every dtype x op, tails of count % n, in place, the scalar path (odd 2-byte
    # chunks, a misaligned base), repeated calls on varying data -- bit-exact vs the oracle, the
    # reference ring's association order
    cases = [_case(dtype=d, op=o, count=n * 997 + i % n, algo=3, seed=700 + i, special=o in ("max", "min"),
                   inplace=(i % 3 == 1)) for i, (d, o) in enumerate((d, o) for d in DTYPES for o in OPS)]
    cases += [_case(count=n * 1024, algo=3, seed=720),                          # one 1 KiB piece
              _case(count=(1 << 18) + 3, algo=3, seed=721, inplace=True),       # many pipelines, tail
              _case(dtype="f16", count=n * 333 + 1, algo=3, seed=722),          # odd chunks: scalar path
              _case(count=12345, algo=3, seed=723, offset=2),                   # misaligned: scalar path
              _case(count=n - 1, algo=3, seed=724),                             # count < n: copy only
              _case(count=5000, algo=3, calls=5, seed=725, vary=True)]          # slots and credits reused
    _run_allreduce(n, cases, timeout=600)


def test_oneshot_10_ranks(dev):
    # past a node's 8 ranks (up to 16 per communicator): the one-shot's per-peer lanes and pieces
    # beyond 8, interleaved with ring and read calls; 10 rank processes on the one GPU with 64
    # pipelines and one hardware queue each (all resident at once), bit-exact vs the oracle
    cases = [_case(count=10 * 997 + 3, algo=3, seed=40),
             _case(dtype="bf16", count=10 * 3001, algo=3, seed=41, inplace=True),
             _case(op="max", count=10 * 512 + 9, algo=3, seed=42, special=True),
             _case(count=10 * 70001, algo=0, seed=43),
             _case(count=4099, algo=-1, seed=44, mem="pinned", expect_algo=3),
             _case(count=10 * 5000, algo=2, seed=45, calls=2, vary=True),
             _case(count=12345, algo=3, seed=46, calls=3, vary=True)]
    env = {"MINI_NCCL_CHANNELS": "64", "GPU_MAX_HW_QUEUES": "1"}
    _run_allreduce(10, cases, env, timeout=600)


@pytest.mark.parametrize("n,algo,env", [(2, 2, {}), (3, 2, {}), (8, 2, {"GPU_MAX_HW_QUEUES": "2"}), (3, 0, {})],
                         ids=["read_n2", "read_n3", "read_n8", "ring_n3"])
def test_read_push_visible_to_cached_consumers(dev, n, algo, env):
    # recv's lines pre-warmed into its owner's L2 by an ordinary kernel, then a call
    # whose peers push into that recv (other GPUs over xGMI when the placement spreads the ranks,
    # other XCDs' L2s when they share one), then an ordinary plain-load consumer right behind the
    # call on the same stream: seeded uniform data, every call bit-exact vs the oracle's ring fold
    port = GW.free_port()
    count = (1 << 20) + 2 * n + 1
    e = {"MINI_NCCL_TIMEOUT_MS": "30000", "MINI_NCCL_BLOCKING": "0", "TEST_ALGO": str(algo), **env}
    out = GW.run_ranks(GW.cached_consumer_rank, n, lambda r: (r, n, port, e, count, 6), 600, barrier=True)
    assert sorted(out) == list(range(n)), out
    for r in range(n):
        o = out[r]
        assert "error" not in o, o["error"]
        _check_placement(r, n, o["info"])
        assert o["rcs"] == [0] * 6 and o["async"] == 0 and o["destroy"] == 0, o
        assert o["algos"] == [algo] * 6, o["algos"]
        assert o["bad"] == [0] * 6, (r, o["bad"])


@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_read_grid_parity(dev, n):
    # mncclAlgoReadGrid, the push form's large calls as start / grid fold / done
    # launches (chunks >= 4 MiB, whole 16-byte vectors): ring-order bits vs the oracle, tails, in
    # place, 2-byte types, every op, repeated calls on varying data; a chunk just below the
    # threshold and an odd one stay on the persistent kernel
    m = 1 << 20  # 4 MiB of fp32 per chunk
    g = 4        # mncclAlgoReadGrid
    cases = [_case(count=n * m + n - 1, algo=g, seed=900, expect_grid=True, expect_algo=2),
             _case(count=n * m, algo=g, seed=901, inplace=True, expect_grid=True),
             _case(dtype="bf16", count=n * 2 * m + 1, algo=g, seed=902, expect_grid=True),
             _case(dtype="f64", op="max", count=n * (m // 2) + n * 64, algo=g, seed=903, special=True, expect_grid=True),
             _case(op="prod", count=n * (m + 4), algo=g, seed=904, calls=3, vary=True, expect_grid=True),
             _case(dtype="i32", op="min", count=n * (m + 4) + 1, algo=g, seed=905, expect_grid=True),
             _case(count=n * (m - 256), algo=g, seed=906, expect_grid=False, expect_algo=2),  # below 4 MiB
             _case(dtype="f16", count=n * (2 * m + 1), algo=g, seed=907, expect_grid=False),  # chunk % 16 != 0
             # auto: the grid form for the calls it fits, co-located ranks too (schedule.h read_grid_form)
             _case(count=n * m + 1, algo=-1, seed=908, expect_algo=2, expect_grid=True),
             _case(count=n * m + 1, algo=2, seed=909, expect_algo=2, expect_grid=False)]  # forced persistent
    _run_allreduce(n, cases, {"GPU_MAX_HW_QUEUES": "2"} if n > 4 else None, timeout=600)


@pytest.mark.parametrize("n,vectors", [(2, 4), (2, 2), (5, 1), (8, 4)])
def test_read_grid_vectors_knob(dev, n, vectors):
    # MINI_NCCL_GRID_VECTORS (the node sweep's tuning knob): fp32 Sum calls in the grid form with
    # 1 / 2 / 4 vectors per lane per workgroup, tails and in place; other types and ops follow the
    # rule -- the same bits either way
    m = 1 << 20
    cases = [_case(count=n * m + n - 1, algo=4, seed=1900, expect_grid=True),
             _case(count=n * (m + 256), algo=4, seed=1901, inplace=True, expect_grid=True, calls=2, vary=True),
             _case(count=n * (3 * m + 64), algo=-1, seed=1902, expect_grid=True),
             _case(dtype="bf16", op="max", count=n * 2 * m + n - 1, algo=4, seed=1903, special=True, expect_grid=True)]
    env = {"MINI_NCCL_GRID_VECTORS": str(vectors)}
    if n > 4:
        env["GPU_MAX_HW_QUEUES"] = "2"
    _run_allreduce(n, cases, env, timeout=600)


@pytest.mark.parametrize("n", [2, 8])
def test_read_grid_min_knob(dev, n):
    # MINI_NCCL_GRID_MIN lowered to 256 KiB: auto's DDP-bucket-sized calls (25 MiB) and forced grid
    # calls with chunks from 256 KiB take the grid form, smaller ones the persistent kernel; bit-exact
    m = (256 << 10) // 4  # 256 KiB of fp32
    cases = [_case(count=(25 << 20) // 4 + n - 1, algo=-1, seed=2000, expect_grid=True),
             _case(count=n * m, algo=4, seed=2001, inplace=True, expect_grid=True),
             _case(count=n * (m - 64), algo=4, seed=2002, expect_grid=False, expect_algo=2),
             _case(dtype="bf16", op="min", count=n * 2 * m + 1, algo=-1, seed=2003, special=True, expect_grid=True)]
    env = {"MINI_NCCL_GRID_MIN": str(256 << 10)}
    if n > 4:
        env["GPU_MAX_HW_QUEUES"] = "2"
    _run_allreduce(n, cases, env, timeout=600)


def test_read_grid_skewed_and_interleaved(dev):
    # grid-form calls between persistent read, ring and one-shot calls on one communicator (the
    # grid form moves pipeline 0's counters only), ranks entering every call out of step
    n = 4
    plan = [(4, n * (1 << 20)), (0, 70001), (2, 5000), (4, n * (1 << 20) + 3), (3, 3000), (4, n * (3 << 20)),
            (2, n * (1 << 20))]
    cases = [_case(count=c, algo=a, calls=2, vary=True, seed=950 + i, skew_ms=20, inplace=(i % 2 == 1))
             for i, (a, c) in enumerate(plan)]
    _run_allreduce(n, cases, timeout=600)


def _run_windows(n, scenario, env=None, timeout=300):
    port = GW.free_port()
    e = {"MINI_NCCL_TIMEOUT_MS": "20000", "MINI_NCCL_WINDOW_RENDEZVOUS": "0", **(env or {})}
    out = GW.run_ranks(GW.window_rank, n, lambda r: (r, n, port, e, scenario), timeout, barrier=True)
    assert sorted(out) == list(range(n)), out
    for r in range(n):
        assert "error" not in out[r], out[r]["error"]
        _check_placement(r, n, out[r]["info"], env)
    return out


@pytest.mark.parametrize("n", [2, 3, 8])
def test_registered_windows_parity(dev, n):
    # calls inside registered windows (same windows, same offsets on every rank) run
    # the read schedule with no host rendezvous; every dtype class, in place and out of place,
    # ragged counts, the grid form, interleaved with negotiated and ring calls: bit-exact vs the oracle
    out = _run_windows(n, "parity", {"GPU_MAX_HW_QUEUES": "2"} if n > 4 else None, timeout=600)
    for r in range(n):
        o = out[r]
        assert o["windows"] == 2 and o["windows_after"] == 0 and o["destroy"] == 0, o
        assert all(rc == 0 for rc in o["rcs"]) and all(b == 0 for b in o["bad"]), (r, o["rcs"], o["bad"])
        assert o["kinds"] == [2] * len(o["kinds"]), o["kinds"]  # the read schedule, every window call
        assert o["wc"] == [1] * len(o["wc"]), o["wc"]           # ... each without a rendezvous
        assert o["info"]["read_map_failures"] == 0 and o["info"]["ipc_open_failures"] == 0


@pytest.mark.parametrize("knob", ["-1", "1"])
def test_registered_windows_auto_rendezvous(dev, knob):
    # MINI_NCCL_WINDOW_RENDEZVOUS unset (-1, auto): window calls skip the host rendezvous only when
    # no two ranks share a GPU; co-located ranks negotiate them like any other call (they meet faster
    # on the host: profiles/r6_small_calls_windows.txt); 1: always negotiated -- the same bits
    n = 3
    out = _run_windows(n, "parity", {"MINI_NCCL_WINDOW_RENDEZVOUS": knob}, timeout=600)
    shared = knob == "1" or any(out[r]["info"]["ranks_on_device"] > 1 for r in range(n))
    for r in range(n):
        o = out[r]
        assert all(rc == 0 for rc in o["rcs"]) and all(b == 0 for b in o["bad"]), (r, o["rcs"], o["bad"])
        assert o["kinds"] == [2] * len(o["kinds"]), o["kinds"]
        assert o["info"]["window_fast"] == (0 if shared else 1), o["info"]["window_fast"]
        assert o["wc"] == [0 if shared else 1] * len(o["wc"]), o["wc"]


def test_registered_windows_host_independent(dev):
    # MINI_NCCL_BLOCKING=0 and windows: rank 0's call returns while rank 1 still sleeps 50 ms before
    # its own -- no host rendezvous -- and every result is bit-exact
    out = _run_windows(2, "async", {"MINI_NCCL_BLOCKING": "0"})
    o0, o1 = out[0], out[1]
    assert o0["bad"] == [0] * 4 and o1["bad"] == [0] * 4, (o0["bad"], o1["bad"])
    assert o0["window_calls"] == 4 and o1["window_calls"] == 4
    print(f"\n[windows] rank 0 host time per call (rank 1 50 ms late): "
          f"{[round(t * 1e6, 1) for t in o0['call_s']]} us")
    assert max(o0["call_s"]) < 0.01, o0["call_s"]  # far below the 50 ms a rendezvous would wait


@pytest.mark.parametrize("scenario", ["mismatch", "mismatch_algo"])
def test_registered_windows_mismatch_is_invalid_usage(dev, scenario):
    # a window call whose ranks pass different offsets (or, ADVICE r5, made different schedule
    # choices: auto's grid form against a forced persistent read): the kernels see the signatures
    # differ at START and give up before touching a buffer -- ncclInvalidUsage on every rank, sticky
    import mini_nccl as M
    out = _run_windows(3, scenario)
    for r in range(3):
        o = out[r]
        assert o["rc"] == M.ncclInvalidUsage and o["rc2"] == M.ncclInvalidUsage, (r, o)
        assert o["secs"] < 5, o


def test_registered_windows_unregistered_peer_fails_fast(dev):
    # rank 0 passes window buffers, the others buffers outside any window: the others see rank 0's
    # window record in their rendezvous and fail the call at once (ncclInvalidUsage), raising rank
    # 0's ABORT so its kernel does not wait for a START that never comes
    import mini_nccl as M
    out = _run_windows(3, "unregistered")
    for r in range(3):
        o = out[r]
        assert o["rc"] in (M.ncclInvalidUsage, M.ncclRemoteError), (r, o)
        assert o["rc2"] != 0 and o["secs"] < 5, (r, o)


def test_schedules_interleaved_on_one_communicator(dev):
    # the one-shot, the ring and the read schedule share the per-(pair, pipeline) FIFO counters,
    # READY words, credits and scratch slots: calls of all three (and auto's choice by size)
    # alternate on one communicator, on changing data, every call checked
    n = 4
    plan = [(3, 3000), (0, 70001), (2, 1 << 18), (-1, 4096), (3, 16384), (0, 1000), (-1, 1 << 20), (2, 777),
            (3, 100003), (-1, 65536 // 4), (0, 5), (3, 8 * 1024), (4, 4 * (1 << 20) + 3)]
    # (auto: device buffers every rank shares run the read schedule at every size); five read /
    # auto cases on registered windows (no host rendezvous for their calls)
    cases = [_case(count=c, algo=a, calls=2, vary=True, seed=800 + i, inplace=(i % 2 == 0), window=i in (2, 3, 6, 7, 12),
                   **({"expect_algo": 2} if a == -1 else {})) for i, (a, c) in enumerate(plan)]
    _run_allreduce(n, cases, timeout=600)


@pytest.mark.parametrize("mem", ["pinned", "pageable"])
def test_oneshot_host_buffers(dev, mem):
    # auto's small calls on host buffers (the ring's domain before one-shot): pinned memory read
    # and written through its device mapping, pageable memory staged through HBM; above 64 KiB
    # the ring again
    cases = [_case(count=4099, algo=-1, mem=mem, seed=30, expect_algo=3),
             _case(count=3 * 5000 + 2, algo=-1, mem=mem, inplace=True, seed=31, expect_algo=3),
             _case(dtype="bf16", count=3001, algo=-1, mem=mem, recv_mem="device", seed=32, expect_algo=3),
             _case(count=3 * (1 << 14) + 1, algo=-1, mem=mem, seed=33, expect_algo=0)]
    _run_allreduce(3, cases)


@pytest.mark.parametrize("what", ["count", "algo"])
def test_read_schedule_count_mismatch_is_invalid_usage(dev, what):
    # MINI_NCCL_ALGO=read: every rank sees every rank's (count, dtype, op, schedule choice) in the
    # per-call rendezvous, so a call whose ranks disagree fails on all of them alike, and nothing is
    # left half-done: the next (matching) call is bit-exact.  "algo": one rank on auto, the others
    # on mncclAlgoRead (they would launch different kernel forms)
    port = GW.free_port()
    env = {"MINI_NCCL_ALGO": "read", "MINI_NCCL_TIMEOUT_MS": "20000", "MISMATCH": what}
    out = GW.run_ranks(GW.mismatch_rank, 3, lambda r: (r, 3, port, env), 180)
    for r in range(3):
        assert "error" not in out[r], out[r].get("error")
        o = out[r]
        assert o["rc_bad"] == 5 and o["rc_ok"] == 0 and o["bad"] == 0 and o["last_algo"] == 2, o
        assert o["async"] == 0 and o["destroy"] == 0


def test_read_schedule_allocation_churn(dev):
    # a fresh hipMalloc'd send and recv for each of 70 calls, freed after it (addresses come back
    # with new allocation ids, often in the same buffer object): every call runs the read schedule
    # (a new allocation is a new dma-buf export, csrc/ipcreg.h); every freed allocation a peer
    # mapped is reported by its owner at its next call and the peer unmaps its import -- mappings
    # stay bounded, no import fails, every call bit-exact
    n = 3
    cases = [_case(count=4099 + 13 * i, algo=2, seed=900 + i, inplace=(i % 3 == 0), fresh=True) for i in range(70)]
    out = _run_allreduce(n, cases, timeout=600)
    for r in range(n):
        res = out[r]["results"]
        assert all(x["last_algo"] == 2 for x in res), [x["last_algo"] for x in res]
        # the peers' user allocations of this call and at most those of the call before (an owner
        # reports a free with its next call)
        assert all(x["peer_mappings"] <= 4 * (n - 1) for x in res), [x["peer_mappings"] for x in res]
        assert res[-1]["closed_freed"] >= _freed_imports(res, n), [x["closed_freed"] for x in res]
        assert all(x["live_exports"] <= 2 for x in res)


def test_same_gpu_freed_imports_leave_later_exports_intact(dev):
    # the round-5 stress's failure, bisected (tools/r5_export_bisect.py, 5 ranks): fresh 20 MiB
    # buffers that every peer imported, freed by their owners, then new allocations registered as
    # windows and run.  On one GPU the driver gives an import the exporter's handle; had the peers
    # unmapped their imports of the freed buffers, that second delete would take the handle of a
    # buffer allocated since (its export then fails, or names another buffer: wrong results,
    # profiles/r5_export_alias.txt).  Same-GPU imports are retired instead (csrc/ipcreg.h
    # close_import): every registration succeeds, every call bit-exact
    n = 5
    cases = []
    for i in range(4):
        cases += [_case(dtype="i32", count=n << 20, algo=-1, seed=2100 + 3 * i, fresh=True),
                  _case(dtype="i32", op="max", count=n + i, algo=0, seed=2101 + 3 * i, window=True),
                  _case(count=4099 + i, algo=2, seed=2102 + 3 * i, window=True, calls=2, vary=True)]
    out = _run_allreduce(n, cases, timeout=400)
    for r in range(n):
        colocated = out[r]["info"]["ranks_on_device"]
        res = out[r]["results"]
        assert all(x["window_calls"] >= 1 for x in res if x["case"].get("window") and x["case"]["algo"] == 2), \
            [x["window_calls"] for x in res]
        if colocated == n:  # every peer on this GPU: every freed import retired, none unmapped
            assert res[-1]["retired_imports"] >= res[-1]["closed_freed"] > 0, res[-1]


def _churn(n, env, calls, nbytes, timeout):
    port = GW.free_port()
    e = {"MINI_NCCL_TIMEOUT_MS": "30000", **env}
    out = GW.run_ranks(GW.churn_rank, n, lambda r: (r, n, port, e, calls, nbytes), timeout, barrier=True)
    assert sorted(out) == list(range(n)), out
    for r in range(n):
        assert "error" not in out[r], out[r]["error"]
        o = out[r]
        _check_placement(r, n, o["info"])
        assert o["destroy"] == 0 and o["rcs"] == [0] * calls and o["bad"] == 0, (r, o["bad"], o["rcs"][:8])
        assert o["info"]["ipc_open_failures"] == 0, o["info"]
    return out


def test_retired_imports_bounded_by_byte_budget(dev):
    # 2 ranks, 200 calls, each on a fresh 64 MiB allocation freed after it.  Co-located,
    # every peer import of a freed buffer stays mapped (the driver's shared handle, csrc/ipcreg.h):
    # MINI_NCCL_RETIRED_MB = 1024 bounds what that pins -- the calls past it run the ring on every
    # rank alike, counted in budget_refusals, each still exact -- and the device's free memory never
    # drops by more than both processes' budgets plus the live buffers
    n, calls, nbytes, budget = 2, 200, 64 << 20, 1024 << 20
    out = _churn(n, {"MINI_NCCL_RETIRED_MB": str(budget >> 20)}, calls, nbytes, 600)
    for r in range(n):
        o, i = out[r], out[r]["info"]
        if i["ranks_on_device"] == 1:  # a GPU of its own: nothing is retired, every call reads
            assert i["retired_bytes"] == 0 and set(o["algos"]) == {2}, (r, i["retired_bytes"], o["algos"][:8])
            continue
        assert i["retired_budget"] == budget, i["retired_budget"]
        assert budget <= i["retired_bytes"] <= budget + nbytes, i["retired_bytes"]
        assert i["budget_refusals"] > 0, i
        k = o["algos"].index(0)  # the first ring call: past the budget, every call the ring
        assert set(o["algos"][:k]) == {2} and set(o["algos"][k:]) == {0}, o["algos"]
        assert k <= budget // nbytes + 2, k
        drop = o["free0"] - o["min_free"]
        assert drop <= n * (budget + 2 * nbytes) + (512 << 20), (drop >> 20, "MiB")


def test_freed_peer_buffers_beyond_the_import_cap(dev):
    # more freed peer allocations than the import cap (1024, live + retired) across
    # co-located ranks: past the cap every call runs the ring (cap_refusals), still exact, and the
    # memory the retired imports hold is recorded (small buffers: the byte budget is not the bound)
    n, calls, nbytes = 2, 1100, 64 << 10
    out = _churn(n, {}, calls, nbytes, 600)
    for r in range(n):
        o, i = out[r], out[r]["info"]
        if i["ranks_on_device"] == 1:
            assert i["retired_imports"] == 0 and set(o["algos"]) == {2}
            continue
        assert i["retired_imports"] >= 1000 and i["retired_bytes"] >= i["retired_imports"] * nbytes, i
        assert i["cap_refusals"] > 0 and i["budget_refusals"] == 0, i
        # (the read schedule's fallback for a call this small under auto: the one-shot, else the ring)
        assert o["algos"][:900] == [2] * 900 and set(o["algos"][-50:]) <= {0, 3}, o["algos"][895:910]
        print(f"rank {r}: {i['retired_imports']} retired imports hold {i['retired_bytes'] >> 20} MiB")


def test_more_pipelines_than_stay_resident(dev):
    # every rank's pipeline w waits for its peers' pipeline w, so the waves one call launches on a
    # GPU must all be resident: 8 co-located ranks x 512 channels = 4096 one-wave pipelines for 2048
    # wave slots (256 CUs x 4 SIMDs x 2) timed out in the round-6 proxy sweep.  A call now launches
    # at most run_pipelines (all 512 when every rank has its own GPU); read, ring and one-shot
    # calls bit-exact
    n = 8
    cases = [_case(count=(64 << 20) // 4 + 5, algo=2, seed=930), _case(count=(64 << 20) // 4, algo=0, seed=931),
             _case(count=(1 << 20) + 3, algo=2, seed=932, calls=2, vary=True), _case(count=n * 512, algo=3, seed=933),
             _case(count=(16 << 20) // 4, algo=4, seed=934)]
    out = _run_allreduce(n, cases, {"MINI_NCCL_CHANNELS": "512", "GPU_MAX_HW_QUEUES": "2"}, timeout=600)
    most = max(out[r]["info"]["ranks_on_device"] for r in range(n))
    for r in range(n):
        i = out[r]["info"]
        # (512 workgroups, fewer where the scratch cap bounds them: 292 at 8 ranks)
        assert 256 < i["pipelines"] <= 512 and i["run_pipelines"] <= i["pipelines"], i
        assert i["run_pipelines"] * most <= 2048, (i["pipelines"], i["run_pipelines"], most)
        if most == 1:
            assert i["run_pipelines"] == i["pipelines"]


def test_read_schedule_send_recv_in_one_allocation(dev):
    # out of place with send and recv two regions of ONE allocation on every rank: the owner's
    # descriptor datagram carries that allocation once, both mappings come from one import;
    # cached and fresh allocations, every call run by the read schedule and bit-exact
    n = 3
    cases = [_case(count=300007 + 5 * i, algo=2, seed=1500 + i, one_alloc=True, fresh=(i % 2 == 1), calls=2, vary=True)
             for i in range(6)]
    out = _run_allreduce(n, cases, timeout=300)
    for r in range(n):
        assert all(x["last_algo"] == 2 for x in out[r]["results"])


def test_read_schedule_two_communicators_share_buffers(dev):
    # two communicators per rank process over the same ranks, the same buffers used on both
    # (calls alternate); every other round on fresh allocations that are then freed -- every call
    # read and bit-exact, no import fails, frees reach both communicators
    n = 3
    ports = (GW.free_port(), GW.free_port())
    out = GW.run_ranks(GW.two_comms_rank, n, lambda r: (r, n, ports, {"MINI_NCCL_TIMEOUT_MS": "30000"}, 6), 300)
    assert sorted(out) == list(range(n)), out
    for r in range(n):
        o = out[r]
        assert "error" not in o, o["error"]
        assert o["bad"] == 0 and all(rc == 0 for rc in o["rcs"]) and o["destroy"] == [0, 0], o
        assert all(a == 2 for a in o["algos"]), o["algos"]
        assert o["ipc_open_failures"] == 0 and o["read_map_failures"] == [0, 0], o
        assert sum(o["closed_freed"]) >= 2 * (n - 1) * 2, o  # rounds 1 and 3's fresh buffers at least


def test_read_schedule_frees_mapped_allocations(dev):
    # large allocations (64-96 MiB) mapped by every peer and then freed by their owner while the
    # peers still hold the mappings (hipFree before the importers close: the owner reports the
    # allocation freed with its next call, the peers close their imports then); new allocations
    # of the same and other sizes after them -- every call bit-exact, no open fails, every freed
    # allocation's imports closed
    n = 3
    sizes = [16 << 20, 16 << 20, 24 << 20, 16 << 20, 24 << 20, 20 << 20]  # elements (fp32)
    cases = [_case(count=c + i, algo=2, seed=1300 + i, fresh=True, calls=2, vary=True) for i, c in enumerate(sizes)]
    out = _run_allreduce(n, cases, timeout=600)
    for r in range(n):
        res = out[r]["results"]
        assert res[0]["last_algo"] == 2
        assert _freed_imports(res, n) >= 2 * (n - 1)
        assert res[-1]["closed_freed"] >= _freed_imports(res, n), [x["closed_freed"] for x in res]


def _freed_imports(res, n):
    """imports a rank must have closed by the end: every peer buffer of every read case but the
    last (an owner reports its freed allocations with its next call)"""
    return sum((n - 1) * (1 if x["case"]["inplace"] else 2) for x in res[:-1] if x["last_algo"] == 2)


@pytest.mark.parametrize("dtype,algos,gib,knobs", [
    # -1: the library default (auto: read, its large calls in the grid form), 2: the persistent
    # read kernel, 0: the reference's ring
    ("f32", (-1, 2, 0), 1, {}), ("bf16", (-1, 2), 1, {}), ("f16", (2, -1), 1, {}),
    # C4: 4 GiB fp32, the grid's extreme geometries (WINDOW 16 -> 128 pipelines with 64 KiB
    # slices; 1 MiB slices -> 36 pipelines under the scratch cap), ring as C4 names it
    ("f32", (0, 2, -1), 4, {"MINI_NCCL_SLICE_SIZE": "65536", "MINI_NCCL_WINDOW_SIZE": "16"}),
    ("f32", (0,), 4, {"MINI_NCCL_SLICE_SIZE": "1048576", "MINI_NCCL_WINDOW_SIZE": "64"})],
    ids=["c3_f32_auto_read_ring", "c5_bf16_auto_read", "c5_f16_read_auto", "c4_64k_w16_ring_read_auto",
         "c4_1m_w64_ring"])
def test_allreduce_8_ranks_full_size(dev, dtype, algos, gib, knobs):
    # BASELINE C3 (8 ranks, 1 GiB fp32; the library default in its grid form, the persistent read
    # kernel and the reference's ring), C5 (8 ranks, 1 GiB fp16 / bf16; default and persistent)
    # and C4 (8 ranks, 4 GiB fp32) at their FULL sizes, seeded
    # uniform[-1, 1) inputs (order-sensitive), bit-exact against the oracle's closed-form ring
    # fold -- itself pinned to the loop-by-loop restatement of mini_nccl.cu:108-194
    # (tests/test_oracle.py).  The ranks report 16 MiB block digests of their result; the
    # oracle's digests are computed here.
    n = 8
    count = (gib << 30) // (4 if dtype == "f32" else 2)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(n) as ex:
        xs = list(ex.map(lambda r: GW.fullsize_input(r, count, dtype), range(n)))
    exp = GW.block_digests(O.ring_fold_parallel(xs, dtype, "sum"))
    del xs
    port = GW.free_port()
    env = {"MINI_NCCL_TIMEOUT_MS": "60000", "GPU_MAX_HW_QUEUES": "2", **knobs}
    out = GW.run_ranks(GW.fullsize_rank, n, lambda r: (r, n, port, env, dtype, count, algos), 600, barrier=True)
    assert sorted(out) == list(range(n)), f"only ranks {sorted(out)} reported"
    for r in range(n):
        assert "error" not in out[r], f"rank {r}:\n{out[r]['error']}"
        assert out[r]["destroy"] == 0
        _check_placement(r, n, out[r]["info"], env)
        for res in out[r]["results"]:
            assert res["rc"] == 0 and res["async"] == 0, (r, res["algo"], res["rc"], res["async"])
            assert res["last_algo"] == (2 if res["algo"] == -1 else res["algo"]), (r, res["algo"], res["last_algo"])
            # the default's 1 GiB calls ran in the grid form (chunks of 128 MiB), the forced ones not
            assert res["grid_calls"] == (1 if res["algo"] == -1 else 0), (r, res["algo"], res["grid_calls"])
            bad = [i for i, (g, e) in enumerate(zip(res["digests"], exp)) if g != e]
            assert len(res["digests"]) == len(exp) and not bad, \
                f"rank {r} schedule {res['algo']} in_place={res['inplace']}: 16 MiB blocks {bad[:8]} differ"


def test_allreduce_c2_full_size(dev):
    # BASELINE.json configs[1] (C2): 2 ranks, 256 MiB fp32, MINI_NCCL_SLICE_SIZE = 128 KiB,
    # seeded uniform inputs, bit-exact against the oracle at full size
    cases = [_case(count=64 << 20, algo=a, seed=1234 + a) for a in (0, 2)]
    _run_allreduce(2, cases, env={"MINI_NCCL_SLICE_SIZE": "131072"}, timeout=600)


def test_allreduce_small_slices_many_messages(dev):
    # 1 KiB slices, 4 channels: thousands of flag hand-offs per call, both schedules
    cases = [_case(count=(1 << 19) + 5, algo=a, calls=2, seed=77) for a in (0, 2)]
    _run_allreduce(4, cases, env={"MINI_NCCL_SLICE_SIZE": "1024", "MINI_NCCL_CHANNELS": "4"})


def test_allreduce_misaligned_buffers(dev):
    # dword-aligned but not 16-byte-aligned buffers (vector path with straddling vectors)
    # and 2-byte-aligned halves with odd chunks (element path)
    cases = [_case(count=40001, algo=a, offset=o, seed=5) for a in (0, 2) for o in (4, 8, 12)]
    cases += [_case(dtype="bf16", count=30001, algo=a, offset=2, seed=6) for a in (0, 2)]
    _run_allreduce(3, cases)


def test_allreduce_async_mode(dev):
    cases = [_case(count=1 << 20, algo=a, calls=4, seed=3) for a in (0, 2)]
    _run_allreduce(2, cases, env={"MINI_NCCL_BLOCKING": "0"})


@pytest.mark.parametrize("algo", ["ring", "read"])
def test_destroy_waits_for_calls_in_flight(dev, algo):
    port = GW.free_port()
    env = {"MINI_NCCL_BLOCKING": "0", "MINI_NCCL_ALGO": algo, "MINI_NCCL_TIMEOUT_MS": "30000"}
    out = GW.run_ranks(GW.destroy_inflight_rank, 3, lambda r: (r, 3, port, env), 180)
    assert sorted(out) == [0, 1, 2], out
    for r in range(3):
        assert "error" not in out[r], out[r]["error"]
        assert out[r]["rcs"] == [0, 0, 0] and out[r]["destroy"] == 0 and out[r]["bad"] == 0, out[r]


def test_allreduce_reference_known_answers(dev):
    # perf_test.cpp: all ranks send 1.0 -> every element == nRanks (the oracle agrees)
    cases = [dict(_case(count=(16 << 20) // 4, seed=0), known="ones")]
    out = _run_allreduce(2, cases)
    assert out[0]["info"]["nranks"] == 2


def test_watchdog_timeout_is_internal_error_and_sticky(dev):
    import mini_nccl as M
    port = GW.free_port()
    env = {"MINI_NCCL_TIMEOUT_MS": "1500", "STALL_SECS": "6"}
    out = GW.run_ranks(GW.stall_rank, 2, lambda r: (r, 2, port, env, r == 0), 120)
    assert 0 in out and "error" not in out[0], out
    assert out[0]["rc"] == M.ncclInternalError
    assert out[0]["secs"] < 15
    assert out[0]["rc2"] == M.ncclInternalError  # the communicator stays failed
    assert out[0]["async"] == M.ncclInternalError


@pytest.mark.parametrize("algo", ["ring", "read", "oneshot"])
def test_late_peer_is_aborted_fast(dev, algo):
    # rank 0 gives up on rank 1 (kernel watchdog for ring and one-shot, the read schedule's
    # rendezvous limit for read); either way it raises rank 1's ABORT word, so rank 1's late call fails at once
    import mini_nccl as M
    port = GW.free_port()
    env = {"MINI_NCCL_TIMEOUT_MS": "1500", "STALL_SECS": "7", "LATE_CALL": "1", "MINI_NCCL_ALGO": algo}
    out = GW.run_ranks(GW.stall_rank, 2, lambda r: (r, 2, port, env, r == 0), 120)
    assert sorted(out) == [0, 1] and all("error" not in v for v in out.values()), out
    assert out[0]["rc"] == M.ncclInternalError and out[0]["secs"] < 15
    assert out[1]["rc"] == M.ncclRemoteError, out[1]
    assert out[1]["secs"] < 1.5, out[1]  # well under its own 1.5 s watchdog + 2 s host limit


@pytest.mark.parametrize("algo", ["ring", "read", "oneshot", "read_grid", "read_window"])
def test_allreduce_hip_graph_capture_and_replay(dev, algo):
    # the reference only warns under capture (api.cpp:153-166); here a captured all-reduce
    # replays correctly because the FIFO counters are device state advanced by the kernel (the
    # grid form: three captured launches, its `go` word rewritten by every replay's START)
    port = GW.free_port()
    env = {"MINI_NCCL_TIMEOUT_MS": "20000", "MINI_NCCL_ALGO": algo.replace("_window", "")}
    if algo == "read_grid":
        env["GRAPH_COUNT"] = str(3 * (1 << 20) + 1)
    if algo == "read_window":  # registered windows: the captured launch carries its START signature
        env.update(GRAPH_WINDOW="1", MINI_NCCL_WINDOW_RENDEZVOUS="0")
    out = GW.run_ranks(GW.graph_rank, 3, lambda r: (r, 3, port, env, 4), 240)
    assert sorted(out) == [0, 1, 2], out
    for r in range(3):
        assert "error" not in out[r], out[r]["error"]
        assert out[r]["capture_rc"] == [0]
        assert out[r]["bad"] == [0, 0, 0, 0]
        assert out[r]["eager_rc"] == 0 and out[r]["eager_bad"] == 0
        # the read schedule is captured too (its peer mappings pinned for the replays)
        assert out[r]["captured_algo"] == {"ring": 0, "read": 2, "oneshot": 3, "read_grid": 2, "read_window": 2}[algo]
        assert out[r]["captured_grid"] == (1 if algo == "read_grid" else 0)
        assert out[r]["captured_window"] == (1 if algo == "read_window" else 0)


@pytest.mark.parametrize("algo", ["ring", "read", "oneshot"])
def test_calls_on_alternating_streams_are_ordered(dev, algo):
    port = GW.free_port()
    env = {"MINI_NCCL_TIMEOUT_MS": "20000", "MINI_NCCL_ALGO": algo, "MINI_NCCL_BLOCKING": "0"}
    out = GW.run_ranks(GW.streams_rank, 3, lambda r: (r, 3, port, env, 6), 180)
    assert sorted(out) == [0, 1, 2], out
    for r in range(3):
        assert "error" not in out[r], out[r]["error"]
        assert out[r]["rcs"] == [0] * 6 and out[r]["bad"] == [0] * 6
        assert out[r]["async"] == 0 and out[r]["destroy"] == 0


def test_link_probe_then_allreduce(dev):
    port = GW.free_port()
    out = GW.run_ranks(GW.probe_rank, 3, lambda r: (r, 3, port, {"MINI_NCCL_TIMEOUT_MS": "20000"}), 180)
    assert sorted(out) == [0, 1, 2], out
    for r in range(3):
        assert "error" not in out[r], out[r]["error"]
        assert out[r]["next"] > 0 and out[r]["mesh"] > 0
        assert len(out[r]["variants"]) == 12 and all(g > 0 for g in out[r]["variants"])
        assert out[r]["rc"] == 0 and out[r]["exact"]


def test_single_rank_is_copy_only(dev):
    # nRanks == 1: the reference returns after the send->recv copy (mini_nccl.cu:66)
    cases = [_case(count=100001, seed=4), _case(count=4097, inplace=True, seed=5),
             _case(dtype="f64", op="max", count=3001, seed=6)]
    _run_allreduce(1, cases)


@pytest.mark.parametrize("knob,values", [("MINI_NCCL_SLICE_SIZE", ("131072", "65536")),
                                         ("MINI_NCCL_ALGO", ("ring", "oneshot")),
                                         ("MINI_NCCL_WINDOW_SIZE", ("64", "16")),
                                         ("MINI_NCCL_GRID_MIN", (str(4 << 20), str(1 << 20)))])
def test_mismatched_config_is_system_error(dev, knob, values):
    # every init failure is ncclSystemError, as in the reference (api.cpp:62-65)
    import mini_nccl as M
    port = GW.free_port()
    env = {0: {knob: values[0]}, 1: {knob: values[1]}}
    out = GW.run_ranks(GW.init_rank, 2, lambda r: (r, 2, port, env), 120)
    assert sorted(out) == [0, 1], out
    assert out[0]["rc"] == M.ncclSystemError and out[1]["rc"] == M.ncclSystemError


def test_unparsable_knob_is_system_error(dev):
    import mini_nccl as M
    port = GW.free_port()
    out = GW.run_ranks(GW.init_rank, 1, lambda r: (r, 1, port, {0: {"MINI_NCCL_SLICE_SIZE": "12x"}}), 60)
    assert out[0]["rc"] == M.ncclSystemError, out


def test_watchdog_deadline_starts_with_the_kernel(dev):
    # 6 s of work queued ahead of the call on its stream, a 3 s kernel watchdog: the host's
    # deadline (timeout + 2 s) must count from the kernel's start, not from the call
    port = GW.free_port()
    env = {"MINI_NCCL_TIMEOUT_MS": "3000", "MINI_NCCL_ALGO": "ring"}
    out = GW.run_ranks(GW.delayed_start_rank, 2, lambda r: (r, 2, port, env, 6.0), 120)
    assert sorted(out) == [0, 1], out
    for r in range(2):
        assert "error" not in out[r], out[r]["error"]
        assert out[r]["rc"] == 0 and out[r]["bad"] == 0 and out[r]["async"] == 0, out[r]
        assert out[r]["secs"] >= 5.5 and out[r]["destroy"] == 0, out[r]


@pytest.mark.parametrize("n", [2, 8])
def test_ring_small_calls_run_only_their_pipelines(dev, n):
    # the ring launches one pipeline per slice up to all 256 (schedule.h call_pipelines): calls
    # from 1 slice to the full grid, interleaved with read calls on the same communicator (its
    # idle pipelines' counters must stay in step on every rank), bit-exact vs the oracle
    sizes = [n * 64 + 1, 1000, n * 1024 * 7 + 3, 4099, n * 256 * 1024 + 5, 77, (1 << 20) + 3]
    cases = [_case(count=c, algo=(0 if i % 3 else 2), seed=1700 + i, vary=True, calls=2, inplace=i % 2 == 1)
             for i, c in enumerate(sizes)]
    _run_allreduce(n, cases, {"GPU_MAX_HW_QUEUES": "2"}, timeout=300)


def test_read_schedule_many_live_buffers(dev):
    # ~600 distinct live allocations per rank (300 send / recv pairs), one read call
    # each: bit-exact; past the process's 512-export cap the calls run the ring on every rank
    # alike, counted (cap_refusals) and warned once; the pointer queries per call stay bounded by
    # the call's own buffers + a batch of 4, whatever the number of live exports
    n, pairs = 2, 300
    port = GW.free_port()
    out = GW.run_ranks(GW.many_buffers_rank, n, lambda r: (r, n, port, {"MINI_NCCL_TIMEOUT_MS": "30000"}, pairs), 600)
    assert sorted(out) == list(range(n)), out
    for r in range(n):
        o = out[r]
        assert "error" not in o, o["error"]
        assert o["bad"] == 0 and all(rc == 0 for rc in o["rcs"]) and o["destroy"] == 0, o["bad"]
        assert o["algos"][:256] == [2] * 256, o["algos"][:256]  # 512 exports: 256 pairs share
        assert all(a == 0 for a in o["algos"][256:]), o["algos"][256:]  # beyond the cap: the ring
        assert o["info"]["cap_refusals"] > 0 and o["info"]["live_exports"] == 512, o["info"]
        assert max(o["queries"]) <= 2 + 4, o["queries"]
        assert o["info"]["ipc_open_failures"] == 0 and o["info"]["read_map_failures"] == 0, o["info"]
    assert out[0]["algos"] == out[1]["algos"]


def test_destroy_releases_shared_memory(dev):
    # an allocation a read call exported (dma-buf) and the peers imported is released
    # by its owner's hipFree once every communicator is destroyed (destroy closes the imports of
    # peers no live communicator talks to, and the last one closes the process's exports) -- when
    # no peer shares the owner's GPU.  A same-GPU peer keeps its import while its process lives
    # (csrc/ipcreg.h close_import: the driver's shared handle, DESIGN.md Same-GPU handle loss), so
    # there the memory stays pinned after the free
    n, nbytes = 3, 256 << 20
    port = GW.free_port()
    out = GW.run_ranks(GW.release_rank, n, lambda r: (r, n, port, {"MINI_NCCL_TIMEOUT_MS": "30000"}, nbytes), 300,
                       barrier=True)
    assert sorted(out) == list(range(n)), out
    for r in range(n):
        o = out[r]
        assert "error" not in o, o["error"]
        assert o["rc"] == 0 and o["destroy"] == 0 and o["ok"] and o["last_algo"] == 2, o
        if o["ranks_on_device"] == 1:
            assert o["freed"] >= nbytes * 9 // 10, o  # the memory came back at hipFree
        else:
            assert o["freed"] < nbytes // 2, o  # held by the same-GPU peers' imports until they exit


def test_count_beyond_int32(dev):
    # 2^31 + 7 bf16 elements per rank (4 GiB): 64-bit counts end to end
    port = GW.free_port()
    count = (1 << 31) + 7
    out = GW.run_ranks(GW.huge_rank, 2, lambda r: (r, 2, port, {"MINI_NCCL_TIMEOUT_MS": "60000"}, count), 600)
    assert sorted(out) == [0, 1], out
    for r in range(2):
        assert "error" not in out[r], out[r]["error"]
        assert out[r]["rc"] == 0 and out[r]["bad"] == 0, out[r]


def test_chunks_beyond_4gib(dev):
    # 2 ranks, 2^31 + 2^20 + 9 int32 per rank (8 GiB + 4 MiB): rank 1's chunk starts past 2^32
    # bytes; position-coded values (far_offsets_rank) catch a wrapped offset in any schedule
    port = GW.free_port()
    count = (1 << 31) + (1 << 20) + 9
    algos = [0, 2, 4]  # ring, read (persistent), read's grid form
    env = {"MINI_NCCL_TIMEOUT_MS": "60000", "GPU_MAX_HW_QUEUES": "2"}
    out = GW.run_ranks(GW.far_offsets_rank, 2, lambda r: (r, 2, port, env, count, algos), 900)
    assert sorted(out) == [0, 1], out
    for r in range(2):
        assert "error" not in out[r], out[r]["error"]
        bad, first = out[r]["checker"]  # the device check flags an input that is not the sum
        assert first == 1 and bad >= out[r]["body"] - 2, out[r]
        res = out[r]["results"]
        assert [x["algo"] for x in res] == algos, res
        for x in res:
            assert x["rc"] == 0 and x["bad"] == 0, (r, x)
        assert [x["last_algo"] for x in res][:2] == [0, 2], res
        assert res[2]["grid_calls"] == res[1]["grid_calls"] + 1, res  # the grid form ran
        assert out[r]["destroy"] == 0, out[r]


@pytest.mark.parametrize("n", [2, 3])
def test_ranks_as_threads_of_one_process(dev, n):
    # the same-process peer paths (raw pointers, no IPC) under every schedule, bit-exact
    port = GW.free_port()
    cases = [dict(dtype="f32", count=1000, algo=-1, inplace=False, seed=61),          # auto: small call
             dict(dtype="f32", count=(1 << 20) + 3, algo=0, inplace=False, seed=62),  # ring
             dict(dtype="f32", count=(1 << 20) + 3, algo=2, inplace=True, seed=63),   # read, persistent
             dict(dtype="f32", count=3 << 21, algo=4, inplace=False, seed=64),        # read, grid form
             dict(dtype="bf16", count=3 << 21, algo=-1, inplace=False, seed=65),      # auto, large
             dict(dtype="f64", count=4099, algo=3, inplace=False, seed=66)]           # one-shot
    env = {"MINI_NCCL_TIMEOUT_MS": "30000"}
    out = GW.run_ranks(GW.threaded_ranks_proc, 1, lambda _: (n, port, env, cases), 300)
    assert 0 in out and "error" not in out[0], out
    ranks = out[0]["ranks"]
    assert sorted(ranks) == list(range(n)), ranks
    for r in range(n):
        o = ranks[r]
        assert "error" not in o, o["error"]
        assert o["ranks_on_device"] == n and o["ipc_open_failures"] == 0 and o["destroy"] == 0, o
        assert len(o["results"]) == len(cases), o
        for x in o["results"]:
            assert x["rc"] == 0 and x["bad"] == 0, (r, x)
        algos = [x["last_algo"] for x in o["results"]]
        assert algos[1] == 0 and algos[2] == 2 and algos[5] == 3, algos


def test_sixteen_ranks_as_threads(dev):
    # the largest communicator (kMaxRanks = 16) on the GPU: 16 rank threads of one process (16
    # rank PROCESSES would exceed the box's GPU process limit), one hardware queue per rank's
    # stream so every rank's persistent kernel is resident at once
    port = GW.free_port()
    cases = [dict(dtype="f32", count=(1 << 20) + 5, algo=2, inplace=False, seed=71),   # read
             dict(dtype="f32", count=(1 << 20) + 5, algo=0, inplace=True, seed=72),    # ring
             dict(dtype="bf16", count=4 << 20, algo=-1, inplace=False, seed=73),       # auto, large
             dict(dtype="i32", count=16 * 7 + 3, algo=-1, inplace=False, seed=74),     # auto, tiny
             dict(dtype="f64", count=999, algo=3, inplace=False, seed=75)]             # one-shot
    env = {"MINI_NCCL_TIMEOUT_MS": "60000", "GPU_MAX_HW_QUEUES": "16"}
    out = GW.run_ranks(GW.threaded_ranks_proc, 1, lambda _: (16, port, env, cases), 300)
    assert 0 in out and "error" not in out[0], out
    ranks = out[0]["ranks"]
    assert sorted(ranks) == list(range(16)), ranks
    for r in range(16):
        o = ranks[r]
        assert "error" not in o, o["error"]
        assert o["ranks_on_device"] == 16 and o["destroy"] == 0, o
        for x in o["results"]:
            assert x["rc"] == 0 and x["bad"] == 0, (r, x)
        algos = [x["last_algo"] for x in o["results"]]
        assert algos[0] == 2 and algos[1] == 0 and algos[4] == 3, algos


def _run_procs(cmds, env, timeout):
    import subprocess
    procs = [subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env) for c in cmds]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            o, e = p.communicate()
        outs.append((p.returncode, o, e))
    return outs


@pytest.mark.parametrize("prog", ["app", "app_device", "perf_test", "perf_test_host", "perf_test_8"])
def test_reference_programs_against_this_abi(dev, prog):
    # the reference's own callers (src/main.cpp, tests/perf_test.cpp) rebuilt against
    # include/mini_nccl_api.h + libmini_nccl.so (apps/), one process per rank on GPU 0 as the
    # reference's README runs them: app checks 1.0 + 2.0 == 3.0 on 1 Mi floats (main.cpp:37-61),
    # perf_test the all-ones known answer with its AVX2 scan (perf_test.cpp:81-134)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "apps", "bin", "app" if prog.startswith("app") else "perf_test")
    assert os.path.exists(exe), f"{exe} not built (make -C apps)"
    env = dict(os.environ, MINI_NCCL_PORT=str(GW.free_port()), MINI_NCCL_PERF_DEVICE="0")
    t0 = time.time()
    if prog == "app":
        cmds = [[exe, str(r)] for r in range(2)]  # pinned host buffer, as main.cpp:35
    elif prog == "app_device":
        cmds = [[exe, str(r), "--device-buffer"] for r in range(2)]
    elif prog == "perf_test_host":
        # the reference's own buffers: cudaHostAlloc'd send / recv handed to ncclAllReduce
        cmds = [[exe, str(r), "3", "--mode", "host", "--sizes", "1,16", "--iters", "3", "--warmup", "1"]
                for r in range(3)]
    elif prog == "perf_test_8":
        # `perf_test <r> 8` x 8 on GPU 0 with the default environment (the reference's topology,
        # perf_test.cpp:46): completes within seconds
        env = {k: v for k, v in env.items() if not k.startswith("MINI_NCCL_") or k == "MINI_NCCL_PORT"}
        env["MINI_NCCL_PERF_DEVICE"] = "0"
        cmds = [[exe, str(r), "8", "--sizes", "1,16", "--iters", "3", "--warmup", "1"] for r in range(8)]
    else:
        cmds = [[exe, str(r), "3", "--sizes", "1,16", "--iters", "3", "--warmup", "1"] for r in range(3)]
    outs = _run_procs(cmds, env, 120)
    for rc, o, e in outs:
        assert rc == 0, (rc, o[-2000:], e[-2000:])
    if prog.startswith("app"):
        assert all("Result: [PASS]" in o for _, o, _ in outs)
    else:
        if prog == "perf_test_8":
            assert time.time() - t0 < 60, time.time() - t0
        rows = [ln for ln in outs[0][1].splitlines() if ln.strip() and ln.strip()[0].isdigit()]
        assert len(rows) == 2 and not any("FAIL" in ln for ln in rows), outs[0][1]


def test_bench_self_launch_two_ranks(dev):
    # `python3 bench.py --gpus 2` with no launcher starts its two rank processes
    # itself (here on GPU 0: --same-device) and prints ONE line -- rank 0's -- with n_gpus 2 and
    # every timed schedule's order-sensitive check ok
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(GW.ROOT, "bench.py"), "--gpus", "2", "--same-device", "--no-sweep",
                        "--no-cpu-baseline", "--core-only", "--count", str(16 << 20), "--steps", "5", "--warmup", "2"],
                       capture_output=True, text=True, timeout=280, env=env, cwd=GW.ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert r.returncode == 0 and len(lines) == 1, (r.returncode, r.stdout[-500:], r.stderr[-2000:])
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["result_check"] == "ok", d
    assert {s["verify"]["order_sensitive"] for s in d["schedules"].values()} == {"ok"}, d["schedules"]
