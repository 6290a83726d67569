"""The GPU kernels' protocol, executed on the CPU (mini-nccl_amd/csrc/sim.cpp).

sim.cpp runs, per simulated (rank, channel), the op sequence kernels.hip runs, with the
same csrc/schedule.h index math and the same scratch/mailbox layouts; a wait that is not
satisfied yields.  These tests check the result against the oracle (bit-exact), that
the protocol never deadlocks (for every slot depth >= 1, channel count and size tried,
including pseudo-random interleavings), and that sequence numbers carried across calls
stay consistent.
"""
import numpy as np
import pytest

import oracle_api as O
import sim_api as S

OPS = ["sum", "prod", "max", "min"]


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


@pytest.mark.parametrize("algo", [S.RING, S.READ, S.READ_GRID], ids=["ring", "read", "read_grid"])
@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("count,slice_bytes,channels,slots", [
    (4096, 256, 4, 2),      # several slices per channel
    (4099, 64, 3, 2),       # odd count (tail)
    (1000, 1024, 8, 2),     # fewer slices than channels (padding messages)
    (10007, 128, 5, 4),     # deep FIFO
    (7, 64, 2, 2),          # chunk of 0 or 1 element
])
def test_sim_matches_oracle(oracle_lib, sim_lib, algo, n, count, slice_bytes, channels, slots):
    xs = O.random_inputs(n, count, "f32", seed=7)
    ref = O.allreduce(xs, "f32", "sum", slice_bytes=slice_bytes)
    got, steps = S.allreduce(xs, algo=algo, op=0, slice_bytes=slice_bytes, channels=channels, slots=slots)
    for r in range(n):
        assert same_bits(got[r], ref[r]), f"rank {r}"


@pytest.mark.parametrize("algo", [S.RING, S.READ, S.READ_GRID], ids=["ring", "read", "read_grid"])
@pytest.mark.parametrize("op", OPS)
def test_sim_all_ops(oracle_lib, sim_lib, algo, op):
    xs = O.random_inputs(4, 2050, "f32", seed=11)
    ref = O.allreduce(xs, "f32", op, slice_bytes=96)
    got, _ = S.allreduce(xs, algo=algo, op=O.OPS[op], slice_bytes=96, channels=3, slots=2)
    assert all(same_bits(g, e) for g, e in zip(got, ref))


@pytest.mark.parametrize("algo", [S.RING, S.READ, S.READ_GRID], ids=["ring", "read", "read_grid"])
@pytest.mark.parametrize("seed", range(1, 13))
def test_sim_random_interleavings_no_deadlock(oracle_lib, sim_lib, algo, seed):
    n = 2 + seed % 7
    xs = O.random_inputs(n, 3000 + seed, "f32", seed=seed)
    ref = O.allreduce(xs, slice_bytes=64)
    got, _ = S.allreduce(xs, algo=algo, slice_bytes=64, channels=1 + seed % 4, slots=2 + seed % 3, calls=3,
                         seed=seed)
    assert all(same_bits(g, e) for g, e in zip(got, ref))


@pytest.mark.parametrize("algo", [S.RING, S.READ, S.READ_GRID], ids=["ring", "read", "read_grid"])
def test_sim_sequence_continues_across_calls(oracle_lib, sim_lib, algo):
    # 5 calls on one communicator state: flags are monotone and never reset
    xs = O.random_inputs(4, 5000, "f32", seed=5)
    ref = O.allreduce(xs, slice_bytes=128)
    got, steps5 = S.allreduce(xs, algo=algo, slice_bytes=128, channels=3, slots=2, calls=5)
    _, steps1 = S.allreduce(xs, algo=algo, slice_bytes=128, channels=3, slots=2, calls=1)
    assert steps5 == 5 * steps1
    assert all(same_bits(g, e) for g, e in zip(got, ref))


def test_ring_message_counts(sim_lib):
    # per pipeline iteration: 2n-1 ops for the ring (1 send + (n-1) SR + (n-1) AG receives); a
    # call runs only the pipelines its slices need (schedule.h call_pipelines): 1 slice -> 1
    n, C = 4, 2
    xs = O.random_inputs(n, n * 16, "f32")
    _, steps = S.allreduce(xs, algo=S.RING, slice_bytes=64, channels=C, slots=2)
    assert steps == n * 1 * 1 * (2 * n - 1)  # nslices = 1: one pipeline, one iteration
    xs = O.random_inputs(n, n * 16 * 5, "f32")  # 5 slices over 2 pipelines: 3 iterations
    _, steps = S.allreduce(xs, algo=S.RING, slice_bytes=64, channels=C, slots=2)
    assert steps == n * C * 3 * (2 * n - 1)


def test_single_slot_fifo_deadlocks(sim_lib):
    # why Config clamps MINI_NCCL_SLOTS to >= 2: with one slot per pipeline, op k of every
    # rank waits for the credit its neighbour only returns inside ITS op k -- a cycle
    xs = O.random_inputs(2, 4096, "f32")
    with pytest.raises(RuntimeError, match="deadlock"):
        S.allreduce(xs, algo=S.RING, slice_bytes=256, channels=2, slots=1)


@pytest.mark.parametrize("algos", [[0, 2, 0, 2], [4, 4, 0, 0, 2], [0, 0, 4], [2, 0, 2, 4, 2], [4, 2, 2, 0]])
@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_sim_switching_schedules_on_one_communicator(oracle_lib, sim_lib, algos, n):
    # mncclCommSetAlgo between calls: per-pair FIFO counters keep every link consistent
    # (a single per-channel counter would leave non-neighbour credits behind and hang)
    xs = O.random_inputs(n, 3001, "f32", seed=n)
    ref = O.allreduce(xs, slice_bytes=64)
    got, _ = S.allreduce(xs, slice_bytes=64, channels=3, slots=2, algos=algos, seed=n)
    assert all(same_bits(g, e) for g, e in zip(got, ref))


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("count", [7, 1000, 4099, 70001])
@pytest.mark.parametrize("inplace", [False, True], ids=["out", "inplace"])
def test_sim_oneshot(oracle_lib, sim_lib, n, count, inplace):
    # the one-shot schedule (kernels.hip oneshot_kernel): every rank folds all n chunks from the
    # peers' messages in ring order -- the reference ring's bits on every rank, 3 calls on one
    # communicator state (slots and credits reused), random interleavings
    xs = O.random_inputs(n, count, "f32", seed=count + n)
    ref = O.allreduce(xs, slice_bytes=1024)
    if inplace:  # every call after the first reduces the previous result
        ref = O.allreduce(ref, slice_bytes=1024)
        ref = O.allreduce(ref, slice_bytes=1024)
    got, _ = S.allreduce(xs, algo=S.ONESHOT, slice_bytes=16384, min_slice=1024, channels=64, slots=2, calls=3,
                         seed=count, inplace=inplace)
    assert all(same_bits(g, e) for g, e in zip(got, ref))


@pytest.mark.parametrize("algos", [[1, 0, 1, 2], [4, 1, 1, 0, 2], [0, 0, 1], [2, 1, 2, 4, 1], [1, 2, 2, 0, 1, 1]])
@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_sim_oneshot_switching_schedules(oracle_lib, sim_lib, algos, n):
    # the one-shot shares the per-(pair, pipeline) FIFO counters, READY words, credits and slots
    # with the ring and the read schedule: any order of calls keeps every link consistent
    xs = O.random_inputs(n, 9001, "f32", seed=3 * n)
    ref = O.allreduce(xs, slice_bytes=1024)
    for seed in (0, 5, 11):
        got, _ = S.allreduce(xs, slice_bytes=16384, min_slice=1024, channels=64, slots=2, algos=algos, seed=seed)
        assert all(same_bits(g, e) for g, e in zip(got, ref)), seed


@pytest.mark.parametrize("n", [2, 3, 5, 8, 16])
@pytest.mark.parametrize("chunk", [4, 1000, 4096, 8192, 1 << 15, 100000, 1 << 20, 1 << 24])
def test_oneshot_geometry(sim_lib, n, chunk):
    # schedule.h oneshot_slice / oneshot_fits: a pipeline per slice of every chunk, one round of
    # the pipelines covers the call, a piece fits a slot, whole 1 KiB waves; auto takes it only up
    # to 64 KiB per call
    C, slot = 256, 128 << 10
    sl = S.oneshot_slice(chunk, n, C, slot)
    forced, auto = S.oneshot_fits(chunk, n, C, slot, True), S.oneshot_fits(chunk, n, C, slot, False)
    assert sl % 1024 == 0 and 1024 <= sl <= slot
    if forced:
        assert -(-chunk // sl) * n <= C
    assert auto == (forced and chunk * n <= 64 << 10)
    if chunk * n <= 64 << 10 and n <= 16:
        assert auto  # every call the auto path meant for one-shot fits the default geometry
    assert not S.oneshot_fits(chunk, 1, C, slot, True)


@pytest.mark.parametrize("chunk", [0, 4, 1000, 1 << 16, (1 << 20) + 12, 3 << 22, 1 << 27, 1 << 30])
@pytest.mark.parametrize("C", [1, 7, 256])
def test_effective_slice_properties(sim_lib, chunk, C):
    # adaptive payload (csrc/schedule.h): never above the configured slice, never below the
    # floor, whole 1 KiB waves of vectors, and every pipeline busy when it shrinks
    slice_bytes, floor = 128 * 1024, 1024
    e = S.effective_slice(chunk, C, slice_bytes, floor)
    assert floor <= e <= slice_bytes
    assert e == slice_bytes or e % 1024 == 0
    nslices = -(-chunk // e)
    if e < slice_bytes and e > floor:
        assert nslices <= C and -(-chunk // (e - 1024)) > C  # the smallest payload with <= C slices
    if chunk >= C * slice_bytes:
        assert e == slice_bytes
    assert S.effective_slice(chunk, C, slice_bytes, slice_bytes) == slice_bytes  # MIN_SLICE >= SLICE: off


@pytest.mark.parametrize("algo", [S.RING, S.READ, S.READ_GRID], ids=["ring", "read", "read_grid"])
@pytest.mark.parametrize("n,count,seed", [(2, 70001, 1), (3, 40000, 2), (4, 9000, 3), (8, 123457, 4)])
def test_sim_adaptive_slice(oracle_lib, sim_lib, algo, n, count, seed):
    # payload shrunk below the slot stride, random interleavings over 3 calls: same bits
    xs = O.random_inputs(n, count, "f32", seed=seed)
    ref = O.allreduce(xs, slice_bytes=1024)
    got, _ = S.allreduce(xs, algo=algo, slice_bytes=16384, min_slice=1024, channels=5, slots=2, calls=3, seed=seed)
    assert all(same_bits(g, e) for g, e in zip(got, ref))


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("seed", range(1, 9))
def test_sim_ring_partial_grid_random_interleavings(oracle_lib, sim_lib, n, seed):
    # the ring runs only the pipelines a call's slices need (schedule.h call_pipelines; the
    # reference moves only the slices that exist, mini_nccl.cu:112-115): calls of 1 .. C slices
    # interleaved with full-grid calls and read calls on one communicator state, random
    # interleavings -- the idle pipelines' per-pair counters stay in step on every rank
    C = 8
    sizes = [n * 16, n * 16 * 3 + 1, n * 16 * C * 2 + 5, n * 16 * 5 + 3, 7, n * 16 * C + 16]
    for i, count in enumerate(sizes):
        xs = O.random_inputs(n, count, "f32", seed=100 * seed + i)
        ref = O.allreduce(xs, slice_bytes=64)
        algos = [S.RING, S.RING, S.READ if i % 2 else S.READ_GRID, S.RING]
        got, _ = S.allreduce(xs, slice_bytes=64, channels=C, slots=2, algos=algos, seed=seed + i)
        assert all(same_bits(g, e) for g, e in zip(got, ref)), (count, algos)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_ring_small_calls_run_only_the_pipelines_they_need(oracle_lib, sim_lib, n):
    # a 3-slice ring call on 8 pipelines executes 3 pipelines' ops, not 8
    C, count = 8, n * 48
    xs = O.random_inputs(n, count, "f32", seed=60 + n)
    got, steps = S.allreduce(xs, algo=S.RING, slice_bytes=64, channels=C)
    assert steps == n * 3 * (2 * n - 1)
    assert all(same_bits(g, e) for g, e in zip(got, O.allreduce(xs, slice_bytes=64)))


@pytest.mark.parametrize("nslices,C,waves,want", [(0, 256, 1, 1), (1, 256, 1, 1), (3, 8, 1, 3), (255, 256, 1, 255),
                                                  (256, 256, 1, 256), (10**6, 256, 1, 256), (3, 64, 4, 4),
                                                  (5, 64, 4, 8), (70, 64, 4, 64)])
def test_call_pipelines(sim_lib, nslices, C, waves, want):
    # one pipeline per slice up to all C, whole workgroups of `waves` pipelines
    assert S.call_pipelines(nslices, C, waves) == want


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("seed", range(1, 7))
def test_sim_read_in_place_random_interleavings(oracle_lib, sim_lib, n, seed):
    # the read schedule in place (send == recv): only rank c writes chunk c of any recv, after its
    # own loads of that slice; under random interleavings any other order would leave a wrong
    # value behind
    xs = O.random_inputs(n, 3000 + 7 * seed, "f32", seed=seed)
    ref = O.allreduce(xs, slice_bytes=64)
    for algo in (S.READ, S.READ_GRID):
        got, _ = S.allreduce(xs, algo=algo, slice_bytes=64, channels=1 + seed % 4, calls=1, seed=seed, inplace=True)
        assert all(same_bits(g, e) for g, e in zip(got, ref)), algo


def test_sim_read_needs_no_slots(oracle_lib, sim_lib):
    # no scratch FIFO: even one slot (which deadlocks the ring) is irrelevant
    xs = O.random_inputs(3, 4096, "f32", seed=3)
    got, _ = S.allreduce(xs, algo=S.READ, slice_bytes=256, channels=2, slots=1)
    assert all(same_bits(g, e) for g, e in zip(got, O.allreduce(xs, slice_bytes=256)))


def test_read_message_counts(sim_lib):
    # per pipeline and call: START (publish + wait), one fold-and-push per iteration (no READY,
    # no copies), DONE (publish + wait); the 4.0-5.x load form (schedule code 3) is refused
    n, C = 4, 2
    xs = O.random_inputs(n, n * 64, "f32")
    _, steps = S.allreduce(xs, algo=S.READ, slice_bytes=64, channels=C)
    iters = -(-(64 * 4 // 64) // C)
    assert steps == n * C * (4 + iters)
    with pytest.raises(ValueError):
        S.allreduce(xs, algo=3, slice_bytes=64, channels=C)


@pytest.mark.parametrize("chunk", [0, 4, 1000, 1 << 16, (1 << 20) + 12, 3 << 22, 1 << 27, 1 << 30])
@pytest.mark.parametrize("C", [1, 7, 256])
def test_read_slice_properties(sim_lib, chunk, C):
    # the read schedule's payload (csrc/schedule.h read_slice): never above the configured slice;
    # >= 16 iterations per pipeline while slices stay >= 16 KiB; otherwise 16 KiB or the
    # one-slice-per-pipeline payload of small calls, whichever is smaller
    sl, floor = 128 * 1024, 1024
    e = S.read_slice(chunk, C, sl, floor)
    assert floor <= e <= sl and (e == sl or e % 1024 == 0)
    per_pipe = -(-chunk // C)
    if per_pipe >= 16 * 16384:
        assert -(-per_pipe // e) >= 16 or e == sl and -(-per_pipe // e) >= 1
    if e < 16384:
        assert e == S.effective_slice(chunk, C, sl, floor)


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_read_small_calls_run_only_the_pipelines_they_need(oracle_lib, sim_lib, n):
    # schedule.h call_pipelines: a read call with fewer slices than pipelines runs one pipeline per
    # slice; the rest sit it out on every rank, so their per-pair counters stay in step through
    # later calls of either schedule
    C, count = 8, n * 48  # 192 B chunks of 64 B slices: 3 slices, 3 of the 8 pipelines
    xs = O.random_inputs(n, count, "f32", seed=40 + n)
    ref = O.allreduce(xs, slice_bytes=64)
    _, steps = S.allreduce(xs, algo=2, slice_bytes=64, channels=C)
    assert steps == n * 3 * (4 + 1)  # iters = 1 on 3 pipelines
    for seed in range(3):
        got, _ = S.allreduce(xs, slice_bytes=64, channels=C, algos=[2, 0, 2, 4, 2, 2, 0, 4, 2], seed=seed + 1)
        assert all(same_bits(g, e) for g, e in zip(got, ref))


def _topo(n, kind=S.XGMI, hops=1, devices=None):
    """n x n link / hop matrices: every pair over `kind` at `hops`, or, with `devices`, ranks on the
    same device index reach each other through that GPU (SAME_GPU, 0 hops)"""
    link = [[S.SAME_GPU if p == q or (devices and devices[p] == devices[q]) else kind for p in range(n)]
            for q in range(n)]
    hop = [[0 if link[q][p] == S.SAME_GPU else hops for p in range(n)] for q in range(n)]
    return link, hop


def test_topology_rule_for_the_default_schedule(sim_lib):
    # auto runs the read schedule only when every pair of ranks shares a GPU or is
    # one xGMI hop apart (an MI355X node's full mesh; the co-located rehearsal), otherwise the
    # ring -- decided from every rank's row, so every rank decides alike
    assert S.topology_blocks_read(*_topo(8)) is None                               # the 8-GPU node
    assert S.topology_blocks_read(*_topo(8, devices=[0] * 8)) is None              # 8 ranks, one GPU
    assert S.topology_blocks_read(*_topo(4, devices=[0, 0, 1, 1])) is None         # 2 GPUs x 2 ranks
    assert S.topology_blocks_read(*_topo(2, kind=S.PCIE)) == (0, 1)                # PCIe box
    link, hops = _topo(8)
    link[5][3] = S.PCIE                      # one peer of one rank over PCIe: the whole communicator
    assert S.topology_blocks_read(link, hops) == (5, 3)
    link, hops = _topo(8)
    hops[2][6] = 2                           # xGMI but routed through another GPU
    assert S.topology_blocks_read(link, hops) == (2, 6)
    link, hops = _topo(3)
    link[1][0] = S.UNKNOWN                   # a peer GPU that rank 1's process cannot see
    assert S.topology_blocks_read(link, hops) == (1, 0)
    # the diagonal (a rank and itself) never counts
    link, hops = _topo(3, kind=S.PCIE, devices=[0, 0, 0])
    assert S.topology_blocks_read(link, hops) is None



@pytest.mark.parametrize("n", [2, 3, 8])
def test_sim_registered_window_signatures_random_interleavings(sim_lib, n):
    # a registered-window read call is launched with no host rendezvous; each
    # rank's START carries the call's signature and every pipeline compares its peers' with its
    # own before touching any buffer.  Under random interleavings: equal signatures -> the
    # oracle's bits; any rank differing -> every pipeline of every rank gives up and no recv
    # element is written (the call fails with ncclInvalidUsage instead of reading a wrong buffer)
    import oracle_api as O
    count = n * 2500 + 3
    xs = O.random_inputs(n, count, "f32", seed=77)
    exp = O.allreduce(xs, "f32", "sum")
    for seed in range(1, 13):
        out, mm = S.signed_read(xs, [0x5eed] * n, seed=seed)
        assert mm == [0] * n
        body = (count // n) * n
        for r in range(n):
            assert np.array_equal(out[r][:body].view(np.uint32), exp[r][:body].view(np.uint32)), (seed, r)
        for bad_rank in {0, n - 1, seed % n}:
            sigs = [0x5eed] * n
            sigs[bad_rank] = 0x5eed + 2 * seed  # another window / offset / count on one rank
            out, mm = S.signed_read(xs, sigs, seed=seed)
            assert all(m > 0 for m in mm), (seed, bad_rank, mm)
            assert len(set(mm)) == 1, mm  # every pipeline of every rank, alike
            assert all(np.isnan(o).all() for o in out), (seed, bad_rank)  # nothing written



def test_read_grid_form_rule(sim_lib):
    # forced (mncclAlgoReadGrid) or auto: calls with chunks of >= 4 MiB in whole 16-byte vectors
    # at 2-8 ranks take the grid form; unaligned calls, smaller chunks, more ranks and a forced
    # persistent read (mncclAlgoRead) keep the persistent kernel
    big = 4 << 20
    for n in (2, 3, 5, 8):
        assert S.read_grid_form(True, False, True, big, n)
        assert S.read_grid_form(False, True, True, big, n)
        assert not S.read_grid_form(False, False, True, big, n)  # MINI_NCCL_ALGO=read
        assert not S.read_grid_form(False, True, False, big, n)  # element-wise path
        assert not S.read_grid_form(False, True, True, big - 16, n)
        assert not S.read_grid_form(False, True, True, big + 8, n)
    assert not S.read_grid_form(True, True, True, big, 9)
    assert not S.read_grid_form(True, True, True, big, 1)
    # MINI_NCCL_GRID_MIN moves the threshold (the node's sweep weighs DDP-bucket-sized calls)
    assert S.read_grid_form(False, True, True, 256 << 10, 8, min_bytes=256 << 10)
    assert not S.read_grid_form(False, True, True, (256 << 10) - 16, 8, min_bytes=256 << 10)



@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_sim_grid_form_between_other_schedules(oracle_lib, sim_lib, n):
    # the grid form's protocol (START / DONE on pipeline 0 only, the whole chunk folded and pushed
    # between them) interleaved with every other schedule on one communicator state, under random
    # interleavings: every call bit-exact vs the oracle, no deadlock (the other pipelines' counters
    # stay in step because every rank skips them alike)
    import oracle_api as O
    plans = [[S.READ_GRID, S.RING, S.READ_GRID, S.READ, S.ONESHOT, S.READ_GRID],
             [S.READ, S.READ_GRID, S.RING, S.READ_GRID, S.READ, S.READ]]
    for i, algos in enumerate(plans):
        count = n * 700 + i
        xs = O.random_inputs(n, count, "f32", seed=60 + i)
        ref = O.allreduce(xs, "f32", "sum")
        for seed in range(1, 6):
            got, _ = S.allreduce(xs, slice_bytes=16384, min_slice=1024, channels=64, slots=2, algos=algos, seed=seed)
            body = (count // n) * n
            for r in range(n):
                assert np.array_equal(got[r][:body].view(np.uint32), ref[r][:body].view(np.uint32)), (algos, seed, r)


@pytest.mark.parametrize("P,waves,cus,most,want", [
    (256, 1, 256, 1, 256), (256, 1, 256, 8, 256),     # the default geometry: 8 co-located ranks fill 2048 slots exactly
    (512, 1, 256, 8, 256), (512, 1, 256, 1, 512),     # MINI_NCCL_CHANNELS=512: capped only when ranks share a GPU
    (4096, 4, 256, 1, 2048), (1024, 4, 256, 3, 680),  # 4-wave workgroups: whole workgroups
    (256, 1, 256, 16, 128), (8, 4, 1, 16, 4)])        # never below one workgroup
def test_resident_pipes(sim_lib, P, waves, cus, most, want):
    # csrc/schedule.h resident_pipes: the waves one call launches on the most crowded GPU all fit
    # its cus x 4 SIMDs x 2 slots (every rank's pipeline w waits for its peers' pipeline w)
    got = S.resident_pipes(P, waves, cus, most)
    assert got == want
    assert got % waves == 0 and got <= P
    assert got * most <= max(cus * 4 * 2, waves * most)
