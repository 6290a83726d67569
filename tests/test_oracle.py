"""Pin the CPU oracle (oracle/ring_oracle.c) before anything is checked against it.

* against the reference's own known answers (perf_test.cpp:81-134, main.cpp:37-61),
  stored as fixtures in tests/golden/known_*.npz;
* against the independent numpy restatement's fixtures (tests/golden/make_golden.py);
* against the closed-form fold, written independently in the oracle;
* fp16/bf16 conversions against numpy.
"""
import glob
import os

import numpy as np
import pytest

import oracle_api as O

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


def load_fixture(path):
    z = np.load(path, allow_pickle=False)
    return (list(z["inputs"]), str(z["dtype"]), str(z["op"]), int(z["slice_bytes"]), bool(z["inplace"]),
            list(z["expected"]))


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_oracle_matches_golden_bit_exact(oracle_lib, path):
    xs, dtype, op, sb, inplace, expected = load_fixture(path)
    got = O.allreduce(xs, dtype=dtype, op=op, slice_bytes=sb, inplace=inplace)
    for r, (g, e) in enumerate(zip(got, expected)):
        assert same_bits(g, e), f"rank {r} differs from fixture {os.path.basename(path)}"


def test_golden_set_contains_reference_known_answers():
    names = {os.path.basename(p) for p in GOLDEN}
    assert {"known_allones_n2.npz", "known_allones_n4.npz", "known_allones_n8.npz", "known_app_1plus2.npz"} <= names


@pytest.mark.parametrize("n", [2, 3, 4, 7, 8])
@pytest.mark.parametrize("dtype,op", [("f32", "sum"), ("f32", "max"), ("f64", "prod"), ("i32", "sum"),
                                      ("f16", "sum"), ("bf16", "sum"), ("bf16", "min")])
def test_step_loop_equals_closed_form_fold(oracle_lib, n, dtype, op):
    count = 64 * n + 5  # a tail of count % n elements
    xs = O.random_inputs(n, count, dtype, seed=99)
    outs = O.allreduce(xs, dtype=dtype, op=op, slice_bytes=48)
    fold = O.ring_fold(xs, dtype=dtype, op=op)
    chunk = count // n
    for r in range(n):
        assert same_bits(outs[r][: n * chunk], fold[: n * chunk]), f"rank {r}"
        assert same_bits(outs[r][n * chunk:], xs[r][n * chunk:]), "tail must keep the rank's own input"
    # every rank ends with the same reduced body (the all-gather is a pure copy)
    for r in range(1, n):
        assert same_bits(outs[r][: n * chunk], outs[0][: n * chunk])


def test_slice_size_does_not_change_results(oracle_lib):
    xs = O.random_inputs(5, 5003, "f32", seed=3)
    ref = O.allreduce(xs, slice_bytes=1 << 20)
    for sb in (4, 16, 100, 1024, 0):  # 0 -> 1024 (Config.h:50)
        got = O.allreduce(xs, slice_bytes=sb)
        assert all(same_bits(a, b) for a, b in zip(ref, got)), sb


def test_association_is_ring_order_not_sorted(oracle_lib):
    # (a + b) + c != a + (b + c) in fp32 for these values: the oracle must follow the ring
    xs = [np.array([1e8, 0, 0], np.float32), np.array([1.0, 0, 0], np.float32), np.array([-1e8, 0, 0], np.float32)]
    out = O.allreduce(xs, slice_bytes=4)
    # chunk 0 (count 3, n 3 -> chunk 1): fold starts at rank 0: x2 + (x1 + x0) = -1e8 + (1 + 1e8) = 0
    assert out[0][0] == np.float32(-1e8) + (np.float32(1.0) + np.float32(1e8))


def test_rejects_what_the_reference_rejects(oracle_lib):
    xs = O.random_inputs(2, 16, "f32")
    lib = O.load()
    import ctypes
    sp = (ctypes.c_void_p * 2)(*[x.ctypes.data for x in xs])
    for dtype in (0, 1, 3, 4, 5):  # int8, uint8, uint32, int64, uint64 (api.cpp:101-108)
        assert lib.oracle_allreduce(sp, sp, 2, 16, dtype, 0, 64) == -1
    assert lib.oracle_allreduce(sp, sp, 2, 16, 7, 4, 64) == -1  # ncclAvg (api.cpp:120-127)


def test_half_conversions_match_numpy(oracle_lib):
    g = np.random.default_rng(0)
    f = np.concatenate([g.uniform(-70000, 70000, 20000), g.uniform(-1e-4, 1e-4, 20000),
                        g.standard_normal(20000) * 2.0 ** g.integers(-30, 16, 20000),
                        [0.0, -0.0, np.inf, -np.inf, 65504, 65519.99, 65520, 6.1e-5, 5.96e-8, 2.98e-8, 2.99e-8]]
                       ).astype(np.float32)
    L = O.load()
    h = np.array([L.oracle_f32_to_f16(float(x)) for x in f], np.uint16)
    with np.errstate(over="ignore"):  # values past 65520 round to inf on purpose
        ref = f.astype(np.float16)
    assert np.array_equal(h, ref.view(np.uint16))
    back = np.array([L.oracle_f16_to_f32(int(x)) for x in h[:5000]], np.float32)
    assert np.array_equal(back, h[:5000].view(np.float16).astype(np.float32))
    b = np.array([L.oracle_f32_to_bf16(float(x)) for x in f[:5000]], np.uint16)
    assert np.array_equal(b, O.bf16_from_f32(f[:5000]))


def test_verify_scan_finds_first_mismatch(oracle_lib):
    x = np.full(1001, 4.0, np.float32)
    L = O.load()
    assert L.oracle_verify_avx2(x.ctypes.data, x.size, 4.0) == -1
    x[517] = 3.0
    assert L.oracle_verify_avx2(x.ctypes.data, x.size, 4.0) == 517
    x[517] = 4.0
    x[1000] = 0.0  # scalar tail (perf_test.cpp:128-134)
    assert L.oracle_verify_avx2(x.ctypes.data, x.size, 4.0) == 1000


@pytest.mark.parametrize("dtype", ["f32", "f16", "bf16", "i32"])
@pytest.mark.parametrize("count", [8 * 4099, 8 * 4099 + 5])
def test_ring_fold_parallel_matches_ring_fold(dtype, count):
    # the threaded closed-form fold the full-size GPU tests compare against gives ring_fold's bits
    xs = O.random_inputs(8, count, dtype, seed=77)
    a = O.ring_fold(xs, dtype, "sum")
    b = O.ring_fold_parallel(xs, dtype, "sum", piece=1000)
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
