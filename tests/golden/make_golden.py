"""Generate the committed golden fixtures (tests/golden/*.npz).

An INDEPENDENT numpy restatement of the reference ring (XuDongGong/Mini-NCCL
src/mini_nccl.cu:56-217 with api.cpp:173-178), written step by step with whole-chunk
numpy ops -- no shared code with oracle/ring_oracle.c -- so that the C oracle can be
checked against it.  The reference itself cannot run here (needs CUDA + libibverbs,
SURVEY.md s8c); its own known-answer cases (perf_test.cpp:81-134: all-ones -> nRanks;
main.cpp:37-61: 1.0 + 2.0 -> 3.0) are included as fixtures too.

Each fixture stores: inputs (n x count), dtype, op, slice_bytes, inplace flag and the
expected outputs (n x count).  bf16 is stored as raw uint16 bits.
Run:  python tests/golden/make_golden.py   (deterministic; rewrites the .npz files)
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def bf16_round(f32):
    u = f32.astype(np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_f32(h):
    return (h.astype(np.uint32) << 16).view(np.float32)


def op_apply(op, a, b, dtype):
    """c = op(a = local, b = incoming), reference mini_nccl.cu:38-41"""
    if dtype == "bf16":
        fa, fb = bf16_f32(a), bf16_f32(b)
        if op == "max":
            return np.where(fa > fb, a, b)
        if op == "min":
            return np.where(fa < fb, a, b)
        return bf16_round(fa + fb if op == "sum" else fa * fb)
    if op == "sum":
        with np.errstate(over="ignore", invalid="ignore"):
            return (a + b).astype(a.dtype)
    if op == "prod":
        with np.errstate(over="ignore", invalid="ignore", under="ignore"):
            return (a * b).astype(a.dtype)
    if op == "max":
        return np.where(a > b, a, b)
    return np.where(a < b, a, b)


def ring(inputs, op, dtype, slice_bytes, inplace):
    n = len(inputs)
    bufs = [x.copy() for x in inputs]  # recv after the send->recv copy (api.cpp:173-175)
    if n == 1:
        return bufs
    count = inputs[0].size
    chunk = count // n                               # mini_nccl.cu:69
    # slicing does not change element-wise results; it is kept to mirror :112-117
    esz = inputs[0].itemsize
    slice_elems = max(1, slice_bytes // esz)
    for i in range(n - 1):                           # :108
        for s0 in range(0, chunk, slice_elems):
            s1 = min(chunk, s0 + slice_elems)
            wire = []
            for r in range(n):
                send_idx = (r - i) % n               # :109
                wire.append(bufs[r][send_idx * chunk + s0: send_idx * chunk + s1].copy())
            for r in range(n):
                recv_idx = (r - i - 1) % n           # :110
                t = slice(recv_idx * chunk + s0, recv_idx * chunk + s1)
                bufs[r][t] = op_apply(op, bufs[r][t], wire[(r - 1) % n], dtype)  # :126
    for i in range(n - 1):                           # :159
        for s0 in range(0, chunk, slice_elems):
            s1 = min(chunk, s0 + slice_elems)
            wire = []
            for r in range(n):
                send_idx = (r - i + 1) % n           # :160
                wire.append((send_idx, bufs[r][send_idx * chunk + s0: send_idx * chunk + s1].copy()))
            for r in range(n):
                blk, data = wire[(r - 1) % n]        # peer writes at its own send offset (:172)
                bufs[r][blk * chunk + s0: blk * chunk + s1] = data
    return bufs


NPD = {"f32": np.float32, "f64": np.float64, "i32": np.int32, "f16": np.float16, "bf16": np.uint16}


def make_inputs(n, count, dtype, seed, special=False):
    outs = []
    for r in range(n):
        g = np.random.default_rng(seed + r)
        if dtype == "i32":
            x = g.integers(-(2 ** 31), 2 ** 31 - 1, size=count, dtype=np.int64).astype(np.int32)
        elif dtype == "bf16":
            x = bf16_round(g.uniform(-1, 1, size=count).astype(np.float32))
        else:
            x = g.uniform(-1, 1, size=count).astype(NPD[dtype])
            if special and dtype in ("f32", "f64"):
                # signed zeros, infinities, denormals, NaN (max/min are pure selections:
                # bit-exact even for NaN payloads and -0/+0)
                k = g.choice(count, size=min(count, 48), replace=False)
                vals = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3e-45], dtype=NPD[dtype])
                x[k] = vals[np.arange(k.size) % vals.size]
        outs.append(x)
    return outs


CASES = [
    # name, n, count, dtype, op, slice_bytes, inplace, special
    ("f32_sum_n2", 2, 1003, "f32", "sum", 64, False, False),
    ("f32_sum_n3", 3, 1000, "f32", "sum", 128, True, False),
    ("f32_sum_n4", 4, 4099, "f32", "sum", 256, False, False),
    ("f32_sum_n8", 8, 8191, "f32", "sum", 512, False, False),
    ("f32_sum_n8_denorm", 8, 2048, "f32", "sum", 64, True, True),
    ("f32_max_n4_special", 4, 2050, "f32", "max", 128, False, True),
    ("f32_min_n5_special", 5, 2003, "f32", "min", 96, False, True),
    ("f32_prod_n3", 3, 1500, "f32", "prod", 64, False, False),
    ("f64_sum_n4", 4, 1026, "f64", "sum", 128, False, False),
    ("f64_prod_n8", 8, 1024, "f64", "prod", 64, True, False),
    ("f64_max_n3_special", 3, 999, "f64", "max", 64, False, True),
    ("i32_sum_n4_wrap", 4, 1029, "i32", "sum", 64, False, False),
    ("i32_prod_n3_wrap", 3, 1200, "i32", "prod", 32, False, False),
    ("i32_min_n8", 8, 1031, "i32", "min", 128, True, False),
    ("f16_sum_n4", 4, 2049, "f16", "sum", 64, False, False),
    ("f16_prod_n2", 2, 1002, "f16", "prod", 64, False, False),
    ("bf16_sum_n8", 8, 4100, "bf16", "sum", 256, False, False),
    ("bf16_max_n4", 4, 1002, "bf16", "max", 64, True, False),
    ("f32_sum_n1", 1, 777, "f32", "sum", 64, False, False),
    ("f32_sum_small_count", 4, 3, "f32", "sum", 64, False, False),  # count < n: chunk == 0
]


def known_answer_cases():
    """The reference's own assertions, as fixtures."""
    out = []
    # perf_test.cpp:81-134 -- all ranks send 1.0, every element must equal nRanks
    for n, count in ((2, 262144), (4, 65536), (8, 32768)):
        xs = [np.ones(count, np.float32) for _ in range(n)]
        out.append((f"known_allones_n{n}", xs, "f32", "sum", 131072, False,
                    [np.full(count, float(n), np.float32) for _ in range(n)]))
    # main.cpp:37-61 -- 2 ranks, 1 Mi floats in place, rank0 = 1.0, rank1 = 2.0 -> 3.0
    count = 1 << 20
    xs = [np.full(count, 1.0, np.float32), np.full(count, 2.0, np.float32)]
    out.append(("known_app_1plus2", xs, "f32", "sum", 131072, True, [np.full(count, 3.0, np.float32)] * 2))
    return out


def save(name, inputs, dtype, op, slice_bytes, inplace, expected):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), inputs=np.stack(inputs), expected=np.stack(expected),
                        dtype=np.array(dtype), op=np.array(op), slice_bytes=np.array(slice_bytes),
                        inplace=np.array(inplace))


def main():
    for name, n, count, dtype, op, sb, inplace, special in CASES:
        xs = make_inputs(n, count, dtype, seed=1234, special=special)
        save(name, xs, dtype, op, sb, inplace, ring(xs, op, dtype, sb, inplace))
    for name, xs, dtype, op, sb, inplace, expected in known_answer_cases():
        # the known answers are stated by the reference; check the restatement reproduces them
        got = ring(xs, op, dtype, sb, inplace)
        assert all(np.array_equal(g, e) for g, e in zip(got, expected)), name
        save(name, xs, dtype, op, sb, inplace, expected)
    print("wrote", len(CASES) + len(known_answer_cases()), "fixtures to", HERE)


if __name__ == "__main__":
    main()
