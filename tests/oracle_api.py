"""ctypes + numpy front end of oracle/_build/liboracle.so (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module;
the product never imports it.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")

# dtype name -> (ncclDataType_t, numpy storage dtype)
DTYPES = {
    "f32": (7, np.float32),
    "f64": (8, np.float64),
    "i32": (2, np.int32),
    "f16": (6, np.float16),
    "bf16": (9, np.uint16),  # raw bf16 bits
}
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3}

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise OSError(f"{LIB} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.oracle_elem_size.argtypes = [i]
        L.oracle_reduce.argtypes = [vp, vp, vp, sz, i, i]
        L.oracle_allreduce.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), i, sz, i, i, sz]
        L.oracle_ring_fold.argtypes = [ctypes.POINTER(vp), vp, i, sz, i, i]
        L.oracle_f32_to_f16.argtypes = [ctypes.c_float]
        L.oracle_f32_to_f16.restype = ctypes.c_uint16
        L.oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
        L.oracle_f16_to_f32.restype = ctypes.c_float
        L.oracle_f32_to_bf16.argtypes = [ctypes.c_float]
        L.oracle_f32_to_bf16.restype = ctypes.c_uint16
        L.oracle_bf16_to_f32.argtypes = [ctypes.c_uint16]
        L.oracle_bf16_to_f32.restype = ctypes.c_float
        L.oracle_cpu_local_reduce_avx2.argtypes = [vp, vp, sz, i, i]
        L.oracle_cpu_local_reduce_avx2.restype = ctypes.c_double
        L.oracle_verify_avx2.argtypes = [vp, sz, ctypes.c_float]
        L.oracle_verify_avx2.restype = ctypes.c_long
        L.oracle_cpu_ring_threads_avx2.argtypes = [ctypes.POINTER(vp), i, sz, sz, i]
        L.oracle_cpu_ring_threads_avx2.restype = ctypes.c_double
        L.oracle_cpu_ring_tcp.argtypes = [i, i, ctypes.c_char_p, i, vp, sz, sz, i, ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def allreduce(inputs, dtype="f32", op="sum", slice_bytes=128 * 1024, inplace=False):
    """Reference ring all-reduce (mini_nccl.cu:56-217) on len(inputs) ranks; returns outputs."""
    code, npd = DTYPES[dtype]
    n = len(inputs)
    count = inputs[0].size
    sends = [np.ascontiguousarray(x, dtype=npd) for x in inputs]
    if inplace:
        recvs = [x.copy() for x in sends]
        sp = rp = (ctypes.c_void_p * n)(*[r.ctypes.data for r in recvs])
    else:
        recvs = [np.empty_like(x) for x in sends]
        sp = (ctypes.c_void_p * n)(*[s.ctypes.data for s in sends])
        rp = (ctypes.c_void_p * n)(*[r.ctypes.data for r in recvs])
    rc = load().oracle_allreduce(sp, rp, n, count, code, OPS[op], slice_bytes)
    if rc != 0:
        raise ValueError(f"oracle rejected dtype={dtype} op={op} (rc={rc})")
    return recvs


def ring_fold(inputs, dtype="f32", op="sum"):
    """Closed-form fold (chunk c = x[c-1] op (... op (x[c+1] op x[c])))."""
    code, npd = DTYPES[dtype]
    n = len(inputs)
    ins = [np.ascontiguousarray(x, dtype=npd) for x in inputs]
    out = np.empty_like(ins[0])
    ip = (ctypes.c_void_p * n)(*[x.ctypes.data for x in ins])
    rc = load().oracle_ring_fold(ip, _ptr(out), n, out.size, code, OPS[op])
    if rc != 0:
        raise ValueError("oracle_ring_fold rejected arguments")
    return out


def ring_fold_parallel(inputs, dtype="f32", op="sum", threads=8, piece=1 << 22):
    """ring_fold for full-size buffers: the same closed form (chunk c starts from x[c], then
    acc = op(x[q], acc) for q = c+1, ..., c-1, mini_nccl.cu:108-194), each chunk cut into pieces
    folded by oracle_reduce on a thread pool (ctypes releases the GIL; element-wise work, so the
    bits are ring_fold's).  The count % n tail is rank 0's input, as in ring_fold."""
    from concurrent.futures import ThreadPoolExecutor
    code, npd = DTYPES[dtype]
    n = len(inputs)
    ins = [np.ascontiguousarray(x, dtype=npd) for x in inputs]
    count = ins[0].size
    chunk = count // n
    out = np.empty_like(ins[0])
    out[n * chunk:] = ins[0][n * chunk:]
    L = load()

    def job(c, a, b):
        lo, hi = c * chunk + a, c * chunk + b
        acc = out[lo:hi]
        acc[:] = ins[c][lo:hi]
        for k in range(1, n):
            src = ins[(c + k) % n][lo:hi]
            if L.oracle_reduce(_ptr(acc), _ptr(src), _ptr(acc), hi - lo, code, OPS[op]) != 0:
                raise ValueError("oracle_reduce rejected arguments")

    with ThreadPoolExecutor(threads) as ex:
        futs = [ex.submit(job, c, a, min(chunk, a + piece)) for c in range(n) for a in range(0, chunk, piece)]
        for f in futs:
            f.result()
    return out


def reduce(a, b, dtype="f32", op="sum"):
    """Element-wise c = op(a = local, b = incoming) (mini_nccl.cu:43-47)."""
    code, npd = DTYPES[dtype]
    a = np.ascontiguousarray(a, dtype=npd)
    b = np.ascontiguousarray(b, dtype=npd)
    c = np.empty_like(a)
    rc = load().oracle_reduce(_ptr(c), _ptr(a), _ptr(b), a.size, code, OPS[op])
    if rc != 0:
        raise ValueError("oracle_reduce rejected arguments")
    return c


def random_inputs(n, count, dtype="f32", seed=1234, kind="uniform"):
    """Rank r's buffer: seeded uniform[-1, 1) (seed = 1234 + r)."""
    _, npd = DTYPES[dtype]
    outs = []
    for r in range(n):
        g = np.random.default_rng(seed + r)
        if dtype == "i32":
            x = g.integers(-(2 ** 31), 2 ** 31 - 1, size=count, dtype=np.int64).astype(np.int32)
        elif dtype == "bf16":
            f = g.uniform(-1, 1, size=count).astype(np.float32)
            x = bf16_from_f32(f)
        else:
            x = g.uniform(-1, 1, size=count).astype(npd)
        outs.append(x)
    return outs


def bf16_from_f32(f):
    """float32 array -> bf16 bits (RNE, NaN quieted) -- vectorised twin of oracle_f32_to_bf16."""
    u = np.ascontiguousarray(f, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_to_f32(h):
    return (np.ascontiguousarray(h, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)
