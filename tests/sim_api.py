"""ctypes front end of mini-nccl_amd/lib/libmnccl_sim.so (CPU-only test library).

The simulator executes the GPU kernels' per-channel op sequence (csrc/schedule.h, the
same header kernels.hip includes) on simulated ranks; see csrc/sim.cpp.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mini-nccl_amd", "lib", "libmnccl_sim.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB)
        vp, u64, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.mnccl_sim_allreduce.argtypes = [u64, ctypes.POINTER(vp), ctypes.POINTER(vp), i, u64, i, u64, u64, i, i, i,
                                          u64, ctypes.POINTER(u64)]
        L.mnccl_board_selftest.argtypes = [i, i, ctypes.c_char_p, i, i, i, ctypes.c_double, ctypes.POINTER(i)]
        L.mnccl_read_slice.argtypes = [u64, i, u64, u64, i]
        L.mnccl_read_slice.restype = u64
        L.mnccl_call_pipelines.argtypes = [u64, i, i]
        L.mnccl_resident_pipes.argtypes = [i, i, i, i, i]
        L.mnccl_topology_blocks_read.argtypes = [i, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.mnccl_read_grid_form.argtypes = [i, i, i, u64, i, u64]
        L.mnccl_sim_signed_read.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), i, u64, i, u64,
                                            ctypes.POINTER(u64), u64, ctypes.POINTER(i)]
        L.mnccl_oneshot_slice.argtypes = [u64, i, i, u64]
        L.mnccl_oneshot_slice.restype = u64
        L.mnccl_oneshot_fits.argtypes = [u64, i, i, u64, i]
        L.mnccl_effective_slice.argtypes = [u64, i, u64, u64, i]
        L.mnccl_effective_slice.restype = u64
        L.mnccl_bootstrap_selftest.argtypes = [i, i, ctypes.c_char_p, i, i]
        L.mnccl_config_describe.argtypes = [ctypes.c_char_p, i]
        L.mnccl_pipeline_geometry.argtypes = [i, i, i, i, i, i, u64, u64, ctypes.POINTER(u64)]
        _lib = L
    return _lib


# schedules: the ring, the one-shot, read (the persistent kernel), read's grid form
RING, ONESHOT, READ, READ_GRID = 0, 1, 2, 4  # (3: the load form, removed in 6.0)


def allreduce(inputs, algo=0, op=0, slice_bytes=1024, channels=4, slots=2, calls=1, seed=0, algos=None, min_slice=0,
              inplace=False):
    """fp32 all-reduce of `inputs` (one array per rank) through the simulated kernels,
    `calls` times on one communicator state (schedule `algo` -- RING, ONESHOT, READ (the
    persistent kernel) or READ_GRID (its grid launches) -- for every
    call, or the per-call list `algos`; at most 21 calls).  inplace: send == recv (then every call after the first reduces the previous
    result).  Returns (outputs, steps); raises RuntimeError on deadlock."""
    if algos is None:
        algos = [algo] * calls
    calls = len(algos)
    assert calls <= 21
    mask = sum((a & 7) << (3 * i) for i, a in enumerate(algos))
    n = len(inputs)
    sends = [np.array(x, dtype=np.float32) for x in inputs]  # own copies (in place writes them)
    recvs = sends if inplace else [np.full_like(x, np.nan) for x in sends]
    sp = (ctypes.c_void_p * n)(*[s.ctypes.data for s in sends])
    rp = (ctypes.c_void_p * n)(*[r.ctypes.data for r in recvs])
    steps = ctypes.c_uint64()
    rc = load().mnccl_sim_allreduce(mask, sp, rp, n, sends[0].size, op, slice_bytes, min_slice, channels, slots,
                                    calls, seed, ctypes.byref(steps))
    if rc == -1:
        raise RuntimeError("simulated protocol deadlocked")
    if rc != 0:
        raise ValueError(f"bad simulator arguments (rc={rc})")
    return recvs, steps.value


def config_describe(env=None):
    buf = ctypes.create_string_buffer(512)
    rc = load().mnccl_config_describe(buf, 512)
    return rc, buf.value.decode()


def pipeline_geometry(n, channels=0, threads=64, window=64, signal_batch=16, slots=2, slice_bytes=128 << 10,
                      cap=512 << 20):
    """csrc/schedule.h pipeline_geometry: what a communicator allocates and launches."""
    out = (ctypes.c_uint64 * 4)()
    load().mnccl_pipeline_geometry(n, channels, threads, window, signal_batch, slots, slice_bytes, cap, out)
    return {"workgroups": out[0], "waves": out[1], "slot_bytes": out[2], "scratch_bytes": out[3]}


def effective_slice(chunk_bytes, channels, slice_bytes, min_slice, depth=1):
    return load().mnccl_effective_slice(chunk_bytes, channels, slice_bytes, min_slice, depth)


def read_slice(chunk_bytes, channels, slice_bytes, min_slice, depth=16):
    return load().mnccl_read_slice(chunk_bytes, channels, slice_bytes, min_slice, depth)


def oneshot_slice(chunk_bytes, n, channels, slot_bytes):
    return load().mnccl_oneshot_slice(chunk_bytes, n, channels, slot_bytes)


def oneshot_fits(chunk_bytes, n, channels, slot_bytes, forced=False):
    return bool(load().mnccl_oneshot_fits(chunk_bytes, n, channels, slot_bytes, int(forced)))


def resident_pipes(P, waves, cus, most, waves_per_simd=2):
    """csrc/schedule.h resident_pipes: the pipelines a call may launch with `most` ranks on a GPU."""
    return load().mnccl_resident_pipes(P, waves, cus, most, waves_per_simd)


def call_pipelines(nslices, channels, waves=1):
    """csrc/schedule.h call_pipelines: the pipelines a call of `nslices` slices runs."""
    return load().mnccl_call_pipelines(nslices, channels, waves)


def board_selftest(rank, nranks, port, scenario, calls, timeout_s=2.0):
    """csrc/peerbuf.cpp's per-call rendezvous on real processes (no GPU): (rc, decisions)."""
    dec = (ctypes.c_int * calls)()
    rc = load().mnccl_board_selftest(rank, nranks, b"127.0.0.1", port, scenario, calls, timeout_s, dec)
    return rc, list(dec)


# schedule.h link kinds (how rank q's GPU reaches rank p's)
SAME_GPU, UNKNOWN, PCIE, XGMI = -1, -2, 2, 4


def topology_blocks_read(link, hops):
    """csrc/schedule.h topology_blocks_read on an n x n link / hop matrix (row q: rank q's view):
    None when auto may run the read schedule, else the first offending pair (q, p)."""
    n = len(link)
    flat_l = (ctypes.c_int * (n * n))(*[link[q][p] for q in range(n) for p in range(n)])
    flat_h = (ctypes.c_int * (n * n))(*[hops[q][p] for q in range(n) for p in range(n)])
    bad = load().mnccl_topology_blocks_read(n, flat_l, flat_h)
    return None if bad == 0 else divmod(bad - 1, n)


def signed_read(inputs, sigs, slice_bytes=1024, channels=4, seed=1):
    """One read call (push form) on registered windows through the simulated kernels: rank r's
    START carries sigs[r], every pipeline checks its peers' before touching data (kernels.hip
    starts_agree).  Returns (recv buffers, per-rank count of pipelines that gave up)."""
    n = len(inputs)
    sends = [np.array(x, dtype=np.float32) for x in inputs]
    recvs = [np.full_like(x, np.nan) for x in sends]
    sp = (ctypes.c_void_p * n)(*[s.ctypes.data for s in sends])
    rp = (ctypes.c_void_p * n)(*[r.ctypes.data for r in recvs])
    sg = (ctypes.c_uint64 * n)(*sigs)
    mm = (ctypes.c_int * n)()
    rc = load().mnccl_sim_signed_read(sp, rp, n, sends[0].size, channels, slice_bytes, sg, seed, mm)
    if rc == -1:
        raise RuntimeError("simulated protocol deadlocked")
    if rc not in (0, 1):
        raise ValueError(f"bad simulator arguments (rc={rc})")
    return recvs, list(mm)


def read_grid_form(forced, auto_mode, vec, chunk_bytes, n, min_bytes=4 << 20):
    """csrc/schedule.h read_grid_form: a read-schedule call launches in the grid form (chunks of
    at least min_bytes: MINI_NCCL_GRID_MIN, default kReadGridMin = 4 MiB)."""
    return bool(load().mnccl_read_grid_form(int(forced), int(auto_mode), int(vec), chunk_bytes, n,
                                            min_bytes))
