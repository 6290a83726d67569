"""The drop-in boundary, checked without a GPU (-m "not gpu").

* libmini_nccl.so loads and exports every function include/*.h declares, with C linkage;
* the argument-validation paths that return before any device work behave like the
  reference's src/api.cpp (error codes and strings);
* the bootstrap (TCP star, reference RDMATransport.h:516-593) works across processes;
* the environment knobs (reference include/Config.h) parse as documented.
"""
import ctypes
import os
import re
import subprocess
import threading

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("mini_nccl_api.h", "mini_nccl_ext.h")]


def declared_functions():
    names = []
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_headers_declare_the_reference_entry_points():
    names = declared_functions()
    # reference include/mini_nccl_api.h:55-69
    for f in ("ncclGetErrorString", "ncclCommInitRank", "ncclCommDestroy", "ncclCommUserRank", "ncclCommCount",
              "ncclAllReduce"):
        assert f in names


def test_library_exports_every_declared_symbol(nccl_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", nccl_lib._name], capture_output=True, text=True, check=True)
    exported = {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}
    for f in declared_functions():
        assert f in exported, f"{f} declared in include/ but not exported (C linkage)"
        assert getattr(nccl_lib, f) is not None


def test_enum_values_match_reference(nccl_lib):
    import mini_nccl as M
    # reference include/mini_nccl_api.h:15-49
    assert (M.ncclSuccess, M.ncclUnhandledCudaError, M.ncclSystemError, M.ncclInternalError, M.ncclInvalidArgument,
            M.ncclInvalidUsage, M.ncclRemoteError, M.ncclInProgress) == tuple(range(8))
    assert (M.ncclInt8, M.ncclUint8, M.ncclInt32, M.ncclUint32, M.ncclInt64, M.ncclUint64, M.ncclFloat16,
            M.ncclFloat, M.ncclDouble, M.ncclBfloat16) == tuple(range(10))
    assert (M.ncclSum, M.ncclProd, M.ncclMax, M.ncclMin, M.ncclAvg) == tuple(range(5))
    hdr = open(HEADERS[0]).read()
    for name, val in (("ncclInvalidUsage", 5), ("ncclFloat", 7), ("ncclBfloat16", 9), ("ncclAvg", 4)):
        assert re.search(rf"\b{name}\s*=\s*{val}\b", hdr)


def test_error_strings(nccl_lib):
    import mini_nccl as M
    # reference src/api.cpp:14-26 (the CUDA wording becomes HIP)
    expect = {0: "no error", 2: "system error", 3: "internal error", 4: "invalid argument", 5: "invalid usage",
              6: "remote error", 7: "in progress", 99: "unknown error"}
    for code, s in expect.items():
        assert M.get_error_string(code) == s


def test_argument_checks_before_device_work(nccl_lib):
    import mini_nccl as M
    L = nccl_lib
    fake = ctypes.c_void_p(0x1000)  # never dereferenced on these paths
    # api.cpp:29: NULL comm pointer
    assert L.ncclCommInitRank(None, 2, 0, b"127.0.0.1") == M.ncclInvalidArgument
    h = ctypes.c_void_p()
    # api.cpp:53: rank out of range
    assert L.ncclCommInitRank(ctypes.byref(h), 2, 2, None) == M.ncclInvalidArgument
    assert L.ncclCommInitRank(ctypes.byref(h), 2, -2, None) == M.ncclInvalidArgument
    # api.cpp:38-51: Hera auto-rank is out of scope for this build
    assert L.ncclCommInitRank(ctypes.byref(h), 2, -1, None) == M.ncclInvalidUsage
    # api.cpp:69,80,91
    assert L.ncclCommDestroy(None) == M.ncclInvalidArgument
    assert L.ncclCommUserRank(None, None) == M.ncclInvalidArgument
    assert L.ncclCommCount(None, None) == M.ncclInvalidArgument
    # api.cpp:139-140: NULL buffers / comm, then count == 0 -> success
    assert L.ncclAllReduce(None, fake, 4, M.ncclFloat, M.ncclSum, fake, None) == M.ncclInvalidArgument
    assert L.ncclAllReduce(fake, None, 4, M.ncclFloat, M.ncclSum, fake, None) == M.ncclInvalidArgument
    assert L.ncclAllReduce(fake, fake, 4, M.ncclFloat, M.ncclSum, None, None) == M.ncclInvalidArgument
    assert L.ncclAllReduce(fake, fake, 0, M.ncclFloat, M.ncclSum, fake, None) == M.ncclSuccess
    # api.cpp:101-128 + :182-185: unsupported dtype or op -> ncclInternalError
    for dt in (M.ncclInt8, M.ncclUint8, M.ncclUint32, M.ncclInt64, M.ncclUint64):
        assert L.ncclAllReduce(fake, fake, 4, dt, M.ncclSum, fake, None) == M.ncclInternalError
    assert L.ncclAllReduce(fake, fake, 4, M.ncclFloat, M.ncclAvg, fake, None) == M.ncclInternalError
    assert L.mncclLocalReduce(fake, fake, fake, 4, M.ncclFloat, M.ncclAvg, None) == M.ncclInternalError
    assert L.mncclLocalReduce(None, fake, fake, 4, M.ncclFloat, M.ncclSum, None) == M.ncclInvalidArgument
    assert L.mncclCommSetAlgo(None, 0) == M.ncclInvalidArgument
    assert L.mncclVersion() == 600


def test_info_struct_layout(nccl_lib):
    import mini_nccl as M
    # mncclCommGetInfo (legacy) writes the pre-300 prefix only; mncclCommGetInfoV the whole struct
    names = [f for f, _ in M.CommInfo._fields_]
    assert names.index("ipc_open_failures") < names.index("cap_refusals") < names.index("read_push")
    hdr = open(HEADERS[1]).read()
    body = hdr[hdr.index("typedef struct {"):hdr.index("} mncclCommInfo_t;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    hdr_fields = re.findall(r"(\w+)(?:\[\d+\])?\s*[,;]", body)
    assert hdr_fields == names, (hdr_fields, names)


def test_init_without_gpu_fails_cleanly(nccl_lib):
    import mini_nccl as M
    # no device here: the constructor's HIP calls fail -> ncclSystemError (api.cpp:62-65), no crash
    h = ctypes.c_void_p()
    rc = nccl_lib.ncclCommInitRank(ctypes.byref(h), 1, 0, None)
    assert rc in (M.ncclSystemError, M.ncclSuccess)
    if rc == M.ncclSuccess:  # a GPU is visible after all
        assert nccl_lib.ncclCommDestroy(h) == M.ncclSuccess


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_bootstrap_star_allgather(sim_lib, nranks):
    import gpu_workers as GW
    port = GW.free_port()
    rcs = [None] * nranks

    def run(r):
        rcs[r] = sim_lib.mnccl_bootstrap_selftest(r, nranks, b"127.0.0.1", port, 20000)

    th = [threading.Thread(target=run, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert rcs == [0] * nranks


def test_bootstrap_times_out_without_peers(sim_lib):
    import gpu_workers as GW
    # rank 1 of 2 with nobody listening: bounded retry, then an error (not a hang)
    assert sim_lib.mnccl_bootstrap_selftest(1, 2, b"127.0.0.1", GW.free_port(), 500) == -1


def test_config_from_env(sim_lib, monkeypatch):
    import sim_api as S
    for k in list(os.environ):
        if k.startswith("MINI_NCCL_"):
            monkeypatch.delenv(k)
    rc, s = S.config_describe()
    assert rc == 0
    # reference defaults (Config.h:29-47): 128 KiB, 64, 16; workgroups derived per communicator
    # (channels=0, schedule.h pipeline_geometry); no auto-tune at init; 512 MiB scratch cap
    assert "SLICE_SIZE=131072 B" in s and "WINDOW=64" in s and "BATCH=16" in s and "channels=0" in s
    assert "algo=auto" in s and "threads=64" in s and "sys_fence=0" in s and "read_push" not in s
    assert "scratch_cap=512 MiB" in s
    monkeypatch.setenv("MINI_NCCL_SLICE_SIZE", "0")       # Config.h:50: 0 -> 1024
    monkeypatch.setenv("MINI_NCCL_WINDOW_SIZE", "-3")     # Config.h:51: <= 0 -> 1
    monkeypatch.setenv("MINI_NCCL_SLOTS", "1")            # clamped to 2 (deadlock-free minimum)
    rc, s = S.config_describe()
    assert "SLICE_SIZE=1024 B" in s and "WINDOW=1" in s and "slots=2" in s and "channels=0" in s
    monkeypatch.setenv("MINI_NCCL_SLICE_SIZE", str(8 << 30))  # 32-bit message lengths: clamped
    rc, s = S.config_describe()
    assert rc == 0 and f"SLICE_SIZE={256 << 20} B" in s
    monkeypatch.setenv("MINI_NCCL_ALGO", "ring")
    monkeypatch.setenv("MINI_NCCL_SLICE_SIZE", "100")     # rounded down to whole 16-byte vectors
    monkeypatch.setenv("MINI_NCCL_READ_PUSH", "0")        # the load form, removed in 6.0: warned, ignored
    rc, s = S.config_describe()
    assert rc == 0 and "algo=ring" in s and "SLICE_SIZE=96 B" in s
    monkeypatch.setenv("MINI_NCCL_ALGO", "direct")        # removed in 4.0: an init error, not a silent ring
    rc, s = S.config_describe()
    assert rc == -1 and "no longer" in s
    monkeypatch.setenv("MINI_NCCL_ALGO", "auto")
    rc, s = S.config_describe()
    assert rc == 0 and "algo=auto" in s and "grid_vectors=0" in s
    monkeypatch.setenv("MINI_NCCL_GRID_VECTORS", "4")      # the grid form's tuning knob (fp32 Sum)
    rc, s = S.config_describe()
    assert rc == 0 and "grid_vectors=4" in s
    monkeypatch.setenv("MINI_NCCL_GRID_VECTORS", "3")      # not an instantiated width: an init error
    rc, s = S.config_describe()
    assert rc == -1 and "GRID_VECTORS" in s
    monkeypatch.delenv("MINI_NCCL_GRID_VECTORS")
    rc, s = S.config_describe()
    assert rc == 0 and f"grid_min={4 << 20} B" in s                # the grid form's threshold (tuning knob)
    monkeypatch.setenv("MINI_NCCL_GRID_MIN", str(256 << 10))
    rc, s = S.config_describe()
    assert rc == 0 and f"grid_min={256 << 10} B" in s
    monkeypatch.setenv("MINI_NCCL_GRID_MIN", "1000")          # below 64 KiB / not whole vectors: an init error
    rc, s = S.config_describe()
    assert rc == -1 and "GRID_MIN" in s
    monkeypatch.delenv("MINI_NCCL_GRID_MIN")
    monkeypatch.setenv("MINI_NCCL_ALGO", "oneshot")      # 4.1
    rc, s = S.config_describe()
    assert rc == 0 and "algo=oneshot" in s
    monkeypatch.setenv("MINI_NCCL_ALGO", "tree")
    rc, s = S.config_describe()
    assert rc == -1 and "MINI_NCCL_ALGO" in s


def test_pipeline_geometry(sim_lib):
    import sim_api as S
    MiB = 1 << 20
    # defaults: one pipeline per CU (256), (n-1) peer regions of 256 x 2 x 128 KiB
    g = S.pipeline_geometry(8)
    assert g == {"workgroups": 256, "waves": 1, "slot_bytes": 128 << 10, "scratch_bytes": 7 * 256 * 2 * (128 << 10)}
    assert g["scratch_bytes"] == 448 * MiB
    assert S.pipeline_geometry(2)["scratch_bytes"] == 64 * MiB
    assert S.pipeline_geometry(1)["scratch_bytes"] == 0
    # WINDOW x SIGNAL_BATCH bounds the messages in flight per link (mini_nccl.cu:119,144,167):
    # pipelines x slots <= WINDOW x SIGNAL_BATCH; at WINDOW >= 32 the 256-pipeline default binds
    assert [S.pipeline_geometry(8, window=w)["workgroups"] for w in (16, 32, 64)] == [128, 256, 256]
    assert S.pipeline_geometry(8, window=1)["workgroups"] == 8
    assert S.pipeline_geometry(8, window=16, signal_batch=1)["workgroups"] == 8
    assert S.pipeline_geometry(8, window=64, threads=256)["workgroups"] == 64  # 4 waves each
    # the scratch cap: BASELINE C4's SLICE = 1 MiB at WINDOW 64 keeps 1 MiB messages, fewer pipelines
    for sl in (64 << 10, 128 << 10, 256 << 10, 1 << 20):
        for w in (16, 32, 64):
            g = S.pipeline_geometry(8, window=w, slice_bytes=sl)
            assert g["scratch_bytes"] <= 512 * MiB and g["slot_bytes"] == sl, (sl, w, g)
    assert S.pipeline_geometry(8, slice_bytes=1 << 20)["workgroups"] == 36
    # MINI_NCCL_CHANNELS is honoured up to the cap
    assert S.pipeline_geometry(4, channels=64)["workgroups"] == 64
    assert S.pipeline_geometry(8, channels=1024)["workgroups"] == 292
    # a slice so large that one workgroup cannot fit: the slot shrinks (whole KiB), never the cap
    g = S.pipeline_geometry(8, slice_bytes=256 * MiB)
    assert g["workgroups"] == 1 and g["slot_bytes"] % 1024 == 0 and g["scratch_bytes"] <= 512 * MiB
    g = S.pipeline_geometry(8, cap=16 * MiB, slice_bytes=1 << 20)
    assert g["workgroups"] == 1 and g["scratch_bytes"] <= 16 * MiB


def test_removed_knobs_are_warned_once(sim_lib):
    # a knob removed in 4.0 that is still set (a 3.x deployment's MINI_NCCL_STAGE_HOST=1
    # used to stage pinned buffers) is named on stderr once per process, with what replaced it
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import sim_api as S\n"
            "for _ in range(3): S.config_describe()\n") % os.path.dirname(os.path.abspath(__file__))
    env = {k: v for k, v in os.environ.items() if not k.startswith("MINI_NCCL_")}
    env.update(MINI_NCCL_STAGE_HOST="1", MINI_NCCL_PIPE_DEPTH="4")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stderr.splitlines() if "is ignored" in ln]
    assert len(lines) == 2, r.stderr
    assert any("MINI_NCCL_STAGE_HOST=1" in ln and "always mapped" in ln for ln in lines)
    assert any("MINI_NCCL_PIPE_DEPTH=4" in ln for ln in lines)
    env.pop("MINI_NCCL_STAGE_HOST")
    env.pop("MINI_NCCL_PIPE_DEPTH")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert "is ignored" not in r.stderr
