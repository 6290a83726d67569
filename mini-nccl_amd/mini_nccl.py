"""ctypes binding of libmini_nccl.so -- the host-side mirror of the reference's C ABI.

The reference's callers are C++ programs linking ``libmini_nccl.so``
(``tests/perf_test.cpp``, ``src/main.cpp``); ``apps/`` holds the C++ equivalents.
This module exposes the same six entry points (``include/mini_nccl_api.h``) plus the
extensions of ``include/mini_nccl_ext.h`` to Python for the test suite and
``bench.py``.  Names, argument meaning and return codes are the C ones: every
function returns an ``ncclResult_t`` integer, exactly as the C ABI does.

Device memory and streams are passed as raw integers (device pointers / hipStream_t),
so any allocator works: torch tensors (``t.data_ptr()``, ``torch.cuda.Stream().cuda_stream``)
or the raw HIP runtime (``tests/hip_rt.py``).  There is no CPU fallback: if the
library is missing, :func:`load` raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libmini_nccl.so")

# ncclResult_t (include/mini_nccl_api.h; reference include/mini_nccl_api.h:15-24)
ncclSuccess = 0
ncclUnhandledCudaError = 1
ncclSystemError = 2
ncclInternalError = 3
ncclInvalidArgument = 4
ncclInvalidUsage = 5
ncclRemoteError = 6
ncclInProgress = 7

# ncclDataType_t (reference :29-40)
ncclInt8, ncclUint8, ncclInt32, ncclUint32, ncclInt64, ncclUint64 = 0, 1, 2, 3, 4, 5
ncclFloat16, ncclFloat, ncclDouble, ncclBfloat16 = 6, 7, 8, 9

# ncclRedOp_t (reference :43-49)
ncclSum, ncclProd, ncclMax, ncclMin, ncclAvg = 0, 1, 2, 3, 4

# mncclAlgo_t (mncclAlgoDirect = 1 was removed in mncclVersion 400)
ALGO_AUTO, ALGO_RING, ALGO_READ, ALGO_ONESHOT, ALGO_READ_GRID = -1, 0, 2, 3, 4

DTYPE_SIZE = {ncclInt32: 4, ncclFloat16: 2, ncclFloat: 4, ncclDouble: 8, ncclBfloat16: 2}


class CommInfo(ctypes.Structure):
    _fields_ = [
        ("rank", ctypes.c_int), ("nranks", ctypes.c_int), ("device", ctypes.c_int),
        ("slice_bytes", ctypes.c_size_t), ("window", ctypes.c_int), ("signal_batch", ctypes.c_int),
        ("channels", ctypes.c_int), ("slots", ctypes.c_int), ("threads", ctypes.c_int),
        ("algo", ctypes.c_int), ("blocking", ctypes.c_int), ("sys_fence", ctypes.c_int),
        ("timeout_s", ctypes.c_double), ("scratch_bytes", ctypes.c_size_t), ("tune_ms", ctypes.c_double * 2),
        ("pipelines", ctypes.c_int), ("ranks_on_device", ctypes.c_int), ("slot_bytes", ctypes.c_size_t),
        ("last_algo", ctypes.c_int), ("peer_mappings", ctypes.c_size_t), ("scratch_algo", ctypes.c_int),
        ("calib_choice", ctypes.c_int), ("calib_ms", ctypes.c_double * 2),
        # since mncclVersion 300
        ("ipc_open_failures", ctypes.c_ulonglong), ("read_map_failures", ctypes.c_ulonglong),
        ("read_rounds", ctypes.c_ulonglong), ("closed_freed", ctypes.c_ulonglong), ("live_exports", ctypes.c_size_t),
        # since mncclVersion 400
        ("cap_refusals", ctypes.c_ulonglong), ("liveness_queries", ctypes.c_ulonglong), ("read_push", ctypes.c_int),
        # since mncclVersion 500
        ("auto_read", ctypes.c_int), ("peer_link", ctypes.c_int * 16), ("peer_hops", ctypes.c_int * 16),
        ("auto_reason", ctypes.c_char * 160), ("read_grid_calls", ctypes.c_ulonglong),
        ("window_calls", ctypes.c_ulonglong), ("windows", ctypes.c_int), ("auto_grid", ctypes.c_int),
        # since mncclVersion 501
        ("retired_imports", ctypes.c_int),
        # since mncclVersion 600
        ("retired_bytes", ctypes.c_ulonglong), ("retired_budget", ctypes.c_ulonglong),
        ("budget_refusals", ctypes.c_ulonglong), ("window_fast", ctypes.c_int),
        ("run_pipelines", ctypes.c_int),
    ]


# every entry point of include/mini_nccl_api.h and include/mini_nccl_ext.h: (restype, argtypes)
_VP, _SZ, _I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
SIGNATURES = {
    "ncclGetErrorString": (ctypes.c_char_p, [_I]),
    "ncclCommInitRank": (_I, [ctypes.POINTER(_VP), _I, _I, ctypes.c_char_p]),
    "ncclCommDestroy": (_I, [_VP]),
    "ncclCommUserRank": (_I, [_VP, ctypes.POINTER(_I)]),
    "ncclCommCount": (_I, [_VP, ctypes.POINTER(_I)]),
    "ncclAllReduce": (_I, [_VP, _VP, _SZ, _I, _I, _VP, _VP]),
    "mncclLocalReduce": (_I, [_VP, _VP, _VP, _SZ, _I, _I, _VP]),
    "mncclCommGetAsyncError": (_I, [_VP, ctypes.POINTER(_I)]),
    "mncclCommGetInfo": (_I, [_VP, ctypes.POINTER(CommInfo)]),
    "mncclCommGetInfoV": (_I, [_VP, _VP, _SZ]),
    "mncclCommSetAlgo": (_I, [_VP, _I]),
    "mncclCommLinkProbe": (_I, [_VP, _I, _SZ, _I, ctypes.POINTER(ctypes.c_double)]),
    "mncclCommRegister": (_I, [_VP, _VP, _SZ, ctypes.POINTER(_VP)]),
    "mncclCommDeregister": (_I, [_VP, _VP]),
    "mncclVersion": (_I, []),
}

_lib = None


def load(path=None):
    """Load libmini_nccl.so (raises OSError if it is missing: no fallback)."""
    global _lib
    if _lib is None or path is not None:
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise OSError(f"{p} not built: run `make -C mini-nccl_amd` (or __graft_entry__.build())")
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def get_error_string(result):
    return load().ncclGetErrorString(int(result)).decode()


class NcclError(RuntimeError):
    def __init__(self, code, what=""):
        super().__init__(f"{what}: {get_error_string(code)} ({code})")
        self.code = code


def check(code, what="mini-nccl"):
    if code != ncclSuccess:
        raise NcclError(code, what)
    return code


class Comm:
    """Thin RAII wrapper over ncclComm_t (the calls themselves are the C functions)."""

    def __init__(self, nranks, rank, ip="127.0.0.1"):
        lib = load()
        self.handle = ctypes.c_void_p()
        check(lib.ncclCommInitRank(ctypes.byref(self.handle), nranks, rank, ip.encode() if ip else None),
              "ncclCommInitRank")

    def all_reduce(self, send_ptr, recv_ptr, count, dtype=ncclFloat, op=ncclSum, stream=0):
        """Returns the ncclResult_t (does not raise) -- the reference's calling convention."""
        return load().ncclAllReduce(send_ptr, recv_ptr, count, dtype, op, self.handle, stream)

    def rank(self):
        r = ctypes.c_int()
        check(load().ncclCommUserRank(self.handle, ctypes.byref(r)))
        return r.value

    def count(self):
        c = ctypes.c_int()
        check(load().ncclCommCount(self.handle, ctypes.byref(c)))
        return c.value

    def info(self):
        i = CommInfo()
        check(load().mncclCommGetInfoV(self.handle, ctypes.byref(i), ctypes.sizeof(i)))
        d = {f: getattr(i, f) for f, _ in CommInfo._fields_}
        d["tune_ms"] = list(d["tune_ms"])
        d["calib_ms"] = list(d["calib_ms"])
        n = d["nranks"]
        d["peer_link"] = list(d["peer_link"])[:n]
        d["peer_hops"] = list(d["peer_hops"])[:n]
        d["auto_reason"] = d["auto_reason"].decode(errors="replace")
        return d

    PROBE_FORMS = {"sys": 0, "nt": 1, "plain": 2}

    def link_probe(self, all_peers=False, nbytes=0, iters=10, form="sys", pull=False, user=False):
        """GB/s per destination link (collective: every rank must call it).  form: the remote
        accesses' cache policy ("sys" = the hot path's sc0 sc1, "nt", "plain"); pull: load
        from the peers over the link instead of storing into them; user: the peers' ordinary
        device memory (what the read schedule loads from) instead of their uncached scratch."""
        g = ctypes.c_double()
        mode = int(bool(all_peers)) | (self.PROBE_FORMS[form] << 1) | (8 if pull else 0) | (16 if user else 0)
        check(load().mncclCommLinkProbe(self.handle, mode, nbytes, iters, ctypes.byref(g)), "mncclCommLinkProbe")
        return g.value

    def register(self, ptr, nbytes):
        """mncclCommRegister (collective): returns the window handle."""
        h = ctypes.c_void_p()
        check(load().mncclCommRegister(self.handle, ptr, nbytes, ctypes.byref(h)), "mncclCommRegister")
        return h

    def register_rc(self, ptr, nbytes):
        """mncclCommRegister's result code (does not raise) and the handle."""
        h = ctypes.c_void_p()
        return load().mncclCommRegister(self.handle, ptr, nbytes, ctypes.byref(h)), h

    def deregister(self, h):
        return check(load().mncclCommDeregister(self.handle, h), "mncclCommDeregister")

    def set_algo(self, algo):
        return check(load().mncclCommSetAlgo(self.handle, algo))

    def async_error(self):
        e = ctypes.c_int()
        check(load().mncclCommGetAsyncError(self.handle, ctypes.byref(e)))
        return e.value

    def destroy(self):
        if self.handle:
            code = load().ncclCommDestroy(self.handle)
            self.handle = ctypes.c_void_p()
            return code
        return ncclSuccess


def local_reduce(out_ptr, local_ptr, incoming_ptr, count, dtype=ncclFloat, op=ncclSum, stream=0):
    """out[i] = op(local[i], incoming[i]) on the GPU (the scatter-reduce element-wise kernel)."""
    return load().mncclLocalReduce(out_ptr, local_ptr, incoming_ptr, count, dtype, op, stream)
