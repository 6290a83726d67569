"""Minimal ctypes view of the HIP runtime (libamdhip64.so) for the GPU tests.

Device memory, copies and streams only -- plumbing, so the parity tests exercise
libmini_nccl.so through its C ABI exactly as a C caller would, without torch.
"""
import ctypes

import numpy as np

hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice = 1, 2, 3
_hip = None


def lib():
    global _hip
    if _hip is None:
        try:
            _hip = ctypes.CDLL("libamdhip64.so")
        except OSError:
            _hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        _hip.hipSetDevice.argtypes = [i]
        _hip.hipGetDeviceCount.argtypes = [ctypes.POINTER(i)]
        _hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
        _hip.hipFree.argtypes = [vp]
        _hip.hipMemcpy.argtypes = [vp, vp, sz, i]
        _hip.hipMemset.argtypes = [vp, i, sz]
        _hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
        _hip.hipHostFree.argtypes = [vp]
        _hip.hipDeviceSynchronize.argtypes = []
        _hip.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
        _hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
        _hip.hipStreamSynchronize.argtypes = [vp]
        _hip.hipStreamDestroy.argtypes = [vp]
        _hip.hipGetErrorString.argtypes = [i]
        _hip.hipGetErrorString.restype = ctypes.c_char_p
        _hip.hipStreamBeginCapture.argtypes = [vp, i]
        _hip.hipStreamEndCapture.argtypes = [vp, ctypes.POINTER(vp)]
        _hip.hipGraphInstantiate.argtypes = [ctypes.POINTER(vp), vp, vp, ctypes.c_char_p, sz]
        _hip.hipGraphLaunch.argtypes = [vp, vp]
        _hip.hipGraphExecDestroy.argtypes = [vp]
        _hip.hipGraphDestroy.argtypes = [vp]
        _hip.hipStreamWaitValue32.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
        _hip.hipStreamWaitValue32.restype = i
        _hip.hipMemGetInfo.argtypes = [ctypes.POINTER(sz), ctypes.POINTER(sz)]
        _hip.hipMemGetInfo.restype = i
        for f in ("hipStreamBeginCapture", "hipStreamEndCapture", "hipGraphInstantiate", "hipGraphLaunch",
                  "hipGraphExecDestroy", "hipGraphDestroy"):
            getattr(_hip, f).restype = i
        for f in ("hipSetDevice", "hipGetDeviceCount", "hipMalloc", "hipFree", "hipMemcpy", "hipMemset",
                  "hipHostMalloc", "hipHostFree",
                  "hipDeviceSynchronize", "hipStreamCreate", "hipStreamCreateWithFlags", "hipStreamSynchronize",
                  "hipStreamDestroy"):
            getattr(_hip, f).restype = i
    return _hip


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {lib().hipGetErrorString(rc).decode()} ({rc})")


def device_count():
    n = ctypes.c_int()
    rc = lib().hipGetDeviceCount(ctypes.byref(n))
    return n.value if rc == 0 else 0


def set_device(d):
    check(lib().hipSetDevice(d), "hipSetDevice")


def mem_get_info():
    """(free, total) bytes of the current device (hipMemGetInfo)."""
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    check(lib().hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)), "hipMemGetInfo")
    return f.value, t.value


_cache = {}  # segment bytes -> free segments (device pointers) of that size


def _segment_bytes(nbytes):
    """A caching allocator's segment size, as frameworks use (torch's caching allocator never
    hipFrees a segment it can hand out again): a power of two of at least 2 MiB."""
    s = 2 << 20
    while s < nbytes:
        s <<= 1
    return s


class DeviceBuffer:
    """Device memory.  By default from a per-process cache of whole segments (a freed buffer's
    segment serves the next request of the same segment size: the allocation -- and so its IPC
    export -- is reused, as with torch's caching allocator); fresh=True: its own hipMalloc /
    hipFree, for the tests of allocation churn."""

    def __init__(self, nbytes, fresh=False):
        self.nbytes = nbytes
        self.fresh = fresh
        self.seg = max(nbytes, 16) if fresh else _segment_bytes(nbytes)
        free = [] if fresh else _cache.get(self.seg, [])
        if free:
            self.ptr = free.pop()
            return
        p = ctypes.c_void_p()
        check(lib().hipMalloc(ctypes.byref(p), self.seg), "hipMalloc")
        self.ptr = p.value

    def upload(self, arr, offset=0):
        a = np.ascontiguousarray(arr)
        check(lib().hipMemcpy(self.ptr + offset, a.ctypes.data, a.nbytes, hipMemcpyHostToDevice), "H2D")

    def download(self, dtype, count, offset=0):
        out = np.empty(count, dtype=dtype)
        check(lib().hipMemcpy(out.ctypes.data, self.ptr + offset, out.nbytes, hipMemcpyDeviceToHost), "D2H")
        return out

    def fill_byte(self, value):
        # hipMemset runs on the null stream and may return before it lands; the test
        # streams are non-blocking (not ordered after it), so wait here
        check(lib().hipMemset(self.ptr, value, self.nbytes), "hipMemset")
        check(lib().hipDeviceSynchronize(), "hipDeviceSynchronize")

    def free(self):
        if self.ptr:
            if self.fresh:
                lib().hipFree(self.ptr)
            else:
                _cache.setdefault(self.seg, []).append(self.ptr)
            self.ptr = 0


class View:
    """A region of another buffer (its owner is freed with the view at offset 0)."""

    def __init__(self, owner, offset, nbytes):
        self.owner, self.offset, self.nbytes = owner, offset, nbytes
        self.ptr = owner.ptr + offset

    def upload(self, arr, offset=0):
        self.owner.upload(arr, self.offset + offset)

    def download(self, dtype, count, offset=0):
        return self.owner.download(dtype, count, self.offset + offset)

    def fill_byte(self, value):
        check(lib().hipMemset(self.ptr, value, self.nbytes), "hipMemset")
        check(lib().hipDeviceSynchronize(), "hipDeviceSynchronize")

    def free(self):
        if self.offset == 0:
            self.owner.free()
        self.ptr = 0


class HostBuffer:
    """Pinned host memory (hipHostMalloc, the reference perf_test's cudaHostAlloc buffers,
    tests/perf_test.cpp:78-79): the all-reduce kernel addresses it through its device mapping."""

    def __init__(self, nbytes):
        self.nbytes = nbytes
        p = ctypes.c_void_p()
        check(lib().hipHostMalloc(ctypes.byref(p), max(nbytes, 16), 0), "hipHostMalloc")
        self.ptr = p.value

    def view(self):
        return np.ctypeslib.as_array((ctypes.c_uint8 * max(self.nbytes, 16)).from_address(self.ptr))

    def upload(self, arr, offset=0):
        a = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        self.view()[offset:offset + a.size] = a

    def download(self, dtype, count, offset=0):
        nb = count * np.dtype(dtype).itemsize
        return self.view()[offset:offset + nb].copy().view(dtype)

    def fill_byte(self, value):
        self.view()[:] = value

    def free(self):
        if self.ptr:
            lib().hipHostFree(self.ptr)
            self.ptr = 0


class PageableBuffer(HostBuffer):
    """Ordinary (pageable) host memory, unknown to HIP: the library stages it through HBM."""

    def __init__(self, nbytes):
        self.nbytes = nbytes
        self._a = np.zeros(max(nbytes, 16) + 64, dtype=np.uint8)
        self.ptr = (self._a.ctypes.data + 63) & ~63

    def free(self):
        self._a = None
        self.ptr = 0


def buffer(kind, nbytes, fresh=False):
    if kind == "device":
        return DeviceBuffer(nbytes, fresh=fresh)
    return {"pinned": HostBuffer, "pageable": PageableBuffer}[kind](nbytes)


class Stream:
    """A non-blocking stream (hipStreamNonBlocking): it does not synchronise with the legacy
    null stream, so a synchronous hipMemcpy issued by one rank-thread of a process cannot
    wait behind another rank-thread's running all-reduce kernel."""

    def __init__(self):
        s = ctypes.c_void_p()
        check(lib().hipStreamCreateWithFlags(ctypes.byref(s), 1), "hipStreamCreateWithFlags")
        self.handle = s.value

    def sync(self):
        check(lib().hipStreamSynchronize(self.handle), "hipStreamSynchronize")

    def wait_value32(self, ptr, value):
        """Block the stream (on the GPU) until the 32-bit word at `ptr` (pinned host memory) is
        >= value (hipStreamWaitValueGte)."""
        check(lib().hipStreamWaitValue32(self.handle, ptr, value, 0, 0xFFFFFFFF), "hipStreamWaitValue32")

    def destroy(self):
        if self.handle:
            lib().hipStreamDestroy(self.handle)
            self.handle = None


def sync():
    check(lib().hipDeviceSynchronize(), "hipDeviceSynchronize")


class Graph:
    """Capture the HIP work a callable enqueues on `stream` into a graph; replay it with launch()."""

    def __init__(self, stream, fn):
        self.stream = stream
        check(lib().hipStreamBeginCapture(stream.handle, 0), "hipStreamBeginCapture")  # global mode
        try:
            fn()
        finally:
            g = ctypes.c_void_p()
            check(lib().hipStreamEndCapture(stream.handle, ctypes.byref(g)), "hipStreamEndCapture")
        self.graph = g.value
        ex = ctypes.c_void_p()
        check(lib().hipGraphInstantiate(ctypes.byref(ex), self.graph, None, None, 0), "hipGraphInstantiate")
        self.exec = ex.value

    def launch(self):
        check(lib().hipGraphLaunch(self.exec, self.stream.handle), "hipGraphLaunch")

    def destroy(self):
        lib().hipGraphExecDestroy(self.exec)
        lib().hipGraphDestroy(self.graph)
