"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

SURVEY.md §5 asks for sanitizers on the host side; GPU ASan / XNACK are not available on the
test pool, so the host logic the GPU path relies on -- csrc/schedule.h index math driven by
the kernel-mirroring simulator, the TCP bootstrap, env parsing -- is compiled with
-fsanitize=address,undefined into tests/native/host_selftest and run.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mini-nccl_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_logic_under_asan_ubsan(tmp_path):
    import gpu_workers as GW
    exe = str(tmp_path / "host_selftest")
    srcs = [os.path.join(ROOT, "tests", "native", "host_selftest.cpp")] + \
        [os.path.join(CSRC, f) for f in ("sim.cpp", "bootstrap.cpp", "config.cpp", "peerbuf.cpp", "ipcreg.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-pthread", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           "-I" + CSRC, "-o", exe] + srcs + ["-L/opt/rocm/lib", "-lamdhip64", "-lhsa-runtime64", "-lrt", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, SELFTEST_PORT=str(GW.free_port()), ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    for k in [k for k in env if k.startswith("MINI_NCCL_")]:
        env.pop(k)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "host selftest: ok" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]


def _build_abi_selftest(tmp_path):
    obj = os.path.join(ROOT, "mini-nccl_amd", "build", "kernels.o")
    if not os.path.exists(obj):
        subprocess.run(["make", "-C", os.path.join(ROOT, "mini-nccl_amd")], check=True, capture_output=True,
                       timeout=900)
    exe = str(tmp_path / "abi_selftest")
    srcs = [os.path.join(ROOT, "tests", "native", "abi_selftest.cpp")] + \
        [os.path.join(CSRC, f) for f in ("api.cpp", "comm.cpp", "peerbuf.cpp", "ipcreg.cpp", "bootstrap.cpp", "config.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-Wno-unused-result", "-pthread", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-o", exe] + srcs + \
        [obj, "-L/opt/rocm/lib", "-lamdhip64", "-lhsa-runtime64", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=600)
    return exe


def _run_abi_selftest(exe, expect):
    import gpu_workers as GW
    env = {k: v for k, v in os.environ.items() if not k.startswith("MINI_NCCL_")}
    # the HIP runtime keeps allocations until process exit (leak reports would be its own), and
    # ASan cannot unmap its alternate signal stack in the runtime's threads (a CHECK failure in
    # AsanThread::Destroy, seen on the MI355X box): no sigaltstack
    env.update(MINI_NCCL_PORT=str(GW.free_port()), ASAN_OPTIONS="detect_leaks=0:use_sigaltstack=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert expect in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/rocm/lib/libamdhip64.so"),
                    reason="needs g++ and the HIP runtime")
def test_abi_host_code_under_asan_ubsan(tmp_path):
    # argument checks and the clean init failure without a GPU (api.cpp / comm.cpp host code)
    exe = _build_abi_selftest(tmp_path)
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present: covered by test_abi_host_code_under_asan_on_gpu")
    _run_abi_selftest(exe, "abi selftest (no GPU): ok")


@pytest.mark.gpu
def test_abi_host_code_under_asan_on_gpu(tmp_path):
    # host code sanitized, kernels as shipped: two ranks (threads) all-reduce through the ABI
    exe = _build_abi_selftest(tmp_path)
    _run_abi_selftest(exe, "abi selftest (GPU): ok")
