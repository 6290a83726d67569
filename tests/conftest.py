"""Shared pytest setup: the `gpu` marker, import paths and on-demand CPU builds."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mini-nccl_amd")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    # multi-process GPU tests fork their rank processes from a fork server; start it now,
    # before any test initialises HIP in this process (no exec after GPU init)
    import multiprocessing as mp
    import multiprocessing.forkserver as fs
    mp.set_forkserver_preload(["numpy"])
    fs.ensure_running()


def _make(target_dir, *targets):
    subprocess.run(["make", "-s", "-C", target_dir, *targets], check=True)


@pytest.fixture(scope="session")
def oracle_lib():
    """oracle/_build/liboracle.so (test infrastructure: the checker)."""
    import oracle_api
    _make(os.path.join(ROOT, "oracle"))
    return oracle_api.load()


@pytest.fixture(scope="session")
def sim_lib():
    """mini-nccl_amd/lib/libmnccl_sim.so: the kernels' schedule on simulated ranks (CPU)."""
    import sim_api
    _make(PKG, "lib/libmnccl_sim.so")
    return sim_api.load()


@pytest.fixture(scope="session")
def nccl_lib():
    """The product library (loading it needs no GPU)."""
    import mini_nccl
    if not os.path.exists(mini_nccl.LIB_PATH):
        _make(PKG, "lib/libmini_nccl.so")
    return mini_nccl.load()
