"""bench.py's host-side contract pieces that need no GPU: the crash-line insurance (a process
that dies on a fatal signal after the headline was measured still prints its one JSON line)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(body):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools")], check=True)
    code = ("import os, sys\n"
            f"sys.path.insert(0, {ROOT!r})\n"
            "import bench\n"
            "bench.quiet_stdout()\n" + body)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)


def test_crash_after_arm_prints_the_armed_line_once():
    r = _run("bench.arm({'value': 1.0, 'step': 'a'})\n"
             "bench.arm({'value': 2.0, 'step': 'b'})\n"
             "os.abort()\n")
    assert r.returncode == -6
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    assert json.loads(lines[0]) == {"value": 2.0, "step": "b"}


def test_emit_disarms_so_a_later_crash_prints_nothing_more():
    r = _run("bench.arm({'value': 1.0})\n"
             "bench.emit({'value': 3.0})\n"
             "os.kill(os.getpid(), 11)\n")
    assert r.returncode == -11
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert [json.loads(x) for x in lines] == [{"value": 3.0}]


def test_banners_on_fd1_go_to_stderr():
    r = _run("os.write(1, b'native banner\\n')\n"
             "bench.emit({'value': 4.0})\n")
    assert r.returncode == 0
    assert r.stdout.strip() == json.dumps({"value": 4.0})
    assert "native banner" in r.stderr


def test_sigterm_after_arm_prints_the_armed_line():
    # a launcher's time limit during the extras still leaves the headline on stdout
    r = _run("bench.arm({'value': 5.0})\n"
             "os.kill(os.getpid(), 15)\n"
             "import time; time.sleep(5)\n")
    assert r.returncode == -15
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert [json.loads(x) for x in lines] == [{"value": 5.0}]


class _FakeComm:
    """An all-reduce whose result comes from `result(xs)` (the oracle's ring, or a wrong order)."""

    def __init__(self, torch, rank, n, send, recv, result):
        self.torch, self.rank, self.n, self.send, self.recv, self.result = torch, rank, n, send, recv, result

    def all_reduce(self, sp, rp, count, dt, op, stream):
        import bench
        torch, n = self.torch, self.n
        xs = []
        for q in range(n):  # every rank's input, drawn as verify_order's ranks draw theirs
            g = torch.Generator(device="cpu")
            g.manual_seed(1234 + q)
            x = torch.empty(count)
            for _, a, b in bench.order_ranges(count, n):
                x[a:b] = torch.rand(b - a, generator=g, dtype=torch.float32) * 2 - 1
            xs.append(x.numpy())
        assert (xs[self.rank] == self.send.numpy()).all()
        self.recv.copy_(torch.from_numpy(self.result(xs)[self.rank]))
        return 0

    def async_error(self):
        return 0


def _verify_order_with(monkeypatch, result, n=4, count=4 * 1000 + 3, rank=1):
    import torch

    import bench

    class _Stream:
        cuda_stream = 0

    class _M:
        ncclSum = 0
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)  # CPU tensors: nothing to wait for
    send, recv = torch.empty(count), torch.empty(count)
    comm = _FakeComm(torch, rank, n, send, recv, result)
    return bench.verify_order(_M, torch, comm, torch.device("cpu"), n, rank, send, recv, count, torch.float32,
                              0, _Stream(), lambda: None)


def test_verify_order_accepts_the_reference_ring_association(oracle_lib, monkeypatch):
    # bench.py's order-sensitive check (torch adds in the ring's association) agrees
    # with the oracle's loop-by-loop restatement of mini_nccl.cu:108-194 on seeded uniform data
    import oracle_api as O
    assert _verify_order_with(monkeypatch, lambda xs: O.allreduce(xs, "f32", "sum")) == "ok"


def test_verify_order_rejects_another_association(oracle_lib, monkeypatch):
    import numpy as np

    # the same sums folded from rank 0 for every chunk (a plain left fold): other bits somewhere
    def left_fold(xs):
        acc = xs[0].copy()
        for x in xs[1:]:
            acc = (acc + x).astype(np.float32)
        n, count = len(xs), xs[0].size
        out = []
        for r in range(n):
            y = acc.copy()
            y[(count // n) * n:] = xs[r][(count // n) * n:]
            out.append(y)
        return out
    assert _verify_order_with(monkeypatch, left_fold).startswith("FAILED: element")


def test_size_curve_columns_merge_into_one_row_per_size(monkeypatch):
    # bench.py measures its own column of the perf_test sizes right after the schedules and RCCL's
    # column among the extras (after the link probes, which slowed later co-located small calls,
    # profiles/r5_bench_size_order.txt): the second pass adds to the first's rows, one per size
    import torch
    import torch.distributed as tdist

    import bench

    n, calls = 2, {"ours": 0, "rccl": 0}

    class _Comm:
        def all_reduce(self, s, r, k, dt, op, st):
            calls["ours"] += 1
            recv[:k] = float(n)
            return 0

        def async_error(self):
            return 0

        def info(self):
            return {"last_algo": 2}

    class _Dist:
        @staticmethod
        def barrier():
            pass

    class _Stream:
        cuda_stream = 0

    class _M:
        ncclFloat, ncclSum = 0, 0

        class NcclError(Exception):
            pass

    def rccl(t, group=None):
        calls["rccl"] += 1

    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    monkeypatch.setattr(tdist, "all_reduce", rccl)
    send, recv = torch.ones(4 << 20), torch.empty(4 << 20)  # 16 MiB: the 1 and 16 MiB points
    rows = bench.size_curve(_M, torch, _Dist, _Comm(), None, send, recv, _Stream(), n, lambda x: x, who=("mini_nccl",))
    assert [r["MiB"] for r in rows] == [1, 16] and all(r["ok"] and "mini_nccl_us" in r for r in rows)
    assert all("rccl_us" not in r for r in rows) and calls["rccl"] == 0
    ours = calls["ours"]
    out = bench.size_curve(_M, torch, _Dist, _Comm(), object(), send, recv, _Stream(), n, lambda x: x, who=("rccl",),
                           rows=rows)
    assert out is rows and [r["MiB"] for r in rows] == [1, 16]
    assert all("rccl_us" in r and "mini_nccl_us" in r for r in rows)
    assert calls["ours"] == ours and calls["rccl"] == 2 * (5 + 20)  # RCCL's pass leaves this library alone


def test_run_sweeps_stops_alike_at_its_budget(monkeypatch):
    # the sweep keeps LINK_RESERVE_S of the extras' time for the link probes that run after it:
    # past its deadline every rank stops before its next point (agreed through max_over_ranks)
    import time

    import bench

    seen = []

    def fake_point(M, torch, dist, dev, n, rank, env, algo, count, reps, max_over_ranks, dtype="f32"):
        seen.append((algo, dict(env)))
        return {"GBps": 1.0, "ok": True}

    monkeypatch.setattr(bench, "sweep_point", fake_point)
    out = bench.run_sweeps(None, None, None, None, 2, 0, lambda x: x, with_c4=False, out={}, deadline=None)
    assert len(seen) == len(bench.SWEEP_POINTS) + len(bench.MID_POINTS) and "stopped" not in out
    seen.clear()
    out = bench.run_sweeps(None, None, None, None, 2, 0, lambda x: x, with_c4=True, out={},
                           deadline=time.time() - 1)
    assert seen == [] and "stopped" in out
    # a peer past its deadline stops this rank too (max over ranks of the flag)
    seen.clear()
    out = bench.run_sweeps(None, None, None, None, 2, 0, lambda x: 1.0, with_c4=False, out={},
                           deadline=time.time() + 3600)
    assert seen == [] and "stopped" in out


# ------------------------------------------------------------------ the self-launch
def test_launch_plan_decisions():
    import bench
    assert bench.launch_plan(1, None, 0, False) == ("ranks", None)      # N = 1: this process
    assert bench.launch_plan(8, "8", 8, False) == ("ranks", None)       # a launcher set WORLD_SIZE
    assert bench.launch_plan(8, None, 8, False) == ("spawn", None)      # no launcher: 8 rank processes
    assert bench.launch_plan(2, None, 1, True) == ("spawn", None)       # the one-GPU rehearsal
    kind, why = bench.launch_plan(8, None, 1, False)                    # never a silent co-location
    assert kind == "error" and "--gpus 8" in why and "1 GPU(s) visible" in why


def test_spawn_ranks_sets_the_launcher_env_and_keeps_rank0_line():
    sys.path.insert(0, ROOT)
    import bench
    child = ("import json, os\n"
             "if os.environ['RANK'] == '0':\n"
             "    print('banner before the line')\n"
             "    print(json.dumps({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR')}))\n"
             "else:\n"
             "    print(json.dumps({'rank': os.environ['RANK']}))\n")
    rc, line = bench.spawn_ranks([sys.executable, "-c", child], 3, timeout=60)
    assert rc == 0
    assert json.loads(line) == {"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "3", "MASTER_ADDR": "127.0.0.1"}


def test_spawn_ranks_ends_the_rest_when_a_rank_fails():
    sys.path.insert(0, ROOT)
    import bench
    child = ("import os, sys, time\n"
             "if os.environ['RANK'] == '1':\n"
             "    sys.exit(3)\n"
             "time.sleep(120)\n")
    t0 = __import__("time").time()
    rc, line = bench.spawn_ranks([sys.executable, "-c", child], 2, timeout=60, grace=1.0)
    assert rc == 3 and line is None
    assert __import__("time").time() - t0 < 30


def test_bench_gpus_n_without_enough_gpus_prints_one_error_line():
    # this container has no GPU: `python3 bench.py --gpus 4` (no launcher) must neither co-locate
    # nor fall back to N = 1 -- one line, value 0, the reason, exit status 2
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=300, cwd=ROOT, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert r.returncode == 2, r.stderr[-2000:]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 0.0 and d["n_gpus"] == 4 and "GPU(s) visible" in d["error"]


def test_summarize_proxy_line():
    # proxy_allreduce's reading of the rank processes' --core-only line
    sys.path.insert(0, ROOT)
    import bench

    def sched(v, ok="ok", order="ok"):
        return {"value": v, "ms_per_step": 1.0, "kernel_ms": 0.9, "result_check": ok,
                "roofline": {"frac": 0.2, "fused_frac": 0.35}, "verify": {"order_sensitive": order}}

    line = {"config": {"algo": "read_grid"}, "schedules": {"ring": sched(800.0), "read_grid": sched(1400.0)}}
    s = bench.summarize_proxy(line, 2, 0)
    assert s["ok"] and s["default"]["schedule"] == "read_grid" and s["ring"]["GBps"] == 800.0
    assert s["default"]["fused_frac_all_ranks"] == 0.7
    line["schedules"]["read_grid"] = sched(1400.0, order="FAILED: element 3")
    assert not bench.summarize_proxy(line, 2, 0)["ok"]
    assert not bench.summarize_proxy({"error": "boom"}, 2, 1)["ok"]
    assert not bench.summarize_proxy({"config": {"algo": "read"}, "schedules": {"ring": sched(1.0)}}, 2, 0)["ok"]


def test_spawned_ranks_die_with_a_killed_launcher(tmp_path):
    # a launcher stopped at its time limit (SIGKILL: no handler runs) must not leave rank processes
    # behind holding the GPU: every rank gets SIGTERM from the kernel when its parent dies
    import signal
    import time
    pidfile = tmp_path / "pids"
    child = ("import os, sys, time\n"
             f"sys.path.insert(0, {ROOT!r})\n"
             "import bench\n"
             "bench.die_with_parent()\n"  # what bench.py's main() does first
             f"open({str(pidfile)!r}, 'a').write(str(os.getpid()) + '\\n')\n"
             "time.sleep(120)\n")
    parent = ("import sys\n"
              f"sys.path.insert(0, {ROOT!r})\n"
              "import bench\n"
              f"bench.spawn_ranks([sys.executable, '-c', {child!r}], 2, timeout=100)\n")
    p = subprocess.Popen([sys.executable, "-c", parent])
    for _ in range(200):
        if pidfile.exists() and len(pidfile.read_text().split()) == 2:
            break
        time.sleep(0.05)
    pids = [int(x) for x in pidfile.read_text().split()]
    os.kill(p.pid, signal.SIGKILL)
    p.wait()
    deadline = time.time() + 10
    alive = pids
    while alive and time.time() < deadline:
        alive = []
        for pid in pids:
            try:
                os.kill(pid, 0)
                st = open(f"/proc/{pid}/stat").read().split()[2]
                if st != "Z":
                    alive.append(pid)
            except (ProcessLookupError, FileNotFoundError):
                pass
        time.sleep(0.1)
    assert not alive, f"rank processes {alive} outlived their launcher"
