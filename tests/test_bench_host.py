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
