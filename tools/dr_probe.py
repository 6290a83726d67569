#!/usr/bin/env python3
"""Diagnostic: which 8-rank read calls stall?  Each variant runs on a fresh set of 8 rank processes
sharing the GPU, 5 s watchdog.  Round 3 found with it that a copy kernel queued in front of the
persistent kernel (the count % n tail, then a hipMemcpyAsync) can stall every co-located rank:
the tail is now copied inside the kernels (kernels.hip copy_tail)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mini-nccl_amd")]


def case(count, inplace=False, dtype="f32", **kw):
    return dict(dtype=dtype, op="sum", count=count, inplace=inplace, algo=2, calls=1, seed=7, special=False, offset=0, **kw)


def main():
    import gpu_workers as GW
    c0 = case(4099, inplace=True)
    c1 = case(1 << 20, dtype="bf16", vary=True)
    c1["calls"] = 2
    c2 = case(77)
    variants = [
        ("c1 then 77 out of place (tail copy)", [c1, c2], {}),
        ("c1 then 72 out of place (no tail)", [c1, case(72)], {}),
        ("c1 then 77 in place (no tail copy)", [c1, case(77, inplace=True)], {}),
        ("c1 then 77 out of place (tail copy), again", [c1, c2], {}),
        ("c1 then 72 out of place (no tail), again", [c1, case(72)], {}),
        ("c1 then 77 in place, again", [c1, case(77, inplace=True)], {}),
    ]
    for name, cases, env in variants:
        e = {"MINI_NCCL_TIMEOUT_MS": "5000", "GPU_MAX_HW_QUEUES": "2", **env}
        port = GW.free_port()
        out = GW.run_ranks(GW.allreduce_rank, 8, lambda r: (r, 8, port, cases, e), 120, barrier=True)
        rcs = [[x["rc"] for x in out[r]["results"]] if r in out and "results" in out[r] else "ERR" for r in range(8)]
        bad = [[x["bad"] for x in out[r]["results"]] if r in out and "results" in out[r] else "ERR" for r in range(8)]
        secs = [[round(x["secs"], 2) for x in out[r]["results"]] if r in out and "results" in out[r] else "ERR"
                for r in range(8)]
        print(f"{name}: rc {rcs} bad {bad} secs {secs}", flush=True)


if __name__ == "__main__":
    main()
