#!/usr/bin/env python3
"""Which earlier call makes a later dma-buf export fail?  Round 5's mixed stress at 5 ranks (seed 22)
failed its 4th case: mncclCommRegister of a cached 2 MiB test segment, export refused with
HSA_STATUS_ERROR_OUT_OF_RESOURCES on two of the five ranks.  This runs the stress's first cases
in subsets (one communicator per subset, the stress's own worker), so the trigger is named.

    python tools/r5_export_bisect.py [--ranks 5] [--seed 22] [--first 4] [--subsets "0123 123 023 23 3 13"]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mini-nccl_amd")]


def stress_cases(n, calls, seed):
    """the stress's case list (tools/r4_stress_mixed.py), same draws"""
    import numpy as np
    rng = np.random.default_rng(seed)
    cases = []
    for i in range(calls):
        algo = int(rng.choice([-1, 0, 2, 3, 4]))
        dtype = str(rng.choice(["f32", "f64", "i32", "f16", "bf16"]))
        op = str(rng.choice(["sum", "prod", "max", "min"]))
        count = int(rng.choice([n - 1, n, 77, 1000, 4099, 16384, 65536 + 3, 1 << 18, (1 << 20) + 5, 1 << 22,
                                n << 20]))
        mem = "pinned" if rng.random() < 0.1 else "device"
        cases.append(dict(dtype=dtype, op=op, count=count, inplace=bool(rng.random() < 0.3), algo=algo, calls=1,
                          seed=7000 + i, special=op in ("max", "min"), offset=0, mem=mem,
                          fresh=bool(mem == "device" and rng.random() < 0.2), skew_ms=3,
                          window=bool(mem == "device" and rng.random() < 0.25)))
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=5)
    ap.add_argument("--seed", type=int, default=22)
    ap.add_argument("--first", type=int, default=4)
    ap.add_argument("--subsets", default="0123 123 023 23 3 13")
    a = ap.parse_args()
    import gpu_workers as GW
    n = a.ranks
    cases = stress_cases(n, a.first, a.seed)
    for i, c in enumerate(cases):
        print(f"case {i}: {c}", flush=True)
    env = {"MINI_NCCL_TIMEOUT_MS": "30000", "GPU_MAX_HW_QUEUES": "2"}
    for sub in a.subsets.split():
        picked = [cases[int(ch)] for ch in sub]
        print(f"== subset {sub}", flush=True)
        port = GW.free_port()
        out = GW.run_ranks(GW.allreduce_rank, n, lambda r: (r, n, port, picked, env), 300, barrier=True)
        ok = len(out) == n
        for r in sorted(out):
            o = out[r]
            if "error" in o:
                ok = False
                print(f"   rank {r}: ERROR {o['error'].strip().splitlines()[-1][:200]}", flush=True)
            else:
                bad = [x for x in o["results"] if x["rc"] != 0 or x["bad"] != 0]
                ok = ok and not bad
        print(f"== subset {sub}: {'OK' if ok else 'FAILED'}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
