#!/usr/bin/env python3
"""Mixed-schedule stress through the library: N rank processes on one GPU run CALLS all-reduces on
ONE communicator, each call's schedule drawn from auto / ring / read (push form) / one-shot / read's
grid form, a quarter of the device-buffer calls on registered windows (no host rendezvous), its
size from a few bytes to 16 MiB (one-shot's small calls, read's persistent and large slices, the
ring's partial grids), its dtype and op from the whole matrix, in place or not, device / pinned
host buffers, fresh allocations or cached ones, ranks entering out of step (0-3 ms skew) --
every call checked bit-exact against the oracle.  A window registration the library refuses (on
every rank alike: co-located ranks can hit the GPU driver's lost export handles) is
counted and its case runs unregistered.  Schedules share the per-pair FIFO counters,
READY words, credits and slots; any protocol slip shows as a wrong result, a hang (watchdog) or
an error.  One summary line per rank and a verdict.

    python tools/stress_mixed.py [--ranks 8] [--calls 300] [--seed 11]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mini-nccl_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--seed", type=int, default=11)
    a = ap.parse_args()
    import numpy as np
    import gpu_workers as GW
    rng = np.random.default_rng(a.seed)
    n = a.ranks
    cases = []
    for i in range(a.calls):
        algo = int(rng.choice([-1, 0, 2, 3, 4]))
        dtype = str(rng.choice(["f32", "f64", "i32", "f16", "bf16"]))
        op = str(rng.choice(["sum", "prod", "max", "min"]))
        count = int(rng.choice([n - 1, n, 77, 1000, 4099, 16384, 65536 + 3, 1 << 18, (1 << 20) + 5, 1 << 22,
                                n << 20]))
        mem = "pinned" if rng.random() < 0.1 else "device"
        cases.append(dict(dtype=dtype, op=op, count=count, inplace=bool(rng.random() < 0.3), algo=algo, calls=1,
                          seed=7000 + i, special=op in ("max", "min"), offset=0, mem=mem,
                          fresh=bool(mem == "device" and rng.random() < 0.2), skew_ms=3,
                          window=bool(mem == "device" and rng.random() < 0.25), window_optional=True))
    port = GW.free_port()
    # window calls on the device-checked path (auto would negotiate them: the ranks share a GPU)
    env = {"MINI_NCCL_TIMEOUT_MS": "30000", "GPU_MAX_HW_QUEUES": "2", "MINI_NCCL_WINDOW_RENDEZVOUS": "0"}
    out = GW.run_ranks(GW.allreduce_rank, n, lambda r: (r, n, port, cases, env), 2400, barrier=True)
    ok = len(out) == n
    names = {0: "ring", 2: "read", 3: "oneshot", -1: "none"}
    refusals = set()
    for r in sorted(out):
        o = out[r]
        if "error" in o:
            print(f"rank {r}: ERROR {o['error'][-500:]}")
            ok = False
            continue
        res = o["results"]
        bad = [x for x in res if x["rc"] != 0 or x["bad"] != 0 or x["async"] != 0]
        ran = collections.Counter(names.get(x["last_algo"], "?") for x in res)
        last = res[-1]
        refused = sum(1 for x in res if x.get("register_refused"))
        refusals.add(tuple(i for i, x in enumerate(res) if x.get("register_refused")))
        print(f"rank {r}: calls {len(res)}, wrong/failed {len(bad)}, ran {dict(ran)}, windows refused {refused}, "
              f"ipc open failures "
              f"{last['ipc_open_failures']}, read map failures {last['read_map_failures']}, destroy {o['destroy']}")
        for x in bad[:3]:
            print(f"   bad: {x['case']} rc={x['rc']} bad={x['bad']} first={x['first']} {x.get('detail', '')}")
        ok = ok and not bad and last["ipc_open_failures"] == 0 and last["read_map_failures"] == 0 and o["destroy"] == 0
    if len(refusals) > 1:  # registration is collective: every rank refuses the same cases
        print(f"registrations refused on different cases by different ranks: {sorted(refusals)}")
        ok = False
    print("STRESS", "OK" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
