#!/usr/bin/env python3
"""Stress of the read schedule's IPC lifecycle through the library (not the probe): N rank
processes on one GPU run CALLS read calls of changing size / dtype / placement, a third of them
on fresh hipMalloc'd buffers that are freed after the call (addresses come back, owners report
frees, peers close imports), the rest from the caching allocator; every call checked bit-exact
against the oracle.  Prints one summary line per rank and a verdict.

    python tools/r3_stress_read.py [--ranks 8] [--calls 200]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mini-nccl_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    import numpy as np
    import gpu_workers as GW
    rng = np.random.default_rng(7)
    cases = []
    for i in range(a.calls):
        count = int(rng.choice([77, 4099, 65536 + 3, 1 << 18, (1 << 20) + 5, 3 << 20, 1 << 22]))
        cases.append(dict(dtype=("f32", "bf16", "f16")[i % 3], op="sum", count=max(count, a.ranks), inplace=bool(i % 4 == 0),
                          algo=2, calls=1, seed=5000 + i, special=False, offset=0, fresh=bool(i % 3 == 1)))
    port = GW.free_port()
    env = {"MINI_NCCL_TIMEOUT_MS": "30000", "GPU_MAX_HW_QUEUES": "2"}
    out = GW.run_ranks(GW.allreduce_rank, a.ranks, lambda r: (r, a.ranks, port, cases, env), 1800, barrier=True)
    ok = len(out) == a.ranks
    for r in sorted(out):
        o = out[r]
        if "error" in o:
            print(f"rank {r}: ERROR {o['error'][-500:]}")
            ok = False
            continue
        res = o["results"]
        bad = sum(1 for x in res if x["rc"] != 0 or x["bad"] != 0 or x["async"] != 0)
        reads = sum(1 for x in res if x["last_algo"] == 2)
        fresh_reads = sum(1 for x in res if x["last_algo"] == 2 and x["case"]["fresh"])
        last = res[-1]
        print(f"rank {r}: calls {len(res)}, wrong/failed {bad}, read {reads} (on fresh allocations {fresh_reads}), "
              f"ring {len(res) - reads}, ipc open failures {last['ipc_open_failures']}, read map failures "
              f"{last['read_map_failures']}, imports closed on owner frees {last['closed_freed']}, "
              f"max imports {max(x['peer_mappings'] for x in res)}, destroy {o['destroy']}")
        ok = ok and bad == 0 and last["ipc_open_failures"] == 0 and last["read_map_failures"] == 0 and o["destroy"] == 0
    print("STRESS", "OK" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
