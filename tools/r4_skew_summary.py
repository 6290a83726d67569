#!/usr/bin/env python3
"""Summary of tools/r4_skew_trace.sh: per config, the all-reduce kernels of every rank matched by
call (k-th launch on each rank), and per call

  skew_us      = latest start - earliest start (the ranks' kernels do not start together);
  span_us      = latest end - earliest start;
  all_in_us    = latest end - latest start (every rank's kernel running);
  rank0_us     = rank 0's kernel duration (what a per-rank kernel trace reports).

Rates over the GPU (the proxy's n ranks share one HBM): n x fused bytes / rank0 time, and over
the all-in window, against the pure-stream ceiling of the same read:write mix (tools/mix_probe).

Usage: r4_skew_summary.py <dir> [out.json]
"""
import csv
import glob
import json
import os
import statistics
import sys

COUNT = 268435456


def fused(form, n):
    return 4 * (COUNT // n) * {"ring": 6 * n - 4, "read": 2 * n}[form]


def main():
    root = sys.argv[1]
    res = {}
    for d in sorted(glob.glob(os.path.join(root, "*_n*"))):
        if not os.path.isdir(d):
            continue
        name = os.path.basename(d)
        algo, n = name.split("_n")[0], int(name.split("_n")[1])
        per_rank = []
        for r in range(n):
            f = glob.glob(os.path.join(d, f"r{r}", "**", "*kernel_trace.csv"), recursive=True)
            if not f:
                break
            rows = [x for x in csv.DictReader(open(f[0])) if f"{algo}_kernel" in x["Kernel_Name"]]
            rows.sort(key=lambda x: int(x["Start_Timestamp"]))
            per_rank.append([(int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in rows])
        if len(per_rank) != n:
            continue
        calls = min(len(x) for x in per_rank)
        sk, sp, ai, r0 = [], [], [], []
        for k in range(2, calls):  # the timed calls (after perf_test's 2 warm-ups)
            st = [per_rank[r][k][0] for r in range(n)]
            en = [per_rank[r][k][1] for r in range(n)]
            sk.append((max(st) - min(st)) / 1e3)
            sp.append((max(en) - min(st)) / 1e3)
            ai.append((max(en) - max(st)) / 1e3)
            r0.append((per_rank[0][k][1] - per_rank[0][k][0]) / 1e3)
        b = fused(algo, n)
        med = statistics.median
        res[name] = {
            "calls": len(sk), "skew_us_median": round(med(sk), 1), "skew_us_max": round(max(sk), 1),
            "span_us_median": round(med(sp), 1), "all_in_us_median": round(med(ai), 1),
            "rank0_kernel_us_median": round(med(r0), 1), "fused_bytes_per_rank": b,
            "gpu_TBps_over_rank0_kernel": round(n * b / (med(r0) * 1e-6) / 1e12, 3),
            "gpu_TBps_over_all_in_window": round(n * b / (med(ai) * 1e-6) / 1e12, 3),
        }
    txt = json.dumps(res, indent=1, sort_keys=True)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
