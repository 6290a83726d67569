#!/usr/bin/env python3
"""tools/profile_proxy.sh output (gpurun_out/<tag>/) -> profiles/<round>_proxy_kernel_stats.csv:
per schedule kernel of rank 0, calls / mean / min / max and the median after the first 5
dispatches (the first ones include waiting for the other rank processes to start).

  python tools/proxy_stats.py <tag> <round>
"""
import csv
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [("trace_n2", "2 ranks on one GPU, 1 GiB fp32, perf_test rank 0, library defaults"),
          ("trace_n4", "4 ranks on one GPU, 1 GiB fp32, perf_test rank 0, library defaults (auto-tune at init)")]


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    out = os.path.join(ROOT, "profiles", f"{rnd}_proxy_kernel_stats.csv")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Config", "Name", "Calls", "AverageNs", "MinNs", "MaxNs", "median_ns_after_first_5", "note"])
        for pas, cfg in PASSES:
            path = os.path.join(ROOT, "gpurun_out", tag, pas, "run_kernel_trace.csv")
            by = {}
            with open(path, newline="") as g:
                for r in csv.DictReader(g):
                    if "mnccl::" in r["Kernel_Name"]:
                        by.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for name, ds in by.items():
                tail = ds[5:] if len(ds) > 5 else ds
                note = "first call includes waiting for the other ranks to start (max)" if len(ds) > 5 else \
                    "auto-tune calls at init (64 MiB)"
                w.writerow([cfg, name, len(ds), f"{statistics.mean(ds):.1f}", min(ds), max(ds),
                            int(statistics.median(tail)), note])
    print(open(out).read())


if __name__ == "__main__":
    main()
