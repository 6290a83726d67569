#!/usr/bin/env python3
"""PMC passes of tools/profile_proxy_kernels.sh (gpurun_out/<tag>/{fetch,write}_<form>_n<N>) -> per-launch
HBM bytes of rank 0's kernel on the N-rank one-GPU proxy, with the gfx950 corrections (FETCH x2,
KiB x1024, MI355X_MICROARCH.md), against the fused algorithmic bytes of its kernel form (bench.py
fused_bytes: ring (6n-4) chunks, read_push / read_grid 2n), next to the kernel-trace durations.

  python tools/proxy_pmc_n.py <tag> <round> <n> ring read_push read_grid ...
      -> profiles/<round>_proxy_pmc_n<N>.csv, profiles/<round>_proxy_kernel_stats_n<N>.csv,
         and the "<form>_f32_1GiB_n<N>_same_gpu" entries of profiles/pmc_summary.json, each
         carrying its kernel_form (bench.py refuses an entry of another form)
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNT = 268435456  # 1 GiB fp32 per rank


def rows(path, kernel, counter=None):
    out = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if kernel not in r.get("Kernel_Name", ""):
                continue
            if counter is not None and r.get("Counter_Name") != counter:
                continue
            out.append(r)
    return out


def med_after5(vals):
    return statistics.median(vals[5:] if len(vals) > 5 else vals)


def main():
    tag, rnd, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    algos = sys.argv[4:] or ["ring", "read_push"]
    base = os.path.join(ROOT, "gpurun_out", tag)
    def fused_of(form):  # bench.py fused_bytes
        return 4 * (COUNT // n) * {"ring": 6 * n - 4, "read_push": 2 * n, "read_grid": 2 * n}[form]
    summ_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    summ = json.load(open(summ_path)) if os.path.exists(summ_path) else {}
    pmc_csv = os.path.join(ROOT, "profiles", f"{rnd}_proxy_pmc_n{n}.csv")
    st_csv = os.path.join(ROOT, "profiles", f"{rnd}_proxy_kernel_stats_n{n}.csv")
    with open(pmc_csv, "w", newline="") as fp, open(st_csv, "w", newline="") as fs:
        wp, ws = csv.writer(fp), csv.writer(fs)
        wp.writerow(["Algo", "Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value_KiB"])
        ws.writerow(["Algo", "Kernel_Name", "Calls", "median_ns_after_first_5", "MinNs", "MaxNs",
                     "fused_alg_bytes", "fused_GBps_one_rank", "ranks_x_fused_GBps"])
        for algo in algos:
            fused = fused_of(algo)
            # the kernel's template arguments name its form: read_kernel<float, 0, true>
            # (the grid form: its fold grid, read_grid_kernel<float, 0, G, V>; START / DONE are one wave each)
            k = {"ring": "ring_kernel<float, 0, true>", "read_push": "read_kernel<float, 0, true>",
                 "read_grid": "read_grid_kernel<float, 0,"}[algo]
            tr = rows(os.path.join(base, f"trace_{algo}_n{n}", "run_kernel_trace.csv"), k)
            durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
            md = med_after5(durs)
            ws.writerow([algo, tr[0]["Kernel_Name"], len(durs), int(md), min(durs), max(durs), fused,
                         round(fused / md, 2), round(n * fused / md, 2)])
            fe = rows(os.path.join(base, f"fetch_{algo}_n{n}", "run_counter_collection.csv"), k, "FETCH_SIZE")
            wr = rows(os.path.join(base, f"write_{algo}_n{n}", "run_counter_collection.csv"), k, "WRITE_SIZE")
            for r in fe + wr:
                wp.writerow([algo, r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"], r["Counter_Value"]])
            rd = med_after5([float(r["Counter_Value"]) for r in fe]) * 1024 * 2
            wb = med_after5([float(r["Counter_Value"]) for r in wr]) * 1024
            summ[f"{algo}_f32_1GiB_n{n}_same_gpu"] = {
                "kernel": tr[0]["Kernel_Name"], "kernel_form": algo,
                "read_bytes_per_launch": int(rd), "write_bytes_per_launch": int(wb),
                "hbm_bytes_per_launch": int(rd + wb), "fused_algorithmic_bytes_per_launch": fused,
                "traffic_over_fused_algorithmic": round((rd + wb) / fused, 4),
                "kernel_median_ns": int(md),
                "dispatches": [len(fe), len(wr)],
                "note": f"{n} ranks sharing ONE MI355X (proxy); rank 0 profiled (apps/bin/perf_test --sizes 1024, "
                        "default knobs); medians after the first 5 dispatches; fused bytes = 4 B x chunk x (6n-4) for "
                        "the ring, x 2n for the read schedule (either form)",
                "source": f"profiles/{rnd}_proxy_pmc_n{n}.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate "
                          "passes; FETCH x2, KiB x1024)",
            }
            print(algo, json.dumps(summ[f"{algo}_f32_1GiB_n{n}_same_gpu"], indent=1))
    json.dump(summ, open(summ_path, "w"), indent=1, sort_keys=True)
    print(open(st_csv).read())


if __name__ == "__main__":
    main()
