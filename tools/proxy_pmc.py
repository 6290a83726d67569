#!/usr/bin/env python3
"""tools/profile_proxy.sh PMC passes (gpurun_out/<tag>/{fetch_n2,write_n2}) -> per-launch HBM bytes
of rank 0's ring kernel on the 2-rank proxy, with the gfx950 corrections (FETCH x2, KiB x1024),
against the fused algorithmic bytes 4 B x chunk x (6n - 4).

  python tools/proxy_pmc.py <tag> <round>     (updates profiles/pmc_summary.json, writes
                                               profiles/<round>_proxy_pmc.csv)
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNT, N = 268435456, 2


def per_dispatch(path, counter):
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if "ring_kernel" in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                rows.append((r["Kernel_Name"], int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return rows


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    base = os.path.join(ROOT, "gpurun_out", tag)
    fetch = per_dispatch(os.path.join(base, "fetch_n2", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(base, "write_n2", "run_counter_collection.csv"), "WRITE_SIZE")
    with open(os.path.join(ROOT, "profiles", f"{rnd}_proxy_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value_KiB"])
        for name, d, v in fetch:
            w.writerow([name, d, "FETCH_SIZE", f"{v:.6f}"])
        for name, d, v in write:
            w.writerow([name, d, "WRITE_SIZE", f"{v:.6f}"])

    def med(rows):
        vals = [v for _, _, v in rows]
        return statistics.median(vals[5:] if len(vals) > 5 else vals)

    rd, wr = med(fetch) * 1024 * 2, med(write) * 1024
    fused = 4 * (COUNT // N) * (6 * N - 4)
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    d = json.load(open(p)) if os.path.exists(p) else {}
    d["ring_f32_1GiB_n2_same_gpu"] = {
        "kernel": fetch[0][0] if fetch else None,
        "read_bytes_per_launch": int(rd), "write_bytes_per_launch": int(wr), "hbm_bytes_per_launch": int(rd + wr),
        "fused_algorithmic_bytes_per_launch": fused, "traffic_over_fused_algorithmic": round((rd + wr) / fused, 4),
        "dispatches": [len(fetch), len(write)],
        "note": "2 ranks sharing ONE MI355X (proxy); rank 0 profiled (perf_test --sizes 1024); medians over the "
                "dispatches after the first 5; the counts match ONE rank's bytes (the other rank process's "
                "concurrent kernel is not in them); fused bytes = 4 B x chunk x (6n-4)",
        "source": f"profiles/{rnd}_proxy_pmc.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                  "FETCH x2, KiB x1024)",
    }
    json.dump(d, open(p, "w"), indent=1, sort_keys=True)
    print(json.dumps(d["ring_f32_1GiB_n2_same_gpu"], indent=1))


if __name__ == "__main__":
    main()
