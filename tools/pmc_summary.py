#!/usr/bin/env python3
"""Turn a tools/profile_n1.sh run (gpurun_out/<tag>/) into committed evidence under profiles/.

  python tools/pmc_summary.py <tag> <round>      e.g. prof_n1_r6 r6

Writes (<head>: the commit tools/profile_n1.sh was given, gpurun_out/<tag>/head.txt)
  profiles/<round>_n1_<head>_kernel_stats.csv  rocprofv3 --kernel-trace --stats of bench.py's headline
                                          (the kernel rows of this library, plus every row's totals)
  profiles/<round>_n1_<head>_line_traced.json  the bench line printed by that same traced process
  profiles/<round>_n1_<head>_line_plain.json   `python3 bench.py --gpus 1` in the same lease
  profiles/<round>_n1_<head>_pmc.csv     per-dispatch FETCH_SIZE / WRITE_SIZE of this library's kernels
  profiles/pmc_summary.json              per-launch HBM bytes read by bench.py's roofline.traffic, and
                                          the trace's mean launch (roofline.kernel_source)

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in KiB
(x 1024); FETCH_SIZE counts exactly half of the bytes of a wide coalesced streaming read
(16 B per lane), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


GRID_1GIB = (268435456 * 4) // 16  # threads of local_reduce_vec's exact grid over 1 GiB (one 16-B vector each)


def ours(name):
    return "mnccl::" in name


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    src = os.path.join(ROOT, "gpurun_out", tag)
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)

    head = open(os.path.join(src, "head.txt")).read().strip()
    stem = f"{rnd}_n1_{head}"
    stats = rows(os.path.join(src, "trace", "run_kernel_stats.csv"))
    lines = {}
    for which in ("traced", "plain"):
        txt = [ln for ln in open(os.path.join(src, f"line_{which}.json")).read().splitlines() if ln.startswith("{")]
        lines[which] = json.loads(txt[-1])
        with open(os.path.join(prof, f"{stem}_line_{which}.json"), "w") as f:
            f.write(txt[-1] + "\n")
    trace_mean = None
    with open(os.path.join(prof, f"{stem}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        other = [0, 0.0, 0.0]
        for r in stats:
            if ours(r["Name"]):
                if "local_reduce_vec<float, 0>" in r["Name"]:
                    trace_mean = float(r["AverageNs"])
                w.writerow([r["Name"], r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["Percentage"], r["MinNs"],
                            r["MaxNs"], r["StdDev"]])
            else:
                other[0] += int(r["Calls"])
                other[1] += float(r["TotalDurationNs"])
                other[2] += float(r["Percentage"])
        w.writerow(["(all other kernels: torch fills / checks)", other[0], int(other[1]), "", round(other[2], 2), "", "",
                    ""])

    per = {}
    pmc_rows = []
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        for r in rows(os.path.join(src, sub, "run_counter_collection.csv")):
            if ours(r["Kernel_Name"]) and r["Counter_Name"] == counter:
                # per-launch bytes of the 1 GiB launch only (exact grid: 2^26 threads); smaller
                # launches of the same kernel (e.g. bench's host-inclusive pieces) stay in the CSV
                if int(r["Grid_Size"]) == GRID_1GIB:
                    per.setdefault((r["Kernel_Name"], counter), []).append(float(r["Counter_Value"]))
                pmc_rows.append([r["Kernel_Name"], r["Dispatch_Id"], r["Grid_Size"], r["Workgroup_Size"],
                                 r["VGPR_Count"], r["SGPR_Count"], counter, r["Counter_Value"]])
    with open(os.path.join(prof, f"{stem}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Grid_Size", "Workgroup_Size", "VGPR_Count", "SGPR_Count",
                    "Counter_Name", "Counter_Value_KiB"])
        w.writerows(pmc_rows)

    out_path = os.path.join(prof, "pmc_summary.json")
    summary = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for kname in sorted({k for k, _ in per}):
        if "local_reduce_vec<float, 0>" not in kname:
            continue
        fetch = per.get((kname, "FETCH_SIZE"), [])
        write = per.get((kname, "WRITE_SIZE"), [])
        f_b = 2 * 1024 * sum(fetch) / len(fetch)
        w_b = 1024 * sum(write) / len(write)
        alg = 3 * 268435456 * 4
        summary["local_reduce_f32_1GiB"] = {
            "kernel": kname,
            "hbm_bytes_per_launch": int(round(f_b + w_b)),
            "read_bytes_per_launch": int(round(f_b)),
            "write_bytes_per_launch": int(round(w_b)),
            "algorithmic_bytes_per_launch": alg,
            "kernel_form": "local_reduce",
            "traffic_over_algorithmic": round((f_b + w_b) / alg, 4),
            "dispatches": [len(fetch), len(write)],
            "source": f"profiles/{stem}_pmc.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                      "FETCH x2 and KiB x1024 per MI355X_MICROARCH.md)",
            "head": head,
            "trace_source": f"profiles/{stem}_kernel_stats.csv",
            "trace_mean_ns": trace_mean,
            "paired_line": f"profiles/{stem}_line_traced.json",
        }
        t = lines["traced"]
        rf = t.get("roofline", {})
        summary["local_reduce_f32_1GiB"]["pairing"] = {
            "line_ms_per_step": t.get("ms_per_step"), "line_kernel_ms": rf.get("kernel_ms"),
            "line_frac": rf.get("frac"), "trace_kernel_ms": round(trace_mean / 1e6, 4),
            "trace_frac": round(alg / (trace_mean / 1e9) / 1e9 / 8000.0, 4),
            "trace_mean_le_step": trace_mean / 1e6 <= t.get("ms_per_step", 0),
            "frac_rel_diff": round(abs(alg / (trace_mean / 1e9) / 1e9 / 8000.0 - rf.get("frac", 0)) / rf.get("frac", 1), 4),
        }
    json.dump(summary, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
