#!/usr/bin/env python3
"""Summary of tools/r4_read_counters.sh: per config (schedule, ranks), the median per launch of
every counter over the all-reduce kernel's launches on rank 0, and derived figures.

Usage: r4_counters_summary.py <dir> [out.json]
Derived (per launch, rank 0's kernel, while the other rank processes' kernels run beside it):
  * vmem_latency_cycles = SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM (SQ counters are per wave-cycle
    samples: mean cycles a vector-memory instruction is outstanding);
  * ea_rd_latency / ea_wr_latency = TCC_EA0_{RD,WR}REQ_LEVEL / TCC_EA0_{RD,WR}REQ (cycles a
    request to memory is outstanding at the L2's memory-side interface);
  * tcp_rd_latency / tcp_wr_latency = TCP_TCC_{READ,WRITE}_REQ_LATENCY / TCP_TCC_{READ,WRITE}_REQ;
  * *_per_cycle = a counter / GRBM_GUI_ACTIVE (the kernel's busy cycles).
"""
import csv
import glob
import json
import os
import statistics
import sys


def launches(path, kernel_sub):
    """{dispatch_id: {counter: value}} of the kernels whose name contains kernel_sub."""
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub not in row["Kernel_Name"]:
                    continue
                d = out.setdefault(row["Dispatch_Id"], {})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                d["_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return out


def main():
    root = sys.argv[1]
    res = {}
    for cfg_dir in sorted(glob.glob(os.path.join(root, "*_n*_p*"))):
        if not os.path.isdir(cfg_dir):
            continue
        name = os.path.basename(cfg_dir)
        cfg = name.rsplit("_p", 1)[0]
        algo = cfg.split("_")[0]
        L = launches(cfg_dir, {"read": "read_kernel", "ring": "ring_kernel", "mix": "mix2"}[algo])
        # the timed launches only: drop the first (warm-up) ones, keep the 1 GiB calls
        vals = {}
        for d in L.values():
            for k, v in d.items():
                vals.setdefault(k, []).append(v)
        agg = res.setdefault(cfg, {"launches": 0})
        agg["launches"] = max(agg["launches"], len(L))
        for k, v in vals.items():
            if k == "_ns":
                agg.setdefault("kernel_ns_median", statistics.median(v))
            else:
                agg[k] = statistics.median(v)
    for cfg, a in res.items():
        def g(k):
            return a.get(k)
        der = {}
        vm = (g("SQ_INSTS_VMEM_RD") or 0) + (g("SQ_INSTS_VMEM_WR") or 0)
        if g("SQ_INST_LEVEL_VMEM") and vm:
            der["vmem_latency_cycles"] = g("SQ_INST_LEVEL_VMEM") / vm
        for kind in ("RD", "WR"):
            lv, rq = g(f"TCC_EA0_{kind}REQ_LEVEL_sum"), g(f"TCC_EA0_{kind}REQ_sum")
            if lv and rq:
                der[f"ea_{kind.lower()}_latency_cycles"] = lv / rq
        for kind in ("READ", "WRITE"):
            lt, rq = g(f"TCP_TCC_{kind}_REQ_LATENCY_sum"), g(f"TCP_TCC_{kind}_REQ_sum")
            if lt and rq:
                der[f"tcp_{kind.lower()}_latency_cycles"] = lt / rq
        gui = g("GRBM_GUI_ACTIVE")
        if gui:
            for k in ("TCC_EA0_WRREQ_STALL_sum", "TCC_TOO_MANY_EA_WRREQS_STALL_sum", "TCC_TAG_STALL_sum",
                      "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum",
                      "TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum", "TA_TA_BUSY_sum",
                      "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TD_TC_STALL_sum", "TCC_BUSY_sum",
                      "TCC_EA0_RDREQ_LEVEL_sum", "TCC_EA0_WRREQ_LEVEL_sum"):
                if g(k) is not None:
                    der[k.replace("_sum", "") + "_per_cycle"] = g(k) / gui
        if g("SQ_WAVE_CYCLES") and g("SQ_WAIT_INST_ANY") is not None:
            der["wait_inst_any_frac"] = g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES")
        if g("SQ_WAVE_CYCLES") and g("SQ_ACTIVE_INST_VMEM") is not None:
            der["active_vmem_frac"] = g("SQ_ACTIVE_INST_VMEM") / g("SQ_WAVE_CYCLES")
        for kind in ("RD", "WR"):  # requests the L2 sent to DRAM vs all its memory-side requests (MALL hits)
            dr, rq = g(f"TCC_EA0_{kind}REQ_DRAM_sum"), g(f"TCC_EA0_{kind}REQ_sum")
            if dr is not None and rq:
                der[f"ea_{kind.lower()}_dram_fraction"] = dr / rq
        if g("FETCH_SIZE") is not None:
            der["fetch_bytes"] = g("FETCH_SIZE") * 1024 * 2  # KiB; gfx950 FETCH x2 (MI355X_MICROARCH.md)
        if g("WRITE_SIZE") is not None:
            der["write_bytes"] = g("WRITE_SIZE") * 1024
        a["derived"] = der
    txt = json.dumps(res, indent=1, sort_keys=True)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
