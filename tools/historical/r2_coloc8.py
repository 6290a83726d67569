"""8 rank processes on ONE GPU (the reference perf_test topology) through the Python binding, at
the library defaults (256 pipelines, 10 s watchdog): does each schedule / dtype complete, how
long does each call take, and is it bit-exact against the oracle.  One JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mini-nccl_amd")]


def main():
    import multiprocessing.forkserver as fs
    fs.ensure_running()
    import gpu_workers as GW
    cases = [("ring_f32", dict(dtype="f32", op="sum", count=(1 << 20) + 5, inplace=False, algo=0, calls=1, seed=8)),
             ("direct_f32", dict(dtype="f32", op="sum", count=(1 << 20) + 5, inplace=False, algo=1, calls=1, seed=8)),
             ("ring_f16", dict(dtype="f16", op="sum", count=(1 << 20) + 3, inplace=True, algo=0, calls=1, seed=9)),
             ("direct_f16", dict(dtype="f16", op="sum", count=(1 << 20) + 3, inplace=True, algo=1, calls=1, seed=9))]
    extra = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
    for name, c in cases:
        port = GW.free_port()
        env = {"MINI_NCCL_TUNE": "0"}
        env.update(extra)
        t0 = time.time()
        out = GW.run_ranks(GW.allreduce_rank, 8, lambda r: (r, 8, port, [c], env), 90)
        res = {"case": name, "env": extra, "wall_s": round(time.time() - t0, 2), "ranks": len(out)}
        errs = [out[r]["error"][-300:] for r in out if "error" in out[r]]
        if errs:
            res["error"] = errs[0]
        else:
            rs = [out[r]["results"][0] for r in sorted(out)]
            res.update(rc=[x["rc"] for x in rs], bad=[x["bad"] for x in rs], secs=[round(x["secs"], 3) for x in rs])
        print(json.dumps(res), flush=True)
        if len(out) < 8 or errs:
            sys.exit(3)


if __name__ == "__main__":
    main()
