"""Debug helper (not a test): run a list of all-reduce cases on N rank processes sharing GPU 0
and print per-rank results and timings."""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mini-nccl_amd")]
import multiprocessing as mp  # noqa: E402

import gpu_workers as GW  # noqa: E402


def case(dtype="f32", op="sum", count=1 << 18, inplace=False, algo=0, calls=1, seed=1234):
    return dict(dtype=dtype, op=op, count=count, inplace=inplace, algo=algo, calls=calls, seed=seed, special=False,
                offset=0)


if __name__ == "__main__":
    mp.set_forkserver_preload(["numpy"])
    n = int(sys.argv[1])
    spec = json.loads(sys.argv[2])
    env = {"MINI_NCCL_TIMEOUT_MS": "15000"}
    env.update(json.loads(sys.argv[3]) if len(sys.argv) > 3 else {})
    cases = [case(**c) for c in spec]
    port = GW.free_port()
    out = GW.run_ranks(GW.allreduce_rank, n, lambda r: (r, n, port, cases, env), 120)
    for r in sorted(out):
        if "error" in out[r]:
            print(r, out[r]["error"][-800:])
            continue
        print(r, [(x["case"]["dtype"], x["case"]["inplace"], x["case"]["algo"], x["rc"], x["bad"], round(x["secs"], 3))
                  for x in out[r]["results"]])
