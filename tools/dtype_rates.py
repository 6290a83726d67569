#!/usr/bin/env python3
"""The element-wise kernel (mncclLocalReduce, the scatter-reduce op) for every dtype x op the
library supports: out = op(a, b) in place over 1 GiB per operand on one MI355X, HIP events
around each launch (20 timed after 5 warm-up), HBM rate = 3 x 1 GiB / kernel time.

    python tools/dtype_rates.py            (GPU box)

Each case is also spot-checked on its first 1 Mi elements against torch (one correctly
rounded op per element; max / min are selections) before timing.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-nccl_amd"))

import torch  # noqa: E402

import mini_nccl as M  # noqa: E402

GIB = 1 << 30
DTYPES = [("f32", torch.float32, M.ncclFloat), ("f64", torch.float64, M.ncclDouble),
          ("i32", torch.int32, M.ncclInt32), ("f16", torch.float16, M.ncclFloat16),
          ("bf16", torch.bfloat16, M.ncclBfloat16)]
OPS = [("sum", M.ncclSum), ("prod", M.ncclProd), ("max", M.ncclMax), ("min", M.ncclMin)]


def ref_op(name, a, b):
    if a.dtype in (torch.float16, torch.bfloat16):
        a32, b32 = a.float(), b.float()
        r = {"sum": a32 + b32, "prod": a32 * b32, "max": torch.where(a32 > b32, a32, b32),
             "min": torch.where(a32 < b32, a32, b32)}[name]
        return r.to(a.dtype)
    return {"sum": a + b, "prod": a * b, "max": torch.where(a > b, a, b), "min": torch.where(a < b, a, b)}[name]


def main():
    M.load()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    out = []
    for dname, tdt, code in DTYPES:
        esz = torch.empty(0, dtype=tdt).element_size()
        count = GIB // esz
        if tdt == torch.int32:
            a = torch.randint(-1000, 1000, (count,), device=dev, dtype=tdt)
            b = torch.randint(-1000, 1000, (count,), device=dev, dtype=tdt)
        else:
            a = torch.rand(count, device=dev, dtype=torch.float32).to(tdt) + 0.5
            b = torch.rand(count, device=dev, dtype=torch.float32).to(tdt) + 0.5
        a0 = a[: 1 << 20].clone()
        for oname, opc in OPS:
            a[: 1 << 20].copy_(a0)
            torch.cuda.synchronize()
            exp = ref_op(oname, a0, b[: 1 << 20])
            rc = M.local_reduce(a.data_ptr(), a.data_ptr(), b.data_ptr(), count, code, opc, st.cuda_stream)
            assert rc == 0, rc
            st.synchronize()
            exact = bool(torch.equal(a[: 1 << 20], exp))
            ms = []
            for i in range(25):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                M.local_reduce(a.data_ptr(), a.data_ptr(), b.data_ptr(), count, code, opc, st.cuda_stream)
                e1.record(st)
                if i >= 5:
                    ms.append((e0, e1))
            st.synchronize()
            t = sum(x.elapsed_time(y) for x, y in ms) / len(ms)
            tbs = 3 * GIB / (t / 1e3) / 1e12
            row = {"dtype": dname, "op": oname, "kernel_ms": round(t, 4), "TBps": round(tbs, 3),
                   "frac_of_8TBps": round(tbs / 8.0, 4), "first_MiEl_exact": exact}
            print(json.dumps(row), flush=True)
            out.append(row)
            a.copy_(b)  # keep values bounded before the next op (prod / sum drift)
        del a, b
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
