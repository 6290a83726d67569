#!/usr/bin/env python3
"""One table from bench lines, wherever they are: the driver's BENCH_rNN.json / SCALE_rNN.json
(the line inside run.stdout_tail, or a list / dict of such runs), or a file holding the JSON line
itself (profiles/r4_bench_n*_same_gpu.json).  Per line: N, value, the schedules' values and
result checks, headline_check, link fractions, RCCL on the same buffer, small calls by schedule,
fallbacks -- what deciding the node's defaults needs.

    python tools/bench_summary.py BENCH_r04.json SCALE_r04.json profiles/r4_bench_n8_same_gpu.json
"""
import json
import sys


def lines_in(obj):
    """every bench JSON line found in a parsed driver record (recursively)"""
    if isinstance(obj, dict):
        if "metric" in obj and "value" in obj:
            yield obj
            return
        for v in obj.values():
            yield from lines_in(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from lines_in(v)
    elif isinstance(obj, str) and '"metric"' in obj:
        for ln in obj.splitlines():
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                try:
                    yield json.loads(ln)
                except ValueError:
                    pass


def load(path):
    text = open(path).read()
    try:
        return list(lines_in(json.loads(text)))
    except ValueError:
        return list(lines_in(text))


def show(path, d):
    c = d.get("config", {})
    sch = {k: (v.get("value"), v.get("result_check")) for k, v in d.get("schedules", {}).items()}
    hc = c.get("headline_check", {})
    link = d.get("link", {})
    print(f"{path}: N={d.get('n_gpus')} value={d.get('value')} {d.get('unit')} check={c.get('result_check', '-')!s:.40}")
    print(f"   workload: {c.get('workload', '-')}")
    if sch:
        print(f"   schedules: {sch}; headline_check holds={hc.get('holds')} read/ring={hc.get('read_over_ring')}")
    r = d.get("roofline", {})
    print(f"   roofline: frac={r.get('frac')} fused_frac={r.get('fused_frac')} kernel_ms={r.get('kernel_ms')} "
          f"traffic={r.get('traffic')} note={r.get('traffic_note')}")
    if link:
        print("   link: " + ", ".join(f"{k}={v}" for k, v in link.items() if "frac" in k or k.startswith("probe_")))
    if "rccl_reference" in d:
        print(f"   rccl_reference: {d['rccl_reference']}")
    if "small_calls" in d:
        print(f"   small_calls: {d['small_calls']}")
    if c.get("fallbacks"):
        print(f"   FALLBACKS: {c['fallbacks']}")
    cb = d.get("cpu_baseline") or {}
    print(f"   cpu_baseline: {cb.get('value')} {cb.get('unit')} ({cb.get('kind')}, {cb.get('cores')} cores)")


def main():
    for p in sys.argv[1:]:
        found, seen = [], set()
        for d in load(p):  # a driver record may hold the same line twice (tail and parsed)
            key = json.dumps(d, sort_keys=True)
            if key not in seen:
                seen.add(key)
                found.append(d)
        if not found:
            print(f"{p}: no bench line ({open(p).read()[:160]!r})")
        for d in found:
            show(p, d)


if __name__ == "__main__":
    main()
