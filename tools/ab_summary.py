#!/usr/bin/env python3
"""Summarise an interleaved A/B log of tools/small_calls.sh / ab_perf_test.sh
("== <tag> round=R n=N ..." headers, perf_test rows "bytes us algbw busbw schedule"): per
(ranks, bytes, tag) the us of every round, the median and the ratio to the first tag's median."""
import collections
import re
import statistics
import sys

d = collections.defaultdict(list)
tags = []
tag = None
for line in open(sys.argv[1]):
    m = re.match(r"== (\S+) (?:round=\d+ )?n=(\d+)", line) or re.match(r"== n=(\d+) algo=(\S+)", line)
    if m:
        if line.startswith("== n="):
            t, n = m.group(2), m.group(1)
        else:
            t, n = m.group(1), m.group(2)
        tag = (t, int(n))
        if t not in tags:
            tags.append(t)
        continue
    f = line.split()
    if tag and len(f) >= 3 and f[0].isdigit():
        d[(tag[1], int(f[0]), tag[0])].append(float(f[1]))
keys = sorted({(n, b) for n, b, _ in d})
for n, b in keys:
    base = None
    for t in tags:
        v = d.get((n, b, t))
        if not v:
            continue
        med = statistics.median(v)
        base = base or med
        print(f"n={n} {b:>11} {t:>10}: median {med:9.2f} us  x{base / med:5.3f}  [{' '.join(f'{x:.1f}' for x in v)}]")
