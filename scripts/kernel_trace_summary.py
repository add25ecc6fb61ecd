#!/usr/bin/env python3
"""Summarize a rocprofv3 kernel-trace CSV: per kernel, duration clusters (µs)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("dissem::kern::", "").split("(")[0]
    d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    v = sorted(v)
    print(f"{k:50s} n={len(v):4d} min={v[0]:9.1f} med={v[len(v) // 2]:9.1f} max={v[-1]:9.1f}")
