#!/usr/bin/env python3
"""Per-launch device times of the verify kernels in a rocprofv3 kernel trace,
grouped by kernel and grid size (the grid tells a 1-, 4-, 8- or 16-chunk batch
apart): launches, mean / min us, and us per 64 MiB source chunk when the
grid's workgroups say how many segments it covered.

    python scripts/trace_groups.py <kernel_trace.csv> [--chunk-mib 64] [--match crc_walk]
"""

import argparse
import csv
import re
from collections import OrderedDict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="verify_once16|crc_walk|crc32c|fold")
    args = ap.parse_args()
    pat = re.compile(args.match)
    groups = OrderedDict()
    with open(args.trace) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if not pat.search(name):
                continue
            short = name.replace("(anonymous namespace)::", "").replace("dissem::kern::", "").replace("void ", "")
            short = re.sub(r"\(.*", "", short)
            key = (short, int(row["Grid_Size_X"]), int(row["Workgroup_Size_X"]))
            us = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            groups.setdefault(key, []).append(us)
    print(f"{'kernel':70s} {'grid':>8s} {'wg':>5s} {'n':>4s} {'mean_us':>9s} {'min_us':>9s} {'median_us':>9s}")
    for (k, grid, wg), v in groups.items():
        s = sorted(v)
        print(f"{k[:70]:70s} {grid:8d} {wg:5d} {len(v):4d} {sum(v) / len(v):9.1f} {s[0]:9.1f} {s[len(s) // 2]:9.1f}")


if __name__ == "__main__":
    main()
