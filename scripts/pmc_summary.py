"""Summarise rocprofv3 --pmc counter CSVs: per kernel name, the mean of each
counter over its dispatches plus a few derived ratios, as a markdown table.

    python scripts/pmc_summary.py DIR [DIR ...] > profiles/.../pmc_summary.md
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta[k] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"],
                           r["Scratch_Size"], r["VGPR_Count"])
    return rows, meta


def main(dirs):
    for d in dirs:
        rows, meta = load(d)
        print(f"### {d}\n")
        ctrs = sorted({c for k in rows for c in rows[k]})
        print("| kernel | grid | wg | lds | scratch | vgpr | " + " | ".join(ctrs) + " |")
        print("|---" * (6 + len(ctrs)) + "|")
        for k in sorted(rows):
            g, w, l, s, v = meta[k]
            vals = [sum(rows[k][c]) / len(rows[k][c]) if rows[k][c] else float("nan") for c in ctrs]
            print(f"| `{k.split('::')[-1]}` | {g} | {w} | {l} | {s} | {v} | " +
                  " | ".join(f"{x:.4g}" for x in vals) + " |")
        print()


if __name__ == "__main__":
    main(sys.argv[1:])
