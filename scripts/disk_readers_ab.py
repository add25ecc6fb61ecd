#!/usr/bin/env python3
"""A/B of the disk tier's reader threads and bounce ring at N = 1 (bench.py
--tier disk with engine options patched in): which setting reads the NVMe
fastest. Prints a {"disk_readers", "disk_ring"} line, then that run's bench JSON line.

    python scripts/disk_readers_ab.py --storage /tmp/dl_disk [--layers 16]
"""
import argparse
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import distributed_llm_dissemination_amd.__main__ as cli  # noqa: E402  (bench's worker imports engine_opts from it)


def run_one(storage, layers, readers, ring):
    orig = cli.engine_opts
    cli.engine_opts = lambda a: {**orig(a), "disk_readers": readers, "disk_ring": ring}
    # bench prints its own JSON line after this one (and ends the process)
    print(json.dumps({"disk_readers": readers, "disk_ring": ring}), flush=True)
    return bench.main(["--tier", "disk", "--storage", storage, "--layers", str(layers), "--steps", "3",
                       "--warmup", "1"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--storage", required=True)
    ap.add_argument("--layers", type=int, default=16)
    ap.add_argument("--settings", default="4:8,8:16,12:24",
                    help="readers:ring pairs (ring = pinned bounce buffers of one chunk each)")
    ap.add_argument("--one", default="", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.one:
        readers, ring = (int(x) for x in args.one.split(":"))
        return run_one(args.storage, args.layers, readers, ring)
    rc = 0
    for spec in args.settings.split(","):  # one process per setting (bench ends its process)
        rc = subprocess.call([sys.executable, os.path.abspath(__file__), "--storage", args.storage, "--layers",
                              str(args.layers), "--one", spec]) or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
