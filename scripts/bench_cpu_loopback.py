#!/usr/bin/env python3
"""BASELINE config #1 (and a larger variant): two CLI processes on one host,
TCP loopback, host (RAM) engine - the reference's own data plane, no GPU.

    python scripts/bench_cpu_loopback.py [--layers 4 --layer-mib 1 --mode 0]

Prints one JSON line per run with the leader's time to deliver and GB/s.
"""

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_cli_multiprocess import free_ports, run_nodes, write_config  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--layer-mib", type=int, default=1)
    ap.add_argument("--mode", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--repeat", type=int, default=3)
    args = ap.parse_args()
    from pathlib import Path

    for mode in args.mode:
        best = None
        for _ in range(args.repeat):
            with tempfile.TemporaryDirectory() as d:
                ports = free_ports(2)
                cfg = write_config(Path(d), ports, layers=args.layers, size=args.layer_mib << 20)
                outs = run_nodes(cfg, [0, 1], mode)
                if any(rc != 0 for rc, _, _ in outs):
                    print(json.dumps({"mode": mode, "error": outs[0][2][-500:]}))
                    return 1
                s = json.loads(outs[0][1].strip().splitlines()[-1])
                if best is None or s["time_to_full_placement_s"] < best["time_to_full_placement_s"]:
                    best = s
        print(json.dumps({"config": f"2 processes, TCP loopback, {args.layers} x {args.layer_mib} MiB, mode {mode}",
                          "time_to_deliver_s": best["time_to_full_placement_s"],
                          "GBps": round(best["aggregate_GBps"], 3), "bytes": best["bytes_moved"],
                          "best_of": args.repeat}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
