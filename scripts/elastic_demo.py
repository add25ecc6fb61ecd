#!/usr/bin/env python3
"""Elastic-recovery demo: N rank processes of the CLI (RCCL engine), one of them
killed mid-session. Writes each rank's stdout/stderr under OUT and prints the
leader's summary.

    python scripts/elastic_demo.py --ranks 3 --out gpurun_out/elastic_demo

On a one-GPU box the ranks share device 0 (DISSEM_SHARED_GPU, RCCL over
loopback sockets). Plain processes rather than torchrun: its agent tears every
worker down as soon as one exits.
"""

import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=3)
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--layer-mib", type=int, default=64)
    ap.add_argument("--out", default="gpurun_out/elastic_demo")
    args = ap.parse_args()
    import torch

    from distributed_llm_dissemination_amd.models.catalog import make_workload

    os.makedirs(args.out, exist_ok=True)
    n = args.ranks
    cfg = make_workload(n, args.layers, args.layer_mib << 20, tier="host", seeding="uniform", copies=2, seed=7,
                        chunk_bytes=8 << 20)
    path = os.path.join(args.out, "cfg.json")
    with open(path, "w") as f:
        json.dump(cfg.to_json(), f)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ngpu = torch.cuda.device_count()
    victim = n - 1
    procs = []
    for r in range(n):
        env = dict(os.environ, PYTHONPATH=ROOT, RANK=str(r), LOCAL_RANK=str(r if ngpu >= n else 0),
                   WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if ngpu < n:
            env["DISSEM_SHARED_GPU"] = "1"
        out = open(os.path.join(args.out, f"rank{r}.out"), "w")
        err = open(os.path.join(args.out, f"rank{r}.err"), "w")
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "distributed_llm_dissemination_amd", "-f", path, "-m", "1", "--engine", "rccl",
             "--json-summary", "--suspect-timeout", "2", "--timeout", "120", "--inject", f"kill-rank={victim}@0"],
            stdout=out, stderr=err, cwd=ROOT, env=env))
    rcs = [p.wait(timeout=200) for p in procs]
    print(json.dumps({"returncodes": rcs, "victim": victim}))
    with open(os.path.join(args.out, "rank0.out")) as f:
        lines = f.read().strip().splitlines()
    print(lines[-1] if lines else "")
    return 0 if all(rc == (86 if r == victim else 0) for r, rc in enumerate(rcs)) else 1


if __name__ == "__main__":
    sys.exit(main())
