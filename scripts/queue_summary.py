#!/usr/bin/env python3
"""Which hardware queue ran which kernels: summarize rocprofv3 kernel traces by
Queue_Id (and Stream_Id when present), per trace file (one per rank process).

    python scripts/queue_summary.py gpurun_out/queues

Kernel classes: rccl (RCCL P2P/broadcast kernels on the comm lanes), crc
(verify queue), fp8 (pack on the copy queues), fill, other. The planned engine
is safe from cross-queue stalls only if no queue that runs an rccl kernel also
runs crc/fp8 kernels (a copy or a check parked behind a P2P kernel that waits
for a peer).

With a marker trace next to a kernel trace (rocprofv3 --marker-trace), every
kernel is also put in a phase by its start time: inside a "bench.step" roctx
range (timed), inside "bench.warmup", or outside both (setup: communicator
init, probe, staging set-up)."""
import collections
import csv
import glob
import os
import sys


def kclass(name: str) -> str:
    n = name.lower()
    if "nccl" in n or "rccl" in n:
        return "rccl"
    if "crc" in n:
        return "crc"
    if "fp8" in n:
        return "fp8"
    if "fill" in n:
        return "fill"
    return "other"


def _ranges(marker_csv: str):
    """{"bench.step": [(t0, t1)], "bench.warmup": [...]} from a rocprofv3 marker trace."""
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(marker_csv)):
        text = " ".join(str(v) for v in r.values())
        for name in ("bench.step", "bench.warmup"):
            if name in text and r.get("Start_Timestamp") and r.get("End_Timestamp"):
                out[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def _phase(t: int, ranges) -> str:
    for name, tag in (("bench.step", "timed"), ("bench.warmup", "warmup")):
        if any(a <= t <= b for a, b in ranges.get(name, ())):
            return tag
    return "setup"


def main(root: str) -> int:
    files = sorted(glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True))
    if not files:
        print(f"no kernel traces under {root}")
        return 1
    bad = 0
    for f in files:
        rows = list(csv.DictReader(open(f)))
        markers = glob.glob(os.path.join(os.path.dirname(f), "*marker_api_trace.csv"))
        ranges = _ranges(markers[0]) if markers else None
        phases = collections.defaultdict(collections.Counter)
        q = collections.defaultdict(collections.Counter)
        streams = collections.defaultdict(set)
        for r in rows:
            qid = r.get("Queue_Id", "?")
            q[qid][kclass(r.get("Kernel_Name", ""))] += 1
            if ranges is not None and r.get("Start_Timestamp"):
                phases[qid][f"{kclass(r.get('Kernel_Name', ''))}@{_phase(int(r['Start_Timestamp']), ranges)}"] += 1
            if "Stream_Id" in r:
                streams[qid].add(r["Stream_Id"])
        print(f"== {os.path.relpath(f, root)}: {len(rows)} kernels on {len(q)} queues")
        for qid, c in sorted(q.items()):
            mixed = c.get("rccl", 0) and (c.get("crc", 0) or c.get("fp8", 0))
            bad += bool(mixed)
            st = f" streams={sorted(streams[qid])}" if streams[qid] else ""
            print(f"  queue {qid}: {dict(c)}{st}{'  <-- RCCL shares a queue with verify/copy kernels' if mixed else ''}")
            if ranges is not None:
                print(f"    by phase: {dict(sorted(phases[qid].items()))}")
        if ranges is not None:
            other = collections.Counter()
            for r in rows:
                if kclass(r.get("Kernel_Name", "")) == "other" and r.get("Start_Timestamp"):
                    other[(r.get("Kernel_Name", "")[:60], _phase(int(r["Start_Timestamp"]), ranges))] += 1
            print(f"  'other' kernels by name and phase: {dict(other.most_common(8))}")
    print("verdict:", "SHARED (rccl + verify/copy on one queue)" if bad else "separate queues for rccl vs verify/copy")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/queues"))
