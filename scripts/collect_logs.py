#!/usr/bin/env python3
"""Merge per-node JSONL logs and rebase time on the leader's "timer start"
(reference: conf/collect_logs.sh:8-19, which uses scp + jq).

    python scripts/collect_logs.py log0.jsonl log1.jsonl ... -o merged.jsonl

Writes merged.jsonl (sorted by `time`) and merged_elapsed.jsonl where `time` is
seconds since the first "timer start" event. Non-JSON lines (banners, Python
tracebacks) are skipped.
"""

import argparse
import json
import sys


def load(paths):
    events = []
    for p in paths:
        with open(p, encoding="utf-8", errors="replace") as f:
            for line in f:
                line = line.strip()
                if not line.startswith("{"):
                    continue
                try:
                    ev = json.loads(line)
                except json.JSONDecodeError:
                    continue
                if "time" in ev:
                    events.append(ev)
    events.sort(key=lambda e: e["time"])
    return events


def rebase(events):
    start = next((e["time"] for e in events if e.get("message") == "timer start"), None)
    if start is None:
        return None
    out = []
    for e in events:
        e2 = dict(e)
        e2["time"] = (e["time"] - start) / 1000.0
        out.append(e2)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("logs", nargs="+")
    ap.add_argument("-o", "--out", default="merged.jsonl")
    args = ap.parse_args(argv)
    events = load(args.logs)
    with open(args.out, "w") as f:
        for e in events:
            f.write(json.dumps(e, separators=(",", ":")) + "\n")
    reb = rebase(events)
    if reb is not None:
        el = args.out.replace(".jsonl", "") + "_elapsed.jsonl"
        with open(el, "w") as f:
            for e in reb:
                f.write(json.dumps(e, separators=(",", ":")) + "\n")
    print(f"saved and merged ({len(events)} events)", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
