#!/usr/bin/env python3
"""Where a schedule leaves links idle: per-link and per-rank staging timelines
of one simulated session in model time (predict_scaling.predict(trace=True)).

    python scripts/sim_timeline.py --n 8 --mode 2
    python scripts/sim_timeline.py --n 8 --mode 1 --json

For every directed link: bytes, busy ms (transfer time at the link rate),
idle ms before its first transfer, inside its run (gaps between transfers)
and after its last one up to the session's end. The same for every rank's
PCIe staging. Full-size milliseconds (the run is at 1/scale size with the
rates scaled alike).
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import predict_scaling  # noqa: E402


def intervals_idle(iv, t0, t1):
    """(busy, head idle, gaps, tail idle) of sorted intervals within [t0, t1]."""
    iv = sorted(iv)
    if not iv:
        return 0.0, t1 - t0, 0.0, 0.0
    busy = gaps = 0.0
    end = iv[0][0]
    for a, b in iv:
        if a > end:
            gaps += a - end
        busy += max(0.0, b - max(a, end))
        end = max(end, b)
    return busy, iv[0][0] - t0, gaps, t1 - end


def timeline(r) -> dict:
    transfers, stages = r["trace_last"]
    t0 = min([t[2] for t in transfers] + [s[1] for s in stages])
    t1 = max([t[3] for t in transfers] + [s[2] for s in stages])
    links = {}
    for s, d, a, b, n in transfers:
        links.setdefault(f"{s}->{d}", []).append((a, b))
    ranks = {}
    for k, a, b, n in stages:
        ranks.setdefault(k, []).append((a, b))
    ms = lambda x: round(x * 1e3, 2)  # noqa: E731
    out = {"session_ms": ms(t1 - t0), "links": {}, "staging": {}}
    for k, iv in sorted(links.items()):
        busy, head, gaps, tail = intervals_idle(iv, t0, t1)
        out["links"][k] = {"busy": ms(busy), "head_idle": ms(head), "gaps": ms(gaps), "tail_idle": ms(tail)}
    for k, iv in sorted(ranks.items()):
        busy, head, gaps, tail = intervals_idle(iv, t0, t1)
        out["staging"][k] = {"busy": ms(busy), "head_idle": ms(head), "gaps": ms(gaps), "tail_idle": ms(tail)}
    for key in ("links", "staging"):
        vals = list(out[key].values())
        if vals:
            out[key + "_mean"] = {f: round(sum(v[f] for v in vals) / len(vals), 2) for f in vals[0]}
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--scale", type=int, default=1024)
    ap.add_argument("--pull-window", type=int, default=0)
    ap.add_argument("--pull-job-mib", type=int, default=0)
    ap.add_argument("--json", action="store_true", help="print the whole timeline as JSON")
    args = ap.parse_args()
    policy = {"owner_policy": "links"}
    if args.pull_window:
        policy["pull_window"] = args.pull_window
    if args.pull_job_mib:
        policy["pull_job_bytes"] = (args.pull_job_mib << 20) // args.scale
    r = predict_scaling.predict(args.n, mode=args.mode, layers=args.layers, scale=args.scale, steps=1, warmup=1,
                                policy=policy, trace=True)
    tl = timeline(r)
    tl["model_ms"] = r["model_ms"]
    tl["closed_form_ms"] = round(predict_scaling.closed_form_ms(args.n, layers=args.layers), 1)
    if args.json:
        print(json.dumps(tl))
        return 0
    print(f"session {tl['session_ms']} ms (model {r['model_ms']}, bound {tl['closed_form_ms']})")
    print("links   mean:", tl.get("links_mean"))
    print("staging mean:", tl.get("staging_mean"))
    worst = sorted(tl["links"].items(), key=lambda kv: -(kv[1]["gaps"] + kv[1]["head_idle"] + kv[1]["tail_idle"]))[:6]
    for k, v in worst:
        print(f"  {k}: {v}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
