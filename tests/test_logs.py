"""Log tooling (reference: conf/collect_logs.sh): per-node JSONL logs from a real
two-process run are merged by time and rebased on the leader's "timer start"."""

import json
import os
import subprocess
import sys

import pytest

from test_cli_multiprocess import ROOT, free_ports, run_nodes, write_config


@pytest.mark.slow
def test_collect_logs_merges_and_rebases(tmp_path):
    ports = free_ports(2)
    cfg = write_config(tmp_path, ports)
    outs = run_nodes(cfg, [0, 1], 1)
    assert all(rc == 0 for rc, _, _ in outs), [e[-1500:] for _, _, e in outs]
    logs = []
    for i, (_, _, err) in enumerate(outs):
        p = tmp_path / f"log{i}.jsonl"
        p.write_text(err)  # the reference's operator redirects stderr the same way
        logs.append(str(p))
    merged = tmp_path / "merged.jsonl"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "collect_logs.py"), *logs, "-o", str(merged)],
                   check=True)
    ev = [json.loads(l) for l in merged.read_text().splitlines()]
    times = [e["time"] for e in ev]
    assert times == sorted(times) and {e.get("node") for e in ev} >= {0, 1}
    el = [json.loads(l) for l in (tmp_path / "merged_elapsed.jsonl").read_text().splitlines()]
    start = [e for e in el if e.get("message") == "timer start"]
    assert start and start[0]["time"] == 0.0
    assert any(e.get("message") == "layer fully received" and e["time"] >= 0 for e in el)
