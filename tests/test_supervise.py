"""Supervised fresh-process attempts with fallbacks (utils/supervise.py), the
insurance bench.py takes for multi-rank runs: an attempt that fails on any rank,
hangs without heartbeats, or lingers in teardown after success is handled by
every rank's supervisor, and the next attempt runs with fallback settings in
fresh processes. CPU only: torchrun + gloo + the agent store (127.0.0.1)."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(n, script_args, env_extra, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + script_args
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    env.pop("DLD_SUP_PREFIX", None)
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


def _result(r):
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_first_attempt_succeeds(tmp_path):
    out = _result(_torchrun(3, ["tests/sup_fake.py"], {"FAKE_TMP": str(tmp_path)}))
    assert out == {"value": 6.0, "fallback": None, "failed": []}


def test_failed_attempt_falls_back_in_fresh_processes(tmp_path):
    r = _torchrun(3, ["tests/sup_fake.py"], {"FAKE_TMP": str(tmp_path), "FAKE_FAIL": "2@0"})
    out = _result(r)
    assert out["fallback"] == "fallback-1" and out["value"] == 6.0
    assert len(out["failed"]) == 1 and out["failed"][0]["failed_rank"] == 2
    assert "injected failure" in out["failed"][0]["why"]
    assert "attempt 1 (fallback-1): starting worker" in r.stderr


def test_hung_worker_is_stopped_and_retried(tmp_path):
    """Rank 1 hangs before the collective (no heartbeat): its supervisor stops
    it after stall_s; the others, blocked in the collective, are stopped too."""
    r = _torchrun(2, ["tests/sup_fake.py"], {"FAKE_TMP": str(tmp_path), "FAKE_HANG": "1@0", "FAKE_STALL_S": "4"})
    out = _result(r)
    assert out["fallback"] == "fallback-1"
    assert "worker hung" in out["failed"][0]["why"]


def test_teardown_hang_after_success_is_not_a_failure(tmp_path):
    r = _torchrun(2, ["tests/sup_fake.py"], {"FAKE_TMP": str(tmp_path), "FAKE_LINGER": "1"})
    out = _result(r)
    assert out["fallback"] is None and out["failed"] == []
    assert "still in teardown" in r.stderr


def test_every_attempt_failing_fails_the_run(tmp_path):
    r = _torchrun(2, ["tests/sup_fake.py"], {"FAKE_TMP": str(tmp_path), "FAKE_FAIL": "1@*"})
    assert r.returncode != 0
    assert "{" not in r.stdout  # no result line
    assert "attempt 2 failed on rank 1: injected failure" in r.stderr


def test_bench_supervisor_runs_the_fallback_attempts_on_cpu(tmp_path):
    """bench.py itself under torchrun on a GPU-less host: every worker attempt
    fails (no GPU visible), and the supervisors walk through the fallback list
    (as given, then world-1 lanes, then RCCL without P2P) before failing."""
    pytest.importorskip("torch")
    r = _torchrun(3, ["bench.py", "--gpus", "3", "--steps", "1", "--warmup", "0", "--layers", "3",
                      "--layer-mib", "1"], {})
    assert r.returncode != 0
    for k, label in enumerate(["", " (lanes=2)", " (lanes=2, NCCL_P2P_DISABLE=1)"]):
        assert f"attempt {k}{label}: starting worker" in r.stderr, r.stderr[-3000:]
