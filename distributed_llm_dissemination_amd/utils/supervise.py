"""Fresh-process attempts with fallbacks for multi-rank runs (bench.py at N > 1).

The first real 8-GPU run is also the first time 8 processes map each other's
HBM through IPC and drive 14 RCCL communicators over xGMI. If that attempt
fails - an error, a stalled lane, a hang in communicator set-up - the run
should still produce a measurement with a more conservative data plane instead
of nothing. torchrun starts one *supervisor* per rank (this module); it never
touches the GPU. Each supervisor starts its rank's worker as a child process
(never an exec), and the supervisors agree through torchrun's own TCPStore
(the agent store) on whether the attempt succeeded:

* a worker heartbeats ``hb/<rank>`` at every phase (set-up, probe, each step);
  no heartbeat for ``stall_s`` seconds = a hung worker;
* a worker that fails (or hangs, or exits non-zero) marks ``fail``; every other
  supervisor then stops its own worker, whose peers are gone;
* rank 0's worker marks ``ok`` once the timed steps are done everywhere and its
  JSON line is written; then teardown problems no longer fail the run.

On failure every supervisor starts the next attempt (fresh worker processes, a
fresh store namespace for their process group) with that attempt's extra
arguments and environment. The reference protects the same outcome - every
receiver completes and the leader prints "Time to deliver"
(reference: cmd/main.go:167-181) - with a single attempt.
"""

from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

ENV_PREFIX = "DLD_SUP_PREFIX"   # worker: store namespace of this attempt
ENV_ATTEMPT = "DLD_SUP_ATTEMPT"  # worker: attempt index
ENV_LABEL = "DLD_SUP_LABEL"      # worker: fallback label ("" on the first attempt)
ENV_JSON = "DLD_SUP_JSON"        # worker rank 0: where to write its result line
ENV_HISTORY = "DLD_SUP_HISTORY"  # worker: JSON list of the failed attempts before this one


@dataclass
class Attempt:
    label: str = ""
    argv: List[str] = field(default_factory=list)
    env: Dict[str, str] = field(default_factory=dict)


def agent_store_available() -> bool:
    """torchrun with its agent store (static rendezvous: --master-addr/--master-port)."""
    return (os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True" and "MASTER_ADDR" in os.environ
            and "MASTER_PORT" in os.environ and int(os.environ.get("WORLD_SIZE", "1")) > 1)


def _tcp_store(timeout_s: float = 300.0):
    from datetime import timedelta

    import torch.distributed as dist

    return dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]),
                         int(os.environ["WORLD_SIZE"]), False, timeout=timedelta(seconds=timeout_s))


def _get(store, key: str) -> Optional[str]:
    if store.check([key]):
        return store.get(key).decode()
    return None


class WorkerChannel:
    """The worker's end: heartbeats, failure reason, success, and the store its
    process group rendezvous on (a namespace of its own per attempt)."""

    def __init__(self, store=None, prefix: Optional[str] = None, rank: Optional[int] = None):
        import torch.distributed as dist

        self.prefix = prefix if prefix is not None else os.environ[ENV_PREFIX]
        self.rank = rank if rank is not None else int(os.environ["RANK"])
        self._base = store if store is not None else _tcp_store()
        self.store = dist.PrefixStore(self.prefix, self._base)
        self.attempt = int(os.environ.get(ENV_ATTEMPT, "0"))
        self.label = os.environ.get(ENV_LABEL, "")
        try:
            self.history = json.loads(os.environ.get(ENV_HISTORY, "[]"))
        except ValueError:
            self.history = []

    @staticmethod
    def from_env() -> Optional["WorkerChannel"]:
        return WorkerChannel() if os.environ.get(ENV_PREFIX) else None

    def pg_store(self):
        import torch.distributed as dist

        return dist.PrefixStore("pg/", self.store)

    def heartbeat(self, phase: str) -> None:
        self.store.set(f"hb/{self.rank}", f"{time.time():.3f} {phase}")

    def fail(self, why: str) -> None:
        self.store.set(f"why/{self.rank}", why[-2000:])
        self.store.compare_set("fail", "", str(self.rank))

    def ok(self) -> None:
        self.store.set("ok", "1")


@dataclass
class AttemptResult:
    label: str
    rc: int
    ok: bool
    failed_rank: Optional[int] = None
    why: str = ""


def run_attempts(worker_cmd: List[str], attempts: List[Attempt], *, store=None, run_id: str = "",
                 stall_s: float = 150.0, finish_grace_s: float = 60.0, kill_grace_s: float = 5.0,
                 json_path: Optional[str] = None, log: Callable[[str], None] = lambda m: None,
                 poll_s: float = 0.2) -> tuple:
    """Run `worker_cmd` (+ each attempt's argv/env) as this rank's child until an
    attempt succeeds on every rank. Returns (rc, [AttemptResult...]). Rank 0 gets
    the worker's result line back in `json_path` (the caller prints it)."""
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    base = store if store is not None else _tcp_store()
    run_id = run_id or os.environ.get("TORCHELASTIC_RUN_ID", "run") + "." + os.environ.get(
        "TORCHELASTIC_RESTART_COUNT", "0")
    history: List[AttemptResult] = []
    rc = 1
    for k, att in enumerate(attempts):
        prefix = f"dld_sup/{run_id}/{k}/"
        sup = dist.PrefixStore(prefix, base)
        env = dict(os.environ)
        env.update(att.env)
        env[ENV_PREFIX] = prefix
        env[ENV_ATTEMPT] = str(k)
        env[ENV_LABEL] = att.label
        env[ENV_HISTORY] = json.dumps([h.__dict__ for h in history])
        if json_path:
            env[ENV_JSON] = json_path
            if rank == 0 and os.path.exists(json_path):
                os.unlink(json_path)
        log(f"attempt {k}{' (' + att.label + ')' if att.label else ''}: starting worker")
        child = subprocess.Popen(worker_cmd + att.argv, env=env, start_new_session=True)
        rc = _watch(child, sup, rank, stall_s, finish_grace_s, kill_grace_s, log, poll_s)
        ok = _get(sup, "ok") == "1"
        sup.set(f"rc/{rank}", str(rc))
        if rc != 0 and not ok:
            sup.compare_set("fail", "", str(rank))
        # every rank's outcome (a rank whose worker is stopped reports within kill_grace_s)
        deadline = time.monotonic() + stall_s
        while time.monotonic() < deadline and not all(sup.check([f"rc/{r}"]) for r in range(world)):
            time.sleep(poll_s)
        ok = _get(sup, "ok") == "1"
        rcs = {r: int(_get(sup, f"rc/{r}") or -999) for r in range(world)}
        failed = _get(sup, "fail")
        res = AttemptResult(att.label, rc, ok)
        if not ok:
            fr = int(failed) if failed not in (None, "") else next((r for r, c in rcs.items() if c != 0), None)
            res.failed_rank = fr
            res.why = (_get(sup, f"why/{fr}") or f"rank {fr} exited {rcs.get(fr)}") if fr is not None else "unknown"
        history.append(res)
        if ok:
            log(f"attempt {k} succeeded (worker rc {rc})")
            return 0, history
        log(f"attempt {k} failed on rank {res.failed_rank}: {res.why}")
    return (rc if rc != 0 else 1), history


def _watch(child, sup, rank, stall_s, finish_grace_s, kill_grace_s, log, poll_s) -> int:
    """Wait for this rank's worker; stop it if it hangs, if another rank failed,
    or if it lingers in teardown after the run succeeded."""
    t_start = time.monotonic()
    last_hb, t_hb = None, t_start
    t_ok = t_fail = None
    while True:
        rc = child.poll()
        if rc is not None:
            return rc
        now = time.monotonic()
        hb = _get(sup, f"hb/{rank}")
        if hb != last_hb:
            last_hb, t_hb = hb, now
        ok = _get(sup, "ok") == "1"
        if ok and t_ok is None:
            t_ok = now
        failed = _get(sup, "fail")
        if failed not in (None, "") and not ok and t_fail is None:
            t_fail = now
        reason = None
        if t_ok is not None and now - t_ok > finish_grace_s:
            reason = f"still in teardown {finish_grace_s:.0f} s after the run succeeded"
        elif t_fail is not None and now - t_fail > kill_grace_s:
            reason = f"rank {failed} failed"
        elif not ok and now - t_hb > stall_s:
            reason = f"no progress for {stall_s:.0f} s (last: {last_hb or 'no heartbeat'})"
            sup.set(f"why/{rank}", f"worker hung: {reason}")
            sup.compare_set("fail", "", str(rank))
        if reason is not None:
            log(f"stopping worker pid {child.pid}: {reason}")
            _kill_group(child, kill_grace_s)
            rc = child.wait()
            return 0 if t_ok is not None else (rc if rc != 0 else 1)
        time.sleep(poll_s)


def _kill_group(child, grace_s: float) -> None:
    for sig in (signal.SIGTERM, signal.SIGKILL):
        try:
            os.killpg(child.pid, sig)
        except ProcessLookupError:
            return
        t0 = time.monotonic()
        while time.monotonic() - t0 < grace_s:
            if child.poll() is not None:
                return
            time.sleep(0.05)


def emit_json(json_path: str, out=None) -> bool:
    """Rank 0's supervisor: pass the worker's result line to stdout."""
    out = out or sys.stdout
    try:
        with open(json_path) as f:
            line = f.read().strip().splitlines()[-1]
    except (OSError, IndexError):
        return False
    out.write(line + "\n")
    out.flush()
    return True
