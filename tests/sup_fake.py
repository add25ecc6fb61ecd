"""Stand-in for bench.py's supervisor and worker (tests/test_supervise.py, CPU).

Supervisor (torchrun rank): run_attempts over this script in --worker mode.
Worker: forms a gloo group on the attempt's store, optionally fails or hangs
as FAKE_* asks, and rank 0 writes a result line naming the attempt.
"""

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import importlib.util  # noqa: E402

spec = importlib.util.spec_from_file_location(
    "dld_supervise", os.path.join(os.path.dirname(HERE), "distributed_llm_dissemination_amd", "utils", "supervise.py"))
sup = importlib.util.module_from_spec(spec)
sys.modules["dld_supervise"] = sup
spec.loader.exec_module(sup)


def worker():
    import torch
    import torch.distributed as dist

    chan = sup.WorkerChannel.from_env()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    chan.heartbeat("start")
    dist.init_process_group("gloo", store=chan.pg_store(), rank=rank, world_size=world)
    chan.heartbeat("pg")
    fail = os.environ.get("FAKE_FAIL", "")  # "rank@attempt"
    if fail and fail in (f"{rank}@{chan.attempt}", f"{rank}@*"):
        chan.fail("injected failure")
        os._exit(3)
    hang = os.environ.get("FAKE_HANG", "")
    if hang and hang == f"{rank}@{chan.attempt}":
        time.sleep(3600)  # no heartbeat: the supervisor must stop it
    t = torch.tensor([rank + 1.0])
    dist.all_reduce(t)  # the other ranks wait here for a hung one
    chan.heartbeat("measured")
    if rank == 0:
        line = json.dumps({"value": float(t.item()), "fallback": chan.label or None, "failed": chan.history})
        with open(os.environ[sup.ENV_JSON], "w") as f:
            f.write(line + "\n")
        chan.ok()
    linger = os.environ.get("FAKE_LINGER", "")
    if linger and linger == str(rank):
        time.sleep(3600)  # teardown hang after success
    dist.destroy_process_group()
    return 0


def supervisor():
    rank = int(os.environ["RANK"])
    json_path = os.path.join(os.environ["FAKE_TMP"], "result.json") if rank == 0 else None
    attempts = [sup.Attempt(""), sup.Attempt("fallback-1", ["--tag", "one"]),
                sup.Attempt("fallback-2", ["--tag", "two"], {"FAKE_EXTRA": "1"})]
    rc, hist = sup.run_attempts([sys.executable, os.path.abspath(__file__), "--worker"], attempts,
                                json_path=json_path, stall_s=float(os.environ.get("FAKE_STALL_S", "20")),
                                finish_grace_s=1.5, kill_grace_s=1.0,
                                log=lambda m: print(f"[sup {rank}] {m}", file=sys.stderr, flush=True))
    if rank == 0 and rc == 0:
        sup.emit_json(json_path)
    return rc


if __name__ == "__main__":
    sys.exit(worker() if "--worker" in sys.argv else supervisor())
