"""Cross-process HBM sharing on this image's driver, the mechanism RCCL's
intra-node P2P transport uses to map a peer's buffers: one process exports a
hipMalloc buffer (hipIpcGetMemHandle), another opens it (hipIpcOpenMemHandle)
and reads it back byte-exact. Run with HSA_ENABLE_IPC_MODE_LEGACY unset, =0
(dmabuf IPC, what bench.py and the CLI set) and =1 (legacy IPC). The outcome
of every variant goes to DISSEM_TEST_LOGDIR/ipc.json (profiles/r3_ipc/); the
test requires the variant the framework uses (=0) to work."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEER = os.path.join(ROOT, "tests", "ipc_peer.py")


def _exchange(legacy):
    env = dict(os.environ)
    env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    if legacy is not None:
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = legacy
    exp = subprocess.Popen([sys.executable, PEER, "export"], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True, env=env)
    try:
        first = exp.stdout.readline().strip()
        if first.startswith("{"):  # the exporter failed before it had a handle
            exp.communicate(timeout=60)
            return {"export": json.loads(first), "import": None}
        imp = subprocess.run([sys.executable, PEER, "import", first], capture_output=True, text=True, timeout=90,
                             env=env)
        got_imp = json.loads(imp.stdout.strip().splitlines()[-1]) if imp.stdout.strip() else {
            "ok": False, "error": imp.stderr[-500:]}
        out, _ = exp.communicate("done\n", timeout=60)
        return {"export": json.loads(out.strip().splitlines()[-1]), "import": got_imp}
    finally:
        if exp.poll() is None:
            exp.kill()


def test_ipc_handle_exchange_between_processes():
    import torch

    if torch.cuda.device_count() < 1:
        pytest.skip("needs a GPU")
    results = {str(v): _exchange(v) for v in (None, "0", "1")}
    d = os.environ.get("DISSEM_TEST_LOGDIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "ipc.json"), "w") as f:
            json.dump(results, f, indent=1)
    print(json.dumps(results))
    dmabuf = results["0"]
    assert dmabuf["import"] is not None and dmabuf["import"]["ok"], dmabuf
