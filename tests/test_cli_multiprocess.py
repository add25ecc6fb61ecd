"""BASELINE config #1: 2-process loopback TCP on CPU, 4 layers x 1 MiB, mode 0,
through the reference-compatible CLI (one OS process per node)."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def write_config(tmp_path, ports, layers=4, size=1 << 20, holders=None, assign=None):
    holders = holders or {0: list(range(layers))}
    assign = assign or {1: list(range(layers))}
    nodes = []
    for i, p in enumerate(ports):
        nodes.append({
            "Id": i, "Addr": f"127.0.0.1:{p}", "NetworkBW": 1562500000, "IsLeader": i == 0,
            "Sources": {"2": 0},
            "InitialLayers": {"2": {str(l): {"LayerSize": size} for l in holders.get(i, [])}},
        })
    cfg = {"Nodes": nodes, "Assignment": {str(k): {str(l): {} for l in v} for k, v in assign.items()}}
    path = tmp_path / "config.json"
    path.write_text(json.dumps(cfg))
    return str(path)


def run_nodes(cfg_path, ids, mode, extra=()):
    env = dict(os.environ, PYTHONPATH=ROOT)
    procs = [
        subprocess.Popen([sys.executable, "-m", "distributed_llm_dissemination_amd", "-id", str(i), "-f", cfg_path,
                          "-m", str(mode), "--json-summary", *extra],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=ROOT)
        for i in ids
    ]
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out, err))
    return outs


@pytest.mark.slow
@pytest.mark.parametrize("mode", [0, 1])
def test_two_process_loopback_mode(tmp_path, mode):
    ports = free_ports(2)
    cfg = write_config(tmp_path, ports)
    (rc0, out0, err0), (rc1, out1, err1) = run_nodes(cfg, [0, 1], mode)
    assert rc0 == 0, err0
    assert rc1 == 0, err1
    assert "launching leader..." in out0 and "launching receiver..." in out1
    assert "Time to deliver:" in out0
    summary = json.loads(out0.strip().splitlines()[-1])
    assert summary["bytes_moved"] == 4 << 20 and summary["mode"] == mode


@pytest.mark.slow
def test_torchrun_launch_host_engine(tmp_path):
    """torchrun (3 ranks, gloo bootstrap on CPU): -id comes from RANK, nodes have
    no fixed Addr and exchange their ephemeral ports through the process group."""
    from distributed_llm_dissemination_amd.models.catalog import make_workload

    cfg = make_workload(3, 6, 512 << 10, tier="host", seeding="random")
    path = tmp_path / "cfg.json"
    path.write_text(json.dumps(cfg.to_json()))
    port = free_ports(1)[0]
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        "-m", "distributed_llm_dissemination_amd", "-f", str(path), "-m", "1", "--engine", "host",
                        "--json-summary"], capture_output=True, text=True, env=env, cwd=ROOT, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Time to deliver:" in r.stdout
    summary = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert summary["bytes_moved"] == 2 * 6 * (512 << 10)


def test_usage_without_flags():
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "distributed_llm_dissemination_amd"], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("usage: -id 0 -f config.json -s . -m 2 -l -v")


def test_go_duration_format():
    from distributed_llm_dissemination_amd.__main__ import go_duration

    assert go_duration(59.87) == "59.87s"
    assert go_duration(0.1502) == "150.2ms"
    assert go_duration(62.5) == "1m2.5s"
    assert go_duration(12e-6) == "12µs"
    assert go_duration(0) == "0s"


def write_config_rates(tmp_path, ports, size, holders, assign, rates):
    nodes = []
    for i, p in enumerate(ports):
        nodes.append({
            "Id": i, "Addr": f"127.0.0.1:{p}", "NetworkBW": 1562500000, "IsLeader": i == 0,
            "Sources": {"2": rates.get(i, 0)},
            "InitialLayers": {"2": {str(l): {"LayerSize": size} for l in holders.get(i, [])}},
        })
    cfg = {"Nodes": nodes, "Assignment": {str(k): {str(l): {} for l in v} for k, v in assign.items()}}
    path = tmp_path / "config.json"
    path.write_text(json.dumps(cfg))
    return str(path)


@pytest.mark.slow
def test_kill_rank_injection_recovers_via_job_deadline(tmp_path):
    """--inject kill-rank=1@T: node 1 (a rate-limited owner) dies mid-transfer;
    the leader's job deadline re-dispatches its layers to node 2."""
    ports = free_ports(4)
    size = 2 << 20
    holders = {1: [0, 1, 2, 3], 2: [0, 1, 2, 3]}
    assign = {1: [0], 2: [0], 3: [0, 1, 2, 3]}  # 1 and 2 are keys so the leader waits for their announce
    cfg = write_config_rates(tmp_path, ports, size, holders, assign, rates={1: 2 << 20})
    extra = ["--inject", "kill-rank=1@0.5", "--job-timeout", "1.5", "--owner-policy", "balanced"]
    (rc0, out0, err0), (rc1, _, err1), (rc2, _, err2), (rc3, _, err3) = run_nodes(cfg, [0, 1, 2, 3], 1, extra)
    assert rc1 == 86, err1  # killed by the injection
    assert rc0 == 0, err0[-3000:]
    assert rc3 == 0, err3[-3000:]
    summary = json.loads(out0.strip().splitlines()[-1])
    assert summary["redispatched"] >= 1
    assert "job deadline expired" in err0


@pytest.mark.slow
def test_persist_dir_resume_skips_network(tmp_path):
    ports = free_ports(2)
    cfg = write_config(tmp_path, ports)
    pdir = str(tmp_path / "persist")
    outs = run_nodes(cfg, [0, 1], 1, ["--persist-dir", pdir])
    assert all(rc == 0 for rc, _, _ in outs), [e[-2000:] for _, _, e in outs]
    assert "layers persisted" in outs[1][2]
    assert "start receiving layer" in outs[1][2]
    ports2 = free_ports(2)
    cfg = write_config(tmp_path, ports2)
    outs = run_nodes(cfg, [0, 1], 1, ["--persist-dir", pdir])
    assert all(rc == 0 for rc, _, _ in outs), [e[-2000:] for _, _, e in outs]
    assert "start receiving layer" not in outs[1][2]  # promoted from the persisted copies


@pytest.mark.slow
def test_two_process_weights_preset(tmp_path):
    """--weights: the layers are random-init Llama-family decoder layers (models/weights.py);
    the receiver reads its layers back as named parameters and runs their forward pass."""
    from distributed_llm_dissemination_amd.models.weights import PRESETS, layer_nbytes

    ports = free_ports(2)
    cfg = write_config(tmp_path, ports, layers=2, size=layer_nbytes(PRESETS["tiny"]))
    (rc0, out0, err0), (rc1, out1, err1) = run_nodes(cfg, [0, 1], 1, extra=("--weights", "tiny"))
    assert rc0 == 0, err0
    assert rc1 == 0, err1
    check = [json.loads(line) for line in err1.splitlines() if "weights forward check" in line]
    assert check and check[0]["layers"] == 2 and check[0]["max_rel_err"] == 0.0
    bad = run_nodes(write_config(tmp_path, ports, layers=1, size=4096), [0], 1, extra=("--weights", "tiny"))
    assert bad[0][0] == 2 and "needs LayerSize" in bad[0][2]
