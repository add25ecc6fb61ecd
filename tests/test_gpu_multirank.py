"""Multi-GPU runs through torchrun. One rank per GPU over
RCCL/xGMI: every mode, fp8 packing and the ncclBroadcast path, with CRC
verification on the receivers. Skipped when fewer than 2 GPUs are visible (the
CPU suite covers the same schedules on the simulated fabric)."""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ngpus():
    import torch

    return torch.cuda.device_count()


def _keep_logs(outs):
    """Copy each rank's output where a GPU-box run can read it (DISSEM_TEST_LOGDIR)."""
    d = os.environ.get("DISSEM_TEST_LOGDIR")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    for r, (out, err) in enumerate(outs):
        with open(os.path.join(d, f"rank{r}.log"), "w") as f:
            f.write((out or "") + "\n----- stderr -----\n" + (err or ""))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(n, args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    env = dict(os.environ, PYTHONPATH=ROOT)
    if _ngpus() < n:
        # one-GPU box: every rank on device 0, RCCL over loopback sockets (utils/launch.py)
        env["DISSEM_SHARED_GPU"] = "1"
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


@pytest.fixture(scope="module", params=["odd", "full"])
def n(request):
    """Ranks. With >= 2 GPUs: every GPU (at most 8). On a one-GPU box every rank
    shares device 0: 3 ranks (odd on purpose: relay/scatter schedules with an
    uneven split) and 8 ranks, the driver's `bench.py --gpus 8` world (8-way
    communicator init, 7 peers in every group)."""
    k = _ngpus()
    if k < 1:
        pytest.skip("needs a GPU")
    if k >= 2:
        if request.param == "odd":
            pytest.skip("multi-GPU box: one run over every GPU")
        return min(k, 8)
    return 3 if request.param == "odd" else 8


@pytest.mark.parametrize("mode,extra", [(1, []), (2, ["--pull-window", "2"]), (3, []), (0, ["--seeding", "leader"]),
                                        (0, ["--seeding", "leader", "--bcast", "collective"]),
                                        (1, ["--pack", "fp8", "--layer-mib", "96"]),
                                        (1, ["--pack", "fp8", "--store", "bf16", "--layer-mib", "96"]),
                                        (1, ["--inject", "slow-link=0:1:2G"]),
                                        # every rank holds every layer: mode 2 loads a dest's own copy and
                                        # may let an idle peer steal it - scratch landings on the HIP backend
                                        (2, ["--pull-window", "2", "--copies", "3"]),
                                        (1, ["--seeding", "uniform", "--source-pool", "3"])])
def test_bench_modes(n, mode, extra, request):
    if n == 8 and _ngpus() < 2 and (extra or mode != 1) and os.environ.get("DISSEM_FULL_REHEARSAL") != "1":
        # one-GPU box: the default suite runs the headline mode 1 at 8 shared
        # ranks (~100 s each: 14 communicators per rank); every variant runs at
        # 3 ranks, and DISSEM_FULL_REHEARSAL=1 / scripts/gpu.sh shared8 run
        # modes 0-3 and the variants at 8
        pytest.skip("variant covered at 3 ranks")
    r = _torchrun(n, ["bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1", "--layers", "16",
                      "--layer-mib", "64", "--chunk-mib", "16", "--mode", str(mode)] + extra)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == n and out["value"] > 0
    st = out["config"]["engine_stats_rank0"]
    assert st["verify_failures"] == 0 and st["unverified_pieces"] == 0
    if _ngpus() >= n and not any(a.startswith("slow-link") for a in extra):
        # real GPUs: RCCL's P2P over xGMI on every directed link, not a fallback (tests/benchcheck.py)
        from distributed_llm_dissemination_amd import _core
        from benchcheck import real_multi_gpu_problems

        assert real_multi_gpu_problems(out, n, _core.resolve_lanes(n, 0)) == [], out["config"]


@pytest.mark.parametrize("mode,extra", [(1, []), (0, ["--seeding", "leader"])])
def test_bench_fake_hosts(mode, extra):
    """4 ranks posing as 2 hosts x 2 GPUs (DISSEM_FAKE_HOSTS=2) over real RCCL:
    host-aware comm lanes, mode 1's once-per-host imports with xGMI relays and
    mode 0's three-level tree. Mode 0 with the leader holding every layer is the
    run that hung before the CRC tables were uploaded without a host sync
    (profiles/r3_multihost/hang_diag/): the other host's ranks start by
    receiving, so their first check comes after posted receives."""
    if _ngpus() < 1:
        pytest.skip("needs a GPU")
    os.environ["DISSEM_FAKE_HOSTS"] = "2"
    try:
        r = _torchrun(4, ["bench.py", "--gpus", "4", "--steps", "1", "--warmup", "1", "--layers", "8",
                          "--layer-mib", "64", "--chunk-mib", "16", "--probe-mib", "16", "--mode", str(mode)] + extra)
    finally:
        del os.environ["DISSEM_FAKE_HOSTS"]
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["config"]["hosts"] == 2 and out["config"].get("fallback") is None
    st = out["config"]["engine_stats_rank0"]
    assert st["verify_failures"] == 0 and st["unverified_pieces"] == 0 and st["order_violations"] == 0


@pytest.mark.parametrize("size", [32 << 20, (32 << 20) + 13])
def test_cli_torchrun_rccl(n, size, tmp_path):
    """The CLI over RCCL; the second size is not a multiple of 16 (like the
    reference's experiment layers): every layer ends in an odd-length chunk that
    crosses RCCL and the batched CRC check."""
    from distributed_llm_dissemination_amd.models.catalog import make_workload

    cfg = make_workload(n, 8, size, tier="host", seeding="random", chunk_bytes=8 << 20)
    path = tmp_path / "cfg.json"
    path.write_text(json.dumps(cfg.to_json()))
    r = _torchrun(n, ["-m", "distributed_llm_dissemination_amd", "-f", str(path), "-m", "1", "--engine", "rccl",
                      "--json-summary"])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "Time to deliver:" in r.stdout


def test_cli_rank_death_elastic_recovery(n, tmp_path):
    """A rank process dies mid-session (--inject kill-rank, os._exit): the
    survivors' RCCL groups with it fail or stall, the leader's probe finds it
    gone, the survivors abort the communicator and re-form one without it
    (fresh unique id from the leader), and the leader re-plans the unacked
    layers from live holders. Plain processes, not torchrun: its agent would
    tear every worker down when one exits."""
    if n == 8 and _ngpus() < 2 and os.environ.get("DISSEM_FULL_REHEARSAL") != "1":
        # DISSEM_FULL_REHEARSAL=1 (scripts/gpu.sh insure): 8 ranks on one GPU,
        # 14 lanes aborted in parallel and re-formed as 7 ranks (18 lanes)
        pytest.skip("one-GPU box: rank death is rehearsed at 3 ranks")
    from distributed_llm_dissemination_amd.models.catalog import make_workload

    cfg = make_workload(n, 24, 64 << 20, tier="host", seeding="uniform", copies=2, seed=7, chunk_bytes=8 << 20)
    path = tmp_path / "cfg.json"
    path.write_text(json.dumps(cfg.to_json()))
    victim = n - 1
    port = _port()
    procs = []
    for r in range(n):
        env = dict(os.environ, PYTHONPATH=ROOT, RANK=str(r), LOCAL_RANK=str(r if _ngpus() >= n else 0),
                   WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if _ngpus() < n:
            env["DISSEM_SHARED_GPU"] = "1"
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "distributed_llm_dissemination_amd", "-f", str(path), "-m", "1", "--engine", "rccl",
             "--json-summary", "--suspect-timeout", "2", "--timeout", "120", "--inject", f"kill-rank={victim}@0"],
            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT, env=env))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=150))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            outs = [q.communicate() for q in procs]
            _keep_logs(outs)
            raise
    _keep_logs(outs)
    rcs = [p.returncode for p in procs]
    assert rcs[victim] == 86, outs[victim][1][-3000:]
    for r in range(n):
        if r != victim:
            assert rcs[r] == 0, (r, outs[r][1][-4000:])
    summary = json.loads(outs[0][0].strip().splitlines()[-1])
    assert summary["recoveries"] >= 1, summary
