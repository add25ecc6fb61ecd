"""Checks of a `bench.py` result line from a run on real GPUs, one per rank
(tests/test_gpu_multirank.py; tests/test_benchcheck.py covers them on CPU).

On a box with 2+ GPUs a multi-rank bench must have driven RCCL's P2P/IPC
transport over xGMI: no supervised fallback attempt (utils/supervise.py), one
comm lane per directed link, and a pre-flight probe that saw every link move
data at link speed. A run that fell back to NCCL_P2P_DISABLE=1 (host memory
between the GPUs) or to fewer lanes moves the same bytes and passes every
correctness check, so these are what tell the two apart."""

PROBE_FLOOR_GBPS = 10.0  # an xGMI link moves 50-64 GB/s per direction under RCCL P2P; host bounce ~ a few


def real_multi_gpu_problems(out: dict, n: int, lanes: int, probe_floor: float = PROBE_FLOOR_GBPS) -> list:
    """What is wrong with `out` (a bench.py JSON line) for an n-rank run on n
    real GPUs with `lanes` expected comm lanes; [] if nothing."""
    bad = []
    cfg = out.get("config", {})
    if out.get("n_gpus") != n:
        bad.append(f"n_gpus {out.get('n_gpus')} != {n}")
    engine = str(cfg.get("engine", ""))
    if not engine.startswith("rccl-p2p-xgmi"):
        bad.append(f"engine {engine!r} is not rccl-p2p-xgmi")
    if cfg.get("fallback") is not None:
        bad.append(f"ran on a fallback attempt: {cfg.get('fallback')!r}")
    if cfg.get("comm_lanes") != lanes:
        bad.append(f"comm_lanes {cfg.get('comm_lanes')} != {lanes} (one per directed link)")
    probe = cfg.get("probe_lane_GBps")
    if not probe or not probe.get("concurrent"):
        bad.append("no pre-flight link probe in the result")
    else:
        conc = probe["concurrent"]
        if len(conc) != n * (n - 1):
            bad.append(f"probe covered {len(conc)} directed links, not {n * (n - 1)}")
        slow = {k: v for k, v in conc.items() if v is None or v < probe_floor}
        if slow:
            bad.append(f"probe: links below {probe_floor} GB/s: {slow}")
    return bad
