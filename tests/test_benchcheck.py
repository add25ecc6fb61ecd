"""The multi-GPU result checks (tests/benchcheck.py) on hand-made result lines."""

from benchcheck import real_multi_gpu_problems


def _line(n=8, engine="rccl-p2p-xgmi, 14 comm lanes", fallback=None, lanes=14, rate=55.0, drop=None):
    conc = {f"{s}->{d}": rate for s in range(n) for d in range(n) if s != d}
    if drop:
        conc.pop(drop)
    return {"n_gpus": n, "config": {"engine": engine, "fallback": fallback, "comm_lanes": lanes,
                                    "probe_lane_GBps": {"MiB": 256, "concurrent": conc, "solo": {}}}}


def test_a_real_8_gpu_run_passes():
    assert real_multi_gpu_problems(_line(), 8, 14) == []


def test_fallbacks_and_shared_gpu_runs_fail():
    assert real_multi_gpu_problems(_line(fallback="lanes=7, NCCL_P2P_DISABLE=1"), 8, 14)
    assert real_multi_gpu_problems(_line(engine="rccl-socket, all ranks on one GPU (schedule rehearsal)"), 8, 14)
    assert real_multi_gpu_problems(_line(lanes=7), 8, 14)


def test_slow_or_missing_probe_links_fail():
    probs = real_multi_gpu_problems(_line(rate=3.0), 8, 14)
    assert any("below" in p for p in probs), probs
    assert real_multi_gpu_problems(_line(drop="3->4"), 8, 14)
    line = _line()
    del line["config"]["probe_lane_GBps"]
    assert real_multi_gpu_problems(line, 8, 14)
