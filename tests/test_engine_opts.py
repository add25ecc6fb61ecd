"""CLI -> planned-engine knobs (the rccl engine's PlannedConfig), CPU only."""

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.__main__ import build_parser, engine_opts


def test_verify_partition_flags_reach_the_engine_config():
    args = build_parser().parse_args(["-id", "0", "-f", "x.json", "--verify-cus", "48",
                                      "--comm-init", "parallel", "--nccl-ctas", "2:8"])
    opts = engine_opts(args)
    assert opts["verify_cus"] == 48 and opts["comm_init"] == "parallel"
    assert (opts["nccl_min_ctas"], opts["nccl_max_ctas"]) == (2, 8)
    cfg = _core.PlannedConfig()
    for k in ("verify_cus", "comm_init", "nccl_min_ctas", "nccl_max_ctas"):
        setattr(cfg, k, opts[k])
    assert (cfg.verify_cus, cfg.comm_init) == (48, "parallel")


def test_defaults_leave_the_choice_to_the_backend():
    """-1: the backend picks (32 verify CUs with peers, 128 with the fused unpack, 0 alone);
    split communicator init."""
    opts = engine_opts(build_parser().parse_args(["-id", "0", "-f", "x.json"]))
    assert opts["verify_cus"] == -1 and opts["comm_init"] == "split"
    cfg = _core.PlannedConfig()
    assert cfg.verify_cus == -1 and cfg.comm_init == "split"
