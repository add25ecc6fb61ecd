"""CLI -> planned-engine knobs (the rccl engine's PlannedConfig), CPU only."""

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.__main__ import build_parser, engine_opts


def test_verify_partition_flags_reach_the_engine_config():
    args = build_parser().parse_args(["-id", "0", "-f", "x.json", "--verify-cus", "48", "--lanes", "7",
                                      "--suspect-timeout", "2"])
    opts = engine_opts(args)
    assert (opts["verify_cus"], opts["lanes"], opts["suspect_s"]) == (48, 7, 2.0)
    cfg = _core.PlannedConfig()
    for k, v in opts.items():
        setattr(cfg, k, v)  # every knob is a PlannedConfig field
    assert (cfg.verify_cus, cfg.lanes) == (48, 7)


def test_defaults_leave_the_choice_to_the_backend():
    """-1: the backend picks (32 verify CUs with peers, 128 with the fused unpack, 0 alone);
    split communicator init."""
    opts = engine_opts(build_parser().parse_args(["-id", "0", "-f", "x.json"]))
    assert opts["verify_cus"] == -1 and opts["comm_init"] == "split"
    cfg = _core.PlannedConfig()
    assert cfg.verify_cus == -1 and cfg.comm_init == "split"


def test_cli_stays_small():
    """The reference's seven flags plus the extensions a recipe or test uses (<= 30)."""
    flags = [a for a in build_parser()._actions if a.option_strings and a.dest != "help"]
    assert len(flags) <= 30, [a.option_strings[0] for a in flags]
