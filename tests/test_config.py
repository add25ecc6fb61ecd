"""Config schema (reference: cmd/config.go, readme.md, conf/config.json)."""

import json

import pytest

from distributed_llm_dissemination_amd.utils.config import (
    SOURCE_DISK,
    SOURCE_MEM,
    ConfigError,
    example_config,
    load_config,
    parse_config,
)

# Same shape as the reference experiment conf/config.json: 8 nodes, nodes 0-6 hold
# layers 0-7 on disk (source 1), node 7 holds nothing and is assigned all 8.
LAYER = 10930691768


def reference_like():
    nodes = []
    for i in range(8):
        n = {"Id": i, "Addr": f":{8080 + i}", "NetworkBW": 1562500000, "IsLeader": i == 0}
        if i < 7:
            n["Sources"] = {"0": 16257500, "1": 209715200}
            n["InitialLayers"] = {"1": {str(l): {"LayerSize": LAYER} for l in range(8)}}
        else:
            n["InitialLayers"] = {}
        nodes.append(n)
    return {"Nodes": nodes, "Assignment": {"7": {str(l): {} for l in range(8)}}}


def test_nested_schema_like_reference_experiment():
    cfg = parse_config(reference_like())
    assert cfg.leader().id == 0
    assert cfg.node(3).initial_layers[SOURCE_DISK][5] == LAYER
    assert cfg.node(3).sources == {0: 16257500, 1: 209715200}
    assert cfg.assignment == {7: list(range(8))}
    assert cfg.node(7).initial_layers == {}
    assert cfg.layer_sizes()[2] == LAYER
    assert cfg.network_bw()[5] == 1562500000


def test_readme_flat_schema():
    raw = {
        "Nodes": [
            {"Id": 0, "Addr": "a:8080", "IsLeader": True, "InitialLayers": {"1": {}, "3": {}}},
            {"Id": 1, "Addr": "b:8080", "IsLeader": False, "InitialLayers": {"1": {}}},
            {"Id": 2, "Addr": "c:8080", "IsLeader": False, "InitialLayers": {}},
        ],
        "Assignment": {"1": {"1": {}}, "2": {"1": {}, "3": {}}},
        "LayerSize": 1048576,
    }
    cfg = parse_config(raw)
    assert cfg.node(0).initial_layers == {SOURCE_MEM: {1: 1048576, 3: 1048576}}
    assert cfg.node(2).initial_layers == {}
    assert cfg.assignment == {1: [1], 2: [1, 3]}


def test_case_insensitive_keys_and_negative_sizes_clamped():
    raw = {"nodes": [{"ID": 0, "isleader": True, "initiallayers": {"2": {"4": {"layersize": -5}}}}]}
    cfg = parse_config(raw)
    assert cfg.node(0).initial_layers == {2: {4: 0}}


def test_errors_are_raised_not_swallowed(tmp_path):
    p = tmp_path / "bad.json"
    p.write_text("{not json")
    with pytest.raises(ConfigError):
        load_config(str(p))
    with pytest.raises(ConfigError):
        parse_config({"Nodes": [{"Id": 0}]})  # no leader
    with pytest.raises(ConfigError):
        parse_config({"Nodes": [{"Id": 0, "IsLeader": True}], "Assignment": {"9": {}}})


def test_roundtrip_and_example(tmp_path):
    cfg = parse_config(reference_like())
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg.to_json()))
    again = load_config(str(p))
    assert again.assignment == cfg.assignment and again.node(4).initial_layers == cfg.node(4).initial_layers
    ex = example_config()
    assert ex.leader().id == 0 and ex.assignment[2] == [1, 3]


def test_clients_section():
    raw = reference_like()
    raw["Clients"] = [{"ID": 7, "Addr": ":9000", "Layers": {"3": 100}}]
    raw["LayerSize"] = 4096
    cfg = parse_config(raw)
    assert cfg.client(7).layers == {3: 100} and cfg.client(1) is None


# ---- the shipped configs (conf/*.json), parsed by the strict loader
import glob  # noqa: E402
import os  # noqa: E402

CONF = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conf")
CONF_FILES = sorted(glob.glob(os.path.join(CONF, "*.json")))


def test_conf_dir_holds_the_shipped_configs():
    names = {os.path.basename(p) for p in CONF_FILES}
    assert {"reference_ec2_mode3.json", "loopback_4x1MiB.json"} <= names, names


@pytest.mark.parametrize("path", CONF_FILES, ids=os.path.basename)
def test_every_shipped_config_loads(path):
    """Every conf/*.json parses under the strict loader; its assignment names
    only known nodes and every assigned layer has a size (held somewhere, a
    client's, or the top-level LayerSize)."""
    cfg = load_config(path)
    ids = {n.id for n in cfg.nodes}
    assert cfg.leader().id in ids
    sizes = cfg.layer_sizes()
    for node, layers in cfg.assignment.items():
        assert node in ids
        for l in layers:
            assert sizes.get(l, 0) > 0, (path, node, l)


def test_reference_experiment_file_parses_unchanged():
    """conf/reference_ec2_mode3.json is the reference's conf/config.json
    (/root/reference/conf/config.json:1-289) with loopback addresses: the
    nested schema of cmd/config.go:14-45 exactly as ReadJson reads it."""
    cfg = load_config(os.path.join(CONF, "reference_ec2_mode3.json"))
    assert [n.id for n in cfg.nodes] == list(range(8)) and cfg.leader().id == 0
    for i in range(7):
        n = cfg.node(i)
        assert n.network_bw == 1562500000
        assert n.sources == {0: 16257500, 1: 209715200}
        assert n.initial_layers == {SOURCE_DISK: {l: LAYER for l in range(8)}}
    assert cfg.node(7).initial_layers in ({}, {SOURCE_DISK: {}})
    assert cfg.assignment == {7: list(range(8))}


def test_reference_experiment_mode3_plan_is_60_s():
    """The reference's solver on its own experiment file (flow.go:146-219,
    whole-second bisection): the binding cut is the 7 senders' disk tiers,
    7 x 200 MiB/s = 1.468 GB/s against 8 x 10.93 GB = 87.45 GB, so T = 59.57 s
    rounds up to 60 s (derived). Our planner on the same problem
    (runtime.mode3_plan: what the mode-3 leader builds from the announces)
    gives T = 60 s, and its byte ranges partition every layer exactly once."""
    from distributed_llm_dissemination_amd.parallel.runtime import mode3_plan

    cfg = load_config(os.path.join(CONF, "reference_ec2_mode3.json"))
    p = mode3_plan(cfg, integer_seconds=True)
    assert p.feasible and p.T == 60.0, (p.T, p.feasible)
    assert p.required == 8 * LAYER
    per_layer = {}
    for j in p.jobs:
        assert j.dest == 7 and 0 <= j.sender <= 6 and j.size > 0
        per_layer.setdefault(j.layer, []).append((j.offset, j.size))
    assert sorted(per_layer) == list(range(8))
    for l, rs in per_layer.items():
        pos = 0
        for off, sz in sorted(rs):
            assert off == pos, (l, rs)
            pos += sz
        assert pos == LAYER, (l, pos)
    # at T each sender's disk tier carries at most its rate x T (the binding budget)
    sent = {}
    for j in p.jobs:
        sent[j.sender] = sent.get(j.sender, 0) + j.size
    assert all(b <= 209715200 * 60 for b in sent.values()), sent
    # without whole seconds the same cut gives the continuous T
    q = mode3_plan(cfg, integer_seconds=False)
    assert q.T == pytest.approx(8 * LAYER / (7 * 209715200), rel=1e-6)
