"""NUMA placement helpers (utils/numa.py) on fake sysfs trees (CPU)."""

import os

from distributed_llm_dissemination_amd.utils import numa


def test_parse_cpulist():
    assert numa.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa.parse_cpulist("") == set()


def test_node_cpus_and_gpu_node_from_sysfs(tmp_path, monkeypatch):
    node = tmp_path / "devices/system/node/node1"
    node.mkdir(parents=True)
    (node / "cpulist").write_text("4-7\n")
    dev = tmp_path / "bus/pci/devices/0000:75:00.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text("1\n")
    monkeypatch.setattr(numa, "pci_bdf", lambda d: "0000:75:00.0")
    assert numa.gpu_numa_node(0, sysfs=str(tmp_path)) == 1
    assert numa.node_cpus(1, sysfs=str(tmp_path)) == {4, 5, 6, 7}
    assert numa.node_cpus(3, sysfs=str(tmp_path)) == set()


def test_bind_is_a_no_op_when_the_node_is_unknown(monkeypatch):
    before = os.sched_getaffinity(0)
    monkeypatch.setattr(numa, "gpu_numa_node", lambda d: -1)
    assert numa.bind_to_gpu(0) == {}
    monkeypatch.setattr(numa, "gpu_numa_node", lambda d: 0)
    monkeypatch.setattr(numa, "node_cpus", lambda n: set())  # cpuset excludes the node
    assert numa.bind_to_gpu(0) == {}
    assert os.sched_getaffinity(0) == before


def test_bind_restricts_to_the_nodes_cpus_in_this_cpuset(monkeypatch):
    import threading

    allowed = sorted(os.sched_getaffinity(0))
    got = {}

    def run():  # on a thread of its own: affinity is per thread
        monkeypatch.setattr(numa, "gpu_numa_node", lambda d: 0)
        monkeypatch.setattr(numa, "node_cpus", lambda n: set(allowed[:1]) | {10_000})
        monkeypatch.setattr(numa, "_prefer_node", lambda n: True)
        got["r"] = numa.bind_to_gpu(0)
        got["aff"] = os.sched_getaffinity(0)

    t = threading.Thread(target=run)
    t.start()
    t.join()
    assert got["r"] == {"numa_node": 0, "cpus": 1, "mempolicy": 1}
    assert got["aff"] == {allowed[0]}
