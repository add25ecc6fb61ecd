"""--inject spec parsing (utils/faults.py)."""

import pytest

from distributed_llm_dissemination_amd.utils.faults import FaultPlan, parse_inject, parse_rate


def test_parse_rate_units():
    assert parse_rate("1000") == 1000
    assert parse_rate("2.5G") == 2_500_000_000
    assert parse_rate("40MB/s") == 40_000_000
    assert parse_rate("8k") == 8000


def test_parse_inject_all_kinds():
    p = parse_inject(["drop-chunk=0.01", "kill-rank=3@2.5", "slow-link=0:1:20G", "slow-link=0:2:1M"])
    assert p.drop_chunk == 0.01
    assert p.kill == {3: 2.5}
    assert p.slow_links == {(0, 1): 20_000_000_000, (0, 2): 1_000_000}
    assert p.link_rates_from(0) == {1: 20_000_000_000, 2: 1_000_000}
    assert p.link_rates_from(1) == {}
    assert parse_inject(None) == FaultPlan()


@pytest.mark.parametrize("bad", ["drop-chunk", "drop-chunk=1.5", "kill-rank=3", "slow-link=0:1", "boom=1"])
def test_parse_inject_rejects_malformed_specs(bad):
    with pytest.raises(ValueError):
        parse_inject([bad])
