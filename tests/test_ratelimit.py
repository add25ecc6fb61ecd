"""Token bucket (reference: x/time/rate with a 256 KiB bucket, transport.go:407-424),
run on a virtual clock: the waits are the bucket's own schedule, exact."""

import pytest


def test_unlimited_is_one_piece(core):
    secs, pieces = core.token_bucket_pace(10 << 20, 0)
    assert pieces == [10 << 20] and secs == 0.0  # quirk Q1: rate 0 = unlimited


def test_pieces_are_burst_sized(core):
    _, pieces = core.token_bucket_pace(1_000_000, 100 << 20)
    assert sum(pieces) == 1_000_000
    assert all(p == 256 << 10 for p in pieces[:-1]) and 0 < pieces[-1] <= 256 << 10


def test_rate_is_enforced_after_the_initial_burst(core):
    # 1 MiB at 2 MiB/s with a 256 KiB bucket: the first 256 KiB passes at once,
    # the remaining 768 KiB take ~0.375 s.
    secs, _ = core.token_bucket_pace(1 << 20, 2 << 20)
    assert secs == pytest.approx(0.375, rel=1e-9), secs


def test_small_burst(core):
    secs, pieces = core.token_bucket_pace(64 << 10, 256 << 10, 16 << 10)
    assert len(pieces) == 4 and secs == pytest.approx(0.1875, rel=1e-9), secs  # 48 KiB after the burst
