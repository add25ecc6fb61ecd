"""Transport unit tests (reference: distributor/transport_test.go), for the
in-process fake and the TCP transport on ephemeral loopback ports."""

import itertools

import pytest

_ids = itertools.count()


def make_pair(core, kind):
    if kind == "inproc":
        tag = next(_ids)
        reg = {1: f"p1-{tag}", 2: f"p2-{tag}"}
        return core.inproc_transport(reg[1], reg), core.inproc_transport(reg[2], reg)
    p1 = core.tcp_transport("127.0.0.1:0")
    p2 = core.tcp_transport("127.0.0.1:0")
    reg = {1: p1.address(), 2: p2.address()}
    p1.set_registry(reg)
    p2.set_registry(reg)
    return p1, p2


@pytest.fixture(params=["inproc", "tcp"])
def pair(core, request):
    p1, p2 = make_pair(core, request.param)
    yield p1, p2
    p1.close()
    p2.close()


def test_send_single(core, pair):
    p1, p2 = pair
    p1.send(2, core.simple_msg(p1.address(), "hi from peer1"))
    m = p2.deliver(1.0)
    assert m is not None and m.payload_str == "hi from peer1" and m.src_addr == p1.address()


def test_send_three_in_order(core, pair):
    p1, p2 = pair
    for i in range(3):
        p1.send(2, core.simple_msg(p1.address(), f"hi{i}"))
    got = [p2.deliver(1.0) for _ in range(3)]
    assert [m.payload_str for m in got] == ["hi0", "hi1", "hi2"]


def test_broadcast_single(core, pair):
    p1, p2 = pair
    p1.broadcast(core.simple_msg(p1.address(), "broadcast value"))
    m = p2.deliver(1.0)
    assert m is not None and m.payload_str == "broadcast value"


def test_send_to_unknown_peer_raises(core, pair):
    p1, _ = pair
    with pytest.raises(Exception):
        p1.send(99, core.simple_msg("x", "y"))


def test_tcp_self_send_short_circuits(core):
    t = core.tcp_transport("127.0.0.1:0")
    t.set_registry({5: t.address()})
    t.send(5, core.simple_msg("me", "loop"))
    assert t.deliver(1.0).payload_str == "loop"
    t.close()


def test_many_messages_stream_framing(core):
    p1, p2 = make_pair(core, "tcp")
    for i in range(500):
        p1.send(2, core.simple_msg("a", "x" * (i % 37) + str(i)))
    got = [p2.deliver(2.0) for _ in range(500)]
    assert [m.payload_str for m in got] == ["x" * (i % 37) + str(i) for i in range(500)]
    p1.close()
    p2.close()
