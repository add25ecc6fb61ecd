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


# ---- a misbehaving peer is disconnected before this process buffers or
# allocates what it claims (tcp.cc read_loop / receive_layer)

def _raw_conn(t):
    import socket

    host, port = t.address().rsplit(":", 1)
    s = socket.create_connection((host, int(port)), timeout=5)
    return s


def _closed_by_peer(s, timeout=5.0):
    """True once the transport closed the connection (EOF or reset)."""
    import socket

    s.settimeout(timeout)
    try:
        while True:
            if not s.recv(65536):
                return True
    except (ConnectionResetError, BrokenPipeError):
        return True
    except socket.timeout:
        return False


def test_tcp_drops_oversized_envelope(core):
    t = core.tcp_transport("127.0.0.1:0")
    t.set_max_envelope(1 << 16)
    s = _raw_conn(t)
    try:
        chunk = b'{"type":7,"src":"x","payload":{"PayloadStr":"' + b"a" * 4096
        try:
            for _ in range(64):  # 256 KiB of one never-terminated envelope, 4x the limit
                s.sendall(b"a" * 4096 if _ else chunk)
        except (ConnectionResetError, BrokenPipeError):
            pass
        assert _closed_by_peer(s)
        assert t.deliver(0.2) is None
        # the transport still serves other peers
        t.set_registry({5: t.address()})
        t.send(5, core.simple_msg("me", "still here"))
        assert t.deliver(2.0).payload_str == "still here"
    finally:
        s.close()
        t.close()


def test_tcp_drops_garbage_and_keeps_framing_across_recvs(core):
    t = core.tcp_transport("127.0.0.1:0")
    s = _raw_conn(t)
    try:
        # one valid envelope split into 1-byte sends (incremental framing), a brace inside a string
        env = core.encode_envelope(core.simple_msg("p", 'a}b{"c\\\\'))
        for b in env:
            s.sendall(bytes([b]))
        assert t.deliver(2.0).payload_str == 'a}b{"c\\\\'
        s.sendall(b"xyz")  # not an envelope
        assert _closed_by_peer(s)
    finally:
        s.close()
        t.close()


@pytest.mark.parametrize("hdr", [
    dict(data_size=1 << 40, total_size=1 << 40, offset=0),   # beyond the payload limit
    dict(data_size=4096, total_size=1024, offset=0),         # range past its own TotalSize
    dict(data_size=-1, total_size=1024, offset=0),           # negative
])
def test_tcp_refuses_lying_layer_header(core, hdr):
    t = core.tcp_transport("127.0.0.1:0")
    t.set_max_payload(1 << 30)
    s = _raw_conn(t)
    try:
        m = core.Message()
        m.type = core.MsgType.Layer
        m.src = 3
        m.layer = 9
        for k, v in hdr.items():
            setattr(m, k, v)
        s.sendall(core.encode_envelope(m) + b"\0" * 64)
        assert _closed_by_peer(s)
        assert t.deliver(0.2) is None
    finally:
        s.close()
        t.close()
