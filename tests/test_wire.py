"""Wire codec: JSON envelope + every message kind (reference: distributor/message.go)."""

import json

import pytest


def _env(core, msg):
    return json.loads(core.encode_envelope(msg))


def _msg(core, t, **kw):
    m = core.Message()
    m.type = t
    for k, v in kw.items():
        setattr(m, k, v)
    return m


def test_announce_envelope_field_names(core):
    m = _msg(core, core.MsgType.Announce, src=3)
    m.layers = {5: core.LayerMeta(core.Location.Disk, 1000, core.SourceType.Disk, 64)}
    env = _env(core, m)
    assert env["type"] == 0 and env["src"] == "3"
    assert env["payload"]["SrcID"] == 3
    assert env["payload"]["LayerIDs"]["5"] == {"Location": 1, "LimitRate": 1000, "SourceType": 1, "DataSize": 64}
    back = core.decode_envelope(core.encode_envelope(m))
    assert back.type == core.MsgType.Announce and back.src == 3
    assert back.layers[5].location == core.Location.Disk and back.layers[5].limit_rate == 1000


@pytest.mark.parametrize(
    "t,fields,keys",
    [
        ("Ack", dict(src=2, layer=7, location=None), {"SrcID", "LayerID", "Location"}),
        ("Retransmit", dict(src=0, layer=4, dest=6), {"SrcID", "LayerID", "DestID"}),
        ("FlowRetransmit", dict(src=0, layer=4, dest=6, data_size=100, offset=50, rate=9),
         {"SrcID", "LayerID", "DestID", "DataSize", "Offset", "Rate"}),
        ("ClientReq", dict(src=1, layer=2, save_disk=True), {"SrcID", "LayerID", "SaveDisk"}),
        ("Startup", dict(src=0), {"SrcID"}),
    ],
)
def test_control_messages_roundtrip(core, t, fields, keys):
    if "location" in fields:
        fields["location"] = core.Location.Device
    m = _msg(core, getattr(core.MsgType, t), **fields)
    env = _env(core, m)
    assert set(env["payload"]) == keys
    back = core.decode_envelope(core.encode_envelope(m))
    for k, v in fields.items():
        assert getattr(back, k) == v, k


def test_simple_message_uses_src_addr(core):
    m = core.simple_msg("peer1", "hi from peer1")
    env = _env(core, m)
    assert env == {"type": 7, "src": "peer1", "payload": {"SrcAddr": "peer1", "PayloadStr": "hi from peer1"}}


def test_layer_header_keeps_reference_typo(core):
    m = _msg(core, core.MsgType.Layer, src=1, layer=3, data_size=10, total_size=40, offset=20)
    env = _env(core, m)
    assert env["type"] == 2
    assert env["payload"] == {"SrcID": 1, "LayerID": 3, "LayerSize": 10, "TotalSize": 40, "Offert": 20}
    back = core.decode_envelope(core.encode_envelope(m))
    assert (back.offset, back.data_size, back.total_size) == (20, 10, 40)


def test_client_id_is_max_uint64(core):
    assert core.CLIENT_ID == 2**64 - 1
    m = _msg(core, core.MsgType.Ack, src=core.CLIENT_ID, layer=1)
    assert core.decode_envelope(core.encode_envelope(m)).src == core.CLIENT_ID


def test_reference_style_ack_without_location(core):
    # The reference's ackMsg.location is unexported, so it never reaches the wire.
    back = core.decode_envelope('{"type":1,"src":"4","payload":{"SrcID":4,"LayerID":9}}')
    assert back.layer == 9 and back.location == core.Location.Inmem


def test_unknown_type_rejected(core):
    with pytest.raises(Exception):
        core.decode_envelope('{"type":200,"src":"1","payload":{}}')


def test_stream_framing_parse_prefix(core):
    a = core.encode_envelope(core.simple_msg("x", "one")).decode()
    b = core.encode_envelope(core.simple_msg("x", "two")).decode()
    stream = a + b
    n, first = core.json_parse_prefix(stream)
    assert n == len(a) and json.loads(first)["payload"]["PayloadStr"] == "one"
    # Truncated value -> need more bytes.
    assert core.json_parse_prefix(stream[: len(a) - 3])[0] == 0
    with pytest.raises(Exception):
        core.json_parse_prefix("{]")


def test_json_unicode_and_big_ints(core):
    s = '{"a":"\\u00e9\\ud83d\\ude00","b":18446744073709551615,"c":-5,"d":1.5e3}'
    out = json.loads(core.json_roundtrip(s))
    assert out == {"a": "é😀", "b": 18446744073709551615, "c": -5, "d": 1500.0}


@pytest.mark.parametrize("order", [0, 1])
def test_xfer_batch_fast_path_matches_dom(core, order):
    """Transfer batches are written straight to text and read back by a cursor
    (wire.cc fast path): the text must equal the JSON DOM's, and both decoders
    give back every job field, the CRCs and the lane order (Message.order:
    1 = job-major lanes for mode-2 pull batches, omitted when 0)."""
    m = _msg(core, core.MsgType.XferBatch, src=0, epoch=3, batch=7, order=order)
    jobs = []
    for k in range(3):
        j = core.XferJob()
        j.seq, j.src, j.dst, j.layer = 10 + k, k, k + 1, 40 + k
        j.offset, j.size, j.total, j.chunk_bytes = k * 4096, 8192, 65536, 4096
        j.crc = [0xDEADBEEF, k, 0xFFFFFFFF]
        j.rate = 0 if k else 123456
        jobs.append(j)
    m.jobs = jobs
    text = core.encode_envelope(m)
    env = json.loads(text)
    assert ("Order" in env["payload"]) == (order == 1)
    assert core.json_roundtrip(text.decode()) == text.decode()  # sorted keys, no whitespace: the DOM's own text
    for back in (core.decode_envelope(text.decode()), core.decode_envelope_text(text.decode())):
        assert back.type == core.MsgType.XferBatch and back.batch == 7 and back.order == order and back.epoch == 3
        got = [(j.seq, j.src, j.dst, j.layer, j.offset, j.size, j.total, j.chunk_bytes, list(j.crc), j.rate)
               for j in back.jobs]
        want = [(j.seq, j.src, j.dst, j.layer, j.offset, j.size, j.total, j.chunk_bytes, list(j.crc), j.rate)
                for j in jobs]
        assert got == want
