"""Pin the CPU oracle against the reference's own known-answer tests (CPU only).

Each fixture vector cites the snf4j test assertion it transcribes
(tests/golden/make_golden.py).  The oracle is the parity checker for the HIP
path, so it must reproduce every one of them exactly.
"""
import pytest

from tests.golden import fixtures, make_golden


def test_frame_builder_matches_reference_testFrame():
    # FrameDecoderTest.testFrame :189-219 — the fixture builder is itself pinned
    for v in fixtures.load("builder"):
        assert make_golden.frame(v["spec"]).hex() == fixtures.unhex(v["bytes"]).hex(), v["spec"]


def _check_frame(f, exp):
    assert f is not None
    assert f.opcode == exp["opcode"]
    assert f.fin == exp["fin"]
    assert f.rsv == exp["rsv"]
    assert f.payload == fixtures.unhex(exp["payload"])


@pytest.mark.parametrize("idx", range(len(fixtures.load("decode"))))
def test_decode_kat(oracle, idx):
    v = fixtures.load("decode")[idx]
    dec = oracle.Decoder(v["client_mode"], v["allow_extensions"], v["max_payload"], True)
    for st in v["steps"]:
        if "available" in st:
            data = fixtures.unhex(st["available"])
            assert dec.available(data, 0, len(data)) == st["expect"], v["src"]
            continue
        data = fixtures.unhex(st["data"])
        if "error" in st:
            with pytest.raises(oracle.InvalidFrame) as ei:
                dec.decode(data)
            assert str(ei.value) == st["error"], v["src"]
            assert ei.value.close_code == st["close_code"]
            assert dec.closed
        elif st.get("none"):
            assert dec.decode(data) is None, v["src"]
        else:
            _check_frame(dec.decode(data), st["frame"])


def _assert_available(oracle, data, off, expected_len, payload_len):
    # FrameDecoderTest.assertAvailable :221-232
    dec = oracle.Decoder(True, True, 2400)
    min_len = expected_len - payload_len
    assert dec.available(data, off, expected_len) == expected_len
    assert dec.available(data, off, expected_len + 1) == expected_len
    lens = range(expected_len)
    if expected_len > 1024:  # every value near the header, a stride through the payload
        lens = list(range(0, min_len + 256)) + list(range(min_len + 256, expected_len, 97))
    for ln in lens:
        assert dec.available(data, off, ln) == (ln if ln >= min_len else 0), (off, ln)


def test_available_kat(oracle):
    av = fixtures.load("available")
    for c in av["frames"]:
        data = make_golden.frame(c["data_spec"], c["off"])
        _assert_available(oracle, data, c["off"], c["expected_len"], c["payload_len"])
    for c in av["big"]:
        dec = oracle.Decoder(True, True, 2400)
        data = fixtures.unhex(c["data"])
        if "error" in c:
            with pytest.raises(oracle.InvalidFrame) as ei:
                dec.available(data, 0, c["len"])
            assert str(ei.value) == c["error"]
            assert dec.closed
        else:
            assert dec.available(data, 0, c["len"]) == c["expect"]


def test_available_every_length_kat(oracle):
    # FrameDecoderTest.testAvailableArray :310-322: off 5, every payload length 0..65534
    dec = oracle.Decoder(True, True, 2400)
    for i in list(range(0, 126)) + list(range(126, 0xFFFF, 61)):
        f = make_golden.frame(f"FRRR1|{i}|M|-|", 5)
        n = make_golden.frame_len(i, True)
        assert dec.available(f, 5, n) == n


def test_split_frame_available_kat(oracle):
    # FrameDecoderTest.testSplittedFrameAvailable :678-696
    sp = fixtures.load("available")["split"]
    dec = oracle.Decoder(True, True, 0x20000)
    first = fixtures.unhex(sp["first"])
    assert dec.available(first, 0, len(first)) == sp["checks"][0]["expect_before"]
    assert dec.decode(first) is None
    for c in sp["checks"][1:]:
        d = fixtures.unhex(c["data"])
        assert dec.available(d, 0, len(d)) == c["expect"]


def test_validator_kat(oracle):
    # FrameUtf8ValidatorTest.testDecode :81-133
    for seq in fixtures.load("validator"):
        v = oracle.Validator()
        for f in seq["frames"]:
            ok = v.decode(f["opcode"], f["fin"], bytes.fromhex(f["payload"]))
            assert ok == ("error" not in f), (seq["src"], f)
            if not ok:
                v = oracle.Validator()  # the reference test uses a fresh validator after a throw


def _encoder_layout(b: bytes) -> str:
    """FrameEncoderTest.frame(ByteBuffer) :45-104 — the layout string of an encoded frame."""
    i = 0
    b0 = b[i]; i += 1
    s = ("F" if b0 & 0x80 else "f") + ("R" if b0 & 0x40 else "r") + ("R" if b0 & 0x20 else "r")
    s += ("R" if b0 & 0x10 else "r") + str(b0 & 0x0F)
    b1 = b[i]; i += 1
    masked = bool(b1 & 0x80)
    s += ("M" if masked else "m") + "|" + str(b1 & 0x7F) + "|"
    ln = b1 & 0x7F
    if ln == 126:
        ln = int.from_bytes(b[i:i + 2], "big"); i += 2
        s += f"{ln}(2)"
    elif ln == 127:
        ln = int.from_bytes(b[i:i + 8], "big"); i += 8
        s += f"{ln}(8)"
    mask = b""
    if masked:
        mask = b[i:i + 4]; i += 4
        s += "M(4)"
    rest = bytearray(b[i:])
    if ln == len(rest):
        s += "="
    if rest:
        if masked:
            for j in range(len(rest)):
                rest[j] ^= mask[j % 4]
        t = rest.decode("latin-1")
        s += (t[:10] + "..." + t[-10:]) if len(t) > 20 else t
    return s


def test_encoder_kat(oracle):
    # FrameEncoderTest.testEncode :136-207 (masks are injected instead of java.util.Random)
    for i, v in enumerate(fixtures.load("encoder")):
        enc = oracle.Encoder(v["client_mode"])
        payload = fixtures.unhex(v["payload"])
        mask = (0x11 * (i % 7 + 1), 0x5A, 0xA5, i & 0xFF)
        out = enc.encode(v["opcode"], v["fin"], v["rsv"], payload, mask)
        assert len(out) == oracle.encoded_length(len(payload), v["client_mode"])
        assert _encoder_layout(out) == v["expect"], v["expect"]


def test_encoder_masking_and_close_latch(oracle):
    # FrameEncoderTest.testMasking :209-226 and FrameEncoder.java:71-76
    enc = oracle.Encoder(True)
    p = b"ABCDEFGHIJ"
    out = enc.encode(2, True, 0, p, (9, 8, 7, 6))
    assert len(out) == 16
    assert bytes(out[6 + i] ^ out[2 + i % 4] for i in range(10)) == p
    assert enc.encode(8, True, 0, b"", (0, 0, 0, 0)) != b""
    assert enc.encode(2, True, 0, p, (1, 2, 3, 4)) == b""  # closed: dropped
    enc = oracle.Encoder(False)
    assert enc.encode(2, True, 0, p)[2:] == p


@pytest.mark.parametrize("idx", range(len(fixtures.load("session"))))
def test_session_stream_kat(oracle, idx):
    # WebSocketSessionTest stream cases through the session read loop
    v = fixtures.load("session")[idx]
    chunks = [fixtures.unhex(c) for c in v["chunks"]]
    stream = b"".join(chunks)
    frames, err = oracle.stream_decode(stream, [len(c) for c in chunks], client_mode=v["client_mode"],
                                       allow_extensions=False, max_payload_len=v["max_payload"])
    assert len(frames) == len(v["frames"])
    for f, e in zip(frames, v["frames"]):
        _check_frame(f, e)
    if "error" in v:
        assert err is not None and str(err) == v["error"]
        assert err.close_code == v["close_code"]
    else:
        assert err is None


def test_stream_chunking_independence(oracle):
    """Outputs do not depend on how bytes are chunked (SURVEY.md §8a notes)."""
    import numpy as np
    rng = np.random.default_rng(7)
    enc = oracle.Encoder(True)
    parts = []
    for k in range(60):
        n = int(rng.integers(0, 3000))
        op = 1 if k % 3 == 0 else 2
        payload = ("é" * (n // 2)).encode() if op == 1 else rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        parts.append(enc.encode(op, True, 0, payload, tuple(int(x) for x in rng.integers(0, 256, 4))))
    stream = b"".join(parts)
    ref, err = oracle.stream_decode(stream, [len(stream)])
    assert err is None and len(ref) == 60
    for chunks in ([1], [7], [13, 2, 8192], [8192]):
        got, err = oracle.stream_decode(stream, chunks)
        assert err is None
        assert [(f.opcode, f.payload) for f in got] == [(f.opcode, f.payload) for f in ref]


def test_aggregator_kat(oracle):
    """FrameAggregatorTest / WebSocketSessionTest.testFrameAggregation vectors through the
    oracle's FrameAggregator restatement."""
    for seq in fixtures.load("aggregator"):
        agg = oracle.Aggregator(seq["max"])
        for i, f in enumerate(seq["frames"]):
            exp = f["expect"]
            payload = fixtures.unhex(f["payload"])
            if "error" in exp:
                with pytest.raises(oracle.InvalidFrame) as ei:
                    agg.decode(f["opcode"], f["fin"], f["rsv"], payload)
                assert str(ei.value) == exp["error"] and ei.value.close_code == exp["close_code"], (seq["src"], i)
                break
            got = agg.decode(f["opcode"], f["fin"], f["rsv"], payload)
            if not exp["out"]:
                assert got is None, (seq["src"], i)
                continue
            o = exp["out"][0]
            assert (got.opcode, got.fin, got.rsv, got.payload) == \
                   (o["opcode"], o["fin"], o["rsv"], fixtures.unhex(o["payload"])), (seq["src"], i)


def test_deflate_kat(oracle):
    """PerMessageDeflateCodecTest vectors through the oracle's PerMessageDeflateDecoder
    restatement (inputs deflated as PerMessageDeflateEncoder does, tests/wsgen.py)."""
    from tests.wsgen import pm_deflate_encode
    for seq in fixtures.load("deflate"):
        frames = [(f["opcode"], f["fin"], f["rsv"], fixtures.unhex(f["payload"])) for f in seq["frames"]]
        if seq["kind"] == "pass_through":
            d = oracle.PerMessageDeflateDecoder(seq["no_context"])
            for fr in frames:
                assert d.decode(*fr) == (fr[0], fr[1], fr[2], fr[3]), seq["src"]
            continue
        enc = pm_deflate_encode(frames, seq["level"], seq["no_context"])
        for e, f, src in zip(enc, frames, seq["frames"]):
            assert e[2] == f[2] | src["rsv_mask"], seq["src"]
        if seq["kind"] == "round_trip":
            d = oracle.PerMessageDeflateDecoder(seq["no_context"])
            for e, f in zip(enc, frames):
                assert d.decode(*e) == f, seq["src"]
        else:  # the second message of a context-takeover stream, to a fresh decoder
            d = oracle.PerMessageDeflateDecoder(seq["no_context"])
            with pytest.raises(oracle.InvalidFrame) as ei:
                d.decode(*enc[1])
            assert oracle.format_error(ei.value.err) == seq["error"], seq["src"]


HS_KIND = {"need_more": 0, "defer": 1, "parse_error": 2, "accept": 3, "finished": 4, "closing": 5}


def _hs_cause(name):
    from snf4j_amd.handshake import CAUSE_NAMES
    return {v: k for k, v in CAUSE_NAMES.items()}[name]


def hs_cfg(c):
    return dict(max_length=c.get("max_length", 65536), ignore_host=bool(c.get("ignore_host", 0)))


@pytest.mark.parametrize("idx", range(len(fixtures.load("handshake"))))
def test_handshake_kat(idx):
    """The handshake restatement against HttpUtilsTest / HandshakeUtilsTest /
    HandshakeDecoderTest / HanshakerTest vectors."""
    from oracle import handshake_oracle as H
    v = fixtures.load("handshake")[idx]
    if v["kind"] == "available":
        data = fixtures.unhex(v["data"])
        n, lines, _ = H.available(data, v["lines_len"])
        assert n == v["expect"], v
        assert [data[b:e].decode() for b, e in lines] == v["lines"], v
    elif v["kind"] == "split_request_line":
        data = fixtures.unhex(v["data"])
        assert [data[b:e].decode() for b, e in H.split_request_line(data, 0, len(data), 50)] == v["items"], v
    elif v["kind"] == "answer_key":
        assert H.answer_key(v["key"]) == v["accept"]
    elif v["kind"] == "parse_key":
        k = H.base64_decode(v["key"])
        assert (k is not None and len(k) == 16) == v["valid"], v
    else:
        r = H.accept(fixtures.unhex(v["request"]), **hs_cfg(v["cfg"]))
        e = v["expect"]
        assert r["kind"] == HS_KIND[e["kind"]], (v, r)
        assert r["status"] == e["status"] and r["cause"] == _hs_cause(e["cause"]), (v, r)
        assert r["detail"] == e["detail"], (v, r)
        if "response" in e:
            assert r["response"] == fixtures.unhex(e["response"]), (v, r)


@pytest.mark.parametrize("idx", range(len(fixtures.load("handshake_client"))))
def test_handshake_client_kat(idx):
    """The client-side restatement (response parse + Handshaker.validate) against the
    HandshakeFactoryTest / HandshakeDecoderTest / HanshakerTest client vectors."""
    from oracle import handshake_oracle as H
    v = fixtures.load("handshake_client")[idx]
    c = v["cfg"]
    r = H.validate(fixtures.unhex(v["response"]), v["key"], c.get("max_length", 65536), c.get("subprotocols"),
                   bool(c.get("extensions", False)))
    e = v["expect"]
    assert r["kind"] == HS_KIND[e["kind"]], (v, r)
    assert r["status"] == e["status"] and r["cause"] == _hs_cause(e["cause"]), (v, r)
    assert r["detail"] == e["detail"] and r["subprotocol"] == e["subprotocol"], (v, r)
    if e["cause"] == "INVALID_ACCEPT":  # "... Expected: " + generateAnswerKey(key), ending in "="
        assert r["expected"] == H.answer_key(v["key"]) and r["expected"].endswith("=")
