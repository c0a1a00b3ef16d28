"""Client side of the opening handshake on the GPU (k_hs_validate through the C ABI):
HandshakeDecoder(clientMode) + Handshaker.validate against the CPU restatement
(oracle/handshake_oracle.py: validate), which tests/test_oracle_golden.py pins to the
reference's HandshakeFactoryTest / HandshakeDecoderTest / HanshakerTest vectors."""
import random

import pytest

from oracle import handshake_oracle as H
from tests.golden import fixtures
from tests.test_oracle_golden import HS_KIND, _hs_cause

pytestmark = pytest.mark.gpu

RFC_KEY = "dGhlIHNhbXBsZSBub25jZQ=="


def _gpu(responses, keys, max_length=65536, subprotocols=(), extensions=False):
    from snf4j_amd import BatchClientHandshaker, ClientConfig
    return BatchClientHandshaker(ClientConfig(max_length, tuple(subprotocols or ()), extensions)).validate(
        responses, keys)


def _oracle_message(r):
    m = H.MESSAGES.get(r["cause"]) if r["kind"] in (H.PARSE_ERROR, H.CLOSING) else None
    if m and "%s" in m:
        m = m % ((r["detail"], r["expected"]) if r["cause"] == H.C_INVALID_ACCEPT else r["detail"])
    return m


def _expect_equal(resp, key, g, cfg):
    d = H.gpu_defers_client(resp, key, **cfg)
    if d is not None:
        assert (g.kind, g.cause) == (H.DEFER, d), (resp, g)
        return
    r = H.validate(resp, key, **cfg)
    assert r["kind"] is not None, (resp, g)
    assert (g.kind, g.status, g.cause) == (r["kind"], r["status"], r["cause"]), (resp, g, r)
    assert g.message == _oracle_message(r), (resp, g, r)
    if r["frame_len"]:
        assert g.frame_len == r["frame_len"], (resp, g, r)
    if r["expected"] is not None:
        assert g.expected == r["expected"], (resp, g, r)


def test_handshake_client_kat_gpu():
    vs = fixtures.load("handshake_client")
    for v in vs:
        c = v["cfg"]
        cfg = dict(max_length=c.get("max_length", 65536), subprotocols=c.get("subprotocols"),
                   extensions=bool(c.get("extensions", False)))
        resp = fixtures.unhex(v["response"])
        g = _gpu([resp], [v["key"]], **cfg)[0]
        d = H.gpu_defers_client(resp, v["key"], **cfg)
        if d is not None:  # a subprotocol answer against a configured list: Java's string match
            assert (g.kind, g.cause) == (H.DEFER, d), (v, g)
            continue
        e = v["expect"]
        assert (g.kind, g.status, g.cause) == (HS_KIND[e["kind"]], e["status"], _hs_cause(e["cause"])), (v, g)
        if e["detail"] is not None and e["cause"] != "INVALID_ACCEPT":
            assert g.message.endswith(": " + e["detail"]), (v, g)
        if e["cause"] == "INVALID_ACCEPT":
            assert g.message == "Invalid websocket key challenge. Actual: %s. Expected: %s" % (
                e["detail"], "s3pPLMBiTxaQ9kYGzzhZRbK+xOo="), (v, g)
    # the RFC 6455 / HandshakeUtilsTest answer key
    ok = H.response(101, "Switching Protocols", [("Upgrade", "websocket"), ("Connection", "Upgrade"),
                                                ("Sec-WebSocket-Accept", "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=")])
    g = _gpu([ok, ok + b"\x81\x02hi"], [RFC_KEY, RFC_KEY])
    assert all(x.finished and x.expected == "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=" for x in g)
    assert g[1].frame_len == len(ok)  # the rest is the session's first WebSocket bytes


def gen_response(rng: random.Random, key: str) -> bytes:
    """A server's answer to a client handshake: mostly valid, with the variants the
    reference's validation distinguishes, and forms the lane defers."""
    acc = H.answer_key(key)
    r = rng.random()
    if r < 0.7:
        line = b"HTTP/1.1 101 Switching Protocols"
    else:
        line = rng.choice([b"HTTP/1.1 400 Bad Request", b"HTTP/1.1 200 OK", b"HTTP/1.0 101 Switching Protocols",
                           b"HTTP/1.1 1O1 X", b"HTTP/1.1  101   Switching Protocols ", b"HTTP/1.1 101",
                           b"HTTP/1.1 101 ", b" HTTP/1.1 101 X", b"HTTP/1.1 0101 X", b"HTTP/1.1 426 Upgrade Required",
                           b"HTTP/1.1 101 a b c d e f", b""])
    fields = []
    u = rng.random()
    if u < 0.85:
        fields.append(("Upgrade", rng.choice(["websocket", "WebSocket", "h2c, websocket", " websocket ", "WEBSOCKET"])))
    elif u < 0.93:
        fields.append(("Upgrade", rng.choice(["xxx", "web socket", "", "websockets"])))
    c = rng.random()
    if c < 0.85:
        fields.append(("Connection", rng.choice(["Upgrade", "upgrade", "keep-alive, Upgrade", "Upgrade,close"])))
    elif c < 0.93:
        fields.append(("Connection", rng.choice(["close", "", "Upgraded", "keep-alive"])))
    a = rng.random()
    if a < 0.8:
        fields.append(("Sec-WebSocket-Accept", acc if rng.random() < 0.9 else acc + "  "))
    elif a < 0.92:
        fields.append(("Sec-WebSocket-Accept", rng.choice(["AAAA", acc.lower(), acc[:-1], H.answer_key("x" * 24),
                                                           " " + acc[1:], ""])))
    if rng.random() < 0.15:
        fields.append(("Sec-WebSocket-Protocol", rng.choice(["chat", "superchat", "", "chat, superchat"])))
    if rng.random() < 0.1:
        fields.append(("Sec-WebSocket-Extensions", rng.choice(["permessage-deflate", "", "x; y=1"])))
    for _ in range(rng.randrange(0, 4)):
        fields.append((rng.choice(["Server", "Date", "Set-Cookie", "X-Powered-By", "Via"]), "v%d" % rng.randrange(99)))
    rng.shuffle(fields)
    out = [line]
    for n, v in fields:
        n = rng.choice([n, n.upper(), n.lower()]) if rng.random() < 0.2 else n
        out.append(n.encode() + (b": " if rng.random() < 0.9 else b":\t ") + v.encode())
    x = rng.random()  # the forms the lane defers, and odd but plain lines
    if x < 0.03:
        out.insert(rng.randrange(1, len(out) + 1), b" folded continuation")
    elif x < 0.05:
        out.insert(rng.randrange(1, len(out) + 1), b"NameOnly")
    elif x < 0.07 and len(out) > 1:
        out.insert(rng.randrange(1, len(out) + 1), out[rng.randrange(1, len(out))])  # a repeat
    elif x < 0.09:
        out.insert(rng.randrange(1, len(out) + 1), b"Upgrade: web\xe9socket")
    elif x < 0.11:
        out.insert(rng.randrange(1, len(out) + 1), b"Upgrade : websocket")
    msg = b"\r\n".join(out) + b"\r\n\r\n"
    t = rng.random()
    if t < 0.1:
        msg = msg[:rng.randrange(0, len(msg))]             # not complete yet
    elif t < 0.2:
        msg += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40)))  # first frame bytes
    return msg


@pytest.mark.parametrize("seed", range(4))
def test_handshake_client_random_gpu(seed):
    from snf4j_amd.handshake import generate_key
    rng = random.Random(2000 + seed)
    cfgs = [dict(), dict(subprotocols=("chat",)), dict(extensions=True), dict(subprotocols=("chat", "x"),
                                                                                  extensions=True)]
    for cfg in cfgs:
        keys = [generate_key(rng) for _ in range(3000)]
        resps = [gen_response(rng, k) for k in keys]
        for resp, key, g in zip(resps, keys, _gpu(resps, keys, **cfg)):
            _expect_equal(resp, key, g, dict(max_length=65536, subprotocols=cfg.get("subprotocols"),
                                             extensions=cfg.get("extensions", False)))


def test_handshake_client_edges_gpu():
    ok = H.response(101, "Switching Protocols", [("Upgrade", "websocket"), ("Connection", "Upgrade"),
                                                ("Sec-WebSocket-Accept", H.answer_key(RFC_KEY))])
    cases = [(ok, {}), (ok, dict(max_length=len(ok))), (ok, dict(max_length=len(ok) - 1)),
             (ok[:20], dict(max_length=10)), (ok[:40], {}), (b"", {}), (b"\r\n", {}), (b"\r\n\r\n", {})]
    # the 50-line chunk: 49 header lines fit, 50 do not
    for n in (48, 49, 50):
        cases.append((b"HTTP/1.1 101 X\r\n" + b"".join(b"X-%d: v\r\n" % i for i in range(n)) + b"\r\n", {}))
    # every prefix of a valid response
    cases += [(ok[:i], {}) for i in range(len(ok) + 1)]
    for resp, cfg in cases:
        full = dict(max_length=cfg.get("max_length", 65536), subprotocols=None, extensions=False)
        g = _gpu([resp], [RFC_KEY], **cfg)[0]
        _expect_equal(resp, RFC_KEY, g, full)
