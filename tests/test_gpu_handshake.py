"""Server opening handshake on the GPU (k_hs_accept through the C ABI) against the
CPU restatement (oracle/handshake_oracle.py), which tests/test_oracle_golden.py pins
to the reference's handshake tests."""
import random

import numpy as np
import pytest

from oracle import handshake_oracle as H
from tests import hsgen
from tests.golden import fixtures
from tests.test_oracle_golden import HS_KIND, _hs_cause, hs_cfg


def test_available_matches_oracle():
    """wsg_handshake_available (host framing, like wsg_frame_available) vs HttpUtils.available."""
    from snf4j_amd import handshake
    for v in fixtures.load("handshake"):
        if v["kind"] == "available":
            data = fixtures.unhex(v["data"])
            assert handshake.available(data) == H.available(data)[0] == v["expect"]
    rng = random.Random(7)
    for _ in range(3000):
        r = hsgen.request(rng)
        assert handshake.available(r) == H.available(r)[0], r
    # the 50-line chunk: 49 header lines fit, 50 do not (HandshakeDecoder.java:50,224-231)
    for n in (48, 49, 50):
        r = b"GET / HTTP/1.1\r\n" + b"".join(b"X-%d: v\r\n" % i for i in range(n)) + b"\r\n"
        assert handshake.available(r) == H.available(r)[0] == (len(r) if n <= 49 else 0)


def _gpu(requests, **cfg):
    from snf4j_amd import BatchHandshaker, HandshakeConfig
    c = HandshakeConfig(cfg.get("max_length", 65536), cfg.get("ignore_host", False), cfg.get("subprotocols", False),
                        cfg.get("extensions", False), cfg.get("host_policy", False))
    return BatchHandshaker(c).accept(requests)


def _expect_equal(req, g, cfg):
    d = H.gpu_defers(req, **cfg)
    if d is not None:
        assert (g.kind, g.cause) == (H.DEFER, d), (req, g)
        return
    r = H.accept(req, **cfg)
    assert r["kind"] is not None, (req, g)
    assert g.kind == r["kind"] and g.status == r["status"] and g.cause == r["cause"], (req, g, r)
    assert g.response == r["response"], (req, g, r)
    if r["kind"] != H.NEED_MORE:
        exp_msg = H.MESSAGES.get(r["cause"])
        if exp_msg and "%s" in exp_msg:
            exp_msg = exp_msg % r["detail"]
        assert g.message == exp_msg, (req, g, r)
    if r["frame_len"]:
        assert g.frame_len == r["frame_len"]


@pytest.mark.gpu
def test_handshake_kat_gpu():
    vs = [v for v in fixtures.load("handshake") if v["kind"] == "accept"]
    for v in vs:
        req = fixtures.unhex(v["request"])
        g = _gpu([req], **hs_cfg(v["cfg"]))[0]
        e = v["expect"]
        assert (g.kind, g.status, g.cause) == (HS_KIND[e["kind"]], e["status"], _hs_cause(e["cause"])), (v, g)
        if "response" in e:
            assert g.response == fixtures.unhex(e["response"]), (v, g)
        if e["detail"] is not None:
            assert g.message.endswith(": " + e["detail"]), (v, g)
    # the RFC 6455 / HandshakeUtilsTest answer key through the whole path
    g = _gpu([H.request("/uri", [("Host", "snf4j.org"), ("Upgrade", "websocket"), ("Connection", "Upgrade"),
                                 ("Sec-WebSocket-Key", "dGhlIHNhbXBsZSBub25jZQ=="),
                                 ("Sec-WebSocket-Version", "13")])])[0]
    assert g.switched and b"Sec-WebSocket-Accept: s3pPLMBiTxaQ9kYGzzhZRbK+xOo=\r\n" in g.response


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_handshake_random_gpu(seed):
    rng = random.Random(1000 + seed)
    cfgs = [dict(), dict(ignore_host=True), dict(subprotocols=True, extensions=True), dict(host_policy=True),
            dict(max_length=180)]
    cfg = cfgs[seed % len(cfgs)]
    reqs = [hsgen.request(rng) for _ in range(4000)]
    outs = _gpu(reqs, **cfg)
    kinds = {}
    for req, g in zip(reqs, outs):
        _expect_equal(req, g, cfg)
        kinds[g.kind] = kinds.get(g.kind, 0) + 1
    assert kinds.get(H.ACCEPT, 0) > 100   # the random mix exercises the decided path
    if seed == 0:
        assert sum(1 for g in outs if g.switched) > 300


@pytest.mark.gpu
def test_handshake_edges_gpu():
    base = H.request("/uri", [("Host", "snf4j.org"), ("Upgrade", "websocket"), ("Connection", "Upgrade"),
                              ("Sec-WebSocket-Key", "dGhlIHNhbXBsZSBub25jZQ=="), ("Sec-WebSocket-Version", "13")])
    reqs = [b"", b"G", base[:20], base[:-1], base, base + b"\x81\x80abcd",
            b"GET / HTTP/1.1\r\n" + b"".join(b"X-%d: v\r\n" % i for i in range(60)) + b"\r\n",
            b"\r\n\r\n", b"GET  / HTTP/1.1\r\n\r\n", b" GET / HTTP/1.1\r\n\r\n", b"GET / HTTP/1.1 \r\n\r\n",
            b"GET / HTTP/1.1\r\nHost: a\r\n", b"XXXX / HTTP/1.1\r\n", b"GET / HTTP/1.1\r\n\n\r\n",
            b"GET / HTTP/1.1\r\r\n\r\n", base.replace(b"13\r\n", b"13\r\n\tx\r\n"),
            base.replace(b"Host", b"\xe9Host"), base.replace(b"snf4j.org", b"sn\xe9f")]
    for cfg in (dict(), dict(max_length=100), dict(max_length=10)):
        outs = _gpu(reqs, **cfg)
        for req, g in zip(reqs, outs):
            _expect_equal(req, g, cfg)
