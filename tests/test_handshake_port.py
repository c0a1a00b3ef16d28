"""The compiled handshake port (oracle/handshake_port.c, bench.py's cpu_baseline of kind
"port") against the Python restatement it follows (oracle/handshake_oracle.py, pinned by
the reference's test vectors in tests/test_oracle_golden.py): the same kind, HTTP status
and response bytes wherever the port takes the request (it leaves folded / repeated
header lines and java.net.URI's cases to the restatement)."""
import base64
import random

import numpy as np

from oracle import handshake_oracle as H
from oracle import handshake_port as P
from tests import hsgen
from tests.golden import fixtures

KIND = {H.NEED_MORE: P.NEED_MORE, H.PARSE_ERROR: P.PARSE_ERROR, H.ACCEPT: P.ACCEPT}


def _same(req):
    k, st, resp = P.accept(req)
    if k == P.UNSUPPORTED:
        return False
    e = H.accept(req)
    assert e["kind"] is not None, req
    assert k == KIND[e["kind"]], (req, k, e)
    if k != P.NEED_MORE:
        assert st == e["status"] and resp == e["response"], (req, st, resp, e)
    return True


def test_rfc_answer_key():
    req = H.request("/uri", [("Host", "snf4j.org"), ("Upgrade", "websocket"), ("Connection", "Upgrade"),
                             ("Sec-WebSocket-Key", "dGhlIHNhbXBsZSBub25jZQ=="), ("Sec-WebSocket-Version", "13")])
    k, st, resp = P.accept(req)
    assert k == P.ACCEPT and st == 101 and b"Sec-WebSocket-Accept: s3pPLMBiTxaQ9kYGzzhZRbK+xOo=\r\n" in resp


def test_port_equals_restatement_on_the_vectors():
    n = 0
    for v in fixtures.load("handshake"):
        if v["kind"] != "accept" or v["cfg"].get("max_length", 65536) != 65536 or v["cfg"].get("ignore_host"):
            continue
        n += _same(fixtures.unhex(v["request"]))
    assert n >= 10


def test_port_equals_restatement_on_random_requests():
    rng = random.Random(77)
    taken = sum(_same(hsgen.request(rng)) for _ in range(3000))
    assert taken > 1000


def test_client_validate():
    rng = np.random.default_rng(5)
    for i in range(200):
        key = base64.b64encode(rng.integers(0, 256, 16, dtype=np.uint8).tobytes()).decode()
        acc = H.answer_key(key) if i % 5 else H.answer_key(key[::-1])
        fields = [("Upgrade", "websocket"), ("Connection", "Upgrade"), ("Sec-WebSocket-Accept", acc)]
        if i % 7 == 3:
            fields = fields[1:]
        resp = H.response(101 if i % 11 else 200, "X", fields)
        want = H.validate(resp, key)["kind"]
        assert P.validate(resp, key) == {H.FINISHED: P.FINISHED, H.CLOSING: P.CLOSING}[want], (i, resp)


def test_rate_runs_on_threads():
    reqs = [H.request("/chat", [("Host", "a.example"), ("Upgrade", "websocket"), ("Connection", "Upgrade"),
                                ("Sec-WebSocket-Key", base64.b64encode(bytes([i]) * 16).decode()),
                                ("Sec-WebSocket-Version", "13")]) for i in range(64)]
    buf = np.frombuffer(b"".join(reqs), np.uint8)
    off = np.concatenate([[0], np.cumsum([len(r) for r in reqs])]).astype(np.uint64)
    r1, d1 = P.rate(buf, off, None, 1, 0.05)
    r2, d2 = P.rate(buf, off, None, 2, 0.05)
    assert r1 > 1e4 and r2 > 1e4 and d1 > 0 and d2 > 0
