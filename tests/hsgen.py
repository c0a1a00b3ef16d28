"""Random server handshake requests for the parity tests: valid requests from the
reference's test builder (HanshakerTest.request, :111-133) mutated toward every rule
of HttpUtils / HandshakeFactory / Handshaker the GPU path decides or defers."""
from __future__ import annotations

import base64
import random

NAMES = ["Host", "Upgrade", "Connection", "Sec-WebSocket-Key", "Sec-WebSocket-Version"]


def _case(rng, s):
    r = rng.random()
    return s if r < 0.6 else (s.upper() if r < 0.8 else s.lower())


def request(rng: random.Random) -> bytes:
    key = base64.b64encode(bytes(rng.randrange(256) for _ in range(16))).decode()
    if rng.random() < 0.08:
        key = rng.choice([key[:22], key[:23], key[:-1], "AAAA", "", key + "==", key[:21] + "?" + key[22:],
                          key.replace("=", "A"), " " + key])
    uri = rng.choice(["/uri", "/chat?room=1&x=%20a", "//host/uri", "host/uri", "/", "?q", "/a;b,c$d+e=f~g'h(i)*!"])
    if rng.random() < 0.05:
        uri = rng.choice(["/u%2", "/a:b", "http://host/x", "/é", "/a[b]", "/a\tb", "/a#frag", "/%zz"])
    version = "13"
    if rng.random() < 0.1:
        version = rng.choice(["14", "13, 14", "12, 13", "ab", "", " 13 ", "+13", "-13", "013", "8, ab, 13",
                              "99999999999", "13,", ",13", "1 3"])
    fields = [("Host", rng.choice(["snf4j.org", "snf4j.org:8080", "127.0.0.1", "", "a_b.org", "h@st"])),
              ("Upgrade", rng.choice(["websocket"] * 6 + ["WebSocket", "h2c, websocket", "xxx", " websocket "])),
              ("Connection", rng.choice(["Upgrade"] * 6 + ["keep-alive, Upgrade", "upgrade", "close", "Up grade"])),
              ("Sec-WebSocket-Key", key), ("Sec-WebSocket-Version", version)]
    if rng.random() < 0.2:
        fields.append(("Sec-WebSocket-Protocol", rng.choice(["chat", "", "a, b"])))
    if rng.random() < 0.2:
        fields.append(("Sec-WebSocket-Extensions", rng.choice(["permessage-deflate", "", "x; y=1"])))
    if rng.random() < 0.3:
        fields.append(("User-Agent", "Mozilla/5.0 (X11) \xe9t\xe9"))
    rng.shuffle(fields)
    if rng.random() < 0.1:
        fields = [f for f in fields if f[0] != rng.choice(NAMES)]
    if rng.random() < 0.05:
        fields.append(rng.choice(fields))
    lines = [rng.choice(["GET"] * 12 + ["POST", "get"]) + " " + uri + " " +
             rng.choice(["HTTP/1.1"] * 12 + ["HTTP/1.0", "HTTP/1.1 x"])]
    for n, v in fields:
        sep = rng.choice([": "] * 8 + [":", ":\t", " : "])
        trail = rng.choice([""] * 8 + [" ", "\t "])
        lines.append(_case(rng, n) + sep + v + trail)
    if rng.random() < 0.05:
        i = rng.randrange(1, len(lines) + 1)
        lines.insert(i, rng.choice([" folded", "\tfolded: x", "NoColon", ""]))
    raw = ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")
    if rng.random() < 0.05:
        raw = raw.replace(b"\r\n", b"\n", 1)
    tail = b""
    if rng.random() < 0.2:
        tail = bytes([0x81, 0x85]) + bytes(rng.randrange(256) for _ in range(9))  # first frame bytes
    raw += tail
    if rng.random() < 0.08:
        raw = raw[:rng.randrange(len(raw))]
    return raw
