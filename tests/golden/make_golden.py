"""Generate the golden fixtures for the frame codec from the reference's own tests.

Every vector below transcribes one assertion of snf4j-websocket's JUnit tests
(paths relative to snf4j-websocket/src/test/java/org/snf4j/websocket/): the
input bytes are rebuilt with the same frame-description mini-language the
reference tests use (FrameDecoderTest.frame(), :117-173) and the expected
outcome is the value the reference test asserts.  The reference itself cannot
run here (pure Java, no JDK), so these assertions are what pins the oracle.

Run:  python tests/golden/make_golden.py   (writes tests/golden/*.json)
"""
from __future__ import annotations

import base64
import json
import os
import struct
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
MASK = (1, 2, 3, 4)  # FrameDecoderTest.mask, :49


def fill_bytes(c: str, n: int, masked: bool) -> bytearray:
    """FrameDecoderTest.bytes(c, len, masked), :96-113."""
    b = bytearray(n)
    for i in range(n):
        b[i] = (i & 0xFF) if c == "*" else ord(c)
        if masked:
            b[i] ^= MASK[i % 4]
    return b


def frame(text: str, off: int = 0) -> bytes:
    """FrameDecoderTest.frame(text, off), :117-173: "FRRR<op>|<len>|<M|m>|<fill>|"."""
    s = text.split("|")
    out = bytearray(b"\xff" * off)
    s0 = s[0]
    b = 0
    if s0[0] == "F":
        b |= 0x80
    if s0[1] == "R":
        b |= 0x40
    if s0[2] == "R":
        b |= 0x20
    if s0[3] == "R":
        b |= 0x10
    op = int(s0[4:])
    b |= op
    out.append(b)
    ln = int(s[1])
    m = 0x80 if s[2][0] == "M" else 0
    if ln < 126:
        out.append(ln | m)
    elif ln <= 0xFFFF:
        out.append(126 | m)
        out += struct.pack(">H", ln)
    else:
        out.append(127 | m)
        out += struct.pack(">Q", ln & 0xFFFFFFFFFFFFFFFF)
    if m:
        out += bytes(MASK)
    c = s[3][0]
    if c != "-":
        payload = fill_bytes(c, ln, bool(m))
        if op == 8 and len(payload) > 1:
            payload[0] = 3
            payload[1] = 0xE8
            if m:
                payload[0] ^= MASK[0]
                payload[1] ^= MASK[1]
        out += payload
    return bytes(out)


def frame_len(ln: int, mask: bool) -> int:
    """FrameDecoderTest.frameLen, :57-71."""
    n = 2 + (4 if mask else 0)
    if ln > 0xFFFF:
        n += 8
    elif ln > 125:
        n += 2
    return n + ln


def hx(b: bytes) -> str:
    """Byte strings: hex up to 128 bytes, else "z:" + base64(zlib) (see fixtures.unhex)."""
    b = bytes(b)
    if len(b) <= 128:
        return b.hex()
    return "z:" + base64.b64encode(zlib.compress(b, 9)).decode()


def expect_frame(op, fin, rsv, payload: bytes):
    return {"frame": {"opcode": op, "fin": fin, "rsv": rsv, "payload": hx(payload)}}


def expect_error(msg, close_code=1002):
    return {"error": msg, "close_code": close_code}


OPS = {"CONTINUATION": 0, "TEXT": 1, "BINARY": 2, "CLOSE": 8, "PING": 9, "PONG": 10}
SRC_DEC = "frame/FrameDecoderTest.java"


def builder_kats():
    """FrameDecoderTest.testFrame, :189-219 — pins the frame() restatement itself."""
    cases = [
        ("FRRR1|0|M|*|", [0xf1, 0x80, 1, 2, 3, 4]),
        ("fRRR1|0|m|*|", [0x71, 0]),
        ("frRR15|0|m|*|", [0x3f, 0]),
        ("fRrR0|0|m|*|", [0x50, 0]),
        ("fRRr15|0|m|*|", [0x6f, 0]),
        ("fRRr2|1|m|*|", [0x62, 1, 0]),
        ("fRRr2|1|M|*|", [0x62, 0x81, 1, 2, 3, 4, 0 ^ 1]),
        ("fRRr2|2|M|*|", [0x62, 0x82, 1, 2, 3, 4, 0 ^ 1, 1 ^ 2]),
        ("fRRr2|3|M|*|", [0x62, 0x83, 1, 2, 3, 4, 0 ^ 1, 1 ^ 2, 2 ^ 3]),
        ("fRRr2|4|M|*|", [0x62, 0x84, 1, 2, 3, 4, 0 ^ 1, 1 ^ 2, 2 ^ 3, 3 ^ 4]),
        ("fRRr2|5|M|*|", [0x62, 0x85, 1, 2, 3, 4, 0 ^ 1, 1 ^ 2, 2 ^ 3, 3 ^ 4, 4 ^ 1]),
        ("fRRr2|2|m|*|", [0x62, 2, 0, 1]),
        ("fRRr2|5|m|*|", [0x62, 5, 0, 1, 2, 3, 4]),
        ("fRRr2|125|m|-|", [0x62, 0x7d]),
        ("fRRr2|125|M|-|", [0x62, 0xfd, 1, 2, 3, 4]),
        ("fRRr2|126|m|-|", [0x62, 0x7e, 0, 0x7e]),
        ("fRRr2|126|M|-|", [0x62, 0xfe, 0, 0x7e, 1, 2, 3, 4]),
        ("fRRr2|65535|m|-|", [0x62, 0x7e, 0xff, 0xff]),
        ("fRRr2|65535|M|-|", [0x62, 0xfe, 0xff, 0xff, 1, 2, 3, 4]),
        ("fRRr2|65536|m|-|", [0x62, 0x7f, 0, 0, 0, 0, 0, 1, 0, 0]),
        ("fRRr2|65536|M|-|", [0x62, 0xff, 0, 0, 0, 0, 0, 1, 0, 0, 1, 2, 3, 4]),
        ("fRRr2|9223372036854775807|m|-|", [0x62, 0x7f, 0x7f, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff]),
        ("fRRr2|9223372036854775807|M|-|",
         [0x62, 0xff, 0x7f, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 1, 2, 3, 4]),
    ]
    out = []
    for t, exp in cases:
        got = frame(t)
        assert list(got) == exp, (t, list(got), exp)
        out.append({"src": SRC_DEC + ":189-219", "spec": t, "bytes": hx(got)})
    return out


def decode_kats():
    """Sequences of decode() calls on one decoder, with the asserted outcome of each."""
    V = []

    def seq(src, cm, ext, maxp, steps):
        V.append({"src": src, "client_mode": cm, "allow_extensions": ext, "max_payload": maxp,
                  "steps": steps})

    def one(src, data, expected, cm, ext=True, maxp=0x20000):
        seq(src, cm, ext, maxp, [{"data": hx(data), **expected}])

    z = b""
    # testDecodeFinRsv :397-426
    s = SRC_DEC + ":397-426"
    one(s, frame("FRRR1|0|m|-|"), expect_frame(1, True, 7, z), True)
    one(s, frame("fRRR1|0|m|-|"), expect_frame(1, False, 7, z), True)
    one(s, frame("FrRR1|0|m|-|"), expect_frame(1, True, 3, z), True)
    one(s, frame("FrrR1|0|m|-|"), expect_frame(1, True, 1, z), True)
    one(s, frame("frrr1|0|m|-|"), expect_frame(1, False, 0, z), True)
    for op in (8, 9, 10):
        one(s, frame(f"frrr{op}|0|m|-|"), expect_error("Fragmented control frame"), True)
    seq(s, True, True, 0x20000, [
        {"data": hx(frame("FRRR1|0|m|-|")), **expect_frame(1, True, 7, z)},
        {"data": hx(frame("Frrr1|0|m|-|")), **expect_frame(1, True, 0, z)}])
    seq(s, True, False, 0x20000, [
        {"data": hx(frame("Frrr1|0|m|-|")), **expect_frame(1, True, 0, z)}])
    one(s, frame("FRrr1|0|m|-|"), expect_error("Unexpected non-zero RSV bits (4)"), True, ext=False)

    # testDecodeOpcode :428-446
    s = SRC_DEC + ":428-446"
    seq(s, True, True, 0x20000, [
        {"data": hx(frame("fRrR1|0|m|-|")), **expect_frame(1, False, 5, z)},
        {"data": hx(frame("fRrR0|0|m|-|")), **expect_frame(0, False, 5, z)}])
    one(s, frame("FrrR2|0|m|-|"), expect_frame(2, True, 1, z), True)
    one(s, frame("FrrR8|0|m|-|"), expect_frame(8, True, 1, z), True)
    one(s, frame("FRrR9|0|m|-|"), expect_frame(9, True, 5, z), True)
    one(s, frame("FRRR10|0|m|-|"), expect_frame(10, True, 7, z), True)
    for i in list(range(3, 8)) + list(range(11, 16)):
        one(s, frame(f"FRRR{i}|0|m|-|"), expect_error(f"Unexpected opcode value ({i})"), True)

    # testDecodeLengthMask :448-513
    s = SRC_DEC + ":448-513"

    def star(n):
        return bytes(i & 0xFF for i in range(n))

    for n in (0, 1, 125, 126, 65535, 65536):
        fill = "-" if n == 0 else "*"
        one(s, frame(f"FRRR2|{n}|M|{fill}|"), expect_frame(2, True, 7, star(n)), False)
        one(s, frame(f"FRRR2|{n}|m|{fill}|"), expect_frame(2, True, 7, star(n)), True)
    one(s, frame("FRRR2|0|M|*|"), expect_error("Unexpected payload masking"), True)
    one(s, frame("FRRR2|0|m|*|"), expect_error("Unexpected payload masking"), False)
    one(s, frame("FRRR8|0|M|*|"), expect_frame(8, True, 7, z), False)
    one(s, frame("FRRR8|1|M|*|"), expect_error("Invalid payload length (1) in close frame"), False)
    one(s, frame("FRRR8|2|M|*|"), expect_frame(8, True, 7, bytes([3, 0xe8])), False)
    b = bytearray(star(125))
    b[0], b[1] = 3, 0xE8
    one(s, frame("FRRR8|125|M|*|"), expect_frame(8, True, 7, bytes(b)), False)
    one(s, frame("FRRR9|125|M|*|"), expect_frame(9, True, 7, star(125)), False)
    one(s, frame("FRRR10|125|M|*|"), expect_frame(10, True, 7, star(125)), False)
    for i in (8, 9, 10):
        one(s, frame(f"FRRR{i}|126|M|-|"), expect_error("Invalid payload length (126) in control frame"),
            False)
    one(s, bytes([0xf2, 126, 0, 125]), expect_error("Invalid minimal payload length"), True)
    one(s, bytes([0xf2, 127, 0, 0, 0, 0, 0, 0, 0, 125]), expect_error("Invalid minimal payload length"),
        True)
    one(s, bytes([0xf2, 127, 0, 0, 0, 0, 0, 0, 0xff, 0xff]),
        expect_error("Invalid minimal payload length"), True)
    for hi in ([0xff] * 8, [0x80] + [0xff] * 7, [0x7f] + [0xff] * 7, [0, 0, 0, 0, 0x80, 0xff, 0xff, 0xff]):
        one(s, bytes([0xf2, 127] + hi), expect_error("Invalid maximum payload length"), True)
    one(s, bytes([0xf2, 127, 0, 0, 0, 0, 0, 2, 0, 1]),
        expect_error("Maximum frame length (131072) has been exceeded"), True)
    one(s, frame("FRRR2|131072|m|*|"), expect_frame(2, True, 7, star(131072)), True)

    # testDecodeFragemntation :566-617  (decoder: FrameDecoder(true, true, 0x20000))
    s = SRC_DEC + ":566-617"

    def frag(op, fin, err=None):
        name = (("F" if fin else "f") + "RRR" + str(OPS[op]) + "|0|m|-|")
        st = {"data": hx(frame(name))}
        if err:
            st.update(expect_error(err))
        else:
            st.update(expect_frame(OPS[op], fin, 7, z))
        return st

    ctl = [frag("CLOSE", True), frag("PING", True), frag("PONG", True)]
    COUT = "Continuation frame outside fragmented message"
    NINS = "Non-continuation frame while inside fragmented massage"
    seq(s, True, True, 0x20000,
        [frag("TEXT", True), frag("BINARY", True)] + ctl + [frag("CONTINUATION", True, COUT)])
    for second in (("TEXT", True), ("BINARY", True), ("TEXT", False), ("BINARY", False)):
        seq(s, True, True, 0x20000, [frag("TEXT", False), frag(second[0], second[1], NINS)])
    seq(s, True, True, 0x20000, [frag("TEXT", False)] + ctl)
    seq(s, True, True, 0x20000,
        [frag("TEXT", False), frag("CONTINUATION", False)] + ctl + [frag("TEXT", True, NINS)])
    for second in (("BINARY", True), ("TEXT", False), ("BINARY", False)):
        seq(s, True, True, 0x20000,
            [frag("TEXT", False), frag("CONTINUATION", False), frag(second[0], second[1], NINS)])
    seq(s, True, True, 0x20000,
        [frag("TEXT", False), frag("CONTINUATION", False), frag("CONTINUATION", True),
         frag("TEXT", True), frag("BINARY", True)] + ctl)

    # testSplittedFrame :633-676 (partial frames across decode() calls)
    s = SRC_DEC + ":633-676"
    b = frame("FRRR2|100|m|*|")
    b2 = b[50:]
    b3, b4 = b2[: len(b2) // 2], b2[len(b2) // 2:]
    seq(s, True, True, 0x20000, [
        {"data": hx(b[:50]), "none": True},
        {"data": hx(b2), **expect_frame(2, True, 7, star(100))},
        {"data": hx(frame("FRRR2|1|m|*|")), **expect_frame(2, True, 7, star(1))},
        {"data": hx(b[:50]), "none": True},
        {"data": hx(b3), "none": True},
        {"data": hx(b4), **expect_frame(2, True, 7, star(100))},
        {"data": hx(frame("FRRR2|1|m|*|")), **expect_frame(2, True, 7, star(1))}])
    b = frame("FRRR2|100|M|*|")
    seq(s, False, True, 0x20000, [
        {"data": hx(b[:50]), "none": True},
        {"data": hx(b[50:]), **expect_frame(2, True, 7, star(100))},
        {"data": hx(frame("FRRR2|1|M|*|")), **expect_frame(2, True, 7, star(1))}])

    # testCloseFrame :698-740
    s = SRC_DEC + ":698-740"
    one(s, frame("FRRR8|0|m|*|"), expect_frame(8, True, 7, z), True)
    base = bytearray(frame("FRRR8|2|m|*|"))
    i = len(base) - 2
    for st0, st1, res in ((0, 0, "Invalid close frame status code (0)"),
                          (0xff, 0xff, "Invalid close frame status code (65535)"),
                          (3, 0xe7, "Invalid close frame status code (999)"),
                          (3, 0xe8, None), (3, 0xe9, None), (0x13, 0x87, None),
                          (0x13, 0x88, "Invalid close frame status code (5000)")):
        f = bytearray(base)
        f[i], f[i + 1] = st0, st1
        one(s, bytes(f), expect_error(res) if res else expect_frame(8, True, 7, bytes([st0, st1])), True)
    f = bytearray(frame("FRRR8|5|m|*|"))
    i = len(f) - 5
    f[i:i + 5] = bytes([3, 0xe8, 0xdf, 0xdf, 0xbf])
    one(s, bytes(f), expect_error("Invalid close frame reason value: bytes are not UTF-8", 1007), True)

    # testClosedDecoder :742-762
    s = SRC_DEC + ":742-762"
    f = bytearray(frame("FRRR8|2|m|*|"))
    f[-2], f[-1] = 0, 0
    seq(s, True, True, 0x20000, [
        {"data": hx(f), **expect_error("Invalid close frame status code (0)")},
        {"data": hx(f), "none": True},
        {"available": hx(bytes(f) + bytes(len(f))), "expect": 2 * len(f)}])
    return V


def available_kats():
    """FrameDecoderTest.testAvailableArray :282-367 and testSplittedFrameAvailable :678-696."""
    s = SRC_DEC + ":282-367"
    cases = []
    for off in (0, 5):
        for n in (0, 1, 125, 126, 65535, 65536):
            for m in ("M", "m"):
                data = frame(f"FRRR1|{n}|{m}|-|", off)
                cases.append({"src": s, "data_spec": f"FRRR1|{n}|{m}|-|", "off": off,
                              "expected_len": frame_len(n, m == "M"), "payload_len": n})
    big = []
    d = frame_len(0x7FFFFFFF, True) - 0x7FFFFFFF  # 14
    big.append({"src": s, "data": hx(frame(f"FRRR1|{0x7FFFFFFF - d}|M|-|")),
                "len": frame_len(0x7FFFFFFF - d, True), "expect": frame_len(0x7FFFFFFF - d, True)})
    big.append({"src": s, "data": hx(frame(f"FRRR1|{0x7FFFFFFF - d}|M|-|")),
                "len": 0x7FFFFFFF, "expect": 0x7FFFFFFF})
    big.append({"src": s, "data": hx(frame(f"FRRR1|{0x7FFFFFFF - d + 1}|M|-|")),
                "len": 0x7FFFFFFF, "error": "Extended payload length (2147483634) > 2147483633"})
    big.append({"src": s, "data": hx(frame(f"FRRR1|{0x7FFFFFFFFFFFFFFF - d}|M|-|")),
                "len": 0x7FFFFFFF,
                "error": "Extended payload length (9223372036854775793) > 2147483633"})
    f = bytearray(frame(f"FRRR1|{0x7FFFFFFFFFFFFFFF}|M|-|"))
    f[2] = 0xFF
    big.append({"src": s, "data": hx(f), "len": 0x7FFFFFFF, "error": "Negative payload length (-1)"})
    # Java long/int overflow in available(): need += plen wraps to 0 (FrameDecoder.java:392-395)
    big.append({"src": s, "data": hx(frame(f"FRRR1|{0x7FFFFFFFFFFFFFFF - d + 1}|M|-|")),
                "len": 0x7FFFFFFF, "expect": 0})

    # testSplittedFrameAvailable :678-696 (decoder in client mode, pending payload)
    s2 = SRC_DEC + ":678-696"
    b = frame("FRRR2|100|m|*|")
    sp1 = (b[: len(b) // 2], b[len(b) // 2:])
    sp2 = (sp1[0][: len(sp1[0]) // 2], sp1[0][len(sp1[0]) // 2:])
    split = {"src": s2, "first": hx(sp1[0]),
             "checks": [{"data": hx(sp1[0]), "expect_before": len(sp1[0])},
                        {"data": "00", "expect": 1},
                        {"data": hx(sp2[0]), "expect": len(sp2[0])},
                        {"data": hx(sp1[1]), "expect": len(sp1[1])},
                        {"data": hx(bytes(len(sp1[1]) + 1)), "expect": len(sp1[1])}]}
    return {"frames": cases, "big": big, "split": split}


def validator_kats():
    """FrameUtf8ValidatorTest.testDecode :81-133 — the validator stage alone."""
    s = "frame/FrameUtf8ValidatorTest.java:81-133"
    NON, OKU, INC, TAIL = "dfdf", "dfbf", "df", "bf"
    E = "Invalid text frame payload: bytes are not UTF-8"

    def f(op, fin, p, err=None):
        d = {"opcode": OPS[op], "fin": fin, "payload": p}
        if err:
            d["error"] = E
        return d

    seqs = [
        [f("CONTINUATION", True, NON), f("BINARY", True, NON), f("CLOSE", True, NON), f("PING", True, NON),
         f("PONG", True, NON), f("TEXT", True, OKU), f("CONTINUATION", True, NON)],
        [f("TEXT", True, NON, 1)],
        [f("TEXT", True, INC, 1)],
        [f("CONTINUATION", False, NON), f("BINARY", False, NON), f("TEXT", False, INC), f("BINARY", True, NON),
         f("CLOSE", True, NON), f("PING", True, NON), f("PONG", True, NON), f("CONTINUATION", True, TAIL),
         f("CONTINUATION", True, NON), f("TEXT", False, INC), f("CONTINUATION", False, TAIL),
         f("BINARY", True, NON), f("CLOSE", True, NON), f("PING", True, NON), f("PONG", True, NON),
         f("CONTINUATION", False, INC), f("CONTINUATION", False, ""), f("CONTINUATION", True, TAIL),
         f("CONTINUATION", True, NON), f("TEXT", False, INC), f("CONTINUATION", True, "", 1)],
        [f("TEXT", False, INC), f("CONTINUATION", False, ""), f("CONTINUATION", False, OKU, 1)],
    ]
    return [{"src": s, "frames": q} for q in seqs]


def encoder_kats():
    """FrameEncoderTest.testEncode :136-207: header layout strings."""
    s = "frame/FrameEncoderTest.java:136-207"

    def bytes_fill(n, c):  # FrameEncoderTest.bytes(length, fill), :128-134
        b = bytearray([ord(c)] * n)
        b[0] = ord(c) + 1
        b[-1] = ord(c) + 2
        return bytes(b)

    rows = [(0, True, 0, b""), (0, True, 0, b"A"), (0, True, 0, b"ABCDEFGH"),
            (7, True, 0, bytes_fill(125, "D")), (4, True, 0, bytes_fill(126, "E")),
            (2, True, 0, bytes_fill(127, "E")), (0, True, 0, bytes_fill(0xFFFE, "C")),
            (0, True, 0, bytes_fill(0xFFFF, "C")), (0, True, 0, bytes_fill(0x10000, "D")),
            (1, False, 0, bytes_fill(100000, "D"))]
    exp_masked = ["Frrr2M|0|M(4)=", "Frrr2M|1|M(4)=A", "Frrr2M|8|M(4)=ABCDEFGH",
                  "FRRR2M|125|M(4)=EDDDDDDDDD...DDDDDDDDDF", "FRrr2M|126|126(2)M(4)=FEEEEEEEEE...EEEEEEEEEG",
                  "FrRr2M|126|127(2)M(4)=FEEEEEEEEE...EEEEEEEEEG",
                  "Frrr2M|126|65534(2)M(4)=DCCCCCCCCC...CCCCCCCCCE",
                  "Frrr2M|126|65535(2)M(4)=DCCCCCCCCC...CCCCCCCCCE",
                  "Frrr2M|127|65536(8)M(4)=EDDDDDDDDD...DDDDDDDDDF",
                  "frrR2M|127|100000(8)M(4)=EDDDDDDDDD...DDDDDDDDDF"]
    out = []
    for cm in (True, False):
        for (rsv, fin, _, payload), em in zip(rows, exp_masked):
            e = em if cm else em.replace("M|", "m|", 1).replace("M(4)", "")
            out.append({"src": s, "client_mode": cm, "opcode": 2, "fin": fin, "rsv": rsv,
                        "payload": hx(payload), "expect": e})
    return out


def session_kats():
    """WebSocketSessionTest stream cases (a client decoding server frames: unmasked)."""
    s = "WebSocketSessionTest.java"
    out = []
    out.append({"src": s + ":568-575", "client_mode": True, "max_payload": 65536,
                "chunks": [hx(bytes([0x82, 0x0A, ord("A")])), hx(b"BCDEFGHI"), hx(b"J")],
                "frames": [{"opcode": 2, "fin": True, "rsv": 0, "payload": hx(b"ABCDEFGHIJ")}]})
    out.append({"src": s + ":595-599", "client_mode": True, "max_payload": 65536,
                "chunks": [hx(bytes([0x80, 0x00]))], "frames": [],
                "error": "Continuation frame outside fragmented message", "close_code": 1002})
    out.append({"src": s + ":605-610", "client_mode": True, "max_payload": 65536,
                "chunks": [hx(bytes([0x80, 0x7F] + [0xFF] * 8))], "frames": [],
                "error": "Negative payload length (-1)", "close_code": 1002})
    out.append({"src": s + ":627-631", "client_mode": True, "max_payload": 65536,
                "chunks": [hx(bytes([0x81, 0x02, 0xDF, 0xDF]))], "frames": [],
                "error": "Invalid text frame payload: bytes are not UTF-8", "close_code": 1007})
    out.append({"src": s + ":636-642", "client_mode": True, "max_payload": 65536,
                "chunks": [hx(bytes([0x88, 0x04, 3, 0xE8, 0xDF, 0xDF]))], "frames": [],
                "error": "Invalid close frame reason value: bytes are not UTF-8", "close_code": 1007})
    for maxp, n_ok in ((65536, 65536), (512, 512)):
        ok = bytes([0x82]) + (bytes([126]) + struct.pack(">H", n_ok) if n_ok <= 0xFFFF
                              else bytes([127]) + struct.pack(">Q", n_ok)) + bytes(n_ok)
        n_bad = n_ok + 1
        bad = bytes([0x82]) + (bytes([126]) + struct.pack(">H", n_bad) if n_bad <= 0xFFFF
                               else bytes([127]) + struct.pack(">Q", n_bad)) + bytes(n_bad)
        out.append({"src": s + ":676-708", "client_mode": True, "max_payload": maxp,
                    "chunks": [hx(ok)], "frames": [{"opcode": 2, "fin": True, "rsv": 0,
                                                    "payload": hx(bytes(n_ok))}]})
        out.append({"src": s + ":676-708", "client_mode": True, "max_payload": maxp,
                    "chunks": [hx(bad)], "frames": [],
                    "error": f"Maximum frame length ({maxp}) has been exceeded", "close_code": 1002})
    return out


def aggregator_kats():
    """FrameAggregatorTest.testMaxLength :48-89 and testDecode :91-139, and
    WebSocketSessionTest.testFrameAggregation :1334-1365, all FrameAggregator(100).
    Each input frame lists what the reference asserts comes out of decode():
    nothing, the input itself ("passthrough", the tests' `f == out.get(0)`), the
    aggregated frame, or the 1009 exception."""
    E = "Too big payload for aggregated frame"

    def f(op, fin, rsv, payload, out=None, passthrough=False, err=False):
        d = {"opcode": OPS[op], "fin": fin, "rsv": rsv, "payload": hx(payload)}
        if err:
            d["expect"] = {"error": E, "close_code": 1009}
        elif passthrough:
            d["expect"] = {"out": [{"opcode": OPS[op], "fin": fin, "rsv": rsv, "payload": hx(payload),
                                    "passthrough": True}]}
        elif out is not None:
            o_op, o_rsv, o_payload = out
            d["expect"] = {"out": [{"opcode": OPS[o_op], "fin": True, "rsv": o_rsv, "payload": hx(o_payload),
                                    "passthrough": False}]}
        else:
            d["expect"] = {"out": []}
        return d

    src = "frame/FrameAggregatorTest.java"
    max_length = [
        f("BINARY", True, 0, bytes(101), passthrough=True),                  # :55-58
        f("BINARY", False, 4, bytes(50)),                                     # :60-64
        f("CONTINUATION", True, 0, bytes(50), out=("BINARY", 4, bytes(100))),  # :65-73
        f("TEXT", False, 0, bytes(50)),                                       # :75-78
        f("CONTINUATION", True, 0, bytes(51), err=True),                      # :79-88
    ]
    decode = [
        f("TEXT", True, 0, b"ABC", passthrough=True),                         # :97-100
        f("PING", True, 0, b"", passthrough=True),                            # :102-106
        f("TEXT", False, 0, b"ABC"),                                          # :108-110
        f("CONTINUATION", False, 0, b"DEF"),                                  # :111-112
        f("PING", True, 0, b"", passthrough=True),                            # :113-115
        f("CONTINUATION", True, 0, b"GH", out=("TEXT", 0, b"ABCDEFGH")),      # :117-119
        f("BINARY", False, 0, b"ABC"),                                        # :121-123
        f("CONTINUATION", False, 0, b"DEF"),                                  # :124-125
        f("PING", True, 0, b"", passthrough=True),                            # :126-128
        f("CONTINUATION", True, 0, b"GH", out=("BINARY", 0, b"ABCDEFGH")),    # :130-132
        f("CONTINUATION", True, 0, b"GH", passthrough=True),                  # :134-138
    ]
    session = [
        f("TEXT", True, 0, b"ABC", passthrough=True),                         # :1340-1343
        f("TEXT", False, 0, b"BCD"),                                          # :1345-1347
        f("PING", True, 0, b"", passthrough=True),                            # :1348-1350
        f("CONTINUATION", False, 0, b"EFG"),                                  # :1351-1353
        f("CONTINUATION", True, 0, b"HIJ", out=("TEXT", 0, b"BCDEFGHIJ")),    # :1354-1357
        f("BINARY", False, 0, bytes(99)),                                     # :1359-1361
        f("CONTINUATION", False, 0, bytes(2), err=True),                      # :1362-1365 (CLOSE=1009)
    ]
    return [{"src": src + ":48-89", "max": 100, "frames": max_length},
            {"src": src + ":91-139", "max": 100, "frames": decode},
            {"src": "WebSocketSessionTest.java:1334-1365", "max": 100, "frames": session}]


def deflate_kats():
    """PerMessageDeflateCodecTest (extensions/compress/PerMessageDeflateCodecTest.java):
    testEncodeDecode :96-131 (frames that must come back unchanged after
    PerMessageDeflateEncoder(8, noContext) -> PerMessageDeflateDecoder(noContext); the
    rsv mask is 4 for compressed TEXT/BINARY, 0 otherwise), testDecodeUncompressed :235-260
    (frames without RSV1 pass through as the same object) and testDecompressionFailure
    :312-324 (a context-takeover stream decoded by a fresh decoder fails)."""
    src = "extensions/compress/PerMessageDeflateCodecTest.java"

    def seq_bytes(n):  # PerMessageDeflateCodecTest.bytes(len), :88-94
        return bytes(i & 0xFF for i in range(n))

    def f(op, fin, rsv, payload, mask):
        return {"opcode": OPS[op], "fin": fin, "rsv": rsv, "payload": hx(payload), "rsv_mask": mask}

    round_trip = [f("TEXT", True, 0, b"ABCDEFG", 4), f("TEXT", True, 3, b"1", 4), f("TEXT", True, 1, b"", 4),
                  f("BINARY", True, 1, seq_bytes(1024), 4), f("PING", True, 0, seq_bytes(10), 0),
                  f("PONG", True, 0, seq_bytes(10), 0),
                  f("CLOSE", True, 0, bytes([0x03, 0xE8]) + b"XXX", 0),
                  f("CONTINUATION", True, 1, seq_bytes(10), 0),
                  f("TEXT", False, 0, b"ABCDEFG", 4), f("CONTINUATION", False, 0, b"IJKLMNOP", 0),
                  f("CONTINUATION", True, 0, b"XYZ", 0)]
    uncompressed = [f("TEXT", True, 0, b"TEXT", 0), f("TEXT", False, 0, b"TEXT", 0),
                    f("CONTINUATION", False, 3, b"TEXT", 0), f("CONTINUATION", True, 0, b"TEXT", 0)]
    return [{"src": src + ":96-131", "kind": "round_trip", "level": 8, "no_context": False, "frames": round_trip},
            {"src": src + ":96-131", "kind": "round_trip", "level": 8, "no_context": True, "frames": round_trip},
            {"src": src + ":235-260", "kind": "pass_through", "no_context": False, "frames": uncompressed},
            {"src": src + ":312-324", "kind": "failure", "level": 8, "no_context": False,
             "frames": [f("BINARY", True, 0, seq_bytes(2024), 4), f("BINARY", True, 0, seq_bytes(2024), 4)],
             "error": "org.snf4j.core.codec.zip.DecompressionException: decompression failure: "
                      "invalid compressed data format"}]


def deflate_encode_kats():
    """PerMessageDeflateCodecTest's encoder cases (extensions/compress/
    PerMessageDeflateCodecTest.java): testEncodeDecode :96-131 (PerMessageDeflateEncoder(8,
    noContext) for noContext false and true), testEncodeWithoutRsv1 :151-166 (frames that
    must come back as the same object), testEncodeCompressed :262-286 (a message whose
    first frame already has RSV1: every frame of it passes through), testMinInflateBound
    :289-309 and testDecompressionFailure :312-324 (2024-byte BINARY frames, one encoder).
    The expected bytes are what zlib (java.util.zip.Deflater's engine) writes, driven the
    way ZlibEncoder drives Deflater (oracle/deflate_ref.c); out_rsv and pass_through are the
    reference's own assertions (rsv | 4 on compressed TEXT/BINARY, the same frame object
    otherwise)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle.deflateref import encode_frames
    src = "extensions/compress/PerMessageDeflateCodecTest.java"

    def seq_bytes(n):
        return bytes(i & 0xFF for i in range(n))

    def case(where, kind, level, nc, frames):
        fr = [(OPS[op], fin, rsv, payload) for op, fin, rsv, payload in frames]
        got = encode_frames(fr, level, nc)
        out = []
        for (op, fin, rsv, payload), g in zip(fr, got):
            allow = (op in (1, 2) and not rsv & 4)
            out.append({"opcode": op, "fin": fin, "rsv": rsv, "payload": hx(payload), "out": hx(g[3]),
                        "out_rsv": g[2], "pass_through": g[3] == payload and g[2] == rsv and not allow
                        and not (op == 0 and g[3] != payload)})
        return {"src": src + where, "kind": kind, "level": level, "no_context": nc, "frames": out}

    round_trip = [("TEXT", True, 0, b"ABCDEFG"), ("TEXT", True, 3, b"1"), ("TEXT", True, 1, b""),
                  ("BINARY", True, 1, seq_bytes(1024)), ("PING", True, 0, seq_bytes(10)),
                  ("PONG", True, 0, seq_bytes(10)), ("CLOSE", True, 0, bytes([0x03, 0xE8]) + b"XXX"),
                  ("CONTINUATION", True, 1, seq_bytes(10)), ("TEXT", False, 0, b"ABCDEFG"),
                  ("CONTINUATION", False, 0, b"IJKLMNOP"), ("CONTINUATION", True, 0, b"XYZ")]
    without_rsv1 = [("TEXT", True, 4, b"ABC"), ("BINARY", True, 7, seq_bytes(10)),
                    ("CONTINUATION", True, 0, seq_bytes(10)), ("PING", True, 0, seq_bytes(10)),
                    ("PONG", True, 0, seq_bytes(10)), ("CLOSE", True, 0, bytes([0x03, 0xE8]))]
    compressed = [("TEXT", True, 4, b"TEXT"), ("TEXT", False, 4, b"TEXT"), ("CONTINUATION", False, 3, b"TEXT"),
                  ("CONTINUATION", True, 0, b"TEXT")]
    return [case(":96-131", "round_trip", 8, False, round_trip),
            case(":96-131", "round_trip", 8, True, round_trip),
            case(":151-166", "pass_through", 8, False, without_rsv1),
            case(":262-286", "pass_through", 8, False, compressed),
            case(":289-309", "round_trip", 8, False, [("BINARY", True, 0, bytes(2024))]),
            case(":312-324", "round_trip", 8, False,
                 [("BINARY", True, 0, seq_bytes(2024)), ("BINARY", True, 0, seq_bytes(2024))])]


def handshake_kats():
    """Opening-handshake vectors (server side), transcribed from the reference's tests
    under snf4j-websocket/src/test/java/org/snf4j/websocket/handshake/:
    HttpUtilsTest.testAvailable :113-129 and testSplitRequestLine :211-230 ('|' = CRLF,
    HandshakeTest.bytes :36-63), HandshakeUtilsTest.testGenerateAnswerKey :153-159 and
    testParseKey :162-175, HandshakeDecoderTest.testDecode :76-107 / testDecodeTooBigFrame
    :120-138 / testDecodeFailures :141-160, and the server cases of HanshakerTest
    (request() :111-133 builds Host, Upgrade, Connection, Sec-WebSocket-Key,
    Sec-WebSocket-Version in that order; testServerHandshake :206-236, testAcceptVersion
    :245-270, testAcceptBasicFields :274-299, testAssertUri :311-356, testAcceptKey :359-382).
    A Handshaker case is the request bytes HandshakeFactory.format writes for the test's
    HandshakeRequest, with the status and closing reason the test asserts."""
    src = "snf4j-websocket/src/test/java/org/snf4j/websocket/handshake/"

    def pipe(s):
        return s.replace("|", "\r\n").encode()

    avail = [("", 0, []), ("x", 0, []), ("xx", 0, []), ("\n", 0, []), ("\r", 0, []), ("\r\n", 0, [""]),
             ("1|22|333|", 0, ["1", "22", "333"]), ("1|22|333|4444", 0, ["1", "22", "333"]),
             ("||", 4, [""]), ("||ccc", 4, [""]), ("xxx|yy||", 11, ["xxx", "yy"]),
             ("xxx|yy||6", 11, ["xxx", "yy"]), ("xxx|yy||86", 11, ["xxx", "yy"]),
             ("xxx|yy||86|", 11, ["xxx", "yy"]), ("xxx|yy|||", 11, ["xxx", "yy"])]
    split = [("", [""]), (" ", ["", ""]), ("  ", ["", ""]), ("a", ["a"]), ("ab", ["ab"]), ("a ", ["a", ""]),
             ("ab ", ["ab", ""]), (" a", ["", "a"]), (" ab", ["", "ab"]), (" a ", ["", "a", ""]),
             (" ab ", ["", "ab", ""]), ("   ab     ", ["", "ab", ""]), ("a b", ["a", "b"]), ("a  b", ["a", "b"]),
             ("ac bd", ["ac", "bd"]), ("ac  bd", ["ac", "bd"]), (" ac  bd ", ["", "ac", "bd", ""])]
    out = []
    for s, n, lines in avail:
        out.append({"src": src + "HttpUtilsTest.java:113-129", "kind": "available", "data": hx(pipe(s)),
                    "lines_len": 100, "expect": n, "lines": lines})
    for s, items in split:
        out.append({"src": src + "HttpUtilsTest.java:211-230", "kind": "split_request_line", "data": hx(s.encode()),
                    "items": items})
    out.append({"src": src + "HandshakeUtilsTest.java:153-159", "kind": "answer_key",
                "key": "dGhlIHNhbXBsZSBub25jZQ==", "accept": "s3pPLMBiTxaQ9kYGzzhZRbK+xOo="})
    b16 = bytes(range(1, 17))
    for key, ok in [(base64.b64encode(b16).decode(), True), (base64.b64encode(b16[:15]).decode(), False),
                    (base64.b64encode(b16 + b"\x11").decode(), False), ("A???", False)]:
        out.append({"src": src + "HandshakeUtilsTest.java:162-175", "kind": "parse_key", "key": key, "valid": ok})

    def case(where, req, status, kind, cause, detail=None, response=None, **cfg):
        c = {"src": src + where, "kind": "accept", "request": hx(req), "cfg": cfg,
             "expect": {"kind": kind, "status": status, "cause": cause, "detail": detail}}
        if response is not None:
            c["expect"]["response"] = hx(response)
        return c

    dec = pipe("GET /uri HTTP/1.1|Host: snf4j.org||")
    # the decoder passes these frames on: the combined outcome is Handshaker.accept's (no version field)
    out.append(case("HandshakeDecoderTest.java:76-107", dec, 400, "accept", "MISSING_VERSION"))
    out.append(case("HandshakeDecoderTest.java:120-128", dec, 400, "accept", "MISSING_VERSION", max_length=len(dec)))
    out.append(case("HandshakeDecoderTest.java:130-138", dec, 413, "parse_error", "TOO_LARGE",
                    response=b"HTTP/1.1 413 Request Entity Too Large\r\n\r\n", max_length=len(dec) - 1))
    out.append(case("HandshakeDecoderTest.java:141-151", pipe("POST /uri HTTP/1.1|Host: snf4j.org||"), 403,
                    "parse_error", "FORBIDDEN", response=b"HTTP/1.1 403 Forbidden\r\n\r\n"))
    out.append(case("HandshakeDecoderTest.java:152-160", pipe("GET /uri HTTP/1.2|Host: snf4j.org||"), 400,
                    "parse_error", "BAD_VERSION", response=b"HTTP/1.1 400 Bad Request\r\n\r\n"))
    out.append(case("HandshakeDecoderTest.java:94-97", dec[:4], 0, "need_more", "NONE"))

    def req(uri="/uri", upper=None, host="snf4j.org", upgrade=None, connection=None, key=None, version=None):
        def v(s):
            return s if upper is None else (s.upper() if upper else s.lower())
        f = []
        if host is not None:
            f.append((v("Host"), host))
        if upgrade != "no":
            f.append((v("Upgrade"), v(upgrade or "websocket")))
        if connection != "no":
            f.append((v("Connection"), v(connection or "Upgrade")))
        if key != "no":
            f.append((v("Sec-WebSocket-Key"), key or "dGhlIHNhbXBsZSBub25jZQ=="))
        if version != "no":
            f.append((v("Sec-WebSocket-Version"), version or "13"))
        b = b"GET " + uri.encode() + b" HTTP/1.1\r\n"
        for n, val in f:
            b += n.encode() + b": " + val.encode() + b"\r\n"
        return b + b"\r\n"

    ok101 = (b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
             b"Sec-WebSocket-Accept: s3pPLMBiTxaQ9kYGzzhZRbK+xOo=\r\n\r\n")
    bad = b"HTTP/1.1 400 Bad Request\r\n\r\n"
    h = "HanshakerTest.java:"
    for up in (None, True, False):
        out.append(case(h + "206-221", req(upper=up), 101, "accept", "NONE", response=ok101))
    out.append(case(h + "249-252", req(version="no"), 400, "accept", "MISSING_VERSION", response=bad))
    out.append(case(h + "253-256", req(version="ab"), 400, "accept", "INCORRECT_VERSION", "ab", response=bad))
    v426 = b"HTTP/1.1 426 Upgrade Required\r\nSec-WebSocket-Version: 13\r\n\r\n"
    out.append(case(h + "257-260", req(version="14"), 426, "accept", "UNSUPPORTED_VERSION", "14", response=v426))
    out.append(case(h + "261-263", req(version="13, 14"), 101, "accept", "NONE", response=ok101))
    out.append(case(h + "264-266", req(version="12, 13, 14"), 101, "accept", "NONE", response=ok101))
    out.append(case(h + "267-270", req(version="12, 14"), 426, "accept", "UNSUPPORTED_VERSION", "12, 14",
                    response=v426))
    out.append(case(h + "278-282", req(upgrade="no"), 400, "accept", "MISSING_UPGRADE", response=bad))
    out.append(case(h + "283-287", req(upgrade="xxx"), 400, "accept", "INVALID_UPGRADE", "xxx", response=bad))
    out.append(case(h + "289-293", req(connection="no"), 400, "accept", "MISSING_CONNECTION", response=bad))
    out.append(case(h + "294-298", req(connection="xxx"), 400, "accept", "INVALID_CONNECTION", "xxx", response=bad))
    for uri in ("/uri?find%20c", "//host/uri", "host/uri"):
        out.append(case(h + "327-329", req(uri=uri), 101, "accept", "NONE", response=ok101))
    out.append(case(h + "348-353", req(host=None), 400, "accept", "MISSING_HOST", response=bad))
    out.append(case(h + "354-355", req(uri="/find", host=None), 101, "accept", "NONE", response=ok101,
                    ignore_host=1))
    out.append(case(h + "363-367", req(key="no"), 400, "accept", "MISSING_KEY", response=bad))
    out.append(case(h + "368-372", req(key="AAAA"), 400, "accept", "INVALID_KEY", "AAAA", response=bad))
    return out


def handshake_client_kats():
    """Client-side handshake vectors: a response buffer, the key the session sent and
    the combined outcome of HandshakeDecoder(clientMode) + Handshaker.handshake(response).
    Transcribed from the reference's tests under snf4j-websocket/src/test/java/org/snf4j/
    websocket/handshake/: HandshakeFactoryTest.testParse :80-99 (the response rows, and
    the request rows parsed as responses), HandshakeDecoderTest.testDecode :113-120 and
    testDecodeFailures :173-183, and HanshakerTest's client cases (response() :135-154
    adds Upgrade, Connection, Sec-WebSocket-Accept, -Protocol, -Extensions in that order;
    testValidateStatus :482-493, testValidateBasicFields :496-536, testValidateAnswerKey
    :539-547, testValidateSubProtocol :550-589, testValidateExtensions :612-622 for the
    configs without IExtension objects).  Key: the RFC 6455 sample the tests'
    assertValidate answers with generateAnswerKey."""
    src = "snf4j-websocket/src/test/java/org/snf4j/websocket/handshake/"
    key, acc = "dGhlIHNhbXBsZSBub25jZQ==", "s3pPLMBiTxaQ9kYGzzhZRbK+xOo="

    def pipe(s):
        return s.replace("|", "\r\n").encode()

    def case(where, resp, kind, cause, status=0, detail=None, subprotocol=None, **cfg):
        return {"src": src + where, "kind": "validate", "response": hx(resp), "key": key, "cfg": cfg,
                "expect": {"kind": kind, "status": status, "cause": cause, "detail": detail,
                           "subprotocol": subprotocol}}
    out = []
    f = "HandshakeFactoryTest.java:"
    # parsed responses; the Handshaker then judges them (no Upgrade field / not 101)
    out.append(case(f + "91", pipe("HTTP/1.1 101 Switching Protocols|x: y||"), "closing", "MISSING_UPGRADE", 101))
    out.append(case(f + "92", pipe("HTTP/1.1   102   Switching Protocols |x: y||"), "closing", "INVALID_STATUS", 102,
                    "102"))
    for row, s, cause in [("80", "GET /chat HTTP/1.1|xxx: yyy||", "BAD_RESPONSE_VERSION"),
                          ("82", "GET /chat HTTP/1.1 |xxx: yyy||", "BAD_RESPONSE_VERSION"),
                          ("85", "GET /chat|xxx: yyy||", "BAD_RESPONSE_LINE"),
                          ("86", "GET /chat |xxx: yyy||", "BAD_RESPONSE_VERSION"),
                          ("87", "GET|xxx: yyy||", "BAD_RESPONSE_LINE"),
                          ("88", "GET |xxx: yyy||", "BAD_RESPONSE_LINE"),
                          ("89", "|xxx: yyy||", "BAD_RESPONSE_LINE"),
                          ("94", " HTTP/1.1 A01 Switching Protocols|x: y||", "BAD_RESPONSE_VERSION"),
                          ("95", "HTTP/1.1 A01 Switching Protocols|x: y||", "BAD_RESPONSE_STATUS"),
                          ("96", "HTTP/1.1 0A1 Switching Protocols|x: y||", "BAD_RESPONSE_STATUS"),
                          ("97", "HTTP/1.1 10A Switching Protocols|x: y||", "BAD_RESPONSE_STATUS"),
                          ("98", "HTTP/1.1 1010 Switching Protocols|x: y||", "BAD_RESPONSE_STATUS"),
                          ("99", "HTTP/1.0 10A Switching Protocols|x: y||", "BAD_RESPONSE_VERSION")]:
        out.append(case(f + row, pipe(s), "parse_error", cause))
    d = "HandshakeDecoderTest.java:"
    out.append(case(d + "113-120", pipe("HTTP/1.1 400 Bad Request||"), "closing", "INVALID_STATUS", 400, "400"))
    out.append(case(d + "173-182", pipe("HTTP/1.3 400 Bad Request||"), "parse_error", "BAD_RESPONSE_VERSION"))

    def resp(status=101, upper=None, upgrade=None, connection=None, accept=None, protocols=None, extensions=None):
        def v(x):
            return x if upper is None else (x.upper() if upper else x.lower())
        fl = []
        if upgrade != "no":
            fl.append((v("Upgrade"), v(upgrade or "websocket")))
        if connection != "no":
            fl.append((v("Connection"), v(connection or "Upgrade")))
        if accept != "no":
            fl.append((v("Sec-WebSocket-Accept"), accept or acc))
        if protocols is not None:
            fl.append((v("Sec-WebSocket-Protocol"), protocols))
        if extensions is not None:
            fl.append((v("Sec-WebSocket-Extensions"), extensions))
        b = b"HTTP/1.1 %03d X\r\n" % status       # HandshakeFactory.format (:141-157), reason "X"
        for n, val in fl:
            b += n.encode() + b": " + val.encode() + b"\r\n"
        return b + b"\r\n"
    h = "HanshakerTest.java:"
    out.append(case(h + "482-493", resp(100), "closing", "INVALID_STATUS", 100, "100"))
    for up in (None, True):
        out.append(case(h + "497-500", resp(upper=up), "finished", "NONE", 101))
    for u in ("websocket", "Websocket", "Websocket,xxx", "yyy, Websocket ", "yyy, websocket , xxx"):
        out.append(case(h + "501-516", resp(upgrade=u), "finished", "NONE", 101))
    out.append(case(h + "518-520", resp(upgrade="no"), "closing", "MISSING_UPGRADE", 101))
    out.append(case(h + "521-523", resp(upgrade="xxx"), "closing", "INVALID_UPGRADE", 101, "xxx"))
    out.append(case(h + "527-529", resp(connection="no"), "closing", "MISSING_CONNECTION", 101))
    out.append(case(h + "530-532", resp(connection="xxx"), "closing", "INVALID_CONNECTION", 101, "xxx"))
    out.append(case(h + "533-535", resp(connection="xxx,yyy, zzz"), "closing", "INVALID_CONNECTION", 101,
                    "xxx,yyy, zzz"))
    out.append(case(h + "540", resp(), "finished", "NONE", 101))
    out.append(case(h + "541-542", resp(accept="no"), "closing", "MISSING_ACCEPT", 101))
    out.append(case(h + "543-546", resp(accept="AAAA"), "closing", "INVALID_ACCEPT", 101, "AAAA"))
    out.append(case(h + "553", resp(), "finished", "NONE", 101))
    out.append(case(h + "554-556", resp(), "finished", "NONE", 101, subprotocols=[]))
    out.append(case(h + "557-559", resp(protocols="proto1"), "closing", "INVALID_SUBPROTOCOL", 101, "proto1",
                    subprotocols=[]))
    p1, p12 = ["proto1"], ["proto1", "proto2"]
    out.append(case(h + "563-564", resp(), "closing", "MISSING_SUBPROTOCOL", 101, subprotocols=p1))
    out.append(case(h + "565-567", resp(protocols="proto1"), "finished", "NONE", 101, None, "proto1", subprotocols=p1))
    out.append(case(h + "568-570", resp(protocols="proto2"), "closing", "INVALID_SUBPROTOCOL", 101, "proto2",
                    subprotocols=p1))
    out.append(case(h + "574-575", resp(), "closing", "MISSING_SUBPROTOCOL", 101, subprotocols=p12))
    out.append(case(h + "576-578", resp(protocols="proto3"), "closing", "INVALID_SUBPROTOCOL", 101, "proto3",
                    subprotocols=p12))
    out.append(case(h + "579-581", resp(protocols="proto1, proto2"), "closing", "INVALID_SUBPROTOCOL", 101,
                    "proto1, proto2", subprotocols=p12))
    out.append(case(h + "582-584", resp(protocols="proto2"), "finished", "NONE", 101, None, "proto2",
                    subprotocols=p12))
    out.append(case(h + "585-587", resp(protocols=""), "closing", "INVALID_SUBPROTOCOL", 101, "", subprotocols=p12))
    out.append(case(h + "616", resp(), "finished", "NONE", 101))
    out.append(case(h + "617-619", resp(), "finished", "NONE", 101, extensions=False))
    out.append(case(h + "620-622", resp(extensions="ext1; param1"), "closing", "INVALID_EXTENSIONS", 101))
    return out


def main():
    data = {
        "handshake_client": handshake_client_kats(),
        "handshake": handshake_kats(),
        "deflate": deflate_kats(),
        "deflate_encode": deflate_encode_kats(),
        "aggregator": aggregator_kats(),
        "builder": builder_kats(),
        "decode": decode_kats(),
        "available": available_kats(),
        "validator": validator_kats(),
        "encoder": encoder_kats(),
        "session": session_kats(),
    }
    for name, obj in data.items():
        with open(os.path.join(HERE, f"{name}_kat.json"), "w") as fh:
            json.dump(obj, fh, indent=0, separators=(",", ":"))
    sizes = {k: os.path.getsize(os.path.join(HERE, f"{k}_kat.json")) for k in data}
    print(sizes)


if __name__ == "__main__":
    main()
