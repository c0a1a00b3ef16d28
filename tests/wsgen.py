"""Random WebSocket frame streams for parity tests (test infrastructure).

Builds per-session frame sequences — text (multi-byte UTF-8, code points split
across fragments), binary, control frames interleaved between fragments — and
optionally injects exactly the protocol violations the reference checks
(FrameDecoder.java:197-256, :121-136; FrameUtf8Validator.java:65-70).
"""
from __future__ import annotations

import struct

import numpy as np

TEXT_SAMPLES = ["hello", "é", "ß", "€", "中文", "한국어", "😀", "𐍈", "ऄ", "ﬀ", "a" * 7, "Ж", "߿", "ࠀ",
                "퟿", "", "￿", "\U00010000", "\U0010ffff"]
BAD_UTF8 = [b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf0\x80\x80\x80", b"\xf4\x90\x80\x80",
            b"\xf5\x80", b"\xff", b"\x80", b"\xbf", b"\xe2\x82", b"\xc3", b"\xe2\x28\xa1", b"\xf0\x9f\x98"]


def build_frame(opcode, fin, rsv, payload, masked, mask=(0, 0, 0, 0), len_form=None, len_value=None) -> bytes:
    """Wire bytes of one frame; len_form forces 7/16/64-bit length encoding."""
    payload = bytes(payload)
    n = len(payload) if len_value is None else len_value
    b0 = (0x80 if fin else 0) | ((rsv & 7) << 4) | (opcode & 0x0F)
    mb = 0x80 if masked else 0
    form = len_form or (7 if n <= 125 else 16 if n <= 0xFFFF else 64)
    if form == 7:
        hdr = bytes([b0, mb | n])
    elif form == 16:
        hdr = bytes([b0, mb | 126]) + struct.pack(">H", n)
    else:
        hdr = bytes([b0, mb | 127]) + struct.pack(">Q", n & 0xFFFFFFFFFFFFFFFF)
    if masked:
        m = bytes(mask)
        hdr += m
        payload = bytes(b ^ m[i & 3] for i, b in enumerate(payload)) if payload else payload
    return hdr + payload


def rand_text(rng, n_chars) -> bytes:
    parts = []
    for _ in range(n_chars):
        r = rng.random()
        if r < 0.6:
            parts.append(chr(int(rng.integers(0x20, 0x7F))))
        else:
            parts.append(TEXT_SAMPLES[int(rng.integers(0, len(TEXT_SAMPLES)))])
    return "".join(parts).encode("utf-8")


def split_points(rng, n, k):
    if k <= 1 or n == 0:
        return [0, n]
    pts = sorted(set(int(x) for x in rng.integers(0, n + 1, size=k - 1)))
    return [0] + pts + [n]


def session_frames(rng, n_msgs, client_mode=False, allow_ext=False, max_payload=65536, inject=None,
                   big=False):
    """Frames (wire bytes) of one session's stream, as a client (masked) sends them
    to a server decoder (client_mode=False), or unmasked for a client decoder."""
    masked = not client_mode
    frames = []

    def mk(opcode, fin, payload, rsv=0):
        m = tuple(int(x) for x in rng.integers(0, 256, 4))
        frames.append(build_frame(opcode, fin, rsv, payload, masked, m))

    for _ in range(n_msgs):
        kind = rng.random()
        if kind < 0.45:
            body = rand_text(rng, int(rng.integers(0, 400 if not big else 3000)))
            op = 1
        elif kind < 0.85:
            body = rng.integers(0, 256, int(rng.integers(0, 600 if not big else 20000)), dtype=np.uint8).tobytes()
            op = 2
        else:
            c = rng.random()
            if c < 0.4:
                mk(9, True, rng.integers(0, 256, int(rng.integers(0, 126)), dtype=np.uint8).tobytes())
            elif c < 0.8:
                mk(10, True, rng.integers(0, 256, int(rng.integers(0, 126)), dtype=np.uint8).tobytes())
            else:
                reason = rand_text(rng, int(rng.integers(0, 20)))[:100]
                mk(8, True, struct.pack(">H", int(rng.integers(1000, 5000))) + reason)
            continue
        nfrag = 1 if rng.random() < 0.7 else int(rng.integers(2, 6))
        pts = split_points(rng, len(body), nfrag)
        for i in range(len(pts) - 1):
            fin = i == len(pts) - 2
            mk(op if i == 0 else 0, fin, body[pts[i]:pts[i + 1]], rsv=(int(rng.integers(0, 8)) if allow_ext else 0))
            if not fin and rng.random() < 0.3:  # control frame between fragments
                mk(9, True, b"p")
    if inject is not None and frames:
        pos = int(rng.integers(0, len(frames) + 1))
        frames.insert(pos, bad_frame(rng, inject, masked, max_payload))
    return frames


INJECT_KINDS = ["opcode", "rsv", "masking", "frag_control", "control_len", "close_len", "cont_outside",
                "min_len16", "min_len64", "max_payload", "too_long", "close_status", "close_reason", "utf8",
                "utf8_fin_incomplete"]


def bad_frame(rng, kind, masked, max_payload) -> bytes:
    m = tuple(int(x) for x in rng.integers(0, 256, 4))
    if kind == "opcode":
        return build_frame(int(rng.choice([3, 4, 5, 6, 7, 11, 12, 13, 14, 15])), True, 0, b"xy", masked, m)
    if kind == "rsv":
        return build_frame(2, True, int(rng.integers(1, 8)), b"xy", masked, m)
    if kind == "masking":
        return build_frame(2, True, 0, b"xy", not masked, m)
    if kind == "frag_control":
        return build_frame(int(rng.choice([8, 9, 10])), False, 0, b"", masked, m)
    if kind == "control_len":
        return build_frame(int(rng.choice([9, 10])), True, 0, bytes(126), masked, m)
    if kind == "close_len":
        return build_frame(8, True, 0, b"\x03", masked, m)
    if kind == "cont_outside":
        return build_frame(0, True, 0, b"abc", masked, m)
    if kind == "min_len16":
        return build_frame(2, True, 0, bytes(100), masked, m, len_form=16)
    if kind == "min_len64":
        return build_frame(2, True, 0, bytes(1000), masked, m, len_form=64)
    if kind == "max_payload":  # u64 length > Integer.MAX_VALUE: decode() rule (the host never frames it)
        return build_frame(2, True, 0, b"", masked, m, len_form=64, len_value=0x80000000)[:14 if masked else 10]
    if kind == "too_long":
        return build_frame(2, True, 0, bytes(max_payload + 1), masked, m)
    if kind == "close_status":
        return build_frame(8, True, 0, struct.pack(">H", int(rng.choice([0, 999, 5000, 65535]))), masked, m)
    if kind == "close_reason":
        return build_frame(8, True, 0, b"\x03\xe8" + BAD_UTF8[int(rng.integers(0, len(BAD_UTF8)))], masked, m)
    if kind == "utf8":
        bad = BAD_UTF8[int(rng.integers(0, len(BAD_UTF8)))]
        body = rand_text(rng, 5) + bad + rand_text(rng, 5)
        return build_frame(1, True, 0, body, masked, m)
    if kind == "utf8_fin_incomplete":
        return build_frame(1, True, 0, rand_text(rng, 3) + b"\xe2\x82", masked, m)
    raise ValueError(kind)


def make_batch(sessions_frames):
    """Concatenate per-session frame lists into (wire, frame_off, session_first)."""
    chunks, off, first = [], [0], [0]
    for fr in sessions_frames:
        for f in fr:
            chunks.append(f)
            off.append(off[-1] + len(f))
        first.append(len(off) - 1)
    wire = np.frombuffer(b"".join(chunks), dtype=np.uint8).copy() if chunks else np.zeros(0, np.uint8)
    return wire, np.array(off, dtype=np.uint64), np.array(first, dtype=np.uint32)


def pm_deflate_encode(frames, level=8, no_context=False):
    """PerMessageDeflateEncoder(level, noContext) restated for test inputs
    (PerMessageDeflateEncoder.java:55-98, DeflateEncoder.java:60-106): TEXT/BINARY frames
    without RSV1 and the continuations of such a message are deflated (raw, sync flush;
    the tail 00 00 FF FF removed from a final fragment; an empty payload becomes 00) and
    TEXT/BINARY get RSV1.  Input/output: (opcode, fin, rsv, payload) tuples."""
    import zlib
    out = []
    comp = None
    compressing = False
    for op, fin, rsv, p in frames:
        allow = (op in (1, 2) and not (rsv & 4)) or (op == 0 and compressing)
        if allow:
            if comp is None:
                comp = zlib.compressobj(level, zlib.DEFLATED, -15)
            b = (comp.compress(p) + comp.flush(zlib.Z_SYNC_FLUSH)) if p else b""
            if fin and no_context:
                comp = None
            if not b:
                b = b"\x00"
            elif fin:
                b = b[:-4]
            out.append((op, fin, rsv | 4 if op in (1, 2) else rsv, b))
        else:
            out.append((op, fin, rsv, p))
        if op < 8:
            if fin:
                compressing = False
            elif not (rsv & 4) and op in (1, 2):
                compressing = True
    return out
