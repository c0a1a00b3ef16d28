"""Host planner of synthetic mixed batches (BASELINE.json configs[2]; SURVEY.md §8d
"Config 3"): the host decides message sizes, text/binary, fragmentation, session
placement and injected invalid UTF-8; wsb_synth_frames (libwsbench.so) writes the
bytes on the device.  Bench and test infrastructure only — the decode path never
calls it.
"""
from __future__ import annotations

import numpy as np

# wsb_synth_frame (include/wsbench.h)
SYNTH_DTYPE = np.dtype([("wire_off", "<u8"), ("msg_seed", "<u8"), ("payload_len", "<u4"), ("msg_pos", "<u4"),
                        ("msg_len", "<u4"), ("mask", "<u4"), ("inject_pos", "<i4"), ("opcode", "u1"),
                        ("flags", "u1"), ("text", "u1"), ("inject_kind", "u1")])
assert SYNTH_DTYPE.itemsize == 40


def header_len(payload_len, masked: bool):
    """FrameEncoder.length() header part (FrameEncoder.java:122-135), vectorised."""
    pl = np.asarray(payload_len, dtype=np.int64)
    return 2 + np.where(pl > 0xFFFF, 8, np.where(pl > 125, 2, 0)) + (4 if masked else 0)


def mixed_plan(seed: int, n_sessions: int, target_wire_bytes: int, min_len: int = 64, max_len: int = 65536,
               text_frac: float = 0.5, frag_frac: float = 0.1, bad_frac: float = 0.01, max_frags: int = 4,
               masked: bool = True):
    """Messages with log-uniform sizes in [min_len, max_len], `text_frac` TEXT (valid
    UTF-8, ~70 % ASCII bytes) else BINARY; `frag_frac` of them fragmented into 2..max_frags
    frames cut at arbitrary bytes (code points split across fragments); `bad_frac` of the
    text messages carry one injected invalid sequence.  Sessions own contiguous frames.
    The wire holds at least target_wire_bytes.

    Returns (table[SYNTH_DTYPE], frame_off u64[n+1], session_first u32[n_sessions+1], wire_len,
    info dict)."""
    rng = np.random.default_rng(seed)
    lo, hi = np.log(min_len), np.log(max_len + 1)
    mean = (max_len - min_len) / (hi - lo)
    n_msgs = max(n_sessions, int(1.25 * target_wire_bytes / (mean + 10)) + 16)
    L = np.exp(rng.uniform(lo, hi, n_msgs)).astype(np.int64).clip(min_len, max_len)
    # a message's wire bytes are >= its payload + the smallest header (2 B, + 4 B mask),
    # so cutting where these lower bounds reach the target gives wire_len >= target
    approx = np.cumsum(L + (6 if masked else 2))
    n_msgs = max(min(n_msgs, int(np.searchsorted(approx, target_wire_bytes)) + 1), 1)
    L = L[:n_msgs]
    is_text = rng.random(n_msgs) < text_frac
    nfrag = np.where(rng.random(n_msgs) < frag_frac, rng.integers(2, max_frags + 1, n_msgs), 1)
    nfrag = np.minimum(nfrag, L)  # every fragment >= 1 byte
    bad = is_text & (rng.random(n_msgs) < bad_frac)
    inject_pos = np.where(bad, (rng.random(n_msgs) * np.maximum(L - 1, 1)).astype(np.int64), -1)
    inject_kind = rng.integers(0, 5, n_msgs)
    msg_seed = rng.integers(0, 2**63, n_msgs, dtype=np.int64).astype(np.uint64)
    sess = rng.integers(0, n_sessions, n_msgs)
    order = np.argsort(sess, kind="stable")  # a session's messages stay in generation order

    # fragments, in session order
    m_of_f = np.repeat(order, nfrag[order])
    n_frames = len(m_of_f)
    pos = np.zeros(n_frames, dtype=np.int64)
    plen = L[m_of_f].copy()
    first = np.ones(n_frames, dtype=bool)
    fin = np.ones(n_frames, dtype=bool)
    starts = np.concatenate([[0], np.cumsum(nfrag[order])[:-1]])
    for i in np.nonzero(nfrag[order] > 1)[0]:
        m = order[i]
        k = int(nfrag[m])
        while True:
            cuts = np.unique(rng.integers(1, int(L[m]), k - 1))
            if len(cuts) == k - 1:
                break
        edges = np.concatenate([[0], cuts, [int(L[m])]])
        f0 = int(starts[i])
        pos[f0:f0 + k] = edges[:-1]
        plen[f0:f0 + k] = np.diff(edges)
        first[f0 + 1:f0 + k] = False
        fin[f0:f0 + k - 1] = False

    t = np.zeros(n_frames, dtype=SYNTH_DTYPE)
    flen = header_len(plen, masked) + plen
    off = np.zeros(n_frames + 1, dtype=np.uint64)
    off[1:] = np.cumsum(flen)
    t["wire_off"] = off[:-1]
    t["msg_seed"] = msg_seed[m_of_f]
    t["payload_len"] = plen
    t["msg_pos"] = pos
    t["msg_len"] = L[m_of_f]
    t["mask"] = rng.integers(0, 2**32, n_frames, dtype=np.int64).astype(np.uint32)
    t["inject_pos"] = inject_pos[m_of_f]
    t["opcode"] = np.where(first, np.where(is_text[m_of_f], 1, 2), 0)
    t["flags"] = np.where(fin, 0x80, 0) | (1 if masked else 0)
    t["text"] = is_text[m_of_f]
    t["inject_kind"] = inject_kind[m_of_f]
    counts = np.bincount(sess, weights=nfrag, minlength=n_sessions).astype(np.int64)
    sf = np.zeros(n_sessions + 1, dtype=np.uint32)
    sf[1:] = np.cumsum(counts)
    info = {"messages": int(n_msgs), "frames": int(n_frames), "text_messages": int(is_text.sum()),
            "fragmented_messages": int((nfrag > 1).sum()), "bad_messages": int(bad.sum()),
            "payload_bytes": int(plen.sum()), "bad_sessions": sorted(set(sess[bad].tolist()))}
    return t, off, sf, int(off[-1]), info


def deflate_plain(seed: int, n_sessions: int, msgs_per_session: int, msg_bytes: int, unique: int = 64):
    """The plain TEXT messages deflate_batch compresses: word-salad ASCII (a 3,000-word
    random vocabulary plus JSON-ish tokens and numbers, ~3x compressible by zlib level 6).
    `unique` distinct sessions are generated and tiled over n_sessions (shared objects).
    Returns [session][message] -> bytes."""
    rng = np.random.default_rng(seed)
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)
    vocab = [bytes(letters[rng.integers(0, 26, int(rng.integers(2, 10)))]) for _ in range(3000)]
    vocab += [b'{"id":', b'"name":', b'"value":', b'},', b'"ts":', b'true', b'false', b'null']
    u = min(unique, n_sessions)
    out = []
    for _ in range(u):
        msgs = []
        for _ in range(msgs_per_session):
            words, n = [], 0
            while n < msg_bytes:
                w = vocab[int(rng.integers(0, len(vocab)))] if rng.random() < 0.9 else str(
                    int(rng.integers(0, 100000))).encode()
                words.append(w)
                n += len(w) + 1
            msgs.append(b" ".join(words)[:msg_bytes])
        out.append(msgs)
    return [out[s % u] for s in range(n_sessions)]


def deflate_batch(seed: int, n_sessions: int, msgs_per_session: int, msg_bytes: int, level: int = 6,
                  unique: int = 64):
    """A decoded batch of permessage-deflate TEXT messages (one FIN frame each, RSV1) as
    PerMessageDeflateEncoder sends them with context takeover: per session one raw
    DEFLATE stream, Z_SYNC_FLUSH after every message, the 00 00 FF FF tail stripped
    (DeflateEncoder.java / PerMessageDeflateEncoder.java).  Message text is word-salad
    ASCII (chat/JSON-like, ~3x compressible).  `unique` distinct session streams are
    compressed on the host and tiled over n_sessions (each copy at its own offset).
    Returns (desc[n], session_first[n_s+1], payload, plain_bytes_per_batch)."""
    import zlib
    from snf4j_amd._lib import DESC_DTYPE
    u = min(unique, n_sessions)
    bodies = deflate_plain(seed, u, msgs_per_session, msg_bytes, unique=u)
    streams, plain = [], []
    for s in range(u):
        comp = zlib.compressobj(level, zlib.DEFLATED, -15)
        msgs, tot = [], 0
        for body in bodies[s]:
            tot += len(body)
            msgs.append((comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH))[:-4])
        streams.append(msgs)
        plain.append(tot)
    n = n_sessions * msgs_per_session
    desc = np.zeros(n, dtype=DESC_DTYPE)
    sizes = np.array([[len(m) for m in streams[s % u]] for s in range(n_sessions)], dtype=np.uint64).reshape(-1)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(sizes, out=off[1:])
    desc["payload_off"] = off[:-1]
    desc["payload_len"] = sizes
    desc["opcode"] = 1
    desc["flags"] = 0x80 | (4 << 4)
    blob = [b"".join(streams[s]) for s in range(u)]
    payload = np.frombuffer(b"".join(blob[s % u] for s in range(n_sessions)) + bytes(16), dtype=np.uint8)
    sf = (np.arange(n_sessions + 1) * msgs_per_session).astype(np.uint32)
    return desc, sf, payload, int(sum(plain[s % u] for s in range(n_sessions)))


def deflate_wire(seed: int, n_sessions: int, msgs_per_session: int, msg_bytes: int, unique: int = 64):
    """deflate_batch's messages as a client sends them on the wire: one masked TEXT frame
    per message with RSV1 set (FrameEncoder.java:81-118 over PerMessageDeflateEncoder's
    output), each session's frames back to back.  Returns (wire u8, session start
    offsets [n_s + 1], plain bytes per batch)."""
    desc, sf, payload, plain = deflate_batch(seed, n_sessions, msgs_per_session, msg_bytes, unique=unique)
    rng = np.random.default_rng(seed ^ 0x3A5C)
    u = min(unique, n_sessions)
    per = []
    for s in range(u):
        parts = []
        for k in range(int(sf[s]), int(sf[s + 1])):
            o, n = int(desc[k]["payload_off"]), int(desc[k]["payload_len"])
            p = payload[o:o + n]
            hl = int(header_len(n, True))
            fr = np.empty(hl + n, dtype=np.uint8)
            fr[0] = 0x80 | 0x40 | 1
            if n <= 125:
                fr[1] = 0x80 | n
            elif n <= 0xFFFF:
                fr[1], fr[2], fr[3] = 0x80 | 126, n >> 8, n & 0xFF
            else:
                fr[1] = 0x80 | 127
                fr[2:10] = np.frombuffer(n.to_bytes(8, "big"), np.uint8)
            m = rng.integers(0, 256, 4, dtype=np.uint8)
            fr[hl - 4:hl] = m
            fr[hl:] = p ^ np.resize(m, n)
            parts.append(fr)
        per.append(np.concatenate(parts))
    sizes = np.array([per[s % u].size for s in range(n_sessions)], dtype=np.int64)
    starts = np.zeros(n_sessions + 1, dtype=np.int64)
    np.cumsum(sizes, out=starts[1:])
    wire = np.concatenate([per[s % u] for s in range(n_sessions)])
    return wire, starts, plain
