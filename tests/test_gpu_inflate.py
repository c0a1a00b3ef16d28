"""GPU parity of permessage-deflate decode (inflate.hip, wsg_inflate_batch_*) against the
oracle (PerMessageDeflateDecoder / DeflateDecoder / ZlibDecoder restated over zlib) and the
reference's PerMessageDeflateCodecTest vectors."""
import zlib

import numpy as np
import pytest

from tests import wsgen
from tests.golden import fixtures

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from snf4j_amd import Context
    c = Context(0)
    yield c
    c.close()


def test_deflate_kat_through_gpu(ctx, oracle):
    """PerMessageDeflateCodecTest through the GPU PerMessageDeflateDecoder, one frame per
    batch: round trips (context takeover and not), pass-through identity, failure."""
    from snf4j_amd import InvalidFrameException, PerMessageDeflateDecoder
    from snf4j_amd.frame import make_frame
    for seq in fixtures.load("deflate"):
        frames = [(f["opcode"], f["fin"], f["rsv"], fixtures.unhex(f["payload"])) for f in seq["frames"]]
        d = PerMessageDeflateDecoder(seq["no_context"], ctx=ctx)
        if seq["kind"] == "pass_through":
            for fr in frames:
                x = make_frame(*fr)
                out = []
                d.decode(None, x, out)
                assert out == [x] and out[0] is x, seq["src"]
            continue
        enc = wsgen.pm_deflate_encode(frames, seq["level"], seq["no_context"])
        if seq["kind"] == "round_trip":
            for e, f in zip(enc, frames):
                out = []
                d.decode(None, make_frame(*e), out)
                assert len(out) == 1, seq["src"]
                g = out[0]
                assert (int(g.getOpcode()), g.isFinalFragment(), g.getRsvBits(), g.getPayload()) == f, seq["src"]
        else:
            with pytest.raises(InvalidFrameException) as ei:
                d.decode(None, make_frame(*enc[1]), [])
            assert ei.value.getMessage() == seq["error"]


def _message(rng, big):
    r = rng.random()
    if r < 0.5:
        body = wsgen.rand_text(rng, int(rng.integers(0, 6000 if big else 400)))
    elif r < 0.75:
        body = rng.integers(0, 256, int(rng.integers(0, 70000 if big else 500)), dtype=np.uint8).tobytes()
    else:  # compressible binary: runs and repeats (long matches, short distances)
        unit = rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
        body = unit * int(rng.integers(1, 3000 if big else 50))
    return body


def _session(rng, n_msgs, level, no_context, big, corrupt):
    """A compressed frame stream: messages deflated as PerMessageDeflateEncoder does, the
    compressed bytes of a message cut into fragments at arbitrary byte positions, pings
    between fragments, uncompressed messages, and (optionally) damaged bytes or a stream
    that ends with a final block."""
    comp = zlib.compressobj(level, zlib.DEFLATED, -15)
    out = []
    for _ in range(n_msgs):
        r = rng.random()
        if r < 0.15:  # an uncompressed message (no RSV1): passes through
            out.append((int(rng.choice([1, 2])), True, 0, _message(rng, False)))
            continue
        if r < 0.22:
            out.append((9, True, 0, b"ping"))
            continue
        body = _message(rng, big)
        if no_context:
            comp = zlib.compressobj(level, zlib.DEFLATED, -15)
        if rng.random() < 0.03:  # a final block: the stream ends, later data passes raw
            data = comp.compress(body) + comp.flush(zlib.Z_FINISH)
            comp = zlib.compressobj(level, zlib.DEFLATED, -15)
        else:
            data = comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH)
            data = data[:-4] if body else b"\x00"
        if corrupt and rng.random() < 0.1 and data:
            b = bytearray(data)
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            data = bytes(b)
        cuts = sorted(set(int(x) for x in rng.integers(0, len(data) + 1, int(rng.integers(0, 4)))))
        parts = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
        op = int(rng.choice([1, 2]))
        for i, p in enumerate(parts):
            out.append((op if i == 0 else 0, i == len(parts) - 1, (4 if i == 0 else 0) | int(rng.integers(0, 2)) * 2,
                        p))
            if i + 1 < len(parts) and rng.random() < 0.2:
                out.append((10, True, 0, b""))
    return out


def _run(ctx, oracle, sessions, no_context, n_batches, rng):
    from snf4j_amd import BatchInflater
    from snf4j_amd._lib import DESC_DTYPE
    n_s = len(sessions)
    cuts = [[0] + sorted(int(x) for x in rng.integers(0, len(f) + 1, n_batches - 1)) + [len(f)] for f in sessions]
    bi = BatchInflater(n_s, no_context, ctx=ctx)
    got = [[] for _ in range(n_s)]
    err = [None] * n_s
    base = [0] * n_s
    for b in range(n_batches):
        rows, chunks, sf, pos = [], [], [0], 0
        for s in range(n_s):
            part = sessions[s][cuts[s][b]:cuts[s][b + 1]] if err[s] is None else []
            for (op, fin, rsv, p) in part:
                r = np.zeros((), dtype=DESC_DTYPE)
                r["payload_off"], r["payload_len"], r["opcode"] = pos, len(p), op
                r["flags"] = (0x80 if fin else 0) | (rsv << 4)
                rows.append(r)
                chunks.append(p)
                pos += len(p)
            sf.append(len(rows))
        desc = np.array(rows, dtype=DESC_DTYPE) if rows else np.zeros(0, DESC_DTYPE)
        payload = np.frombuffer(b"".join(chunks) + bytes(16), dtype=np.uint8)
        for s, (frames, exc) in enumerate(bi.run(desc, np.array(sf, np.uint32), payload)):
            got[s] += frames
            if exc is not None and err[s] is None:
                err[s] = (base[s] + exc.frame_index, exc.getMessage())
            base[s] += sf[s + 1] - sf[s]
    for s in range(n_s):
        d = oracle.PerMessageDeflateDecoder(no_context)
        exp, e = [], None
        for i, fr in enumerate(sessions[s]):
            try:
                exp.append(d.decode(*fr))
            except oracle.InvalidFrame as ex:
                e = (i, str(ex))
                break
        assert err[s] == e, (s, err[s], e)
        assert len(got[s]) == len(exp), s
        for i, (g, o) in enumerate(zip(got[s], exp)):
            assert (int(g.getOpcode()), g.isFinalFragment(), g.getRsvBits()) == o[:3], (s, i)
            assert g.getPayload() == o[3], (s, i, len(g.getPayload()), len(o[3]))


@pytest.mark.parametrize("seed", range(6))
def test_inflate_random_batches(ctx, oracle, seed):
    rng = np.random.default_rng(1300 + seed)
    no_context = bool(seed & 1)
    level = [1, 6, 9][seed % 3]
    n_s = int(rng.integers(1, 48))
    sessions = [_session(rng, int(rng.integers(0, 10)), level, no_context, big=seed >= 4, corrupt=seed in (2, 5))
                for _ in range(n_s)]
    _run(ctx, oracle, sessions, no_context, 1 + seed % 3, rng)


def test_inflate_long_context_window(ctx, oracle):
    """Context takeover over many messages: back-references reach 32 KiB into earlier
    messages and earlier batches (the window carried in state/window)."""
    rng = np.random.default_rng(77)
    sessions = []
    for _ in range(6):
        comp = zlib.compressobj(9, zlib.DEFLATED, -15)
        seed_text = wsgen.rand_text(rng, 3000)
        frames = []
        for m in range(30):
            body = seed_text[int(rng.integers(0, 1000)):][:int(rng.integers(100, 3000))] + bytes([m])
            data = comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH)
            frames.append((1, True, 4, data[:-4]))
        sessions.append(frames)
    _run(ctx, oracle, sessions, False, 4, rng)


def test_inflate_predecode_matches_serial_and_zlib(oracle):
    """k_infl_tok + token replay against the serial decoder alone (set_tuning inflate_tokens 0) and
    zlib, on a bench-shaped batch (single-frame messages, context takeover), split over
    two batches so the second replays tokens against a carried-in window."""
    import os
    import zlib
    from snf4j_amd import Context
    from snf4j_amd._lib import DESC_DTYPE, INFLATE_STATE_DTYPE
    from benchsupport.synth import deflate_batch
    n_s, msgs, mb = 96, 8, 2048
    desc, sf, payload, plain = deflate_batch(0xD1F, n_s, msgs, mb, unique=12)
    outs = []
    for flag in (1, 0):
        c = Context(0)
        c.set_tuning("inflate_tokens", flag)
        state = np.zeros(n_s, dtype=INFLATE_STATE_DTYPE)
        window = np.zeros(n_s * 32768, dtype=np.uint8)
        got = [[] for _ in range(n_s)]
        for half in (0, 1):  # messages [0, msgs/2) then [msgs/2, msgs) of every session
            idx = np.concatenate([np.arange(s * msgs, (s + 1) * msgs)[half * msgs // 2:(half + 1) * msgs // 2]
                                  for s in range(n_s)])
            d = desc[idx].copy()
            sfh = (np.arange(n_s + 1) * (msgs // 2)).astype(np.uint32)
            out_off = (np.arange(n_s + 1) * (msgs // 2) * mb).astype(np.uint64)
            out, od, res, rf = c.inflate_host(False, d, sfh, payload, state, window, out_off)
            assert (res["error"] == 0).all() and (rf == 0xFFFFFFFF).all()
            for s in range(n_s):
                for j in range(msgs // 2):
                    o = od[s * (msgs // 2) + j]
                    got[s].append(out[int(o["payload_off"]):int(o["payload_off"]) + int(o["payload_len"])].tobytes())
        c.close()
        outs.append(got)
    assert outs[0] == outs[1]
    for s in range(n_s):
        z = zlib.decompressobj(-15)
        for j in range(msgs):
            o = desc[s * msgs + j]
            exp = z.decompress(payload[int(o["payload_off"]):int(o["payload_off"]) + int(o["payload_len"])].tobytes()
                               + b"\x00\x00\xff\xff")
            assert outs[0][s][j] == exp, (s, j)


def test_inflate_parallel_replay_fallbacks(ctx, oracle):
    """k_infl_fast (the parallel token replay) next to sessions it must leave to the
    serial decoder, in the same batches: a message whose back-reference reaches before
    the decoder's history ("invalid distance too far back"), fragmented messages, an
    uncompressed message, a final block; and sessions it takes, with context carried
    across batches and with no_context.  Every session against the oracle."""
    rng = np.random.default_rng(2024)
    for no_context in (False, True):
        sessions = []
        for i in range(40):
            comp = zlib.compressobj(6, zlib.DEFLATED, -15)
            text = wsgen.rand_text(rng, 4000)
            msgs = []
            for m in range(int(rng.integers(2, 12))):
                if no_context:
                    comp = zlib.compressobj(6, zlib.DEFLATED, -15)
                body = text[int(rng.integers(0, 2000)):][:int(rng.integers(50, 2000))] + bytes([m])
                data = comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH)
                msgs.append((1, True, 4, data[:-4]))
            kind = i % 6
            if kind == 1 and len(msgs) > 2 and not no_context:
                msgs = msgs[1:]  # its first message now refers to history it never had
            elif kind == 2:  # a fragmented message in the middle
                op, fin, rsv, p = msgs[1]
                cut = len(p) // 2
                msgs[1:2] = [(op, False, 4, p[:cut]), (0, True, 0, p[cut:])]
            elif kind == 3:
                msgs.insert(1, (2, True, 0, b"plain"))
            elif kind == 4:
                comp2 = zlib.compressobj(6, zlib.DEFLATED, -15)
                msgs.append((1, True, 4, comp2.compress(b"the end") + comp2.flush(zlib.Z_FINISH)))
            sessions.append(msgs)
        _run(ctx, oracle, sessions, no_context, 3, rng)


@pytest.mark.parametrize("no_context", [False, True])
def test_inflate_fragmented_messages_predecoded(ctx, oracle, no_context):
    """Compressed messages cut into 2-6 fragments at arbitrary bytes (tiny fragments
    that complete no symbol included), pings and uncompressed frames between them:
    k_infl_tok decodes whole multi-frame messages and attributes each symbol to the
    fragment that supplies its last bit's byte (zlib's rule), so k_infl_fast can take
    these sessions; every frame against the oracle."""
    rng = np.random.default_rng(4242 + no_context)
    sessions = []
    for i in range(48):
        comp = zlib.compressobj(int(rng.choice([1, 6, 9])), zlib.DEFLATED, -15)
        text = wsgen.rand_text(rng, 3000)
        frames = []
        for m in range(int(rng.integers(1, 8))):
            if no_context:
                comp = zlib.compressobj(6, zlib.DEFLATED, -15)
            body = text[int(rng.integers(0, 1500)):][:int(rng.integers(20, 3000))] + bytes([m])
            data = (comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH))[:-4]
            n_cuts = int(rng.integers(1, 6))
            cuts = sorted(set(int(x) for x in rng.integers(1, len(data), n_cuts))) if len(data) > 1 else []
            parts = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
            op = int(rng.choice([1, 2]))
            for j, p in enumerate(parts):
                frames.append((op if j == 0 else 0, j == len(parts) - 1, 4 if j == 0 else 0, p))
                if j + 1 < len(parts) and rng.random() < 0.3:
                    frames.append((9, True, 0, b"ping"))
            if rng.random() < 0.2:
                frames.append((1, True, 0, b"plain text"))
        sessions.append(frames)
    _run(ctx, oracle, sessions, no_context, 2, rng)


def test_inflate_after_reserve(oracle):
    """wsg_reserve_inflate pre-sizes the lane pre-decode's workspace (token and literal
    regions, table pool, order): a batch within the reservation decodes as without it."""
    from snf4j_amd import Context
    rng = np.random.default_rng(9200)
    sessions = []
    for i in range(24):
        comp = zlib.compressobj(6, zlib.DEFLATED, -15)
        frames = []
        for m in range(int(rng.integers(1, 6))):
            body = wsgen.rand_text(rng, int(rng.integers(50, 2500)))
            frames.append((1, True, 4, (comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH))[:-4]))
        sessions.append(frames)
    c = Context(0)
    try:
        c.reserve_inflate(4096, 64, 1 << 22)
        _run(c, oracle, sessions, False, 2, rng)
    finally:
        c.close()


@pytest.mark.parametrize("tabs", [0, 5])
def test_inflate_table_pool_exhausted(oracle, tabs):
    """Multi-frame compressed messages need the lane pre-decode's HBM tables, taken from a
    pool (set_tuning inflate_tabs): with none or only a few, the lanes left without one
    hand their messages to the serial decoder, and every frame still matches the oracle."""
    from snf4j_amd import Context
    rng = np.random.default_rng(9100 + tabs)
    sessions = []
    for i in range(40):
        comp = zlib.compressobj(6, zlib.DEFLATED, -15)
        text = wsgen.rand_text(rng, 3000)
        frames = []
        for m in range(int(rng.integers(1, 6))):
            body = text[int(rng.integers(0, 1500)):][:int(rng.integers(200, 3000))] + bytes([m])
            data = (comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH))[:-4]
            cuts = sorted(set(int(x) for x in rng.integers(1, len(data), int(rng.integers(1, 4))))) \
                if len(data) > 1 else []
            parts = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
            for j, p in enumerate(parts):
                frames.append((1 if j == 0 else 0, j == len(parts) - 1, 4 if j == 0 else 0, p))
        sessions.append(frames)
    c = Context(0)
    c.set_tuning("inflate_tabs", tabs)
    try:
        _run(c, oracle, sessions, False, 2, rng)
    finally:
        c.close()


def test_inflate_fast_replay_takes_fragmented_sessions(oracle):
    """With set_tuning inflate_fast 2 the serial pass does not run at all, so every session must
    be finished by the pre-decode + parallel replay: fragmented compressed messages
    (fragments of >= 200 bytes, so each completes a symbol), pings, uncompressed frames,
    context carried over three batches."""
    import os
    from snf4j_amd import Context
    rng = np.random.default_rng(777)
    sessions = []
    for i in range(32):
        comp = zlib.compressobj(6, zlib.DEFLATED, -15)
        text = wsgen.rand_text(rng, 4000)
        frames = []
        for m in range(int(rng.integers(1, 6))):
            body = text[int(rng.integers(0, 1000)):][:int(rng.integers(1500, 3500))] + bytes([m])
            data = (comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH))[:-4]
            cuts, c = [], 0
            while len(data) - c >= 400 and rng.random() < 0.7:
                c += int(rng.integers(200, len(data) - c - 199))
                cuts.append(c)
            parts = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
            op = int(rng.choice([1, 2]))
            for j, p in enumerate(parts):
                frames.append((op if j == 0 else 0, j == len(parts) - 1, 4 if j == 0 else 0, p))
                if j + 1 < len(parts) and rng.random() < 0.3:
                    frames.append((9, True, 0, b"ping"))
            if rng.random() < 0.3:
                frames.append((2, True, 0, b"raw"))
        sessions.append(frames)
    c = Context(0)
    c.set_tuning("inflate_fast", 2)
    try:
        # cut each session only after a FIN data frame (a message boundary)
        n_b = 3
        cut_sessions = []
        for fr in sessions:
            e = [j + 1 for j, f in enumerate(fr) if f[1] and f[0] < 8]
            pts = sorted(rng.choice(e, size=min(n_b - 1, len(e)), replace=False).tolist()) if e else []
            cut_sessions.append((fr, pts))
        _run_cuts(c, oracle, cut_sessions, False, n_b)
    finally:
        c.close()


def _run_cuts(ctx, oracle, cut_sessions, no_context, n_batches):
    """_run with given cut points per session (frame indices where batches split)."""
    from snf4j_amd import BatchInflater
    from snf4j_amd._lib import DESC_DTYPE
    sessions = [fr for fr, _ in cut_sessions]
    n_s = len(sessions)
    cuts = []
    for fr, pts in cut_sessions:
        pts = (pts + [len(fr)] * n_batches)[:n_batches - 1]
        cuts.append([0] + sorted(pts) + [len(fr)])
    bi = BatchInflater(n_s, no_context, ctx=ctx)
    got = [[] for _ in range(n_s)]
    for b in range(n_batches):
        rows, chunks, sf, pos = [], [], [0], 0
        for s in range(n_s):
            for (op, fin, rsv, p) in sessions[s][cuts[s][b]:cuts[s][b + 1]]:
                r = np.zeros((), dtype=DESC_DTYPE)
                r["payload_off"], r["payload_len"], r["opcode"] = pos, len(p), op
                r["flags"] = (0x80 if fin else 0) | (rsv << 4)
                rows.append(r)
                chunks.append(p)
                pos += len(p)
            sf.append(len(rows))
        desc = np.array(rows, dtype=DESC_DTYPE) if rows else np.zeros(0, DESC_DTYPE)
        payload = np.frombuffer(b"".join(chunks) + bytes(16), dtype=np.uint8)
        for s, (frames, exc) in enumerate(bi.run(desc, np.array(sf, np.uint32), payload)):
            assert exc is None, (s, b, exc)
            got[s] += frames
    for s in range(n_s):
        d = oracle.PerMessageDeflateDecoder(no_context)
        exp = [d.decode(*fr) for fr in sessions[s]]
        assert len(got[s]) == len(exp), s
        for i, (g, o) in enumerate(zip(got[s], exp)):
            assert (int(g.getOpcode()), g.isFinalFragment(), g.getRsvBits()) == o[:3], (s, i)
            assert g.getPayload() == o[3], (s, i)


def _lds_path_messages(rng):
    """Single-frame compressed messages aimed at the pre-decode's LDS table paths:
    fixed-code blocks (Z_FIXED), stored blocks (level 0), near-uniform bytes over all
    256 values (most literal codes 8-9 bits: every 7-bit root prefix needs a sub-table,
    far more than the LDS sub-table room of a lane, so the lane falls back to its HBM
    tables), skewed far back-references (distance codes longer than the 6-bit LDS root),
    tiny and multi-block messages."""
    kinds = []
    for i in range(48):
        k = i % 6
        if k == 0:
            body = bytes(rng.integers(97, 123, int(rng.integers(1, 600)), dtype=np.uint8))
            kinds.append(("fixed", body, zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_FIXED)))
        elif k == 1:
            body = bytes(rng.integers(0, 256, int(rng.integers(1, 3000)), dtype=np.uint8))
            kinds.append(("stored", body, zlib.compressobj(0, zlib.DEFLATED, -15)))
        elif k == 2:
            p = np.where(np.arange(256) < 128, 3.0, 1.0)
            body = bytes(rng.choice(256, int(rng.integers(4000, 9000)), p=p / p.sum()).astype(np.uint8))
            kinds.append(("wide", body, zlib.compressobj(6, zlib.DEFLATED, -15)))
        elif k == 3:
            # repeats of chunks at geometric distances: a long tail of distance codes
            base = bytes(rng.integers(97, 123, 30000, dtype=np.uint8))
            parts = []
            for _ in range(400):
                d = int(min(29999, rng.geometric(0.002)))
                s = int(rng.integers(0, 30000 - 8))
                parts.append(base[s:s + 6] + base[max(0, s - d):max(0, s - d) + 5])
            kinds.append(("far", b"".join(parts), zlib.compressobj(9, zlib.DEFLATED, -15)))
        elif k == 4:
            body = bytes(rng.integers(97, 100, int(rng.integers(1, 8)), dtype=np.uint8))
            kinds.append(("tiny", body, zlib.compressobj(6, zlib.DEFLATED, -15)))
        else:
            # several blocks in one message: a small memLevel forces block splits
            words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9)), dtype=np.uint8)) for _ in range(300)]
            body = b" ".join(words[int(j)] for j in rng.integers(0, 300, 6000))
            kinds.append(("blocks", body, zlib.compressobj(6, zlib.DEFLATED, -15, 1)))
    return kinds


def test_inflate_lds_table_paths(oracle):
    """The pre-decode's LDS path (default) against its HBM tables (set_tuning inflate_lds 0), the
    serial decoder alone (set_tuning inflate_tokens 0) and zlib, one session per message (no
    context), every message a single FIN frame."""
    import os
    from snf4j_amd import Context
    from snf4j_amd._lib import DESC_DTYPE, INFLATE_STATE_DTYPE
    rng = np.random.default_rng(0x1D5)
    kinds = _lds_path_messages(rng)
    comp = []
    for _, body, c in kinds:
        comp.append((c.compress(body) + c.flush(zlib.Z_SYNC_FLUSH))[:-4])
    n = len(kinds)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(x) for x in comp], out=off[1:])
    desc["payload_off"] = off[:-1]
    desc["payload_len"] = [len(x) for x in comp]
    desc["opcode"] = 1
    desc["flags"] = 0x80 | (4 << 4)
    payload = np.frombuffer(b"".join(comp) + bytes(16), dtype=np.uint8)
    sf = np.arange(n + 1, dtype=np.uint32)
    cap = max(len(b) for _, b, _ in kinds) + 64
    out_off = (np.arange(n + 1) * cap).astype(np.uint64)
    results = []
    for env in ({}, {"inflate_lds": 0}, {"inflate_tokens": 0}):
        c = Context(0)
        for k, v in env.items():
            c.set_tuning(k, v)
        state = np.zeros(n, dtype=INFLATE_STATE_DTYPE)
        window = np.zeros(n * 32768, dtype=np.uint8)
        out, od, res, rf = c.inflate_host(True, desc, sf, payload, state, window, out_off)
        c.close()
        assert (res["error"] == 0).all(), (env, res["error"])
        results.append([out[int(o["payload_off"]):int(o["payload_off"]) + int(o["payload_len"])].tobytes() for o in od])
    for i, (kind, body, _) in enumerate(kinds):
        assert zlib.decompressobj(-15).decompress(comp[i] + b"\x00\x00\xff\xff") == body
        for r in results:
            assert r[i] == body, (i, kind)


def _split_ctx(mode):
    from snf4j_amd import Context
    c = Context(0)
    c.set_tuning("inflate_split", mode)
    return c


@pytest.mark.parametrize("msg_bytes", [4096, 16384])
def test_inflate_split_lanes_match_zlib(oracle, msg_bytes):
    """The split-lane decode (k_infl_tok<true>: a head lane from the block's first code, a
    tail lane from the middle, joined where the head meets one of the tail's code starts)
    on the bench's message shape (context takeover, one FIN frame a message, ~3x
    compressible text): with it forced (inflate_split 2) every message must equal zlib's
    and the serial decoder's (inflate_tokens 0), and the split must have taken most
    messages (wsg_inflate_split_count); with it off (inflate_split 0) the one-lane decode
    gives the same bytes.  (Only messages whose code tables fit a lane's LDS room split:
    the others take the HBM-table decoder, tok_message, alone.  At 16 KiB, with more
    distinct codes, that is most of them.)"""
    import zlib
    from snf4j_amd._lib import INFLATE_STATE_DTYPE
    from benchsupport.synth import deflate_batch
    n_s, msgs = 64, 6
    desc, sf, payload, plain = deflate_batch(0x5B1 + msg_bytes, n_s, msgs, msg_bytes, unique=16)
    n_big = int((desc["payload_len"] >= 1024).sum())
    assert n_big >= n_s * msgs // 2  # the shape this test is about: messages a split takes
    outs = []
    for env in ({"inflate_split": 2}, {"inflate_split": 0}, {"inflate_tokens": 0}):
        from snf4j_amd import Context
        c = Context(0)
        for k, v in env.items():
            c.set_tuning(k, v)
        state = np.zeros(n_s, dtype=INFLATE_STATE_DTYPE)
        window = np.zeros(n_s * 32768, dtype=np.uint8)
        out_off = (np.arange(n_s + 1) * msgs * (msg_bytes + 4096)).astype(np.uint64)
        out, od, res, rf = c.inflate_host(False, desc, sf, payload, state, window, out_off)
        assert (res["error"] == 0).all()
        outs.append([out[int(o["payload_off"]):int(o["payload_off"]) + int(o["payload_len"])].tobytes() for o in od])
        n_split = c.inflate_split_count()
        c.close()
        if env.get("inflate_split") == 2:
            assert n_split >= (0.9 if msg_bytes <= 4096 else 0.25) * n_big, (n_split, n_big)
        else:
            assert n_split == 0, (env, n_split)
    assert outs[0] == outs[1] == outs[2]
    for s in range(n_s):
        z = zlib.decompressobj(-15)
        for j in range(msgs):
            o = desc[s * msgs + j]
            exp = z.decompress(payload[int(o["payload_off"]):int(o["payload_off"]) + int(o["payload_len"])].tobytes()
                               + b"\x00\x00\xff\xff")
            assert outs[0][s * msgs + j] == exp, (s, j)


@pytest.mark.parametrize("seed", range(6))
def test_inflate_random_batches_split_modes(oracle, seed):
    """test_inflate_random_batches' sessions (fragments, pings, raw messages, final
    blocks, damaged bytes) with the split-lane decode forced on every message, and off."""
    for mode in (2, 0):
        rng = np.random.default_rng(1300 + seed)
        no_context = bool(seed & 1)
        level = [1, 6, 9][seed % 3]
        n_s = int(rng.integers(1, 48))
        sessions = [_session(rng, int(rng.integers(0, 10)), level, no_context, big=True, corrupt=seed in (2, 5))
                    for _ in range(n_s)]
        c = _split_ctx(mode)
        try:
            _run(c, oracle, sessions, no_context, 1 + seed % 3, rng)
        finally:
            c.close()


def test_inflate_lds_table_paths_split(oracle):
    """_lds_path_messages (fixed codes, stored blocks, wide and far codes, several blocks a
    message) with the split-lane decode forced, against zlib: a first block that is
    stored leaves the message to the head, a split whose window falls past the first
    block's end is dropped, and the tail's later blocks rebuild its tables."""
    from snf4j_amd._lib import DESC_DTYPE, INFLATE_STATE_DTYPE
    rng = np.random.default_rng(0x5D5)
    kinds = _lds_path_messages(rng)
    comp = [(c.compress(body) + c.flush(zlib.Z_SYNC_FLUSH))[:-4] for _, body, c in kinds]
    n = len(kinds)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(x) for x in comp], out=off[1:])
    desc["payload_off"] = off[:-1]
    desc["payload_len"] = [len(x) for x in comp]
    desc["opcode"] = 1
    desc["flags"] = 0x80 | (4 << 4)
    payload = np.frombuffer(b"".join(comp) + bytes(16), dtype=np.uint8)
    sf = np.arange(n + 1, dtype=np.uint32)
    cap = max(len(b) for _, b, _ in kinds) + 64
    out_off = (np.arange(n + 1) * cap).astype(np.uint64)
    c = _split_ctx(2)
    try:
        state = np.zeros(n, dtype=INFLATE_STATE_DTYPE)
        window = np.zeros(n * 32768, dtype=np.uint8)
        out, od, res, rf = c.inflate_host(True, desc, sf, payload, state, window, out_off)
        assert (res["error"] == 0).all(), res["error"]
        assert c.inflate_split_count() > 0
    finally:
        c.close()
    for i, (kind, body, _) in enumerate(kinds):
        o = od[i]
        assert out[int(o["payload_off"]):int(o["payload_off"]) + int(o["payload_len"])].tobytes() == body, (i, kind)
