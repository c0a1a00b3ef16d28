"""permessage-deflate compression on the GPU (wsg_deflate_batch_*, deflate.hip) against zlib
driven as java.util.zip.Deflater is (oracle/deflate_ref.c): every output byte, the RSV bits,
the pass-through frames and the carried state, at levels 0-9, with and without context
takeover, over many sessions a batch and several batches; the parallel form (levels 4-9)
and zlib's loop per session (levels 1-3, and forced for 4-9) both."""
import json
import os
import zlib

import numpy as np
import pytest

from oracle.deflateref import encode_frames
from tests import deflatehost as dh
from tests.golden.fixtures import unhex

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "deflate_encode_kat.json")


@pytest.fixture(scope="module")
def ctx():
    from snf4j_amd.context import Context
    return Context(0, stream="own")


def _deflater(ctx, n, level, nc, serial=False):
    from snf4j_amd.codec import BatchDeflater
    ctx.set_tuning("deflate_serial", 1 if serial else 0)
    return BatchDeflater(n, level, nc, ctx)


def _check_batches(ctx, sessions, level, nc, n_batches, rng, serial=False):
    """sessions[s] = frame list; runs them over n_batches batches (random cut per session)
    and compares every session with the oracle."""
    n = len(sessions)
    bd = _deflater(ctx, n, level, nc, serial)
    cuts = []
    for fr in sessions:
        c = sorted(int(x) for x in rng.integers(0, len(fr) + 1, n_batches - 1))
        cuts.append([0] + c + [len(fr)])
    got = [[] for _ in range(n)]
    for b in range(n_batches):
        batch = [fr[cuts[s][b]:cuts[s][b + 1]] for s, fr in enumerate(sessions)]
        for s, o in enumerate(bd.run(batch)):
            got[s] += o
    for s, fr in enumerate(sessions):
        ref = encode_frames(fr, level, nc)
        assert got[s] == ref, ("session", s, "level", level, "nc", nc, "serial", serial)
    return bd


def test_golden_encode_vectors(ctx):
    """PerMessageDeflateCodecTest's encoder cases (tests/golden/deflate_encode_kat.json), one
    session a case, all in one batch, both forms."""
    cases = json.load(open(GOLDEN))
    for serial in (False, True):
        for c in cases:
            fr = [(f["opcode"], f["fin"], f["rsv"], unhex(f["payload"])) for f in c["frames"]]
            bd = _deflater(ctx, 1, c["level"], c["no_context"], serial)
            got = bd.run([fr])[0]
            assert [(g[2], g[3]) for g in got] == [(f["out_rsv"], unhex(f["out"])) for f in c["frames"]], c["src"]


def test_encoder_mirror_pass_through_identity(ctx):
    """PerMessageDeflateEncoder.encode hands frames it does not compress on as the same object
    (PerMessageDeflateCodecTest.testEncodeWithoutRsv1 :151-166)."""
    from snf4j_amd.codec import PerMessageDeflateEncoder
    from snf4j_amd.frame import make_frame
    e = PerMessageDeflateEncoder(8, False, ctx)
    for f in [make_frame(1, True, 4, b"ABC"), make_frame(2, True, 7, bytes(range(10))),
              make_frame(0, True, 0, bytes(range(10))), make_frame(9, True, 0, bytes(range(10)))]:
        out = []
        e.encode(None, f, out)
        assert len(out) == 1 and out[0] is f
    out = []
    f = make_frame(1, True, 0, b"ABCDEFG")
    e.encode(None, f, out)
    assert out[0] is not f and out[0].getRsvBits() == 4
    assert zlib.decompressobj(-15).decompress(out[0].getPayload() + b"\x00\x00\xff\xff") == b"ABCDEFG"


@pytest.mark.parametrize("level", range(10))
def test_random_sessions_all_levels(ctx, level):
    rng = np.random.default_rng(100 + level)
    kinds = ["text", "bin", "rand", "tiny", "text"]
    for nc in (False, True):
        sessions = [dh.random_frames(rng, int(rng.integers(1, 24)), kinds[s % 5]) for s in range(40)]
        _check_batches(ctx, sessions, level, nc, 3, rng)


@pytest.mark.parametrize("level", [4, 6, 9])
def test_serial_form_forced(ctx, level):
    """zlib's own loop per session (the form levels 1-3 take) at the parallel levels."""
    rng = np.random.default_rng(200 + level)
    sessions = [dh.random_frames(rng, int(rng.integers(1, 16)), "text") for _ in range(24)]
    _check_batches(ctx, sessions, level, False, 2, rng, serial=True)


@pytest.mark.parametrize("level", [4, 6, 8, 9])
def test_window_slides_nil_edge_runs_big(ctx, level):
    """Window slides at a call start and inside a frame's last bytes, the NIL head exactly
    MAX_DIST back after a slide, one-byte runs, frames longer than the window."""
    rng = np.random.default_rng(300 + level)
    sessions = []
    for s in range(16):
        t = s % 4
        if t == 0:
            sessions.append(dh.nil_edge_frames(rng))
        elif t == 1:
            sessions.append(dh.slide_frames(rng))
        elif t == 2:
            sessions.append([(2, True, 0, (rng.integers(0, 2, int(rng.integers(1, 70000)), dtype=np.uint8)
                                           * int(rng.integers(1, 256))).astype(np.uint8).tobytes())
                             for _ in range(3)])
        else:
            sessions.append(dh.random_frames(rng, 6, "big"))
    _check_batches(ctx, sessions, level, False, 2, rng)


def test_parallel_state_equals_serial(ctx):
    """After the same batches the parallel form leaves the state zlib's loop leaves: the
    scalars, the window up to high_water, the hash heads."""
    rng = np.random.default_rng(400)
    sessions = [dh.random_frames(rng, 12, "text") + dh.slide_frames(rng) for _ in range(8)]
    a = _check_batches(ctx, sessions, 6, False, 1, rng)
    b = _check_batches(ctx, sessions, 6, False, 1, rng, serial=True)
    assert np.array_equal(a.state, b.state)
    ma = a.session_mem.reshape(len(sessions), -1)
    mb = b.session_mem.reshape(len(sessions), -1)
    for s in range(len(sessions)):
        hw = int(a.state[s]["high_water"])
        assert np.array_equal(ma[s, :hw], mb[s, :hw])
        assert np.array_equal(ma[s, 65536:131072], mb[s, 65536:131072])   # head


def test_round_trip_through_gpu_inflater(ctx):
    """Frames compressed on the GPU inflate back on the GPU (BatchInflater, context kept)."""
    from snf4j_amd._lib import DESC_DTYPE
    from snf4j_amd.codec import BatchInflater
    rng = np.random.default_rng(500)
    sessions = [[(1, True, 0, dh.text(rng, int(rng.integers(1, 5000)))) for _ in range(10)] for _ in range(16)]
    enc = _deflater(ctx, 16, 6, False).run(sessions)
    inf = BatchInflater(16, False, ctx)
    rows, chunks, sf, pos = [], [], [0], 0
    for s in range(16):
        for op, fin, rsv, p in enc[s]:
            r = np.zeros((), DESC_DTYPE)
            r["payload_off"], r["payload_len"], r["opcode"] = pos, len(p), op
            r["flags"] = (0x80 if fin else 0) | (rsv << 4)
            rows.append(r)
            chunks.append(p)
            pos += len(p)
        sf.append(len(rows))
    res = inf.run(np.array(rows, DESC_DTYPE), np.array(sf, np.uint32), np.frombuffer(b"".join(chunks), np.uint8))
    for s in range(16):
        frames, exc = res[s]
        assert exc is None
        assert [bytes(f.getPayload()) for f in frames] == [p for (_, _, _, p) in sessions[s]]


def test_bench_shaped_batch(ctx):
    """The bench's shape (word-salad TEXT messages of 4 KiB, level 6, context takeover) over
    256 sessions x 16 messages in one batch."""
    from benchsupport.synth import deflate_plain
    msgs = deflate_plain(0xDEF1, 256, 16, 4096)
    sessions = [[(1, True, 0, m) for m in msgs[s]] for s in range(256)]
    got = _deflater(ctx, 256, 6, False).run(sessions)
    for s in range(0, 256, 5):
        assert got[s] == encode_frames(sessions[s], 6, False), s


def _pmd_stream(rng, n_frames):
    """A session's outgoing frames: messages of 1-3 fragments (TEXT / BINARY then
    continuations), PINGs between fragments, now and then a message already carrying RSV1
    (passed through, PerMessageDeflateEncoder.allowEncoding) and empty payloads."""
    fr, i = [], 0
    while i < n_frames:
        nfrag = int(rng.integers(1, 4))
        op = int(rng.choice([1, 2]))
        rsv = 4 if rng.random() < 0.08 else 0
        for j in range(nfrag):
            n = 0 if rng.random() < 0.05 else int(rng.integers(1, 9000))
            fr.append((op if j == 0 else 0, j == nfrag - 1, rsv if j == 0 else 0, dh.text(rng, n)))
            if rng.random() < 0.1:
                fr.append((9, True, 0, bytes(rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8))))
            i += 1
    return fr


@pytest.mark.parametrize("level,nc", [(6, False), (6, True), (1, False), (9, False), (0, True)])
def test_encode_batcher_deflate(ctx, oracle, level, nc):
    """The permessage-deflate-encoder stage inside the encode batcher
    (wsg_enc_batcher_set_deflate): frames of many sessions added interleaved over several
    pipelined flushes (two in flight), compressed and framed on the device; every session's
    wire bytes equal the reference chain's — PerMessageDeflateEncoder (zlib as Deflater,
    oracle/deflate_ref.c) then FrameEncoder (the oracle's) — with the deflater kept across
    flushes, a CLOSE latching its session, and a slot reset giving a new session a new
    deflater while its old frames are in flight."""
    from snf4j_amd import EncodeBatcher
    from snf4j_amd.frame import make_frame
    for cm in (False, True):
        rng = np.random.default_rng(1000 + 10 * level + nc + 2 * cm)
        n = 24
        b = EncodeBatcher(n, cm, ctx=ctx)
        b.set_deflate(level, nc)
        streams = [_pmd_stream(rng, 40) for _ in range(n)]
        streams[7] = streams[7][:5] + [(8, True, 0, b"\x03\xe8")] + streams[7][5:]   # CLOSE mid-stream
        hist = [[] for _ in range(n)]       # frames since the slot's last reset
        enc = [oracle.Encoder(cm) for _ in range(n)]
        pos = [0] * n
        pending = []
        for flush in range(6):
            want = [b""] * n
            adds = []
            for s in range(n):
                k = int(rng.integers(0, 10))
                for f in streams[s][pos[s]:pos[s] + k]:
                    adds.append((s, f))
                pos[s] += k
            rng.shuffle(adds)
            per = [[] for _ in range(n)]
            for s, f in adds:   # a session's frames keep their order (the shuffle mixes sessions only)
                per[s].append(f)
            order = sorted(range(len(adds)), key=lambda i: rng.random())
            qs = [list(p) for p in per]
            for i in order:
                s = adds[i][0]
                if not qs[s]:
                    continue
                op, fin, rsv, p = qs[s].pop(0)
                mask = tuple(int(x) for x in rng.integers(0, 256, 4))
                b.add(s, make_frame(op, fin, rsv, p), mask)
                h0 = len(hist[s])
                hist[s].append((op, fin, rsv, p))
                out = encode_frames(hist[s], level, nc)[h0]
                want[s] += enc[s].encode(out[0], out[1], out[2], out[3], mask if cm else (0, 0, 0, 0))
            b.flush_async()
            pending.append(want)
            if flush == 3:   # slot 11 to a new session while its frames are in flight
                b.reset_session(11)
                hist[11] = []
                enc[11] = oracle.Encoder(cm)
                for w in pending:
                    w[11] = b""
            if len(pending) == 2:
                assert b.wait() == pending.pop(0), (level, nc, cm, flush)
        while pending:
            assert b.wait() == pending.pop(0), (level, nc, cm)
        b.close()


@pytest.mark.parametrize("level", [5, 9])
def test_match_paths_agree(level):
    """The chain walks out of the LDS ring (k_defl_match_lds, the default) and all in global
    memory (WSG_TUNE_DEFLATE_LDS 0): both byte-identical to zlib, over frames short enough for
    the ring, ones too long for it (> DEFL_LDS_MAXLEN) between them, and runs the ring must
    reload after a long frame."""
    from snf4j_amd.context import Context
    rng = np.random.default_rng(600 + level)
    sessions = []
    for s in range(12):
        fr = []
        for i in range(int(rng.integers(3, 12))):
            n = int(rng.integers(17000, 40000)) if rng.random() < 0.2 else int(rng.integers(0, 9000))
            fr.append((1 if i % 3 == 0 else 0, i % 3 == 2, 0, dh.text(rng, n)))
        sessions.append(fr)
    for lds in (1, 0):
        c = Context(0, stream="own")
        try:
            c.set_tuning("deflate_lds", lds)
            _check_batches(c, sessions, level, False, 2, rng)
        finally:
            c.close()
