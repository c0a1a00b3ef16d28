"""GPU parity of the decode path (libwsgpu HIP kernels) against the CPU oracle and
the reference's golden vectors.  Bit-exact payloads, identical frame sequences,
identical first-error frame / message / close code per session."""
import numpy as np
import pytest

import benchsupport

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


def _cfg(cm, ext, maxp, val=True):
    from snf4j_amd import decoder_cfg
    return decoder_cfg(cm, ext, maxp, val)


def compare(gpu, ora, sf, tag=""):
    gp, gd, gr = gpu
    op, od, orr = ora
    for s in range(len(sf) - 1):
        g, o = gr[s], orr[s]
        assert (int(g["n_delivered"]), int(g["error"]), int(g["close_code"]), int(g["detail"])) == \
               (int(o["n_delivered"]), int(o["error"]), int(o["close_code"]), int(o["detail"])), (tag, s)
        for k in range(int(sf[s]), int(sf[s]) + int(g["n_delivered"])):
            a, b = gd[k], od[k]
            assert int(a["opcode"]) == int(b["opcode"]), (tag, s, k)
            assert int(a["flags"]) & 0xF0 == int(b["flags"]) & 0xF0, (tag, s, k)
            assert int(a["payload_len"]) == int(b["payload_len"]), (tag, s, k)
            assert int(a["payload_off"]) % 16 == 0
            n = int(a["payload_len"])
            ga = gp[int(a["payload_off"]):int(a["payload_off"]) + n]
            ob = op[int(b["payload_off"]):int(b["payload_off"]) + n]
            assert np.array_equal(ga, ob), (tag, s, k)


def run_parity(ctx, oracle, sessions, cm=False, ext=False, maxp=65536, val=True, n_batches=1, rng=None, tag=""):
    from snf4j_amd._lib import STATE_DTYPE
    n_s = len(sessions)
    state = np.zeros(n_s, dtype=STATE_DTYPE)
    ob = oracle.Batch(cm, ext, maxp, val, n_s)
    # cut every session's stream into n_batches consecutive parts
    cuts = []
    for fr in sessions:
        pts = sorted(int(x) for x in (rng.integers(0, len(fr) + 1, n_batches - 1) if rng is not None and n_batches > 1
                                      else []))
        cuts.append([0] + pts + [len(fr)])
    for b in range(n_batches):
        part = [fr[cuts[i][b]:cuts[i][b + 1]] for i, fr in enumerate(sessions)]
        wire, off, sf = wsgen.make_batch(part)
        gpu = ctx.decode_host(_cfg(cm, ext, maxp, val), wire, off, sf, state)
        ora = ob.decode(wire, off, sf)
        compare(gpu, ora, sf, f"{tag} batch {b}")


def test_single_frames_basic(ctx, oracle):
    rng = np.random.default_rng(0)
    sess = [[wsgen.build_frame(2, True, 0, bytes(range(n % 256)) * (n // 256 + 1), True, (1, 2, 3, 4))]
            for n in (0, 1, 2, 3, 15, 16, 17, 63, 64, 65, 125, 126, 1000, 4096, 65535, 65536)]
    run_parity(ctx, oracle, sess, rng=rng, tag="basic")


@pytest.mark.parametrize("seed", range(12))
def test_random_sessions_with_injected_errors(ctx, oracle, seed):
    rng = np.random.default_rng(100 + seed)
    cm = bool(seed & 1)
    ext = bool(seed & 2)
    maxp = [65536, 512, 131072][seed % 3]
    sessions = []
    for s in range(int(rng.integers(1, 120))):
        inj = None
        if rng.random() < 0.35:
            inj = wsgen.INJECT_KINDS[int(rng.integers(0, len(wsgen.INJECT_KINDS)))]
            if inj == "max_payload":
                inj = "too_long"
        sessions.append(wsgen.session_frames(rng, int(rng.integers(0, 12)), client_mode=cm, allow_ext=ext,
                                             max_payload=maxp, inject=inj))
    run_parity(ctx, oracle, sessions, cm=cm, ext=ext, maxp=maxp, val=seed % 4 != 3, n_batches=1 + seed % 3,
               rng=rng, tag=f"seed{seed}")


def test_fragment_seams_utf8(ctx, oracle):
    """Every split of multi-byte code points across 2-3 fragments, empty fragments,
    pings between fragments (FrameUtf8Validator carry, FrameUtf8Validator.java:78-96)."""
    rng = np.random.default_rng(9)
    texts = ["aé€😀b", "😀😀", "€", "é", "ab", "中文字", "\U0010ffff!"]
    bad = [b"\xe2\x82", b"\xed\xa0\x80", b"\xf0\x9f\x98", b"\xc3", b"\xf4\x90\x80\x80", b"\x80"]
    sessions = []
    for t in texts:
        body = t.encode()
        for i in range(len(body) + 1):
            for j in range(i, len(body) + 1):
                fr = [wsgen.build_frame(1, False, 0, body[:i], True, (9, 8, 7, 6)),
                      wsgen.build_frame(9, True, 0, b"", True, (1, 1, 1, 1)),
                      wsgen.build_frame(0, False, 0, body[i:j], True, (5, 4, 3, 2)),
                      wsgen.build_frame(0, True, 0, body[j:], True, (0, 1, 0, 1))]
                sessions.append(fr)
    for b in bad:
        for i in range(len(b) + 1):
            sessions.append([wsgen.build_frame(1, False, 0, b"x" + b[:i], True, (1, 2, 3, 4)),
                             wsgen.build_frame(0, True, 0, b[i:] + b"y", True, (4, 3, 2, 1))])
        sessions.append([wsgen.build_frame(1, False, 0, b, True, (1, 2, 3, 4)),
                         wsgen.build_frame(0, False, 0, b"", True, (1, 2, 3, 4)),
                         wsgen.build_frame(0, True, 0, b"", True, (1, 2, 3, 4))])
    run_parity(ctx, oracle, sessions, n_batches=3, rng=rng, tag="seams")


def test_utf8_sweeps(ctx, oracle):
    """Utf8Test sweeps (:107-207) as one TEXT frame per session, unmasked, client mode."""
    from snf4j_amd._lib import STATE_DTYPE
    strings = []
    strings += [bytes([a, b]) for a in range(256) for b in range(256)]
    v = np.arange(0, 0x10000)
    three = np.stack([0xE0 | (v >> 12), 0x80 | ((v >> 6) & 0x3F), 0x80 | (v & 0x3F)], axis=-1).astype(np.uint8)
    strings += [r.tobytes() for r in three] + [r[:2].tobytes() for r in three[::7]]
    v = np.arange(0x10000, 0x110100, 3)
    four = np.stack([0xF0 | (v >> 18), 0x80 | ((v >> 12) & 0x3F), 0x80 | ((v >> 6) & 0x3F), 0x80 | (v & 0x3F)],
                    axis=-1).astype(np.uint8)
    strings += [r.tobytes() for r in four] + [r[:3].tobytes() for r in four[::11]]
    rng = np.random.default_rng(4)
    strings += [rng.integers(0x80, 0x100, int(rng.integers(1, 9)), dtype=np.uint8).tobytes() for _ in range(20000)]
    sessions = [[wsgen.build_frame(1, True, 0, s, False)] for s in strings]
    wire, off, sf = wsgen.make_batch(sessions)
    state = np.zeros(len(sessions), dtype=STATE_DTYPE)
    _, _, res = ctx.decode_host(_cfg(True, False, 65536), wire, off, sf, state)
    exp = np.array([oracle.utf8_is_valid(s) for s in strings])
    got = res["error"] == 0
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [strings[i].hex() for i in bad[:10]]
    assert (res["error"][~exp] == 14).all() and (res["close_code"][~exp] == 1007).all()


def test_decoder_kat_through_gpu_frame_decoder(ctx):
    """FrameDecoderTest sequences through the GPU-backed FrameDecoder mirror."""
    from snf4j_amd import FrameDecoder, InvalidFrameException
    for v in fixtures.load("decode"):
        dec = FrameDecoder(v["client_mode"], v["allow_extensions"], v["max_payload"], True, ctx=ctx)
        for st in v["steps"]:
            if "available" in st:
                d = fixtures.unhex(st["available"])
                assert dec.available(None, d, 0, len(d)) == st["expect"]
                continue
            data = fixtures.unhex(st["data"])
            out = []
            if "error" in st:
                with pytest.raises(InvalidFrameException) as ei:
                    dec.decode(None, data, out)
                assert str(ei.value) == st["error"], v["src"]
                assert dec.closed
            else:
                dec.decode(None, data, out)
                if st.get("none"):
                    assert out == [], v["src"]
                else:
                    f = out[0]
                    e = st["frame"]
                    assert (int(f.getOpcode()), f.isFinalFragment(), f.getRsvBits()) == \
                           (e["opcode"], e["fin"], e["rsv"]), v["src"]
                    assert f.getPayload() == fixtures.unhex(e["payload"]), v["src"]


def _batcher(kind):
    from snf4j_amd import NativeBatcher, SessionBatcher
    return SessionBatcher if kind == "python" else NativeBatcher


@pytest.mark.parametrize("kind", ["python", "native"])
def test_session_kat_through_batcher(ctx, kind):
    """WebSocketSessionTest stream cases through the cross-session batcher (the
    Python SessionBatcher and the native wsg_batcher)."""
    cases = fixtures.load("session")
    by_max = {}
    for i, v in enumerate(cases):
        by_max.setdefault(v["max_payload"], []).append(i)
    for maxp, idx in by_max.items():
        b = _batcher(kind)(len(idx), clientMode=True, maxPayloadLen=maxp, ctx=ctx)
        for sid, i in enumerate(idx):
            for ch in cases[i]["chunks"]:
                b.feed(sid, fixtures.unhex(ch))
        res = b.flush()
        for sid, i in enumerate(idx):
            frames, exc = res[sid]
            v = cases[i]
            assert [(int(f.getOpcode()), f.getPayload()) for f in frames] == \
                   [(e["opcode"], fixtures.unhex(e["payload"])) for e in v["frames"]], v["src"]
            if "error" in v:
                assert exc is not None and str(exc) == v["error"] and exc.close_code == v["close_code"], v["src"]
            else:
                assert exc is None


@pytest.mark.parametrize("kind", ["python", "native"])
def test_batcher_matches_stream_oracle(ctx, oracle, kind):
    """Random streams fed in random socket-read chunks through the batcher, several
    flushes, against the oracle's session read loop."""
    rng = np.random.default_rng(21)
    n = 40
    streams = [b"".join(wsgen.session_frames(rng, int(rng.integers(1, 10)),
                                             inject=(wsgen.INJECT_KINDS[int(rng.integers(0, 15))]
                                                     if rng.random() < 0.3 else None)))
               for _ in range(n)]
    b = _batcher(kind)(n, clientMode=False, maxPayloadLen=65536, ctx=ctx)
    got = [[] for _ in range(n)]
    err = [None] * n
    pos = [0] * n
    while any(pos[s] < len(streams[s]) for s in range(n)):
        for s in range(n):
            if pos[s] < len(streams[s]):
                c = int(rng.integers(1, 3000))
                b.feed(s, streams[s][pos[s]:pos[s] + c])
                pos[s] += c
        for s, (fr, e) in enumerate(b.flush()):
            got[s] += fr
            if e is not None and err[s] is None:
                err[s] = e
    for s in range(n):
        frames, e = oracle.stream_decode(streams[s], [len(streams[s])])
        assert [(f.opcode, f.fin, f.rsv, f.payload) for f in frames] == \
               [(int(f.getOpcode()), f.isFinalFragment(), f.getRsvBits(), f.getPayload()) for f in got[s]], s
        assert (str(e) if e else None) == (str(err[s]) if err[s] else None), s


def test_device_resident_synth_parity(ctx, oracle):
    """Device-generated batch (wsg_synth_uniform) decoded in HBM; checked frame by
    frame against the oracle on the same bytes."""
    import torch
    from snf4j_amd import decoder_cfg
    from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE, STATE_DTYPE
    for (nf, plen, fps, op, text) in [(4096, 4096, 64, 1, 1), (8192, 1024, 32, 2, 0), (2000, 65536, 50, 1, 1),
                                     (3000, 100, 7, 1, 1)]:
        flen = ctx_len = plen + (14 if plen > 0xFFFF else 8 if plen > 125 else 6)
        n_s = (nf + fps - 1) // fps
        dev = torch.device("cuda:0")
        wire = torch.empty(nf * flen + 64, dtype=torch.uint8, device=dev)
        off = torch.empty(nf + 1, dtype=torch.int64, device=dev)
        sf = torch.empty(n_s + 1, dtype=torch.int32, device=dev)
        benchsupport.synth_uniform(ctx, 77, nf, plen, fps, op, True, text, wire, off, sf)
        state = torch.zeros(n_s * 8, dtype=torch.uint8, device=dev)
        payload = torch.empty(nf * flen + 16 * nf + 16, dtype=torch.uint8, device=dev)
        desc = torch.empty(nf * 16, dtype=torch.uint8, device=dev)
        res = torch.empty(n_s * 16, dtype=torch.uint8, device=dev)
        ctx.decode_device(decoder_cfg(False, False, 65536, True), wire, off, sf, state, payload, desc, res,
                          wire_len=nf * flen)
        ctx.sync()
        w = wire[:nf * flen].cpu().numpy()
        o = off.cpu().numpy().view(np.uint64)
        s = sf.cpu().numpy().view(np.uint32)
        ow, oo, osf = oracle.synth_uniform(77, nf, plen, fps, opcode=op, masked=True, text=bool(text))
        assert np.array_equal(w, ow) and np.array_equal(o, oo) and np.array_equal(s, osf)
        gpu = (payload.cpu().numpy(), desc.cpu().numpy().view(DESC_DTYPE), res.cpu().numpy().view(RESULT_DTYPE))
        ora = oracle.Batch(False, False, 65536, True, n_s).decode(w, o, s)
        compare(gpu, ora, s, f"synth {nf}x{plen}")
        st = state.cpu().numpy().view(STATE_DTYPE)
        assert (st["closed"] == 0).all() and (st["fragmentation"] == 0).all()


def test_empty_and_closed_sessions(ctx, oracle):
    from snf4j_amd._lib import STATE_DTYPE
    # no frames at all
    state = np.zeros(3, dtype=STATE_DTYPE)
    p, d, r = ctx.decode_host(_cfg(False, False, 65536), np.zeros(0, np.uint8), np.zeros(1, np.uint64),
                              np.zeros(4, np.uint32), state)
    assert (r["n_delivered"] == 0).all() and (r["error"] == 0).all()
    # a closed session swallows everything (FrameDecoder.java:185-187)
    state[1]["closed"] = 1
    sessions = [[wsgen.build_frame(2, True, 0, b"abc", True, (1, 2, 3, 4))] for _ in range(3)]
    wire, off, sf = wsgen.make_batch(sessions)
    p, d, r = ctx.decode_host(_cfg(False, False, 65536), wire, off, sf, state)
    assert list(r["n_delivered"]) == [1, 0, 1] and (r["error"] == 0).all()


def test_host_async_matches_sync(ctx, oracle):
    """wsg_decode_batch_host_async (pipelined host path): two back-to-back batches that
    share sessions and one host state array == the sync host path batch by batch."""
    import torch
    from snf4j_amd import Context
    from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE, STATE_DTYPE
    rng = np.random.default_rng(77)
    sessions = [wsgen.session_frames(rng, int(rng.integers(0, 14)),
                                     inject=wsgen.INJECT_KINDS[i % len(wsgen.INJECT_KINDS)] if i % 4 == 0 else None)
                for i in range(40)]
    cuts = [int(rng.integers(0, len(fr) + 1)) for fr in sessions]
    batches = [wsgen.make_batch([fr[:c] for fr, c in zip(sessions, cuts)]),
               wsgen.make_batch([fr[c:] for fr, c in zip(sessions, cuts)])]
    cfg = _cfg(False, False, 65536)
    n_s = len(sessions)
    st_sync = np.zeros(n_s, dtype=STATE_DTYPE)
    want = [ctx.decode_host(cfg, w, o, f, st_sync) for w, o, f in batches]
    c2 = Context(0, stream=torch.cuda.Stream())
    st = np.zeros(n_s, dtype=STATE_DTYPE)
    got = []
    try:
        for w, o, f in batches:
            n = len(o) - 1
            pay = np.zeros(w.size + 16 * n + 16, np.uint8)
            desc = np.zeros(max(1, n), DESC_DTYPE)
            res = np.zeros(n_s, RESULT_DTYPE)
            c2.decode_host_async(cfg, w if w.size else np.zeros(1, np.uint8), o, f, st, pay, desc, res,
                                 wire_len=w.size)
            got.append((pay, desc[:n], res))
        c2.sync()
    finally:
        c2.close()
    assert np.array_equal(st, st_sync)
    for (gp, gd, gr), (wp, wd, wr), (w, o, f) in zip(got, want, batches):
        assert np.array_equal(gr, wr) and np.array_equal(gd, wd)
        compare((gp, gd, gr), (wp, wd, wr), f, "async")


@pytest.mark.parametrize("empties", [0, 70, 300])
def test_dense_small_frames(ctx, oracle, empties):
    """Pieces holding many frames: tiny text/binary frames (the lane-parallel frame
    lookup of the multi-frame piece path) and runs of zero-length frames longer
    than a wave (its walking fallback), with UTF-8 split across tiny fragments."""
    rng = np.random.default_rng(500 + empties)
    sessions = []
    for s in range(24):
        fr = []
        for m in range(int(rng.integers(20, 60))):
            if rng.random() < 0.5:
                body = wsgen.rand_text(rng, int(rng.integers(0, 12)))
                pts = wsgen.split_points(rng, len(body), int(rng.integers(1, 4)))
                for i in range(len(pts) - 1):
                    fr.append(wsgen.build_frame(1 if i == 0 else 0, i == len(pts) - 2, 0, body[pts[i]:pts[i + 1]], True,
                                                tuple(int(x) for x in rng.integers(0, 256, 4))))
            else:
                fr.append(wsgen.build_frame(2, True, 0, rng.integers(0, 256, int(rng.integers(0, 40)),
                                                                       dtype=np.uint8).tobytes(), True, (9, 8, 7, 6)))
            if empties and rng.random() < 0.05:
                fr.extend(wsgen.build_frame(9, True, 0, b"", True, (1, 1, 1, 1)) for _ in range(empties))
        if s % 5 == 0:
            fr.insert(len(fr) // 2, wsgen.bad_frame(rng, "utf8", True, 65536))
        sessions.append(fr)
    run_parity(ctx, oracle, sessions, rng=rng, n_batches=2, tag=f"dense {empties}")


@pytest.mark.parametrize("masked", [True, False])
def test_tail_utf8_large_frames(ctx, oracle, masked):
    """A frame's last byte and the end of a FIN message are tested by the piece
    kernel on the bytes it holds (decode.hip tail_error): invalid leads, stray
    continuation bytes and truncated sequences at the end of frames whose last
    piece is full, partial, 1-3 bytes long, or the frame's only piece, with the
    frame FIN, followed by a continuation, or ending a fragmented message."""
    rng = np.random.default_rng(21)
    tails = [b"", b"\xff", b"\xc3", b"\xe2\x82", b"\xf0\x9f\x98", b"\xc3\xa9", b"\x80", b"\xed\xa0", b"\xf4\x90",
             b"\xe2\x82\xac", b"\xf0\x9f\x98\x80", b"\xc0"]
    lens = [1, 2, 3, 4, 15, 16, 17, 18, 31, 1020, 1021, 1022, 1023, 1024, 1025, 1026, 1027, 2047, 2048, 2049,
            3071, 3072, 3073, 4096, 4097, 4098, 6000]
    sessions = []
    cm = not masked
    for n in lens:
        for t in tails:
            if len(t) > n:
                continue
            body = b"a" * (n - len(t)) + t
            m = tuple(int(x) for x in rng.integers(0, 256, 4))
            sessions.append([wsgen.build_frame(1, True, 0, body, masked, m)])
            sessions.append([wsgen.build_frame(1, False, 0, body, masked, m),
                             wsgen.build_frame(0, True, 0, b"\x80\x80z", masked, m)])
            sessions.append([wsgen.build_frame(1, False, 0, b"x\xe2", masked, m),
                             wsgen.build_frame(0, True, 0, body, masked, m)])
            sessions.append([wsgen.build_frame(1, False, 0, b"\xf0\x9f", masked, m),
                             wsgen.build_frame(0, True, 0, t[:2], masked, m)])
    run_parity(ctx, oracle, sessions, cm=cm, n_batches=2, rng=rng, tag="tails")


def test_native_batcher_large_random_chunks(ctx, oracle):
    """The native batcher's threaded gather (> 8 MiB per flush) with frames split
    across many feeds, against the oracle's read loop."""
    from snf4j_amd import NativeBatcher
    rng = np.random.default_rng(33)
    n = 64
    streams = [b"".join(wsgen.session_frames(rng, int(rng.integers(5, 40)), big=True)) for _ in range(n)]
    b = NativeBatcher(n, ctx=ctx)
    got = [[] for _ in range(n)]
    err = [None] * n
    pos = [0] * n
    while any(pos[s] < len(streams[s]) for s in range(n)):
        for s in range(n):
            c = int(rng.integers(1, 200000))
            if pos[s] < len(streams[s]):
                b.feed(s, streams[s][pos[s]:pos[s] + c])
                pos[s] += c
        for s, (fr, e) in enumerate(b.flush()):
            got[s] += fr
            if e is not None and err[s] is None:
                err[s] = e
    for s in range(n):
        frames, e = oracle.stream_decode(streams[s], [len(streams[s])])
        assert [(f.opcode, f.fin, f.payload) for f in frames] == \
               [(int(f.getOpcode()), f.isFinalFragment(), f.getPayload()) for f in got[s]], s
        assert (str(e) if e else None) == (str(err[s]) if err[s] else None), s


def test_native_batcher_feed_many_threaded(ctx, oracle):
    """wsg_batcher_feed_many with every session's reads of a round in one call (the
    sessions framed in place by several threads, > 4 MiB a call), big frames that stay
    partial over several rounds (carried, then landed once complete), then one flush:
    the same frames and verdicts as the oracle's read loop."""
    from snf4j_amd import NativeBatcher
    rng = np.random.default_rng(34)
    n = 48
    streams = [b"".join(wsgen.session_frames(rng, int(rng.integers(5, 30)), big=bool(s % 3 == 0))) for s in range(n)]
    cuts = [[0] + sorted(int(x) for x in rng.integers(0, len(st) + 1, int(rng.integers(1, 12)))) + [len(st)]
            for st in streams]
    b = NativeBatcher(n, ctx=ctx)
    for r in range(max(len(c) for c in cuts) - 1):
        sids, chunks = [], []
        for s in range(n):
            if r + 1 < len(cuts[s]) and cuts[s][r + 1] > cuts[s][r]:
                # a round's read of a session, sometimes split in two reads of the same call
                a0, a1 = cuts[s][r], cuts[s][r + 1]
                m = int(rng.integers(a0, a1 + 1))
                for x0, x1 in ((a0, m), (m, a1)):
                    if x1 > x0:
                        sids.append(s)
                        chunks.append(streams[s][x0:x1])
        b.feed_many(sids, chunks)
    res = b.flush()
    for s in range(n):
        fr, e = res[s]
        frames, oe = oracle.stream_decode(streams[s], [len(streams[s])])
        assert [(f.opcode, f.fin, f.payload) for f in frames] == \
               [(int(f.getOpcode()), f.isFinalFragment(), f.getPayload()) for f in fr], s
        assert (str(oe) if oe else None) == (str(e) if e else None), s


def test_pinned_pool(ctx):
    from snf4j_amd.codec import pinned_alloc, pinned_release
    a = pinned_alloc(5000)
    assert a.size == 8192
    a[:] = 7
    addr = a.ctypes.data
    pinned_release(a)
    b2 = pinned_alloc(6000)  # recycled from the same size class
    assert b2.ctypes.data == addr
    pinned_release(b2)
    with pytest.raises(ValueError):
        pinned_release(np.zeros(16, np.uint8))


def test_native_batcher_session_reset_reuses_slot(ctx, oracle):
    """A slot handed to a new session (wsg_batcher_session_reset) decodes exactly as
    a fresh FrameDecoder + FrameUtf8Validator: the old session's closed latch (it
    failed), its open fragmented text message with a split code point, its partial
    frame and bytes fed but never flushed are all gone."""
    from snf4j_amd import NativeBatcher
    rng = np.random.default_rng(404)
    m = (1, 2, 3, 4)
    old = [
        # failed: a bad opcode closes the session
        wsgen.build_frame(1, True, 0, b"hi", True, m) + bytes([0x83, 0x80]) + bytes(m),
        # an open text message ending inside a code point, and half of the next frame
        wsgen.build_frame(1, False, 0, b"ab\xe2\x82", True, m) + wsgen.build_frame(0, True, 0, b"\xac!", True, m)[:5],
        # a fragmented binary message left open (FrameDecoder.fragmentation)
        wsgen.build_frame(2, False, 0, b"\x00" * 300, True, m),
        b"",
    ]
    unflushed = [b"", b"", wsgen.build_frame(0, True, 0, b"zz", True, m)[:3], wsgen.build_frame(1, True, 0, b"x", True, m)]
    n = len(old)
    b = NativeBatcher(n, ctx=ctx)
    for s in range(n):
        if old[s]:
            b.feed(s, old[s])
    first = b.flush()
    assert first[0][1] is not None and first[1][1] is None and first[2][1] is None
    for s in range(n):
        if unflushed[s]:
            b.feed(s, unflushed[s])
        b.reset_session(s)
    # the new sessions start with a continuation (an error for a fresh decoder: it must
    # not continue the old session's message) or with ordinary traffic
    new = [b"".join(wsgen.session_frames(rng, int(rng.integers(1, 8)))) for _ in range(n)]
    new[1] = wsgen.build_frame(0, True, 0, b"\xac", True, m) + new[1]
    new[2] = wsgen.build_frame(0, True, 0, b"more", True, m) + new[2]
    got = [[] for _ in range(n)]
    err = [None] * n
    pos = [0] * n
    while any(pos[s] < len(new[s]) for s in range(n)):
        for s in range(n):
            if pos[s] < len(new[s]):
                c = int(rng.integers(1, 700))
                b.feed(s, new[s][pos[s]:pos[s] + c])
                pos[s] += c
        for s, (fr, e) in enumerate(b.flush()):
            got[s] += fr
            if e is not None and err[s] is None:
                err[s] = e
    for s in range(n):
        frames, e = oracle.stream_decode(new[s], [len(new[s])])
        assert [(f.opcode, f.fin, f.payload) for f in frames] == \
               [(int(f.getOpcode()), f.isFinalFragment(), f.getPayload()) for f in got[s]], s
        assert (str(e) if e else None) == (str(err[s]) if err[s] else None), s
    assert err[1] is not None and err[2] is not None  # a fresh decoder rejects the leading continuation
    b.close()


def test_native_batcher_pipelined_flushes(ctx, oracle):
    """wsg_batcher_feed_many + flush_async/wait with two flushes in flight: the next
    reads and gather overlap the device work, the carry chains through the batches on
    the device.  Random socket chunks (threaded feeds above 4 MiB), header errors the
    host finds (opcode 3), sessions reset while a flush is in flight; every session's
    frames and first error == the oracle's read loop (a reset session: its new stream)."""
    from snf4j_amd import NativeBatcher
    rng = np.random.default_rng(515)
    n = 96
    streams = [b"".join(wsgen.session_frames(rng, int(rng.integers(1, 12)), big=(s % 3 == 0),
                                            inject=(wsgen.INJECT_KINDS[int(rng.integers(0, 15))]
                                                    if rng.random() < 0.2 else None)))
               for s in range(n)]
    for s in range(0, n, 13):  # a header error the host sees first: a bad opcode after some frames
        streams[s] += bytes([0x83, 0x85, 1, 2, 3, 4]) + b"\x00" * 5
    b = NativeBatcher(n, ctx=ctx)
    got = [[] for _ in range(n)]
    err = [None] * n
    pos = [0] * n
    reset_at = {7: 1, 31: 2, 50: 3}  # session -> round at which its slot gets a new session
    new = {}
    pending = 0

    def collect():
        for s, (fr, e) in enumerate(b.wait()):
            got[s] += fr
            if e is not None and err[s] is None:
                err[s] = e

    rnd = 0
    while any(pos[s] < len(streams[s]) for s in range(n)) or pending:
        sids, chunks = [], []
        for s in range(n):
            if reset_at.get(s) == rnd:
                b.reset_session(s)  # (a flush may be in flight: its results for s are dropped)
                streams[s] = new[s] = b"".join(wsgen.session_frames(rng, int(rng.integers(1, 8))))
                pos[s], got[s], err[s] = 0, [], None
            for _ in range(int(rng.integers(0, 3))):
                if pos[s] < len(streams[s]):
                    c = int(rng.integers(1, 150000))
                    sids.append(s)
                    chunks.append(streams[s][pos[s]:pos[s] + c])
                    pos[s] += c
        if sids:
            b.feed_many(sids, chunks)
        if pending == 2:
            collect()
            pending -= 1
        if any(pos[s] < len(streams[s]) for s in range(n)) or sids:
            b.flush_async()
            pending += 1
        else:
            collect()
            pending -= 1
        rnd += 1
    for s in range(n):
        frames, e = oracle.stream_decode(streams[s], [len(streams[s])])
        assert [(f.opcode, f.fin, f.payload) for f in frames] == \
               [(int(f.getOpcode()), f.isFinalFragment(), f.getPayload()) for f in got[s]], s
        assert (str(e) if e else None) == (str(err[s]) if err[s] else None), s
    assert set(new) == set(reset_at)
    b.close()
