"""GPU parity of the native batcher with the decoders after "ws-decoder" in the same
flush (wsg_batcher_set_stages): FrameDecoder -> PerMessageDeflateDecoder ->
FrameUtf8Validator -> FrameAggregator, the pipeline snf4j builds when
permessage-deflate is negotiated (DefaultWebSocketSessionConfig.java:276-281,
PerMessageDeflateExtension.java:316-326) with an application FrameAggregator after
it.  The oracle runs the same chain frame by frame per session: the C restatement's
session read loop, then the restated PerMessageDeflateDecoder (over zlib), the
restated FrameUtf8Validator and FrameAggregator, stopping at the first exception."""
import zlib

import numpy as np
import pytest

from tests import wsgen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from snf4j_amd import Context
    c = Context(0)
    yield c
    c.close()


def _messages(rng, n_msgs, no_context, bad_utf8, big=False):
    """(opcode, fin, rsv, payload) of one session: compressed text/binary messages cut
    into fragments with pings between them, uncompressed messages, invalid UTF-8 in a
    few compressed text messages, corrupt compressed bytes now and then."""
    comp = zlib.compressobj(6, zlib.DEFLATED, -15)
    out = []
    for _ in range(n_msgs):
        r = rng.random()
        if r < 0.15:
            op = int(rng.choice([1, 2]))
            body = wsgen.rand_text(rng, int(rng.integers(0, 300))) if op == 1 else \
                rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
            out.append((op, True, 0, body))
            continue
        if r < 0.2:
            out.append((9, True, 0, b"ping"))
            continue
        op = 1 if rng.random() < 0.7 else 2
        top = 12000 if big else 3000
        body = wsgen.rand_text(rng, int(rng.integers(0, top))) if op == 1 else \
            rng.integers(0, 256, int(rng.integers(0, top)), dtype=np.uint8).tobytes()
        if op == 1 and rng.random() < bad_utf8:
            bad = wsgen.BAD_UTF8[int(rng.integers(0, len(wsgen.BAD_UTF8)))]
            at = int(rng.integers(0, len(body) + 1))
            body = body[:at] + bad + body[at:]
        if no_context:
            comp = zlib.compressobj(6, zlib.DEFLATED, -15)
        data = comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH)
        data = data[:-4] if body else b"\x00"
        if rng.random() < 0.02 and data:
            b = bytearray(data)
            b[int(rng.integers(0, len(b)))] ^= 0x10
            data = bytes(b)
        cuts = sorted(set(int(x) for x in rng.integers(0, len(data) + 1, int(rng.integers(0, 4)))))
        parts = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
        for i, p in enumerate(parts):
            out.append((op if i == 0 else 0, i == len(parts) - 1, 4 if i == 0 else 0, p))
            if i + 1 < len(parts) and rng.random() < 0.2:
                out.append((10, True, 0, b""))
    return out


def _oracle_chain(oracle, stream, no_context, validate, aggregate, max_agg):
    """[(opcode, fin, rsv, payload)] the handler receives, and the first error
    (message, close code) or None."""
    frames, derr = oracle.stream_decode(stream, [len(stream)], client_mode=False, allow_extensions=True, max_payload_len=1 << 20,
                                        validate_utf8=False)
    inf = oracle.PerMessageDeflateDecoder(no_context)
    val = oracle.Validator()
    agg = oracle.Aggregator(max_agg) if aggregate else None
    out = []
    for f in frames:
        try:
            op, fin, rsv, p = inf.decode(f.opcode, f.fin, f.rsv, f.payload)
        except oracle.InvalidFrame as e:
            return out, (str(e), e.close_code)
        if validate and not val.decode(op, fin, p):
            return out, (oracle.format_error(14), 1007)
        if agg is not None:
            try:
                g = agg.decode(op, fin, rsv, p)
            except oracle.InvalidFrame as e:
                return out, (oracle.format_error(18), 1009)
            if g is None:
                continue
            op, fin, rsv, p = g.opcode, g.fin, g.rsv, g.payload
        out.append((op, fin, rsv, p))
    if derr is not None:
        return out, (str(derr), derr.close_code)
    return out, None


@pytest.mark.parametrize("seed,no_context,aggregate", [(0, False, True), (1, True, True), (2, False, False),
                                                       (3, False, True)])
def test_batcher_stage_chain_matches_oracle(ctx, oracle, seed, no_context, aggregate):
    _chain_case(ctx, oracle, seed, no_context, aggregate)


def test_batcher_stage_chain_split_lanes(oracle):
    """The chain with the split-lane inflate forced (set_tuning inflate_split 2 on the
    batcher's context, which its stage context takes over), with and without context
    takeover; the split must have taken some messages (a message cut into fragments, or
    whose tables need the HBM decoder, is decoded by one lane)."""
    from snf4j_amd import Context
    c = Context(0)
    try:
        c.set_tuning("inflate_split", 2)
        n_split = sum(_chain_case(c, oracle, seed, no_context, True, big=True)
                      for seed, no_context in ((0, False), (1, True)))
        assert n_split > 0
    finally:
        c.close()


def _chain_case(ctx, oracle, seed, no_context, aggregate, big=False):
    from snf4j_amd import NativeBatcher
    rng = np.random.default_rng(6100 + seed)
    n = 48
    max_agg = 4000 if seed == 3 else 1 << 20
    streams = []
    for s in range(n):
        msgs = _messages(rng, int(rng.integers(1, 14)), no_context, bad_utf8=0.05, big=big)
        wire = b"".join(wsgen.build_frame(op, fin, rsv, p, True, tuple(int(x) for x in rng.integers(0, 256, 4)))
                        for (op, fin, rsv, p) in msgs)
        if s % 11 == 5:  # a protocol error after some frames (opcode 3)
            wire += bytes([0x83, 0x80, 1, 2, 3, 4])
        streams.append(wire)
    b = NativeBatcher(n, clientMode=False, allowExtensions=True, maxPayloadLen=1 << 20, ctx=ctx)
    b.set_stages(inflate=True, noContext=no_context, validate=True, aggregate=aggregate,
                 maxAggregatedLength=max_agg)
    got = [[] for _ in range(n)]
    err = [None] * n
    pos = [0] * n
    while any(pos[s] < len(streams[s]) for s in range(n)):
        for s in range(n):
            if pos[s] < len(streams[s]):
                c = int(rng.integers(1, 4000))
                b.feed(s, streams[s][pos[s]:pos[s] + c])
                pos[s] += c
        for s, (fr, e) in enumerate(b.flush()):
            got[s] += fr
            if e is not None:
                assert err[s] is None, s  # one error per session, then it is closed
                err[s] = (e.getMessage(), e.close_code)
    n_err = 0
    for s in range(n):
        exp, eerr = _oracle_chain(oracle, streams[s], no_context, True, aggregate, max_agg)
        assert err[s] == eerr, (s, err[s], eerr)
        assert [(int(f.getOpcode()), f.isFinalFragment(), f.getRsvBits(), f.getPayload()) for f in got[s]] == exp, s
        n_err += eerr is not None
    assert n_err  # the generator produced failures of some kind
    n_split = b.stage_split_count()
    b.close()
    return n_split


@pytest.mark.parametrize("seed,aggregate,depth", [(10, True, 2), (11, False, 2), (12, True, 3), (13, False, 3),
                                                   (14, True, 4), (15, False, 4)])
def test_batcher_stage_chain_pipelined(ctx, oracle, seed, aggregate, depth):
    """The same chain with `depth` flushes in flight (wsg_batcher_flush_async / wait; 4 =
    WSG_BATCHER_MAX_INFLIGHT: flush_async and feed_many start the queued chains, each
    wait collects the next flush's chain and begins the one after): a session a stage fails in one flush gets nothing from the flushes
    already in flight behind it (the session is closed), a slot reset while its chains
    are begun or collected delivers nothing of the old session, and a reset slot starts
    from fresh stage decoders."""
    from snf4j_amd import NativeBatcher
    rng = np.random.default_rng(6200 + seed)
    n = 40
    streams = []
    for s in range(n):
        msgs = _messages(rng, int(rng.integers(4, 16)), False, bad_utf8=0.15)
        streams.append(b"".join(wsgen.build_frame(op, fin, rsv, p, True, tuple(int(x) for x in rng.integers(0, 256, 4)))
                                for (op, fin, rsv, p) in msgs))
    b = NativeBatcher(n, clientMode=False, allowExtensions=True, maxPayloadLen=1 << 20, ctx=ctx)
    b.set_stages(inflate=True, noContext=False, validate=True, aggregate=aggregate, maxAggregatedLength=1 << 20)
    for rnd in range(2):  # round 1: every slot reset, the same streams again from fresh sessions
        if rnd:
            for s in range(n):
                b.reset_session(s)
        got = [[] for _ in range(n)]
        err = [None] * n
        pos = [0] * n
        pending = 0

        def collect():
            for s, (fr, e) in enumerate(b.wait()):
                got[s] += fr
                if e is not None:
                    assert err[s] is None, s
                    err[s] = (e.getMessage(), e.close_code)

        it = 0
        while any(pos[s] < len(streams[s]) for s in range(n)):
            it += 1
            if rnd == 0 and it == 3:  # slots to new sessions mid-stream, flushes in flight
                for s in range(0, n, 7):
                    b.reset_session(s)
                    got[s], err[s], pos[s] = [], None, 0
            for s in range(n):
                if pos[s] < len(streams[s]):
                    c = int(rng.integers(1, 1500))
                    b.feed(s, streams[s][pos[s]:pos[s] + c])
                    pos[s] += c
            if pending == depth:
                collect()
                pending -= 1
            b.flush_async()
            pending += 1
        while pending:
            collect()
            pending -= 1
        n_err = 0
        for s in range(n):
            exp, eerr = _oracle_chain(oracle, streams[s], False, True, aggregate, 1 << 20)
            assert err[s] == eerr, (rnd, s, err[s], eerr)
            assert [(int(f.getOpcode()), f.isFinalFragment(), f.getRsvBits(), f.getPayload()) for f in got[s]] == exp, (rnd, s)
            n_err += eerr is not None
        assert n_err
    b.close()


def test_batcher_stage_chain_capacity_rerun(ctx, oracle):
    """Messages that inflate far more than the stage's first output region per session
    (4 KiB + 8x the compressed bytes): those sessions are re-run with larger regions,
    nothing of the first run having been committed, beside sessions that fit."""
    from snf4j_amd import NativeBatcher
    rng = np.random.default_rng(6300)
    n = 24
    streams = []
    for s in range(n):
        comp = zlib.compressobj(9, zlib.DEFLATED, -15)
        wire = b""
        for m in range(int(rng.integers(1, 5))):
            if s % 3 == 0:
                body = bytes([65 + m]) * int(rng.integers(20000, 120000))  # ~1000:1
            else:
                body = wsgen.rand_text(rng, int(rng.integers(10, 2000)))
            data = (comp.compress(body) + comp.flush(zlib.Z_SYNC_FLUSH))[:-4]
            wire += wsgen.build_frame(1, True, 4, data, True, tuple(int(x) for x in rng.integers(0, 256, 4)))
        streams.append(wire)
    b = NativeBatcher(n, clientMode=False, allowExtensions=True, maxPayloadLen=1 << 20, ctx=ctx)
    b.set_stages(inflate=True, noContext=False, validate=True, aggregate=False)
    got = [[] for _ in range(n)]
    for s in range(n):
        b.feed(s, streams[s])
    for s, (fr, e) in enumerate(b.flush()):
        assert e is None, (s, e)
        got[s] += fr
    for s in range(n):
        exp, eerr = _oracle_chain(oracle, streams[s], False, True, False, 1 << 20)
        assert eerr is None
        assert [(int(f.getOpcode()), f.isFinalFragment(), f.getRsvBits(), f.getPayload()) for f in got[s]] == exp, s
    b.close()


def test_batcher_stage_chain_threaded_feeds(ctx, oracle):
    """Feeds big enough for wsg_batcher_feed_many's thread pool (8 MB a round), so the
    chains of the flushes in flight advance on the calling thread while the workers
    copy (stage_advance beside the copies), WSG_BATCHER_MAX_INFLIGHT flushes deep, with
    slots reset mid-stream; every session's frames and first error equal the oracle
    chain's."""
    from snf4j_amd import NativeBatcher
    from snf4j_amd._lib import BATCHER_MAX_INFLIGHT
    rng = np.random.default_rng(6400)
    n, u, chunk = 1024, 32, 8192
    uniq = []
    for _ in range(u):
        msgs = _messages(rng, 20, False, bad_utf8=0.04)
        uniq.append(b"".join(wsgen.build_frame(op, fin, rsv, p, True, tuple(int(x) for x in rng.integers(0, 256, 4)))
                             for (op, fin, rsv, p) in msgs))
    wire = np.frombuffer(b"".join(uniq), dtype=np.uint8).copy()
    ustart = np.concatenate([[0], np.cumsum([len(x) for x in uniq])])
    base = wire.ctypes.data
    b = NativeBatcher(n, clientMode=False, allowExtensions=True, maxPayloadLen=1 << 20, ctx=ctx)
    b.set_stages(inflate=True, noContext=False, validate=True)
    got = [[] for _ in range(n)]
    err = [None] * n
    pos = np.zeros(n, dtype=np.int64)
    end = np.array([len(uniq[s % u]) for s in range(n)], dtype=np.int64)
    off = np.array([ustart[s % u] for s in range(n)], dtype=np.int64)

    def collect():
        for s, (fr, e) in enumerate(b.wait()):
            got[s] += fr
            if e is not None:
                assert err[s] is None, s
                err[s] = (e.getMessage(), e.close_code)

    pending, it = 0, 0
    while (pos < end).any():
        it += 1
        if it == 2:  # slots to new sessions mid-stream, flushes in flight
            for s in range(0, n, 97):
                b.reset_session(s)
                got[s], err[s], pos[s] = [], None, 0
        live = np.nonzero(pos < end)[0]
        ln = np.minimum(end[live] - pos[live], chunk)
        assert ln.sum() >= (4 << 20) or it > 2  # (the pool's threshold: the first rounds are threaded)
        b.feed_many_ptrs(live.astype(np.uint32), (base + off[live] + pos[live]).astype(np.uint64), ln.astype(np.uint64))
        pos[live] += ln
        if pending == BATCHER_MAX_INFLIGHT:
            collect()
            pending -= 1
        b.flush_async()
        pending += 1
    while pending:
        collect()
        pending -= 1
    b.close()
    want = [_oracle_chain(oracle, uniq[k], False, True, False, 1 << 20) for k in range(u)]
    n_err = 0
    for s in range(n):
        exp, eerr = want[s % u]
        assert err[s] == eerr, (s, err[s], eerr)
        assert [(int(f.getOpcode()), f.isFinalFragment(), f.getRsvBits(), f.getPayload()) for f in got[s]] == exp, s
        n_err += eerr is not None
    assert n_err


def test_stage_failure_reported_by_wait_not_by_flush():
    """A stage-chain step that fails while flush_async or a feed advances the chains of
    flushes already queued (WSG_TUNE_STAGE_FAIL injects it, as a device error would come):
    those calls still return OK — the flush is queued, the reads copied — and a later
    wsg_batcher_wait reports the error; the batcher goes on with the flushes after it."""
    from snf4j_amd import Context, NativeBatcher
    from snf4j_amd._lib import WsgError
    rng = np.random.default_rng(6500)
    n = 16
    c = Context(0)
    try:
        b = NativeBatcher(n, clientMode=False, allowExtensions=True, maxPayloadLen=1 << 20, ctx=c)
        b.set_stages(inflate=True, noContext=False, validate=True)
        streams = [b"".join(wsgen.build_frame(op, fin, rsv, p, True, (1, 2, 3, 4))
                            for (op, fin, rsv, p) in _messages(rng, 12, False, bad_utf8=0.0)) for _ in range(n)]
        c.set_tuning("stage_fail", 2)
        errors, pending, pos = [], 0, [0] * n
        for it in range(8):
            for s in range(n):
                if pos[s] < len(streams[s]):
                    b.feed(s, streams[s][pos[s]:pos[s] + 700])   # never raises for the side step
                    pos[s] += 700
            if pending == 3:
                try:
                    b.wait()
                except WsgError as e:
                    errors.append(str(e))
                pending -= 1
            b.flush_async()   # queued: OK whatever the stage step it ran on the side did
            pending += 1
        while pending:
            try:
                b.wait()
            except WsgError as e:
                errors.append(str(e))
            pending -= 1
        assert len(errors) == 1 and "injected stage failure" in errors[0], errors
        b.close()
    finally:
        c.close()
