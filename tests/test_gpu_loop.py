"""The drop-in's loop scheduling (snf4j_amd/loop.py, the restatement of
WsgBatcher.java's) on the GPU: reads fed once per loop iteration, flushes collected in
a later iteration after the completion thread re-enters the loop, two flushes in
flight, sessions ending and their slots reused mid-stream, the encode side with a
CLOSE draining what is in flight.  Every session's frames and first error == the
oracle's read loop (FrameDecoder.java:180-401, FrameUtf8Validator.java:59-98 over
StreamSession.java:798-854); every session's written bytes == the oracle encoder's
(FrameEncoder.java:69-135)."""
import random

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


def test_loop_decode_matches_oracle(ctx, oracle):
    from benchsupport.selector import SelectorLoop, run_until_idle
    from snf4j_amd.loop import LoopBatcher
    rng = random.Random(2024)
    nrng = np.random.default_rng(2024)
    n = 64
    streams = [b"".join(wsgen.session_frames(nrng, rng.randrange(1, 14), big=(s % 7 == 0),
                                            inject=(wsgen.INJECT_KINDS[rng.randrange(15)]
                                                    if rng.random() < 0.2 else None)))
               for s in range(n)]
    for s in range(0, n, 11):  # a header error the host finds first
        streams[s] += bytes([0x83, 0x85, 1, 2, 3, 4]) + b"\x00" * 5
    got = [[] for _ in range(n)]
    err = [None] * n
    closed = [False] * n  # GpuFrameDecoder.closed: after its first error a session's input is swallowed
    gen = [0] * n  # the session occupying each slot

    def deliver(sid, frames, exc):
        got[sid] += frames
        if exc is not None and err[sid] is None:
            err[sid] = exc
            closed[sid] = True

    loop = SelectorLoop()
    lb = LoopBatcher(loop, n, deliver, ctx=ctx, max_wire=4 << 20, max_frames=1 << 14)
    pos = [0] * n
    end_at = {3: 4, 20: 7, 41: 2}  # slot -> iteration its session ends (the slot then serves a new one)
    it = 0
    while any(pos[s] < len(streams[s]) for s in range(n)):
        it += 1
        reads = []
        for s in range(n):
            if end_at.get(s) == it:
                lb.reset_session(s)  # IEventDrivenCodec ENDING -> unregister
                gen[s] += 1
                streams[s] = b"".join(wsgen.session_frames(nrng, rng.randrange(1, 8)))
                pos[s], got[s], err[s], closed[s] = 0, [], None, False
            if pos[s] < len(streams[s]) and rng.random() < 0.6:
                c = rng.randrange(1, 40000)
                chunk = streams[s][pos[s]:pos[s] + c]
                pos[s] += c

                def read(s=s, chunk=chunk):
                    if not closed[s]:
                        lb.enqueue(s, chunk)
                reads.append(read)
        loop.run_iteration(reads)
        if not reads:  # nothing readable: the loop sleeps until the completion thread wakes it
            loop.select(0.05)
    run_until_idle(loop, lb)
    for s in range(n):
        frames, e = oracle.stream_decode(streams[s], [len(streams[s])])
        assert [(f.opcode, f.fin, f.rsv, f.payload) for f in frames] == \
               [(int(f.getOpcode()), f.isFinalFragment(), f.getRsvBits(), f.getPayload()) for f in got[s]], s
        assert (str(e) if e else None) == (str(err[s]) if err[s] else None), s
    st = lb.stats
    # one flush per iteration with reads, each delivered after its iteration's reads
    # (two in flight needs the device to lag the loop: tests/test_gpu_jni.py queues them
    # explicitly; the bench's drop_in_loop line reports how often it happens)
    assert st["flushes"] >= 5 and st["max_inflight"] >= 1, st
    lb.close()


def test_loop_encode_matches_oracle(ctx, oracle):
    from snf4j_amd import frame as F
    from benchsupport.selector import SelectorLoop, run_until_idle
    from snf4j_amd.loop import LoopEncodeBatcher
    rng = random.Random(77)
    n = 24
    written = [b"" for _ in range(n)]
    loop = SelectorLoop()
    eb = LoopEncodeBatcher(loop, n, lambda sid, b: written.__setitem__(sid, written[sid] + b), clientMode=True,
                           ctx=ctx, max_frames=1024, max_payload=8 << 20)
    enc = [oracle.Encoder(True) for _ in range(n)]
    expect = [b"" for _ in range(n)]
    for it in range(12):
        writes = []
        for s in range(n):
            for _ in range(rng.randrange(0, 3)):
                op = rng.choice([1, 2, 2, 9]) if it < 9 or rng.random() < 0.8 else 8
                payload = bytes(rng.randrange(256) for _ in range(rng.choice([0, 10, 126, 5000, 70000])))
                if op >= 8:
                    payload = b"\x03\xe8" if op == 8 else payload[:125]
                fin = op >= 8 or rng.random() < 0.7
                mask = tuple(rng.randrange(256) for _ in range(4))
                fr = F.make_frame(op, fin, 0, payload)
                expect[s] += enc[s].encode(op, fin, 0, payload, mask)

                def write(s=s, fr=fr, mask=mask, op=op):
                    if op == 8:  # GpuFrameEncoder: a CLOSE first writes out everything before it
                        eb.enqueue(s, fr, mask)
                        eb.flush_encodes()
                    else:
                        eb.enqueue(s, fr, mask)
                writes.append(write)
        loop.run_iteration(writes)
    run_until_idle(loop, eb)
    for s in range(n):
        assert written[s] == expect[s], s
    eb.close()


def test_reserve_refused_with_flushes_in_flight(ctx, oracle):
    """wsg_batcher_reserve / wsg_enc_batcher_reserve move the slots' buffers, which a
    queued flush still reads and writes: with flushes in flight they return
    WSG_API_ERANGE and change nothing; the queued flushes' results stay exact."""
    from snf4j_amd import frame as F
    from snf4j_amd._lib import WsgError
    from snf4j_amd.codec import EncodeBatcher, NativeBatcher
    rng = random.Random(5)
    nrng = np.random.default_rng(5)
    n = 8
    nb = NativeBatcher(n, ctx=ctx)
    nb.reserve(1 << 16, 256)
    streams = [[b"".join(wsgen.session_frames(nrng, rng.randrange(1, 6))) for _ in range(2)] for _ in range(n)]
    for k in range(2):
        for s in range(n):
            nb.feed(s, streams[s][k])
        nb.flush_async()
    with pytest.raises(WsgError):
        nb.reserve(64 << 20, 1 << 20)  # larger: every buffer would move
    for k in range(2):
        got = nb.wait()
        for s in range(n):
            frames, e = oracle.stream_decode(streams[s][k])
            assert [(f.opcode, f.payload) for f in frames] == \
                   [(int(f.getOpcode()), f.getPayload()) for f in got[s][0]], (k, s)
    nb.reserve(64 << 20, 1 << 20)  # idle: fine
    nb.close()
    eb = EncodeBatcher(n, True, ctx=ctx)
    eb.reserve(64, 1 << 16)
    enc = [oracle.Encoder(True) for _ in range(n)]
    expect = []
    for k in range(2):
        exp = []
        for s in range(n):
            p = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 3000)))
            eb.add(s, F.make_frame(2, True, 0, p), (1, 2, 3, 4))
            exp.append(enc[s].encode(2, True, 0, p, (1, 2, 3, 4)))
        expect.append(exp)
        eb.flush_async()
    with pytest.raises(WsgError):
        eb.reserve(1 << 16, 64 << 20)
    for k in range(2):
        assert list(eb.wait()) == expect[k], k
    eb.close()
