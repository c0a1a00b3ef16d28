"""GPU parity of the encode path (FrameEncoder) against the oracle and the
reference's FrameEncoderTest layouts; encode -> decode round trips."""
import numpy as np
import pytest

from tests.golden import fixtures

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from snf4j_amd import Context
    c = Context(0)
    yield c
    c.close()


def _frames(specs):
    from snf4j_amd._lib import ENCODE_DTYPE
    fr = np.zeros(len(specs), dtype=ENCODE_DTYPE)
    payload = []
    off = 0
    for i, (op, fin, rsv, p, mask) in enumerate(specs):
        fr[i]["payload_off"] = off
        fr[i]["payload_len"] = len(p)
        fr[i]["opcode"] = op
        fr[i]["flags"] = (0x80 if fin else 0) | (rsv << 4)
        fr[i]["mask"] = mask
        payload.append(p)
        off += len(p)
    return np.frombuffer(b"".join(payload), dtype=np.uint8).copy() if off else np.zeros(0, np.uint8), fr


def test_encoder_kat(ctx):
    from tests.test_oracle_golden import _encoder_layout
    for i, v in enumerate(fixtures.load("encoder")):
        payload = fixtures.unhex(v["payload"])
        mask = (0x11 * (i % 7 + 1), 0x5A, 0xA5, i & 0xFF)
        pl, fr = _frames([(v["opcode"], v["fin"], v["rsv"], payload, mask)])
        closed = np.zeros(1, np.uint8)
        wire, off = ctx.encode_host(v["client_mode"], pl, fr, np.array([0, 1], np.uint32), closed)
        assert _encoder_layout(wire.tobytes()) == v["expect"]


@pytest.mark.parametrize("cm", [True, False])
def test_random_encode_batches(ctx, oracle, cm):
    rng = np.random.default_rng(31 + cm)
    specs, first = [], [0]
    exp = []
    for s in range(150):
        enc = oracle.Encoder(cm)
        for _ in range(int(rng.integers(0, 9))):
            r = rng.random()
            op = 8 if r < 0.05 else 9 if r < 0.1 else int(rng.choice([0, 1, 2]))
            n = int(rng.integers(0, 125 if op >= 8 else 70000 if rng.random() < 0.1 else 300))
            p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            fin, rsv = bool(rng.integers(0, 2)) or op >= 8, int(rng.integers(0, 8))
            mask = tuple(int(x) for x in rng.integers(0, 256, 4))
            specs.append((op, fin, rsv, p, mask))
            exp.append(enc.encode(op, fin, rsv, p, mask))
        first.append(len(specs))
    pl, fr = _frames(specs)
    closed = np.zeros(len(first) - 1, np.uint8)
    wire, off = ctx.encode_host(cm, pl, fr, np.array(first, np.uint32), closed)
    for k in range(len(specs)):
        assert wire[int(off[k]):int(off[k + 1])].tobytes() == exp[k], k
    # the close latch carried out: sessions that sent CLOSE are closed
    for s in range(len(first) - 1):
        assert closed[s] == any(specs[k][0] == 8 for k in range(first[s], first[s + 1]))


def test_encode_decode_round_trip(ctx, oracle):
    """16 MiB messages fragmented into 64 KiB frames (BASELINE config 5 at reduced count)."""
    from snf4j_amd import decoder_cfg
    from snf4j_amd._lib import STATE_DTYPE
    rng = np.random.default_rng(2)
    msg = rng.integers(0, 256, 1 << 22, dtype=np.uint8).tobytes()
    specs = []
    for i in range(0, len(msg), 65536):
        specs.append((2 if i == 0 else 0, i + 65536 >= len(msg), 0, msg[i:i + 65536],
                      tuple(int(x) for x in rng.integers(0, 256, 4))))
    pl, fr = _frames(specs)
    closed = np.zeros(1, np.uint8)
    wire, off = ctx.encode_host(True, pl, fr, np.array([0, len(specs)], np.uint32), closed)
    state = np.zeros(1, dtype=STATE_DTYPE)
    payload, desc, res = ctx.decode_host(decoder_cfg(False, False, 65536), wire, off, np.array([0, len(specs)],
                                                                                                np.uint32), state)
    assert res[0]["n_delivered"] == len(specs) and res[0]["error"] == 0
    got = b"".join(payload[int(d["payload_off"]):int(d["payload_off"]) + int(d["payload_len"])].tobytes()
                   for d in desc)
    assert got == msg


@pytest.mark.parametrize("cm", [True, False])
def test_large_encode_batch_multipass(ctx, oracle, cm):
    """More frames than the one-workgroup plan takes (encode.hip ENC_PLAN1_MAX):
    the multi-pass latch / offset scans and the coarse piece index, with CLOSE
    frames mid-session and sessions already closed on entry (FrameEncoder.java:71-76)."""
    rng = np.random.default_rng(77 + cm)
    n_s = 3000
    counts = rng.integers(0, 50, n_s)
    pre_closed = rng.random(n_s) < 0.05
    specs, first, exp = [], [0], []
    for s in range(n_s):
        enc = oracle.Encoder(cm)
        for _ in range(int(counts[s])):
            r = rng.random()
            op = 8 if r < 0.01 else 9 if r < 0.03 else int(rng.choice([0, 1, 2]))
            n = int(rng.integers(0, 125 if op >= 8 else (3000 if rng.random() < 0.05 else 200)))
            p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            fin, rsv = bool(rng.integers(0, 2)) or op >= 8, int(rng.integers(0, 8))
            mask = tuple(int(x) for x in rng.integers(0, 256, 4))
            specs.append((op, fin, rsv, p, mask))
            e = enc.encode(op, fin, rsv, p, mask)
            exp.append(b"" if pre_closed[s] else e)
        first.append(len(specs))
    assert len(specs) > 65536
    pl, fr = _frames(specs)
    closed = pre_closed.astype(np.uint8)
    wire, off = ctx.encode_host(cm, pl, fr, np.array(first, np.uint32), closed)
    assert int(off[-1]) == sum(len(e) for e in exp)
    for k in range(len(specs)):
        assert wire[int(off[k]):int(off[k + 1])].tobytes() == exp[k], k
    for s in range(n_s):
        assert closed[s] == (pre_closed[s] or any(specs[k][0] == 8 for k in range(first[s], first[s + 1])))


def test_encode_batcher_matches_oracle(ctx, oracle):
    """The native cross-session encode batcher (wsg_enc_batcher_*): frames of many
    sessions added interleaved over several flushes, 64 KiB frames and small ones,
    CLOSE latches (frames after it dropped, also in later flushes), a slot reset
    for a new session; every session's wire bytes == the oracle FrameEncoder's."""
    from snf4j_amd import EncodeBatcher
    from snf4j_amd.frame import make_frame
    for cm in (True, False):
        rng = np.random.default_rng(808 + cm)
        n = 37
        b = EncodeBatcher(n, cm, ctx=ctx)
        enc = [oracle.Encoder(cm) for _ in range(n)]
        for flush in range(4):
            want = [b""] * n
            for _ in range(int(rng.integers(50, 300))):
                s = int(rng.integers(0, n))
                r = rng.random()
                op = 8 if r < 0.01 else 9 if r < 0.05 else int(rng.choice([0, 1, 2]))
                ln = int(rng.integers(0, 126)) if op >= 8 else 65536 if rng.random() < 0.1 else \
                    int(rng.integers(0, 3000))
                if op == 8 and ln == 1:
                    ln = 2
                p = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
                fin, rsv = bool(rng.integers(0, 2)) or op >= 8, int(rng.integers(0, 8))
                mask = tuple(int(x) for x in rng.integers(0, 256, 4))
                b.add(s, make_frame(op, fin, rsv, p), mask)
                want[s] += enc[s].encode(op, fin, rsv, p, mask if cm else (0, 0, 0, 0))
            if flush == 2:  # slot 3 goes to a new session: queued frames dropped, latch cleared
                b.reset_session(3)
                enc[3] = oracle.Encoder(cm)
                want[3] = b""
            got = b.flush()
            assert got == want, (cm, flush)
        b.close()


def test_encode_batcher_pipelined(ctx, oracle):
    """wsg_enc_batcher_flush_async / wait with two flushes in flight: each flush's view
    equals the oracle FrameEncoders' output for the frames added before it; a CLOSE in
    a flush still in flight latches the frames added after it (the latch is known on
    the host); a slot reset while its frames are in flight drops them from the view."""
    from snf4j_amd import EncodeBatcher
    from snf4j_amd.frame import make_frame
    for cm in (True, False):
        rng = np.random.default_rng(909 + cm)
        n = 29
        b = EncodeBatcher(n, cm, ctx=ctx)
        enc = [oracle.Encoder(cm) for _ in range(n)]
        pending = []  # expected views of the flushes in flight, oldest first
        for flush in range(8):
            want = [b""] * n
            many = []  # odd flushes: the frames go in with one wsg_enc_batcher_add_many
            for _ in range(int(rng.integers(30, 200))):
                s = int(rng.integers(0, n))
                r = rng.random()
                op = 8 if r < 0.01 else 9 if r < 0.05 else int(rng.choice([0, 1, 2]))
                ln = int(rng.integers(0, 126)) if op >= 8 else 65536 if rng.random() < 0.1 else \
                    int(rng.integers(0, 3000))
                if op == 8 and ln == 1:
                    ln = 2
                p = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
                fin, rsv = bool(rng.integers(0, 2)) or op >= 8, int(rng.integers(0, 8))
                mask = tuple(int(x) for x in rng.integers(0, 256, 4))
                if flush & 1:
                    many.append((s, op, (0x80 if fin else 0) | (rsv << 4), mask, np.frombuffer(p, np.uint8)))
                else:
                    b.add(s, make_frame(op, fin, rsv, p), mask)
                want[s] += enc[s].encode(op, fin, rsv, p, mask if cm else (0, 0, 0, 0))
            if many:
                b.add_many_ptrs([m[0] for m in many], [m[1] for m in many], [m[2] for m in many],
                                np.array([m[3] for m in many], dtype=np.uint8),
                                [m[4].ctypes.data if m[4].size else 0 for m in many], [m[4].size for m in many])
            b.flush_async()
            pending.append(want)
            if flush == 4:  # slot 5 to a new session while two flushes hold its frames
                b.reset_session(5)
                enc[5] = oracle.Encoder(cm)
                for w in pending:
                    w[5] = b""
            if len(pending) == 2:
                assert b.wait() == pending.pop(0), (cm, flush)
        while pending:
            assert b.wait() == pending.pop(0), cm
        b.close()
