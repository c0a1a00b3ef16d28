"""GPU parity of the standalone FrameUtf8Validator stage (wsg_validate_batch_*,
the "ws-utf8-validator" stage kept separate when permessage-deflate is on)
against the oracle (FrameUtf8Validator.java:59-98) and FrameUtf8ValidatorTest."""
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


def test_validator_kat_through_gpu(ctx):
    """FrameUtf8ValidatorTest.testDecode :81-133, one frame per batch (the carry
    crosses every batch boundary)."""
    from snf4j_amd import FrameUtf8Validator, InvalidFrameException
    from snf4j_amd.frame import make_frame
    for seq in fixtures.load("validator"):
        v = FrameUtf8Validator(ctx=ctx)
        for f in seq["frames"]:
            fr = make_frame(f["opcode"], f["fin"], 0, bytes.fromhex(f["payload"]))
            out = []
            if "error" in f:
                with pytest.raises(InvalidFrameException) as ei:
                    v.decode(None, fr, out)
                assert ei.value.getMessage() == "Invalid text frame payload: bytes are not UTF-8"
                v = FrameUtf8Validator(ctx=ctx)  # the reference test uses a fresh validator after a throw
            else:
                v.decode(None, fr, out)
                assert out == [fr] and out[0] is fr


def _plain_batch(parts, rng, aligned=False):
    """desc / session_first / payload of plain frames, payload offsets unaligned
    (or each payload at a 16-B boundary)."""
    from snf4j_amd._lib import DESC_DTYPE
    n = sum(len(p) for p in parts)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    chunks, pos, k, sf = [], 0, 0, [0]
    for fr in parts:
        for (op, fin, p) in fr:
            gap = (-pos) % 16 if aligned else int(rng.integers(0, 7))
            chunks.append(bytes(gap))
            pos += gap
            desc[k]["payload_off"] = pos
            desc[k]["payload_len"] = len(p)
            desc[k]["opcode"] = op
            desc[k]["flags"] = 0x80 if fin else 0
            chunks.append(p)
            pos += len(p)
            k += 1
        sf.append(k)
    payload = np.frombuffer(b"".join(chunks) + bytes(32), dtype=np.uint8).copy()
    return desc, np.array(sf, np.uint32), payload


def _text_messages(rng, n_msgs, big):
    """(opcode, fin, payload) frames: text messages split at arbitrary bytes (code
    points across fragments), binary and control frames between fragments, with
    some invalid sequences injected."""
    out = []
    for _ in range(n_msgs):
        r = rng.random()
        if r < 0.6:
            body = wsgen.rand_text(rng, int(rng.integers(0, 3000 if big else 300)))
            if rng.random() < 0.15:
                bad = wsgen.BAD_UTF8[int(rng.integers(0, len(wsgen.BAD_UTF8)))]
                at = int(rng.integers(0, len(body) + 1))
                body = body[:at] + bad + body[at:]
            cuts = sorted(int(x) for x in rng.integers(0, len(body) + 1, int(rng.integers(0, 4))))
            pieces = [body[a:b] for a, b in zip([0] + cuts, cuts + [len(body)])]
            for i, pc in enumerate(pieces):
                out.append((1 if i == 0 else 0, i == len(pieces) - 1, pc))
                if rng.random() < 0.2 and i + 1 < len(pieces):
                    out.append((9, True, b"p"))
        elif r < 0.85:
            out.append((2, True, rng.integers(0, 256, int(rng.integers(0, 2000)), dtype=np.uint8).tobytes()))
        else:
            out.append((10, True, b""))
    return out


@pytest.mark.parametrize("seed", range(6))
def test_validate_random_batches(ctx, oracle, seed):
    from snf4j_amd._lib import STATE_DTYPE
    rng = np.random.default_rng(900 + seed)
    n_s = int(rng.integers(1, 120))
    sessions = [_text_messages(rng, int(rng.integers(0, 12)), big=seed >= 3) for _ in range(n_s)]
    n_batches = 1 + seed % 3
    cuts = [[0] + sorted(int(x) for x in rng.integers(0, len(f) + 1, n_batches - 1)) + [len(f)] for f in sessions]
    state = np.zeros(n_s, dtype=STATE_DTYPE)
    passed = [0] * n_s
    failed = [None] * n_s
    for b in range(n_batches):
        parts = [sessions[s][cuts[s][b]:cuts[s][b + 1]] for s in range(n_s)]
        desc, sf, payload = _plain_batch(parts, rng)
        res = ctx.validate_host(desc, sf, payload, state)
        for s in range(n_s):
            if failed[s] is not None:
                continue
            passed[s] += int(res[s]["n_delivered"])
            if res[s]["error"]:
                assert int(res[s]["error"]) == 14 and int(res[s]["close_code"]) == 1007
                failed[s] = passed[s]
    for s in range(n_s):
        v = oracle.Validator()
        exp_fail = None
        for i, (op, fin, p) in enumerate(sessions[s]):
            if not v.decode(op, fin, p):
                exp_fail = i
                break
        assert failed[s] == exp_fail, (seed, s)
        if exp_fail is None:
            assert passed[s] == len(sessions[s]), (seed, s)


def _check_sessions(ctx, oracle, rng, sessions, n_batches, aligned=False):
    from snf4j_amd._lib import STATE_DTYPE
    n_s = len(sessions)
    cuts = [[0] + sorted(int(x) for x in rng.integers(0, len(f) + 1, n_batches - 1)) + [len(f)] for f in sessions]
    state = np.zeros(n_s, dtype=STATE_DTYPE)
    passed = [0] * n_s
    failed = [None] * n_s
    for b in range(n_batches):
        parts = [sessions[s][cuts[s][b]:cuts[s][b + 1]] for s in range(n_s)]
        desc, sf, payload = _plain_batch(parts, rng, aligned)
        res = ctx.validate_host(desc, sf, payload, state)
        for s in range(n_s):
            if failed[s] is not None:
                continue
            passed[s] += int(res[s]["n_delivered"])
            if res[s]["error"]:
                assert int(res[s]["error"]) == 14 and int(res[s]["close_code"]) == 1007
                failed[s] = passed[s]
    for s in range(n_s):
        v = oracle.Validator()
        exp_fail = None
        for i, (op, fin, p) in enumerate(sessions[s]):
            if not v.decode(op, fin, p):
                exp_fail = i
                break
        assert failed[s] == exp_fail, s
        if exp_fail is None:
            assert passed[s] == len(sessions[s]), s


@pytest.mark.parametrize("seed,aligned", [(0, False), (1, True), (2, False), (3, True)])
def test_validate_large_frames(ctx, oracle, seed, aligned):
    """Frames of 1-40 KiB, so that whole 4 KiB groups of pieces take the
    lane-contiguous validate path: invalid sequences planted anywhere (piece and
    lane boundaries, the last bytes, the first bytes of a continuation), code
    points cut by fragment ends, 16-B aligned and unaligned payload offsets."""
    rng = np.random.default_rng(4200 + seed)
    sessions = []
    for _ in range(int(rng.integers(20, 60))):
        frames = []
        for _ in range(int(rng.integers(1, 5))):
            body = wsgen.rand_text(rng, int(rng.integers(400, 16000)))
            if rng.random() < 0.3:
                bad = wsgen.BAD_UTF8[int(rng.integers(0, len(wsgen.BAD_UTF8)))]
                r = rng.random()
                at = (len(body) if r < 0.2 else int(rng.integers(0, 3)) if r < 0.3
                      else (int(rng.integers(1, max(2, len(body) // 1024))) * 1024 + int(rng.integers(-3, 4))) if r < 0.6
                      else int(rng.integers(0, len(body) + 1)))
                at = max(0, min(len(body), at))
                body = body[:at] + bad + body[at:]
            if rng.random() < 0.15 and len(body) > 1:  # truncated last code point: fails at FIN
                body = body[:-1]
            cuts = sorted(int(x) for x in rng.integers(0, len(body) + 1, int(rng.integers(0, 3))))
            pieces = [body[a:b] for a, b in zip([0] + cuts, cuts + [len(body)])]
            for i, pc in enumerate(pieces):
                frames.append((1 if i == 0 else 0, i == len(pieces) - 1, pc))
        sessions.append(frames)
    _check_sessions(ctx, oracle, rng, sessions, 1 + seed % 2, aligned)


_SNIPS = [b"", b"a", b"ab", b"\xdf", b"\xbf", b"\xdf\xbf", b"\xdf\xdf", b"\xe2", b"\x82", b"\xac", b"\xe2\x82",
          b"\x82\xac", b"\xe2\x82\xac", b"\xf0\x9f", b"\x98\x80", b"\xed\xa0", b"\xc0\xaf", b"\xff", b"hello "]


def _arbitrary_frames(rng, n):
    """(opcode, fin, payload) in ANY order, decoder-illegal ones included: TEXT
    inside an open text message (FrameUtf8Validator continues the context), BINARY
    between fragments (leaves it alone), CONTINUATION with no open context (not
    validated), control frames anywhere."""
    out = []
    for _ in range(n):
        op = int(rng.choice([0, 0, 0, 1, 1, 1, 2, 2, 8, 9, 10]))
        fin = bool(rng.random() < 0.45)
        if rng.random() < 0.15:
            body = wsgen.rand_text(rng, int(rng.integers(0, 2500)))
            if rng.random() < 0.5 and len(body) > 2:  # cut a code point at either end
                body = body[int(rng.integers(0, 3)):len(body) - int(rng.integers(0, 3))]
        else:
            body = b"".join(_SNIPS[int(i)] for i in rng.integers(0, len(_SNIPS), int(rng.integers(0, 4))))
        out.append((op, fin, body))
    return out


def _check_cut(ctx, oracle, rng, sessions, cuts, aligned=False):
    """Batches b = frames [cuts[s][b], cuts[s][b+1]) of every session; every
    session's first failure (frame index) and delivered count vs the oracle."""
    from snf4j_amd._lib import STATE_DTYPE
    n_s = len(sessions)
    n_batches = len(cuts[0]) - 1
    state = np.zeros(n_s, dtype=STATE_DTYPE)
    passed, failed = [0] * n_s, [None] * n_s
    for b in range(n_batches):
        parts = [sessions[s][cuts[s][b]:cuts[s][b + 1]] for s in range(n_s)]
        desc, sf, payload = _plain_batch(parts, rng, aligned)
        res = ctx.validate_host(desc, sf, payload, state)
        for s in range(n_s):
            if failed[s] is not None:
                continue
            passed[s] += int(res[s]["n_delivered"])
            if res[s]["error"]:
                assert int(res[s]["error"]) == 14 and int(res[s]["close_code"]) == 1007
                failed[s] = passed[s]
    for s in range(n_s):
        v = oracle.Validator()
        exp_fail = None
        for i, (op, fin, p) in enumerate(sessions[s]):
            if not v.decode(op, fin, p):
                exp_fail = i
                break
        assert failed[s] == exp_fail, (s, sessions[s][: (exp_fail or failed[s] or 0) + 1])
        if exp_fail is None:
            assert passed[s] == len(sessions[s]), s


def test_validate_context_rule_counterexample(ctx, oracle):
    """TEXT(fin=0, DF), BINARY(fin=1), CONTINUATION(fin=1, DF DF): the BINARY frame
    leaves the open context alone, so the continuation is validated and fails 1007
    (FrameUtf8Validator.java:63-75); and TEXT(fin=0, E2 82), TEXT(fin=1, AC): the
    second TEXT continues the context and passes."""
    cases = [
        [(1, False, b"\xdf"), (2, True, b"\x00\xff"), (0, True, b"\xdf\xdf")],   # fails at 2
        [(1, False, b"\xe2\x82"), (1, True, b"\xac")],                           # passes
        [(1, False, b"\xe2\x82"), (1, True, b"\xe2\x82\xac")],                   # fails at 1
        [(0, False, b"\xdf"), (1, True, b"ok")],                                 # cont not validated
        [(1, True, b"a"), (0, True, b"\xff")],                                   # closed: not validated
        [(1, False, b""), (9, True, b"p"), (1, False, b"\xf0"), (2, False, b"\xff"), (0, True, b"\x9f\x98\x80")],
    ]
    rng = np.random.default_rng(7)
    # one frame per batch (the carry crosses every boundary), and each session whole
    per_frame = [list(range(len(c) + 1)) for c in cases]
    m = max(len(c) for c in per_frame)
    per_frame = [c + [c[-1]] * (m - len(c)) for c in per_frame]
    _check_cut(ctx, oracle, rng, cases, per_frame)
    _check_cut(ctx, oracle, rng, cases, [[0, len(c)] for c in cases])
    v = oracle.Validator()
    assert [v.decode(*f) for f in cases[0]] == [True, True, False]


@pytest.mark.parametrize("seed", range(8))
def test_validate_arbitrary_opcode_orders(ctx, oracle, seed):
    """Arbitrary opcode/FIN orders vs or_validator_decode: one frame per batch, one
    batch, and random multi-frame batches."""
    rng = np.random.default_rng(31000 + seed)
    n_s = int(rng.integers(1, 200))
    sessions = [_arbitrary_frames(rng, int(rng.integers(0, 24))) for _ in range(n_s)]
    if seed % 3 == 0:
        m = max(len(f) for f in sessions)
        cuts = [[min(i, len(f)) for i in range(m + 1)] for f in sessions]
    elif seed % 3 == 1:
        cuts = [[0, len(f)] for f in sessions]
    else:
        nb = 2 + seed % 4
        cuts = [[0] + sorted(int(x) for x in rng.integers(0, len(f) + 1, nb - 1)) + [len(f)] for f in sessions]
    _check_cut(ctx, oracle, rng, sessions, cuts, aligned=seed % 2 == 1)


def test_validate_arbitrary_orders_many_blocks(ctx, oracle):
    """> 256 frames per block boundary and thousands of sessions, so the context
    function composes across the block aggregates (the k_vlink fold)."""
    rng = np.random.default_rng(4711)
    sessions = [_arbitrary_frames(rng, int(rng.integers(0, 40))) for _ in range(3000)]
    cuts = [[0] + sorted(int(x) for x in rng.integers(0, len(f) + 1, 2)) + [len(f)] for f in sessions]
    _check_cut(ctx, oracle, rng, sessions, cuts)


def _long_valid_session(rng, n, bad_at=None):
    """n frames in arbitrary-but-valid orders: the generator tracks the reference's
    context, so TEXT frames continue open contexts, a code point is split across
    the validated frames of a context (BINARY and pings between them), orphan
    CONTINUATIONs carry invalid bytes that must not be validated.  bad_at: a
    validated frame there gets an invalid byte."""
    out, is_open, split = [], False, False
    r = rng.random(n)
    for k in range(n):
        x = r[k]
        if x < 0.08:
            out.append((2, bool(x < 0.04), b"\xff\x80"))
            continue
        if x < 0.12:
            out.append((9, True, b"\xc3"))
            continue
        if not is_open and x < 0.25:
            out.append((0, bool(x < 0.18), b"\xa9\xff"))  # orphan: not validated
            continue
        op = 1 if (not is_open or x < 0.45) else 0
        fin = bool(rng.random() < 0.3)
        body = b"\xa9" if split else b""
        split = False
        if fin:
            body += b"a" if x < 0.7 else b"\xe2\x82\xac"
        else:
            body += b"" if x < 0.5 else (b"\xc3" if x < 0.8 else b"b")
            split = body.endswith(b"\xc3")
        if k == bad_at:
            body = b"\xff" + body
        out.append((op, fin, body))
        is_open = not fin
    return out


def test_validate_arbitrary_orders_multi_chunk(ctx, oracle):
    """More than 4096 x 256 frames in one batch: the k_scan<VAgg> chunk path, with
    the context (open state and split code points) composed across blocks and
    chunks; one session fails late, where the oracle says."""
    from snf4j_amd._lib import DESC_DTYPE, STATE_DTYPE
    rng = np.random.default_rng(99)
    n_s, per = 4, 300_000
    sessions = [_long_valid_session(rng, per, bad_at=(per - 1000 if s == 2 else None)) for s in range(n_s)]
    flat = [f for fr in sessions for f in fr]
    n = len(flat)
    lens = np.array([len(p) for _, _, p in flat], np.int64)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(lens)
    payload = np.frombuffer(b"".join(p for _, _, p in flat) + bytes(32), np.uint8).copy()
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["payload_off"], desc["payload_len"] = off[:-1], lens
    desc["opcode"] = [op for op, _, _ in flat]
    desc["flags"] = [0x80 if fin else 0 for _, fin, _ in flat]
    sf = (np.arange(n_s + 1) * per).astype(np.uint32)
    state = np.zeros(n_s, dtype=STATE_DTYPE)
    res = ctx.validate_host(desc, sf, payload, state)
    for s in range(n_s):
        v = oracle.Validator()
        exp = None
        for i, f in enumerate(sessions[s]):
            if not v.decode(*f):
                exp = i
                break
        got = int(res[s]["n_delivered"]) if res[s]["error"] else None
        assert got == exp, s
        assert (exp is None) == (s != 2)
