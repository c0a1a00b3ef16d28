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
