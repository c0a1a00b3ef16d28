"""GPU parity of FrameAggregator (aggregate.hip) against the oracle's restatement
(FrameAggregator.java:72-104) and the reference's own test vectors."""
import numpy as np
import pytest

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


class _Session:
    def __init__(self):
        self.msgs = []

    def writenf(self, frame):
        self.msgs.append(frame)


def test_aggregator_kat_through_gpu(ctx):
    """FrameAggregatorTest :48-139 and WebSocketSessionTest :1334-1365 through the
    GPU FrameAggregator, one frame per batch (every fragment crosses a batch)."""
    from snf4j_amd import AggregatedBinaryFrame, AggregatedTextFrame, FrameAggregator, InvalidFrameException
    from snf4j_amd.frame import make_frame
    for seq in fixtures.load("aggregator"):
        agg = FrameAggregator(seq["max"], ctx=ctx)
        sess = _Session()
        for i, f in enumerate(seq["frames"]):
            exp = f["expect"]
            fr = make_frame(f["opcode"], f["fin"], f["rsv"], fixtures.unhex(f["payload"]))
            out = []
            if "error" in exp:
                with pytest.raises(InvalidFrameException) as ei:
                    agg.decode(sess, fr, out)
                assert ei.value.getMessage() == exp["error"], (seq["src"], i)
                assert sess.msgs and sess.msgs[-1].getStatus() == exp["close_code"]
                break
            agg.decode(sess, fr, out)
            assert len(out) == len(exp["out"]), (seq["src"], i)
            for g, o in zip(out, exp["out"]):
                if o["passthrough"]:
                    assert g is fr, (seq["src"], i)  # the reference asserts f == out.get(0)
                else:
                    assert isinstance(g, AggregatedTextFrame if o["opcode"] == 1 else AggregatedBinaryFrame)
                    assert (int(g.getOpcode()), g.isFinalFragment(), g.getRsvBits(), g.getPayload()) == \
                           (o["opcode"], True, o["rsv"], fixtures.unhex(o["payload"])), (seq["src"], i)
        assert not sess.msgs or "error" in seq["frames"][-1]["expect"]


def _batch(parts, truncate=None):
    """Decoded-batch arrays (as wsg_decode_batch_host returns them) from per-session
    frame lists [(opcode, fin, rsv, payload)]: 16-B aligned payload slots."""
    from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE
    n = sum(len(p) for p in parts)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    res = np.zeros(len(parts), dtype=RESULT_DTYPE)
    sf = [0]
    chunks, pos, k = [], 0, 0
    for s, fr in enumerate(parts):
        for (op, fin, rsv, p) in fr:
            desc[k]["payload_off"] = pos
            desc[k]["payload_len"] = len(p)
            desc[k]["opcode"] = op
            desc[k]["flags"] = (0x80 if fin else 0) | (rsv << 4) | 1
            slot = (len(p) + 15) & ~15
            chunks.append(p + bytes(slot - len(p)))
            pos += slot
            k += 1
        sf.append(k)
        res[s]["n_delivered"] = len(fr) if truncate is None else min(len(fr), truncate[s])
    payload = np.frombuffer(b"".join(chunks) + bytes(16), dtype=np.uint8).copy()
    return desc, np.array(sf, np.uint32), res, payload


def _rand_session(rng, n, big):
    out = []
    for _ in range(n):
        r = rng.random()
        op = 0 if r < 0.45 else 1 if r < 0.62 else 2 if r < 0.8 else int(rng.choice([8, 9, 10]))
        fin = op >= 8 or bool(rng.random() < 0.4)  # a control Frame is always final (ControlFrame.java:44-49)
        ln = int(rng.integers(0, 126)) if op >= 8 else int(rng.choice(
            [0, int(rng.integers(1, 40)), int(rng.integers(40, 600)), int(rng.integers(600, 5000))] +
            ([int(rng.integers(5000, 70000))] if big else [])))
        if op == 8 and ln == 1:
            ln = 2  # a CloseFrame cannot hold 1 byte (CloseFrame.java:158-163)
        out.append((op, fin, int(rng.integers(0, 8)), rng.integers(0, 256, ln, dtype=np.uint8).tobytes()))
    return out


@pytest.mark.parametrize("fold", [True, False])
@pytest.mark.parametrize("seed", range(6))
def test_aggregate_random_batches(ctx, oracle, seed, fold):
    """Arbitrary frame sequences (also ones a decoder would reject: continuations
    outside a message pass through, a new start replaces an open message), split
    over several batches with the carry, vs the oracle fed the same frames.  fold=False
    forces the plan's k_agg_scan path (WSG_TUNE_AGG_FOLD_MAX 0), which the default
    takes only above 3,072 blocks (1.5 M frames)."""
    from snf4j_amd import BatchAggregator
    ctx.set_tuning("agg_fold_max", 1 << 30 if fold else 0)
    try:
        _random_batches(ctx, oracle, seed)
    finally:
        ctx.set_tuning("agg_fold_max", 1 << 30)


def _random_batches(ctx, oracle, seed):
    from snf4j_amd import BatchAggregator
    rng = np.random.default_rng(500 + seed)
    n_s = int(rng.integers(1, 90))
    max_len = [100, 3000, 1 << 20][seed % 3]
    sessions = [_rand_session(rng, int(rng.integers(0, 40)), big=seed >= 3) for _ in range(n_s)]
    n_batches = 1 + seed % 4
    cuts = [[0] + sorted(int(x) for x in rng.integers(0, len(f) + 1, n_batches - 1)) + [len(f)] for f in sessions]
    gpu = BatchAggregator(n_s, max_len, ctx=ctx)
    got = [[] for _ in range(n_s)]
    err = [None] * n_s
    for b in range(n_batches):
        parts = [sessions[s][cuts[s][b]:cuts[s][b + 1]] if err[s] is None else [] for s in range(n_s)]
        desc, sf, res, payload = _batch(parts)
        for s, (frames, exc) in enumerate(gpu.run(desc, sf, res, payload)):
            got[s] += frames
            if exc is not None and err[s] is None:
                err[s] = (cuts[s][b] + exc.frame_index, str(exc), exc.close_code)
    for s in range(n_s):
        agg = oracle.Aggregator(max_len)
        exp, e = [], None
        for i, (op, fin, rsv, p) in enumerate(sessions[s]):
            try:
                f = agg.decode(op, fin, rsv, p)
            except oracle.InvalidFrame as ex:
                e = (i, str(ex), ex.close_code)
                break
            if f is not None:
                exp.append((f, op))
        assert err[s] == e, (seed, s)
        assert len(got[s]) == len(exp), (seed, s)
        for g, (o, in_op) in zip(got[s], exp):
            assert (int(g.getOpcode()), g.isFinalFragment(), g.getRsvBits()) == (o.opcode, o.fin, o.rsv), (seed, s)
            assert g.getPayload() == o.payload, (seed, s)
            aggregated = in_op == 0 and o.opcode in (1, 2)
            assert aggregated == hasattr(g, "getFragments"), (seed, s)


def test_aggregate_truncated_sessions(ctx, oracle):
    """Only the frames the decoder delivered are aggregated (dec_result.n_delivered)."""
    from snf4j_amd import BatchAggregator
    rng = np.random.default_rng(77)
    sessions = [_rand_session(rng, 30, big=True) for _ in range(40)]
    trunc = [int(rng.integers(0, 31)) for _ in sessions]
    desc, sf, res, payload = _batch(sessions, trunc)
    out = BatchAggregator(len(sessions), 1 << 20, ctx=ctx).run(desc, sf, res, payload)
    for s, (frames, exc) in enumerate(out):
        agg = oracle.Aggregator(1 << 20)
        exp = [f for f in (agg.decode(*fr) for fr in sessions[s][:trunc[s]]) if f is not None]
        assert exc is None and len(frames) == len(exp), s
        for g, o in zip(frames, exp):
            assert g.getPayload() == o.payload and int(g.getOpcode()) == o.opcode, s


def test_aggregate_multi_pass_block_scan(ctx, oracle):
    """1.1 M tiny frames: 2,150 plan blocks of 512, folded by k_agg_b / k_agg_c (the
    default up to 3,072 blocks) and through k_agg_scan, which then carries its scans
    across passes of 1,024 (forced): every session's output against the oracle."""
    from snf4j_amd import BatchAggregator
    rng = np.random.default_rng(4097)
    n_s, per = 128, 8600
    ops = rng.choice([0, 0, 1, 2, 9], size=(n_s, per))
    fins = rng.random((n_s, per)) < 0.35
    lens = rng.integers(0, 4, size=(n_s, per))
    sessions = []
    for s in range(n_s):
        fr = []
        for i in range(per):
            op = int(ops[s, i])
            fr.append((op, True if op >= 8 else bool(fins[s, i]), 0, bytes([i & 255]) * int(lens[s, i])))
        sessions.append(fr)
    desc, sf, res, payload = _batch(sessions)
    assert len(desc) > 4096 * 256
    for fold in (True, False):  # 2,150 blocks of 512: folded by default, k_agg_scan forced
        ctx.set_tuning("agg_fold_max", 1 << 30 if fold else 0)
        try:
            out = BatchAggregator(n_s, 1 << 20, ctx=ctx).run(desc, sf, res, payload)
        finally:
            ctx.set_tuning("agg_fold_max", 1 << 30)
        _check_multi(oracle, sessions, out)


def _check_multi(oracle, sessions, out):
    for s, (frames, exc) in enumerate(out):
        agg = oracle.Aggregator(1 << 20)
        exp = [f for f in (agg.decode(*fr) for fr in sessions[s]) if f is not None]
        assert exc is None and len(frames) == len(exp), s
        for g, o in zip(frames, exp):
            assert g.getPayload() == o.payload and int(g.getOpcode()) == o.opcode, s
