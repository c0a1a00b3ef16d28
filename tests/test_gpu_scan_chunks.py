"""GPU parity of the multi-chunk scan path: a batch of more than SCAN_CHUNK x DBLOCK
(4096 x 256) frames is scanned by several k_scan workgroups, and k_link folds the
chunk totals in order.  The frames are tiny fragments (0-3 payload bytes) of long
TEXT messages with pings between them, so the UTF-8 carry (the last <= 3 message
bytes, FrameUtf8Validator.java:59-98) crosses frame, block and chunk boundaries, and
two batches carry the session tails across the batch seam.  Checked frame by frame
against the oracle."""
import numpy as np
import pytest

from tests.test_gpu_mixed import compare_vec

pytestmark = pytest.mark.gpu


def _session_frames(rng, n_frames, bad_at=None):
    """(opcode, fin, payload bytes) arrays of one session: one TEXT message cut into
    n_frames fragments of 0-3 bytes with pings in between, the code points split at
    arbitrary bytes."""
    lens = rng.integers(0, 4, n_frames)
    target = int(lens[:-1].sum())
    # code points until their bytes reach the target; the final fragment takes the rest (0-3 bytes)
    cps = rng.choice(np.array([0x41, 0x7A, 0xE9, 0x20AC, 0x4E2D, 0x1F600]), size=target + 1)
    nb = np.where(cps < 0x80, 1, np.where(cps < 0x800, 2, np.where(cps < 0x10000, 3, 4)))
    m = int(np.searchsorted(np.cumsum(nb), target)) + 1
    body = np.frombuffer("".join(map(chr, cps[:m])).encode(), np.uint8).copy()
    lens[-1] = len(body) - target
    assert 0 <= lens[-1] <= 3
    if bad_at is not None:
        body[int(bad_at * len(body))] = 0xFF
    op = np.zeros(n_frames, np.uint8)
    op[0] = 1
    fin = np.zeros(n_frames, bool)
    fin[-1] = True
    pings = rng.random(n_frames) < 0.05
    pings[0] = pings[-1] = False
    # a ping is a frame of its own before the fragment
    n = n_frames + int(pings.sum())
    o_op = np.full(n, 9, np.uint8)
    o_fin = np.ones(n, bool)
    o_len = np.zeros(n, np.int64)
    pos = np.arange(n_frames) + np.cumsum(pings)
    o_op[pos], o_fin[pos], o_len[pos] = op, fin, lens
    o_src = np.zeros(n, np.int64)
    o_src[pos] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    return o_op, o_fin, o_len, o_src, body


def _wire(parts):
    """Unmasked frames (client mode) of the sessions' (op, fin, len, src, body) lists."""
    ops, fins, lens, bodies, src = [], [], [], [], []
    base = 0
    for op, fin, ln, sr, body in parts:
        ops.append(op), fins.append(fin), lens.append(ln), src.append(sr + base), bodies.append(body)
        base += len(body)
    op, fin, ln, sr = (np.concatenate(x) for x in (ops, fins, lens, src))
    body = np.concatenate(bodies)
    flen = 2 + ln
    off = np.zeros(len(op) + 1, np.uint64)
    off[1:] = np.cumsum(flen)
    wire = np.zeros(int(off[-1]), np.uint8)
    o = off[:-1].astype(np.int64)
    wire[o] = (fin.astype(np.uint8) << 7) | op
    wire[o + 1] = ln.astype(np.uint8)
    # payload bytes: frame k's bytes body[sr[k] : sr[k] + ln[k]] at o[k] + 2
    idx = np.repeat(np.arange(len(op)), ln)
    within = np.arange(int(ln.sum())) - np.repeat(np.cumsum(ln) - ln, ln)
    wire[o[idx] + 2 + within] = body[sr[idx] + within]
    return wire, off


def test_multi_chunk_scan_tiny_fragments(oracle):
    from snf4j_amd import Context, decoder_cfg
    from snf4j_amd._lib import STATE_DTYPE

    rng = np.random.default_rng(77)
    n_s = 5
    per = 500_000  # 5 x ~525 K frames in 2 batches: each > 4096 x 256, so k_scan runs 2 workgroups
    sessions = [_session_frames(rng, per, bad_at=(0.9 if s == n_s - 1 else None)) for s in range(n_s)]
    # two batches: every session's frames cut at its own point
    cuts = [int(rng.integers(len(op) // 3, 2 * len(op) // 3)) for op, *_ in sessions]
    state = np.zeros(n_s, dtype=STATE_DTYPE)
    ob = oracle.Batch(True, False, 65536, True, n_s)
    ctx = Context(0)
    try:
        total = 0
        for b in range(2):
            parts, counts = [], []
            for (op, fin, ln, sr, body), c in zip(sessions, cuts):
                sl = slice(0, c) if b == 0 else slice(c, len(op))
                parts.append((op[sl], fin[sl], ln[sl], sr[sl], body))
                counts.append(len(op[sl]))
            wire, off = _wire(parts)
            sf = np.zeros(n_s + 1, np.uint32)
            sf[1:] = np.cumsum(counts)
            total += int(sf[-1])
            gpu = ctx.decode_host(decoder_cfg(True, False, 65536, True), wire, off, sf, state)
            ora = ob.decode(wire, off, sf)
            compare_vec(gpu, [(0, n_s, ora)], sf, f"chunks batch {b}")
            assert int(sf[-1]) > 4096 * 256
        # the session with the invalid byte (in the second batch) fails with 1007
        assert int(gpu[2]["error"][n_s - 1]) == 14 and (gpu[2]["error"][:n_s - 1] == 0).all()
    finally:
        ctx.close()
