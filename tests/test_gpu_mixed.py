"""GPU parity on the mixed configuration (BASELINE configs[2]): log-uniform 64 B-64 KiB
text+binary messages, fragmented at arbitrary bytes (code points split across
fragments), injected invalid UTF-8; bytes generated on the device by wsg_synth_frames,
decoded on the device, checked frame by frame against the oracle."""
import numpy as np
import pytest

import benchsupport

from tests.test_gpu_decode import compare

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,sessions,mib,bad", [(1, 64, 24, 0.05), (2, 7, 8, 0.0), (3, 256, 32, 0.01)])
def test_mixed_batch_parity(oracle, seed, sessions, mib, bad):
    import torch

    from snf4j_amd import Context, decoder_cfg
    from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE, STATE_DTYPE, lib
    from benchsupport.synth import mixed_plan

    t, off, sf, wl, info = mixed_plan(seed, sessions, mib << 20, bad_frac=bad, frag_frac=0.2)
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    try:
        tab = torch.from_numpy(t.view(np.uint8).copy()).to(dev)
        wire = torch.zeros(wl + 64, dtype=torch.uint8, device=dev)
        benchsupport.synth_frames(ctx, tab, wire)
        n, n_s = len(t), len(sf) - 1
        cap = int(lib.wsg_decode_payload_bound(wl, n))
        payload = torch.empty(cap, dtype=torch.uint8, device=dev)
        desc = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        res = torch.empty(n_s * 16, dtype=torch.uint8, device=dev)
        state = torch.zeros(n_s * 8, dtype=torch.uint8, device=dev)
        ctx.decode_device(decoder_cfg(False, False, 65536, True), wire, torch.from_numpy(off.astype(np.int64)).to(dev),
                          torch.from_numpy(sf.astype(np.int32)).to(dev), state, payload, desc, res, wire_len=wl)
        torch.cuda.synchronize(dev)
        h_wire = wire[:wl].cpu().numpy()
        gpu = (payload.cpu().numpy(), desc.cpu().numpy().view(DESC_DTYPE), res.cpu().numpy().view(RESULT_DTYPE))
    finally:
        ctx.close()
    ora = oracle.Batch(False, False, 65536, True, n_s).decode(h_wire, off, sf)
    compare(gpu, ora, sf, f"mixed seed {seed}")
    # the generator: exactly the sessions holding an injected sequence fail, with 1007
    err = gpu[2]["error"]
    bad_s = set(info["bad_sessions"])
    for s in range(n_s):
        assert (int(err[s]) == 14) == (s in bad_s), s
        assert int(err[s]) in (0, 14)


def oracle_decode_groups(oracle, wire, off, sf, groups=8):
    """The oracle's decode of a batch, in `groups` independent session ranges run on
    host threads (ctypes releases the GIL; sessions are independent, so this is the
    same result as one Batch over all sessions).  Yields (s0, s1, (payload, desc, result))
    with payload offsets relative to the group."""
    import threading
    n_s = len(sf) - 1
    bounds = [round(i * n_s / groups) for i in range(groups + 1)]
    out = [None] * groups

    def run(g):
        s0, s1 = bounds[g], bounds[g + 1]
        f0, f1 = int(sf[s0]), int(sf[s1])
        b0 = int(off[f0])
        w = wire[b0:int(off[f1])]
        o = off[f0:f1 + 1].astype(np.uint64) - np.uint64(b0)
        s = (sf[s0:s1 + 1].astype(np.int64) - f0).astype(np.uint32)
        out[g] = (s0, s1, oracle.Batch(False, False, 65536, True, s1 - s0).decode(w, o, s))

    ts = [threading.Thread(target=run, args=(g,)) for g in range(groups)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


def compare_vec(gpu, groups, sf, tag=""):
    """compare() for large batches: results, descriptors and payload bytes of every
    delivered frame, vectorised per oracle session group."""
    gp, gd, gr = gpu
    n_checked = 0
    for s0, s1, (op, od, orr) in groups:
        g = gr[s0:s1]
        for f in ("n_delivered", "error", "close_code", "detail"):
            bad = np.nonzero(g[f] != orr[f])[0]
            assert bad.size == 0, (tag, f, s0 + int(bad[0]), g[bad[0]], orr[bad[0]])
        f0, f1 = int(sf[s0]), int(sf[s1])
        cnt = np.diff(sf[s0:s1 + 1].astype(np.int64))
        sess = np.repeat(np.arange(s1 - s0), cnt)
        idx = np.arange(f1 - f0) - (sf[s0:s1].astype(np.int64) - f0)[sess]
        deliv = np.nonzero(idx < g["n_delivered"].astype(np.int64)[sess])[0]
        a, b = gd[f0:f1][deliv], od[deliv]
        assert np.array_equal(a["opcode"], b["opcode"]), tag
        assert np.array_equal(a["flags"] & 0xF0, b["flags"] & 0xF0), tag
        assert np.array_equal(a["payload_len"], b["payload_len"]), tag
        assert (a["payload_off"] % 16 == 0).all(), tag
        ga_off, gl = a["payload_off"].astype(np.int64), a["payload_len"].astype(np.int64)
        ob_off = b["payload_off"].astype(np.int64)
        for c in range(0, len(deliv), 65536):  # payload bytes, 64 K frames at a time
            sl = slice(c, c + 65536)
            ga = np.concatenate([gp[o:o + n] for o, n in zip(ga_off[sl], gl[sl])] or [np.zeros(0, np.uint8)])
            ob = np.concatenate([op[o:o + n] for o, n in zip(ob_off[sl], gl[sl])] or [np.zeros(0, np.uint8)])
            assert np.array_equal(ga, ob), (tag, s0, c)
        n_checked += len(deliv)
    return n_checked


@pytest.mark.parametrize("bad", [0.01, 0.0], ids=["configs2_1pct_bad", "configs2_no_errors"])
def test_mixed_full_size_parity(oracle, bad):
    """BASELINE configs[2] at full size (>= 4 GiB of wire, 1024 sessions, the bench's
    plan): GPU decode vs the oracle, frame by frame.  With bad_frac = 0 no session
    closes early, so every frame of every session is compared."""
    import torch

    from snf4j_amd import Context, decoder_cfg
    from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE, lib
    from benchsupport.synth import mixed_plan

    t, off, sf, wl, info = mixed_plan(0xC0F3, 1024, 4 << 30, bad_frac=bad)
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    try:
        tab = torch.from_numpy(t.view(np.uint8).copy()).to(dev)
        wire = torch.zeros(wl + 64, dtype=torch.uint8, device=dev)
        benchsupport.synth_frames(ctx, tab, wire)
        del tab
        n, n_s = len(t), len(sf) - 1
        payload = torch.empty(int(lib.wsg_decode_payload_bound(wl, n)), dtype=torch.uint8, device=dev)
        desc = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        res = torch.empty(n_s * 16, dtype=torch.uint8, device=dev)
        state = torch.zeros(n_s * 8, dtype=torch.uint8, device=dev)
        ctx.decode_device(decoder_cfg(False, False, 65536, True), wire, torch.from_numpy(off.astype(np.int64)).to(dev),
                          torch.from_numpy(sf.astype(np.int32)).to(dev), state, payload, desc, res, wire_len=wl)
        torch.cuda.synchronize(dev)
        h_wire = wire[:wl].cpu().numpy()
        del wire
        gpu = (payload.cpu().numpy(), desc.cpu().numpy().view(DESC_DTYPE), res.cpu().numpy().view(RESULT_DTYPE))
        del payload
        torch.cuda.empty_cache()
    finally:
        ctx.close()
    assert wl >= 4 << 30
    groups = oracle_decode_groups(oracle, h_wire, off, sf)
    checked = compare_vec(gpu, groups, sf, f"configs[2] full size, bad {bad}")
    err = gpu[2]["error"]
    assert set(np.nonzero(err)[0].tolist()) == set(info["bad_sessions"])
    assert set(np.unique(err).tolist()) <= {0, 14}
    if bad == 0:
        assert checked == n  # every frame of every session delivered and compared
    print(f"configs[2] full size (bad {bad}): {n} frames, {wl} wire bytes, {checked} frames compared")
