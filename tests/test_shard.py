"""Multi-GPU path on the CPU: sessions sharded over ranks (snf4j_amd/shard.py),
world_size-2 gloo (per-session state, no data-path collective).

Per rank the shard is decoded by the oracle (the GPU is not available here); the
test checks that the union of per-rank results equals the single-process decode
of the whole batch, that shards partition the sessions, and that the timed
region reports the max over ranks."""
from __future__ import annotations

import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import pyoracle
from snf4j_amd.shard import ShardPlan, assign_by_bytes, contiguous_shard, rank_seed, time_steps
from tests.wsgen import INJECT_KINDS, make_batch, session_frames


def _batch(seed=7, n_sessions=24):
    rng = np.random.default_rng(seed)
    sess = []
    for s in range(n_sessions):
        inject = INJECT_KINDS[s % len(INJECT_KINDS)] if s % 3 == 0 else None
        sess.append(session_frames(rng, int(rng.integers(0, 12)), inject=inject))
    return make_batch(sess)


def _decode_by_session(wire, off, sf):
    """{session index: (result row, [(opcode, flags, status, payload bytes)])} via the oracle."""
    payload, desc, res = pyoracle.Batch(False, False, 65536, True, len(sf) - 1).decode(wire, off, sf)
    out = []
    for s in range(len(sf) - 1):
        frames = []
        for k in range(int(sf[s]), int(sf[s + 1])):
            d = desc[k]
            o, n = int(d["payload_off"]), int(d["payload_len"])
            frames.append((int(d["opcode"]), int(d["flags"]), int(d["status"]), payload[o:o + n].tobytes()))
        r = res[s]
        out.append(((int(r["n_delivered"]), int(r["error"]), int(r["close_code"]), int(r["detail"])), frames))
    return out


def test_contiguous_shard_partitions():
    for n in (0, 1, 7, 1024, 1025):
        for w in (1, 2, 3, 8):
            spans = [contiguous_shard(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_assign_by_bytes_balanced():
    rng = np.random.default_rng(3)
    sb = rng.integers(64, 65536, 1000)
    owner = assign_by_bytes(sb, 8)
    loads = np.bincount(owner, weights=sb, minlength=8)
    assert loads.max() - loads.min() <= sb.max()  # greedy LPT bound
    assert set(owner.tolist()) == set(range(8))
    assert rank_seed(0x5EED, 0) == 0x5EED and rank_seed(0x5EED, 1) != rank_seed(0x5EED, 2)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_local_batches_reassemble(world):
    wire, off, sf = _batch()
    full = _decode_by_session(wire, off, sf)
    plan = ShardPlan.by_bytes(off, sf, world)
    seen = []
    for r in range(world):
        lw, loff, lsf, sids = plan.local_batch(r, wire, off, sf)
        assert int(loff[-1]) == lw.size
        part = _decode_by_session(lw, loff, lsf)
        for i, s in enumerate(sids):
            assert part[i] == full[s], f"session {s} differs on rank {r}"
        seen.extend(sids.tolist())
    assert sorted(seen) == list(range(len(sf) - 1))


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wire, off, sf = _batch(seed=11, n_sessions=30)
        plan = ShardPlan.by_bytes(off, sf, world)
        lw, loff, lsf, sids = plan.local_batch(rank, wire, off, sf)
        # the data path: only this rank's sessions, no collective
        mine = _decode_by_session(lw, loff, lsf)
        # timing contract: barrier + sync around the steps, max over ranks
        elapsed = time_steps(lambda: time.sleep(0.05 * (rank + 1)), 2, sync=lambda: None, dist=dist)
        # verification only (test side): gather every shard's verdicts on rank 0
        got = [None] * world
        dist.all_gather_object(got, (sids.tolist(), mine))
        if rank == 0:
            full = _decode_by_session(wire, off, sf)
            merged = {}
            for s_list, res in got:
                for s, v in zip(s_list, res):
                    merged[s] = v
            ok = sorted(merged) == list(range(len(sf) - 1)) and all(merged[s] == full[s] for s in merged)
            q.put((ok, elapsed))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_decode():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, elapsed = q.get(timeout=5)
    assert ok, "sharded decode differs from the single-process decode"
    assert elapsed >= 0.2 - 1e-3  # rank 1's 2 x 0.1 s dominates: max over ranks


def test_native_loop_device_policy():
    """wsg_device_for_loop (the JNI shim's WsgDevices): a new selector loop goes to
    the device with the fewest loops, ties to the fewest wire bytes accounted; a
    loop keeps its device; a released loop frees its share."""
    from snf4j_amd._lib import lib
    assert lib.wsg_device_policy_init(8) == 0
    devs = [lib.wsg_device_for_loop(100 + i) for i in range(8)]
    assert sorted(devs) == list(range(8))
    assert [lib.wsg_device_for_loop(100 + i) for i in range(8)] == devs  # stable
    # bytes break the ties of the second round: the least loaded devices first
    for d in range(8):
        assert lib.wsg_device_account(d, (8 - d) * 1000) == 0
    second = [lib.wsg_device_for_loop(200 + i) for i in range(8)]
    assert second == list(range(7, -1, -1))
    # a released loop's device takes the next loop
    assert lib.wsg_device_release_loop(100 + devs.index(3)) == 0
    assert lib.wsg_device_for_loop(999) == 3
    assert lib.wsg_device_release_loop(12345) != 0
    assert lib.wsg_device_account(8, 1) != 0
