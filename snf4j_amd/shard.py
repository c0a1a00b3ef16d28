"""Multi-GPU sharding of frame batches: sessions -> GPUs, one process per GPU.

All decoder and validator state is per session (FrameDecoder.java:43-63,
FrameUtf8Validator.java:42; one decoder per session, DefaultWebSocketSessionConfig.java:276-281),
so a node-wide batch splits into independent per-GPU batches of whole sessions
and no data moves between GPUs: the only cross-rank traffic is the timing
barrier/max.  Nothing here touches a GPU, so the logic is
tested with gloo on the CPU (tests/test_shard.py).
"""
from __future__ import annotations

import heapq
import time

import numpy as np


def rank_seed(seed: int, rank: int) -> int:
    """Synthetic-data seed of a rank's shard (bench.py): independent streams per rank."""
    return (int(seed) ^ (int(rank) * 0x1000003)) & 0xFFFFFFFFFFFFFFFF


def contiguous_shard(n_sessions: int, world: int, rank: int) -> tuple[int, int]:
    """Global sessions [lo, hi) of `rank` for uniform sessions (session_id blocks)."""
    q, r = divmod(int(n_sessions), int(world))
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def assign_by_bytes(session_bytes, world: int) -> np.ndarray:
    """Greedy byte-balanced assignment (largest session first to the least loaded
    GPU, ties to the lower rank).  Returns the rank of every session."""
    sb = np.asarray(session_bytes, dtype=np.int64)
    order = sorted(range(len(sb)), key=lambda i: (-int(sb[i]), i))
    heap = [(0, g) for g in range(world)]
    owner = np.zeros(len(sb), dtype=np.int32)
    for i in order:
        load, g = heapq.heappop(heap)
        owner[i] = g
        heapq.heappush(heap, (load + int(sb[i]), g))
    return owner


class ShardPlan:
    """Sessions of one node-wide batch split over `world` GPUs.  The batch layout
    is the C ABI's (include/wsgpu.h): wire bytes, frame_off[n_frames+1] (frames
    of a session contiguous), session_first[n_sessions+1]."""

    def __init__(self, owner: np.ndarray, world: int):
        self.owner = np.asarray(owner, dtype=np.int32)
        self.world = int(world)
        self.sessions = [np.nonzero(self.owner == g)[0] for g in range(self.world)]

    @classmethod
    def by_bytes(cls, frame_off, session_first, world: int) -> "ShardPlan":
        off = np.asarray(frame_off, dtype=np.int64)
        sf = np.asarray(session_first, dtype=np.int64)
        return cls(assign_by_bytes(off[sf[1:]] - off[sf[:-1]], world), world)

    @classmethod
    def contiguous(cls, n_sessions: int, world: int) -> "ShardPlan":
        owner = np.zeros(n_sessions, dtype=np.int32)
        for g in range(world):
            lo, hi = contiguous_shard(n_sessions, world, g)
            owner[lo:hi] = g
        return cls(owner, world)

    def local_batch(self, rank: int, wire, frame_off, session_first):
        """(wire, frame_off, session_first, global_session_ids) of rank's sessions,
        gathered on the host into one contiguous per-GPU batch."""
        wire = np.asarray(wire, dtype=np.uint8)
        off = np.asarray(frame_off, dtype=np.uint64)
        sf = np.asarray(session_first, dtype=np.uint32)
        sids = self.sessions[rank]
        parts, loff, lsf = [], [0], [0]
        pos = 0
        for s in sids:
            f0, f1 = int(sf[s]), int(sf[s + 1])
            a, b = int(off[f0]), int(off[f1])
            parts.append(wire[a:b])
            loff.extend(pos + (off[f0 + 1:f1 + 1].astype(np.int64) - a))
            pos += b - a
            lsf.append(lsf[-1] + (f1 - f0))
        lw = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        return lw, np.array(loff, dtype=np.uint64), np.array(lsf, dtype=np.uint32), sids

    def session_state(self, rank: int, state):
        """Rank-local view (copy) of the per-session carry state."""
        return np.ascontiguousarray(np.asarray(state)[self.sessions[rank]])


def time_steps(step, steps: int, sync=None, dist=None) -> float:
    """Time exactly `steps` calls of step(), bracketed by a barrier and a device
    sync on both sides; returns the max over ranks (bench.py contract)."""
    if dist is not None:
        dist.barrier()
    if sync:
        sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if sync:
        sync()
    # this rank's time ends at its own device sync; the barrier after it only lines
    # the ranks up (its latency is not work), and the max over ranks is the job time
    elapsed = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed
