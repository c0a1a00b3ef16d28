"""The selector-loop side of the drop-in: the scheduling of
java/org/snf4j/websocket/gpu/WsgBatcher.java over the native batchers, restated in
Python so that it runs here (there is no JDK in this image) — the same calls in the
same order, driven by the same kind of loop.

snf4j's loop (InternalSelectorLoop.java): one thread repeats select() -> the reads
of the ready sessions, each going through its decoder (StreamSession.java:798-854 ->
GpuFrameDecoder.decode -> LoopBatcher.enqueue) -> handleTasks (:641, :751-758),
which polls the task queue until it is empty, so a task queued while tasks run runs
in the same phase; executenf from another thread queues a task and wakes select()
(:990-1011, :1038-1046).

The batching on that loop:
- enqueue() only records a read; the first of an iteration schedules flush() with
  executenf, which runs after every read of the iteration;
- flush() feeds the iteration's reads with one wsg_batcher_feed_many, collects every
  earlier flush whose device work has finished (wsg_batcher_await with no wait),
  collects the oldest one blocking only when two are in flight, then queues this one
  (wsg_batcher_flush_async) and hands its ticket to the completion thread;
- the completion thread waits for the ticket (wsg_batcher_await) and re-enters the
  loop with executenf(collect_ready): the loop thread never waits on the device for a
  flush it queued in the same iteration, and a flush is delivered in a later
  iteration even when no further reads arrive;
- frames go to each session in flush order; a session's slot reset while a flush is
  in flight drops that flush's results for it (wsg_batcher_session_reset);
- the encode side is the same over wsg_enc_batcher_*; flush_encodes() (a CLOSE
  frame) first writes out everything in flight, then encodes what is queued now.
"""
from __future__ import annotations

import collections
import queue
import threading

from .codec import EncodeBatcher, NativeBatcher


class SelectorLoop:
    """The task side of InternalSelectorLoop: executenf queues (any thread) and wakes
    the selector; handle_tasks runs tasks until the queue is empty."""

    def __init__(self):
        self._tasks = collections.deque()
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self.iteration = 0

    def executenf(self, task):
        with self._lock:
            self._tasks.append(task)
        self._wake.set()

    def handle_tasks(self):
        while True:
            with self._lock:
                if not self._tasks:
                    return
                task = self._tasks.popleft()
            task()

    def select(self, timeout: float | None) -> bool:
        """Block until woken (executenf) or the timeout; True if woken."""
        woke = self._wake.wait(timeout)
        self._wake.clear()
        return woke

    def run_iteration(self, reads):
        """One loop iteration: the reads (callables, each a session's read -> decode),
        then the task phase."""
        self.iteration += 1
        for r in reads:
            r()
        self.handle_tasks()

    def has_tasks(self) -> bool:
        with self._lock:
            return bool(self._tasks)


class _Completion(threading.Thread):
    """Waits for the tickets it is given (await on the native batcher) and re-enters
    the loop with executenf(task) for each one that finished."""

    def __init__(self, loop: SelectorLoop, await_fn, task, name: str):
        super().__init__(name=name, daemon=True)
        self.loop, self.await_fn, self.task = loop, await_fn, task
        self.q: queue.Queue = queue.Queue()
        self.stop = False

    def watch(self, ticket: int):
        self.q.put(ticket)

    def run(self):
        while not self.stop:
            try:
                t = self.q.get(timeout=0.1)
            except queue.Empty:
                continue
            while not self.stop and self.await_fn(t - 1, 100) < t:
                pass
            if not self.stop:
                self.loop.executenf(self.task)

    def close(self):
        self.stop = True
        self.join()


class LoopBatcher:
    """WsgBatcher's decode side.  deliver(sid, frames, exc) is called on the loop
    thread, per session in flush order (frames as NativeBatcher returns them)."""

    def __init__(self, loop: SelectorLoop, n_sessions: int, deliver, ctx=None, clientMode: bool = False,
                 allowExtensions: bool = False, maxPayloadLen: int = 65536, validate_utf8: bool = True,
                 max_wire: int = 0, max_frames: int = 0, raw: bool = False):
        self.loop = loop
        self.nb = NativeBatcher(n_sessions, clientMode, allowExtensions, maxPayloadLen, validate_utf8, ctx=ctx)
        if max_wire:
            self.nb.reserve(max_wire, max_frames)
        self.deliver = deliver
        self.raw = raw  # deliver the raw views (sf, desc, payload, result, wire_bytes) once per flush
        self.n = n_sessions
        self._sids: list[int] = []
        self._data: list = []
        self.inflight: collections.deque = collections.deque()  # (ticket, loop iteration queued)
        self.flush_scheduled = False
        self.stats = {"flushes": 0, "collected_later": 0, "collected_blocking": 0, "max_inflight": 0}
        self._completion = _Completion(loop, self.nb.await_done, self.collect_ready, "wsg-completion")
        self._completion.start()

    # ---- the loop thread
    def enqueue(self, sid: int, data):
        """A session's read (GpuFrameDecoder.decode): recorded; the flush feeds it."""
        self._sids.append(int(sid))
        self._data.append(data)
        self.schedule()

    def enqueue_ptr(self, sid: int, ptr: int, length: int):
        """A read given as a host address and length (the bytes stay valid until the
        flush feeds them, as the Java side holds the ByteBuffer until then)."""
        self._sids.append(int(sid))
        self._data.append((int(ptr), int(length)))
        self.schedule()

    def enqueue_many_ptr(self, sids, ptrs, lens):
        """Many sessions' reads of one iteration at once (numpy arrays): what the
        iteration's enqueue() calls record, one at a time in Java (a few array stores
        each); recorded in bulk here so Python's per-call cost stays out of the bench."""
        self._sids.append(sids)
        self._data.append(("many", ptrs, lens))
        self.schedule()

    def reset_session(self, sid: int):
        """The session ended (unregister): its unfed reads are dropped, its slot reset."""
        keep = [i for i, s in enumerate(self._sids) if s != sid]
        self._sids = [self._sids[i] for i in keep]
        self._data = [self._data[i] for i in keep]
        self.nb.reset_session(sid)

    def schedule(self):
        if not self.flush_scheduled:
            self.flush_scheduled = True
            self.loop.executenf(self.flush)

    def flush(self):
        self.flush_scheduled = False
        if self._sids:  # one feed call for the iteration's reads
            if isinstance(self._data[0], tuple) and self._data[0][0] == "many":
                import numpy as np
                self.nb.feed_many_ptrs(np.concatenate(self._sids), np.concatenate([d[1] for d in self._data]),
                                       np.concatenate([d[2] for d in self._data]))
            elif isinstance(self._data[0], tuple):
                ptrs, lens = zip(*self._data)
                self.nb.feed_many_ptrs(self._sids, ptrs, lens)
            else:
                self.nb.feed_many(self._sids, self._data)
            self._sids, self._data = [], []
        self.collect_ready()
        if len(self.inflight) == 2:
            self._collect_oldest(blocking=True)
        self.nb.flush_async()
        t = self.nb.ticket()
        self.inflight.append((t, self.loop.iteration))
        self.stats["flushes"] += 1
        self.stats["max_inflight"] = max(self.stats["max_inflight"], len(self.inflight))
        self._completion.watch(t)

    def collect_ready(self):
        """Every in-flight flush whose device work has finished (no wait)."""
        if not self.inflight:
            return
        done = self.nb.await_done(0, 0)
        while self.inflight and self.inflight[0][0] <= done:
            self._collect_oldest(blocking=False)

    def _collect_oldest(self, blocking: bool):
        t, it = self.inflight.popleft()
        if self.loop.iteration > it:
            self.stats["collected_later"] += 1
        if blocking:
            self.stats["collected_blocking"] += 1
        if self.raw:
            self.deliver(None, self.nb.wait_raw(), None)
            return
        for sid, (frames, exc) in enumerate(self.nb.wait()):
            if frames or exc is not None:
                self.deliver(sid, frames, exc)

    def drain(self):
        while self.inflight:
            self._collect_oldest(blocking=True)

    def close(self):
        self._completion.close()
        self.drain()
        self.nb.close()


class LoopEncodeBatcher:
    """WsgBatcher's encode side: write(sid, wire bytes) on the loop thread."""

    def __init__(self, loop: SelectorLoop, n_sessions: int, write, clientMode: bool = True, ctx=None,
                 max_frames: int = 0, max_payload: int = 0):
        self.loop = loop
        self.eb = EncodeBatcher(n_sessions, clientMode, ctx=ctx)
        if max_frames:
            self.eb.reserve(max_frames, max_payload)
        self.write = write
        self.dirty = False
        self.inflight: collections.deque = collections.deque()
        self.flush_scheduled = False
        self._completion = _Completion(loop, self.eb.await_done, self.collect_ready, "wsg-enc-completion")
        self._completion.start()

    def enqueue(self, sid: int, frame, mask=(0, 0, 0, 0)):
        self.eb.add(sid, frame, mask)
        self.dirty = True
        self.schedule()

    def reset_session(self, sid: int):
        self.eb.reset_session(sid)

    def schedule(self):
        if not self.flush_scheduled:
            self.flush_scheduled = True
            self.loop.executenf(self.flush)

    def flush(self):
        self.flush_scheduled = False
        self.collect_ready()
        if not self.dirty:
            return
        if len(self.inflight) == 2:
            self._collect_oldest()
        self.eb.flush_async()
        self.dirty = False
        t = self.eb.ticket()
        self.inflight.append(t)
        self._completion.watch(t)

    def flush_encodes(self):
        """Before a CLOSE frame: everything in flight written, then what is queued."""
        while self.inflight:
            self._collect_oldest()
        if self.dirty:
            self._write(self.eb.flush())
            self.dirty = False

    def collect_ready(self):
        if not self.inflight:
            return
        done = self.eb.await_done(0, 0)
        while self.inflight and self.inflight[0] <= done:
            self._collect_oldest()

    def _collect_oldest(self):
        self.inflight.popleft()
        self._write(self.eb.wait())

    def _write(self, per_session):
        for sid, b in enumerate(per_session):
            if b:
                self.write(sid, b)

    def close(self):
        self._completion.close()
        while self.inflight:
            self._collect_oldest()
        self.eb.close()


def run_until_idle(loop: SelectorLoop, *batchers, timeout: float = 60.0):
    """Loop iterations without reads until every batcher's flushes are delivered
    (woken by the completion threads)."""
    import time
    end = time.monotonic() + timeout
    while any(b.inflight or b.flush_scheduled for b in batchers) or loop.has_tasks():
        if time.monotonic() > end:
            raise TimeoutError("flushes still in flight")
        loop.select(0.05)
        loop.run_iteration([])


__all__ = ["SelectorLoop", "LoopBatcher", "LoopEncodeBatcher", "run_until_idle"]
