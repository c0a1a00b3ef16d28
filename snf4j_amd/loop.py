"""The selector-loop side of the drop-in: the scheduling of
java/org/snf4j/websocket/gpu/WsgBatcher.java over the native batchers, restated in
Python so that it runs here (there is no JDK in this image) — the same calls in the
same order, driven by the same kind of loop.

The loop object these classes take is anything with snf4j's task-queue calls
(executenf, iteration): the SelectorLoop model the tests and the bench drive them with
is benchsupport/selector.py; the session around the decoder stage (snf4j-core's read
loop and exception path) is modelled in tests/harness/session.py.

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
  collects the oldest one blocking only when WSG_BATCHER_MAX_INFLIGHT (4) are in
  flight, then queues this one
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

from ._lib import BATCHER_MAX_INFLIGHT
from .codec import EncodeBatcher, NativeBatcher


class _Completion(threading.Thread):
    """Waits for the tickets it is given (await on the native batcher) and re-enters
    the loop with executenf(task) for each one that finished."""

    def __init__(self, loop, await_fn, task, name: str):
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

    def __init__(self, loop, n_sessions: int, deliver, ctx=None, clientMode: bool = False,
                 allowExtensions: bool = False, maxPayloadLen: int = 65536, validate_utf8: bool = True,
                 max_wire: int = 0, max_frames: int = 0, raw: bool = False,
                 max_inflight: int = BATCHER_MAX_INFLIGHT):
        self.loop = loop
        self.max_inflight = max_inflight  # (WsgBatcher: Wsg.BATCHER_MAX_INFLIGHT)
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
        fed = bool(self._sids)
        if fed:  # one feed call for the iteration's reads
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
        if not fed:  # (the reads went with a drain)
            return
        if len(self.inflight) == self.max_inflight:
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

    def __init__(self, loop, n_sessions: int, write, clientMode: bool = True, ctx=None,
                 max_frames: int = 0, max_payload: int = 0, deflate: tuple | None = None):
        self.loop = loop
        self.eb = EncodeBatcher(n_sessions, clientMode, ctx=ctx)
        if deflate is not None:  # (level, noContext): WsgBatcher.EncNative's wsg_enc_batcher_set_deflate
            self.eb.set_deflate(*deflate)
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


class CloseType:
    """ICloseControllingException.CloseType (ICloseControllingException.java:40-60)."""
    GENTLE, DEFAULT, NONE = "GENTLE", "DEFAULT", "NONE"



class GpuFrameDecoder:
    """java/org/snf4j/websocket/gpu/GpuFrameDecoder.java restated over DecoderBatcher
    (WsgBatcher's decode side): available() delimits on the loop thread, decode()
    hands the bytes to the batch, deliver() runs each frame through the rest of the
    pipeline and the handler, the first error does what FrameDecoder.java:92-102
    does, and an exception from downstream ends the session as controlClose does.
    Same methods, same order of effects as the Java class."""

    batched = False

    def __init__(self, clientMode: bool, allowExtensions: bool, maxPayloadLen: int, batcher: "DecoderBatcher"):
        self.batcher = batcher
        self.clientMode, self.allowExtensions, self.maxPayloadLen = clientMode, allowExtensions, maxPayloadLen
        self.sid = -1
        self.session = None
        self.closed = False     # FrameDecoder.closed (:63)
        self.released_ = False  # the session ended: the slot went back
        self.remaining = 0      # bytes of the current frame still to come (:348-355)

    # FrameDecoder.available(ISession, byte[], int, int) (FrameDecoder.java:357-401)
    def available(self, session, buffer, off: int, length: int) -> int:
        if self.closed:
            return length
        if self.remaining > 0:
            return min(length, self.remaining)
        from .context import frame_available
        hdr = bytes(buffer[off:off + min(length, 14)])
        return self._checked(session, frame_available(hdr, length), hdr, length)

    # FrameDecoder.available(ISession, ByteBuffer, boolean) (:290-332); the buffer is not moved
    def available_buffer(self, session, buffer: ByteBuffer, flipped: bool) -> int:
        b = buffer.duplicate() if flipped else buffer.duplicate().flip()
        length = b.remaining()
        if self.closed:
            return length
        if self.remaining > 0:
            return min(length, self.remaining)
        from .context import frame_available
        hdr = bytes(b.buf[b.pos:b.pos + min(length, 14)])
        return self._checked(session, frame_available(hdr, length), hdr, length)

    def _checked(self, session, res, hdr, length) -> int:
        r, err, d1, d2 = res
        if r < 0:  # Negative / Extended payload length (FrameDecoder.java:388-394)
            self.session = session
            if self.sid >= 0:
                self.batcher.drain(self)  # the frames read before this header first
            if self.closed:  # one of them failed first: the reference never reached this header
                return length
            self._fail(session, err, d1, d2, in_available=True)
        if r > 0:
            from .context import frame_available
            whole = frame_available(hdr, 0x7FFFFFFF)[0]  # the frame's length (the JNI err[3])
            if whole > r:  # a partial frame: the rest follows in later reads
                self.remaining = whole
        return r

    # FrameDecoder.decode (:180-288): the bytes go to the device batch
    def decode(self, session, data: ByteBuffer, out: list):
        self.session = session
        if self.closed or self.released_:
            session.release(data)
            return
        try:
            if self.sid < 0:
                self.sid = self.batcher.register(self)
        except RuntimeError:
            session.release(data)
            raise
        if self.remaining > 0:
            self.remaining -= data.remaining()
        self.batcher.enqueue(self, session, data)

    def _chain(self):
        """The decoders after "ws-decoder" the batch did not run."""
        after, chain = False, []
        for key, c in self.session.getCodecPipeline():
            if not after:
                after = key == "ws-decoder"
                continue
            if getattr(c, "batched", False):
                continue
            chain.append(c)
        return chain

    def deliver(self, frames, exc):
        """The session's frames of one device batch, on the loop thread."""
        if self.closed or self.released_:
            return
        chain = self._chain()
        for f in frames:
            if not self._downstream(f, chain):
                return
        if exc is not None:
            self._fail(self.session, None, 0, 0, in_available=False, exc=exc)

    def _downstream(self, frame, chain) -> bool:
        """One frame through the rest of the pipeline, then the handler
        (DefaultCodecExecutor.java:557-584); an exception goes to controlClose."""
        objs = [frame]
        try:
            for c in chain:
                nxt = []
                for o in objs:
                    c.decode(self.session, o, nxt)
                objs = nxt
            for o in objs:
                self.session.read_object(o)
        except Exception as e:  # noqa: BLE001
            return self._control_close(e)
        return True

    def _control_close(self, t) -> bool:
        """InternalSession.exception / controlClose (InternalSession.java:804-848):
        True if the session stays open (close type NONE)."""
        s = self.session
        ct = getattr(t, "getCloseType", None)
        if ct is not None:
            kind, cause = ct(), t.getClosingCause()
            if kind == CloseType.GENTLE:
                self.closed = True
                s.handler_exception(cause)
                s.close()
                return False
            if kind == CloseType.NONE:
                s.handler_exception(cause)
                return True
            t = cause
        self.closed = True
        s.handler_exception(t)
        s.quickClose()
        return False

    def fail_batch(self, e):
        """The device batch this session's bytes were in failed (not a protocol error)."""
        if self.closed or self.released_ or self.session is None:
            return
        self._control_close(e)

    def _fail(self, session, status, detail, detail2, in_available: bool, exc=None):
        from .context import error_message
        from .frame import CloseFrame, InvalidFrameException
        self.closed = True
        self.remaining = 0
        if exc is None:
            from .codec import _close_code
            code = _close_code(status)
            exc = InvalidFrameException(error_message(status, detail, detail2))
        else:
            code = exc.close_code
        session.writenf(CloseFrame.of_status(code))
        if in_available:
            raise exc  # FrameDecoder.available throws here too (:388-394)
        self._control_close(exc)  # InvalidFrameException: GENTLE (:75-77)

    # ---- IEventDrivenCodec
    def event_ending(self):
        self.release()

    def release(self):
        if not self.released_:
            self.released_ = True
            if self.sid >= 0:
                self.batcher.unregister(self)


class DecoderBatcher(LoopBatcher):
    """WsgBatcher's decode side with its session slots (register / unregister /
    enqueue / drain, WsgBatcher.java): deliveries go to the decoder holding the slot."""

    def __init__(self, loop, n_sessions: int, **kw):
        self.slots: list = [None] * n_sessions
        self.next = 0
        super().__init__(loop, n_sessions, self._route, **kw)

    def _route(self, sid, frames, exc):
        d = self.slots[sid]
        if d is not None:
            d.deliver(frames, exc)

    def register(self, d: GpuFrameDecoder) -> int:
        for i in range(self.n):
            sid = (self.next + i) % self.n
            if self.slots[sid] is None:
                self.nb.reset_session(sid)
                self.slots[sid] = d
                self.next = sid + 1
                return sid
        raise RuntimeError(f"no free session slot (maxSessions {self.n})")

    def unregister(self, d: GpuFrameDecoder):
        if d.sid < 0 or self.slots[d.sid] is not d:
            return
        self.reset_session(d.sid)
        self.slots[d.sid] = None

    def enqueue(self, d, session, data: ByteBuffer):  # noqa: D401 - WsgBatcher.enqueue
        super().enqueue(d.sid, data.peek())
        session.release(data)  # (Java releases it once the flush has fed it; the copy is taken here)

    def drain(self, d: GpuFrameDecoder | None = None):
        """WsgBatcher.drain: the iteration's reads fed and flushed, every flush collected
        (with no decoder: LoopBatcher.drain, what close() does)."""
        if d is None:
            return super().drain()
        fed = bool(self._sids)
        if fed:
            ids, data = self._sids, self._data
            self._sids, self._data = [], []
            self.nb.feed_many(ids, data)
            if len(self.inflight) == self.max_inflight:
                self._collect_oldest(blocking=True)
            self.nb.flush_async()
            self.inflight.append((self.nb.ticket(), self.loop.iteration))
        while self.inflight:
            self._collect_oldest(blocking=True)


__all__ = ["LoopBatcher", "LoopEncodeBatcher", "CloseType", "GpuFrameDecoder", "DecoderBatcher"]
