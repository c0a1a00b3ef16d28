"""The drop-in codec stages: FrameDecoder / FrameEncoder with the reference's
interface (same names, argument meaning and error behaviour), executed by the
HIP kernels of libwsgpu through its C ABI, plus the cross-session batcher that
feeds many sessions' frames to one GPU launch.

Reference (snf4j-websocket/src/main/java/org/snf4j/websocket/frame/):
  FrameDecoder.java:41-403       IBaseDecoder<ByteBuffer,Frame>: available() + decode()
  FrameUtf8Validator.java:40-100 fused into the decode pass (validate_utf8=True)
  FrameEncoder.java:41-136       IEncoder<Frame,ByteBuffer>
Errors: the stage writes CloseFrame(code) to the session and raises
InvalidFrameException(message) exactly where the reference does
(FrameDecoder.java:92-102, FrameUtf8Validator.java:54-57).
"""
from __future__ import annotations

import os
import struct

import numpy as np

from ._lib import AGG_STATE_DTYPE, DESC_DTYPE, ENCODE_DTYPE, RESULT_DTYPE, STATE_DTYPE
from .context import Context, check_header, decoder_cfg, error_message, frame_available
from .frame import (AggregatedBinaryFrame, AggregatedTextFrame, CloseFrame, Frame, InvalidFrameException, Opcode,
                    make_frame)

AGG_IN_AGG, AGG_PREFIXED, AGG_PENDING = 0x02, 0x04, 0x08  # wsg_frame_desc.flags of aggregator output

_CLOSE_FOR = {13: CloseFrame.NON_UTF8, 14: CloseFrame.NON_UTF8, 18: 1009}


def _close_code(err: int) -> int:
    return _CLOSE_FOR.get(err, CloseFrame.PROTOCOL_ERROR)


def _header_len(buf: bytes) -> int:
    b1 = buf[1]
    n = 2 + (4 if b1 & 0x80 else 0)
    ln = b1 & 0x7F
    return n + (2 if ln == 126 else 8 if ln == 127 else 0)


def _frame_total(buf) -> int:
    """Header + payload length of the frame starting at buf[0] (header complete)."""
    ln = buf[1] & 0x7F
    hl = _header_len(buf)
    if ln == 126:
        ln = struct.unpack(">H", bytes(buf[2:4]))[0]
    elif ln == 127:
        ln = struct.unpack(">Q", bytes(buf[2:10]))[0]
    return hl + ln


def _writenf(session, frame):
    if session is not None and hasattr(session, "writenf"):
        session.writenf(frame)


def _release(session, data):
    if session is not None and hasattr(session, "release"):
        session.release(data)


_default_ctx = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


class FrameDecoder:
    """GPU-backed FrameDecoder (+ the fused "ws-utf8-validator" stage).

    decode() of a complete frame runs one batch on the GPU; for throughput use
    SessionBatcher, which puts many sessions' frames into one launch.
    """

    def __init__(self, clientMode: bool, allowExtensions: bool, maxPayloadLen: int, validate_utf8: bool = True,
                 ctx: Context | None = None):
        self.cfg = decoder_cfg(clientMode, allowExtensions, maxPayloadLen, validate_utf8)
        self.ctx = ctx
        self.state = np.zeros(1, dtype=STATE_DTYPE)
        self._pending = None  # bytearray of a frame whose payload is incomplete
        self._need = 0

    def getInboundType(self):
        return bytes

    def getOutboundType(self):
        return Frame

    @property
    def closed(self) -> bool:
        return bool(self.state[0]["closed"])

    def _protocol_error(self, session, err, detail=0, detail2=0):
        self.state[0]["closed"] = 1
        _writenf(session, CloseFrame.of_status(_close_code(err)))
        return InvalidFrameException(error_message(err, detail, detail2))

    # FrameDecoder.available(ISession, byte[], off, len), :357-401
    def available(self, session, buffer, off: int = 0, length: int | None = None) -> int:
        buf = bytes(buffer)[off:]
        n = len(buf) if length is None else int(length)
        if self.closed:
            return n
        if self._pending is not None:
            return min(n, self._need - len(self._pending))
        r, err, d1, d2 = frame_available(buf, n)
        if r < 0:
            raise self._protocol_error(session, err, d1, d2)
        return r

    # FrameDecoder.decode(ISession, ByteBuffer, List<Frame>), :180-288
    def decode(self, session, data, out: list):
        data = bytes(data)
        try:
            if self.closed:
                return
            if self._pending is not None:
                self._pending += data
                if len(self._pending) < self._need:
                    return
                frame, self._pending = bytes(self._pending), None
            else:
                hl = _header_len(data) if len(data) >= 2 else 2
                if len(data) < hl:
                    raise ValueError("incomplete frame header (reference: BufferUnderflowException)")
                err, det = check_header(self.cfg, bool(self.state[0]["fragmentation"]), data[:hl])
                if err:
                    raise self._protocol_error(session, err, det)
                total = _frame_total(data)
                if len(data) < total:
                    self._pending, self._need = bytearray(data), total
                    return
                frame = data
            self._run(session, frame, out)
        finally:
            _release(session, data)

    def _run(self, session, frame: bytes, out: list):
        ctx = self.ctx or default_context()
        wire = np.frombuffer(frame, dtype=np.uint8)
        payload, desc, result = ctx.decode_host(self.cfg, wire, np.array([0, len(frame)], np.uint64),
                                                np.array([0, 1], np.uint32), self.state)
        r = result[0]
        if r["n_delivered"] == 1:
            d = desc[0]
            off, ln = int(d["payload_off"]), int(d["payload_len"])
            out.append(make_frame(int(d["opcode"]), bool(d["flags"] & 0x80), (int(d["flags"]) >> 4) & 7,
                                  payload[off:off + ln].tobytes()))
        elif r["error"]:
            _writenf(session, CloseFrame.of_status(int(r["close_code"])))
            raise InvalidFrameException(error_message(int(r["error"]), int(r["detail"])))


class FrameEncoder:
    """GPU-backed FrameEncoder. The mask key comes from `mask_source()` (default:
    os.urandom, standing in for the reference's java.util.Random, FrameEncoder.java:43)."""

    def __init__(self, clientMode: bool, ctx: Context | None = None, mask_source=None):
        self.clientMode = bool(clientMode)
        self.ctx = ctx
        self.mask_source = mask_source or (lambda: os.urandom(4))
        self.closed = np.zeros(1, dtype=np.uint8)

    def getInboundType(self):
        return Frame

    def getOutboundType(self):
        return bytes

    def length(self, frame: Frame) -> int:
        from .context import encoded_length
        return encoded_length(frame.getPayloadLength(), self.clientMode)

    def encode(self, session, frame: Frame, out: list):
        if self.closed[0]:
            return
        ctx = self.ctx or default_context()
        payload = np.frombuffer(frame.getPayload(), dtype=np.uint8)
        fr = np.zeros(1, dtype=ENCODE_DTYPE)
        fr[0]["payload_off"] = 0
        fr[0]["payload_len"] = len(payload)
        fr[0]["opcode"] = int(frame.getOpcode())
        fr[0]["flags"] = (0x80 if frame.isFinalFragment() else 0) | ((frame.getRsvBits() & 7) << 4)
        if self.clientMode:
            fr[0]["mask"] = np.frombuffer(bytes(self.mask_source()), dtype=np.uint8)
        wire, _ = ctx.encode_host(self.clientMode, payload, fr, np.array([0, 1], np.uint32), self.closed)
        buf = wire.tobytes()
        if session is not None and hasattr(session, "allocate"):
            b = session.allocate(len(buf))
            b[:] = buf
            buf = b
        out.append(buf)


class SessionBatcher:
    """Cross-session batching: bytes from many sessions' socket reads are framed on
    the host (the session loop's available() calls, StreamSession.java:798-854),
    complete frames are queued, and flush() decodes all queued frames of all
    sessions in ONE device batch.  Per-session state (fragmentation, UTF-8 carry,
    closed) persists across flushes.  Header rules are applied as soon as a
    header is complete, so a frame announcing a too-long payload fails without
    waiting for its bytes, as in the reference (FrameDecoder.java:238-256)."""

    def __init__(self, n_sessions: int, clientMode: bool = False, allowExtensions: bool = False,
                 maxPayloadLen: int = 65536, validate_utf8: bool = True, ctx: Context | None = None):
        self.cfg = decoder_cfg(clientMode, allowExtensions, maxPayloadLen, validate_utf8)
        self.ctx = ctx
        self.n = n_sessions
        self.state = np.zeros(n_sessions, dtype=STATE_DTYPE)
        self.inbuf = [bytearray() for _ in range(n_sessions)]
        self.queue = [[] for _ in range(n_sessions)]
        self.host_error = [None] * n_sessions
        self._frag_host = np.zeros(n_sessions, dtype=bool)  # fragmentation as of the queued frames

    def feed(self, sid: int, data: bytes):
        if self.state[sid]["closed"] or self.host_error[sid] is not None:
            return
        buf = self.inbuf[sid]
        buf += data
        pos = 0
        while True:
            r, err, d1, d2 = frame_available(bytes(buf[pos:pos + 14]), len(buf) - pos)
            if r < 0:
                self.host_error[sid] = (err, d1, d2)
                break
            if r == 0:
                break
            hl = _header_len(buf[pos:pos + 2]) if len(buf) - pos >= 2 else 2
            e, det = check_header(self.cfg, bool(self._frag_host[sid]), bytes(buf[pos:pos + hl]))
            if e and e != 17:  # a header rule fails: report it now (the frame may never complete)
                self.host_error[sid] = (e, det, 0)
                break
            total = _frame_total(buf[pos:pos + hl])
            if len(buf) - pos < total:
                break
            op = buf[pos] & 0x0F
            if op <= 2:
                self._frag_host[sid] = not (buf[pos] & 0x80)
            self.queue[sid].append(bytes(buf[pos:pos + total]))
            pos += total
        del buf[:pos]

    def flush(self):
        """Decode everything queued. Returns [(frames, InvalidFrameException | None)] per session."""
        ctx = self.ctx or default_context()
        frames_all, first, off = [], [0], [0]
        for q in self.queue:
            for f in q:
                frames_all.append(f)
                off.append(off[-1] + len(f))
            first.append(len(frames_all))
        wire = np.frombuffer(b"".join(frames_all), dtype=np.uint8) if frames_all else np.zeros(0, np.uint8)
        payload, desc, result = ctx.decode_host(self.cfg, wire, np.array(off, np.uint64),
                                                np.array(first, np.uint32), self.state)
        out = []
        for s in range(self.n):
            r = result[s]
            frames = []
            for k in range(first[s], first[s] + int(r["n_delivered"])):
                d = desc[k]
                o, ln = int(d["payload_off"]), int(d["payload_len"])
                frames.append(make_frame(int(d["opcode"]), bool(d["flags"] & 0x80), (int(d["flags"]) >> 4) & 7,
                                         payload[o:o + ln].tobytes()))
            exc = None
            if r["error"]:
                exc = InvalidFrameException(error_message(int(r["error"]), int(r["detail"])))
                exc.close_code = int(r["close_code"])
            elif self.host_error[s] is not None and not self.state[s]["closed"]:
                e, d1, d2 = self.host_error[s]
                exc = InvalidFrameException(error_message(e, d1, d2))
                exc.close_code = _close_code(e)
                self.state[s]["closed"] = 1
            out.append((frames, exc))
            self.queue[s] = []
        return out


class BatchAggregator:
    """FrameAggregator (FrameAggregator.java:72-104) for every session of a batch
    flow, run on the GPU over each decoded batch (wsg_aggregate_batch_*).  The
    device lays every fragmented message's bytes back to back; the bytes of a
    message still open at the end of a batch are held here per session, as the
    reference's PayloadAggregator holds its fragment list (PayloadAggregator.java:34),
    and put in front of the message's remaining bytes when it completes."""

    def __init__(self, n_sessions: int, maxAggregatedLength: int, ctx: Context | None = None):
        self.max_len = int(maxAggregatedLength)
        self.ctx = ctx
        self.state = np.zeros(n_sessions, dtype=AGG_STATE_DTYPE)
        self.held = [[] for _ in range(n_sessions)]

    def run(self, desc, session_first, dec_result, payload):
        """Aggregate one decoded batch (host arrays as wsg_decode_batch_host returns
        them).  Returns [(frames, InvalidFrameException | None)] per session."""
        ctx = self.ctx or default_context()
        sf = np.ascontiguousarray(session_first, dtype=np.uint32)
        agg, od, ores = ctx.aggregate_host(self.max_len, desc, sf, dec_result, payload, self.state)
        out = []
        for s in range(len(sf) - 1):
            base = int(sf[s]) + s
            r = ores[s]
            frames = []
            for i in range(int(r["n_delivered"])):
                d = od[base + i]
                fl, o, ln = int(d["flags"]), int(d["payload_off"]), int(d["payload_len"])
                rsv = (fl >> 4) & 7
                if fl & AGG_IN_AGG:
                    part = agg[o:o + ln].tobytes()
                    parts = (self.held[s] if fl & AGG_PREFIXED else []) + [part]
                    self.held[s] = []
                    cls = AggregatedTextFrame if int(d["opcode"]) == 1 else AggregatedBinaryFrame
                    frames.append(cls(rsv, b"".join(parts), parts))
                else:
                    frames.append(make_frame(int(d["opcode"]), bool(fl & 0x80), rsv, payload[o:o + ln].tobytes()))
            exc = None
            if r["error"]:
                exc = InvalidFrameException(error_message(int(r["error"]), int(r["detail"])))
                exc.close_code = int(r["close_code"])
                exc.frame_index = int(r["detail"])
            elif self.state[s]["open"]:
                d = od[base + int(r["n_delivered"])]
                assert int(d["flags"]) & AGG_PENDING
                o, ln = int(d["payload_off"]), int(d["payload_len"])
                kept = self.held[s] if int(d["flags"]) & AGG_PREFIXED else []
                self.held[s] = kept + ([agg[o:o + ln].tobytes()] if ln else [])
            else:
                self.held[s] = []
            out.append((frames, exc))
        return out


class FrameAggregator:
    """GPU-backed FrameAggregator(maxAggregatedLength): IDecoder<Frame,Frame>
    (FrameAggregator.java:40-104).  decode() of one frame runs a one-frame batch;
    for throughput, BatchAggregator aggregates whole decoded batches."""

    def __init__(self, maxAggregatedLength: int, ctx: Context | None = None):
        self._b = BatchAggregator(1, maxAggregatedLength, ctx)

    def getInboundType(self):
        return Frame

    def getOutboundType(self):
        return Frame

    def decode(self, session, data: Frame, out: list):
        payload = bytes(data.getPayload())
        desc = np.zeros(1, dtype=DESC_DTYPE)
        desc[0]["payload_len"] = len(payload)
        desc[0]["opcode"] = int(data.getOpcode())
        desc[0]["flags"] = (0x80 if data.isFinalFragment() else 0) | ((data.getRsvBits() & 7) << 4)
        res = np.zeros(1, dtype=RESULT_DTYPE)
        res[0]["n_delivered"] = 1
        pl = np.frombuffer(payload + bytes(16), dtype=np.uint8)
        frames, exc = self._b.run(desc, np.array([0, 1], np.uint32), res, pl)[0]
        if exc is not None:
            _writenf(session, CloseFrame.of_status(exc.close_code))  # tooBig: CloseFrame.TOO_BIG (:66-69)
            raise exc
        for f in frames:
            out.append(data if not isinstance(f, (AggregatedTextFrame, AggregatedBinaryFrame)) else f)


class FrameUtf8Validator:
    """GPU-backed FrameUtf8Validator: the "ws-utf8-validator" stage alone
    (FrameUtf8Validator.java:40-100), for pipelines where validation cannot be fused
    into the decode pass (permessage-deflate inflates between the two,
    PerMessageDeflateExtension.java:316-326).  decode() of one frame runs a
    one-frame batch (wsg_validate_batch_host); frames pass through unchanged."""

    def __init__(self, ctx: Context | None = None):
        self.ctx = ctx
        self.state = np.zeros(1, dtype=STATE_DTYPE)

    def getInboundType(self):
        return Frame

    def getOutboundType(self):
        return Frame

    def decode(self, session, frame: Frame, out: list):
        ctx = self.ctx or default_context()
        payload = bytes(frame.getPayload())
        desc = np.zeros(1, dtype=DESC_DTYPE)
        desc[0]["payload_len"] = len(payload)
        desc[0]["opcode"] = int(frame.getOpcode())
        desc[0]["flags"] = (0x80 if frame.isFinalFragment() else 0) | ((frame.getRsvBits() & 7) << 4)
        self.state[0]["closed"] = 0  # the stage itself does not latch; the session closes on the exception
        r = ctx.validate_host(desc, np.array([0, 1], np.uint32), np.frombuffer(payload + bytes(16), np.uint8),
                              self.state)[0]
        if r["error"]:
            # the reference clears its context on FIN before validating (:83-88): a failed
            # non-final frame leaves the context as it stands; the session closes anyway
            _writenf(session, CloseFrame.of_status(int(r["close_code"])))
            raise InvalidFrameException(error_message(int(r["error"]), int(r["detail"])))
        out.append(frame)


class NativeBatcher:
    """The native cross-session batcher (wsg_batcher_*, batcher.hip): the C++ core a
    JNI shim drives.  feed() takes a session's socket bytes, delimits frames on the
    host as the session read loop does (FrameDecoder.available,
    StreamSession.java:798-854) and applies the header rules as soon as a header is
    complete; flush() decodes every complete frame of every session in one device
    batch.  Same results as SessionBatcher, without Python in the per-frame loop."""

    def __init__(self, n_sessions: int, clientMode: bool = False, allowExtensions: bool = False,
                 maxPayloadLen: int = 65536, validate_utf8: bool = True, ctx: Context | None = None):
        from ._lib import check, lib
        import ctypes as C
        self.ctx = ctx or default_context()
        self.cfg = decoder_cfg(clientMode, allowExtensions, maxPayloadLen, validate_utf8)
        self.n = n_sessions
        h = C.c_void_p()
        check(lib.wsg_batcher_open(self.ctx._h, C.byref(self.cfg), n_sessions, C.byref(h)), self.ctx._h)
        self._h = h

    def close(self):
        from ._lib import lib
        if getattr(self, "_h", None):
            lib.wsg_batcher_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        from ._lib import WsgError, lib
        if rc != 0:
            raise WsgError(f"libwsgpu batcher error {rc}: {lib.wsg_batcher_last_error(self._h).decode()}")

    def feed(self, sid: int, data):
        from ._lib import lib
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        if a.size:
            self._check(lib.wsg_batcher_feed(self._h, int(sid), a.ctypes.data, a.size))

    def set_stages(self, inflate: bool = False, noContext: bool = False, validate: bool = True,
                   aggregate: bool = False, maxAggregatedLength: int = 0):
        """The decoders after "ws-decoder" that each flush runs in the same device batch
        (wsg_batcher_set_stages): PerMessageDeflateDecoder(noContext) -> FrameUtf8Validator
        -> FrameAggregator(maxAggregatedLength), as the pipeline orders them."""
        import ctypes as C
        from ._lib import StageCfg, lib
        c = StageCfg(int(inflate), int(noContext), int(validate), int(aggregate), 0, int(maxAggregatedLength))
        self._check(lib.wsg_batcher_set_stages(self._h, C.byref(c)))

    def stage_split_count(self) -> int:
        """Messages the stage chain's inflate took with the split-lane decode
        (wsg_inflate_split_count on wsg_batcher_stage_context); 0 before set_stages."""
        import ctypes as C
        from ._lib import lib
        h = lib.wsg_batcher_stage_context(self._h)
        if not h:
            return 0
        n = C.c_uint64()
        if lib.wsg_inflate_split_count(C.c_void_p(h), C.byref(n)) != 0:
            raise RuntimeError("wsg_inflate_split_count failed")
        return int(n.value)

    def reset_session(self, sid: int):
        """Hand slot `sid` to a new session (wsg_batcher_session_reset): the partial
        frame and the carry are dropped, as a fresh FrameDecoder would start."""
        from ._lib import lib
        self._check(lib.wsg_batcher_session_reset(self._h, int(sid)))

    def feed_many(self, sids, chunks):
        """Many socket reads in one call (wsg_batcher_feed_many): chunks[i] of session
        sids[i]; each session's reads in order, the sessions fed by several threads."""
        import ctypes as C
        from ._lib import lib
        n = len(sids)
        arrs = [c if isinstance(c, np.ndarray) else np.frombuffer(bytes(c), dtype=np.uint8) for c in chunks]
        sid_a = np.ascontiguousarray(sids, dtype=np.uint32)
        ptrs = (C.c_void_p * max(1, n))(*[a.ctypes.data if a.size else None for a in arrs])
        lens = np.array([a.size for a in arrs], dtype=np.uint64)
        self._check(lib.wsg_batcher_feed_many(self._h, n, sid_a.ctypes.data, C.addressof(ptrs), lens.ctypes.data))

    def feed_many_ptrs(self, sids, ptrs, lens):
        """feed_many over numpy arrays: session ids (u32), host addresses (u64) and
        lengths (u64) of the reads — no per-read Python objects."""
        from ._lib import lib
        sids = np.ascontiguousarray(sids, dtype=np.uint32)
        ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        self._check(lib.wsg_batcher_feed_many(self._h, len(sids), sids.ctypes.data, ptrs.ctypes.data,
                                              lens.ctypes.data))

    def flush_async(self):
        """Queue the decode of everything complete (wsg_batcher_flush_async); collect it
        with wait().  At most two in flight."""
        from ._lib import lib
        self._check(lib.wsg_batcher_flush_async(self._h))

    def ticket(self) -> int:
        """The last queued flush's ticket (wsg_batcher_ticket: flushes are 1, 2, ...)."""
        from ._lib import lib
        return int(lib.wsg_batcher_ticket(self._h))

    def await_done(self, seen: int, timeout_ms: int) -> int:
        """wsg_batcher_await: the highest ticket whose device work has finished, once one
        above `seen` has or `timeout_ms` passed (0: no wait).  Safe from another thread."""
        from ._lib import lib
        return int(lib.wsg_batcher_await(self._h, int(seen), int(timeout_ms)))

    def reserve(self, max_wire: int, max_frames: int):
        """wsg_batcher_reserve: flushes up to these sizes allocate nothing."""
        from ._lib import lib
        self._check(lib.wsg_batcher_reserve(self._h, int(max_wire), int(max_frames)))

    def reserve_stages(self, max_out_bytes: int, max_out_frames: int):
        """wsg_batcher_reserve_stages (after set_stages and reserve): flushes whose stages
        deliver up to these sizes allocate nothing."""
        from ._lib import lib
        self._check(lib.wsg_batcher_reserve_stages(self._h, int(max_out_bytes), int(max_out_frames)))

    def wait_raw(self):
        """The oldest queued flush's results (wsg_batcher_wait), as flush_raw returns them."""
        import ctypes as C
        from ._lib import BatchView, lib
        v = BatchView()
        self._check(lib.wsg_batcher_wait(self._h, C.byref(v)))
        return self._views(v)

    def wait(self):
        return self._frames(*self.wait_raw()[:4])

    def flush_raw(self):
        """Decode everything complete; returns numpy views (valid until the next flush):
        (session_first, desc, payload, result, wire_bytes)."""
        import ctypes as C
        from ._lib import BatchView, lib
        v = BatchView()
        self._check(lib.wsg_batcher_flush(self._h, C.byref(v)))
        return self._views(v)

    def _views(self, v):
        import ctypes as C
        n, s = int(v.n_frames), int(v.n_sessions)

        def view(ptr, count, dtype):
            if not count:
                return np.zeros(0, dtype=dtype)
            buf = (C.c_uint8 * (count * np.dtype(dtype).itemsize)).from_address(ptr)
            return np.frombuffer(buf, dtype=dtype)

        sf = view(v.session_first, s + 1, np.uint32)
        desc = view(v.desc, n, DESC_DTYPE)
        res = view(v.result, s, RESULT_DTYPE)
        end = int((desc["payload_off"] + desc["payload_len"]).max()) if n else 0
        payload = view(v.payload, end, np.uint8)
        self._detail2 = view(v.detail2, s, np.int64) if v.detail2 else np.zeros(s, np.int64)
        return sf, desc, payload, res, int(v.wire_bytes)

    def flush(self):
        """[(frames, InvalidFrameException | None)] per session, like SessionBatcher.flush."""
        return self._frames(*self.flush_raw()[:4])

    def _frames(self, sf, desc, payload, res):
        d2 = self._detail2
        out = []
        for s in range(self.n):
            r = res[s]
            frames = []
            for k in range(int(sf[s]), int(sf[s]) + int(r["n_delivered"])):
                d = desc[k]
                o, ln = int(d["payload_off"]), int(d["payload_len"])
                data, rsv = payload[o:o + ln].tobytes(), (int(d["flags"]) >> 4) & 7
                if int(d["flags"]) & AGG_IN_AGG:  # WSG_OUT_AGGREGATED: a FrameAggregator message
                    cls = AggregatedTextFrame if int(d["opcode"]) == 1 else AggregatedBinaryFrame
                    frames.append(cls(rsv, data, [data]))
                else:
                    frames.append(make_frame(int(d["opcode"]), bool(d["flags"] & 0x80), rsv, data))
            exc = None
            if r["error"]:
                exc = InvalidFrameException(error_message(int(r["error"]), int(r["detail"]), int(d2[s])))
                exc.close_code = int(r["close_code"])
            out.append((frames, exc))
        return out


class EncodeBatcher:
    """The native cross-session encode batcher (wsg_enc_batcher_*, batcher.hip):
    FrameEncoder.encode (FrameEncoder.java:69-120) for every session of a loop in
    one device batch per flush.  add() queues a frame (the payload is copied to a
    pinned arena); flush() returns each session's wire bytes, its frames in the
    order they were added, with the close latch (:71-76) kept across flushes."""

    def __init__(self, n_sessions: int, clientMode: bool, ctx: Context | None = None):
        from ._lib import check, lib
        import ctypes as C
        self.ctx = ctx or default_context()
        self.n = n_sessions
        h = C.c_void_p()
        check(lib.wsg_enc_batcher_open(self.ctx._h, int(bool(clientMode)), n_sessions, C.byref(h)), self.ctx._h)
        self._h = h

    def close(self):
        from ._lib import lib
        if getattr(self, "_h", None):
            lib.wsg_enc_batcher_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        from ._lib import WsgError, lib
        if rc != 0:
            raise WsgError(f"libwsgpu encode batcher error {rc}: {lib.wsg_enc_batcher_last_error(self._h).decode()}")

    def add(self, sid: int, frame: Frame, mask=(0, 0, 0, 0)):
        from ._lib import lib
        p = np.frombuffer(bytes(frame.getPayload()), dtype=np.uint8)
        m = np.asarray(mask, dtype=np.uint8)
        flags = (0x80 if frame.isFinalFragment() else 0) | ((frame.getRsvBits() & 7) << 4)
        self._check(lib.wsg_enc_batcher_add(self._h, int(sid), int(frame.getOpcode()), flags, m.ctypes.data,
                                            p.ctypes.data if p.size else None, int(p.size)))

    def add_many_ptrs(self, sids, opcodes, flags, masks, ptrs, lens):
        """wsg_enc_batcher_add_many over numpy arrays: per frame its session (u32),
        opcode and FIN/RSV flags (u8), 4-byte mask (u8 [n, 4], or None), payload host
        address (u64) and length (u32), in the order add() would take them."""
        from ._lib import lib
        sids = np.ascontiguousarray(sids, dtype=np.uint32)
        opcodes = np.ascontiguousarray(opcodes, dtype=np.uint8)
        flags = np.ascontiguousarray(flags, dtype=np.uint8)
        ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        m = np.ascontiguousarray(masks, dtype=np.uint8) if masks is not None else None
        self._check(lib.wsg_enc_batcher_add_many(self._h, len(sids), sids.ctypes.data, opcodes.ctypes.data,
                                                 flags.ctypes.data, m.ctypes.data if m is not None else None,
                                                 ptrs.ctypes.data, lens.ctypes.data))

    def set_deflate(self, compressionLevel: int, noContext: bool):
        """PerMessageDeflateEncoder(compressionLevel, noContext) in front of the encoder for
        every session (wsg_enc_batcher_set_deflate): each flush compresses on the device first."""
        from ._lib import lib
        self._check(lib.wsg_enc_batcher_set_deflate(self._h, int(compressionLevel), int(bool(noContext))))

    def reset_session(self, sid: int):
        from ._lib import lib
        self._check(lib.wsg_enc_batcher_session_reset(self._h, int(sid)))

    def flush(self):
        """[wire bytes of session s] (its frames back to back)."""
        import ctypes as C
        from ._lib import EncView, lib
        v = EncView()
        self._check(lib.wsg_enc_batcher_flush(self._h, C.byref(v)))
        return self._sessions(v)

    def flush_async(self):
        """Queue the encode of everything added so far (wsg_enc_batcher_flush_async);
        collect it with wait().  At most two in flight."""
        from ._lib import lib
        self._check(lib.wsg_enc_batcher_flush_async(self._h))

    def ticket(self) -> int:
        from ._lib import lib
        return int(lib.wsg_enc_batcher_ticket(self._h))

    def await_done(self, seen: int, timeout_ms: int) -> int:
        """wsg_enc_batcher_await (see NativeBatcher.await_done)."""
        from ._lib import lib
        return int(lib.wsg_enc_batcher_await(self._h, int(seen), int(timeout_ms)))

    def reserve(self, max_frames: int, max_payload: int):
        from ._lib import lib
        self._check(lib.wsg_enc_batcher_reserve(self._h, int(max_frames), int(max_payload)))

    def wait_raw(self):
        """The oldest queued flush (wsg_enc_batcher_wait) as numpy views, valid until
        that slot is flushed again: (session_first, wire_off, wire)."""
        import ctypes as C
        from ._lib import EncView, lib
        v = EncView()
        self._check(lib.wsg_enc_batcher_wait(self._h, C.byref(v)))
        n, s = int(v.n_frames), int(v.n_sessions)
        sf = np.ctypeslib.as_array((C.c_uint32 * (s + 1)).from_address(v.session_first))
        off = np.ctypeslib.as_array((C.c_uint64 * (n + 1)).from_address(v.wire_off))
        wire = np.ctypeslib.as_array((C.c_uint8 * int(v.wire_bytes)).from_address(v.wire)) if v.wire_bytes \
            else np.zeros(0, np.uint8)
        return sf, off, wire

    def wait(self):
        """[wire bytes of session s] of the oldest queued flush."""
        import ctypes as C
        from ._lib import EncView, lib
        v = EncView()
        self._check(lib.wsg_enc_batcher_wait(self._h, C.byref(v)))
        return self._sessions(v)

    def _sessions(self, v):
        import ctypes as C
        n, s = int(v.n_frames), int(v.n_sessions)
        sf = np.ctypeslib.as_array((C.c_uint32 * (s + 1)).from_address(v.session_first))
        off = np.ctypeslib.as_array((C.c_uint64 * (n + 1)).from_address(v.wire_off))
        wire = (C.c_uint8 * int(v.wire_bytes)).from_address(v.wire) if v.wire_bytes else b""
        wb = bytes(wire)
        return [wb[int(off[sf[i]]):int(off[sf[i + 1]])] for i in range(s)]


def pinned_alloc(capacity: int):
    """A pinned host buffer from the library's pool (wsg_host_alloc), as a numpy
    uint8 array of its class capacity; return it with pinned_release()."""
    import ctypes as C
    from ._lib import lib
    p = lib.wsg_host_alloc(int(capacity))
    if not p:
        raise MemoryError("wsg_host_alloc failed")
    n = int(lib.wsg_host_capacity(p))
    return np.frombuffer((C.c_uint8 * n).from_address(p), dtype=np.uint8)


def pinned_release(arr) -> None:
    from ._lib import lib
    rc = lib.wsg_host_release(arr.ctypes.data)
    if rc != 0:
        raise ValueError("buffer not from the pinned pool")


class BatchInflater:
    """PerMessageDeflateDecoder (PerMessageDeflateDecoder.java:68-105) for every session of a
    batch flow, run on the GPU over each decoded batch (wsg_inflate_batch_host).  The
    per-session inflater state and its 32 KiB window stay in `state` / `window`; the
    frames of a message a batch leaves open are re-sent with the next batch (replay),
    so the device always restarts a message from its first frame.  Output regions are
    sized from the compressed bytes and grown for a session that overflows."""

    def __init__(self, n_sessions: int, noContext: bool = False, ctx: Context | None = None, ratio: int = 16):
        from ._lib import INFLATE_STATE_DTYPE
        self.no_context = bool(noContext)
        self.ctx = ctx
        self.n = n_sessions
        self.state = np.zeros(n_sessions, dtype=INFLATE_STATE_DTYPE)
        self.window = np.zeros(n_sessions * 32768, dtype=np.uint8)
        self.held = [[] for _ in range(n_sessions)]   # (desc, payload bytes) of an open message
        self.ratio = ratio

    def _run(self, sids, per_session, caps):
        """One device batch over sessions `sids` (frames: lists of (desc row, payload bytes, replay))."""
        from ._lib import INFLATE_STATE_DTYPE
        ctx = self.ctx or default_context()
        rows, chunks, sf, pos = [], [], [0], 0
        for s in sids:
            for (d, p, rep) in per_session[s]:
                r = np.array(d, dtype=DESC_DTYPE).reshape(())
                r = r.copy()
                r["payload_off"] = pos
                r["payload_len"] = len(p)
                r["flags"] = (int(d["flags"]) & ~0x02) | (0x02 if rep else 0)
                rows.append(r)
                chunks.append(p)
                pos += len(p)
            sf.append(len(rows))
        desc = np.array(rows, dtype=DESC_DTYPE) if rows else np.zeros(0, DESC_DTYPE)
        payload = np.frombuffer(b"".join(chunks) + bytes(16), dtype=np.uint8)
        st = np.ascontiguousarray(self.state[sids]).astype(INFLATE_STATE_DTYPE)
        win = np.ascontiguousarray(self.window.reshape(self.n, 32768)[sids]).reshape(-1)
        out_off = np.zeros(len(sids) + 1, dtype=np.uint64)
        out_off[1:] = np.cumsum([caps[s] for s in sids])
        out, odesc, res, rf = ctx.inflate_host(self.no_context, desc, np.array(sf, np.uint32), payload, st, win,
                                               out_off)
        return sf, out, odesc, res, rf, st, win, payload

    def run(self, desc, session_first, payload):
        """Inflate one decoded batch (host arrays; the frames each session's decoder delivered).
        Returns [(frames, InvalidFrameException | None)] per session."""
        sf = np.asarray(session_first, dtype=np.int64)
        payload = np.asarray(payload, dtype=np.uint8)
        per = []
        for s in range(self.n):
            fr = [(d, b, True) for (d, b) in self.held[s]]
            for k in range(int(sf[s]), int(sf[s + 1])):
                d = desc[k]
                o, ln = int(d["payload_off"]), int(d["payload_len"])
                fr.append((d, payload[o:o + ln].tobytes(), False))
            per.append(fr)
        caps = {s: 65536 + self.ratio * sum(len(p) + 4 for (_, p, _) in per[s]) for s in range(self.n)}
        results = [None] * self.n
        todo = list(range(self.n))
        while todo:
            bsf, out, odesc, res, rf, st, win, _ = self._run(todo, per, caps)
            retry = []
            for i, s in enumerate(todo):
                r = res[i]
                if int(r["error"]) == 21:  # the output region overflowed: nothing committed, grow it
                    caps[s] *= 8
                    retry.append(s)
                    continue
                self.state[s] = st[i]
                self.window.reshape(self.n, 32768)[s] = win.reshape(len(todo), 32768)[i]
                frames = []
                nd = int(r["n_delivered"])
                ks = [k for k in range(int(bsf[i]), int(bsf[i + 1])) if not per[s][k - int(bsf[i])][2]]
                for k in ks[:nd]:
                    d = odesc[k]
                    o, ln = int(d["payload_off"]), int(d["payload_len"])
                    if int(d["flags"]) & 0x02:
                        data = out[o:o + ln].tobytes()
                    else:
                        data = per[s][k - int(bsf[i])][1]
                    f = make_frame(int(d["opcode"]), bool(d["flags"] & 0x80), (int(d["flags"]) >> 4) & 7, data)
                    f.inflated = bool(int(d["flags"]) & 0x02)
                    frames.append(f)
                exc = None
                if int(r["error"]):
                    exc = InvalidFrameException(error_message(int(r["error"])))
                    exc.close_code = int(r["close_code"])
                    exc.frame_index = int(r["detail"])
                    self.held[s] = []
                elif int(rf[i]) != 0xFFFFFFFF:  # a message left open: re-send its frames next time
                    self.held[s] = [(d, b) for (d, b, _) in per[s][int(rf[i]):]]
                else:
                    self.held[s] = []
                results[s] = (frames, exc)
            todo = retry
        return results


class BatchDeflater:
    """PerMessageDeflateEncoder(compressionLevel, noContext) (PerMessageDeflateEncoder.java:
    39-100) for every session of a batch flow, run on the GPU over each batch of outgoing
    frames (wsg_deflate_batch_host): zlib's raw deflate with a Z_SYNC_FLUSH per frame,
    byte-identical to java.util.zip.Deflater's.  The per-session deflater state (zlib's
    strstart / high_water / insert and its window, head and prev arrays) stays in `state` /
    `session_mem` between batches (context takeover)."""

    def __init__(self, n_sessions: int, compressionLevel: int = 6, noContext: bool = False,
                 ctx: Context | None = None):
        from ._lib import DEFLATE_STATE_DTYPE
        from .context import DEFLATE_SESSION_BYTES
        if compressionLevel < 0 or compressionLevel > 9:
            raise ValueError("compression level is out of range")   # ZlibEncoder.java:102-104
        self.level = int(compressionLevel)
        self.no_context = bool(noContext)
        self.ctx = ctx
        self.n = n_sessions
        self.state = np.zeros(n_sessions, dtype=DEFLATE_STATE_DTYPE)
        self.session_mem = np.zeros(n_sessions * DEFLATE_SESSION_BYTES, dtype=np.uint8)

    def run(self, frames, with_flags: bool = False):
        """frames[s] = [(opcode, fin, rsv, payload)] of session s, in order.  Returns the
        encoded frames of every session, [(opcode, fin, rsv, payload)] (with_flags: a fifth
        element, True when the payload was produced by the deflater)."""
        ctx = self.ctx or default_context()
        rows, chunks, sf, pos = [], [], [0], 0
        for s in range(self.n):
            for op, fin, rsv, p in frames[s]:
                r = np.zeros((), dtype=DESC_DTYPE)
                r["payload_off"] = pos
                r["payload_len"] = len(p)
                r["opcode"] = int(op)
                r["flags"] = (0x80 if fin else 0) | ((int(rsv) & 7) << 4)
                rows.append(r)
                chunks.append(bytes(p))
                pos += len(p)
            sf.append(len(rows))
        desc = np.array(rows, dtype=DESC_DTYPE) if rows else np.zeros(0, DESC_DTYPE)
        payload = np.frombuffer(b"".join(chunks) + bytes(16), dtype=np.uint8)
        out, odesc = ctx.deflate_host(self.level, self.no_context, desc, np.array(sf, np.uint32), payload,
                                      self.state, self.session_mem)
        res = []
        for s in range(self.n):
            fs = []
            for k in range(sf[s], sf[s + 1]):
                d = odesc[k]
                o, ln = int(d["payload_off"]), int(d["payload_len"])
                deflated = bool(int(d["flags"]) & 0x02)
                data = out[o:o + ln].tobytes() if deflated else chunks[k]
                t = (int(d["opcode"]), bool(int(d["flags"]) & 0x80), (int(d["flags"]) >> 4) & 7, data)
                fs.append(t + (deflated,) if with_flags else t)
            res.append(fs)
        return res


class PerMessageDeflateEncoder:
    """GPU-backed PerMessageDeflateEncoder(compressionLevel, noContext): IEncoder<Frame,Frame>
    (PerMessageDeflateEncoder.java:39-100).  encode() of one frame runs a one-frame batch;
    BatchDeflater compresses whole batches of every session's outgoing frames."""

    def __init__(self, compressionLevel: int, noContext: bool, ctx: Context | None = None):
        self._b = BatchDeflater(1, compressionLevel, noContext, ctx)

    def getInboundType(self):
        return Frame

    def getOutboundType(self):
        return Frame

    def encode(self, session, frame: Frame, out: list):
        src = (int(frame.getOpcode()), frame.isFinalFragment(), frame.getRsvBits(), bytes(frame.getPayload()))
        op, fin, rsv, data, deflated = self._b.run([[src]], with_flags=True)[0][0]
        if not deflated:
            out.append(frame)   # allowEncoding false: the same frame object (DeflateEncoder.java:103)
        else:
            out.append(make_frame(op, fin, rsv, data))


class PerMessageDeflateDecoder:
    """GPU-backed PerMessageDeflateDecoder(noContext): IDecoder<Frame,Frame>
    (PerMessageDeflateDecoder.java:33-107).  decode() of one frame runs a one-frame
    batch (so every fragment crosses a batch boundary); BatchInflater inflates whole
    decoded batches."""

    def __init__(self, noContext: bool = False, ctx: Context | None = None):
        self._b = BatchInflater(1, noContext, ctx)

    def getInboundType(self):
        return Frame

    def getOutboundType(self):
        return Frame

    def decode(self, session, frame: Frame, out: list):
        payload = bytes(frame.getPayload())
        desc = np.zeros(1, dtype=DESC_DTYPE)
        desc[0]["payload_len"] = len(payload)
        desc[0]["opcode"] = int(frame.getOpcode())
        desc[0]["flags"] = (0x80 if frame.isFinalFragment() else 0) | ((frame.getRsvBits() & 7) << 4)
        frames, exc = self._b.run(desc, np.array([0, 1], np.uint32), np.frombuffer(payload, np.uint8))[0]
        if exc is not None:
            _writenf(session, CloseFrame.of_status(exc.close_code))  # protocolError (DeflateDecoder.java:64-72)
            raise exc
        for f in frames:
            out.append(f if f.inflated else frame)  # a frame not inflated is the same object (:140)
