"""Context: a libwsgpu context on one GPU, with device-resident and host batch calls.

Device buffers are torch tensors (plumbing only: HIP allocations + the stream);
all work runs in libwsgpu's HIP kernels.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import AGG_STATE_DTYPE, DESC_DTYPE, ENCODE_DTYPE, RESULT_DTYPE, STATE_DTYPE, DecoderCfg, check, lib

DEFLATE_SESSION_BYTES = 65536 + 2 * 32768 * 2   # WSG_DEFLATE_SESSION_BYTES: window + head + prev

MESSAGES = {
    1: "Unexpected opcode value ({d})",
    2: "Unexpected non-zero RSV bits ({d})",
    3: "Unexpected payload masking",
    4: "Fragmented control frame",
    5: "Invalid payload length ({d}) in control frame",
    6: "Invalid payload length ({d}) in close frame",
    7: "Continuation frame outside fragmented message",
    8: "Non-continuation frame while inside fragmented massage",
    9: "Invalid minimal payload length",
    10: "Invalid maximum payload length",
    11: "Maximum frame length ({d}) has been exceeded",
    12: "Invalid close frame status code ({d})",
    13: "Invalid close frame reason value: bytes are not UTF-8",
    14: "Invalid text frame payload: bytes are not UTF-8",
    15: "Negative payload length ({d})",
    16: "Extended payload length ({d}) > {d2}",
    17: "Malformed batch (frame extent does not match its header)",
    18: "Too big payload for aggregated frame",
    19: "org.snf4j.core.codec.zip.DecompressionException: decompression failure: invalid compressed data format",
    20: "Inflating of input data produced no data",
    21: "Inflate output region too small (batch contract)",
}


def error_message(code: int, detail: int = 0, detail2: int = 0) -> str:
    """The InvalidFrameException message the reference builds for a wsg_status
    (FrameDecoder.java:200-255, :390-393; FrameUtf8Validator.java:31)."""
    return MESSAGES[int(code)].format(d=int(detail), d2=int(detail2))


def decoder_cfg(client_mode: bool, allow_extensions: bool, max_payload_len: int,
                validate_utf8: bool = True) -> DecoderCfg:
    return DecoderCfg(int(bool(client_mode)), int(bool(allow_extensions)), int(max_payload_len),
                      int(bool(validate_utf8)), 0)


def _p(a) -> int:
    """Device pointer of a torch tensor, host pointer of a numpy array."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


def _stream_handle(stream) -> int:
    return int(stream) if isinstance(stream, int) else int(stream.cuda_stream)


class Context:
    """A libwsgpu context on one device.

    stream: "torch" (default) = torch's current stream on `device`, so the codec's
    kernels are ordered with the torch operations that fill and free the device
    buffers; "own" = a private non-blocking stream; or a hipStream_t handle /
    torch.cuda.Stream.  Torch's default stream has handle 0, which is passed on
    with wsg_set_stream (wsg_open(NULL) would create a private stream instead)."""

    TUNING = {"inflate_tokens": 1, "inflate_fast": 2, "inflate_lds": 3, "inflate_order": 4, "inflate_lanes": 5,
              "fused_scan": 6, "agg_units": 7, "agg_grid": 8, "inflate_tabs": 9, "inflate_split": 10,
              "agg_fold_max": 11, "deflate_serial": 12, "stage_fail": 13,
              "deflate_lds": 14}

    def set_tuning(self, name: str, value: int):
        """A measurement / test switch of this context (wsg_set_tuning; wsgpu.h lists them)."""
        check(lib.wsg_set_tuning(self._h, self.TUNING[name], int(value)), self._h)

    def __init__(self, device: int = 0, stream="torch"):
        h = C.c_void_p()
        rc = lib.wsg_open(int(device), None, C.byref(h))
        if rc != 0:
            raise _lib.WsgError(f"wsg_open(device={device}) failed: {rc} (no HIP device?)")
        self._h = h
        self.device = device
        if isinstance(stream, str) and stream == "torch":
            import torch
            stream = torch.cuda.current_stream(device)
        if not (isinstance(stream, str) and stream == "own"):
            self.set_stream(stream)

    # -------------------------------------------------------------- plumbing
    def close(self):
        if getattr(self, "_h", None):
            lib.wsg_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_stream(self, stream):
        check(lib.wsg_set_stream(self._h, C.c_void_p(_stream_handle(stream))), self._h)

    @property
    def stream_handle(self) -> int:
        """The hipStream_t the context enqueues on (wsg_get_stream)."""
        h = C.c_void_p()
        check(lib.wsg_get_stream(self._h, C.byref(h)), self._h)
        return int(h.value or 0)

    def sync(self):
        check(lib.wsg_sync(self._h), self._h)

    def reserve(self, max_frames: int, max_sessions: int, max_wire_len: int = 0):
        check(lib.wsg_reserve(self._h, int(max_frames), int(max_sessions), int(max_wire_len)), self._h)

    def reserve_inflate(self, max_frames: int, max_sessions: int, max_payload_len: int):
        """wsg_reserve_inflate: pre-size the permessage-deflate workspace."""
        check(lib.wsg_reserve_inflate(self._h, int(max_frames), int(max_sessions), int(max_payload_len)), self._h)

    def inflate_split_count(self) -> int:
        """wsg_inflate_split_count: messages the split-lane decode took on this context."""
        n = C.c_uint64()
        check(lib.wsg_inflate_split_count(self._h, C.byref(n)), self._h)
        return int(n.value)

    def set_timing(self, on=True):
        """True: time every kernel; "hot": only the streaming kernels (an event pair
        costs queue time, so timed steps bracket only the kernel the roofline needs)."""
        check(lib.wsg_set_timing(self._h, 2 if on == "hot" else int(bool(on))), self._h)

    def set_timing_every(self, every: int):
        """'hot' timing brackets one launch in `every` of each streaming kernel."""
        check(lib.wsg_set_timing_every(self._h, int(every)), self._h)

    def reset_timing(self):
        check(lib.wsg_reset_timing(self._h), self._h)

    def timing(self) -> dict:
        n = lib.wsg_num_kernels()
        ms = (C.c_double * n)()
        cnt = (C.c_uint64 * n)()
        lib.wsg_get_timing(self._h, ms, cnt, n)
        return {lib.wsg_kernel_name(i).decode(): (ms[i], cnt[i]) for i in range(n)}

    # -------------------------------------------------------------- decode
    def decode_device(self, cfg: DecoderCfg, wire, frame_off, session_first, state, payload_out, desc_out,
                      result_out, wire_len: int | None = None):
        """Enqueue a device-resident batch decode (all arguments cuda tensors)."""
        n_frames = frame_off.numel() - 1
        n_sessions = session_first.numel() - 1
        wl = wire.numel() if wire_len is None else int(wire_len)
        check(lib.wsg_decode_batch_device(self._h, C.byref(cfg), _p(wire), wl, _p(frame_off), n_frames,
                                          _p(session_first), n_sessions, _p(state), _p(payload_out),
                                          payload_out.numel(), _p(desc_out), _p(result_out)), self._h)

    def decode_host(self, cfg: DecoderCfg, wire: np.ndarray, frame_off: np.ndarray, session_first: np.ndarray,
                    state: np.ndarray):
        """Host batch decode (H2D, kernels, D2H). `state` (STATE_DTYPE) is updated in place.
        Returns (payload, desc, result)."""
        wire = np.ascontiguousarray(wire, dtype=np.uint8)
        frame_off = np.ascontiguousarray(frame_off, dtype=np.uint64)
        session_first = np.ascontiguousarray(session_first, dtype=np.uint32)
        assert state.dtype == STATE_DTYPE and state.flags.c_contiguous
        n_frames = len(frame_off) - 1
        n_sessions = len(session_first) - 1
        cap = int(lib.wsg_decode_payload_bound(wire.size, n_frames))
        payload = np.zeros(cap, dtype=np.uint8)
        desc = np.zeros(max(1, n_frames), dtype=DESC_DTYPE)
        result = np.zeros(max(1, n_sessions), dtype=RESULT_DTYPE)
        w = wire if wire.size else np.zeros(1, np.uint8)
        check(lib.wsg_decode_batch_host(self._h, C.byref(cfg), w.ctypes.data, wire.size, frame_off.ctypes.data,
                                        n_frames, session_first.ctypes.data, n_sessions, state.ctypes.data,
                                        payload.ctypes.data, cap, desc.ctypes.data, result.ctypes.data), self._h)
        return payload, desc[:n_frames], result[:n_sessions]

    def decode_host_async(self, cfg: DecoderCfg, wire, frame_off, session_first, state, payload, desc, result,
                          wire_len: int | None = None):
        """Enqueue H2D + decode + D2H of a host batch and return (wsg_decode_batch_host_async).
        All buffers are host tensors/arrays (pinned for real overlap) that must stay alive
        until sync(); `payload` holds >= wire_len + 16 * n_frames bytes."""
        n_frames = int(np.prod(frame_off.shape)) - 1
        n_sessions = int(np.prod(session_first.shape)) - 1
        wl = int(np.prod(wire.shape)) if wire_len is None else int(wire_len)
        check(lib.wsg_decode_batch_host_async(self._h, C.byref(cfg), _p(wire), wl, _p(frame_off), n_frames,
                                              _p(session_first), n_sessions, _p(state), _p(payload),
                                              int(np.prod(payload.shape)), _p(desc), _p(result)), self._h)

    # -------------------------------------------------------------- validate (FrameUtf8Validator alone)
    def validate_device(self, desc, session_first, payload, state, result_out, n_frames: int | None = None,
                        payload_len: int | None = None):
        """Enqueue the standalone UTF-8 validator stage over plain payloads (wsg_validate_batch_device)."""
        n = desc.numel() // DESC_DTYPE.itemsize if n_frames is None else int(n_frames)
        pl = payload.numel() if payload_len is None else int(payload_len)
        check(lib.wsg_validate_batch_device(self._h, _p(desc), n, _p(session_first), session_first.numel() - 1,
                                            _p(payload), pl, _p(state), _p(result_out)), self._h)

    def validate_host(self, desc: np.ndarray, session_first: np.ndarray, payload: np.ndarray, state: np.ndarray):
        """FrameUtf8Validator over a host batch of plain payloads; `state` updated in place.
        Returns the per-session results."""
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        session_first = np.ascontiguousarray(session_first, dtype=np.uint32)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        assert state.dtype == STATE_DTYPE and state.flags.c_contiguous
        n, n_s = len(desc), len(session_first) - 1
        res = np.zeros(max(1, n_s), dtype=RESULT_DTYPE)
        d = desc if n else np.zeros(1, DESC_DTYPE)
        pl = payload if payload.size else np.zeros(16, np.uint8)
        check(lib.wsg_validate_batch_host(self._h, d.ctypes.data, n, session_first.ctypes.data, n_s, pl.ctypes.data,
                                          payload.size, state.ctypes.data, res.ctypes.data), self._h)
        return res[:n_s]

    # -------------------------------------------------------------- inflate (permessage-deflate decode)
    def inflate_device(self, no_context: bool, desc, session_first, payload, state, window, out, out_off, out_desc,
                       out_result, replay_from, n_frames: int | None = None):
        """Enqueue PerMessageDeflateDecoder over a decoded device batch (wsg_inflate_batch_device);
        all arguments cuda tensors (desc / state / results as uint8 byte views, out_off int64)."""
        n = desc.numel() // DESC_DTYPE.itemsize if n_frames is None else int(n_frames)
        n_s = session_first.numel() - 1
        assert window.numel() >= n_s * 32768 and out_off.numel() == n_s + 1
        check(lib.wsg_inflate_batch_device(self._h, int(bool(no_context)), _p(desc), n, _p(session_first), n_s,
                                           _p(payload), payload.numel(), _p(state), _p(window), _p(out), _p(out_off),
                                           _p(out_desc), _p(out_result), _p(replay_from)), self._h)

    def inflate_host(self, no_context: bool, desc: np.ndarray, session_first: np.ndarray, payload: np.ndarray,
                     state: np.ndarray, window: np.ndarray, out_off: np.ndarray):
        """PerMessageDeflateDecoder over a host batch of decoded frames (wsg_inflate_batch_host).
        `state` (INFLATE_STATE_DTYPE) and `window` (uint8, n_sessions x 32768) are updated in
        place.  Returns (out, out_desc, results, replay_from)."""
        from ._lib import INFLATE_STATE_DTYPE
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        session_first = np.ascontiguousarray(session_first, dtype=np.uint32)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
        assert state.dtype == INFLATE_STATE_DTYPE and state.flags.c_contiguous
        assert window.dtype == np.uint8 and window.flags.c_contiguous
        n, n_s = len(desc), len(session_first) - 1
        assert window.size >= n_s * 32768 and len(out_off) == n_s + 1
        out = np.zeros(max(1, int(out_off[-1])), dtype=np.uint8)
        odesc = np.zeros(max(1, n), dtype=DESC_DTYPE)
        res = np.zeros(max(1, n_s), dtype=RESULT_DTYPE)
        rf = np.zeros(max(1, n_s), dtype=np.uint32)
        d = desc if n else np.zeros(1, DESC_DTYPE)
        pl = payload if payload.size else np.zeros(16, np.uint8)
        check(lib.wsg_inflate_batch_host(self._h, int(bool(no_context)), d.ctypes.data, n, session_first.ctypes.data,
                                         n_s, pl.ctypes.data, payload.size, state.ctypes.data, window.ctypes.data,
                                         out.ctypes.data, out_off.ctypes.data, odesc.ctypes.data, res.ctypes.data,
                                         rf.ctypes.data), self._h)
        return out, odesc[:n], res[:n_s], rf[:n_s]

    # -------------------------------------------------------------- deflate (permessage-deflate encode)
    def deflate_device(self, level: int, no_context: bool, desc, session_first, payload, state, session_mem, out,
                       out_desc, n_frames: int | None = None) -> int:
        """PerMessageDeflateEncoder over a device batch of outgoing frames (wsg_deflate_batch_device);
        all arguments cuda tensors (desc / state as uint8 byte views, session_mem uint8 of
        n_sessions x SESSION_BYTES).  Synchronises once; returns the out bytes used."""
        n = desc.numel() // DESC_DTYPE.itemsize if n_frames is None else int(n_frames)
        n_s = session_first.numel() - 1
        assert session_mem.numel() >= n_s * DEFLATE_SESSION_BYTES and state.numel() >= n_s * 16
        tot = C.c_uint64(0)
        check(lib.wsg_deflate_batch_device(self._h, int(level), int(bool(no_context)), _p(desc), n, _p(session_first),
                                           n_s, _p(payload), payload.numel(), _p(state), _p(session_mem), _p(out),
                                           out.numel(), _p(out_desc), C.byref(tot)), self._h)
        return int(tot.value)

    def deflate_host(self, level: int, no_context: bool, desc: np.ndarray, session_first: np.ndarray,
                     payload: np.ndarray, state: np.ndarray, session_mem: np.ndarray):
        """PerMessageDeflateEncoder over a host batch (wsg_deflate_batch_host).  `state`
        (DEFLATE_STATE_DTYPE) and `session_mem` (uint8, n_sessions x SESSION_BYTES) are updated
        in place.  Returns (out, out_desc)."""
        from ._lib import DEFLATE_STATE_DTYPE
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        session_first = np.ascontiguousarray(session_first, dtype=np.uint32)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        assert state.dtype == DEFLATE_STATE_DTYPE and state.flags.c_contiguous
        assert session_mem.dtype == np.uint8 and session_mem.flags.c_contiguous
        n, n_s = len(desc), len(session_first) - 1
        assert session_mem.size >= n_s * DEFLATE_SESSION_BYTES
        lens = desc["payload_len"].astype(np.uint64)
        cap = int((((lens + ((lens + 7) >> 3) + ((lens + 63) >> 6) + 15 + 15) >> 4) << 4).sum()) + 16 * n + 16
        out = np.zeros(cap, dtype=np.uint8)
        odesc = np.zeros(max(1, n), dtype=DESC_DTYPE)
        d = desc if n else np.zeros(1, DESC_DTYPE)
        pl = payload if payload.size else np.zeros(16, np.uint8)
        tot = C.c_uint64(0)
        check(lib.wsg_deflate_batch_host(self._h, int(level), int(bool(no_context)), d.ctypes.data, n,
                                         session_first.ctypes.data, n_s, pl.ctypes.data, payload.size,
                                         state.ctypes.data, session_mem.ctypes.data, out.ctypes.data, cap,
                                         odesc.ctypes.data, C.byref(tot)), self._h)
        return out[:int(tot.value)], odesc[:n]

    # -------------------------------------------------------------- handshake
    def handshake_accept_device(self, cfg, req, req_off, resp, result, n: int | None = None):
        """Enqueue the server handshake over a device batch (wsg_handshake_accept_batch_device):
        req uint8, req_off int64 (n + 1), resp uint8 (n * HS_RESP_STRIDE), result uint8 byte view
        (n * 16), all cuda tensors."""
        n = req_off.numel() - 1 if n is None else int(n)
        assert resp.numel() >= n * _lib.HS_RESP_STRIDE and result.numel() >= n * 16
        check(lib.wsg_handshake_accept_batch_device(self._h, C.byref(cfg), _p(req), _p(req_off), n, _p(resp),
                                                    _p(result)), self._h)

    def handshake_accept_host(self, cfg, req: np.ndarray, req_off: np.ndarray):
        """The server handshake over a host batch (wsg_handshake_accept_batch_host).
        Returns (resp [n, HS_RESP_STRIDE] uint8, result HS_RESULT_DTYPE[n])."""
        from ._lib import HS_RESULT_DTYPE
        req = np.ascontiguousarray(req, dtype=np.uint8)
        req_off = np.ascontiguousarray(req_off, dtype=np.uint64)
        n = len(req_off) - 1
        resp = np.zeros((max(1, n), _lib.HS_RESP_STRIDE), dtype=np.uint8)
        res = np.zeros(max(1, n), dtype=HS_RESULT_DTYPE)
        r = req if req.size else np.zeros(16, np.uint8)
        check(lib.wsg_handshake_accept_batch_host(self._h, C.byref(cfg), r.ctypes.data, req_off.ctypes.data, n,
                                                  resp.ctypes.data, res.ctypes.data), self._h)
        return resp[:n], res[:n]

    def handshake_validate_device(self, cfg, resp, resp_off, keys, expected, result, n: int | None = None):
        """Enqueue the client handshake over a device batch (wsg_handshake_validate_batch_device):
        resp uint8, resp_off int64 (n + 1), keys uint8 (n * 24), expected uint8
        (n * HS_EXPECTED_STRIDE), result uint8 byte view (n * 16), all cuda tensors."""
        n = resp_off.numel() - 1 if n is None else int(n)
        assert keys.numel() >= n * 24 and expected.numel() >= n * _lib.HS_EXPECTED_STRIDE and result.numel() >= n * 16
        check(lib.wsg_handshake_validate_batch_device(self._h, C.byref(cfg), _p(resp), _p(resp_off), _p(keys), n,
                                                      _p(expected), _p(result)), self._h)

    def handshake_validate_host(self, cfg, resp: np.ndarray, resp_off: np.ndarray, keys: np.ndarray):
        """The client handshake over a host batch (wsg_handshake_validate_batch_host).
        Returns (expected [n, HS_EXPECTED_STRIDE] uint8, result HS_RESULT_DTYPE[n])."""
        from ._lib import HS_RESULT_DTYPE
        resp = np.ascontiguousarray(resp, dtype=np.uint8)
        resp_off = np.ascontiguousarray(resp_off, dtype=np.uint64)
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = len(resp_off) - 1
        assert keys.size >= n * 24
        exp = np.zeros((max(1, n), _lib.HS_EXPECTED_STRIDE), dtype=np.uint8)
        res = np.zeros(max(1, n), dtype=HS_RESULT_DTYPE)
        r = resp if resp.size else np.zeros(16, np.uint8)
        k = keys if keys.size else np.zeros(24, np.uint8)
        check(lib.wsg_handshake_validate_batch_host(self._h, C.byref(cfg), r.ctypes.data, resp_off.ctypes.data,
                                                    k.ctypes.data, n, exp.ctypes.data, res.ctypes.data), self._h)
        return exp[:n], res[:n]

    # -------------------------------------------------------------- aggregate
    def aggregate_device(self, max_aggregated_len: int, desc, session_first, dec_result, payload, state, agg_out,
                         out_desc, out_result, agg_total, n_frames: int | None = None):
        """Enqueue FrameAggregator over a decoded device batch (wsg_aggregate_batch_device);
        all arguments cuda tensors (desc / results / state as uint8 byte views)."""
        n = desc.numel() // DESC_DTYPE.itemsize if n_frames is None else int(n_frames)
        n_s = session_first.numel() - 1
        check(lib.wsg_aggregate_batch_device(self._h, int(max_aggregated_len), _p(desc), n, _p(session_first), n_s,
                                             _p(dec_result), _p(payload), payload.numel(), _p(state), _p(agg_out),
                                             agg_out.numel(), _p(out_desc), _p(out_result), _p(agg_total)), self._h)

    def aggregate_host(self, max_aggregated_len: int, desc: np.ndarray, session_first: np.ndarray,
                       dec_result: np.ndarray, payload: np.ndarray, state: np.ndarray):
        """FrameAggregator over a decoded host batch (wsg_aggregate_batch_host).  `state`
        (AGG_STATE_DTYPE) is updated in place.  Returns (agg_out, out_desc, out_result):
        session s's outputs are out_desc[session_first[s] + s + i]."""
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        session_first = np.ascontiguousarray(session_first, dtype=np.uint32)
        dec_result = np.ascontiguousarray(dec_result, dtype=RESULT_DTYPE)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        assert state.dtype == AGG_STATE_DTYPE and state.flags.c_contiguous
        n, n_s = len(desc), len(session_first) - 1
        cap = int(desc["payload_len"].astype(np.uint64).sum()) + 16
        agg = np.zeros(cap, dtype=np.uint8)
        out_desc = np.zeros(n + n_s + 1, dtype=DESC_DTYPE)
        out_res = np.zeros(max(1, n_s), dtype=RESULT_DTYPE)
        total = C.c_uint64(0)
        d = desc if n else np.zeros(1, DESC_DTYPE)
        pl = payload if payload.size else np.zeros(16, np.uint8)
        check(lib.wsg_aggregate_batch_host(self._h, int(max_aggregated_len), d.ctypes.data, n,
                                           session_first.ctypes.data, n_s, dec_result.ctypes.data, pl.ctypes.data,
                                           payload.size, state.ctypes.data, agg.ctypes.data, cap,
                                           out_desc.ctypes.data, out_res.ctypes.data, C.byref(total)), self._h)
        return agg[:total.value], out_desc[:n + n_s], out_res[:n_s]

    # -------------------------------------------------------------- encode
    def encode_device(self, client_mode: bool, payload, frames, session_first, closed, wire_out, wire_off):
        n_frames = frames.numel() // ENCODE_DTYPE.itemsize if frames.dtype.itemsize == 1 else frames.shape[0]
        n_sessions = session_first.numel() - 1
        check(lib.wsg_encode_batch_device(self._h, int(client_mode), _p(payload), payload.numel(), _p(frames),
                                          n_frames, _p(session_first), n_sessions, _p(closed), _p(wire_out),
                                          wire_out.numel(), _p(wire_off)), self._h)

    def encode_host(self, client_mode: bool, payload: np.ndarray, frames: np.ndarray, session_first: np.ndarray,
                    closed: np.ndarray):
        """Host batch encode; `closed` (uint8 per session) updated in place.
        Returns (wire, wire_off)."""
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        frames = np.ascontiguousarray(frames, dtype=ENCODE_DTYPE)
        session_first = np.ascontiguousarray(session_first, dtype=np.uint32)
        n_frames, n_sessions = len(frames), len(session_first) - 1
        cap = int(sum(int(lib.wsg_encoded_length(int(f), int(client_mode))) for f in frames["payload_len"])) + 16
        wire = np.zeros(cap, dtype=np.uint8)
        wire_off = np.zeros(n_frames + 1, dtype=np.uint64)
        p = payload if payload.size else np.zeros(1, np.uint8)
        fr = frames if n_frames else np.zeros(1, ENCODE_DTYPE)
        check(lib.wsg_encode_batch_host(self._h, int(client_mode), p.ctypes.data, payload.size, fr.ctypes.data,
                                        n_frames, session_first.ctypes.data, n_sessions, closed.ctypes.data,
                                        wire.ctypes.data, cap, wire_off.ctypes.data), self._h)
        return wire[:int(wire_off[-1])], wire_off


def frame_available(buf: bytes, length: int | None = None):
    """wsg_frame_available: FrameDecoder.available(session, byte[], off, len) without
    a pending payload. Returns (n, err, detail, detail2)."""
    b = bytes(buf) + bytes(16)
    n = len(buf) if length is None else int(length)
    a = np.frombuffer(b, dtype=np.uint8)
    err, d1, d2 = C.c_int32(0), C.c_int64(0), C.c_int64(0)
    r = lib.wsg_frame_available(a.ctypes.data, n, C.byref(err), C.byref(d1), C.byref(d2))
    return int(r), int(err.value), int(d1.value), int(d2.value)


def check_header(cfg: DecoderCfg, fragmentation: bool, buf: bytes):
    a = np.frombuffer(bytes(buf) + bytes(16), dtype=np.uint8)
    d = C.c_int64(0)
    e = lib.wsg_check_header(C.byref(cfg), int(bool(fragmentation)), a.ctypes.data, len(buf), C.byref(d))
    return int(e), int(d.value)


def encoded_length(payload_len: int, client_mode: bool) -> int:
    return int(lib.wsg_encoded_length(int(payload_len), int(bool(client_mode))))
