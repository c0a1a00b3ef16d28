"""ctypes binding of the CPU ORACLE (oracle/libwsoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by snf4j_amd/.  The oracle restates
snf4j-websocket's FrameDecoder / Utf8 / FrameUtf8Validator / FrameEncoder
(see ws_oracle.h for the cited reference lines and how it is pinned).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libwsoracle.so")

# wsg_status values (include/wsgpu.h)
OK = 0
E_OPCODE, E_RSV, E_MASKING, E_FRAG_CONTROL, E_CONTROL_LEN, E_CLOSE_LEN = 1, 2, 3, 4, 5, 6
E_CONT_OUTSIDE, E_NONCONT_INSIDE, E_MIN_LEN, E_MAX_PAYLOAD, E_TOO_LONG = 7, 8, 9, 10, 11
E_CLOSE_STATUS, E_CLOSE_REASON, E_TEXT_UTF8, E_NEG_LEN, E_EXT_LEN, E_BATCH = 12, 13, 14, 15, 16, 17

DESC_DTYPE = np.dtype([("payload_off", "<u8"), ("payload_len", "<u4"), ("opcode", "u1"),
                       ("flags", "u1"), ("status", "<u2")])
RESULT_DTYPE = np.dtype([("n_delivered", "<u4"), ("error", "<u2"), ("close_code", "<u2"),
                         ("detail", "<i8")])


def build() -> str:
    """Compile the oracle (gcc) if it is missing or stale; returns the .so path."""
    src = [os.path.join(_HERE, f) for f in ("ws_oracle.c", "ws_oracle.h")]
    if (not os.path.exists(_LIB_PATH)
            or any(os.path.getmtime(s) > os.path.getmtime(_LIB_PATH) for s in src)):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        p, i64, i32, u32, u64 = C.c_void_p, C.c_int64, C.c_int, C.c_uint32, C.c_uint64
        P = C.POINTER
        L.or_utf8_validate.argtypes = [P(C.c_int * 2), p, i64]
        L.or_utf8_is_valid.argtypes = [p, i64]
        L.or_utf8_is_valid_batch.argtypes = [p, p, i64, p]
        L.or_utf8_reject_pos.argtypes = [i32, p, i64]
        L.or_utf8_reject_pos.restype = i64
        L.or_validator_decode.argtypes = [p, i32, i32, p, i64]
        L.or_decoder_new.argtypes = [i32, i32, i64, i32]
        L.or_decoder_new.restype = p
        L.or_decoder_free.argtypes = [p]
        L.or_decoder_closed.argtypes = [p]
        L.or_decoder_fragmentation.argtypes = [p]
        L.or_decoder_available.argtypes = [p, p, i64, P(i32), P(i64), P(i64)]
        L.or_decoder_available.restype = i64
        L.or_decoder_decode.argtypes = [p, p, i64, p, P(i32), P(i64), P(i32)]
        L.or_format_error.argtypes = [i32, i64, i64, C.c_char_p, i32]
        L.or_batch_new.argtypes = [i32, i32, i64, i32, u32]
        L.or_batch_new.restype = p
        L.or_batch_free.argtypes = [p]
        L.or_batch_decode.argtypes = [p, p, p, u64, p, u32, p, p, p]
        L.or_batch_decode.restype = i64
        L.or_stream_decode.argtypes = [i32, i32, i64, i32, p, i64, p, i32, p, p, i64,
                                       P(i32), P(i64), P(i64), P(i32)]
        L.or_stream_decode.restype = i64
        L.or_encoded_length.argtypes = [i64, i32]
        L.or_encoded_length.restype = i64
        L.or_encode.argtypes = [p, i32, i32, i32, p, i64, p, p]
        L.or_encode.restype = i64
        L.or_aggregator_init.argtypes = [p, i64]
        L.or_aggregator_free.argtypes = [p]
        L.or_aggregate.argtypes = [p, i32, i32, i32, p, i64, p]
        L.or_splitmix64.argtypes = [u64]
        L.or_splitmix64.restype = u64
        L.or_synth_uniform.argtypes = [u64, u64, u32, u32, i32, i32, i32, p, p, p]
        _lib = L
    return _lib


def _ptr(a) -> int:
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return C.cast(C.c_char_p(bytes(a)), C.c_void_p).value


def format_error(err: int, detail: int = 0, detail2: int = 0) -> str:
    buf = C.create_string_buffer(256)
    lib().or_format_error(err, detail, detail2, buf, 256)
    return buf.value.decode()


# ---------------------------------------------------------------- Utf8.java
def utf8_is_valid(data: bytes) -> bool:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    return bool(lib().or_utf8_is_valid(a.ctypes.data, len(data)))


def utf8_validate(state: list, data: bytes) -> bool:
    """Utf8.validate(ctx, data, 0, len); state = [state, codep] updated in place."""
    ctx = (C.c_int * 2)(*state)
    a = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    ok = bool(lib().or_utf8_validate(C.byref(ctx), a.ctypes.data, len(data)))
    state[0], state[1] = ctx[0], ctx[1]
    return ok


def utf8_is_valid_batch(strings_u8: np.ndarray, lengths: np.ndarray) -> np.ndarray:
    """Rows of a 2-D uint8 array, each valid for its length: returns bool array."""
    strings_u8 = np.ascontiguousarray(strings_u8, dtype=np.uint8)
    n, w = strings_u8.shape
    flat = strings_u8.reshape(-1)
    lengths = np.asarray(lengths, dtype=np.int64)
    # offsets of row i's string within flat, packed end-to-end: repack
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lengths, out=offs[1:])
    mask = np.arange(w)[None, :] < lengths[:, None]
    packed = np.ascontiguousarray(flat[mask.reshape(-1)])
    if packed.size == 0:
        packed = np.zeros(1, np.uint8)
    out = np.zeros(n, dtype=np.uint8)
    lib().or_utf8_is_valid_batch(packed.ctypes.data, offs.ctypes.data, n, out.ctypes.data)
    return out.astype(bool)


def utf8_reject_pos(data: bytes, state: int = 0) -> int:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    return int(lib().or_utf8_reject_pos(state, a.ctypes.data, len(data)))


# ---------------------------------------------------------------- FrameUtf8Validator
class _CVal(C.Structure):
    _fields_ = [("open", C.c_int), ("state", C.c_int), ("codep", C.c_int)]


class Validator:
    """FrameUtf8Validator alone; decode() returns False where the reference throws."""

    def __init__(self):
        self._v = _CVal(0, 0, 0)

    def decode(self, opcode, fin, payload: bytes) -> bool:
        p = bytes(payload)
        a = np.frombuffer(p, dtype=np.uint8) if p else np.zeros(1, np.uint8)
        return lib().or_validator_decode(C.byref(self._v), opcode, int(fin), a.ctypes.data, len(p)) == 0


# ---------------------------------------------------------------- FrameDecoder
class InvalidFrame(Exception):
    def __init__(self, err, detail=0, detail2=0, close_code=0):
        self.err, self.detail, self.detail2, self.close_code = err, detail, detail2, close_code
        super().__init__(format_error(err, detail, detail2))


class OracleFrame:
    def __init__(self, opcode, fin, rsv, payload):
        self.opcode, self.fin, self.rsv, self.payload = opcode, fin, rsv, payload

    def __repr__(self):
        return f"OracleFrame(op={self.opcode},fin={self.fin},rsv={self.rsv},len={len(self.payload)})"


class _CFrame(C.Structure):
    _fields_ = [("opcode", C.c_int), ("fin", C.c_int), ("rsv", C.c_int),
                ("len", C.c_int64), ("payload", C.c_void_p)]


class Decoder:
    """FrameDecoder(+FrameUtf8Validator) restated in C; raises InvalidFrame like the reference."""

    def __init__(self, client_mode, allow_extensions, max_payload_len, validate_utf8=True):
        self._h = lib().or_decoder_new(int(client_mode), int(allow_extensions),
                                       int(max_payload_len), int(validate_utf8))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_decoder_free(self._h)
            self._h = None

    @property
    def closed(self):
        return bool(lib().or_decoder_closed(self._h))

    def available(self, buf: bytes, off: int = 0, length: int | None = None) -> int:
        """available(session, buf, off, len).  `length` may exceed the bytes given
        (the reference tests pass Integer.MAX_VALUE with header-only arrays): only
        the header bytes are ever read."""
        b = bytes(buf)[off:]
        n = len(b) if length is None else int(length)
        a = np.frombuffer(b + bytes(16), dtype=np.uint8)
        err, d1, d2 = C.c_int(0), C.c_int64(0), C.c_int64(0)
        r = lib().or_decoder_available(self._h, a.ctypes.data, n, C.byref(err), C.byref(d1),
                                       C.byref(d2))
        if r < 0:
            raise InvalidFrame(err.value, d1.value, d2.value, 1002)
        return int(r)

    def decode(self, data: bytes):
        """Returns an OracleFrame, None (partial / closed), or raises InvalidFrame."""
        b = bytes(data)
        a = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8)
        f = _CFrame()
        err, det, cc = C.c_int(0), C.c_int64(0), C.c_int(0)
        rc = lib().or_decoder_decode(self._h, a.ctypes.data, len(b), C.byref(f), C.byref(err),
                                     C.byref(det), C.byref(cc))
        if rc == 1:
            payload = C.string_at(f.payload, f.len) if f.len else b""
            return OracleFrame(f.opcode, bool(f.fin), f.rsv, payload)
        if rc == 0:
            return None
        if rc == -1:
            raise InvalidFrame(err.value, det.value, 0, cc.value)
        raise ValueError("decode() contract violation (reference: BufferUnderflowException)")


class Batch:
    """or_batch: per-session decoders driven one complete frame per decode()."""

    def __init__(self, client_mode, allow_extensions, max_payload_len, validate_utf8, n_sessions):
        self.n_sessions = n_sessions
        self._h = lib().or_batch_new(int(client_mode), int(allow_extensions), int(max_payload_len),
                                     int(validate_utf8), n_sessions)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_batch_free(self._h)
            self._h = None

    def decode(self, wire: np.ndarray, frame_off: np.ndarray, session_first: np.ndarray):
        wire = np.ascontiguousarray(wire, dtype=np.uint8)
        frame_off = np.ascontiguousarray(frame_off, dtype=np.uint64)
        session_first = np.ascontiguousarray(session_first, dtype=np.uint32)
        n_frames = len(frame_off) - 1
        n_sessions = len(session_first) - 1
        payload = np.zeros(max(1, int(wire.size)), dtype=np.uint8)
        desc = np.zeros(max(1, n_frames), dtype=DESC_DTYPE)
        res = np.zeros(max(1, n_sessions), dtype=RESULT_DTYPE)
        w = wire if wire.size else np.zeros(1, np.uint8)
        n = lib().or_batch_decode(self._h, w.ctypes.data, frame_off.ctypes.data, n_frames,
                                  session_first.ctypes.data, n_sessions, payload.ctypes.data,
                                  desc.ctypes.data, res.ctypes.data)
        return payload[:n], desc[:n_frames], res[:n_sessions]


def stream_decode(stream: bytes, chunks=(), client_mode=False, allow_extensions=False,
                  max_payload_len=65536, validate_utf8=True, max_frames=1 << 20):
    """The session read loop over `stream`; returns (frames, error or None)."""
    b = bytes(stream)
    a = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8)
    ch = np.asarray(list(chunks) or [len(b) or 1], dtype=np.int64)
    payload = np.zeros(max(1, len(b)), dtype=np.uint8)
    desc = np.zeros(max(1, max_frames), dtype=DESC_DTYPE)
    err, d1, d2, cc = C.c_int(0), C.c_int64(0), C.c_int64(0), C.c_int(0)
    n = lib().or_stream_decode(int(client_mode), int(allow_extensions), int(max_payload_len),
                               int(validate_utf8), a.ctypes.data, len(b), ch.ctypes.data, len(ch),
                               payload.ctypes.data, desc.ctypes.data, max_frames, C.byref(err),
                               C.byref(d1), C.byref(d2), C.byref(cc))
    frames = []
    for k in range(n):
        d = desc[k]
        off, ln = int(d["payload_off"]), int(d["payload_len"])
        frames.append(OracleFrame(int(d["opcode"]), bool(d["flags"] & 0x80),
                                  (int(d["flags"]) >> 4) & 7, payload[off:off + ln].tobytes()))
    error = InvalidFrame(err.value, d1.value, d2.value, cc.value) if err.value else None
    return frames, error


# ---------------------------------------------------------------- FrameAggregator
class _CAgg(C.Structure):
    _fields_ = [("max_len", C.c_int64), ("open", C.c_int), ("opcode", C.c_int), ("rsv", C.c_int),
                ("length", C.c_int64), ("data", C.c_void_p), ("cap", C.c_int64)]


E_AGG_TOO_BIG = 18


class Aggregator:
    """FrameAggregator(maxAggregatedLength) restated in C (FrameAggregator.java:72-104).
    decode() returns the emitted OracleFrame, None, or raises InvalidFrame(18, close 1009)."""

    def __init__(self, max_aggregated_len):
        self._a = _CAgg()
        lib().or_aggregator_init(C.byref(self._a), int(max_aggregated_len))

    def __del__(self):
        if getattr(self, "_a", None) is not None:
            lib().or_aggregator_free(C.byref(self._a))
            self._a = None

    @property
    def state(self):
        return bool(self._a.open), int(self._a.opcode), int(self._a.rsv), int(self._a.length)

    def decode(self, opcode, fin, rsv, payload: bytes):
        b = bytes(payload)
        a = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8)
        f = _CFrame()
        rc = lib().or_aggregate(C.byref(self._a), int(opcode), int(bool(fin)), int(rsv), a.ctypes.data, len(b),
                                C.byref(f))
        if rc == -1:
            raise InvalidFrame(E_AGG_TOO_BIG, 0, 0, 1009)
        if rc == 0:
            return None
        return OracleFrame(f.opcode, bool(f.fin), f.rsv, C.string_at(f.payload, f.len) if f.len else b"")


# ---------------------------------------------------------------- permessage-deflate decode
E_INFLATE, E_INFLATE_NO_DATA = 19, 20
INFLATE_MESSAGE = ("org.snf4j.core.codec.zip.DecompressionException: "
                   "decompression failure: invalid compressed data format")


class _ZlibRawDecoder:
    """ZlibDecoder(Mode.RAW) (snf4j-core ZlibDecoder.java:180-280) over java.util.zip.Inflater,
    i.e. zlib's raw inflate.  The inflate itself is zlib's: Python's zlib module binds the same
    library (third-party dependency of the reference's JDK, version zlib.ZLIB_RUNTIME_VERSION);
    the wrapper logic (finished stream, leftover bytes) is restated from ZlibDecoder."""

    def __init__(self):
        import zlib
        self._zlib = zlib
        self.d = zlib.decompressobj(-15)
        self.finished = False

    def decode(self, data: bytes) -> list:
        if self.finished:              # :186-191: later data passes through
            return [data] if data else []
        if not data:                   # :193-195
            return []
        try:
            out = self.d.decompress(data)
        except self._zlib.error as e:  # DataFormatException -> DecompressionException (:255-257)
            raise InvalidFrame(E_INFLATE, 0, 0, 1002) from e
        bufs = [out] if out else []
        if self.d.eof:                 # inflater.finished(): postFinish, leftover input added (:262-270)
            self.finished = True
            if self.d.unused_data:
                bufs.append(self.d.unused_data)
        return bufs


class PerMessageDeflateDecoder:
    """PerMessageDeflateDecoder(noContext) + DeflateDecoder restated (PerMessageDeflateDecoder.java:
    68-105, DeflateDecoder.java:78-141).  decode() returns (opcode, fin, rsv, payload) or raises
    InvalidFrame (19: the DecompressionException, 20: "Inflating of input data produced no data")."""
    TAIL = b"\x00\x00\xff\xff"  # DeflateCodec.java:43

    def __init__(self, no_context: bool):
        self.no_context = bool(no_context)
        self.compressing = False
        self.decoder = None

    def decode(self, opcode, fin, rsv, payload: bytes):
        payload = bytes(payload)
        allow = (opcode in (1, 2) and (rsv & 4)) or (opcode == 0 and self.compressing)
        out = (opcode, bool(fin), rsv, payload)
        if allow:
            if self.decoder is None:
                self.decoder = _ZlibRawDecoder()
            bufs = self.decoder.decode(payload)
            if fin:                                   # appendTail (:78-80)
                bufs += self.decoder.decode(self.TAIL)
            if fin and self.no_context:
                self.decoder = None
            if not bufs:
                if len(payload) == 1 and payload[0] == 0:
                    data = b""
                else:
                    raise InvalidFrame(E_INFLATE_NO_DATA, 0, 0, 1002)
            else:
                data = b"".join(bufs)
            out = (opcode, bool(fin), rsv ^ 4 if rsv & 4 else rsv, data)   # rsvBits (:83-85)
        if opcode < 8:
            if fin:
                self.compressing = False
            elif (rsv & 4) and opcode in (1, 2):
                self.compressing = True
        return out


def deflate_message(comp, data: bytes, fin: bool) -> bytes:
    """PerMessageDeflateEncoder's payload for one fragment: zlib raw deflate with a sync
    flush; the trailing 00 00 FF FF is removed from a final fragment (DeflateEncoder)."""
    import zlib
    b = comp.compress(data) + comp.flush(zlib.Z_SYNC_FLUSH)
    if fin and b.endswith(b"\x00\x00\xff\xff"):
        b = b[:-4]
    return b


# ---------------------------------------------------------------- FrameEncoder
class _CEnc(C.Structure):
    _fields_ = [("client_mode", C.c_int), ("closed", C.c_int)]


class Encoder:
    def __init__(self, client_mode):
        self._e = _CEnc(int(client_mode), 0)

    def encode(self, opcode, fin, rsv, payload: bytes, mask=(0, 0, 0, 0)) -> bytes:
        p = bytes(payload)
        a = np.frombuffer(p, dtype=np.uint8) if p else np.zeros(1, np.uint8)
        m = np.asarray(mask, dtype=np.uint8)
        out = np.zeros(len(p) + 14, dtype=np.uint8)
        n = lib().or_encode(C.byref(self._e), opcode, int(fin), rsv, a.ctypes.data, len(p),
                            m.ctypes.data, out.ctypes.data)
        return out[:n].tobytes()


def encoded_length(payload_len: int, client_mode: bool) -> int:
    return int(lib().or_encoded_length(payload_len, int(client_mode)))


# ---------------------------------------------------------------- synthetic data
def splitmix64(x: int) -> int:
    return int(lib().or_splitmix64(x & 0xFFFFFFFFFFFFFFFF))


def synth_uniform(seed, n_frames, payload_len, frames_per_session, opcode=2, masked=True,
                  text=False):
    flen = encoded_length(payload_len, masked)
    n_sessions = (n_frames + frames_per_session - 1) // frames_per_session
    wire = np.zeros(n_frames * flen + 1, dtype=np.uint8)
    frame_off = np.zeros(n_frames + 1, dtype=np.uint64)
    session_first = np.zeros(n_sessions + 1, dtype=np.uint32)
    lib().or_synth_uniform(seed, n_frames, payload_len, frames_per_session, opcode, int(masked),
                           int(text), wire.ctypes.data, frame_off.ctypes.data,
                           session_first.ctypes.data)
    return wire[:n_frames * flen], frame_off, session_first
