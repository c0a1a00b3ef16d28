"""ctypes binding of the permessage-deflate compression ORACLE (oracle/libdeflateref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by snf4j_amd/.  deflate_ref.c drives the system zlib (the
engine java.util.zip.Deflater wraps) exactly as PerMessageDeflateEncoder / DeflateEncoder
/ ZlibEncoder drive Deflater (PerMessageDeflateEncoder.java:55-99, DeflateEncoder.java:
62-104, ZlibEncoder.java:158-287): one deflate(Z_SYNC_FLUSH) per non-empty frame into a
deflateBound(len) buffer, the 00 00 FF FF tail removed from a final fragment, 00 for an
empty payload, RSV1 on TEXT/BINARY.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libdeflateref.so")
_lib = None


def build() -> str:
    src = os.path.join(_HERE, "deflate_ref.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(src) > os.path.getmtime(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE, "libdeflateref.so"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        p, i32, u32, u64, i64 = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64, C.c_int64
        L.dref_open.argtypes = [i32, i32]
        L.dref_open.restype = p
        L.dref_close.argtypes = [p]
        L.dref_encode_frame.argtypes = [p, i32, i32, i32, p, u64, p, u64, C.POINTER(C.c_int)]
        L.dref_encode_frame.restype = i64
        L.dref_stream_bytes.argtypes = [i32, u32, p, p, p, u64]
        L.dref_stream_bytes.restype = i64
        _lib = L
    return _lib


class PerMessageDeflateEncoderRef:
    """One session's PerMessageDeflateEncoder(level, noContext), state kept across calls."""

    def __init__(self, level: int = 6, no_context: bool = False):
        self._h = lib().dref_open(level, 1 if no_context else 0)
        if not self._h:
            raise ValueError("bad level")

    def close(self):
        if self._h:
            lib().dref_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def encode(self, opcode: int, fin: bool, rsv: int, payload: bytes) -> tuple[int, bytes]:
        """(rsv after encoding, payload after encoding) of one frame."""
        payload = bytes(payload)
        cap = len(payload) + (len(payload) >> 3) + (len(payload) >> 6) + 64
        out = C.create_string_buffer(cap)
        r = C.c_int(0)
        n = lib().dref_encode_frame(self._h, opcode, 1 if fin else 0, rsv, payload, len(payload), out, cap,
                                    C.byref(r))
        if n < 0:
            raise RuntimeError("zlib deflate failed")
        return r.value, out.raw[:n]


def encode_frames(frames, level=6, no_context=False):
    """[(opcode, fin, rsv, payload)] -> [(opcode, fin, rsv', payload')] for one session."""
    enc = PerMessageDeflateEncoderRef(level, no_context)
    try:
        out = []
        for op, fin, rsv, p in frames:
            r, b = enc.encode(op, fin, rsv, p)
            out.append((op, fin, r, b))
        return out
    finally:
        enc.close()


def stream_bytes(level: int, lens: np.ndarray, data: np.ndarray) -> int:
    """zlib deflate(SYNC_FLUSH) over one context-takeover stream of len(lens) calls (the
    CPU baseline's unit of work); returns the compressed byte count."""
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    cap = int(lens.max(initial=0)) * 2 + 64
    scratch = np.empty(cap, np.uint8)
    n = lib().dref_stream_bytes(level, len(lens), lens.ctypes.data, data.ctypes.data, scratch.ctypes.data, cap)
    if n < 0:
        raise RuntimeError("zlib deflate failed")
    return int(n)
