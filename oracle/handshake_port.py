"""ctypes binding of oracle/handshake_port.c, the compiled CPU port of the opening
handshake (bench.py's cpu_baseline, kind "port"; tests/test_handshake_port.py checks it
against oracle/handshake_oracle.py).  TEST / BENCH INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_LIB = None
UNSUPPORTED, NEED_MORE, PARSE_ERROR, ACCEPT, FINISHED, CLOSING = -1, 0, 2, 3, 4, 5


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhsport.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-s", "-C", os.path.dirname(path), "libhsport.so"], check=True)
        L = C.CDLL(path)
        L.hsp_accept.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_int)]
        L.hsp_accept.restype = C.c_int
        L.hsp_validate.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        L.hsp_validate.restype = C.c_int
        L.hsp_rate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.c_double,
                               C.POINTER(C.c_uint64)]
        L.hsp_rate.restype = C.c_double
        _LIB = L
    return _LIB


def accept(data: bytes):
    """(kind, status, response bytes) of one request."""
    resp = C.create_string_buffer(512)
    rl, st = C.c_size_t(), C.c_int()
    k = lib().hsp_accept(data, len(data), resp, C.byref(rl), C.byref(st))
    return k, st.value, resp.raw[:rl.value]


def validate(data: bytes, key: str) -> int:
    return lib().hsp_validate(data, len(data), key.encode(), len(key))


def rate(buf: np.ndarray, off: np.ndarray, keys: np.ndarray | None, threads: int, seconds: float):
    """(handshakes per second, handshakes done) on `threads` host threads; buf: the
    requests (or responses) back to back, off: their n + 1 offsets, keys: 24 B a response
    (client side) or None."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    kp = np.ascontiguousarray(keys, dtype=np.uint8).ctypes.data if keys is not None else None
    done = C.c_uint64()
    r = lib().hsp_rate(buf.ctypes.data, off.ctypes.data, kp, len(off) - 1, int(threads), float(seconds),
                       C.byref(done))
    if r < 0:
        raise RuntimeError("the handshake port rejected a request of the sample")
    return r, int(done.value)
