"""ctypes binding of tests/cpp/deflate_host.cpp (test infrastructure): the GPU deflate
algorithm (snf4j_amd/csrc/deflate_core.h) run on the host, serially (mode 0) or in the
decomposed form the GPU uses for levels 4-9 (mode 1), plus input generators shared by the
host and GPU deflate tests."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpp", "deflate_host.cpp")
DEPS = [SRC, os.path.join(HERE, "..", "snf4j_amd", "csrc", "deflate_core.h"),
        os.path.join(HERE, "..", "snf4j_amd", "csrc", "deflate_pmd.h"), os.path.join(HERE, "..", "include", "wsgpu.h")]
OUT = os.path.join(HERE, "cpp", "_build", "libzdh.so")
STATE_BYTES = 16
SESSION_BYTES = 65536 + 2 * 32768 * 2
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in DEPS):
            os.makedirs(os.path.dirname(OUT), exist_ok=True)
            subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-Werror", "-o",
                            OUT + ".tmp", SRC], check=True)
            os.replace(OUT + ".tmp", OUT)
        L = C.CDLL(OUT)
        p = C.c_void_p
        L.zdh_session.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint32, p, p, p, p, p, p, p, p, p, p, p, C.c_uint64,
                                  p, p]
        _lib = L
    return _lib


def new_state():
    """(wsg_deflate_state bytes, window, head, prev) of a new session."""
    return (np.zeros(STATE_BYTES, np.uint8), np.zeros(65536, np.uint8), np.zeros(32768, np.uint16),
            np.zeros(32768, np.uint16))


def run_session(frames, level, no_context, mode, state=None):
    """frames [(opcode, fin, rsv, payload)] of one session -> ([(opcode, fin, rsv', payload')], state)."""
    n = len(frames)
    op = np.array([f[0] for f in frames], np.uint8)
    fin = np.array([1 if f[1] else 0 for f in frames], np.uint8)
    rsv = np.array([f[2] for f in frames], np.uint8)
    lens = np.array([len(f[3]) for f in frames], np.uint32)
    off = np.zeros(n, np.uint64)
    if n:
        off[1:] = np.cumsum(lens, dtype=np.uint64)[:-1]
    pay = np.frombuffer(b"".join(bytes(f[3]) for f in frames) + bytes(16), np.uint8)
    if state is None:
        state = new_state()
    st, win, head, prev = state
    cap = int(lens.sum()) * 2 + 64 * n + 64
    out = np.zeros(cap, np.uint8)
    oo = np.zeros(n + 1, np.uint64)
    orsv = np.zeros(max(n, 1), np.uint8)
    r = lib().zdh_session(level, 1 if no_context else 0, mode, n, op.ctypes.data, fin.ctypes.data, rsv.ctypes.data,
                          off.ctypes.data, lens.ctypes.data, pay.ctypes.data, st.ctypes.data, win.ctypes.data,
                          head.ctypes.data, prev.ctypes.data, out.ctypes.data, cap, oo.ctypes.data, orsv.ctypes.data)
    assert r == 0
    res = [(frames[i][0], frames[i][1], int(orsv[i]), out[int(oo[i]):int(oo[i + 1])].tobytes()) for i in range(n)]
    return res, state


def text(rng, n, vocab=200):
    words = [bytes(rng.integers(97, 123, int(rng.integers(1, 9)), dtype=np.uint8)) for _ in range(vocab)]
    out = bytearray()
    while len(out) < n:
        out += words[int(rng.integers(0, len(words)))] + b" "
    return bytes(out[:n])


def random_frames(rng, n, kind):
    """A session's frame list: messages of 1-4 frames (TEXT/BINARY then continuations)."""
    fr = []
    for i in range(n):
        if kind == "text":
            p = text(rng, int(rng.integers(0, 6000)))
        elif kind == "big":
            p = text(rng, int(rng.integers(0, 90000)))
        elif kind == "bin":
            p = rng.integers(0, 4, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        elif kind == "rand":
            p = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        else:
            p = rng.integers(97, 100, int(rng.integers(0, 50)), dtype=np.uint8).tobytes()
        fr.append((1 if i % 4 == 0 else 0, i % 4 == 3, 0, p))
    return fr


def nil_edge_frames(rng):
    """A new session whose second frame starts at window index 65274: zlib's slide there
    leaves the head of its first string at window index 0 (NIL), exactly MAX_DIST back,
    so that string must not match although an 8-byte copy sits 32506 bytes earlier."""
    while True:
        buf = bytearray(text(rng, 65274 + 4000))
        tri = rng.integers(128, 256, 8, dtype=np.uint8).tobytes()
        buf[32768:32776] = tri
        buf[65274:65282] = tri
        a = np.frombuffer(bytes(buf), np.uint8).astype(np.int64)
        hh = ((a[:-2] << 10) ^ (a[1:-1] << 5) ^ a[2:]) & 32767
        if not (hh[32769:65274] == hh[65274]).any():
            break
    return [(2, False, 0, bytes(buf[:65274])), (0, True, 0, bytes(buf[65274:]))]


def slide_frames(rng):
    """Text frames whose running total crosses 65274 near a frame end (tail slides)."""
    tot, s = [], 0
    target = 65274 + int(rng.integers(-300, 300))
    while s < target - 5000:
        n = int(rng.integers(1000, 5000))
        tot.append(n)
        s += n
    tot.append(target - s)
    tot += [int(rng.integers(1, 5000)) for _ in range(int(rng.integers(1, 20)))]
    fr = [(1 if i == 0 else 0, False, 0, text(rng, n)) for i, n in enumerate(tot)]
    fr[-1] = (fr[-1][0], True, 0, fr[-1][3])
    return fr
