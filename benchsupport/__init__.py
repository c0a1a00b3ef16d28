"""Bench and test support: synthetic frame batches generated in HBM and the
device's streaming-copy ceiling (libwsbench.so, include/wsbench.h).

Not part of the codec: snf4j_amd/ never imports this package and libwsgpu.so does
not contain these kernels.  Work is enqueued on a snf4j_amd.Context's stream, so
it is ordered with the codec's kernels on that context.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libwsbench.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libwsbench.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        p, i32, u32, u64 = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64
        L.wsb_synth_uniform.argtypes = [i32, p, u64, u64, u32, u32, i32, i32, i32, p, p, p]
        L.wsb_synth_frames.argtypes = [i32, p, p, u64, p]
        L.wsb_copy_ceiling.argtypes = [i32, p, p, p, u64, i32, C.POINTER(C.c_double)]
        for f in (L.wsb_synth_uniform, L.wsb_synth_frames, L.wsb_copy_ceiling):
            f.restype = i32
        _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {rc}")


def _where(ctx):
    return int(ctx.device), C.c_void_p(ctx.stream_handle)


def synth_uniform(ctx, seed, n_frames, payload_len, frames_per_session, opcode, masked, text, wire, frame_off,
                  session_first):
    """wsb_synth_uniform into device tensors (wire uint8, frame_off int64, session_first int32)."""
    dev, st = _where(ctx)
    _check(lib().wsb_synth_uniform(dev, st, int(seed), int(n_frames), int(payload_len), int(frames_per_session),
                                   int(opcode), int(masked), int(text), wire.data_ptr(), frame_off.data_ptr(),
                                   session_first.data_ptr()), "wsb_synth_uniform")


def synth_frames(ctx, table, wire):
    """Table-driven synthetic batch (wsb_synth_frames); `table` is a device uint8
    tensor holding synth.SYNTH_DTYPE records (benchsupport/synth.py)."""
    dev, st = _where(ctx)
    _check(lib().wsb_synth_frames(dev, st, table.data_ptr(), int(table.numel() // 40), wire.data_ptr()),
           "wsb_synth_frames")


def copy_ceiling(ctx, src, dst, nbytes: int, reps: int = 5) -> float:
    """GB/s (read+write) of the device's best streaming copy over nbytes (tensors)."""
    dev, st = _where(ctx)
    g = C.c_double(0)
    _check(lib().wsb_copy_ceiling(dev, st, src.data_ptr(), dst.data_ptr(), int(nbytes), int(reps), C.byref(g)),
           "wsb_copy_ceiling")
    return float(g.value)
