"""ctypes binding of libwsgpu.so (include/wsgpu.h).

The product path is the HIP library: if it is missing this module raises at
import time — there is no CPU fallback anywhere in snf4j_amd.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# WSG_LIB: another build of the same library (A/B runs of kernel variants, scripts/ab_lib.sh)
LIB_PATH = os.environ.get("WSG_LIB") or os.path.join(HERE, "libwsgpu.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "wsgpu.h")


class WsgError(RuntimeError):
    pass


class DecoderCfg(C.Structure):
    _fields_ = [("client_mode", C.c_int32), ("allow_extensions", C.c_int32),
                ("max_payload_len", C.c_int64), ("validate_utf8", C.c_int32), ("flags", C.c_int32)]


class SessionState(C.Structure):
    _fields_ = [("fragmentation", C.c_uint8), ("text_open", C.c_uint8), ("closed", C.c_uint8),
                ("tail_len", C.c_uint8), ("tail", C.c_uint8 * 3), ("reserved", C.c_uint8)]


class FrameDesc(C.Structure):
    _fields_ = [("payload_off", C.c_uint64), ("payload_len", C.c_uint32), ("opcode", C.c_uint8),
                ("flags", C.c_uint8), ("status", C.c_uint16)]


class SessionResult(C.Structure):
    _fields_ = [("n_delivered", C.c_uint32), ("error", C.c_uint16), ("close_code", C.c_uint16),
                ("detail", C.c_int64)]


class BatchView(C.Structure):
    _fields_ = [("n_frames", C.c_uint64), ("wire_bytes", C.c_uint64), ("n_sessions", C.c_uint32),
                ("reserved", C.c_uint32), ("session_first", C.c_void_p), ("desc", C.c_void_p),
                ("payload", C.c_void_p), ("result", C.c_void_p), ("detail2", C.c_void_p)]


class StageCfg(C.Structure):
    _fields_ = [("inflate", C.c_uint8), ("inflate_no_context", C.c_uint8), ("validate", C.c_uint8),
                ("aggregate", C.c_uint8), ("reserved", C.c_uint32), ("max_aggregated_len", C.c_int64)]


class EncView(C.Structure):
    _fields_ = [("n_frames", C.c_uint64), ("wire_bytes", C.c_uint64), ("n_sessions", C.c_uint32),
                ("reserved", C.c_uint32), ("session_first", C.c_void_p), ("wire_off", C.c_void_p),
                ("wire", C.c_void_p)]


class EncodeFrame(C.Structure):
    _fields_ = [("payload_off", C.c_uint64), ("payload_len", C.c_uint32), ("opcode", C.c_uint8),
                ("flags", C.c_uint8), ("reserved", C.c_uint8 * 2), ("mask", C.c_uint8 * 4),
                ("reserved2", C.c_uint32)]


class HsConfig(C.Structure):
    _fields_ = [("max_length", C.c_uint32), ("ignore_host", C.c_uint8), ("subprotocols", C.c_uint8),
                ("extensions", C.c_uint8), ("host_policy", C.c_uint8)]


BATCHER_MAX_INFLIGHT = 4  # WSG_BATCHER_MAX_INFLIGHT: decode flushes a batcher keeps in flight
HS_RESP_STRIDE = 160
HS_EXPECTED_STRIDE = 32   # wsg_handshake_validate_batch_*: expected Sec-WebSocket-Accept per session


assert C.sizeof(SessionState) == 8 and C.sizeof(FrameDesc) == 16
assert C.sizeof(SessionResult) == 16 and C.sizeof(EncodeFrame) == 24

# numpy views of the same records
try:
    import numpy as np

    STATE_DTYPE = np.dtype([("fragmentation", "u1"), ("text_open", "u1"), ("closed", "u1"),
                            ("tail_len", "u1"), ("tail", "u1", (3,)), ("reserved", "u1")])
    DESC_DTYPE = np.dtype([("payload_off", "<u8"), ("payload_len", "<u4"), ("opcode", "u1"),
                           ("flags", "u1"), ("status", "<u2")])
    RESULT_DTYPE = np.dtype([("n_delivered", "<u4"), ("error", "<u2"), ("close_code", "<u2"),
                             ("detail", "<i8")])
    ENCODE_DTYPE = np.dtype([("payload_off", "<u8"), ("payload_len", "<u4"), ("opcode", "u1"),
                             ("flags", "u1"), ("reserved", "u1", (2,)), ("mask", "u1", (4,)),
                             ("reserved2", "<u4")])
    AGG_STATE_DTYPE = np.dtype([("open", "u1"), ("opcode", "u1"), ("rsv", "u1"), ("reserved", "u1"),
                                ("length", "<u4")])
    INFLATE_STATE_DTYPE = np.dtype([("compressing", "u1"), ("has_decoder", "u1"), ("finished", "u1"),
                                    ("reserved", "u1"), ("window_len", "<u2"), ("window_phase", "<u2")])
    DEFLATE_STATE_DTYPE = np.dtype([("strstart", "<u4"), ("high_water", "<u4"), ("insert", "<u2"),
                                    ("has_deflater", "u1"), ("compressing", "u1"), ("reserved", "<u4")])
    HS_RESULT_DTYPE = np.dtype([("frame_len", "<u4"), ("http_status", "<u2"), ("kind", "u1"), ("cause", "u1"),
                                ("resp_len", "<u2"), ("detail_len", "<u2"), ("detail_off", "<u4")])
    assert HS_RESULT_DTYPE.itemsize == 16
except ImportError:  # pragma: no cover
    np = None


def _load():
    # torch (when installed) bundles its own libamdhip64.so.7, the soname libwsgpu.so
    # links against: load torch first so the process has ONE HIP runtime (torch's) and
    # device pointers / streams pass between them; loaded the other way round, torch
    # would bind to the system runtime and fail to initialise.
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover  (a JNI/ctypes host without torch uses the system runtime)
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libwsgpu.so not built ({LIB_PATH}); run snf4j_amd.build.build() — "
                          "the HIP extension is required, there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    p, i32, i64, u32, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
    P = C.POINTER
    sig = {
        "wsg_version": ([], i32),
        "wsg_open": ([i32, p, P(p)], i32),
        "wsg_close": ([p], i32),
        "wsg_set_stream": ([p, p], i32),
        "wsg_get_stream": ([p, P(p)], i32),
        "wsg_last_error": ([p], C.c_char_p),
        "wsg_reserve": ([p, u64, u32, u64], i32),
        "wsg_reserve_inflate": ([p, u64, u32, u64], i32),
        "wsg_inflate_split_count": ([p, p], i32),
        "wsg_batcher_stage_context": ([p], p),
        "wsg_sync": ([p], i32),
        "wsg_set_timing": ([p, i32], i32),
        "wsg_set_timing_every": ([p, u32], i32),
        "wsg_get_timing": ([p, P(C.c_double), P(u64), i32], i32),
        "wsg_reset_timing": ([p], i32),
        "wsg_kernel_name": ([i32], C.c_char_p),
        "wsg_num_kernels": ([], i32),
        "wsg_decode_payload_bound": ([u64, u64], u64),
        "wsg_decode_batch_device": ([p, P(DecoderCfg), p, u64, p, u64, p, u32, p, p, u64, p, p], i32),
        "wsg_decode_batch_host": ([p, P(DecoderCfg), p, u64, p, u64, p, u32, p, p, u64, p, p], i32),
        "wsg_decode_batch_host_async": ([p, P(DecoderCfg), p, u64, p, u64, p, u32, p, p, u64, p, p], i32),
        "wsg_frame_available": ([p, u64, P(i32), P(i64), P(i64)], i64),
        "wsg_check_header": ([P(DecoderCfg), i32, p, u64, P(i64)], i32),
        "wsg_encoded_length": ([u32, i32], u64),
        "wsg_encode_batch_device": ([p, i32, p, u64, p, u64, p, u32, p, p, u64, p], i32),
        "wsg_encode_batch_host": ([p, i32, p, u64, p, u64, p, u32, p, p, u64, p], i32),
        "wsg_batcher_open": ([p, P(DecoderCfg), u32, P(p)], i32),
        "wsg_batcher_close": ([p], i32),
        "wsg_batcher_last_error": ([p], C.c_char_p),
        "wsg_batcher_feed": ([p, u32, p, u64], i32),
        "wsg_batcher_flush": ([p, P(BatchView)], i32),
        "wsg_batcher_session_state": ([p, u32, P(SessionState)], i32),
        "wsg_batcher_session_reset": ([p, u32], i32),
        "wsg_batcher_feed_many": ([p, u32, p, p, p], i32),
        "wsg_batcher_flush_async": ([p], i32),
        "wsg_batcher_wait": ([p, P(BatchView)], i32),
        "wsg_batcher_set_stages": ([p, P(StageCfg)], i32),
        "wsg_batcher_ticket": ([p], u64),
        "wsg_batcher_await": ([p, u64, i64], i64),
        "wsg_batcher_reserve": ([p, u64, u64], i32),
        "wsg_batcher_reserve_stages": ([p, u64, u64], i32),
        "wsg_batcher_alloc_count": ([], u64),
        "wsg_enc_batcher_ticket": ([p], u64),
        "wsg_enc_batcher_await": ([p, u64, i64], i64),
        "wsg_enc_batcher_reserve": ([p, u64, u64], i32),
        "wsg_enc_batcher_set_deflate": ([p, i32, i32], i32),
        "wsg_set_tuning": ([p, i32, C.c_int64], i32),
        "wsg_device_policy_init": ([i32], i32),
        "wsg_device_for_loop": ([u64], i32),
        "wsg_device_account": ([i32, u64], i32),
        "wsg_device_release_loop": ([u64], i32),
        "wsg_enc_batcher_open": ([p, i32, u32, P(p)], i32),
        "wsg_enc_batcher_close": ([p], i32),
        "wsg_enc_batcher_last_error": ([p], C.c_char_p),
        "wsg_enc_batcher_add": ([p, u32, C.c_uint8, C.c_uint8, p, p, u32], i32),
        "wsg_enc_batcher_flush": ([p, P(EncView)], i32),
        "wsg_enc_batcher_flush_async": ([p], i32),
        "wsg_enc_batcher_add_many": ([p, u32, p, p, p, p, p, p], i32),
        "wsg_enc_batcher_wait": ([p, P(EncView)], i32),
        "wsg_enc_batcher_session_reset": ([p, u32], i32),
        "wsg_host_alloc": ([u64], p),
        "wsg_host_release": ([p], i32),
        "wsg_host_capacity": ([p], u64),
        "wsg_host_trim": ([], i32),
        "wsg_inflate_batch_device": ([p, i32, p, u64, p, u32, p, u64, p, p, p, p, p, p, p], i32),
        "wsg_inflate_batch_host": ([p, i32, p, u64, p, u32, p, u64, p, p, p, p, p, p, p], i32),
        "wsg_deflate_batch_device": ([p, i32, i32, p, u64, p, u32, p, u64, p, p, p, u64, p, P(u64)], i32),
        "wsg_deflate_batch_host": ([p, i32, i32, p, u64, p, u32, p, u64, p, p, p, u64, p, P(u64)], i32),
        "wsg_validate_batch_device": ([p, p, u64, p, u32, p, u64, p, p], i32),
        "wsg_validate_batch_host": ([p, p, u64, p, u32, p, u64, p, p], i32),
        "wsg_aggregate_batch_device": ([p, i64, p, u64, p, u32, p, p, u64, p, p, u64, p, p, p], i32),
        "wsg_aggregate_batch_host": ([p, i64, p, u64, p, u32, p, p, u64, p, p, u64, p, p, P(u64)], i32),
        "wsg_handshake_available": ([p, u64], i32),
        "wsg_handshake_accept_batch_device": ([p, P(HsConfig), p, p, u32, p, p], i32),
        "wsg_handshake_accept_batch_host": ([p, P(HsConfig), p, p, u32, p, p], i32),
        "wsg_handshake_validate_batch_device": ([p, P(HsConfig), p, p, p, u32, p, p], i32),
        "wsg_handshake_validate_batch_host": ([p, P(HsConfig), p, p, p, u32, p, p], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


lib = _load()


def header_symbols() -> list[str]:
    """Every function the C ABI header declares."""
    with open(HEADER) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wsg_[a-z0-9_]+)\s*\(", text)))


def check(rc: int, ctx=None):
    if rc != 0:
        msg = lib.wsg_last_error(ctx).decode() if ctx else ""
        raise WsgError(f"libwsgpu error {rc}: {msg}")
