"""snf4j_amd — MI355X-native RFC 6455 frame codec for snf4j's codec pipeline.

The hot path (frame decode: header parse, length prefix-scan, unmask, UTF-8
validation; frame encode: header emit + masking) runs in hand-written HIP
kernels for gfx950 (snf4j_amd/csrc, built into snf4j_amd/libwsgpu.so) behind the
C ABI declared in include/wsgpu.h.  This package is the host-side mirror of the
reference's codec interface over that ABI.
"""
from . import _lib  # noqa: F401  (fails loudly if libwsgpu.so is missing)
from .codec import (BatchAggregator, BatchInflater, EncodeBatcher, FrameAggregator, FrameDecoder, FrameEncoder,
                    FrameUtf8Validator, NativeBatcher, PerMessageDeflateDecoder, SessionBatcher)
from .context import Context, decoder_cfg, encoded_length, error_message, frame_available
from .handshake import (BatchClientHandshaker, BatchHandshaker, ClientConfig, ClientHandshakeOutcome, HandshakeConfig,
                        HandshakeOutcome)
from .frame import (AggregatedBinaryFrame, AggregatedTextFrame, BinaryFrame, CloseFrame, ContinuationFrame, Frame,
                    InvalidFrameException, Opcode, PingFrame, PongFrame, TextFrame)

__all__ = ["Context", "FrameDecoder", "FrameEncoder", "EncodeBatcher", "SessionBatcher", "FrameAggregator", "BatchAggregator",
           "FrameUtf8Validator", "NativeBatcher", "BatchInflater", "PerMessageDeflateDecoder",
           "AggregatedTextFrame", "AggregatedBinaryFrame", "decoder_cfg", "encoded_length",
           "error_message", "frame_available",
           "BatchHandshaker", "HandshakeConfig", "HandshakeOutcome", "Frame", "Opcode", "TextFrame", "BinaryFrame", "ContinuationFrame",
           "CloseFrame", "PingFrame", "PongFrame", "InvalidFrameException"]
