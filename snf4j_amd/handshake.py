"""Opening handshake over libwsgpu: the host mirror of HandshakeDecoder +
Handshaker.handshake for a batch of new sessions, server side (k_hs_accept:
BatchHandshaker) and client side (k_hs_validate: BatchClientHandshaker).

Reference (snf4j-websocket/src/main/java/org/snf4j/websocket/handshake/):
  HandshakeDecoder.available/decode   HandshakeDecoder.java:141-235
  Handshaker.handshake / accept       Handshaker.java:375-405, 555-578
  Handshaker.request / validate       Handshaker.java:177-206, 420-544, 546-566 (client)
  HandshakeEncoder / HandshakeFactory.format   HandshakeEncoder.java:81-118, HandshakeFactory.java:129-158

A BatchHandshaker outcome is what the reference's server session does with the
request: write `response` and either switch the session to the frame codec (101)
or close it with `message` (the exception message or the Handshaker closing
reason).  DEFER means the Java Handshaker takes the request (include/wsgpu.h lists
the forms); NEED_MORE means the frame is not complete yet.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import HsConfig, lib

NEED_MORE, DEFER, PARSE_ERROR, ACCEPT, FINISHED, CLOSING = 0, 1, 2, 3, 4, 5

MESSAGES = {1: "Invalid http request", 2: "Invalid http request version", 3: "Forbidden http request command",
            4: "Handshake frame too large", 5: "Missing websocket version", 6: "Incorrect websocket version: %s",
            7: "Unsupported websocket version: %s", 8: "Missing websocket upgrade",
            9: "Missing websocket connection", 10: "Invalid websocket upgrade: %s",
            11: "Invalid websocket connection: %s", 12: "Missing websocket request host",
            13: "Missing websocket key", 14: "Invalid websocket key: %s",
            15: "Invalid http response", 16: "Invalid http response version", 17: "Invalid http response status",
            18: "Invalid websocket response status: %s", 19: "Missing websocket key challenge",
            20: "Invalid websocket key challenge. Actual: %s. Expected: %s", 21: "Missing websocket sub protocol",
            22: "Invalid websocket sub protocol: %s"}
CAUSE_NAMES = {0: "NONE", 1: "BAD_REQUEST_LINE", 2: "BAD_VERSION", 3: "FORBIDDEN", 4: "TOO_LARGE",
               5: "MISSING_VERSION", 6: "INCORRECT_VERSION", 7: "UNSUPPORTED_VERSION", 8: "MISSING_UPGRADE",
               9: "MISSING_CONNECTION", 10: "INVALID_UPGRADE", 11: "INVALID_CONNECTION", 12: "MISSING_HOST",
               13: "MISSING_KEY", 14: "INVALID_KEY", 15: "BAD_RESPONSE_LINE", 16: "BAD_RESPONSE_VERSION",
               17: "BAD_RESPONSE_STATUS", 18: "INVALID_STATUS", 19: "MISSING_ACCEPT", 20: "INVALID_ACCEPT",
               21: "MISSING_SUBPROTOCOL", 22: "INVALID_SUBPROTOCOL", 23: "INVALID_EXTENSIONS", 32: "D_LINE_FORM", 33: "D_REPEATED", 34: "D_NON_ASCII",
               35: "D_URI", 36: "D_HOST", 37: "D_SUBPROTOCOL", 38: "D_EXTENSION", 39: "D_POLICY", 40: "D_LINES"}
KIND_NAMES = {NEED_MORE: "need_more", DEFER: "defer", PARSE_ERROR: "parse_error", ACCEPT: "accept",
              FINISHED: "finished", CLOSING: "closing"}


def available(data: bytes) -> int:
    """HttpUtils.available with HandshakeDecoder's default 50-line chunk (wsg_handshake_available)."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    r = lib.wsg_handshake_available(buf.ctypes.data if buf.size else None, buf.size)
    if r < 0:
        raise _lib.WsgError("wsg_handshake_available: %d" % r)
    return r


@dataclass
class HandshakeConfig:
    """The IWebSocketSessionConfig values the server handshake reads
    (DefaultWebSocketSessionConfig.java:59-63,129-189,289-309)."""
    max_handshake_frame_length: int = 65536
    ignore_host_header_field: bool = False
    supported_subprotocols: bool = False   # getSupportedSubProtocols() != null
    supported_extensions: bool = False     # getSupportedExtensions() != null
    custom_policy: bool = False            # acceptRequestUri / customizeHeaders overridden

    def native(self) -> HsConfig:
        return HsConfig(self.max_handshake_frame_length, int(self.ignore_host_header_field),
                        int(self.supported_subprotocols), int(self.supported_extensions), int(self.custom_policy))


@dataclass
class HandshakeOutcome:
    kind: int
    status: int
    cause: int
    frame_len: int
    response: bytes
    message: str | None

    @property
    def switched(self) -> bool:
        """The session switches to the frame codec (HandshakeEncoder.encode :83-96)."""
        return self.kind == ACCEPT and self.status == 101


class BatchHandshaker:
    """Server handshakes of many sessions in one k_hs_accept launch."""

    def __init__(self, config: HandshakeConfig | None = None, ctx=None):
        from .context import Context
        self.config = config or HandshakeConfig()
        self.ctx = ctx or Context(0)

    def accept(self, requests) -> list:
        """requests: the bytes each session has received so far.  One outcome per request."""
        reqs = [bytes(r) for r in requests]
        off = np.zeros(len(reqs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(r) for r in reqs]) if reqs else []
        buf = np.frombuffer(b"".join(reqs), dtype=np.uint8)
        resp, res = self.ctx.handshake_accept_host(self.config.native(), buf, off)
        return [self._outcome(reqs[i], resp[i], res[i]) for i in range(len(reqs))]

    @staticmethod
    def _outcome(req: bytes, resp, r) -> HandshakeOutcome:
        kind, cause = int(r["kind"]), int(r["cause"])
        msg = MESSAGES.get(cause)
        if msg and "%s" in msg:
            d0 = int(r["detail_off"])
            msg = msg % "".join(chr(b) if b < 0x80 else "�" for b in req[d0:d0 + int(r["detail_len"])])
        return HandshakeOutcome(kind, int(r["http_status"]), cause, int(r["frame_len"]),
                                bytes(resp[:int(r["resp_len"])]), msg)


# ------------------------------------------------------------------ client side
GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"


def generate_key(rng=None) -> str:
    """HandshakeUtils.generateKey (HandshakeUtils.java:87-91): Base64 of 16 random bytes."""
    import base64
    import os
    raw = rng.randbytes(16) if rng is not None else os.urandom(16)
    return base64.b64encode(raw).decode()


def client_request(uri: str, host: str, key: str, origin: str | None = None, subprotocols=(), extension_offers=(),
                   extra=()) -> bytes:
    """The request Handshaker.request (:177-206) builds, as HandshakeFactory.format writes
    it (:133-140,150-156): Host, Upgrade, Connection, Sec-WebSocket-Key, [Origin],
    Sec-WebSocket-Version, [Sec-WebSocket-Protocol], [Sec-WebSocket-Extensions], then
    the fields customizeHeaders adds.  uri = HandshakeUtils.requestUri(uri), host =
    HandshakeUtils.host(uri), both already derived by the caller."""
    fields = [("Host", host), ("Upgrade", "websocket"), ("Connection", "Upgrade"), ("Sec-WebSocket-Key", key)]
    if origin is not None:
        fields.append(("Origin", origin))
    fields.append(("Sec-WebSocket-Version", "13"))
    if subprotocols:
        fields.append(("Sec-WebSocket-Protocol", ", ".join(subprotocols)))
    if extension_offers:
        fields.append(("Sec-WebSocket-Extensions", ", ".join(extension_offers)))
    fields += list(extra)
    out = b"GET " + uri.encode() + b" HTTP/1.1\r\n"
    for n, v in fields:
        out += n.encode() + b": " + v.encode() + b"\r\n"
    return out + b"\r\n"


@dataclass
class ClientConfig:
    """The IWebSocketSessionConfig values the client handshake reads."""
    max_handshake_frame_length: int = 65536
    supported_subprotocols: tuple = ()      # getSupportedSubProtocols()
    supported_extensions: bool = False      # getSupportedExtensions() non-empty

    def native(self) -> HsConfig:
        return HsConfig(self.max_handshake_frame_length, 0, int(bool(self.supported_subprotocols)),
                        int(self.supported_extensions), 0)


@dataclass
class ClientHandshakeOutcome:
    kind: int                 # NEED_MORE / DEFER / PARSE_ERROR / FINISHED / CLOSING
    status: int               # the response status (0 before the status line is parsed)
    cause: int
    frame_len: int
    expected: str | None      # generateAnswerKey(key), once the frame is complete
    message: str | None       # the exception message (PARSE_ERROR) or getClosingReason() (CLOSING)

    @property
    def finished(self) -> bool:
        return self.kind == FINISHED


class BatchClientHandshaker:
    """Client handshakes of many sessions: each session's received response bytes and
    the key its request carried, validated in one k_hs_validate launch."""

    def __init__(self, config: ClientConfig | None = None, ctx=None):
        from .context import Context
        self.config = config or ClientConfig()
        self.ctx = ctx or Context(0)

    def validate(self, responses, keys) -> list:
        rs = [bytes(r) for r in responses]
        ks = [k.encode("ascii") if isinstance(k, str) else bytes(k) for k in keys]
        if len(ks) != len(rs) or any(len(k) != 24 for k in ks):
            raise ValueError("one 24-character Sec-WebSocket-Key per response")
        off = np.zeros(len(rs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(r) for r in rs]) if rs else []
        buf = np.frombuffer(b"".join(rs), dtype=np.uint8)
        kb = np.frombuffer(b"".join(ks), dtype=np.uint8)
        exp, res = self.ctx.handshake_validate_host(self.config.native(), buf, off, kb)
        return [self._outcome(rs[i], exp[i], res[i]) for i in range(len(rs))]

    @staticmethod
    def _outcome(resp: bytes, exp, r) -> ClientHandshakeOutcome:
        kind, cause = int(r["kind"]), int(r["cause"])
        expected = bytes(exp[:int(r["resp_len"])]).decode("ascii") if int(r["resp_len"]) else None
        msg = MESSAGES.get(cause) if kind in (PARSE_ERROR, CLOSING) else None
        if msg and "%s" in msg:
            d0 = int(r["detail_off"])
            detail = "".join(chr(b) if b < 0x80 else "\ufffd" for b in resp[d0:d0 + int(r["detail_len"])])
            if cause == 18:
                msg = msg % int(r["http_status"])
            elif cause == 20:
                msg = msg % (detail, expected)
            else:
                msg = msg % detail
        return ClientHandshakeOutcome(kind, int(r["http_status"]), cause, int(r["frame_len"]), expected, msg)
