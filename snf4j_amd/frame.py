"""Frame model — the host-side mirror of snf4j-websocket's frame classes.

Same names, constructor arguments and checks as the reference
(snf4j-websocket/src/main/java/org/snf4j/websocket/frame/):
  Opcode.java:33-98, Frame.java:33-143, ControlFrame.java:44-49,
  CloseFrame.java:35-272, TextFrame/BinaryFrame/ContinuationFrame/PingFrame/PongFrame,
  InvalidFrameException.java:35-117.
"""
from __future__ import annotations

from enum import IntEnum


class Opcode(IntEnum):
    CONTINUATION = 0
    TEXT = 1
    BINARY = 2
    CLOSE = 8
    PING = 9
    PONG = 10

    @staticmethod
    def findByValue(value: int):
        """Opcode.findByValue (Opcode.java:48-50): None for an unknown value."""
        try:
            return Opcode(value)
        except ValueError:
            return None

    def value_(self) -> int:
        return int(self)

    def isControl(self) -> bool:
        return int(self) >= 8


EMPTY_PAYLOAD = b""


class Frame:
    RSV1, RSV2, RSV3 = 0x04, 0x02, 0x01

    def __init__(self, opcode: Opcode, finalFragment: bool, rsvBits: int, payload):
        self._opcode = Opcode(opcode)
        self._fin = bool(finalFragment)
        self._rsv = int(rsvBits)
        self._payload = EMPTY_PAYLOAD if payload is None else bytes(payload)

    def getOpcode(self) -> Opcode:
        return self._opcode

    def isFinalFragment(self) -> bool:
        return self._fin

    def getRsvBits(self) -> int:
        return self._rsv

    def isRsvBit1(self) -> bool:
        return bool(self._rsv & Frame.RSV1)

    def isRsvBit2(self) -> bool:
        return bool(self._rsv & Frame.RSV2)

    def isRsvBit3(self) -> bool:
        return bool(self._rsv & Frame.RSV3)

    def getPayload(self) -> bytes:
        return self._payload

    def getPayloadLength(self) -> int:
        return len(self._payload)

    def __eq__(self, other):
        return (type(self) is type(other) and self._opcode == other._opcode and self._fin == other._fin
                and self._rsv == other._rsv and self._payload == other._payload)

    def __repr__(self):
        return (f"{type(self).__name__}(fin={self._fin}, rsv={self._rsv}, "
                f"len={len(self._payload)})")


class DataFrame(Frame):
    pass


class ControlFrame(Frame):
    def __init__(self, opcode, rsvBits, payload):
        super().__init__(opcode, True, rsvBits, payload)
        if len(self._payload) > 125:
            raise ValueError("payload length is too big for control frame")


class TextFrame(DataFrame):
    def __init__(self, finalFragment=True, rsvBits=0, payload=EMPTY_PAYLOAD):
        if isinstance(payload, str):
            payload = payload.encode("utf-8")
        super().__init__(Opcode.TEXT, finalFragment, rsvBits, payload)

    def getText(self) -> str:
        return self._payload.decode("utf-8")


class BinaryFrame(DataFrame):
    def __init__(self, finalFragment=True, rsvBits=0, payload=EMPTY_PAYLOAD):
        super().__init__(Opcode.BINARY, finalFragment, rsvBits, payload)


class ContinuationFrame(DataFrame):
    def __init__(self, finalFragment=True, rsvBits=0, payload=EMPTY_PAYLOAD):
        super().__init__(Opcode.CONTINUATION, finalFragment, rsvBits, payload)


class CloseFrame(ControlFrame):
    NORMAL, GOING_AWAY, PROTOCOL_ERROR, NOT_ACCEPTED = 1000, 1001, 1002, 1003
    NO_CODE, ABNORMAL, NON_UTF8, POLICY_VALIDATION, TOO_BIG = 1005, 1006, 1007, 1008, 1009

    def __init__(self, rsvBits=0, payload=EMPTY_PAYLOAD):
        super().__init__(Opcode.CLOSE, rsvBits, payload)
        if len(self._payload) == 1:
            raise ValueError("illegal data length (1)")

    @staticmethod
    def of_status(status: int, reason: str | None = None, rsvBits: int = 0) -> "CloseFrame":
        body = b"" if reason is None else reason.encode("utf-8")
        return CloseFrame(rsvBits, bytes([(status >> 8) & 0xFF, status & 0xFF]) + body)

    def getStatus(self) -> int:
        if self._payload:
            return (self._payload[0] << 8) | self._payload[1]
        return -1

    def getReason(self) -> str:
        return self._payload[2:].decode("utf-8", "replace") if len(self._payload) > 2 else ""


class PingFrame(ControlFrame):
    def __init__(self, rsvBits=0, payload=EMPTY_PAYLOAD):
        super().__init__(Opcode.PING, rsvBits, payload)


class PongFrame(ControlFrame):
    def __init__(self, rsvBits=0, payload=EMPTY_PAYLOAD):
        super().__init__(Opcode.PONG, rsvBits, payload)


class AggregatedTextFrame(TextFrame):
    """AggregatedTextFrame (AggregatedTextFrame.java:35-90): a final TEXT frame built by
    FrameAggregator from a fragmented message; `fragments` lists the parts it was
    assembled from on the host (one per batch the message spanned)."""

    def __init__(self, rsvBits: int, payload, fragments=None):
        super().__init__(True, rsvBits, payload)
        self.fragments = fragments if fragments is not None else [bytes(payload)]

    def getFragments(self):
        return self.fragments


class AggregatedBinaryFrame(BinaryFrame):
    """AggregatedBinaryFrame (AggregatedBinaryFrame.java:35-72)."""

    def __init__(self, rsvBits: int, payload, fragments=None):
        super().__init__(True, rsvBits, payload)
        self.fragments = fragments if fragments is not None else [bytes(payload)]

    def getFragments(self):
        return self.fragments


def make_frame(opcode: int, fin: bool, rsv: int, payload: bytes) -> Frame:
    """FrameDecoder.createFrame's opcode -> class dispatch (FrameDecoder.java:104-145)."""
    op = Opcode(opcode)
    if op == Opcode.CONTINUATION:
        return ContinuationFrame(fin, rsv, payload)
    if op == Opcode.TEXT:
        return TextFrame(fin, rsv, payload)
    if op == Opcode.BINARY:
        return BinaryFrame(fin, rsv, payload)
    if op == Opcode.CLOSE:
        return CloseFrame(rsv, payload)
    if op == Opcode.PING:
        return PingFrame(rsv, payload)
    return PongFrame(rsv, payload)


class InvalidFrameException(RuntimeError):
    """InvalidFrameException (InvalidFrameException.java:35-117); close type GENTLE."""

    GENTLE, DEFAULT = "GENTLE", "DEFAULT"

    def __init__(self, message: str | None = None, gentleClose: bool = True):
        super().__init__(message)
        self.message = message
        self.closeType = InvalidFrameException.GENTLE if gentleClose else InvalidFrameException.DEFAULT

    def getMessage(self):
        return self.message

    def getCloseType(self):
        return self.closeType

    def getClosingCause(self):
        """ICloseControllingException.getClosingCause (InvalidFrameException.java:112-115)."""
        return self
