"""CPU restatement of snf4j's WebSocket opening handshake (server side, and the
client side's response validation).

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this as the checker; the product path is k_hs_accept
(snf4j_amd/csrc/handshake.hip) behind the C ABI.

Restated from (paths under snf4j-websocket/src/main/java/org/snf4j/websocket/):
  handshake/HttpUtils.java:77-110     available (CRLF lines, `end` latch, chunk cap)
  handshake/HttpUtils.java:125-157    splitRequestLine
  handshake/HttpUtils.java:159-196    splitHeaderField
  handshake/HttpUtils.java:226-249    rtrimAscii / ascii (US-ASCII decoding)
  handshake/HttpUtils.java:311-333    values (split ',', trim, drop empty)
  handshake/HandshakeFrame.java:74-101  addValue / appendValue / pendingName
  handshake/HandshakeFactory.java:47-127  parse / parseFields
  handshake/HandshakeFactory.java:129-158 format
  handshake/HandshakeDecoder.java:141-219 decode (frame length cap, server error response)
  handshake/Handshaker.java:208-405    acceptVersion / acceptBasicFields / acceptUri /
                                       acceptKey / acceptSubProtocol / acceptExtensions / accept
  handshake/HandshakeUtils.java:93-120 generateAnswerKey / parseKey
  snf4j-core/.../util/Base64Util.java:253-350 decode (not MIME)
  client side:
  handshake/HandshakeFactory.java:108-123  parse, response branch (HttpUtils.digits :271-284)
  handshake/HandshakeDecoder.java:141-210  decode in client mode (exceptions are thrown)
  handshake/Handshaker.java:420-544    validateBasicFields / validateKeyChallenge /
                                       validateSubProtocol / validateExtensions / validate

java.net.URI is not restated: `accept` answers only for the forms whose
validity follows from RFC 2396's grammar as java.net.URI implements it (relative
references over unreserved / punctuation characters and %XX escapes, and Host
values of [A-Za-z0-9.-:]); for every other form it returns None ("unknown").
"""
from __future__ import annotations

import base64
import hashlib

CR, LF, SP, HT = 13, 10, 32, 9
MAX_LINES = 50                      # HandshakeDecoder.DEFAULT_MAX_LINES_IN_CHUNK
GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"

REASONS = {101: "Switching Protocols", 400: "Bad Request", 403: "Forbidden", 404: "Not Found",
           413: "Request Entity Too Large", 426: "Upgrade Required"}   # HttpStatus.java:30-35

# wsg_hs_kind / wsg_hs_cause (include/wsgpu.h)
NEED_MORE, DEFER, PARSE_ERROR, ACCEPT = 0, 1, 2, 3
C_NONE, C_BAD_REQUEST_LINE, C_BAD_VERSION, C_FORBIDDEN, C_TOO_LARGE = 0, 1, 2, 3, 4
C_MISSING_VERSION, C_INCORRECT_VERSION, C_UNSUPPORTED_VERSION = 5, 6, 7
C_MISSING_UPGRADE, C_MISSING_CONNECTION, C_INVALID_UPGRADE, C_INVALID_CONNECTION = 8, 9, 10, 11
C_MISSING_HOST, C_MISSING_KEY, C_INVALID_KEY = 12, 13, 14
FINISHED, CLOSING = 4, 5
C_BAD_RESPONSE_LINE, C_BAD_RESPONSE_VERSION, C_BAD_RESPONSE_STATUS, C_INVALID_STATUS = 15, 16, 17, 18
C_MISSING_ACCEPT, C_INVALID_ACCEPT, C_MISSING_SUBPROTOCOL, C_INVALID_SUBPROTOCOL, C_INVALID_EXTENSIONS = 19, 20, 21, 22, 23
D_LINE_FORM, D_REPEATED, D_NON_ASCII, D_URI, D_HOST, D_SUBPROTOCOL, D_EXTENSION, D_POLICY, D_LINES = range(32, 41)

MESSAGES = {C_BAD_REQUEST_LINE: "Invalid http request", C_BAD_VERSION: "Invalid http request version",
            C_FORBIDDEN: "Forbidden http request command", C_TOO_LARGE: "Handshake frame too large",
            C_MISSING_VERSION: "Missing websocket version", C_INCORRECT_VERSION: "Incorrect websocket version: %s",
            C_UNSUPPORTED_VERSION: "Unsupported websocket version: %s",
            C_MISSING_UPGRADE: "Missing websocket upgrade", C_MISSING_CONNECTION: "Missing websocket connection",
            C_INVALID_UPGRADE: "Invalid websocket upgrade: %s",
            C_INVALID_CONNECTION: "Invalid websocket connection: %s",
            C_MISSING_HOST: "Missing websocket request host", C_MISSING_KEY: "Missing websocket key",
            C_INVALID_KEY: "Invalid websocket key: %s",
            C_BAD_RESPONSE_LINE: "Invalid http response", C_BAD_RESPONSE_VERSION: "Invalid http response version",
            C_BAD_RESPONSE_STATUS: "Invalid http response status",
            C_INVALID_STATUS: "Invalid websocket response status: %s",
            C_MISSING_ACCEPT: "Missing websocket key challenge",
            C_INVALID_ACCEPT: "Invalid websocket key challenge. Actual: %s. Expected: %s",
            C_MISSING_SUBPROTOCOL: "Missing websocket sub protocol",
            C_INVALID_SUBPROTOCOL: "Invalid websocket sub protocol: %s"}


class InvalidHandshake(Exception):
    def __init__(self, cause, status=400):
        super().__init__(MESSAGES.get(cause, ""))
        self.cause, self.status = cause, status


def ascii_str(data: bytes) -> str:
    """new String(bytes, US_ASCII): bytes >= 0x80 decode to U+FFFD."""
    return "".join(chr(b) if b < 0x80 else "�" for b in data)


def java_trim(s: str) -> str:
    i, j = 0, len(s)
    while i < j and ord(s[i]) <= 0x20:
        i += 1
    while j > i and ord(s[j - 1]) <= 0x20:
        j -= 1
    return s[i:j]


def values(s: str) -> list:
    """HttpUtils.values(s) (:311-333)."""
    if not s:
        return []
    return [java_trim(t) for t in s.split(",") if java_trim(t)]


def available(data: bytes, lines_len: int = MAX_LINES * 2 + 1):
    """HttpUtils.available (:77-110) with lines = int[lines_len]:
    (frame length or 0, list of (begin, end) lines, capped)."""
    max_count = lines_len - 3
    lines, line0, count, curr, end = [], 0, 0, 0, False
    for i, c in enumerate(data):
        prev, curr = curr, c
        if curr == LF:
            if prev == CR:
                if end:
                    return i + 1, lines, False
                if count > max_count:
                    return 0, lines, True
                end = True
                lines.append((line0, i - 1))
                count += 2
                line0 = i + 1
        elif curr != CR:
            end = False
    return 0, lines, False


def split_request_line(data: bytes, b: int, e: int, max_tokens: int = 5):
    """HttpUtils.splitRequestLine (:132-157) with out = int[10]."""
    max_count = max_tokens * 2 - 2
    out, line0, curr = [], b, 0
    for i in range(b, e):
        prev, curr = curr, data[i]
        if curr == SP:
            if prev != SP:
                out.append((line0, i))
                if len(out) * 2 > max_count:
                    return out
        elif prev == SP:
            line0 = i
    out.append((e, e) if curr == SP else (line0, e))
    return out


def split_header_field(data: bytes, b: int, e: int):
    """HttpUtils.splitHeaderField (:159-196): (code, tokens)."""
    i, sign = b, 1
    while i < e and data[i] in (SP, HT):
        sign = -1
        i += 1
    t = [i]
    while i < e:
        if data[i] == ord(":"):
            t.append(i)
            i += 1
            break
        i += 1
    if len(t) == 1:
        t.append(e)
        return 2 * sign, t
    while i < e and data[i] in (SP, HT):
        i += 1
    t += [i, e]
    return 4 * sign, t


def rtrim(data: bytes, b: int, e: int) -> str:
    while e > b and data[e - 1] in (SP, HT):
        e -= 1
    return ascii_str(data[b:e])


class Frame:
    """HandshakeFrame (:33-150): upper-cased keys, ", "-joined repeats, folding."""

    def __init__(self, uri=None):
        self.uri, self.values, self.names = uri, {}, []
        self.pending, self.last_key = None, None
        self.adds = {}     # key -> number of addValue calls (the GPU defers repeats)

    def add(self, name, value):
        if self.pending is not None:
            name = self.pending + name
            self.pending = None
        self.last_key = name.upper()
        self.adds[self.last_key] = self.adds.get(self.last_key, 0) + 1
        old = self.values.get(self.last_key)
        if old is not None:
            value = old + ", " + value
        else:
            self.names.append(name)
        self.values[self.last_key] = value

    def append(self, value):
        if self.last_key is None:
            raise InvalidHandshake(-1)   # "No header field to extend"
        self.values[self.last_key] = self.values[self.last_key] + value

    def get(self, name):
        return self.values.get(name.upper())


def parse_request(data: bytes, lines) -> Frame:
    """HandshakeFactory.parse (:94-127) for a request, parseFields (:47-92) from line 1."""
    b, e = lines[0]
    tok = split_request_line(data, b, e)
    if len(tok) != 3:
        raise InvalidHandshake(C_BAD_REQUEST_LINE)
    if data[tok[2][0]:tok[2][1]] != b"HTTP/1.1":
        raise InvalidHandshake(C_BAD_VERSION)
    if data[tok[0][0]:tok[0][1]] != b"GET":
        raise InvalidHandshake(C_FORBIDDEN, 403)
    f = Frame(ascii_str(data[tok[1][0]:tok[1][1]]))
    for (b, e) in lines[1:]:
        code, t = split_header_field(data, b, e)
        if code == 4:
            if f.pending is not None:
                raise InvalidHandshake(-2)   # "No value in header field"
            f.add(ascii_str(data[t[0]:t[1]]), rtrim(data, t[2], t[3]))
        elif code == 2:
            if f.pending is not None:
                raise InvalidHandshake(-2)
            f.pending = ascii_str(data[t[0]:t[1]])
        elif code == -4:
            if f.pending is not None:
                f.add(ascii_str(data[t[0]:t[1]]), rtrim(data, t[2], t[3]))
            else:
                f.append(" ")
                f.append(rtrim(data, t[0], t[3]))
        elif code == -2:
            if f.pending is not None:
                f.pending += ascii_str(data[t[0]:t[1]])
            else:
                f.append(" ")
                f.append(rtrim(data, t[0], t[1]))
    return f


def parse_int(s: str):
    """Integer.parseInt over the characters the oracle sees (ASCII)."""
    if not s:
        return None
    i, neg = 0, False
    if s[0] in "+-":
        if len(s) == 1:
            return None
        neg, i = s[0] == "-", 1
    if not all("0" <= ch <= "9" for ch in s[i:]):
        return None
    v = int(s[i:]) * (-1 if neg else 1)
    return v if -2**31 <= v < 2**31 else None


def base64_decode(s: str):
    """Base64Util.decode(data, isMime=false) (:253-350) over HttpUtils.bytes(s)."""
    data = s.encode("ascii", errors="replace")
    n = len(data)
    if n == 0:
        return b""
    if n < 2:
        return None
    end = n
    if data[end - 1] == ord("="):
        end -= 1
        if data[end - 1] == ord("="):
            end -= 1
    length = end
    if length == 0:
        return b""
    if (length & 3) == 1:
        return None
    alphabet = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"
    out, v, cnt = bytearray(), 0, 0
    for c in data[:end]:
        k = alphabet.find(bytes([c]))
        if k < 0:
            return None
        v = (v << 6) | k
        if cnt == 3:
            out += bytes([(v >> 16) & 255, (v >> 8) & 255, v & 255])
            v, cnt = 0, 0
        else:
            cnt += 1
    if cnt:
        shift = (4 - cnt) * 6
        out.append((v >> (16 - shift)) & 255)
        if shift == 6:
            out.append((v >> (8 - shift)) & 255)
    return bytes(out)


def answer_key(key: str) -> str:
    """HandshakeUtils.generateAnswerKey (:98-111)."""
    return base64.b64encode(hashlib.sha1(key.encode("ascii", errors="replace") + GUID).digest()).decode()


_URI_OK = set(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-._~!*'()/?=&+,;$")
_HOST_OK = set(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789.-:")
_HEX = set(b"0123456789abcdefABCDEF")


def uri_fast(u: str) -> bool:
    b = u.encode("latin-1", errors="replace")
    i = 0
    while i < len(b):
        c = b[i]
        if c == ord("%"):
            if i + 2 < len(b) and b[i + 1] in _HEX and b[i + 2] in _HEX:
                i += 3
                continue
            return False
        if c not in _URI_OK:
            return False
        i += 1
    return True


def host_fast(h: str) -> bool:
    return all(ord(ch) < 128 and ord(ch) in _HOST_OK for ch in h)


def format_response(status: int, fields) -> bytes:
    """HandshakeFactory.format of a HandshakeResponse (:141-157)."""
    out = b"HTTP/1.1 %03d %s\r\n" % (status, REASONS[status].encode())
    for n, v in fields:
        out += n.encode() + b": " + v.encode() + b"\r\n"
    return out + b"\r\n"


def accept(data: bytes, max_length=65536, ignore_host=False, subprotocols=False, extensions=False,
           host_policy=False):
    """HandshakeDecoder.decode + Handshaker.accept for one server request buffer.
    Returns dict(kind, status, cause, detail, frame_len, response) where kind is
    NEED_MORE / PARSE_ERROR / ACCEPT, or UNKNOWN (None) when the verdict depends on
    java.net.URI or on config callbacks the oracle does not restate."""
    flen, lines, capped = available(data)
    r = dict(kind=NEED_MORE, status=0, cause=C_NONE, detail=None, frame_len=flen, response=b"")
    if capped:
        return dict(r, kind=DEFER, cause=D_LINES)
    if flen == 0:
        # HandshakeDecoder.available0 (:221-233) hands the complete lines to decode as a
        # chunk: its length and the request line are judged before the frame completes
        if not lines:
            return r
        end = lines[-1][1] + 2
        if end > max_length:
            return dict(r, kind=PARSE_ERROR, status=413, cause=C_TOO_LARGE, response=format_response(413, []))
        try:
            parse_request(data[:end], lines[:1])
        except InvalidHandshake as e:
            return dict(r, kind=PARSE_ERROR, status=e.status, cause=e.cause, response=format_response(e.status, []))
        return r
    if flen > max_length:
        return dict(r, kind=PARSE_ERROR, status=413, cause=C_TOO_LARGE, response=format_response(413, []))
    try:
        f = parse_request(data[:flen], lines)
    except InvalidHandshake as e:
        if e.cause < 0:   # the folding exceptions: 400, message not among the GPU causes
            return dict(r, kind=PARSE_ERROR, status=400, cause=e.cause, response=format_response(400, []))
        return dict(r, kind=PARSE_ERROR, status=e.status, cause=e.cause, response=format_response(e.status, []))

    def refuse(status, cause, detail=None, fields=()):
        return dict(r, kind=ACCEPT, status=status, cause=cause, detail=detail,
                    response=format_response(status, list(fields)))
    # acceptVersion (:208-234)
    s = f.get("Sec-WebSocket-Version")
    if s is None:
        return refuse(400, C_MISSING_VERSION)
    ok = False
    for v in values(s):
        x = parse_int(v)
        if x is None:
            return refuse(400, C_INCORRECT_VERSION, v)
        if x == 13:
            ok = True
            break
    if not ok:
        return refuse(426, C_UNSUPPORTED_VERSION, s, [("Sec-WebSocket-Version", "13")])
    # acceptBasicFields (:236-240, :420-444)
    u, c = f.get("Upgrade"), f.get("Connection")
    if u is None:
        return refuse(400, C_MISSING_UPGRADE)
    if c is None:
        return refuse(400, C_MISSING_CONNECTION)
    if not any(t.lower() == "websocket" for t in values(u)):
        return refuse(400, C_INVALID_UPGRADE, u)
    if not any(t.lower() == "upgrade" for t in values(c)):
        return refuse(400, C_INVALID_CONNECTION, c)
    # acceptUri (:327-373)
    host = f.get("Host")
    if not uri_fast(f.uri):
        return dict(r, kind=None)           # new URI(request.getUri()): java.net.URI decides
    if host is None:
        if not ignore_host:
            return refuse(400, C_MISSING_HOST)
    elif not host_fast(host):
        return dict(r, kind=None)           # new URI("ws://" + host + uri)
    if host_policy:
        return dict(r, kind=None)           # config.acceptRequestUri(uri)
    # acceptKey (:242-257)
    key = f.get("Sec-WebSocket-Key")
    if key is None:
        return refuse(400, C_MISSING_KEY)
    k = base64_decode(key)
    if k is None or len(k) != 16:
        return refuse(400, C_INVALID_KEY, key)
    # acceptSubProtocol / acceptExtensions: decided by the configured lists (host side)
    if (subprotocols and f.get("Sec-WebSocket-Protocol")) or (extensions and f.get("Sec-WebSocket-Extensions")):
        return dict(r, kind=None)
    return dict(r, kind=ACCEPT, status=101, cause=C_NONE,
                response=format_response(101, [("Upgrade", "websocket"), ("Connection", "Upgrade"),
                                               ("Sec-WebSocket-Accept", answer_key(key))]))


TARGETS = ("HOST", "UPGRADE", "CONNECTION", "SEC-WEBSOCKET-KEY", "SEC-WEBSOCKET-VERSION",
           "SEC-WEBSOCKET-PROTOCOL", "SEC-WEBSOCKET-EXTENSIONS")


def gpu_defers(data: bytes, max_length=65536, ignore_host=False, subprotocols=False, extensions=False,
               host_policy=False):
    """The forms k_hs_accept hands to the Java Handshaker (include/wsgpu.h), as a
    deferral cause, or None.  Walks the request in the reference's order, so a
    definite verdict found before a deferred form wins."""
    flen, lines, capped = available(data)
    if capped:
        return D_LINES
    if flen == 0:
        return None
    if flen > max_length:
        return None
    b, e = lines[0]
    tok = split_request_line(data, b, e)
    if len(tok) != 3 or data[tok[2][0]:tok[2][1]] != b"HTTP/1.1" or data[tok[0][0]:tok[0][1]] != b"GET":
        return None
    seen, fields = set(), {}
    for (b, e) in lines[1:]:
        code, t = split_header_field(data, b, e)
        if code != 4:
            return D_LINE_FORM
        name = ascii_str(data[t[0]:t[1]]).upper()
        if name in TARGETS:
            if name in seen:
                return D_REPEATED
            seen.add(name)
            v = data[t[2]:t[3]]
            if any(x >= 0x80 for x in v):
                return D_NON_ASCII
            fields[name] = rtrim(data, t[2], t[3])
    if any(x >= 0x80 for x in data[tok[1][0]:tok[1][1]]):
        return D_NON_ASCII
    r = accept(data, max_length, ignore_host, False, False, False)
    if r["kind"] is not None and r["cause"] in (C_MISSING_VERSION, C_INCORRECT_VERSION, C_UNSUPPORTED_VERSION,
                                                  C_MISSING_UPGRADE, C_MISSING_CONNECTION, C_INVALID_UPGRADE,
                                                  C_INVALID_CONNECTION):
        return None
    if not uri_fast(ascii_str(data[tok[1][0]:tok[1][1]])):
        return D_URI
    host = fields.get("HOST")
    if host is None:
        if not ignore_host:
            return None
    elif not host_fast(host):
        return D_HOST
    if host_policy:
        return D_POLICY
    if r["kind"] is not None and r["cause"] in (C_MISSING_KEY, C_INVALID_KEY):
        return None
    if subprotocols and fields.get("SEC-WEBSOCKET-PROTOCOL"):
        return D_SUBPROTOCOL
    if extensions and fields.get("SEC-WEBSOCKET-EXTENSIONS"):
        return D_EXTENSION
    return None


def request(uri="/uri", fields=None) -> bytes:
    """A request the way HandshakeFactory.format writes one (:133-140, :150-156)."""
    out = b"GET " + uri.encode() + b" HTTP/1.1\r\n"
    for n, v in (fields or []):
        out += n.encode() + b": " + v.encode() + b"\r\n"
    return out + b"\r\n"


# ----------------------------------------------------------------- client side
def parse_response(data: bytes, lines) -> tuple:
    """HandshakeFactory.parse (:108-123) for a response: (status, Frame)."""
    b, e = lines[0]
    tok = split_request_line(data, b, e)           # splitResponseLine = splitRequestLine
    if len(tok) < 3:
        raise InvalidHandshake(C_BAD_RESPONSE_LINE)
    if data[tok[0][0]:tok[0][1]] != b"HTTP/1.1":
        raise InvalidHandshake(C_BAD_RESPONSE_VERSION)
    st = data[tok[1][0]:tok[1][1]]
    if not all(0x30 <= c <= 0x39 for c in st) or len(st) != 3:   # HttpUtils.digits, STATUS_CODE_LENGTH
        raise InvalidHandshake(C_BAD_RESPONSE_STATUS)
    status = int(st)
    f = Frame()
    for (b, e) in lines[1:]:
        code, t = split_header_field(data, b, e)
        if code == 4:
            if f.pending is not None:
                raise InvalidHandshake(-2)
            f.add(ascii_str(data[t[0]:t[1]]), rtrim(data, t[2], t[3]))
        elif code == 2:
            if f.pending is not None:
                raise InvalidHandshake(-2)
            f.pending = ascii_str(data[t[0]:t[1]])
        elif code == -4:
            if f.pending is not None:
                f.add(ascii_str(data[t[0]:t[1]]), rtrim(data, t[2], t[3]))
            else:
                f.append(" ")
                f.append(rtrim(data, t[0], t[3]))
        elif code == -2:
            if f.pending is not None:
                f.pending += ascii_str(data[t[0]:t[1]])
            else:
                f.append(" ")
                f.append(rtrim(data, t[0], t[1]))
    return status, f


def validate(data: bytes, key: str, max_length=65536, subprotocols=None, extensions=False):
    """HandshakeDecoder(clientMode).decode + Handshaker.handshake(response) for one
    response buffer and the key the session sent.  subprotocols: the configured list
    (None or empty: none); extensions: the configured list is non-empty.  Returns
    dict(kind, status, cause, detail, frame_len, expected, subprotocol); kind is None
    when IExtension.validateResponse decides (not restated)."""
    flen, lines, capped = available(data)
    r = dict(kind=NEED_MORE, status=0, cause=C_NONE, detail=None, frame_len=flen, expected=None, subprotocol=None)
    if capped:
        return dict(r, kind=DEFER, cause=D_LINES)
    if flen == 0:
        if not lines:
            return r
        end = lines[-1][1] + 2
        if end > max_length:
            return dict(r, kind=PARSE_ERROR, cause=C_TOO_LARGE)
        try:
            status, _ = parse_response(data[:end], lines[:1])
        except InvalidHandshake as e:
            return dict(r, kind=PARSE_ERROR, cause=e.cause)
        return dict(r, status=status)
    if flen > max_length:
        return dict(r, kind=PARSE_ERROR, cause=C_TOO_LARGE)
    try:
        status, f = parse_response(data[:flen], lines)
    except InvalidHandshake as e:
        return dict(r, kind=PARSE_ERROR, cause=e.cause)
    r["status"] = status

    def closing(cause, detail=None):
        return dict(r, kind=CLOSING, cause=cause, detail=detail)
    if status != 101:                                          # validate (:535-544)
        return closing(C_INVALID_STATUS, str(status))
    u, c = f.get("Upgrade"), f.get("Connection")                 # validateBasicFields (:420-444)
    if u is None:
        return closing(C_MISSING_UPGRADE)
    if c is None:
        return closing(C_MISSING_CONNECTION)
    if not any(t.lower() == "websocket" for t in values(u)):
        return closing(C_INVALID_UPGRADE, u)
    if not any(t.lower() == "upgrade" for t in values(c)):
        return closing(C_INVALID_CONNECTION, c)
    expected = answer_key(key)                                   # validateKeyChallenge (:446-460)
    r["expected"] = expected
    actual = f.get("Sec-WebSocket-Accept")
    if actual is None:
        return closing(C_MISSING_ACCEPT)
    if actual != expected:
        return closing(C_INVALID_ACCEPT, actual)
    received = f.get("Sec-WebSocket-Protocol")                   # validateSubProtocol (:462-485)
    if subprotocols:
        if received is None:
            return closing(C_MISSING_SUBPROTOCOL)
        if received not in subprotocols:
            return closing(C_INVALID_SUBPROTOCOL, received)
        r["subprotocol"] = received
    elif received is not None:
        return closing(C_INVALID_SUBPROTOCOL, received)
    ext = f.get("Sec-WebSocket-Extensions")                      # validateExtensions (:487-533)
    if ext is not None:
        if extensions:
            return dict(r, kind=None)
        return closing(C_INVALID_EXTENSIONS)
    return dict(r, kind=FINISHED)


CLIENT_TARGETS = ("UPGRADE", "CONNECTION", "SEC-WEBSOCKET-ACCEPT", "SEC-WEBSOCKET-PROTOCOL", "SEC-WEBSOCKET-EXTENSIONS")


def gpu_defers_client(data: bytes, key: str, max_length=65536, subprotocols=None, extensions=False):
    """The forms k_hs_validate hands to the Java Handshaker, in its walk order (the
    status line, then the header lines, then validate), or None."""
    flen, lines, capped = available(data)
    if capped:
        return D_LINES
    if flen == 0 or flen > max_length:
        return None
    try:
        parse_response(data[:flen], lines[:1])
    except InvalidHandshake:
        return None
    seen = set()
    for (b, e) in lines[1:]:
        code, t = split_header_field(data, b, e)
        if code != 4:
            return D_LINE_FORM
        name = ascii_str(data[t[0]:t[1]]).upper()
        if name in CLIENT_TARGETS:
            if name in seen:
                return D_REPEATED
            seen.add(name)
            if any(x >= 0x80 for x in data[t[2]:t[3]]):
                return D_NON_ASCII
    r = validate(data, key, max_length, None, False)
    if r["kind"] == CLOSING and r["cause"] in (C_INVALID_STATUS, C_MISSING_UPGRADE, C_MISSING_CONNECTION,
                                                 C_INVALID_UPGRADE, C_INVALID_CONNECTION, C_MISSING_ACCEPT,
                                                 C_INVALID_ACCEPT):
        return None
    _, f = parse_response(data[:flen], lines)
    if subprotocols:  # a missing answer closes; a present one is Java's list match
        return D_SUBPROTOCOL if f.get("Sec-WebSocket-Protocol") is not None else None
    if f.get("Sec-WebSocket-Protocol") is not None:
        return None
    if extensions and f.get("Sec-WebSocket-Extensions") is not None:
        return D_EXTENSION
    return None


def response(status=101, reason="Switching Protocols", fields=None) -> bytes:
    """A response the way HandshakeFactory.format writes one (:141-157)."""
    out = b"HTTP/1.1 %03d %s\r\n" % (status, reason.encode())
    for n, v in (fields or []):
        out += n.encode() + b": " + v.encode() + b"\r\n"
    return out + b"\r\n"
