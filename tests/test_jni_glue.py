"""The JNI glue (jni/wsgpu_jni.c) compiled and run without a JVM: against the stub
tests/jni/jni.h, in the fake JNIEnv of tests/jni/fake_jni.c (tests/jni_harness.py).
CPU only: the calls here are those that reach no device (header framing, the
argument checks that return before any libwsgpu call).  The device lifecycle is
tests/test_gpu_jni.py.  Reference contract: IBaseDecoder.java:49-94 (available must
not move the buffer, decode owns it), FrameDecoder.java:357-401 (available)."""
import os
import subprocess

import numpy as np
import pytest

from tests import jni_harness
from tests.golden import fixtures, make_golden

ROOT = jni_harness.ROOT
EINVAL = -1
DUMMY = 0x1000  # a batcher / context handle the glue must never dereference in these calls


@pytest.fixture(scope="module")
def jni():
    jni_harness.build()
    j = jni_harness.Jni()
    yield j
    j.free_all()


@pytest.mark.parametrize("src", ["jni/wsgpu_jni.c", "tests/jni/fake_jni.c"])
def test_glue_compiles_warning_free(tmp_path, src):
    """-Wall -Wextra -Werror, C11, against the stub header (every JNI call the glue
    makes must exist in the stub with the specification's signature)."""
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-Wshadow", "-Wformat=2",
                        "-I", os.path.join(ROOT, "tests", "jni"), "-c", os.path.join(ROOT, src),
                        "-o", str(tmp_path / "x.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_java_natives_match_the_c_definitions():
    """Every native of Wsg.java has its Java_..._Wsg_ function with the JNI types javah
    would generate (int -> jint, long -> jlong, boolean -> jboolean, ByteBuffer ->
    jobject, byte[] -> jbyteArray, T[] of objects -> jobjectArray, String -> jstring)."""
    java = jni_harness.java_signatures()
    c = jni_harness.glue_signatures()
    assert set(java) == set(c), (set(java) ^ set(c))
    for name in java:
        assert java[name] == c[name], (name, java[name], c[name])


def _avail_array(jni, data: bytes, off: int, ln: int):
    err = jni.longs(4)
    r = jni.call("frameAvailable", jni.bytes_(data), off, ln, err)
    return r, jni.long_values(err)


def _avail_direct(jni, data: bytes, off: int, ln: int):
    err = jni.longs(4)
    buf = np.frombuffer(data, np.uint8).copy()
    r = jni.call("frameAvailableDirect", jni.direct(buf), off, ln, err)
    return r, jni.long_values(err)


@pytest.mark.parametrize("form", ["array", "direct"])
def test_available_kat_through_jni(jni, form):
    """FrameDecoderTest's available KATs (:229-367) through both available natives:
    the frame length when complete, else 0 below the header; the u64 length errors as
    -1 with {status, detail, detail2} that Wsg.message turns into the reference text."""
    from snf4j_amd.context import error_message
    call = _avail_array if form == "array" else _avail_direct
    av = fixtures.load("available")
    for c in av["frames"]:
        data = make_golden.frame(c["data_spec"], c["off"])
        n = c["expected_len"]
        hdr = n - c["payload_len"]
        for ln in sorted({0, 1, hdr - 1, hdr, n - 1, n, n + 7}):
            if ln < 0 or c["off"] + min(ln, 14) > len(data):
                continue
            r, err = call(jni, data, c["off"], ln)
            assert r == (n if ln >= n else (ln if ln >= hdr else 0)), (c, ln, r)
            if r > 0:
                assert err[3] == n  # the whole frame (GpuFrameDecoder tracks the rest with it)
    for c in av["big"]:
        data = fixtures.unhex(c["data"])
        if form == "direct":  # a direct buffer holds the bytes the call reads
            data = data + b"\x00" * 16
        r, err = call(jni, data, 0, min(c["len"], len(data)) if form == "direct" else c["len"])
        if "error" in c:
            assert r == -1
            assert error_message(int(err[0]), int(err[1]), int(err[2])) == c["error"]
        elif form == "array":
            assert r == c["expect"]


def test_available_does_not_read_past_the_caller_bytes(jni):
    """-2 (never an exception, never a read) when the header bytes are not there."""
    frame = bytes([0x82, 0x85, 1, 2, 3, 4]) + b"hello"
    err = jni.longs(4)
    assert jni.call("frameAvailable", jni.bytes_(frame), 8, 6, err) == -2       # off + header past the array
    assert jni.call("frameAvailable", jni.bytes_(frame), -1, 4, err) == -2
    assert jni.call("frameAvailable", jni.bytes_(frame), 0, -1, err) == -2
    assert jni.call("frameAvailable", 0, 0, 4, err) == -2                        # null array
    assert jni.call("frameAvailable", jni.bytes_(frame), 0, 11, jni.longs(3)) == -2  # err too short
    buf = np.frombuffer(frame, np.uint8).copy()
    assert jni.call("frameAvailableDirect", jni.bytes_(frame), 0, 11, err) == -2   # not a direct buffer
    assert jni.call("frameAvailableDirect", jni.direct(buf, cap=4), 0, 11, err) == -2  # capacity short
    assert jni.call("frameAvailableDirect", jni.direct(buf), 0, 11, err) == 11


def test_check_header_through_jni(jni):
    """wsg_check_header (the header rules of FrameDecoder.decode, :197-256) through the
    glue: opcode, RSV, masking, control rules, with detail = the message argument."""
    from snf4j_amd import _lib
    det = jni.longs(1)
    cases = [(bytes([0x83, 0x80, 1, 2, 3, 4]), 1, 3),   # Unexpected opcode value (3)
             (bytes([0xC2, 0x80, 1, 2, 3, 4]), 2, 4),   # Unexpected non-zero RSV bits (4)
             (bytes([0x82, 0x00]), 3, 0),               # Unexpected payload masking (server side)
             (bytes([0x09, 0x80, 1, 2, 3, 4]), 4, 0),   # Fragmented control frame
             (bytes([0x82, 0x85, 1, 2, 3, 4]), 0, 0)]
    for hdr, status, detail in cases:
        buf = np.frombuffer(hdr, np.uint8).copy()
        s = jni.call("checkHeader", 0, 0, 65536, 0, jni.direct(buf), 0, len(hdr), det)
        assert (s, int(jni.long_values(det)[0])) == (status, detail), hdr.hex()
        cfg = _lib.DecoderCfg(0, 0, 65536, 0, 0)
        d = _lib.C.c_int64()
        assert s == _lib.lib.wsg_check_header(_lib.C.byref(cfg), 0, buf.ctypes.data, len(hdr), _lib.C.byref(d))
    buf = np.zeros(8, np.uint8)
    assert jni.call("checkHeader", 0, 0, 65536, 0, jni.direct(buf), 4, 6, det) == EINVAL
    assert jni.call("checkHeader", 0, 0, 65536, 0, jni.direct(buf), 0, 2, jni.longs(0)) == EINVAL


def test_argument_checks_return_einval(jni):
    """Every call whose buffers or ranges do not hold what it would read or write
    returns WSG_API_EINVAL before any libwsgpu call (the handles here are dummies the
    glue never dereferences), with no JNI exception pending and no critical region."""
    a16 = np.zeros(16, np.uint8)
    d16 = jni.direct(a16)
    heap = jni.bytes_(b"\x00" * 16)
    # batcherFeed: direct buffers only, inside their capacity
    for args in [(DUMMY, 0, 0, 0, 4), (DUMMY, 0, heap, 0, 4), (DUMMY, 0, d16, 8, 9), (DUMMY, 0, d16, -1, 2),
                 (DUMMY, 0, d16, 0, -2), (DUMMY, -1, d16, 0, 4), (0, 0, d16, 0, 4)]:
        assert jni.call("batcherFeed", *args) == EINVAL, args
    for args in [(DUMMY, 0, heap, 10, 7), (DUMMY, 0, 0, 0, 1), (DUMMY, 0, heap, -3, 1), (DUMMY, -2, heap, 0, 1)]:
        assert jni.call("batcherFeedArray", *args) == EINVAL, args
    # batcherFeedMany: every read checked before any is fed (one bad read feeds nothing)
    good = (jni.ints([0, 1]), jni.objs([d16, 0]), jni.objs([0, heap]), jni.ints([0, 0]), jni.ints([16, 16]))
    bad_reads = [
        (jni.ints([0, 1]), jni.objs([d16, 0]), jni.objs([0, heap]), jni.ints([0, 0]), jni.ints([16, 17])),
        (jni.ints([0, 1]), jni.objs([d16, 0]), jni.objs([0, 0]), jni.ints([0, 0]), jni.ints([16, 1])),
        (jni.ints([0, -1]), jni.objs([d16, 0]), jni.objs([0, heap]), jni.ints([0, 0]), jni.ints([16, 1])),
        (jni.ints([0, 1]), jni.objs([d16, 0]), jni.objs([0, heap]), jni.ints([-1, 0]), jni.ints([4, 1])),
        (jni.ints([0]), jni.objs([d16, 0]), jni.objs([0, heap]), jni.ints([0, 0]), jni.ints([16, 16])),
    ]
    for arrays in bad_reads:
        assert jni.call("batcherFeedMany", DUMMY, 2, *arrays) == EINVAL
    assert jni.call("batcherFeedMany", 0, 2, *good) == EINVAL
    assert jni.call("batcherFeedMany", DUMMY, -1, *good) == EINVAL
    # views / counts arrays too short: refused before the flush is taken
    assert jni.call("batcherWait", DUMMY, jni.objs_empty(3), jni.longs(2)) == EINVAL
    assert jni.call("batcherWait", DUMMY, jni.objs_empty(5), jni.longs(1)) == EINVAL
    assert jni.call("batcherFlush", DUMMY, 0, jni.longs(2)) == EINVAL
    assert jni.call("encBatcherFlush", DUMMY, jni.objs_empty(2)) == EINVAL
    assert jni.call("encBatcherWait", DUMMY, jni.objs_empty(1)) == EINVAL
    assert jni.call("batcherSessionState", DUMMY, 0, jni.bytes_(b"1234567")) == EINVAL
    assert jni.call("batcherSessionReset", DUMMY, -1) == EINVAL
    assert jni.call("encBatcherSessionReset", DUMMY, -1) == EINVAL
    assert jni.call("encBatcherAdd", DUMMY, -1, 2, 0x80, 0, heap) == EINVAL
    assert jni.call("batcherAwait", 0, 0, 0) == EINVAL
    assert jni.call("batcherReserve", DUMMY, -1, 0) == EINVAL
    # the batch host calls: each buffer must cover its count
    z = lambda n: jni.direct(np.zeros(max(n, 1), np.uint8), cap=n)  # noqa: E731
    ok = dict(payload=z(64), frames=z(2 * 24), sf=z(3 * 4), closed=z(2), wire=z(256), woff=z(3 * 8))
    args = lambda **kw: (DUMMY, 1, kw.get("payload", ok["payload"]), 64, kw.get("frames", ok["frames"]), 2,  # noqa: E731
                         kw.get("sf", ok["sf"]), 2, kw.get("closed", ok["closed"]), kw.get("wire", ok["wire"]), 256,
                         kw.get("woff", ok["woff"]))
    for k, short in [("payload", z(63)), ("frames", z(47)), ("sf", z(11)), ("closed", z(1)), ("wire", z(255)),
                     ("woff", z(23)), ("frames", heap)]:
        assert jni.call("encodeBatchHost", *args(**{k: short})) == EINVAL, k
    assert jni.call("validateBatchHost", DUMMY, z(2 * 16), 2, z(3 * 4), 2, z(64), 64, z(2 * 8), z(2 * 16 - 1)) == EINVAL
    assert jni.call("validateBatchHost", DUMMY, z(2 * 16 - 1), 2, z(3 * 4), 2, z(64), 64, z(2 * 8), z(32)) == EINVAL
    offs = np.array([0, 10, 5], np.uint64)  # descending: not a request list
    assert jni.call("handshakeAcceptBatchHost", DUMMY, 0, z(64), jni.direct(offs), 2, z(320), z(32)) == EINVAL
    offs = np.array([0, 10, 70], np.uint64)  # past the request buffer
    assert jni.call("handshakeAcceptBatchHost", DUMMY, 0, z(64), jni.direct(offs), 2, z(320), z(32)) == EINVAL
    assert jni.call("handshakeValidateBatchHost", DUMMY, 0, z(64), jni.direct(np.array([0, 10, 20], np.uint64)),
                    z(47), 2, z(64), z(32)) == EINVAL
    assert jni.call("handshakeAvailable", heap, 10, 7) == -2
    assert jni.call("releasePinned", 0) == EINVAL
    assert jni.call("encodedLength", -1, 1) == EINVAL
    assert jni.call("reserve", DUMMY, -1, 1, 1) == EINVAL


def test_handshake_available_through_jni(jni):
    """HttpUtils.available (HttpUtils.java:77-111) through the glue == the C ABI, on the
    reference handshake vectors and every prefix of one request."""
    from snf4j_amd import _lib
    reqs = [fixtures.unhex(v["request"]) for v in fixtures.load("handshake") if v["kind"] == "accept"][:20]
    assert reqs
    for rq in reqs:
        for ln in sorted({0, 1, len(rq) // 2, len(rq) - 1, len(rq)}):
            a = np.frombuffer(rq[:ln] or b"\x00", np.uint8).copy()
            assert jni.call("handshakeAvailable", jni.bytes_(rq), 0, ln) == \
                _lib.lib.wsg_handshake_available(a.ctypes.data, ln)
    big = b"GET / HTTP/1.1\r\n" + b"X: y\r\n" * 2000
    assert jni.call("handshakeAvailable", jni.bytes_(big), 0, len(big)) == -1  # > 8 KiB: the Java decoder's


def test_feed_many_local_references_stay_bounded(jni):
    """Thousands of reads in one feedMany call: the glue holds at most a group's local
    references at once (the JVM guarantees 16 without EnsureLocalCapacity; the glue
    ensures FEED_GROUP + 8), checked here with a bad last read so nothing is fed."""
    n = 3000
    heaps = [jni.bytes_(b"x") for _ in range(n)]
    lens = [1] * n
    lens[-1] = 2  # outside its array: EINVAL from the checking pass
    assert jni.call("batcherFeedMany", DUMMY, n, jni.ints(range(n)), jni.objs_empty(n), jni.objs(heaps),
                    jni.ints([0] * n), jni.ints(lens)) == EINVAL
    assert jni.peak <= 136, jni.peak
