"""The Java integration sources (java/, jni/) against the C ABI, without a JDK:
every native method of Wsg.java has its JNI function in jni/wsgpu_jni.c (and no
JNI function lacks its declaration), every libwsgpu entry point the glue calls
is declared in include/wsgpu.h and exported by libwsgpu.so, and the stage
classes keep the reference's keys, types and lifecycle hooks."""
import ctypes as C
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "org", "snf4j", "websocket", "gpu")


def _read(*p):
    with open(os.path.join(ROOT, *p)) as fh:
        return fh.read()


def _java(name):
    return _read("java/org/snf4j/websocket/gpu", name)


def test_every_native_method_has_its_jni_function():
    natives = set(re.findall(r"static native \S+ (\w+)\(", _java("Wsg.java")))
    jni = set(re.findall(r"Java_org_snf4j_websocket_gpu_Wsg_(\w+)\(", _read("jni/wsgpu_jni.c")))
    assert natives and natives == jni, (natives - jni, jni - natives)


def test_every_native_method_is_used():
    natives = set(re.findall(r"static native \S+ (\w+)\(", _java("Wsg.java")))
    body = "".join(_java(f) for f in os.listdir(JAVA) if f != "Wsg.java")
    unused = {n for n in natives if f"Wsg.{n}(" not in body}
    # the handshake natives are bound for the handshake stages INTEGRATION.md §1.3d-e describes
    assert unused <= {"handshakeAvailable", "handshakeAcceptBatchHost", "handshakeValidateBatchHost",
                      "batcherSessionState", "checkHeader", "encodedLength", "encodeBatchHost",
                      "validateBatchHost", "batcherFlush", "batcherFeed", "batcherFeedArray"}, unused


def test_glue_calls_only_declared_exported_entry_points():
    from snf4j_amd import _lib
    called = set(re.findall(r"\b(wsg_[a-z_]+)\(", _read("jni/wsgpu_jni.c")))
    declared = set(re.findall(r"\b(wsg_[a-z_]+)\(", _read("include/wsgpu.h")))
    assert called <= declared, called - declared
    lib = C.CDLL(_lib.LIB_PATH)
    assert all(hasattr(lib, f) for f in called)


def test_stage_classes_keep_the_reference_keys_and_types():
    cfg = _java("GpuWebSocketSessionConfig.java")
    assert "pipeline.replace(HANDSHAKE_DECODER, WEBSOCKET_DECODER" in cfg
    assert "pipeline.replace(HANDSHAKE_ENCODER, WEBSOCKET_ENCODER" in cfg
    # the validator stage is the GPU one now (fused or after GPU inflate), not the CPU FrameUtf8Validator
    assert "addAfter(WEBSOCKET_DECODER, WEBSOCKET_UTF8_VALIDATOR, new GpuFrameUtf8Validator())" in cfg
    assert "new FrameUtf8Validator()" not in cfg
    dec = _java("GpuFrameDecoder.java")
    assert "implements IBaseDecoder<ByteBuffer, Frame>, IEventDrivenCodec" in dec
    # (release exactly once, FrameDecoder.java:285-287: test_decode_releases_data_exactly_once)
    assert "implements IEncoder<Frame, ByteBuffer>, IEventDrivenCodec" in _java("GpuFrameEncoder.java")
    for f in ("GpuPerMessageDeflateDecoder.java", "GpuFrameAggregator.java", "GpuFrameUtf8Validator.java"):
        assert "implements IDecoder<Frame, Frame>" in _java(f) and "GpuStage" in _java(f), f
    ext = _java("GpuPerMessageDeflateExtension.java")
    assert "implements IExtension" in ext and "PERMESSAGE_DEFLATE_DECODER" in ext
    assert "implements IEncoder<Frame, Frame>" in _java("GpuPerMessageDeflateEncoder.java")
    files = sorted(os.listdir(JAVA))
    assert files == ["GpuFrameAggregator.java", "GpuFrameDecoder.java", "GpuFrameEncoder.java",
                     "GpuFrameUtf8Validator.java", "GpuPerMessageDeflateDecoder.java",
                     "GpuPerMessageDeflateEncoder.java", "GpuPerMessageDeflateExtension.java", "GpuStage.java",
                     "GpuWebSocketSessionConfig.java", "PinnedByteBufferAllocator.java", "Wsg.java",
                     "WsgBatcher.java", "WsgDevices.java"]


def test_deflate_encoder_marker_is_installed_and_batched():
    """PerMessageDeflateExtension.updateEncoders (PerMessageDeflateExtension.java:303-313)
    puts PerMessageDeflateEncoder under "permessage-deflate-encoder"; the GPU extension
    wraps it there in GpuPerMessageDeflateEncoder with the negotiated noContext (the
    server's parameter for a server, :310) and attaches it to the GpuFrameEncoder, whose
    encode batcher then runs the deflate stage (wsg_enc_batcher_set_deflate) for every data
    frame of the session, whatever its size."""
    ext = _java("GpuPerMessageDeflateExtension.java")
    up = _body(ext, "public void updateEncoders(ICodecPipeline pipeline)", "public void updateDecoders(")
    order = ["delegate.updateEncoders(pipeline)", "pipeline.get(PerMessageDeflateExtension.PERMESSAGE_DEFLATE_ENCODER)",
             "SERVER_NO_CONTEXT : CLIENT_NO_CONTEXT", "pipeline.replace(PerMessageDeflateExtension.PERMESSAGE_DEFLATE_ENCODER",
             "pipeline.get(IWebSocketSessionConfig.WEBSOCKET_ENCODER)", ".attachDeflate(g)"]
    pos = [up.index(x) for x in order]
    assert pos == sorted(pos), order
    marker = _java("GpuPerMessageDeflateEncoder.java")
    enc = _body(marker, "public void encode(ISession session, Frame frame", "public void added(")
    assert "if (batched)" in enc and "out.add(frame)" in enc and "fallback.encode(session, frame, out)" in enc
    fe = _java("GpuFrameEncoder.java")
    att = fe[fe.index("void attachDeflate(GpuPerMessageDeflateEncoder d)"):fe.index("public void encode(ISession")]
    assert "if (sid >= 0 || deflate != null)" in att and "d.setBatched()" in att
    assert "!(deflate != null && data)" in fe and "batcher.registerEncoder(this, clientMode, deflate)" in fe
    b = _java("WsgBatcher.java")
    en = b[b.index("EncNative(boolean clientMode, GpuPerMessageDeflateEncoder deflate)"):]
    assert en.index("Wsg.encBatcherSetDeflate(handle, deflate.level, deflate.noContext)") < \
        en.index("Wsg.encBatcherReserve(handle")
    assert "wsg_enc_batcher_set_deflate(ENC_BATCHER(b)" in _read("jni/wsgpu_jni.c")


def test_session_lifecycle_reaches_the_native_reset():
    """ENDING / removed -> unregister -> wsg_batcher_session_reset (and the encoder's)."""
    dec = _java("GpuFrameDecoder.java")
    assert "event == SessionEvent.ENDING" in dec and "batcher.unregister(this)" in dec
    assert "public void removed(ISession session, ICodecPipeline pipeline)" in dec
    enc = _java("GpuFrameEncoder.java")
    assert "event == SessionEvent.ENDING" in enc and "batcher.unregisterEncoder(this)" in enc
    b = _java("WsgBatcher.java")
    assert "Wsg.batcherSessionReset(n.handle, d.sid)" in b and "Wsg.encBatcherSessionReset(n.handle, e.sid)" in b
    assert "wsg_batcher_session_reset" in _read("jni/wsgpu_jni.c")


def test_flush_is_deferred_not_inline():
    """The flush is queued on the loop (SelectorLoop.executenf always queues), never
    ISession.executenf, which runs the task inline on the loop thread."""
    b = _java("WsgBatcher.java")
    assert "loop.executenf(flushTask)" in b
    assert "session.executenf" not in b and ".executenf(new Runnable" not in b


def test_feed_handles_every_buffer_kind():
    b = _java("WsgBatcher.java")
    assert "data.hasArray()" in b and "data.isDirect()" in b and "data.duplicate().get(b)" in b
    jni = _read("jni/wsgpu_jni.c")
    assert "GetDirectBufferCapacity" in jni and "if (!p || cap < 0 || (uint64_t)cap < need)" in jni


def test_java_messages_match_the_python_mirror():
    """Wsg.message() builds the reference's exception texts: the same table as
    snf4j_amd/context.py MESSAGES (checked against the oracle in test_abi)."""
    from snf4j_amd.context import MESSAGES
    java = _java("Wsg.java")
    for code in range(1, 21):
        if code == 17:
            continue
        text = MESSAGES[code].split("{")[0].rstrip(" (")
        assert text in java, (code, text)


def _body(src, start, end):
    return src[src.index(start):src.index(end)]


def test_loop_scheduling_matches_the_python_restatement():
    """WsgBatcher's flush does what snf4j_amd/loop.py (run on the GPU by
    tests/test_gpu_loop.py) does, in the same order: the iteration's reads in one
    batcherFeedMany, the finished flushes collected without waiting (await 0, 0), the
    oldest collected only when two are in flight, then flushAsync + ticket handed to the
    completion thread; the completion thread calls only the await natives and re-enters
    the loop with executenf (never schedule() from inside the task phase)."""
    b = _java("WsgBatcher.java")
    flush = _body(b, "synchronized void flush()", "private static void check(")
    order = ["feedReads(n)", "collectReady(n)", "n.inflight.size() == Wsg.BATCHER_MAX_INFLIGHT",
             "Wsg.batcherFlushAsync(n.handle)",
             "Wsg.batcherTicket(n.handle)", "completion.watch(n.handle, t, false)"]
    pos = [flush.index(x) for x in order]
    assert pos == sorted(pos), order
    enc = ["collectReady(n)", "n.inflight.size() == 2", "Wsg.encBatcherFlushAsync(n.handle)",
           "Wsg.encBatcherTicket(n.handle)", "completion.watch(n.handle, t, true)"]
    encflush = flush[flush.index("for (EncNative n : encNatives)"):]
    pos = [encflush.index(x) for x in enc]
    assert pos == sorted(pos), enc
    assert "schedule()" not in flush
    feed = _body(b, "private void feedReads(Native n)", "synchronized void collectReady()")
    assert feed.count("Wsg.batcherFeedMany(") == 1 and "release(n.owned[i])" in feed
    comp = _body(b, "private final class Completion", "final long ctx;")
    natives = set(re.findall(r"Wsg\.(\w+)\(", comp))
    assert natives == {"batcherAwait", "encBatcherAwait"}, natives
    assert "loop.executenf(collectTask)" in comp
    ready = _body(b, "private void collectReady(Native n)", "private void collectReady(EncNative n)")
    assert "Wsg.batcherAwait(n.handle, 0, 0)" in ready
    loop = _read("snf4j_amd/loop.py")
    for x in ("feed_many", "collect_ready()", "len(self.inflight) == self.max_inflight", "flush_async()", "ticket()",
              "_completion.watch(t)", "await_done(0, 0)", "executenf(self.task)"):
        assert x in loop, x


def test_decode_releases_data_exactly_once():
    """FrameDecoder.java:285-287: the decoder releases its input once — GpuFrameDecoder
    when it swallows it (closed, released, a failed registration), else the batcher
    after the flush copied it (feedReads), when the session ends first (unregister), or
    at close."""
    dec = _java("GpuFrameDecoder.java")
    body = _body(dec, "public void decode(ISession session, ByteBuffer data", "private WsgBatcher.Cfg stages(")
    assert body.count("session.release(data)") == 2 and "batcher.enqueue(this, session, data)" in body
    b = _java("WsgBatcher.java")
    assert b.count(".release(n.owned[i])") == 3  # feedReads, unregister, close


def test_encode_flush_is_pipelined():
    """The encode batch queued by a flush is written by a later collect (its await
    done) or, with two in flight, before the next is queued; a CLOSE frame
    (flushEncodes) first writes out everything in flight, so writes keep their order;
    hasQueued is a per-encoder count, not a scan."""
    b = _java("WsgBatcher.java")
    sync = _body(b, "synchronized void flushEncodes()", "private void writeOldest(")
    assert sync.index("writeOldest(n)") < sync.index("Wsg.encBatcherFlush(n.handle, views)")
    hq = _body(b, "boolean hasQueued(GpuFrameEncoder e)", "/* ------------------------------------------------------------------ flush */")
    assert "e.batches > 0" in hq and "for (" not in hq
    assert "e.batches--" in _body(b, "private void write(EncNative n", "private void failSessions(Native n")
    jni = _read("jni/wsgpu_jni.c")
    assert "wsg_enc_batcher_flush_async(ENC_BATCHER(b))" in jni and "wsg_enc_batcher_wait(ENC_BATCHER(b), &v)" in jni


def test_close_releases_the_loop_device():
    b = _java("WsgBatcher.java")
    close = b[b.index("public void close()"):]
    assert "completion.join()" in close and "if (ownsDevice)" in close and "WsgDevices.release(loop)" in close


def test_decoder_close_control_matches_the_restatement():
    """GpuFrameDecoder ends a session as InternalSession.exception/controlClose does
    (InternalSession.java:804-848) — GENTLE: exception(closing cause) + close(); NONE:
    the exception only, the next frame goes on; DEFAULT or any other exception:
    quickClose() — for exceptions of the decoders behind it and of the handler's read,
    and delivers the frames before a u64 length error (WsgBatcher.drain) before
    available() throws it (FrameDecoder.java:388-394).  snf4j_amd/loop.py's
    GpuFrameDecoder does the same, run against the reference by
    tests/test_session_model.py (CPU batcher) and tests/test_gpu_session.py (GPU)."""
    dec = _java("GpuFrameDecoder.java")
    cc = _body(dec, "private boolean controlClose(Throwable t)", "void failBatch(Exception e)")
    assert "t instanceof ICloseControllingException" in cc and "c.getClosingCause()" in cc
    gentle = _body(cc, "case GENTLE:", "case NONE:")
    assert "handler.exception(cause)" in gentle and "session.close()" in gentle and "return false" in gentle
    none = _body(cc, "case NONE:", "default:")
    assert "handler.exception(cause)" in none and "return true" in none and "close" not in none
    tail = cc[cc.index("default:"):]
    assert "t = cause" in tail and "handler.exception(t)" in tail and "session.quickClose()" in tail
    down = _body(dec, "private boolean downstream(Frame frame", "private boolean controlClose(")
    # the handler's read is inside the try: its exceptions end the session the same way
    assert down.index("try {") < down.index("session.getHandler().read(o)") < down.index("catch (Exception e)")
    assert "return controlClose(e)" in down
    deliver = _body(dec, "void deliver(List<Frame> frames", "/** The decoders after")
    assert "if (!downstream(f, chain))" in deliver
    chk = _body(dec, "private int checked(ISession session, long r, int len)", "/**\n\t * FrameDecoder.decode")
    assert chk.index("batcher.drain(this)") < chk.index("if (closed)") < chk.index("fail(session")
    fail = _body(dec, "private void fail(ISession session", "/* ---- IEventDrivenCodec")
    assert fail.index("writenf(new CloseFrame(") < fail.index("if (inAvailable)") < fail.index("controlClose(e)")
    b = _java("WsgBatcher.java")
    drain = _body(b, "synchronized void drain(GpuFrameDecoder d)", "/* ------------------------------------------------------------------ encode side */")
    order = ["feedReads(n)", "Wsg.batcherFlushAsync(n.handle)", "while (!n.inflight.isEmpty())"]
    pos = [drain.index(x) for x in order]
    assert pos == sorted(pos), order
    assert "collectOldest(n)" in drain[pos[-1]:]
    loop = _read("snf4j_amd/loop.py")
    for x in ("def _control_close(self, t)", "self.batcher.drain(self)", "kind == CloseType.NONE",
              "s.quickClose()", "def drain(self, d: GpuFrameDecoder | None = None)"):
        assert x in loop, x


def test_inflight_limit_agrees():
    """WSG_BATCHER_MAX_INFLIGHT (wsgpu.h) = Wsg.BATCHER_MAX_INFLIGHT = _lib.BATCHER_MAX_INFLIGHT."""
    from snf4j_amd import _lib
    h = re.search(r"#define WSG_BATCHER_MAX_INFLIGHT (\d+)", _read("include/wsgpu.h"))
    j = re.search(r"static final int BATCHER_MAX_INFLIGHT = (\d+);", _java("Wsg.java"))
    assert h and j and int(h.group(1)) == int(j.group(1)) == _lib.BATCHER_MAX_INFLIGHT
