"""The Java integration sources (java/, jni/) against the C ABI, without a JDK:
every native method of Wsg.java has its JNI function in jni/wsgpu_jni.c (and no
JNI function lacks its declaration), and every libwsgpu entry point the glue calls
is declared in include/wsgpu.h and exported by libwsgpu.so."""
import ctypes as C
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "org", "snf4j", "websocket", "gpu")


def _read(*p):
    with open(os.path.join(ROOT, *p)) as fh:
        return fh.read()


def test_every_native_method_has_its_jni_function():
    natives = set(re.findall(r"static native \S+ (\w+)\(", _read("java/org/snf4j/websocket/gpu/Wsg.java")))
    jni = set(re.findall(r"Java_org_snf4j_websocket_gpu_Wsg_(\w+)\(", _read("jni/wsgpu_jni.c")))
    assert natives and natives == jni, (natives - jni, jni - natives)


def test_glue_calls_only_declared_exported_entry_points():
    from snf4j_amd import _lib
    called = set(re.findall(r"\b(wsg_[a-z_]+)\(", _read("jni/wsgpu_jni.c")))
    declared = set(re.findall(r"\b(wsg_[a-z_]+)\(", _read("include/wsgpu.h")))
    assert called <= declared, called - declared
    lib = C.CDLL(_lib.LIB_PATH)
    assert all(hasattr(lib, f) for f in called)


def test_stage_classes_keep_the_reference_keys_and_types():
    cfg = _read("java/org/snf4j/websocket/gpu/GpuWebSocketSessionConfig.java")
    assert "pipeline.replace(HANDSHAKE_DECODER, WEBSOCKET_DECODER" in cfg
    assert "pipeline.replace(HANDSHAKE_ENCODER, WEBSOCKET_ENCODER" in cfg
    assert "WEBSOCKET_UTF8_VALIDATOR" in cfg
    dec = _read("java/org/snf4j/websocket/gpu/GpuFrameDecoder.java")
    assert "implements IBaseDecoder<ByteBuffer, Frame>" in dec
    assert "session.release(data)" in dec  # exactly once, FrameDecoder.java:285-287
    assert "executenf" in _read("java/org/snf4j/websocket/gpu/WsgBatcher.java")
    files = sorted(os.listdir(JAVA))
    assert files == ["GpuFrameDecoder.java", "GpuFrameEncoder.java", "GpuWebSocketSessionConfig.java",
                     "PinnedByteBufferAllocator.java", "Wsg.java", "WsgBatcher.java"]


def test_java_messages_match_the_python_mirror():
    """Wsg.message() builds the reference's exception texts: the same table as
    snf4j_amd/context.py MESSAGES (checked against the oracle in test_abi)."""
    from snf4j_amd.context import MESSAGES
    java = _read("java/org/snf4j/websocket/gpu/Wsg.java")
    for code in range(1, 17):
        text = MESSAGES[code].split("{")[0].rstrip(" (")
        assert text in java, (code, text)
