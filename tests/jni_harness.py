"""Drive the JNI glue (jni/wsgpu_jni.c) without a JVM: the glue compiled against the
stub tests/jni/jni.h with the fake JNIEnv of tests/jni/fake_jni.c
(tests/jni/_build/libwsgpu_jni_test.so, built by `make -C jni harness`).

Jni.call("batcherFeed", b, sid, buf, off, len) calls
Java_org_snf4j_websocket_gpu_Wsg_batcherFeed(env, NULL, ...), as the JVM would for
Wsg.batcherFeed(...).  The argument and return types come from the C definitions
(jint -> c_int, jlong -> c_long, jboolean -> c_ubyte, every reference -> c_void_p).
Objects: direct(array) wraps a numpy array as a direct ByteBuffer, bytes_(data) a
byte[], ints/longs/objs the other arrays.  After every call the harness checks the
glue's JNI discipline (no exception left pending, no critical region left open, no
call inside one, no leaked local reference beyond what the call returns) — the
checks a JVM's -Xcheck:jni makes.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLUE = os.path.join(ROOT, "jni", "wsgpu_jni.c")
HARNESS = os.path.join(ROOT, "tests", "jni", "_build", "libwsgpu_jni_test.so")

_CTYPE = {"jint": C.c_int, "jlong": C.c_long, "jboolean": C.c_ubyte, "void": None}
_JAVA_TO_JNI = {"int": "jint", "long": "jlong", "boolean": "jboolean", "void": "void", "String": "jstring",
                "ByteBuffer": "jobject", "byte[]": "jbyteArray", "int[]": "jintArray", "long[]": "jlongArray",
                "ByteBuffer[]": "jobjectArray", "byte[][]": "jobjectArray", "Object[]": "jobjectArray"}


def glue_signatures() -> dict[str, tuple[str, list[str]]]:
    """name -> (return JNI type, [JNI parameter types after env and jclass])."""
    with open(GLUE) as fh:
        src = fh.read()
    out = {}
    for ret, name, params in re.findall(
            r"JNIEXPORT\s+(\w+)\s+JNICALL\s+Java_org_snf4j_websocket_gpu_Wsg_(\w+)\s*\(([^)]*)\)", src, re.S):
        types = [p.strip().rsplit(None, 1)[0].replace(" ", "") for p in params.split(",")]
        assert types[0] == "JNIEnv*" and types[1] == "jclass", name
        out[name] = (ret, types[2:])
    return out


def java_signatures() -> dict[str, tuple[str, list[str]]]:
    """name -> (JNI return type, [JNI parameter types]) of Wsg.java's natives, as javah maps them."""
    with open(os.path.join(ROOT, "java", "org", "snf4j", "websocket", "gpu", "Wsg.java")) as fh:
        src = fh.read()
    out = {}
    for ret, name, params in re.findall(r"static native ([\w\[\]]+) (\w+)\(([^)]*)\)", src, re.S):
        ps = [p.strip().rsplit(None, 1)[0] for p in params.split(",") if p.strip()]
        out[name] = (_JAVA_TO_JNI[ret], [_JAVA_TO_JNI[p] for p in ps])
    return out


def build() -> str:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "jni"), "harness"], check=True)
    return HARNESS


class JniError(AssertionError):
    pass


class Jni:
    """The glue in a fake JVM.  Objects live until free_all()."""

    def __init__(self, path: str = HARNESS):
        from snf4j_amd import _lib  # noqa: F401  (loads libwsgpu.so with torch's HIP runtime first)
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built: make -C jni harness")
        self.L = C.CDLL(path)
        L = self.L
        vp = C.c_void_p
        for name, (args, res) in {
            "fj_env": ([], vp), "fj_direct": ([vp, C.c_long], vp), "fj_bytes": ([C.c_long], vp),
            "fj_ints": ([C.c_long], vp), "fj_longs": ([C.c_long], vp), "fj_objs": ([C.c_long], vp),
            "fj_kind": ([vp], C.c_int), "fj_data": ([vp], vp), "fj_len": ([vp], C.c_long),
            "fj_cap": ([vp], C.c_long), "fj_get": ([vp, C.c_long], vp), "fj_set": ([vp, C.c_long, vp], None),
            "fj_exception": ([], C.c_int), "fj_exception_msg": ([], C.c_char_p), "fj_clear": ([], None),
            "fj_violations": ([], C.c_long), "fj_critical": ([], C.c_int), "fj_local_refs": ([], C.c_long),
            "fj_local_peak": ([], C.c_long), "fj_calls": ([], C.c_long), "fj_return": ([], None),
            "fj_free_all": ([], None),
        }.items():
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        self.env = L.fj_env()
        self.sigs = glue_signatures()
        self._fn = {}
        for name, (ret, params) in self.sigs.items():
            f = getattr(L, "Java_org_snf4j_websocket_gpu_Wsg_" + name)
            f.argtypes = [vp, vp] + [_CTYPE.get(p, vp) for p in params]
            f.restype = _CTYPE.get(ret, vp)
            self._fn[name] = f
        self._keep = []  # numpy arrays wrapped as direct buffers stay alive

    # ---- objects
    def direct(self, arr: np.ndarray, cap: int | None = None):
        """A direct ByteBuffer over a (contiguous) numpy array's bytes."""
        assert arr.flags.c_contiguous
        self._keep.append(arr)
        return self.L.fj_direct(arr.ctypes.data, arr.nbytes if cap is None else cap)

    def bytes_(self, data) -> int:
        b = bytes(data)
        o = self.L.fj_bytes(len(b))
        if b:
            C.memmove(self.L.fj_data(o), b, len(b))
        return o

    def ints(self, vals) -> int:
        v = np.asarray(vals, dtype=np.int32)
        o = self.L.fj_ints(len(v))
        if len(v):
            C.memmove(self.L.fj_data(o), v.ctypes.data, v.nbytes)
        return o

    def longs(self, n: int) -> int:
        return self.L.fj_longs(n)

    def long_values(self, o) -> np.ndarray:
        n = self.L.fj_len(o)
        return np.ctypeslib.as_array((C.c_long * n).from_address(self.L.fj_data(o))).copy() if n else np.zeros(0)

    def objs(self, items) -> int:
        items = list(items)
        o = self.L.fj_objs(len(items))
        for i, x in enumerate(items):
            if x:
                self.L.fj_set(o, i, x)
        return o

    def objs_empty(self, n: int) -> int:
        return self.L.fj_objs(n)

    def element(self, arr, i):
        return self.L.fj_get(arr, i)

    def buffer(self, o, dtype=np.uint8) -> np.ndarray:
        """A direct buffer's bytes as a numpy view (the glue's NewDirectByteBuffer)."""
        assert self.L.fj_kind(o) == 1, "not a direct buffer"
        cap = self.L.fj_cap(o)
        if cap == 0:
            return np.zeros(0, dtype=dtype)
        raw = np.ctypeslib.as_array((C.c_uint8 * cap).from_address(self.L.fj_data(o)))
        return raw.view(dtype) if np.dtype(dtype).itemsize > 1 else raw

    def string(self, o) -> str:
        return C.string_at(self.L.fj_data(o), self.L.fj_len(o)).decode()

    # ---- calls
    def call(self, name, *args, returns_refs: int = 0):
        """Wsg.<name>(args) through the glue, then the JNI discipline checks."""
        v0 = self.L.fj_violations()
        r = self._fn[name](self.env, None, *args)
        if self.L.fj_exception():
            msg = self.L.fj_exception_msg().decode()
            self.L.fj_clear()
            raise JniError(f"{name} left a pending exception: {msg}")
        if self.L.fj_critical():
            raise JniError(f"{name} returned inside a critical region")
        if self.L.fj_violations() != v0:
            raise JniError(f"{name}: JNI call inside a critical region or with an exception pending")
        if self.L.fj_local_refs() > returns_refs:
            raise JniError(f"{name} leaked {self.L.fj_local_refs() - returns_refs} local references")
        self.peak = self.L.fj_local_peak()
        self.L.fj_return()
        return r

    def free_all(self):
        self.L.fj_free_all()
        self._keep.clear()
