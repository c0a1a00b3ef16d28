/* A fake JNIEnv for running jni/wsgpu_jni.c without a JVM (test infrastructure;
 * built with the stub tests/jni/jni.h into tests/jni/_build/libwsgpu_jni_test.so).
 *
 * Objects are C records: direct ByteBuffers (an address and a capacity), byte /
 * int / long arrays, object arrays and strings.  The functions behave as the JNI
 * specification describes for a JVM:
 *  - Get/Set<Type>ArrayRegion outside the array, or on null, leave a pending
 *    ArrayIndexOutOfBoundsException / NullPointerException and copy nothing;
 *  - GetDirectBufferAddress returns NULL and GetDirectBufferCapacity -1 for an
 *    object that is not a direct buffer;
 *  - between GetPrimitiveArrayCritical and its release only critical calls are
 *    allowed: any other call there counts as a violation;
 *  - a JNI call (other than ExceptionCheck and DeleteLocalRef) with an exception
 *    pending counts as a violation.
 * The harness (tests/test_jni_glue.py, tests/test_gpu_jni.py) builds objects with
 * the fj_* functions, calls the Java_* entry points with fj_env(), and reads the
 * counters to check the glue's discipline. */
#define _POSIX_C_SOURCE 200809L /* strdup */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_DIRECT = 1, K_BYTES, K_INTS, K_LONGS, K_OBJS, K_STRING };

struct _jobject {
    int kind;
    jlong len;      /* array elements / string bytes */
    void* data;     /* array storage, string bytes, or the direct buffer's address */
    jlong cap;      /* direct buffer capacity */
    int owned;      /* data is ours to free */
    struct _jobject* next;
};

static struct _jobject* g_all;
static int g_exc;                 /* 0 none, 1 AIOOBE, 2 NPE, 3 thrown by ThrowNew */
static char g_exc_msg[256];
static int g_critical;            /* critical regions open */
static long g_violations;
static long g_local_refs;         /* live local references the glue holds */
static long g_local_peak;
static long g_calls;

/* a local reference handed to the glue (a new object, or an array element) */
static void local_ref(void) {
    if (++g_local_refs > g_local_peak) g_local_peak = g_local_refs;
}

static struct _jobject* obj_new(int kind, jlong len, int local) {
    struct _jobject* o = (struct _jobject*)calloc(1, sizeof *o);
    o->kind = kind;
    o->len = len;
    o->next = g_all;
    g_all = o;
    if (local) local_ref();
    return o;
}

static void enter(int critical_ok) {
    ++g_calls;
    if (g_critical && !critical_ok) ++g_violations;
    if (g_exc) ++g_violations;
}

static void throw_(int kind, const char* msg) {
    if (!g_exc) {
        g_exc = kind;
        snprintf(g_exc_msg, sizeof g_exc_msg, "%s", msg);
    }
}


static size_t elem(int kind) {
    switch (kind) {
    case K_BYTES: return 1;
    case K_INTS: return 4;
    case K_LONGS: return 8;
    case K_OBJS: return sizeof(jobject);
    default: return 0;
    }
}

/* the region functions: copy between an array and a C buffer, or throw */
static void region(jarray a, int kind, jsize start, jsize len, void* buf, int set) {
    enter(0);
    if (!a) {
        throw_(2, "java/lang/NullPointerException");
        return;
    }
    if (a->kind != kind) {  /* a JVM would crash or corrupt; the glue must never do it */
        ++g_violations;
        return;
    }
    if (start < 0 || len < 0 || (jlong)start + len > a->len) {
        throw_(1, "java/lang/ArrayIndexOutOfBoundsException");
        return;
    }
    const size_t e = elem(kind);
    if (set)
        memcpy((uint8_t*)a->data + (size_t)start * e, buf, (size_t)len * e);
    else
        memcpy(buf, (uint8_t*)a->data + (size_t)start * e, (size_t)len * e);
}

static jint JNICALL f_EnsureLocalCapacity(JNIEnv* env, jint capacity) {
    (void)env;
    enter(0);
    return capacity < 0 ? JNI_ERR : JNI_OK;
}

static void JNICALL f_DeleteLocalRef(JNIEnv* env, jobject obj) {
    (void)env;
    ++g_calls;
    if (g_critical) ++g_violations;
    if (obj) --g_local_refs;
}

static jint JNICALL f_ThrowNew(JNIEnv* env, jclass clazz, const char* msg) {
    (void)env;
    (void)clazz;
    enter(0);
    throw_(3, msg ? msg : "");
    return JNI_OK;
}

static jclass JNICALL f_FindClass(JNIEnv* env, const char* name) {
    (void)env;
    enter(0);
    struct _jobject* o = obj_new(K_STRING, (jlong)strlen(name), 1);
    o->data = strdup(name);
    o->owned = 1;
    return o;
}

static jboolean JNICALL f_ExceptionCheck(JNIEnv* env) {
    (void)env;
    ++g_calls;
    return g_exc ? JNI_TRUE : JNI_FALSE;
}

static jstring JNICALL f_NewStringUTF(JNIEnv* env, const char* utf) {
    (void)env;
    enter(0);
    if (!utf) return NULL;
    struct _jobject* o = obj_new(K_STRING, (jlong)strlen(utf), 1);
    o->data = strdup(utf);
    o->owned = 1;
    return o;
}

static jsize JNICALL f_GetArrayLength(JNIEnv* env, jarray array) {
    (void)env;
    enter(0);
    if (!array) {
        throw_(2, "java/lang/NullPointerException");
        return 0;
    }
    if (!elem(array->kind)) {
        ++g_violations;
        return 0;
    }
    return (jsize)array->len;
}

static jobject JNICALL f_GetObjectArrayElement(JNIEnv* env, jobjectArray array, jsize index) {
    (void)env;
    enter(0);
    if (!array) {
        throw_(2, "java/lang/NullPointerException");
        return NULL;
    }
    if (array->kind != K_OBJS) {
        ++g_violations;
        return NULL;
    }
    if (index < 0 || index >= array->len) {
        throw_(1, "java/lang/ArrayIndexOutOfBoundsException");
        return NULL;
    }
    jobject v = ((jobject*)array->data)[index];
    if (v) local_ref();
    return v;
}

static void JNICALL f_SetObjectArrayElement(JNIEnv* env, jobjectArray array, jsize index, jobject val) {
    (void)env;
    enter(0);
    if (!array) {
        throw_(2, "java/lang/NullPointerException");
        return;
    }
    if (array->kind != K_OBJS) {
        ++g_violations;
        return;
    }
    if (index < 0 || index >= array->len) {
        throw_(1, "java/lang/ArrayIndexOutOfBoundsException");
        return;
    }
    ((jobject*)array->data)[index] = val;
}

static void JNICALL f_GetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize n, jbyte* buf) {
    (void)env;
    region(a, K_BYTES, s, n, buf, 0);
}
static void JNICALL f_SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize n, const jbyte* buf) {
    (void)env;
    region(a, K_BYTES, s, n, (void*)buf, 1);
}
static void JNICALL f_GetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, jint* buf) {
    (void)env;
    region(a, K_INTS, s, n, buf, 0);
}
static void JNICALL f_GetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize n, jlong* buf) {
    (void)env;
    region(a, K_LONGS, s, n, buf, 0);
}
static void JNICALL f_SetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize n, const jlong* buf) {
    (void)env;
    region(a, K_LONGS, s, n, (void*)buf, 1);
}

static void* JNICALL f_GetPrimitiveArrayCritical(JNIEnv* env, jarray array, jboolean* isCopy) {
    (void)env;
    enter(1);
    if (isCopy) *isCopy = JNI_FALSE;
    if (!array) {
        throw_(2, "java/lang/NullPointerException");
        return NULL;
    }
    if (array->kind != K_BYTES && array->kind != K_INTS && array->kind != K_LONGS) {
        ++g_violations;
        return NULL;
    }
    ++g_critical;
    return array->data ? array->data : (void*)array;  /* (a zero-length array still pins) */
}

static void JNICALL f_ReleasePrimitiveArrayCritical(JNIEnv* env, jarray array, void* carray, jint mode) {
    (void)env;
    (void)mode;
    ++g_calls;
    if (!array || !carray || g_critical <= 0) {
        ++g_violations;
        return;
    }
    --g_critical;
}

static jobject JNICALL f_NewDirectByteBuffer(JNIEnv* env, void* address, jlong capacity) {
    (void)env;
    enter(0);
    if (capacity < 0 || capacity > INT32_MAX) {  /* a ByteBuffer's capacity is an int */
        throw_(3, "java/lang/IllegalArgumentException");
        return NULL;
    }
    struct _jobject* o = obj_new(K_DIRECT, 0, 1);
    o->data = address;
    o->cap = capacity;
    return o;
}

static void* JNICALL f_GetDirectBufferAddress(JNIEnv* env, jobject buf) {
    (void)env;
    enter(0);
    return buf && buf->kind == K_DIRECT ? buf->data : NULL;
}

static jlong JNICALL f_GetDirectBufferCapacity(JNIEnv* env, jobject buf) {
    (void)env;
    enter(0);
    return buf && buf->kind == K_DIRECT ? buf->cap : -1;
}

static const struct JNINativeInterface_ g_table = {
    NULL,
    f_EnsureLocalCapacity,
    f_DeleteLocalRef,
    f_ThrowNew,
    f_FindClass,
    f_ExceptionCheck,
    f_NewStringUTF,
    f_GetArrayLength,
    f_GetObjectArrayElement,
    f_SetObjectArrayElement,
    f_GetByteArrayRegion,
    f_SetByteArrayRegion,
    f_GetIntArrayRegion,
    f_GetLongArrayRegion,
    f_SetLongArrayRegion,
    f_GetPrimitiveArrayCritical,
    f_ReleasePrimitiveArrayCritical,
    f_NewDirectByteBuffer,
    f_GetDirectBufferAddress,
    f_GetDirectBufferCapacity,
};
static JNIEnv g_env = &g_table;

/* ---- harness side ---- */
JNIEXPORT JNIEnv* fj_env(void) { return &g_env; }

JNIEXPORT jobject fj_direct(void* addr, jlong cap) {
    struct _jobject* o = obj_new(K_DIRECT, 0, 0);
    o->data = addr;
    o->cap = cap;
    return o;
}

static jobject fj_array(int kind, jlong n) {
    struct _jobject* o = obj_new(kind, n, 0);
    o->data = calloc((size_t)(n ? n : 1), elem(kind));
    o->owned = 1;
    return o;
}
JNIEXPORT jobject fj_bytes(jlong n) { return fj_array(K_BYTES, n); }
JNIEXPORT jobject fj_ints(jlong n) { return fj_array(K_INTS, n); }
JNIEXPORT jobject fj_longs(jlong n) { return fj_array(K_LONGS, n); }
JNIEXPORT jobject fj_objs(jlong n) { return fj_array(K_OBJS, n); }

JNIEXPORT int fj_kind(jobject o) { return o ? o->kind : 0; }
JNIEXPORT void* fj_data(jobject o) { return o ? o->data : NULL; }
JNIEXPORT jlong fj_len(jobject o) { return o ? o->len : -1; }
JNIEXPORT jlong fj_cap(jobject o) { return o && o->kind == K_DIRECT ? o->cap : -1; }
JNIEXPORT jobject fj_get(jobject arr, jlong i) {
    return arr && arr->kind == K_OBJS && i >= 0 && i < arr->len ? ((jobject*)arr->data)[i] : NULL;
}
JNIEXPORT void fj_set(jobject arr, jlong i, jobject v) {
    if (arr && arr->kind == K_OBJS && i >= 0 && i < arr->len) ((jobject*)arr->data)[i] = v;
}

JNIEXPORT int fj_exception(void) { return g_exc; }
JNIEXPORT const char* fj_exception_msg(void) { return g_exc_msg; }
JNIEXPORT void fj_clear(void) {
    g_exc = 0;
    g_exc_msg[0] = 0;
}
JNIEXPORT long fj_violations(void) { return g_violations; }
JNIEXPORT int fj_critical(void) { return g_critical; }
JNIEXPORT long fj_local_refs(void) { return g_local_refs; }
JNIEXPORT long fj_local_peak(void) { return g_local_peak; }
JNIEXPORT long fj_calls(void) { return g_calls; }

/* the end of a native method: its local references are released (as the JVM does
 * when a native call returns) */
JNIEXPORT void fj_return(void) {
    g_local_refs = 0;
    g_local_peak = 0;
}

JNIEXPORT void fj_free_all(void) {
    while (g_all) {
        struct _jobject* o = g_all;
        g_all = o->next;
        if (o->owned) free(o->data);
        free(o);
    }
    g_exc = 0;
    g_critical = 0;
    g_violations = 0;
    g_local_refs = g_local_peak = 0;
    g_calls = 0;
}
