/* Test stub of <jni.h> for compiling jni/wsgpu_jni.c without a JDK (the image has
 * none).  It is test infrastructure, not a JVM header:
 *  - the primitive and reference types follow the JNI specification's C mapping on
 *    LP64 Linux (jni.h + jni_md.h: jint = int, jlong = long, jboolean = unsigned
 *    char, jbyte = signed char; every array and jclass/jstring is a jobject);
 *  - JNIEnv is a pointer to a function table, called as (*env)->Fn(env, ...), with
 *    the JNI specification's signature for each function;
 *  - but the table holds ONLY the functions the glue calls, in an order of its own,
 *    so code built against it runs only with the fake environment of
 *    tests/jni/fake_jni.c, never inside a JVM.
 * A call the glue adds that this table lacks fails to compile: add it here, with
 * its specification signature, and to fake_jni.c. */
#ifndef WSG_TEST_JNI_H
#define WSG_TEST_JNI_H

#include <stdarg.h>

typedef unsigned char jboolean;
typedef signed char jbyte;
typedef unsigned short jchar;
typedef short jshort;
typedef int jint;
typedef long jlong;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbooleanArray;
typedef jarray jbyteArray;
typedef jarray jcharArray;
typedef jarray jshortArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_OK 0
#define JNI_ERR (-1)
#define JNI_COMMIT 1
#define JNI_ABORT 2

#define JNIEXPORT __attribute__((visibility("default")))
#define JNIIMPORT __attribute__((visibility("default")))
#define JNICALL

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    void* reserved0;
    jint (JNICALL* EnsureLocalCapacity)(JNIEnv* env, jint capacity);
    void (JNICALL* DeleteLocalRef)(JNIEnv* env, jobject obj);
    jint (JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    jclass (JNICALL* FindClass)(JNIEnv* env, const char* name);
    jboolean (JNICALL* ExceptionCheck)(JNIEnv* env);
    jstring (JNICALL* NewStringUTF)(JNIEnv* env, const char* utf);
    jsize (JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
    jobject (JNICALL* GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
    void (JNICALL* SetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index, jobject val);
    void (JNICALL* GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
    void (JNICALL* SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
    void (JNICALL* GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
    void (JNICALL* GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
    void (JNICALL* SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
    void* (JNICALL* GetPrimitiveArrayCritical)(JNIEnv* env, jarray array, jboolean* isCopy);
    void (JNICALL* ReleasePrimitiveArrayCritical)(JNIEnv* env, jarray array, void* carray, jint mode);
    jobject (JNICALL* NewDirectByteBuffer)(JNIEnv* env, void* address, jlong capacity);
    void* (JNICALL* GetDirectBufferAddress)(JNIEnv* env, jobject buf);
    jlong (JNICALL* GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
};

#endif
