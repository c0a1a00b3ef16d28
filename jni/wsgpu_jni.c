/* libwsgpu_jni.so: the JNI glue between org.snf4j.websocket.gpu.Wsg (java/) and
 * the C ABI of libwsgpu.so (include/wsgpu.h).  Every array crosses as a direct
 * ByteBuffer (GetDirectBufferAddress, no copy); byte[] only for the <= 14 header
 * bytes available() looks at and for batcher feeds from heap buffers.
 * Build: jni/Makefile (needs a JDK for jni.h; this repository's image has none). */
#include <jni.h>
#include <stdint.h>
#include <string.h>

#include "../include/wsgpu.h"

#define CTX(x) ((wsg_ctx*)(intptr_t)(x))
#define BATCHER(x) ((wsg_batcher*)(intptr_t)(x))

static uint8_t* addr(JNIEnv* env, jobject bb) {
    return bb ? (uint8_t*)(*env)->GetDirectBufferAddress(env, bb) : NULL;
}

static wsg_decoder_cfg decoder_cfg(jboolean client, jboolean ext, jlong max_payload, jboolean validate) {
    wsg_decoder_cfg c;
    memset(&c, 0, sizeof c);
    c.client_mode = client ? 1 : 0;
    c.allow_extensions = ext ? 1 : 0;
    c.max_payload_len = max_payload;
    c.validate_utf8 = validate ? 1 : 0;
    return c;
}

/* ---- context ---- */
JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_open(JNIEnv* env, jclass c, jint device) {
    wsg_ctx* ctx = NULL;
    return wsg_open(device, NULL, &ctx) == WSG_API_OK ? (jlong)(intptr_t)ctx : 0;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_reserve(JNIEnv* env, jclass c, jlong ctx, jlong frames,
                                                                jint sessions, jlong wire) {
    return wsg_reserve(CTX(ctx), (uint64_t)frames, (uint32_t)sessions, (uint64_t)wire);
}

JNIEXPORT void JNICALL Java_org_snf4j_websocket_gpu_Wsg_close(JNIEnv* env, jclass c, jlong ctx) {
    wsg_close(CTX(ctx));
}

JNIEXPORT jstring JNICALL Java_org_snf4j_websocket_gpu_Wsg_lastError(JNIEnv* env, jclass c, jlong ctx) {
    return (*env)->NewStringUTF(env, wsg_last_error(CTX(ctx)));
}

/* ---- FrameDecoder.available (FrameDecoder.java:357-401) ----
 * err[0..2] = {status, detail, detail2} when the result is -1; err[3] = the whole
 * frame's length once its header is complete (the decoder tracks the rest of a
 * partial frame with it, as FrameDecoder.availablePayload does, :348-355). */
static jlong available(JNIEnv* env, const uint8_t* hdr, jint len, jlongArray err) {
    int32_t e = 0;
    int64_t d1 = 0, d2 = 0;
    int64_t r = wsg_frame_available(hdr, (uint64_t)len, &e, &d1, &d2);
    jlong v[4] = {e, d1, d2, 0};
    if (r > 0) {
        int32_t e2 = 0;
        int64_t t1 = 0, t2 = 0;
        int64_t whole = wsg_frame_available(hdr, (uint64_t)INT32_MAX, &e2, &t1, &t2);
        v[3] = whole > 0 ? whole : r;
    }
    (*env)->SetLongArrayRegion(env, err, 0, 4, v);
    return (jlong)r;
}

JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_frameAvailable(JNIEnv* env, jclass c, jbyteArray b, jint off,
                                                                        jint len, jlongArray err) {
    uint8_t hdr[16] = {0}; /* only the header is ever read: <= 14 bytes */
    jint n = len < 14 ? len : 14;
    (*env)->GetByteArrayRegion(env, b, off, n, (jbyte*)hdr);
    return available(env, hdr, len, err);
}

JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_frameAvailableDirect(JNIEnv* env, jclass c, jobject b,
                                                                              jint off, jint len, jlongArray err) {
    uint8_t hdr[16] = {0};
    uint8_t* p = addr(env, b);
    jlong cap = b ? (*env)->GetDirectBufferCapacity(env, b) : -1;
    jint n = len < 14 ? len : 14;
    if (!p || cap < 0 || off < 0 || len < 0 || (jlong)off + (jlong)n > cap) return -2; /* not a direct buffer */
    memcpy(hdr, p + off, (size_t)n);
    return available(env, hdr, len, err);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_checkHeader(JNIEnv* env, jclass c, jboolean client,
                                                                    jboolean ext, jlong max_payload, jboolean frag,
                                                                    jobject data, jint off, jint len,
                                                                    jlongArray detail) {
    wsg_decoder_cfg cfg = decoder_cfg(client, ext, max_payload, 0);
    int64_t d = 0;
    uint8_t* p = addr(env, data);
    jlong cap = data ? (*env)->GetDirectBufferCapacity(env, data) : -1;
    if (!p || cap < 0 || off < 0 || len < 0 || (jlong)off + (jlong)len > cap) return WSG_API_EINVAL;
    int32_t s = wsg_check_header(&cfg, frag ? 1 : 0, p + off, (uint64_t)len, &d);
    jlong v = d;
    (*env)->SetLongArrayRegion(env, detail, 0, 1, &v);
    return s;
}

/* ---- cross-session batcher ---- */
JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherOpen(JNIEnv* env, jclass c, jlong ctx, jboolean client,
                                                                     jboolean ext, jlong max_payload,
                                                                     jboolean validate, jint sessions) {
    wsg_decoder_cfg cfg = decoder_cfg(client, ext, max_payload, validate);
    wsg_batcher* b = NULL;
    return wsg_batcher_open(CTX(ctx), &cfg, (uint32_t)sessions, &b) == WSG_API_OK ? (jlong)(intptr_t)b : 0;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherClose(JNIEnv* env, jclass c, jlong b) {
    return wsg_batcher_close(BATCHER(b));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFeed(JNIEnv* env, jclass c, jlong b, jint sid,
                                                                    jobject data, jint off, jint len) {
    /* a direct buffer only: a heap buffer has no address (the Java side copies those) */
    uint8_t* p = addr(env, data);
    jlong cap = data ? (*env)->GetDirectBufferCapacity(env, data) : -1;
    if (!p || cap < 0 || off < 0 || len < 0 || (jlong)off + (jlong)len > cap) return WSG_API_EINVAL;
    return wsg_batcher_feed(BATCHER(b), (uint32_t)sid, p + off, (uint64_t)len);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherSessionReset(JNIEnv* env, jclass c, jlong b,
                                                                            jint sid) {
    return wsg_batcher_session_reset(BATCHER(b), (uint32_t)sid);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherSetStages(JNIEnv* env, jclass c, jlong b,
                                                                         jboolean inflate, jboolean no_context,
                                                                         jboolean validate, jboolean aggregate,
                                                                         jlong max_aggregated) {
    wsg_stage_cfg st;
    memset(&st, 0, sizeof st);
    st.inflate = inflate ? 1 : 0;
    st.inflate_no_context = no_context ? 1 : 0;
    st.validate = validate ? 1 : 0;
    st.aggregate = aggregate ? 1 : 0;
    st.max_aggregated_len = (int64_t)max_aggregated;
    return wsg_batcher_set_stages(BATCHER(b), &st);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFeedArray(JNIEnv* env, jclass c, jlong b, jint sid,
                                                                         jbyteArray data, jint off, jint len) {
    /* the batcher copies the bytes, so a critical section is enough */
    jbyte* p = (jbyte*)(*env)->GetPrimitiveArrayCritical(env, data, NULL);
    if (!p) return WSG_API_ENOMEM;
    int rc = wsg_batcher_feed(BATCHER(b), (uint32_t)sid, (const uint8_t*)p + off, (uint64_t)len);
    (*env)->ReleasePrimitiveArrayCritical(env, data, p, JNI_ABORT);
    return rc;
}

static int batch_views(JNIEnv* env, const wsg_batch_view* pv, jobjectArray views, jlongArray counts);

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFlush(JNIEnv* env, jclass c, jlong b,
                                                                     jobjectArray views, jlongArray counts) {
    wsg_batch_view v;
    int rc = wsg_batcher_flush(BATCHER(b), &v);
    if (rc != WSG_API_OK) return rc;
    return batch_views(env, &v, views, counts);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFlushAsync(JNIEnv* env, jclass c, jlong b) {
    return wsg_batcher_flush_async(BATCHER(b));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherWait(JNIEnv* env, jclass c, jlong b,
                                                                    jobjectArray views, jlongArray counts) {
    wsg_batch_view v;
    int rc = wsg_batcher_wait(BATCHER(b), &v);
    if (rc != WSG_API_OK) return rc;
    return batch_views(env, &v, views, counts);
}

/* the flush view as four direct buffers: session_first, desc, payload, result */
static int batch_views(JNIEnv* env, const wsg_batch_view* pv, jobjectArray views, jlongArray counts) {
    wsg_batch_view v = *pv;
    /* payload offsets run to the last descriptor's end; the region is < 2 GiB by contract */
    uint64_t pay = 0;
    for (uint64_t k = 0; k < v.n_frames; ++k) {
        uint64_t e = v.desc[k].payload_off + v.desc[k].payload_len;
        if (e > pay) pay = e;
    }
    (*env)->SetObjectArrayElement(env, views, 0,
                                  (*env)->NewDirectByteBuffer(env, (void*)v.session_first,
                                                              (jlong)(v.n_sessions + 1) * sizeof(uint32_t)));
    (*env)->SetObjectArrayElement(env, views, 1,
                                  (*env)->NewDirectByteBuffer(env, (void*)v.desc,
                                                              (jlong)v.n_frames * sizeof(wsg_frame_desc)));
    (*env)->SetObjectArrayElement(env, views, 2, (*env)->NewDirectByteBuffer(env, (void*)v.payload, (jlong)pay));
    (*env)->SetObjectArrayElement(env, views, 3,
                                  (*env)->NewDirectByteBuffer(env, (void*)v.result,
                                                              (jlong)v.n_sessions * sizeof(wsg_session_result)));
    if ((*env)->GetArrayLength(env, views) > 4)
        (*env)->SetObjectArrayElement(env, views, 4,
                                      (*env)->NewDirectByteBuffer(env, (void*)v.detail2,
                                                                  (jlong)v.n_sessions * sizeof(int64_t)));
    jlong n[2] = {(jlong)v.n_frames, (jlong)v.wire_bytes};
    (*env)->SetLongArrayRegion(env, counts, 0, 2, n);
    return WSG_API_OK;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherSessionState(JNIEnv* env, jclass c, jlong b, jint sid,
                                                                            jbyteArray st) {
    wsg_session_state s;
    int rc = wsg_batcher_session_state(BATCHER(b), (uint32_t)sid, &s);
    if (rc == WSG_API_OK) (*env)->SetByteArrayRegion(env, st, 0, sizeof s, (const jbyte*)&s);
    return rc;
}

/* ---- device per selector loop ---- */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_deviceForLoop(JNIEnv* env, jclass c, jlong loop) {
    return wsg_device_for_loop((uint64_t)loop);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_deviceAccount(JNIEnv* env, jclass c, jint device,
                                                                      jlong bytes) {
    return wsg_device_account(device, (uint64_t)bytes);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_deviceReleaseLoop(JNIEnv* env, jclass c, jlong loop) {
    return wsg_device_release_loop((uint64_t)loop);
}

/* ---- cross-session encode batcher ---- */
#define ENC_BATCHER(x) ((wsg_enc_batcher*)(intptr_t)(x))

JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherOpen(JNIEnv* env, jclass c, jlong ctx,
                                                                        jboolean client, jint sessions) {
    wsg_enc_batcher* b = NULL;
    return wsg_enc_batcher_open(CTX(ctx), client ? 1 : 0, (uint32_t)sessions, &b) == WSG_API_OK ? (jlong)(intptr_t)b
                                                                                                  : 0;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherClose(JNIEnv* env, jclass c, jlong b) {
    return wsg_enc_batcher_close(ENC_BATCHER(b));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherAdd(JNIEnv* env, jclass c, jlong b, jint sid,
                                                                      jint opcode, jint flags, jint mask,
                                                                      jbyteArray payload) {
    uint8_t m[4] = {(uint8_t)(mask >> 24), (uint8_t)(mask >> 16), (uint8_t)(mask >> 8), (uint8_t)mask};
    jsize n = payload ? (*env)->GetArrayLength(env, payload) : 0;
    /* the batcher copies the payload into its pinned arena */
    jbyte* p = n ? (jbyte*)(*env)->GetPrimitiveArrayCritical(env, payload, NULL) : NULL;
    if (n && !p) return WSG_API_ENOMEM;
    int rc = wsg_enc_batcher_add(ENC_BATCHER(b), (uint32_t)sid, (uint8_t)opcode, (uint8_t)flags, m,
                                 (const uint8_t*)p, (uint32_t)n);
    if (p) (*env)->ReleasePrimitiveArrayCritical(env, payload, p, JNI_ABORT);
    return rc;
}

static void enc_views(JNIEnv* env, jobjectArray views, const wsg_enc_view* pv) {
    const wsg_enc_view v = *pv;
    (*env)->SetObjectArrayElement(env, views, 0,
                                  (*env)->NewDirectByteBuffer(env, (void*)v.session_first,
                                                              (jlong)(v.n_sessions + 1) * sizeof(uint32_t)));
    (*env)->SetObjectArrayElement(env, views, 1,
                                  (*env)->NewDirectByteBuffer(env, (void*)v.wire_off,
                                                              (jlong)(v.n_frames + 1) * sizeof(uint64_t)));
    (*env)->SetObjectArrayElement(env, views, 2,
                                  (*env)->NewDirectByteBuffer(env, (void*)v.wire, (jlong)v.wire_bytes));
}

/* views[0] = session_first, views[1] = wire_off, views[2] = wire (valid until the next add/flush) */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherFlush(JNIEnv* env, jclass c, jlong b,
                                                                        jobjectArray views) {
    wsg_enc_view v;
    int rc = wsg_enc_batcher_flush(ENC_BATCHER(b), &v);
    if (rc != WSG_API_OK) return rc;
    enc_views(env, views, &v);
    return WSG_API_OK;
}

/* pipelined form: flushAsync queues the encode of everything added so far; wait
 * returns the oldest in-flight flush's views (valid until that slot flushes again) */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherFlushAsync(JNIEnv* env, jclass c, jlong b) {
    return wsg_enc_batcher_flush_async(ENC_BATCHER(b));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherWait(JNIEnv* env, jclass c, jlong b,
                                                                       jobjectArray views) {
    wsg_enc_view v;
    int rc = wsg_enc_batcher_wait(ENC_BATCHER(b), &v);
    if (rc != WSG_API_OK) return rc;
    if (views) enc_views(env, views, &v);
    return WSG_API_OK;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherSessionReset(JNIEnv* env, jclass c, jlong b,
                                                                               jint sid) {
    return wsg_enc_batcher_session_reset(ENC_BATCHER(b), (uint32_t)sid);
}

/* ---- encode ---- */
JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_encodedLength(JNIEnv* env, jclass c, jint len,
                                                                       jboolean client) {
    return (jlong)wsg_encoded_length((uint32_t)len, client ? 1 : 0);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encodeBatchHost(
        JNIEnv* env, jclass c, jlong ctx, jboolean client, jobject payload, jlong payload_len, jobject frames,
        jlong n_frames, jobject session_first, jint n_sessions, jobject closed, jobject wire_out, jlong wire_cap,
        jobject wire_off) {
    return wsg_encode_batch_host(CTX(ctx), client ? 1 : 0, addr(env, payload), (uint64_t)payload_len,
                                 (const wsg_encode_frame*)addr(env, frames), (uint64_t)n_frames,
                                 (const uint32_t*)addr(env, session_first), (uint32_t)n_sessions, addr(env, closed),
                                 addr(env, wire_out), (uint64_t)wire_cap, (uint64_t*)addr(env, wire_off));
}

/* ---- the validator stage alone ---- */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_validateBatchHost(
        JNIEnv* env, jclass c, jlong ctx, jobject desc, jlong n_frames, jobject session_first, jint n_sessions,
        jobject payload, jlong payload_len, jobject state, jobject result) {
    return wsg_validate_batch_host(CTX(ctx), (const wsg_frame_desc*)addr(env, desc), (uint64_t)n_frames,
                                   (const uint32_t*)addr(env, session_first), (uint32_t)n_sessions,
                                   addr(env, payload), (uint64_t)payload_len, (wsg_session_state*)addr(env, state),
                                   (wsg_session_result*)addr(env, result));
}

/* ---- opening handshake (HandshakeDecoder + Handshaker, server and client side) ---- */
static int hs_config(JNIEnv* env, jintArray a, wsg_hs_config* c) {
    jint v[5] = {65536, 0, 0, 0, 0};
    if (a) {
        jsize n = (*env)->GetArrayLength(env, a);
        (*env)->GetIntArrayRegion(env, a, 0, n < 5 ? n : 5, v);
    }
    memset(c, 0, sizeof *c);
    c->max_length = (uint32_t)v[0];
    c->ignore_host = v[1] ? 1 : 0;
    c->subprotocols = v[2] ? 1 : 0;
    c->extensions = v[3] ? 1 : 0;
    c->host_policy = v[4] ? 1 : 0;
    return 0;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_handshakeAvailable(JNIEnv* env, jclass c, jbyteArray b,
                                                                           jint off, jint len) {
    uint8_t buf[8192];
    if (len < 0 || len > (jint)sizeof buf) return -1;  /* larger frames go to the Java HandshakeDecoder */
    (*env)->GetByteArrayRegion(env, b, off, len, (jbyte*)buf);
    return wsg_handshake_available(buf, (uint64_t)len);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_handshakeAcceptBatchHost(
        JNIEnv* env, jclass c, jlong ctx, jintArray config, jobject req, jobject req_off, jint n, jobject resp,
        jobject result) {
    wsg_hs_config cfg;
    hs_config(env, config, &cfg);
    return wsg_handshake_accept_batch_host(CTX(ctx), &cfg, addr(env, req), (const uint64_t*)addr(env, req_off),
                                           (uint32_t)n, addr(env, resp), (wsg_hs_result*)addr(env, result));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_handshakeValidateBatchHost(
        JNIEnv* env, jclass c, jlong ctx, jintArray config, jobject resp, jobject resp_off, jobject keys, jint n,
        jobject expected, jobject result) {
    wsg_hs_config cfg;
    hs_config(env, config, &cfg);
    return wsg_handshake_validate_batch_host(CTX(ctx), &cfg, addr(env, resp), (const uint64_t*)addr(env, resp_off),
                                             addr(env, keys), (uint32_t)n, addr(env, expected),
                                             (wsg_hs_result*)addr(env, result));
}

/* ---- pinned host pool (IByteBufferAllocator.allocate / release) ---- */
JNIEXPORT jobject JNICALL Java_org_snf4j_websocket_gpu_Wsg_allocPinned(JNIEnv* env, jclass c, jint capacity) {
    void* p = wsg_host_alloc((uint64_t)capacity);
    return p ? (*env)->NewDirectByteBuffer(env, p, (jlong)wsg_host_capacity(p)) : NULL;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_releasePinned(JNIEnv* env, jclass c, jobject b) {
    return wsg_host_release(addr(env, b));
}
