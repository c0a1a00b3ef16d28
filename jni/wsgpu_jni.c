/* libwsgpu_jni.so: the JNI glue between org.snf4j.websocket.gpu.Wsg (java/) and
 * the C ABI of libwsgpu.so (include/wsgpu.h).  Every array crosses as a direct
 * ByteBuffer (GetDirectBufferAddress, no copy); byte[] only for the <= 14 header
 * bytes available() looks at and for batcher feeds from heap buffers.
 *
 * Argument checks: no libwsgpu call is made with a range the Java objects do not
 * hold.  A direct buffer must exist and its capacity cover what the call reads or
 * writes, an array must hold off + len elements; otherwise the call returns
 * WSG_API_EINVAL (available(): -2) without touching any buffer, so no JNI exception
 * is ever left pending.  Critical sections (GetPrimitiveArrayCritical) enclose only
 * the libwsgpu call, no other JNI call.
 *
 * Build: jni/Makefile (needs a JDK for jni.h; this repository's image has none).
 * Without a JDK the glue is compiled against tests/jni/jni.h and run with the fake
 * JNIEnv of tests/jni/fake_jni.c (tests/test_jni_glue.py, tests/test_gpu_jni.py). */
#include <jni.h>
#include <stdint.h>
#include <string.h>

#include "../include/wsgpu.h"

#define CTX(x) ((wsg_ctx*)(intptr_t)(x))
#define BATCHER(x) ((wsg_batcher*)(intptr_t)(x))
#define ENC_BATCHER(x) ((wsg_enc_batcher*)(intptr_t)(x))

/* A direct buffer's address if its capacity covers `need` bytes, else NULL. */
static uint8_t* span(JNIEnv* env, jobject bb, uint64_t need) {
    if (!bb) return NULL;
    uint8_t* p = (uint8_t*)(*env)->GetDirectBufferAddress(env, bb);
    jlong cap = (*env)->GetDirectBufferCapacity(env, bb);
    if (!p || cap < 0 || (uint64_t)cap < need) return NULL;
    return p;
}

/* off + len inside a direct buffer: its address at off, else NULL */
static uint8_t* span_at(JNIEnv* env, jobject bb, jint off, jint len) {
    if (off < 0 || len < 0) return NULL;
    uint8_t* p = span(env, bb, (uint64_t)off + (uint64_t)len);
    return p ? p + off : NULL;
}

/* an array holding at least `n` elements */
static int holds(JNIEnv* env, jarray a, jlong n) {
    return a && n >= 0 && (jlong)(*env)->GetArrayLength(env, a) >= n;
}

/* [off, off + len) inside an array */
static int range_in(JNIEnv* env, jarray a, jint off, jint len) {
    return off >= 0 && len >= 0 && holds(env, a, (jlong)off + (jlong)len);
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
    (void)env;
    (void)c;
    return wsg_open(device, NULL, &ctx) == WSG_API_OK ? (jlong)(intptr_t)ctx : 0;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_reserve(JNIEnv* env, jclass c, jlong ctx, jlong frames,
                                                                jint sessions, jlong wire) {
    (void)env;
    (void)c;
    if (!ctx || frames < 0 || sessions < 0 || wire < 0) return WSG_API_EINVAL;
    return wsg_reserve(CTX(ctx), (uint64_t)frames, (uint32_t)sessions, (uint64_t)wire);
}

JNIEXPORT void JNICALL Java_org_snf4j_websocket_gpu_Wsg_close(JNIEnv* env, jclass c, jlong ctx) {
    (void)env;
    (void)c;
    if (ctx) wsg_close(CTX(ctx));
}

JNIEXPORT jstring JNICALL Java_org_snf4j_websocket_gpu_Wsg_lastError(JNIEnv* env, jclass c, jlong ctx) {
    (void)c;
    return (*env)->NewStringUTF(env, wsg_last_error(CTX(ctx)));
}

/* ---- FrameDecoder.available (FrameDecoder.java:357-401) ----
 * err[0..2] = {status, detail, detail2} when the result is -1; err[3] = the whole
 * frame's length once its header is complete (the decoder tracks the rest of a
 * partial frame with it, as FrameDecoder.availablePayload does, :348-355).
 * -2: the arguments do not describe bytes the caller holds (or err is too short). */
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
    uint8_t hdr[16] = {0}; /* only the header is ever read: <= 14 bytes (the reference reads no
                              more either, so len may exceed the array: FrameDecoderTest.java:336-366) */
    (void)c;
    jint n = len < 14 ? len : 14;
    if (!range_in(env, b, off, n) || !holds(env, err, 4)) return -2;
    (*env)->GetByteArrayRegion(env, b, off, n, (jbyte*)hdr);
    return available(env, hdr, len, err);
}

JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_frameAvailableDirect(JNIEnv* env, jclass c, jobject b,
                                                                              jint off, jint len, jlongArray err) {
    uint8_t hdr[16] = {0};
    (void)c;
    jint n = len < 14 ? len : 14;
    const uint8_t* p = span_at(env, b, off, n);
    if (!p || !holds(env, err, 4)) return -2; /* not a direct buffer, or its header bytes are not there */
    memcpy(hdr, p, (size_t)n);
    return available(env, hdr, len, err);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_checkHeader(JNIEnv* env, jclass c, jboolean client,
                                                                    jboolean ext, jlong max_payload, jboolean frag,
                                                                    jobject data, jint off, jint len,
                                                                    jlongArray detail) {
    (void)c;
    wsg_decoder_cfg cfg = decoder_cfg(client, ext, max_payload, 0);
    int64_t d = 0;
    const uint8_t* p = span_at(env, data, off, len);
    if (!p || !holds(env, detail, 1)) return WSG_API_EINVAL;
    int32_t s = wsg_check_header(&cfg, frag ? 1 : 0, p, (uint64_t)len, &d);
    jlong v = d;
    (*env)->SetLongArrayRegion(env, detail, 0, 1, &v);
    return s;
}

/* ---- cross-session batcher ---- */
JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherOpen(JNIEnv* env, jclass c, jlong ctx, jboolean client,
                                                                     jboolean ext, jlong max_payload,
                                                                     jboolean validate, jint sessions) {
    (void)env;
    (void)c;
    if (!ctx || sessions < 0) return 0;
    wsg_decoder_cfg cfg = decoder_cfg(client, ext, max_payload, validate);
    wsg_batcher* b = NULL;
    return wsg_batcher_open(CTX(ctx), &cfg, (uint32_t)sessions, &b) == WSG_API_OK ? (jlong)(intptr_t)b : 0;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherClose(JNIEnv* env, jclass c, jlong b) {
    (void)env;
    (void)c;
    return wsg_batcher_close(BATCHER(b));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFeed(JNIEnv* env, jclass c, jlong b, jint sid,
                                                                    jobject data, jint off, jint len) {
    /* a direct buffer only: a heap buffer has no address (batcherFeedArray takes those) */
    (void)c;
    const uint8_t* p = span_at(env, data, off, len);
    if (!b || !p || sid < 0) return WSG_API_EINVAL;
    return wsg_batcher_feed(BATCHER(b), (uint32_t)sid, p, (uint64_t)len);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFeedArray(JNIEnv* env, jclass c, jlong b, jint sid,
                                                                         jbyteArray data, jint off, jint len) {
    (void)c;
    if (!b || sid < 0 || !range_in(env, data, off, len)) return WSG_API_EINVAL;
    /* the batcher copies the bytes, so a critical section is enough */
    jbyte* p = (jbyte*)(*env)->GetPrimitiveArrayCritical(env, data, NULL);
    if (!p) return WSG_API_ENOMEM;
    int rc = wsg_batcher_feed(BATCHER(b), (uint32_t)sid, (const uint8_t*)p + off, (uint64_t)len);
    (*env)->ReleasePrimitiveArrayCritical(env, data, p, JNI_ABORT);
    return rc;
}

/* One selector-loop iteration's reads in one call (wsg_batcher_feed_many): read i is
 * session sids[i]'s bytes [offs[i], offs[i] + lens[i]) of direct[i] (a direct
 * ByteBuffer) or, when that is null, of heap[i] (a byte[]).  Every read is checked
 * before any is fed, so an invalid one feeds nothing.  The reads go to the batcher in
 * groups of FEED_GROUP, with at most that many local references live and the group's
 * heap arrays pinned (critical) only around the libwsgpu call. */
#define FEED_GROUP 128
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFeedMany(JNIEnv* env, jclass c, jlong b, jint n,
                                                                        jintArray sids, jobjectArray direct,
                                                                        jobjectArray heap, jintArray offs,
                                                                        jintArray lens) {
    (void)c;
    if (!b || n < 0 || !holds(env, sids, n) || !holds(env, direct, n) || !holds(env, heap, n) ||
        !holds(env, offs, n) || !holds(env, lens, n))
        return WSG_API_EINVAL;
    if ((*env)->EnsureLocalCapacity(env, FEED_GROUP + 8) != JNI_OK) return WSG_API_ENOMEM;
    jint so[FEED_GROUP], oo[FEED_GROUP], lo[FEED_GROUP];
    /* pass 1: every read inside its buffer */
    for (jint base = 0; base < n; base += FEED_GROUP) {
        const jint m = n - base < FEED_GROUP ? n - base : FEED_GROUP;
        (*env)->GetIntArrayRegion(env, sids, base, m, so);
        (*env)->GetIntArrayRegion(env, offs, base, m, oo);
        (*env)->GetIntArrayRegion(env, lens, base, m, lo);
        for (jint k = 0; k < m; ++k) {
            int ok = so[k] >= 0 && oo[k] >= 0 && lo[k] >= 0;
            jobject d = (*env)->GetObjectArrayElement(env, direct, base + k);
            if (d) {
                ok = ok && span_at(env, d, oo[k], lo[k]) != NULL;
                (*env)->DeleteLocalRef(env, d);
            } else {
                jobject h = (*env)->GetObjectArrayElement(env, heap, base + k);
                ok = ok && (h ? range_in(env, h, oo[k], lo[k]) : lo[k] == 0);
                if (h) (*env)->DeleteLocalRef(env, h);
            }
            if (!ok) return WSG_API_EINVAL;
        }
    }
    /* pass 2: feed, a group at a time */
    uint32_t gs[FEED_GROUP];
    const uint8_t* gp[FEED_GROUP];
    uint64_t gl[FEED_GROUP];
    jobject ref[FEED_GROUP];
    void* pin[FEED_GROUP];
    for (jint base = 0; base < n; base += FEED_GROUP) {
        const jint m = n - base < FEED_GROUP ? n - base : FEED_GROUP;
        (*env)->GetIntArrayRegion(env, sids, base, m, so);
        (*env)->GetIntArrayRegion(env, offs, base, m, oo);
        (*env)->GetIntArrayRegion(env, lens, base, m, lo);
        int rc = WSG_API_OK;
        for (jint k = 0; k < m; ++k) {  /* checked again: pass 1's values are not trusted across the passes */
            gs[k] = (uint32_t)so[k];
            gl[k] = (uint64_t)lo[k];
            gp[k] = NULL;
            pin[k] = NULL;
            ref[k] = NULL;
            if (rc != WSG_API_OK) continue;
            if (so[k] < 0 || oo[k] < 0 || lo[k] < 0) {
                rc = WSG_API_EINVAL;
                continue;
            }
            ref[k] = (*env)->GetObjectArrayElement(env, direct, base + k);
            if (ref[k]) {  /* a direct buffer: its address, never pinned as an array */
                gp[k] = span_at(env, ref[k], oo[k], lo[k]);
                if (!gp[k]) rc = WSG_API_EINVAL;
            } else {
                ref[k] = (*env)->GetObjectArrayElement(env, heap, base + k);  /* byte[] or null (empty read) */
                if (ref[k] ? !range_in(env, ref[k], oo[k], lo[k]) : lo[k] != 0) rc = WSG_API_EINVAL;
            }
        }
        for (jint k = 0; k < m && rc == WSG_API_OK; ++k)  /* the heap arrays pinned: only critical calls until released */
            if (ref[k] && !gp[k]) {
                pin[k] = (*env)->GetPrimitiveArrayCritical(env, ref[k], NULL);
                if (pin[k]) gp[k] = (const uint8_t*)pin[k] + oo[k];
                else rc = WSG_API_ENOMEM;
            }
        if (rc == WSG_API_OK) rc = wsg_batcher_feed_many(BATCHER(b), (uint32_t)m, gs, gp, gl);
        for (jint k = m; k-- > 0;)
            if (pin[k]) (*env)->ReleasePrimitiveArrayCritical(env, ref[k], pin[k], JNI_ABORT);
        for (jint k = 0; k < m; ++k)
            if (ref[k]) (*env)->DeleteLocalRef(env, ref[k]);
        if (rc != WSG_API_OK) return rc;
    }
    return WSG_API_OK;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherSessionReset(JNIEnv* env, jclass c, jlong b,
                                                                            jint sid) {
    (void)env;
    (void)c;
    if (sid < 0) return WSG_API_EINVAL;
    return wsg_batcher_session_reset(BATCHER(b), (uint32_t)sid);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherSetStages(JNIEnv* env, jclass c, jlong b,
                                                                         jboolean inflate, jboolean no_context,
                                                                         jboolean validate, jboolean aggregate,
                                                                         jlong max_aggregated) {
    (void)env;
    (void)c;
    wsg_stage_cfg st;
    memset(&st, 0, sizeof st);
    st.inflate = inflate ? 1 : 0;
    st.inflate_no_context = no_context ? 1 : 0;
    st.validate = validate ? 1 : 0;
    st.aggregate = aggregate ? 1 : 0;
    st.max_aggregated_len = (int64_t)max_aggregated;
    return wsg_batcher_set_stages(BATCHER(b), &st);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherReserve(JNIEnv* env, jclass c, jlong b,
                                                                       jlong max_wire, jlong max_frames) {
    (void)env;
    (void)c;
    if (max_wire < 0 || max_frames < 0) return WSG_API_EINVAL;
    return wsg_batcher_reserve(BATCHER(b), (uint64_t)max_wire, (uint64_t)max_frames);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherReserveStages(JNIEnv* env, jclass c, jlong b,
                                                                             jlong max_out, jlong max_frames) {
    (void)env;
    (void)c;
    if (max_out < 0 || max_frames < 0) return WSG_API_EINVAL;
    return wsg_batcher_reserve_stages(BATCHER(b), (uint64_t)max_out, (uint64_t)max_frames);
}

/* the flush view as direct buffers: session_first, desc, payload, result (+ detail2) */
static int batch_views(JNIEnv* env, const wsg_batch_view* pv, jobjectArray views, jlongArray counts) {
    wsg_batch_view v = *pv;
    /* payload offsets run to the last descriptor's end; the region is < 2 GiB by contract */
    uint64_t pay = 0;
    for (uint64_t k = 0; k < v.n_frames; ++k) {
        uint64_t e = v.desc[k].payload_off + v.desc[k].payload_len;
        if (e > pay) pay = e;
    }
    const void* base[5] = {v.session_first, v.desc, v.payload, v.result, v.detail2};
    const jlong size[5] = {(jlong)(v.n_sessions + 1) * (jlong)sizeof(uint32_t),
                           (jlong)v.n_frames * (jlong)sizeof(wsg_frame_desc), (jlong)pay,
                           (jlong)v.n_sessions * (jlong)sizeof(wsg_session_result),
                           (jlong)v.n_sessions * (jlong)sizeof(int64_t)};
    const jint nv = (*env)->GetArrayLength(env, views) > 4 ? 5 : 4;
    for (jint i = 0; i < nv; ++i) {
        jobject bb = (*env)->NewDirectByteBuffer(env, (void*)base[i], size[i]);
        if (!bb) return WSG_API_ENOMEM; /* (the JVM's exception is pending) */
        (*env)->SetObjectArrayElement(env, views, i, bb);
        (*env)->DeleteLocalRef(env, bb);
    }
    jlong n[2] = {(jlong)v.n_frames, (jlong)v.wire_bytes};
    (*env)->SetLongArrayRegion(env, counts, 0, 2, n);
    return WSG_API_OK;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFlush(JNIEnv* env, jclass c, jlong b,
                                                                     jobjectArray views, jlongArray counts) {
    (void)c;
    if (!holds(env, views, 4) || !holds(env, counts, 2)) return WSG_API_EINVAL;
    wsg_batch_view v;
    int rc = wsg_batcher_flush(BATCHER(b), &v);
    if (rc != WSG_API_OK) return rc;
    return batch_views(env, &v, views, counts);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherFlushAsync(JNIEnv* env, jclass c, jlong b) {
    (void)env;
    (void)c;
    return wsg_batcher_flush_async(BATCHER(b));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherWait(JNIEnv* env, jclass c, jlong b,
                                                                    jobjectArray views, jlongArray counts) {
    (void)c;
    if (!holds(env, views, 4) || !holds(env, counts, 2)) return WSG_API_EINVAL; /* checked before the flush is taken */
    wsg_batch_view v;
    int rc = wsg_batcher_wait(BATCHER(b), &v);
    if (rc != WSG_API_OK) return rc;
    return batch_views(env, &v, views, counts);
}

JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherTicket(JNIEnv* env, jclass c, jlong b) {
    (void)env;
    (void)c;
    return (jlong)wsg_batcher_ticket(BATCHER(b));
}

/* (called on the completion thread, not the loop's) */
JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherAwait(JNIEnv* env, jclass c, jlong b, jlong seen,
                                                                      jlong timeout_ms) {
    (void)env;
    (void)c;
    if (!b || seen < 0) return WSG_API_EINVAL;
    return (jlong)wsg_batcher_await(BATCHER(b), (uint64_t)seen, (int64_t)timeout_ms);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_batcherSessionState(JNIEnv* env, jclass c, jlong b, jint sid,
                                                                            jbyteArray st) {
    (void)c;
    if (sid < 0 || !holds(env, st, (jlong)sizeof(wsg_session_state))) return WSG_API_EINVAL;
    wsg_session_state s;
    int rc = wsg_batcher_session_state(BATCHER(b), (uint32_t)sid, &s);
    if (rc == WSG_API_OK) (*env)->SetByteArrayRegion(env, st, 0, sizeof s, (const jbyte*)&s);
    return rc;
}

/* ---- device per selector loop ---- */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_deviceForLoop(JNIEnv* env, jclass c, jlong loop) {
    (void)env;
    (void)c;
    return wsg_device_for_loop((uint64_t)loop);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_deviceAccount(JNIEnv* env, jclass c, jint device,
                                                                      jlong bytes) {
    (void)env;
    (void)c;
    if (bytes < 0) return WSG_API_EINVAL;
    return wsg_device_account(device, (uint64_t)bytes);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_deviceReleaseLoop(JNIEnv* env, jclass c, jlong loop) {
    (void)env;
    (void)c;
    return wsg_device_release_loop((uint64_t)loop);
}

/* ---- cross-session encode batcher ---- */
JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherOpen(JNIEnv* env, jclass c, jlong ctx,
                                                                        jboolean client, jint sessions) {
    (void)env;
    (void)c;
    if (!ctx || sessions < 0) return 0;
    wsg_enc_batcher* b = NULL;
    return wsg_enc_batcher_open(CTX(ctx), client ? 1 : 0, (uint32_t)sessions, &b) == WSG_API_OK ? (jlong)(intptr_t)b
                                                                                                  : 0;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherClose(JNIEnv* env, jclass c, jlong b) {
    (void)env;
    (void)c;
    return wsg_enc_batcher_close(ENC_BATCHER(b));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherAdd(JNIEnv* env, jclass c, jlong b, jint sid,
                                                                      jint opcode, jint flags, jint mask,
                                                                      jbyteArray payload) {
    (void)c;
    if (!b || sid < 0) return WSG_API_EINVAL;
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

static int enc_views(JNIEnv* env, jobjectArray views, const wsg_enc_view* pv) {
    const wsg_enc_view v = *pv;
    const void* base[3] = {v.session_first, v.wire_off, v.wire};
    const jlong size[3] = {(jlong)(v.n_sessions + 1) * (jlong)sizeof(uint32_t),
                           (jlong)(v.n_frames + 1) * (jlong)sizeof(uint64_t), (jlong)v.wire_bytes};
    for (jint i = 0; i < 3; ++i) {
        jobject bb = (*env)->NewDirectByteBuffer(env, (void*)base[i], size[i]);
        if (!bb) return WSG_API_ENOMEM;
        (*env)->SetObjectArrayElement(env, views, i, bb);
        (*env)->DeleteLocalRef(env, bb);
    }
    return WSG_API_OK;
}

/* views[0] = session_first, views[1] = wire_off, views[2] = wire (valid until the next add/flush) */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherFlush(JNIEnv* env, jclass c, jlong b,
                                                                        jobjectArray views) {
    (void)c;
    if (!holds(env, views, 3)) return WSG_API_EINVAL;
    wsg_enc_view v;
    int rc = wsg_enc_batcher_flush(ENC_BATCHER(b), &v);
    if (rc != WSG_API_OK) return rc;
    return enc_views(env, views, &v);
}

/* pipelined form: flushAsync queues the encode of everything added so far; wait
 * returns the oldest in-flight flush's views (valid until that slot flushes again) */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherFlushAsync(JNIEnv* env, jclass c, jlong b) {
    (void)env;
    (void)c;
    return wsg_enc_batcher_flush_async(ENC_BATCHER(b));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherWait(JNIEnv* env, jclass c, jlong b,
                                                                       jobjectArray views) {
    (void)c;
    if (views && !holds(env, views, 3)) return WSG_API_EINVAL;
    wsg_enc_view v;
    int rc = wsg_enc_batcher_wait(ENC_BATCHER(b), &v);
    if (rc != WSG_API_OK) return rc;
    return views ? enc_views(env, views, &v) : WSG_API_OK;
}

JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherTicket(JNIEnv* env, jclass c, jlong b) {
    (void)env;
    (void)c;
    return (jlong)wsg_enc_batcher_ticket(ENC_BATCHER(b));
}

/* (called on the completion thread, not the loop's) */
JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherAwait(JNIEnv* env, jclass c, jlong b, jlong seen,
                                                                         jlong timeout_ms) {
    (void)env;
    (void)c;
    if (!b || seen < 0) return WSG_API_EINVAL;
    return (jlong)wsg_enc_batcher_await(ENC_BATCHER(b), (uint64_t)seen, (int64_t)timeout_ms);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherSetDeflate(JNIEnv* env, jclass c, jlong b,
                                                                             jint level, jboolean no_context) {
    (void)env;
    (void)c;
    return wsg_enc_batcher_set_deflate(ENC_BATCHER(b), (int)level, no_context ? 1 : 0);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherReserve(JNIEnv* env, jclass c, jlong b,
                                                                          jlong max_frames, jlong max_payload) {
    (void)env;
    (void)c;
    if (max_frames < 0 || max_payload < 0) return WSG_API_EINVAL;
    return wsg_enc_batcher_reserve(ENC_BATCHER(b), (uint64_t)max_frames, (uint64_t)max_payload);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encBatcherSessionReset(JNIEnv* env, jclass c, jlong b,
                                                                               jint sid) {
    (void)env;
    (void)c;
    if (sid < 0) return WSG_API_EINVAL;
    return wsg_enc_batcher_session_reset(ENC_BATCHER(b), (uint32_t)sid);
}

/* ---- encode ---- */
JNIEXPORT jlong JNICALL Java_org_snf4j_websocket_gpu_Wsg_encodedLength(JNIEnv* env, jclass c, jint len,
                                                                       jboolean client) {
    (void)env;
    (void)c;
    if (len < 0) return WSG_API_EINVAL;
    return (jlong)wsg_encoded_length((uint32_t)len, client ? 1 : 0);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_encodeBatchHost(
        JNIEnv* env, jclass c, jlong ctx, jboolean client, jobject payload, jlong payload_len, jobject frames,
        jlong n_frames, jobject session_first, jint n_sessions, jobject closed, jobject wire_out, jlong wire_cap,
        jobject wire_off) {
    (void)c;
    if (!ctx || payload_len < 0 || n_frames < 0 || n_sessions < 0 || wire_cap < 0) return WSG_API_EINVAL;
    const uint64_t F = (uint64_t)n_frames, S = (uint64_t)n_sessions;
    const uint8_t* pay = span(env, payload, (uint64_t)payload_len);
    const wsg_encode_frame* fr = (const wsg_encode_frame*)span(env, frames, F * sizeof(wsg_encode_frame));
    const uint32_t* sf = (const uint32_t*)span(env, session_first, (S + 1) * sizeof(uint32_t));
    uint8_t* cl = span(env, closed, S);
    uint8_t* wire = span(env, wire_out, (uint64_t)wire_cap);
    uint64_t* woff = (uint64_t*)span(env, wire_off, (F + 1) * sizeof(uint64_t));
    if ((payload_len && !pay) || (F && !fr) || !sf || (S && !cl) || !wire || !woff) return WSG_API_EINVAL;
    return wsg_encode_batch_host(CTX(ctx), client ? 1 : 0, pay, (uint64_t)payload_len, fr, F, sf, (uint32_t)S, cl,
                                 wire, (uint64_t)wire_cap, woff);
}

/* ---- the validator stage alone ---- */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_validateBatchHost(
        JNIEnv* env, jclass c, jlong ctx, jobject desc, jlong n_frames, jobject session_first, jint n_sessions,
        jobject payload, jlong payload_len, jobject state, jobject result) {
    (void)c;
    if (!ctx || n_frames < 0 || n_sessions < 0 || payload_len < 0) return WSG_API_EINVAL;
    const uint64_t F = (uint64_t)n_frames, S = (uint64_t)n_sessions;
    const wsg_frame_desc* d = (const wsg_frame_desc*)span(env, desc, F * sizeof(wsg_frame_desc));
    const uint32_t* sf = (const uint32_t*)span(env, session_first, (S + 1) * sizeof(uint32_t));
    const uint8_t* pay = span(env, payload, (uint64_t)payload_len);
    wsg_session_state* st = (wsg_session_state*)span(env, state, S * sizeof(wsg_session_state));
    wsg_session_result* res = (wsg_session_result*)span(env, result, S * sizeof(wsg_session_result));
    if ((F && !d) || !sf || (payload_len && !pay) || (S && (!st || !res))) return WSG_API_EINVAL;
    return wsg_validate_batch_host(CTX(ctx), d, F, sf, (uint32_t)S, pay, (uint64_t)payload_len, st, res);
}

/* ---- opening handshake (HandshakeDecoder + Handshaker, server and client side) ---- */
static void hs_config(JNIEnv* env, jintArray a, wsg_hs_config* c) {
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
}

/* HttpUtils.available over b[off, off + len): the frame length or 0; -1 for a buffer
 * over 8 KiB (the Java HandshakeDecoder takes those); -2 for a range outside b */
JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_handshakeAvailable(JNIEnv* env, jclass c, jbyteArray b,
                                                                           jint off, jint len) {
    uint8_t buf[8192];
    (void)c;
    if (!range_in(env, b, off, len)) return -2;
    if (len > (jint)sizeof buf) return -1;
    (*env)->GetByteArrayRegion(env, b, off, len, (jbyte*)buf);
    return wsg_handshake_available(buf, (uint64_t)len);
}

/* request / response i is data[offs[i], offs[i+1]): offs holds n + 1 offsets, ascending,
 * inside data */
static const uint8_t* hs_input(JNIEnv* env, jobject data, jobject offs, jint n, const uint64_t** off_out) {
    const uint64_t* off = (const uint64_t*)span(env, offs, ((uint64_t)n + 1) * sizeof(uint64_t));
    if (!off) return NULL;
    for (jint i = 0; i < n; ++i)
        if (off[i + 1] < off[i]) return NULL;
    const uint8_t* p = span(env, data, off[n]);
    *off_out = off;
    return p;
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_handshakeAcceptBatchHost(
        JNIEnv* env, jclass c, jlong ctx, jintArray config, jobject req, jobject req_off, jint n, jobject resp,
        jobject result) {
    (void)c;
    if (!ctx || n < 0) return WSG_API_EINVAL;
    const uint64_t* off = NULL;
    const uint8_t* rq = hs_input(env, req, req_off, n, &off);
    uint8_t* rs = span(env, resp, (uint64_t)n * WSG_HS_RESP_STRIDE);
    wsg_hs_result* res = (wsg_hs_result*)span(env, result, (uint64_t)n * sizeof(wsg_hs_result));
    if (!rq || (n && (!rs || !res))) return WSG_API_EINVAL;
    wsg_hs_config cfg;
    hs_config(env, config, &cfg);
    return wsg_handshake_accept_batch_host(CTX(ctx), &cfg, rq, off, (uint32_t)n, rs, res);
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_handshakeValidateBatchHost(
        JNIEnv* env, jclass c, jlong ctx, jintArray config, jobject resp, jobject resp_off, jobject keys, jint n,
        jobject expected, jobject result) {
    (void)c;
    if (!ctx || n < 0) return WSG_API_EINVAL;
    const uint64_t* off = NULL;
    const uint8_t* rs = hs_input(env, resp, resp_off, n, &off);
    const uint8_t* k = span(env, keys, (uint64_t)n * 24);
    uint8_t* ex = span(env, expected, (uint64_t)n * WSG_HS_EXPECTED_STRIDE);
    wsg_hs_result* res = (wsg_hs_result*)span(env, result, (uint64_t)n * sizeof(wsg_hs_result));
    if (!rs || (n && (!k || !ex || !res))) return WSG_API_EINVAL;
    wsg_hs_config cfg;
    hs_config(env, config, &cfg);
    return wsg_handshake_validate_batch_host(CTX(ctx), &cfg, rs, off, k, (uint32_t)n, ex, res);
}

/* ---- pinned host pool (IByteBufferAllocator.allocate / release) ---- */
JNIEXPORT jobject JNICALL Java_org_snf4j_websocket_gpu_Wsg_allocPinned(JNIEnv* env, jclass c, jint capacity) {
    (void)c;
    if (capacity < 0) return NULL;
    void* p = wsg_host_alloc((uint64_t)capacity);
    if (!p) return NULL;
    uint64_t cap = wsg_host_capacity(p); /* the size class; a ByteBuffer's capacity is an int */
    return (*env)->NewDirectByteBuffer(env, p, (jlong)(cap > INT32_MAX ? INT32_MAX : cap));
}

JNIEXPORT jint JNICALL Java_org_snf4j_websocket_gpu_Wsg_releasePinned(JNIEnv* env, jclass c, jobject b) {
    (void)c;
    uint8_t* p = span(env, b, 0);
    return p ? wsg_host_release(p) : WSG_API_EINVAL;
}
