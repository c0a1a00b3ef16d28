/*
 * ws_oracle.c — CPU ORACLE (test infrastructure only; see ws_oracle.h).
 *
 * Each function restates one piece of snf4j-websocket's frame codec; the
 * reference line it follows is cited next to it.  This file is never linked
 * into libwsgpu.so.
 */
#include "ws_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Utf8.java:32-50 — the DFA tables, kept as data.                           */
/* ------------------------------------------------------------------------ */
static const uint8_t UTF8_TYPES[256] = {
    0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,
    0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,
    0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,
    0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,
    1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,9,9,9,9,9,9,9,9,9,9,9,9,9,9,9,9,
    7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,7,
    8,8,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,2,
    10,3,3,3,3,3,3,3,3,3,3,3,3,4,3,3, 11,6,6,6,5,8,8,8,8,8,8,8,8,8,8,8,
};
static const uint8_t UTF8_STATES[108] = {
     0,12,24,36,60,96,84,12,12,12,48,72, 12,12,12,12,12,12,12,12,12,12,12,12,
    12, 0,12,12,12,12,12, 0,12, 0,12,12, 12,24,12,12,12,12,12,24,12,24,12,12,
    12,12,12,12,12,12,12,24,12,12,12,12, 12,24,12,12,12,12,12,12,12,24,12,12,
    12,12,12,12,12,12,12,36,12,36,12,12, 12,36,12,12,12,12,12,36,12,36,12,12,
    12,36,12,12,12,12,12,12,12,12,12,12,
};
#define U8_ACCEPT 0
#define U8_REJECT 12

/* Utf8.validate (Utf8.java:73-92): stops at the first REJECT. */
int or_utf8_validate(or_utf8_ctx* ctx, const uint8_t* data, int64_t len) {
    int state = ctx->state, codep = ctx->codep;
    for (int64_t i = 0; i < len; ++i) {
        int b = data[i], type = UTF8_TYPES[b];
        codep = state != U8_ACCEPT ? ((b & 0x3f) | (codep << 6)) : ((0xff >> type) & b);
        state = UTF8_STATES[state + type];
        if (state == U8_REJECT) return 0;
    }
    ctx->state = state;
    ctx->codep = codep;
    return 1;
}

/* Utf8.isValid(byte[], off, len) (Utf8.java:60-66) */
int or_utf8_is_valid(const uint8_t* data, int64_t len) {
    or_utf8_ctx c = {0, 0};
    return or_utf8_validate(&c, data, len) && c.state == U8_ACCEPT;
}

void or_utf8_is_valid_batch(const uint8_t* data, const int64_t* offs, int64_t n, uint8_t* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = (uint8_t)or_utf8_is_valid(data + offs[i], offs[i + 1] - offs[i]);
}

int64_t or_utf8_reject_pos(int state, const uint8_t* data, int64_t len) {
    for (int64_t i = 0; i < len; ++i) {
        state = UTF8_STATES[state + UTF8_TYPES[data[i]]];
        if (state == U8_REJECT) return i;
    }
    return -1;
}

/* ------------------------------------------------------------------------ */
/* FrameDecoder + FrameUtf8Validator                                         */
/* ------------------------------------------------------------------------ */
struct or_decoder {
    /* constructor arguments, FrameDecoder.java:76-80 */
    int client_mode, allow_ext, validate_utf8;
    int64_t max_payload;
    /* FrameDecoder state, :49-63 */
    int fragmentation;
    int pending;          /* this.opcode != null */
    int p_opcode, p_fin, p_rsv, p_masked;
    uint8_t p_mask[4];
    uint8_t* payload;     /* this.payload */
    int64_t payload_len;  /* payload.length */
    int64_t payload_have; /* this.payloadLen */
    int64_t payload_cap;
    int closed;
    /* FrameUtf8Validator.context (:42) */
    int vopen;
    or_utf8_ctx vctx;
};

or_decoder* or_decoder_new(int client_mode, int allow_extensions, int64_t max_payload_len,
                           int validate_utf8) {
    or_decoder* d = (or_decoder*)calloc(1, sizeof(or_decoder));
    d->client_mode = client_mode != 0;
    d->allow_ext = allow_extensions != 0;
    d->max_payload = max_payload_len;
    d->validate_utf8 = validate_utf8 != 0;
    return d;
}

void or_decoder_free(or_decoder* d) {
    if (!d) return;
    free(d->payload);
    free(d);
}

int or_decoder_closed(const or_decoder* d) { return d->closed; }
int or_decoder_fragmentation(const or_decoder* d) { return d->fragmentation; }

static int is_known_opcode(int v) { return v == 0 || v == 1 || v == 2 || v == 8 || v == 9 || v == 10; }

/* len16 / len64 (FrameDecoder.java:334-346), big-endian */
static int64_t be16(const uint8_t* p) { return ((int64_t)p[0] << 8) | p[1]; }
static int64_t be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return (int64_t)v;
}

/* available(session, byte[], off, len), FrameDecoder.java:357-401 */
int64_t or_decoder_available(or_decoder* d, const uint8_t* buf, int64_t len, int* err,
                             int64_t* detail, int64_t* detail2) {
    if (d->closed) return len;
    if (d->pending) { /* availablePayload :348-355 */
        int64_t needed = d->payload_len - d->payload_have;
        return len >= needed ? needed : len;
    }
    /* `need` is a Java int and `plen` a Java long: the arithmetic below wraps
     * exactly as the JVM's does (:392-395 can overflow for huge u64 lengths). */
    int32_t need = 2;
    if (len < need) return 0;
    if (buf[1] & 0x80) {
        need += 4;
        if (len < need) return 0;
    }
    int64_t plen = buf[1] & 0x7f;
    if (plen < 126) {
        need += (int32_t)plen;
    } else if (plen == 126) {
        need += 2;
        if (len < need) return 0;
        need += (int32_t)be16(buf + 2);
    } else {
        need += 8;
        if (len < need) return 0;
        plen = be64(buf + 2);
        if (plen < 0) {
            d->closed = 1;
            *err = WSG_E_NEG_LEN; *detail = plen; *detail2 = 0;
            return -1;
        }
        if ((int64_t)((uint64_t)plen + (uint64_t)(int64_t)need) > (int64_t)INT32_MAX) {
            d->closed = 1;
            *err = WSG_E_EXT_LEN; *detail = plen; *detail2 = (int64_t)INT32_MAX - need;
            return -1;
        }
        need = (int32_t)(uint32_t)((uint64_t)(int64_t)need + (uint64_t)plen);
    }
    return len > need ? need : len;
}

static void ensure_payload(or_decoder* d, int64_t n) {
    if (d->payload_cap < n || !d->payload) {
        free(d->payload);
        d->payload_cap = n > 16 ? n : 16;
        d->payload = (uint8_t*)malloc((size_t)d->payload_cap);
    }
}

/* FrameUtf8Validator.decode, FrameUtf8Validator.java:59-98. Returns 0 ok, -1 error.
 * `vopen` is (context != null), `vctx` the carried context. */
static int validator_step2(int* vopen, or_utf8_ctx* vctx, int opcode, int fin, const uint8_t* p,
                           int64_t len) {
    int validate;
    if (opcode == WSG_OP_CONTINUATION) validate = *vopen;
    else validate = opcode == WSG_OP_TEXT;
    if (!validate) return 0;
    or_utf8_ctx ctx;
    if (*vopen) ctx = *vctx;
    else { ctx.state = 0; ctx.codep = 0; }
    /* the field is cleared on FIN before validating (:83-88); the local keeps the state.
     * A non-final frame stores the SAME context object, so a later frame continues
     * from wherever this one stopped (also after a REJECT). */
    int ok = or_utf8_validate(&ctx, p, len);
    if (fin) *vopen = 0;
    else { *vopen = 1; *vctx = ctx; }
    if (!ok) return -1;
    if (fin && ctx.state != U8_ACCEPT) return -1;
    return 0;
}

static int validator_step(or_decoder* d, int opcode, int fin, const uint8_t* p, int64_t len) {
    return validator_step2(&d->vopen, &d->vctx, opcode, fin, p, len);
}

int or_validator_decode(or_validator* v, int opcode, int fin, const uint8_t* p, int64_t len) {
    return validator_step2(&v->open, &v->ctx, opcode, fin, p, len);
}

/* createFrame, FrameDecoder.java:104-157 (+ the validator stage after it) */
static int emit_frame(or_decoder* d, int opcode, int fin, int rsv, or_frame* out, int* err,
                      int64_t* detail, int* close_code) {
    const uint8_t* p = d->payload;
    int64_t len = d->payload_len;
    if (opcode == WSG_OP_CLOSE && len > 0) {
        int64_t status = be16(p);
        if (status <= 999 || status > 4999) {
            d->closed = 1;
            *err = WSG_E_CLOSE_STATUS; *detail = status; *close_code = WSG_CLOSE_PROTOCOL_ERROR;
            return -1;
        }
        if (len > 2 && !or_utf8_is_valid(p + 2, len - 2)) {
            d->closed = 1;
            *err = WSG_E_CLOSE_REASON; *detail = 0; *close_code = WSG_CLOSE_NON_UTF8;
            return -1;
        }
    }
    /* fragmentation update (:147-154); control frames are always final */
    if (fin) {
        if (opcode < 8) d->fragmentation = 0;
    } else {
        d->fragmentation = 1;
    }
    if (d->validate_utf8 && validator_step(d, opcode, fin, p, len) != 0) {
        /* the session is closed by the pipeline exception (FrameUtf8Validator.java:54-57) */
        d->closed = 1;
        *err = WSG_E_TEXT_UTF8; *detail = 0; *close_code = WSG_CLOSE_NON_UTF8;
        return -1;
    }
    out->opcode = opcode; out->fin = fin; out->rsv = rsv;
    out->len = len; out->payload = p;
    return 1;
}

#define PROTO_ERR(code, det) do { d->closed = 1; *err = (code); *detail = (det); \
    *close_code = WSG_CLOSE_PROTOCOL_ERROR; return -1; } while (0)

/* decode(session, data, out), FrameDecoder.java:180-288 */
int or_decoder_decode(or_decoder* d, const uint8_t* data, int64_t len, or_frame* out,
                      int* err, int64_t* detail, int* close_code) {
    *err = 0; *detail = 0; *close_code = 0;
    if (d->closed) return 0;

    if (d->pending) { /* decodePayload :159-178 */
        int64_t off = d->payload_have;
        if (len > d->payload_len - off) return -2;
        memcpy(d->payload + off, data, (size_t)len);
        if (len == d->payload_len - off) {
            if (d->p_masked)
                for (int64_t i = 0; i < d->payload_len; ++i) d->payload[i] ^= d->p_mask[i & 3];
            d->pending = 0;
            return emit_frame(d, d->p_opcode, d->p_fin, d->p_rsv, out, err, detail, close_code);
        }
        d->payload_have = off + len;
        return 0;
    }

    int64_t pos = 0;
    if (len < 2) return -2;
    int b = data[pos++];
    int opcode = b & 0x0f;
    if (!is_known_opcode(opcode)) PROTO_ERR(WSG_E_OPCODE, opcode);
    int fin = (b & 0x80) != 0;
    int rsv = (b >> 4) & 7;
    if (rsv != 0 && !d->allow_ext) PROTO_ERR(WSG_E_RSV, rsv);
    b = data[pos++];
    int masked = (b & 0x80) != 0;
    int64_t plen = b & 0x7f;
    if (masked == d->client_mode) PROTO_ERR(WSG_E_MASKING, 0);
    if (opcode >= 8) {
        if (!fin) PROTO_ERR(WSG_E_FRAG_CONTROL, 0);
        if (plen > 125) PROTO_ERR(WSG_E_CONTROL_LEN, plen);
        if (opcode == WSG_OP_CLOSE && plen == 1) PROTO_ERR(WSG_E_CLOSE_LEN, plen);
    } else if (opcode == WSG_OP_CONTINUATION) {
        if (!d->fragmentation) PROTO_ERR(WSG_E_CONT_OUTSIDE, 0);
    } else if (d->fragmentation) {
        PROTO_ERR(WSG_E_NONCONT_INSIDE, 0);
    }
    if (plen == 126) {
        if (len < pos + 2) return -2;
        plen = be16(data + pos); pos += 2;
        if (plen < 126) PROTO_ERR(WSG_E_MIN_LEN, 0);
    } else if (plen == 127) {
        if (len < pos + 8) return -2;
        plen = be64(data + pos); pos += 8;
        if (plen < 0 || plen > (int64_t)INT32_MAX) PROTO_ERR(WSG_E_MAX_PAYLOAD, 0);
        if (plen <= 0xffff) PROTO_ERR(WSG_E_MIN_LEN, 0);
    }
    if (plen > d->max_payload) PROTO_ERR(WSG_E_TOO_LONG, d->max_payload);
    uint8_t mask[4] = {0, 0, 0, 0};
    if (masked) {
        if (len < pos + 4) return -2;
        memcpy(mask, data + pos, 4);
        pos += 4;
    }
    ensure_payload(d, plen);
    d->payload_len = plen;
    int64_t remaining = len - pos;
    if (remaining > plen) return -2;
    memcpy(d->payload, data + pos, (size_t)remaining);
    if (remaining == plen) {
        if (masked)
            for (int64_t i = 0; i < plen; ++i) d->payload[i] ^= mask[i & 3];
        return emit_frame(d, opcode, fin, rsv, out, err, detail, close_code);
    }
    d->pending = 1;
    d->p_opcode = opcode; d->p_fin = fin; d->p_rsv = rsv; d->p_masked = masked;
    memcpy(d->p_mask, mask, 4);
    d->payload_have = remaining;
    return 0;
}

int or_format_error(int err, int64_t detail, int64_t detail2, char* buf, int cap) {
    switch (err) {
    case WSG_E_OPCODE: return snprintf(buf, cap, "Unexpected opcode value (%lld)", (long long)detail);
    case WSG_E_RSV: return snprintf(buf, cap, "Unexpected non-zero RSV bits (%lld)", (long long)detail);
    case WSG_E_MASKING: return snprintf(buf, cap, "Unexpected payload masking");
    case WSG_E_FRAG_CONTROL: return snprintf(buf, cap, "Fragmented control frame");
    case WSG_E_CONTROL_LEN: return snprintf(buf, cap, "Invalid payload length (%lld) in control frame", (long long)detail);
    case WSG_E_CLOSE_LEN: return snprintf(buf, cap, "Invalid payload length (%lld) in close frame", (long long)detail);
    case WSG_E_CONT_OUTSIDE: return snprintf(buf, cap, "Continuation frame outside fragmented message");
    case WSG_E_NONCONT_INSIDE: return snprintf(buf, cap, "Non-continuation frame while inside fragmented massage");
    case WSG_E_MIN_LEN: return snprintf(buf, cap, "Invalid minimal payload length");
    case WSG_E_MAX_PAYLOAD: return snprintf(buf, cap, "Invalid maximum payload length");
    case WSG_E_TOO_LONG: return snprintf(buf, cap, "Maximum frame length (%lld) has been exceeded", (long long)detail);
    case WSG_E_CLOSE_STATUS: return snprintf(buf, cap, "Invalid close frame status code (%lld)", (long long)detail);
    case WSG_E_CLOSE_REASON: return snprintf(buf, cap, "Invalid close frame reason value: bytes are not UTF-8");
    case WSG_E_TEXT_UTF8: return snprintf(buf, cap, "Invalid text frame payload: bytes are not UTF-8");
    case WSG_E_NEG_LEN: return snprintf(buf, cap, "Negative payload length (%lld)", (long long)detail);
    case WSG_E_EXT_LEN: return snprintf(buf, cap, "Extended payload length (%lld) > %lld", (long long)detail, (long long)detail2);
    case WSG_E_BATCH: return snprintf(buf, cap, "Malformed batch");
    case WSG_E_AGG_TOO_BIG: return snprintf(buf, cap, "Too big payload for aggregated frame");  /* FrameAggregator.java:93 */
    /* InvalidFrameException(cause): the message is cause.toString() (DeflateDecoder.java:73-76, ZlibDecoder.java:256) */
    case WSG_E_INFLATE: return snprintf(buf, cap, "org.snf4j.core.codec.zip.DecompressionException: decompression failure: invalid compressed data format");
    case WSG_E_INFLATE_NO_DATA: return snprintf(buf, cap, "Inflating of input data produced no data");  /* DeflateDecoder.java:129 */
    default: if (cap > 0) buf[0] = 0; return 0;
    }
}

/* ------------------------------------------------------------------------ */
/* Batch form: one decode() per complete frame, sessions independent.        */
/* ------------------------------------------------------------------------ */
struct or_batch {
    uint32_t n;
    or_decoder** dec;
};

or_batch* or_batch_new(int client_mode, int allow_extensions, int64_t max_payload_len,
                       int validate_utf8, uint32_t n_sessions) {
    or_batch* b = (or_batch*)calloc(1, sizeof(or_batch));
    b->n = n_sessions;
    b->dec = (or_decoder**)calloc(n_sessions ? n_sessions : 1, sizeof(or_decoder*));
    for (uint32_t i = 0; i < n_sessions; ++i)
        b->dec[i] = or_decoder_new(client_mode, allow_extensions, max_payload_len, validate_utf8);
    return b;
}

void or_batch_free(or_batch* b) {
    if (!b) return;
    for (uint32_t i = 0; i < b->n; ++i) or_decoder_free(b->dec[i]);
    free(b->dec);
    free(b);
}

int64_t or_batch_decode(or_batch* b, const uint8_t* wire, const uint64_t* frame_off,
                        uint64_t n_frames, const uint32_t* session_first, uint32_t n_sessions,
                        uint8_t* payload_out, wsg_frame_desc* desc_out,
                        wsg_session_result* result_out) {
    int64_t pos = 0;
    (void)n_frames;
    for (uint32_t s = 0; s < n_sessions && s < b->n; ++s) {
        or_decoder* d = b->dec[s];
        wsg_session_result* r = &result_out[s];
        memset(r, 0, sizeof(*r));
        for (uint64_t k = session_first[s]; k < session_first[s + 1]; ++k) {
            wsg_frame_desc* dk = &desc_out[k];
            memset(dk, 0, sizeof(*dk));
            if (d->closed) continue;
            or_frame f;
            int err = 0, cc = 0;
            int64_t det = 0;
            int rc = or_decoder_decode(d, wire + frame_off[k], (int64_t)(frame_off[k + 1] - frame_off[k]),
                                       &f, &err, &det, &cc);
            if (rc == 1) {
                dk->payload_off = (uint64_t)pos;
                dk->payload_len = (uint32_t)f.len;
                dk->opcode = (uint8_t)f.opcode;
                dk->flags = (uint8_t)((f.fin ? 0x80 : 0) | (f.rsv << 4));
                memcpy(payload_out + pos, f.payload, (size_t)f.len);
                pos += f.len;
                r->n_delivered++;
            } else if (rc == -1) {
                dk->status = (uint16_t)err;
                r->error = (uint16_t)err;
                r->close_code = (uint16_t)cc;
                r->detail = det;
            } else {
                /* a partial (rc 0) or overlong (rc -2) batch frame: the batch contract is broken */
                d->closed = 1;
                dk->status = WSG_E_BATCH;
                r->error = WSG_E_BATCH;
                r->close_code = WSG_CLOSE_PROTOCOL_ERROR;
            }
        }
    }
    return pos;
}

/* ------------------------------------------------------------------------ */
/* StreamSession.consumeBuffer (copying path, StreamSession.java:798-854).   */
/* ------------------------------------------------------------------------ */
int64_t or_stream_decode(int client_mode, int allow_extensions, int64_t max_payload_len,
                         int validate_utf8, const uint8_t* stream, int64_t len,
                         const int64_t* chunk, int n_chunk, uint8_t* payload_out,
                         wsg_frame_desc* desc_out, int64_t max_frames, int* err,
                         int64_t* detail, int64_t* detail2, int* close_code) {
    or_decoder* d = or_decoder_new(client_mode, allow_extensions, max_payload_len, validate_utf8);
    uint8_t* inbuf = (uint8_t*)malloc((size_t)(len > 0 ? len : 1));
    int64_t have = 0, fed = 0, nf = 0, pos = 0;
    int ci = 0;
    *err = 0; *detail = 0; *detail2 = 0; *close_code = 0;
    while (fed < len && !*err) {
        int64_t c = n_chunk > 0 ? chunk[ci++ % n_chunk] : len;
        if (c <= 0) c = 1;
        if (c > len - fed) c = len - fed;
        memcpy(inbuf + have, stream + fed, (size_t)c); /* SocketChannel.read into inBuffer */
        have += c;
        fed += c;
        int64_t start = 0;
        for (;;) {
            int64_t e2 = 0;
            int64_t a = or_decoder_available(d, inbuf + start, have - start, err, detail, &e2);
            if (a < 0) { *detail2 = e2; *close_code = WSG_CLOSE_PROTOCOL_ERROR; break; }
            if (a == 0) break;
            or_frame f;
            int rc = or_decoder_decode(d, inbuf + start, a, &f, err, detail, close_code);
            start += a;
            if (rc == 1 && nf < max_frames) {
                desc_out[nf].payload_off = (uint64_t)pos;
                desc_out[nf].payload_len = (uint32_t)f.len;
                desc_out[nf].opcode = (uint8_t)f.opcode;
                desc_out[nf].flags = (uint8_t)((f.fin ? 0x80 : 0) | (f.rsv << 4));
                desc_out[nf].status = 0;
                memcpy(payload_out + pos, f.payload, (size_t)f.len);
                pos += f.len;
                ++nf;
            } else if (rc < 0) {
                if (rc == -2) { *err = WSG_E_BATCH; }
                break;
            }
            if (start == have) break;
        }
        memmove(inbuf, inbuf + start, (size_t)(have - start)); /* inBuffer.compact() */
        have -= start;
    }
    free(inbuf);
    or_decoder_free(d);
    return nf;
}

/* ------------------------------------------------------------------------ */
/* FrameEncoder.encode / length, FrameEncoder.java:69-135.                   */
/* ------------------------------------------------------------------------ */
int64_t or_encoded_length(int64_t len, int client_mode) {
    int64_t n = len;
    if (len > 0xffff) n += 8;
    else if (len > 125) n += 2;
    if (client_mode) n += 4;
    return n + 2;
}

int64_t or_encode(or_encoder* e, int opcode, int fin, int rsv, const uint8_t* payload,
                  int64_t len, const uint8_t mask[4], uint8_t* out) {
    if (e->closed) return 0;
    if (opcode == WSG_OP_CLOSE) e->closed = 1;
    int64_t p = 0;
    out[p++] = (uint8_t)(((rsv << 4) & 0x70) | (fin ? 0x80 : 0) | opcode);
    uint8_t b1 = e->client_mode ? 0x80 : 0;
    if (len > 0xffff) {
        out[p++] = b1 | 127;
        for (int i = 7; i >= 0; --i) out[p++] = (uint8_t)((uint64_t)len >> (8 * i));
    } else if (len > 125) {
        out[p++] = b1 | 126;
        out[p++] = (uint8_t)(len >> 8);
        out[p++] = (uint8_t)len;
    } else {
        out[p++] = b1 | (uint8_t)len;
    }
    if (e->client_mode) {
        memcpy(out + p, mask, 4);
        p += 4;
        for (int64_t i = 0; i < len; ++i) out[p + i] = payload[i] ^ mask[i & 3];
    } else {
        memcpy(out + p, payload, (size_t)len);
    }
    return p + len;
}

/* ------------------------------------------------------------------------ */
/* Synthetic workload generator (must match the device generator bit for bit) */
/* ------------------------------------------------------------------------ */
/* ------------------------------------------------------------------------ */
/* FrameAggregator.decode, FrameAggregator.java:72-104.                      */
/* ------------------------------------------------------------------------ */
void or_aggregator_init(or_aggregator* a, int64_t max_aggregated_len) {
    memset(a, 0, sizeof(*a));
    a->max_len = max_aggregated_len;
}

void or_aggregator_free(or_aggregator* a) {
    free(a->data);
    a->data = NULL;
    a->cap = 0;
}

static void agg_append(or_aggregator* a, const uint8_t* p, int64_t len) {
    if (a->length + len > a->cap) {
        int64_t c = a->cap ? a->cap : 64;
        while (c < a->length + len) c *= 2;
        a->data = (uint8_t*)realloc(a->data, (size_t)c);
        a->cap = c;
    }
    if (len) memcpy(a->data + a->length, p, (size_t)len);
    a->length += len;
}

int or_aggregate(or_aggregator* a, int opcode, int fin, int rsv, const uint8_t* payload, int64_t len,
                 or_frame* out) {
    switch (opcode) {
    case WSG_OP_BINARY:
    case WSG_OP_TEXT:
        if (fin) break;  /* a final data frame passes through (:77-79, :84-86) */
        /* new AggregatedBinaryFrame/AggregatedTextFrame(true, rsv, payload) (:80, :87) */
        a->open = 1;
        a->opcode = opcode;
        a->rsv = rsv;
        a->length = 0;
        agg_append(a, payload, len);
        return 0;
    case WSG_OP_CONTINUATION:
        if (a->open) {
            if (a->length + len > a->max_len) return -1;  /* tooBig (:92-94) */
            agg_append(a, payload, len);                  /* addFragment (:95) */
            if (!fin) return 0;
            a->open = 0;                                  /* data = frame; frame = null (:99-100) */
            out->opcode = a->opcode;
            out->fin = 1;
            out->rsv = a->rsv;
            out->len = a->length;
            out->payload = a->data;
            return 1;
        }
        break;  /* falls through to out.add(data) (:103) */
    default:
        break;
    }
    out->opcode = opcode;
    out->fin = fin;
    out->rsv = rsv;
    out->len = len;
    out->payload = payload;
    return 1;
}

uint64_t or_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

/* Valid UTF-8 for one 16-byte chunk: code points never straddle a chunk. */
static void synth_text16(uint64_t h, uint8_t out[16]) {
    int i = 0;
    uint64_t r = h;
    int draws = 0;
    while (i < 16) {
        if (draws == 8) { r = or_splitmix64(r); draws = 0; }
        unsigned v = (unsigned)(r & 0xff);
        r >>= 8; ++draws;
        int room = 16 - i;
        unsigned kind = v % 10; /* 0..6 ASCII, 7 two-byte, 8 three-byte, 9 four-byte */
        if (kind <= 6 || room < 2) {
            out[i++] = (uint8_t)(0x20 + (v % 95));
        } else if (kind == 7 || room < 3) {
            unsigned cp = 0x80 + (v * 7u) % (0x800 - 0x80);
            out[i++] = (uint8_t)(0xC0 | (cp >> 6));
            out[i++] = (uint8_t)(0x80 | (cp & 0x3f));
        } else if (kind == 8 || room < 4) {
            unsigned cp = 0x800 + (v * 211u) % (0x10000 - 0x800);
            if (cp >= 0xD800 && cp <= 0xDFFF) cp += 0x800;
            out[i++] = (uint8_t)(0xE0 | (cp >> 12));
            out[i++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3f));
            out[i++] = (uint8_t)(0x80 | (cp & 0x3f));
        } else {
            unsigned cp = 0x10000 + (v * 4099u) % (0x110000 - 0x10000);
            out[i++] = (uint8_t)(0xF0 | (cp >> 18));
            out[i++] = (uint8_t)(0x80 | ((cp >> 12) & 0x3f));
            out[i++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3f));
            out[i++] = (uint8_t)(0x80 | (cp & 0x3f));
        }
    }
}

void or_synth_uniform(uint64_t seed, uint64_t n_frames, uint32_t payload_len,
                      uint32_t frames_per_session, int opcode, int masked, int text,
                      uint8_t* wire, uint64_t* frame_off, uint32_t* session_first) {
    uint64_t flen = (uint64_t)or_encoded_length(payload_len, masked);
    uint64_t n_sessions = (n_frames + frames_per_session - 1) / frames_per_session;
    for (uint64_t s = 0; s <= n_sessions; ++s) {
        uint64_t f = s * frames_per_session;
        session_first[s] = (uint32_t)(f < n_frames ? f : n_frames);
    }
    for (uint64_t k = 0; k <= n_frames; ++k) frame_off[k] = k * flen;
    for (uint64_t k = 0; k < n_frames; ++k) {
        uint8_t* w = wire + k * flen;
        uint64_t sess = k / frames_per_session;
        uint64_t sseed = seed ^ sess;
        uint64_t fh = or_splitmix64(sseed ^ (k * 0x9E3779B97F4A7C15ull));
        uint8_t mask[4] = {(uint8_t)fh, (uint8_t)(fh >> 8), (uint8_t)(fh >> 16), (uint8_t)(fh >> 24)};
        int p = 0;
        w[p++] = (uint8_t)(0x80 | (opcode & 0x0f));
        uint8_t b1 = masked ? 0x80 : 0;
        if (payload_len > 0xffff) {
            w[p++] = b1 | 127;
            for (int i = 7; i >= 0; --i) w[p++] = (uint8_t)((uint64_t)payload_len >> (8 * i));
        } else if (payload_len > 125) {
            w[p++] = b1 | 126;
            w[p++] = (uint8_t)(payload_len >> 8);
            w[p++] = (uint8_t)payload_len;
        } else {
            w[p++] = b1 | (uint8_t)payload_len;
        }
        if (masked) { memcpy(w + p, mask, 4); p += 4; }
        uint8_t* pl = w + p;
        for (uint32_t c = 0; c * 16 < payload_len; ++c) {
            uint64_t h = or_splitmix64(fh + c);
            uint8_t tmp[16];
            if (text) {
                synth_text16(h, tmp);
            } else {
                uint64_t h2 = or_splitmix64(h);
                memcpy(tmp, &h, 8);
                memcpy(tmp + 8, &h2, 8);
            }
            uint32_t n = payload_len - c * 16 < 16 ? payload_len - c * 16 : 16;
            /* a text chunk cut at the payload end must stay valid: pad with ASCII */
            if (text && n < 16) {
                uint32_t cut = n;
                while (cut > 0 && (tmp[cut] & 0xC0) == 0x80) --cut; /* cut before a split code point */
                for (uint32_t i = cut; i < n; ++i) tmp[i] = 'a';
            }
            for (uint32_t i = 0; i < n; ++i) pl[c * 16 + i] = masked ? (uint8_t)(tmp[i] ^ mask[i & 3]) : tmp[i];
        }
    }
}
