/* CPU ORACLE for permessage-deflate compression — TEST INFRASTRUCTURE ONLY.
 *
 * Drives the system zlib (the engine java.util.zip.Deflater wraps; zlib 1.2.11 in
 * this image) exactly the way snf4j's encoder chain drives Deflater:
 *
 *   PerMessageDeflateEncoder.encode   PerMessageDeflateEncoder.java:81-99 (compressing state)
 *     allowEncoding                   :55-62  (TEXT/BINARY without RSV1, or CONTINUATION
 *                                             while compressing)
 *     rsvBits                         :69-79  (RSV1 added to TEXT/BINARY)
 *   DeflateEncoder.encode             DeflateEncoder.java:62-104
 *     new ZlibEncoder(level, RAW) on first use, dropped after a final fragment when
 *     noContext (:65-76); empty payload -> one 00 byte (:88-93); tail removed from a
 *     final fragment (:84, removeTail = isFinalFragment)
 *   ZlibEncoder.encode                ZlibEncoder.java:223-287
 *     Deflater(level, nowrap=true) (:101-112): deflateInit2(level, Z_DEFLATED, -15, 8,
 *     Z_DEFAULT_STRATEGY); an empty payload does not call the deflater (:263-265);
 *     setInput(data), then deflate(buf, pos, remaining, SYNC_FLUSH) until needsInput(),
 *     the first buffer deflateBound(len) bytes (:158-165, :267), later ones
 *     deflateBound(0) (:279).  Each Java deflate() call is one zlib deflate(strm,
 *     Z_SYNC_FLUSH) with avail_in = the input left and avail_out = the buffer space.
 *
 * No product code loads this file: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg (through oracle/deflateref.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

typedef struct dref_session {
    z_stream zs;
    int has_deflater; /* DeflateEncoder.encoder != null */
    int compressing;  /* PerMessageDeflateEncoder.compressing */
    int level;
    int no_context;
} dref_session;

/* ZlibEncoder.deflateBound (ZlibEncoder.java:158-165) */
static uint64_t java_deflate_bound(uint64_t len) { return len + ((len + 7) >> 3) + ((len + 63) >> 6) + 5 + 10; }

dref_session* dref_open(int level, int no_context) {
    if (level < 0 || level > 9) return NULL;
    dref_session* s = (dref_session*)calloc(1, sizeof(dref_session));
    if (!s) return NULL;
    s->level = level;
    s->no_context = no_context;
    return s;
}

static void drop_deflater(dref_session* s) {
    if (s->has_deflater) {
        deflateEnd(&s->zs);
        s->has_deflater = 0;
    }
}

void dref_close(dref_session* s) {
    if (!s) return;
    drop_deflater(s);
    free(s);
}

/* ZlibEncoder.encode(data) for a non-empty payload: appends the deflated bytes to out,
 * returns their count, or -1 on a zlib error / out overflow. */
static int64_t zlib_encode(dref_session* s, const uint8_t* data, uint64_t len, uint8_t* out, uint64_t cap) {
    if (!s->has_deflater) {
        memset(&s->zs, 0, sizeof(s->zs));
        if (deflateInit2(&s->zs, s->level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
        s->has_deflater = 1;
    }
    uint64_t w = 0;
    uint64_t buf = java_deflate_bound(len);       /* first ByteBuffer */
    uint64_t room = buf;
    s->zs.next_in = (Bytef*)data;
    s->zs.avail_in = (uInt)len;
    while (s->zs.avail_in != 0) {                 /* while (!deflater.needsInput()) */
        for (;;) {
            if (w + room > cap) return -1;
            s->zs.next_out = out + w;
            s->zs.avail_out = (uInt)room;
            int r = deflate(&s->zs, Z_SYNC_FLUSH);
            if (r != Z_OK && r != Z_BUF_ERROR) return -1;
            uint64_t n = room - s->zs.avail_out;
            w += n;
            room -= n;
            if (room == 0) {                      /* buffer full: a new deflateBound(0) one */
                room = java_deflate_bound(0);
                continue;
            }
            room = java_deflate_bound(0);         /* the next buffer, if the loop goes on */
            break;
        }
    }
    return (int64_t)w;
}

/* One frame through PerMessageDeflateEncoder: returns the output payload length (written
 * at out) or -1; *out_rsv = the frame's RSV bits after encoding (bit 2 = RSV1). */
int64_t dref_encode_frame(dref_session* s, int opcode, int fin, int rsv, const uint8_t* payload, uint64_t len,
                          uint8_t* out, uint64_t cap, int* out_rsv) {
    int allow = ((opcode == 1 || opcode == 2) && !(rsv & 4)) || (opcode == 0 && s->compressing);
    int64_t n;
    if (allow) {
        uint64_t raw = 0;
        if (len) {
            int64_t r = zlib_encode(s, payload, len, out, cap);
            if (r < 0) return -1;
            raw = (uint64_t)r;
        } else if (!s->has_deflater) {
            /* new ZlibEncoder is created but the empty payload never reaches it */
        }
        if (fin && s->no_context) drop_deflater(s);
        if (raw == 0) {
            if (len != 0) return -1;              /* "Deflating of input data produced no data" */
            if (cap < 1) return -1;
            out[0] = 0;
            n = 1;
        } else {
            n = fin ? (int64_t)raw - 4 : (int64_t)raw;
        }
        *out_rsv = (opcode == 1 || opcode == 2) ? (rsv | 4) : rsv;
    } else {
        if (len > cap) return -1;
        memcpy(out, payload, len);
        n = (int64_t)len;
        *out_rsv = rsv;
    }
    if (opcode < 8) {
        if (fin) s->compressing = 0;
        else if (!(rsv & 4) && (opcode == 1 || opcode == 2)) s->compressing = 1;
    }
    return n;
}

/* A session's frames in order: frame i is payload[off[i], off[i] + len[i]) with opcode[i],
 * fin[i], rsv[i]; writes out[out_off[i], out_off[i + 1]) and out_rsv[i].  Returns 0 or -1. */
int dref_encode_frames(dref_session* s, uint32_t n, const uint8_t* opcode, const uint8_t* fin, const uint8_t* rsv,
                       const uint64_t* off, const uint32_t* len, const uint8_t* payload, uint8_t* out, uint64_t cap,
                       uint64_t* out_off, uint8_t* out_rsv) {
    uint64_t w = 0;
    out_off[0] = 0;
    for (uint32_t i = 0; i < n; i++) {
        int r8 = 0;
        int64_t k = dref_encode_frame(s, opcode[i], fin[i], rsv[i], payload + off[i], len[i], out + w, cap - w, &r8);
        if (k < 0) return -1;
        w += (uint64_t)k;
        out_off[i + 1] = w;
        out_rsv[i] = (uint8_t)r8;
    }
    return 0;
}

/* Plain zlib per call, for the CPU baseline: `n` calls of deflate(SYNC_FLUSH) on one raw
 * stream (context takeover), inputs back to back in `in` with lengths `lens`; returns the
 * total output bytes or -1. */
int64_t dref_stream_bytes(int level, uint32_t n, const uint32_t* lens, const uint8_t* in, uint8_t* scratch,
                          uint64_t scratch_cap) {
    dref_session* s = dref_open(level, 0);
    if (!s) return -1;
    int64_t tot = 0;
    uint64_t o = 0;
    for (uint32_t i = 0; i < n; i++) {
        int64_t k = lens[i] ? zlib_encode(s, in + o, lens[i], scratch, scratch_cap) : 0;
        if (k < 0) { tot = -1; break; }
        tot += k;
        o += lens[i];
    }
    dref_close(s);
    return tot;
}
