/* handshake_port.c — a compiled CPU port of snf4j's opening handshake for the bench's
 * cpu_baseline (kind "port"): the per-request work the Java side does for a connection
 * storm, in C on one or more host cores.
 *
 * TEST / BENCH INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and tests/ use it; the
 * product path is k_hs_accept / k_hs_validate (snf4j_amd/csrc/handshake.hip).
 *
 * It follows oracle/handshake_oracle.py (the checker, pinned by the reference's test
 * vectors) step for step, on the forms a browser sends (request and header lines of the
 * "Name: value" form; folded or repeated lines return HSP_UNSUPPORTED):
 *   HttpUtils.available (:77-110), splitRequestLine (:125-157), splitHeaderField
 *     (:159-196), values (:311-333)
 *   HandshakeFactory.parse / parseFields (:47-127), format (:129-158)
 *   Handshaker.acceptVersion / acceptBasicFields / acceptUri / acceptKey (:208-373),
 *     validateBasicFields / validateKeyChallenge / validate (:420-544)
 *   HandshakeUtils.generateAnswerKey / parseKey (:93-120), Base64Util (:253-350)
 * SHA-1 is FIPS 180-4's.  The Java side also builds a HashMap of every field and
 * Strings for each name and value; the port keeps byte ranges, so it is the faster of
 * the two per core. */
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

enum { HSP_NEED_MORE = 0, HSP_PARSE_ERROR = 2, HSP_ACCEPT = 3, HSP_FINISHED = 4, HSP_CLOSING = 5,
       HSP_UNSUPPORTED = -1 };

#define MAX_LINES 50
#define MAX_FIELDS 64

/* ------------------------------------------------------------------ SHA-1 */
static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void sha1_block(uint32_t h[5], const uint8_t* p) {
    uint32_t w[80];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 80; i++) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; i++) {
        uint32_t f, k;
        if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
        else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
        else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
        else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
        const uint32_t t = rol(a, 5) + f + e + k + w[i];
        e = d; d = c; c = rol(b, 30); b = a; a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

static void sha1(const uint8_t* m, size_t n, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    size_t i = 0;
    for (; i + 64 <= n; i += 64) sha1_block(h, m + i);
    uint8_t blk[128];
    const size_t r = n - i;
    memcpy(blk, m + i, r);
    blk[r] = 0x80;
    const size_t tot = r + 9 <= 64 ? 64 : 128;
    memset(blk + r + 1, 0, tot - r - 1);
    const uint64_t bits = (uint64_t)n * 8;
    for (int j = 0; j < 8; j++) blk[tot - 1 - j] = (uint8_t)(bits >> (8 * j));
    sha1_block(h, blk);
    if (tot == 128) sha1_block(h, blk + 64);
    for (int j = 0; j < 5; j++) {
        out[4 * j] = (uint8_t)(h[j] >> 24); out[4 * j + 1] = (uint8_t)(h[j] >> 16);
        out[4 * j + 2] = (uint8_t)(h[j] >> 8); out[4 * j + 3] = (uint8_t)h[j];
    }
}

/* ------------------------------------------------------------------ Base64 */
static const char B64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

static size_t b64_encode(const uint8_t* s, size_t n, char* d) {
    size_t o = 0, i = 0;
    for (; i + 3 <= n; i += 3) {
        const uint32_t v = (uint32_t)s[i] << 16 | (uint32_t)s[i + 1] << 8 | s[i + 2];
        d[o++] = B64[v >> 18]; d[o++] = B64[(v >> 12) & 63]; d[o++] = B64[(v >> 6) & 63]; d[o++] = B64[v & 63];
    }
    if (n - i == 1) {
        const uint32_t v = (uint32_t)s[i] << 16;
        d[o++] = B64[v >> 18]; d[o++] = B64[(v >> 12) & 63]; d[o++] = '='; d[o++] = '=';
    } else if (n - i == 2) {
        const uint32_t v = (uint32_t)s[i] << 16 | (uint32_t)s[i + 1] << 8;
        d[o++] = B64[v >> 18]; d[o++] = B64[(v >> 12) & 63]; d[o++] = B64[(v >> 6) & 63]; d[o++] = '=';
    }
    return o;
}

static int b64_val(uint8_t c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
}

/* Base64Util.decode (not MIME): decoded length, or -1 for an invalid form */
static int b64_decoded_len(const uint8_t* s, size_t n) {
    if (n == 0) return 0;
    if (n < 2) return -1;
    size_t end = n;
    if (s[end - 1] == '=') {
        end--;
        if (s[end - 1] == '=') end--;
    }
    if (end == 0) return 0;
    if ((end & 3) == 1) return -1;
    for (size_t i = 0; i < end; i++)
        if (b64_val(s[i]) < 0) return -1;
    return (int)(end / 4 * 3 + ((end & 3) ? (end & 3) - 1 : 0));
}

/* ------------------------------------------------------------------ HTTP framing */
typedef struct { uint32_t b, e; } Rng;

/* HttpUtils.available: the frame length (0: incomplete) and its lines */
static size_t available(const uint8_t* d, size_t n, Rng* lines, int* nl, int* capped) {
    const int max_count = MAX_LINES * 2 + 1 - 3;
    int count = 0, end = 0;
    uint32_t line0 = 0;
    uint8_t curr = 0;
    *nl = 0;
    *capped = 0;
    for (size_t i = 0; i < n; i++) {
        const uint8_t prev = curr;
        curr = d[i];
        if (curr == '\n') {
            if (prev == '\r') {
                if (end) return i + 1;
                if (count > max_count) {
                    *capped = 1;
                    return 0;
                }
                end = 1;
                lines[(*nl)++] = (Rng){line0, (uint32_t)(i - 1)};
                count += 2;
                line0 = (uint32_t)(i + 1);
            }
        } else if (curr != '\r') {
            end = 0;
        }
    }
    return 0;
}

/* HttpUtils.splitRequestLine with out = int[10]: the number of tokens */
static int split_line(const uint8_t* d, uint32_t b, uint32_t e, Rng* t) {
    const int max_count = 5 * 2 - 2;
    int nt = 0;
    uint32_t line0 = b;
    uint8_t curr = 0;
    for (uint32_t i = b; i < e; i++) {
        const uint8_t prev = curr;
        curr = d[i];
        if (curr == ' ') {
            if (prev != ' ') {
                t[nt++] = (Rng){line0, i};
                if (nt * 2 > max_count) return nt;
            }
        } else if (prev == ' ') {
            line0 = i;
        }
    }
    t[nt++] = curr == ' ' ? (Rng){e, e} : (Rng){line0, e};
    return nt;
}

typedef struct { Rng name, value; } Field;

/* HttpUtils.splitHeaderField, "Name: value" lines only (code 4); 0 for any other form */
static int split_field(const uint8_t* d, uint32_t b, uint32_t e, Field* f) {
    uint32_t i = b;
    if (i < e && (d[i] == ' ' || d[i] == '\t')) return 0;  /* a folded line */
    const uint32_t n0 = i;
    while (i < e && d[i] != ':') i++;
    if (i == e) return 0;
    f->name = (Rng){n0, i};
    i++;
    while (i < e && (d[i] == ' ' || d[i] == '\t')) i++;
    uint32_t ve = e;
    while (ve > i && (d[ve - 1] == ' ' || d[ve - 1] == '\t')) ve--;  /* rtrimAscii */
    f->value = (Rng){i, ve};
    return 1;
}

static int ieq(const uint8_t* d, Rng r, const char* s) {
    const size_t n = strlen(s);
    if (r.e - r.b != n) return 0;
    for (size_t i = 0; i < n; i++) {
        uint8_t c = d[r.b + i];
        if (c >= 'a' && c <= 'z') c -= 32;
        uint8_t x = (uint8_t)s[i];
        if (x >= 'a' && x <= 'z') x -= 32;
        if (c != x) return 0;
    }
    return 1;
}

static int eq(const uint8_t* d, Rng r, const char* s) {
    const size_t n = strlen(s);
    return r.e - r.b == n && memcmp(d + r.b, s, n) == 0;
}

/* the parsed frame: fields by name (HandshakeFrame keys are upper-cased; a repeated name is
 * outside the port's forms) */
typedef struct { Field f[MAX_FIELDS]; int n; } Frame;

static int find(const uint8_t* d, const Frame* fr, const char* name, Rng* v) {
    for (int i = 0; i < fr->n; i++)
        if (ieq(d, fr->f[i].name, name)) {
            *v = fr->f[i].value;
            return 1;
        }
    return 0;
}

static int parse_fields(const uint8_t* d, const Rng* lines, int nl, Frame* fr) {
    fr->n = 0;
    for (int i = 1; i < nl; i++) {
        Field f;
        if (!split_field(d, lines[i].b, lines[i].e, &f) || fr->n == MAX_FIELDS) return HSP_UNSUPPORTED;
        for (int j = 0; j < fr->n; j++)
            if (fr->f[j].name.e - fr->f[j].name.b == f.name.e - f.name.b) {
                Rng r = fr->f[j].name;
                int same = 1;
                for (uint32_t k = 0; k < r.e - r.b && same; k++) {
                    uint8_t a = d[r.b + k], c = d[f.name.b + k];
                    if (a >= 'a' && a <= 'z') a -= 32;
                    if (c >= 'a' && c <= 'z') c -= 32;
                    same = a == c;
                }
                if (same) return HSP_UNSUPPORTED;  /* a repeated field: ", "-joined in Java */
            }
        fr->f[fr->n++] = f;
    }
    return 0;
}

/* HttpUtils.values + a test on each trimmed token: any token equal (ignoring case) to s */
static int has_token(const uint8_t* d, Rng v, const char* s) {
    uint32_t i = v.b;
    while (i <= v.e) {
        uint32_t j = i;
        while (j < v.e && d[j] != ',') j++;
        uint32_t a = i, b = j;
        while (a < b && d[a] <= 0x20) a++;
        while (b > a && d[b - 1] <= 0x20) b--;
        if (b > a && ieq(d, (Rng){a, b}, s)) return 1;
        i = j + 1;
    }
    return 0;
}

/* acceptVersion: 1 if a token parses as 13; 0 none does; -1 a token is not an integer */
static int version_ok(const uint8_t* d, Rng v) {
    uint32_t i = v.b;
    while (i <= v.e) {
        uint32_t j = i;
        while (j < v.e && d[j] != ',') j++;
        uint32_t a = i, b = j;
        while (a < b && d[a] <= 0x20) a++;
        while (b > a && d[b - 1] <= 0x20) b--;
        if (b > a) {
            uint32_t k = a;
            int neg = 0;
            if (d[k] == '+' || d[k] == '-') {
                neg = d[k] == '-';
                k++;
                if (k == b) return -1;
            }
            int64_t x = 0;
            for (; k < b; k++) {
                if (d[k] < '0' || d[k] > '9') return -1;
                x = x * 10 + (d[k] - '0');
                if (x > 2147483648LL) return -1;
            }
            if (neg) x = -x;
            if (x > 2147483647LL) return -1;
            if (x == 13) return 1;
        }
        i = j + 1;
    }
    return 0;
}

static int uri_ok(const uint8_t* d, Rng r) {
    for (uint32_t i = r.b; i < r.e; i++) {
        const uint8_t c = d[i];
        if (c == '%') {
            if (i + 2 < r.e && strchr("0123456789abcdefABCDEF", d[i + 1]) && d[i + 1] &&
                strchr("0123456789abcdefABCDEF", d[i + 2]) && d[i + 2]) {
                i += 2;
                continue;
            }
            return 0;
        }
        if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
              (c && strchr("-._~!*'()/?=&+,;$", c))))
            return 0;
    }
    return 1;
}

static int host_ok(const uint8_t* d, Rng r) {
    for (uint32_t i = r.b; i < r.e; i++) {
        const uint8_t c = d[i];
        if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '.' || c == '-' ||
              c == ':'))
            return 0;
    }
    return 1;
}

static size_t put(uint8_t* o, size_t at, const char* s) {
    const size_t n = strlen(s);
    memcpy(o + at, s, n);
    return at + n;
}

/* generateAnswerKey: base64(SHA-1(key + GUID)), 28 characters */
static void answer_key(const uint8_t* key, size_t n, char out[28]) {
    uint8_t m[128], h[20];
    static const char GUID[] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
    if (n > 128 - 36) n = 128 - 36;
    memcpy(m, key, n);
    memcpy(m + n, GUID, 36);
    sha1(m, n + 36, h);
    b64_encode(h, 20, out);
}

static size_t status_response(uint8_t* o, int status) {
    switch (status) {
        case 400: return put(o, 0, "HTTP/1.1 400 Bad Request\r\n\r\n");
        case 403: return put(o, 0, "HTTP/1.1 403 Forbidden\r\n\r\n");
        case 413: return put(o, 0, "HTTP/1.1 413 Request Entity Too Large\r\n\r\n");
        default: return put(o, 0, "HTTP/1.1 426 Upgrade Required\r\nSec-WebSocket-Version: 13\r\n\r\n");
    }
}

/* HandshakeDecoder.decode + Handshaker.accept of one complete request: the kind, the HTTP
 * status (*status) and the response bytes (resp, >= 160 B; *resp_len). */
int hsp_accept(const uint8_t* d, size_t n, uint8_t* resp, size_t* resp_len, int* status) {
    Rng lines[MAX_LINES + 2];
    int nl, capped;
    *resp_len = 0;
    *status = 0;
    const size_t flen = available(d, n, lines, &nl, &capped);
    if (capped) return HSP_UNSUPPORTED;
    if (flen == 0 && nl == 0) return HSP_NEED_MORE;
    /* (HandshakeDecoder.available0: the complete lines of an unfinished request are judged
     * as a chunk, its length and request line) */
    if ((flen ? flen : (size_t)lines[nl - 1].e + 2) > 65536) {
        *status = 413;
        *resp_len = status_response(resp, 413);
        return HSP_PARSE_ERROR;
    }
    Rng t[8];
    const int nt = split_line(d, lines[0].b, lines[0].e, t);
    int st = 0;
    if (nt != 3) st = 400;
    else if (!eq(d, t[2], "HTTP/1.1")) st = 400;
    else if (!eq(d, t[0], "GET")) st = 403;
    if (st) {
        *status = st;
        *resp_len = status_response(resp, st);
        return HSP_PARSE_ERROR;
    }
    if (flen == 0) return HSP_NEED_MORE;
    Frame fr;
    if (parse_fields(d, lines, nl, &fr)) return HSP_UNSUPPORTED;
    Rng v, u, c, h;
    st = 0;
    if (!find(d, &fr, "Sec-WebSocket-Version", &v)) st = 400;
    else {
        const int ok = version_ok(d, v);
        if (ok < 0) st = 400;
        else if (!ok) st = 426;
    }
    if (!st) {
        if (!find(d, &fr, "Upgrade", &u) || !find(d, &fr, "Connection", &c)) st = 400;
        else if (!has_token(d, u, "websocket") || !has_token(d, c, "upgrade")) st = 400;
    }
    if (!st) {
        if (!uri_ok(d, t[1])) return HSP_UNSUPPORTED;  /* java.net.URI decides */
        if (!find(d, &fr, "Host", &h)) st = 400;
        else if (!host_ok(d, h)) return HSP_UNSUPPORTED;
    }
    Rng k;
    if (!st) {
        if (!find(d, &fr, "Sec-WebSocket-Key", &k)) st = 400;
        else if (b64_decoded_len(d + k.b, k.e - k.b) != 16) st = 400;
    }
    *status = st ? st : 101;
    if (st) {
        *resp_len = status_response(resp, st);
        return HSP_ACCEPT;
    }
    size_t o = put(resp, 0, "HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                            "Sec-WebSocket-Accept: ");
    answer_key(d + k.b, k.e - k.b, (char*)resp + o);
    o = put(resp, o + 28, "\r\n\r\n");
    *resp_len = o;
    return HSP_ACCEPT;
}

/* HandshakeDecoder(clientMode).decode + Handshaker.validate of one complete 101 response
 * against the key the session sent: HSP_FINISHED or HSP_CLOSING (or a parse error) */
int hsp_validate(const uint8_t* d, size_t n, const uint8_t* key, size_t key_len) {
    Rng lines[MAX_LINES + 2];
    int nl, capped;
    const size_t flen = available(d, n, lines, &nl, &capped);
    if (capped) return HSP_UNSUPPORTED;
    if (flen == 0) return HSP_NEED_MORE;
    if (flen > 65536) return HSP_PARSE_ERROR;
    Rng t[8];
    const int nt = split_line(d, lines[0].b, lines[0].e, t);
    if (nt < 3 || !eq(d, t[0], "HTTP/1.1") || t[1].e - t[1].b != 3) return HSP_PARSE_ERROR;
    int status = 0;
    for (uint32_t i = t[1].b; i < t[1].e; i++) {
        if (d[i] < '0' || d[i] > '9') return HSP_PARSE_ERROR;
        status = status * 10 + (d[i] - '0');
    }
    Frame fr;
    if (parse_fields(d, lines, nl, &fr)) return HSP_UNSUPPORTED;
    if (status != 101) return HSP_CLOSING;
    Rng u, c, a, x;
    if (!find(d, &fr, "Upgrade", &u) || !find(d, &fr, "Connection", &c)) return HSP_CLOSING;
    if (!has_token(d, u, "websocket") || !has_token(d, c, "upgrade")) return HSP_CLOSING;
    char exp[28];
    answer_key(key, key_len, exp);
    if (!find(d, &fr, "Sec-WebSocket-Accept", &a)) return HSP_CLOSING;
    if (a.e - a.b != 28 || memcmp(d + a.b, exp, 28) != 0) return HSP_CLOSING;
    if (find(d, &fr, "Sec-WebSocket-Protocol", &x)) return HSP_CLOSING;
    if (find(d, &fr, "Sec-WebSocket-Extensions", &x)) return HSP_CLOSING;
    return HSP_FINISHED;
}

/* ------------------------------------------------------------------ timing */
typedef struct {
    const uint8_t* buf;
    const uint64_t* off;
    const uint8_t* keys;  /* client: 24 B a response, else NULL */
    uint32_t n, first;
    double seconds;
    uint64_t done, bad;
} Job;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* run_job(void* p) {
    Job* j = (Job*)p;
    uint8_t resp[512];
    size_t rl;
    int st;
    const double t0 = now_s();
    uint64_t done = 0, bad = 0;
    uint32_t i = j->first;
    do {
        for (int r = 0; r < 64; r++) {
            const uint8_t* q = j->buf + j->off[i];
            const size_t len = j->off[i + 1] - j->off[i];
            const int k = j->keys ? hsp_validate(q, len, j->keys + 24 * (uint64_t)i, 24)
                                  : hsp_accept(q, len, resp, &rl, &st);
            bad += k != (j->keys ? HSP_FINISHED : HSP_ACCEPT);
            done++;
            if (++i == j->n) i = 0;
        }
    } while (now_s() - t0 < j->seconds);
    j->done = done;
    j->bad = bad;
    return NULL;
}

/* Handshakes per second on `threads` host threads over n requests (keys: client mode),
 * each thread for `seconds`; *done = handshakes, returns -1 if any was not accepted /
 * finished. */
double hsp_rate(const uint8_t* buf, const uint64_t* off, const uint8_t* keys, uint32_t n, int threads,
                double seconds, uint64_t* done) {
    Job jobs[256];
    pthread_t th[256];
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    const double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        jobs[t] = (Job){buf, off, keys, n, (uint32_t)((uint64_t)n * t / threads), seconds, 0, 0};
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    uint64_t tot = 0, bad = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        tot += jobs[t].done;
        bad += jobs[t].bad;
    }
    const double el = now_s() - t0;
    *done = tot;
    return bad ? -1.0 : tot / el;
}
