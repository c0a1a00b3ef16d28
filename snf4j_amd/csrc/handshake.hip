// handshake.hip — the WebSocket opening handshake on gfx950, one lane per session:
//   server side (k_hs_accept): HandshakeDecoder (HandshakeDecoder.java:141-235) +
//     Handshaker.accept (Handshaker.java:208-405) + the response format of
//     HandshakeFactory.format (HandshakeFactory.java:129-158), for a batch of requests;
//   client side (k_hs_validate): HandshakeDecoder in client mode (the response branch
//     of HandshakeFactory.parse, HandshakeFactory.java:108-123) + Handshaker.validate
//     (Handshaker.java:420-544), for a batch of responses and the keys the sessions sent.
//
// A request is a few hundred bytes of serial HTTP parsing, so the lane is the unit:
// 64 requests per wave, each lane walking its own bytes (they stay in the L1/L2
// lines the first pass brought in).  No LDS, no cross-lane traffic.  The lane
// decides every request whose form it can reproduce exactly and defers the rest to
// the Java Handshaker (wsgpu.h lists the deferred forms).
#include <type_traits>

#include "wsgpu_internal.h"

namespace ws {

namespace {

constexpr uint8_t CR = 13, LF = 10, SP = ' ', HT = '\t';
constexpr int MAX_LINES = 50;  // HandshakeDecoder.DEFAULT_MAX_LINES_IN_CHUNK (HandshakeDecoder.java:50)

struct Span {
  int32_t b, e;  // [b, e) in the request; b < 0: absent
};

// Every function taking a Req is force-inlined: a Req passed by reference to an
// outlined call lives in scratch, and then every byte access went through memory.
// A lane's view of its request: bytes come from 16-B aligned blocks held in
// registers, so a forward scan costs one load per 16 bytes instead of one per byte
// (the batch buffer is 16-B aligned: a block never leaves the allocation's granule).
// waves a SIMD the kernels are built for (their register budget; A/B build switches)
#ifndef WSG_HS_WAVES
#define WSG_HS_WAVES 6  // k_hs_accept: 79 VGPRs, 6 waves a SIMD: 2.12 -> 1.79 ms with key_words (4, 5, 7, 8 slower: DESIGN 8b)
#endif
#ifndef WSG_HS_VWAVES
#define WSG_HS_VWAVES 4
#endif
struct Req {
  const uint4* base;  // the aligned block holding byte 0
  uint32_t lead;      // byte 0's offset in that block
  int32_t cq = -1;    // cached block index
  uint4 blk;
  __device__ uint8_t operator[](int32_t i) {
    const uint32_t a = lead + (uint32_t)i;
    const int32_t q = (int32_t)(a >> 4);
    if (q != cq) {
      cq = q;
      blk = base[q];
    }
    // (shifts of computed halves: a select among blk's fields became a dynamically
    // indexed load, which kept the whole Req in scratch)
    const uint32_t o = a & 15u;
    const uint64_t lo = (uint64_t)blk.x | ((uint64_t)blk.y << 32), hi = (uint64_t)blk.z | ((uint64_t)blk.w << 32);
    return (uint8_t)(((o & 8u) ? hi : lo) >> (8u * (o & 7u)));
  }
};

// Target fields (upper-cased names, HandshakeFrame.key: HandshakeFrame.java:128-130).
enum Field : int { F_HOST = 0, F_UPGRADE, F_CONNECTION, F_KEY, F_VERSION, F_PROTOCOL, F_EXTENSIONS, F_COUNT };

__device__ __constant__ char kFieldNames[F_COUNT][25] = {"HOST", "UPGRADE", "CONNECTION", "SEC-WEBSOCKET-KEY",
                                                         "SEC-WEBSOCKET-VERSION", "SEC-WEBSOCKET-PROTOCOL",
                                                         "SEC-WEBSOCKET-EXTENSIONS"};
__device__ __constant__ uint8_t kFieldLen[F_COUNT] = {4, 7, 10, 17, 21, 22, 24};

__device__ __constant__ char kGuid[37] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";  // HandshakeUtils.KEY_GUID
__device__ __constant__ char kB64[65] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

__device__ __forceinline__ uint8_t up(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

// Base64Util.DECODING (Base64Util.java:48-68): -1 for bytes outside the alphabet ('=' included).
__device__ __forceinline__ int b64v(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

// String.trim(): chars <= ' ' off both ends.
__device__ __forceinline__ Span trim(Req& d, Span s) {
  while (s.b < s.e && d[s.b] <= SP) ++s.b;
  while (s.e > s.b && d[s.e - 1] <= SP) --s.e;
  return s;
}

// Iterate HttpUtils.values(s) (HttpUtils.java:311-333): split at ',', trim, skip empty.
// f(token) returns true to stop; returns that token (b < 0 when none stopped).
template <typename F>
__device__ __forceinline__ Span each_value(Req& d, Span s, F&& f) {
  int32_t t0 = s.b;
  for (int32_t i = s.b; i <= s.e; ++i) {
    if (i == s.e || d[i] == ',') {
      const Span t = trim(d, Span{t0, i});
      if (t.e > t.b && f(t)) return t;
      t0 = i + 1;
    }
  }
  return Span{-1, -1};
}

// Integer.parseInt over ASCII: optional sign, decimal digits, int range.
__device__ __forceinline__ bool parse_int(Req& d, Span t, int64_t* v) {
  int32_t i = t.b;
  bool neg = false;
  if (d[i] == '-' || d[i] == '+') {
    neg = d[i] == '-';
    if (t.e - t.b == 1) return false;
    ++i;
  }
  int64_t x = 0;
  for (; i < t.e; ++i) {
    const uint8_t c = d[i];
    if (c < '0' || c > '9') return false;
    x = x * 10 + (c - '0');
    if (x > 2147483648ll) return false;
  }
  if (!neg && x > 2147483647ll) return false;
  *v = neg ? -x : x;
  return true;
}

// equalsIgnoreCase against an upper-case ASCII literal.
__device__ __forceinline__ bool eq_icase(Req& d, Span t, const char* lit, int n) {
  if (t.e - t.b != n) return false;
  for (int i = 0; i < n; ++i)
    if (up(d[t.b + i]) != (uint8_t)lit[i]) return false;
  return true;
}

__device__ __forceinline__ bool eq_exact(Req& d, Span t, const char* lit, int n) {
  if (t.e - t.b != n) return false;
  for (int i = 0; i < n; ++i)
    if (d[t.b + i] != (uint8_t)lit[i]) return false;
  return true;
}

// Handshaker.contains (Handshaker.java:407-418)
__device__ __forceinline__ bool contains(Req& d, Span s, const char* lit, int n) {
  return each_value(d, s, [&](Span t) { return eq_icase(d, t, lit, n); }).b >= 0;
}

// --- SHA-1 (MessageDigest "SHA1") over key bytes + KEY_GUID: at most 24 + 36 bytes.
__device__ __forceinline__ uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

__device__ __forceinline__ void sha1_block(uint32_t h[5], const uint32_t w0[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = w0[i];
  uint32_t a = h[0], b = h[1], c = h[2], dd = h[3], e = h[4];
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    if (t >= 16) w[t & 15] = rol(w[(t + 13) & 15] ^ w[(t + 8) & 15] ^ w[(t + 2) & 15] ^ w[t & 15], 1);
    uint32_t f, k;
    if (t < 20) { f = (b & c) | (~b & dd); k = 0x5A827999u; }
    else if (t < 40) { f = b ^ c ^ dd; k = 0x6ED9EBA1u; }
    else if (t < 60) { f = (b & c) | (b & dd) | (c & dd); k = 0x8F1BBCDCu; }
    else { f = b ^ c ^ dd; k = 0xCA62C1D6u; }
    const uint32_t tmp = rol(a, 5) + f + e + k + w[t & 15];
    e = dd;
    dd = c;
    c = rol(b, 30);
    b = a;
    a = tmp;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += dd; h[4] += e;
}

#ifndef WSG_HS_KEY_BLOCKS
#define WSG_HS_KEY_BLOCKS 1  // 0: the key bytes one by one through Req (A/B)
#endif
// The KL key bytes at request offset kb as big-endian words, from the (at most three)
// 16-B blocks that hold them: loaded once and funnel-shifted with selects (no
// dynamically indexed register array), instead of a byte-at-a-time walk whose block
// reloads the compiler kept as separate spilled copies.  Only blocks holding key
// bytes are loaded (they hold request bytes, so they stay in the allocation).
template <int KL>
__device__ __forceinline__ void key_words(const Req& d, int32_t kb, uint32_t* kw) {
  const uint32_t a0 = d.lead + (uint32_t)kb, sh = a0 & 15u;
  const uint4* const blk = d.base + (a0 >> 4);
  const uint4 b0 = blk[0], b1 = blk[1];  // (sh + KL > 16: KL >= 22)
  const uint4 b2 = sh + (uint32_t)KL > 32u ? blk[2] : make_uint4(0u, 0u, 0u, 0u);
  const uint32_t W[12] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b2.z, b2.w};
  const uint32_t qd = sh >> 2, sb = sh & 3u;
  uint32_t V[(KL + 3) / 4 + 1];
#pragma unroll
  for (int j = 0; j < (KL + 3) / 4 + 1; ++j)
    V[j] = qd == 0u ? W[j] : (qd == 1u ? W[j + 1] : (qd == 2u ? W[j + 2] : W[j + 3]));
#pragma unroll
  for (int j = 0; j < (KL + 3) / 4; ++j) {
    const uint32_t le = __builtin_amdgcn_alignbyte(V[j + 1], V[j], sb);  // key bytes 4j..4j+3
    uint32_t be = __builtin_bswap32(le);
    if (4 * j + 4 > KL) be &= 0xffffffffu << (8 * (4 * j + 4 - KL));  // bytes past the key: zero
    kw[j] = be;
  }
}

// Sec-WebSocket-Accept = Base64(SHA1(key + GUID)) (HandshakeUtils.generateAnswerKey,
// HandshakeUtils.java:98-111): 28 characters to the response.  Specialised on the key length,
// so that every message byte's source (key byte, GUID constant, padding) is known at
// compile time and the message words stay in registers.
template <int KL, class S, class O>
__device__ __forceinline__ void accept_key_n(S& d, int32_t kb, O& out) {
  constexpr int total = KL + 36;  // <= 60: two blocks after padding
  uint32_t kw[(KL + 3) / 4];      // the key bytes, big-endian words
#if WSG_HS_KEY_BLOCKS
  if constexpr (std::is_same<S, Req>::value) {
    key_words<KL>(d, kb, kw);
  } else
#endif
  {
#pragma unroll
    for (int j = 0; j < (KL + 3) / 4; ++j) {
      uint32_t v = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) v = (v << 8) | (j * 4 + q < KL ? (uint32_t)d[kb + j * 4 + q] : 0u);
      kw[j] = v;
    }
  }
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t v = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = blk * 64 + j * 4 + q;
        uint32_t byte;
        if (i < KL) byte = (kw[i >> 2] >> (24 - 8 * (i & 3))) & 0xffu;
        else if (i < total) byte = (uint8_t)"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"[i - KL];  // KEY_GUID
        else if (i == total) byte = 0x80u;
        else byte = 0u;
        v = (v << 8) | byte;
      }
      w[j] = v;
    }
    if (blk == 1) w[15] = (uint32_t)total * 8u;  // 60 bytes > 55: the length lands in block 2
    sha1_block(h, w);
  }
  // Base64Util.encode (padding '='): 20 bytes -> 6 full groups + 2 bytes
  uint32_t dg[7];  // digest bytes in 3-byte groups
#pragma unroll
  for (int g = 0; g < 7; ++g) {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int i = g * 3 + q;
      v = (v << 8) | (i < 20 ? (h[i >> 2] >> (24 - 8 * (i & 3))) & 0xffu : 0u);
    }
    dg[g] = v;
  }
#pragma unroll
  for (int g = 0; g < 7; ++g) {
    out.byte((uint8_t)kB64[(dg[g] >> 18) & 63]);
    out.byte((uint8_t)kB64[(dg[g] >> 12) & 63]);
    out.byte((uint8_t)kB64[(dg[g] >> 6) & 63]);
    out.byte(g < 6 ? (uint8_t)kB64[dg[g] & 63] : (uint8_t)'=');
  }
}
template <class O>
__device__ __forceinline__ void accept_key(Req& d, Span key, O& out) {
  switch (key.e - key.b) {  // 22..24 (a parseable key)
    case 22: accept_key_n<22>(d, key.b, out); break;
    case 23: accept_key_n<23>(d, key.b, out); break;
    default: accept_key_n<24>(d, key.b, out); break;
  }
}

// HandshakeUtils.parseKey (HandshakeUtils.java:113-120) over Base64Util.decode
// (Base64Util.java:253-350, not MIME): true when the key decodes to 16 bytes.
__device__ __forceinline__ bool key_ok(Req& d, Span k) {
  int32_t len = k.e - k.b, end = k.e;
  if (len < 2) return false;  // EMPTY (0 bytes) or null
  if (d[end - 1] == '=') {
    --end;
    --len;
    if (d[end - 1] == '=') {
      --end;
      --len;
    }
  }
  if (len == 0) return false;
  int calc = (len / 4) * 3;
  switch (len & 3) {
    case 1: return false;
    case 2: calc += 1; break;
    case 3: calc += 2; break;
    default: break;
  }
  for (int32_t i = k.b; i < end; ++i)
    if (b64v(d[i]) < 0) return false;
  return calc == 16;
}

// The request URI forms the lane accepts as java.net.URI would (a relative
// reference without scheme, authority-safe characters, well-formed escapes).
__device__ __forceinline__ bool uri_fast(Req& d, Span u) {
  for (int32_t i = u.b; i < u.e; ++i) {
    const uint8_t c = d[i];
    if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9')) continue;
    switch (c) {
      case '-': case '.': case '_': case '~': case '!': case '*': case '\'': case '(': case ')':
      case '/': case '?': case '=': case '&': case '+': case ',': case ';': case '$':
        continue;
      case '%': {
        auto hx = [](uint8_t x) { return (x >= '0' && x <= '9') || (x >= 'a' && x <= 'f') || (x >= 'A' && x <= 'F'); };
        if (i + 2 < u.e && hx(d[i + 1]) && hx(d[i + 2])) {
          i += 2;
          continue;
        }
        return false;
      }
      default:
        return false;
    }
  }
  return true;
}

__device__ __forceinline__ bool host_fast(Req& d, Span h) {
  for (int32_t i = h.b; i < h.e; ++i) {
    const uint8_t c = d[i];
    if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '.' || c == '-' ||
          c == ':'))
      return false;
  }
  return true;
}

__device__ __forceinline__ bool ascii(Req& d, Span s) {
  for (int32_t i = s.b; i < s.e; ++i)
    if (d[i] >= 0x80) return false;
  return true;
}

// Response bytes gathered into 16-B blocks: one aligned 16-B store per 16 bytes (resp
// is 16-B aligned and the stride a multiple of 16; dword stores to 64 strided lanes
// cost a partial line each).  done() stores the last partial block.
struct Out {
  uint8_t* p;
  int n = 0;
  uint64_t lo = 0, hi = 0;
  __device__ void byte(uint32_t c) {
    const int k = n & 15;
    if (k < 8) lo |= (uint64_t)c << (8 * k);
    else hi |= (uint64_t)c << (8 * (k - 8));
    if (k == 15) {
      reinterpret_cast<uint4*>(p)[n >> 4] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
      lo = hi = 0;
    }
    ++n;
  }
  __device__ void put(const char* s) {
    while (*s) byte((uint8_t)*s++);
  }
  __device__ void put(const uint8_t* s, int len) {
    for (int i = 0; i < len; ++i) byte(s[i]);
  }
  __device__ int done() {
    if (n & 15)
      reinterpret_cast<uint4*>(p)[n >> 4] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    return n;
  }
};

// HandshakeFactory.format of a HandshakeResponse(status) (HandshakeFactory.java:141-157)
__device__ int status_response(uint8_t* resp, int status) {
  Out o{resp};
  switch (status) {
    case 400: o.put("HTTP/1.1 400 Bad Request\r\n\r\n"); break;
    case 403: o.put("HTTP/1.1 403 Forbidden\r\n\r\n"); break;
    case 413: o.put("HTTP/1.1 413 Request Entity Too Large\r\n\r\n"); break;
    case 426: o.put("HTTP/1.1 426 Upgrade Required\r\nSec-WebSocket-Version: 13\r\n\r\n"); break;
    default: break;
  }
  return o.done();
}

}  // namespace

// HttpUtils.available (HttpUtils.java:77-110) with HandshakeDecoder's lines array of
// MAX_LINES*2+1 entries: frame length, or 0 (incomplete, or *capped: the chunk is
// full).  *lines_end: the end of the last complete line recorded, the chunk
// HandshakeDecoder.available0 (:221-233) hands to decode when no frame is complete.
template <typename D>
__host__ __device__ __forceinline__ int frame_len_t(D& d, int64_t len, int* capped, int64_t* lines_end) {
  const int max_count = MAX_LINES * 2 + 1 - 3;
  int line_count = 0;
  uint8_t prev, curr = 0;
  bool end = false;
  *capped = 0;
  *lines_end = 0;
  for (int64_t i = 0; i < len; ++i) {
    prev = curr;
    curr = d[i];
    if (curr == LF) {
      if (prev == CR) {
        if (end) return (int)(i + 1);
        if (line_count > max_count) {
          *capped = 1;
          return 0;
        }
        end = true;
        line_count += 2;
        *lines_end = i + 1;
      }
    } else if (curr != CR) {
      end = false;
    }
  }
  return 0;
}

__host__ __device__ int hs_frame_len(const uint8_t* d, int64_t len, int* capped, int64_t* lines_end) {
  return frame_len_t(d, len, capped, lines_end);
}

namespace {

__device__ __forceinline__ void accept_one(Req& d, int64_t n, const wsg_hs_config& cfg, uint8_t* resp, wsg_hs_result* res) {
  wsg_hs_result r = {0u, 0, WSG_HS_NEED_MORE, WSG_HSC_NONE, 0, 0, 0u};
  auto finish = [&](int kind, int status, int cause, Span detail) {
    r.kind = (uint8_t)kind;
    r.http_status = (uint16_t)status;
    r.cause = (uint8_t)cause;
    if (detail.b >= 0) {
      r.detail_off = (uint32_t)detail.b;
      r.detail_len = (uint16_t)(detail.e - detail.b);
    }
    if (kind == WSG_HS_PARSE_ERROR || (kind == WSG_HS_ACCEPT && status != 101))
      r.resp_len = (uint16_t)status_response(resp, status);
    *res = r;
  };
  const Span none{-1, -1};
  int capped = 0;
  int64_t lines_end = 0;
  const int flen = frame_len_t(d, n, &capped, &lines_end);
  if (capped) {
    finish(WSG_HS_DEFER, 0, WSG_HSC_D_LINES, none);
    return;
  }
  // No complete frame: HandshakeDecoder still decodes the complete lines as a chunk
  // (available0, :221-233), so the length cap and the request line are judged now.
  const bool partial = flen == 0;
  const int32_t limit = partial ? (int32_t)lines_end : flen;
  if (partial && limit == 0) {
    finish(WSG_HS_NEED_MORE, 0, WSG_HSC_NONE, none);
    return;
  }
  r.frame_len = (uint32_t)flen;
  // HandshakeDecoder.decode (:166-171): frameLength > maxLength -> 413
  if ((uint32_t)limit > cfg.max_length) {
    finish(WSG_HS_PARSE_ERROR, 413, WSG_HSC_TOO_LARGE, none);
    return;
  }
  // second pass over the lines of the frame: the request line, then header fields
  Span fld[F_COUNT];
  for (int f = 0; f < F_COUNT; ++f) fld[f] = none;
  Span uri = none;
  {
    // the lines HttpUtils.available recorded: CRLF-ended, up to the CRLF met with
    // `end` still set (the scan of hs_frame_len, replayed)
    int32_t line0 = 0;
    uint8_t prev, curr = 0;
    bool end = false;
    int line_no = 0;
    for (int32_t i = 0; i < limit; ++i) {
      prev = curr;
      curr = d[i];
      if (curr != LF) {
        if (curr != CR) end = false;
        continue;
      }
      if (prev != CR) continue;
      if (end) break;
      end = true;
      const int32_t lb = line0, le = i - 1;
      line0 = i + 1;
      if (line_no++ == 0) {
        // HandshakeFactory.parse (:96-107) with HttpUtils.splitRequestLine (:125-157), out[10]
        Span tok0 = none, tok1 = none, tok2 = none;  // (named: a dynamically indexed array goes to scratch)
        auto set_tok = [&](int c, Span t) {  // (selects, not stores through a chosen pointer)
          tok0 = c == 0 ? t : tok0;
          tok1 = c == 1 ? t : tok1;
          tok2 = c == 2 ? t : tok2;
        };
        int count = 0;
        int32_t t0 = lb;
        uint8_t p2, c2 = 0;
        bool over = false;
        for (int32_t j = lb; j < le && !over; ++j) {
          p2 = c2;
          c2 = d[j];
          if (c2 == SP) {
            if (p2 != SP) {
              set_tok(count, Span{t0, j});
              ++count;
              if (count * 2 > 8) over = true;
            }
          } else if (p2 == SP) {
            t0 = j;
          }
        }
        if (!over) {
          set_tok(count, (c2 == SP) ? Span{le, le} : Span{t0, le});
          ++count;
        }
        if (count != 3) {
          finish(WSG_HS_PARSE_ERROR, 400, WSG_HSC_BAD_REQUEST_LINE, none);
          return;
        }
        if (!eq_exact(d, tok2, "HTTP/1.1", 8)) {  // HttpUtils.equals (:198-215)
          finish(WSG_HS_PARSE_ERROR, 400, WSG_HSC_BAD_VERSION, none);
          return;
        }
        if (!eq_exact(d, tok0, "GET", 3)) {
          finish(WSG_HS_PARSE_ERROR, 403, WSG_HSC_FORBIDDEN, none);
          return;
        }
        uri = tok1;
        if (partial) {  // the fields are judged once the frame is complete
          finish(WSG_HS_NEED_MORE, 0, WSG_HSC_NONE, none);
          return;
        }
        continue;
      }
      // HttpUtils.splitHeaderField (:159-196): only the plain "name: value" form (4)
      // is taken here; folded lines (-4/-2) and bare names (2) go to the host
      if (lb < le && (d[lb] == SP || d[lb] == HT)) {
        finish(WSG_HS_DEFER, 0, WSG_HSC_D_LINE_FORM, none);
        return;
      }
      int32_t fs = -1;
      for (int32_t j = lb; j < le; ++j)
        if (d[j] == ':') {
          fs = j;
          break;
        }
      if (fs < 0) {
        finish(WSG_HS_DEFER, 0, WSG_HSC_D_LINE_FORM, none);
        return;
      }
      int32_t vb = fs + 1;
      while (vb < le && (d[vb] == SP || d[vb] == HT)) ++vb;
      int32_t ve = le;  // rtrimAscii (:230-239)
      while (ve > vb && (d[ve - 1] == SP || d[ve - 1] == HT)) --ve;
      const int nl = fs - lb;
      int fi = -1;
      for (int f = 0; f < F_COUNT && fi < 0; ++f) {
        if (nl != kFieldLen[f]) continue;
        bool m = true;
        for (int q = 0; q < nl && m; ++q) m = up(d[lb + q]) == (uint8_t)kFieldNames[f][q];
        if (m) fi = f;
      }
      if (fi >= 0) {
        // fld is touched with constant indices only (a switch), so it stays in registers
        bool seen = false;
#pragma unroll
        for (int f = 0; f < F_COUNT; ++f)
          if (f == fi) {
            seen = fld[f].b >= 0;
            if (!seen) fld[f] = Span{vb, ve};
          }
        if (seen) {  // a repeated field joins its values with ", " (HandshakeFrame.java:80-85)
          finish(WSG_HS_DEFER, 0, WSG_HSC_D_REPEATED, none);
          return;
        }
        if (!ascii(d, Span{vb, ve})) {
          finish(WSG_HS_DEFER, 0, WSG_HSC_D_NON_ASCII, none);
          return;
        }
      }
    }
  }
  if (!ascii(d, uri)) {
    finish(WSG_HS_DEFER, 0, WSG_HSC_D_NON_ASCII, none);
    return;
  }
  // Handshaker.accept (:375-405): version, basic fields, uri, key, subprotocol, extensions
  if (fld[F_VERSION].b < 0) {
    finish(WSG_HS_ACCEPT, 400, WSG_HSC_MISSING_VERSION, none);
    return;
  }
  {
    bool bad = false, found = false;
    const Span t = each_value(d, fld[F_VERSION], [&](Span v) {
      int64_t x = 0;
      if (!parse_int(d, v, &x)) {
        bad = true;
        return true;
      }
      if (x == 13) {
        found = true;
        return true;
      }
      return false;
    });
    if (bad) {
      finish(WSG_HS_ACCEPT, 400, WSG_HSC_INCORRECT_VERSION, t);
      return;
    }
    if (!found) {
      finish(WSG_HS_ACCEPT, 426, WSG_HSC_UNSUPPORTED_VERSION, fld[F_VERSION]);
      return;
    }
  }
  if (fld[F_UPGRADE].b < 0) {
    finish(WSG_HS_ACCEPT, 400, WSG_HSC_MISSING_UPGRADE, none);
    return;
  }
  if (fld[F_CONNECTION].b < 0) {
    finish(WSG_HS_ACCEPT, 400, WSG_HSC_MISSING_CONNECTION, none);
    return;
  }
  if (!contains(d, fld[F_UPGRADE], "WEBSOCKET", 9)) {
    finish(WSG_HS_ACCEPT, 400, WSG_HSC_INVALID_UPGRADE, fld[F_UPGRADE]);
    return;
  }
  if (!contains(d, fld[F_CONNECTION], "UPGRADE", 7)) {
    finish(WSG_HS_ACCEPT, 400, WSG_HSC_INVALID_CONNECTION, fld[F_CONNECTION]);
    return;
  }
  // acceptUri (:327-373)
  if (!uri_fast(d, uri)) {
    finish(WSG_HS_DEFER, 0, WSG_HSC_D_URI, none);
    return;
  }
  if (fld[F_HOST].b < 0) {
    if (!cfg.ignore_host) {
      finish(WSG_HS_ACCEPT, 400, WSG_HSC_MISSING_HOST, none);
      return;
    }
  } else if (!host_fast(d, fld[F_HOST])) {
    finish(WSG_HS_DEFER, 0, WSG_HSC_D_HOST, none);
    return;
  }
  if (cfg.host_policy) {  // acceptRequestUri / customizeHeaders are Java callbacks
    finish(WSG_HS_DEFER, 0, WSG_HSC_D_POLICY, none);
    return;
  }
  // acceptKey (:242-257)
  if (fld[F_KEY].b < 0) {
    finish(WSG_HS_ACCEPT, 400, WSG_HSC_MISSING_KEY, none);
    return;
  }
  if (!key_ok(d, fld[F_KEY])) {
    finish(WSG_HS_ACCEPT, 400, WSG_HSC_INVALID_KEY, fld[F_KEY]);
    return;
  }
  // acceptSubProtocol / acceptExtensions (:259-325): only with supported ones configured
  if (cfg.subprotocols && fld[F_PROTOCOL].b >= 0 && fld[F_PROTOCOL].e > fld[F_PROTOCOL].b) {
    finish(WSG_HS_DEFER, 0, WSG_HSC_D_SUBPROTOCOL, none);
    return;
  }
  if (cfg.extensions && fld[F_EXTENSIONS].b >= 0 && fld[F_EXTENSIONS].e > fld[F_EXTENSIONS].b) {
    finish(WSG_HS_DEFER, 0, WSG_HSC_D_EXTENSION, none);
    return;
  }
  // 101 with Upgrade, Connection, Sec-WebSocket-Accept (:386-391)
  Out o{resp};
  o.put("HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\nSec-WebSocket-Accept: ");
  accept_key(d, fld[F_KEY], o);  // 28 characters
  o.put("\r\n\r\n");
  const int rl = o.done();
  finish(WSG_HS_ACCEPT, 101, WSG_HSC_NONE, none);
  res->resp_len = (uint16_t)rl;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WSG_HS_WAVES))) void k_hs_accept(wsg_hs_config cfg, const uint8_t* req, const uint64_t* req_off,
                                                   uint32_t n, uint8_t* resp, wsg_hs_result* result) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = req_off[i], e = req_off[i + 1];
  Req d;
  d.base = reinterpret_cast<const uint4*>(req + (b & ~(uint64_t)15));
  d.lead = (uint32_t)(b & 15u);
  accept_one(d, (int64_t)(e - b), cfg, resp + (uint64_t)i * WSG_HS_RESP_STRIDE, result + i);
}

// ------------------------------------------------------------------ client side
// Target fields of a response (upper-cased names, HandshakeFrame.key).
enum CField : int { C_UPGRADE = 0, C_CONNECTION, C_ACCEPT, C_PROTOCOL, C_EXTENSIONS, C_COUNT };
__device__ __constant__ char kCliNames[C_COUNT][25] = {"UPGRADE", "CONNECTION", "SEC-WEBSOCKET-ACCEPT",
                                                       "SEC-WEBSOCKET-PROTOCOL", "SEC-WEBSOCKET-EXTENSIONS"};
__device__ __constant__ uint8_t kCliLen[C_COUNT] = {7, 10, 20, 22, 24};

// The 24 characters of the key a session sent, as six dwords in registers.
struct KeyWords {
  uint32_t w0, w1, w2, w3, w4, w5;
  __device__ uint8_t operator[](int32_t i) const {
    const int q = i >> 2;
    const uint32_t w = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : q == 3 ? w3 : q == 4 ? w4 : w5;
    return (uint8_t)(w >> (8 * (i & 3)));
  }
};

// The expected Sec-WebSocket-Accept, gathered in registers (named words and selects:
// an indexed member array went to scratch).
struct KeySink {
  uint32_t w0 = 0u, w1 = 0u, w2 = 0u, w3 = 0u, w4 = 0u, w5 = 0u, w6 = 0u;
  int n = 0;
  __device__ void byte(uint32_t c) {
    const uint32_t v = c << (8 * (n & 3));
    switch (n >> 2) {
      case 0: w0 |= v; break;
      case 1: w1 |= v; break;
      case 2: w2 |= v; break;
      case 3: w3 |= v; break;
      case 4: w4 |= v; break;
      case 5: w5 |= v; break;
      default: w6 |= v; break;
    }
    ++n;
  }
  __device__ uint8_t at(int i) const {
    const int q = i >> 2;
    const uint32_t w = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : q == 3 ? w3 : q == 4 ? w4 : q == 5 ? w5 : w6;
    return (uint8_t)(w >> (8 * (i & 3)));
  }
};

__device__ __forceinline__ void validate_one(Req& d, int64_t n, const wsg_hs_config& cfg, const KeyWords& key,
                                             uint8_t* expected, wsg_hs_result* res) {
  wsg_hs_result r = {0u, 0, WSG_HS_NEED_MORE, WSG_HSC_NONE, 0, 0, 0u};
  auto finish = [&](int kind, int cause, Span detail) {
    r.kind = (uint8_t)kind;
    r.cause = (uint8_t)cause;
    if (detail.b >= 0) {
      r.detail_off = (uint32_t)detail.b;
      r.detail_len = (uint16_t)(detail.e - detail.b);
    }
    *res = r;
  };
  const Span none{-1, -1};
  int capped = 0;
  int64_t lines_end = 0;
  const int flen = frame_len_t(d, n, &capped, &lines_end);
  if (capped) {
    finish(WSG_HS_DEFER, WSG_HSC_D_LINES, none);
    return;
  }
  // no complete frame: the complete lines are decoded as a chunk (available0,
  // HandshakeDecoder.java:212-224), so the length cap and the status line are judged now
  const bool partial = flen == 0;
  const int32_t limit = partial ? (int32_t)lines_end : flen;
  if (partial && limit == 0) {
    finish(WSG_HS_NEED_MORE, WSG_HSC_NONE, none);
    return;
  }
  r.frame_len = (uint32_t)flen;
  if ((uint32_t)limit > cfg.max_length) {  // :168-170; client mode throws (:192-193)
    finish(WSG_HS_PARSE_ERROR, WSG_HSC_TOO_LARGE, none);
    return;
  }
  Span fld[C_COUNT];
  for (int f = 0; f < C_COUNT; ++f) fld[f] = none;
  int status = 0;
  {
    int32_t line0 = 0;
    uint8_t prev, curr = 0;
    bool end = false;
    int line_no = 0;
    for (int32_t i = 0; i < limit; ++i) {
      prev = curr;
      curr = d[i];
      if (curr != LF) {
        if (curr != CR) end = false;
        continue;
      }
      if (prev != CR) continue;
      if (end) break;
      end = true;
      const int32_t lb = line0, le = i - 1;
      line0 = i + 1;
      if (line_no++ == 0) {
        // HandshakeFactory.parse, response branch (:108-123): HttpUtils.splitResponseLine
        // (= splitRequestLine, HttpUtils.java:138-176, out[10]) gives >= 3 tokens
        Span tok0 = none, tok1 = none;
        int count = 0;
        int32_t t0 = lb;
        uint8_t p2, c2 = 0;
        bool over = false;
        for (int32_t j = lb; j < le && !over; ++j) {
          p2 = c2;
          c2 = d[j];
          if (c2 == SP) {
            if (p2 != SP) {
              const Span t{t0, j};
              tok0 = count == 0 ? t : tok0;
              tok1 = count == 1 ? t : tok1;
              ++count;
              if (count * 2 > 8) over = true;
            }
          } else if (p2 == SP) {
            t0 = j;
          }
        }
        if (!over) {
          const Span t = (c2 == SP) ? Span{le, le} : Span{t0, le};
          tok0 = count == 0 ? t : tok0;
          tok1 = count == 1 ? t : tok1;
          ++count;
        }
        if (count < 3) {
          finish(WSG_HS_PARSE_ERROR, WSG_HSC_BAD_RESPONSE_LINE, none);
          return;
        }
        if (!eq_exact(d, tok0, "HTTP/1.1", 8)) {
          finish(WSG_HS_PARSE_ERROR, WSG_HSC_BAD_RESPONSE_VERSION, none);
          return;
        }
        // HttpUtils.digits (:271-284) and STATUS_CODE_LENGTH (3)
        bool digits = tok1.e - tok1.b == 3;
        for (int32_t j = tok1.b; j < tok1.e && digits; ++j) {
          const uint8_t c = d[j];
          if (c < '0' || c > '9') digits = false;
          else status = status * 10 + (c - '0');
        }
        if (!digits) {
          finish(WSG_HS_PARSE_ERROR, WSG_HSC_BAD_RESPONSE_STATUS, none);
          return;
        }
        r.http_status = (uint16_t)status;
        if (partial) {
          finish(WSG_HS_NEED_MORE, WSG_HSC_NONE, none);
          return;
        }
        continue;
      }
      // header fields: the plain "name: value" form only, as on the server side
      if (lb < le && (d[lb] == SP || d[lb] == HT)) {
        finish(WSG_HS_DEFER, WSG_HSC_D_LINE_FORM, none);
        return;
      }
      int32_t fs = -1;
      for (int32_t j = lb; j < le; ++j)
        if (d[j] == ':') {
          fs = j;
          break;
        }
      if (fs < 0) {
        finish(WSG_HS_DEFER, WSG_HSC_D_LINE_FORM, none);
        return;
      }
      int32_t vb = fs + 1;
      while (vb < le && (d[vb] == SP || d[vb] == HT)) ++vb;
      int32_t ve = le;
      while (ve > vb && (d[ve - 1] == SP || d[ve - 1] == HT)) --ve;
      const int nl = fs - lb;
      int fi = -1;
      for (int f = 0; f < C_COUNT && fi < 0; ++f) {
        if (nl != kCliLen[f]) continue;
        bool m = true;
        for (int q = 0; q < nl && m; ++q) m = up(d[lb + q]) == (uint8_t)kCliNames[f][q];
        if (m) fi = f;
      }
      if (fi >= 0) {
        bool seen = false;
#pragma unroll
        for (int f = 0; f < C_COUNT; ++f)
          if (f == fi) {
            seen = fld[f].b >= 0;
            if (!seen) fld[f] = Span{vb, ve};
          }
        if (seen) {
          finish(WSG_HS_DEFER, WSG_HSC_D_REPEATED, none);
          return;
        }
        if (!ascii(d, Span{vb, ve})) {
          finish(WSG_HS_DEFER, WSG_HSC_D_NON_ASCII, none);
          return;
        }
      }
    }
  }
  // Handshaker.validate (:535-544)
  if (status != 101) {
    finish(WSG_HS_CLOSING, WSG_HSC_INVALID_STATUS, none);
    return;
  }
  // validateBasicFields (:420-444)
  if (fld[C_UPGRADE].b < 0) {
    finish(WSG_HS_CLOSING, WSG_HSC_MISSING_UPGRADE, none);
    return;
  }
  if (fld[C_CONNECTION].b < 0) {
    finish(WSG_HS_CLOSING, WSG_HSC_MISSING_CONNECTION, none);
    return;
  }
  if (!contains(d, fld[C_UPGRADE], "WEBSOCKET", 9)) {
    finish(WSG_HS_CLOSING, WSG_HSC_INVALID_UPGRADE, fld[C_UPGRADE]);
    return;
  }
  if (!contains(d, fld[C_CONNECTION], "UPGRADE", 7)) {
    finish(WSG_HS_CLOSING, WSG_HSC_INVALID_CONNECTION, fld[C_CONNECTION]);
    return;
  }
  // validateKeyChallenge (:446-460): HandshakeUtils.generateAnswerKey(key)
  KeySink ex;
  accept_key_n<24>(key, 0, ex);
  reinterpret_cast<uint4*>(expected)[0] = make_uint4(ex.w0, ex.w1, ex.w2, ex.w3);
  reinterpret_cast<uint4*>(expected)[1] = make_uint4(ex.w4, ex.w5, ex.w6, 0u);
  r.resp_len = 28;
  const Span act = fld[C_ACCEPT];
  if (act.b < 0) {
    finish(WSG_HS_CLOSING, WSG_HSC_MISSING_ACCEPT, none);
    return;
  }
  bool same = act.e - act.b == 28;
#pragma unroll
  for (int i = 0; i < 28; ++i) same = same && d[act.b + (same ? i : 0)] == ex.at(i);
  if (!same) {
    finish(WSG_HS_CLOSING, WSG_HSC_INVALID_ACCEPT, act);
    return;
  }
  // validateSubProtocol (:462-485): a match against the configured list is Java's
  const Span pr = fld[C_PROTOCOL];
  if (cfg.subprotocols) {
    if (pr.b < 0) {
      finish(WSG_HS_CLOSING, WSG_HSC_MISSING_SUBPROTOCOL, none);
      return;
    }
    finish(WSG_HS_DEFER, WSG_HSC_D_SUBPROTOCOL, none);
    return;
  }
  if (pr.b >= 0) {
    finish(WSG_HS_CLOSING, WSG_HSC_INVALID_SUBPROTOCOL, pr);
    return;
  }
  // validateExtensions (:487-533): IExtension.validateResponse is Java's
  if (fld[C_EXTENSIONS].b >= 0) {
    if (cfg.extensions) {
      finish(WSG_HS_DEFER, WSG_HSC_D_EXTENSION, none);
      return;
    }
    finish(WSG_HS_CLOSING, WSG_HSC_INVALID_EXTENSIONS, none);
    return;
  }
  finish(WSG_HS_FINISHED, WSG_HSC_NONE, none);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WSG_HS_VWAVES))) void k_hs_validate(
    wsg_hs_config cfg, const uint8_t* resp, const uint64_t* resp_off, const uint8_t* keys, uint32_t n,
    uint8_t* expected, wsg_hs_result* result) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = resp_off[i], e = resp_off[i + 1];
  Req d;
  d.base = reinterpret_cast<const uint4*>(resp + (b & ~(uint64_t)15));
  d.lead = (uint32_t)(b & 15u);
  const uint32_t* kp = reinterpret_cast<const uint32_t*>(keys + (uint64_t)i * 24u);
  const KeyWords k{kp[0], kp[1], kp[2], kp[3], kp[4], kp[5]};
  validate_one(d, (int64_t)(e - b), cfg, k, expected + (uint64_t)i * WSG_HS_EXPECTED_STRIDE, result + i);
}

}  // namespace

void launch_hs_validate(const wsg_hs_config& cfg, const uint8_t* resp, const uint64_t* resp_off, const uint8_t* keys,
                        uint32_t n, uint8_t* expected, wsg_hs_result* result, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_hs_validate, dim3((n + 255) / 256), dim3(256), 0, s, cfg, resp, resp_off, keys, n, expected,
                       result);
}

void launch_hs_accept(const wsg_hs_config& cfg, const uint8_t* req, const uint64_t* req_off, uint32_t n,
                      uint8_t* resp, wsg_hs_result* result, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_hs_accept, dim3((n + 255) / 256), dim3(256), 0, s, cfg, req, req_off, n, resp, result);
}

}  // namespace ws
