// ws_rules.h — RFC 6455 header rules and the UTF-8 position rule, shared by the
// HIP kernels and the host side of libwsgpu (wsg_check_header / wsg_frame_available).
//
// Semantics follow snf4j-websocket (paths under .../websocket/frame/):
//   header rules and their order ........ FrameDecoder.java:197-256
//   available() framing ................. FrameDecoder.java:357-401
//   close status / reason ............... FrameDecoder.java:121-136
//   UTF-8 verdicts ...................... Utf8.java:73-92 (Hoehrmann DFA)
#pragma once
#include <stdint.h>

#include "../../include/wsgpu.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define WS_HD __host__ __device__ __forceinline__
#else  // plain C++ host build of the rules (tests/cpp: exhaustive rule-vs-DFA check)
#define WS_HD static inline
#endif

namespace ws {

// Opcode.findByValue(v) != null (Opcode.java:48-50)
WS_HD bool known_opcode(uint32_t v) { return v <= 2u || (v >= 8u && v <= 10u); }
WS_HD bool is_control(uint32_t v) { return v >= 8u; }

// Parsed frame header.
struct Header {
  uint32_t opcode, fin, rsv, masked, len7;
  uint32_t hdr_len;  // 2 + ext + (masked ? 4 : 0)
  uint64_t plen;     // payload length as read (u16 / u64 big-endian)
  uint32_t mask;     // mask key as a little-endian u32 of the 4 wire bytes
};

// Parse the header from the first n (<= 14 used) bytes; returns false when the
// header is not complete within n bytes.
// ---------------------------------------------------------------------------
// UTF-8.  The Hoehrmann DFA (Utf8.java) rejects at byte p exactly when, with
// the bytes before p a valid prefix, byte p is not allowed after the last <=3
// bytes.  That condition needs only the 3 preceding bytes, so every byte can be
// checked independently; the first flagged byte is the DFA's REJECT byte
// (proved exhaustively against the DFA in tests/test_utf8_rule.py).
// All masks below carry one flag per byte in bit 7 (0x80 lanes of a u32).
// ---------------------------------------------------------------------------
WS_HD uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, s);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * (s & 3u)));
#endif
}

// The 4 bytes at byte offset off (0..16) of the 20-byte window w0..w4 (little
// endian): word selects + one funnel shift, no indexed array (a device-side
// indexed array would live in scratch).
WS_HD uint32_t bytes_at(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4, uint32_t off) {
  const uint32_t q = off >> 2;
  const uint32_t lo = q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : (q == 3 ? w3 : w4)));
  const uint32_t hi = q == 0 ? w1 : (q == 1 ? w2 : (q == 2 ? w3 : w4));
  return alignbyte(hi, lo, off & 3u);
}

WS_HD uint32_t bswap32(uint32_t v) {
  return (v >> 24) | ((v >> 8) & 0xff00u) | ((v << 8) & 0xff0000u) | (v << 24);
}

// RFC 6455 header from the first 20 wire bytes of a frame (w0..w4, zero past the
// data); n = bytes available.  FrameDecoder.java:189-262 header reads.
WS_HD bool parse_header_words(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4, uint64_t n,
                              Header& o) {
  if (n < 2) return false;
  const uint32_t b0 = w0 & 0xffu, b1 = (w0 >> 8) & 0xffu;
  o.opcode = b0 & 0x0fu;
  o.fin = b0 >> 7;
  o.rsv = (b0 >> 4) & 7u;
  o.masked = b1 >> 7;
  o.len7 = b1 & 0x7fu;
  const uint32_t ext = o.len7 == 126 ? 2u : (o.len7 == 127 ? 8u : 0u);
  o.hdr_len = 2u + ext + (o.masked ? 4u : 0u);
  if (n < o.hdr_len) return false;
  if (ext == 0) {
    o.plen = o.len7;
  } else if (ext == 2) {
    o.plen = ((w0 >> 8) & 0xff00u) | (w0 >> 24);  // bytes 2, 3 big-endian
  } else {                                         // bytes 2..9 big-endian
    o.plen = ((uint64_t)bswap32(alignbyte(w1, w0, 2)) << 32) | bswap32(alignbyte(w2, w1, 2));
  }
  o.mask = o.masked ? bytes_at(w0, w1, w2, w3, w4, 2u + ext) : 0u;
  return true;
}

WS_HD bool parse_header(const uint8_t* h, uint64_t n, Header& o) {
  uint32_t w[5] = {0u, 0u, 0u, 0u, 0u};
  for (int i = 0; i < 20 && (uint64_t)i < n; ++i) w[i >> 2] |= (uint32_t)h[i] << (8 * (i & 3));
  return parse_header_words(w[0], w[1], w[2], w[3], w[4], n, o);
}

// The header checks of FrameDecoder.decode that run before the fragmentation
// test (:197-228): opcode, RSV, masking, control-frame rules.
WS_HD uint32_t rules_pre(const Header& h, int client_mode, int allow_ext) {
  if (!known_opcode(h.opcode)) return WSG_E_OPCODE;
  if (h.rsv != 0 && !allow_ext) return WSG_E_RSV;
  if ((int)h.masked == (client_mode ? 1 : 0)) return WSG_E_MASKING;
  if (is_control(h.opcode)) {
    if (!h.fin) return WSG_E_FRAG_CONTROL;
    if (h.len7 > 125) return WSG_E_CONTROL_LEN;
    if (h.opcode == WSG_OP_CLOSE && h.len7 == 1) return WSG_E_CLOSE_LEN;
  }
  return WSG_OK;
}

// Fragmentation test (:229-236) given FrameDecoder.fragmentation before the frame.
WS_HD uint32_t rules_frag(uint32_t opcode, bool fragmentation) {
  if (opcode == WSG_OP_CONTINUATION) return fragmentation ? WSG_OK : WSG_E_CONT_OUTSIDE;
  if (opcode == WSG_OP_TEXT || opcode == WSG_OP_BINARY) return fragmentation ? WSG_E_NONCONT_INSIDE : WSG_OK;
  return WSG_OK;
}

// Length checks after the fragmentation test (:238-256).
WS_HD uint32_t rules_post(const Header& h, int64_t max_payload) {
  if (h.len7 == 126) {
    if (h.plen < 126) return WSG_E_MIN_LEN;
  } else if (h.len7 == 127) {
    int64_t v = (int64_t)h.plen;
    if (v < 0 || v > 0x7fffffffLL) return WSG_E_MAX_PAYLOAD;
    if (v <= 0xffff) return WSG_E_MIN_LEN;
  }
  if ((int64_t)h.plen > max_payload) return WSG_E_TOO_LONG;
  return WSG_OK;
}

// Close status range (:124-128).
WS_HD bool close_status_ok(uint32_t status) { return status > 999u && status <= 4999u; }

WS_HD uint16_t close_code_of(uint32_t err) {
  if (err == WSG_OK) return 0;
  return (err == WSG_E_CLOSE_REASON || err == WSG_E_TEXT_UTF8) ? WSG_CLOSE_NON_UTF8 : WSG_CLOSE_PROTOCOL_ERROR;
}


constexpr uint32_t H80 = 0x80808080u;

// Error flags of the 4 bytes of `w` (little-endian: byte 0 first) given the
// word `p` holding the 4 bytes before it.
WS_HD uint32_t utf8_err_word(uint32_t w, uint32_t p) {
  const uint32_t w2 = w << 2, w3 = w << 3;
  const uint32_t hw = w & H80;
  const uint32_t cw = hw & (w << 1);  // byte >= C0
  const uint32_t gw = cw & w2;        // byte >= E0
  const uint32_t fw = gw & w3;        // byte >= F0
  const uint32_t hp = p & H80;
  const uint32_t cp = hp & (p << 1);
  const uint32_t gp = cp & (p << 2);
  const uint32_t fp = gp & (p << 3);
  // a continuation byte is expected after a lead within the last 1/2/3 bytes
  const uint32_t expect = alignbyte(cw, cp, 3) | alignbyte(gw, gp, 2) | alignbyte(fw, fp, 1);
  const uint32_t cont = hw ^ cw;  // 10xxxxxx
  uint32_t err = expect ^ cont;
  // C0, C1 (overlong 2-byte leads) and F5..FF are rejected at the byte itself
  err |= cw & ~((w & 0x3E3E3E3Eu) + 0x7F7F7F7Fu);
  err |= ((w & 0x7F7F7F7Fu) + 0x0B0B0B0Bu) & hw;
  // second-byte ranges after E0 (A0..BF), ED (80..9F), F0 (90..BF), F4 (80..8F)
  const uint32_t g1 = alignbyte(gw, gp, 3);  // previous byte >= E0
  if (g1) {
    const uint32_t p1 = alignbyte(w, p, 3);
    const uint32_t n = p1 & 0x0F0F0F0Fu;
    const uint32_t n0 = ~(n + 0x7F7F7F7Fu);
    const uint32_t nd = ~((n ^ 0x0D0D0D0Du) + 0x7F7F7F7Fu);
    const uint32_t n4 = ~((n ^ 0x04040404u) + 0x7F7F7F7Fu);
    const uint32_t isf = p1 << 3;  // previous byte >= F0 (given >= E0)
    const uint32_t b5 = w2, b54 = w2 | w3;
    err |= g1 & ((n0 & ~isf & ~b5) | (nd & ~isf & b5) | (n0 & isf & ~b54) | (n4 & isf & b54));
  }
  return err & H80;
}

// v_perm_b32 byte permute: each selector byte 0..7 picks byte of {hi:lo}.
WS_HD uint32_t perm_bytes(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const uint64_t t = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) r |= (uint32_t)((t >> (8 * ((sel >> (8 * i)) & 7))) & 0xffu) << (8 * i);
  return r;
#endif
}

// The kernels' UTF-8 rule (k_pieces): the continuation count is checked at the
// byte itself exactly as utf8_err_word does; the lead-specific rules (C0/C1,
// F5..FF, and the second-byte ranges after E0/ED/F0/F4) are checked on the
// (previous byte, byte) pair with three v_perm nibble-table lookups and are
// flagged on the SECOND byte of the pair.  So an invalid lead (C0, C1, F5..FF)
// is flagged one byte late; the frame-level verdict stays exact because the
// last byte of every validated frame is also tested with utf8_bad_last
// (k_pieces).  Exhaustively checked against the DFA in tests/cpp/utf8_rule_check.cpp.
// Unmasked form: bit 7 of each byte is the flag, the other bits are don't-care
// (the kernels OR the words of a lane and mask once).  24 VALU operations a word:
//   continuation count: w<<1, w<<2, w<<3 and three ANDs give ">= C0/E0/F0" in bit 7,
//   three byte-aligns move them 1/2/3 bytes on, one OR3 and one XOR with "10xxxxxx";
//   pair tables: th on previous-byte bits 5..3, tl on its bits 2..0, tb on the
//   byte's bits 5..4 (80/90/A0/B0 class); a common class bit is an error.
WS_HD uint32_t utf8_err_word_raw(uint32_t w, uint32_t p) {
  const uint32_t t1 = w << 1;
  const uint32_t cw = w & t1;          // bit 7: byte >= C0
  const uint32_t gw = cw & (w << 2);   // >= E0
  const uint32_t fw = gw & (w << 3);   // >= F0
  const uint32_t cont = w & ~t1;       // bit 7: 10xxxxxx
  const uint32_t tp = p << 1;
  const uint32_t cp = p & tp;
  const uint32_t gp = cp & (p << 2);
  const uint32_t fp = gp & (p << 3);
  const uint32_t c1 = alignbyte(cw, cp, 3);  // previous byte >= C0
  const uint32_t expect = c1 | alignbyte(gw, gp, 2) | alignbyte(fw, fp, 1);
  const uint32_t err = expect ^ cont;
  // pair tables: bits A=1 C0/C1, B=2 F5..F7, C=4 E0, D=8 ED, E=16 F0, F=32 F4, G=64 F8..FF
  const uint32_t p1 = alignbyte(w, p, 3);
  const uint32_t th = perm_bytes(0x40320804u, 0x00000001u, (p1 >> 3) & 0x07070707u);  // C0-7,C8-F,...,F8-F
  const uint32_t tl = perm_bytes(0x42424A60u, 0x40404155u, p1 & 0x07070707u);
  const uint32_t tb = perm_bytes(0u, 0x6B6B6757u, (w >> 4) & 0x03030303u);  // second byte 80/90/A0/B0 class
  return err | (((th & tl & tb) + 0x7F7F7F7Fu) & c1);
}

WS_HD uint32_t utf8_err_word_fast(uint32_t w, uint32_t p) { return utf8_err_word_raw(w, p) & H80; }

// The same rule split into per-word values, so that a word's shifts and masks are
// computed once and serve it both as the current word and as the next word's
// predecessor: the kernels run utf8_err_word_raw over runs of consecutive words.
//   t1 = w << 1; c/g/f = ">= C0/E0/F0" in bit 7; z = bits 5..3 of each byte (the
//   previous-byte table index, and the byte's own 80/88/.../B8 class: tb is the
//   bits 5..4 table with each entry doubled); l = bits 2..0.
// Two consecutive words share 64-bit shifts (v_lshlrev_b64: the bits that cross
// from the low word into the high one land in bits 0..2 of its byte 0, which the
// rule never reads).  u8w_err(x, p) == utf8_err_word_raw(x.w, p.w) in bit 7 of
// each byte (tests/cpp/utf8_rule_check.cpp).
struct U8W {
  uint32_t w, t1, c, g, f, z, l;
};

WS_HD void u8w_finish(U8W& x, uint32_t w, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t r3) {
  x.w = w;
  x.t1 = s1;
  x.c = w & s1;
  x.g = x.c & s2;
  x.f = x.g & s3;
  x.z = r3 & 0x07070707u;
  x.l = w & 0x07070707u;
}

WS_HD void u8w_one(uint32_t w, U8W& x) { u8w_finish(x, w, w << 1, w << 2, w << 3, w >> 3); }

WS_HD void u8w_pair(uint32_t wa, uint32_t wb, U8W& a, U8W& b) {
  const uint64_t P = ((uint64_t)wb << 32) | wa;
  uint64_t S1, S2, S3, R3;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(WSG_U8W_SHIFT32)
  // (written out: the compiler splits a 64-bit shift by a constant into two 32-bit ops)
  asm("v_lshlrev_b64 %0, 1, %1" : "=v"(S1) : "v"(P));
  asm("v_lshlrev_b64 %0, 2, %1" : "=v"(S2) : "v"(P));
  asm("v_lshlrev_b64 %0, 3, %1" : "=v"(S3) : "v"(P));
  asm("v_lshrrev_b64 %0, 3, %1" : "=v"(R3) : "v"(P));
#else
  S1 = P << 1; S2 = P << 2; S3 = P << 3; R3 = P >> 3;
#endif
  u8w_finish(a, wa, (uint32_t)S1, (uint32_t)S2, (uint32_t)S3, (uint32_t)R3);
  u8w_finish(b, wb, (uint32_t)(S1 >> 32), (uint32_t)(S2 >> 32), (uint32_t)(S3 >> 32), (uint32_t)(R3 >> 32));
}

WS_HD uint32_t u8w_err(const U8W& x, const U8W& p) {
  const uint32_t c1 = alignbyte(x.c, p.c, 3);  // previous byte >= C0
  const uint32_t expect = c1 | alignbyte(x.g, p.g, 2) | alignbyte(x.f, p.f, 1);
  const uint32_t err = expect ^ (x.w & ~x.t1);
  const uint32_t th = perm_bytes(0x40320804u, 0x00000001u, alignbyte(x.z, p.z, 3));
  const uint32_t tl = perm_bytes(0x42424A60u, 0x40404155u, alignbyte(x.l, p.l, 3));
  const uint32_t tb = perm_bytes(0x6B6B6B6Bu, 0x67675757u, x.z);
  return err | (((th & tl & tb) + 0x7F7F7F7Fu) & c1);
}

// Last byte of a frame is a lead the DFA rejects on its own (C0, C1, F5..FF):
// the pair rule above would flag it only at the next byte.
WS_HD bool utf8_bad_last(uint32_t b) { return b == 0xC0u || b == 0xC1u || b >= 0xF5u; }

// Error flag of a single byte b given its 3 predecessors (p1 nearest).
WS_HD bool utf8_err_byte(uint32_t p3, uint32_t p2, uint32_t p1, uint32_t b) {
  uint32_t p = (p3 << 8) | (p2 << 16) | (p1 << 24);
  return (utf8_err_word(b, p) & 0x80u) != 0;
}

// DFA state after a valid prefix is not ACCEPT (a continuation is still due),
// from the last 3 bytes (l1 = last).
WS_HD bool utf8_incomplete(uint32_t l3, uint32_t l2, uint32_t l1) {
  return l1 >= 0xC0u || l2 >= 0xE0u || l3 >= 0xF0u;
}

}  // namespace ws
