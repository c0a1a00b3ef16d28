// decode.hip — the frame decode pipeline on gfx950 (FrameDecoder + FrameUtf8Validator).
//
//   k_parse   thread per frame: header parse + the per-frame rules of
//             FrameDecoder.decode (:197-256), close status/reason (:121-136),
//             first/last payload bytes; block aggregates for the scans.
//   k_scan    a workgroup per 4096 block aggregates: exclusive scan within the
//             chunk (payload slot bytes = the length prefix-scan; last data /
//             message start / nonempty frame indices = max-scans; the UTF-8
//             carry).  Grids up to FUSED_SCAN_MAX_BLOCKS skip it: k_link reduces
//             the aggregates itself.
//   k_link    thread per frame: payload slot offset, the fragmentation rule
//             (:229-236) from the previous data frame's FIN, text-message
//             membership for the validator (FrameUtf8Validator.java:59-70), the
//             UTF-8 seam of a continuation frame against the scanned carry, the
//             frame's wsg_frame_desc with its status in the reference's check
//             order, the piece descriptors.
//   k_piecesN one wave per 2 KiB of payload output: coalesced 16-B loads, 4-byte
//             XOR unmask (:268-273), aligned 16-B stores into the frame slots,
//             per-lane SWAR UTF-8 rule with the 3-byte carry taken from the
//             neighbour lane (DPP) and the verdict folded by wavefront ballot.
//             A UTF-8 error sets its frame's status and the session's first
//             failing frame (atomicMin) directly.
//   k_final   thread per session: wsg_session_result + carry-out state.
#include "wsgpu_internal.h"
#include "wsgpu_scan.h"

namespace ws {

// UTF-8 validity of a short byte run (close reason), by the per-byte rule
__device__ bool utf8_valid_run(const uint8_t* wire, uint64_t off, uint32_t n, uint32_t mask, uint32_t phase0) {
  uint32_t p1 = 0, p2 = 0, p3 = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t b = wire[off + i] ^ ((mask >> (8 * ((phase0 + i) & 3))) & 0xffu);
    if (utf8_err_byte(p3, p2, p1, b)) return false;
    p3 = p2; p2 = p1; p1 = b;
  }
  return !utf8_incomplete(p3, p2, p1);
}

// ------------------------------------------------------------------ scan element
// Per-frame scan input: payload slot bytes, the "last frame of a kind" max fields as
// (k << 1) | bit carrying what k_link needs about that frame (FIN of the last data
// frame, TEXT-ness of the last message start), and the UTF-8 carry c3, so k_link
// never reads another frame's record.  Frame indices < 2^30 (wsg_decode_batch_device).
//
// c3 is the FrameUtf8Validator state a frame inherits (FrameUtf8Validator.java:59-98):
// the last <= 3 payload bytes of the data frames since the last reset, newest in bits
// 16-23 (the edge layout), their count in bits 24-25, bit 26 = reset, bit 27 = the
// session's tail from the previous batch still goes in front.  A message start resets
// it (FrameUtf8Validator.java:64-67), and so does a session's first frame, marked
// pending: k_parse reads no session state (so it can run while the previous batch
// still streams), and k_link puts the tail in front where a carry is used
// (resolve_c3).  A FIN frame contributes zero bytes (its message ended complete, or
// the frame failed).  carry_op is the associative "last 3 bytes of the concatenation,
// restarted at a reset".
struct DAgg {
  uint64_t sum;
  int32_t m0, m1, m2;
  uint32_t c3;
};
constexpr DAgg DAGG_ID = {0ull, -1, -1, -1, 0u};
constexpr uint32_t C3_RESET = 1u << 26;
constexpr uint32_t C3_PENDING = 1u << 27;

__device__ __forceinline__ uint32_t carry_op(uint32_t x, uint32_t y) {
  if (y & C3_RESET) return y;
  const uint32_t nx = (x >> 24) & 3u, ny = (y >> 24) & 3u;
  const uint32_t n = nx + ny < 3u ? nx + ny : 3u;
  return ((x & 0xffffffu) >> (8 * ny)) | (y & 0xffffffu) | (n << 24) | (x & (C3_RESET | C3_PENDING));
}
__device__ __forceinline__ DAgg agg_op(const DAgg& x, const DAgg& y) {
  DAgg r;
  r.sum = x.sum + y.sum;
  r.m0 = x.m0 > y.m0 ? x.m0 : y.m0;
  r.m1 = x.m1 > y.m1 ? x.m1 : y.m1;
  r.m2 = x.m2 > y.m2 ? x.m2 : y.m2;
  r.c3 = carry_op(x.c3, y.c3);
  return r;
}
template <int CTRL, int RM>
__device__ __forceinline__ DAgg agg_dpp(const DAgg& v) {
  DAgg t;
  t.sum = dpp_u64<CTRL, RM>(v.sum, 0ull);
  t.m0 = (int32_t)dpp_u32<CTRL, RM>((uint32_t)v.m0, 0xffffffffu);
  t.m1 = (int32_t)dpp_u32<CTRL, RM>((uint32_t)v.m1, 0xffffffffu);
  t.m2 = (int32_t)dpp_u32<CTRL, RM>((uint32_t)v.m2, 0xffffffffu);
  t.c3 = dpp_u32<CTRL, RM>(v.c3, 0u);  // (carry_op(0, y) == y: DAGG_ID.c3)
  return t;
}

// the session's carry from the previous batch, as a reset element
__device__ __forceinline__ uint32_t tail_c3(const wsg_session_state& st) {
  const uint32_t n = st.tail_len < 3 ? st.tail_len : 3u;  // tail[0] the oldest
  const uint32_t t = (uint32_t)st.tail[0] | ((uint32_t)st.tail[1] << 8) | ((uint32_t)st.tail[2] << 16);
  return C3_RESET | (n << 24) | ((t << (24 - 8 * n)) & 0xffffffu);
}

// a carry of frame k's session with its pending tail put in front
__device__ __forceinline__ uint32_t resolve_c3(uint32_t c, const wsg_session_state& st) {
  return (c & C3_PENDING) ? carry_op(tail_c3(st), c & ~(C3_RESET | C3_PENDING)) : c;
}

// l3: the frame's last 3 payload bytes (edge layout; 0 for a FIN frame)
__device__ __forceinline__ DAgg frame_agg(uint64_t k, const FrameRec& r, uint32_t l3, bool sess_first) {
  DAgg v;
  v.sum = (uint64_t)((r.len + 15u) & ~15u);
  const bool data = code_is_data(r.code);
  v.m0 = data ? (int32_t)((k << 1) | ((r.code & CODE_FIN) ? 1u : 0u)) : -1;
  v.m1 = code_is_start(r.code) ? (int32_t)((k << 1) | (code_op(r.code) == WSG_OP_TEXT ? 1u : 0u)) : -1;
  v.m2 = (data && r.len) ? (int32_t)(k << 1) : -1;
  uint32_t c = (data && r.len) ? (l3 & 0xffffffu) | ((r.len < 3 ? r.len : 3u) << 24) : 0u;
  if (code_is_start(r.code)) c |= C3_RESET;
  else if (sess_first) c |= C3_RESET | C3_PENDING;
  v.c3 = c;
  return v;
}

// ------------------------------------------------------------------ validator-only scan element
// The ws-utf8-validator stage alone (wsg_validate_batch_*) sees frame orders the
// decoder would reject, so it follows FrameUtf8Validator.java:59-98 literally: one
// context per session, opened by a TEXT frame when none is open, CONTINUED by a TEXT
// frame when one is, carried by a CONTINUATION only while open, closed by any
// validated FIN frame; BINARY and control frames leave it alone.  Per frame that is
// a function of the state (open, last <= 3 bytes of the context's payload):
//   TEXT !FIN, bytes t : (o, b) -> (1, o ? b.t : t)        OPENS  A = B = t
//   CONT !FIN, bytes t : (o, b) -> (o, b.t)  (garbage if !o) PASS   A = t
//   TEXT / CONT FIN    : -> (0, -)                          CONST  o = 0
//   BINARY, control    : identity                           PASS   A = empty
// and the composition of any run of them is one of
//   PASS  (o, b) -> (o, b.A)     OPENS (o, b) -> (1, o ? b.A : B)     CONST -> (o_out, B)
// fa = A (c3 layout, bits 0-25) | kind << 28 | o_out << 30; fb = B (0 unless a state
// with an open context can come out of it).  A session's first frame is composed
// with CONST(its carried-in state), so every exclusive prefix inside a session is a
// CONST: the context open before the frame and its last bytes.
struct VAgg {
  uint64_t sum;
  uint32_t fa, fb;
};
constexpr VAgg VAGG_ID = {0ull, 0u, 0u};
constexpr uint32_t VK_PASS = 0u, VK_OPENS = 1u, VK_CONST = 2u;
constexpr uint32_t VC_MASK = 0x3ffffffu;  // bytes + count
__device__ __forceinline__ uint32_t vkind(uint32_t fa) { return (fa >> 28) & 3u; }
__device__ __forceinline__ uint32_t vopen(uint32_t fa) { return (fa >> 30) & 1u; }
__device__ __forceinline__ uint32_t vcat(uint32_t x, uint32_t y) { return carry_op(x & VC_MASK, y & VC_MASK); }

__device__ __forceinline__ VAgg agg_op(const VAgg& x, const VAgg& y) {
  VAgg r;
  r.sum = x.sum + y.sum;
  const uint32_t kx = vkind(x.fa), ky = vkind(y.fa);
  if (ky == VK_CONST) {
    r.fa = y.fa; r.fb = y.fb;
    return r;
  }
  // bytes of an open context after x, then y appends to them; else y's own opening
  const bool xb = kx == VK_OPENS || (kx == VK_CONST && vopen(x.fa));
  r.fb = xb ? vcat(x.fb, y.fa) : (ky == VK_OPENS ? y.fb : 0u);
  if (kx == VK_CONST) {
    r.fa = (VK_CONST << 28) | ((vopen(x.fa) || ky == VK_OPENS) ? (1u << 30) : 0u);
    if (!(r.fa >> 30)) r.fb = 0u;
  } else {
    r.fa = vcat(x.fa, y.fa) | ((kx == VK_OPENS || ky == VK_OPENS ? VK_OPENS : VK_PASS) << 28);
  }
  return r;
}
template <int CTRL, int RM>
__device__ __forceinline__ VAgg agg_dpp(const VAgg& v) {
  VAgg t;
  t.sum = dpp_u64<CTRL, RM>(v.sum, 0ull);
  t.fa = dpp_u32<CTRL, RM>(v.fa, 0u);
  t.fb = dpp_u32<CTRL, RM>(v.fb, 0u);
  return t;
}

// frame k's element (l3: its last 3 payload bytes, 0 for a FIN frame)
__device__ __forceinline__ VAgg vframe_agg(const FrameRec& r, uint32_t l3, bool sess_first, const wsg_session_state* st) {
  VAgg v;
  v.sum = (uint64_t)((r.len + 15u) & ~15u);
  const uint32_t op = code_op(r.code);
  const uint32_t t = r.len ? (l3 & 0xffffffu) | ((r.len < 3 ? r.len : 3u) << 24) : 0u;
  v.fb = 0u;
  if (op != WSG_OP_TEXT && op != WSG_OP_CONTINUATION) v.fa = 0u;
  else if (r.code & CODE_FIN) v.fa = VK_CONST << 28;
  else if (op == WSG_OP_TEXT) { v.fa = t | (VK_OPENS << 28); v.fb = t; }
  else v.fa = t;
  if (sess_first) {  // the state carried in from the previous batch
    VAgg c;
    c.sum = 0;
    c.fa = (VK_CONST << 28) | (st->text_open ? (1u << 30) : 0u);
    c.fb = st->text_open ? (tail_c3(*st) & VC_MASK) : 0u;
    v = agg_op(c, v);
  }
  return v;
}

// Block aggregates: blk_sum[b], and the maxima / carry in four rows of blk_max
// whose stride is nblk rounded up to 4, so that every row is 16-B aligned (k_link
// folds them with 16-B loads).
__device__ __forceinline__ uint32_t blk_stride(const DecodeArgs& a) { return (a.nblk + 3u) & ~3u; }
__device__ __forceinline__ DAgg load_blk(const DecodeArgs& a, uint32_t b) {
  const uint32_t st = blk_stride(a);
  DAgg e;
  e.sum = a.blk_sum[b];
  e.m0 = a.blk_max[b];
  e.m1 = a.blk_max[st + b];
  e.m2 = a.blk_max[2 * st + b];
  e.c3 = (uint32_t)a.blk_max[3 * st + b];
  return e;
}
__device__ __forceinline__ void store_blk(const DecodeArgs& a, uint32_t b, const DAgg& e) {
  const uint32_t st = blk_stride(a);
  a.blk_sum[b] = e.sum;
  a.blk_max[b] = e.m0;
  a.blk_max[st + b] = e.m1;
  a.blk_max[2 * st + b] = e.m2;
  a.blk_max[3 * st + b] = (int32_t)e.c3;
}
// (validator-only mode: fa, fb in rows 0 and 1)
__device__ __forceinline__ void load_blk(const DecodeArgs& a, uint32_t b, VAgg& e) {
  e.sum = a.blk_sum[b];
  e.fa = (uint32_t)a.blk_max[b];
  e.fb = (uint32_t)a.blk_max[blk_stride(a) + b];
}
__device__ __forceinline__ void store_blk(const DecodeArgs& a, uint32_t b, const VAgg& e) {
  a.blk_sum[b] = e.sum;
  a.blk_max[b] = (int32_t)e.fa;
  a.blk_max[blk_stride(a) + b] = (int32_t)e.fb;
}
__device__ __forceinline__ void load_blk(const DecodeArgs& a, uint32_t b, DAgg& e) { e = load_blk(a, b); }

__device__ __forceinline__ uint32_t wave_session(const DecodeArgs& a, uint64_t k) {
  return wave_find_session(a.session_first, a.n_sessions, a.n_frames, k);
}

// ------------------------------------------------------------------ k_parse
// Frame k's header rules and record; returns its scan element.  d[0..5]: the wire
// words from o & ~3 (zero past the wire end).
__device__ __forceinline__ DAgg parse_one(const DecodeArgs& a, uint64_t k, uint64_t o, uint64_t e, const uint32_t d[6],
                                          uint32_t s) {
  const uint64_t ext = e > o ? e - o : 0;
  const uint32_t sh = (uint32_t)(o & 3);
  const uint32_t w0 = alignbyte(d[1], d[0], sh), w1 = alignbyte(d[2], d[1], sh), w2 = alignbyte(d[3], d[2], sh);
  const uint32_t w3 = alignbyte(d[4], d[3], sh), w4 = alignbyte(d[5], d[4], sh);
  Header hd;
  uint32_t pre = 0, post = 0, len = 0, f3 = 0, l3 = 0;
  uint64_t src = o;
  if (!parse_header_words(w0, w1, w2, w3, w4, ext, hd)) {
    pre = WSG_E_BATCH;
    hd.opcode = w0 & 15u; hd.fin = (w0 >> 7) & 1u; hd.rsv = (w0 >> 4) & 7u; hd.masked = 0; hd.mask = 0;
  } else {
    pre = rules_pre(hd, a.client_mode, a.allow_ext);
    post = rules_post(hd, a.max_payload);
    // the batch's frame extent must be the header's (sparse: the frame must fit before the wire end)
    if (!pre && !post && (a.sparse ? (uint64_t)hd.hdr_len + hd.plen > ext : (uint64_t)hd.hdr_len + hd.plen != ext))
      pre = WSG_E_BATCH;
    if (!pre && !post) {
      len = (uint32_t)hd.plen;
      src = o + hd.hdr_len;
      if (hd.opcode == WSG_OP_CLOSE && len >= 2) {  // createFrame, FrameDecoder.java:121-136
        uint32_t b0 = a.wire[src] ^ (hd.mask & 0xffu);
        uint32_t b1 = a.wire[src + 1] ^ ((hd.mask >> 8) & 0xffu);
        if (!close_status_ok((b0 << 8) | b1)) post = WSG_E_CLOSE_STATUS;
        else if (len > 2 && !utf8_valid_run(a.wire, src + 2, len - 2, hd.mask, 2)) post = WSG_E_CLOSE_REASON;
      }
      if (hd.opcode <= WSG_OP_TEXT) {  // fragment-boundary bytes for the UTF-8 carry
        // first 3 payload bytes: within the header's 20 loaded bytes (hdr_len <= 14)
        const uint32_t nf = len < 3 ? len : 3;
        const uint32_t keep3 = nf >= 3 ? 0xffffffu : (nf == 2 ? 0xffffu : (nf == 1 ? 0xffu : 0u));
        f3 = (bytes_at(w0, w1, w2, w3, w4, hd.hdr_len) ^ hd.mask) & keep3;
        // last 3 payload bytes: only a non-FIN fragment's are needed (the carry into the
        // next fragment or batch); a frame's own last-byte and end-of-message tests
        // run in k_pieces on bytes it holds, so a FIN frame costs no second line here
        if (nf && !hd.fin) {
          const uint64_t e3 = src + len - nf;  // first of the last nf bytes
          const uint64_t q = e3 & ~3ull;
          uint32_t lo, hi;
          if (q + 8 <= a.wire_len) {
            lo = *(const uint32_t*)(a.wire + q);
            hi = *(const uint32_t*)(a.wire + q + 4);
          } else {
            lo = hi = 0;
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i)
              if (q + i < a.wire_len) (i < 4 ? lo : hi) |= (uint32_t)a.wire[q + i] << (8 * (i & 3));
          }
          const uint32_t t = alignbyte(hi, lo, (uint32_t)(e3 & 3));  // bytes e3.. e3+3
          const uint32_t ph = (uint32_t)(len - nf) & 3u;            // mask phase of byte e3
          const uint32_t m = (hd.mask >> (8 * ph)) | (ph ? hd.mask << (32 - 8 * ph) : 0u);
          const uint32_t u = t ^ m;                                  // unmasked bytes e3..e3+3
          for (uint32_t i = 0; i < nf; ++i) {  // byte len-1-i (newest first) -> bits 16-8i
            const uint32_t j = nf - 1 - i;     // its index in u
            l3 |= ((u >> (8 * j)) & 0xffu) << (8 * (2 - i));
          }
        }
      }
    }
  }
  a.edge[k] = f3;
  a.edge[a.n_frames + k] = l3;
  if (pre || post) len = 0;
  FrameRec r;
  r.src = src;
  r.len = len;
  r.mask = hd.mask;
  r.code = (pre << CODE_PRE_SHIFT) | (post << CODE_POST_SHIFT) | (hd.fin ? CODE_FIN : 0u) |
           (hd.rsv << CODE_RSV_SHIFT) | (hd.masked ? CODE_MASKED : 0u) | (hd.opcode << CODE_OP_SHIFT);
  r.sess = s;
  a.rec[k] = r;
  return frame_agg(k, r, l3, k == a.session_first[s]);
}

__global__ __launch_bounds__(DBLOCK) void k_parse(DecodeArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * DBLOCK + threadIdx.x;
  DAgg v = DAGG_ID;
  if (k < a.n_frames) {
    const uint64_t o = a.frame_off[k], e = a.sparse ? a.wire_len : a.frame_off[k + 1];
    // wire words from o & ~3 (zero past the wire end)
    uint32_t d[6];
    const uint64_t a4 = o & ~3ull;
    if (a4 + 24 <= a.wire_len) {
      const uint32_t* p = (const uint32_t*)(a.wire + a4);
#pragma unroll
      for (int j = 0; j < 6; ++j) d[j] = p[j];
    } else {
#pragma unroll
      for (int j = 0; j < 6; ++j) d[j] = 0u;
#pragma unroll
      for (uint32_t b = 0; b < 24u; ++b)
        if (a4 + b < a.wire_len) d[b >> 2] |= (uint32_t)a.wire[a4 + b] << (8 * (b & 3));
    }
    v = parse_one(a, k, o, e, d, wave_session(a, k));
  }
  DAgg tot;
  block_excl_scan_t(v, &tot, DAGG_ID);
  if (threadIdx.x == 0) store_blk(a, blockIdx.x, tot);
}

// ------------------------------------------------------------------ k_vparse
// Validator-only mode (the "ws-utf8-validator" stage alone, FrameUtf8Validator.java:
// 59-98, e.g. after permessage-deflate inflated the payloads): frame k is
// in_desc[k], its plain payload at wire[payload_off, +len).  Builds the same
// FrameRec / edges / block aggregates as k_parse, with no header rules.
__device__ __forceinline__ uint32_t plain_byte(const DecodeArgs& a, uint64_t i) { return i < a.wire_len ? a.wire[i] : 0u; }
// the 4 plain bytes at i (zero past the end), from two aligned dword loads
__device__ __forceinline__ uint32_t plain_word(const DecodeArgs& a, uint64_t i) {
  const uint64_t q = i & ~3ull;
  if (q + 8 <= a.wire_len) {
    const uint32_t lo = *(const uint32_t*)(a.wire + q), hi = *(const uint32_t*)(a.wire + q + 4);
    return alignbyte(hi, lo, (uint32_t)(i & 3u));
  }
  return plain_byte(a, i) | (plain_byte(a, i + 1) << 8) | (plain_byte(a, i + 2) << 16) | (plain_byte(a, i + 3) << 24);
}

__global__ __launch_bounds__(DBLOCK) void k_vparse(DecodeArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * DBLOCK + threadIdx.x;
  VAgg v = VAGG_ID;
  if (k < a.n_frames) {
    const uint32_t s = wave_session(a, k);
    const wsg_frame_desc d = a.in_desc[k];
    const uint32_t op = d.opcode & 15u, fin = (d.flags >> 7) & 1u, rsv = (d.flags >> 4) & 7u;
    const uint32_t len = d.payload_len;
    const uint64_t src = d.payload_off;
    uint32_t l3 = 0;
    // the last bytes of a non-FIN text/continuation frame: the carry into what follows.
    // (a frame's first bytes matter only at a seam, which k_link knows: it loads them)
    if (op <= WSG_OP_TEXT && len && !fin) {
      const uint32_t nf = len < 3 ? len : 3;
      const uint32_t keep = nf >= 3 ? 0xffffffu : (nf == 2 ? 0xffffu : 0xffu);
      l3 = (plain_word(a, src + len - nf) & keep) << (8 * (3 - nf));  // newest in bits 16-23
    }
    a.edge[a.n_frames + k] = l3;
    FrameRec r;
    r.src = src;
    r.len = len;
    r.mask = 0;
    r.code = (fin ? CODE_FIN : 0u) | (rsv << CODE_RSV_SHIFT) | (op << CODE_OP_SHIFT);
    r.sess = s;
    a.rec[k] = r;
    const bool first = k == a.session_first[s];
    v = vframe_agg(r, l3, first, first ? &a.state[s] : nullptr);
  }
  VAgg tot;
  block_excl_scan_t(v, &tot, VAGG_ID);
  if (threadIdx.x == 0) store_blk(a, blockIdx.x, tot);
}

// ------------------------------------------------------------------ k_scan
// Grids beyond FUSED_SCAN_MAX_BLOCKS: one workgroup per chunk of SCAN_CHUNK block
// aggregates scans its chunk in place (exclusive within the chunk, 4 entries per
// thread) and leaves the chunk's total; k_link folds the totals of the chunks
// before its own (a handful) in order.
__device__ __forceinline__ void store_chunk(const DecodeArgs& a, uint32_t c, const DAgg& t) {
  a.chunk_sum[c] = t.sum;
  a.chunk_max[4 * c + 0] = t.m0;
  a.chunk_max[4 * c + 1] = t.m1;
  a.chunk_max[4 * c + 2] = t.m2;
  a.chunk_max[4 * c + 3] = (int32_t)t.c3;
}
__device__ __forceinline__ void store_chunk(const DecodeArgs& a, uint32_t c, const VAgg& t) {
  a.chunk_sum[c] = t.sum;
  a.chunk_max[4 * c + 0] = (int32_t)t.fa;
  a.chunk_max[4 * c + 1] = (int32_t)t.fb;
}
__device__ __forceinline__ void load_chunk(const DecodeArgs& a, uint32_t c, DAgg& e) {
  e.sum = a.chunk_sum[c];
  e.m0 = a.chunk_max[4 * c + 0];
  e.m1 = a.chunk_max[4 * c + 1];
  e.m2 = a.chunk_max[4 * c + 2];
  e.c3 = (uint32_t)a.chunk_max[4 * c + 3];
}
__device__ __forceinline__ void load_chunk(const DecodeArgs& a, uint32_t c, VAgg& e) {
  e.sum = a.chunk_sum[c];
  e.fa = (uint32_t)a.chunk_max[4 * c + 0];
  e.fb = (uint32_t)a.chunk_max[4 * c + 1];
}

__device__ __forceinline__ DAgg agg_ident(const DAgg*) { return DAGG_ID; }
__device__ __forceinline__ VAgg agg_ident(const VAgg*) { return VAGG_ID; }

template <class T>
__global__ __launch_bounds__(1024) void k_scan(DecodeArgs a) {
  const T ident = agg_ident((const T*)nullptr);
  const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
  T e[4], t = ident;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    e[i] = ident;
    if (b0 + i < a.nblk) load_blk(a, b0 + i, e[i]);
    t = agg_op(t, e[i]);
  }
  T tot;
  T ex = block_excl_scan_t(t, &tot, ident);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (b0 + i < a.nblk) store_blk(a, b0 + i, ex);
    ex = agg_op(ex, e[i]);
  }
  if (threadIdx.x == 0) store_chunk(a, blockIdx.x, tot);
}

// ------------------------------------------------------------------ UTF-8 seams
// UTF-8 verdict of a validated continuation frame's first (<= 3) bytes after the
// message carry c3, and of the message end when a FIN frame shorter than 3 bytes
// ends on the carry: FrameUtf8Validator.java:78-96 at the fragment seams (every
// other byte of the frame is checked by k_pieces).
__device__ bool seam_utf8_error(uint32_t c3, uint32_t f3, uint32_t len, bool fin) {
  // the carry then the frame's head bytes, oldest in bits 0-7 (registers, no array)
  const uint32_t nc = (c3 >> 24) & 3u, nh = len < 3 ? len : 3u, n = nc + nh;
  const uint64_t win = (uint64_t)((c3 & 0xffffffu) >> (24 - 8 * nc)) | ((uint64_t)f3 << (8 * nc));
  for (uint32_t i = nc; i < n; ++i) {
    const uint32_t p1 = i >= 1 ? (uint32_t)(win >> (8 * (i - 1))) & 0xffu : 0u;
    const uint32_t p2 = i >= 2 ? (uint32_t)(win >> (8 * (i - 2))) & 0xffu : 0u;
    const uint32_t p3 = i >= 3 ? (uint32_t)(win >> (8 * (i - 3))) & 0xffu : 0u;
    if (utf8_err_byte(p3, p2, p1, (uint32_t)(win >> (8 * i)) & 0xffu)) return true;
  }
  // the frame's last byte, and the end of a FIN message of >= 3 bytes in this frame,
  // are tested by k_pieces (tail_error); a shorter FIN frame ends on the carry
  if (fin && len < 3) {
    const uint32_t t1 = n >= 1 ? (uint32_t)(win >> (8 * (n - 1))) & 0xffu : 0u;
    const uint32_t t2 = n >= 2 ? (uint32_t)(win >> (8 * (n - 2))) & 0xffu : 0u;
    const uint32_t t3 = n >= 3 ? (uint32_t)(win >> (8 * (n - 3))) & 0xffu : 0u;
    if (utf8_incomplete(t3, t2, t1)) return true;
  }
  return false;
}

// Descriptors of the pieces whose first output byte falls in a frame's slot,
// written cooperatively: the wave's pieces are contiguous, lane i writes the
// wave's pieces i, i+64, ... (coalesced 16-B stores) after finding the owning
// frame with a shuffle search over the exclusive piece counts.  cont: the frame's
// head bytes are checked against a carry by k_link (PDF_CONT).
__device__ __forceinline__ void write_pieces(const DecodeArgs& a, bool live, uint64_t k, const FrameRec& r,
                                             uint64_t ex_sum, bool validate, bool cont, int lane) {
  const uint64_t slot = live ? (uint64_t)((r.len + 15u) & ~15u) : 0ull;
  const uint64_t slot_end = ex_sum + slot;
  const uint32_t pc0 = (uint32_t)((ex_sum + PIECE - 1) / PIECE);
  const uint32_t cnt = slot ? (uint32_t)((slot_end + PIECE - 1) / PIECE) - pc0 : 0u;
  uint32_t cum = cnt;  // inclusive wave scan of the counts
  cum = wave_incl_sum_u32(cum);
  const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)cum, 63);
  cum -= cnt;  // exclusive
  if (!T) return;
  // per-frame fields a piece needs: src, slot start, len, mask, frame | validate << 31
  const uint32_t fk = (uint32_t)k | (validate ? 0x80000000u : 0u) | ((live && (r.code & CODE_FIN)) ? 0x40000000u : 0u);
  for (uint32_t t = lane; t < ((T + 63u) & ~63u); t += 64) {
    int o = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1)
      if ((uint32_t)__shfl((int)cum, o + step, 64) <= t) o += step;
    const uint32_t o_cum = (uint32_t)__shfl((int)cum, o, 64);
    const uint32_t o_pc0 = (uint32_t)__shfl((int)pc0, o, 64);
    const uint64_t o_out = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(ex_sum >> 32), o, 64) << 32) |
                           (uint32_t)__shfl((int)(uint32_t)ex_sum, o, 64);
    const uint64_t o_src = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(r.src >> 32), o, 64) << 32) |
                           (uint32_t)__shfl((int)(uint32_t)r.src, o, 64);
    const uint32_t o_len = (uint32_t)__shfl((int)r.len, o, 64);
    const uint32_t o_mask = (uint32_t)__shfl((int)r.mask, o, 64);
    const uint32_t o_fk = (uint32_t)__shfl((int)fk, o, 64);
    const bool o_cont = __shfl((int)cont, o, 64) != 0;
    if (t >= T) continue;
    const uint64_t pc = (uint64_t)o_pc0 + (t - o_cum);
    if (pc >= a.n_pieces) continue;  // beyond the grid: the frame failed with WSG_E_BATCH above
    const uint64_t ps = pc * PIECE;
    const uint64_t o_end = o_out + ((o_len + 15u) & ~15u);
    const uint32_t j0 = (uint32_t)(ps - o_out);
    const uint32_t left = o_len - j0;
    // runs past its frame's slot: other frames' bytes follow, unless it is the batch's
    // last frame (a slot ending the payload region)
    const bool single = o_end >= ps + PIECE || (uint64_t)(o_fk & 0x3fffffffu) + 1 == a.n_frames;
    PieceDesc d;
    d.info = ((o_src + j0) & PD_SRC_MASK) | ((uint64_t)(left < PIECE ? left : PIECE) << PD_NB_SHIFT) |
             ((o_fk & 0x80000000u) ? PD_VALIDATE : 0ull) | (j0 == 0 ? PD_FIRST : 0ull) | (single ? 0ull : PD_MULTI) |
             (left <= PIECE ? PD_LAST : 0ull) | ((o_fk & 0x40000000u) ? PD_FIN : 0ull);
    d.mask = o_mask;
    d.frame = (o_fk & PDF_INDEX) | (o_cont ? PDF_CONT : 0u);
    a.pieces[pc] = d;
  }
}

// ------------------------------------------------------------------ k_link
__global__ __launch_bounds__(DBLOCK) void k_link(DecodeArgs a) {
  const int lane = threadIdx.x & 63;
  // the aggregate of every frame before this block: k_scan's exclusive scan, or (small
  // grids, no k_scan launch) this block's own reduction of k_parse's block aggregates.
  // Coalesced loads (entry i * DBLOCK + t); the sums and maxima commute and fold as
  // loaded, the order-sensitive carries go through LDS so that each thread folds a
  // contiguous run of them, in order.
  DAgg bp;
  if (a.fused_scan) {
    __shared__ uint32_t c3s[FUSED_SCAN_MAX_BLOCKS];
    DAgg t = DAGG_ID;
    // four consecutive blocks a thread: 16-B loads of each row (6 loads per 4 blocks)
    const uint32_t nb = blockIdx.x, st = blk_stride(a);
    for (uint32_t b = threadIdx.x * 4u; b < nb; b += DBLOCK * 4u) {
      if (b + 4u <= nb) {
        const int4 x0 = *reinterpret_cast<const int4*>(a.blk_max + b);
        const int4 x1 = *reinterpret_cast<const int4*>(a.blk_max + st + b);
        const int4 x2 = *reinterpret_cast<const int4*>(a.blk_max + 2 * st + b);
        const int4 x3 = *reinterpret_cast<const int4*>(a.blk_max + 3 * st + b);
        const ulonglong2 s0 = *reinterpret_cast<const ulonglong2*>(a.blk_sum + b);
        const ulonglong2 s1 = *reinterpret_cast<const ulonglong2*>(a.blk_sum + b + 2);
        t.sum += s0.x + s0.y + s1.x + s1.y;
        t.m0 = max(max(t.m0, max(x0.x, x0.y)), max(x0.z, x0.w));
        t.m1 = max(max(t.m1, max(x1.x, x1.y)), max(x1.z, x1.w));
        t.m2 = max(max(t.m2, max(x2.x, x2.y)), max(x2.z, x2.w));
        c3s[b] = (uint32_t)x3.x;
        c3s[b + 1] = (uint32_t)x3.y;
        c3s[b + 2] = (uint32_t)x3.z;
        c3s[b + 3] = (uint32_t)x3.w;
      } else {
        for (uint32_t i = b; i < nb; ++i) {
          const DAgg e = load_blk(a, i);
          t.sum += e.sum;
          t.m0 = t.m0 > e.m0 ? t.m0 : e.m0;
          t.m1 = t.m1 > e.m1 ? t.m1 : e.m1;
          t.m2 = t.m2 > e.m2 ? t.m2 : e.m2;
          c3s[i] = e.c3;
        }
      }
    }
    __syncthreads();
    const uint32_t per = (blockIdx.x + DBLOCK - 1) / DBLOCK;
    const uint32_t b0 = threadIdx.x * per, b1 = b0 + per < blockIdx.x ? b0 + per : blockIdx.x;
    for (uint32_t b = b0; b < b1; ++b) t.c3 = carry_op(t.c3, c3s[b]);
    block_excl_scan_t(t, &bp, DAGG_ID);
  } else {  // k_scan's chunks: the totals of the chunks before this block's, then its own prefix
    bp = DAGG_ID;
    for (uint32_t c = 0; c < blockIdx.x / SCAN_CHUNK; ++c) {
      DAgg e;
      e.sum = a.chunk_sum[c];
      e.m0 = a.chunk_max[4 * c + 0];
      e.m1 = a.chunk_max[4 * c + 1];
      e.m2 = a.chunk_max[4 * c + 2];
      e.c3 = (uint32_t)a.chunk_max[4 * c + 3];
      bp = agg_op(bp, e);
    }
    bp = agg_op(bp, load_blk(a, blockIdx.x));
  }
  {
    const uint64_t k = (uint64_t)blockIdx.x * DBLOCK + threadIdx.x;
    const bool live = k < a.n_frames;
    FrameRec r = {0ull, 0u, 0u, 0u, 0u};
    DAgg v = DAGG_ID;
    wsg_session_state st = {};
    bool first = false;
    if (live) {
      r = a.rec[k];
      const uint32_t l3 = (code_is_data(r.code) && r.len && !(r.code & CODE_FIN)) ? a.edge[a.n_frames + k] : 0u;
      first = k == a.session_first[r.sess];
      st = a.state[r.sess];
      v = frame_agg(k, r, l3, first);
    }
    DAgg tot;
    DAgg ex = agg_op(bp, block_excl_scan_t(v, &tot, DAGG_ID));
    if (blockIdx.x + 1 == a.nblk && threadIdx.x == 0) *a.total = bp.sum + tot.sum;
    uint32_t validate = 0;
    if (live) {
      const int32_t jd = ex.m0 >> 1, jm = ex.m1 >> 1;  // (-1 >> 1 == -1)
      const uint32_t s = r.sess;
      const int32_t sf = (int32_t)a.session_first[s];
      const uint32_t op = code_op(r.code);
      uint32_t frag_err = 0;
      bool text = false;
      if (!code_pre(r.code)) {
        // FrameDecoder.fragmentation before this frame: FIN of the previous data frame
        const bool frag = jd >= sf ? !(ex.m0 & 1) : (st.fragmentation != 0);
        if (!a.validator_only) frag_err = rules_frag(op, frag);
        if (a.validate) {
          text = op == WSG_OP_TEXT;
          if (op == WSG_OP_CONTINUATION) text = jm >= sf ? (ex.m1 & 1) != 0 : (st.text_open != 0);
        }
      }
      // the frame's status in the reference's check order (header rules, fragmentation,
      // lengths / close, then the validator); a failed frame is never validated
      uint32_t status = code_pre(r.code) ? code_pre(r.code) : (frag_err ? frag_err : code_post(r.code));
      if (!status && ex.sum + r.len > a.n_pieces * PIECE) status = WSG_E_BATCH;  // slots beyond the piece grid
      // a validated continuation's head against the message carry (the inherited
      // validator state: the session tail for its first frame)
      if (!status && text && op == WSG_OP_CONTINUATION &&
          seam_utf8_error(first ? tail_c3(st) : resolve_c3(ex.c3, st), a.edge[k], r.len, (r.code & CODE_FIN) != 0))
        status = WSG_E_TEXT_UTF8;
      validate = (text && !status) ? 1u : 0u;
      // bit 1: the head is checked against a carry here (piece_general masks it)
      a.vflag[k] = (uint8_t)(validate | ((validate && op == WSG_OP_CONTINUATION) ? 2u : 0u));
      wsg_frame_desc d;
      d.payload_off = ex.sum;
      d.payload_len = r.len;
      d.opcode = (uint8_t)op;
      d.flags = (uint8_t)(((r.code & CODE_FIN) ? 0x80u : 0u) | (((r.code >> CODE_RSV_SHIFT) & 7u) << 4) |
                          ((r.code & CODE_MASKED) ? 1u : 0u));
      d.status = (uint16_t)status;
      a.desc[k] = d;
      if (status) atomicMin((unsigned long long*)&a.sess_err[s], (unsigned long long)k);
      // the session's last frame: what k_final needs for the carry-out state (the last
      // data frame, the last message start, the validator carry through this frame)
      if (k + 1 == a.session_first[s + 1]) {
        a.slink[s] = code_is_data(r.code) ? (int32_t)k : jd;
        a.slink[a.n_sessions + s] = code_is_start(r.code) ? (int32_t)k : jm;
        a.slink[2 * a.n_sessions + s] = (int32_t)resolve_c3(first ? v.c3 : carry_op(ex.c3, v.c3), st);
      }
    }
    write_pieces(a, live, k, r, ex.sum, validate != 0, live && code_op(r.code) == WSG_OP_CONTINUATION, lane);
  }
}

// ------------------------------------------------------------------ k_vlink
// k_link of the validator-only stage: the exclusive scan of the VAgg elements
// gives every frame the FrameUtf8Validator context it meets (open or not, its last
// <= 3 bytes).  A frame is validated when it is TEXT, or a CONTINUATION while a
// context is open (FrameUtf8Validator.java:63-75); a validated frame that meets an
// open context (a CONTINUATION, or a TEXT frame continuing it) has its head bytes
// checked against that carry here, the rest by the piece kernel.
__global__ __launch_bounds__(DBLOCK) void k_vlink(DecodeArgs a) {
  const int lane = threadIdx.x & 63;
  VAgg bp;
  if (a.fused_scan) {  // fold the block aggregates before this block (in order: staged in LDS)
    __shared__ uint32_t fas[FUSED_SCAN_MAX_BLOCKS], fbs[FUSED_SCAN_MAX_BLOCKS];
    const uint32_t nb = blockIdx.x, st = blk_stride(a);
    uint64_t sum = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += DBLOCK) {
      sum += a.blk_sum[b];
      fas[b] = (uint32_t)a.blk_max[b];
      fbs[b] = (uint32_t)a.blk_max[st + b];
    }
    __syncthreads();
    const uint32_t per = (nb + DBLOCK - 1) / DBLOCK;
    const uint32_t b0 = threadIdx.x * per, b1 = b0 + per < nb ? b0 + per : nb;
    VAgg t = VAGG_ID;
    for (uint32_t b = b0; b < b1; ++b) t = agg_op(t, VAgg{0ull, fas[b], fbs[b]});
    t.sum = sum;  // (the sums commute: folded as loaded)
    block_excl_scan_t(t, &bp, VAGG_ID);
  } else {
    bp = VAGG_ID;
    for (uint32_t c = 0; c < blockIdx.x / SCAN_CHUNK; ++c) {
      VAgg e;
      load_chunk(a, c, e);
      bp = agg_op(bp, e);
    }
    VAgg e;
    load_blk(a, blockIdx.x, e);
    bp = agg_op(bp, e);
  }
  const uint64_t k = (uint64_t)blockIdx.x * DBLOCK + threadIdx.x;
  const bool live = k < a.n_frames;
  FrameRec r = {0ull, 0u, 0u, 0u, 0u};
  VAgg v = VAGG_ID;
  wsg_session_state st = {};
  bool first = false;
  if (live) {
    r = a.rec[k];
    const uint32_t l3 = (r.len && !(r.code & CODE_FIN)) ? a.edge[a.n_frames + k] : 0u;
    first = k == a.session_first[r.sess];
    if (first) st = a.state[r.sess];
    v = vframe_agg(r, l3, first, &st);
  }
  VAgg tot;
  const VAgg ex = agg_op(bp, block_excl_scan_t(v, &tot, VAGG_ID));
  if (blockIdx.x + 1 == a.nblk && threadIdx.x == 0) *a.total = bp.sum + tot.sum;
  bool validate = false, seam = false;
  if (live) {
    const uint32_t s = r.sess;
    const uint32_t op = code_op(r.code);
    // the context this frame meets: the session's carried-in state, or the (CONST) prefix
    const bool open = first ? st.text_open != 0 : vopen(ex.fa) != 0;
    const uint32_t carry = first ? (st.text_open ? tail_c3(st) & VC_MASK : 0u) : ex.fb;
    validate = op == WSG_OP_TEXT || (op == WSG_OP_CONTINUATION && open);
    seam = validate && open;
    uint32_t status = 0;
    if (ex.sum + r.len > a.n_pieces * PIECE) status = WSG_E_BATCH;  // slots beyond the piece grid
    if (!status && seam) {
      const uint32_t nh = r.len < 3 ? r.len : 3u;
      const uint32_t f3 = nh ? plain_word(a, r.src) & (0xffffffu >> (8 * (3 - nh))) : 0u;
      if (seam_utf8_error(carry, f3, r.len, (r.code & CODE_FIN) != 0)) status = WSG_E_TEXT_UTF8;
    }
    validate = validate && !status;
    seam = seam && validate;
    a.vflag[k] = (uint8_t)((validate ? 1u : 0u) | (seam ? 2u : 0u));
    wsg_frame_desc d;
    d.payload_off = ex.sum;
    d.payload_len = r.len;
    d.opcode = (uint8_t)op;
    d.flags = (uint8_t)(((r.code & CODE_FIN) ? 0x80u : 0u) | (((r.code >> CODE_RSV_SHIFT) & 7u) << 4));
    d.status = (uint16_t)status;
    a.desc[k] = d;
    if (status) atomicMin((unsigned long long*)&a.sess_err[s], (unsigned long long)k);
    if (k + 1 == a.session_first[s + 1]) {  // the context after the session's last frame (k_final)
      const VAgg inc = agg_op(ex, v);      // (a CONST: v of a session's first frame is one)
      a.slink[a.n_sessions + s] = (int32_t)vopen(inc.fa);
      a.slink[2 * a.n_sessions + s] = (int32_t)inc.fb;
    }
  }
  write_pieces(a, live, k, r, ex.sum, validate, seam, lane);
}

// ------------------------------------------------------------------ k_pieces
// One wave per 1 KiB piece of the payload OUTPUT (16-B aligned frame slots laid
// end to end): lane i owns output bytes [1024p + 16i, +16).  The grid size is
// known on the host (piece_bound), every store is an aligned full-line store,
// and a wave's footprint is 1 KiB in and 1 KiB out — the streaming shape that
// reaches the chip's copy ceiling.  A piece inside one frame (the common case)
// reads 16-B ALIGNED source blocks and builds the misaligned payload bytes with
// a wave-shift DPP funnel; a piece spanning frame slots takes the general path.
__device__ __forceinline__ uint32_t dpp_from_next(uint32_t v, uint32_t old) {
  // lane i <- lane i+1 (wave_shl:1); lane 63 keeps `old`
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_from_prev(uint32_t v, uint32_t old) {
  // lane i <- lane i-1 (wave_shr:1); lane 0 keeps `old`
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}

__device__ __forceinline__ uint32_t keep_bytes(uint32_t w, int keep) {
  return keep >= 4 ? w : (keep <= 0 ? 0u : (w & ((1u << (8 * keep)) - 1u)));
}
__device__ __forceinline__ uint32_t keep_flags(int keep) {  // UTF-8 flag mask of the first `keep` bytes
  return keep >= 4 ? 0x80808080u : (keep <= 0 ? 0u : (0x80808080u >> (8 * (4 - keep))));
}

// The 3 payload bytes before position `keep` (1..16) of a lane's chunk w[0..3],
// pw = the 4 bytes before the chunk, in the edge layout (oldest byte in bits 0-7).
// The lane holding a frame's last byte tests them: the SWAR pair rule flags a lone
// invalid lead one byte late, so the frame's last byte is tested alone, and a FIN
// frame of >= 3 bytes must not end inside a sequence (FrameUtf8Validator.java:83-96).
__device__ __forceinline__ bool tail_error(uint32_t l3, bool fin) {
  return utf8_bad_last((l3 >> 16) & 0xffu) || (fin && utf8_incomplete(l3 & 0xffu, (l3 >> 8) & 0xffu, (l3 >> 16) & 0xffu));
}
__device__ __forceinline__ uint32_t last3(uint32_t pw, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int keep) {
  const int t = keep + 1;  // window (pw ++ w) index of the first of the 3 bytes
  const int q = t >> 2;
  const uint32_t lo = q == 0 ? pw : (q == 1 ? w0 : (q == 2 ? w1 : (q == 3 ? w2 : w3)));
  const uint32_t hi = q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : w3));
  return alignbyte(hi, lo, (uint32_t)t & 3u) & 0xffffffu;
}

// A piece found invalid UTF-8 in frame k (which passed every other rule: k_link
// validates no failed frame): FrameUtf8Validator's 1007 (FrameUtf8Validator.java:
// 54-57, 78-96) as the frame's status, and the session's first failing frame.
__device__ __forceinline__ void report_utf8(const DecodeArgs& a, uint32_t k) {
  a.desc[k].status = (uint16_t)WSG_E_TEXT_UTF8;
  atomicMin((unsigned long long*)&a.sess_err[a.rec[k].sess], (unsigned long long)k);
}

// 4 source bytes ending right before wire offset `pos`, unmasked (payload phase 0)
__device__ __forceinline__ uint32_t prev_word(const DecodeArgs& a, uint64_t pos, uint32_t mask) {
  uint32_t w = 0;
  for (int i = 0; i < 4; ++i) w |= (uint32_t)a.wire[pos - 4 + i] << (8 * i);
  return w ^ mask;
}

// Fast path: the piece is payload of ONE frame.  Every lane loads one 16-B
// ALIGNED source block; output dword j of lane i is bytes sh+4j.. of
// (block i ++ block i+1), the next block arriving by a wave-shift DPP move
// (block 64 by a scalar load).  Returns the lane's UTF-8 error flags.
template <int NT>
__device__ __forceinline__ uint32_t piece_fast(const DecodeArgs& a, const PieceDesc d, uint64_t pstart, int lane) {
  const uint32_t aux = (NT & 1) ? 2 : 0;  // NT bit 0: nontemporal; bit 2: validate only, no stores
  constexpr bool ST = !(NT & 4);
  const uint64_t s = d.info & PD_SRC_MASK;
  const uint32_t nb = (uint32_t)(d.info >> PD_NB_SHIFT) & 2047u;
  const uint64_t a16 = s & ~15ull;
  const uint32_t sh = (uint32_t)(s & 15u);
  const uint32_t boff = (uint32_t)lane * 16u;
  const __amdgpu_buffer_rsrc_t rout =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.payload_out + pstart), 0, (int)PIECE, 0x00020000);
  // the 4 payload bytes before the piece (UTF-8 carry from the previous piece of the
  // same frame): scalar loads issued up front, beside the payload load
  const uint32_t b = sh & 3u;
  const uint64_t pva = a16 >= 16u ? a16 - 16u : 0u;  // bytes a16-16 .. a16+15
  const uint32_t i0 = 3u + (sh >> 2);                 // dword holding byte (s - 4)
  // (kept in VGPRs: a readfirstlane here would force a wait before the payload load)
  const uint32_t pv_lo = ((const uint32_t*)(a.wire + pva))[i0];
  const uint32_t pv_hi = ((const uint32_t*)(a.wire + pva))[i0 + 1];
  u32x4 A;
  uint32_t e0, e1, e2, e3;
  if (a16 + PIECE + 16u <= a.wire_len) {  // wave-uniform: the usual case
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.wire + a16), 0, (int)(PIECE + 16u), 0x00020000);
    A = __builtin_amdgcn_raw_buffer_load_b128(rin, boff, 0, aux);
    const u32x4 nx = *(const u32x4*)(a.wire + a16 + PIECE);  // block 64 (lane 63's next block)
    e0 = nx.x; e1 = nx.y; e2 = nx.z; e3 = nx.w;
  } else {  // the wire's last KiB: byte loads (the buffer range check is per dword)
    uint32_t dd[4] = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < 16u; ++i)
      if (a16 + boff + i < a.wire_len) dd[i >> 2] |= (uint32_t)a.wire[a16 + boff + i] << (8 * (i & 3));
    A = (u32x4){dd[0], dd[1], dd[2], dd[3]};
    uint32_t ee[4] = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < 16u; ++i)
      if (a16 + PIECE + i < a.wire_len) ee[i >> 2] |= (uint32_t)a.wire[a16 + PIECE + i] << (8 * (i & 3));
    e0 = ee[0]; e1 = ee[1]; e2 = ee[2]; e3 = ee[3];
  }
  const uint32_t W0 = A.x, W1 = A.y, W2 = A.z, W3 = A.w;
  const uint32_t W4 = dpp_from_next(A.x, e0), W5 = dpp_from_next(A.y, e1);
  const uint32_t W6 = dpp_from_next(A.z, e2), W7 = dpp_from_next(A.w, e3);
  uint32_t w[4];
  switch (sh >> 2) {  // wave-uniform
    case 0: w[0] = alignbyte(W1, W0, b); w[1] = alignbyte(W2, W1, b); w[2] = alignbyte(W3, W2, b); w[3] = alignbyte(W4, W3, b); break;
    case 1: w[0] = alignbyte(W2, W1, b); w[1] = alignbyte(W3, W2, b); w[2] = alignbyte(W4, W3, b); w[3] = alignbyte(W5, W4, b); break;
    case 2: w[0] = alignbyte(W3, W2, b); w[1] = alignbyte(W4, W3, b); w[2] = alignbyte(W5, W4, b); w[3] = alignbyte(W6, W5, b); break;
    default: w[0] = alignbyte(W4, W3, b); w[1] = alignbyte(W5, W4, b); w[2] = alignbyte(W6, W5, b); w[3] = alignbyte(W7, W6, b); break;
  }
  const bool full = nb >= PIECE;        // wave-uniform: every lane holds 16 payload bytes
  const int keep = (int)nb - lane * 16;  // payload bytes in this lane's chunk
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] ^= d.mask;
  if (full) {
    if (ST) __builtin_amdgcn_raw_buffer_store_b128((u32x4){w[0], w[1], w[2], w[3]}, rout, boff, 0, aux);
  } else {  // the frame's last piece: zero the slot padding past the payload
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = keep_bytes(w[i], keep - 4 * i);
    if (ST && keep > 0) __builtin_amdgcn_raw_buffer_store_b128((u32x4){w[0], w[1], w[2], w[3]}, rout, boff, 0, aux);
  }
  if (!(d.info & PD_VALIDATE)) return 0u;
  const uint32_t first_prev = (d.info & PD_FIRST) ? 0u : (alignbyte(pv_hi, pv_lo, b) ^ d.mask);
  const uint32_t pw = dpp_from_prev(w[3], first_prev);
  uint32_t f0 = utf8_err_word_raw(w[0], pw), f1 = utf8_err_word_raw(w[1], w[0]);
  uint32_t f2 = utf8_err_word_raw(w[2], w[1]), f3 = utf8_err_word_raw(w[3], w[2]);
  // a continuation's bytes 0..2 are checked against the message carry (k_link); a
  // message start has no carry, and the zero word before it is exact
  const bool cont_head = lane == 0 && (d.info & PD_FIRST) && (d.frame & PDF_CONT);
  if (cont_head) f0 &= 0x80000000u;
  if (!full) {
    f0 &= keep_flags(keep); f1 &= keep_flags(keep - 4); f2 &= keep_flags(keep - 8); f3 &= keep_flags(keep - 12);
  }
  uint32_t te = 0;
  if ((d.info & PD_LAST) && keep >= 1 && keep <= 16) {
    const bool whole = !(cont_head && keep < 3);  // (a short continuation ends on the carry: k_link)
    te = tail_error(last3(pw, w[0], w[1], w[2], w[3], keep), whole && (d.info & PD_FIN)) ? 1u : 0u;
  }
  return ((f0 | f1 | f2 | f3) & H80) | te;
}


// General path: the piece spans several frame slots (small frames).  Each lane
// finds the frame owning its 16 output bytes by walking the records from the
// piece's first frame; the UTF-8 carry is taken per lane.
template <int NT>
__device__ __forceinline__ void piece_general(const DecodeArgs& a, const PieceDesc d, uint64_t pstart, uint64_t total,
                                              int lane) {
  const uint32_t aux = (NT & 1) ? 2 : 0;  // NT bit 0: nontemporal; bit 2: validate only, no stores
  constexpr bool ST = !(NT & 4);
  const __amdgpu_buffer_rsrc_t rout =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.payload_out + pstart), 0, (int)PIECE, 0x00020000);
  const uint64_t pend = pstart + PIECE < total ? pstart + PIECE : total;
  const uint64_t my = pstart + (uint64_t)lane * 16u;
  const bool live = my < pend;
  const uint32_t fr0 = d.frame & PDF_INDEX;
  uint32_t lk = fr0;  // frame owning this lane's 16 output bytes
  uint64_t lout;       // its slot (desc: k_link's payload_off / payload_len)
  uint32_t llen;
  {
    // lane-parallel lookup: lane l takes record d.frame + l and the 16-B chunk of the
    // piece where that frame's slot starts (0 for the piece's first frame, 64 past
    // the piece end); the chunks are non-decreasing over the lanes, so the owner of
    // chunk i is the last lane whose chunk is <= i: a 6-step search over shuffles
    const uint64_t fl = (uint64_t)fr0 + (uint64_t)lane;
    const bool have = fl < a.n_frames;
    wsg_frame_desc fd = {};
    if (have) fd = a.desc[fl];
    const uint64_t fs = have ? fd.payload_off : ~0ull;
    const uint64_t fslot = have ? (uint64_t)((fd.payload_len + 15u) & ~15u) : 0ull;
    if (__any(have && fslot && fs + fslot >= pend)) {  // the 64 records reach the piece end
      const int c = fs >= pend ? 64 : (fs <= pstart ? 0 : (int)((fs - pstart) >> 4));
      int pos = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1)
        if (__shfl(c, pos + step, 64) <= lane) pos += step;
      lk = fr0 + (uint32_t)pos;
      lout = (uint64_t)__shfl((int)(uint32_t)fs, pos, 64) | ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(fs >> 32), pos, 64) << 32);
      llen = (uint32_t)__shfl((int)fd.payload_len, pos, 64);
    } else {  // more than 64 frames (empty ones) in the piece: walk the records
      uint32_t kk = fr0;
      wsg_frame_desc rd = a.desc[kk];
      lout = rd.payload_off;
      llen = rd.payload_len;
      uint64_t send = rd.payload_off + ((rd.payload_len + 15u) & ~15u);
      for (;;) {
        const bool beyond = live && my >= send;
        if (!__any(beyond)) break;
        ++kk;
        rd = a.desc[kk];
        if (beyond) { lk = kk; lout = rd.payload_off; llen = rd.payload_len; }
        send = rd.payload_off + ((rd.payload_len + 15u) & ~15u);
      }
    }
  }
  const FrameRec lr = a.rec[lk];  // (src, mask, code: k_parse's record)
  const uint32_t j = (uint32_t)(my - lout);
  const int keep = live ? (int)llen - (int)j : 0;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  if (live) {
    const uint64_t s = lr.src + j;
    const uint64_t a4 = s & ~3ull;
    const uint32_t sh = (uint32_t)(s & 3u);
    uint32_t dd[5];
    if (a4 + 20u <= a.wire_len) {
      const uint32_t* q = (const uint32_t*)(a.wire + a4);
      dd[0] = q[0]; dd[1] = q[1]; dd[2] = q[2]; dd[3] = q[3]; dd[4] = q[4];
    } else {
      for (int i = 0; i < 5; ++i) dd[i] = 0u;
#pragma unroll
      for (uint32_t i = 0; i < 20u; ++i)  // constant indices: dd stays in registers
        if (a4 + i < a.wire_len) dd[i >> 2] |= (uint32_t)a.wire[a4 + i] << (8 * (i & 3));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = keep_bytes(alignbyte(dd[i + 1], dd[i], sh) ^ lr.mask, keep - 4 * i);
    if (ST) __builtin_amdgcn_raw_buffer_store_b128((u32x4){w[0], w[1], w[2], w[3]}, rout, (uint32_t)lane * 16u, 0, aux);
  }
  const bool lval = live && a.vflag[lk];
  if (__any(lval)) {
    uint32_t pw = dpp_from_prev(w[3], 0u);
    const uint32_t prev_k = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffffu, (int)lk, 0x138, 0xf, 0xf, false);
    if (j == 0) pw = 0u;
    else if (prev_k != lk) pw = prev_word(a, lr.src + j, lr.mask);  // lane 0 inside a frame
    if (lval) {
      const bool cont = (a.vflag[lk] & 2u) != 0;  // a seam frame: its head is k_link's
      uint32_t e0 = utf8_err_word_raw(w[0], pw), e1 = utf8_err_word_raw(w[1], w[0]);
      uint32_t e2 = utf8_err_word_raw(w[2], w[1]), e3 = utf8_err_word_raw(w[3], w[2]);
      if (j == 0 && cont) e0 &= 0x80000000u;  // a continuation's head: k_link
      e0 &= keep_flags(keep); e1 &= keep_flags(keep - 4); e2 &= keep_flags(keep - 8); e3 &= keep_flags(keep - 12);
      const bool te = keep >= 1 && keep <= 16 &&
                      tail_error(last3(pw, w[0], w[1], w[2], w[3], keep),
                                 (j + keep >= 3 || !cont) && (lr.code & CODE_FIN));
      if (e0 | e1 | e2 | e3 | (te ? 1u : 0u)) report_utf8(a, lk);
    }
  }
}

template <int NT, int WPB, int XCD>
__global__ __launch_bounds__(64 * WPB) void k_pieces(DecodeArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t blk = XCD ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint64_t p = (uint64_t)__builtin_amdgcn_readfirstlane(blk * (uint32_t)WPB + (threadIdx.x >> 6));
  const PieceDesc d = a.pieces[p];
  const uint64_t total = *a.total;
  // keep both scalar loads in flight together (the exit test below would
  // otherwise let the compiler wait for `total` before issuing the descriptor load)
  asm volatile("" ::"s"(d.info), "s"(d.mask), "s"(d.frame), "s"(total));
  const uint64_t pstart = p * PIECE;
  if (pstart >= total) return;
  if (!(d.info & PD_MULTI)) {
    const uint32_t err = piece_fast<NT>(a, d, pstart, lane);
    if (__any(err != 0) && lane == 0) report_utf8(a, d.frame & PDF_INDEX);
    return;
  }
  piece_general<NT>(a, d, pstart, total, lane);
}

// output dwords of a lane from its aligned source block (W0..W3) and the next
// lane's (W4..W7): bytes sh.. of the 32-byte window (sh wave-uniform)
__device__ __forceinline__ void funnel16(uint32_t sh, uint32_t W0, uint32_t W1, uint32_t W2, uint32_t W3, uint32_t W4,
                                         uint32_t W5, uint32_t W6, uint32_t W7, uint32_t w[4]) {
  const uint32_t b = sh & 3u;
  switch (sh >> 2) {
    case 0: w[0] = alignbyte(W1, W0, b); w[1] = alignbyte(W2, W1, b); w[2] = alignbyte(W3, W2, b); w[3] = alignbyte(W4, W3, b); break;
    case 1: w[0] = alignbyte(W2, W1, b); w[1] = alignbyte(W3, W2, b); w[2] = alignbyte(W4, W3, b); w[3] = alignbyte(W5, W4, b); break;
    case 2: w[0] = alignbyte(W3, W2, b); w[1] = alignbyte(W4, W3, b); w[2] = alignbyte(W5, W4, b); w[3] = alignbyte(W6, W5, b); break;
    default: w[0] = alignbyte(W4, W3, b); w[1] = alignbyte(W5, W4, b); w[2] = alignbyte(W6, W5, b); w[3] = alignbyte(W7, W6, b); break;
  }
}

// N consecutive pieces of one frame per wave (N KiB in flight per wave).  All
// but the last piece are full, so the source is contiguous: block 64 of piece i
// is lane 0's block of piece i+1 (readlane), the last piece's block 64 is one
// extra load, and the UTF-8 carry of piece i+1 is lane 63's last word of piece i.
template <int NT, int N>
__device__ __forceinline__ uint32_t piece_fastN(const DecodeArgs& a, const PieceDesc d, const uint64_t info_last,
                                                uint64_t pstart, int lane) {
  const uint32_t nb_last = (uint32_t)(info_last >> PD_NB_SHIFT) & 2047u;
  const uint32_t aux = (NT & 1) ? 2 : 0;  // NT bit 0: nontemporal; bit 2: validate only, no stores
  constexpr bool ST = !(NT & 4);
  const uint64_t s = d.info & PD_SRC_MASK;
  const uint64_t a16 = s & ~15ull;
  const uint32_t sh = (uint32_t)(s & 15u);
  const uint32_t boff = (uint32_t)lane * 16u;
  const __amdgpu_buffer_rsrc_t rout =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.payload_out + pstart), 0, (int)(N * PIECE), 0x00020000);
  const uint32_t b = sh & 3u;
  const uint64_t pva = a16 >= 16u ? a16 - 16u : 0u;
  const uint32_t i0 = 3u + (sh >> 2);
  const uint32_t pv_lo = ((const uint32_t*)(a.wire + pva))[i0];
  const uint32_t pv_hi = ((const uint32_t*)(a.wire + pva))[i0 + 1];
  u32x4 A[N];
  u32x4 nx;
  if (a16 + N * PIECE + 16u <= a.wire_len) {
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.wire + a16), 0, (int)(N * PIECE + 16u), 0x00020000);
#pragma unroll
    for (int i = 0; i < N; ++i) A[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, boff + i * PIECE, 0, aux);
    nx = *(const u32x4*)(a.wire + a16 + N * PIECE);
  } else {  // the wire's last bytes: byte loads (the buffer range check is per dword)
#pragma unroll
    for (int i = 0; i <= N; ++i) {
      uint32_t dd[4] = {0u, 0u, 0u, 0u};
      const uint64_t base = a16 + (uint64_t)i * PIECE + (i < N ? boff : 0u);
      for (uint32_t k = 0; k < 16u; ++k)
        if (base + k < a.wire_len) dd[k >> 2] |= (uint32_t)a.wire[base + k] << (8 * (k & 3));
      if (i < N) A[i] = (u32x4){dd[0], dd[1], dd[2], dd[3]};
      else nx = (u32x4){dd[0], dd[1], dd[2], dd[3]};
    }
  }
  uint32_t w[N][4];
  if (sh == 0) {  // wave-uniform: a 16-B aligned source (plain payload slots) needs no funnel
#pragma unroll
    for (int i = 0; i < N; ++i) {
      w[i][0] = A[i].x; w[i][1] = A[i].y; w[i][2] = A[i].z; w[i][3] = A[i].w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      u32x4 n;
      if (i + 1 < N) {
        n.x = (uint32_t)__builtin_amdgcn_readlane((int)A[i + 1].x, 0);
        n.y = (uint32_t)__builtin_amdgcn_readlane((int)A[i + 1].y, 0);
        n.z = (uint32_t)__builtin_amdgcn_readlane((int)A[i + 1].z, 0);
        n.w = (uint32_t)__builtin_amdgcn_readlane((int)A[i + 1].w, 0);
      } else {
        n = nx;
      }
      funnel16(sh, A[i].x, A[i].y, A[i].z, A[i].w, dpp_from_next(A[i].x, n.x), dpp_from_next(A[i].y, n.y),
               dpp_from_next(A[i].z, n.z), dpp_from_next(A[i].w, n.w), w[i]);
    }
  }
  if (ST) {  // (validate only: plain payloads, no mask)
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) w[i][k] ^= d.mask;
  }
  const bool full = nb_last >= PIECE;
  const int keep = (int)nb_last - lane * 16;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (!ST) continue;
    if (i + 1 < N || full) {
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){w[i][0], w[i][1], w[i][2], w[i][3]}, rout, boff + i * PIECE, 0,
                                             aux);
    } else {  // the frame's last piece: zero the slot padding past the payload
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = keep_bytes(w[i][k], keep - 4 * k);
      if (keep > 0) __builtin_amdgcn_raw_buffer_store_b128((u32x4){v[0], v[1], v[2], v[3]}, rout, boff + i * PIECE, 0, aux);
    }
  }
  if (!(d.info & PD_VALIDATE)) return 0u;
  uint32_t err = 0;
  uint32_t carry = (d.info & PD_FIRST) ? 0u : (alignbyte(pv_hi, pv_lo, b) ^ d.mask);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t pw = dpp_from_prev(w[i][3], carry);
    U8W up, u0, u1, u2, u3;
    u8w_one(pw, up);
    u8w_pair(w[i][0], w[i][1], u0, u1);
    u8w_pair(w[i][2], w[i][3], u2, u3);
    uint32_t f0 = u8w_err(u0, up), f1 = u8w_err(u1, u0), f2 = u8w_err(u2, u1), f3 = u8w_err(u3, u2);
    const bool cont_head = i == 0 && lane == 0 && (d.info & PD_FIRST) && (d.frame & PDF_CONT);
    if (cont_head) f0 &= 0x80000000u;  // a continuation's bytes 0..2: k_link
    if (i + 1 == N && !full) {
      f0 &= keep_flags(keep); f1 &= keep_flags(keep - 4); f2 &= keep_flags(keep - 8); f3 &= keep_flags(keep - 12);
    }
    if (i + 1 == N && (info_last & PD_LAST) && keep >= 1 && keep <= 16) {
      // (a frame of N > 1 pieces has >= 3 bytes; with N == 1 the piece may start it)
      const bool ge3 = N > 1 || !(lane == 0 && (d.info & PD_FIRST) && (d.frame & PDF_CONT) && keep < 3);
      if (tail_error(last3(pw, w[i][0], w[i][1], w[i][2], w[i][3], keep), ge3 && (info_last & PD_FIN))) err |= 1u;
    }
    err |= (f0 | f1 | f2 | f3) & H80;
    if (i + 1 < N) carry = (uint32_t)__builtin_amdgcn_readlane((int)w[i][3], 63);
  }
  return err;
}

template <int NT, int XCD, int N, int WPB = 1, int MINW = 1>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MINW))) void k_piecesN(DecodeArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t blk = XCD ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint64_t p = (uint64_t)N * (uint64_t)__builtin_amdgcn_readfirstlane(blk * (uint32_t)WPB + (threadIdx.x >> 6));
  if (WPB > 1 && p >= a.n_pieces) return;  // (a wave of the last workgroup past the grid)
  PieceDesc d[N];
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = a.pieces[p + i];
  const uint64_t total = *a.total;
  asm volatile("" ::"s"(d[0].info), "s"(d[0].mask), "s"(d[0].frame), "s"(d[N - 1].info), "s"(d[N - 1].frame),
               "s"(total));
  const uint64_t pstart = p * PIECE;
  if (pstart >= total) return;
  // fast: all N pieces exist and are payload of the same frame (then all but the last are full)
  bool fast = pstart + (uint64_t)(N - 1) * PIECE < total && d[0].frame == d[N - 1].frame;
#pragma unroll
  for (int i = 0; i < N; ++i) fast = fast && !(d[i].info & PD_MULTI);
  if (fast) {
    const uint32_t err = piece_fastN<NT, N>(a, d[0], d[N - 1].info, pstart, lane);
    if (__any(err != 0) && lane == 0) report_utf8(a, d[0].frame & PDF_INDEX);
    return;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t ps = pstart + (uint64_t)i * PIECE;
    if (ps >= total) return;
    if (!(d[i].info & PD_MULTI)) {
      const uint32_t err = piece_fast<NT>(a, d[i], ps, lane);
      if (__any(err != 0) && lane == 0) report_utf8(a, d[i].frame & PDF_INDEX);
    } else {
      piece_general<NT>(a, d[i], ps, total, lane);
    }
  }
}

// ------------------------------------------------------------------ k_final
__device__ int64_t error_detail(const DecodeArgs& a, uint64_t k, uint32_t err) {
  if (a.validator_only) return 0;  // (no wire headers: only the validator's 1007, which has no argument)
  const uint64_t o = a.frame_off[k];
  const uint32_t b0 = a.wire[o], b1 = a.wire[o + 1];
  switch (err) {
    case WSG_E_OPCODE: return b0 & 15;
    case WSG_E_RSV: return (b0 >> 4) & 7;
    case WSG_E_CONTROL_LEN:
    case WSG_E_CLOSE_LEN: return b1 & 0x7f;
    case WSG_E_TOO_LONG: return a.max_payload;
    case WSG_E_CLOSE_STATUS: {
      const FrameRec r = a.rec[k];
      const uint32_t s0 = a.wire[r.src] ^ (r.mask & 0xffu), s1 = a.wire[r.src + 1] ^ ((r.mask >> 8) & 0xffu);
      return (int64_t)((s0 << 8) | s1);
    }
    default: return 0;
  }
}

__global__ __launch_bounds__(256) void k_final(DecodeArgs a) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= a.n_sessions) return;
  wsg_session_state st = a.state[s];
  wsg_session_result res = {0u, 0u, 0u, 0};
  const uint32_t sf = a.session_first[s], se = a.session_first[s + 1];
  const uint64_t fe = a.sess_err[s];
  if (fe != ~0ull) a.sess_err[s] = ~0ull;  // back to the idle state for the next batch
  if (st.closed) {  // FrameDecoder.closed: all further input is swallowed (:185-187)
    a.result[s] = res;
    return;
  }
  if (fe != ~0ull) {
    const uint32_t err = a.desc[fe].status;
    res.n_delivered = (uint32_t)(fe - sf);
    res.error = (uint16_t)err;
    res.close_code = close_code_of(err);
    res.detail = error_detail(a, fe, err);
    st.closed = 1;
  } else {
    res.n_delivered = se - sf;
    if (se > sf && a.validator_only) {  // k_vlink: the validator context after the last frame
      const bool open = a.slink[a.n_sessions + s] != 0;
      const uint32_t c3 = (uint32_t)a.slink[2 * a.n_sessions + s];
      const uint32_t n = open ? (c3 >> 24) & 3u : 0u;
      for (uint32_t i = 0; i < n; ++i) st.tail[i] = (uint8_t)(c3 >> (24 - 8 * (n - i)));
      st.tail_len = (uint8_t)n;
      st.text_open = open;
    } else if (se > sf) {  // k_link's record of the session's last frame
      const int32_t ld = a.slink[s];                          // last data frame
      if (ld >= (int32_t)sf) {
        const bool frag = !(a.rec[ld].code & CODE_FIN);
        st.fragmentation = frag;
        bool text = false;
        if (a.validate && frag) {
          const int32_t ls = a.slink[a.n_sessions + s];         // last message start
          text = ls >= (int32_t)sf ? code_op(a.rec[ls].code) == WSG_OP_TEXT : (st.text_open != 0);
        }
        if (text) {  // tail = last <= 3 bytes of the open text message: the validator carry
          const uint32_t c3 = (uint32_t)a.slink[2 * a.n_sessions + s];
          const uint32_t n = (c3 >> 24) & 3u;
          for (uint32_t i = 0; i < n; ++i) st.tail[i] = (uint8_t)(c3 >> (24 - 8 * (n - i)));
          st.tail_len = (uint8_t)n;
        } else {
          st.tail_len = 0;
        }
        st.text_open = text;
      }
    }
  }
  a.state[s] = st;
  a.result[s] = res;
}

// ------------------------------------------------------------------ launchers
void launch_parse(const DecodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_parse, dim3(a.nblk), dim3(DBLOCK), 0, s, a);
}
void launch_scan(const DecodeArgs& a, hipStream_t s) {
  const dim3 g((a.nblk + SCAN_CHUNK - 1) / SCAN_CHUNK);
  if (a.validator_only) hipLaunchKernelGGL(k_scan<VAgg>, g, dim3(1024), 0, s, a);
  else hipLaunchKernelGGL(k_scan<DAgg>, g, dim3(1024), 0, s, a);
}
void launch_link(const DecodeArgs& a, hipStream_t s) {
  if (a.validator_only) hipLaunchKernelGGL(k_vlink, dim3(a.nblk), dim3(DBLOCK), 0, s, a);
  else hipLaunchKernelGGL(k_link, dim3(a.nblk), dim3(DBLOCK), 0, s, a);
}
#ifndef WSG_DWPB
#define WSG_DWPB 1  // waves a workgroup of the decode piece kernel (A/B build switch)
#endif
void launch_pieces(const DecodeArgs& a, hipStream_t s, uint64_t n_pieces_bound) {
  // one 64-lane workgroup per two pieces, nontemporal loads/stores, XCD-aware
  // (fastest in tools/ubench_unmask: 2 KiB in flight per wave)
  const uint64_t waves = (n_pieces_bound + PIECES_PER_WAVE - 1) / PIECES_PER_WAVE;
  hipLaunchKernelGGL((k_piecesN<1, 1, PIECES_PER_WAVE, WSG_DWPB>), dim3((uint32_t)((waves + WSG_DWPB - 1) / WSG_DWPB)),
                     dim3(64 * WSG_DWPB), 0, s, a);
}
void launch_vparse(const DecodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_vparse, dim3(a.nblk), dim3(DBLOCK), 0, s, a);
}
#ifndef WSG_VWPB
#define WSG_VWPB 1  // waves a workgroup of the validate-only piece kernel (A/B build switch)
#endif
#ifndef WSG_VMINW
#define WSG_VMINW 1  // its minimum waves a SIMD (a register budget: 8 -> 64 VGPRs; A/B build switch)
#endif
void launch_vpieces(const DecodeArgs& a, hipStream_t s, uint64_t n_pieces_bound) {
  // validate only: the piece kernel with its stores compiled out (NT bit 2)
  // (read-only streaming wants more bytes in flight per wave than the copy does:
  // VPIECES_PER_WAVE KiB)
  const uint64_t waves = (n_pieces_bound + VPIECES_PER_WAVE - 1) / VPIECES_PER_WAVE;
  hipLaunchKernelGGL((k_piecesN<5, 1, VPIECES_PER_WAVE, WSG_VWPB, WSG_VMINW>), dim3((uint32_t)((waves + WSG_VWPB - 1) / WSG_VWPB)),
                     dim3(64 * WSG_VWPB), 0, s, a);
}
void launch_final(const DecodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_final, dim3((a.n_sessions + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace ws
