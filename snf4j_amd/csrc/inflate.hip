// inflate.hip — permessage-deflate decode on gfx950: PerMessageDeflateDecoder
// (PerMessageDeflateDecoder.java:68-105) over DeflateDecoder (DeflateDecoder.java:
// 78-141) over a raw ZlibDecoder (ZlibDecoder.java:180-280, java.util.zip.Inflater,
// i.e. zlib's inflate, RFC 1951).
//
// DEFLATE is a serial bit stream per session (Huffman codes, back-references into
// a 32 KiB window that persists across messages unless no_context), so the unit
// of parallelism is the session: one 64-lane workgroup per session, the sessions
// of a batch in parallel.  The decoder itself is wave-uniform code (its registers
// live in SGPRs, every LDS value it reads is made uniform with readfirstlane); the
// lanes split the work that is wide: staging the input from HBM in aligned 16-byte
// loads, building the Huffman lookup tables (one symbol per lane, ranks by ballot),
// back-reference and stored-block copies, flushing output from the LDS window ring
// to HBM in dwords, and the window carry.
//
// Decoding is table driven: a 9-bit root table for literal/length codes and an 8-bit
// one for distances (longer codes, rare, fall back to a canonical walk), a 64-bit
// bit buffer refilled 8 bytes at a time while at least 8 input bytes of the frame
// remain, and the lazy byte-at-a-time path of zlib's inflate() for a frame's last
// bytes, so that symbol completion at frame ends is zlib's exactly.
//
// zlib semantics the reference depends on, reproduced exactly:
//   * a symbol completes (and its output belongs to the frame) when its last bit's
//     byte has been supplied; a frame's inflate call decodes as far as its bytes
//     allow (Java's Inflater loop until needsInput, ZlibDecoder.java:223-241), the
//     tail 00 00 FF FF of a final fragment is fed in the same call
//     (DeflateDecoder.java:96-99);
//   * the error checks of zlib's inflate/inflate_table at the same bits: invalid
//     block type, stored lengths, too many length/distance symbols, over-subscribed
//     or incomplete code sets (an incomplete set is allowed only for a single
//     1-bit code of the literal/length or distance table), bit-length repeat
//     errors, missing end-of-block, invalid literal/length and distance codes
//     (286/287, 30/31), distance too far back; all map to one exception
//     (DecompressionException, ZlibDecoder.java:255-257);
//   * a final block ends the stream: the rest of the frame and every later frame
//     pass through unchanged (ZlibDecoder.java:186-191, 262-270);
//   * a frame that produces no bytes fails unless its payload is the single byte
//     00 (DeflateDecoder.java:122-131).
#include "wsgpu_internal.h"
#include "wsgpu_scan.h"

namespace ws {

namespace {

constexpr uint32_t WMASK = WSG_INFLATE_WINDOW - 1;
constexpr uint32_t IB = 2048;        // input stage bytes
constexpr int LROOT = 9, DROOT = 8, CROOT = 7;
constexpr int32_t FLUSH_AT = 8192;   // ring bytes held back before a flush to HBM
// positions are 32-bit: a session's output per batch is capped below 2 GiB (else CAP)
constexpr int32_t POS_LIMIT = 0x7fff0000;

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                       33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum Mode : int { M_HEAD = 0, M_STORED, M_COPY, M_TABLE, M_LENLENS, M_CODELENS, M_LEN, M_LENEXT, M_DIST, M_DISTEXT, M_DONE };

enum Err : int { E_NONE = 0, E_DATA = 1, E_NODATA = 2, E_CAP = 3 };

// Table entry: [0,4) code length, [4,8) extra bits, [8,11) op, [16,32) value.
enum Op : uint32_t { OP_LIT = 0, OP_BASE = 1, OP_EOB = 2, OP_BAD = 3, OP_LONG = 4 };
enum Kind : int { T_LIT = 0, T_DIST = 1, T_CODES = 2 };

__device__ __forceinline__ uint32_t ent(uint32_t len, uint32_t extra, uint32_t op, uint32_t val) {
  return len | (extra << 4) | (op << 8) | (val << 16);
}
__device__ __forceinline__ uint32_t e_len(uint32_t e) { return e & 15u; }
__device__ __forceinline__ uint32_t e_extra(uint32_t e) { return (e >> 4) & 15u; }
__device__ __forceinline__ uint32_t e_op(uint32_t e) { return (e >> 8) & 7u; }
__device__ __forceinline__ uint32_t e_val(uint32_t e) { return e >> 16; }

// What symbol s of a table decodes to (zlib's inflate_table base/extra arrays: 286/287
// and 30/31 are codes that decode as invalid).
__device__ __forceinline__ uint32_t sym_entry(int kind, uint32_t s, uint32_t len) {
  if (kind == T_CODES) return ent(len, 0, OP_LIT, s);
  if (kind == T_DIST) return s < 30 ? ent(len, kDistExt[s], OP_BASE, kDistBase[s]) : ent(len, 0, OP_BAD, 0);
  if (s < 256) return ent(len, 0, OP_LIT, s);
  if (s == 256) return ent(len, 0, OP_EOB, 0);
  if (s < 286) return ent(len, kLenExt[s - 257], OP_BASE, kLenBase[s - 257]);
  return ent(len, 0, OP_BAD, 0);
}

// The lane decoders' entry tables hold the length and distance symbols only (a literal's
// entry is its byte): ents[0, 32) length symbols 256..287, ents[32, 64) distance 0..31.
constexpr int N_ENTS = 64;
__device__ __forceinline__ uint32_t ents_init(uint32_t i) {
  return i < 32u ? sym_entry(T_LIT, 256u + i, 0) : sym_entry(T_DIST, i - 32u, 0);
}
__device__ __forceinline__ uint32_t tok_ent(const uint32_t* ents, uint32_t sym, bool dist) {
  const uint32_t e = ents[(sym + (dist ? 32u : 0u - 256u)) & 63u];
  return (!dist && sym < 256u) ? ent(0, 0, OP_LIT, sym) : e;
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) { return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x); }

// Canonical code arrays (count per length, symbols in code order) for codes longer
// than the root table.
template <int N>
struct Huff {
  uint16_t cnt[16];
  uint16_t sym[N];
};

struct alignas(16) Lds {
  uint8_t ring[WSG_INFLATE_WINDOW];  // the inflate window / output stage (a ring image)
  uint8_t ibuf[IB + 16];             // input stage
  uint32_t lroot[1 << LROOT];        // literal/length root table (the code-length table in a header)
  uint32_t droot[1 << DROOT];        // distance root table
  Huff<288> lit;
  Huff<32> dist;
  uint8_t lens[320];
};

// Build the root table (and the canonical arrays) of the n code lengths lens[0..n):
// every lane takes symbols, ranks among equal lengths come from ballots.  Returns
// the longest length (0: no codes — every entry is an invalid 1-bit code) or -1 for
// a set zlib's inflate_table rejects: over-subscribed, or incomplete unless a single
// 1-bit code of a literal/length or distance table.
template <int N>
__device__ int build_tab(uint32_t* root, int rbits, Huff<N>* h, const uint8_t* lens, int n, int kind, int lane) {
  int cnt[16];
#pragma unroll
  for (int l = 0; l < 16; ++l) cnt[l] = 0;
  for (int b = 0; b < n; b += 64) {
    const int s = b + lane;
    const int l = s < n ? lens[s] : 0;
#pragma unroll
    for (int L = 1; L < 16; ++L) cnt[L] += __popcll(__ballot(l == L));
  }
  int maxl = 0;
#pragma unroll
  for (int L = 1; L < 16; ++L)
    if (cnt[L]) maxl = L;
  const uint32_t rsize = 1u << rbits;
  if (maxl == 0) {  // zlib: a table of invalid 1-bit entries (only a distance table gets here)
    for (uint32_t i = lane; i < rsize; i += 64) root[i] = ent(1, 0, OP_BAD, 0);
    return 0;
  }
  int left = 1;
#pragma unroll
  for (int L = 1; L < 16; ++L) {
    left = (left << 1) - cnt[L];
    if (left < 0) return -1;  // over-subscribed
  }
  if (left > 0 && (kind == T_CODES || maxl != 1)) return -1;  // incomplete
  int first[16], offs[16];
  {
    int code = 0, off = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
      code = (code + cnt[L - 1]) << 1;
      first[L] = code;
      offs[L] = off;
      off += cnt[L];
    }
  }
  if (h) {
    int v = 0;
#pragma unroll
    for (int L = 0; L < 16; ++L)
      if (lane == L) v = cnt[L];
    if (lane < 16) h->cnt[lane] = (uint16_t)v;
  }
  if (left > 0)  // the single-code case: the other half of the table is invalid (1 bit)
    for (uint32_t i = lane; i < rsize; i += 64) root[i] = ent(1, 0, OP_BAD, 0);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int seen[16];
#pragma unroll
  for (int L = 0; L < 16; ++L) seen[L] = 0;
  for (int b = 0; b < n; b += 64) {
    const int s = b + lane;
    const int l = s < n ? lens[s] : 0;
    int rank = 0, fc = 0, of = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
      const uint64_t m = __ballot(l == L);
      if (l == L) {
        rank = seen[L] + __popcll(m & below);
        fc = first[L];
        of = offs[L];
      }
      seen[L] += __popcll(m);
    }
    if (l) {
      if (h) h->sym[of + rank] = (uint16_t)s;
      const uint32_t code = (uint32_t)(fc + rank);
      const uint32_t rev = __builtin_bitreverse32(code) >> (32 - l);
      if (l <= rbits) {
        const uint32_t e = sym_entry(kind, (uint32_t)s, (uint32_t)l);
        for (uint32_t j = rev; j < rsize; j += (1u << l)) root[j] = e;
      } else {
        root[rev & (rsize - 1)] = ent(0, 0, OP_LONG, 0);
      }
    }
  }
  return maxl;
}

// Canonical walk for a code longer than the root table: >= 0 the symbol (*nb its
// length), -1 more bits needed.  Only complete codes reach here.
template <int N>
__device__ __forceinline__ int canon(const Huff<N>& h, int maxl, uint64_t hold, int bits, int* nb) {
  int code = 0, first = 0, index = 0;
  for (int len = 1; len <= maxl; ++len) {
    if (len > bits) return -1;
    code |= (int)((hold >> (len - 1)) & 1u);
    const int count = (int)uni(h.cnt[len]);
    if (code - count < first) {
      *nb = len;
      return (int)uni(h.sym[index + (code - first)]);
    }
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  *nb = maxl;
  return -1;
}

// Table decode from the low `bits` bits of hold (bits above them zero or the stream's
// own next bits): true with the entry when its code is complete.
template <int N>
__device__ __forceinline__ bool tdec(const uint32_t* root, int rbits, const Huff<N>* h, int maxl, int kind,
                                     uint64_t hold, int bits, uint32_t* e) {
  uint32_t x = uni(root[(uint32_t)hold & ((1u << rbits) - 1u)]);
  if (e_op(x) == OP_LONG) {
    int nb = 0;
    const int s = canon(*h, maxl, hold, bits, &nb);
    if (s < 0) return false;
    x = sym_entry(kind, (uint32_t)s, (uint32_t)nb);
  } else if ((int)e_len(x) > bits) {
    return false;
  }
  *e = x;
  return true;
}

}  // namespace

namespace {

constexpr uint32_t TOK_SLACK = 80;  // per-frame slack of the token / literal regions

// ---------------------------------------------------------------------------------
// Message-parallel pre-decode (k_infl_tok).  permessage-deflate ends every message
// with a sync flush (the stripped 00 00 FF FF), so a message that is one FIN frame
// starts a new block on a byte boundary with an empty bit buffer: its Huffman decode
// does not depend on anything before it.  One LANE per such frame decodes the frame
// (payload + tail) into a token stream: literal runs (bytes in a side stream) and
// (length, distance) pairs.  k_inflate then replays the tokens into its window ring
// instead of decoding, when its own state at that frame is the clean one the lane
// assumed; back-reference bounds are checked there, against the real history.  A
// frame the lane cannot finish cleanly (a final block, data errors, input ending
// inside a block, an incomplete code set, token space exhausted) is marked not ok
// and k_inflate decodes it itself: the serial decoder stays the authority.
// ---------------------------------------------------------------------------------

// Phase clocks for tools/prof_inflate.hip and tools/prof_infl_tok.hip (compiled out of the library).
#ifdef WSG_INFLATE_PROF
__device__ unsigned long long g_infl_prof[24];
#define PROF_T(v) const uint64_t v = clock64()
#define PROF_ACC(i, v) pf_[i] += clock64() - (v)
#define PROF_CNT(i, n) pf_[i] += (uint64_t)(n)
#else
#define PROF_T(v)
#define PROF_ACC(i, v)
#define PROF_CNT(i, n)
#endif
#ifdef WSG_INFLATE_TOK_PROF
__device__ unsigned long long g_fast_prof[8];
#define FPROF_T(v) const uint64_t v = clock64()
#define FPROF_ACC(i, v) if (threadIdx.x == 0) atomicAdd(&g_fast_prof[i], (unsigned long long)(clock64() - (v)))
#else
#define FPROF_T(v)
#define FPROF_ACC(i, v)
#endif
#ifdef WSG_INFLATE_TOK_PROF
__device__ unsigned long long g_tok_prof[8];
#define TPROF_T(v) const uint64_t v = clock64()
#define TPROF_ACC(i, v) pf_[i] += clock64() - (v)
#define TPROF_CNT(i, n) pf_[i] += (uint64_t)(n)
#else
#define TPROF_T(v)
#define TPROF_ACC(i, v)
#define TPROF_CNT(i, n)
#endif

// per-lane tables in HBM scratch.  Two levels: a root entry is len | symbol << 4 for a
// code of at most rbits bits; for a longer code it points at a sub-table after the
// root (len 0 | sub-table bits << 4 | offset << 7), indexed by the code's next bits, whose
// entries carry the full length.  Any symbol is two dependent loads at most (a walk
// of the canonical counts costs one load per code bit, and the wave waits for its
// slowest lane).
constexpr int LSUB = 340;  // zlib's bound for 286 codes of <= 15 bits over a 9-bit root (852 - 512)
constexpr int DSUB = 256;  // a distance set needing more goes to the serial decoder
struct LaneTab {
  uint16_t lroot[(1 << LROOT) + LSUB];
  uint16_t droot[(1 << DROOT) + DSUB];
  uint16_t croot[1 << CROOT];
  uint16_t sym[288];  // symbols in canonical order (table build)
  uint8_t lens[320];
};

// A lane's input: the frame's payload through a 16-B block held in registers, then the tail.
struct Src {
  const uint8_t* pay;    // batch payload
  uint64_t pay_len;
  uint64_t off;          // the frame's payload offset
  uint32_t plen;
  int64_t cq;
  uint4 blk;
  __device__ uint4 ld(int64_t q) const {
    if ((uint64_t)q * 16 + 16 <= pay_len) return reinterpret_cast<const uint4*>(pay)[q];
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (int t = 0; t < 16; ++t)
      if ((uint64_t)q * 16 + t < pay_len) w[t >> 2] |= (uint32_t)pay[(uint64_t)q * 16 + t] << (8 * (t & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

// Canonical two-level table of lens[0..n) (rbits root bits, at most sub entries after
// the root): the longest length, or -1 for any set that is not complete (over-subscribed,
// incomplete, empty) or that needs more sub-table room: the serial decoder then takes
// the frame and applies zlib's exact rules.  Sub-tables are sized as zlib's
// inflate_table sizes them: grown while the codes left at the next length do not fill it.
__device__ int lane_build(uint16_t* root, int rbits, int sub, uint16_t* sym, const uint8_t* lens, int n) {
  // counts and running offsets live in registers (a select chain per symbol): a
  // read-modify-write of counters in HBM scratch would chain every symbol on its latency
  int c[16];
#pragma unroll
  for (int l = 0; l < 16; ++l) c[l] = 0;
  for (int s = 0; s < n; ++s) {
    const int l = lens[s];
#pragma unroll
    for (int L = 1; L < 16; ++L) c[L] += (l == L) ? 1 : 0;
  }
  int left = 1, maxl = 0;
  bool bad = false;
#pragma unroll
  for (int l = 1; l < 16; ++l) {
    left = (left << 1) - c[l];
    bad |= left < 0;
    if (c[l]) maxl = l;
  }
  if (bad || left != 0 || maxl == 0) return -1;
  int o[16];
  {
    int off = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) {
      o[l] = off;
      off += c[l];
    }
  }
  for (int s = 0; s < n; ++s) {
    const int l = lens[s];
    if (!l) continue;
    int at = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L)
      if (l == L) at = o[L]++;
    sym[at] = (uint16_t)s;
  }
  const uint32_t rsize = 1u << rbits;
  uint32_t code = 0, pfx = 0xffffffffu, next = rsize, sbase = 0, sbits = 0;
  int idx = 0;
  for (int l = 1; l <= maxl; ++l) {
    int cl = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L)
      if (l == L) cl = c[L];
    for (int i = 0; i < cl; ++i, ++idx, ++code) {
      const uint32_t sy = sym[idx];
      const uint32_t rev = __builtin_bitreverse32(code) >> (32 - l);
      const uint16_t e = (uint16_t)((uint32_t)l | (sy << 4));
      if (l <= rbits) {
        for (uint32_t j = rev; j < rsize; j += (1u << l)) root[j] = e;
      } else {
        if ((rev & (rsize - 1u)) != pfx) {  // a new root prefix: its sub-table
          pfx = rev & (rsize - 1u);
          // c[] holds the codes not yet placed at each length (this one included)
          int curr = l - rbits, room = 1 << curr;
          while (curr + rbits < maxl) {
            int cn = 0;
#pragma unroll
            for (int L = 1; L < 16; ++L)
              if (curr + rbits == L) cn = c[L];
            room -= cn;
            if (room <= 0) break;
            ++curr;
            room <<= 1;
          }
          if (next + (1u << curr) > rsize + (uint32_t)sub) return -1;
          sbase = next;
          sbits = (uint32_t)curr;
          next += 1u << curr;
          root[pfx] = (uint16_t)((sbits << 4) | ((sbase - rsize) << 7));
        }
        for (uint32_t j = rev >> rbits; j < (1u << sbits); j += 1u << (l - rbits)) root[sbase + j] = e;
      }
#pragma unroll
      for (int L = 1; L < 16; ++L)
        if (l == L) --c[L];
    }
    code <<= 1;
  }
  return maxl;
}

// The symbol at the bit buffer: the table entry, or OP_BAD with len 0 when the code
// runs past the bits held (the rest of the input: a complete set fills every slot).
__device__ __forceinline__ uint32_t lane_sym(const uint16_t* root, int rbits, const uint32_t* ents, uint64_t hold,
                                             int bits) {
  uint32_t r = root[(uint32_t)hold & ((1u << rbits) - 1u)];
  if ((r & 15u) == 0)
    r = root[(1u << rbits) + (r >> 7) + ((uint32_t)(hold >> rbits) & ((1u << ((r >> 4) & 7u)) - 1u))];
  const uint32_t len = r & 15u, sy = r >> 4;
  if ((int)len > bits) return ent(0, 0, OP_BAD, 0);
  return ents ? (ents[sy] | len) : ent(len, 0, OP_LIT, sy);
}


__device__ __forceinline__ uint64_t tok_base(uint64_t po, uint64_t k) { return po + (uint64_t)TOK_SLACK * k; }
__device__ __forceinline__ uint64_t lit_base(uint64_t po, uint64_t k) {
  return (3 * po + (uint64_t)TOK_SLACK * k + 3) & ~(uint64_t)3;
}
__device__ __forceinline__ uint32_t lit_cap_of(uint32_t plen) { return 3u * (plen + 4u) + 60u; }

// One message's pre-decode into per-frame token regions (MULTI: several frames; the
// single-frame instantiation keeps the segment and attribution steps out of its loop).
template <bool MULTI>
__device__ __forceinline__ void tok_message(const InflArgs& a, LaneTab* T, const uint32_t* lit_ent,
                                            uint64_t k, uint64_t kend, uint32_t in_len, uint64_t* pf_) {
  (void)pf_;
  TPROF_T(t_msg);
  const wsg_frame_desc d = a.desc[k];
  // the next data frame of the message after j (j < kend)
  auto next_frame = [&](uint64_t j) -> uint64_t {
    for (++j; j < kend; ++j)
      if ((a.desc[j].opcode & 15u) < 8u) break;
    return j;
  };
  const uint32_t total = in_len + 4u;
  constexpr bool multi = MULTI;
  // input reader: segment = a frame's payload, message offsets [seg_lo, seg_lo + seg_len)
  uint64_t seg_k = k, seg_off = d.payload_off;
  uint32_t seg_lo = 0, seg_len = d.payload_len;
  Src src{a.payload, a.payload_len, d.payload_off, d.payload_len, -1, make_uint4(0, 0, 0, 0)};
  // output attribution: the frame whose bytes complete a symbol (zlib: a symbol belongs
  // to the inflate call that supplies its last bit's byte), per-frame token regions
  uint64_t fa = k;
  uint32_t fa_hi = k == kend ? total : d.payload_len;  // message offset where frame fa's bytes end
  uint32_t tok_cap = d.payload_len + 68u, lit_cap = lit_cap_of(d.payload_len);
  uint32_t* tok = a.tok + tok_base(d.payload_off, k);
  uint8_t* lit = a.lit + lit_base(d.payload_off, k);
  uint64_t hold = 0;
  int bits = 0;
  uint32_t ip = 0, ntok = 0, nlit = 0, run = 0, outlen = 0, litw = 0;
  bool ok = true;
  // The bit buffer is refilled with up to 8 bytes at once from a 32-byte window of
  // two 16-B blocks held in registers (one funnel shift, no per-byte branches); the
  // window moves on by one block when the lane leaves the first one.
  int64_t wq = (int64_t)(seg_off >> 4);
  uint4 wc = src.ld(wq), wn = src.ld(wq + 1);
  auto refill = [&]() {
    if (bits > 56 || ip >= total) return;
    while (multi && seg_k != kend && ip == seg_lo + seg_len) {  // on to the next frame's payload
      seg_lo += seg_len;
      seg_k = next_frame(seg_k);
      const wsg_frame_desc dn = a.desc[seg_k];
      seg_off = dn.payload_off;
      seg_len = dn.payload_len;
      wq = (int64_t)(seg_off >> 4);
      wc = src.ld(wq);
      wn = src.ld(wq + 1);
    }
    const uint64_t g = seg_off + (ip - seg_lo);  // payload address of input byte ip
    const uint32_t o = (uint32_t)(g & 15u);
    const uint32_t q = o >> 2, sh = o & 3u;
    const uint32_t D0 = wc.x, D1 = wc.y, D2 = wc.z, D3 = wc.w, D4 = wn.x, D5 = wn.y;
    const uint32_t A = q == 0 ? D0 : q == 1 ? D1 : q == 2 ? D2 : D3;
    const uint32_t B = q == 0 ? D1 : q == 1 ? D2 : q == 2 ? D3 : D4;
    const uint32_t C = q == 0 ? D2 : q == 1 ? D3 : q == 2 ? D4 : D5;
    const uint32_t lo = __builtin_amdgcn_alignbyte(B, A, sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(C, B, sh);
    uint64_t v = ((uint64_t)hi << 32) | lo;
    const int32_t k0 = (int32_t)(seg_lo + seg_len) - (int32_t)ip;  // bytes left in this segment
    uint32_t nb = (uint32_t)(64 - bits) >> 3;
    if (seg_k == kend) {
      // the last segment: the tail 00 00 FF FF from its end on (DeflateCodec TAIL)
      if (k0 < 8) {
        const uint64_t tail = 0xFFFF0000ull;
        v = k0 > 0 ? ((v & ((1ull << (8 * k0)) - 1ull)) | (tail << (8 * k0))) : (tail >> (8 * (-k0 < 8 ? -k0 : 7)));
      }
      if (nb > total - ip) nb = total - ip;
    } else if (nb > (uint32_t)k0) {
      nb = (uint32_t)k0;  // a segment's bytes only: the next one is elsewhere
    }
    if (nb < 8) v &= (1ull << (8 * nb)) - 1ull;
    hold |= v << bits;
    bits += 8 * (int)nb;
    ip += nb;
    if ((int64_t)((seg_off + (ip - seg_lo)) >> 4) > wq) {
      ++wq;
      wc = wn;
      wn = src.ld(wq + 1);
    }
  };
  auto drop = [&](int n) {
    hold >>= n;
    bits -= n;
  };
  auto put_lit = [&](uint32_t b) -> bool {
    if (nlit >= lit_cap) return false;
    litw |= b << (8 * (nlit & 3u));
    if ((++nlit & 3u) == 0) {
      reinterpret_cast<uint32_t*>(lit)[(nlit >> 2) - 1] = litw;
      litw = 0;
    }
    ++run;
    ++outlen;
    return true;
  };
  auto put_tok = [&](uint32_t t) -> bool {
    if (ntok >= tok_cap) return false;
    tok[ntok++] = t;
    return true;
  };
  auto end_run = [&]() -> bool {
    if (!run) return true;
    const bool r = put_tok(run);
    run = 0;
    return r;
  };
  // close frame fa (its stats), open the next data frame's regions
  auto close_frame = [&]() -> bool {
    if (!end_run()) return false;
    if (nlit & 3u) reinterpret_cast<uint32_t*>(lit)[nlit >> 2] = litw;
    a.tstat[fa] = InflTokStat{1u, ntok, nlit, outlen};
    if (fa == kend) return true;
    const uint32_t lo = fa_hi;
    fa = next_frame(fa);
    const wsg_frame_desc df = a.desc[fa];
    fa_hi = fa == kend ? total : lo + df.payload_len;
    tok_cap = df.payload_len + 68u;
    lit_cap = lit_cap_of(df.payload_len);
    tok = a.tok + tok_base(df.payload_off, fa);
    lit = a.lit + lit_base(df.payload_off, fa);
    ntok = nlit = run = outlen = litw = 0;
    return true;
  };
  // a symbol just completed: its last bit's byte decides its frame
  auto attrib = [&]() -> bool {
    if (!multi) return true;
    const uint32_t lb = (8u * ip - (uint32_t)bits - 1u) >> 3;
    while (lb >= fa_hi && fa != kend)
      if (!close_frame()) return false;
    return true;
  };
  for (;;) {
    refill();
    if (bits == 0 && ip >= total) break;  // clean: all input used, on a block boundary
    if (bits < 3) { ok = false; break; }
    const uint32_t last = (uint32_t)(hold & 1u), type = (uint32_t)((hold >> 1) & 3u);
    drop(3);
    if (last) { ok = false; break; }      // a final block: the stream ends (k_inflate handles it)
    if (type == 0) {                      // stored
      drop(bits & 7);
      refill();
      if (bits < 32) { ok = false; break; }
      const uint32_t ln = (uint32_t)(hold & 0xffffu), nl = (uint32_t)((hold >> 16) & 0xffffu);
      if (ln != (nl ^ 0xffffu)) { ok = false; break; }
      drop(32);
      for (uint32_t i = 0; i < ln && ok; ++i) {
        refill();
        if (bits < 8) { ok = false; break; }
        const uint32_t b = (uint32_t)(hold & 0xffu);
        drop(8);
        ok = attrib() && put_lit(b);
      }
      if (!ok) break;
      continue;
    }
    int lmax, dmax;
    TPROF_CNT(5, 1);
    TPROF_T(t_hdr);
    if (type == 1) {  // fixed codes
      for (int i = 0; i < 288; ++i) T->lens[i] = i < 144 ? 8 : (i < 256 ? 9 : (i < 280 ? 7 : 8));
      lmax = lane_build(T->lroot, LROOT, LSUB, T->sym, T->lens, 288);
      for (int i = 0; i < 30; ++i) T->lens[i] = 5;
      // zlib's fixed distance set has 30 codes of 5 bits + the 2 invalid ones: complete with 32
      T->lens[30] = 5;
      T->lens[31] = 5;
      dmax = lane_build(T->droot, DROOT, DSUB, T->sym, T->lens, 32);
    } else if (type == 2) {  // dynamic codes
      refill();
      if (bits < 14) { ok = false; break; }
      const int nlen = (int)(hold & 31u) + 257, ndist = (int)((hold >> 5) & 31u) + 1,
                ncode = (int)((hold >> 10) & 15u) + 4;
      drop(14);
      if (nlen > 286 || ndist > 30) { ok = false; break; }
      for (int i = 0; i < 19; ++i) T->lens[kClenOrder[i]] = 0;
      for (int i = 0; i < ncode; ++i) {
        refill();
        if (bits < 3) { ok = false; break; }
        T->lens[kClenOrder[i]] = (uint8_t)(hold & 7u);
        drop(3);
      }
      if (!ok) break;
      const int cmax = lane_build(T->croot, CROOT, 0, T->sym, T->lens, 19);
      if (cmax < 0) { ok = false; break; }
      int have = 0;
      while (have < nlen + ndist) {
        refill();
        const uint32_t e = lane_sym(T->croot, CROOT, nullptr, hold, bits);
        const int nb = (int)e_len(e);
        if (nb == 0 || nb > bits) { ok = false; break; }
        const int sy = (int)e_val(e);
        if (sy < 16) {
          drop(nb);
          T->lens[have++] = (uint8_t)sy;
          continue;
        }
        const int xb = sy == 16 ? 2 : (sy == 17 ? 3 : 7);
        if (nb + xb > bits) { ok = false; break; }
        drop(nb);
        int len = 0, copy;
        if (sy == 16) {
          if (have == 0) { ok = false; break; }
          len = T->lens[have - 1];
          copy = 3 + (int)(hold & 3u);
        } else if (sy == 17) {
          copy = 3 + (int)(hold & 7u);
        } else {
          copy = 11 + (int)(hold & 127u);
        }
        drop(xb);
        if (have + copy > nlen + ndist) { ok = false; break; }
        for (int i = 0; i < copy; ++i) T->lens[have + i] = (uint8_t)len;
        have += copy;
      }
      if (!ok) break;
      if (T->lens[256] == 0) { ok = false; break; }
      TPROF_T(t_bld);
      lmax = lane_build(T->lroot, LROOT, LSUB, T->sym, T->lens, nlen);
      // the distance lengths follow the literal/length ones in lens[]: move them first
      for (int i = 0; i < ndist; ++i) T->lens[i] = T->lens[nlen + i];
      dmax = lane_build(T->droot, DROOT, DSUB, T->sym, T->lens, ndist);
      TPROF_ACC(2, t_bld);
    } else {
      ok = false;
      break;
    }
    TPROF_ACC(1, t_hdr);
    if (lmax < 0 || dmax < 0) { ok = false; break; }
    TPROF_T(t_sym);
    // the block's symbols, one code a step: a literal/length code, or the distance code
    // of the length before it.  One lookup path for both keeps the 64 lanes in step (a
    // length and its distance as one step runs both paths on every step, as some lane
    // of 64 almost always has a match).
    uint32_t mlen = 0;  // a length waiting for its distance
    for (;;) {
      TPROF_CNT(4, 1);
      if (bits < 32) refill();  // a step takes at most 15 + 13 bits
      const bool dist = mlen != 0;
      const uint16_t* const root = dist ? T->droot : T->lroot;
      const int rb = dist ? DROOT : LROOT;
      uint32_t r = root[(uint32_t)hold & ((1u << rb) - 1u)];
      if ((r & 15u) == 0)
        r = root[(1u << rb) + (r >> 7) + ((uint32_t)(hold >> rb) & ((1u << ((r >> 4) & 7u)) - 1u))];
      const uint32_t len = r & 15u;
      const uint32_t e = tok_ent(lit_ent, r >> 4, dist);
      const uint32_t x = e_extra(e), eo = e_op(e);
      if ((int)(len + x) > bits || eo == OP_BAD) { ok = false; break; }
      const uint32_t v = e_val(e) + ((uint32_t)(hold >> len) & ((1u << x) - 1u));
      drop((int)(len + x));
      if (dist) {
        if (!attrib() || !end_run() || !put_tok(0x80000000u | ((mlen - 3u) << 16) | (v - 1u))) { ok = false; break; }
        outlen += mlen;
        mlen = 0;
      } else if (eo == OP_LIT) {
        if (!attrib() || !put_lit(v)) { ok = false; break; }
      } else if (eo == OP_EOB) {
        break;
      } else {
        mlen = v;
      }
    }
    TPROF_ACC(3, t_sym);
    if (!ok) break;
  }
  // the frames left: the last symbol's frame and any after it (no output: the
  // serial decoder then decides, DeflateDecoder.java:122-131)
  while (ok) {
    const bool last = fa == kend;
    if (!close_frame()) ok = false;
    if (last) break;
  }
  if (!ok) a.tstat[k] = InflTokStat{0u, 0u, 0u, 0u};  // the message goes to the serial decoder
  TPROF_ACC(0, t_msg);
  TPROF_CNT(6, 1);
}

// ---------------------------------------------------------------------------------
// Single-frame messages from LDS (the common case).  A lane's tables in HBM scratch
// made every step wait on a global load (and, through the in-order vector memory
// counter, on the window loads and the output stores issued before it), and 128K
// lanes' tables do not fit L2.  Here a lane's tables and its input live in LDS:
//   * literal/length table: 7-bit root + up to QL_SUB sub-table entries; distance:
//     6-bit root + QD_SUB (a set needing more runs on the HBM tables instead).  With
//     the code lengths kept as nibbles that is 47 KB a workgroup, 3 per CU (8/96 and
//     7/32 with byte lengths took 76 KB, 2 per CU: k_infl_tok 4.39 -> 4.11 ms);
//     fixed-code blocks use shared 9/5-bit tables built once per workgroup;
//   * the input: a 64-B ring of the payload's 32-B aligned chunks, topped up at
//     wave-uniform points (when some lane is about to run dry) from a chunk already
//     loaded into registers, so the only wait on global memory is there;
//   * the code lengths of a header in the distance table's space (nibble q of a lane
//     in dword q / 8), the code-length code table in the literal table's.
// The output (literal bytes, tokens) goes to HBM as in tok_message; nothing waits on
// those stores until the next ring top-up.
// ---------------------------------------------------------------------------------
// Root widths and sub-table room (build overrides for A/B): what the bench's headers
// need per width is in DESIGN.md §9 (tools/infl_table_sizes.py).
#ifndef WSG_QL_ROOT
#define WSG_QL_ROOT 7
#endif
#ifndef WSG_QL_SUB
#define WSG_QL_SUB 44
#endif
#ifndef WSG_TOK_WG_PER_CU
#define WSG_TOK_WG_PER_CU 4
#endif
#ifndef WSG_QD_ROOT
#define WSG_QD_ROOT 6
#endif
#ifndef WSG_QD_SUB
#define WSG_QD_SUB 20
#endif
constexpr int QL_ROOT = WSG_QL_ROOT, QD_ROOT = WSG_QD_ROOT, QC_ROOT = 7;  // per-lane root bits
constexpr int QL_SUB = WSG_QL_SUB, QD_SUB = WSG_QD_SUB;                  // sub-table entries a lane may use
constexpr int QL_N = (1 << QL_ROOT) + QL_SUB;        // u16 entries per lane
constexpr int QD_N = (1 << QD_ROOT) + QD_SUB;
constexpr int QF_LROOT = 9, QF_DROOT = 5;            // fixed codes (shared tables)
constexpr uint32_t QF_L = 0, QF_D = 1u << QF_LROOT;  // their u16 offsets
constexpr uint32_t Q_LT = QF_D + (1u << QF_DROOT);   // lane tables: entry j of lane i at Q_LT + j * 64 + i
constexpr uint32_t Q_DT = Q_LT + QL_N * 64;
constexpr uint32_t Q_TAB = Q_DT + QD_N * 64;
#ifndef WSG_TOK_MATCH1
// a match's length and distance in one lane-decoder step: k_infl_tok 2.377 -> 2.168 ms,
// the inflate line 132.3 -> 140.2 GiB/s (same box, 3 interleaved rounds,
// profiles/r05_ab/r05aj_ab_match1.txt); 0 restores two steps a match (A/B)
#define WSG_TOK_MATCH1 1
#endif
#ifndef WSG_TOK_MATCH1_SUB
#define WSG_TOK_MATCH1_SUB 0  // (A/B) the one-step match also through the distance sub-tables
#endif
#ifndef WSG_TOK_EAGER
// the lane's bit buffer refilled to 57-64 bits every step (not only below 32): more
// one-step matches and literal pairs, k_infl_tok 2.168 -> 2.133 ms (same box, 3 rounds,
// profiles/r05_ab/r05ak_ab_eager.txt); 0 for the below-32 refill (A/B)
#define WSG_TOK_EAGER 1
#endif
#ifndef WSG_TOK_MIRROR
#define WSG_TOK_MIRROR 1
#endif
constexpr int Q_RING = 16 + WSG_TOK_MIRROR;          // ring dwords per lane (+ slot 0 mirrored: no wrap test)
constexpr int Q_LENW = 40;                           // code-length dwords per lane (320 nibbles)
static_assert(QD_N * 2 >= Q_LENW * 4, "the code lengths of a header fit a lane's distance table");
static_assert(QL_N >= (1 << QC_ROOT), "the code-length code table fits a lane's literal table");
static_assert(QL_SUB < 256 && QD_SUB < 256, "sub-table offsets fit a root entry's 8 bits");
static_assert((Q_DT * 2) % 4 == 0, "code-length dwords are aligned");

struct TokLds {
  uint32_t ents[N_ENTS];       // length / distance symbol -> entry (tok_ent)
  uint16_t tab[Q_TAB];         // fixed tables, then the lanes' tables
  uint32_t ring[Q_RING * 64];  // input ring: dword slot s of lane i at s * 64 + i
  uint32_t cnt[8 * 64];        // literal/length table build: count, then next code, of length L in
                               // half L & 1 of dword (L >> 1) * 64 + i (both < 2^16); a split's
                               // window bitmap (split_bm), then the head's hand-over
  uint32_t mbox[64];           // a split's mailboxes: lane i's position << 2 | state
};
static_assert(sizeof(TokLds) <= 160 * 1024 / WSG_TOK_WG_PER_CU || WSG_QL_ROOT != 7 || WSG_QD_ROOT != 6,
              "the default tables fit WSG_TOK_WG_PER_CU workgroups per CU (160 KiB of LDS)");

enum : int { Q_OK = 0, Q_BAD = 1, Q_BAIL = 2, Q_SYNC = 3, Q_IDLE = 4 };

// Canonical two-level table of n code lengths into tab (entry j at base + (j << 6)):
// root entries len | symbol << 4; a prefix of longer codes points at its sub-table
// (len 0 | sub bits << 4 | offset << 8), sized by the longest code under the prefix.
// Codes are canonical, so the long codes take the top root prefixes and, code order
// and length order agreeing, the longest code under a prefix is the one that ends
// it.  Returns the longest length, -1 for a set that is not complete (the serial
// decoder applies zlib's rules), -2 when the sub-tables need more than sub entries.
template <class LensF>
__device__ int q_build(uint16_t* tab, uint32_t base, int rb, int sub, LensF lens, int n) {
  int c[16];
#pragma unroll
  for (int l = 0; l < 16; ++l) c[l] = 0;
  for (int s = 0; s < n; ++s) {
    const int l = lens(s);
#pragma unroll
    for (int L = 1; L < 16; ++L) c[L] += (l == L) ? 1 : 0;
  }
  int left = 1, maxl = 0;
  bool bad = false;
#pragma unroll
  for (int l = 1; l < 16; ++l) {
    left = (left << 1) - c[l];
    bad |= left < 0;
    if (c[l]) maxl = l;
  }
  if (bad || left != 0 || maxl == 0) return -1;
  int nx[16];  // first code of each length (MSB-first)
  {
    int code = 0;
    nx[0] = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) {
      code = (code + c[l - 1]) << 1;
      nx[l] = code;
    }
  }
  const uint32_t rsize = 1u << rb;
  if (maxl > rb) {
    // the long prefixes: from the first rb-bit code no shorter code takes
    int P = 0, L = rb + 1;
#pragma unroll
    for (int l = 1; l < 16; ++l)
      if (l == rb) P = nx[l] + c[l];
    uint32_t used = 0;
    for (; P < (int)rsize; ++P) {
      const int pend = (P + 1) << (15 - rb);
      for (;;) {  // the end (left-justified to 15 bits) of the codes of length <= L
        int e = 0;
#pragma unroll
        for (int l = 1; l < 16; ++l)
          if (l == L) e = (nx[l] + c[l]) << (15 - l);
        if (e >= pend) break;
        ++L;
      }
      const uint32_t sb = (uint32_t)(L - rb);
      if (used + (1u << sb) > (uint32_t)sub) return -2;
      const uint32_t slot = __builtin_bitreverse32((uint32_t)P) >> (32 - rb);
      tab[base + (slot << 6)] = (uint16_t)((sb << 4) | (used << 8));
      used += 1u << sb;
    }
  }
  for (int s = 0; s < n; ++s) {
    const int l = lens(s);
    if (!l) continue;
    int code = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L)
      if (l == L) code = nx[L]++;
    const uint32_t rev = __builtin_bitreverse32((uint32_t)code) >> (32 - l);
    const uint16_t e = (uint16_t)((uint32_t)l | ((uint32_t)s << 4));
    if (l <= rb) {
      for (uint32_t j = rev; j < rsize; j += 1u << l) tab[base + (j << 6)] = e;
    } else {
      const uint32_t r = tab[base + ((rev & (rsize - 1u)) << 6)];
      const uint32_t sb = (r >> 4) & 15u, off = r >> 8;
      for (uint32_t j = rev >> rb; j < (1u << sb); j += 1u << (l - rb)) tab[base + ((rsize + off + j) << 6)] = e;
    }
  }
  return maxl;
}

// q_build for the literal/length set (up to 286 codes): the counts and each symbol's
// code come from per-lane LDS counters (an atomic add a symbol, four lengths a read)
// instead of a 15-way select chain a symbol in registers.
__device__ int q_build_lit(TokLds& Q, uint32_t lane, const uint32_t* lw, int n) {
  uint16_t* const tab = Q.tab;
  const uint32_t base = Q_LT + lane;
  constexpr int rb = QL_ROOT;
  uint32_t* const cnt = Q.cnt;  // length L: half L & 1 of dword (L >> 1) * 64 + lane
#pragma unroll
  for (int L = 0; L < 8; ++L) cnt[L * 64 + lane] = 0;
  const int nw = (n + 7) >> 3;  // code length s: nibble s & 7 of dword (s >> 3) * 64 + lane (zero past n)
  for (int q = 0; q < nw; ++q) {
    const uint32_t w = lw[q * 64 + lane];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint32_t l = (w >> (4 * b)) & 15u;
      atomicAdd(&cnt[(l >> 1) * 64 + lane], 1u << (16u * (l & 1u)));  // length 0 counts into slot 0, unused
    }
  }
  int c[16];
  c[0] = 0;
#pragma unroll
  for (int l = 1; l < 16; ++l) c[l] = (int)((cnt[(l >> 1) * 64 + lane] >> (16 * (l & 1))) & 0xffffu);
  int left = 1, maxl = 0;
  bool bad = false;
#pragma unroll
  for (int l = 1; l < 16; ++l) {
    left = (left << 1) - c[l];
    bad |= left < 0;
    if (c[l]) maxl = l;
  }
  if (bad || left != 0 || maxl == 0) return -1;
  int nx[16];
  {
    int code = 0;
    nx[0] = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) {
      code = (code + c[l - 1]) << 1;
      nx[l] = code;
    }
#pragma unroll
    for (int L = 0; L < 8; ++L)  // the next code of each length (length 0's slot unused)
      cnt[L * 64 + lane] = (uint32_t)nx[2 * L] | ((uint32_t)nx[2 * L + 1] << 16);
  }
  const uint32_t rsize = 1u << rb;
  if (maxl > rb) {
    int P = nx[rb] + c[rb], L = rb + 1;
    uint32_t used = 0;
    for (; P < (int)rsize; ++P) {
      const int pend = (P + 1) << (15 - rb);
      for (;;) {
        int e = 0;
#pragma unroll
        for (int l = 1; l < 16; ++l)
          if (l == L) e = (nx[l] + c[l]) << (15 - l);
        if (e >= pend) break;
        ++L;
      }
      const uint32_t sb = (uint32_t)(L - rb);
      if (used + (1u << sb) > (uint32_t)QL_SUB) return -2;
      const uint32_t slot = __builtin_bitreverse32((uint32_t)P) >> (32 - rb);
      tab[base + (slot << 6)] = (uint16_t)((sb << 4) | (used << 8));
      used += 1u << sb;
    }
  }
  for (int q = 0; q < nw; ++q) {
    const uint32_t w = lw[q * 64 + lane];
    uint32_t l4[8], code4[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      l4[b] = (w >> (4 * b)) & 15u;
      code4[b] = (atomicAdd(&cnt[(l4[b] >> 1) * 64 + lane], 1u << (16u * (l4[b] & 1u))) >> (16u * (l4[b] & 1u))) & 0xffffu;
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint32_t l = l4[b];
      if (!l) continue;
      const uint32_t rev = __builtin_bitreverse32(code4[b]) >> (32 - l);
      const uint16_t e = (uint16_t)(l | ((uint32_t)(8 * q + b) << 4));
      if (l <= (uint32_t)rb) {
        for (uint32_t j = rev; j < rsize; j += 1u << l) tab[base + (j << 6)] = e;
      } else {
        const uint32_t r = tab[base + ((rev & (rsize - 1u)) << 6)];
        const uint32_t sb = (r >> 4) & 15u, off = r >> 8;
        for (uint32_t j = rev >> rb; j < (1u << sb); j += 1u << (l - rb)) tab[base + ((rsize + off + j) << 6)] = e;
      }
    }
  }
  return maxl;
}

// The fixed-code tables (RFC 1951 3.2.6), shared by the workgroup.
__device__ void q_fixed_tables(uint16_t* tab, int t) {
  for (int s = t; s < 288; s += 64) {
    int l, code;
    if (s < 144) { l = 8; code = 0x30 + s; }
    else if (s < 256) { l = 9; code = 0x190 + (s - 144); }
    else if (s < 280) { l = 7; code = s - 256; }
    else { l = 8; code = 0xC0 + (s - 280); }
    const uint32_t rev = __builtin_bitreverse32((uint32_t)code) >> (32 - l);
    for (uint32_t j = rev; j < (1u << QF_LROOT); j += 1u << l) tab[QF_L + j] = (uint16_t)(l | (s << 4));
  }
  if (t < 32) tab[QF_D + (__builtin_bitreverse32((uint32_t)t) >> 27)] = (uint16_t)(5 | (t << 4));
}

// Split-lane decode (k_infl_tok<true>; tools/split_decode_proto.py is
// the CPU model of these rules).  The two lanes of a pair take one message.  Both read
// its first block's header (same bits, same tables); then the HEAD decodes from the
// block's first code and the TAIL from a bit near the middle of the payload.  An
// arbitrary bit is not a code boundary, but a Huffman decode started anywhere falls into
// step with the true one within a few codes: the tail marks every literal/length code
// start it meets in a window of SPLIT_WIN bits from its start (a bitmap in the pair's
// cnt dwords) and keeps its counters there (snapshots at the top of its region).  When
// the head reaches a marked position with no length pending, both decodes are at the
// same code of the same block with the same tables, so they agree from there on: the
// head stops at that point S, and after the loop the tail moves its tokens and literals
// after S behind the head's (the run it counted before S comes off its first run token)
// and writes the message's stats.  The tail writes to its own scratch regions (tok2 /
// lit2, laid out as tok / lit), so the head never has to wait for it or stay in half a
// region, and the lanes talk only at the window: the tail's mailbox dword (Q.mbox:
// window start << 2 | state) is read by the head when it reaches the window.  A tail
// decode that fails (a bad code, an end of block far from the payload's end) while the
// head cannot have come near the window (the head moves at most 28 bits a step) starts
// again one bit later; a head that passes the window unmarked, finds the tail still
// marking or failed, or leaves the first block carries on alone (the tail's output is
// dropped).  Every step of the loop pays only a compare for the split; the instructions
// a step issues are what this one-wave-a-SIMD kernel runs on.
constexpr uint32_t SPLIT_MIN = 1024;   // payload bytes a message needs for a split
constexpr uint32_t SPLIT_WIN = 512;    // the tail's window, bits
constexpr uint32_t SPLIT_MARKS = 96;   // snapshots it keeps (the window ends early past them)
constexpr uint32_t SPLIT_SNAPW = 4 * SPLIT_MARKS + 4;  // tail-region token words they take (16-B aligned inside)
constexpr uint32_t SPLIT_STEP_BITS = 28;  // the most bits a step consumes (15-bit code + 13 extra)
constexpr uint32_t SPLIT_RESTARTS = 48;
enum : uint32_t { TS_MARK = 0, TS_RUN = 1, TS_FAIL = 2 };  // tail states
enum : uint32_t { HS_WAIT = 0, HS_OFF = 1, HS_SYNC = 2 };  // head states (the head's own)

// bitmap dword q (0..15) of the pair holding `lane`: the pair's cnt dwords
__device__ __forceinline__ uint32_t split_bm(uint32_t lane, uint32_t q) {
  return (q >> 1) * 64u + (lane & ~1u) + (q & 1u);
}

// One single-frame message from LDS.  Q_BAIL: a table needs more sub-table room than
// the LDS gives a lane; the caller decodes the message with the HBM tables instead.
// PAIR (split-lane decode above): Q_SYNC, the head stopped where the tail took over;
// Q_IDLE, the tail had nothing to do (no split, or the head carried on alone).
template <bool PAIR>
__device__ __forceinline__ int tok_single_lds(const InflArgs& a, TokLds& Q, const wsg_frame_desc& d, uint64_t k,
                                              uint64_t* pf_) {
  (void)pf_;
  const uint32_t lane = threadIdx.x;
  const uint32_t role = PAIR ? (lane & 1u) : 0u;  // 0: the head (or the only lane), 1: the tail
  const uint32_t plen = d.payload_len, total = plen + 4u;
  const uint64_t off = d.payload_off;
  const uint32_t tok_cap = plen + 68u, lit_cap = lit_cap_of(plen);
  uint32_t* const tok = a.tok + tok_base(off, k);
  uint8_t* const lit = a.lit + lit_base(off, k);
  uint32_t* tokp = tok;  // this lane's output (a split's tail: its scratch regions)
  uint8_t* litp = lit;
  uint32_t tcap = tok_cap, lcap = lit_cap;
  uint16_t* const tab = Q.tab;
  uint32_t* const lw32 = reinterpret_cast<uint32_t*>(Q.tab + Q_DT);  // code length s: nibble s & 7 of dword (s >> 3) * 64 + lane
  const uint32_t lt = Q_LT + lane, dt = Q_DT + lane;
  // --- the input ring ---
  const uint8_t* const pay = a.payload;
  const uint64_t pay_len = a.payload_len;
  auto chunk = [&](uint64_t g, uint32_t* w) {  // the 32 bytes at g (32-B aligned), zeros past the payload
    if (g + 32 <= pay_len) {
      const uint4 x = reinterpret_cast<const uint4*>(pay + g)[0], y = reinterpret_cast<const uint4*>(pay + g)[1];
      w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w; w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint32_t v = 0;
        for (int b = 0; b < 4; ++b)
          if (g + 4 * i + b < pay_len) v |= (uint32_t)pay[g + 4 * i + b] << (8 * b);
        w[i] = v;
      }
    }
  };
  auto put_chunk = [&](uint64_t g, const uint32_t* w) {
    const uint32_t s0 = (uint32_t)(g >> 2) & 15u;  // 0 or 8
#pragma unroll
    for (int i = 0; i < 8; ++i) Q.ring[(s0 + i) * 64 + lane] = w[i];
    if (WSG_TOK_MIRROR && s0 == 0) Q.ring[16 * 64 + lane] = w[0];
  };
  uint64_t fill = off & ~(uint64_t)31;  // the next chunk to enter the ring
  const uint64_t pe = off + plen;        // where the payload ends: the tail 00 00 FF FF goes there
  auto top_up = [&]() {
    uint32_t w[8];
    chunk(fill, w);
    if (fill + 32 > pe) {  // DeflateCodec TAIL after the payload, in the ring itself
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint64_t g = fill + 4 * i + b;
          if (g >= pe) {
            const uint64_t q = g - pe;
            const uint32_t by = q < 2 ? 0x00u : (q < 4 ? 0xffu : 0x00u);
            w[i] = (w[i] & ~(0xffu << (8 * b))) | (by << (8 * b));
          }
        }
    }
    put_chunk(fill, w);
    fill += 32;
  };
  top_up();
  top_up();
  uint64_t hold = 0;
  int bits = 0;
  uint32_t ip = 0;                                   // message offset of the next input byte
  uint32_t avail = (uint32_t)(fill - off);           // ring bytes from ip on
  const uint32_t off32 = (uint32_t)off;
  auto ring_word = [&](uint32_t q) -> uint32_t {  // the 4 bytes at message offset q
    const uint32_t ipg = off32 + q;
    const uint32_t sl = (ipg >> 2) & 15u;
    const uint32_t sn = WSG_TOK_MIRROR ? sl + 1u : ((sl + 1u) & 15u);
    return __builtin_amdgcn_alignbyte(Q.ring[sn * 64 + lane], Q.ring[sl * 64 + lane], ipg & 3u);
  };
  // Input, a step: at least 32 bits held (or the rest of the input), up to 4 bytes
  // from the ring word at ip, read a step ahead so its latency overlaps the step.
  // Top-up: at a point every active lane reaches, when some lane has under 4 bytes in
  // the ring, every lane with room loads a chunk into it.  The load is waited on right
  // there: a chunk loaded ahead into registers kept a load pending across the step
  // loop, and the compiler then waited on the vector memory counter at every step.
  uint32_t rw = ring_word(0);
  auto in_step = [&]() {
    if (__any(ip < total && avail < 4u)) {
      if (avail <= 32u) {
        top_up();
        avail += 32u;
      }
      rw = ring_word(ip);
    }
    const uint32_t rem = total - ip;
#if WSG_TOK_EAGER
    // as many whole bytes of the ring word as the 64-bit buffer has room for, so a step
    // holds 57-64 bits and the one-step match and second literal fire more often
    const uint32_t room = (uint32_t)(64 - bits) >> 3;
    const uint32_t nb = min(min(room, 4u), rem);
#else
    const uint32_t nb = bits < 32 ? (rem < 4u ? rem : 4u) : 0u;
#endif
    hold |= (uint64_t)(rw & (nb == 4u ? 0xffffffffu : ((1u << (8u * nb)) - 1u))) << bits;
    bits += 8 * (int)nb;
    ip += nb;
    avail -= nb;
    rw = ring_word(ip);
  };
  auto drop = [&](int n) {
    hold >>= n;
    bits -= n;
  };
  // the input from message bit p (a split's tail)
  auto seek = [&](uint32_t p) {
    ip = p >> 3;
    fill = (off + ip) & ~(uint64_t)31;
    top_up();
    top_up();
    avail = (uint32_t)(fill - (off + ip));
    hold = 0;
    bits = 0;
    rw = ring_word(ip);
    in_step();
    drop((int)(p & 7u));
  };
  // --- the output ---
  uint32_t ntok = 0, nlit = 0, run = 0, outlen = 0, litw = 0;
  auto put_lit = [&](uint32_t b) -> bool {
    if (nlit >= lcap) return false;
    litw |= b << (8 * (nlit & 3u));
    if ((++nlit & 3u) == 0) {
      reinterpret_cast<uint32_t*>(litp)[(nlit >> 2) - 1] = litw;
      litw = 0;
    }
    ++run;
    ++outlen;
    return true;
  };
  auto put_tok = [&](uint32_t t) -> bool {
    if (ntok >= tcap) return false;
    tokp[ntok++] = t;
    return true;
  };
  auto end_run = [&]() -> bool {
    if (!run) return true;
    const bool r = put_tok(run);
    run = 0;
    return r;
  };
  // --- the split (PAIR) ---
  bool split = false;  // open for this message (both lanes decide alike)
  bool blk1 = false;   // in the first block's symbol loop, where the split lives
  uint32_t ss = 0;     // HS_* (head) / TS_* (tail)
  uint32_t win0 = 0;   // the tail's window start (the head: as last seen)
  uint32_t nmarks = 0, restarts = 0, sync_j = 0;
  uint32_t tsteps = 0, rlimit = 0;  // the tail's steps; it may start again while tsteps < rlimit
  uint4* snap = nullptr;
  bool first = true;   // the message's first block
  int st = Q_OK;
  for (;;) {
    in_step();
    if (bits == 0 && ip >= total) break;  // clean: all input used, on a block boundary
    if (bits < 3) { st = Q_BAD; break; }
    const uint32_t last = (uint32_t)(hold & 1u), type = (uint32_t)((hold >> 1) & 3u);
    drop(3);
    if (last) { st = Q_BAD; break; }  // a final block: the stream ends (k_inflate handles it)
    if (type == 0) {                  // stored
      if (PAIR && first && role) { st = Q_IDLE; break; }  // no split: the head decodes it
      first = false;
      drop(bits & 7);
      in_step();
      if (bits < 32) { st = Q_BAD; break; }
      const uint32_t ln = (uint32_t)(hold & 0xffffu), nl = (uint32_t)((hold >> 16) & 0xffffu);
      if (ln != (nl ^ 0xffffu)) { st = Q_BAD; break; }
      drop(32);
      for (uint32_t i = 0; i < ln; ++i) {
        in_step();
        if (bits < 8 || !put_lit((uint32_t)(hold & 0xffu))) { st = Q_BAD; break; }
        drop(8);
      }
      if (st != Q_OK) break;
      continue;
    }
    if (type == 3) { st = Q_BAD; break; }
    const bool fixed = type == 1;
    TPROF_CNT(5, 1);
    TPROF_T(t_hdr);
    if (!fixed) {  // dynamic codes
      in_step();
      if (bits < 14) { st = Q_BAD; break; }
      const int nlen = (int)(hold & 31u) + 257, ndist = (int)((hold >> 5) & 31u) + 1,
                ncode = (int)((hold >> 10) & 15u) + 4;
      drop(14);
      if (nlen > 286 || ndist > 30) { st = Q_BAD; break; }
      // code-length code lengths: 19 nibbles in registers, by symbol
      uint32_t cl0 = 0, cl1 = 0, cl2 = 0;
      for (int i = 0; i < ncode; ++i) {
        in_step();
        if (bits < 3) { st = Q_BAD; break; }
        const uint32_t v = (uint32_t)(hold & 7u), s = kClenOrder[i], sh = 4u * (s & 7u);
        if (s < 8) cl0 |= v << sh;
        else if (s < 16) cl1 |= v << sh;
        else cl2 |= v << sh;
        drop(3);
      }
      if (st != Q_OK) break;
      auto clen = [&](int s) -> int {
        const uint32_t w = s < 8 ? cl0 : (s < 16 ? cl1 : cl2);
        return (int)((w >> (4 * (s & 7))) & 15u);
      };
      const int cmax = q_build(tab, lt, QC_ROOT, 0, clen, 19);
      if (cmax < 0) { st = Q_BAD; break; }
      // the code lengths, into the distance table's space (zeroed first: runs of zeros
      // then write nothing)
      for (int q = 0; q < Q_LENW; ++q) lw32[q * 64 + lane] = 0;
      int have = 0, prev = 0, len256 = 0;
      while (have < nlen + ndist) {
        in_step();
        const uint32_t r = tab[lt + (((uint32_t)hold & ((1u << QC_ROOT) - 1u)) << 6)];
        const int nb = (int)(r & 15u), sy = (int)(r >> 4);
        if (nb == 0 || nb > bits) { st = Q_BAD; break; }
        int copy = 1, len = sy, xb = 0;
        if (sy >= 16) {
          xb = sy == 16 ? 2 : (sy == 17 ? 3 : 7);
          if (nb + xb > bits) { st = Q_BAD; break; }
          const int x = (int)((hold >> nb) & ((1u << xb) - 1u));
          if (sy == 16) {
            if (have == 0) { st = Q_BAD; break; }
            len = prev;
            copy = 3 + x;
          } else {
            len = 0;
            copy = (sy == 17 ? 3 : 11) + x;
          }
        }
        drop(nb + xb);
        if (have + copy > nlen + ndist) { st = Q_BAD; break; }
        for (int i = 0; len && i < copy; ++i) {
          const uint32_t q = (uint32_t)(have + i);
          lw32[(q >> 3) * 64u + lane] |= (uint32_t)len << (4u * (q & 7u));
        }
        if (have <= 256 && 256 < have + copy) len256 = len;
        have += copy;
        prev = len;
      }
      if (st != Q_OK) break;
      if (len256 == 0) { st = Q_BAD; break; }
      // the distance lengths into registers (their space becomes the distance table)
      uint32_t dl[4] = {0u, 0u, 0u, 0u};
      for (int i = 0; i < ndist; ++i) {
        const uint32_t q = (uint32_t)(nlen + i);
        const uint32_t v = (lw32[(q >> 3) * 64u + lane] >> (4u * (q & 7u))) & 15u;
        const uint32_t w = (uint32_t)i >> 3, sh = 4u * ((uint32_t)i & 7u);
        if (w == 0) dl[0] |= v << sh;
        else if (w == 1) dl[1] |= v << sh;
        else if (w == 2) dl[2] |= v << sh;
        else dl[3] |= v << sh;
      }
      auto dlen = [&](int s) -> int {
        const uint32_t w = (uint32_t)s >> 3;
        const uint32_t x = w == 0 ? dl[0] : (w == 1 ? dl[1] : (w == 2 ? dl[2] : dl[3]));
        return (int)((x >> (4 * (s & 7))) & 15u);
      };
      TPROF_T(t_bld);
      // (the distance lengths after the literal ones are in the same dwords: cleared
      // first, so the literal build counts only its own)
      for (int i = 0; i < ndist; ++i) {
        const uint32_t q = (uint32_t)(nlen + i);
        lw32[(q >> 3) * 64u + lane] &= ~(15u << (4u * (q & 7u)));
      }
      const int lmax = q_build_lit(Q, lane, lw32, nlen);
      if (lmax == -2) { st = Q_BAIL; break; }
      if (lmax < 0) { st = Q_BAD; break; }
      const int dmax = q_build(tab, dt, QD_ROOT, QD_SUB, dlen, ndist);
      if (dmax == -2) { st = Q_BAIL; break; }
      if (dmax < 0) { st = Q_BAD; break; }
      TPROF_ACC(2, t_bld);
    }
    TPROF_ACC(1, t_hdr);
    if (PAIR && first) {  // open a split, or leave the message to the head
      const uint32_t pos0 = 8u * ip - (uint32_t)bits, endb = 8u * plen;
      split = a.split != 0 && plen >= SPLIT_MIN && plen < (1u << 26) && endb > pos0 + 4096u;
      if (!split) {
        if (role) { st = Q_IDLE; break; }
      } else {
        blk1 = true;
        win0 = pos0 + (uint32_t)(((uint64_t)(endb - pos0) * 15u) >> 5);
        // the head is at most pos0 + 28 t after t steps: while t < rlimit it is two
        // windows short of win0, so a restart cannot pull the bitmap from under it
        rlimit = (win0 - pos0 > 2u * SPLIT_WIN) ? (win0 - pos0 - 2u * SPLIT_WIN) / SPLIT_STEP_BITS : 0u;
        if (role == 0) {
          ss = HS_WAIT;
        } else {
          tokp = a.tok2 + tok_base(off, k);
          litp = a.lit2 + lit_base(off, k);
          tcap = tok_cap - SPLIT_SNAPW;
          snap = reinterpret_cast<uint4*>((reinterpret_cast<uintptr_t>(tokp + tcap) + 15u) & ~(uintptr_t)15u);
          ss = TS_MARK;
#pragma unroll
          for (uint32_t q = 0; q < 16; ++q) Q.cnt[split_bm(lane, q)] = 0u;
          seek(win0);
          Q.mbox[lane] = (win0 << 2) | TS_MARK;
        }
      }
    }
    first = false;
    TPROF_T(t_sym);
    // the block's symbols, one code a step (literal/length, or the distance of the
    // length before it) through one lookup path
    const uint32_t lbase = fixed ? QF_L : lt, dbase = fixed ? QF_D : dt;
    const uint32_t lrb = fixed ? QF_LROOT : QL_ROOT, drb = fixed ? QF_DROOT : QD_ROOT;
    const uint32_t tsh = fixed ? 0u : 6u;  // entry j at base + (j << tsh)
    uint32_t mlen = 0;                     // a length waiting for its distance
    // Branch-light: one instruction stream for the 64 lanes; the stores are masked to
    // the lanes that complete something (a literal word, a match and the literal run
    // before it), so every output byte is written once.  (Unconditional stores of the
    // partial word and of a token slot every step wrote ~6x the token + literal bytes
    // per launch, and each ring top-up waited for all of them.)
    for (;;) {
      TPROF_CNT(4, 1);
      in_step();  // a step takes at most 15 + 13 bits
      const bool dist = mlen != 0;
      const uint32_t base = dist ? dbase : lbase, rb = dist ? drb : lrb;
      uint32_t r = tab[base + (((uint32_t)hold & ((1u << rb) - 1u)) << tsh)];
      if ((r & 15u) == 0)
        r = tab[base + (((1u << rb) + (r >> 8) + ((uint32_t)(hold >> rb) & ((1u << ((r >> 4) & 15u)) - 1u))) << tsh)];
      const uint32_t len = r & 15u;
      const uint32_t e = tok_ent(Q.ents, r >> 4, dist);
      // a second literal in the same step (text is mostly literals): the root entry of the
      // code after this one, read beside the symbol entry, taken when both are literals
      // whose codes the root resolves
      const uint32_t r2 = !PAIR ? tab[lbase + ((((uint32_t)(hold >> len)) & ((1u << lrb) - 1u)) << tsh)] : 0u;
      const uint32_t x = e_extra(e), eo = e_op(e);
      const uint32_t v = e_val(e) + ((uint32_t)(hold >> len) & ((1u << x) - 1u));
      if (PAIR && split) {
        const uint32_t cur = 8u * ip - (uint32_t)bits;
        if (role == 0) {
          if (ss == HS_WAIT && !dist && cur >= win0) {  // at the tail's window: its mailbox
            const uint32_t pm = Q.mbox[lane ^ 1u];
            const uint32_t w0 = pm >> 2, ts = pm & 3u;
            if (w0 > win0) {
              win0 = w0;  // the tail started again further on: look again there
            } else if (ts != TS_RUN || cur >= w0 + SPLIT_WIN) {
              ss = HS_OFF;  // the tail failed or is still marking, or the window passed unmarked
            } else {
              const uint32_t b = cur - w0, q = b >> 5;
              const uint32_t wq = Q.cnt[split_bm(lane, q)];
              if ((wq >> (b & 31u)) & 1u) {  // S: the tail decoded from here too
                uint32_t j = (uint32_t)__builtin_popcount(wq & ((1u << (b & 31u)) - 1u));
                for (uint32_t q2 = 0; q2 < q; ++q2) j += (uint32_t)__builtin_popcount(Q.cnt[split_bm(lane, q2)]);
                sync_j = j;
                ss = HS_SYNC;
                st = Q_SYNC;
                break;
              }
            }
          }
        } else {
          ++tsteps;
          if (blk1 && ss == TS_MARK && !dist) {
            if (cur < win0 + SPLIT_WIN && nmarks < SPLIT_MARKS) {
              const uint32_t b = cur - win0;
              Q.cnt[split_bm(lane, b >> 5)] |= 1u << (b & 31u);
              snap[nmarks++] = make_uint4(ntok, nlit, outlen, run);
            } else {
              ss = TS_RUN;
              Q.mbox[lane] = (win0 << 2) | TS_RUN;
            }
          }
        }
      }
      const bool is_lit = !dist && eo == OP_LIT, is_len = !dist && eo == OP_BASE;
#if WSG_TOK_MATCH1
      // A length's distance in the same step (a match in one step instead of two) when its
      // code resolves at the distance root, is a valid distance, and all its bits are held
      // (a step holds 32-63 bits; otherwise the next step decodes it as before).
      bool m1 = false;
      uint32_t dv = 0, dbits = 0;
      if (!PAIR) {
        const uint32_t sh1 = len + x;
        const uint64_t h2 = hold >> sh1;
        uint32_t rd = tab[dbase + (((uint32_t)h2 & ((1u << drb) - 1u)) << tsh)];
#if WSG_TOK_MATCH1_SUB
        if ((rd & 15u) == 0)  // a longer distance code: its sub-table, as the main lookup does
          rd = tab[dbase + (((1u << drb) + (rd >> 8) + ((uint32_t)(h2 >> drb) & ((1u << ((rd >> 4) & 15u)) - 1u))) << tsh)];
#endif
        const uint32_t dl = rd & 15u;
        const uint32_t ed = tok_ent(Q.ents, rd >> 4, true);
        const uint32_t dx = e_extra(ed);
        dv = e_val(ed) + ((uint32_t)(h2 >> dl) & ((1u << dx) - 1u));
        dbits = dl + dx;
        m1 = is_len && dl != 0u && e_op(ed) == OP_BASE && (int)(sh1 + dbits) <= bits;
      }
      const bool emit = dist | m1;  // a match token this step
#else
      constexpr bool m1 = false;
      constexpr uint32_t dv = 0, dbits = 0;
      const bool emit = dist;
#endif
      const uint32_t has_run = (emit && run) ? 1u : 0u;
      // (bitwise: one exit test, no short-circuit branches)
      const bool bad = ((int)(len + x) > bits) | (eo == OP_BAD) | (is_lit & (nlit >= lcap)) |
                       (emit & (ntok + 1u + has_run > tcap));
      const bool eob = !dist & (eo == OP_EOB);
      if (bad | eob) {
        if (PAIR && split && role && ss != TS_FAIL &&
            (bad || (blk1 && tsteps < rlimit && 8u * total - (8u * ip - (uint32_t)bits + len) > 48u))) {
          // the tail off the true stream (an end of block far from the payload's end is
          // taken for one): again one bit on while the head cannot be near, else give up
          // (a failure after the head stopped at S is the message's: the serial decoder's)
          if (blk1 && tsteps < rlimit && restarts < SPLIT_RESTARTS) {
            ++restarts;
            ++win0;
#pragma unroll
            for (uint32_t q = 0; q < 16; ++q) Q.cnt[split_bm(lane, q)] = 0u;
            seek(win0);
            ntok = nlit = run = outlen = litw = 0;
            mlen = 0;
            nmarks = 0;
            ss = TS_MARK;
            Q.mbox[lane] = (win0 << 2) | TS_MARK;
            continue;
          }
          ss = TS_FAIL;
          Q.mbox[lane] = (win0 << 2) | TS_FAIL;
          st = Q_IDLE;
          break;
        }
        if (bad) st = Q_BAD;
        else drop((int)len);
        break;
      }
      const uint32_t len2 = r2 & 15u, sym2 = r2 >> 4;
      const bool two = !PAIR && is_lit && len2 != 0u && sym2 < 256u && (int)(len + len2) <= bits && nlit + 2u <= lcap;
      drop((int)(len + x + (two ? len2 : 0u) + (m1 ? dbits : 0u)));
      uint32_t* const lit32 = reinterpret_cast<uint32_t*>(litp);
      const uint32_t nadd = is_lit ? (two ? 2u : 1u) : 0u;
      const uint32_t sh = 8u * (nlit & 3u);
      const uint64_t acc = (uint64_t)litw | ((uint64_t)(is_lit ? v : 0u) << sh) | ((uint64_t)(two ? sym2 : 0u) << (sh + 8u));
      const bool word_done = (nlit & 3u) + nadd >= 4u;
      if (word_done) lit32[nlit >> 2] = (uint32_t)acc;  // the word just filled
      if (emit) {
        if (has_run) tokp[ntok] = run;
        const uint32_t ml = dist ? mlen : v, md = dist ? v : dv;
        tokp[ntok + has_run] = 0x80000000u | ((ml - 3u) << 16) | (md - 1u);
      }
      ntok += emit ? 1u + has_run : 0u;
      litw = word_done ? (uint32_t)(acc >> 32) : (uint32_t)acc;
      nlit += nadd;
      outlen += is_lit ? nadd : (dist ? mlen : (m1 ? v : 0u));
      run = emit ? 0u : run + nadd;
      mlen = (is_len && !m1) ? v : (dist ? 0u : mlen);
    }
    TPROF_ACC(3, t_sym);
    if (PAIR && blk1) {  // leaving the first block: the head's split ends, the tail's window closes
      if (role == 0 && ss == HS_WAIT) ss = HS_OFF;
      if (role == 1 && ss == TS_MARK) {
        ss = TS_RUN;
        Q.mbox[lane] = (win0 << 2) | TS_RUN;
      }
      blk1 = false;
    }
    if (st != Q_OK) break;
  }
  if (PAIR && split) {
    // both lanes are past the loop here (the wave leaves it together): the head hands
    // its counters to the tail through its own cnt dwords
    if (role == 0) {
      if (st == Q_SYNC) {
        end_run();  // (room: checked at S)
        Q.cnt[0 * 64 + lane] = 1u;
        Q.cnt[1 * 64 + lane] = sync_j;
        Q.cnt[2 * 64 + lane] = ntok;
        Q.cnt[3 * 64 + lane] = nlit;
        Q.cnt[4 * 64 + lane] = outlen;
        Q.cnt[5 * 64 + lane] = litw;
      } else {
        Q.cnt[0 * 64 + lane] = 0u;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
    if (role == 1) {
      const uint32_t hl = lane ^ 1u;
      if (Q.cnt[0 * 64 + hl] != 1u) return Q_IDLE;  // the head decoded the message alone
      if (st == Q_BAIL) return Q_BAIL;             // (a later block's tables: the caller's HBM decoder)
      if (st != Q_OK || !end_run()) {              // the message's own error: the serial decoder's
        a.tstat[k] = InflTokStat{0u, 0u, 0u, 0u};
        return Q_BAD;
      }
      if (nlit & 3u) reinterpret_cast<uint32_t*>(litp)[nlit >> 2] = litw;
      const uint32_t j = Q.cnt[1 * 64 + hl], nth = Q.cnt[2 * 64 + hl], nlh = Q.cnt[3 * 64 + hl],
                     outh = Q.cnt[4 * 64 + hl], litwh = Q.cnt[5 * 64 + hl];
      const uint4 sn = snap[j];  // the tail's counters at S: tokens, literals, output, run
      // its tokens after S behind the head's; the run before S comes off the first run token
      const uint32_t* src = tokp + sn.x;
      uint32_t n = ntok - sn.x, nt = nth;
      const uint32_t m = nlit - sn.y;
      if (nth + n > tok_cap || nlh + m > lit_cap) {  // (room as the one-lane decode has it)
        a.tstat[k] = InflTokStat{0u, 0u, 0u, 0u};
        return Q_BAD;
      }
      if (sn.w && n) {
        const uint32_t v0 = src[0] - sn.w;
        if (v0) tok[nt++] = v0;
        ++src;
        --n;
      }
      uint32_t i = 0;
      for (; i + 8 <= n; i += 8) {  // (8 loads in flight a lane)
        uint32_t t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = src[i + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) tok[nt + i + u] = t[u];
      }
      for (; i < n; ++i) tok[nt + i] = src[i];
      nt += n;
      // its literals after S behind the head's, byte-shifted word by word (the head's
      // partial last word merged into the first)
      const uint32_t sb = sn.y, db = nlh;
      const uint32_t* const s32 = reinterpret_cast<const uint32_t*>(litp);
      uint32_t* const l32 = reinterpret_cast<uint32_t*>(lit);
      const uint32_t w0 = db >> 2, we = (db + m + 3u) >> 2;
      for (uint32_t w = w0; w < we; w += 4) {
        uint32_t vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          // source byte of the word's first byte: below 0 only for the first word, whose
          // bytes there are the head's (kept below)
          const int32_t sp = (int32_t)(4u * (w + u) + sb) - (int32_t)db;
          const int32_t q = sp >> 2;
          vv[u] = __builtin_amdgcn_alignbyte(s32[q + 1], q >= 0 ? s32[q] : 0u, (uint32_t)sp & 3u);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t ww = w + u;
          if (ww >= we) break;
          uint32_t x = vv[u];
          if (ww == w0 && (db & 3u)) {
            const uint32_t keep = (1u << (8u * (db & 3u))) - 1u;
            x = (x & ~keep) | (litwh & keep);
          }
          l32[ww] = x;
        }
      }
      a.tstat[k] = InflTokStat{1u, nt, nlh + m, outh + (outlen - sn.z)};
      if (a.split_cnt) atomicAdd(a.split_cnt, 1ull);
      return Q_SYNC;
    }
    if (st == Q_SYNC) return Q_SYNC;
  }
  if (PAIR && role) return Q_IDLE;  // (no split: every outcome is the head's)
  if (st == Q_OK) {
    if (!end_run()) st = Q_BAD;
    else {
      if (nlit & 3u) reinterpret_cast<uint32_t*>(lit)[nlit >> 2] = litw;
      a.tstat[k] = InflTokStat{1u, ntok, nlit, outlen};
    }
  }
  if (st == Q_BAD) a.tstat[k] = InflTokStat{0u, 0u, 0u, 0u};  // the message goes to the serial decoder
  return st;
}

// PAIR: the two lanes of a pair take the same frames (the split-lane decode above);
// otherwise a lane takes its own.
template <bool PAIR>
__global__ __launch_bounds__(64) void k_infl_tok(InflArgs a) {
  // symbol -> entry (base, extra bits, op) for the 16-bit root entries
  __shared__ TokLds Q;
  uint32_t* const ents = Q.ents;  // length entries, then distance entries (tok_ent)
  for (int i = threadIdx.x; i < N_ENTS; i += 64) ents[i] = ents_init((uint32_t)i);
  q_fixed_tables(Q.tab, threadIdx.x);
  __syncthreads();
  const uint32_t lane_id = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane_id >= a.n_lanes) return;  // (n_lanes: whole waves)
#ifdef WSG_INFLATE_TOK_PROF
  uint64_t pf_[8] = {};
#define PF_PTR pf_
#else
#define PF_PTR nullptr
#endif
  const uint32_t unit = PAIR ? lane_id >> 1 : lane_id, n_units = PAIR ? a.n_lanes >> 1 : a.n_lanes;
  const bool tail = PAIR && (lane_id & 1u);
  LaneTab* T = nullptr;  // the lane's HBM tables, taken from the pool when first needed
  for (uint64_t i = unit; i < a.n_frames; i += n_units) {
    const uint64_t k = a.order ? a.order[i] : i;
    const wsg_frame_desc d = a.desc[k];
    const uint32_t op = d.opcode & 15u, fin = (d.flags >> 7) & 1u, rsv = (d.flags >> 4) & 7u;
    const bool start = (op == WSG_OP_TEXT || op == WSG_OP_BINARY) && (rsv & 4u) && !(d.flags & WSG_DESC_REPLAY) &&
                       d.payload_off + d.payload_len <= a.payload_len;
    if (!start) {
      // a continuation's stats are its message's (the start frame's lane writes them)
      if (!tail && op != WSG_OP_CONTINUATION) a.tstat[k] = InflTokStat{0u, 0u, 0u, 0u};
      continue;
    }
    // The message: frame k and, if it is not FIN, the session's continuation frames up
    // to the FIN one (control frames between them are not part of the stream).  A
    // message the batch does not hold whole goes to the serial decoder.
    uint64_t kend = k, se = k + 1;
    uint32_t in_len = d.payload_len;  // compressed bytes of the whole message
    bool whole = fin != 0;
    if (!fin) {
      se = a.session_first[find_session(a.session_first, a.n_sessions, k) + 1];
      for (uint64_t j = k + 1; j < se; ++j) {
        const wsg_frame_desc dj = a.desc[j];
        const uint32_t oj = dj.opcode & 15u;
        if (oj >= 8u) continue;
        if (oj != WSG_OP_CONTINUATION || (dj.flags & WSG_DESC_REPLAY) || dj.payload_off + dj.payload_len > a.payload_len)
          break;
        in_len += dj.payload_len;
        if (dj.flags & 0x80u) {
          kend = j;
          whole = true;
          break;
        }
      }
    }
    if (!whole) {
      if (!tail) a.tstat[k] = InflTokStat{0u, 0u, 0u, 0u};
      continue;
    }
    if (kend == k && a.tok_lds) {
      TPROF_T(t_msg);
      const int st = tok_single_lds<PAIR>(a, Q, d, k, PF_PTR);
      TPROF_ACC(0, t_msg);
      TPROF_CNT(6, 1);
      TPROF_CNT(7, st == Q_BAIL);
      if (st != Q_BAIL) continue;  // (a tail's Q_BAIL: its part of a split needs the HBM tables)
    } else if (tail) {
      continue;  // the head takes it alone
    }
    if (!T) {
      const uint32_t slot = atomicAdd(a.tab_cnt, 1u);
      if (slot < a.n_tab) T = reinterpret_cast<LaneTab*>(a.tab) + slot;
    }
    if (!T) {  // no table block left: the serial decoder takes the message
      a.tstat[k] = InflTokStat{0u, 0u, 0u, 0u};
      continue;
    }
    if (kend == k)
      tok_message<false>(a, T, ents, k, kend, in_len, PF_PTR);
    else
      tok_message<true>(a, T, ents, k, kend, in_len, PF_PTR);
  }
#ifdef WSG_INFLATE_TOK_PROF
  for (int i = 0; i < 8; ++i) atomicAdd(&g_tok_prof[i], (unsigned long long)pf_[i]);
#endif
#undef PF_PTR
}

}  // namespace


// One workgroup (one wave) per session.
__global__ __launch_bounds__(64) void k_inflate(InflArgs a) {
  __shared__ Lds L;
  const int lane = threadIdx.x;
  const uint32_t s = blockIdx.x;
  if (s >= a.n_sessions) return;
  if (a.fast_done && a.fast_done[s]) return;  // replayed in parallel by k_infl_fast
#ifdef WSG_INFLATE_PROF
  uint64_t pf_[24] = {};
#endif
  PROF_T(t_all);
  const uint32_t f0 = a.session_first[s], f1 = a.session_first[s + 1];
  const uint64_t obase = a.out_off[s], ocap64 = a.out_off[s + 1] - a.out_off[s];
  const int32_t ocap = ocap64 < (uint64_t)POS_LIMIT ? (int32_t)ocap64 : POS_LIMIT;
  const wsg_inflate_state st0 = a.state[s];
  uint8_t* const win = a.window + (uint64_t)s * WSG_INFLATE_WINDOW;
  uint8_t* const out = a.out + obase;
  const bool pl_aligned = (((uintptr_t)a.payload) & 15u) == 0;
  const bool win_aligned = (((uintptr_t)win) & 15u) == 0;

  // carry-in: the window image goes to the ring as is; position 0 of this batch sits
  // at ring slot ph, the history at positions [-wl0, 0)
  int compressing = st0.compressing, has_dec = st0.has_decoder, finished = st0.finished;
  const int wl0 = (has_dec && !finished) ? (int)(st0.window_len < WSG_INFLATE_WINDOW ? st0.window_len : WSG_INFLATE_WINDOW) : 0;
  const uint32_t ph = wl0 ? (uint32_t)st0.window_phase & WMASK : 0u;
  PROF_T(t_cin);
  if (wl0) {
    if (win_aligned)
      for (uint32_t c = lane; c < WSG_INFLATE_WINDOW / 16; c += 64)
        reinterpret_cast<uint4*>(L.ring)[c] = reinterpret_cast<const uint4*>(win)[c];
    else
      for (uint32_t i = lane; i < WSG_INFLATE_WINDOW; i += 64) L.ring[i] = win[i];
  }
  __syncthreads();
  PROF_ACC(1, t_cin);
  auto ri = [&](int32_t p) -> uint32_t { return ((uint32_t)p + ph) & WMASK; };

  int32_t pos = 0;            // output bytes of this batch (session region offset)
  int32_t flushed = 0;        // ring bytes [flushed, pos) not yet in HBM
  int32_t wstart = -wl0;      // position where the current inflater's history starts
  // inflater registers (persist across frames: one continuous stream)
  int mode = M_HEAD, last = 0;
  uint64_t hold = 0;
  int bits = 0;
  int lmax = 0, dmax = 0, cmax = 0;
  int nlen = 0, ndist = 0, ncode = 0, have = 0;
  uint32_t length = 0, dist = 0, extra = 0;
  // the message-start snapshot (a batch ending inside a message commits it)
  int snap_k = -1, snap_has = 0, snap_fin = 0;
  int32_t snap_pos = 0, snap_wstart = 0;
  int err = E_NONE;
  uint32_t err_idx = 0, delivered = 0;
  int32_t err_end = 0;        // on a data error: output of the frames delivered before it

  // flush ring bytes [flushed, end) to HBM in dwords (all lanes); false past the region's end
  auto flush_to = [&](int32_t end) -> bool {
    if (end > ocap) return false;
    PROF_T(t_fl);
    int32_t i0 = flushed;
    int32_t head = (int32_t)((4u - (uint32_t)(((uintptr_t)(out + i0)) & 3u)) & 3u);
    if (head > end - i0) head = end - i0;
    if (lane < head) out[i0 + lane] = L.ring[ri(i0 + lane)];
    i0 += head;
    const int32_t nw = (end - i0) >> 2;
    uint32_t* const ow = reinterpret_cast<uint32_t*>(out + i0);
    if ((ri(i0) & 3u) == 0) {
      for (int32_t w = lane; w < nw; w += 64) ow[w] = *reinterpret_cast<const uint32_t*>(L.ring + ri(i0 + 4 * w));
    } else {
      for (int32_t w = lane; w < nw; w += 64) {
        const int32_t q = i0 + 4 * w;
        ow[w] = (uint32_t)L.ring[ri(q)] | ((uint32_t)L.ring[ri(q + 1)] << 8) | ((uint32_t)L.ring[ri(q + 2)] << 16) |
                ((uint32_t)L.ring[ri(q + 3)] << 24);
      }
    }
    i0 += nw * 4;
    if (lane < end - i0) out[i0 + lane] = L.ring[ri(i0 + lane)];
    flushed = end;
    PROF_ACC(6, t_fl);
    return true;
  };
  auto flush = [&]() -> bool { return flush_to(pos); };
  // a back-reference: every byte comes from [pos - dist, pos), so a chunk of 64 lanes
  // never reads a byte of its own chunk
  auto copy_match = [&](uint32_t len, uint32_t d) {
    if (d >= len) {
      for (uint32_t b = 0; b < len; b += 64) {
        const uint32_t i = b + (uint32_t)lane;
        if (i < len) {
          const uint8_t v = L.ring[ri(pos - d + i)];
          L.ring[ri(pos + i)] = v;
        }
      }
    } else {
      for (uint32_t b = 0; b < len; b += 64) {
        const uint32_t i = b + (uint32_t)lane;
        if (i < len) {
          const uint8_t v = L.ring[ri(pos - d + i % d)];
          L.ring[ri(pos + i)] = v;
        }
      }
    }
    pos += len;
  };

  for (uint32_t k = f0; k < f1 && err == E_NONE; ++k) {
    PROF_T(t_fr);
    const wsg_frame_desc d = a.desc[k];
    PROF_CNT(15, 1);
    const bool replay = (d.flags & WSG_DESC_REPLAY) != 0;
    const uint32_t op = d.opcode & 15u, fin = (d.flags >> 7) & 1u, rsv = (d.flags >> 4) & 7u;
    const bool allow = ((op == WSG_OP_TEXT || op == WSG_OP_BINARY) && (rsv & 4u)) || (op == WSG_OP_CONTINUATION && compressing);
    if (allow && !compressing) {  // a compressed message starts here: snapshot
      snap_k = (int)(k - f0);
      snap_has = has_dec;
      snap_fin = finished;
      snap_pos = pos;
      snap_wstart = wstart;
    }
    if (allow) {
      if (!has_dec) {  // new ZlibDecoder(RAW): a fresh inflater, empty window (DeflateDecoder.java:80-93)
        has_dec = 1;
        finished = 0;
        mode = M_HEAD;
        last = 0;
        hold = 0;
        bits = 0;
        wstart = pos;
      }
      const int32_t fstart = pos;
      PROF_ACC(8, t_fr);
      // the frame's input: its payload, then the tail 00 00 FF FF if final
      const uint64_t src0 = d.payload_off;
      const uint32_t plen = d.payload_len;
      const uint32_t total_in = plen + (fin ? 4u : 0u);
      uint32_t ip = 0;                              // bytes of this frame's input pulled
      uint32_t ib_lo = 0, ib_hi = 0, ib_off = 0;    // ibuf[ib_off..] holds input bytes [ib_lo, ib_hi)
      // stage input from byte i: aligned 16-byte loads by all lanes
      auto restage = [&](uint32_t i) {
        const uint64_t g = src0 + i;
        const uint64_t A = g & ~(uint64_t)15;
        ib_off = (uint32_t)(g - A);
        PROF_CNT(12, 1);
        ib_lo = i;
        ib_hi = (i + IB - ib_off) < total_in ? (i + IB - ib_off) : total_in;
        for (uint32_t c = lane; c < IB / 16; c += 64) {
          const uint64_t o = A + 16u * c;
          uint4 v;
          if (pl_aligned && o + 16 <= a.payload_len) {
            v = *reinterpret_cast<const uint4*>(a.payload + o);
          } else {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (int t = 0; t < 16; ++t)
              if (o + t < a.payload_len) w[t >> 2] |= (uint32_t)a.payload[o + t] << (8 * (t & 3));
            v = make_uint4(w[0], w[1], w[2], w[3]);
          }
          reinterpret_cast<uint4*>(L.ibuf)[c] = v;
        }
        if (fin && lane < 4) {
          const uint32_t t = plen + (uint32_t)lane;
          if (t >= ib_lo && t < ib_hi) L.ibuf[ib_off + (t - ib_lo)] = lane < 2 ? 0x00u : 0xffu;
        }
      };
      auto in_byte = [&](uint32_t i) -> uint32_t {  // i < total_in
        if (i < ib_lo || i >= ib_hi) restage(i);
        return uni(L.ibuf[ib_off + (i - ib_lo)]);
      };
      // pull bytes until `n` bits are held; false when the frame's input is exhausted
      auto need = [&](int n) -> bool {
        while (bits < n) {
          if (ip >= total_in) return false;
          hold |= (uint64_t)in_byte(ip++) << bits;
          bits += 8;
        }
        return true;
      };
      auto drop = [&](int n) {
        hold >>= n;
        bits -= n;
      };
      // n input bytes from ip straight to the output (stored blocks, a finished stream)
      auto copy_in = [&](uint32_t n) {
        while (n) {
          if (pos - flushed >= FLUSH_AT && !flush()) { err = E_CAP; return; }
          if (ip < ib_lo || ip >= ib_hi) restage(ip);
          uint32_t m = ib_hi - ip;
          if (m > n) m = n;
          if (m > 4096u) m = 4096u;
          const uint32_t base = ib_off + (ip - ib_lo);
          for (uint32_t t = lane; t < m; t += 64) L.ring[ri(pos + t)] = L.ibuf[base + t];
          pos += m;
          ip += m;
          n -= m;
        }
      };
      auto raw_rest = [&]() { copy_in(total_in - ip); };

      // A single-frame message met in the clean state k_infl_tok assumed: replay its
      // tokens instead of decoding.
      bool tok_use = false;
      const uint64_t tk = a.tmap ? (uint64_t)a.tmap[k] : k;  // frame k in the pre-decode's list
      if (a.tstat && tk != 0xFFFFFFFFull && !finished && !compressing && fin && !replay &&
          (op == WSG_OP_TEXT || op == WSG_OP_BINARY) && mode == M_HEAD && bits == 0 && !last)
        tok_use = uni(a.tstat[tk].ok) != 0u;
      if (finished) {
        raw_rest();
      } else if (tok_use) {
        const uint32_t n_tok = uni(a.tstat[tk].n_tok), n_lit = uni(a.tstat[tk].n_lit);
        const uint32_t* const T = a.tok + tok_base(d.payload_off, tk);
        const uint64_t lb = lit_base(d.payload_off, tk);
        uint32_t li = 0, lw_lo = 0, lw_hi = 0, lw_off = 0;  // ibuf holds literal bytes [lw_lo, lw_hi) from lw_off
        auto lit_stage = [&](uint32_t i) {
          const uint64_t g = lb + i;
          const uint64_t A = g & ~(uint64_t)15;
          lw_off = (uint32_t)(g - A);
          lw_lo = i;
          lw_hi = (i + IB - lw_off) < n_lit ? (i + IB - lw_off) : n_lit;
          for (uint32_t c = lane; c < IB / 16; c += 64) {
            const uint64_t o = A + 16u * c;
            if (o + 16 <= a.lit_len) reinterpret_cast<uint4*>(L.ibuf)[c] = reinterpret_cast<const uint4*>(a.lit)[o >> 4];
          }
        };
        uint32_t nxt = (uint32_t)lane < n_tok ? T[lane] : 0u;
        for (uint32_t t0 = 0; t0 < n_tok && err == E_NONE; t0 += 64) {
          const uint32_t cur = nxt;
          if (t0 + 64 < n_tok) nxt = (t0 + 64 + (uint32_t)lane < n_tok) ? T[t0 + 64 + lane] : 0u;
          const uint32_t cnt = (n_tok - t0) < 64u ? (n_tok - t0) : 64u;
          for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t tk = (uint32_t)__builtin_amdgcn_readlane((int)cur, (int)j);
            pos = (int32_t)uni((uint32_t)pos);
            if (pos - flushed >= FLUSH_AT && !flush()) { err = E_CAP; break; }
            if (tk & 0x80000000u) {
              const uint32_t mlen = ((tk >> 16) & 255u) + 3u, md = (tk & 0x7fffu) + 1u;
              if ((int32_t)md > pos - wstart) { err = E_DATA; break; }  // "invalid distance too far back"
              if (md >= mlen && mlen <= 64u) {
                if ((uint32_t)lane < mlen) {
                  const uint8_t v = L.ring[ri(pos - (int32_t)md + lane)];
                  L.ring[ri(pos + lane)] = v;
                }
                pos += (int32_t)mlen;
              } else {
                copy_match(mlen, md);
              }
            } else {
              uint32_t run = tk;
              while (run) {
                if (li < lw_lo || li >= lw_hi) lit_stage(li);
                uint32_t m = lw_hi - li;
                if (m > run) m = run;
                const uint32_t base = lw_off + (li - lw_lo);
                for (uint32_t t = lane; t < m; t += 64) L.ring[ri(pos + (int32_t)t)] = L.ibuf[base + t];
                pos += (int32_t)m;
                li += m;
                run -= m;
                if (run && pos - flushed >= FLUSH_AT && !flush()) { err = E_CAP; break; }
              }
              if (err) break;
            }
          }
        }
      } else {
        // the inflate state machine: runs until the frame's input is exhausted
        bool more = true;
        while (more && err == E_NONE) {
          if (pos - flushed >= FLUSH_AT && !flush()) { err = E_CAP; break; }
          PROF_T(t_it);
#ifdef WSG_INFLATE_PROF
          const int mode0 = mode;
          if (mode0 == M_HEAD) PROF_CNT(14, 1);
#endif
          switch (mode) {
            case M_HEAD: {
              if (last) {  // after a final block: the stream is done
                mode = M_DONE;
                break;
              }
              if (!need(3)) { more = false; break; }
              last = (int)(hold & 1u);
              const int type = (int)((hold >> 1) & 3u);
              drop(3);
              if (type == 0) mode = M_STORED;
              else if (type == 1) {  // fixed tables
                for (int i = lane; i < 288; i += 64) L.lens[i] = i < 144 ? 8 : (i < 256 ? 9 : (i < 280 ? 7 : 8));
                lmax = build_tab(L.lroot, LROOT, &L.lit, L.lens, 288, T_LIT, lane);
                for (int i = lane; i < 32; i += 64) L.lens[i] = 5;
                dmax = build_tab(L.droot, DROOT, &L.dist, L.lens, 32, T_DIST, lane);
                mode = M_LEN;
              } else if (type == 2) mode = M_TABLE;
              else err = E_DATA;  // "invalid block type"
              break;
            }
            case M_STORED: {
              drop(bits & 7);  // to a byte boundary
              if (!need(32)) { more = false; break; }
              const uint32_t ln = (uint32_t)(hold & 0xffffu), nl = (uint32_t)((hold >> 16) & 0xffffu);
              if (ln != (nl ^ 0xffffu)) { err = E_DATA; break; }  // "invalid stored block lengths"
              drop(32);
              length = ln;
              mode = M_COPY;
              break;
            }
            case M_COPY: {
              if (length == 0) { mode = M_HEAD; break; }
              // bits is 0 here: the stored bytes come straight from the input
              if (ip >= total_in) { more = false; break; }
              uint32_t take = length;
              if (take > total_in - ip) take = total_in - ip;
              copy_in(take);
              length -= take;
              break;
            }
            case M_TABLE: {
              if (!need(14)) { more = false; break; }
              nlen = (int)(hold & 31u) + 257;
              ndist = (int)((hold >> 5) & 31u) + 1;
              ncode = (int)((hold >> 10) & 15u) + 4;
              drop(14);
              if (nlen > 286 || ndist > 30) { err = E_DATA; break; }  // "too many length or distance symbols"
              have = 0;
              mode = M_LENLENS;
              break;
            }
            case M_LENLENS: {
              while (have < ncode) {
                if (!need(3)) break;
                L.lens[kClenOrder[have++]] = (uint8_t)(hold & 7u);
                drop(3);
              }
              if (have < ncode) { more = false; break; }
              while (have < 19) L.lens[kClenOrder[have++]] = 0;
              cmax = build_tab<1>(L.lroot, CROOT, nullptr, L.lens, 19, T_CODES, lane);
              if (cmax < 0) { err = E_DATA; break; }  // "invalid code lengths set"
              have = 0;
              mode = M_CODELENS;
              break;
            }
            case M_CODELENS: {
              while (have < nlen + ndist) {
                uint32_t e = 0;
                bool ok;
                if (cmax == 0) {  // zlib's empty code table: 1 bit, value 0, no check
                  ok = need(1);
                  e = ent(1, 0, OP_LIT, 0);
                } else {
                  ok = tdec<1>(L.lroot, CROOT, nullptr, cmax, T_CODES, hold, bits, &e);
                  while (!ok) {
                    if (!need(bits + 1)) break;
                    ok = tdec<1>(L.lroot, CROOT, nullptr, cmax, T_CODES, hold, bits, &e);
                  }
                }
                if (!ok) break;  // more input needed
                const int nb = (int)e_len(e);
                const int sym = (int)e_val(e);
                if (sym < 16) {
                  drop(nb);
                  L.lens[have++] = (uint8_t)sym;
                  continue;
                }
                const int xb = sym == 16 ? 2 : (sym == 17 ? 3 : 7);
                if (!need(nb + xb)) break;
                drop(nb);
                int len = 0, copy;
                if (sym == 16) {
                  if (have == 0) { err = E_DATA; break; }  // "invalid bit length repeat"
                  len = L.lens[have - 1];
                  copy = 3 + (int)(hold & 3u);
                } else if (sym == 17) {
                  copy = 3 + (int)(hold & 7u);
                } else {
                  copy = 11 + (int)(hold & 127u);
                }
                drop(xb);
                if (have + copy > nlen + ndist) { err = E_DATA; break; }  // "invalid bit length repeat"
                for (int i = lane; i < copy; i += 64) L.lens[have + i] = (uint8_t)len;
                have += copy;
              }
              if (err) break;
              if (have < nlen + ndist) { more = false; break; }
              if (L.lens[256] == 0) { err = E_DATA; break; }  // "invalid code -- missing end-of-block"
              lmax = build_tab(L.lroot, LROOT, &L.lit, L.lens, nlen, T_LIT, lane);
              if (lmax < 0) { err = E_DATA; break; }  // "invalid literal/lengths set"
              dmax = build_tab(L.droot, DROOT, &L.dist, L.lens + nlen, ndist, T_DIST, lane);
              if (dmax < 0) { err = E_DATA; break; }  // "invalid distances set"
              mode = M_LEN;
              break;
            }
            case M_LEN: {
              // fast path: whole symbols from a 64-bit buffer while >= 8 input bytes of
              // the frame remain; on the way out the unused whole bytes go back, so the
              // byte-at-a-time path below sees zlib's lazy state
              if (bits < 8 && ip + 8 <= total_in) {
                hold &= (1ull << bits) - 1ull;
                PROF_T(t_fast);
                // whole dwords of the stage from here on: align to its 4-byte grid (the
                // stage grid is the absolute address's, so this holds across restages)
                while (((uint32_t)(src0 + ip)) & 3u) {
                  hold |= (uint64_t)in_byte(ip++) << bits;
                  bits += 8;
                }
                if (ip + 4 > ib_hi || ip < ib_lo) restage(ip);
                const uint32_t* const ib32 = reinterpret_cast<const uint32_t*>(L.ibuf);
                uint32_t nxt = ib32[(ib_off + (ip - ib_lo)) >> 2];  // prefetched: made uniform at use
                // + 32 bits (bits < 32); false when fewer than 4 input bytes of the frame remain
                auto refill = [&]() -> bool {
                  if (ip + 4 > total_in) return false;
                  hold |= (uint64_t)uni(nxt) << bits;
                  bits += 32;
                  ip += 4;
                  if (ip + 4 <= total_in) {
                    if (ip + 4 > ib_hi) restage(ip);
                    nxt = ib32[(ib_off + (ip - ib_lo)) >> 2];
                  }
                  return true;
                };
                for (;;) {
                  // the decoder registers are wave-uniform: keep them in SGPRs
                  hold = uni64(hold);
                  bits = (int)uni((uint32_t)bits);
                  pos = (int32_t)uni((uint32_t)pos);
                  ip = uni(ip);
                  // >= 32 bits at every lookup: a literal/length code and its extra bits fit
                  if (bits < 32) {
                    if (pos - flushed >= FLUSH_AT && !flush()) { err = E_CAP; break; }
                    if (!refill()) break;
                  }
                  PROF_T(t_sym);
                  uint32_t e = uni(L.lroot[(uint32_t)hold & ((1u << LROOT) - 1u)]);
                  if ((e & 0x700u) == 0u) {  // a literal (the common case first)
                    PROF_ACC(16, t_sym);
                    L.ring[ri(pos)] = (uint8_t)(e >> 16);
                    ++pos;
                    hold >>= (e & 15u);
                    bits -= (int)(e & 15u);
                    PROF_CNT(9, 1);
                    continue;
                  }
                  if (e_op(e) == OP_LONG) {
                    PROF_T(t_long);
                    int nb = 0;
                    const int sy = canon(L.lit, lmax, hold, bits, &nb);
                    e = sym_entry(T_LIT, (uint32_t)sy, (uint32_t)nb);
                    PROF_ACC(17, t_long);
                    PROF_CNT(18, 1);
                  }
                  const uint32_t eo = e_op(e);
                  if (eo == OP_BAD) { err = E_DATA; break; }  // "invalid literal/length code"
                  drop((int)e_len(e));
                  if (eo == OP_LIT) {
                    L.ring[ri(pos)] = (uint8_t)e_val(e);
                    ++pos;
                    continue;
                  }
                  PROF_T(t_m);
                  if (eo == OP_EOB) { mode = M_HEAD; break; }
                  const uint32_t lx = e_extra(e);
                  const uint32_t mlen = e_val(e) + (uint32_t)(hold & ((1ull << lx) - 1ull));
                  drop((int)lx);
                  // a distance code and its extra bits need up to 28 bits
                  if (bits < 28 && !refill()) {
                    length = mlen;  // the lazy path goes on at the distance
                    mode = M_DIST;
                    break;
                  }
                  uint32_t g = uni(L.droot[(uint32_t)hold & ((1u << DROOT) - 1u)]);
                  if (e_op(g) == OP_LONG) {
                    int nb = 0;
                    const int sy = canon(L.dist, dmax, hold, bits, &nb);
                    g = sym_entry(T_DIST, (uint32_t)sy, (uint32_t)nb);
                    PROF_CNT(19, 1);
                  }
                  if (e_op(g) == OP_BAD) { err = E_DATA; break; }  // "invalid distance code"
                  drop((int)e_len(g));
                  PROF_ACC(20, t_m);
                  PROF_T(t_c);
                  const uint32_t dx = e_extra(g);
                  const uint32_t md = e_val(g) + (uint32_t)(hold & ((1ull << dx) - 1ull));
                  drop((int)dx);
                  if ((int32_t)md > pos - wstart) { err = E_DATA; break; }  // "invalid distance too far back"
                  PROF_CNT(10, 1);
                  PROF_CNT(11, mlen);
                  if (md >= mlen && mlen <= 64u) {  // one chunk, no overlap
                    if ((uint32_t)lane < mlen) {
                      const uint8_t v = L.ring[ri(pos - (int32_t)md + lane)];
                      L.ring[ri(pos + lane)] = v;
                    }
                    pos += (int32_t)mlen;
                  } else {
                    copy_match(mlen, md);
                  }
                  PROF_ACC(21, t_c);
                  PROF_ACC(22, t_sym);
                }
                ip -= (uint32_t)(bits >> 3);
                bits &= 7;
                hold &= (1ull << bits) - 1ull;
                PROF_ACC(2, t_fast);
                if (err || mode != M_LEN) break;
              }
              PROF_CNT(13, 1);
              // one symbol, pulling bytes lazily
              uint32_t e = 0;
              bool ok = tdec(L.lroot, LROOT, &L.lit, lmax, T_LIT, hold, bits, &e);
              while (!ok) {
                if (!need(bits + 1)) break;
                ok = tdec(L.lroot, LROOT, &L.lit, lmax, T_LIT, hold, bits, &e);
              }
              if (!ok) { more = false; break; }
              const uint32_t eo = e_op(e);
              if (eo == OP_BAD) { err = E_DATA; break; }  // "invalid literal/length code"
              drop((int)e_len(e));
              if (eo == OP_LIT) {
                L.ring[ri(pos)] = (uint8_t)e_val(e);
                ++pos;
                break;
              }
              if (eo == OP_EOB) { mode = M_HEAD; break; }  // end of block
              length = e_val(e);
              extra = e_extra(e);
              mode = M_LENEXT;
              break;
            }
            case M_LENEXT: {
              if (extra) {
                if (!need((int)extra)) { more = false; break; }
                length += (uint32_t)(hold & ((1u << extra) - 1u));
                drop((int)extra);
              }
              mode = M_DIST;
              break;
            }
            case M_DIST: {
              uint32_t e = 0;
              bool ok = tdec(L.droot, DROOT, &L.dist, dmax, T_DIST, hold, bits, &e);
              while (!ok) {
                if (!need(bits + 1)) break;
                ok = tdec(L.droot, DROOT, &L.dist, dmax, T_DIST, hold, bits, &e);
              }
              if (!ok) { more = false; break; }
              if (e_op(e) == OP_BAD) { err = E_DATA; break; }  // "invalid distance code"
              drop((int)e_len(e));
              dist = e_val(e);
              extra = e_extra(e);
              mode = M_DISTEXT;
              break;
            }
            case M_DISTEXT: {
              if (extra) {
                if (!need((int)extra)) { more = false; break; }
                dist += (uint32_t)(hold & ((1u << extra) - 1u));
                drop((int)extra);
              }
              if ((int32_t)dist > pos - wstart) { err = E_DATA; break; }  // "invalid distance too far back"
              copy_match(length, dist);
              mode = M_LEN;
              break;
            }
            case M_DONE: {
              // the stream ended (ZlibDecoder.finished): the rest of the frame passes through
              finished = 1;
              drop(bits & 7);  // the partial byte's bits are discarded
              // whole bytes already pulled into hold are unused input: give them back
              ip -= (uint32_t)(bits >> 3);
              hold = 0;
              bits = 0;
              raw_rest();
              more = false;
              break;
            }
          }
#ifdef WSG_INFLATE_PROF
          if (mode0 <= M_CODELENS) PROF_ACC(3, t_it);
          else if (mode0 <= M_DISTEXT) PROF_ACC(4, t_it);
          else PROF_ACC(5, t_it);
#endif
        }
        if (err == E_NONE && mode == M_DONE && !finished) {
          finished = 1;
          raw_rest();
        }
      }
      if (err == E_DATA || err == E_CAP) {
        err_idx = delivered;
        err_end = fstart;
        break;
      }
      if (fin && a.no_context) has_dec = 0;  // decoder.event(ENDING); decoder = null (DeflateDecoder.java:107-110)
      const int32_t produced = pos - fstart;
      if (produced == 0) {  // no buffer came out (DeflateDecoder.java:122-131)
        const bool single_zero = plen == 1 && a.payload[src0] == 0;
        if (!single_zero) {
          err = E_NODATA;
          err_idx = delivered;
          err_end = fstart;
          break;
        }
      }
      if (!replay) {
        wsg_frame_desc o;
        o.payload_off = obase + (uint64_t)fstart;
        o.payload_len = (uint32_t)produced;
        o.opcode = (uint8_t)op;
        const uint32_t orsv = (rsv & 4u) ? (rsv ^ 4u) : rsv;  // rsvBits(): RSV1 cleared (:83-85)
        o.flags = (uint8_t)((fin << 7) | (orsv << 4) | WSG_DESC_INFLATED);
        o.status = 0;
        if (lane == 0) a.out_desc[k] = o;
      }
    } else if (!replay) {  // passed through unchanged (DeflateDecoder.java:140)
      wsg_frame_desc o = d;
      o.flags = (uint8_t)(d.flags & 0xF1u);
      o.status = 0;
      if (lane == 0) a.out_desc[k] = o;
    }
    // PerMessageDeflateDecoder.compressing (:94-104)
    if (op < 8u) {
      if (fin) compressing = 0;
      else if ((rsv & 4u) && (op == WSG_OP_TEXT || op == WSG_OP_BINARY)) compressing = 1;
    }
    if (!replay) ++delivered;
  }
  if (err == E_NONE && !flush()) err = E_CAP;
  // frames delivered before a data error keep their output (DeflateDecoder.java:122-131
  // fails only the frame at hand); the erroring frame's partial output is dropped
  if ((err == E_DATA || err == E_NODATA) && err_end > flushed && !flush_to(err_end)) err = E_CAP;
  __syncthreads();

  PROF_T(t_cm);
  wsg_session_result res = {delivered, 0u, 0u, 0};
  uint32_t rf = 0xffffffffu;
  if (err == E_CAP) {  // nothing committed: the caller retries with a larger region
    res.n_delivered = 0;
    res.error = WSG_E_INFLATE_CAPACITY;
  } else if (err != E_NONE) {
    res.n_delivered = err_idx;
    res.error = err == E_NODATA ? WSG_E_INFLATE_NO_DATA : WSG_E_INFLATE;
    res.close_code = WSG_CLOSE_PROTOCOL_ERROR;
    res.detail = err_idx;
  } else {
    // commit: at the start of a message left open, else at the end
    const bool open = compressing && snap_k >= 0;
    const int32_t P = open ? snap_pos : pos;
    const int32_t W = open ? snap_wstart : wstart;
    const int chas = open ? snap_has : has_dec, cfin = open ? snap_fin : finished;
    wsg_inflate_state st = st0;
    st.compressing = open ? 0 : (uint8_t)compressing;
    st.has_decoder = (uint8_t)chas;
    st.finished = (uint8_t)cfin;
    st.window_len = 0;
    st.window_phase = 0;
    if (chas && !cfin) {
      const int32_t n = (P - W) < (int32_t)WSG_INFLATE_WINDOW ? (P - W) : (int32_t)WSG_INFLATE_WINDOW;
      // the new image: slot j holds position q(j) in [P - 32768, P).  q < 0: the old
      // image already has it (same phase); q >= pos - 32768: the ring; else this
      // batch's output in HBM (flushed).  Slots below the history are don't-care.
      const uint32_t nph = ri(P);
      const int32_t ring_lo = pos - (int32_t)WSG_INFLATE_WINDOW;
      const int32_t lo = (P - n) > 0 ? (P - n) : 0;
      __threadfence_block();
      for (uint32_t c = lane; c < WSG_INFLATE_WINDOW / 16; c += 64) {
        const uint32_t j0 = 16u * c;
        const int32_t q0 = P - (int32_t)WSG_INFLATE_WINDOW + (int32_t)((j0 - nph) & WMASK);
        const bool wraps = nph > j0 && nph < j0 + 16u;
        if (!wraps && q0 + 16 <= lo) continue;  // nothing to write
        if (!wraps && win_aligned && q0 >= 0 && q0 >= ring_lo) {
          reinterpret_cast<uint4*>(win)[c] = reinterpret_cast<const uint4*>(L.ring)[c];
          continue;
        }
        for (uint32_t t = 0; t < 16u; ++t) {
          const uint32_t j = j0 + t;
          const int32_t q = P - (int32_t)WSG_INFLATE_WINDOW + (int32_t)((j - nph) & WMASK);
          if (q < lo) continue;
          win[j] = q >= ring_lo ? L.ring[j] : out[q];
        }
      }
      st.window_len = (uint16_t)n;
      st.window_phase = (uint16_t)nph;
    }
    if (open) rf = (uint32_t)snap_k;
    if (lane == 0) a.state[s] = st;
  }
  if (lane == 0) {
    a.result[s] = res;
    a.replay_from[s] = rf;
  }
  PROF_ACC(7, t_cm);
  PROF_ACC(0, t_all);
#ifdef WSG_INFLATE_PROF
  if (lane == 0)
    for (int i = 0; i < 24; ++i) atomicAdd(&g_infl_prof[i], (unsigned long long)pf_[i]);
#endif
}

// ---------------------------------------------------------------------------------
// Parallel token replay (k_infl_fast).  A session whose compressed messages in this
// batch k_infl_tok all decoded cleanly (whole messages, one frame or several), met in
// the clean state (no message open, no final block seen), needs no serial decoder and
// no LDS window (its other frames pass through): per message, in chunks of FC output
// bytes, the threads expand the tokens into one descriptor per output byte (a literal,
// or the absolute session position it copies: a back-reference byte i of (length,
// distance) at p copies p - distance + i mod distance) — each token marks its first
// byte and the 64-byte row starts it covers, and a lane a byte finds its token by a
// max-scan of its row's marks, so the work is the chunk's bytes whatever the match
// lengths — chase the copies that land inside the chunk through LDS, gather the ones
// that land before it from the session's output in HBM (or the carried window image)
// with no branch a byte, and store the chunk.  Every output byte is resolved independently, so nothing serialises on a
// window round trip; a session is one 256-thread workgroup (4 waves, 16 KiB of LDS).  A
// session it cannot finish (a distance too far back, capacity, any frame that does
// not qualify) is left to k_inflate, which runs the serial decoder for exactly the
// sessions without fast_done and overwrites whatever this kernel wrote.
// ---------------------------------------------------------------------------------
namespace {

#ifndef WSG_FAST_GU
#define WSG_FAST_GU 16  // gather loads in flight a thread (of the FC / FNT bytes it resolves)
#endif
#ifndef WSG_FAST_CU
#define WSG_FAST_CU 8  // window-commit dwords in flight a thread
#endif
#ifndef WSG_FAST_CHUNK
#define WSG_FAST_CHUNK 4096
#endif
constexpr uint32_t FC = WSG_FAST_CHUNK;   // output bytes resolved per chunk (a multiple of FNT)
// the replay's token records pack (start - c0 + 512) into 13 bits and a literal's lb
// index - jj + 8192 into 14: both must stay below their field for every chunk size built
static_assert(FC + 512u + 258u < 8192u, "WSG_FAST_CHUNK too large for the 13-bit match start field");
static_assert(FC + 4u < 8192u, "WSG_FAST_CHUNK too large for the 14-bit literal offset field");
constexpr uint32_t FD_LIT = 0x80000000u;  // descriptor: a resolved byte (bits 0-7)
constexpr int32_t FD_BIAS = 32768;        // descriptor: position + FD_BIAS (history positions are >= -32768)

constexpr int FNT = 256;  // threads per session (4 waves)
#ifndef WSG_FAST_TPT
#define WSG_FAST_TPT 2  // tokens a thread a round (records: 8 B a token of LDS; 3 spills, 4 holds 5 sessions a CU)
#endif
constexpr int FTPT = WSG_FAST_TPT;
#ifndef WSG_FAST_WAVES
#define WSG_FAST_WAVES 6  // waves a SIMD: the register budget (80 VGPRs) that keeps 6 sessions a CU
#endif

// block-wide exclusive sum of a packed (hi, lo) pair of 32-bit counts, and the totals;
// no trailing barrier: the caller alternates two wsum buffers
__device__ __forceinline__ uint64_t blk_excl_add2(uint64_t v, uint64_t* total, uint64_t* wsum) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t inc = v;
  inc += dpp_u64<DPP_ROW_SHR1, 0xf>(inc, 0ull);
  inc += dpp_u64<DPP_ROW_SHR2, 0xf>(inc, 0ull);
  inc += dpp_u64<DPP_ROW_SHR4, 0xf>(inc, 0ull);
  inc += dpp_u64<DPP_ROW_SHR8, 0xf>(inc, 0ull);
  inc += dpp_u64<DPP_ROW_BCAST15, 0xa>(inc, 0ull);
  inc += dpp_u64<DPP_ROW_BCAST31, 0xc>(inc, 0ull);
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < FNT / 64; ++w) {
    pre += w < wid ? wsum[w] : 0ull;
    tot += wsum[w];
  }
  *total = tot;
  return pre + inc - v;
}

__global__ __launch_bounds__(FNT) __attribute__((amdgpu_waves_per_eu(WSG_FAST_WAVES))) void k_infl_fast(InflArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t fd[FC + 4];  // (+ a slot the marks of tokens outside the chunk go to)
  __shared__ uint32_t lbuf[FC / 4 + 2];  // the chunk's literal bytes (at most FC), from a dword boundary
  // a round's token records (below), its wave sums and the token holding byte c1; two of
  // each, rounds alternating, so a round needs two barriers (sums, records) and not four
  __shared__ uint32_t tokrec[2][FTPT * FNT];
  __shared__ uint64_t wsum2[2][FNT / 64];
  __shared__ uint32_t xs[3][4];  // (row 2: the spare the other lanes write)
  __shared__ uint32_t xbad;  // a lane of the chunk's rounds met a distance too far back
  const int lane = threadIdx.x;  // (the block's thread: FNT per session)
  const uint32_t s = blockIdx.x;
  if (s >= a.n_sessions) return;
  const uint32_t f0 = a.session_first[s], f1 = a.session_first[s + 1];
  const uint64_t obase = a.out_off[s], ocap64 = a.out_off[s + 1] - a.out_off[s];
  const int64_t ocap = ocap64 < (uint64_t)POS_LIMIT ? (int64_t)ocap64 : (int64_t)POS_LIMIT;
  const wsg_inflate_state st0 = a.state[s];
  // the state must be clean (no message open, no final block seen); every frame is
  // checked as it comes (a session that fails a check is left to k_inflate)
  if (st0.compressing || (st0.has_decoder && st0.finished)) {
    if (lane == 0) a.fast_done[s] = 0;
    return;
  }
  FPROF_T(f_all);
  const uint8_t* const win = a.window + (uint64_t)s * WSG_INFLATE_WINDOW;
  uint8_t* const out = a.out + obase;
  const int wl0 = (st0.has_decoder && !st0.finished) ? (int)(st0.window_len < WSG_INFLATE_WINDOW ? st0.window_len : WSG_INFLATE_WINDOW) : 0;
  const uint32_t ph = wl0 ? (uint32_t)st0.window_phase & WMASK : 0u;
  // the session's output so far, read around L1 (bytes this wave stored a chunk ago)
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)ocap, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(win), 0, (int)WSG_INFLATE_WINDOW, 0x00020000);
  int has_dec = st0.has_decoder;
  int32_t pos = 0, wstart = -wl0;
  bool bad = false;
  int compressing = 0;
  for (uint32_t k = f0; k < f1 && !bad; ++k) {
    const wsg_frame_desc d = a.desc[k];
    const uint32_t op = d.opcode & 15u, fin = (d.flags >> 7) & 1u, rsv = (d.flags >> 4) & 7u;
    if (d.flags & WSG_DESC_REPLAY) { bad = true; break; }
    // PerMessageDeflateDecoder (:69-105): a TEXT/BINARY frame with RSV1 starts a compressed
    // message, its continuations belong to it; anything else passes through unchanged
    const bool start = (op == WSG_OP_TEXT || op == WSG_OP_BINARY) && (rsv & 4u);
    if (!start && !(op == WSG_OP_CONTINUATION && compressing)) {
      if (lane == 0) {
        wsg_frame_desc o = d;
        o.flags = (uint8_t)(d.flags & 0xF1u);
        o.status = 0;
        a.out_desc[k] = o;
      }
      if (op < 8u && fin) compressing = 0;
      continue;
    }
    if (start && compressing) { bad = true; break; }
    // the message's pre-decode (its start frame's lane wrote every frame's stats)
    const uint64_t tk = a.tmap ? (uint64_t)a.tmap[k] : k;  // frame k in the pre-decode's list
    if (tk == 0xFFFFFFFFull) { bad = true; break; }
    const InflTokStat ts = a.tstat[tk];
    if (!ts.ok || !ts.out_len || (int64_t)pos + ts.out_len > ocap) { bad = true; break; }
    if (!has_dec) {  // new ZlibDecoder(RAW): a fresh history (DeflateDecoder.java:80-93)
      has_dec = 1;
      wstart = pos;
    }
    const int32_t P0 = pos;
    const uint32_t L = ts.out_len, n_tok = ts.n_tok;
    const uint32_t* const T = a.tok + tok_base(d.payload_off, tk);
    const uint8_t* const lit = a.lit + lit_base(d.payload_off, tk);
    uint32_t tt = 0, t_off = 0, t_li = 0;  // the first token not fully emitted: index, output offset, literal index
    uint32_t l_first = 0;                  // the index of the chunk's first literal
    for (uint32_t c0 = 0; c0 < L && !bad; c0 += FC) {
      const uint32_t c1 = c0 + FC < L ? c0 + FC : L, n = c1 - c0;
      const int32_t C0 = P0 + (int32_t)c0;  // absolute position of the chunk's first byte
      FPROF_T(f_ex);
      // 0. the chunk's literal bytes into LDS (one coalesced read; the expansion below
      //    reads a literal run's bytes one by one)
      const uint64_t lg = (uint64_t)(lit - a.lit) + l_first;  // the chunk's first literal, in a.lit
      const uint64_t lw0 = lg >> 2;
      // only the message's literals from l_first on (at most a chunk's worth): text is mostly
      // matches, so this is a fraction of the FC bytes the buffer holds
      const uint32_t lrem = ts.n_lit > l_first ? ts.n_lit - l_first : 0u;
      const uint32_t lw_n = (lrem < FC ? lrem : FC) / 4u + 2u;
      for (uint32_t w = (uint32_t)lane; w < lw_n; w += FNT)
        lbuf[w] = (lw0 + w) * 4 + 4 <= a.lit_len ? reinterpret_cast<const uint32_t*>(a.lit)[lw0 + w] : 0u;
      const uint32_t lsh = (uint32_t)(lg & 3u) - l_first;  // literal index i is byte i + lsh of lbuf
      for (uint32_t w = (uint32_t)lane; w < FC / 4; w += FNT) reinterpret_cast<uint4*>(fd)[w] = make_uint4(0u, 0u, 0u, 0u);
      if (threadIdx.x == 0) xbad = 0u;
      __syncthreads();
      const uint8_t* const lb = reinterpret_cast<const uint8_t*>(lbuf);
      // 1. expand the tokens that overlap [c0, c1) into fd, 2 * FNT tokens a round.  A
      //    block scan of a thread's two token lengths places its tokens; each token
      //    leaves a record (below) and its round index at its first byte in the chunk
      //    and at every 64-byte row start it covers (fd was cleared: the other bytes
      //    hold 0, the round's first token); then a wave resolves whole rows, a lane a
      //    byte, the byte's token being the max-scan of the row's marks up to it.  The
      //    work is the chunk's bytes, not a loop over each token's bytes.
      const int lw = threadIdx.x & 63, wv = threadIdx.x >> 6;
      uint32_t t = tt, o = t_off, li = t_li, rp = 0;
      bool crossed = false;
      const uint32_t tq = (uint32_t)FTPT * (uint32_t)lane;
      const uint32_t mb = (uint32_t)(P0 + (int32_t)c0 + FD_BIAS);  // a match's source, + jj - distance
      uint32_t nk[FTPT];
#pragma unroll
      for (int i = 0; i < FTPT; ++i) nk[i] = t + tq + i < n_tok ? T[t + tq + i] : 0u;
      while (t < n_tok && o < c1) {
        uint32_t kk[FTPT], ll[FTPT], lsum = 0u, lit_sum = 0u;
#pragma unroll
        for (int i = 0; i < FTPT; ++i) {
          const bool v = t + tq + i < n_tok;
          kk[i] = v ? nk[i] : 0u;
          const uint32_t tn = t + (uint32_t)(FTPT * FNT) + tq + i;  // the next round's, read ahead
          nk[i] = tn < n_tok ? T[tn] : 0u;
          const bool ism = (kk[i] & 0x80000000u) != 0;
          ll[i] = !v ? 0u : (ism ? ((kk[i] >> 16) & 255u) + 3u : kk[i]);
          lsum += ll[i];
          lit_sum += ism ? 0u : ll[i];
        }
        uint32_t* const rec_r = tokrec[rp];
        uint32_t* const xs_r = xs[rp];
        if (threadIdx.x == 0) xs_r[0] = 0xffffffffu;
        uint64_t tot;
        const uint64_t ex = blk_excl_add2(((uint64_t)lsum << 32) | lit_sum, &tot, wsum2[rp]);
        const uint32_t tot_len = uni((uint32_t)(tot >> 32)), tot_lit = uni((uint32_t)tot);
        uint32_t to = o + (uint32_t)(ex >> 32), tli = li + (uint32_t)ex;
#pragma unroll
        for (int i = 0; i < FTPT; ++i) {
          const uint32_t tk = kk[i], len = ll[i];
          const bool v = t + tq + i < n_tok, ism = (tk & 0x80000000u) != 0;
          const uint32_t idx = tq + (uint32_t)i;
          const bool here = v && len && to < c1 && to + len > c0;  // has bytes in the chunk
          const uint32_t toc = to - c0;                             // (mod 2^32: may be "negative")
          // the record (read only for a token with bytes in the chunk, whose fields fit): a
          // match: flag | distance - 1 | (start - c0 + 512) << 15; a literal run: the lb
          // index of chunk byte jj's literal, minus jj, + 8192 (14 bits)
          uint32_t rec;
          if (ism) {
            const uint32_t md = (tk & 0x7fffu) + 1u;
            if (here && (int32_t)md > P0 + (int32_t)to - wstart) xbad = 1u;  // "invalid distance too far back"
            rec = 0x80000000u | (md - 1u) | (((toc + 512u) & 0x1fffu) << 15);
          } else {
            rec = (tli + lsh - toc + 8192u) & 0x3fffu;
          }
          rec_r[idx] = rec;
          {  // (no exec-mask branch: a token outside the chunk marks the spare slot)
            const uint32_t s = !here ? FC : (to > c0 ? toc : 0u), e = here ? (to + len < c1 ? to + len : c1) - c0 : 0u;
            fd[s] = idx;
            for (uint32_t r = (s + 64u) & ~63u; r < e; r += 64u) fd[r] = idx;
          }
          {  // the token holding byte c1 (one at most): the next chunk starts from it (the
             // others write a spare row: no exec-mask branch)
            uint32_t* const xw = (v && to <= c1 && to + len > c1) ? xs_r : xs[2];
            xw[0] = idx;
            xw[1] = to;
            xw[2] = tli;
            xw[3] = ism ? tli : tli + (c1 - to);  // the next chunk's first literal
          }
          to += len;
          tli += ism ? 0u : len;
        }
        __syncthreads();
        const uint32_t xf = uni(xs_r[0]), xo = uni(xs_r[1]), xl = uni(xs_r[2]), xlf = uni(xs_r[3]);
        const uint32_t rs = (o > c0 ? o : c0) - c0;
        const uint32_t re = (o + tot_len < c1 ? o + tot_len : c1) - c0;
        for (uint32_t row = (rs >> 6) + (uint32_t)wv; (row << 6) < re; row += FNT / 64) {
          const uint32_t jj = (row << 6) + (uint32_t)lw;
          const bool in = jj >= rs && jj < re;
          // (read and written back by every lane, no exec-mask branch: a lane outside the
          // round's bytes rewrites what it read — the rounds either side are past a barrier)
          const uint32_t orig = fd[jj];
          uint32_t m = in ? orig : 0u;
          m = max(m, dpp_u32<DPP_ROW_SHR1, 0xf>(m, 0u));
          m = max(m, dpp_u32<DPP_ROW_SHR2, 0xf>(m, 0u));
          m = max(m, dpp_u32<DPP_ROW_SHR4, 0xf>(m, 0u));
          m = max(m, dpp_u32<DPP_ROW_SHR8, 0xf>(m, 0u));
          m = max(m, dpp_u32<DPP_ROW_BCAST15, 0xa>(m, 0u));
          m = max(m, dpp_u32<DPP_ROW_BCAST31, 0xc>(m, 0u));
          {  // (no branch a byte: literal and match values both formed, one kept)
            const uint32_t rec = rec_r[m];
            const bool ism = (rec & 0x80000000u) != 0;
            const uint32_t md = (rec & 0x7fffu) + 1u;
            const uint32_t toc = ((rec >> 15) & 0x1fffu) - 512u;
            const uint32_t x = jj - toc;  // the byte's index in its match
            const uint32_t lv = FD_LIT | lb[ism || !in ? 0u : (rec & 0x3fffu) - 8192u + jj];
            const uint32_t base = mb - md;
            uint32_t v = ism ? base + jj : lv;
            if (in && ism && x >= md) v = base + toc + x % md;  // (rare: a match longer than its distance)
            fd[jj] = in ? v : orig;
          }
        }
        if (xf != 0xffffffffu) {  // the chunk ends inside token xf
          tt = t + xf;
          t_off = xo;
          t_li = xl;
          l_first = xlf;
          crossed = true;
          break;
        }
        rp ^= 1u;  // (no barrier: the next round writes the other records, sums and xs)
        t += (uint32_t)(FTPT * FNT);
        o += tot_len;
        li += tot_lit;
      }
      if (!crossed) {
        tt = t < n_tok ? t : n_tok;
        t_off = o;
        t_li = li;
        l_first = li;
      }
      __syncthreads();
      if (uni(xbad)) {
        bad = true;
        break;
      }
      FPROF_ACC(0, f_ex);
      FPROF_T(f_ch);
      // 2. chase copies inside the chunk: a byte's source precedes it, so a chain
      //    ends at a literal or at a byte before the chunk (kept as a position)
#pragma unroll
      for (int u = 0; u < (int)(FC / FNT); ++u) {
        // the first hop unmasked (a byte with no source in the chunk re-reads itself), the
        // rest of a chain (rarer) by the loop; fd read and written unmasked (j < FC)
        const uint32_t j = (uint32_t)FNT * u + (uint32_t)lane;
        uint32_t v = fd[j];
        v = j < n ? v : FD_LIT;
        const bool p1 = !(v & FD_LIT) && (int32_t)v - FD_BIAS >= C0;
        const uint32_t h = fd[p1 ? (uint32_t)((int32_t)v - FD_BIAS - C0) : j];
        v = p1 ? h : v;
        while (!(v & FD_LIT) && (int32_t)v - FD_BIAS >= C0) v = fd[(int32_t)v - FD_BIAS - C0];
        fd[j] = v;
      }
      __syncthreads();
      FPROF_ACC(1, f_ch);
      FPROF_T(f_ga);
      // 3. gather the bytes that come from before the chunk: this batch's output (HBM),
      //    or the window carried in
      // a thread's FC / FNT bytes, WSG_FAST_GU loads in flight at once
#pragma unroll
      for (int u0 = 0; u0 < (int)(FC / FNT); u0 += WSG_FAST_GU) {
        constexpr int GU = WSG_FAST_GU;
        uint32_t v[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          const uint32_t j = (uint32_t)FNT * (u0 + u) + (uint32_t)lane;
          v[u] = u0 + u < (int)(FC / FNT) ? fd[j] : FD_LIT;  // (read unmasked: j < FC)
          v[u] = j < n ? v[u] : FD_LIT;
          // no branch a byte (a branch each cost more than the loads): both loads are
          // issued, the one not wanted at an offset out of its buffer's range (reads 0)
          const bool isp = !(v[u] & FD_LIT);
          const int32_t q = (int32_t)v[u] - FD_BIAS;
          const uint32_t oq = isp && q >= 0 ? (uint32_t)q : 0xffffffffu;
          uint32_t b = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rout, oq, 0, 1);
          if (wl0) {  // (session-uniform) a carried window
            const uint32_t wq = isp && q < 0 ? (((uint32_t)q + ph) & WMASK) : 0xffffffffu;
            b |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rwin, wq, 0, 1);
          }
          v[u] = isp ? (FD_LIT | b) : v[u];
        }
#pragma unroll
        for (int u = 0; u < GU; ++u) {
          const uint32_t j = (uint32_t)FNT * (u0 + u) + (uint32_t)lane;
          if (u0 + u < (int)(FC / FNT)) fd[j] = v[u];  // (unmasked: past n it is unused)
        }
      }
      __syncthreads();
      FPROF_ACC(2, f_ga);
      FPROF_T(f_st);
      // 4. store the chunk: head bytes to a 4-B boundary, dwords, tail bytes
      uint8_t* const dst = out + C0;
      uint32_t head = (uint32_t)((4u - (uint32_t)((uintptr_t)dst & 3u)) & 3u);
      if (head > n) head = n;
      if ((uint32_t)lane < head) dst[lane] = (uint8_t)fd[lane];
      const uint32_t nw = (n - head) >> 2;
#pragma unroll
      for (int q = 0; q < (int)(FC / 4 / FNT); ++q) {  // (descriptors read unmasked: b + 3 < FC + 4)
        const uint32_t w = (uint32_t)FNT * q + (uint32_t)lane, b = head + 4u * w;
        const uint32_t x = (fd[b] & 0xffu) | ((fd[b + 1] & 0xffu) << 8) | ((fd[b + 2] & 0xffu) << 16) | ((fd[b + 3] & 0xffu) << 24);
        if (w < nw) reinterpret_cast<uint32_t*>(dst + head)[w] = x;
      }
      const uint32_t tb = head + 4u * nw;
      if ((uint32_t)lane < n - tb) dst[tb + lane] = (uint8_t)fd[tb + lane];
      // the stores complete before the next chunk gathers from them
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __syncthreads();
      FPROF_ACC(3, f_st);
    }
    if (bad) break;
    pos += (int32_t)L;
    if (lane == 0) {
      wsg_frame_desc o;
      o.payload_off = obase + (uint64_t)P0;
      o.payload_len = L;
      o.opcode = (uint8_t)op;
      const uint32_t orsv = (rsv & 4u) ? (rsv ^ 4u) : rsv;  // rsvBits(): RSV1 cleared (:83-85)
      o.flags = (uint8_t)((fin << 7) | (orsv << 4) | WSG_DESC_INFLATED);
      o.status = 0;
      a.out_desc[k] = o;
    }
    if (fin && a.no_context) has_dec = 0;  // decoder.event(ENDING); decoder = null (DeflateDecoder.java:107-110)
    compressing = fin ? 0 : 1;
  }
  if (compressing) bad = true;  // a message left open: k_inflate's snapshot and replay_from
  if (bad) {
    if (lane == 0) a.fast_done[s] = 0;
    return;
  }
  // commit (k_inflate's, with no message left open): the state and the window image
  wsg_inflate_state st = st0;
  st.compressing = 0;
  st.has_decoder = (uint8_t)has_dec;
  st.finished = 0;
  st.window_len = 0;
  st.window_phase = 0;
  if (has_dec) {
    const int32_t P = pos, nh = (P - wstart) < (int32_t)WSG_INFLATE_WINDOW ? (P - wstart) : (int32_t)WSG_INFLATE_WINDOW;
    const uint32_t nph = ((uint32_t)P + ph) & WMASK;
    const int32_t lo = (P - nh) > 0 ? (P - nh) : 0;
    // slot j holds position q(j) in [P - 32768, P); q < 0: the old image has it already
    uint8_t* const wout = a.window + (uint64_t)s * WSG_INFLATE_WINDOW;
    // a dword of slots a thread, 8 dwords (32 byte loads) in flight; slots whose position
    // is before lo keep the old image's byte
    uint32_t* const wout32 = reinterpret_cast<uint32_t*>(wout);
    const uint32_t mis = (uint32_t)((uintptr_t)out & 3u);  // the output's offset from a dword boundary
    for (uint32_t w0 = 0; w0 < WSG_INFLATE_WINDOW / 4; w0 += WSG_FAST_CU * FNT) {
      uint32_t v[WSG_FAST_CU];
#pragma unroll
      for (int u = 0; u < WSG_FAST_CU; ++u) {
        const uint32_t w = w0 + (uint32_t)FNT * u + (uint32_t)lane;
        // a slot dword whose 4 positions are consecutive output bytes (not across the
        // ring's end, none before lo): two aligned dword loads and a funnel, not 4 byte loads
        const uint32_t i0 = (4u * w - nph) & WMASK;
        const int32_t q0 = P - (int32_t)WSG_INFLATE_WINDOW + (int32_t)i0;
        const uint32_t sh = (uint32_t)(q0 + (int32_t)mis) & 3u;
        if (i0 <= WMASK - 3u && q0 >= lo && q0 >= (int32_t)sh) {
          const int32_t qa = q0 - (int32_t)sh;  // out + qa is dword-aligned
          const uint32_t l = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rout, (uint32_t)qa, 0, 1);
          const uint32_t h = sh ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rout, (uint32_t)qa + 4u, 0, 1) : 0u;
          v[u] = __builtin_amdgcn_alignbyte(h, l, sh);
          continue;
        }
        uint32_t x = 0;
        bool all = true;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int32_t q = P - (int32_t)WSG_INFLATE_WINDOW + (int32_t)((4 * w + b - nph) & WMASK);
          if (q >= lo) x |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rout, (uint32_t)q, 0, 1) << (8 * b);
          else all = false;
        }
        if (!all) {  // merge with the old image
          const uint32_t old = wout32[w];
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int32_t q = P - (int32_t)WSG_INFLATE_WINDOW + (int32_t)((4 * w + b - nph) & WMASK);
            if (q < lo) x |= old & (0xffu << (8 * b));
          }
        }
        v[u] = x;
      }
#pragma unroll
      for (int u = 0; u < WSG_FAST_CU; ++u) wout32[w0 + (uint32_t)FNT * u + (uint32_t)lane] = v[u];
    }
    st.window_len = (uint16_t)nh;
    st.window_phase = (uint16_t)nph;
  }
  if (lane == 0) {
    a.state[s] = st;
    wsg_session_result res = {f1 - f0, 0u, 0u, 0};
    a.result[s] = res;
    a.replay_from[s] = 0xffffffffu;
    a.fast_done[s] = 1;
  }
  FPROF_ACC(4, f_all);
}

// Message order for the pre-decode: a wave's 64 lanes step in lock-step until its
// longest message ends, so lanes are given messages of similar size (a counting sort
// of the frames by payload length, longest first; the order within a size bucket
// does not matter: every frame writes only its own regions).
constexpr uint32_t ORD_BUCKETS = 4096;
__device__ __forceinline__ uint32_t ord_bucket(uint32_t len) {
  const uint32_t b = len >> 4;
  return ORD_BUCKETS - 1u - (b < ORD_BUCKETS - 1u ? b : ORD_BUCKETS - 1u);
}

__global__ __launch_bounds__(256) void k_ord_hist(InflArgs a) {
  __shared__ uint32_t h[ORD_BUCKETS];
  for (uint32_t i = threadIdx.x; i < ORD_BUCKETS; i += 256) h[i] = 0;
  __syncthreads();
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < a.n_frames; k += (uint64_t)gridDim.x * 256)
    atomicAdd(&h[ord_bucket(a.desc[k].payload_len)], 1u);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ORD_BUCKETS; i += 256)
    if (h[i]) atomicAdd(&a.ord_cnt[i], h[i]);
}

__global__ __launch_bounds__(1024) void k_ord_scan(InflArgs a) {
  // exclusive scan of the bucket counts, 4 per thread
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x;
  uint32_t v[4], sum = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = a.ord_cnt[4 * t + i];
    sum += v[i];
  }
  part[t] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t x = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a.ord_cnt[4 * t + i] = run;
    run += v[i];
  }
}

// One frame a thread: ranks within the block's bucket from LDS counters, then one
// global atomic per (block, bucket) reserves the block's run of each bucket.  (A
// global atomic per frame serialised on the few buckets similar messages share:
// 342 us for 131 K frames.)
__global__ __launch_bounds__(256) void k_ord_scatter(InflArgs a) {
  __shared__ uint32_t cnt[ORD_BUCKETS];
  for (uint32_t i = threadIdx.x; i < ORD_BUCKETS; i += 256) cnt[i] = 0;
  __syncthreads();
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = k < a.n_frames;
  const uint32_t b = live ? ord_bucket(a.desc[k].payload_len) : 0u;
  const uint32_t r = live ? atomicAdd(&cnt[b], 1u) : 0u;
  __syncthreads();
  // the first frame of each bucket in the block reserves the bucket's run
  if (live && r == 0) cnt[b] = atomicAdd(&a.ord_cnt[b], cnt[b]);
  __syncthreads();
  if (live) a.order[cnt[b] + r] = (uint32_t)k;
}

}  // namespace

void launch_infl_fast(const InflArgs& a, hipStream_t s) {
  if (a.n_sessions && a.tstat && a.fast_done) hipLaunchKernelGGL(k_infl_fast, dim3(a.n_sessions), dim3(FNT), 0, s, a);
}

void launch_infl_tok(const InflArgs& a, hipStream_t s) {
  if (!a.n_lanes || !a.n_frames) return;
  if (a.order) {
    const uint32_t g = (uint32_t)((a.n_frames + 255) / 256 < 1024 ? (a.n_frames + 255) / 256 : 1024);
    (void)hipMemsetAsync(a.ord_cnt, 0, ORD_BUCKETS * sizeof(uint32_t), s);  // errors show at the launch check
    hipLaunchKernelGGL(k_ord_hist, dim3(g), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_ord_scan, dim3(1), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_ord_scatter, dim3((uint32_t)((a.n_frames + 255) / 256)), dim3(256), 0, s, a);
  }
  if (a.split)
    hipLaunchKernelGGL(k_infl_tok<true>, dim3((a.n_lanes + 63) / 64), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_infl_tok<false>, dim3((a.n_lanes + 63) / 64), dim3(64), 0, s, a);
}
uint64_t infl_ord_words(uint64_t n_frames) { return n_frames + ORD_BUCKETS; }

uint64_t infl_tok_words(uint64_t payload_len, uint64_t n_frames) { return payload_len + (uint64_t)TOK_SLACK * n_frames + 64; }
uint64_t infl_lit_bytes(uint64_t payload_len, uint64_t n_frames) {
  return 3 * payload_len + (uint64_t)TOK_SLACK * n_frames + 256;
}
uint64_t infl_tab_bytes() { return sizeof(LaneTab); }

void launch_inflate(const InflArgs& a, hipStream_t s) {
  if (a.n_sessions) hipLaunchKernelGGL(k_inflate, dim3(a.n_sessions), dim3(64), 0, s, a);
}

}  // namespace ws
