// inflate.hip — permessage-deflate decode on gfx950: PerMessageDeflateDecoder
// (PerMessageDeflateDecoder.java:68-105) over DeflateDecoder (DeflateDecoder.java:
// 78-141) over a raw ZlibDecoder (ZlibDecoder.java:180-280, java.util.zip.Inflater,
// i.e. zlib's inflate, RFC 1951).
//
// DEFLATE is a serial bit stream per session (Huffman codes, back-references into
// a 32 KiB window that persists across messages unless no_context), so the unit
// of parallelism is the session: one 64-lane workgroup per session, the sessions
// of a batch in parallel.  Inside a workgroup the decoder is uniform code (every
// lane runs the same state machine on the same LDS data); the lanes split the
// work that is wide: refilling the input stage from HBM, long back-reference
// copies, flushing output from the LDS window ring to HBM, and the window carry.
//
// zlib semantics the reference depends on, reproduced exactly:
//   * bytes are pulled lazily: a symbol completes (and its output belongs to the
//     frame) when its last bit's byte is read; a frame's inflate call decodes as
//     far as its bytes allow (Java's Inflater loop until needsInput, ZlibDecoder
//     .java:223-241), the tail 00 00 FF FF of a final fragment is fed in the same
//     call (DeflateDecoder.java:96-99);
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

namespace ws {

namespace {

constexpr uint32_t WMASK = WSG_INFLATE_WINDOW - 1;
constexpr int IB = 2048;  // input stage bytes

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

// Canonical Huffman table in LDS (count per length, symbols by code order).
struct Huff {
  uint16_t cnt[16];
  uint16_t sym[320];
};

struct Lds {
  uint8_t ring[WSG_INFLATE_WINDOW];  // the inflate window / output stage
  uint8_t ibuf[IB];                  // input stage
  Huff lit, dist, clen;
  uint8_t lens[320];
  uint16_t offs[16];
};

// Build a table over n lengths; returns the longest code length (0: no codes),
// or -1 for an over-subscribed or (except a single 1-bit code of a LENS/DISTS
// table) incomplete set, as zlib's inflate_table decides.
__device__ int build(Huff& h, const uint8_t* length, int n, bool codes_type, uint16_t* offs) {
  for (int l = 0; l < 16; ++l) h.cnt[l] = 0;
  for (int s = 0; s < n; ++s) h.cnt[length[s]]++;
  int maxl = 15;
  while (maxl >= 1 && h.cnt[maxl] == 0) --maxl;
  if (maxl == 0) return 0;
  int left = 1;
  for (int l = 1; l <= 15; ++l) {
    left <<= 1;
    left -= h.cnt[l];
    if (left < 0) return -1;  // over-subscribed
  }
  if (left > 0 && (codes_type || maxl != 1)) return -1;  // incomplete
  offs[1] = 0;
  for (int l = 1; l < 15; ++l) offs[l + 1] = offs[l] + h.cnt[l];
  for (int s = 0; s < n; ++s)
    if (length[s]) h.sym[offs[length[s]]++] = (uint16_t)s;
  return maxl;
}

// Decode one symbol from the low `bits` bits of hold (first stream bit = code
// MSB).  >= 0: the symbol, *nb its length; -1: more bits needed; -2: no code of
// the table starts with these bits (zlib's invalid entry), *nb bits decide it.
__device__ __forceinline__ int decode(const Huff& h, int maxl, uint64_t hold, int bits, int* nb) {
  if (maxl == 0) {  // no codes at all: zlib's table of two invalid 1-bit entries
    if (bits < 1) return -1;
    *nb = 1;
    return -2;
  }
  int code = 0, first = 0, index = 0;
  for (int len = 1; len <= maxl; ++len) {
    if (len > bits) return -1;
    code |= (int)((hold >> (len - 1)) & 1u);
    const int count = h.cnt[len];
    if (code - count < first) {
      *nb = len;
      return h.sym[index + (code - first)];
    }
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  *nb = maxl;
  return -2;
}

}  // namespace

// One workgroup (one wave) per session.
__global__ __launch_bounds__(64) void k_inflate(InflArgs a) {
  __shared__ Lds L;
  const int lane = threadIdx.x;
  const uint32_t s = blockIdx.x;
  if (s >= a.n_sessions) return;
  const uint32_t f0 = a.session_first[s], f1 = a.session_first[s + 1];
  const uint64_t obase = a.out_off[s], ocap = a.out_off[s + 1] - a.out_off[s];
  const wsg_inflate_state st0 = a.state[s];
  uint8_t* const win = a.window + (uint64_t)s * WSG_INFLATE_WINDOW;

  // carry-in: the inflater's history sits at ring positions [-wl, 0)
  int compressing = st0.compressing, has_dec = st0.has_decoder, finished = st0.finished;
  const int wl0 = (has_dec && !finished) ? (int)(st0.window_len < WSG_INFLATE_WINDOW ? st0.window_len : WSG_INFLATE_WINDOW) : 0;
  for (int i = lane; i < wl0; i += 64) L.ring[(uint32_t)(i - wl0) & WMASK] = win[i];
  __syncthreads();

  int64_t pos = 0;            // output bytes of this batch (session region offset)
  int64_t flushed = 0;        // ring bytes [flushed, pos) not yet in HBM
  int64_t wstart = -wl0;      // position where the current inflater's history starts
  // inflater registers (persist across frames: one continuous stream)
  int mode = M_HEAD, last = 0;
  uint64_t hold = 0;
  int bits = 0;
  int lmax = 0, dmax = 0, cmax = 0;
  int nlen = 0, ndist = 0, ncode = 0, have = 0;
  uint32_t length = 0, dist = 0, extra = 0;
  // the message-start snapshot (a batch ending inside a message commits it)
  int snap_k = -1, snap_has = 0, snap_fin = 0;
  int64_t snap_pos = 0, snap_wstart = 0;
  int err = E_NONE;
  uint32_t err_idx = 0, delivered = 0;
  int64_t err_end = 0;        // on a data error: output of the frames delivered before it

  // flush ring bytes to HBM (all lanes); returns false past the region's end
  auto flush_to = [&](int64_t end) -> bool {
    if (end > (int64_t)ocap) return false;
    for (int64_t i = flushed + lane; i < end; i += 64) a.out[obase + (uint64_t)i] = L.ring[(uint32_t)i & WMASK];
    flushed = end;
    return true;
  };
  auto flush = [&]() -> bool { return flush_to(pos); };

  for (uint32_t k = f0; k < f1 && err == E_NONE; ++k) {
    const wsg_frame_desc d = a.desc[k];
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
      const int64_t fstart = pos;
      // the frame's input: its payload, then the tail 00 00 FF FF if final
      const uint64_t src0 = d.payload_off;
      const uint32_t plen = d.payload_len;
      const uint32_t total_in = plen + (fin ? 4u : 0u);
      uint32_t ip = 0;                 // bytes of this frame's input pulled
      uint32_t ib_lo = 0, ib_hi = 0;   // ibuf holds payload bytes [ib_lo, ib_hi)
      auto in_byte = [&](uint32_t i) -> uint32_t {  // i < total_in
        if (i >= plen) {
          const uint32_t t = i - plen;
          return t < 2 ? 0x00u : 0xffu;
        }
        if (i >= ib_hi || i < ib_lo) {  // refill the input stage (all lanes, coalesced)
          __syncthreads();
          ib_lo = i;
          ib_hi = i + IB < plen ? i + IB : plen;
          for (uint32_t j = ib_lo + lane; j < ib_hi; j += 64)
            L.ibuf[j - ib_lo] = (src0 + j < a.payload_len) ? a.payload[src0 + j] : 0u;
          __syncthreads();
        }
        return L.ibuf[i - ib_lo];
      };
      auto out_byte = [&](uint32_t b) {
        L.ring[(uint32_t)pos & WMASK] = (uint8_t)b;
        ++pos;
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
      // raw pass-through of the rest of the frame's input (a finished stream)
      auto raw_rest = [&]() {
        while (ip < total_in) {
          if (pos - flushed >= 8192 && !flush()) { err = E_CAP; return; }
          out_byte(in_byte(ip++));
        }
      };

      if (finished) {
        raw_rest();
      } else {
        // the inflate state machine: runs until the frame's input is exhausted
        bool more = true;
        while (more && err == E_NONE) {
          if (pos - flushed >= 8192 && !flush()) { err = E_CAP; break; }
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
                for (int i = 0; i < 144; ++i) L.lens[i] = 8;
                for (int i = 144; i < 256; ++i) L.lens[i] = 9;
                for (int i = 256; i < 280; ++i) L.lens[i] = 7;
                for (int i = 280; i < 288; ++i) L.lens[i] = 8;
                lmax = build(L.lit, L.lens, 288, false, L.offs);
                for (int i = 0; i < 32; ++i) L.lens[i] = 5;
                dmax = build(L.dist, L.lens, 32, false, L.offs);
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
              uint32_t take = length;
              if (ip >= total_in) { more = false; break; }
              if (take > total_in - ip) take = total_in - ip;
              if (take > 4096) take = 4096;
              for (uint32_t i = 0; i < take; ++i) out_byte(in_byte(ip++));
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
              cmax = build(L.clen, L.lens, 19, true, L.offs);
              if (cmax < 0) { err = E_DATA; break; }  // "invalid code lengths set"
              have = 0;
              mode = M_CODELENS;
              break;
            }
            case M_CODELENS: {
              while (have < nlen + ndist) {
                int nb = 0, sym;
                if (cmax == 0) {  // zlib's empty code table: 1 bit, value 0, no check
                  if (!need(1)) { sym = -1; } else { sym = 0; nb = 1; }
                } else {
                  sym = decode(L.clen, cmax, hold, bits, &nb);
                  while (sym == -1) {
                    if (!need(bits + 1)) break;
                    sym = decode(L.clen, cmax, hold, bits, &nb);
                  }
                }
                if (sym < 0) break;  // more input needed (an incomplete CODES set cannot be built)
                if (sym < 16) {
                  drop(nb);
                  L.lens[have++] = (uint8_t)sym;
                  continue;
                }
                const int xb = sym == 16 ? 2 : (sym == 17 ? 3 : 7);
                if (!need(nb + xb)) { sym = -1; break; }
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
                while (copy--) L.lens[have++] = (uint8_t)len;
              }
              if (err) break;
              if (have < nlen + ndist) { more = false; break; }
              if (L.lens[256] == 0) { err = E_DATA; break; }  // "invalid code -- missing end-of-block"
              lmax = build(L.lit, L.lens, nlen, false, L.offs);
              if (lmax < 0) { err = E_DATA; break; }  // "invalid literal/lengths set"
              dmax = build(L.dist, L.lens + nlen, ndist, false, L.offs);
              if (dmax < 0) { err = E_DATA; break; }  // "invalid distances set"
              mode = M_LEN;
              break;
            }
            case M_LEN: {
              // literals in a run, flushing as the stage fills
              for (int guard = 0; guard < 4096; ++guard) {
                int nb = 0;
                int sym = decode(L.lit, lmax, hold, bits, &nb);
                while (sym == -1) {
                  if (!need(bits + 1)) break;
                  sym = decode(L.lit, lmax, hold, bits, &nb);
                }
                if (sym == -1) { more = false; break; }
                if (sym == -2 || sym >= 286) { err = E_DATA; break; }  // "invalid literal/length code"
                drop(nb);
                if (sym < 256) {
                  out_byte((uint32_t)sym);
                  continue;
                }
                if (sym == 256) { mode = M_HEAD; break; }  // end of block
                length = kLenBase[sym - 257];
                extra = kLenExt[sym - 257];
                mode = M_LENEXT;
                break;
              }
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
              int nb = 0;
              int sym = decode(L.dist, dmax, hold, bits, &nb);
              while (sym == -1) {
                if (!need(bits + 1)) break;
                sym = decode(L.dist, dmax, hold, bits, &nb);
              }
              if (sym == -1) { more = false; break; }
              if (sym == -2 || sym >= 30) { err = E_DATA; break; }  // "invalid distance code"
              drop(nb);
              dist = kDistBase[sym];
              extra = kDistExt[sym];
              mode = M_DISTEXT;
              break;
            }
            case M_DISTEXT: {
              if (extra) {
                if (!need((int)extra)) { more = false; break; }
                dist += (uint32_t)(hold & ((1u << extra) - 1u));
                drop((int)extra);
              }
              if ((int64_t)dist > pos - wstart) { err = E_DATA; break; }  // "invalid distance too far back"
              // the copy: lanes in chunks that never read a byte of their own chunk
              const uint32_t step = dist < 64u ? dist : 64u;
              for (uint32_t b = 0; b < length; b += step) {
                const uint32_t i = b + (uint32_t)lane;
                if ((uint32_t)lane < step && i < length)
                  L.ring[(uint32_t)(pos + i) & WMASK] = L.ring[(uint32_t)(pos + i - dist) & WMASK];
                __syncthreads();
              }
              pos += length;
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
      const int64_t produced = pos - fstart;
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
    const int64_t P = open ? snap_pos : pos;
    const int64_t W = open ? snap_wstart : wstart;
    const int chas = open ? snap_has : has_dec, cfin = open ? snap_fin : finished;
    wsg_inflate_state st = st0;
    st.compressing = open ? 0 : (uint8_t)compressing;
    st.has_decoder = (uint8_t)chas;
    st.finished = (uint8_t)cfin;
    if (chas && !cfin) {
      const int64_t n = (P - W) < WSG_INFLATE_WINDOW ? (P - W) : WSG_INFLATE_WINDOW;
      // bytes [P-n, P): the ring holds [pos-32768, pos), earlier ones are in HBM (this
      // batch's output) or in the old window; the old window moves only downwards
      __threadfence_block();
      for (int64_t b = 0; b < n; b += 64) {
        const int64_t j = b + lane;
        uint32_t v = 0;
        if (j < n) {
          const int64_t q = P - n + j;
          if (q >= pos - (int64_t)WSG_INFLATE_WINDOW) v = L.ring[(uint32_t)q & WMASK];
          else if (q >= 0) v = a.out[obase + (uint64_t)q];
          else v = win[wl0 + q];
        }
        __syncthreads();
        if (j < n) win[j] = (uint8_t)v;
        __syncthreads();
      }
      st.window_len = (uint32_t)n;
    } else {
      st.window_len = 0;
    }
    if (open) rf = (uint32_t)snap_k;
    if (lane == 0) a.state[s] = st;
  }
  if (lane == 0) {
    a.result[s] = res;
    a.replay_from[s] = rf;
  }
}

void launch_inflate(const InflArgs& a, hipStream_t s) {
  if (a.n_sessions) hipLaunchKernelGGL(k_inflate, dim3(a.n_sessions), dim3(64), 0, s, a);
}

}  // namespace ws
