// deflate_core.h — permessage-deflate compression (PerMessageDeflateEncoder.java:55-99 over
// DeflateEncoder.java:62-104 over ZlibEncoder.java:223-287 over java.util.zip.Deflater) for
// the GPU: zlib's raw deflate (windowBits -15, memLevel 8, Z_DEFAULT_STRATEGY), one
// deflate(Z_SYNC_FLUSH) per frame, restated exactly so that every output byte equals the
// one zlib writes.  zlib itself is not in /root/reference (java.util.zip's native engine);
// the restatement follows zlib 1.2.11's deflate.c (fill_window, longest_match, deflate_fast,
// deflate_slow, deflate_stored for Z_SYNC_FLUSH) and trees.c (build_tree with its heap and
// depth tie-break, gen_bitlen with the overflow fix, gen_codes, scan_tree/send_tree,
// build_bl_tree, _tr_flush_block's stored/static/dynamic choice, compress_block), and is
// pinned against the system zlib driven exactly as Deflater drives it (oracle/deflate_ref.c).
//
// Two ways to run it, both exact:
//   * Serial: zlib's own loop over a session's window/head/prev (SerialState) — one lane a
//     session; the only form for levels 1-3 (deflate_fast inserts hash strings depending on
//     the matches it takes, so its hash chains are a product of the parse).
//   * Decomposed (levels 4-9, deflate_slow): every string is inserted in position order, so
//     the hash chain seen at any position is a function of the input alone.  The expensive
//     part — longest_match at every position, for both chain budgets (max_chain, and
//     max_chain >> 2 once prev_length >= good_match) — runs one lane a position
//     (match_at); the lazy-evaluation loop then replays deflate_slow's control flow over
//     those results (ParseCall), one lane a frame.  What deflate_slow reads beyond the data
//     (longest_match scans up to strstart + 258) is the window image zlib keeps: the bytes
//     after a frame's end are supplied per frame, before and after the one window slide
//     that can fall inside a frame's last 261 bytes (the parse knows which applies).
//
// Everything here is __host__ __device__ so the CPU test harness (tests/cpp/deflate_host.cpp)
// checks the decomposition against zlib without a GPU; the product runs it only on the GPU.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ZD_FN __host__ __device__ inline
#define ZD_MFN __host__ __device__ inline
#else
#define ZD_FN static inline
#define ZD_MFN inline
#endif

namespace zd {

enum : int {
    WSIZE = 32768, WMASK = WSIZE - 1, WINDOW_SIZE = 2 * WSIZE, HASH_MASK = 32767,
    MIN_MATCH = 3, MAX_MATCH = 258, MIN_LOOKAHEAD = MAX_MATCH + MIN_MATCH + 1,
    MAX_DIST = WSIZE - MIN_LOOKAHEAD, TOO_FAR = 4096, WIN_INIT = MAX_MATCH,
    LIT_BUFSIZE = 16384, SYM_END = LIT_BUFSIZE - 1,
    L_CODES = 286, D_CODES = 30, BL_CODES = 19, HEAP_SIZE = 2 * L_CODES + 1,
    MAX_BITS = 15, MAX_BL_BITS = 7, END_BLOCK = 256, REP_3_6 = 16, REPZ_3_10 = 17, REPZ_11_138 = 18,
    STRIP = 260   // window bytes kept after a frame's end (longest_match reads up to +258)
};

// configuration_table (deflate.c): good_length, max_lazy, nice_length, max_chain
struct Cfg { uint16_t good, lazy, nice, chain; };
ZD_FN Cfg level_cfg(int level) {
    switch (level) {
    case 1: return {4, 4, 8, 4};
    case 2: return {4, 5, 16, 8};
    case 3: return {4, 6, 32, 32};
    case 4: return {4, 4, 16, 16};
    case 5: return {8, 16, 32, 32};
    case 6: return {8, 16, 128, 128};
    case 7: return {8, 32, 128, 256};
    case 8: return {32, 128, 258, 1024};
    case 9: return {32, 258, 258, 4096};
    default: return {0, 0, 0, 0};
    }
}

ZD_FN uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) { return ((a << 10) ^ (b << 5) ^ c) & HASH_MASK; }
ZD_FN int flog2(uint32_t x) { return 31 - __builtin_clz(x); }

// _length_code / base_length / extra_lbits (trees.c tr_static_init) as formulas;
// lc = match length - 3
ZD_FN int len_code(int lc) {
    if (lc < 8) return lc;
    if (lc == 255) return 28;
    int e = flog2((uint32_t)lc) - 2;
    return 4 * e + 4 + ((lc >> e) & 3);
}
ZD_FN int len_extra(int code) { return (code < 8 || code == 28) ? 0 : (code - 4) >> 2; }
ZD_FN int len_base(int code) { return code < 8 ? code : code == 28 ? 0 : (4 + (code & 3)) << ((code - 4) >> 2); }
// d_code / base_dist / extra_dbits; d = distance - 1
ZD_FN int dist_code(int d) {
    if (d < 4) return d;
    int l = flog2((uint32_t)d);
    return 2 * l + ((d >> (l - 1)) & 1);
}
ZD_FN int dist_extra(int code) { return code < 4 ? 0 : (code >> 1) - 1; }
ZD_FN int dist_base(int code) { return code < 4 ? code : (2 | (code & 1)) << ((code >> 1) - 1); }
ZD_FN int bl_extra(int n) { return n == 16 ? 2 : n == 17 ? 3 : n == 18 ? 7 : 0; }
// bl_order = {16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15}, 5 bits an entry
ZD_FN int bl_order(int i) {
    const uint64_t lo = 16ull | 17ull << 5 | 18ull << 10 | 0ull << 15 | 8ull << 20 | 7ull << 25 | 9ull << 30 |
                        6ull << 35 | 10ull << 40 | 5ull << 45 | 11ull << 50 | 4ull << 55;
    const uint64_t hi = 12ull | 3ull << 5 | 13ull << 10 | 2ull << 15 | 14ull << 20 | 1ull << 25 | 15ull << 30;
    return (int)((i < 12 ? lo >> (5 * i) : hi >> (5 * (i - 12))) & 31);
}
// static_ltree / static_dtree lengths; codes are canonical (gen_codes) then bit-reversed
ZD_FN int static_llen(int n) { return n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8; }
ZD_FN uint32_t bi_reverse(uint32_t code, int len) {
    code = ((code >> 1) & 0x55555555u) | ((code & 0x55555555u) << 1);
    code = ((code >> 2) & 0x33333333u) | ((code & 0x33333333u) << 2);
    code = ((code >> 4) & 0x0F0F0F0Fu) | ((code & 0x0F0F0F0Fu) << 4);
    code = ((code >> 8) & 0x00FF00FFu) | ((code & 0x00FF00FFu) << 8);
    code = (code >> 16) | (code << 16);
    return code >> (32 - len);
}
ZD_FN uint32_t static_lcode(int n) {
    uint32_t c = n < 144 ? 0x30u + n : n < 256 ? 0x190u + (n - 144) : n < 280 ? (uint32_t)(n - 256) : 0xC0u + (n - 280);
    return bi_reverse(c, static_llen(n));
}
ZD_FN uint32_t static_dcode(int n) { return bi_reverse((uint32_t)n, 5); }

// ------------------------------------------------------------------ bit output (send_bits)
struct BitWriter {
    uint8_t* out;
    uint64_t pos;   // bytes written
    uint64_t acc;
    int n;          // bits in acc
    ZD_MFN void put(uint32_t v, int len) {
        acc |= (uint64_t)v << n;
        n += len;
        while (n >= 8) {
            out[pos++] = (uint8_t)acc;
            acc >>= 8;
            n -= 8;
        }
    }
    ZD_MFN void windup() {   // bi_windup
        if (n > 0) out[pos++] = (uint8_t)acc;
        acc = 0;
        n = 0;
    }
    ZD_MFN void byte(uint8_t b) { out[pos++] = b; }
};

// _tr_stored_block: block type 000, byte align, LEN, NLEN, the bytes (buf may be null for len 0)
ZD_FN void stored_block(BitWriter* bw, const uint8_t* buf, uint32_t len) {
    bw->put(0, 3);
    bw->windup();
    bw->byte((uint8_t)len);
    bw->byte((uint8_t)(len >> 8));
    bw->byte((uint8_t)~len);
    bw->byte((uint8_t)(~len >> 8));
    for (uint32_t i = 0; i < len; i++) bw->byte(buf[i]);
}

// ------------------------------------------------------------------ trees.c
// ct_data split into fc (Freq, then Code) and dl (Dad, then Len), as zlib's unions are used
// The heap proper holds keys freq << 15 | depth << 10 | node: zlib's smaller() (freq, then
// depth; equal keys count as smaller) is a compare of key >> 10, with no lookup of the two
// nodes' freq and depth a heap step.  (A block has at most 16384 symbols with its end code,
// so a freq fits 15 bits; a Huffman tree over weights >= 1 totalling at most 16384 is at
// most 19 levels high, so a depth fits 5.)  zlib's heap[heap_max..HEAP_SIZE) (the node
// order gen_bitlen walks) shares the keys' storage from its far end: a merge frees one key
// (4 B) as it adds two nodes (2 B each), so the two never meet (node h at u16 slot h + 1).
// fc / dl: leaves' freqs then codes; dads then lengths.
struct TreeWork {
    uint16_t lfc[L_CODES], ldl[HEAP_SIZE];
    uint16_t dfc[D_CODES], ddl[2 * D_CODES + 1];
    uint16_t bfc[BL_CODES], bdl[2 * BL_CODES + 1];
    union {
        uint32_t kheap[L_CODES + 1];
        int16_t hsort[2 * L_CODES + 2];
    };
    uint16_t bl_count[MAX_BITS + 1];
    uint32_t opt_len, static_len;
    int16_t l_max, d_max;
};
ZD_FN int16_t& heap_node(TreeWork* t, int h) { return t->hsort[h + 1]; }   // zlib's heap[h], h >= heap_max

ZD_FN void init_block(TreeWork* t) {
    for (int n = 0; n < L_CODES; n++) t->lfc[n] = 0;
    for (int n = 0; n < D_CODES; n++) t->dfc[n] = 0;
    for (int n = 0; n < BL_CODES; n++) t->bfc[n] = 0;
    t->lfc[END_BLOCK] = 1;
    t->opt_len = t->static_len = 0;
}

// a symbol: literal byte (dist 0) or (dist, lc = length - 3); as zlib's d_buf/l_buf pair
ZD_FN uint32_t sym_lit(uint32_t c) { return c; }
ZD_FN uint32_t sym_match(uint32_t dist, uint32_t lc) { return dist << 8 | lc; }
ZD_FN void tally(TreeWork* t, uint32_t sym) {
    uint32_t dist = sym >> 8, lc = sym & 255;
    if (dist == 0) {
        t->lfc[lc]++;
    } else {
        t->lfc[len_code((int)lc) + 257]++;
        t->dfc[dist_code((int)dist - 1)]++;
    }
}

template <int KIND> ZD_FN int tree_elems() { return KIND == 0 ? L_CODES : KIND == 1 ? D_CODES : BL_CODES; }
template <int KIND> ZD_FN int tree_stree_len(int n) { return KIND == 0 ? static_llen(n) : 5; }
template <int KIND> ZD_FN int tree_xbits(int n) {
    return KIND == 0 ? (n >= 257 ? len_extra(n - 257) : 0) : KIND == 1 ? dist_extra(n) : bl_extra(n);
}

ZD_FN uint32_t heap_key(uint32_t freq, uint32_t depth, uint32_t node) { return freq << 15 | depth << 10 | node; }
// pqdownheap over the keys (zlib's smaller(a, b): key(a) >> 10 <= key(b) >> 10)
ZD_FN void pqdownheap(uint32_t* kh, int k, int heap_len) {
    const uint32_t v = kh[k];
    int j = k << 1;
    while (j <= heap_len) {
        uint32_t kj = kh[j];
        if (j < heap_len) {
            const uint32_t kj1 = kh[j + 1];
            if ((kj1 >> 10) <= (kj >> 10)) {
                j++;
                kj = kj1;
            }
        }
        if ((v >> 10) <= (kj >> 10)) break;
        kh[k] = kj;
        k = j;
        j <<= 1;
    }
    kh[k] = v;
}

template <int KIND> ZD_FN void gen_bitlen(TreeWork* t, const uint16_t* fc, uint16_t* dl, int max_code, int heap_max) {
    const int max_length = KIND == 2 ? MAX_BL_BITS : MAX_BITS;
    int h, n, m, bits, overflow = 0;
    for (bits = 0; bits <= MAX_BITS; bits++) t->bl_count[bits] = 0;
    dl[heap_node(t, heap_max)] = 0;   // root
    for (h = heap_max + 1; h < HEAP_SIZE; h++) {
        n = heap_node(t, h);
        bits = dl[dl[n]] + 1;
        if (bits > max_length) bits = max_length, overflow++;
        dl[n] = (uint16_t)bits;
        if (n > max_code) continue;   // not a leaf
        t->bl_count[bits]++;
        int xbits = tree_xbits<KIND>(n);
        uint32_t f = fc[n];
        t->opt_len += f * (uint32_t)(bits + xbits);
        if (KIND != 2) t->static_len += f * (uint32_t)(tree_stree_len<KIND>(n) + xbits);
    }
    if (overflow == 0) return;
    do {
        bits = max_length - 1;
        while (t->bl_count[bits] == 0) bits--;
        t->bl_count[bits]--;
        t->bl_count[bits + 1] += 2;
        t->bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (bits = max_length; bits != 0; bits--) {
        n = t->bl_count[bits];
        while (n != 0) {
            m = heap_node(t, --h);
            if (m > max_code) continue;
            if (dl[m] != (uint32_t)bits) {
                t->opt_len += ((uint32_t)bits - dl[m]) * fc[m];
                dl[m] = (uint16_t)bits;
            }
            n--;
        }
    }
}

ZD_FN void gen_codes(uint16_t* fc, const uint16_t* dl, int max_code, const uint16_t* bl_count) {
    uint32_t next_code[MAX_BITS + 1];
    uint32_t code = 0;
    next_code[0] = 0;
    for (int bits = 1; bits <= MAX_BITS; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = code;
    }
    for (int n = 0; n <= max_code; n++) {
        int len = dl[n];
        if (len == 0) continue;
        fc[n] = (uint16_t)bi_reverse(next_code[len]++, len);
    }
}

// build_tree: Huffman code lengths (fc = freqs in, codes out; dl = lengths out); returns max_code
template <int KIND> ZD_FN int build_tree(TreeWork* t, uint16_t* fc, uint16_t* dl) {
    const int elems = tree_elems<KIND>();
    uint32_t* kh = t->kheap;
    int n, m, max_code = -1, node, heap_len = 0, heap_max = HEAP_SIZE;
    for (n = 0; n < elems; n++) {
        if (fc[n] != 0) {
            kh[++heap_len] = heap_key(fc[n], 0, (uint32_t)(max_code = n));
        } else {
            dl[n] = 0;
        }
    }
    while (heap_len < 2) {   // at least two codes of non-zero frequency
        node = max_code < 2 ? ++max_code : 0;
        kh[++heap_len] = heap_key(1, 0, (uint32_t)node);
        fc[node] = 1;
        t->opt_len--;
        if (KIND != 2) t->static_len -= (uint32_t)tree_stree_len<KIND>(node);
    }
    for (n = heap_len / 2; n >= 1; n--) pqdownheap(kh, n, heap_len);
    node = elems;
    do {
        const uint32_t kn = kh[1];   // pqremove
        kh[1] = kh[heap_len--];
        pqdownheap(kh, 1, heap_len);
        const uint32_t km = kh[1];
        n = (int)(kn & 1023);
        m = (int)(km & 1023);
        heap_node(t, --heap_max) = (int16_t)n;
        heap_node(t, --heap_max) = (int16_t)m;
        const uint32_t dn = (kn >> 10) & 31, dm = (km >> 10) & 31;
        dl[n] = dl[m] = (uint16_t)node;
        kh[1] = heap_key((kn >> 15) + (km >> 15), (dn >= dm ? dn : dm) + 1, (uint32_t)node++);
        pqdownheap(kh, 1, heap_len);
    } while (heap_len >= 2);
    const int16_t root = (int16_t)(kh[1] & 1023);
    heap_node(t, --heap_max) = root;
    gen_bitlen<KIND>(t, fc, dl, max_code, heap_max);
    gen_codes(fc, dl, max_code, t->bl_count);
    return max_code;
}

// scan_tree: bit-length code frequencies of one tree's lengths (guard at max_code + 1)
ZD_FN void scan_tree(uint16_t* bfc, uint16_t* dl, int max_code) {
    int prevlen = -1, curlen, nextlen = dl[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    dl[max_code + 1] = 0xffff;
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = dl[n + 1];
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            bfc[curlen] = (uint16_t)(bfc[curlen] + count);
        } else if (curlen != 0) {
            if (curlen != prevlen) bfc[curlen]++;
            bfc[REP_3_6]++;
        } else if (count <= 10) {
            bfc[REPZ_3_10]++;
        } else {
            bfc[REPZ_11_138]++;
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

ZD_FN void send_tree(BitWriter* bw, const uint16_t* dl, int max_code, const uint16_t* bfc, const uint16_t* bdl) {
    int prevlen = -1, curlen, nextlen = dl[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = dl[n + 1];
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            do { bw->put(bfc[curlen], bdl[curlen]); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) {
                bw->put(bfc[curlen], bdl[curlen]);
                count--;
            }
            bw->put(bfc[REP_3_6], bdl[REP_3_6]);
            bw->put((uint32_t)(count - 3), 2);
        } else if (count <= 10) {
            bw->put(bfc[REPZ_3_10], bdl[REPZ_3_10]);
            bw->put((uint32_t)(count - 3), 3);
        } else {
            bw->put(bfc[REPZ_11_138], bdl[REPZ_11_138]);
            bw->put((uint32_t)(count - 11), 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

// compress_block with the static trees (STATIC) or the block's dynamic ones
template <bool STATIC, class SYMS>
ZD_FN void compress_block(BitWriter* bw, const TreeWork* t, const SYMS& syms, uint32_t nsym) {
    for (uint32_t i = 0; i < nsym; i++) {
        uint32_t s = syms(i);
        uint32_t dist = s >> 8;
        int lc = (int)(s & 255);
        if (dist == 0) {
            if (STATIC) bw->put(static_lcode(lc), static_llen(lc));
            else bw->put(t->lfc[lc], t->ldl[lc]);
        } else {
            int code = len_code(lc);
            if (STATIC) bw->put(static_lcode(code + 257), static_llen(code + 257));
            else bw->put(t->lfc[code + 257], t->ldl[code + 257]);
            int extra = len_extra(code);
            if (extra) bw->put((uint32_t)(lc - len_base(code)), extra);
            int d = (int)dist - 1;
            code = dist_code(d);
            if (STATIC) bw->put(static_dcode(code), 5);
            else bw->put(t->dfc[code], t->ddl[code]);
            extra = dist_extra(code);
            if (extra) bw->put((uint32_t)(d - dist_base(code)), extra);
        }
    }
    if (STATIC) bw->put(static_lcode(END_BLOCK), 7);
    else bw->put(t->lfc[END_BLOCK], t->ldl[END_BLOCK]);
}

// The decision half of _tr_flush_block over a block whose frequencies t holds (init_block
// + tally): the trees (codes in fc, lengths in dl), max_blindex, and the block type zlib
// picks — 0 stored (only when `stored_ok`, zlib's block_start >= 0), 1 static, 2 dynamic.
// *bits: the block's size after its 3-bit header (static_len or opt_len; stored blocks are
// byte-aligned: 5 bytes + the data).
ZD_FN int plan_block(TreeWork* t, bool stored_ok, uint32_t stored_len, uint32_t* bits, int* max_blindex_out) {
    t->l_max = (int16_t)build_tree<0>(t, t->lfc, t->ldl);
    t->d_max = (int16_t)build_tree<1>(t, t->dfc, t->ddl);
    scan_tree(t->bfc, t->ldl, t->l_max);   // build_bl_tree
    scan_tree(t->bfc, t->ddl, t->d_max);
    build_tree<2>(t, t->bfc, t->bdl);
    int max_blindex;
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (t->bdl[bl_order(max_blindex)] != 0) break;
    t->opt_len += 3u * ((uint32_t)max_blindex + 1) + 5 + 5 + 4;
    *max_blindex_out = max_blindex;
    uint32_t opt_lenb = (t->opt_len + 3 + 7) >> 3;
    uint32_t static_lenb = (t->static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    if (stored_len + 4 <= opt_lenb && stored_ok) {
        *bits = 0;
        return 0;
    }
    if (static_lenb == opt_lenb) {
        *bits = t->static_len;
        return 1;
    }
    *bits = t->opt_len;
    return 2;
}

// _tr_flush_block (last = 0) over a block whose frequencies t holds (init_block + tally);
// stored = the block's bytes (window + block_start) or null when block_start < 0
template <class SYMS>
ZD_FN void flush_block(TreeWork* t, BitWriter* bw, const SYMS& syms, uint32_t nsym, const uint8_t* stored,
                       uint32_t stored_len) {
    uint32_t bits;
    int max_blindex;
    const int type = plan_block(t, stored != nullptr, stored_len, &bits, &max_blindex);
    if (type == 0) {
        stored_block(bw, stored, stored_len);
    } else if (type == 1) {
        bw->put(2, 3);   // (STATIC_TREES << 1) + last
        compress_block<true>(bw, t, syms, nsym);
    } else {
        bw->put(4, 3);   // (DYN_TREES << 1) + last
        int lcodes = t->l_max + 1, dcodes = t->d_max + 1, blcodes = max_blindex + 1;
        bw->put((uint32_t)(lcodes - 257), 5);   // send_all_trees
        bw->put((uint32_t)(dcodes - 1), 5);
        bw->put((uint32_t)(blcodes - 4), 4);
        for (int rank = 0; rank < blcodes; rank++) bw->put(t->bdl[bl_order(rank)], 3);
        send_tree(bw, t->ldl, lcodes - 1, t->bfc, t->bdl);
        send_tree(bw, t->ddl, dcodes - 1, t->bfc, t->bdl);
        compress_block<false>(bw, t, syms, nsym);
    }
    init_block(t);
}

// the empty stored block deflate() adds after a block_done Z_SYNC_FLUSH (the 00 00 FF FF tail)
ZD_FN void sync_marker(BitWriter* bw) { stored_block(bw, nullptr, 0); }

// ------------------------------------------------------------------ deflate.c, serial
struct ArraySyms {
    const uint32_t* p;
    ZD_MFN uint32_t operator()(uint32_t i) const { return p[i]; }
};

// deflate_state for one session (raw, 32 KiB window, 32 K hash heads); window/head/prev are
// the session's own arrays (zlib layout: window indices, NIL = 0)
struct SerialState {
    uint8_t* window;
    uint16_t* head;
    uint16_t* prev;
    uint32_t strstart, lookahead, insert, high_water, ins_h;
    int32_t block_start;
    uint32_t match_length, prev_length, match_available, match_start, prev_match;
    const uint8_t* next_in;
    uint32_t avail_in;
    Cfg cfg;
    uint32_t* sym;
    uint32_t nsym;
    TreeWork* tw;
    BitWriter bw;
};

ZD_FN void slide_hash(SerialState* s) {
    for (int n = 0; n < WSIZE; n++) {
        uint32_t m = s->head[n];
        s->head[n] = (uint16_t)(m >= (uint32_t)WSIZE ? m - WSIZE : 0);
    }
    for (int n = 0; n < WSIZE; n++) {
        uint32_t m = s->prev[n];
        s->prev[n] = (uint16_t)(m >= (uint32_t)WSIZE ? m - WSIZE : 0);
    }
}

ZD_FN void fill_window(SerialState* s) {
    uint32_t more;
    do {
        more = WINDOW_SIZE - s->lookahead - s->strstart;
        if (s->strstart >= (uint32_t)(WSIZE + MAX_DIST)) {
            for (uint32_t i = 0; i < WSIZE - more; i++) s->window[i] = s->window[i + WSIZE];
            s->match_start -= WSIZE;
            s->strstart -= WSIZE;
            s->block_start -= WSIZE;
            slide_hash(s);
            more += WSIZE;
        }
        if (s->avail_in == 0) break;
        uint32_t n = s->avail_in < more ? s->avail_in : more;   // read_buf
        uint8_t* dst = s->window + s->strstart + s->lookahead;
        for (uint32_t i = 0; i < n; i++) dst[i] = s->next_in[i];
        s->next_in += n;
        s->avail_in -= n;
        s->lookahead += n;
        if (s->lookahead + s->insert >= MIN_MATCH) {
            uint32_t str = s->strstart - s->insert;
            s->ins_h = s->window[str];
            s->ins_h = ((s->ins_h << 5) ^ s->window[str + 1]) & HASH_MASK;
            while (s->insert) {
                s->ins_h = ((s->ins_h << 5) ^ s->window[str + MIN_MATCH - 1]) & HASH_MASK;
                s->prev[str & WMASK] = s->head[s->ins_h];
                s->head[s->ins_h] = (uint16_t)str;
                str++;
                s->insert--;
                if (s->lookahead + s->insert < MIN_MATCH) break;
            }
        }
    } while (s->lookahead < MIN_LOOKAHEAD && s->avail_in != 0);
    if (s->high_water < (uint32_t)WINDOW_SIZE) {
        uint32_t curr = s->strstart + s->lookahead, init;
        if (s->high_water < curr) {
            init = WINDOW_SIZE - curr;
            if (init > WIN_INIT) init = WIN_INIT;
            for (uint32_t i = 0; i < init; i++) s->window[curr + i] = 0;
            s->high_water = curr + init;
        } else if (s->high_water < curr + WIN_INIT) {
            init = curr + WIN_INIT - s->high_water;
            if (init > WINDOW_SIZE - s->high_water) init = WINDOW_SIZE - s->high_water;
            for (uint32_t i = 0; i < init; i++) s->window[s->high_water + i] = 0;
            s->high_water += init;
        }
    }
}

ZD_FN uint32_t insert_string(SerialState* s, uint32_t str) {   // INSERT_STRING, returns the old head
    s->ins_h = ((s->ins_h << 5) ^ s->window[str + MIN_MATCH - 1]) & HASH_MASK;
    uint32_t h = s->head[s->ins_h];
    s->prev[str & WMASK] = (uint16_t)h;
    s->head[s->ins_h] = (uint16_t)str;
    return h;
}

ZD_FN uint32_t longest_match(SerialState* s, uint32_t cur_match) {
    uint32_t chain_length = s->cfg.chain;
    const uint8_t* scan = s->window + s->strstart;
    int best_len = (int)s->prev_length;
    int nice_match = s->cfg.nice;
    uint32_t limit = s->strstart > (uint32_t)MAX_DIST ? s->strstart - MAX_DIST : 0;
    uint8_t scan_end1 = scan[best_len - 1];
    uint8_t scan_end = scan[best_len];
    if (s->prev_length >= s->cfg.good) chain_length >>= 2;
    if ((uint32_t)nice_match > s->lookahead) nice_match = (int)s->lookahead;
    do {
        const uint8_t* match = s->window + cur_match;
        if (match[best_len] != scan_end || match[best_len - 1] != scan_end1 || match[0] != scan[0] ||
            match[1] != scan[1])
            continue;
        int len = 3;   // scan[2] == match[2]: equal hash and equal first two bytes
        while (len < MAX_MATCH && scan[len] == match[len]) len++;
        if (len > best_len) {
            s->match_start = cur_match;
            best_len = len;
            if (len >= nice_match) break;
            scan_end1 = scan[best_len - 1];
            scan_end = scan[best_len];
        }
    } while ((cur_match = s->prev[cur_match & WMASK]) > limit && --chain_length != 0);
    if ((uint32_t)best_len <= s->lookahead) return (uint32_t)best_len;
    return s->lookahead;
}

ZD_FN void serial_flush(SerialState* s) {   // FLUSH_BLOCK_ONLY(s, 0)
    flush_block(s->tw, &s->bw, ArraySyms{s->sym}, s->nsym,
                s->block_start >= 0 ? s->window + s->block_start : nullptr,
                (uint32_t)((int32_t)s->strstart - s->block_start));
    s->block_start = (int32_t)s->strstart;
    s->nsym = 0;
}
ZD_FN bool serial_tally(SerialState* s, uint32_t sym) {
    s->sym[s->nsym++] = sym;
    tally(s->tw, sym);
    return s->nsym == SYM_END;
}

ZD_FN void deflate_fast(SerialState* s) {
    for (;;) {
        if (s->lookahead < MIN_LOOKAHEAD) {
            fill_window(s);
            if (s->lookahead == 0) break;
        }
        uint32_t hash_head = 0;
        if (s->lookahead >= MIN_MATCH) hash_head = insert_string(s, s->strstart);
        if (hash_head != 0 && s->strstart - hash_head <= (uint32_t)MAX_DIST) s->match_length = longest_match(s, hash_head);
        bool bflush;
        if (s->match_length >= MIN_MATCH) {
            bflush = serial_tally(s, sym_match(s->strstart - s->match_start, s->match_length - MIN_MATCH));
            s->lookahead -= s->match_length;
            if (s->match_length <= s->cfg.lazy && s->lookahead >= MIN_MATCH) {   // max_insert_length
                s->match_length--;
                do {
                    s->strstart++;
                    insert_string(s, s->strstart);
                } while (--s->match_length != 0);
                s->strstart++;
            } else {
                s->strstart += s->match_length;
                s->match_length = 0;
                s->ins_h = s->window[s->strstart];
                s->ins_h = ((s->ins_h << 5) ^ s->window[s->strstart + 1]) & HASH_MASK;
            }
        } else {
            bflush = serial_tally(s, sym_lit(s->window[s->strstart]));
            s->lookahead--;
            s->strstart++;
        }
        if (bflush) serial_flush(s);
    }
    s->insert = s->strstart < MIN_MATCH - 1 ? s->strstart : MIN_MATCH - 1;
    if (s->nsym) serial_flush(s);
}

ZD_FN void deflate_slow(SerialState* s) {
    for (;;) {
        if (s->lookahead < MIN_LOOKAHEAD) {
            fill_window(s);
            if (s->lookahead == 0) break;
        }
        uint32_t hash_head = 0;
        if (s->lookahead >= MIN_MATCH) hash_head = insert_string(s, s->strstart);
        s->prev_length = s->match_length;
        s->prev_match = s->match_start;
        s->match_length = MIN_MATCH - 1;
        if (hash_head != 0 && s->prev_length < s->cfg.lazy && s->strstart - hash_head <= (uint32_t)MAX_DIST) {
            s->match_length = longest_match(s, hash_head);
            if (s->match_length <= 5 && s->match_length == MIN_MATCH && s->strstart - s->match_start > (uint32_t)TOO_FAR)
                s->match_length = MIN_MATCH - 1;
        }
        if (s->prev_length >= MIN_MATCH && s->match_length <= s->prev_length) {
            uint32_t max_insert = s->strstart + s->lookahead - MIN_MATCH;
            bool bflush = serial_tally(s, sym_match(s->strstart - 1 - s->prev_match, s->prev_length - MIN_MATCH));
            s->lookahead -= s->prev_length - 1;
            s->prev_length -= 2;
            do {
                if (++s->strstart <= max_insert) insert_string(s, s->strstart);
            } while (--s->prev_length != 0);
            s->match_available = 0;
            s->match_length = MIN_MATCH - 1;
            s->strstart++;
            if (bflush) serial_flush(s);
        } else if (s->match_available) {
            bool bflush = serial_tally(s, sym_lit(s->window[s->strstart - 1]));
            if (bflush) serial_flush(s);
            s->strstart++;
            s->lookahead--;
        } else {
            s->match_available = 1;
            s->strstart++;
            s->lookahead--;
        }
    }
    if (s->match_available) {
        serial_tally(s, sym_lit(s->window[s->strstart - 1]));
        s->match_available = 0;
    }
    s->insert = s->strstart < MIN_MATCH - 1 ? s->strstart : MIN_MATCH - 1;
    if (s->nsym) serial_flush(s);
}

// One Deflater.deflate(buf, SYNC_FLUSH) over a non-empty frame payload (levels 1-9): the
// blocks and the sync marker go to s->bw.  Between calls zlib's match_length is below 3,
// prev_length 2, nothing is available and block_start == strstart.
ZD_FN void serial_call(SerialState* s, const uint8_t* data, uint32_t len, int level) {
    s->next_in = data;
    s->avail_in = len;
    s->lookahead = 0;
    s->match_length = s->prev_length = MIN_MATCH - 1;
    s->match_available = 0;
    s->block_start = (int32_t)s->strstart;
    s->nsym = 0;
    init_block(s->tw);
    if (level <= 3) deflate_fast(s);
    else deflate_slow(s);
    sync_marker(&s->bw);
}

// Level 0 (deflate_stored with Java's deflateBound(len) output buffer: every call emits
// its input as stored blocks of at most 65535 bytes, then the sync marker)
ZD_FN void stored_call(BitWriter* bw, const uint8_t* data, uint32_t len) {
    uint32_t o = 0;
    while (o < len) {
        uint32_t n = len - o < 65535u ? len - o : 65535u;
        stored_block(bw, data + o, n);
        o += n;
    }
    sync_marker(bw);
}

// ------------------------------------------------------------------ decomposition (levels 4-9)
// Per-position longest_match results, packed: bits 0-8 best length - 2 (0 = no match of >= 3),
// bits 9-23 distance, bit 24 (full word only): the head candidate is exactly MAX_DIST back
// (window index 0, NIL, when a slide has just put strstart at MAX_DIST).
enum : uint32_t { MR_HEAD_AT_MAX = 1u << 24 };
ZD_FN uint32_t mr_len(uint32_t r) { return (r & 511) ? (r & 511) + 2 : 0; }
ZD_FN uint32_t mr_dist(uint32_t r) { return (r >> 9) & 32767; }

// longest_match at stream position s of a frame ending at `end` (s + 2 < end), for both
// chain budgets and a start threshold of 2: the first candidate of the longest length, the
// search stopping at the first candidate of >= nice_match (nice clamped to end - s) or after
// the budget.  byte(p): the window byte at stream position p (past `end`: the frame's strip);
// link(p): distance from p to the previous string with its hash (0: none / not a candidate).
template <class BYTE, class LINK>
ZD_FN void match_at(const BYTE& byte, const LINK& link, uint32_t s, uint32_t end, Cfg c, uint32_t* out_full,
                    uint32_t* out_quarter) {
    uint32_t d = link(s);
    if (d == 0 || d > (uint32_t)MAX_DIST) {   // hash_head NIL or too far: no lookup
        *out_full = *out_quarter = 0;
        return;
    }
    uint32_t flags = d == (uint32_t)MAX_DIST ? (uint32_t)MR_HEAD_AT_MAX : 0u;
    uint32_t nice = c.nice;
    if (nice > end - s) nice = end - s;
    const uint32_t qbudget = c.chain >> 2;
    uint32_t best = 2, best_d = 0, qres = 0;
    uint32_t b0 = byte(s), b1 = byte(s + 1);
    uint32_t q = s - d;
    uint32_t dist = d;
    uint32_t k = 1;   // candidates visited
    for (;; k++) {
        if (byte(q) == b0 && byte(q + 1) == b1 && byte(q + best) == byte(s + best)) {
            uint32_t len = 3;
            while (len < (uint32_t)MAX_MATCH && byte(q + len) == byte(s + len)) len++;
            if (len > best) {
                best = len;
                best_d = dist;
                if (len >= nice) break;
            }
        }
        if (k == qbudget) qres = best > 2 ? ((best - 2) | best_d << 9) : 0;
        if (k >= c.chain) break;
        uint32_t l = link(q);
        if (l == 0) break;
        dist += l;
        if (dist >= (uint32_t)MAX_DIST) break;
        q -= l;
    }
    uint32_t full = best > 2 ? ((best - 2) | best_d << 9) : 0;
    *out_full = full | flags;
    *out_quarter = k <= qbudget ? full : qres;   // the walk ended inside the quarter budget
}

// What a frame's parse needs about its place in the window (computed by the window walk):
struct CallGeom {
    uint32_t start_w;     // strstart after the call-start fill_window (slide applied)
    uint8_t start_slid;   // that fill slid the window with strstart exactly WSIZE + MAX_DIST
};

// deflate_slow over one frame from the per-position results.  res(s, variant, &full,
// &quarter) gives the packed pair at stream position s; variant 1 = after a slide in the
// frame's tail (the window bytes past the end differ).  byte(p) is the stream byte (the
// literals).  Symbols go to symw.put(v); every block zlib would flush is closed by
// symw.block_done() and handed to sink(nsym, stored_s, stored_len, stored_ok): its symbol
// count, and for the stored choice the stream range it covers (stored_ok: zlib's
// block_start >= 0).  The caller adds the sync marker.  Returns whether the window slid
// inside the frame's tail (the next call then starts without a slide).
template <class RES, class BYTE, class SYMW, class SINK>
ZD_FN bool parse_call(RES&& res, BYTE&& byte, uint32_t start, uint32_t len, CallGeom g, Cfg c, SYMW& symw,
                      SINK& sink) {
    uint32_t sw = g.start_w;                 // strstart, window index
    uint32_t s = start;                      // strstart, stream position
    uint32_t more = WINDOW_SIZE - sw;
    uint32_t rem = len;
    uint32_t n0 = rem < more ? rem : more;
    uint32_t loaded = sw + n0;               // window index of the loaded end
    rem -= n0;
    int32_t block_start_w = (int32_t)sw;
    uint32_t block_start_s = s;
    uint32_t match_length = MIN_MATCH - 1, prev_length, match_start = 0, prev_match;
    bool match_available = false, tail_slid = false;
    bool slid_here = g.start_slid != 0;      // a slide put strstart at MAX_DIST at this loop top
    uint32_t nsym = 0;
    auto flush = [&](uint32_t cur_s, int32_t cur_w) {
        symw.block_done();
        sink(nsym, block_start_s, cur_s - block_start_s, block_start_w >= 0);
        block_start_s = cur_s;
        block_start_w = cur_w;
        nsym = 0;
    };
    for (;;) {
        uint32_t lookahead = loaded - sw;
        if (lookahead < (uint32_t)MIN_LOOKAHEAD) {
            if (sw >= (uint32_t)(WSIZE + MAX_DIST)) {
                slid_here = sw == (uint32_t)(WSIZE + MAX_DIST);
                sw -= WSIZE;
                loaded -= WSIZE;
                block_start_w -= WSIZE;
                if (rem == 0) tail_slid = true;
            }
            if (rem) {
                uint32_t m = WINDOW_SIZE - loaded;
                uint32_t n = rem < m ? rem : m;
                loaded += n;
                rem -= n;
            }
            lookahead = loaded - sw;
            if (lookahead == 0) break;
        }
        bool lookup = lookahead >= (uint32_t)MIN_MATCH;
        prev_length = match_length;
        prev_match = match_start;
        match_length = MIN_MATCH - 1;
        if (lookup && prev_length < c.lazy) {
            uint32_t full, quarter;
            res(s, tail_slid ? 1 : 0, &full, &quarter);
            bool nil_edge = slid_here && (full & MR_HEAD_AT_MAX);
            uint32_t r = prev_length >= c.good ? quarter : full;
            if ((full & 511) != 0 && !nil_edge) {
                uint32_t m = mr_len(r);
                uint32_t ml;
                if (m > prev_length) {
                    match_start = s - mr_dist(r);
                    ml = m;
                } else {
                    ml = prev_length;
                }
                if (ml > lookahead) ml = lookahead;
                match_length = ml;
                if (match_length == (uint32_t)MIN_MATCH && s - match_start > (uint32_t)TOO_FAR)
                    match_length = MIN_MATCH - 1;
            }
        }
        slid_here = false;
        if (prev_length >= (uint32_t)MIN_MATCH && match_length <= prev_length) {
            symw.put(sym_match(s - 1 - prev_match, prev_length - MIN_MATCH));
            nsym++;
            uint32_t adv = prev_length - 1;   // strstart moves to the match end
            s += adv;
            sw += adv;
            match_available = false;
            match_length = MIN_MATCH - 1;
            if (nsym == (uint32_t)SYM_END) flush(s, (int32_t)sw);
        } else if (match_available) {
            symw.put(sym_lit(byte(s - 1)));
            nsym++;
            if (nsym == (uint32_t)SYM_END) flush(s, (int32_t)sw);
            s++;
            sw++;
        } else {
            match_available = true;
            s++;
            sw++;
        }
    }
    if (match_available) {
        symw.put(sym_lit(byte(s - 1)));
        nsym++;
    }
    if (nsym) flush(s, (int32_t)sw);
    return tail_slid;
}

// The host forms: a symbol buffer reused per block, and a sink that runs _tr_flush_block
// right away (trees, bits), as zlib does.
struct SymBuf {
    uint32_t* buf;
    uint32_t n;
    ZD_MFN void put(uint32_t v) { buf[n++] = v; }
    ZD_MFN void block_done() {}
};
struct FlushNow {
    TreeWork* t;
    BitWriter* bw;
    const uint8_t* S;   // stream bytes (stored blocks)
    SymBuf* sb;
    ZD_MFN void operator()(uint32_t nsym, uint32_t stored_s, uint32_t stored_len, bool stored_ok) {
        init_block(t);
        for (uint32_t i = 0; i < nsym; i++) tally(t, sb->buf[i]);
        flush_block(t, bw, ArraySyms{sb->buf}, nsym, stored_ok ? S + stored_s : nullptr, stored_len);
        sb->n = 0;
    }
};

}  // namespace zd
