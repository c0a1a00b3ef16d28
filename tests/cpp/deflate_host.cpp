// CPU harness of snf4j_amd/csrc/deflate_core.h — TEST INFRASTRUCTURE ONLY.
//
// Runs the GPU deflate algorithm's pieces on the host so tests/test_deflate_host.py can
// compare them byte for byte with zlib (oracle/deflate_ref.c) without a GPU:
//   mode 0: the serial restatement (zlib's own loop, SerialState) per session;
//   mode 1: the decomposition the GPU runs for levels 4-9 — the window walk (history,
//           strips past each frame's end, call geometry), hash links, match_at at every
//           position for both chain budgets, parse_call per frame, and the conversion of
//           the links back into zlib's head/prev arrays — written serially.
// Both run PerMessageDeflateEncoder's frame logic (pmd_step) over one session's frames and
// carry the session state (wsg_deflate_state + window/head/prev) between calls.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../snf4j_amd/csrc/deflate_core.h"
#include "../../snf4j_amd/csrc/deflate_pmd.h"

using namespace zd;

namespace {

struct Session {
    wsg_deflate_state* st;
    uint8_t* win;
    uint16_t* head;
    uint16_t* prev;
};

void fresh(Session& S) {
    S.st->strstart = 0;
    S.st->high_water = 0;
    S.st->insert = 0;
    memset(S.win, 0, WINDOW_SIZE);
    memset(S.head, 0, WSIZE * 2);
    memset(S.prev, 0, WSIZE * 2);
}

// ---- mode 0: serial
uint64_t serial_call_host(Session& S, int level, const uint8_t* data, uint32_t len, uint8_t* out) {
    std::vector<uint32_t> sym(LIT_BUFSIZE);
    TreeWork tw;
    SerialState s;
    memset(&s, 0, sizeof(s));
    s.window = S.win;
    s.head = S.head;
    s.prev = S.prev;
    s.strstart = S.st->strstart;
    s.insert = S.st->insert;
    s.high_water = S.st->high_water;
    s.cfg = level_cfg(level);
    s.sym = sym.data();
    s.tw = &tw;
    s.bw = BitWriter{out, 0, 0, 0};
    serial_call(&s, data, len, level);
    S.st->strstart = s.strstart;
    S.st->insert = (uint16_t)s.insert;
    S.st->high_water = s.high_water;
    return s.bw.pos;
}

// ---- mode 1: the decomposition over one deflater segment (calls without a reset between)
struct Call {
    const uint8_t* p;
    uint32_t len;
    uint8_t* out;
    uint64_t out_len;
};

struct StreamBytes {
    const uint8_t* S;
    uint32_t end;
    const uint8_t* strip;
    uint32_t operator()(uint32_t p) const { return p < end ? S[p] : strip[p - end]; }
};
struct Links {
    const uint16_t* l;
    uint32_t operator()(uint32_t p) const { return l[p]; }
};
struct PlainBytes {
    const uint8_t* S;
    uint32_t operator()(uint32_t p) const { return S[p]; }
    const uint8_t* ptr(uint32_t p) const { return S + p; }
};

void zero_hw(uint8_t* W, uint32_t& hw, uint32_t curr) {
    if (hw >= (uint32_t)WINDOW_SIZE) return;
    if (hw < curr) {
        uint32_t init = std::min<uint32_t>(WIN_INIT, WINDOW_SIZE - curr);
        memset(W + curr, 0, init);
        hw = curr + init;
    } else if (hw < curr + WIN_INIT) {
        uint32_t init = std::min<uint32_t>(curr + WIN_INIT - hw, WINDOW_SIZE - hw);
        memset(W + hw, 0, init);
        hw += init;
    }
}

void decomp_segment(Session& S, int level, std::vector<Call>& calls) {
    const Cfg c = level_cfg(level);
    const uint32_t strstart0 = S.st->strstart, insert0 = S.st->insert;
    const uint32_t H = std::min<uint32_t>(strstart0, WSIZE);
    uint64_t total = 0;
    for (auto& k : calls) total += k.len;
    const uint32_t SL = H + (uint32_t)total;
    std::vector<uint8_t> Sb(SL + 16);
    memcpy(Sb.data(), S.win + strstart0 - H, H);
    {
        uint32_t o = H;
        for (auto& k : calls) {
            memcpy(Sb.data() + o, k.p, k.len);
            o += k.len;
        }
    }
    const int64_t base0 = (int64_t)H - strstart0;   // stream position of window index 0
    // links: history from prev[], then every new string in position order from head[]
    std::vector<uint16_t> link(SL + 1, 0);
    std::vector<int64_t> pred(SL + 1, -1);
    for (uint32_t p = 0; p < H; p++) {
        uint32_t w = strstart0 - H + p;
        if (w >= strstart0 - insert0) break;
        uint32_t pv = S.prev[w & WMASK];
        if (pv != 0) {
            pred[p] = (int64_t)pv + base0;
            if (w - pv < (uint32_t)WSIZE) link[p] = (uint16_t)(w - pv);
        }
    }
    std::vector<int64_t> hpos(WSIZE, -1);
    for (uint32_t h = 0; h < (uint32_t)WSIZE; h++)
        if (S.head[h]) hpos[h] = (int64_t)S.head[h] + base0;
    const uint32_t ins_from = H - std::min(insert0, H);
    for (uint32_t p = ins_from; p + 2 < SL; p++) {
        uint32_t h = hash3(Sb[p], Sb[p + 1], Sb[p + 2]);
        int64_t q = hpos[h];
        pred[p] = q;
        if (q >= 0 && (int64_t)p - q < WSIZE) link[p] = (uint16_t)(p - q);
        if ((int64_t)p != base0) hpos[h] = p;   // window index 0 is NIL (a deflater's first string)
    }
    // the window walk: strips after each frame's end, call geometry
    std::vector<uint8_t> W(S.win, S.win + WINDOW_SIZE);
    uint32_t sw = strstart0, hw = S.st->high_water;
    const size_t nc = calls.size();
    std::vector<CallGeom> geom(nc);
    std::vector<uint8_t> strip0(nc * STRIP), strip1(nc * STRIP);
    std::vector<uint8_t> tail_ok(nc);
    std::vector<uint32_t> cstart(nc);
    {
        uint32_t o = H;
        for (size_t k = 0; k < nc; k++) {
            uint32_t L = calls[k].len;
            cstart[k] = o;
            geom[k].start_slid = 0;
            if (sw >= (uint32_t)(WSIZE + MAX_DIST)) {
                geom[k].start_slid = sw == (uint32_t)(WSIZE + MAX_DIST);
                memmove(W.data(), W.data() + WSIZE, sw - WSIZE);
                sw -= WSIZE;
            }
            geom[k].start_w = sw;
            uint32_t n = std::min<uint32_t>(L, WINDOW_SIZE - sw);
            memcpy(W.data() + sw, calls[k].p, n);
            uint32_t loaded = sw + n, rem = L - n;
            zero_hw(W.data(), hw, loaded);
            while (rem) {
                memmove(W.data(), W.data() + WSIZE, loaded - WSIZE);
                loaded -= WSIZE;
                uint32_t m = std::min<uint32_t>(rem, WINDOW_SIZE - loaded);
                memcpy(W.data() + loaded, calls[k].p + (L - rem), m);
                loaded += m;
                rem -= m;
                zero_hw(W.data(), hw, loaded);
            }
            for (uint32_t j = 0; j < (uint32_t)STRIP; j++) {
                strip0[k * STRIP + j] = loaded + j < (uint32_t)WINDOW_SIZE ? W[loaded + j] : 0;
                strip1[k * STRIP + j] = loaded - WSIZE + j < (uint32_t)WINDOW_SIZE ? W[loaded - WSIZE + j] : 0;
            }
            tail_ok[k] = loaded > (uint32_t)(WSIZE + MAX_DIST);
            sw = loaded;
            o += L;
        }
    }
    // match_at everywhere, then the parse per frame
    std::vector<uint32_t> full(SL), quarter(SL), sym(LIT_BUFSIZE);
    TreeWork tw;
    bool last_tail = false;
    for (size_t k = 0; k < nc; k++) {
        uint32_t start = cstart[k], end = start + calls[k].len;
        StreamBytes b0{Sb.data(), end, &strip0[k * STRIP]};
        StreamBytes b1{Sb.data(), end, &strip1[k * STRIP]};
        for (uint32_t s = start; s + 2 < end; s++) match_at(b0, Links{link.data()}, s, end, c, &full[s], &quarter[s]);
        uint32_t t0 = end > (uint32_t)MAX_MATCH + start ? end - MAX_MATCH : start;
        std::vector<uint32_t> full1(end - t0 + 1), quarter1(end - t0 + 1);
        if (tail_ok[k])
            for (uint32_t s = t0; s + 2 < end; s++)
                match_at(b1, Links{link.data()}, s, end, c, &full1[s - t0], &quarter1[s - t0]);
        auto res = [&](uint32_t s, int variant, uint32_t* f, uint32_t* q) {
            if (variant && s >= t0) {
                *f = full1[s - t0];
                *q = quarter1[s - t0];
            } else {
                *f = full[s];
                *q = quarter[s];
            }
        };
        BitWriter bw{calls[k].out, 0, 0, 0};
        SymBuf sbuf{sym.data(), 0};
        FlushNow sink{&tw, &bw, Sb.data(), &sbuf};
        last_tail = parse_call(res, PlainBytes{Sb.data()}, start, calls[k].len, geom[k], c, sbuf, sink);
        sync_marker(&bw);
        calls[k].out_len = bw.pos;
    }
    if (nc && last_tail) {
        memmove(W.data(), W.data() + WSIZE, sw - WSIZE);
        sw -= WSIZE;
    }
    // state back in zlib's layout
    const int64_t base = (int64_t)SL - sw;
    const uint32_t ins_final = std::min<uint32_t>(sw, 2);
    const int64_t ins_end = (int64_t)SL - ins_final;
    for (uint32_t h = 0; h < (uint32_t)WSIZE; h++) {
        int64_t v = hpos[h] >= 0 ? hpos[h] - base : 0;
        S.head[h] = (uint16_t)(v > 0 ? v : 0);
    }
    for (uint32_t j = 0; j < (uint32_t)WSIZE; j++) {
        uint32_t v = S.prev[j];
        int64_t nv = v ? (int64_t)v + base0 - base : 0;
        S.prev[j] = (uint16_t)(nv > 0 ? nv : 0);
    }
    for (int64_t p = ins_from; p < ins_end; p++) {
        int64_t v = pred[p] >= 0 ? pred[p] - base : 0;
        S.prev[(uint32_t)((p - base) & WMASK)] = (uint16_t)(v > 0 ? v : 0);
    }
    memcpy(S.win, W.data(), WINDOW_SIZE);
    S.st->strstart = sw;
    S.st->high_water = hw;
    S.st->insert = (uint16_t)ins_final;
}

}  // namespace

extern "C" {

// One session's frames through PerMessageDeflateEncoder(level, noContext).  Frame i:
// opcode/fin/rsv, payload[off[i], +len[i]).  Writes out[out_off[i], out_off[i+1]) and
// out_rsv[i].  st/win/head/prev: the session's carried state (fresh = zeros).
// mode 0 = serial restatement, 1 = decomposition (levels 4-9; levels 0-3 run serially).
int zdh_session(int level, int no_context, int mode, uint32_t n, const uint8_t* opcode, const uint8_t* fin,
                const uint8_t* rsv, const uint64_t* off, const uint32_t* len, const uint8_t* payload,
                wsg_deflate_state* st, uint8_t* win, uint16_t* head, uint16_t* prev, uint8_t* out, uint64_t cap,
                uint64_t* out_off, uint8_t* out_rsv) {
    Session S{st, win, head, prev};
    std::vector<std::vector<uint8_t>> raw(n);
    std::vector<Call> seg;
    std::vector<uint32_t> seg_frames;
    std::vector<uint8_t> kind(n), drop(n);
    auto run_segment = [&]() {
        if (seg.empty()) return;
        if (!st->has_deflater) {
            fresh(S);
            st->has_deflater = 1;
        }
        if (level == 0) {
            for (auto& k : seg) {
                BitWriter bw{k.out, 0, 0, 0};
                stored_call(&bw, k.p, k.len);
                k.out_len = bw.pos;
            }
        } else if (mode == 1 && level >= 4) {
            decomp_segment(S, level, seg);
        } else {
            for (auto& k : seg) k.out_len = serial_call_host(S, level, k.p, k.len, k.out);
        }
        for (size_t i = 0; i < seg.size(); i++) raw[seg_frames[i]].resize(seg[i].out_len);
        seg.clear();
        seg_frames.clear();
    };
    for (uint32_t i = 0; i < n; i++) {
        uint8_t r8 = 0, dr = 0;
        kind[i] = (uint8_t)pmd_step(&st->compressing, opcode[i], fin[i], rsv[i], len[i], no_context, &r8, &dr);
        out_rsv[i] = r8;
        drop[i] = dr;
        if (kind[i] == PMD_CALL) {
            raw[i].resize((size_t)len[i] + (len[i] >> 3) + 64 + 5 * (len[i] / 16000 + 1));
            seg.push_back(Call{payload + off[i], len[i], raw[i].data(), 0});
            seg_frames.push_back(i);
        }
        if (dr) {
            run_segment();
            st->has_deflater = 0;
        }
    }
    run_segment();
    uint64_t w = 0;
    out_off[0] = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t k;
        if (kind[i] == PMD_PASS) {
            k = len[i];
            if (w + k > cap) return -1;
            memcpy(out + w, payload + off[i], k);
        } else if (kind[i] == PMD_EMPTY) {
            k = 1;
            if (w + 1 > cap) return -1;
            out[w] = 0;
        } else {
            k = raw[i].size() - (fin[i] ? 4 : 0);
            if (w + k > cap) return -1;
            memcpy(out + w, raw[i].data(), k);
        }
        w += k;
        out_off[i + 1] = w;
    }
    return 0;
}
}
