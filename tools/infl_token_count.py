"""Token-stream size of the inflate bench batch (CPU, diagnostic): a minimal raw-DEFLATE
decoder (RFC 1951) that counts what k_infl_tok writes per message — one 32-bit word per
literal run and per (length, distance) pair, plus the literal bytes — so the kernel's
PMC write bytes can be set against it.
  python tools/infl_token_count.py [sessions]   (default: the bench's 8192)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchsupport.synth import deflate_batch  # noqa: E402

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]


class Bits:
    def __init__(self, data):
        self.d, self.p = data, 0

    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.d[self.p >> 3] >> (self.p & 7)) & 1) << i
            self.p += 1
        return v


def huff(lens):
    """canonical code -> {(length, code): symbol}"""
    cnt = [0] * 16
    for ln in lens:
        cnt[ln] += 1
    cnt[0] = 0
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + cnt[b - 1]) << 1
        nxt[b] = code
    t = {}
    for s, ln in enumerate(lens):
        if ln:
            t[(ln, nxt[ln])] = s
            nxt[ln] += 1
    return t


def sym(b, t):
    code, ln = 0, 0
    while True:
        code = (code << 1) | b.get(1)
        ln += 1
        if (ln, code) in t:
            return t[(ln, code)]


FIXED = (huff([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8), huff([5] * 30))


def count(data):
    """(tokens, literals) of one sync-flushed message (its blocks end on the stripped tail)"""
    b = Bits(data + b"\x00\x00\xff\xff")
    tok = lit = 0
    run = 0
    while b.p < len(data) * 8:
        _final, typ = b.get(1), b.get(2)
        if typ == 0:
            b.p = (b.p + 7) & ~7
            n = b.get(16)
            b.get(16)
            b.p += 8 * n
            lit += n
            run += n
            continue
        if typ == 1:
            lt, dt = FIXED
        else:
            hl, hd, hc = b.get(5) + 257, b.get(5) + 1, b.get(4) + 4
            order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
            cl = [0] * 19
            for i in range(hc):
                cl[order[i]] = b.get(3)
            ct = huff(cl)
            lens = []
            while len(lens) < hl + hd:
                s = sym(b, ct)
                if s < 16:
                    lens.append(s)
                elif s == 16:
                    lens += [lens[-1]] * (3 + b.get(2))
                elif s == 17:
                    lens += [0] * (3 + b.get(3))
                else:
                    lens += [0] * (11 + b.get(7))
            lt, dt = huff(lens[:hl]), huff(lens[hl:])
        while True:
            s = sym(b, lt)
            if s < 256:
                lit += 1
                run += 1
            elif s == 256:
                break
            else:
                b.get(LEXT[s - 257])
                d = sym(b, dt)
                b.get(DEXT[d])
                if run:
                    tok += 1
                    run = 0
                tok += 1
    if run:
        tok += 1
    return tok, lit


def main():
    n_s = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    desc, sf, pl, plain = deflate_batch(0x1F1A, n_s, 16, 4096)
    u = 64  # deflate_batch tiles 64 distinct session streams
    tok = lit = 0
    for s in range(u):
        for k in range(int(sf[s]), int(sf[s + 1])):
            o, ln = int(desc[k]["payload_off"]), int(desc[k]["payload_len"])
            t, li = count(bytes(pl[o:o + ln]))
            tok += t
            lit += li
    scale = n_s / u
    print(f"{n_s} sessions: {tok * scale:.0f} tokens, {lit * scale:.0f} literal bytes; token+literal bytes "
          f"{(4 * tok + lit) * scale / 1e9:.3f} GB for {plain / 1e9:.3f} GB inflated")


if __name__ == "__main__":
    main()
