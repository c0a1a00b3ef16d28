"""Sizing study for k_infl_tok's per-lane LDS tables.

Parses the dynamic-Huffman block header at the start of every message of the
bench's inflate batch (benchsupport.synth.deflate_batch: zlib level 6, raw
DEFLATE, Z_SYNC_FLUSH per message, so every message starts a new block on a
byte boundary) and reports, per root width, how many sub-table entries the
literal/length and distance tables need.  The count follows q_build in
inflate.hip: every root prefix with longer codes under it gets a sub-table of
2^(longest length under it - root) entries.  Runs on the CPU, no GPU.

  python tools/infl_table_sizes.py [--sessions 64] [--msgs 16] [--bytes 4096]
"""
import argparse
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

CL_ORDER = (16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15)  # RFC 1951 3.2.7


class Bits:
    def __init__(self, data: bytes):
        self.d, self.p = data, 0

    def get(self, n: int) -> int:
        v = 0
        for i in range(n):
            v |= ((self.d[self.p >> 3] >> (self.p & 7)) & 1) << i
            self.p += 1
        return v


def canonical(lens):
    """(code, length) of each symbol with a non-zero length (RFC 1951 3.2.2)."""
    bl = collections.Counter(l for l in lens if l)
    code, nxt = 0, {}
    for l in range(1, 16):
        code = (code + bl.get(l - 1, 0)) << 1
        nxt[l] = code
    out = []
    for l in lens:
        if l:
            out.append((nxt[l], l))
            nxt[l] += 1
    return out


def decode_sym(bits: Bits, codes):
    """One symbol of a small canonical code (the code-length code) by linear search."""
    c, l = 0, 0
    while True:
        c = (c << 1) | bits.get(1)
        l += 1
        for s, (cc, ll) in codes.items():
            if ll == l and cc == c:
                return s


def header_lengths(data: bytes):
    """Literal/length and distance code lengths of the block at the start of data, or
    None for a stored / fixed-code block."""
    b = Bits(data)
    b.get(1)
    btype = b.get(2)
    if btype != 2:
        return None
    hlit, hdist, hclen = b.get(5) + 257, b.get(5) + 1, b.get(4) + 4
    cl = [0] * 19
    for i in range(hclen):
        cl[CL_ORDER[i]] = b.get(3)
    codes = {s: cw for s, cw in zip([s for s in range(19) if cl[s]], canonical(cl))}
    lens = []
    while len(lens) < hlit + hdist:
        s = decode_sym(b, codes)
        if s < 16:
            lens.append(s)
        elif s == 16:
            lens += [lens[-1]] * (3 + b.get(2))
        elif s == 17:
            lens += [0] * (3 + b.get(3))
        else:
            lens += [0] * (11 + b.get(7))
    return lens[:hlit], lens[hlit:hlit + hdist]


def sub_entries(lens, root: int) -> int:
    longest = {}
    for code, l in canonical(lens):
        if l > root:
            p = code >> (l - root)
            longest[p] = max(longest.get(p, 0), l)
    return sum(1 << (l - root) for l in longest.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=64)
    ap.add_argument("--msgs", type=int, default=16)
    ap.add_argument("--bytes", type=int, default=4096)
    args = ap.parse_args()
    from benchsupport.synth import deflate_batch
    desc, sf, payload, _ = deflate_batch(7, args.sessions, args.msgs, args.bytes, unique=args.sessions)
    pl = np.asarray(payload).tobytes() if not isinstance(payload, (bytes, bytearray)) else bytes(payload)
    lit = {r: [] for r in (7, 8, 9)}
    dist = {r: [] for r in (5, 6, 7)}
    maxl = collections.Counter()
    n_dyn = n_other = 0
    for d in desc:
        o, n = int(d["payload_off"]), int(d["payload_len"])
        h = header_lengths(pl[o:o + n])
        if h is None:
            n_other += 1
            continue
        n_dyn += 1
        ll, dl = h
        maxl[max(ll)] += 1
        for r in lit:
            lit[r].append(sub_entries(ll, r))
        for r in dist:
            dist[r].append(sub_entries(dl, r))
    print(f"messages: {n_dyn} dynamic-code blocks, {n_other} stored/fixed")
    print("longest literal/length code:", dict(sorted(maxl.items())))
    for name, tab in (("literal/length", lit), ("distance", dist)):
        for r, v in tab.items():
            a = np.array(v)
            print(f"{name} root {r} bits: sub-table entries p50 {int(np.percentile(a, 50))} "
                  f"p99 {int(np.percentile(a, 99))} max {int(a.max())}; "
                  f"lane table {1 << r} + max {int(a.max())} = {(1 << r) + int(a.max())} u16")


if __name__ == "__main__":
    main()
