"""How fast does a DEFLATE symbol stream self-synchronise?  A design study for
splitting one message's Huffman decode over several lanes:
a lane that starts at a guessed bit offset inside a block, with the block's tables
and in the literal/length context, decodes garbage until one of its symbol
boundaries coincides with a true one (same bit position, literal/length context);
from there on its symbols are the true ones.  The lane that decodes from the true
start stops at that boundary.

For the bench's inflate workload (benchsupport.synth.deflate_batch: level 6, context
takeover, chat/JSON-like text, 4 KiB messages) this decodes every message's first
dynamic block exactly (restated RFC 1951, checked against zlib's output), starts a
speculative decode at several fractions of the block, and reports how many symbols
and bits the speculation needs before it meets the true stream, and how often it
never does within the block.  CPU only.

  python tools/huff_sync_study.py [--sessions 16] [--fractions 0.25 0.5 0.75]
"""
from __future__ import annotations

import argparse
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227,
         258]
LEXT = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
         6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
CLORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self, data: bytes):
        self.d = data
        self.n = 8 * len(data)

    def get(self, pos: int, k: int) -> int:
        v = 0
        for i in range(k):
            p = pos + i
            if p >= self.n:
                raise EOFError
            v |= ((self.d[p >> 3] >> (p & 7)) & 1) << i
        return v


def canon(lens):
    """{(length, code reversed): symbol} for canonical codes of `lens`."""
    maxl = max(lens) if lens else 0
    cnt = [0] * (maxl + 1)
    for l in lens:
        if l:
            cnt[l] += 1
    code, nxt = 0, [0] * (maxl + 2)
    for l in range(1, maxl + 1):
        code = (code + cnt[l - 1]) << 1
        nxt[l] = code
    tab = {}
    for s, l in enumerate(lens):
        if l:
            c = nxt[l]
            nxt[l] += 1
            r = int(format(c, f"0{l}b")[::-1], 2)
            tab[(l, r)] = s
    return tab, maxl


def dec(bits: Bits, pos: int, tab, maxl):
    v = 0
    for l in range(1, maxl + 1):
        v |= bits.get(pos + l - 1, 1) << (l - 1)
        s = tab.get((l, v))
        if s is not None:
            return s, l
    raise ValueError("invalid code")


def header(bits: Bits, pos: int):
    """Block header at pos: (final, type, tables or None, bit position of the first symbol)."""
    final, typ = bits.get(pos, 1), bits.get(pos + 1, 2)
    pos += 3
    if typ != 2:
        return final, typ, None, pos
    hlit, hdist, hclen = bits.get(pos, 5) + 257, bits.get(pos + 5, 5) + 1, bits.get(pos + 10, 4) + 4
    pos += 14
    cl = [0] * 19
    for i in range(hclen):
        cl[CLORDER[i]] = bits.get(pos, 3)
        pos += 3
    ctab, cmax = canon(cl)
    lens = []
    while len(lens) < hlit + hdist:
        s, l = dec(bits, pos, ctab, cmax)
        pos += l
        if s < 16:
            lens.append(s)
        elif s == 16:
            lens += [lens[-1]] * (3 + bits.get(pos, 2))
            pos += 2
        elif s == 17:
            lens += [0] * (3 + bits.get(pos, 3))
            pos += 3
        else:
            lens += [0] * (11 + bits.get(pos, 7))
            pos += 7
    return final, typ, (canon(lens[:hlit]), canon(lens[hlit:])), pos


def symbols(bits: Bits, pos: int, tables, stop_pos=None, limit=1 << 30):
    """Decode from pos in the literal/length context: [(bit position, context)] of every
    code's start (context 0 literal/length, 1 distance), and the output length; stops at
    end of block, an invalid code, `limit` codes, or once past stop_pos."""
    (ltab, lmax), (dtab, dmax) = tables
    out, bounds = 0, []
    try:
        while len(bounds) < limit:
            if stop_pos is not None and pos >= stop_pos:
                break
            bounds.append((pos, 0))
            s, l = dec(bits, pos, ltab, lmax)
            pos += l
            if s < 256:
                out += 1
                continue
            if s == 256:
                break
            i = s - 257
            if i >= 29:
                raise ValueError("bad length")
            n = LBASE[i] + bits.get(pos, LEXT[i])
            pos += LEXT[i]
            bounds.append((pos, 1))
            ds, dl = dec(bits, pos, dtab, dmax)
            pos += dl
            if ds >= 30:
                raise ValueError("bad distance")
            pos += DEXT[ds]
            out += n
    except (ValueError, EOFError):
        return bounds, out, False
    return bounds, out, True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=16)
    ap.add_argument("--fractions", type=float, nargs="+", default=[0.25, 0.5, 0.75])
    ap.add_argument("--restart", action="store_true",
                    help="a speculative decode that hits an invalid code, or an end of block more than "
                         "--eob-slack bits before the stream's end, restarts one bit after where it "
                         "started (the lane cannot tell a false end of block otherwise)")
    ap.add_argument("--eob-slack", type=int, default=48)
    ap.add_argument("--window", type=int, default=1024, help="bits after the start a sync is looked for in")
    a = ap.parse_args()
    from benchsupport.synth import deflate_batch
    desc, sf, payload, plain = deflate_batch(0x1F1A, a.sessions, 16, 4096, unique=a.sessions)
    sync_syms, sync_bits, never, total = [], [], 0, 0
    blocks_per_msg = []
    for k in range(len(desc)):
        o, n = int(desc[k]["payload_off"]), int(desc[k]["payload_len"])
        data = bytes(payload[o:o + n]) + b"\x00\x00\xff\xff"
        bits = Bits(data)
        pos, nblk, first = 0, 0, None
        while pos + 3 <= bits.n:  # walk the message's blocks (the true decode)
            final, typ, tabs, p = header(bits, pos)
            nblk += 1
            if typ == 0:  # stored (the sync flush's empty block)
                p = (p + 7) & ~7
                pos = p + 32 + 8 * bits.get(p, 16)
            elif typ == 2:
                b, _, ok = symbols(bits, p, tabs)
                assert ok
                if first is None:
                    first = (tabs, b, p)
                s_, l_ = dec(bits, b[-1][0], tabs[0][0], tabs[0][1])
                assert s_ == 256
                pos = b[-1][0] + l_
            else:
                break  # (fixed-code blocks: not in this workload)
            if final:
                break
        blocks_per_msg.append(nblk)
        if first is None:
            continue
        tabs, truth, p0 = first
        true_set = set(truth)
        end = truth[-1][0]
        for f in a.fractions:
            total += 1
            start = p0 + int((end - p0) * f)
            wasted = 0  # codes decoded by starts that were abandoned
            for _ in range(64 if a.restart else 1):
                spec, _, ok = symbols(bits, start, tabs, limit=4096)
                # (a literal/length boundary: at a distance code the length before it would differ)
                hit = next((i for i, bnd in enumerate(spec) if bnd[1] == 0 and bnd in true_set
                            and bnd[0] - start < a.window), None)
                if hit is not None or not a.restart:
                    break
                # what the lane sees: an invalid code, or an end of block far from the stream's end
                last = spec[-1][0] if spec else start
                if ok and bits.n - last <= a.eob_slack:
                    break  # a plausible end: the lane would stop here (no sync: the head decodes alone)
                wasted += len(spec)
                start += 1
            if hit is None:
                never += 1
            else:
                sync_syms.append(hit + wasted)
                sync_bits.append(spec[hit][0] - (p0 + int((end - p0) * f)))
    ss, sb = np.array(sync_syms), np.array(sync_bits)
    print(f"messages {len(desc)}, blocks per message: mean {np.mean(blocks_per_msg):.2f}, max {max(blocks_per_msg)}")
    print(f"speculative starts {total}: synchronised {len(ss)}, never within the block {never}")
    for name, v in (("codes before sync", ss), ("bits before sync", sb)):
        print(f"  {name}: p50 {np.percentile(v, 50):.0f}  p90 {np.percentile(v, 90):.0f}  "
              f"p99 {np.percentile(v, 99):.0f}  max {v.max()}")
    # the true decode of message 0 against zlib (the restatement is exact)
    o, n = int(desc[0]["payload_off"]), int(desc[0]["payload_len"])
    ref = zlib.decompressobj(-15).decompress(bytes(payload[o:o + n]) + b"\x00\x00\xff\xff")
    print(f"message 0: zlib inflates {len(ref)} bytes")


if __name__ == "__main__":
    main()
