"""CPU prototype of the split-lane lane decode planned for k_infl_tok (DESIGN.md §9
item 1): two lanes decode one message's dynamic block, the head from its start, the
tail speculatively from the middle; they are joined where the head meets one of the
tail's literal/length boundaries, and the tail's tokens and literals after that point
are moved behind the head's.  This checks the splice rules on the bench's inflate
workload: the joined token and literal streams, in k_infl_tok's format (a literal-run
token = its count; a match = 0x80000000 | (length - 3) << 16 | (distance - 1)), must
replay to exactly zlib's output.  Test/design infrastructure, CPU only.

  python tools/split_decode_proto.py [--sessions 8] [--window 1024] [--split 0.5]
"""
from __future__ import annotations

import argparse
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from huff_sync_study import DBASE, DEXT, LBASE, LEXT, Bits, dec, header  # noqa: E402


def lane(bits: Bits, pos: int, tables, stop=None, window=None):
    """One lane's decode of a block from bit `pos` (literal/length context), in
    k_infl_tok's output format.  stop(pos) -> True ends it at that literal/length
    boundary (the head's join test); window = (g, w): the literal/length boundaries in
    [g, g + w) and the counters there, {pos: (ntok, nlit, run)} (what the tail's bitmap
    and its counting re-decode give).  Returns (tokens, lits, run, end, state, marks)
    with state 'eob' | 'stop' | 'bad'."""
    (ltab, lmax), (dtab, dmax) = tables
    toks, lits, run, marks = [], bytearray(), 0, {}
    try:
        while True:
            if window is not None and window[0] <= pos < window[0] + window[1]:
                marks[pos] = (len(toks), len(lits), run)
            if stop is not None and stop(pos):
                return toks, lits, run, pos, "stop", marks
            s, n = dec(bits, pos, ltab, lmax)
            pos += n
            if s < 256:
                lits.append(s)
                run += 1
                continue
            if s == 256:
                return toks, lits, run, pos, "eob", marks
            i = s - 257
            if i >= 29:
                return toks, lits, run, pos, "bad", marks
            ml = LBASE[i] + bits.get(pos, LEXT[i])
            pos += LEXT[i]
            ds, dn = dec(bits, pos, dtab, dmax)
            pos += dn
            if ds >= 30:
                return toks, lits, run, pos, "bad", marks
            dist = DBASE[ds] + bits.get(pos, DEXT[ds])
            pos += DEXT[ds]
            if run:
                toks.append(run)
                run = 0
            toks.append(0x80000000 | ((ml - 3) << 16) | (dist - 1))
    except (ValueError, EOFError):
        return toks, lits, run, pos, "bad", marks


def replay(toks, lits, history=b""):
    out = bytearray(history)
    li = 0
    for t in toks:
        if t & 0x80000000:
            ml, d = ((t >> 16) & 255) + 3, (t & 0x7FFF) + 1
            for _ in range(ml):
                out.append(out[-d])
        else:
            out += lits[li:li + t]
            li += t
    return bytes(out[len(history):])


def split_block(bits: Bits, p0: int, tables, frac: float, window: int, eob_slack: int = 48):
    """The head/tail decode of the block at p0 and their join.  Returns (toks, lits,
    run, end, how) as one lane's decode of the block would."""
    whole = lane(bits, p0, tables)
    if whole[4] != "eob":
        return whole[:4] + ("whole",)
    # the tail: from the middle of what is left of the stream, restarting one bit later
    # after an invalid code or an end of block far from the stream's end
    g = p0 + int((bits.n - p0) * frac)
    for _ in range(64):
        t = lane(bits, g, tables, window=(g, window))
        if t[4] == "eob" and bits.n - t[3] <= eob_slack:
            break
        g += 1
    else:
        return whole[:4] + ("no tail",)
    tmarks = {p for p in t[5]}
    # the head: from the start, ending at its first literal/length boundary the tail also had
    h = lane(bits, p0, tables, stop=lambda p: p in tmarks)
    if h[4] != "stop":
        return h[:4] + ("no join",)
    P = h[3]
    ntok_p, nlit_p, run_p = t[5][P]  # the tail's counters there (its counting re-decode)
    # splice: the head closes its literal run at P; the tail's first token after P, if a
    # literal run, loses the run_p literals it counted before P
    toks = list(h[0]) + ([h[2]] if h[2] else [])
    rest = list(t[0][ntok_p:])
    run = t[2]
    if rest and not (rest[0] & 0x80000000):
        rest[0] -= run_p
        if rest[0] == 0:
            rest.pop(0)
    elif not rest:
        run -= run_p  # no token after P: the pending run is what follows P
    toks += rest
    lits = h[1] + t[1][nlit_p:]
    return toks, lits, run, t[3], "split"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=8)
    ap.add_argument("--window", type=int, default=1024)
    ap.add_argument("--split", type=float, default=0.5)
    a = ap.parse_args()
    from benchsupport.synth import deflate_batch
    desc, sf, payload, plain = deflate_batch(0x5B1, a.sessions, 16, 4096, unique=a.sessions)
    counts, head_steps, tail_steps, whole_steps = {}, [], [], []
    for s in range(a.sessions):
        d = zlib.decompressobj(-15)
        history = b""
        for k in range(int(sf[s]), int(sf[s + 1])):
            o, n = int(desc[k]["payload_off"]), int(desc[k]["payload_len"])
            data = bytes(payload[o:o + n]) + b"\x00\x00\xff\xff"
            ref = d.decompress(data)
            bits = Bits(data)
            final, typ, tabs, p0 = header(bits, 0)
            assert typ == 2 and not final
            toks, lits, run, end, how = split_block(bits, p0, tabs, a.split, a.window)
            counts[how] = counts.get(how, 0) + 1
            if run:
                toks.append(run)  # end_run (the stored empty block after it adds nothing)
            got = replay(toks, lits, history)
            assert got == ref, (s, k, how)
            history = (history + ref)[-32768:]
    print(f"messages {sum(counts.values())}: {counts}; every joined stream replays to zlib's output")


if __name__ == "__main__":
    main()
