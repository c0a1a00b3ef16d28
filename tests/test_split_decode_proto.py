"""The splice rules of the planned split-lane inflate decode,
on the CPU prototype (tools/split_decode_proto.py): head and tail lane streams joined
at the head's first literal/length boundary the tail also had replay to exactly
zlib's output, with context takeover across messages."""
import os
import sys
import zlib

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_split_join_replays_to_zlib():
    import split_decode_proto as sp
    from benchsupport.synth import deflate_batch
    from huff_sync_study import Bits, header
    desc, sf, payload, _ = deflate_batch(0x5B1, 2, 16, 4096, unique=2)
    how = {}
    for s in range(2):
        d = zlib.decompressobj(-15)
        history = b""
        for k in range(int(sf[s]), int(sf[s + 1])):
            o, n = int(desc[k]["payload_off"]), int(desc[k]["payload_len"])
            data = bytes(payload[o:o + n]) + b"\x00\x00\xff\xff"
            ref = d.decompress(data)
            bits = Bits(data)
            _, typ, tabs, p0 = header(bits, 0)
            assert typ == 2
            toks, lits, run, _, h = sp.split_block(bits, p0, tabs, 0.5, 1024)
            how[h] = how.get(h, 0) + 1
            if run:
                toks.append(run)
            assert sp.replay(toks, lits, history) == ref, (s, k, h)
            history = (history + ref)[-32768:]
    assert how.get("split", 0) >= 28, how  # the join is the common case
