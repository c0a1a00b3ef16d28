"""The mixed-batch planner (snf4j_amd/synth.py, BASELINE configs[2]): structure only, CPU."""
import numpy as np

from benchsupport.synth import header_len, mixed_plan


def test_plan_structure():
    t, off, sf, wl, info = mixed_plan(3, 37, 8 << 20, frag_frac=0.3, bad_frac=0.2)
    n = len(t)
    assert info["frames"] == n and int(off[-1]) == wl and sf[-1] == n and sf[0] == 0
    assert np.all(np.diff(sf.astype(np.int64)) >= 0)
    assert np.array_equal(off[:-1], t["wire_off"])
    assert np.array_equal(np.diff(off.astype(np.int64)), header_len(t["payload_len"], True) + t["payload_len"])
    # fragments tile their message exactly, first fragment carries the opcode, last one FIN
    k = 0
    msgs = 0
    while k < n:
        assert t["opcode"][k] in (1, 2) and t["msg_pos"][k] == 0
        L = int(t["msg_len"][k])
        pos = 0
        while True:
            assert int(t["msg_pos"][k]) == pos and t["payload_len"][k] >= 1
            pos += int(t["payload_len"][k])
            fin = bool(t["flags"][k] & 0x80)
            k += 1
            if fin:
                break
            assert t["opcode"][k] == 0
        assert pos == L
        msgs += 1
    assert msgs == info["messages"]
    assert (t["text"][t["inject_pos"] >= 0] == 1).all()
    assert 64 <= t["msg_len"].min() and t["msg_len"].max() <= 65536


def test_deflate_batch_plan_inflates_with_zlib():
    """The permessage-deflate bench batch (benchsupport.synth.deflate_batch): every
    session's messages inflate with zlib, context takeover, tail appended."""
    import zlib
    from benchsupport.synth import deflate_batch
    desc, sf, pl, plain = deflate_batch(7, 4, 3, 512, unique=2)
    total = 0
    for s in range(len(sf) - 1):
        d = zlib.decompressobj(-15)
        for k in range(int(sf[s]), int(sf[s + 1])):
            o, n = int(desc[k]["payload_off"]), int(desc[k]["payload_len"])
            total += len(d.decompress(pl[o:o + n].tobytes() + b"\x00\x00\xff\xff"))
    assert total == plain
