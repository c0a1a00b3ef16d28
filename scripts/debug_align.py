"""GPU probe: decode one masked frame at every source alignment and payload length
class; print payload / verdict mismatches against the oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import pyoracle as O
from tests import wsgen
import snf4j_amd
from snf4j_amd._lib import STATE_DTYPE
ctx = snf4j_amd.Context(0)
cfg = snf4j_amd.decoder_cfg(False, False, 65536, True)
rng = np.random.default_rng(1)
bad = 0
for pad in range(0, 8):
    for n in (1, 5, 16, 17, 33, 100, 272, 1000):
        body = wsgen.rand_text(rng, n)
        pre = [wsgen.build_frame(2, True, 0, b"x" * pad, True, (1, 2, 3, 4))]
        f = wsgen.build_frame(1, True, 0, body, True, (5, 6, 7, 8))
        wire, off, sf = wsgen.make_batch([pre + [f]])
        st = np.zeros(1, dtype=STATE_DTYPE)
        p, d, r = ctx.decode_host(cfg, wire, off, sf, st)
        po, do, ro = O.Batch(False, False, 65536, True, 1).decode(wire, off, sf)
        gp = p[int(d[1]["payload_off"]):][:len(body)].tobytes()
        if int(r[0]["n_delivered"]) != 2 or gp != body:
            bad += 1
            print("pad", pad, "src&3", (int(off[1]) + (8 if len(body) > 125 else 6)) & 3, "n", len(body),
                  "res", r[0], "oracle", ro[0])
            diff = [i for i in range(min(len(gp), len(body))) if gp[i] != body[i]]
            print("  first diffs", diff[:8], gp[:24].hex(), body[:24].hex())
print("mismatches", bad)
