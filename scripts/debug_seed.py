"""GPU probe: rerun the random-session parity case of one seed, report mismatching
sessions and retry each alone."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import pyoracle as O
from tests import wsgen
import snf4j_amd
from snf4j_amd._lib import STATE_DTYPE
ctx = snf4j_amd.Context(0)
for seed in [int(x) for x in sys.argv[1:]] or [0]:
    rng = np.random.default_rng(100 + seed)
    cm = bool(seed & 1); ext = bool(seed & 2); maxp = [65536, 512, 131072][seed % 3]
    sessions = []
    for s in range(int(rng.integers(1, 120))):
        inj = None
        if rng.random() < 0.35:
            inj = wsgen.INJECT_KINDS[int(rng.integers(0, len(wsgen.INJECT_KINDS)))]
            if inj == "max_payload":
                inj = "too_long"
        sessions.append(wsgen.session_frames(rng, int(rng.integers(0, 12)), client_mode=cm, allow_ext=ext,
                                             max_payload=maxp, inject=inj))
    cfg = snf4j_amd.decoder_cfg(cm, ext, maxp, seed % 4 != 3)
    wire, off, sf = wsgen.make_batch(sessions)
    st = np.zeros(len(sessions), dtype=STATE_DTYPE)
    p, d, r = ctx.decode_host(cfg, wire, off, sf, st)
    po, do, ro = O.Batch(cm, ext, maxp, seed % 4 != 3, len(sessions)).decode(wire, off, sf)
    for s in range(len(sessions)):
        a = (int(r[s]["n_delivered"]), int(r[s]["error"]), int(r[s]["detail"]))
        b = (int(ro[s]["n_delivered"]), int(ro[s]["error"]), int(ro[s]["detail"]))
        if a != b:
            k = int(sf[s]) + min(a[0], b[0])
            print("seed", seed, "session", s, "gpu", a, "oracle", b, "frame", k, "off", int(off[k]),
                  "len", int(off[k + 1] - off[k]), "status", [int(x) for x in d["status"][sf[s]:sf[s + 1]]])
            w2, o2, s2 = wsgen.make_batch([sessions[s]])
            st2 = np.zeros(1, dtype=STATE_DTYPE)
            _, d2, r2 = ctx.decode_host(cfg, w2, o2, s2, st2)
            print("   alone:", r2[0], [int(x) for x in d2["status"]])
print("done")
