"""Debug: mixed batch (configs[2]) at a given size, GPU decode vs oracle, per-session diff."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import pyoracle
from snf4j_amd import Context, decoder_cfg
from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE, lib
from snf4j_amd.synth import mixed_plan

seed, sessions, mib = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
pyoracle.build()
t, off, sf, wl, info = mixed_plan(seed, sessions, mib << 20)
dev = torch.device("cuda", 0)
ctx = Context(0)
tab = torch.from_numpy(t.view(np.uint8).copy()).to(dev)
wire = torch.zeros(wl + 64, dtype=torch.uint8, device=dev)
ctx.synth_frames(tab, wire)
n, n_s = len(t), len(sf) - 1
cap = int(lib.wsg_decode_payload_bound(wl, n))
payload = torch.empty(cap, dtype=torch.uint8, device=dev)
desc = torch.empty(n * 16, dtype=torch.uint8, device=dev)
res = torch.empty(n_s * 16, dtype=torch.uint8, device=dev)
state = torch.zeros(n_s * 8, dtype=torch.uint8, device=dev)
ctx.decode_device(decoder_cfg(False, False, 65536, True), wire, torch.from_numpy(off.astype(np.int64)).to(dev),
                  torch.from_numpy(sf.astype(np.int32)).to(dev), state, payload, desc, res, wire_len=wl)
torch.cuda.synchronize(dev)
hw = wire[:wl].cpu().numpy()
gd = desc.cpu().numpy().view(DESC_DTYPE)
gr = res.cpu().numpy().view(RESULT_DTYPE)
t0 = time.time()
op, od, orr = pyoracle.Batch(False, False, 65536, True, n_s).decode(hw, off, sf)
print(f"wire {wl} frames {n} oracle {time.time()-t0:.1f}s; gpu err sessions {(gr['error']!=0).sum()} "
      f"oracle {(orr['error']!=0).sum()} planned {len(info['bad_sessions'])}", flush=True)
bad = [s for s in range(n_s) if tuple(gr[s]) != tuple(orr[s])]
print("mismatching sessions:", len(bad), bad[:10])
for s in bad[:5]:
    print("session", s, "gpu", gr[s], "oracle", orr[s])
    k = int(sf[s]) + int(min(gr[s]["n_delivered"], orr[s]["n_delivered"]))
    for kk in range(max(int(sf[s]), k - 2), min(k + 2, int(sf[s + 1]))):
        print("  frame", kk, t[kk], "gpu desc", gd[kk], "ora desc", od[kk], "off", off[kk])
