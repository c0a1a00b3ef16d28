"""Probe (round 5): the encode host-to-host line measured again after the stage line,
in one process, then after creating and destroying 1-3 more streams, to tell whether
what slows it is where the runtime puts its new streams (hardware queue sharing)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import snf4j_amd  # noqa: E402

dev = torch.device("cuda:0")
ctx = snf4j_amd.Context(0, stream=torch.cuda.current_stream(dev))
bench.apply_tuning(ctx)


def enc(tag):
    print(json.dumps({"after": tag, "encode": bench.e2e_encode_line(ctx, dev, 3, 2)["value"]}), flush=True)


enc("nothing")
print(json.dumps({"stages": bench.e2e_stages_line(ctx, dev, 3, 2)["value"]}), flush=True)
enc("stages")
keep = []
for k in range(1, 4):
    keep.append(torch.cuda.Stream(dev))  # one more stream alive before the encode line's
    enc(f"stages + {k} extra streams alive")
