"""Probe: the encode and stage host-to-host lines in a fresh process with the in-suite
warm-up count (W=1), to separate warm-up from in-process state (round 5)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import snf4j_amd  # noqa: E402

dev = torch.device("cuda:0")
ctx = snf4j_amd.Context(0)
print(json.dumps({"encode_w1": bench.e2e_encode_line(ctx, dev, 3, 1)["value"]}), flush=True)
print(json.dumps({"stages_w1": bench.e2e_stages_line(ctx, dev, 3, 1)["value"]}), flush=True)
