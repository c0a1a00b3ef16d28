"""Probe (round 5): the stage line, then the encode line (slow placement), then three
more streams and the encode line again (fast placement), with markers in the trace:
run under rocprofv3 --kernel-trace --memory-copy-trace to compare the two encodes."""
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
print(json.dumps({"stages": bench.e2e_stages_line(ctx, dev, 3, 2)["value"]}), flush=True)
torch.cuda.synchronize()
print(json.dumps({"encode_a": bench.e2e_encode_line(ctx, dev, 2, 1)["value"]}), flush=True)
torch.cuda.synchronize()
keep = [torch.cuda.Stream(dev) for _ in range(3)]
print(json.dumps({"encode_b": bench.e2e_encode_line(ctx, dev, 2, 1)["value"]}), flush=True)
