"""Probe (round 5): the stage line (burst) in one process after 0..3 more streams were
created, twice over, to see how much the runtime's placement of the batcher's streams
on hardware queues moves it (run with GPU_MAX_HW_QUEUES 4 and 16)."""
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
keep = []
out = []
for rnd in range(2):
    for k in range(4):
        out.append(round(bench.e2e_stages_line(ctx, dev, 3, 2)["value"], 2))
        keep.append(torch.cuda.Stream(dev))
print(json.dumps({"hwq": os.environ.get("GPU_MAX_HW_QUEUES", "default"), "stages": out}), flush=True)
