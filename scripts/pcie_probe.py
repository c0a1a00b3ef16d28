"""PCIe probe: pinned H2D alone, D2H alone, and both at once on two streams (GB/s)."""
import time

import torch

N = 1 << 30
dev = torch.device("cuda", 0)
h_src = torch.empty(N, dtype=torch.uint8).pin_memory()
h_dst = torch.empty(N, dtype=torch.uint8).pin_memory()
d_a = torch.empty(N, dtype=torch.uint8, device=dev)
d_b = torch.empty(N, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def run(h2d, d2h, reps=4):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_src, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_dst.copy_(d_b, non_blocking=True)
    torch.cuda.synchronize(dev)
    t = time.perf_counter() - t0
    return reps * N * (int(h2d) + int(d2h)) / t / 1e9


run(True, True, 1)
print(f"H2D {run(True, False):.1f} GB/s  D2H {run(False, True):.1f} GB/s  both {run(True, True):.1f} GB/s (sum)")
