"""Probe (round 5): how much the host-to-host encode line depends on which socket its
threads run on.  Prints the GPU's PCI address, NUMA node and local CPU list, then runs
the encode line with the process pinned to the GPU's local CPUs and to the CPUs of the
other node(s)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import snf4j_amd  # noqa: E402

dev = torch.device("cuda:0")
p = torch.cuda.get_device_properties(0)
bus = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
sysd = f"/sys/bus/pci/devices/{bus}"


def read(f):
    try:
        return open(f).read().strip()
    except OSError as e:
        return f"? ({e})"


def cpus(lst):
    out = set()
    for part in lst.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return out


node, local = read(f"{sysd}/numa_node"), read(f"{sysd}/local_cpulist")
allowed = os.sched_getaffinity(0)
print(json.dumps({"bus": bus, "numa_node": node, "local_cpulist": local, "allowed": len(allowed)}), flush=True)
loc = cpus(local) & allowed if not local.startswith("?") else set()
far = allowed - loc
for name, cs in (("local", loc), ("far", far), ("local", loc)):
    if not cs:
        continue
    os.sched_setaffinity(0, cs)
    ctx = snf4j_amd.Context(0)
    v = bench.e2e_encode_line(ctx, dev, 3, 2)["value"]
    ctx.close()
    print(json.dumps({"cpus": name, "n": len(cs), "encode": v}), flush=True)
