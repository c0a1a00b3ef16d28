"""Per-wave averages of the k_inflate counters in a rocprofv3 counter_collection.csv."""
import collections
import csv
import glob
import sys

f = sys.argv[1] if len(sys.argv) > 1 else sorted(glob.glob("gpurun_out/pmc_infl/**/*counter_collection.csv", recursive=True))[-1]
agg = collections.defaultdict(float)
waves = 0.0
for r in csv.DictReader(open(f)):
    if "k_inflate" in r.get("Kernel_Name", ""):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            waves += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"{k:20s} {v / max(1.0, waves):14.1f} per wave")
