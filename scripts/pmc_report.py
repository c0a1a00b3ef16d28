"""Per-kernel report of a scripts/gpu_pmc.sh run (rocprofv3 kernel trace + PMC passes).

  python scripts/pmc_report.py gpurun_out/prof/<tag> [--json out.json] [--kernels k_piecesN,...]

Per kernel: launches and average duration (kernel trace), and per launch the
average of every counter collected.  Derived (MI355X_MICROARCH.md, HBM/rocprofv3
section and PMC table): FETCH_SIZE / WRITE_SIZE are KiB, FETCH_SIZE counts half the
bytes of 16-B-per-lane streaming reads (doubled here); SQ_* cycle counters count
quad-cycles; SIMD VALU utilisation = SQ_INSTS_VALU x 4 cycles (a wave64 VALU op
on a 16-lane SIMD) / (duration x 2.4 GHz x 256 CUs x 4 SIMDs).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

CLOCK_GHZ, CUS, SIMDS = 2.4, 256, 4


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    for p in ("void ", "ws::", "wsb::"):
        n = n.replace(p, "")
    return n.strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--kernels", default="")
    a = ap.parse_args()
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "kt", "*kernel_trace.csv")):
        for row in csv.DictReader(open(f)):
            dur[short(row["Kernel_Name"])].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(a.dir, "*", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            cnt[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    want = [k for k in a.kernels.split(",") if k]
    out = {}
    for k in sorted(set(dur) | set(cnt)):
        if want and k not in want:
            continue
        d = dur.get(k, [])
        r = {"launches": len(d), "avg_us": round(sum(d) / len(d), 2) if d else None}
        c = {n: sum(v) / len(v) for n, v in cnt.get(k, {}).items()}
        r.update({n: round(v, 1) for n, v in c.items()})
        if "FETCH_SIZE" in c:
            r["fetch_bytes"] = round(c["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in c:
            r["write_bytes"] = round(c["WRITE_SIZE"] * 1024)
        w = c.get("SQ_WAVES")
        if w:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES"):
                if n in c:
                    r[n.lower().replace("sq_", "") + "_per_wave"] = round(c[n] / w, 1)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if n in c:
                    r[n.lower().replace("sq_", "") + "_frac_of_wave_cycles"] = round(c[n] / wc, 3)
        if "SQ_INSTS_VALU" in c and r["avg_us"]:
            # a wave64 VALU instruction takes 4 issue cycles for a wave alone on its SIMD, 2 on
            # the SIMD-32's pipe once two or more waves share it (MI355X_MICROARCH.md)
            r["simd_valu_util"] = round(c["SQ_INSTS_VALU"] * 4 / (r["avg_us"] * 1e3 * CLOCK_GHZ * CUS * SIMDS), 3)
            r["valu_pipe_frac"] = round(c["SQ_INSTS_VALU"] * 2 / (r["avg_us"] * 1e3 * CLOCK_GHZ * CUS * SIMDS), 3)
        out[k] = r
    for k, r in out.items():
        print(k, json.dumps(r))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
