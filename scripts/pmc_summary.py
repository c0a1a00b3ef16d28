"""Condense a scripts/gpu_profile.sh run (gpurun_out/prof_*) into profiles/.

  python scripts/pmc_summary.py --round r01 --key text_1048576x4096 [--src gpurun_out]

Writes
  profiles/<round>_<key>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<round>_<key>_pmc.csv            per kernel: launches, FETCH_SIZE/WRITE_SIZE per launch
  profiles/pmc_traffic.json[<key>]          HBM bytes per launch of the dominant kernel (bench.py
                                            roofline.traffic)

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): the counters are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read, so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "ws::"):
        n = n.replace(p, "")
    return n.strip()


def counters(path: str, counter: str):
    per = defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] == counter:
                per[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--kernel", default="k_piecesN")
    ap.add_argument("--alg-bytes", type=float, default=None, help="algorithmic bytes per launch (for the ratio)")
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    tag = f"{a.round}_{a.key}"

    stats = glob.glob(os.path.join(a.src, "prof_kt", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(out_dir, f"{tag}_kernel_stats.csv"))
    fetch = counters(glob.glob(os.path.join(a.src, "prof_fetch", "*counter_collection.csv"))[0], "FETCH_SIZE")
    write = counters(glob.glob(os.path.join(a.src, "prof_write", "*counter_collection.csv"))[0], "WRITE_SIZE")
    rows = []
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        rows.append((k, max(len(f), len(w)), fk, wk, (2 * fk + wk) * 1024))
    with open(os.path.join(out_dir, f"{tag}_pmc.csv"), "w", newline="") as fh:
        wr = csv.writer(fh)
        wr.writerow(["kernel", "launches", "FETCH_SIZE_KiB_per_launch(raw)", "WRITE_SIZE_KiB_per_launch",
                     "hbm_bytes_per_launch(2*FETCH+WRITE)"])
        for r in rows:
            wr.writerow([r[0], r[1], f"{r[2]:.1f}", f"{r[3]:.1f}", f"{r[4]:.0f}"])
    dom = [r for r in rows if r[0].startswith(a.kernel)]
    if not dom:
        raise SystemExit(f"kernel {a.kernel} not in the PMC output")
    k, n, fk, wk, tb = dom[0]
    jpath = os.path.join(out_dir, "pmc_traffic.json")
    data = {}
    if os.path.exists(jpath):
        with open(jpath) as fh:
            data = json.load(fh)
    entry = {
        "kernel": k,
        "launches": n,
        "fetch_bytes_per_launch": 2 * fk * 1024,
        "write_bytes_per_launch": wk * 1024,
        "hbm_bytes_per_launch": tb,
        "raw_FETCH_SIZE_KiB": fk,
        "raw_WRITE_SIZE_KiB": wk,
        "correction": "FETCH_SIZE x2 (gfx950 half-count on 16-B streaming reads), KiB -> bytes",
        "source": f"profiles/{tag}_pmc.csv (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes)",
        "round": a.round,
    }
    if a.alg_bytes:
        entry["alg_bytes_per_launch"] = a.alg_bytes
        entry["traffic_over_alg"] = tb / a.alg_bytes
    data[a.key] = entry
    with open(jpath, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps({a.key: entry}, indent=1))


if __name__ == "__main__":
    main()
