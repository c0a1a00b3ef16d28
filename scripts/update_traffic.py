"""Point profiles/pmc_traffic.json (bench.py's roofline.traffic) at a PMC run:

  python scripts/update_traffic.py --round r04 --line north --key text_1048576x4096
  python scripts/update_traffic.py --round r04 --line configs1 --key binary_1048576x1024

reads profiles/<round>_<line>_pmc.json (scripts/pmc_report.py output of the
scripts/gpu_profiles.sh passes: FETCH_SIZE and WRITE_SIZE in separate rocprofv3
--pmc runs) and stores the dominant kernel's HBM bytes per launch, with the gfx950
FETCH_SIZE correction pmc_report already applied (x2 on 16-B streaming reads, KiB ->
bytes; MI355X_MICROARCH.md HBM/rocprofv3 section)."""
from __future__ import annotations

import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--line", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--kernel", default="k_piecesN<1, 1, 2>")
    a = ap.parse_args()
    src = os.path.join("profiles", f"{a.round}_{a.line}_pmc.json")
    with open(os.path.join(ROOT, src)) as fh:
        pmc = json.load(fh)
    # (the template arguments rocprof prints vary with the defaulted ones: match a prefix)
    name = a.kernel if a.kernel in pmc else next(k for k in pmc if k.startswith(a.kernel.rstrip(">")))
    r = pmc[name]
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    with open(path) as fh:
        out = json.load(fh)
    out[a.key] = {
        "correction": "FETCH_SIZE x2 (gfx950 half-count on 16-B streaming reads), KiB -> bytes",
        "fetch_bytes_per_launch": r["fetch_bytes"],
        "write_bytes_per_launch": r["write_bytes"],
        "hbm_bytes_per_launch": r["fetch_bytes"] + r["write_bytes"],
        "kernel": name,
        "launches": r["launches"],
        "avg_us_under_pmc": r.get("avg_us"),
        "raw_FETCH_SIZE_KiB": r["FETCH_SIZE"],
        "raw_WRITE_SIZE_KiB": r["WRITE_SIZE"],
        "round": a.round,
        "source": f"{src} (scripts/gpu_profiles.sh: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; "
                  "scripts/pmc_report.py)",
    }
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(a.key, out[a.key]["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
