"""Kernel statistics from a rocprofv3 SQLite output (run_results.db): per kernel the
calls, total and mean duration, optionally only dispatches after the first `--skip`
of a given kernel (warm-up).  Usage: python tools/rocpd_stats.py DB [--last-ms N]"""
import argparse
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches in time order")
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = c.execute("select name, start, end, duration, stream_id from kernels order by start").fetchall()
agg = {}
for name, s, e, d, sid in rows:
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[:60]
    t = agg.setdefault(n, [0, 0])
    t[0] += 1
    t[1] += d
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':60s} {'calls':>6s} {'total_ms':>10s} {'mean_us':>10s} {'pct':>6s}")
for n, (k, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{n:60s} {k:6d} {d / 1e6:10.3f} {d / k / 1e3:10.1f} {100 * d / tot:6.1f}")
if a.timeline:
    t0 = rows[-a.timeline][1]
    for name, s, e, d, sid in rows[-a.timeline:]:
        print(f"{(s - t0) / 1e3:10.1f} us +{d / 1e3:8.1f} stream {sid} {re.sub(r'[(<].*', '', name.replace('(anonymous namespace)::', ''))[:50]}")
