"""Device timeline from a rocprofv3 SQLite output (run_results.db): kernels and memory
copies in start order over the last `--ms` milliseconds of the trace, with the spans in
which neither ran (device idle: the host is the bound there).
Usage: python tools/rocpd_timeline.py DB [--ms 20] [--min-us 20]"""
import argparse
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--ms", type=float, default=20.0, help="the trace's last this many ms")
ap.add_argument("--min-us", type=float, default=20.0, help="list only events and gaps at least this long")
a = ap.parse_args()
c = sqlite3.connect(a.db)
ev = [("K", re.sub(r"[(<].*", "", n.replace("(anonymous namespace)::", ""))[:40], s, e, sid, 0)
      for n, s, e, sid in c.execute("select name, start, end, stream_id from kernels")]
ev += [("C", n[:40], s, e, sid, sz)
       for n, s, e, sid, sz in c.execute("select name, start, end, stream_id, size from memory_copies")]
ev.sort(key=lambda x: x[2])
t_end = max(x[3] for x in ev)
t0 = t_end - a.ms * 1e6
ev = [x for x in ev if x[3] >= t0]
t0 = ev[0][2]
busy_to = ev[0][2]
idle = 0
for kind, name, s, e, sid, sz in ev:
    if s > busy_to:
        gap = (s - busy_to) / 1e3
        idle += gap
        if gap >= a.min_us:
            print(f"{(busy_to - t0) / 1e3:10.1f} us   -- idle {gap:8.1f} us --")
    busy_to = max(busy_to, e)
    d = (e - s) / 1e3
    if d >= a.min_us:
        extra = f" {sz / 1e6:8.2f} MB {sz / (e - s):6.1f} GB/s" if kind == "C" and e > s else ""
        print(f"{(s - t0) / 1e3:10.1f} us + {d:8.1f}  {kind} s{sid:<3d} {name}{extra}")
span = (t_end - t0) / 1e3
print(f"span {span:.1f} us, device idle {idle:.1f} us ({100 * idle / span:.1f}%)")
