"""Per-step GPU timeline from a rocprofv3 --kernel-trace --memory-copy-trace
database (diagnostic): kernels and copies in start order with the idle gap
before each, for the last step of the run.

    python tools/timeline.py <run_results.db> [first-kernel-of-step]
"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
marker = sys.argv[2] if len(sys.argv) > 2 else "k_gather_obs"
rows = [("K", n, s, e) for n, s, e in db.execute("select name, start, end from kernels")]
rows += [("C", "%s %dB" % (n, sz), s, e)
         for n, s, e, sz in db.execute("select name, start, end, size from memory_copies")]
rows.sort(key=lambda r: r[2])
starts = [i for i, r in enumerate(rows) if r[0] == "K" and marker in r[1]]
if len(starts) < 2:
    raise SystemExit("need two steps starting with %s" % marker)
seg = rows[starts[-2]:starts[-1]]
t0 = seg[0][2]
prev_end = None
busy = 0
for kind, name, s, e in seg:
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += e - s
    print("%8.1f us  gap %7.1f  dur %7.1f  %s %s" % ((s - t0) / 1e3, gap, (e - s) / 1e3, kind,
                                                     name[:70]))
    prev_end = e if prev_end is None else max(prev_end, e)
span = (seg[-1][3] - t0) / 1e3
print("step span %.1f us, busy %.1f us, next step starts %.1f us after this one's start"
      % (span, busy / 1e3, (rows[starts[-1]][2] - t0) / 1e3))
