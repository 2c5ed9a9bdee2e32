"""Per-level kernel timeline from a rocprofv3 --kernel-trace rocpd database:
for the last level(s) of a run, every dispatch's start offset from the
level's first kernel, duration, queue and the idle gap before it on the GPU
(diagnostic for the multi-GPU critical path).

    python tools/timeline.py gpurun_out/tl8 [levels=2] [first-kernel]

(no first kernel: levels are split at GPU idle gaps of more than 40 us)

The last level of a bench.py trace is its untimed all-groups timer pass
(HIP events around every kernel group, ~10 us each on the stream): look at
the levels before it for the timed steps' timeline.
"""
import glob
import os
import re
import sqlite3
import sys


def short(name):
    m = re.search(r"(k_\w+|__amd_rocclr_\w+|at::native::\w+)", name)
    return m.group(1) if m else name[:40]


def main(src, levels=2, first=None):
    db = sorted(glob.glob(os.path.join(src, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    rows = list(c.execute("select name, start, end%s from kernels order by start"
                          % ((", " + qcol) if qcol else "")))
    starts = []
    if first:
        for i, r in enumerate(rows):  # a level's first `first` kernel (a second one
            if short(r[0]) == first and (not starts or r[1] - rows[starts[-1]][1] > 100e3):
                starts.append(i)      # within 100 us is the same level's, on the side stream)
    else:  # a level starts after the GPU was idle for more than 40 us
        busy = None
        for i, r in enumerate(rows):
            if busy is None or r[1] - busy > 40e3:
                starts.append(i)
            busy = r[2] if busy is None else max(busy, r[2])
    for li in starts[-levels:]:
        nxt = [s for s in starts if s > li]
        seg = rows[li:nxt[0] if nxt else len(rows)]
        t0 = seg[0][1]
        busy_end = t0
        print("level at dispatch %d: %d kernels, span %.1f us" % (
            li, len(seg), (max(r[2] for r in seg) - t0) / 1e3))
        for r in seg:
            gap = max(0, r[1] - busy_end) / 1e3
            busy_end = max(busy_end, r[2])
            print("  %-28s start %7.1f  dur %6.1f  gap %5.1f  q %s" % (
                short(r[0]), (r[1] - t0) / 1e3, (r[2] - r[1]) / 1e3, gap,
                r[3] if qcol else "-"))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) if a.isdigit() else a for a in sys.argv[2:]))
