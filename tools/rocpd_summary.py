"""Summarise rocprofv3 rocpd databases (tools/profile_round.sh output):
per-kernel trace stats as CSV and per-kernel mean PMC values as JSON.

    python tools/rocpd_summary.py gpurun_out/prof_<tag> profiles/<name>
writes <name>_kernel_stats.csv and <name>_counters.json.
"""
import csv
import json
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+|tpe::\w+|at::native::\w+)", name)
    return m.group(1) if m else name[:60]


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration) from kernels group by name order by sum(duration) desc")
    rows = list(rows)
    tot = sum(r[2] for r in rows) or 1
    return [dict(kernel=short(r[0]), calls=r[1], total_us=r[2] / 1e3, avg_us=r[3] / 1e3,
                 min_us=r[4] / 1e3, max_us=r[5] / 1e3, pct=100.0 * r[2] / tot, name=r[0])
            for r in rows]


def counters(db):
    c = sqlite3.connect(db)
    acc = defaultdict(lambda: defaultdict(list))
    for name, cnt, val, disp in c.execute(
            "select kernel_name, counter_name, sum(value), dispatch_id from counters_collection "
            "group by dispatch_id, counter_name"):
        acc[short(name)][cnt].append(val)
    return {k: {cn: sum(v) / len(v) for cn, v in d.items()} for k, d in acc.items()}


def main(src, dst):
    stats = kernel_stats(os.path.join(src, "trace", "run_results.db"))
    with open(dst + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(stats[0]))
        w.writeheader()
        w.writerows(stats)
    out = {}
    for sub in sorted(os.listdir(src)):
        db = os.path.join(src, sub, "run_results.db")
        if sub != "trace" and os.path.exists(db):
            for k, d in counters(db).items():
                out.setdefault(k, {}).update(d)
    with open(dst + "_counters.json", "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for s in stats[:14]:
        print("%-28s %5d calls  avg %9.1f us  %5.1f%%" % (s["kernel"], s["calls"], s["avg_us"],
                                                          s["pct"]))
    for s in stats[:6]:
        k = s["kernel"]
        if k in out:
            print(k, {a: "%.4g" % b for a, b in out[k].items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
