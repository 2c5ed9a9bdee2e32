"""Per-kernel, per-wave PMC averages of a rocprofv3 counter_collection.csv."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    by[m.group(1) if m else r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kn, agg in by.items():
    w = sum(agg["SQ_WAVES"]) / len(agg["SQ_WAVES"]) if "SQ_WAVES" in agg else 1.0
    print(sys.argv[2] if len(sys.argv) > 2 else "", kn, "waves %.0f" % w,
          {k[8:] if k.startswith("SQ_INSTS") else k: "%.1f" % (sum(v) / len(v) / w)
           for k, v in agg.items() if k != "SQ_WAVES"})
