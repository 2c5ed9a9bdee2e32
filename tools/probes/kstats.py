"""Compare rocprofv3 kernel_stats CSVs: python tools/probes/kstats.py a.csv [b.csv ...]"""
import csv
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        n = r["Name"].replace("tpe::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        out[n] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3)
    return out


tabs = [load(p) for p in sys.argv[1:]]
names = sorted(set().union(*tabs), key=lambda n: -max(t.get(n, (0, 0, 0))[2] for t in tabs))
print("%-28s" % "kernel" + "".join("%22s" % ("avg us (calls) #%d" % i) for i in range(len(tabs))))
for n in names[:30]:
    print("%-28s" % n[:28] + "".join(
        "%14.1f (%4d) " % (t[n][1], t[n][0]) if n in t else "%22s" % "-" for t in tabs))
