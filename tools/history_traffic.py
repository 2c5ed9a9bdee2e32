"""Per-kernel memory-side traffic and achieved GB/s of a profiled config
(tools/history_profile.sh output: <prefix>_kernel_stats.csv and
<prefix>_counters.json).

    python tools/history_traffic.py gpurun_out/hist_<tag>

FETCH_SIZE / WRITE_SIZE are per-dispatch means in KiB (rocprofv3).  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE counts half the bytes of wide
coalesced streaming reads on gfx950 and counts Infinity-Cache hits too; both
the raw and the doubled figure are printed (other access widths are
uncalibrated).  GB/s = bytes per dispatch / the kernel's mean duration in the
kernel-trace pass; the HBM peak is 8 TB/s (about 6.3 achievable).
"""
import csv
import json
import sys

PEAK = 8000.0  # GB/s


def main(prefix):
    stats = {r["kernel"]: r for r in csv.DictReader(open(prefix + "_kernel_stats.csv"))}
    ctr = json.load(open(prefix + "_counters.json"))
    rows = []
    for k, r in stats.items():
        c = ctr.get(k, {})
        if "FETCH_SIZE" not in c and "WRITE_SIZE" not in c:
            continue
        us = float(r["avg_us"])
        f = float(c.get("FETCH_SIZE", 0.0)) * 1024.0
        w = float(c.get("WRITE_SIZE", 0.0)) * 1024.0
        rows.append((float(r["total_us"]), k, int(r["calls"]), us, f, w))
    rows.sort(reverse=True)
    print("%-26s %6s %10s %12s %12s %9s %9s %7s" % (
        "kernel", "calls", "avg_us", "fetch_B", "write_B", "GB/s", "GB/s(2F)", "frac2F"))
    for tot, k, n, us, f, w in rows[:24]:
        gbs = (f + w) / (us * 1e3) if us > 0 else 0.0
        gbs2 = (2 * f + w) / (us * 1e3) if us > 0 else 0.0
        print("%-26s %6d %10.1f %12.0f %12.0f %9.1f %9.1f %7.4f" % (
            k, n, us, f, w, gbs, gbs2, gbs2 / PEAK))


if __name__ == "__main__":
    main(sys.argv[1])
