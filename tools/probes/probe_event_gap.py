"""GPU idle time around stream-ordering operations (diagnostic for the gaps
the level timeline shows after event records / waits).

    rocprofv3 --kernel-trace -d gpurun_out/evgap -o run -- python tools/probes/probe_event_gap.py
    python tools/probes/probe_event_gap.py --report gpurun_out/evgap

Each variant runs 20 times between host syncs and 2 ms sleeps; the report
prints, per variant, the median idle gap on the main stream between the
kernel before the operation and the one after it.
"""
import ctypes
import glob
import os
import sqlite3
import sys
import time

VARIANTS = ["plain", "record", "record_nofence", "record_wait_other", "wait_satisfied",
            "write_value", "write_wait_value"]


def run():
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    P = ctypes.c_void_p
    x = torch.ones(1 << 24, device="cuda")
    y = torch.ones(1 << 24, device="cuda")
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    h1, h2 = P(s1.cuda_stream), P(s2.cuda_stream)

    def ev(flags):
        e = P()
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(flags)) == 0
        return e
    e_nt, e_nf = ev(0x2), ev(0x2 | 0x20000000)
    sig = P()  # signal memory (8 bytes) for the stream value operations
    if hip.hipExtMallocWithFlags(ctypes.byref(sig), ctypes.c_size_t(8), ctypes.c_uint(2)) != 0:
        print("no signal memory: value variants skipped", flush=True)
        sig = None
    else:
        assert hip.hipMemset(sig, 0, 8) == 0
    hip.hipStreamWriteValue32.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint]
    hip.hipStreamWaitValue32.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
    cnt = [0]

    def k(s):
        with torch.cuda.stream(s):
            x.mul_(1.0000001)

    def k2(s):
        with torch.cuda.stream(s):
            y.mul_(1.0000001)

    for v in VARIANTS:
        if sig is None and "value" in v:
            v = "plain"
        for _ in range(20):
            torch.cuda.synchronize()
            time.sleep(0.002)
            k(s1)
            if v == "record":
                hip.hipEventRecord(e_nt, h1)
            elif v == "record_nofence":
                hip.hipEventRecord(e_nf, h1)
            elif v == "record_wait_other":
                hip.hipEventRecord(e_nt, h1)
                hip.hipStreamWaitEvent(h2, e_nt, 0)
                k2(s2)
            elif v == "wait_satisfied":
                k2(s2)
                hip.hipEventRecord(e_nt, h2)
                torch.cuda.synchronize()
                k(s1)
                hip.hipStreamWaitEvent(h1, e_nt, 0)
            elif v == "write_value":
                cnt[0] += 1
                hip.hipStreamWriteValue32(h1, sig, cnt[0], 0)
            elif v == "write_wait_value":
                cnt[0] += 1
                hip.hipStreamWaitValue32(h2, sig, cnt[0], 0, 0xFFFFFFFF)  # Gte
                k2(s2)
                hip.hipStreamWriteValue32(h1, sig, cnt[0], 0)
            k(s1)
        torch.cuda.synchronize()
        time.sleep(0.02)
    print("done", flush=True)


def report(src):
    db = sorted(glob.glob(os.path.join(src, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    q = "queue_id" if "queue_id" in cols else "stream_id"
    rows = list(c.execute("select name, start, end, %s from kernels order by start" % q))
    rows = [r for r in rows if "mul" in r[0] or "Mul" in r[0] or "elementwise" in r[0]]
    # bursts separated by >= 1 ms; 20 bursts per variant after any warm-up
    bursts, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[1] - cur[-1][2] > 1e6:
            bursts.append(cur)
            cur = []
        cur.append(r)
    bursts.append(cur)
    bursts = bursts[-20 * len(VARIANTS):]
    for i, v in enumerate(VARIANTS):
        gaps = []
        for b in bursts[20 * i:20 * (i + 1)]:
            main = [r for r in b if r[3] == b[-1][3]]  # the stream of the last kernel
            if len(main) >= 2:
                gaps.append((main[-1][1] - main[-2][2]) / 1e3)
        gaps.sort()
        print("%-20s median gap %6.1f us  (min %.1f, max %.1f, n %d)" % (
            v, gaps[len(gaps) // 2] if gaps else -1, gaps[0] if gaps else -1,
            gaps[-1] if gaps else -1, len(gaps)))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--report"]:
        report(sys.argv[2])
    else:
        run()
