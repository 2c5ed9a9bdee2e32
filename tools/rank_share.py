"""Strong-scaling projection on one GPU: time each rank's share of bench.py's
step (dist.plan_units(world=N)[r]) alone, no process group (diagnostic).

    python tools/rank_share.py 2 4 8
    python tools/rank_share.py --only 8 2     (one share, e.g. under rocprofv3)

For every N, every rank r: the median ms of its level (host plan + upload +
launches + readback, as bench.py's step without the collective) and the
kernel-group times.  The N-GPU step is projected as max_r(rank time) + the
all-gather of the winners (measured separately).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import dist as hdist  # noqa: E402
from hyperopt_amd.engine import DeviceHistory, Engine  # noqa: E402


def main(worlds, only=None):
    torch.cuda.set_device(0)
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    eng = Engine()
    mat = bench.c3_matrix(space, vals)
    hist = DeviceHistory(eng, len(space), cap=bench.T_HIST)
    hist.append(mat)
    rb = bench.below_rows(losses)
    isb = np.zeros(bench.T_HIST, np.uint8)
    isb[rb] = 1
    n = bench.N_CAND
    out = {}
    for N in ([only[0]] if only else [1] + worlds):
        plan = hdist.plan_units([k for _, k, _ in space], n, N)
        ranks = []
        for r, units in enumerate(plan):
            if only and r != only[1]:
                continue
            def step(k, timers=None):
                works = bench.history_batch(space, mat, hist, rb, k, n, 0, units, n)
                return eng.run(works, precision=32, history=hist, is_below=isb, timers=timers)
            for k in range(3):
                step(k)
            torch.cuda.synchronize()
            ts = []
            for k in range(15):
                t0 = time.perf_counter()
                step(10 + k)
                ts.append(time.perf_counter() - t0)
            marks, phases, names = [], [], []
            for k in range(5):  # host phases (Engine.host_marks)
                eng.host_marks = []
                step(50 + k)
                eng.host_marks.append(("returned", time.perf_counter()))
                m = dict(eng.host_marks)
                marks.append((m["score launches"] - m["start"], m["returned"] - m["score launches"]))
                hm = eng.host_marks
                phases.append([b[1] - a[1] for a, b in zip(hm[:-1], hm[1:])])
                names = [b[0] for b in hm[1:]]
            eng.host_marks = None
            host = np.median(np.array(marks), axis=0) * 1e3
            timers = {}
            for k in range(3):
                step(100 + k, timers)
            torch.cuda.synchronize()
            g = {a: round(float(np.mean([e0.elapsed_time(e1) for e0, e1 in v])), 4)
                 for a, v in timers.items()}
            ranks.append({"rank": r, "labels": len(units), "ms": round(float(np.median(ts)) * 1e3, 4),
                          "host_launch_ms": round(float(host[0]), 4),
                          "wait_ms": round(float(host[1]), 4),
                          "phases_us": dict(zip(names, np.round(np.median(np.array(phases), axis=0) * 1e6, 1).tolist())),
                          "group_ms": g, "gpu_ms": round(sum(g.values()), 4)})
        worst = max(x["ms"] for x in ranks)
        if only:
            print(json.dumps(ranks), flush=True)
            return
        out[N] = {"max_rank_ms": worst, "ranks": ranks}
        print(json.dumps({"N": N, "max_rank_ms": worst,
                          "per_rank_ms": [x["ms"] for x in ranks],
                          "host_launch_ms": [x["host_launch_ms"] for x in ranks],
                          "wait_ms": [x["wait_ms"] for x in ranks],
                          "per_rank_gpu_ms": [x["gpu_ms"] for x in ranks]}), flush=True)
        print(json.dumps({"N": N, "rank0_phases_us": ranks[0]["phases_us"]}), flush=True)
    base = out[1]["max_rank_ms"]
    for N in worlds:
        print(json.dumps({"N": N, "projected_speedup_no_collective": round(base / out[N]["max_rank_ms"], 2)}))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--only"]:  # one share (for a kernel trace): --only N r
        main([], (int(sys.argv[2]), int(sys.argv[3])))
    else:
        main([int(a) for a in sys.argv[1:]] or [2, 4, 8])
