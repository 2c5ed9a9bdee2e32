"""Host-side profile of bench.py's step in history mode (diagnostic): wall time
of the host parts and a cProfile of the whole step at a tiny candidate count
(GPU time negligible, so what remains is launch + host work)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd.engine import DeviceHistory, Engine  # noqa: E402

torch.cuda.set_device(0)
space = bench.c3_space()
vals, losses = bench.c3_history(space)
mat = bench.c3_matrix(space, vals)
eng = Engine()
hist = DeviceHistory(eng, len(space), cap=bench.T_HIST)
hist.append(mat)


def prep(k, n):
    rb = bench.below_rows(losses)
    isb = np.zeros(bench.T_HIST, np.uint8)
    isb[rb] = 1
    return bench.history_works(space, mat, hist, rb, k, n, 0), isb


def step(k, n, timers=None):
    works, isb = prep(k, n)
    return eng.run(works, history=hist, is_below=isb, timers=timers)


for n in (1 << 22, 1 << 10):
    for k in range(3):
        step(k, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(10):
        step(k, n)
    t1 = time.perf_counter()
    print("step n=%d: %.3f ms" % (n, (t1 - t0) / 10e-3))
t0 = time.perf_counter()
for k in range(10):
    prep(k, 1 << 10)
print("prep (below rows + works): %.3f ms" % ((time.perf_counter() - t0) / 10e-3))
pr = cProfile.Profile()
pr.enable()
for k in range(10):
    step(k, 1 << 10)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)

# host phase split of Engine.run (Engine.host_marks), full candidate count
eng.host_marks = []
acc = {}
for k in range(20):
    eng.host_marks.clear()
    t0 = time.perf_counter()
    step(k, 1 << 22)
    m = eng.host_marks
    for (a, ta), (b, tb) in zip(m, m[1:]):
        acc[b] = acc.get(b, 0.0) + (tb - ta)
    acc["prep (bench)"] = acc.get("prep (bench)", 0.0) + (m[0][1] - t0)
for k, v in acc.items():
    print("  %-16s %.3f ms" % (k, v / 20e-3))
