"""Host-side profile of bench.py's step (wall split + cProfile of Engine.run)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd.engine import Engine  # noqa: E402

space = bench.c3_space()
vals, losses = bench.c3_history(space)
eng = Engine()
for k in range(3):
    eng.run(bench.make_works(space, bench.split(vals, losses), k, 1 << 22, 0))
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(5):
    sp = bench.split(vals, losses)
t1 = time.perf_counter()
for k in range(5):
    w = bench.make_works(space, sp, k, 1 << 22, 0)
t2 = time.perf_counter()
print("split %.3f ms  make_works %.3f ms" % ((t1 - t0) / 5e-3, (t2 - t1) / 5e-3))
# launch-side cost: run with tiny candidate counts (GPU time negligible)
for n in (1 << 22, 1 << 10):
    ws = [bench.make_works(space, sp, k, n, 0) for k in range(5)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for w in ws:
        eng.run(w)
    t1 = time.perf_counter()
    print("run n=%d: %.3f ms/step" % (n, (t1 - t0) / 5e-3))
pr = cProfile.Profile()
ws = [bench.make_works(space, sp, k, 1 << 10, 0) for k in range(5)]
pr.enable()
for w in ws:
    eng.run(w)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
