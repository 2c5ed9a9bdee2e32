"""Host-side profile of bench.py's step (cProfile + wall split)."""
import cProfile
import pstats
import sys
import time

sys.path.insert(0, ".")
import numpy as np
import torch

import bench
from hyperopt_amd.engine import Engine

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
pr = cProfile.Profile()
pr.enable()
for k in range(5):
    eng.run(bench.make_works(space, sp, k, 1 << 22, 0))
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
