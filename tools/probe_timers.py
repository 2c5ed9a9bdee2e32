"""Step time of bench.py's C3 step with no HIP-event timers, every group
timed, and only the table group timed (diagnostic; GPU box)."""
import os
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
rb = bench.below_rows(losses)
isb = np.zeros(bench.T_HIST, np.uint8)
isb[rb] = 1


def step(k, timers=None, groups=None):
    works = bench.history_works(space, mat, hist, rb, k, bench.N_CAND, 0)
    return eng.run(works, history=hist, is_below=isb, timers=timers, timer_groups=groups,
                   scorer="auto", precision=32)


for rep in range(2):
    for mode in sys.argv[1:] or ("none", "all", "table", "fit"):
        for k in range(3):
            step(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ts = []
        for k in range(20):
            t1 = time.perf_counter()
            if mode == "none":
                step(k)
            else:
                step(k, {}, None if mode == "all" else {mode})
            ts.append(time.perf_counter() - t1)
        torch.cuda.synchronize()
        print("%-6s mean %.3f ms  p50 %.3f ms" % (mode, (time.perf_counter() - t0) / 20e-3,
                                                np.median(ts) * 1e3), flush=True)
