"""Table-kernel time on C3's 30 continuous labels: history mode vs upload mode
(diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd.engine import DeviceHistory, Engine  # noqa: E402

torch.cuda.set_device(0)
space = bench.c3_space()
vals, losses = bench.c3_history(space)
sp = bench.split(vals, losses)
eng = Engine()
n = 1 << 22
mat = bench.c3_matrix(space, vals)
hist = DeviceHistory(eng, len(space), cap=bench.T_HIST)
hist.append(mat)
rb = bench.below_rows(losses)
isb = np.zeros(bench.T_HIST, np.uint8)
isb[rb] = 1
sel = [j for j, s in enumerate(space) if s[1] in ("uniform", "loguniform", "normal")]


def run(mode, k, timers=None, subset=None):
    if mode == "hist":
        works = bench.history_works(space, mat, hist, rb, k, n, 0)
    else:
        works = bench.make_works(space, sp, k, n, 0)
    if subset is not None:
        works = [works[j] for j in subset]
    return eng.run(works, timers=timers, history=hist if mode == "hist" else None,
                   is_below=isb if mode == "hist" else None)


for mode in ("hist", "upload", "hist", "upload"):
    for subset in (None, sel):
        run(mode, 0, subset=subset)
        timers = {}
        for k in range(3):
            run(mode, k + 1, timers, subset)
        torch.cuda.synchronize()
        g = {k: round(float(np.mean([a.elapsed_time(b) for a, b in v])), 4)
             for k, v in timers.items()}
        print(mode, "all50" if subset is None else "cont30", g, flush=True)
