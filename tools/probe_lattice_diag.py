"""Lattice group timing on C3's 10 quniform labels (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd.engine import Engine  # noqa: E402

torch.cuda.set_device(0)
space = [s for s in bench.c3_space() if s[1] == "quniform"]
vals, losses = bench.c3_history(bench.c3_space())
sp = bench.split(vals, losses)
eng = Engine()
n = 1 << 22
eng.run(bench.make_works(space, sp, 0, n, 0))
timers = {}
for k in range(5):
    eng.run(bench.make_works(space, sp, k + 1, n, 0), timers=timers)
torch.cuda.synchronize()
print({k: round(float(np.mean([a.elapsed_time(b) for a, b in v])), 4) for k, v in timers.items()})
