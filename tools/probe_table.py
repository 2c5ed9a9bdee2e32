"""Per-kind timing of the cell-table path on the C3 history (diagnostic)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import bench
from hyperopt_amd.engine import Engine

torch.cuda.set_device(0)
space = bench.c3_space()
vals, losses = bench.c3_history(space)
sp = bench.split(vals, losses)
eng = Engine()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
for kind in ("uniform", "loguniform", "normal"):
    sub = [s for s in space if s[1] == kind]
    for scorer in ("table", "dense") if n <= (1 << 20) else ("table",):
        works = bench.make_works(sub, sp, 0, n, 0)
        eng.run(works, scorer=scorer)
        timers = {}
        for k in range(3):
            eng.run(bench.make_works(sub, sp, k + 1, n, 0), timers=timers, scorer=scorer)
        torch.cuda.synchronize()
        g = {k: round(float(np.mean([a.elapsed_time(b) for a, b in v])), 4) for k, v in timers.items()}
        print(kind, scorer, n, g, eng.last_table_stats, flush=True)
