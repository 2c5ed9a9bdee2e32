"""C3 level with the sorted fit on / off (diagnostic): winners and the
prefix-first need flags (lattice, categorical) of both."""
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
mat = bench.c3_matrix(space, vals)
rb = bench.below_rows(losses)
isb = np.zeros(losses.size, np.uint8)
isb[rb] = 1
for sf in (True, False):
    eng = Engine()
    eng.sorted_fit = sf
    hist = DeviceHistory(eng, len(space), cap=bench.T_HIST)
    hist.append(mat)
    for step in range(2):
        works = bench.history_works(space, mat, hist, rb, step, bench.N_CAND, 0)
        res = eng.run(works, precision=32, history=hist, is_below=isb)
    ln = eng._bufs["lat_need"][:40].cpu().numpy().view(np.int32)
    cn = eng._bufs["cat_need"][:40].cpu().numpy().view(np.int32)
    print("sorted_fit", sf, "lat_need", ln.tolist(), "cat_need", cn.tolist())
    print("  winners", [(r.index, round(float(r.value), 6)) for r in res][:50:5])
