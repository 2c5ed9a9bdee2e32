"""Per-kind timing of the C3 labels through one scorer (diagnostic).

    python tools/probes/probe_table.py [n_cand] [kinds,comma,separated] [scorer]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd.engine import Engine  # noqa: E402

torch.cuda.set_device(0)
space = bench.c3_space()
vals, losses = bench.c3_history(space)
sp = bench.split(vals, losses)
eng = Engine()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
kinds = sys.argv[2].split(",") if len(sys.argv) > 2 else ["uniform", "loguniform", "normal"]
scorers = sys.argv[3].split(",") if len(sys.argv) > 3 else ["table"]
groups = [[s for s in space if s[1] == kind] for kind in kinds]
if len(kinds) > 1:  # and all of them in one launch (the bench's shape)
    groups.append([s for s in space if s[1] in kinds])
for sub in groups:
    kind = "+".join(sorted({s[1] for s in sub}))
    for scorer in scorers:
        eng.run(bench.make_works(sub, sp, 0, n, 0), scorer=scorer)
        timers = {}
        for k in range(3):
            eng.run(bench.make_works(sub, sp, k + 1, n, 0), timers=timers, scorer=scorer)
        torch.cuda.synchronize()
        g = {k: round(float(np.mean([a.elapsed_time(b) for a, b in v])), 4)
             for k, v in timers.items()}
        print(kind, scorer, n, g, eng.last_table_stats, flush=True)

# cell-grid geometry of the last run (tpe_table records)
from hyperopt_amd import _lib as L  # noqa: E402
nt = len(groups[-1])
raw = eng._bufs["tables"][:L.TABLE_DTYPE.itemsize * nt].cpu().numpy().view(L.TABLE_DTYPE)
for t in raw[:nt]:
    print("  nb %6d  h %.3g  span %.3g  wide b/a %d/%d" % (t["nb"], t["h"], t["hi"] - t["lo"],
                                                        t["n_wide_below"], t["n_wide_above"]))
