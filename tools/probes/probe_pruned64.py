"""fp64 scoring time, dense vs pruned, on C4-shaped labels (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hyperopt_amd.engine import Engine, LabelWork  # noqa: E402
from oracle import tpe_oracle as O  # noqa: E402

torch.cuda.set_device(0)
eng = Engine()
T = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
rng = np.random.RandomState(0)
for kind, args, gen in [("uniform", (-5.0, 5.0), lambda k: rng.uniform(-5, 5, k)),
                        ("normal", (0.0, 2.0), lambda k: rng.normal(0, 2, k)),
                        ("loguniform", (-5.0, 0.0), lambda k: np.exp(rng.uniform(-5, 0, k)))]:
    obs = gen(T)
    losses = rng.normal(size=T)
    below, above = O.ap_split_trials(np.arange(T), obs, np.arange(T), losses, 0.25)
    works = [LabelWork("%s%d" % (kind, j), kind, args, below, above, n_cand=n, key=j)
             for j in range(16)]
    for mode in ("dense", "pruned"):
        eng.exact64 = mode
        eng.run(works, precision=64)
        timers = {}
        for k in range(3):
            eng.run(works, precision=64, timers=timers)
        torch.cuda.synchronize()
        g = {k: round(float(np.mean([a.elapsed_time(b) for a, b in v])), 3)
             for k, v in timers.items()}
        print(kind, mode, T, n, g, flush=True)
