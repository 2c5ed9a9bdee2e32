"""cProfile of the drop-in tpe.suggest on config C3 (diagnostic): where the
host time of a suggest call goes beyond the engine's kernels."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402
from hyperopt_amd.base import JOB_STATE_DONE  # noqa: E402

torch.cuda.set_device(0)
space = bench.c3_space()
vals, losses = bench.c3_history(space)
domain, trials = bench.c3_trials(space, vals, losses)
rng = np.random.RandomState(9)


def call(k, n_cand):
    tid = losses.size + k
    docs = tpe.suggest([tid], domain, trials, k, n_EI_candidates=n_cand, verbose=False)
    docs[0]["state"] = JOB_STATE_DONE
    docs[0]["result"] = {"status": "ok", "loss": float(rng.normal())}
    trials.insert_trial_docs(docs)
    trials.refresh()


for k in range(3):
    call(k, 1 << 10)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(3, 13):
    call(k, 1 << 10)
print("suggest+insert+refresh at 2^10 candidates: %.3f ms" % ((time.perf_counter() - t0) / 10e-3))
pr = cProfile.Profile()
pr.enable()
for k in range(13, 23):
    call(k, 1 << 10)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
pstats.Stats(pr).sort_stats("cumtime").print_stats(25)
