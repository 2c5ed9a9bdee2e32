"""Host profile of the drop-in suggest on C3 (bench.dropin_suggest_p50's loop)
under cProfile: where the ~0.5 ms beyond the engine's level goes."""
import cProfile
import io
import pstats
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402
from hyperopt_amd.base import JOB_STATE_DONE  # noqa: E402

space = bench.c3_space()
vals, losses = bench.c3_history(space)
domain, trials = bench.c3_trials(space, vals, losses)
rng = np.random.RandomState(9)


def call(k):
    tid = losses.size + k
    t0 = time.perf_counter()
    docs = tpe.suggest([tid], domain, trials, k, n_EI_candidates=bench.N_CAND, verbose=False)
    dt = time.perf_counter() - t0
    docs[0]["state"] = JOB_STATE_DONE
    docs[0]["result"] = {"status": "ok", "loss": float(rng.normal())}
    trials.insert_trial_docs(docs)
    trials.refresh()
    return dt


for k in range(5):
    call(k)
pr = cProfile.Profile()
ts = []
pr.enable()
for k in range(5, 25):
    ts.append(call(k))
pr.disable()
print("suggest p50 ms %.3f" % (1e3 * np.median(ts)))
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
print(s.getvalue())
eng = tpe.engine()
print("band overflows:", getattr(eng, "band_overflows", 0), getattr(eng, "last_band_overflow", None))
print("last table stats:", eng.last_table_stats)
plan = eng.last_plan
if plan is not None and getattr(eng, "last_band_overflow", None):
    jobs = plan[3]
    for p, fam, n in eng.last_band_overflow:
        print("job", p, jobs[p])
