"""Host-side cost of the drop-in tpe.suggest on C3 (diagnostic), measured
without a GPU: tools/host_cpu_profile.py's stand-in engine (device calls
return at once) behind hyperopt_amd.tpe.engine(), the 10k-document Trials of
bench.dropin_suggest_p50, one document appended per call.

    python tools/dropin_cpu_profile.py [--cprofile]
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402
from hyperopt_amd.base import JOB_STATE_DONE  # noqa: E402
from tools.host_cpu_profile import make_engine  # noqa: E402


def main(prof=False):
    eng = make_engine()
    tpe.engine = lambda slot=0: eng
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
    ts = []
    for k in range(100):
        ts.append(call(10 + k))
    print("tpe.suggest host (refresh excluded): p50 %.1f us  p90 %.1f us" % (np.median(ts) * 1e6,
                                                     np.percentile(ts, 90) * 1e6))
    if prof:
        pr = cProfile.Profile()
        pr.enable()
        for k in range(100):
            call(1000 + k)
        pr.disable()
        pstats.Stats(pr).sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main("--cprofile" in sys.argv)
