"""Max |log-density error| of the cell-table scorer vs the fp64 oracle
(diagnostic behind DESIGN.md §3.1's accuracy figure)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from hyperopt_amd.engine import Engine, LabelWork  # noqa: E402
from oracle import tpe_oracle as O  # noqa: E402

eng = Engine()
KINDS = [("uniform", (-5.0, 5.0), lambda r, n: r.uniform(-5, 5, n)),
         ("loguniform", (-5.0, 0.0), lambda r, n: np.exp(r.uniform(-5, 0, n))),
         ("normal", (0.0, 2.0), lambda r, n: r.normal(0, 2, n)),
         ("lognormal", (0.0, 1.0), lambda r, n: np.exp(r.normal(0, 1, n)))]
worst = 0.0
for kind, args, gen in KINDS:
    for T in (30, 300, 3000, 10000):
        rng = np.random.RandomState(T)
        obs = gen(rng, T)
        below, above = O.ap_split_trials(np.arange(T), obs, np.arange(T), rng.normal(size=T), 0.25)
        w = LabelWork(kind, kind, args, below, above, n_cand=1 << 16, key=31 + T)
        r, = eng.run([w], precision=32, outputs=True, scorer="table")
        pick = np.random.RandomState(1).choice(r.cand.size, 4000, replace=False)
        with np.errstate(all="ignore"):
            ref = O.continuous_label_scores(kind, args, below, above, r.cand[pick])
        eb = np.max(np.abs(r.below_llik[pick] - ref["below_llik"]))
        ea = np.max(np.abs(r.above_llik[pick] - ref["above_llik"]))
        es = np.max(np.abs((r.below_llik - r.above_llik)[pick]
                           - (ref["below_llik"] - ref["above_llik"])))
        worst = max(worst, eb, ea)
        print("%-10s T=%5d  max|d below| %.2e  max|d above| %.2e  max|d score| %.2e  %s"
              % (kind, T, eb, ea, es, eng.last_table_stats), flush=True)
print("worst %.2e" % worst)
