"""Cell-table mismatch finder (diagnostic): runs one golden case through the
table scorer and prints the worst candidates with their cells.

    python tools/probes/debug_table.py [case] [label]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from hyperopt_amd.engine import Engine  # noqa: E402
from tests.test_gpu_parity import _works_from_fixture  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "readme_wide"
label = sys.argv[2] if len(sys.argv) > 2 else None
eng = Engine()
works, golden, meta = _works_from_fixture(case)
res = eng.run(works, prior_weight=meta["prior_weight"], precision=32, outputs=True,
              scorer="table")
print("stats", eng.last_table_stats)
for w, r, (bl, al, best) in zip(works, res, golden):
    if label and w.label != label:
        continue
    if r.below_llik is None:
        continue
    db = np.abs(r.below_llik - bl)
    da = np.abs(r.above_llik - al)
    print(w.label, w.kind, w.args, "n_below", np.size(w.obs_below), "n_above", np.size(w.obs_above),
          "max db %.3g da %.3g" % (np.nanmax(db), np.nanmax(da)))
    bad = np.argsort(-np.nan_to_num(db + da))[:12]
    for i in bad:
        print("   cand %4d x=%.9g  got %.6f/%.6f  want %.6f/%.6f" % (
            i, w.cand[i], r.below_llik[i], r.above_llik[i], bl[i], al[i]))
    print("   below obs", np.sort(np.asarray(w.obs_below))[:30])
