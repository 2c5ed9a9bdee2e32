"""An explicit precision=32 suggest is exact at every size: below the table
path's TABLE_MIN_CAND the "auto" scorer scores the fp32 candidate stream in
fp64 (tpe_score_pruned64 with TPE_F_DRAW32), so its winner is np.argmax of
the exact scores of those candidates (tpe.py:649-658; GMM1_lpdf / LGMM1_lpdf
tpe.py:117-180, 265-307) -- checked here against the fp64 scores of the same
draws, re-read from the dense fp32 path's per-candidate values."""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

KINDS = [("uniform", (-5.0, 5.0), lambda r, n: r.uniform(-5, 5, n)),
         ("normal", (0.0, 2.0), lambda r, n: r.normal(0, 2, n)),
         ("loguniform", (-5.0, 0.0), lambda r, n: np.exp(r.uniform(-5, 0, n)))]


@pytest.fixture(scope="module")
def engine():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from hyperopt_amd.engine import Engine
    return Engine()


@pytest.mark.parametrize("kind,args,gen", KINDS)
@pytest.mark.parametrize("n_cand", [24, 5000, 60000])
@pytest.mark.parametrize("n_hist", [40, 3000])
def test_precision32_small_levels_are_exact(engine, kind, args, gen, n_cand, n_hist):
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(n_hist + n_cand)
    obs = gen(rng, n_hist)
    losses = rng.normal(size=n_hist)
    below, above = O.ap_split_trials(np.arange(n_hist), obs, np.arange(n_hist), losses, 0.25)
    w = LabelWork(kind, kind, args, below, above, n_cand=n_cand, key=1234567 + n_cand)
    r, = engine.run([w], precision=32)  # "auto": pruned64 on the fp32 stream
    assert r.n_scored == n_cand
    # the same fp32 draws (dense fp32 path, per-candidate values) scored in fp64
    d, = engine.run([w], precision=32, scorer="dense", outputs=True)
    w64 = LabelWork(kind, kind, args, below, above, cand=d.cand)
    e, = engine.run([w64], precision=64, outputs=True)
    s = e.below_llik - e.above_llik
    best = int(np.argmax(s))
    # every kind index-exact (LGMM1: scored at log of the returned value, as
    # the injected path and the reference score it)
    assert r.index == best
    assert r.value == d.cand[best]
