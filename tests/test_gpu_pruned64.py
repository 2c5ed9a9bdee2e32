"""The pruned exact fp64 scorer (tpe_score_pruned64) against the dense fp64
kernel (tpe_score_continuous, every component) and the oracle: it may leave
out only components below e^-40 of the mixture sum, so the log-densities
agree to ~1e-15 relative and the argmax is the same candidate.  GMM1_lpdf /
LGMM1_lpdf, tpe.py:117-180, 265-307; argmax tpe.py:650-658."""
import numpy as np
import pytest

from oracle import tpe_oracle as O
from tests.test_gpu_parity import _mixture_case

pytestmark = pytest.mark.gpu

CONT = [("uniform", (-5.0, 5.0)), ("loguniform", (-5.0, 0.0)), ("normal", (0.0, 2.0)),
        ("lognormal", (0.0, 1.0))]


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    e = Engine()
    yield e
    e.exact64 = "auto"


def _both(engine, w):
    engine.exact64 = "pruned"
    timers = {}
    p, = engine.run([w], precision=64, outputs=True, timers=timers)
    assert "pruned64" in timers
    engine.exact64 = "dense"
    d, = engine.run([w], precision=64, outputs=True)
    engine.exact64 = "auto"
    return p, d


@pytest.mark.parametrize("kind,args", CONT)
@pytest.mark.parametrize("n_above", [0, 3, 300, 2000, 20000])
def test_pruned_equals_dense_injected(engine, kind, args, n_above):
    rng = np.random.RandomState(n_above + 5)
    w = _mixture_case(rng, kind, args, min(n_above, 25), n_above, 2048)
    # a few candidates far off the sampler's range take the full sum
    w.cand = np.concatenate([w.cand, w.cand[:4] * 40.0 + 3.0])
    p, d = _both(engine, w)
    np.testing.assert_allclose(p.below_llik, d.below_llik, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(p.above_llik, d.above_llik, rtol=1e-13, atol=1e-13)
    assert (p.index, p.value) == (d.index, d.value)
    with np.errstate(all="ignore"):
        ref = O.continuous_label_scores(kind, args, w.obs_below, w.obs_above, w.cand)
    np.testing.assert_allclose(p.below_llik, ref["below_llik"], rtol=1e-6, equal_nan=True)
    np.testing.assert_allclose(p.above_llik, ref["above_llik"], rtol=1e-6, equal_nan=True)


@pytest.mark.parametrize("kind,args", CONT)
def test_pruned_equals_dense_sampled(engine, kind, args):
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(len(kind))
    gen = _mixture_case(rng, kind, args, 1, 5000, 1)
    losses = rng.normal(size=5000)
    below, above = O.ap_split_trials(np.arange(5000), gen.obs_above, np.arange(5000), losses,
                                     0.25)
    w = LabelWork(kind, kind, args, below, above, n_cand=1 << 14, key=77)
    p, d = _both(engine, w)
    np.testing.assert_array_equal(p.cand, d.cand)  # same fp64 draws
    np.testing.assert_allclose(p.below_llik, d.below_llik, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(p.above_llik, d.above_llik, rtol=1e-13, atol=1e-13)
    assert (p.index, p.value, p.n_scored) == (d.index, d.value, d.n_scored)


def test_plan_cache_follows_scorer_choice():
    """A plan recorded while a label's above mixture was small (dense exact
    scorer) is not reused once it reaches PRUNED64_MIN_COMP: the cached run
    equals an uncached run (history mode caches plans, upload mode does not)."""
    from hyperopt_amd.engine import PRUNED64_MIN_COMP, DeviceHistory, Engine
    from tests import test_gpu_history as H
    eng = Engine()
    for T in (40, 3000):
        assert (T - 2 >= PRUNED64_MIN_COMP) == (T == 3000)
        mat, active, losses = H._history(T, T, 0.0)
        rows = np.arange(T)
        up, _ = H._works(mat, active, losses, rows)
        hist = DeviceHistory(eng, len(H.SPACE), cap=64)
        hist.append(mat, active)
        hw, isb = H._works(mat, active, losses, rows, hist=hist)
        r_up = eng.run(up, precision=64)
        r_h = eng.run(hw, precision=64, history=hist, is_below=isb)
        for a, b in zip(r_up, r_h):
            assert (a.index, a.value, a.score) == (b.index, b.value, b.score), (T, a, b)
