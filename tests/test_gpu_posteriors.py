"""Posterior parameters from the HIP fit (tpe_parzen_fit, tpe_cat_posterior)
vs vectors produced by the reference itself (tests/golden).

north_star: "posterior parameters ... must match the reference numpy
implementation within rtol 1e-6 (fp64) ... Categorical counts ... must be
bit-exact."  Here: means and bandwidths to the last bit (they are copies and
differences of the observations), weights within rtol 1e-12 (the device sums
the normaliser in a different order than numpy's pairwise sum), categorical
probabilities bit-exact (np.bincount order, numpy pairwise normaliser).
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O
from tests.golden_io import E2E_CASES, load

pytestmark = pytest.mark.gpu

UNITS, UMETA = load("units")


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


@pytest.mark.parametrize("i", range(len(UMETA["parzen"])))
def test_adaptive_parzen_normal_units(engine, i):
    """tpe.py:399-467 on the reference's own unit vectors (len 0/1/2, prior
    ties, LF on/off, tie-heavy quantized data)."""
    from hyperopt_amd.engine import LabelWork
    m = UMETA["parzen"][i]
    obs = UNITS["parzen%d_obs" % i]
    w = LabelWork("x", "normal", (m["prior_mu"], m["prior_sigma"]), obs, obs[:0])
    r, = engine.run([w], prior_weight=m["prior_weight"], lf=m["lf"], posteriors=True)
    pw, pmu, psig = r.extra["below"]
    np.testing.assert_array_equal(pmu, UNITS["parzen%d_mu" % i])
    np.testing.assert_array_equal(psig, UNITS["parzen%d_sigma" % i])
    np.testing.assert_allclose(pw, UNITS["parzen%d_w" % i], rtol=1e-12, atol=0)


def _split(arrays, meta, lab):
    return O.ap_split_trials(arrays["obs_idxs/" + lab], arrays["obs_vals/" + lab],
                             arrays["hist_tids"], arrays["hist_losses"], meta["gamma"])


@pytest.mark.parametrize("case", E2E_CASES)
def test_e2e_posteriors(engine, case):
    """The reference's posterior graph (build_posterior, tpe.py:661-757) on its
    own histories: below/above mixtures of every label, every hp kind."""
    from hyperopt_amd.engine import LabelWork
    arrays, meta = load("e2e_" + case)
    labs = [lab for lab in sorted(meta["labels"]) if meta["labels"][lab]["n"] > 0]
    works = []
    for lab in labs:
        spec = meta["specs"][lab]
        below, above = _split(arrays, meta, lab)
        works.append(LabelWork(lab, spec["kind"], tuple(spec["args"]), below, above))
    res = engine.run(works, prior_weight=meta["prior_weight"], posteriors=True)
    for lab, w, r in zip(labs, works, res):
        if w.kind in ("randint", "categorical"):
            np.testing.assert_array_equal(r.extra["p_below"], arrays["bpost0/" + lab],
                                          err_msg=lab)
            np.testing.assert_array_equal(r.extra["p_above"], arrays["apost0/" + lab],
                                          err_msg=lab)
            continue
        for half, key in (("below", "bpost"), ("above", "apost")):
            got = r.extra[half]
            for j, name in enumerate(("w", "mu", "sigma")):
                np.testing.assert_allclose(got[j], arrays["%s%d/%s" % (key, j, lab)],
                                           rtol=1e-12, atol=0,
                                           err_msg="%s %s %s %s" % (case, lab, half, name))


@pytest.mark.parametrize("n", [2, 2047, 2048, 2049, 6000, 20000])
def test_fit_matches_oracle_across_sort_tiles(engine, n):
    """Histories spanning several 2048-observation sort tiles, with heavy ties
    (quantized values) so the cross-tile stable order is exercised."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(n)
    obs = np.round(rng.normal(0, 2, n) * 4) / 4
    w = LabelWork("x", "normal", (0.0, 2.0), obs[:25], obs)
    r, = engine.run([w], posteriors=True)
    for half, o in (("below", obs[:25]), ("above", obs)):
        ow, omu, osig = O.adaptive_parzen_normal(o, 1.0, 0.0, 2.0)
        gw, gmu, gsig = r.extra[half]
        np.testing.assert_array_equal(gmu, omu)
        np.testing.assert_array_equal(gsig, osig)
        np.testing.assert_allclose(gw, ow, rtol=1e-12, atol=0)


def test_p_accept_bounded(engine):
    """p_accept = sum w (Phi(high) - Phi(low)) (tpe.py:145-150)."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(1)
    obs = rng.uniform(-5, 5, 300)
    w = LabelWork("x", "uniform", (-5.0, 5.0), obs[:20], obs)
    r, = engine.run([w], posteriors=True)
    for half, k in (("below", 0), ("above", 1)):
        ww, mm, ss = r.extra[half]
        ref = np.sum(ww * (O.normal_cdf(5.0, mm, ss) - O.normal_cdf(-5.0, mm, ss)))
        np.testing.assert_allclose(r.extra["p_accept"][k], ref, rtol=1e-12)


@pytest.mark.parametrize("n,k", [(3000, 3), (60000, 3), (150000, 7), (40000, 40)])
def test_categorical_counts_long_histories(engine, n, k):
    """Categorical / randint pseudocounts over long LF-ramped histories (the
    wave-parallel exact fold, tpe_fit.hip seq_fold, crossing many binades):
    bit-exact against np.bincount's sequential sums."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(n + k)
    p = rng.dirichlet(np.full(k, 0.5))
    below = rng.choice(k, size=25, p=p).astype(np.int64)
    above = rng.choice(k, size=n, p=p).astype(np.int64)
    works = [LabelWork("c", "categorical", (tuple(p.tolist()),), below, above),
             LabelWork("r", "randint", (3, 3 + k), below + 3, above + 3)]
    rc, rr = engine.run(works, prior_weight=1.0, posteriors=True)
    np.testing.assert_array_equal(rc.extra["p_above"], O.categorical_posterior(above, 1.0, p))
    np.testing.assert_array_equal(rc.extra["p_below"], O.categorical_posterior(below, 1.0, p))
    np.testing.assert_array_equal(rr.extra["p_above"], O.randint_posterior(above + 3, 1.0, 3,
                                                                           3 + k))
