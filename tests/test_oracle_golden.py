"""Pin the CPU oracle (oracle/tpe_oracle.py) against vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import tpe_oracle as O
from tests.golden_io import E2E_CASES, load

UNITS, UMETA = load("units")


def _same(a, b, rtol=0.0):
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    assert a.shape == b.shape, (a.shape, b.shape)
    if rtol == 0.0:
        np.testing.assert_array_equal(a, b)
    else:
        np.testing.assert_allclose(a, b, rtol=rtol, atol=0, equal_nan=True)


@pytest.mark.parametrize("i", range(len(UMETA["parzen"])))
def test_parzen(i):
    m = UMETA["parzen"][i]
    w, mu, sig = O.adaptive_parzen_normal(UNITS["parzen%d_obs" % i], m["prior_weight"],
                                          m["prior_mu"], m["prior_sigma"], m["lf"])
    _same(mu, UNITS["parzen%d_mu" % i])
    _same(sig, UNITS["parzen%d_sigma" % i])
    _same(w, UNITS["parzen%d_w" % i], rtol=1e-15)


@pytest.mark.parametrize("i", range(len(UMETA["split"])))
def test_split(i):
    g = lambda k: UNITS["split%d_%s" % (i, k)]
    b, a = O.ap_split_trials(g("oi"), g("ov"), g("li"), g("lv"), UMETA["split"][i]["gamma"])
    _same(b, g("below"))
    _same(a, g("above"))


@pytest.mark.parametrize("i", range(len(UMETA["lpdf"])))
def test_lpdf(i):
    m = UMETA["lpdf"][i]
    g = lambda k: UNITS["lpdf%d_%s" % (i, k)]
    f = O.gmm1_lpdf if m["family"] == "GMM1" else O.lgmm1_lpdf
    with np.errstate(all="ignore"):
        out = f(g("x"), g("w"), g("mu"), g("sigma"), low=m["low"], high=m["high"], q=m["q"])
    ref = g("out")
    np.testing.assert_array_equal(np.isfinite(out), np.isfinite(ref))
    _same(out, ref, rtol=1e-13)


@pytest.mark.parametrize("i", range(len(UMETA["best"])))
def test_broadcast_best(i):
    g = lambda k: UNITS["best%d_%s" % (i, k)]
    with np.errstate(invalid="ignore"):
        k = O.broadcast_best_index(g("b"), g("a"))
    assert np.all(g("out") == g("s")[k])


@pytest.mark.parametrize("i", range(len(UMETA["cat"])))
@pytest.mark.parametrize("pw", [1.0, 2.5])
def test_categorical_posterior(i, pw):
    m = UMETA["cat"][i]
    obs = UNITS["cat%d_obs" % i]
    if m["kind"] == "randint":
        args = m["args"]
        p = O.randint_posterior(obs, pw, args[0], args[1] if len(args) > 1 else None)
    else:
        p = O.categorical_posterior(obs, pw, m["args"][0])
    _same(p, UNITS["cat%d_pw%g_p" % (i, pw)])


def _label_pipeline(arrays, meta, lab):
    spec = meta["specs"][lab]
    oi = arrays["obs_idxs/" + lab]
    ov = arrays["obs_vals/" + lab]
    below, above = O.ap_split_trials(oi, ov, arrays["hist_tids"], arrays["hist_losses"],
                                     meta["gamma"])
    cand = arrays["cand/" + lab]
    kind = spec["kind"]
    if kind in O.CONTINUOUS:
        with np.errstate(all="ignore"):
            r = O.continuous_label_scores(kind, spec["args"], below, above, cand,
                                          meta["prior_weight"])
        post_b, post_a = r["below"], r["above"]
    else:
        r = O.categorical_label_scores(kind, spec["args"], below, above, cand,
                                       meta["prior_weight"])
        post_b, post_a = (r["p_below"],), (r["p_above"],)
    return r, post_b, post_a


@pytest.mark.parametrize("case", E2E_CASES)
def test_e2e_reference_posterior(case):
    arrays, meta = load("e2e_" + case)
    for lab, lm in meta["labels"].items():
        r, post_b, post_a = _label_pipeline(arrays, meta, lab)
        for j in range(lm["n_post"]):
            _same(post_b[j], arrays["bpost%d/%s" % (j, lab)], rtol=1e-14)
            _same(post_a[j], arrays["apost%d/%s" % (j, lab)], rtol=1e-14)
        if lm["n"] == 0:
            assert arrays["cand/" + lab].size == 0
            continue
        _same(r["below_llik"], arrays["bl/" + lab], rtol=1e-12)
        _same(r["above_llik"], arrays["al/" + lab], rtol=1e-12)
        assert r["best"] == lm["best"], (case, lab)
