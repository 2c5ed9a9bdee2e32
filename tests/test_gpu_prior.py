"""Startup phase on the GPU: prior draws (tpe_prior_sample via
rand.suggest_device) against the reference's prior samplers,
hyperopt/pyll/stochastic.py:36-158 -- KS for the continuous kinds, chi^2 for
the quantized and categorical ones, the reference's own distribution test
(hyperopt/tests/test_vectorize.py:204-275, same space and thresholds) through
fmin, and the conditional structure of a nested choice."""
import numpy as np
import pytest
from scipy import stats

pytestmark = pytest.mark.gpu

N = 200_000


def _domain(space):
    from hyperopt_amd.base import Domain
    return Domain(lambda p: 0.0, space)


def _chi2(a, b):
    lo, hi = min(a.min(), b.min()), max(a.max(), b.max())
    ca = np.bincount(a - lo, minlength=hi - lo + 1)
    cb = np.bincount(b - lo, minlength=hi - lo + 1)
    keep = (ca + cb) >= 20
    table = np.vstack([np.append(ca[keep], ca[~keep].sum()), np.append(cb[keep], cb[~keep].sum())])
    table = table[:, table.sum(0) > 0]
    return stats.chi2_contingency(table)[1]


def test_prior_draws_match_reference_distributions():
    from hyperopt_amd import hp
    from hyperopt_amd.rand import draw_priors
    space = {
        "u": hp.uniform("u", -3, 4), "lu": hp.loguniform("lu", -2, 1),
        "n": hp.normal("n", 1, 2), "ln": hp.lognormal("ln", 0.5, 0.7),
        "qu": hp.quniform("qu", 0, 10, 3), "qlu": hp.qloguniform("qlu", 0, 3, 2),
        "qn": hp.qnormal("qn", 0, 10, 2), "qln": hp.qlognormal("qln", 0, 1, 0.5),
        "ri": hp.randint("ri", 10), "ri2": hp.randint("ri2", 12, 25),
        "pc": hp.pchoice("pc", [(0.1, "a"), (0.3, "b"), (0.6, "c")]),
    }
    dom = _domain(space)
    labels, vals = draw_priors(dom, 123, N)
    v = dict(zip(labels, vals))
    rng = np.random.RandomState(0)  # reference-style numpy draws (stochastic.py:36-158)
    ks = {"u": (v["u"], stats.uniform(-3, 7).cdf),
          "lu": (np.log(v["lu"]), stats.uniform(-2, 3).cdf),
          "n": (v["n"], stats.norm(1, 2).cdf),
          "ln": (np.log(v["ln"]), stats.norm(0.5, 0.7).cdf)}
    for lab, (x, cdf) in ks.items():
        assert stats.kstest(x, cdf).pvalue > 1e-4, lab
    assert v["u"].min() >= -3 and v["u"].max() < 4
    ref = {"qu": np.round(rng.uniform(0, 10, N) / 3) * 3,
           "qlu": np.round(np.exp(rng.uniform(0, 3, N)) / 2) * 2,
           "qn": np.round(rng.normal(0, 10, N) / 2) * 2,
           "qln": np.round(np.exp(rng.normal(0, 1, N)) / 0.5) * 0.5,
           "ri": rng.randint(10, size=N).astype(float),
           "ri2": rng.randint(12, 25, size=N).astype(float),
           "pc": np.argmax(rng.multinomial(1, [0.1, 0.3, 0.6], size=N), axis=1).astype(float)}
    qs = {"qu": 3, "qlu": 2, "qn": 2, "qln": 0.5, "ri": 1, "ri2": 1, "pc": 1}
    for lab, r in ref.items():
        x = v[lab]
        k = np.round(x / qs[lab]).astype(np.int64)
        assert np.all(k * qs[lab] == x), lab
        p = _chi2(k, np.round(r / qs[lab]).astype(np.int64))
        assert p > 1e-4, (lab, p)
    assert set(np.unique(v["ri2"])) == set(range(12, 25))
    # draws are a function of (seed, label, position): same seed, same values
    labels2, vals2 = draw_priors(dom, 123, 1000)
    np.testing.assert_array_equal(vals2, vals[:, :1000])


def test_reference_distributions_test_through_fmin():
    """hyperopt/tests/test_vectorize.py:204-275 (test_distributions): its
    space and its histogram thresholds, with the draws made on the GPU."""
    from hyperopt_amd import Trials, fmin, hp, rand
    space = {"loss": (hp.loguniform("lu", -2, 2) + hp.qloguniform("qlu", np.log(1 + 0.01),
                                                                    np.log(20), 2)
                      + hp.quniform("qu", -4.999, 5, 1) + hp.uniform("u", 0, 10)),
             "status": "ok"}
    trials = Trials()
    N1 = 1000
    fmin(lambda x: x, space=space, algo=rand.suggest_device, trials=trials, max_evals=N1,
         rstate=np.random.RandomState(124), show_progressbar=False)
    assert len(trials) == N1
    vals = {lab: np.array([t["misc"]["vals"][lab][0] for t in trials.trials])
            for lab in ("lu", "qlu", "qu", "u")}
    COUNTMAX, COUNTMIN = 130, 70
    log_lu = np.log(vals["lu"])
    assert -2 < np.min(log_lu) and np.max(log_lu) < 2
    h = np.histogram(log_lu)[0]
    assert np.all(COUNTMIN < h) and np.all(h < COUNTMAX), h
    qlu = vals["qlu"]
    assert np.all(np.fmod(qlu, 2) == 0)
    assert np.min(qlu) == 2 and np.max(qlu) == 20
    bc_qlu = np.bincount(qlu.astype(int))
    assert bc_qlu[2] > bc_qlu[4] > bc_qlu[6] > bc_qlu[8]
    qu = vals["qu"]
    assert np.min(qu) == -5 and np.max(qu) == 5 and np.all(np.fmod(qu, 1) == 0)
    bc_qu = np.bincount(qu.astype(int) + 5)
    assert np.all(40 < bc_qu) and np.all(bc_qu < 125) and np.all(bc_qu < COUNTMAX), bc_qu
    u = vals["u"]
    assert np.min(u) > 0 and np.max(u) < 10
    h = np.histogram(u)[0]
    assert np.all(COUNTMIN < h) and np.all(h < COUNTMAX), h


def test_nested_choice_structure():
    """Each new trial keeps exactly the labels its own choices make live, and
    the root choice is uniform (chi^2)."""
    from hyperopt_amd import Trials, hp, rand
    from tests.golden import spaces
    dom = _domain(spaces.nested(hp))
    n = 30_000
    docs = rand.suggest_device(list(range(n)), dom, Trials(), 5)
    roots = np.array([d["misc"]["vals"]["root"][0] for d in docs])
    counts = np.bincount(roots, minlength=3)
    assert stats.chisquare(counts).pvalue > 1e-4, counts
    branch = {0: {"lin_lr"}, 1: {"tree_depth", "tree_split"}, 2: {"nn_units", "nn_drop"}}
    for d in docs[:3000]:
        live = {lab for lab, v in d["misc"]["vals"].items() if v}
        r = d["misc"]["vals"]["root"][0]
        want = {"root"} | branch[r]
        if r == 1:
            want |= {"gini_w"} if d["misc"]["vals"]["tree_split"][0] == 0 else {"ent_w", "ent_s"}
        assert live == want, (live, want)
        assert all(d["misc"]["idxs"][lab] == ([d["tid"]] if lab in live else [])
                   for lab in d["misc"]["idxs"])


def test_tpe_startup_uses_device_draws():
    from hyperopt_amd import Trials, hp, rand, tpe
    dom = _domain({"x": hp.uniform("x", 0, 1), "c": hp.choice("c", [0, 1, 2])})
    t = Trials()
    a = tpe.suggest([0, 1, 2], dom, t, 9)
    b = rand.suggest_device([0, 1, 2], dom, t, 9)
    assert [d["misc"]["vals"] for d in a] == [d["misc"]["vals"] for d in b]
