"""tpe.suggest / fmin through the HIP engine (GPU).  Mirrors the reference's
tests/test_tpe.py TestSuggest / TestOpt and tests/test_fmin.py."""
import functools

import numpy as np
import pytest

from hyperopt_amd import STATUS_FAIL, STATUS_OK, Trials, fmin, hp, pyll, rand, tpe
from hyperopt_amd.base import Domain
from hyperopt_amd.pyll import scope
from tests.golden import spaces

pytestmark = pytest.mark.gpu


def passthrough(x):
    return x


# reference tests/test_domains.py objectives, written with this package's hp
def quadratic1():
    return {"loss": (hp.uniform("x", -5, 5) - 3) ** 2, "status": STATUS_OK}


def q1_lognormal():
    return {"loss": scope.min(0.1 * (hp.lognormal("x", 0, 2) - 10) ** 2, 10), "status": STATUS_OK}


def n_arms():
    rng = np.random.RandomState(123)
    x = hp.choice("x", [0, 1])
    mus = pyll.as_apply([-1, 0])
    sig = pyll.as_apply([1, 1])
    return {"loss": scope.normal(mus[x], sig[x], rng=rng), "loss_variance": 1.0,
            "status": STATUS_OK}


def distractor():
    x = hp.uniform("x", -15, 15)
    f1 = 1.0 / (1.0 + scope.exp(-x))
    f2 = 2 * scope.exp(-((x + 10) ** 2))
    return {"loss": -f1 - f2, "status": STATUS_OK}


def gauss_wave():
    x = hp.uniform("x", -20, 20)
    t = hp.choice("curve", [x, x + np.pi])
    return {"loss": -(scope.sin(t) + 2 * scope.exp(-((t / 5.0) ** 2))), "status": STATUS_OK}


def gauss_wave2():
    rng = np.random.RandomState(123)
    x = hp.uniform("x", -20, 20)
    amp = hp.uniform("amp", 0, 1)
    t = scope.normal(0, 0.1, rng=rng) + 2 * scope.exp(-((x / 5.0) ** 2))
    return {"loss": -hp.choice("hf", [t, t + scope.sin(x) * amp]), "loss_variance": 0.1,
            "status": STATUS_OK}


def many_dists():
    a = hp.choice("a", [0, 1, 2])
    b = hp.randint("b", 10)
    bb = hp.randint("bb", 12, 25)
    c = hp.uniform("c", 4, 7)
    d = hp.loguniform("d", -2, 0)
    e = hp.quniform("e", 0, 10, 3)
    f = hp.qloguniform("f", 0, 3, 2)
    g = hp.normal("g", 4, 7)
    h = hp.lognormal("h", -2, 2)
    i = hp.qnormal("i", 0, 10, 2)
    j = hp.qlognormal("j", 0, 2, 1)
    k = hp.pchoice("k", [(0.1, 0), (0.9, 1)])
    z = a + b + bb + c + d + e + f + g + h + i + j + k
    return {"loss": scope.float(scope.log(1e-12 + z ** 2)), "status": STATUS_OK}


def branin():
    x = hp.uniform("x", -5.0, 10.0)
    y = hp.uniform("y", 0.0, 15.0)
    pi = float(np.pi)
    loss = ((y - (5.1 / (4 * pi ** 2)) * x ** 2 + 5 * x / pi - 6) ** 2
            + 10 * (1 - 1 / (8 * pi)) * scope.cos(x) + 10)
    return {"loss": loss, "loss_variance": 0, "status": STATUS_OK}


DOMAINS = dict(quadratic1=quadratic1, q1_lognormal=q1_lognormal, n_arms=n_arms,
               distractor=distractor, gauss_wave=gauss_wave, gauss_wave2=gauss_wave2,
               many_dists=many_dists, branin=branin)


@pytest.mark.parametrize("name", sorted(DOMAINS))
def test_suggest_smoke(name):
    """TestSuggest (test_tpe.py:541-552): every domain runs with n_EI=3."""
    trials = Trials()
    fmin(passthrough, space=DOMAINS[name](), algo=functools.partial(tpe.suggest, n_EI_candidates=3),
         trials=trials, max_evals=30, rstate=np.random.RandomState(0), show_progressbar=False)
    assert len(trials) == 30


# TestOpt thresholds (test_tpe.py:567-668)
THRESH = dict(quadratic1=1e-5, q1_lognormal=0.01, distractor=-1.96, gauss_wave=-2.0,
              gauss_wave2=-2.0, n_arms=-2.5, many_dists=0.0005, branin=0.7)
LEN = dict(quadratic1=1000, many_dists=200, distractor=100, q1_lognormal=250, gauss_wave2=75,
           branin=200)
GAMMAS = dict(distractor=0.05)
PRIOR_WEIGHTS = dict(distractor=0.01)
N_EIS = dict(quadratic1=5, distractor=15)


@pytest.mark.parametrize("name", ["quadratic1", "q1_lognormal", "many_dists", "branin",
                                  "gauss_wave", "distractor"])
def test_opt_quality(name):
    algo = functools.partial(tpe.suggest, gamma=GAMMAS.get(name, 0.25),
                             prior_weight=PRIOR_WEIGHTS.get(name, 1.0),
                             n_EI_candidates=N_EIS.get(name, 24))
    trials = Trials()
    n = LEN.get(name, 50)
    fmin(passthrough, space=DOMAINS[name](), algo=algo, trials=trials, max_evals=n,
         rstate=np.random.RandomState(123), show_progressbar=False)
    assert len(trials) == n
    assert min(trials.losses()) < THRESH[name], (name, min(trials.losses()))


def test_quadratic_converges_near_optimum():
    trials = Trials()
    best = fmin(lambda x: (x - 3) ** 2, hp.uniform("x", -5, 5), algo=tpe.suggest, max_evals=100,
                trials=trials, rstate=np.random.RandomState(1), show_progressbar=False)
    assert abs(best["x"] - 3) < 0.15


def test_status_fail_trials_are_above():
    """test_fmin.py:208-226: failed trials get loss=inf and TPE still runs."""
    def fn(x):
        return {"status": STATUS_FAIL} if x > 0 else {"loss": x ** 2, "status": STATUS_OK}
    trials = Trials()
    fmin(fn, hp.uniform("x", -5, 5), algo=tpe.suggest, max_evals=60, trials=trials,
         rstate=np.random.RandomState(2), show_progressbar=False)
    assert len(trials) == 60


def test_suggest_document_and_determinism():
    space = spaces.many_dists(hp)
    dom = Domain(passthrough, space)
    trials = Trials()
    fmin(lambda p: float(np.sum([v for v in p.values()])), space, algo=rand.suggest,
         max_evals=40, trials=trials, rstate=np.random.RandomState(3), show_progressbar=False)
    docs1 = tpe.suggest([40], dom, trials, 1234, n_EI_candidates=4096)
    docs2 = tpe.suggest([40], dom, trials, 1234, n_EI_candidates=4096)
    assert docs1[0]["misc"]["vals"] == docs2[0]["misc"]["vals"]
    doc = docs1[0]
    trials.assert_valid_trial(doc)
    assert doc["tid"] == 40 and doc["misc"]["tid"] == 40 and doc["state"] == 0
    vals = doc["misc"]["vals"]
    assert set(vals) == set(dom.params)
    assert 12 <= vals["bb"][0] < 25  # randint(low, high) offset re-applied
    assert 0 <= vals["b"][0] < 10 and vals["k"][0] in (0, 1, 2)
    assert vals["e"][0] % 3 == 0 and 0 <= vals["e"][0] <= 10
    assert vals["f"][0] % 2 == 0 and vals["j"][0] == round(vals["j"][0])
    assert 4 <= vals["c"][0] < 7 and np.exp(-2) <= vals["d"][0] < 1.0


def test_nested_space_levels():
    """Conditional space: only the chosen branch's labels are active."""
    space = spaces.nested(hp)
    dom = Domain(passthrough, space)
    trials = Trials()
    fmin(lambda p: float(hash(str(p)) % 97) / 97.0, space, algo=rand.suggest, max_evals=60,
         trials=trials, rstate=np.random.RandomState(4), show_progressbar=False)
    for seed in range(5):
        doc = tpe.suggest([60], dom, trials, seed, n_EI_candidates=512)[0]
        vals = doc["misc"]["vals"]
        root = vals["root"][0]
        active = {k for k, v in vals.items() if v}
        expect = {0: {"root", "lin_lr"}, 1: {"root", "tree_depth", "tree_split"},
                  2: {"root", "nn_units", "nn_drop"}}[root]
        if root == 1:
            expect |= {"gini_w"} if vals["tree_split"][0] == 0 else {"ent_w", "ent_s"}
        assert active == expect, (root, active)
        assert all(doc["misc"]["idxs"][k] == ([60] if k in active else []) for k in vals)


def test_startup_delegates_to_rand():
    space = {"x": hp.uniform("x", 0, 1)}
    dom = Domain(passthrough, space)
    trials = Trials()
    docs = tpe.suggest([0], dom, trials, 7)
    assert docs[0]["misc"]["vals"]["x"][0] == \
        rand.suggest_device([0], dom, trials, 7)[0]["misc"]["vals"]["x"][0]


def test_large_candidate_count_fp32_and_fp64_agree():
    """2^20 candidates on a 2k history: both precisions land on (nearly) the same best."""
    space = {"x": hp.uniform("x", -5, 5), "y": hp.loguniform("y", -3, 0)}
    dom = Domain(passthrough, space)
    trials = Trials()
    fmin(lambda p: (p["x"] - 1) ** 2 + np.log(p["y"]) ** 2, space, algo=rand.suggest,
         max_evals=2000, trials=trials, rstate=np.random.RandomState(5), show_progressbar=False)
    d32 = tpe.suggest([2000], dom, trials, 99, n_EI_candidates=1 << 20, precision=32)[0]
    d64 = tpe.suggest([2000], dom, trials, 99, n_EI_candidates=1 << 20, precision=64)[0]
    for k in ("x", "y"):
        assert abs(d32["misc"]["vals"][k][0] - d64["misc"]["vals"][k][0]) < 0.05


def test_suggest_many_matches_single_calls():
    """Batched multi-study suggest (C4 shape, scaled down) == per-study suggest."""
    reqs = []
    for s in range(6):
        space = spaces.many_dists(hp) if s % 2 else spaces.nested(hp)
        dom = Domain(passthrough, space)
        trials = Trials()
        fmin(lambda p: float(hash(str(p)) % 101) / 101.0, space, algo=rand.suggest,
             max_evals=30 + 5 * s, trials=trials, rstate=np.random.RandomState(s),
             show_progressbar=False)
        reqs.append(tpe.SuggestRequest([len(trials)], dom, trials, 1000 + s,
                                       n_EI_candidates=256))
    batched = tpe.suggest_many(reqs)
    for rq, docs in zip(reqs, batched):
        single = tpe.suggest(rq.new_ids, rq.domain, rq.trials, rq.seed, n_EI_candidates=256)
        assert docs[0]["misc"]["vals"] == single[0]["misc"]["vals"]
        assert docs[0]["misc"]["idxs"] == single[0]["misc"]["idxs"]
