"""Config C5 (BASELINE configs[4]) sizes: 100k-trial histories.

* adaptive_parzen_normal (tpe.py:399-467) on ~1e5-observation above sets:
  means and bandwidths bit-identical to the oracle (log-transformed labels:
  within an ulp of numpy's log), weights rtol 1e-12 --
  past every size the round-1 tests reached (fit sort tiles, table plans,
  the 32 768-cell budget).
* GMM1_lpdf / LGMM1_lpdf (tpe.py:117-180, 265-307) of injected candidates
  against 1e5-component above mixtures: exact fp64 path rtol 1e-6, fp32 table
  path rtol 1e-4 (north_star).
* One nested-choice suggest (tpe.py:837-964) at T = 100k: every level's
  winner is re-derived by scoring that level's whole candidate stream with
  the oracle and taking np.argmax (tpe.py:650-658).
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

T = 100_000


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


def _obs(kind, n, rng):
    if kind == "uniform":
        return rng.uniform(-5, 5, n)
    if kind == "loguniform":
        return np.exp(rng.uniform(-5, 0, n))
    if kind == "quniform":
        return np.round(rng.uniform(0, 100, n))
    return rng.normal(0, 2, n)


ARGS = {"uniform": (-5.0, 5.0), "loguniform": (-5.0, 0.0), "quniform": (0.0, 100.0, 1.0),
        "normal": (0.0, 2.0)}


@pytest.mark.parametrize("kind", ["uniform", "loguniform", "quniform", "normal"])
@pytest.mark.parametrize("n", [99_976, 100_000])
def test_fit_at_1e5(engine, kind, n):
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(n % 97 + len(kind))
    obs = _obs(kind, n, rng)
    w = LabelWork("x", kind, ARGS[kind], obs[:25], obs)
    r, = engine.run([w], posteriors=True)
    fam, pmu, psig, tf, low, high, q = O.posterior_spec(kind, ARGS[kind])
    for half, o in (("below", obs[:25]), ("above", obs)):
        ow, omu, osig = O.adaptive_parzen_normal(tf(o), 1.0, pmu, psig)
        gw, gmu, gsig = r.extra[half]
        if kind == "loguniform":
            # the means are log(obs): the device's fp64 log and numpy's may
            # differ in the last bit (neither is correctly rounded)
            np.testing.assert_allclose(gmu, omu, rtol=4.5e-16, atol=0)
            np.testing.assert_allclose(gsig, osig, rtol=1e-12, atol=0)
        else:
            np.testing.assert_array_equal(gmu, omu)
            np.testing.assert_array_equal(gsig, osig)
        np.testing.assert_allclose(gw, ow, rtol=1e-12, atol=0)


@pytest.mark.parametrize("kind", ["uniform", "loguniform", "normal", "quniform"])
def test_scores_at_1e5_vs_oracle(engine, kind):
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(7 + len(kind))
    obs = _obs(kind, T, rng)
    losses = rng.normal(size=T)
    below, above = O.ap_split_trials(np.arange(T), obs, np.arange(T), losses, 0.25)
    cand = _obs(kind, 1024, rng)
    w = LabelWork("x", kind, ARGS[kind], below, above, cand=cand)
    with np.errstate(all="ignore"):
        ref = O.continuous_label_scores(kind, ARGS[kind], below, above, cand)
    r64, = engine.run([w], precision=64, outputs=True)
    np.testing.assert_allclose(r64.below_llik, ref["below_llik"], rtol=1e-6)
    np.testing.assert_allclose(r64.above_llik, ref["above_llik"], rtol=1e-6)
    assert r64.index == ref["best"]
    scorer = "auto" if kind.startswith("q") else "table"
    r32, = engine.run([w], precision=32, outputs=True, scorer=scorer)
    np.testing.assert_allclose(r32.below_llik, ref["below_llik"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(r32.above_llik, ref["above_llik"], rtol=1e-4, atol=1e-4)
    s = ref["below_llik"] - ref["above_llik"]
    assert s[r32.index] >= np.nanmax(s) - 1e-4 * max(1.0, abs(np.nanmax(s)))
    if not kind.startswith("q"):
        st = engine.last_table_stats
        assert st is not None and st["exact_candidates"] <= 0.01 * cand.size, st


@pytest.fixture(scope="module")
def nested_100k():
    from hyperopt_amd import hp
    from hyperopt_amd.base import Domain
    from tests.golden import spaces
    from tools import scale_configs as S
    domain = Domain(lambda p: 0.0, spaces.nested(hp))
    return domain, S.prior_trials(domain, T, 0)


@pytest.mark.parametrize("seed", [3, 11])
def test_nested_suggest_at_100k_rescored_by_oracle(engine, nested_100k, seed):
    from hyperopt_amd import tpe
    domain, trials = nested_100k
    n_ei = 1024
    docs = tpe.suggest([T], domain, trials, seed, n_EI_candidates=n_ei, precision=64,
                       verbose=False)
    got = docs[0]["misc"]["vals"]
    # replay the level walk on the host lists and re-derive every winner
    labels = list(domain.params)
    hist = tpe.collect_history(trials, labels)
    isb, isa = tpe.split_masks(hist, 0.25)
    obs = tpe.LevelInputs(hist, isb, isa, engine, device=False)
    walk, n_levels = {}, 0
    while True:
        level = [lab for lab in domain.reachable(walk) if lab not in walk]
        if not level:
            break
        n_levels += 1
        for lab, key in zip(level, tpe.label_keys(seed, level)):
            spec = domain.specs[lab]
            w = obs.work(lab, spec, labels.index(lab), n_cand=n_ei, key=key, n_total=n_ei)
            if spec.kind in ("randint", "categorical"):
                r, = engine.run([w], precision=64, outputs=True)
                ref = O.categorical_label_scores(spec.kind, tuple(spec.args), w.obs_below,
                                                 w.obs_above, r.cand.astype(np.int64))
                s = ref["below_llik"] - ref["above_llik"]
                cand = r.cand
            else:
                r, = engine.run([w], precision=64, sample_only=True)
                cand = r.cand
                u, inv = np.unique(cand, return_inverse=True)  # equal values score equally
                with np.errstate(all="ignore"):
                    ref = O.continuous_label_scores(spec.kind, tuple(spec.args), w.obs_below,
                                                    w.obs_above, u)
                s = (ref["below_llik"] - ref["above_llik"])[inv]
            best = int(np.argmax(s))
            use, store = tpe._decode(spec, cand[best])
            assert got[lab] == [store], (lab, got[lab], store)
            walk[lab] = use
    assert n_levels >= 2
    live = {lab for lab, v in got.items() if v}
    assert live == set(walk)


@pytest.mark.parametrize("kind", ["uniform", "normal"])
def test_c5_size_fp32_suggest_path_is_the_exact_argmax(kind):
    """BASELINE configs[4] at its stated size on one label: a 100k-trial
    history (above mixture ~1e5 components) and 2^24 EI candidates through the
    fp32 suggest path (cell table, score cubics, exact fp64 re-score of the
    band): the winner is np.argmax (tpe.py:649-658) over the exact fp64 scores
    of the same 2^24 candidates (the stream materialised by sample_only,
    scored by the pruned fp64 kernel) -- index, value and score -- and the
    winner and runner-up agree with the oracle."""
    from hyperopt_amd.engine import Engine, LabelWork
    eng = Engine()
    rng = np.random.RandomState(5 + len(kind))
    obs = _obs(kind, T, rng)
    losses = rng.normal(size=T)
    below, above = O.ap_split_trials(np.arange(T), obs, np.arange(T), losses, 0.25)
    n = 1 << 24
    w = LabelWork("x", kind, ARGS[kind], below, above, n_cand=n, key=0xC5)
    r, = eng.run([w], precision=32)
    assert eng.last_table_stats is not None and r.n_scored == n
    s, = eng.run([w], precision=32, sample_only=True)
    cand = s.cand
    eng.exact64 = "pruned"
    x, = eng.run([LabelWork("x", kind, ARGS[kind], below, above, cand=cand)], precision=64,
                 outputs=True)
    s64 = x.below_llik - x.above_llik
    best = int(np.argmax(s64))
    assert r.index == best, (r.index, best, s64[r.index], s64[best])
    assert r.value == cand[best]
    np.testing.assert_allclose(r.score, s64[best], rtol=1e-12, atol=1e-12)
    second = int(np.argmax(np.where(np.arange(n) == best, -np.inf, s64)))
    pick = np.array([best, second])
    with np.errstate(all="ignore"):
        ref = O.continuous_label_scores(kind, ARGS[kind], below, above, cand[pick])
    np.testing.assert_allclose(ref["below_llik"] - ref["above_llik"], s64[pick], rtol=1e-6,
                               atol=1e-9)
