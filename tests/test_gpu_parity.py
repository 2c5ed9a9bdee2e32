"""HIP path vs the reference's own vectors (tests/golden) and vs the oracle.

Every test here runs the product kernels (libtpe_hip.so) on the GPU through
the C ABI; the oracle / golden vectors are only the checker.
Tolerances (north_star): fp64 rtol 1e-6, fp32 rtol 1e-4 (atol 1e-4 for
log-densities near 0); argmax indices and categorical results bit-exact.
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O
from tests.golden_io import E2E_CASES, load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


def _works_from_fixture(case):
    from hyperopt_amd.engine import LabelWork
    arrays, meta = load("e2e_" + case)
    works, golden = [], []
    for lab, lm in sorted(meta["labels"].items()):
        if lm["n"] == 0:
            continue
        spec = meta["specs"][lab]
        below, above = O.ap_split_trials(arrays["obs_idxs/" + lab], arrays["obs_vals/" + lab],
                                         arrays["hist_tids"], arrays["hist_losses"],
                                         meta["gamma"])
        works.append(LabelWork(label=lab, kind=spec["kind"], args=tuple(spec["args"]),
                               obs_below=below, obs_above=above, cand=arrays["cand/" + lab]))
        golden.append((arrays["bl/" + lab], arrays["al/" + lab], lm["best"]))
    return works, golden, meta


@pytest.mark.parametrize("case", E2E_CASES)
def test_golden_fp64(engine, case):
    works, golden, meta = _works_from_fixture(case)
    res = engine.run(works, prior_weight=meta["prior_weight"], precision=64, outputs=True)
    for w, r, (bl, al, best) in zip(works, res, golden):
        np.testing.assert_allclose(r.below_llik, bl, rtol=1e-6, atol=0, equal_nan=True,
                                   err_msg="%s/%s below" % (case, w.label))
        np.testing.assert_allclose(r.above_llik, al, rtol=1e-6, atol=0, equal_nan=True,
                                   err_msg="%s/%s above" % (case, w.label))
        assert r.index == best, (case, w.label, r.index, best)
        assert r.value == float(w.cand[best])
        assert r.n_scored == len(w.cand)


@pytest.mark.parametrize("case", E2E_CASES)
def test_golden_fp32(engine, case):
    works, golden, meta = _works_from_fixture(case)
    res = engine.run(works, prior_weight=meta["prior_weight"], precision=32, outputs=True)
    for w, r, (bl, al, best) in zip(works, res, golden):
        np.testing.assert_allclose(r.below_llik, bl, rtol=1e-4, atol=1e-4, equal_nan=True,
                                   err_msg="%s/%s below" % (case, w.label))
        np.testing.assert_allclose(r.above_llik, al, rtol=1e-4, atol=1e-4, equal_nan=True,
                                   err_msg="%s/%s above" % (case, w.label))
        # every kind index-exact: the fp32 log-densities are within 1e-4, the
        # argmax is decided on exact scores (Engine._exact_decision)
        assert r.index == best, (case, w.label, r.index, best)
        assert r.value == float(w.cand[best])


def _mixture_case(rng, kind, args, n_obs_b, n_obs_a, n_cand):
    from hyperopt_amd.engine import LabelWork
    fam, pmu, psig, tf, low, high, q = O.posterior_spec(kind, args)
    if kind in ("uniform", "quniform"):
        draw = lambda n: rng.uniform(args[0], args[1], n)  # noqa: E731
    elif kind in ("loguniform", "qloguniform"):
        draw = lambda n: np.exp(rng.uniform(args[0], args[1], n))  # noqa: E731
    elif kind in ("normal", "qnormal"):
        draw = lambda n: rng.normal(args[0], args[1], n)  # noqa: E731
    else:
        draw = lambda n: np.exp(rng.normal(args[0], args[1], n))  # noqa: E731
    obs_b, obs_a, cand = draw(n_obs_b), draw(n_obs_a), draw(n_cand)
    if q is not None:
        obs_b, obs_a, cand = (np.round(v / q) * q for v in (obs_b, obs_a, cand))
    return LabelWork(label=kind, kind=kind, args=args, obs_below=obs_b, obs_above=obs_a,
                     cand=cand)


KINDS = [("uniform", (-5.0, 5.0)), ("loguniform", (-5.0, 0.0)), ("normal", (0.0, 2.0)),
         ("lognormal", (0.0, 1.0)), ("quniform", (0.0, 100.0, 1.0)),
         ("qloguniform", (0.0, 4.0, 1.0)), ("qnormal", (0.0, 10.0, 2.0)),
         ("qlognormal", (0.0, 1.0, 0.5))]


@pytest.mark.parametrize("kind,args", KINDS)
@pytest.mark.parametrize("n_above", [0, 1, 2, 30, 3000])
def test_oracle_random_mixtures(engine, kind, args, n_above):
    """Bigger / edge histories than the goldens: HIP fp64 vs the oracle."""
    rng = np.random.RandomState(hash((kind, n_above)) % (2 ** 31))
    w = _mixture_case(rng, kind, args, min(n_above, 25), n_above, 2048)
    r64, = engine.run([w], precision=64, outputs=True)
    with np.errstate(all="ignore"):
        ref = O.continuous_label_scores(kind, args, w.obs_below, w.obs_above, w.cand)
    np.testing.assert_allclose(r64.below_llik, ref["below_llik"], rtol=1e-6, equal_nan=True)
    np.testing.assert_allclose(r64.above_llik, ref["above_llik"], rtol=1e-6, equal_nan=True)
    assert r64.index == ref["best"]
    r32, = engine.run([w], precision=32, outputs=True)
    np.testing.assert_allclose(r32.below_llik, ref["below_llik"], rtol=1e-4, atol=1e-4,
                               equal_nan=True)
    np.testing.assert_allclose(r32.above_llik, ref["above_llik"], rtol=1e-4, atol=1e-4,
                               equal_nan=True)
    assert r32.index == ref["best"]  # injected at fp32: the exact argmax too
    # injected without outputs (the fp32 scorers' own path) -- the same winner
    r32n, = engine.run([w], precision=32)
    assert (r32n.index, r32n.value) == (ref["best"], float(w.cand[ref["best"]]))


@pytest.mark.parametrize("kind,args", KINDS[:4])
@pytest.mark.parametrize("n_cand", [500, 1 << 17])
def test_fp32_outputs_winner_is_exact(engine, kind, args, n_cand):
    """Sampled candidates with per-candidate outputs at fp32 (the dense fp32
    kernel below TABLE_MIN_CAND, the two-polynomial table scorer above): the
    winner is np.argmax of the oracle's fp64 scores of the very candidates
    returned, index and value."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(n_cand)
    w0 = _mixture_case(rng, kind, args, 25, 4000, 1)
    w = LabelWork(kind, kind, args, w0.obs_below, w0.obs_above, n_cand=n_cand, key=4242,
                  cand_base=77)
    r, = engine.run([w], precision=32, outputs=True)
    with np.errstate(all="ignore"):
        ref = O.continuous_label_scores(kind, args, w.obs_below, w.obs_above, r.cand)
    assert r.index == 77 + ref["best"] and r.value == r.cand[ref["best"]]


def test_argmax_ties_and_far_tails(engine):
    """Duplicate candidates (exact score ties -> first index) and far-tail
    candidates (fp32 exact-LSE fallback path)."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(7)
    obs_b = rng.uniform(-5, 5, 25)
    obs_a = rng.uniform(-5, 5, 4000)
    base = rng.uniform(-5, 5, 300)
    cand = np.concatenate([base, base[::-1], [-1e3, 1e3, 60.0, -60.0]])
    w = LabelWork("x", "uniform", (-5.0, 5.0), obs_b, obs_a, cand=cand)
    with np.errstate(all="ignore"):
        ref = O.continuous_label_scores("uniform", (-5.0, 5.0), obs_b, obs_a, cand)
    r64, = engine.run([w], precision=64, outputs=True)
    assert r64.index == ref["best"]
    np.testing.assert_allclose(r64.above_llik, ref["above_llik"], rtol=1e-6)
    r32, = engine.run([w], precision=32, outputs=True)
    np.testing.assert_allclose(r32.above_llik, ref["above_llik"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(r32.below_llik, ref["below_llik"], rtol=1e-4, atol=1e-4)
    assert r32.index == ref["best"]  # ties: the first index, at fp32 too


SORT_KINDS = [("uniform", (-5.0, 5.0), lambda r, n: r.uniform(-5, 5, n)),
              ("loguniform", (-5.0, 0.0), lambda r, n: np.exp(r.uniform(-5, 0, n))),
              ("normal", (0.0, 2.0), lambda r, n: r.normal(0, 2, n)),
              ("lognormal", (0.0, 1.0), lambda r, n: np.exp(r.normal(0, 1, n)))]


@pytest.mark.parametrize("kind,args,gen", SORT_KINDS)
@pytest.mark.parametrize("n_hist", [3, 40, 2000, 10000])
def test_sorted_pruned_matches_dense(engine, kind, args, gen, n_hist):
    """The sorted + component-pruned fp32 path picks the dense path's winner
    (same Philox candidates) -- or, on a near tie, one whose exact fp64 score
    is within fp32 rounding of it."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(n_hist)
    obs = gen(rng, n_hist)
    losses = rng.normal(size=n_hist)
    below, above = O.ap_split_trials(np.arange(n_hist), obs, np.arange(n_hist), losses, 0.25)
    w = LabelWork(kind, kind, args, below, above, n_cand=1 << 18, key=987654321 + n_hist)
    dense, = engine.run([w], precision=32, scorer="dense")
    pruned, = engine.run([w], precision=32, scorer="sorted")
    pairs = engine.last_pairs
    assert pruned.n_scored == dense.n_scored == 1 << 18
    if pruned.index == dense.index:
        assert pruned.value == dense.value
    else:
        w2 = LabelWork(kind, kind, args, below, above,
                       cand=np.array([dense.value, pruned.value]))
        r, = engine.run([w2], precision=64, outputs=True)
        s = r.below_llik - r.above_llik
        assert abs(s[0] - s[1]) <= 1e-4 * max(1.0, abs(s[0])), (s, dense, pruned)
    dense_pairs = (1 << 18) * (below.size + above.size + 2)
    assert 0 < pairs <= dense_pairs
    if n_hist >= 2000:
        assert pairs < 0.5 * dense_pairs  # pruning is effective on real histories
