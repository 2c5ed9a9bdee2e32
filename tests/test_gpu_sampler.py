"""Sampler distributions (Philox on the GPU) vs the reference's accepted
distribution: one-sample KS against the exact truncated-mixture CDF, and
two-sample KS against draws of the reference-style rejection sampler.
North star: "The sampler's distributions must pass KS tests against the
reference"."""
import numpy as np
import pytest
from scipy import stats

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

N = 200_000


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


CASES = [
    ("uniform", (-5.0, 5.0), lambda r, n: r.uniform(-5, 5, n)),
    ("normal", (1.0, 3.0), lambda r, n: r.normal(1, 3, n)),
    ("loguniform", (-4.0, 1.0), lambda r, n: np.exp(r.uniform(-4, 1, n))),
    ("lognormal", (0.0, 1.0), lambda r, n: np.exp(r.normal(0, 1, n))),
]


def _draw(engine, kind, args, obs_b, precision, key=11):
    from hyperopt_amd.engine import LabelWork
    w = LabelWork("x", kind, args, obs_b, obs_b[:3], n_cand=N, key=key)
    r, = engine.run([w], precision=precision, sample_only=True)
    return r.cand


@pytest.mark.parametrize("precision", [64, 32])
@pytest.mark.parametrize("kind,args,gen", CASES)
def test_ks_continuous(engine, kind, args, gen, precision):
    rng = np.random.RandomState(3)
    obs_b = gen(rng, 25)
    x = _draw(engine, kind, args, obs_b, precision)
    fam, pmu, psig, tf, low, high, q = O.posterior_spec(kind, args)
    w, mu, sig = O.adaptive_parzen_normal(tf(obs_b), 1.0, pmu, psig)
    y = np.log(x) if fam == "LGMM1" else x
    if low is not None:
        assert y.min() >= low and y.max() < high
    cdf = lambda v: O.truncated_mixture_cdf(v, w, mu, sig, low, high)  # noqa: E731
    p1 = stats.kstest(y, cdf).pvalue
    ref = (O.gmm1_sample if fam == "GMM1" else O.lgmm1_sample)(
        w, mu, sig, low=low, high=high, rng=np.random.RandomState(9), size=N)
    p2 = stats.ks_2samp(x, ref).pvalue
    assert p1 > 1e-4 and p2 > 1e-4, (p1, p2)


@pytest.mark.parametrize("kind,args", [("quniform", (0.0, 20.0, 1.0)),
                                       ("qnormal", (0.0, 5.0, 2.0)),
                                       ("qloguniform", (0.0, 3.0, 1.0)),
                                       ("qlognormal", (0.0, 1.0, 0.5))])
def test_chi2_quantized(engine, kind, args):
    rng = np.random.RandomState(4)
    fam, pmu, psig, tf, low, high, q = O.posterior_spec(kind, args)
    if kind == "quniform":
        obs_b = np.round(rng.uniform(0, 20, 25))
    elif kind == "qnormal":
        obs_b = np.round(rng.normal(0, 5, 25) / 2) * 2
    elif kind == "qloguniform":
        obs_b = np.round(np.exp(rng.uniform(0, 3, 25)))
    else:
        obs_b = np.round(np.exp(rng.normal(0, 1, 25)) / 0.5) * 0.5
    x = _draw(engine, kind, args, obs_b, 64)
    k = np.round(x / q).astype(np.int64)
    assert np.all(k * q == x)
    ref = (O.gmm1_sample if fam == "GMM1" else O.lgmm1_sample)(
        *O.adaptive_parzen_normal(tf(obs_b), 1.0, pmu, psig), low=low, high=high, q=q,
        rng=np.random.RandomState(5), size=N)
    kr = np.round(ref / q).astype(np.int64)
    lo, hi = min(k.min(), kr.min()), max(k.max(), kr.max())
    a = np.bincount(k - lo, minlength=hi - lo + 1)
    b = np.bincount(kr - lo, minlength=hi - lo + 1)
    keep = (a + b) >= 20
    table = np.vstack([np.append(a[keep], a[~keep].sum()), np.append(b[keep], b[~keep].sum())])
    table = table[:, table.sum(0) > 0]
    p = stats.chi2_contingency(table)[1]
    assert p > 1e-4, p


@pytest.mark.parametrize("K,n_cand", [(3, N), (8, N), (40, N), (300, 1 << 17), (8, 1001)])
def test_categorical_draws_and_argmax(engine, K, n_cand):
    """Categorical draws follow the below posterior (chi^2 goodness of fit)
    and the chosen candidate is np.argmax's over the drawn candidates' scores
    (first index of the best-scoring category drawn) -- for K in registers,
    K by binary search and K past the rank-key path; n_cand not a multiple
    of the per-thread count exercises the tail."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(K)
    obs_b = rng.randint(0, K, 25)
    obs_a = rng.randint(0, K, 400)
    w = LabelWork("c", "randint", (K,), obs_b, obs_a, n_cand=n_cand, key=97 + K)
    r, = engine.run([w], outputs=True)
    k = r.cand.astype(np.int64)
    assert k.min() >= 0 and k.max() < K
    ref = O.categorical_label_scores("randint", (K,), obs_b, obs_a, k)
    # p is bit-exact (test_gpu_posteriors); its log may differ from numpy's by an ulp
    np.testing.assert_allclose(r.below_llik, ref["below_llik"], rtol=1e-14, atol=0)
    np.testing.assert_allclose(r.above_llik, ref["above_llik"], rtol=1e-14, atol=0)
    s = r.below_llik - r.above_llik
    best = int(np.argmax(s))
    assert (r.index, int(r.value), r.score) == (best, int(k[best]), s[best])
    assert r.index == ref["best"] or abs(s[r.index] - s[ref["best"]]) < 1e-12
    if n_cand >= 1 << 17:
        counts = np.bincount(k, minlength=K)
        expect = ref["p_below"] * n_cand
        keep = expect >= 20
        obs_c = np.append(counts[keep], counts[~keep].sum())
        exp_c = np.append(expect[keep], expect[~keep].sum())
        if exp_c[-1] == 0:
            obs_c, exp_c = obs_c[:-1], exp_c[:-1]
        p = stats.chisquare(obs_c, exp_c)[1]
        assert p > 1e-4, p
