"""Explicit mixtures on the HIP path (hyperopt_amd.mixture): the reference's
own known-answer and statistical tests for GMM1 / GMM1_lpdf / LGMM1 /
LGMM1_lpdf (hyperopt/tests/test_tpe.py:73-538), run at fp64 and fp32, plus
parity of the lpdf against the oracle's restatement (oracle/tpe_oracle.py
gmm1_lpdf / lgmm1_lpdf, tpe.py:117-180, 265-307) on random mixtures.

The statistical tests keep the reference's thresholds (max err < 0.1, mean
and median < 0.01) and its RandomState(234) seeding; the draws themselves come
from the library's Philox streams keyed by that RandomState (same
distribution, not numpy's sequence), so these check the distribution, not a
sequence.  Argument-error tests need no GPU."""
import numpy as np
import pytest

from hyperopt_amd import mixture as M

PREC = [64, 32]


def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


# ---- argument handling (no GPU) ---------------------------------------------

def test_argument_errors():
    with pytest.raises(ValueError):
        M.GMM1([1.0], [0.0], [1.0], low=2.0, high=1.0, size=(3,))
    with pytest.raises(ValueError):
        M.LGMM1([1.0], [0.0], [1.0], low=2.0, high=2.0, size=(3,))
    with pytest.raises(TypeError):
        M.LGMM1([1.0], [0.0], [1.0], low=2.0, size=(3,))  # float(None), as the reference
    with pytest.raises(TypeError):
        M.GMM1_lpdf([1.0], [1.0], [0.0], [1.0], low=0.0)  # one-sided lpdf
    with pytest.raises(TypeError):
        M.GMM1_lpdf([1.0], [[1.0]], [0.0], [1.0])
    with pytest.raises(AssertionError):
        M.GMM1_lpdf([1.0], [1.0, 2.0], [0.0], [1.0])
    with pytest.raises(ValueError):
        M.GMM1_lpdf([1.0], [1.0], [0.0], [1.0], precision=16)
    assert M.GMM1_lpdf([], [1.0], [0.0], [1.0]).shape == (0,)  # tpe.py:124-125
    assert M.LGMM1_lpdf(np.zeros((0, 3)), [1.0], [0.0], [1.0]).shape == (0, 3)


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from hyperopt_amd import _lib as L
    with pytest.raises((L.TpeHipError, ImportError)):
        M.GMM1_lpdf([1.0], [1.0], [0.0], [1.0])


# ---- TestGMM1 (test_tpe.py:73-219) ------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("precision", PREC)
def test_gmm1_sampling_basics(precision):
    _gpu()
    rng = np.random.RandomState(234)
    kw = dict(rng=rng, precision=precision)
    assert np.allclose(10, M.GMM1([1], [10.0], [0.0000001], **kw))
    assert M.GMM1([1], [10.0], [1.0], **kw).shape == ()
    s = M.GMM1([1], [0.0], [10.0], size=[1000], **kw)
    assert 9 < np.std(s) < 11
    s = M.GMM1([0.5, 0.5], [0.0, 1.0], [0.000001, 0.000001], size=[1000], **kw)
    assert 0.45 < np.mean(s) < 0.55 and 0.2 < np.var(s) < 0.3
    s = M.GMM1([0.9999, 0.0001], [0.0, 1.0], [0.000001, 0.000001], size=[1000], **kw)
    assert s.shape == (1000,)
    assert -0.001 < np.mean(s) < 0.001 and np.var(s) < 0.0001
    s = M.GMM1([0.9999, 0.0001], [0.0, 1.0], [0.000001, 0.000001], size=[40, 20], **kw)
    assert s.shape == (40, 20)
    assert -0.001 < np.mean(s) < 0.001 and np.var(s) < 0.0001


def _a1():
    a = 0.25 / np.sqrt(2 * np.pi * 1.0 ** 2) * np.exp(-0.5 * 1.0 ** 2)
    a += 0.25 / np.sqrt(2 * np.pi * 2.0 ** 2)
    a += 0.5 / np.sqrt(2 * np.pi * 5.0 ** 2) * np.exp(-0.5 * (1.0 / 5.0) ** 2)
    return a


def _a0():
    a = 0.25 / np.sqrt(2 * np.pi * 1.0 ** 2)
    a += 0.25 / np.sqrt(2 * np.pi * 2.0 ** 2) * np.exp(-0.5 * (1.0 / 2.0) ** 2)
    a += 0.5 / np.sqrt(2 * np.pi * 5.0 ** 2) * np.exp(-0.5 * (2.0 / 5.0) ** 2)
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PREC)
def test_gmm1_lpdf_known_answers(precision):
    _gpu()
    W, MU, S = [0.25, 0.25, 0.5], [0.0, 1.0, 2.0], [1.0, 2.0, 5.0]
    ll = M.GMM1_lpdf(1.0, [1.0], [1.0], [2.0], precision=precision)
    assert ll.shape == ()
    assert np.allclose(ll, np.log(1.0 / np.sqrt(2 * np.pi * 2.0 ** 2)))
    ll = M.GMM1_lpdf(1.0, W, MU, S, precision=precision)
    assert ll.shape == () and np.allclose(ll, np.log(_a1()))
    ll = M.GMM1_lpdf([1.0, 0.0], W, MU, S, precision=precision)
    assert ll.shape == (2,)
    assert np.allclose(ll[0], np.log(_a1())) and np.allclose(ll[1], np.log(_a0()))
    ll = M.GMM1_lpdf([[1.0, 0.0, 0.0], [0, 0, 1], [0, 0, 1000]], W, MU, S, precision=precision)
    assert ll.shape == (3, 3)
    assert np.allclose(ll[0, 0], np.log(_a1())) and np.allclose(ll[1, 2], np.log(_a1()))
    for i, j in ((0, 1), (0, 2), (1, 0), (1, 1), (2, 0), (2, 1)):
        assert np.allclose(ll[i, j], np.log(_a0()))
    assert np.isfinite(ll[2, 2])


# ---- the Math classes (test_tpe.py:222-538) ---------------------------------
#
# The reference's procedure -- draws, a histogram, exp(lpdf) at the bins,
# thresholds max err < 0.1, mean and median < 0.01 -- is a noisy check: with
# numpy's own sampler it fails on a sizeable share of seeds (TestLGMM1Math
# basic: about a third; the reference's file passes because its seed 234
# happens to).  Our draws are a different stream, so instead of one seed the
# procedure runs on SEEDS seeds with both samplers -- ours (HIP) and the
# reference's (the oracle's numpy restatement, scored by the oracle's lpdf) --
# and our pass count must not fall short of the reference's by more than a
# 3-sigma binomial margin.  The sharp checks follow each class: a
# Kolmogorov-Smirnov test of 2^20 draws against the exact truncated CDF
# (continuous), and every lattice frequency of 2^20 draws against exp(lpdf)
# within 5 binomial sigmas (quantized).

SEEDS = range(24)


def _passes(err):
    return bool(np.max(err) < 0.1 and np.mean(err) < 0.01 and np.median(err) < 0.01)


def _compare_pass_rates(procedure):
    from oracle import tpe_oracle as O
    ours = sum(procedure(True, np.random.RandomState(s), O) for s in SEEDS)
    ref = sum(procedure(False, np.random.RandomState(s), O) for s in SEEDS)
    r = len(SEEDS)
    pbar = (ours + ref) / (2.0 * r)
    margin = 3.0 * np.sqrt(2.0 * r * pbar * (1.0 - pbar)) + 1.0
    assert ours >= ref - margin, (ours, ref, margin)


def _kw(c):
    return dict(weights=c["weights"], mus=c["mus"], sigmas=c["sigmas"], low=c.get("low"),
                high=c.get("high"), q=c.get("q"))


def _sample(ours, lg, c, rng, n, precision, O):
    if ours:
        f = M.LGMM1 if lg else M.GMM1
        return f(rng=rng, size=(n,), precision=precision, **_kw(c))
    f = O.lgmm1_sample if lg else O.gmm1_sample
    return f(c["weights"], c["mus"], c["sigmas"], c.get("low"), c.get("high"), c.get("q"), rng, n)


def _lpdf(ours, lg, c, x, precision, O):
    if ours:
        f = M.LGMM1_lpdf if lg else M.GMM1_lpdf
        return f(x, precision=precision, **_kw(c))
    f = O.lgmm1_lpdf if lg else O.gmm1_lpdf
    return f(x, c["weights"], c["mus"], c["sigmas"], c.get("low"), c.get("high"), c.get("q"))


def _ks(x, lg, c):
    """sqrt(n) D_n of the draws against the exact CDF (oracle's truncated
    mixture CDF, in log space for LGMM1)."""
    from oracle import tpe_oracle as O
    x = np.sort(np.log(x) if lg else x)
    n = x.size
    F = O.truncated_mixture_cdf(x, *(np.asarray(c[k], dtype=np.float64) for k in ("weights", "mus", "sigmas")),
                                c.get("low"), c.get("high"))
    i = np.arange(1, n + 1)
    return np.sqrt(n) * max(np.max(i / n - F), np.max(F - (i - 1) / n))


def _lattice_check(x, lg, c, precision):
    """Every lattice value's frequency in 2^20 q-rounded draws against
    exp(lpdf) (the mass of its rounding interval), within 5 binomial sigmas."""
    q = c["q"]
    k = x / q
    assert np.all(k == np.round(k))
    k = k.astype(np.int64)
    lo = int(k.min())
    counts = np.bincount(k - lo)
    xs = (np.arange(counts.size) + lo) * q
    p = np.exp(_lpdf(True, lg, c, xs, precision, None))
    n = x.size
    dev = np.abs(counts / n - p)
    assert np.all(dev <= 5 * np.sqrt(p * (1 - p) / n) + 2.0 / n), np.max(dev)
    assert 1.0 - 1e-3 < p.sum() <= 1.0 + 1e-9


GMM_W, GMM_MU, GMM_S = [0.1, 0.3, 0.4, 0.2], [1.0, 2.0, 3.0, 4.0], [0.1, 0.4, 0.8, 2.0]
GMM_CASES = [dict(), dict(low=2.5, high=3.5)]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PREC)
@pytest.mark.parametrize("case", range(len(GMM_CASES)))
def test_gmm1_math(precision, case):
    """TestGMM1Math (test_tpe.py:222-278): histograms of 10001 draws (500
    per bin) against exp(GMM1_lpdf) at the bin edges."""
    _gpu()
    c = dict(weights=GMM_W, mus=GMM_MU, sigmas=GMM_S)
    c.update(GMM_CASES[case])

    def procedure(ours, rng, O):
        s = np.sort(_sample(ours, False, c, rng, 10001, precision, O))
        if "low" in c:
            assert c["low"] <= s.min() and s.max() < c["high"]
        edges = s[::500]
        pdf = np.exp(_lpdf(ours, False, c, edges[:-1], precision, O))
        dx = edges[1:] - edges[:-1]
        return _passes((pdf - 1 / dx / len(dx)) ** 2)
    _compare_pass_rates(procedure)
    x = _sample(True, False, c, np.random.RandomState(234), 1 << 20, precision, None)
    assert _ks(x, False, c) < 2.2


QGMM_CASES = [
    dict(q=1), dict(q=2), dict(q=0.5), dict(q=1, low=2, high=4), dict(q=2, low=2, high=4),
    dict(q=1, low=1, high=4.1), dict(q=2, low=1, high=4.1),
    dict(weights=[0.14285714, 0.28571429, 0.28571429, 0.28571429], mus=[5.505, 7.0, 2.0, 10.0],
         sigmas=[8.99, 5.0, 8.0, 8.0], q=1, low=1.01, high=10, n_samples=10000),
    dict(weights=[0.33333333, 0.66666667], mus=[5.505, 5.0], sigmas=[8.99, 5.19], q=1,
         low=1.01, high=10, n_samples=10000),
]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PREC)
@pytest.mark.parametrize("case", range(len(QGMM_CASES)))
def test_qgmm1_math(precision, case):
    """TestQGMM1Math (test_tpe.py:281-381): bincount of the q-rounded draws
    against exp(GMM1_lpdf) on the lattice."""
    _gpu()
    c = dict(weights=GMM_W, mus=GMM_MU, sigmas=GMM_S, n_samples=1001)
    c.update(QGMM_CASES[case])
    n, q = c.pop("n_samples"), c["q"]

    def procedure(ours, rng, O):
        s = _sample(ours, False, c, rng, n, precision, O) / q
        assert np.all(s == s.astype("int"))
        lo, hi = int(s.min()), int(s.max())
        counts = np.bincount(s.astype("int") - lo)
        prob = np.exp(_lpdf(ours, False, c, np.arange(lo, hi + 1) * q, precision, O))
        assert counts.sum() == n
        return _passes((prob - counts / float(n)) ** 2)
    _compare_pass_rates(procedure)
    x = _sample(True, False, c, np.random.RandomState(234), 1 << 20, precision, None)
    _lattice_check(x, False, c, precision)


LGMM_W, LGMM_MU, LGMM_S = [0.1, 0.3, 0.4, 0.2], [-2.0, 1.0, 0.0, 3.0], [0.1, 0.4, 0.8, 2.0]
LGMM_CASES = [dict(), dict(low=2, high=4)]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PREC)
@pytest.mark.parametrize("case", range(len(LGMM_CASES)))
def test_lgmm1_math(precision, case):
    """TestLGMM1Math (test_tpe.py:384-444): 200-draw bins against
    exp(LGMM1_lpdf) at the bin centres."""
    _gpu()
    c = dict(weights=LGMM_W, mus=LGMM_MU, sigmas=LGMM_S)
    c.update(LGMM_CASES[case])

    def procedure(ours, rng, O):
        s = np.sort(_sample(ours, True, c, rng, 10001, precision, O))
        if "low" in c:
            assert np.exp(c["low"]) * (1 - 1e-6) <= s.min() and s.max() <= np.exp(c["high"])
        edges = s[::200]
        centers = 0.5 * edges[:-1] + 0.5 * edges[1:]
        pdf = np.exp(_lpdf(ours, True, c, centers, precision, O))
        dx = edges[1:] - edges[:-1]
        return _passes((pdf - 1 / dx / len(dx)) ** 2)
    _compare_pass_rates(procedure)
    x = _sample(True, True, c, np.random.RandomState(234), 1 << 20, precision, None)
    assert _ks(x, True, c) < 2.2


QLGMM_CASES = [dict(q=1), dict(q=2), dict(q=0.5), dict(q=0.125), dict(q=1, low=2, high=4),
               dict(q=2, low=2, high=4), dict(q=1, low=1, high=4.1), dict(q=2, low=1, high=4.1)]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PREC)
@pytest.mark.parametrize("case", range(len(QLGMM_CASES)))
def test_qlgmm1_math(precision, case):
    """TestQLGMM1Math (test_tpe.py:447-538): bincount of the q-rounded
    log-normal draws against exp(LGMM1_lpdf), first 20 lattice points."""
    _gpu()
    c = dict(weights=[0.1, 0.3, 0.4, 0.2], mus=[-2, 0.0, -3.0, 1.0], sigmas=[2.1, 0.4, 0.8, 2.1])
    c.update(QLGMM_CASES[case])
    q, n = c["q"], 1001

    def procedure(ours, rng, O):
        s = _sample(ours, True, c, rng, n, precision, O) / q
        assert np.all(s == s.astype("int"))
        lo, hi = int(s.min()), int(s.max())
        counts = np.bincount(s.astype("int") - lo)
        prob = np.exp(_lpdf(ours, True, c, np.arange(lo, hi + 0.5) * q, precision, O))
        assert counts.sum() == n
        return _passes(((prob - counts / float(n)) ** 2)[:20])
    _compare_pass_rates(procedure)
    x = _sample(True, True, c, np.random.RandomState(234), 1 << 20, precision, None)
    _lattice_check(x, True, c, precision)

# ---- parity against the oracle on random mixtures ---------------------------

def _random_mixture(rng, k, lg):
    w = rng.uniform(0.05, 2.0, k)  # deliberately not normalised
    mu = rng.normal(0.0 if lg else 3.0, 1.5, k)
    s = rng.uniform(0.05, 2.0, k)
    return w, mu, s


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PREC)
@pytest.mark.parametrize("lg", [False, True])
@pytest.mark.parametrize("bounded", [False, True])
@pytest.mark.parametrize("q", [None, 0.5])
def test_lpdf_matches_oracle(precision, lg, bounded, q):
    """GMM1_lpdf / LGMM1_lpdf against oracle/tpe_oracle.py (tpe.py:117-180,
    265-307) on 3000 values of random unnormalised 37-component mixtures.
    fp64: within 1e-12 relative (1e-8 (1 + |lpdf|) for quantized masses: a
    mass is a difference of CDFs, 0.5 (1 + erf), so one ulp of erf on either
    side moves a small mass by more than fp64 rounding); fp32 (unquantized
    only -- quantized masses are fp64 at either precision): the oracle at the
    fp32-rounded value, within 2e-5 (1 + |lpdf|)."""
    _gpu()
    from oracle import tpe_oracle as O
    rng = np.random.RandomState(11 + 2 * lg + 4 * bounded + 8 * (q is not None))
    w, mu, s = _random_mixture(rng, 37, lg)
    low, high = (-1.0, 2.0) if lg else (0.5, 5.5)
    if not bounded:
        low = high = None
    if lg:
        x = np.exp(rng.uniform(-2.5, 2.5, 3000))
    else:
        x = rng.uniform(-1.0, 7.0, 3000)
    if q is not None:
        x = np.round(x / q) * q
        if lg:
            x = x[x > 0]
        if bounded:  # values the label can take (the rounded support)
            lo_v, hi_v = (np.exp(low), np.exp(high)) if lg else (low, high)
            x = x[(x >= np.round(lo_v / q) * q) & (x <= np.round(hi_v / q) * q)]
    f = M.LGMM1_lpdf if lg else M.GMM1_lpdf
    o = O.lgmm1_lpdf if lg else O.gmm1_lpdf
    got = f(x, w, mu, s, low=low, high=high, q=q, precision=precision)
    if precision == 32 and q is None:
        want = o(x.astype(np.float32).astype(np.float64), w, mu, s, low=low, high=high, q=q)
        tol = 2e-5 * (1 + np.abs(want))
    else:
        want = o(x, w, mu, s, low=low, high=high, q=q)
        tol = 1e-8 * (1 + np.abs(want)) if q is not None else 1e-12 * (1 + np.abs(want))
    fin = np.isfinite(want)
    assert np.array_equal(fin, np.isfinite(got))
    err = np.abs(got - want)[fin]
    assert np.all(err <= tol[fin]), (np.max(err), np.argmax(err - tol[fin]))


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PREC)
@pytest.mark.parametrize("lg", [False, True])
@pytest.mark.parametrize("q", [0.5, 1.0])
def test_quantized_lpdf_outside_the_rounded_support(precision, lg, q):
    """Quantized values the bounded label cannot take (beyond round(low/q)q or
    round(high/q)q, and between the bound and that slot): the reference clips
    the bin to [low, high] with max/min (tpe.py:154-158, 296-300), so a bin
    past a bound has a negative or empty mass -- NaN or -inf, whichever its
    log gives -- and a bin straddling a bound a partial one.  The HIP lpdf
    gives the oracle's value, NaN and -inf included."""
    _gpu()
    from oracle import tpe_oracle as O
    rng = np.random.RandomState(71 + 2 * lg + int(4 * q))
    w, mu, s = _random_mixture(rng, 9, lg)
    low, high = (-1.0, 2.0) if lg else (0.5, 5.5)
    lo_v, hi_v = (np.exp(low), np.exp(high)) if lg else (low, high)
    ks = np.arange(np.floor(lo_v / q) - 4, np.ceil(hi_v / q) + 5)
    x = ks * q
    if lg:
        x = x[x > 0]
    x = x[(x < np.round(lo_v / q) * q + 2 * q) | (x > np.round(hi_v / q) * q - 2 * q)]
    f = M.LGMM1_lpdf if lg else M.GMM1_lpdf
    o = O.lgmm1_lpdf if lg else O.gmm1_lpdf
    with np.errstate(all="ignore"):
        want = o(x, w, mu, s, low=low, high=high, q=q)
    got = f(x, w, mu, s, low=low, high=high, q=q, precision=precision)
    assert (~np.isfinite(want)).any()  # the case is exercised
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    np.testing.assert_array_equal(np.isneginf(got), np.isneginf(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], rtol=1e-8, atol=1e-8)
