"""Component windows of the quantized log-mass (tpe_score_quantized /
tpe_lattice_suggest with reach arrays, k_qreach): a value sums only the
components whose erf pair is not saturated (tpe.py:159-174, 288-305: a term
whose two CDFs are both exactly 0 or 1 adds nothing), and every thread keeps
its own components in its own order -- so the windowed sums are the full
loop's BIT FOR BIT.  Checked on sorted and unsorted mixtures, with NaN
components, small and multi-pass (> 8192 components) sizes, both families,
bounded or not, against the same kernel without windows; plus the oracle."""
import numpy as np
import pytest

from hyperopt_amd import _lib as L
from hyperopt_amd import mixture as M

pytestmark = pytest.mark.gpu


def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _mixture(rng, k, lg, sort, nan):
    mu = rng.uniform(-1.0, 6.0, k) if not lg else rng.uniform(-2.0, 2.0, k)
    if sort:
        mu = np.sort(mu)
    s = np.exp(rng.uniform(np.log(0.01), np.log(2.0), k))
    s[rng.randint(k)] = 30.0  # a wide (prior-like) component anywhere
    w = rng.uniform(0.1, 1.0, k)
    if nan:
        mu[-1] = np.nan
    return w / w.sum(), mu, s


@pytest.mark.parametrize("k", [37, 3000, 20000, 70000])
@pytest.mark.parametrize("lg", [False, True])
@pytest.mark.parametrize("sort", [True, False])
def test_windowed_quantized_sums_are_the_full_loop_bits(k, lg, sort):
    _gpu()
    rng = np.random.RandomState(k + 2 * lg + 4 * sort)
    w, mu, s = _mixture(rng, k, lg, sort, nan=False)
    fam = L.LGMM1 if lg else L.GMM1
    for bounded in (False, True):
        low, high = ((-1.0, 2.0) if lg else (0.0, 5.0)) if bounded else (None, None)
        m = M._Mixture(fam, w, mu, s, low, high)
        q = 0.25
        x = np.round(rng.uniform(0.05, 6.0, 400) / q) * q
        flags = L.F_QUANT | ((L.F_LOW | L.F_HIGH) if bounded else 0)
        full = m.lpdf(x, flags, low, high, q, 64, windows=False)
        win = m.lpdf(x, flags, low, high, q, 64, windows=True)
        assert np.array_equal(full.view(np.uint64), win.view(np.uint64)), (bounded, k)
        assert np.isfinite(full).any()


def test_windowed_sums_keep_nan_components():
    _gpu()
    rng = np.random.RandomState(5)
    w, mu, s = _mixture(rng, 500, False, True, nan=True)
    m = M._Mixture(L.GMM1, w, mu, s, None, None)
    x = np.arange(0.0, 6.0, 0.5)
    full = m.lpdf(x, L.F_QUANT, None, None, 0.5, 64, windows=False)
    win = m.lpdf(x, L.F_QUANT, None, None, 0.5, 64, windows=True)
    assert np.isnan(full).all() and np.isnan(win).all()


def test_windowed_lpdf_matches_oracle():
    _gpu()
    from oracle import tpe_oracle as O
    rng = np.random.RandomState(9)
    w, mu, s = _mixture(rng, 5000, False, True, nan=False)
    x = np.round(rng.uniform(0.0, 5.0, 300) / 0.5) * 0.5
    got = M.GMM1_lpdf(x, w, mu, s, low=0.0, high=5.0, q=0.5)
    want = O.gmm1_lpdf(x, w, mu, s, low=0.0, high=5.0, q=0.5)
    np.testing.assert_allclose(got, want, rtol=1e-8, atol=1e-8)
