"""CPU oracle for the TPE suggest hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The shipped path (``hyperopt_amd``) never imports anything under
``oracle/`` and fails loudly when its HIP library is missing.

It is a from-scratch numpy restatement of the algorithm in the reference's
``hyperopt/tpe.py`` (hyperopt 0.2.4, mounted read-only at /root/reference).
Every function cites the reference lines it restates.  Parity of this
restatement with the reference is pinned by ``tests/golden/*.npz`` — vectors
produced by importing the reference itself (``tests/golden/make_golden.py``) —
and checked by ``tests/test_oracle_golden.py``.

Deliberate, documented choice: every argsort here defaults to
``kind="stable"``.  The reference calls ``np.argsort`` with numpy's default
(introsort / x86-simd-sort), whose tie order depends on the host CPU; the
goldens for tie-heavy data were generated with the reference's argsort forced
to ``kind="stable"`` (recorded in the fixture metadata), and tie-free goldens
use the unpatched reference.  See DESIGN.md "Tie semantics".
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import erf

EPS = 1e-12  # tpe.py:32
DEFAULT_LF = 25  # tpe.py:36
SQRT2 = math.sqrt(2.0)
SQRT_2PI = math.sqrt(2.0 * math.pi)


# ---------------------------------------------------------------------------
# Parzen posterior fit
# ---------------------------------------------------------------------------
def linear_forgetting_weights(n, lf):
    """Ramp weights, oldest observation first (tpe.py:380-392)."""
    if n < 0 or lf <= 0:
        raise AssertionError((n, lf))
    if n == 0:
        return np.zeros(0)
    if n < lf:
        return np.ones(n)
    return np.concatenate([np.linspace(1.0 / n, 1.0, num=n - lf), np.ones(lf)])


def adaptive_parzen_normal(obs, prior_weight, prior_mu, prior_sigma,
                           lf=DEFAULT_LF, sort_kind="stable"):
    """Prior-augmented Parzen mixture, sorted by mean (tpe.py:399-467).

    Returns (weights, mus, sigmas), each of length len(obs) + 1.
    """
    obs = np.asarray(obs, dtype=np.float64)
    if obs.ndim != 1:
        raise TypeError("mus must be vector", obs)
    n = obs.size
    order = None
    if n == 0:
        mus = np.array([prior_mu], dtype=np.float64)
        sig = np.array([prior_sigma], dtype=np.float64)
        pos = 0
    elif n == 1:
        # tpe.py:414-421 -- the prior goes AFTER an equal observation here
        if prior_mu < obs[0]:
            pos = 0
            mus = np.array([prior_mu, obs[0]])
            sig = np.array([prior_sigma, prior_sigma * 0.5])
        else:
            pos = 1
            mus = np.array([obs[0], prior_mu])
            sig = np.array([prior_sigma * 0.5, prior_sigma])
    else:
        # tpe.py:426-439 -- sort, insert prior (searchsorted side='left'),
        # bandwidth = max distance to the two neighbours, edge gaps at the ends
        order = np.argsort(obs, kind=sort_kind)
        srt = obs[order]
        pos = int(np.searchsorted(srt, prior_mu))
        mus = np.insert(srt, pos, prior_mu)
        gap = np.diff(mus)
        sig = np.empty_like(mus)
        sig[1:-1] = np.maximum(gap[:-1], gap[1:])
        sig[0] = gap[0]
        sig[-1] = gap[-1]

    # tpe.py:441-451 -- ramp weights follow the observation (tid) order
    if lf and lf < n:
        ramp = linear_forgetting_weights(n, lf)
        w = np.insert(ramp[order], pos, prior_weight)
    else:
        w = np.ones(mus.size)
        w[pos] = prior_weight

    # tpe.py:453-465 -- clip bandwidths, restore prior sigma, normalise
    hi = prior_sigma / 1.0
    lo = prior_sigma / min(100.0, 1.0 + mus.size)
    sig = np.clip(sig, lo, hi)
    sig[pos] = prior_sigma
    if not (prior_sigma > 0 and hi > 0 and lo > 0 and np.all(sig > 0)):
        raise AssertionError((sig.min(), lo, hi))
    w = w / w.sum()
    return w, mus, sig


def ap_split_trials(o_idxs, o_vals, l_idxs, l_vals, gamma,
                    gamma_cap=DEFAULT_LF, sort_kind="stable"):
    """Below/above split of one label's observations (tpe.py:623-646).

    The best ``min(ceil(gamma*sqrt(T)), gamma_cap)`` trials by loss form the
    "below" set; observation order (tid order) is preserved in both outputs.
    """
    o_idxs = np.asarray(o_idxs)
    o_vals = np.asarray(o_vals)
    l_idxs = np.asarray(l_idxs)
    l_vals = np.asarray(l_vals)
    n_below = min(int(np.ceil(gamma * np.sqrt(len(l_vals)))), gamma_cap)
    l_order = np.argsort(l_vals, kind=sort_kind)
    good = l_idxs[l_order[:n_below]]
    bad = l_idxs[l_order[n_below:]]
    if o_idxs.size == 0:
        return np.zeros(0), np.zeros(0)
    below = o_vals[np.isin(o_idxs, good)]
    above = o_vals[np.isin(o_idxs, bad)]
    return np.asarray(below, dtype=np.float64), np.asarray(above, dtype=np.float64)


# ---------------------------------------------------------------------------
# Densities
# ---------------------------------------------------------------------------
def normal_cdf(x, mu, sigma):
    """0.5*(1+erf((x-mu)/max(sqrt2*sigma, EPS))) (tpe.py:109-114)."""
    z = (x - mu) / np.maximum(SQRT2 * sigma, EPS)
    return 0.5 * (1 + erf(z))


def lognormal_cdf(x, mu, sigma):
    """0.5+0.5*erf((log(max(x,EPS))-mu)/max(sqrt2*sigma,EPS)) (tpe.py:186-205)."""
    x = np.asarray(x, dtype=np.float64)
    if x.size == 0:
        return np.zeros(0)
    if x.min() < 0:
        raise ValueError("negative arg to lognormal_cdf", x)
    with np.errstate(divide="ignore"):
        z = (np.log(np.maximum(x, EPS)) - mu) / np.maximum(SQRT2 * sigma, EPS)
    return 0.5 + 0.5 * erf(z)


def lognormal_lpdf(x, mu, sigma):
    """Per-component log-normal log density (tpe.py:208-217)."""
    sigma = np.maximum(sigma, EPS)
    z = sigma * x * SQRT_2PI
    e = 0.5 * ((np.log(x) - mu) / sigma) ** 2
    return -e - np.log(z)


def _lse_rows(a):
    """Row max then log-sum-exp, as logsum_rows (tpe.py:260-262)."""
    m = a.max(axis=1)
    return np.log(np.exp(a - m[:, None]).sum(axis=1)) + m


def _p_accept(w, mu, sigma, low, high):
    """Truncation mass of the mixture (tpe.py:145-150, 277-282)."""
    if low is None and high is None:
        return 1
    return np.sum(w * (normal_cdf(high, mu, sigma) - normal_cdf(low, mu, sigma)))


def _check_params(w, mu, sigma):
    w, mu, sigma = (np.asarray(a, dtype=np.float64) for a in (w, mu, sigma))
    for name, a in (("weights", w), ("mus", mu), ("sigmas", sigma)):
        if a.ndim != 1:
            raise TypeError("need vector of %s" % name, a.shape)
    if not (len(w) == len(mu) == len(sigma)):
        raise AssertionError("mixture arrays differ in length")
    return w, mu, sigma


def gmm1_lpdf(samples, w, mu, sigma, low=None, high=None, q=None, chunk=1 << 12):
    """Truncated / quantized Gaussian-mixture log density (tpe.py:117-180).

    Unquantized: LSE over components of -0.5*mahal + log(w/Z/p_accept).
    Quantized: log of the linear-space sum of w*(Phi(ub)-Phi(lb)), summed
    component by component in component order, minus log(p_accept).
    Evaluated in row chunks (row results are independent of chunking).
    """
    x_in = np.asarray(samples, dtype=np.float64)
    if x_in.size == 0:
        return np.zeros(0)
    w, mu, sigma = _check_params(w, mu, sigma)
    x = x_in.ravel()
    p_acc = _p_accept(w, mu, sigma, low, high)
    out = np.empty(x.size)
    if q is None:
        coef = np.log(w / np.sqrt(2 * np.pi * sigma ** 2) / p_acc)
        inv = np.maximum(sigma, EPS)
        for s in range(0, x.size, chunk):
            xs = x[s:s + chunk, None]
            out[s:s + chunk] = _lse_rows(-0.5 * ((xs - mu) / inv) ** 2 + coef)
    else:
        for s in range(0, x.size, chunk):
            xs = x[s:s + chunk, None]
            ub = xs + q / 2.0 if high is None else np.minimum(xs + q / 2.0, high)
            lb = xs - q / 2.0 if low is None else np.maximum(xs - q / 2.0, low)
            inc = w * normal_cdf(ub, mu, sigma) - w * normal_cdf(lb, mu, sigma)
            # sequential left-to-right accumulation == `prob += inc` per component
            prob = np.cumsum(inc, axis=1)[:, -1]
            with np.errstate(divide="ignore"):
                out[s:s + chunk] = np.log(prob) - np.log(p_acc)
    return out.reshape(x_in.shape)


def lgmm1_lpdf(samples, w, mu, sigma, low=None, high=None, q=None, chunk=1 << 12):
    """Log-normal mixture log density (tpe.py:265-307).

    Unquantized branch ignores p_accept (reference quirk, tpe.py:284-287).
    ``low``/``high`` are log-space bounds; quantized bounds use exp(low/high)
    and clamp the lower bound at 0 (tpe.py:292-300).
    """
    x_in = np.asarray(samples, dtype=np.float64)
    w, mu, sigma = _check_params(w, mu, sigma)
    x = x_in.ravel()
    if x.size == 0:
        return x_in.astype(np.float64)
    p_acc = _p_accept(w, mu, sigma, low, high)
    out = np.empty(x.size)
    if q is None:
        logw = np.log(w)
        for s in range(0, x.size, chunk):
            xs = x[s:s + chunk, None]
            with np.errstate(divide="ignore", invalid="ignore"):
                out[s:s + chunk] = _lse_rows(lognormal_lpdf(xs, mu, sigma) + logw)
    else:
        for s in range(0, x.size, chunk):
            xs = x[s:s + chunk, None]
            ub = xs + q / 2.0 if high is None else np.minimum(xs + q / 2.0, np.exp(high))
            lb = xs - q / 2.0 if low is None else np.maximum(xs - q / 2.0, np.exp(low))
            lb = np.maximum(0, lb)
            inc = w * lognormal_cdf(ub, mu, sigma) - w * lognormal_cdf(lb, mu, sigma)
            prob = np.cumsum(inc, axis=1)[:, -1]
            with np.errstate(divide="ignore"):
                out[s:s + chunk] = np.log(prob) - np.log(p_acc)
    return out.reshape(x_in.shape)


def categorical_lpdf(sample, p):
    """log(p[sample]) (tpe.py:60-73)."""
    sample = np.asarray(sample)
    if sample.size == 0:
        return np.zeros(0)
    return np.log(np.asarray(p)[sample])


def broadcast_best_index(below_llik, above_llik):
    """np.argmax(below - above): first max, NaN counts as max (tpe.py:649-658)."""
    return int(np.argmax(np.asarray(below_llik) - np.asarray(above_llik)))


# ---------------------------------------------------------------------------
# Categorical posteriors
# ---------------------------------------------------------------------------
def randint_posterior(obs, prior_weight, low, high=None, lf=DEFAULT_LF):
    """Pseudocount posterior for randint (tpe.py:578-593, pyll/base.py:1053-1060).

    np.bincount accumulates the ramp weights sequentially in observation order.
    """
    obs = np.asarray(obs)
    size = low if high is None else high - low
    offset = 0 if high is None else low
    wts = linear_forgetting_weights(len(obs), lf)
    counts = np.bincount(np.asarray(obs, dtype=int) - offset, wts if len(obs) else None,
                         size)
    pseudo = counts + prior_weight
    return pseudo / np.sum(pseudo)


def categorical_posterior(obs, prior_weight, p, lf=DEFAULT_LF):
    """Pseudocount posterior for pchoice/categorical (tpe.py:596-615)."""
    obs = np.asarray(obs)
    p = np.asarray(p, dtype=np.float64)
    if p.ndim == 2:
        p = p[0]
    wts = linear_forgetting_weights(len(obs), lf)
    counts = np.bincount(np.asarray(obs, dtype=int), wts if len(obs) else None, len(p))
    pseudo = counts + p.size * (prior_weight * p)
    return pseudo / np.sum(pseudo)


# ---------------------------------------------------------------------------
# Per-distribution posterior construction (tpe.py:484-572)
# ---------------------------------------------------------------------------
CONTINUOUS = ("uniform", "quniform", "loguniform", "qloguniform",
              "normal", "qnormal", "lognormal", "qlognormal")


def posterior_spec(kind, args):
    """Return (family, prior_mu, prior_sigma, obs_transform, low, high, q).

    family is "GMM1" or "LGMM1"; obs_transform maps raw observations to the
    space the Parzen fit runs in; low/high are the bounds passed to the lpdf.
    """
    if kind in ("uniform", "quniform", "loguniform", "qloguniform"):
        low, high = float(args[0]), float(args[1])
        q = float(args[2]) if kind.startswith("q") else None
        pmu, psig = 0.5 * (high + low), 1.0 * (high - low)
        if kind == "uniform" or kind == "quniform":
            return "GMM1", pmu, psig, (lambda o: o), low, high, q
        if kind == "loguniform":
            return "LGMM1", pmu, psig, np.log, low, high, None
        floor = max(EPS, math.exp(low))
        return "LGMM1", pmu, psig, (lambda o: np.log(np.maximum(o, floor))), low, high, q
    if kind in ("normal", "qnormal", "lognormal", "qlognormal"):
        mu, sigma = float(args[0]), float(args[1])
        q = float(args[2]) if kind.startswith("q") else None
        if kind in ("normal", "qnormal"):
            return "GMM1", mu, sigma, (lambda o: o), None, None, q
        if kind == "lognormal":
            return "LGMM1", mu, sigma, np.log, None, None, None
        return "LGMM1", mu, sigma, (lambda o: np.log(np.maximum(o, EPS))), None, None, q
    raise ValueError(kind)


def continuous_label_scores(kind, args, obs_below, obs_above, candidates,
                            prior_weight=1.0, lf=DEFAULT_LF, sort_kind="stable"):
    """Full per-label pipeline on injected candidates (tpe.py:697-746).

    Returns dict with the two posteriors, both log-likelihood vectors, the
    argmax index and the chosen value.
    """
    family, pmu, psig, tf, low, high, q = posterior_spec(kind, args)
    ob = tf(np.asarray(obs_below, dtype=np.float64))
    oa = tf(np.asarray(obs_above, dtype=np.float64))
    b = adaptive_parzen_normal(ob, prior_weight, pmu, psig, lf, sort_kind)
    a = adaptive_parzen_normal(oa, prior_weight, pmu, psig, lf, sort_kind)
    f = gmm1_lpdf if family == "GMM1" else lgmm1_lpdf
    cand = np.asarray(candidates, dtype=np.float64)
    bl = f(cand, *b, low=low, high=high, q=q)
    al = f(cand, *a, low=low, high=high, q=q)
    out = dict(below=b, above=a, below_llik=bl, above_llik=al)
    if cand.size:
        best = broadcast_best_index(bl, al)
        out.update(best=best, value=float(cand[best]))
    return out


def categorical_label_scores(kind, args, obs_below, obs_above, candidates,
                             prior_weight=1.0, lf=DEFAULT_LF):
    """randint / categorical pipeline on injected candidate indices."""
    if kind == "randint":
        low = int(args[0])
        high = int(args[1]) if len(args) > 1 and args[1] is not None else None
        pb = randint_posterior(obs_below, prior_weight, low, high, lf)
        pa = randint_posterior(obs_above, prior_weight, low, high, lf)
    elif kind == "categorical":
        pb = categorical_posterior(obs_below, prior_weight, args[0], lf)
        pa = categorical_posterior(obs_above, prior_weight, args[0], lf)
    else:
        raise ValueError(kind)
    cand = np.asarray(candidates, dtype=int)
    bl = categorical_lpdf(cand, pb)
    al = categorical_lpdf(cand, pa)
    out = dict(p_below=pb, p_above=pa, below_llik=bl, above_llik=al)
    if cand.size:
        best = broadcast_best_index(bl, al)
        out.update(best=best, value=int(cand[best]))
    return out


# ---------------------------------------------------------------------------
# Samplers (reference distributions for KS tests; RNG streams cannot match)
# ---------------------------------------------------------------------------
def gmm1_sample(w, mu, sigma, low=None, high=None, q=None, rng=None, size=1):
    """Rejection sampler with the reference's accepted distribution (tpe.py:79-106)."""
    rng = np.random.RandomState(0) if rng is None else rng
    w, mu, sigma = (np.asarray(a, dtype=np.float64) for a in (w, mu, sigma))
    n = int(size)
    if low is None and high is None:
        j = rng.choice(len(w), size=n, p=w / w.sum())
        x = rng.normal(mu[j], sigma[j])
    else:
        lo = -np.inf if low is None else float(low)
        hi = np.inf if high is None else float(high)
        if lo >= hi:
            raise ValueError("low >= high", (lo, hi))
        parts, got = [], 0
        while got < n:
            m = max(2 * (n - got), 64)
            j = rng.choice(len(w), size=m, p=w / w.sum())
            d = rng.normal(mu[j], sigma[j])
            d = d[(lo <= d) & (d < hi)]
            parts.append(d)
            got += d.size
        x = np.concatenate(parts)[:n]
    if q is not None:
        x = np.round(x / q) * q
    return x


def lgmm1_sample(w, mu, sigma, low=None, high=None, q=None, rng=None, size=1):
    """Log-domain variant (tpe.py:229-257)."""
    x = np.exp(gmm1_sample(w, mu, sigma, low, high, None, rng, size))
    if q is not None:
        x = np.round(x / q) * q
    return x


def truncated_mixture_cdf(x, w, mu, sigma, low=None, high=None):
    """Exact CDF of the accepted distribution of the rejection sampler."""
    x = np.asarray(x, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64)
    w = w / w.sum()
    lo = -np.inf if low is None else low
    hi = np.inf if high is None else high

    def phi(v):
        return 0.5 * (1 + erf((v - mu) / (SQRT2 * sigma)))

    xc = np.clip(x, lo, hi)[:, None]
    num = np.sum(w * (phi(xc) - phi(lo)), axis=1)
    den = np.sum(w * (phi(hi) - phi(lo)))
    return num / den


# ---------------------------------------------------------------------------
# CPU baseline scorer (the bench's cpu_baseline leg): chunked dense scoring
# ---------------------------------------------------------------------------
def score_label_dense(family, below, above, candidates, low=None, high=None, q=None,
                      chunk=1 << 12):
    """below_llik - above_llik and the argmax, for candidates in row chunks."""
    f = gmm1_lpdf if family == "GMM1" else lgmm1_lpdf
    bl = f(candidates, *below, low=low, high=high, q=q, chunk=chunk)
    al = f(candidates, *above, low=low, high=high, q=q, chunk=chunk)
    s = bl - al
    return s, int(np.argmax(s))
