"""Explicit 1-D mixtures on the GPU: drop-ins for the reference's GMM1,
GMM1_lpdf, LGMM1 and LGMM1_lpdf (hyperopt/tpe.py:79-106, 117-180, 229-257,
265-307), with the reference's names, argument meaning and error behaviour.

These are the same kernels the suggest path runs on fitted Parzen mixtures
(tpe_sample, tpe_score_continuous, tpe_score_quantized); here the mixture is
the caller's (tpe_mixture_prepare: weights normalised, p_accept, cumulative
weights and coefficients computed exactly as for a fitted one, sigmas kept as
given).  Inputs and outputs are host numpy arrays, as in the reference; the
work runs on the current CUDA (HIP) device and there is no CPU fallback.

Differences from the reference, all deliberate:
* draws come from the library's counter-based Philox streams, keyed by one
  63-bit draw from ``rng`` -- the same distribution, not numpy's sequence;
* ``precision=32`` draws / scores in fp32 (the suggest path's fast mode);
  quantized log-masses (q given) are always computed in fp64;
* components are re-ordered by mean (a mixture is order-free).

The reference's normalisation quirks are reproduced: the weights are not
normalised (log(sum w) enters the result) where the reference never divides
by p_accept -- GMM1_lpdf / quantized LGMM1_lpdf without bounds, and
unquantized LGMM1_lpdf always (tpe.py:284-287 ignores p_accept).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L

_P = ctypes.c_void_p


def _torch_device():
    import torch
    if not torch.cuda.is_available():
        raise L.TpeHipError("hyperopt_amd.mixture: no GPU visible; there is no CPU fallback")
    return torch, torch.device("cuda", torch.cuda.current_device())


class _Mixture:
    """One explicit mixture, prepared on the device (tpe_mixture_prepare)."""

    def __init__(self, family, weights, mus, sigmas, low, high):
        w, mu, s = (np.asarray(a, dtype=np.float64) for a in (weights, mus, sigmas))
        if w.ndim != 1:
            raise TypeError("need vector of weights", w.shape)
        if mu.ndim != 1:
            raise TypeError("need vector of mus", mu.shape)
        if s.ndim != 1:
            raise TypeError("need vector of sigmas", s.shape)
        if not (len(w) == len(mu) == len(s)):
            raise AssertionError("len(weights) == len(mus) == len(sigmas)")
        if len(w) == 0:
            raise ValueError("empty mixture")
        order = np.argsort(mu, kind="stable")
        w, mu, s = w[order], mu[order], s[order]
        self.family, self.K = family, len(w)
        self.wsum = float(np.sum(w))
        torch, dev = _torch_device()
        self.torch, self.dev = torch, dev
        lib = self.lib = L.load()
        seg = np.zeros(1, L.SEG_DTYPE)
        pos = int(np.argmax(s))
        seg["n_obs"] = self.K - 1
        seg["family"] = family
        seg["prior_pos"] = pos
        seg["prior_weight"] = w[pos]
        seg["prior_mu"] = mu[pos]  # the fp32 coefficients' origin
        seg["prior_sigma"] = s[pos]
        if low is not None and high is not None:
            seg["bounded"] = 1
            seg["low"], seg["high"] = low, high
        seg["given"] = 1
        f64 = dict(dtype=torch.float64, device=dev)
        self.d_seg = torch.from_numpy(seg.view(np.uint8).copy()).to(dev)
        self.d_w = torch.from_numpy(w.copy()).to(dev)
        self.d_mu = torch.from_numpy(mu.copy()).to(dev)
        self.d_sigma = torch.from_numpy(s.copy()).to(dev)
        self.d_cdf = torch.empty(self.K, **f64)
        self.d_c64 = torch.empty(4 * self.K, **f64)
        self.d_c32 = torch.empty(4 * self.K, dtype=torch.float32, device=dev)
        nscr = lib.tpe_mixture_scratch_bytes(1, self.K)
        scratch = torch.empty(max(int(nscr), 8), dtype=torch.uint8, device=dev)
        self.stream = torch.cuda.current_stream(dev)
        L.check(lib.tpe_mixture_prepare(
            _P(self.d_seg.data_ptr()), 1, self.K, _P(scratch.data_ptr()), _P(self.d_w.data_ptr()),
            _P(self.d_mu.data_ptr()), _P(self.d_sigma.data_ptr()), _P(self.d_cdf.data_ptr()),
            _P(self.d_c64.data_ptr()), _P(self.d_c32.data_ptr()), _P(self.stream.cuda_stream)),
            "tpe_mixture_prepare")
        self._scratch = scratch  # kept alive until the stream has used it

    def ptrs(self):
        return [_P(t.data_ptr()) for t in (self.d_w, self.d_mu, self.d_sigma, self.d_cdf,
                                           self.d_c64, self.d_c32)]

    def job(self, n, flags, low, high, q, key=0):
        job = np.zeros(1, L.JOB_DTYPE)
        job["family"], job["flags"], job["n_cand"] = self.family, flags, n
        job["below"] = job["above"] = 0
        job["low"] = low if low is not None else 0.0
        job["high"] = high if high is not None else 0.0
        job["q"] = q if q is not None else 0.0
        job["key"] = key
        return job

    def upload(self, arr):
        return self.torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy()).to(self.dev)

    def sample(self, n, flags, low, high, q, key, precision):
        job = self.job(n, flags, low, high, q, key)
        d_job = self.upload(job)
        out = self.torch.empty(max(n, 1), dtype=self.torch.float64, device=self.dev)
        w, mu, s, cdf, _, _ = self.ptrs()
        L.check(self.lib.tpe_sample(_P(d_job.data_ptr()), job.ctypes.data_as(_P), 1,
                                    _P(self.d_seg.data_ptr()), mu, s, cdf, precision,
                                    _P(out.data_ptr()), _P(self.stream.cuda_stream)),
                "tpe_sample")
        return out[:n].cpu().numpy()

    def lpdf(self, x, flags, low, high, q, precision, windows=True):
        """Per-value log-density (unquantized) or log-mass (quantized) of the
        normalised-weight mixture, truncation-normalised as the kernels do.
        windows (quantized): each value sums only its window of unsaturated
        components (tpe_score_quantized's reach arrays; the same bits)."""
        torch, lib = self.torch, self.lib
        n = x.size
        job = self.job(n, flags | L.F_INJECTED, low, high, q)
        d_job = self.upload(job)
        d_x = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).to(self.dev)
        out_bl = torch.empty(n, dtype=torch.float64, device=self.dev)
        best = torch.empty(L.BEST_DTYPE.itemsize, dtype=torch.uint8, device=self.dev)
        w, mu, s, cdf, c64, c32 = self.ptrs()
        hj, sp = job.ctypes.data_as(_P), _P(self.stream.cuda_stream)
        if flags & L.F_QUANT:
            npart = int(lib.tpe_quantized_partials(hj, 1, n))
            partial = torch.empty(max(npart, 1) * L.BEST_DTYPE.itemsize, dtype=torch.uint8,
                                  device=self.dev)
            err = torch.zeros(1, dtype=torch.int32, device=self.dev)
            reach = torch.empty(2 * self.K if windows else 1, dtype=torch.float64, device=self.dev)
            rh = _P(reach.data_ptr()) if windows else None
            rl = _P(reach.data_ptr() + 8 * self.K) if windows else None
            L.check(lib.tpe_score_quantized(
                _P(d_job.data_ptr()), hj, 1, _P(self.d_seg.data_ptr()), w, mu, s,
                _P(d_x.data_ptr()), None, None, n, _P(out_bl.data_ptr()), None,
                _P(partial.data_ptr()), npart, _P(best.data_ptr()), _P(err.data_ptr()), rh,
                rl, sp),
                "tpe_score_quantized")
            if int(err.item()):
                raise ValueError("negative arg to lognormal_cdf", x)  # tpe.py:196-197
        else:
            npart = int(lib.tpe_score_partials(hj, 1))
            partial = torch.empty(max(npart, 1) * L.BEST_DTYPE.itemsize, dtype=torch.uint8,
                                  device=self.dev)
            L.check(lib.tpe_score_continuous(
                _P(d_job.data_ptr()), hj, 1, _P(self.d_seg.data_ptr()), w, mu, s, cdf, c64, c32,
                _P(d_x.data_ptr()), precision, _P(out_bl.data_ptr()), None, None,
                _P(partial.data_ptr()), npart, _P(best.data_ptr()), sp),
                "tpe_score_continuous")
        return out_bl.cpu().numpy()


def _key(rng):
    if rng is None:
        rng = np.random
    return int(rng.randint(0, 2 ** 62)) * 2 + int(rng.randint(0, 2))


def _check_precision(precision):
    if precision not in (32, 64):
        raise ValueError("precision must be 32 or 64", precision)


def GMM1(weights, mus, sigmas, low=None, high=None, q=None, rng=None, size=(), precision=64):
    """Sample from a (truncated) 1-D Gaussian mixture -- tpe.py:79-106.
    Truncation keeps draws with low <= draw < high (one-sided allowed);
    q rounds as np.round(x / q) * q."""
    _check_precision(precision)
    n = int(np.prod(size))
    flags = 0
    lo = hi = None
    if not (low is None and high is None):
        lo = float(low) if low is not None else -float("inf")
        hi = float(high) if high is not None else float("inf")
        if lo >= hi:
            raise ValueError("low >= high", (lo, hi))
        flags |= (L.F_LOW if low is not None else 0) | (L.F_HIGH if high is not None else 0)
    if q is not None:
        flags |= L.F_QUANT
    key = _key(rng)
    if n == 0:
        return np.reshape(np.zeros(0), size)
    m = _Mixture(L.GMM1, weights, mus, sigmas, None, None)
    x = m.sample(n, flags, lo, hi, q, key, precision)
    return np.reshape(x, size)


def LGMM1(weights, mus, sigmas, low=None, high=None, q=None, rng=None, size=(), precision=64):
    """Sample from a (truncated) 1-D log-normal mixture -- tpe.py:229-257.
    Bounds are in log space and both are required when one is given (the
    reference's float(None) fails the same way)."""
    _check_precision(precision)
    n = int(np.prod(size))
    flags = 0
    lo = hi = None
    if not (low is None and high is None):
        lo, hi = float(low), float(high)
        if lo >= hi:
            raise ValueError("low >= high", (lo, hi))
        flags |= L.F_LOW | L.F_HIGH
    if q is not None:
        flags |= L.F_QUANT
    key = _key(rng)
    if n == 0:
        return np.reshape(np.zeros(0), size)
    m = _Mixture(L.LGMM1, weights, mus, sigmas, None, None)
    x = m.sample(n, flags, lo, hi, q, key, precision)
    return np.reshape(x, size)


def _lpdf(family, samples, weights, mus, sigmas, low, high, q, precision):
    _check_precision(precision)
    samples = np.asarray(samples, dtype=np.float64)
    bounded = not (low is None and high is None)
    if bounded and (low is None or high is None):
        # the reference evaluates normal_cdf(None, ...) here and fails
        raise TypeError("one-sided bounds are not supported by the lpdf (tpe.py:148-150)")
    m = _Mixture(family, weights, mus, sigmas, low if bounded else None,
                 high if bounded else None)
    flags = (L.F_LOW | L.F_HIGH) if bounded else 0
    if q is not None:
        flags |= L.F_QUANT
    x = samples.reshape(-1)
    r = m.lpdf(x, flags, low, high, q, precision)
    # our mixture has normalised weights; the reference divides by p_accept
    # (which carries the same sum) only where it truncates -- elsewhere its
    # raw weights' log-sum shows up in the result
    if not bounded or (family == L.LGMM1 and q is None):
        r = r + np.log(m.wsum)
    return r.reshape(samples.shape)


def GMM1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None, precision=64):
    """Log-density (q None) or log-mass of the q-rounded value (q given) of a
    truncated Gaussian mixture -- tpe.py:117-180."""
    samples = np.asarray(samples)
    if samples.size == 0:
        return np.asarray([])
    return _lpdf(L.GMM1, samples, weights, mus, sigmas, low, high, q, precision)


def LGMM1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None, precision=64):
    """Log-density (q None) or log-mass (q given) of a log-normal mixture --
    tpe.py:265-307 (bounds in log space; unquantized ignores p_accept)."""
    samples = np.asarray(samples)
    if samples.size == 0:
        return np.zeros(samples.shape)
    return _lpdf(L.LGMM1, samples, weights, mus, sigmas, low, high, q, precision)
