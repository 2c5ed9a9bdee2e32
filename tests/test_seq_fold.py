"""The categorical counts' wave-parallel sequential fp64 sum (seq_fold in
hyperopt_amd/csrc/tpe_fit.hip), restated on the host with Python integers:
it must give the bits of the serial left fold fl(..fl(fl(S + w0) + w1)..)
-- np.bincount's accumulation order (pyll/base.py:1053-1060) -- on LF ramps,
tie-heavy dyadic weights, 24-decade ranges and sums started near 2^53.
Lanes are modelled as consecutive runs of kSE entries (the kernel's layout);
the scans are written sequentially (their results do not depend on how a
scan is evaluated)."""
import math

import numpy as np

KSE, LANES = 8, 64


def _split(x):
    """x >= 0 -> (M, biased exponent) with x = M * 2^(max(eb, 1) - 1075)."""
    b = int(np.float64(x).view(np.uint64))
    eb = (b >> 52) & 0x7FF
    M = (b & ((1 << 52) - 1)) | ((1 << 52) if eb else 0)
    return M, eb


def seq_fold(S, w):
    """The kernel's passes over one list (len(w) <= KSE * LANES)."""
    n, r0, passes = len(w), 0, 0
    while r0 < n:
        passes += 1
        A, es = _split(S)
        if S == 0.0 or es == 0:
            S = float(np.float64(S) + np.float64(w[r0]))
            r0 += 1
            continue
        d, tie, huge = [0] * n, [False] * n, [False] * n
        for i in range(r0, n):
            M, ew = _split(w[i])
            sh = es - max(ew, 1)
            if sh < 0:
                huge[i] = True
            elif sh == 0:
                d[i] = M
            elif sh < 64:
                rem, half = M & ((1 << sh) - 1), 1 << (sh - 1)
                d[i] = (M >> sh) + (rem > half)
                tie[i] = rem == half
        P = A & 1  # (the composed parity maps, evaluated in order)
        for i in range(r0, n):
            if tie[i]:
                d[i] += (P + d[i]) & 1
                P = 0
            else:
                P ^= d[i] & 1
        D, cross = 0, None
        for i in range(r0, n):
            if huge[i] or A + D + d[i] >= 1 << 53:
                cross = i
                break
            D += d[i]
        if cross is None:
            S, r0 = math.ldexp(float(A + D), es - 1075), n
        else:
            S = float(np.float64(math.ldexp(float(A + D), es - 1075)) + np.float64(w[cross]))
            r0 = cross + 1
    return S, passes


def _serial(S, w):
    s = np.float64(S)
    for x in w:
        s = s + np.float64(x)
    return float(s)


def _fold_all(S, w):
    cap = KSE * LANES
    for f0 in range(0, len(w), cap):
        S, _ = seq_fold(S, w[f0:f0 + cap])
    return S


def test_lf_ramp_counts_match_the_serial_chain():
    rng = np.random.RandomState(3)
    for N in (30, 1000, 20000):
        lf = 25
        num = N - lf
        step = (1.0 - 1.0 / N) / (num - 1)
        for p in (0.05, 0.5, 0.9):
            idx = np.flatnonzero(rng.uniform(size=N) < p)
            w = np.where(idx < num - 1, idx * step + 1.0 / N, 1.0).tolist()
            assert _fold_all(0.0, w) == _serial(0.0, w), (N, p)


def test_tie_heavy_and_wide_ranges_match_the_serial_chain():
    rng = np.random.RandomState(4)
    starts = [0.0, 1.0, 2.0 ** 53, 2.0 ** 53 + 2, 2.0 ** 52 + 1, 3 * 2.0 ** 51 + 1, 1e16, 1e-300]
    for trial in range(400):
        n = int(rng.randint(1, 1500))
        kind = trial % 3
        if kind == 0:
            w = [float(rng.choice([1.0, 3.0, 0.5, 2.0, 1.5, 5.0, 2.0 ** -60, 7.0, 0.0]))
                 for _ in range(n)]
        elif kind == 1:
            w = [float(2.0 ** rng.randint(-6, 3)) * int(rng.randint(1, 4)) for _ in range(n)]
        else:
            w = [float(10.0 ** rng.uniform(-12, 12)) for _ in range(n)]
        S0 = float(starts[trial % len(starts)])
        assert _fold_all(S0, w) == _serial(S0, w), (trial, kind, n, S0)


def test_passes_stay_few_on_a_long_chain():
    """60 000 ramp weights (a C5 root category): one pass per list plus one
    per binade crossed."""
    rng = np.random.RandomState(5)
    N = 100000
    step = (1.0 - 1.0 / N) / (N - 25 - 1)
    idx = np.sort(rng.choice(N, size=60000, replace=False))
    w = np.where(idx < N - 26, idx * step + 1.0 / N, 1.0).tolist()
    S, total = 0.0, 0
    cap = KSE * LANES
    for f0 in range(0, len(w), cap):
        S, p = seq_fold(S, w[f0:f0 + cap])
        total += p
    assert S == _serial(0.0, w)
    assert total < len(w) / cap + 64
