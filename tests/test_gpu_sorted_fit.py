"""The Parzen fit from the history's sorted orders (tpe_history_order +
tpe_fit_sorted) against the gather + sort fit (tpe_gather_obs +
tpe_parzen_fit) and the oracle.

Both fits must give the same bits: adaptive_parzen_normal's means and
bandwidths (tpe.py:399-467) are copies and differences of the sorted
observations, and the sorted fit folds its sums in the multi-kernel fit's
order.  Covered: ties (quantized values, stable tid order), values clamped
by a log prior's floor (qloguniform, tpe.py:527-532), inactive rows, the
len 0 / 1 / 2 rules (tpe.py:410-421), histories grown by appends of 1 row
to several 2048-row chunks (the order is merged, not rebuilt), a column
re-used under another transform (rebuilt), and whole levels' winners.
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

SPACE = [("u", "uniform", (-5.0, 5.0)), ("lu", "loguniform", (-5.0, 0.0)),
         ("q", "quniform", (0.0, 20.0, 1.0)), ("n", "normal", (0.0, 2.0)),
         ("ql", "qloguniform", (0.0, 3.0, 1.0)), ("qn", "qnormal", (0.0, 3.0, 0.5)),
         ("ln", "lognormal", (0.0, 1.0)), ("c", "randint", (6,))]


def _cols(T, rng):
    return np.stack([rng.uniform(-5, 5, T), np.exp(rng.uniform(-5, 0, T)),
                     np.round(rng.uniform(0, 20, T)), rng.normal(0, 2, T),
                     # below exp(low) = 1 for a third of the rows: clamped, tied
                     np.round(np.exp(rng.uniform(-1.5, 3, T))),
                     np.round(rng.normal(0, 3, T) / 0.5) * 0.5, np.exp(rng.normal(0, 1, T)),
                     rng.randint(0, 6, T).astype(float)], axis=1)


def _engines():
    from hyperopt_amd.engine import Engine
    a, b = Engine(), Engine()
    a.sorted_fit, b.sorted_fit = True, False
    return a, b


def _level(hist, mat, active, losses, T, n_cand=1 << 16):
    from hyperopt_amd.engine import LabelWork
    n_below = min(int(np.ceil(0.25 * np.sqrt(T))), 25)
    isb = np.zeros(T, np.uint8)
    isb[np.argsort(losses[:T], kind="stable")[:n_below]] = 1
    works = []
    for j, (lab, kind, a) in enumerate(SPACE):
        act = active[:T, j]
        works.append(LabelWork(lab, kind, a, mat[:T, j][act & (isb == 1)], None,
                               n_cand=n_cand, key=991 + j, col=j,
                               n_above=int((act & (isb == 0)).sum())))
    return works, isb


def _same_posteriors(a, b):
    for ra, rb in zip(a, b):
        assert set(ra.extra) == set(rb.extra)
        for k in ra.extra:
            for x, y in zip(np.atleast_1d(ra.extra[k]), np.atleast_1d(rb.extra[k])):
                np.testing.assert_array_equal(x, y, err_msg="%s %s" % (ra.label, k))


@pytest.mark.parametrize("T,inactive", [(1, 0.0), (2, 0.0), (9, 0.3), (700, 0.1),
                                        (5000, 0.0), (12000, 0.2)])
def test_sorted_fit_equals_sort_fit(T, inactive):
    from hyperopt_amd.engine import DeviceHistory
    rng = np.random.RandomState(T)
    mat = _cols(T, rng)
    active = rng.uniform(size=mat.shape) >= inactive
    losses = rng.normal(size=T)
    srt, ref = _engines()
    hs, hr = DeviceHistory(srt, len(SPACE), cap=32), DeviceHistory(ref, len(SPACE), cap=32)
    for h in (hs, hr):
        h.append(mat, active)
    works, isb = _level(hs, mat, active, losses, T)
    _same_posteriors(srt.run(works, posteriors=True, history=hs, is_below=isb),
                     ref.run(works, posteriors=True, history=hr, is_below=isb))
    assert hs.order_rows and all(v == T for v in hs.order_rows.values())
    # and every label's winner of the whole level, both precisions
    for precision in (64, 32):
        a = srt.run(works, precision=precision, history=hs, is_below=isb)
        b = ref.run(works, precision=precision, history=hr, is_below=isb)
        assert [(r.index, r.value, r.score) for r in a] == \
               [(r.index, r.value, r.score) for r in b]


@pytest.mark.parametrize("T", [9, 5000, 12000])
def test_long_column_path_gives_the_same_bits(T, monkeypatch):
    """Columns of more than 4096 chunks globalise the chunk-local ranks in a
    launch of their own (k_fit_globalize) instead of adding the chunk bases
    from LDS; TPE_FIT_GLOBALIZE=1 takes that path at these sizes -- the same
    posteriors and winners as the default path."""
    from hyperopt_amd.engine import DeviceHistory, Engine
    rng = np.random.RandomState(T + 1)
    mat = _cols(T, rng)
    active = rng.uniform(size=mat.shape) >= 0.1
    losses = rng.normal(size=T)
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv("TPE_FIT_GLOBALIZE", env)
        eng = Engine()
        eng.sorted_fit = True
        h = DeviceHistory(eng, len(SPACE), cap=32)
        h.append(mat, active)
        works, isb = _level(h, mat, active, losses, T)
        post = eng.run(works, posteriors=True, history=h, is_below=isb)
        win = eng.run(works, precision=32, history=h, is_below=isb)
        out.append((post, [(r.index, r.value, r.score) for r in win]))
    _same_posteriors(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def test_sorted_fit_through_appends():
    """The order merged in after every append -- 1, 7, 2048, 2049, 3000 rows
    (one and several tpe_history_order chunks) -- gives the sort fit's bits
    at every size, and the oracle's posterior."""
    from hyperopt_amd.engine import DeviceHistory
    rng = np.random.RandomState(3)
    total = 1 + 7 + 2048 + 2049 + 3000 + 5
    mat = _cols(total, rng)
    active = rng.uniform(size=mat.shape) >= 0.15
    losses = rng.normal(size=total)
    srt, ref = _engines()
    hs, hr = DeviceHistory(srt, len(SPACE), cap=16), DeviceHistory(ref, len(SPACE), cap=16)
    T = 0
    for k in (5, 1, 7, 2048, 2049, 3000):
        for h in (hs, hr):
            h.append(mat[T:T + k], active[T:T + k])
        T += k
        works, isb = _level(hs, mat, active, losses, T)
        _same_posteriors(srt.run(works, posteriors=True, history=hs, is_below=isb),
                         ref.run(works, posteriors=True, history=hr, is_below=isb))
    # the qloguniform column against the oracle (clamped ties included)
    j = 4
    res = srt.run(works, posteriors=True, history=hs, is_below=isb)
    act = active[:T, j]
    below, above = O.ap_split_trials(np.flatnonzero(act), mat[:T][act, j], np.arange(T),
                                     losses[:T], 0.25)
    fam, pmu, psig, tf, low, high, q = O.posterior_spec("qloguniform", SPACE[j][2])
    for half, obs in (("below", below), ("above", above)):
        ow, omu, osig = O.adaptive_parzen_normal(tf(obs), 1.0, pmu, psig)
        gw, gmu, gsig = res[j].extra[half]
        np.testing.assert_allclose(gmu, omu, rtol=4.5e-16, atol=0)
        np.testing.assert_allclose(gsig, osig, rtol=1e-12, atol=0)
        np.testing.assert_allclose(gw, ow, rtol=1e-12, atol=0)


def test_column_under_another_transform_is_rebuilt():
    """The same history column fitted as uniform, then as loguniform (log of
    the values, another order near the floor): the order is rebuilt for the
    new transform."""
    from hyperopt_amd.engine import DeviceHistory, LabelWork
    rng = np.random.RandomState(8)
    T = 3000
    v = np.exp(rng.uniform(-5, 0, T))
    losses = rng.normal(size=T)
    srt, ref = _engines()
    hs, hr = DeviceHistory(srt, 1), DeviceHistory(ref, 1)
    for h in (hs, hr):
        h.append(v[:, None])
    n_below = min(int(np.ceil(0.25 * np.sqrt(T))), 25)
    isb = np.zeros(T, np.uint8)
    isb[np.argsort(losses, kind="stable")[:n_below]] = 1
    for kind, a in (("uniform", (0.0, 1.0)), ("qloguniform", (-2.0, 0.0, 0.01)),
                    ("loguniform", (-5.0, 0.0))):
        w = LabelWork("x", kind, a, v[isb == 1], None, n_cand=256, key=5, col=0,
                      n_above=T - n_below)
        _same_posteriors(srt.run([w], posteriors=True, history=hs, is_below=isb),
                         ref.run([w], posteriors=True, history=hr, is_below=isb))


def test_alternating_column_sets_then_append():
    """Levels over different column sets at one row count (X, Y, X -- a
    nested space's branches, or suggest_many requests on one Trials), then an
    append, then Y: the merge must bring Y's own columns up to the new rows
    (the cached spec list once belonged to X)."""
    from hyperopt_amd.engine import DeviceHistory
    rng = np.random.RandomState(12)
    total = 900 + 300
    mat = _cols(total, rng)
    active = rng.uniform(size=mat.shape) >= 0.1
    losses = rng.normal(size=total)
    srt, ref = _engines()
    hs, hr = DeviceHistory(srt, len(SPACE), cap=16), DeviceHistory(ref, len(SPACE), cap=16)
    X, Y = [0, 1, 2], [3, 4, 5, 6]
    T = 0
    for k, seq in ((900, (X, Y, X, Y, X)), (300, (Y, X, Y))):
        for h in (hs, hr):
            h.append(mat[T:T + k], active[T:T + k])
        T += k
        works, isb = _level(hs, mat, active, losses, T)
        for cols in seq:
            sub = [works[j] for j in cols]
            _same_posteriors(srt.run(sub, posteriors=True, history=hs, is_below=isb),
                             ref.run(sub, posteriors=True, history=hr, is_below=isb))
    assert all(hs.order_rows[c] == T for c in X + Y)


def test_sorted_fit_count_mismatch_raises():
    from hyperopt_amd import _lib as L
    from hyperopt_amd.engine import DeviceHistory
    rng = np.random.RandomState(4)
    T = 400
    mat = _cols(T, rng)
    active = np.ones(mat.shape, bool)
    losses = rng.normal(size=T)
    srt, _ = _engines()
    hs = DeviceHistory(srt, len(SPACE))
    hs.append(mat, active)
    works, isb = _level(hs, mat, active, losses, T)
    works[0].n_above -= 2
    with pytest.raises(L.TpeHipError, match="counts"):
        srt.run(works, history=hs, is_below=isb)
