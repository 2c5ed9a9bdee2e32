"""HBM-resident history (DeviceHistory + tpe_gather_obs) vs the upload path.

The gathered observation lists must be exactly the ones ap_split_trials
builds (tpe.py:623-646: active rows of the label, below / above by the
n_below best losses, tid order), so every result of a history-mode run is
bit-identical to the same run with the lists packed on the host.
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

SPACE = [("u", "uniform", (-5.0, 5.0)), ("lu", "loguniform", (-5.0, 0.0)),
         ("q", "quniform", (0.0, 20.0, 1.0)), ("n", "normal", (0.0, 2.0)),
         ("c", "randint", (6,)), ("r", "randint", (3, 11))]


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


def _history(T, seed, inactive=0.0):
    rng = np.random.RandomState(seed)
    cols = [rng.uniform(-5, 5, T), np.exp(rng.uniform(-5, 0, T)),
            np.round(rng.uniform(0, 20, T)), rng.normal(0, 2, T),
            rng.randint(0, 6, T).astype(float), rng.randint(3, 11, T).astype(float)]
    mat = np.stack(cols, axis=1)
    active = rng.uniform(size=mat.shape) >= inactive
    losses = rng.normal(size=T)
    return mat, active, losses


def _works(mat, active, losses, rows, hist=None, n_cand=1 << 14):
    from hyperopt_amd.engine import LabelWork
    T = rows.size
    n_below = min(int(np.ceil(0.25 * np.sqrt(T))), 25)
    order = np.argsort(losses[rows], kind="stable")
    isb = np.zeros(T, np.uint8)
    isb[order[:n_below]] = 1
    works = []
    for j, (lab, kind, a) in enumerate(SPACE):
        act = active[rows, j]
        v = mat[rows, j]
        below, above = v[act & (isb == 1)], v[act & (isb == 0)]
        w = LabelWork(lab, kind, a, below, above, n_cand=n_cand, key=777 + j)
        if hist is not None:
            w.obs_above, w.col, w.n_above = None, j, above.size
        works.append(w)
    return works, isb


@pytest.mark.parametrize("T,inactive,permute", [(40, 0.0, False), (3000, 0.0, False),
                                                 (2500, 0.3, False), (1500, 0.2, True)])
def test_history_gather_matches_upload(engine, T, inactive, permute):
    from hyperopt_amd.engine import DeviceHistory
    mat, active, losses = _history(T, T, inactive)
    hist = DeviceHistory(engine, len(SPACE), cap=64)  # grows while appending
    for a in range(0, T, 700):
        hist.append(mat[a:a + 700], active[a:a + 700])
    rows = np.random.RandomState(1).permutation(T) if permute else np.arange(T)
    up, _ = _works(mat, active, losses, rows)
    hw, isb = _works(mat, active, losses, rows, hist=hist)
    kw = dict(rows=rows.astype(np.int32)) if permute else {}
    for precision in (64, 32):
        r_up = engine.run(up, precision=precision)
        r_h = engine.run(hw, precision=precision, history=hist, is_below=isb, **kw)
        for a, b in zip(r_up, r_h):
            assert (a.index, a.value, a.score) == (b.index, b.value, b.score), (a, b)
    post_up = engine.run(up, posteriors=True)
    post_h = engine.run(hw, posteriors=True, history=hist, is_below=isb, **kw)
    for a, b in zip(post_up, post_h):
        for k in a.extra:
            for x, y in zip(np.atleast_1d(a.extra[k]), np.atleast_1d(b.extra[k])):
                np.testing.assert_array_equal(x, y)


def test_history_posterior_matches_oracle(engine):
    """The gathered lists feed the same Parzen fit the reference computes."""
    from hyperopt_amd.engine import DeviceHistory
    mat, active, losses = _history(2000, 5, 0.1)
    hist = DeviceHistory(engine, len(SPACE))
    hist.append(mat, active)
    rows = np.arange(2000)
    hw, isb = _works(mat, active, losses, rows, hist=hist)
    res = engine.run(hw, posteriors=True, history=hist, is_below=isb)
    j = 3  # normal(0, 2)
    act = active[:, j]
    below, above = O.ap_split_trials(np.flatnonzero(act), mat[act, j], rows, losses, 0.25)
    for half, obs in (("below", below), ("above", above)):
        ref = O.adaptive_parzen_normal(obs, 1.0, 0.0, 2.0)
        for got, want in zip(res[j].extra[half], ref):
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)


@pytest.mark.parametrize("j", [0, 4])
def test_history_count_mismatch_raises(engine, j):
    """A continuous (sorted fit) or categorical (tpe_cat_posterior_hist)
    label whose host count disagrees with the rows the device finds."""
    from hyperopt_amd import _lib as L
    from hyperopt_amd.engine import DeviceHistory
    mat, active, losses = _history(500, 9)
    hist = DeviceHistory(engine, len(SPACE))
    hist.append(mat, active)
    hw, isb = _works(mat, active, losses, np.arange(500), hist=hist)
    hw[j].n_above -= 3  # the host claims fewer rows than the device finds
    with pytest.raises(L.TpeHipError, match="counts"):
        engine.run(hw, history=hist, is_below=isb)


@pytest.mark.parametrize("T,K", [(60000, 3), (120000, 40)])
def test_history_categorical_counts_long(engine, T, K):
    """Categorical posteriors counted in the HBM history (no gathered lists)
    over long LF-ramped histories: bit-exact against np.bincount's
    sequential sums (the oracle) and the upload path."""
    from hyperopt_amd.engine import DeviceHistory, LabelWork
    rng = np.random.RandomState(T + K)
    p = rng.dirichlet(np.full(K, 0.5))
    mat = np.stack([rng.choice(K, size=T, p=p).astype(float),
                    (rng.choice(K, size=T, p=p) + 2).astype(float)], axis=1)
    active = rng.uniform(size=mat.shape) >= 0.1
    losses = rng.normal(size=T)
    hist = DeviceHistory(engine, 2)
    hist.append(mat, active)
    n_below = min(int(np.ceil(0.25 * np.sqrt(T))), 25)
    isb = np.zeros(T, np.uint8)
    isb[np.argsort(losses, kind="stable")[:n_below]] = 1
    specs = [("c", "categorical", (tuple(p.tolist()),)), ("r", "randint", (2, 2 + K))]
    works = []
    for j, (lab, kind, a) in enumerate(specs):
        v = mat[active[:, j], j]
        b = isb[active[:, j]] == 1
        w = LabelWork(lab, kind, a, v[b], None, col=j, n_above=int((~b).sum()))
        works.append(w)
    res = engine.run(works, posteriors=True, history=hist, is_below=isb)
    for j, (lab, kind, a) in enumerate(specs):
        v = mat[active[:, j], j].astype(np.int64)
        b = isb[active[:, j]] == 1
        if kind == "categorical":
            want = O.categorical_posterior(v[~b], 1.0, p)
        else:
            want = O.randint_posterior(v[~b], 1.0, 2, 2 + K)
        np.testing.assert_array_equal(res[j].extra["p_above"], want, err_msg=lab)


def _suggest_both(monkeypatch, trials, domain, n_ei, seed=7):
    from hyperopt_amd import tpe
    out = []
    for dev in (True, False):
        monkeypatch.setattr(tpe, "USE_DEVICE_HISTORY", dev)
        docs = tpe.suggest([100_000], domain, trials, seed, n_EI_candidates=n_ei, verbose=False)
        out.append(docs[0]["misc"]["vals"])
    return out


@pytest.mark.parametrize("kw", [{}, {"dup": 0.3, "nan": 0.1, "none": 0.1},
                                {"cancel": 0.2, "dup": 0.1}])
@pytest.mark.parametrize("n_ei", [24, 1 << 16])
def test_suggest_device_history_matches_host_lists(monkeypatch, kw, n_ei):
    """tpe.suggest gathering from the HBM mirror of the trials' columnar cache
    == tpe.suggest with host-sliced lists (same Philox streams => identical
    documents), on histories with from_tid duplicates, NaN / None losses and
    cancelled documents (fp64 path at n_EI=24, fp32 table path at 2^16)."""
    from hyperopt_amd import hp
    from hyperopt_amd.base import Domain
    from tests.test_history_cache import _random_trials
    domain = Domain(lambda p: 0.0, {"x": hp.uniform("x", -5, 5), "y": hp.loguniform("y", -3, 0),
                                    "k": hp.randint("k", 4)})
    rng = np.random.RandomState(n_ei + len(kw))
    for T in (30, 700):
        trials = _random_trials(rng, T, **kw)
        dev, host = _suggest_both(monkeypatch, trials, domain, n_ei)
        assert dev == host, (T, dev, host)


def test_fmin_device_history_incremental(monkeypatch):
    """fmin appends one row per iteration to the HBM mirror; the whole run is
    identical to the host-list run."""
    from hyperopt_amd import Trials, fmin, hp, tpe
    space = {"x": hp.uniform("x", -5, 5), "c": hp.choice("c", [0, 1, 2]),
             "q": hp.quniform("q", 0, 10, 1)}

    def run(dev):
        monkeypatch.setattr(tpe, "USE_DEVICE_HISTORY", dev)
        t = Trials()
        fmin(lambda p: (p["x"] - 1) ** 2 + p["c"] + 0.1 * p["q"], space, algo=tpe.suggest,
             max_evals=45, trials=t, rstate=np.random.RandomState(4), show_progressbar=False)
        return t
    t_dev, t_host = run(True), run(False)
    assert [d["misc"]["vals"] for d in t_dev.trials] == [d["misc"]["vals"] for d in t_host.trials]
    col = next(iter(t_dev._columnar.values()))
    (dh,) = col._device.values()
    assert dh.rows == 44  # mirrored up to the last suggest's history


def test_suggest_many_multi_history_matches_host_lists(monkeypatch):
    """suggest_many gathering every study's lists from its own HBM mirror in one
    tpe_gather_obs_multi launch == suggest_many with host-sliced lists, for
    studies of different sizes and history shapes (duplicates, NaN / None
    losses, cancelled documents) in one batch."""
    from hyperopt_amd import hp, tpe
    from hyperopt_amd.base import Domain
    from tests.test_history_cache import _random_trials
    domain = Domain(lambda p: 0.0, {"x": hp.uniform("x", -5, 5), "y": hp.loguniform("y", -3, 0),
                                    "k": hp.randint("k", 4)})
    rng = np.random.RandomState(21)
    kws = [{}, {"dup": 0.3, "nan": 0.1}, {"cancel": 0.2, "none": 0.1}, {}, {"dup": 0.1}]
    studies = [_random_trials(rng, T, **kw) for T, kw in zip((40, 300, 120, 900, 64), kws)]
    out = {}
    for dev in (True, False):
        monkeypatch.setattr(tpe, "USE_DEVICE_HISTORY", dev)
        reqs = [tpe.SuggestRequest([10_000], domain, t, 5 + s, n_EI_candidates=n)
                for s, t in enumerate(studies) for n in (24, 1 << 14)]
        out[dev] = [d[0]["misc"]["vals"] for d in tpe.suggest_many(reqs)]
    assert out[True] == out[False]


@pytest.mark.parametrize("T,K,rows", [(32769, 2, False), (40000, 32, False), (70001, 5, True),
                                      (131072, 3, False)])
def test_categorical_counts_chunked_equal_single_block(T, K, rows):
    """The chunked count of a long history (k_cath_count / k_cath_emit /
    k_cath_fold: many blocks, each list folded in order) gives the posterior
    bits of the single block per (segment, category) and of np.bincount:
    chunk and wave boundaries inside the LF ramp, 32 categories, a row list
    (a subset of the history's rows)."""
    from hyperopt_amd.engine import DeviceHistory, Engine, LabelWork
    rng = np.random.RandomState(T + 7 * K)
    p = rng.dirichlet(np.full(K, 0.7))
    col = rng.choice(K, size=T, p=p).astype(float)
    mat = np.stack([col, rng.choice(K, size=T).astype(float) + 1], axis=1)
    active = rng.uniform(size=mat.shape) >= 0.15
    losses = rng.normal(size=T)
    sel = np.sort(rng.choice(T, size=T - T // 7, replace=False)) if rows else np.arange(T)
    out = []
    for chunked in (True, False):
        eng = Engine()
        eng.cat_chunked = chunked
        hist = DeviceHistory(eng, 2)
        hist.append(mat, active)
        n = sel.size
        n_below = min(int(np.ceil(0.25 * np.sqrt(n))), 25)
        isb = np.zeros(n, np.uint8)
        isb[np.argsort(losses[sel], kind="stable")[:n_below]] = 1
        specs = [("c", "categorical", (tuple(p.tolist()),)), ("r", "randint", (1, 1 + K))]
        works = []
        for j, (lab, kind, a) in enumerate(specs):
            act = active[sel, j]
            v = mat[sel, j][act]
            b = isb[act] == 1
            works.append(LabelWork(lab, kind, a, v[b], None, col=j, n_above=int((~b).sum())))
        res = eng.run(works, posteriors=True, history=hist, is_below=isb,
                      rows=None if not rows else sel.astype(np.int32))
        out.append([(r.extra["p_below"].copy(), r.extra["p_above"].copy()) for r in res])
        if not chunked:
            for j, (lab, kind, a) in enumerate(specs):
                act = active[sel, j]
                v = mat[sel, j][act].astype(np.int64)
                b = isb[act] == 1
                if kind == "categorical":
                    want = O.categorical_posterior(v[~b], 1.0, p)
                else:
                    want = O.randint_posterior(v[~b], 1.0, 1, 1 + K)
                np.testing.assert_array_equal(res[j].extra["p_above"], want, err_msg=lab)
    for (ab, aa), (bb, ba) in zip(out[0], out[1]):
        np.testing.assert_array_equal(ab, bb)
        np.testing.assert_array_equal(aa, ba)
