"""Host-side drop-in API (no GPU): hp, Domain, Trials, fmin with rand.suggest,
and the columnar history / split that feeds the GPU engine, pinned against the
oracle on the reference's own histories (tests/golden)."""
import numpy as np
import pytest

from hyperopt_amd import (STATUS_FAIL, STATUS_OK, AllTrialsFailed, Domain, DuplicateLabel,
                          InvalidTrial, Trials, fmin, hp, pyll, rand, space_eval,
                          trials_from_docs)
from hyperopt_amd import tpe
from hyperopt_amd.fmin import generate_trials_to_calculate
from hyperopt_amd.pyll import scope
from oracle import tpe_oracle as O
from tests.golden import spaces
from tests.golden_io import E2E_CASES, load


def test_hp_validation():
    with pytest.raises(TypeError):
        hp.uniform(3, 0, 1)
    with pytest.raises(ValueError):
        hp.uniform("x", 2, 1)
    hp.uniform("x", 0, -1)  # reference quirk: a falsy bound skips the check
    with pytest.raises(DuplicateLabel):
        Domain(lambda x: 0, {"a": hp.uniform("x", 0, 1), "b": hp.normal("x", 0, 1)})


def test_param_specs():
    d = Domain(lambda x: 0, spaces.many_dists(hp))
    kinds = {k: s.kind for k, s in d.specs.items()}
    assert kinds["a"] == "randint" and kinds["k"] == "categorical" and kinds["f"] == "qloguniform"
    assert d.specs["bb"].args == (12, 25)
    assert d.specs["b"].args == (10, None)
    np.testing.assert_allclose(d.specs["k"].args[0], [0.1, 0.3, 0.6])
    d2 = Domain(lambda x: 0, {"x": hp.uniform("x", low=-1, high=2)})
    assert d2.specs["x"].args == (-1, 2)


def test_reachable_nested():
    d = Domain(lambda x: 0, spaces.nested(hp))
    assert d.reachable({}) == ["root"]
    assert set(d.reachable({"root": 1})) == {"root", "tree_depth", "tree_split"}
    assert set(d.reachable({"root": 1, "tree_split": 1})) == {"root", "tree_depth", "tree_split",
                                                                "ent_w", "ent_s"}
    assert set(d.reachable({"root": 2})) == {"root", "nn_units", "nn_drop"}


def test_rand_suggest_docs_and_space_eval():
    sp = spaces.nested(hp)
    d = Domain(lambda x: 0, sp)
    t = Trials()
    docs = rand.suggest([0, 1, 2], d, t, 5)
    assert [doc["tid"] for doc in docs] == [0, 1, 2]
    for doc in docs:
        t.assert_valid_trial(doc)
        vals = doc["misc"]["vals"]
        live = set(d.reachable({k: v[0] for k, v in vals.items() if v}))
        assert {k for k, v in vals.items() if v} == live
        cfg = {k: v[0] for k, v in vals.items() if v}
        out = space_eval(sp, cfg)
        assert out["kind"] in ("lin", "tree", "nn")


def test_fmin_rand_quadratic():
    trials = Trials()
    best = fmin(lambda x: (x - 1) ** 2, hp.uniform("x", -5, 5), algo=rand.suggest,
                max_evals=200, trials=trials, rstate=np.random.RandomState(0),
                show_progressbar=False)
    assert len(trials) == 200 and abs(best["x"] - 1) < 0.3
    assert trials.argmin == best
    assert trials.best_trial["result"]["loss"] == min(trials.losses())


def test_fmin_options():
    # points_to_evaluate, early stop, loss threshold, return_argmin=False
    trials = generate_trials_to_calculate([{"x": 0.5}, {"x": 1.5}])
    fmin(lambda x: (x - 1) ** 2, hp.uniform("x", -5, 5), algo=rand.suggest, max_evals=5,
         trials=trials, rstate=np.random.RandomState(1), show_progressbar=False)
    # like the reference, points are evaluated on top of max_evals (fmin.py:459-465)
    assert len(trials) == 7 and trials.trials[0]["misc"]["vals"]["x"] == [0.5]

    def stop_after(trials, count=0):
        return count + 1 >= 3, [count + 1]

    t2 = Trials()
    fmin(lambda x: x, hp.uniform("x", 0, 1), algo=rand.suggest, max_evals=100, trials=t2,
         early_stop_fn=stop_after, rstate=np.random.RandomState(2), show_progressbar=False)
    assert len(t2) == 3
    t3 = Trials()
    fmin(lambda x: x, hp.uniform("x", 0, 1), algo=rand.suggest, max_evals=1000, trials=t3,
         loss_threshold=0.5, rstate=np.random.RandomState(3), show_progressbar=False)
    assert len(t3) < 1000 and min(t3.losses()) < 0.5
    out = fmin(lambda p: p[1] ** 2 if p[0] == "b" else 1.0,
               hp.choice("c", [("a", 1.0), ("b", hp.uniform("y", -1, 1))]), algo=rand.suggest,
               max_evals=30, rstate=np.random.RandomState(4), return_argmin=False,
               show_progressbar=False)
    assert out[0] in ("a", "b")


def test_fmin_failures():
    def fn(x):
        return {"status": STATUS_FAIL}

    t = Trials()
    with pytest.raises(AllTrialsFailed):  # space_eval(trials.argmin), as fmin.py:546-549
        fmin(fn, hp.uniform("x", 0, 1), algo=rand.suggest, max_evals=5, trials=t,
             rstate=np.random.RandomState(0), show_progressbar=False, return_argmin=False)
    assert len(t) == 5
    with pytest.raises(AllTrialsFailed):
        t.best_trial

    def boom(x):
        raise RuntimeError("x")

    t2 = Trials()
    fmin(boom, hp.uniform("x", 0, 1), algo=rand.suggest, max_evals=3, trials=t2,
         catch_eval_exceptions=True, rstate=np.random.RandomState(0), show_progressbar=False,
         return_argmin=False)
    assert len(t2) == 0 and len(t2._dynamic_trials) == 3
    with pytest.raises(RuntimeError):
        fmin(boom, hp.uniform("x", 0, 1), algo=rand.suggest, max_evals=3,
             rstate=np.random.RandomState(0), show_progressbar=False)


def test_trials_semantics():
    t = Trials()
    with pytest.raises(InvalidTrial):
        t.insert_trial_doc({"tid": 0})
    ids = t.new_trial_ids(3)
    assert ids == [0, 1, 2]
    docs = t.new_trial_docs(ids, [None] * 3, [{"status": "new"}] * 3,
                            [{"tid": i, "cmd": None, "idxs": {"x": [i]}, "vals": {"x": [i * 0.1]}}
                             for i in ids])
    t.insert_trial_docs(docs)
    assert len(t) == 0  # not refreshed yet
    t.refresh()
    assert len(t) == 3 and t.count_by_state_synced(0) == 3
    t._dynamic_trials[1]["state"] = 3  # error jobs disappear on refresh
    t.refresh()
    assert t.tids == [0, 2]
    t2 = trials_from_docs([dict(d) for d in t.trials])
    assert t2.tids == [0, 2]
    assert t.idxs_vals[1]["x"] == [0.0, 0.2]


def test_columnar_cache_incremental():
    trials = Trials()
    sp = spaces.nested(hp)
    fmin(lambda p: 0.0, sp, algo=rand.suggest, max_evals=20, trials=trials,
         rstate=np.random.RandomState(0), show_progressbar=False)
    d = Domain(lambda x: 0, sp)
    labels = list(d.params)
    c1 = trials.columnar(labels)
    assert c1.rows == 20
    fmin(lambda p: 0.0, sp, algo=rand.suggest, max_evals=35, trials=trials,
         rstate=np.random.RandomState(1), show_progressbar=False)
    c2 = trials.columnar(labels)
    assert c2 is c1 and c2.rows == 35
    for r, doc in enumerate(trials._dynamic_trials):
        for j, lab in enumerate(labels):
            v = doc["misc"]["vals"][lab]
            assert c2.active[r, j] == bool(v)
            if v:
                assert c2.vals[r, j] == v[0]


def _trials_from_fixture(arrays, meta):
    tids = arrays["hist_tids"]
    losses = arrays["hist_losses"]
    labels = sorted(meta["specs"])
    docs = []
    for tid, loss in zip(tids, losses):
        idxs, vals = {}, {}
        for lab in labels:
            oi = arrays["obs_idxs/" + lab]
            pos = np.nonzero(oi == tid)[0]
            idxs[lab] = [int(tid)] if pos.size else []
            vals[lab] = [float(arrays["obs_vals/" + lab][pos[0]])] if pos.size else []
        result = {"status": STATUS_OK, "loss": float(loss)} if np.isfinite(loss) else \
            {"status": STATUS_FAIL}
        docs.append({"state": 2, "tid": int(tid), "spec": None, "result": result,
                     "misc": {"tid": int(tid), "cmd": None, "workdir": None, "idxs": idxs,
                              "vals": vals},
                     "exp_key": None, "owner": None, "version": 0, "book_time": None,
                     "refresh_time": None})
    return trials_from_docs(docs), labels


@pytest.mark.parametrize("case", E2E_CASES)
def test_history_split_matches_reference(case):
    """collect_history + split_masks == ap_split_trials on the reference's histories."""
    arrays, meta = load("e2e_" + case)
    trials, labels = _trials_from_fixture(arrays, meta)
    hist = tpe.collect_history(trials, labels)
    np.testing.assert_array_equal(hist.tids, arrays["hist_tids"])
    np.testing.assert_array_equal(hist.losses, arrays["hist_losses"])
    isb, isa = tpe.split_masks(hist, meta["gamma"])
    for j, lab in enumerate(labels):
        act = hist.active[:, j]
        below, above = O.ap_split_trials(arrays["obs_idxs/" + lab], arrays["obs_vals/" + lab],
                                         arrays["hist_tids"], arrays["hist_losses"], meta["gamma"])
        np.testing.assert_array_equal(hist.vals[act & isb, j], below)
        np.testing.assert_array_equal(hist.vals[act & isa, j], above)


def test_history_from_tid_and_duplicates():
    """Per-tid best loss with from_tid aliasing (tpe.py:876-896)."""
    t = Trials()
    mk = lambda tid, loss, x, src=None: {  # noqa: E731
        "state": 2, "tid": tid, "spec": None,
        "result": {"status": "ok", "loss": loss} if loss is not None else {"status": "new"},
        "misc": dict({"tid": tid, "cmd": None, "idxs": {"x": [tid]}, "vals": {"x": [x]}},
                     **({"from_tid": src} if src is not None else {})),
        "exp_key": None, "owner": None, "version": 0, "book_time": None, "refresh_time": None}
    t.insert_trial_docs([mk(0, 3.0, 0.1), mk(1, None, 0.2), mk(2, 1.0, 0.3, src=0),
                         mk(3, 2.0, 0.4)])
    t.refresh()
    h = tpe.collect_history(t, ["x"])
    assert list(h.tids) == [0, 1, 3]
    assert list(h.losses) == [1.0, np.inf, 2.0]
    assert list(h.obs_tids) == [2, 1, 3]


def test_label_key_and_precision():
    assert tpe.label_key(1, "x") == tpe.label_key(1, "x")
    assert tpe.label_key(1, "x") != tpe.label_key(2, "x")
    assert tpe.label_key(1, "x") != tpe.label_key(1, "y")
    assert tpe._precision(None, 24, 100) == 64
    assert tpe._precision(None, 1 << 22, 10_000) == 32
    # fp32 only where the cell-table path (exact argmax by the band re-score) runs
    assert tpe._precision(None, 4096, 1_000_000) == 64
    assert tpe._precision(None, 1 << 16, 1_000) == 32
    with pytest.raises(ValueError):
        tpe._precision(16, 1, 1)


def test_pyll_graph_ops():
    x = hp.uniform("x", 0, 1)
    e = pyll.as_apply({"a": (x + 1) * 2, "b": [x, -x], "c": scope.exp(x) ** 2})
    memo = {n: 0.5 for n in pyll.dfs(e) if n.name == "hyperopt_param"}
    out = pyll.rec_eval(e, memo=memo)
    assert out["a"] == 3.0 and out["b"] == (0.5, -0.5)
    assert np.isclose(out["c"], np.exp(1.0))
    sw = scope.switch(hp.randint("i", 2), 10, scope.Raise(ValueError, "not taken"))
    memo = {n: 0 for n in pyll.dfs(sw) if n.name == "hyperopt_param"}
    assert pyll.rec_eval(sw, memo=memo) == 10
    s = pyll.sample(hp.normal("n", 0, 1), np.random.RandomState(0))
    assert np.isfinite(s)


def test_smallest_rows_matches_stable_argsort():
    """split_masks' O(T) below-set selection == argsort(kind="stable")[:n] as a set
    (ties, inf and NaN losses included; tpe.py:637-640)."""
    from hyperopt_amd.tpe import _smallest_rows
    rng = np.random.RandomState(0)
    for trial in range(2000):
        T, n = rng.randint(1, 120), rng.randint(0, 30)
        if trial % 2:
            losses = rng.choice([0.0, 1.0, 2.0, np.inf, np.nan, -1.0], size=T)
        else:
            losses = rng.normal(size=T)
        want = set(np.argsort(losses, kind="stable")[:n].tolist())
        assert set(_smallest_rows(losses, n).tolist()) == want, (losses, n)


def test_plan_key_rules():
    """Level-plan cache key (engine.Engine._plan_key): history-mode levels of
    hashable structure only; injected candidates, per-candidate outputs, the
    sampler hook and upload mode always plan from scratch; the key follows
    kinds, arguments, candidate counts and columns but not the Philox keys."""
    from hyperopt_amd.engine import Engine, LabelWork
    eng = Engine.__new__(Engine)  # key logic only: no device state
    eng._plans = {}

    def work(**kw):
        base = dict(label="u", kind="uniform", args=(-5.0, 5.0), obs_below=np.zeros(3),
                    obs_above=None, n_cand=24, col=0, n_above=5)
        base.update(kw)
        return LabelWork(**base)

    k = lambda ws, **o: eng._plan_key(ws, 1.0, 25, 32, "auto", o.get("outputs", False),  # noqa
                                      o.get("sample_only", False), o.get("hist", True), False)
    assert k([work()]) is not None
    assert k([work()]) == k([work(key=99, cand_base=7, n_above=9, obs_below=np.ones(5))])
    assert k([work()]) != k([work(n_cand=48)])
    assert k([work()]) != k([work(col=1)])
    assert k([work(cand=np.zeros(4))]) is None
    assert k([work()], outputs=True) is None
    assert k([work()], sample_only=True) is None
    assert k([work()], hist=False) is None
    assert k([work(kind="categorical", args=([0.5, 0.5],))]) is None  # unhashable args


def test_label_keys_match_label_key():
    labs = ["x", "lr", "a_b", "ü", "c%d" % 7]
    for seed in (0, 1, 12345, 2 ** 40 + 7):
        assert tpe.label_keys(seed, labs) == [tpe.label_key(seed, lab) for lab in labs]


def test_reachable_memo_matches_walk():
    """Domain.reachable is memoised on the decided selector values; every
    answer equals a fresh walk of the space."""
    from hyperopt_amd import hp
    space = hp.choice("a", [("x", hp.uniform("u", 0, 1)),
                            ("y", hp.choice("b", [hp.normal("n", 0, 1),
                                                  {"z": hp.loguniform("lz", -3, 0)}])),
                            ("w", hp.randint("r", 5))])
    dom = Domain(lambda p: 0.0, space)
    cases = [{}, {"a": 0}, {"a": 1}, {"a": 1, "b": 0}, {"a": 1, "b": 1}, {"a": 2},
             {"a": 1, "b": 1, "lz": 0.3}, {"a": np.int64(1), "b": 0}]
    for _ in range(2):  # second pass served from the memo
        for d in cases:
            assert dom.reachable(d) == dom._reachable_walk(d), d


def test_smallest_rows_is_stable_argsort_prefix():
    """tpe._smallest_rows (C one-pass split, tpe_smallest_rows) == the rows of
    np.argsort(losses, kind="stable")[:n] -- ties to the earlier row, +inf and
    NaN last -- for random, tied, infinite and NaN-laden losses."""
    from hyperopt_amd.tpe import _smallest_rows
    rng = np.random.RandomState(0)
    for T in (1, 2, 7, 100, 1000, 10007):
        for kind in ("normal", "ties", "inf", "nan", "desc"):
            x = rng.normal(size=T)
            if kind == "ties":
                x = np.round(x * 2) / 2
            elif kind == "inf":
                x[rng.uniform(size=T) < 0.5] = np.inf
            elif kind == "nan":
                x[rng.uniform(size=T) < 0.7] = np.nan
            elif kind == "desc":
                x = -np.arange(T, dtype=float)
            for n in (1, 3, 25, T // 2 + 1, T):
                n = min(n, T)
                want = np.sort(np.argsort(x, kind="stable")[:n])
                got = np.sort(_smallest_rows(x, n))
                np.testing.assert_array_equal(got, want, err_msg="%s T=%d n=%d" % (kind, T, n))


def test_lat_prefix_setting_is_validated():
    """TPE_LAT_PREFIX (engine.lat_prefix): 0 or a multiple of 4096, checked
    when the engine reads it, not at the first quantized launch."""
    from hyperopt_amd.engine import _lat_prefix
    assert _lat_prefix("0") == 0 and _lat_prefix("65536") == 65536
    for bad in ("1000", "-4096", "abc"):
        with pytest.raises(ValueError):
            _lat_prefix(bad)


def test_split_inputs_fast_path_matches_split_masks():
    """LevelInputs.fast (tpe_split_inputs: the split and the level inputs in
    one C pass) gives the flags, below rows' values and the per-label counts
    of split_masks + LevelInputs, on ties, inactive labels and +inf losses."""
    from hyperopt_amd import _lib as L
    from hyperopt_amd.tpe import History, LevelInputs, split_masks

    class _Col:  # the columnar cache's fields the split reads
        pass

    rng = np.random.RandomState(2)
    lib = L.load()
    for T, Lb in ((1, 3), (40, 5), (997, 7), (5000, 4)):
        col = _Col()
        col.labels = tuple("l%d" % j for j in range(Lb))
        col.rows = T
        col.n_alias = 0
        col.vals = rng.normal(size=(T + 3, Lb))
        col.active = np.ascontiguousarray(rng.uniform(size=(T + 3, Lb)) < 0.7)
        col.active[T:] = True  # (rows past the history must not count)
        col.n_active = col.active[:T].sum(0).astype(np.int64)
        losses = np.round(rng.normal(size=T) * 2) / 2
        losses[rng.uniform(size=T) < 0.1] = np.inf
        tids = np.arange(T, dtype=np.int64)
        hist = History(tids, losses, tids, col=col)
        for gamma in (0.25, 0.5):
            isb, isa = split_masks(hist, gamma)
            nb_ref = col.active[:T][isb].sum(0)
            na_ref = col.active[:T][isa].sum(0)
            n_below = min(int(np.ceil(gamma * np.sqrt(T))), 25)
            flags = np.empty(T, np.uint8)
            rows = np.empty(max(n_below, 1), np.int64)
            nb = np.empty(Lb, np.int64)
            na = np.empty(Lb, np.int64)
            act = np.ascontiguousarray(col.active)
            got = lib.tpe_split_inputs(losses.ctypes.data, T, n_below, act.ctypes.data, Lb,
                                       col.n_active.ctypes.data, flags.ctypes.data,
                                       rows.ctypes.data, nb.ctypes.data, na.ctypes.data)
            assert got == min(n_below, T)
            np.testing.assert_array_equal(flags.view(bool), isb)
            np.testing.assert_array_equal(np.sort(rows[:got]), np.flatnonzero(isb))
            np.testing.assert_array_equal(nb, nb_ref)
            np.testing.assert_array_equal(na, na_ref)


def test_level_inputs_fast_equals_general_path():
    """LevelInputs.fast itself (not only tpe_split_inputs) against
    split_masks + LevelInputs on a real Columnar: flags, below values and
    activity, below / above counts, run_kwargs; and its None fallbacks -- a
    history over a row subset, from_tid aliasing, fewer history rows than
    cached rows, no engine.  split_masks' n_alias == 0 shortcut equals its
    np.isin path.  The HBM mirror is stubbed (device_history: no GPU here)."""
    from hyperopt_amd import tpe as T_
    from hyperopt_amd.base import Columnar
    from hyperopt_amd.tpe import History, LevelInputs, split_masks

    labels = ("a", "b", "c")
    rng = np.random.RandomState(4)
    sentinel = object()

    def docs(n, alias=False):
        out = []
        for t in range(n):
            vals = {lab: ([float(rng.normal())] if rng.uniform() < 0.8 else []) for lab in labels}
            misc = {"tid": t, "vals": vals, "idxs": {}}
            if alias and t > 3 and rng.uniform() < 0.3:
                misc["from_tid"] = int(rng.randint(t))
            out.append({"tid": t, "misc": misc, "state": 2,
                        "result": {"loss": float(np.round(rng.normal() * 2) / 2)}})
        return out

    for T in (1, 30, 500):
        col = Columnar(labels)
        col.extend(docs(T))
        col.device_history = lambda eng: sentinel
        losses = col.losses()
        hist = History(col.key_tid[:T], losses, col.obs_tid[:T], col=col)
        for gamma in (0.25, 1.0):
            fast = LevelInputs.fast(hist, gamma, eng=object())
            isb, isa = split_masks(hist, gamma)
            ref = LevelInputs(hist, isb, isa, eng=object())
            assert fast is not None and fast.device and ref.device
            np.testing.assert_array_equal(fast.isb, isb)
            np.testing.assert_array_equal(fast.vb[fast.ab], ref.vb[ref.ab])
            np.testing.assert_array_equal(fast.ab, ref.ab)
            np.testing.assert_array_equal(fast.nb, ref.nb)
            np.testing.assert_array_equal(fast.n_above, ref.n_above)
            assert fast.run_kwargs["history"] is sentinel and fast.run_kwargs["rows"] is None
            np.testing.assert_array_equal(fast.run_kwargs["is_below"], ref.run_kwargs["is_below"])
            # the shortcut of split_masks (no aliasing) equals the np.isin path
            below = np.zeros(T, bool)
            below[T_._smallest_rows(hist.losses, isb.sum())] = True
            np.testing.assert_array_equal(np.isin(hist.obs_tids, hist.tids[below]), isb)
            np.testing.assert_array_equal(np.isin(hist.obs_tids, hist.tids[~below]), isa)
        # the fallbacks
        sub = History(col.key_tid[:T], losses, col.obs_tid[:T], col=col, rows=np.arange(T))
        assert LevelInputs.fast(sub, 0.25, eng=object()) is None
        assert LevelInputs.fast(hist, 0.25, eng=None) is None
        if T > 1:
            short = History(col.key_tid[:T - 1], losses[:T - 1], col.obs_tid[:T - 1], col=col)
            assert LevelInputs.fast(short, 0.25, eng=object()) is None
    col = Columnar(labels)
    col.extend(docs(60, alias=True))
    assert col.n_alias > 0
    h = History(col.key_tid[:60], col.losses(), col.obs_tid[:60], col=col)
    assert LevelInputs.fast(h, 0.25, eng=object()) is None


def test_engine_switch_without_diag_warns(monkeypatch):
    """an engine switch set without TPE_DIAG=1 is ignored with a
    one-time warning; with TPE_DIAG=1 it is honoured."""
    from hyperopt_amd import engine as E
    monkeypatch.delenv("TPE_DIAG", raising=False)
    monkeypatch.setenv("TPE_SIDE_STREAM", "0")
    E._KNOBS_WARNED.discard("TPE_SIDE_STREAM")
    with pytest.warns(RuntimeWarning, match="TPE_SIDE_STREAM"):
        assert E._knob("TPE_SIDE_STREAM", "1") == "1"
    monkeypatch.setenv("TPE_DIAG", "1")
    assert E._knob("TPE_SIDE_STREAM", "1") == "0"
