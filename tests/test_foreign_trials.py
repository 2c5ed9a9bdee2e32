"""The columnar cache beside a foreign ``Trials`` (CPU): the reference's own
``hyperopt.Trials`` has no ``columnar()``, so ``fmin(algo=hyperopt_amd.tpe.suggest)``
with it goes through ``base.foreign_columnar``.  A stand-in with the
reference's shape (``_dynamic_trials``, ``refresh`` filtering to
JOB_VALID_STATES, ``trials`` property, ``delete_all``; base.py:252-698) must
give the history the reference's walk gives (tpe.py:876-896, base.py:200-214)
after appends, refreshes, deletions, state changes and from_tid aliases,
walking only the appended documents between calls."""
import numpy as np

from hyperopt_amd import tpe
from hyperopt_amd.base import (JOB_STATE_DONE, JOB_STATE_ERROR, JOB_VALID_STATES, Columnar,
                               foreign_columnar, invalidate_loss_cache)

LABELS = ["x", "y", "k"]


class RefShapedTrials(object):
    """The reference Trials' document handling only (no columnar cache)."""

    def __init__(self):
        self._dynamic_trials = []
        self.refresh()

    def refresh(self):  # base.py:364-376: a new filtered list every call
        self._trials = [t for t in self._dynamic_trials if t["state"] in JOB_VALID_STATES]

    @property
    def trials(self):
        return self._trials

    def __len__(self):
        return len(self._trials)

    def insert_trial_docs(self, docs):
        self._dynamic_trials.extend(docs)

    def delete_all(self):
        self._dynamic_trials = []
        self.refresh()


def _doc(tid, loss, vals, from_tid=None, state=JOB_STATE_DONE):
    misc = {"tid": tid, "cmd": None, "workdir": None,
            "idxs": {lab: ([tid] if lab in vals else []) for lab in LABELS},
            "vals": {lab: ([vals[lab]] if lab in vals else []) for lab in LABELS}}
    if from_tid is not None:
        misc["from_tid"] = from_tid
    result = {"status": "ok", "loss": loss} if loss is not None else {"status": "new"}
    return {"state": state, "tid": tid, "spec": None, "result": result, "misc": misc,
            "exp_key": None, "owner": None, "version": 0, "book_time": None,
            "refresh_time": None}


def _docs(rng, tid0, n, nan=0.0, alias=0.0):
    out = []
    for tid in range(tid0, tid0 + n):
        vals = {"k": int(rng.randint(4))}
        if rng.rand() < 0.8:
            vals["x"] = float(rng.uniform(-5, 5))
        if rng.rand() < 0.6:
            vals["y"] = float(np.exp(rng.uniform(-3, 0)))
        loss = float("nan") if rng.rand() < nan else float(rng.normal())
        src = int(rng.randint(tid)) if tid and rng.rand() < alias else None
        out.append(_doc(tid, loss, vals, from_tid=src))
    return out


def _same(trials):
    h = tpe.collect_history(trials, LABELS)
    w = tpe.walk_history(list(trials.trials), LABELS)
    np.testing.assert_array_equal(h.tids, w.tids)
    np.testing.assert_array_equal(h.losses, w.losses)
    np.testing.assert_array_equal(h.obs_tids, w.obs_tids)
    np.testing.assert_array_equal(h.active, w.active)
    np.testing.assert_array_equal(h.vals[h.active], w.vals[w.active])
    np.testing.assert_array_equal(h.label_counts(), w.active.sum(0))
    return h


def test_foreign_trials_incremental_cache(monkeypatch):
    rng = np.random.RandomState(0)
    t = RefShapedTrials()
    t.insert_trial_docs(_docs(rng, 0, 300))
    t.refresh()
    h = _same(t)
    col = h.col
    assert col is not None and col.rows == 300
    walked = []
    orig = Columnar.extend

    def counting(self, docs):
        walked.append(len(docs) - self.rows)
        return orig(self, docs)
    monkeypatch.setattr(Columnar, "extend", counting)
    for k in range(5):  # one new document per call, as fmin appends them
        t.insert_trial_docs(_docs(rng, 300 + k, 1))
        t.refresh()
        h = _same(t)
        assert h.col is col and col.rows == 301 + k
    assert walked == [1] * 5  # only the appended documents were walked
    # nothing appended: nothing walked, the same cache
    t.refresh()
    assert _same(t).col is col and walked[-1] == 0


def test_foreign_trials_rebuild_on_filter_delete_alias():
    rng = np.random.RandomState(1)
    t = RefShapedTrials()
    t.insert_trial_docs(_docs(rng, 0, 200, nan=0.05))
    t.refresh()
    col0 = _same(t).col
    # a document moves to ERROR: refresh filters it out, the rows shift -> rebuild
    t._dynamic_trials[57]["state"] = JOB_STATE_ERROR
    t.insert_trial_docs(_docs(rng, 200, 3))
    t.refresh()
    col1 = _same(t).col
    assert col1 is not col0 and col1.rows == 202
    # a document removed from the list by hand, nothing appended
    del t._dynamic_trials[10]
    t.refresh()
    assert _same(t).col is not col1
    # from_tid aliases (source_trial_docs): the general path, still the walk's result
    t.insert_trial_docs(_docs(rng, 203, 40, alias=0.5))
    t.refresh()
    h = _same(t)
    assert h.col is not None and h.col.n_alias > 0
    # delete_all, then a fresh history
    t.delete_all()
    assert _same(t).tids.size == 0
    t.insert_trial_docs(_docs(rng, 0, 30))
    t.refresh()
    assert _same(t).col.rows == 30


def test_foreign_trials_unfinished_and_edited_losses():
    rng = np.random.RandomState(2)
    t = RefShapedTrials()
    docs = _docs(rng, 0, 50)
    docs[-1]["state"], docs[-1]["result"] = 0, {"status": "new"}  # NEW, loss None -> +inf
    t.insert_trial_docs(docs)
    t.refresh()
    h = _same(t)
    assert np.isinf(h.losses[-1])
    docs[-1]["state"], docs[-1]["result"] = JOB_STATE_DONE, {"status": "ok", "loss": -9.0}
    assert _same(t).losses[-1] == -9.0  # unfinished rows are re-read every call
    docs[3]["result"]["loss"] = -11.0  # an edit of a DONE document after it was cached
    invalidate_loss_cache(t)
    assert _same(t).losses[3] == -11.0


def test_foreign_columnar_without_weakref():
    """An object that cannot be weak-referenced keeps the cache as an attribute."""
    class Slotted(object):
        __slots__ = ("trials", "_hyperopt_amd_columnar", "__dict__")

    rng = np.random.RandomState(3)
    t = Slotted()
    t.trials = _docs(rng, 0, 20)
    c0 = foreign_columnar(t, t.trials, LABELS)
    t.trials = t.trials + _docs(rng, 20, 2)
    c1 = foreign_columnar(t, t.trials, LABELS)
    assert c0 is c1 and c1.rows == 22
