"""Trials / Domain / Ctrl: the data model the suggest path reads (hyperopt/base.py).

Same document format and semantics as the reference: a trial document is
``{state, tid, spec, result, misc: {tid, cmd, workdir, idxs, vals}, exp_key,
owner, version, book_time, refresh_time}`` (base.py:459-482), ``refresh``
keeps documents in JOB_VALID_STATES (base.py:364-376), ``Domain`` compiles
the search space and evaluates a configuration (base.py:770-1018).

What is new here: ``Trials.columnar(labels)`` -- a cached, incrementally
extended columnar view of the history (one row per document, one column per
label) so that tpe.suggest reads observations with numpy indexing instead of
the reference's per-document dict walks (base.py:200-214, tpe.py:641-644).
"""
from __future__ import annotations

import datetime
import logging
import numbers
import sys
import weakref

import numpy as np

from . import pyll
from .exceptions import (AllTrialsFailed, DuplicateLabel, InvalidLoss,  # noqa: F401
                         InvalidResultStatus, InvalidTrial)

logger = logging.getLogger(__name__)

STATUS_NEW = "new"
STATUS_RUNNING = "running"
STATUS_SUSPENDED = "suspended"
STATUS_OK = "ok"
STATUS_FAIL = "fail"
STATUS_STRINGS = ("new", "running", "suspended", "ok", "fail")

JOB_STATE_NEW = 0
JOB_STATE_RUNNING = 1
JOB_STATE_DONE = 2
JOB_STATE_ERROR = 3
JOB_STATE_CANCEL = 4
JOB_STATES = [JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR, JOB_STATE_CANCEL]
JOB_VALID_STATES = {JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE}

TRIAL_KEYS = ["tid", "spec", "result", "misc", "state", "owner", "book_time", "refresh_time",
              "exp_key"]
TRIAL_MISC_KEYS = ["tid", "cmd", "idxs", "vals"]


def coarse_utcnow():
    now = datetime.datetime.utcnow()
    return now.replace(microsecond=(now.microsecond // 1000) * 1000)


_SON_PLAIN = (float, int, str, bool, type(None))


def SONify(arg, memo=None):  # noqa: N802
    """Convert numpy scalars/arrays to plain Python (base.py:128-169, no bson)."""
    t = type(arg)
    if t in _SON_PLAIN:  # the common leaves, returned as they are
        return arg
    if t is dict:
        return {SONify(k): SONify(v) for k, v in arg.items()}
    if t is list:
        return [SONify(a) for a in arg]
    if isinstance(arg, np.floating):
        return float(arg)
    if isinstance(arg, np.integer):
        return int(arg)
    if isinstance(arg, np.bool_):
        return bool(arg)
    if isinstance(arg, np.ndarray):
        return SONify(arg.sum()) if arg.ndim == 0 else [SONify(a) for a in arg]
    if isinstance(arg, dict):
        return {SONify(k): SONify(v) for k, v in arg.items()}
    if isinstance(arg, (list, tuple)):
        return type(arg)(SONify(a) for a in arg)
    return arg


def miscs_update_idxs_vals(miscs, idxs, vals, assert_all_vals_used=True, idxs_map=None):
    """Unpack the idxs/vals format into the misc dicts (base.py:172-197)."""
    idxs_map = {} if idxs_map is None else idxs_map
    assert set(idxs.keys()) == set(vals.keys())
    by_id = {m["tid"]: m for m in miscs}
    for m in miscs:
        m["idxs"] = {k: [] for k in idxs}
        m["vals"] = {k: [] for k in idxs}
    for key in idxs:
        assert len(idxs[key]) == len(vals[key])
        for tid, val in zip(idxs[key], vals[key]):
            tid = idxs_map.get(tid, tid)
            if assert_all_vals_used or tid in by_id:
                by_id[tid]["idxs"][key] = [tid]
                by_id[tid]["vals"][key] = [val]
    return miscs


def miscs_to_idxs_vals(miscs, keys=None):
    """Per-label (tids, values) lists from misc dicts (base.py:200-214)."""
    if keys is None:
        if len(miscs) == 0:
            raise ValueError("cannot infer keys from empty miscs")
        keys = list(miscs[0]["idxs"].keys())
    idxs, vals = {k: [] for k in keys}, {k: [] for k in keys}
    for misc in miscs:
        for k in keys:
            ti, tv = misc["idxs"][k], misc["vals"][k]
            assert len(ti) == len(tv)
            assert ti == [] or ti == [misc["tid"]]
            idxs[k].extend(ti)
            vals[k].extend(tv)
    return idxs, vals


def spec_from_misc(misc):
    spec = {}
    for k, v in misc["vals"].items():
        if len(v) == 1:
            spec[k] = v[0]
        elif len(v) > 1:
            raise NotImplementedError("multiple values", (k, v))
    return spec


def validate_timeout(timeout):
    if timeout is not None and (not isinstance(timeout, numbers.Number) or timeout <= 0
                                or isinstance(timeout, bool)):
        raise Exception("The timeout argument should be None or a positive value. "
                        "Given value: {timeout}".format(timeout=timeout))


def validate_loss_threshold(loss_threshold):
    if loss_threshold is not None and (not isinstance(loss_threshold, numbers.Number)
                                       or isinstance(loss_threshold, bool)):
        raise Exception("The loss_threshold argument should be None or a numeric value. "
                        "Given value: {loss_threshold}".format(loss_threshold=loss_threshold))


def doc_loss(doc):
    """A document's loss for tpe.suggest: result['loss'], None -> +inf (tpe.py:880-882)."""
    loss = doc["result"].get("loss")
    return float("inf") if loss is None else float(loss)


class Columnar(object):
    """Cached columnar view of a trials history for a fixed label tuple.

    Row r holds document r of ``Trials._dynamic_trials`` (documents are
    append-only there); ``vals[r, j]`` is the value of label j (NaN when the
    label is inactive in that trial, ``active[r, j]`` False).  Per row it also
    keeps the tid the row's loss is filed under (``misc.from_tid`` or ``tid``,
    tpe.py:879) and the tid its observations are filed under (``misc.tid``),
    the per-label active counts, and -- once tpe.suggest asks for it -- a
    mirror of the matrix in HBM per device (``device_history``), appended with
    the new rows only.
    """

    def __init__(self, labels):
        self.labels = tuple(labels)
        self.col = {lab: j for j, lab in enumerate(self.labels)}
        self.rows = 0
        self.docs = []
        self.row_of = {}
        self.vals = np.zeros((0, len(self.labels)))
        self.active = np.zeros((0, len(self.labels)), bool)
        self.key_tid = np.zeros(0, np.int64)
        self.obs_tid = np.zeros(0, np.int64)
        self.n_active = np.zeros(len(self.labels), np.int64)
        self.keys_increasing = True  # key_tid strictly increasing: one document per tid
        self.n_alias = 0  # rows whose observations are filed under another tid (from_tid)
        self.loss = np.zeros(0)
        self.n_final = 0  # rows [0, n_final) are DONE and their losses cached
        self._device = {}

    def extend(self, docs):
        new = docs[self.rows:]
        if not new:
            return
        need = self.rows + len(new)
        if need > self.vals.shape[0]:
            cap = max(need, 2 * self.vals.shape[0], 64)
            v = np.full((cap, len(self.labels)), np.nan)
            a = np.zeros((cap, len(self.labels)), bool)
            kt = np.zeros(cap, np.int64)
            ot = np.zeros(cap, np.int64)
            ls = np.zeros(cap)
            v[:self.rows] = self.vals[:self.rows]
            a[:self.rows] = self.active[:self.rows]
            kt[:self.rows] = self.key_tid[:self.rows]
            ot[:self.rows] = self.obs_tid[:self.rows]
            ls[:self.n_final] = self.loss[:self.n_final]
            self.vals, self.active, self.key_tid, self.obs_tid, self.loss = v, a, kt, ot, ls
        col = self.col
        last = self.key_tid[self.rows - 1] if self.rows else None
        inc = self.keys_increasing
        for r, doc in enumerate(new, start=self.rows):
            misc = doc["misc"]
            for lab, vv in misc["vals"].items():
                j = col.get(lab)
                if j is not None and len(vv):
                    self.vals[r, j] = float(vv[0])
                    self.active[r, j] = True
            key = misc.get("from_tid", doc["tid"])
            self.key_tid[r] = key
            self.obs_tid[r] = misc["tid"]
            if key != misc["tid"]:
                self.n_alias += 1
            if inc and last is not None and not key > last:
                inc = False
            last = key
            self.row_of[id(doc)] = r
        self.keys_increasing = inc
        self.n_active += self.active[self.rows:need].sum(0)
        self.docs.extend(new)
        self.rows = need

    VALID_SAMPLES = 16  # strided identity probes of valid_for (foreign lists), besides the ends

    def valid_for(self, docs, probes=0):
        """Whether rows [0, rows) are still ``docs``' first documents: the
        first and the last cached row -- and ``probes`` strided rows between,
        for lists this package does not own (foreign_columnar) -- must be the
        same objects.  A removal anywhere shifts the last cached row (or
        shortens the list), so deletions and filtering are caught; a document
        replaced in place by another object between probes is not.
        (``Trials._dynamic_trials`` only grows, or is replaced whole.)"""
        n = min(self.rows, len(docs))
        if n == 0:
            return True
        mine = self.docs
        if docs[n - 1] is not mine[n - 1] or docs[0] is not mine[0]:
            return False
        if not probes:
            return True
        step = max(1, n // probes)
        return all(docs[i] is mine[i] for i in range(step, n - 1, step))

    def losses(self):
        """Loss of every row (tpe.py:880-882: None -> +inf), as a new array.

        A document's loss is read once it is DONE and cached from then on:
        hyperopt's evaluation flow sets ``result`` and then ``state = DONE``
        and never touches a finished document again.  Rows not yet DONE
        (NEW / RUNNING, loss usually None) are re-read on every call.
        """
        docs, n, k = self.docs, self.rows, self.n_final
        while k < n and docs[k]["state"] == JOB_STATE_DONE:
            self.loss[k] = doc_loss(docs[k])
            k += 1
        self.n_final = k
        out = self.loss[:n].copy()
        for r in range(k, n):
            out[r] = doc_loss(docs[r])
        return out

    def device_history(self, engine):
        """The HBM mirror of rows [0, rows) on ``engine``'s device
        (engine.DeviceHistory, device row r == row r here), brought up to date
        by appending the rows added since the last call."""
        from .engine import DeviceHistory
        key = engine.device  # (a torch.device: hashed by type and index)
        dh = self._device.get(key)
        if dh is None or dh.rows > self.rows:
            dh = self._device[key] = DeviceHistory(engine, len(self.labels),
                                                   cap=max(self.rows, 1024))
        if dh.rows < self.rows:
            dh.append(self.vals[dh.rows:self.rows], self.active[dh.rows:self.rows])
        return dh


_FOREIGN = weakref.WeakKeyDictionary()  # foreign trials object -> {labels: Columnar}


def foreign_columnar(trials, docs, labels):
    """The columnar cache of a ``Trials`` object that has no ``columnar()``
    (the reference's own ``hyperopt.Trials``, or a subclass from another
    backend), kept beside it and extended incrementally like
    ``Trials.columnar``: rows are ``docs`` (``trials.trials``, the refreshed
    document list) and a call walks only the documents appended since the last
    one.  The whole cache is rebuilt when ``docs`` no longer starts with the
    cached documents (``Columnar.valid_for``: deletion, ``delete_all``, a
    refresh that filtered a document out).  Returns None when the object can
    be neither weak-referenced nor given an attribute (the caller then walks
    the documents, as the reference does: tpe.py:876-896, base.py:200-214).

    Like ``Trials.columnar`` the losses of finished documents are read once
    (``Columnar.losses``); ``invalidate_loss_cache(trials)`` forgets them."""
    try:
        cache = _FOREIGN.get(trials)
        if cache is None:
            cache = _FOREIGN[trials] = {}
    except TypeError:  # not weak-referenceable / unhashable: an attribute instead
        cache = getattr(trials, "_hyperopt_amd_columnar", None)
        if cache is None:
            try:
                cache = {}
                setattr(trials, "_hyperopt_amd_columnar", cache)
            except (AttributeError, TypeError):
                return None
    if not isinstance(docs, list):
        docs = list(docs)
    key = tuple(labels)
    col = cache.get(key)
    if col is None or col.rows > len(docs) or not col.valid_for(docs, Columnar.VALID_SAMPLES):
        col = cache[key] = Columnar(key)
    col.extend(docs)
    return col


def invalidate_loss_cache(trials):
    """Forget the cached losses of finished documents of any trials object
    (ours: Trials.invalidate_loss_cache; a foreign one: its foreign_columnar
    caches) -- call after editing the ``result`` of a DONE document."""
    if hasattr(trials, "invalidate_loss_cache"):
        trials.invalidate_loss_cache()
        return
    try:
        caches = _FOREIGN.get(trials) or {}
    except TypeError:
        caches = getattr(trials, "_hyperopt_amd_columnar", None) or {}
    for col in caches.values():
        col.n_final = 0


class Trials(object):
    """List-of-documents history (base.py:252-698)."""

    asynchronous = False

    def __init__(self, exp_key=None, refresh=True):
        self._ids = set()
        self._dynamic_trials = []
        self._exp_key = exp_key
        self.attachments = {}
        self._columnar = {}
        if refresh:
            self.refresh()

    def view(self, exp_key=None, refresh=True):
        rval = object.__new__(self.__class__)
        rval._exp_key = exp_key
        rval._ids = self._ids
        rval._dynamic_trials = self._dynamic_trials
        rval.attachments = self.attachments
        rval._columnar = {}
        if refresh:
            rval.refresh()
        return rval

    def aname(self, trial, name):
        return "ATTACH::%s::%s" % (trial["tid"], name)

    def trial_attachments(self, trial):
        trials = self

        class Attachments(object):
            def __contains__(self, name):
                return trials.aname(trial, name) in trials.attachments

            def __getitem__(self, name):
                return trials.attachments[trials.aname(trial, name)]

            def __setitem__(self, name, value):
                trials.attachments[trials.aname(trial, name)] = value

            def __delitem__(self, name):
                del trials.attachments[trials.aname(trial, name)]

        return Attachments()

    def __iter__(self):
        try:
            return iter(self._trials)
        except AttributeError:
            print("You have to refresh before you iterate", file=sys.stderr)
            raise

    def __len__(self):
        try:
            return len(self._trials)
        except AttributeError:
            print("You have to refresh before you compute len", file=sys.stderr)
            raise

    def __getitem__(self, item):
        raise NotImplementedError("")

    def refresh(self):
        if self._exp_key is None:
            self._trials = [t for t in self._dynamic_trials if t["state"] in JOB_VALID_STATES]
        else:
            self._trials = [t for t in self._dynamic_trials
                            if t["state"] in JOB_VALID_STATES and t["exp_key"] == self._exp_key]
        self._ids.update([t["tid"] for t in self._trials])

    @property
    def trials(self):
        return self._trials

    @property
    def tids(self):
        return [t["tid"] for t in self._trials]

    @property
    def specs(self):
        return [t["spec"] for t in self._trials]

    @property
    def results(self):
        return [t["result"] for t in self._trials]

    @property
    def miscs(self):
        return [t["misc"] for t in self._trials]

    @property
    def idxs_vals(self):
        return miscs_to_idxs_vals(self.miscs)

    @property
    def idxs(self):
        return self.idxs_vals[0]

    @property
    def vals(self):
        return self.idxs_vals[1]

    def assert_valid_trial(self, trial):
        if not (hasattr(trial, "keys") and hasattr(trial, "values")):
            raise InvalidTrial("trial should be dict-like", trial)
        for key in TRIAL_KEYS:
            if key not in trial:
                raise InvalidTrial("trial missing key %s", key)
        for key in TRIAL_MISC_KEYS:
            if key not in trial["misc"]:
                raise InvalidTrial('trial["misc"] missing key', key)
        if trial["tid"] != trial["misc"]["tid"]:
            raise InvalidTrial("tid mismatch between root and misc", trial)
        if trial["exp_key"] != self._exp_key:
            raise InvalidTrial("wrong exp_key", (trial["exp_key"], self._exp_key))
        return trial

    def _insert_trial_docs(self, docs):
        rval = [doc["tid"] for doc in docs]
        self._dynamic_trials.extend(docs)
        return rval

    def insert_trial_doc(self, doc):
        doc = self.assert_valid_trial(SONify(doc))
        return self._insert_trial_docs([doc])[0]

    def insert_trial_docs(self, docs):
        docs = [self.assert_valid_trial(SONify(doc)) for doc in docs]
        return self._insert_trial_docs(docs)

    def new_trial_ids(self, n):
        aa = len(self._ids)
        rval = list(range(aa, aa + n))
        self._ids.update(rval)
        return rval

    def new_trial_docs(self, tids, specs, results, miscs):
        assert len(tids) == len(specs) == len(results) == len(miscs)
        return [{"state": JOB_STATE_NEW, "tid": tid, "spec": spec, "result": result,
                 "misc": misc, "exp_key": self._exp_key, "owner": None, "version": 0,
                 "book_time": None, "refresh_time": None}
                for tid, spec, result, misc in zip(tids, specs, results, miscs)]

    def source_trial_docs(self, tids, specs, results, miscs, sources):
        assert len({len(x) for x in (tids, specs, results, miscs, sources)}) == 1
        rval = []
        for tid, spec, result, misc, source in zip(tids, specs, results, miscs, sources):
            doc = dict(version=0, tid=tid, spec=spec, result=result, misc=misc,
                       state=source["state"], exp_key=source["exp_key"], owner=source["owner"],
                       book_time=source["book_time"], refresh_time=source["refresh_time"])
            for k, v in (("tid", tid), ("cmd", None), ("from_tid", source["tid"])):
                assert doc["misc"].setdefault(k, v) == v
            rval.append(doc)
        return rval

    def delete_all(self):
        self._dynamic_trials = []
        self.attachments = {}
        self._columnar = {}
        self.refresh()

    def count_by_state_synced(self, arg, trials=None):
        trials = self._trials if trials is None else trials
        if arg in JOB_STATES:
            return len([d for d in trials if d["state"] == arg])
        if hasattr(arg, "__iter__"):
            states = set(arg)
            assert all(x in JOB_STATES for x in states)
            return len([d for d in trials if d["state"] in states])
        raise TypeError(arg)

    def count_by_state_unsynced(self, arg):
        if self._exp_key is not None:
            exp_trials = [t for t in self._dynamic_trials if t["exp_key"] == self._exp_key]
        else:
            exp_trials = self._dynamic_trials
        return self.count_by_state_synced(arg, trials=exp_trials)

    def losses(self, bandit=None):
        if bandit is None:
            return [r.get("loss") for r in self.results]
        return list(map(bandit.loss, self.results, self.specs))

    def statuses(self, bandit=None):
        if bandit is None:
            return [r.get("status") for r in self.results]
        return list(map(bandit.status, self.results, self.specs))

    def average_best_error(self, bandit=None):
        """Loss of the best trial (base.py:563-614, zero-variance case)."""
        if bandit is None:
            results = [r for r in self.results if r["status"] == STATUS_OK]
            loss = [r["loss"] for r in results]
            true_loss = [r.get("true_loss", r["loss"]) for r in results]
        else:
            pairs = [(r, s) for r, s in zip(self.results, self.specs)
                     if bandit.status(r) == STATUS_OK]
            loss = [bandit.loss(r, s) for r, s in pairs]
            true_loss = [bandit.true_loss(r, s) for r, s in pairs]
        if not loss:
            raise ValueError("Empty loss vector")
        return true_loss[int(np.argmin(loss))]

    @property
    def best_trial(self):
        cands = [t for t in self.trials
                 if t["result"]["status"] == STATUS_OK and not np.isnan(t["result"]["loss"])]
        if not cands:
            raise AllTrialsFailed
        losses = [float(t["result"]["loss"]) for t in cands]
        return cands[int(np.nanargmin(losses))]

    @property
    def argmin(self):
        vals = self.best_trial["misc"]["vals"]
        return {k: v[0] for k, v in vals.items() if v}

    def fmin(self, fn, space, algo, max_evals, timeout=None, loss_threshold=None,
             max_queue_len=1, rstate=None, verbose=False, pass_expr_memo_ctrl=None,
             catch_eval_exceptions=False, return_argmin=True, show_progressbar=True,
             early_stop_fn=None):
        from .fmin import fmin
        return fmin(fn, space, algo, max_evals, timeout=timeout, loss_threshold=loss_threshold,
                    trials=self, rstate=rstate, verbose=verbose, max_queue_len=max_queue_len,
                    allow_trials_fmin=False, pass_expr_memo_ctrl=pass_expr_memo_ctrl,
                    catch_eval_exceptions=catch_eval_exceptions, return_argmin=return_argmin,
                    show_progressbar=show_progressbar, early_stop_fn=early_stop_fn)

    # -- columnar history for the suggest path --------------------------------------
    def invalidate_loss_cache(self):
        """Forget the cached losses of finished trials (Columnar.losses): call
        after editing the ``result`` of a document that was already DONE, so
        the next suggest re-reads every loss (the reference re-reads them on
        every suggest, tpe.py:880-882)."""
        for col in getattr(self, "_columnar", {}).values():
            col.n_final = 0

    def columnar(self, labels):
        key = tuple(labels)
        cache = getattr(self, "_columnar", None)
        if cache is None:
            cache = self._columnar = {}
        col = cache.get(key)
        docs = self._dynamic_trials
        if col is None or not col.valid_for(docs) or col.rows > len(docs):
            col = cache[key] = Columnar(key)
        col.extend(docs)
        return col


def trials_from_docs(docs, validate=True, **kwargs):
    rval = Trials(**kwargs)
    if validate:
        rval.insert_trial_docs(docs)
    else:
        rval._insert_trial_docs(docs)
    rval.refresh()
    return rval


class Ctrl(object):
    """Control object for interruptible, checkpoint-able evaluation (base.py:713-767)."""

    info = logger.info
    warn = logger.warning
    error = logger.error
    debug = logger.debug

    def __init__(self, trials, current_trial=None):
        self.trials = Trials() if trials is None else trials
        self.current_trial = current_trial

    def checkpoint(self, r=None):
        assert self.current_trial in self.trials._trials
        if r is not None:
            self.current_trial["result"] = r

    @property
    def attachments(self):
        return self.trials.trial_attachments(trial=self.current_trial)

    def inject_results(self, specs, results, miscs, new_tids=None):
        trial = self.current_trial
        assert trial is not None
        assert len(specs) == len(results) == len(miscs)
        if new_tids is None:
            new_tids = self.trials.new_trial_ids(len(specs))
        new_trials = self.trials.source_trial_docs(tids=new_tids, specs=specs, results=results,
                                                   miscs=miscs, sources=[trial])
        for t in new_trials:
            t["state"] = JOB_STATE_DONE
        return self.trials.insert_trial_docs(new_trials)


class ParamSpec(object):
    """A hyperparameter's prior: distribution name and constant arguments."""

    _ARGNAMES = {
        "uniform": ("low", "high"), "loguniform": ("low", "high"),
        "quniform": ("low", "high", "q"), "qloguniform": ("low", "high", "q"),
        "normal": ("mu", "sigma"), "lognormal": ("mu", "sigma"),
        "qnormal": ("mu", "sigma", "q"), "qlognormal": ("mu", "sigma", "q"),
        "randint": ("low", "high"), "categorical": ("p",),
    }

    def __init__(self, label, node):
        self.label = label
        self.node = node
        self.kind = node.name
        if self.kind not in self._ARGNAMES:
            raise NotImplementedError("unsupported prior %r for %r" % (self.kind, label))
        named = {k: v for k, v in node.named_args if k not in ("rng", "size")}
        names = self._ARGNAMES[self.kind]
        vals = []
        for i, name in enumerate(names):
            if i < len(node.pos_args):
                a = node.pos_args[i]
            elif name in named:
                a = named[name]
            elif self.kind == "randint" and name == "high":
                vals.append(None)
                continue
            else:
                raise TypeError("%s: missing argument %s" % (label, name))
            if any(n.name == "hyperopt_param" for n in pyll.dfs(a)):
                raise NotImplementedError("hyperparameter %r has a prior argument that depends "
                                          "on another hyperparameter" % label)
            vals.append(pyll.rec_eval(a))
        if self.kind == "categorical":
            vals[0] = np.asarray(vals[0], dtype=np.float64)
        self.args = tuple(vals)

    def sample(self, rng):
        """One prior draw (pyll/stochastic.py:36-158) as a plain Python number."""
        k, a = self.kind, self.args
        if k == "uniform":
            return float(rng.uniform(a[0], a[1]))
        if k == "loguniform":
            return float(np.exp(rng.uniform(a[0], a[1])))
        if k == "quniform":
            return float(np.round(rng.uniform(a[0], a[1]) / a[2]) * a[2])
        if k == "qloguniform":
            return float(np.round(np.exp(rng.uniform(a[0], a[1])) / a[2]) * a[2])
        if k == "normal":
            return float(rng.normal(a[0], a[1]))
        if k == "qnormal":
            return float(np.round(rng.normal(a[0], a[1]) / a[2]) * a[2])
        if k == "lognormal":
            return float(np.exp(rng.normal(a[0], a[1])))
        if k == "qlognormal":
            return float(np.round(np.exp(rng.normal(a[0], a[1])) / a[2]) * a[2])
        if k == "randint":
            return int(rng.randint(a[0], a[1]))
        p = a[0]
        return int(np.argmax(rng.multinomial(1, p / p.sum())))


class Domain(object):
    """Search space + objective (base.py:770-1018)."""

    rec_eval_print_node_on_error = False
    pyll_ctrl = pyll.as_apply(Ctrl)

    def __init__(self, fn, expr, workdir=None, pass_expr_memo_ctrl=None, name=None,
                 loss_target=None):
        self.fn = fn
        if pass_expr_memo_ctrl is None:
            self.pass_expr_memo_ctrl = getattr(fn, "fmin_pass_expr_memo_ctrl", False)
        else:
            self.pass_expr_memo_ctrl = pass_expr_memo_ctrl
        self.expr = pyll.as_apply(expr)
        self.params = {}
        self.hp_nodes = {}
        for node in pyll.dfs(self.expr):
            if node.name == "hyperopt_param":
                label = node.pos_args[0].obj
                if label in self.params:
                    raise DuplicateLabel(label)
                self.params[label] = node.pos_args[1]
                self.hp_nodes[label] = node
        self.specs = {lab: ParamSpec(lab, n) for lab, n in self.params.items()}
        self.loss_target = loss_target
        self.name = name
        self.workdir = workdir
        self.s_new_ids = pyll.Literal("new_ids")
        self.s_rng = pyll.Literal("rng-placeholder")
        self.cmd = ("domain_attachment", "FMinIter_Domain")

    # -- conditional structure: which labels are live given decided values ----------
    def reachable(self, decided):
        """(live labels in dfs order, pending) given decided {label: value}.

        Walks the space from the root; a ``switch`` whose index depends on an
        undecided label contributes that label but none of its branches
        (the level structure of vectorize.py:321-363 / pyll/base.py:863-881).
        The result depends only on the decided values of switch-selector
        labels, so it is memoised on those.
        """
        sel_labels = self.__dict__.get("_selector_labels")
        if sel_labels is None:
            sel_labels = set()
            for n in pyll.dfs(self.expr):
                if n.name == "switch":
                    sel_labels.update(m.pos_args[0].obj for m in pyll.dfs(n.pos_args[0])
                                      if m.name == "hyperopt_param")
            self._selector_labels = sel_labels = tuple(sorted(sel_labels))
            self._reach_memo = {}
        try:
            key = tuple((lab, decided[lab]) for lab in sel_labels if lab in decided)
            hit = self._reach_memo.get(key)
        except TypeError:  # unhashable decided value: walk
            key, hit = None, None
        if hit is not None:
            return list(hit)
        live = self._reachable_walk(decided)
        if key is not None and len(self._reach_memo) < 4096:
            self._reach_memo[key] = tuple(live)
        return live

    def _reachable_walk(self, decided):
        live, seen = [], set()
        order = {lab: i for i, lab in enumerate(self.params)}
        stack = [self.expr]
        visited = set()
        while stack:
            node = stack.pop()
            if id(node) in visited:
                continue
            visited.add(id(node))
            if node.name == "hyperopt_param":
                lab = node.pos_args[0].obj
                if lab not in seen:
                    seen.add(lab)
                    live.append(lab)
                continue
            if node.name == "switch":
                sel = node.pos_args[0]
                labs = [n.pos_args[0].obj for n in pyll.dfs(sel) if n.name == "hyperopt_param"]
                for lab in labs:
                    if lab not in seen:
                        seen.add(lab)
                        live.append(lab)
                if all(lab in decided for lab in labs):
                    memo = {self.hp_nodes[lab]: decided[lab] for lab in labs}
                    i = pyll.rec_eval(sel, memo=memo)
                    stack.append(node.pos_args[int(i) + 1])
                continue
            stack.extend(reversed(node.inputs()))
        live.sort(key=lambda lab: order[lab])
        return live

    def memo_from_config(self, config):
        memo = {}
        for lab, node in self.hp_nodes.items():
            memo[node] = config.get(lab, pyll.GarbageCollected)
        return memo

    def _bind_ctrl(self, memo, ctrl):
        # Literal(Ctrl) nodes in the space receive the live Ctrl (utils.py
        # use_obj_for_literal_in_memo)
        for node in pyll.dfs(self.expr):
            if isinstance(node, pyll.Literal) and node.obj is Ctrl:
                memo[node] = ctrl
        return memo

    def evaluate(self, config, ctrl, attach_attachments=True):
        memo = self._bind_ctrl(self.memo_from_config(config), ctrl)
        if self.pass_expr_memo_ctrl:
            rval = self.fn(expr=self.expr, memo=memo, ctrl=ctrl)
        else:
            rval = self.fn(pyll.rec_eval(self.expr, memo=memo,
                                         print_node_on_error=self.rec_eval_print_node_on_error))
        return self._result(rval, ctrl, attach_attachments)

    def evaluate_async(self, config, ctrl, attach_attachments=True):
        memo = self._bind_ctrl(self.memo_from_config(config), ctrl)
        if self.pass_expr_memo_ctrl:
            return self.fn(expr=self.expr, memo=memo, ctrl=ctrl)
        return (self.fn, pyll.rec_eval(self.expr, memo=memo,
                                       print_node_on_error=self.rec_eval_print_node_on_error))

    def evaluate_async2(self, rval, ctrl, attach_attachments=True):
        return self._result(rval, ctrl, attach_attachments)

    def _result(self, rval, ctrl, attach_attachments):
        if isinstance(rval, (float, int, np.number)):
            d = {"loss": float(rval), "status": STATUS_OK}
        else:
            d = dict(rval)
            status = d["status"]
            if status not in STATUS_STRINGS:
                raise InvalidResultStatus(d)
            if status == STATUS_OK:
                try:
                    d["loss"] = float(d["loss"])
                except (TypeError, KeyError):
                    raise InvalidLoss(d)
        if attach_attachments:
            for key, val in d.pop("attachments", {}).items():
                ctrl.attachments[key] = val
        return d

    def short_str(self):
        return "Domain{%s}" % str(self.fn)

    def loss(self, result, config=None):
        return result.get("loss", None)

    def loss_variance(self, result, config=None):
        return result.get("loss_variance", 0.0)

    def true_loss(self, result, config=None):
        try:
            return result["true_loss"]
        except KeyError:
            return self.loss(result, config=config)

    def true_loss_variance(self, config=None):
        raise NotImplementedError()

    def status(self, result, config=None):
        return result["status"]

    def new_result(self):
        return {"status": STATUS_NEW}


# ---------------------------------------------------------------------------
# reference-shaped domains (the plug point hyperopt.fmin(algo=...) uses)
# ---------------------------------------------------------------------------
def convert_graph(expr):
    """A pyll graph built by another pyll implementation -- the reference's
    ``hyperopt.pyll`` (pyll/base.py:232-560): nodes with ``name``,
    ``pos_args``, ``named_args``, ``o_len``, ``pure``, literals named
    "literal" with ``obj`` -- rebuilt from this package's Apply / Literal
    nodes, node for node (shared nodes stay shared; iterative, so deep
    graphs do not hit the recursion limit)."""
    memo = {}
    stack = [expr]
    while stack:
        n = stack[-1]
        if id(n) in memo:
            stack.pop()
            continue
        if n.name == "literal":
            memo[id(n)] = pyll.Literal(n.obj)
            stack.pop()
            continue
        kids = list(n.pos_args) + [v for _, v in n.named_args]
        pending = [k for k in kids if id(k) not in memo]
        if pending:
            stack.extend(pending)
            continue
        stack.pop()
        memo[id(n)] = pyll.Apply(n.name, [memo[id(a)] for a in n.pos_args],
                                 [(k, memo[id(v)]) for k, v in n.named_args],
                                 o_len=n.o_len, pure=n.pure)
    return memo[id(expr)]


def as_domain(domain):
    """The suggest engine's view of ``domain``.

    This package's Domain (anything with ``specs`` and ``reachable``) is used
    as is.  A reference-shaped Domain -- hyperopt's own (base.py:783-870),
    which ``hyperopt.fmin`` hands to its ``algo`` callable (fmin.py:268-270)
    -- is converted once: its ``expr`` graph rebuilt with this package's
    nodes (``convert_graph``), the same labels, prior kinds and arguments,
    and the same conditional structure; ``cmd`` / ``workdir`` /
    ``new_result`` stay the original's.  The conversion is cached on the
    original object."""
    if hasattr(domain, "specs") and hasattr(domain, "reachable"):
        return domain
    d = getattr(domain, "__dict__", None)
    conv = d.get("_hyperopt_amd_domain") if d is not None else None
    if conv is None:
        conv = Domain(getattr(domain, "fn", None), convert_graph(domain.expr),
                      workdir=getattr(domain, "workdir", None),
                      pass_expr_memo_ctrl=getattr(domain, "pass_expr_memo_ctrl", None),
                      name=getattr(domain, "name", None),
                      loss_target=getattr(domain, "loss_target", None))
        if hasattr(domain, "cmd"):
            conv.cmd = domain.cmd
        if hasattr(domain, "new_result"):
            conv.new_result = domain.new_result
        if set(getattr(domain, "params", conv.params)) != set(conv.params):
            raise ValueError("domain conversion lost labels: %s vs %s"
                             % (sorted(domain.params), sorted(conv.params)))
        if d is not None:
            d["_hyperopt_amd_domain"] = conv
    return conv
