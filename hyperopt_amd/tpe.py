"""Tree-of-Parzen-Estimators suggest on MI355X: drop-in for hyperopt.tpe.suggest.

    fmin(fn, space, algo=hyperopt_amd.tpe.suggest, ...)
    algo = functools.partial(tpe.suggest, n_EI_candidates=2**20, gamma=0.25)

Same signature, defaults, startup rule, history rules and returned document
as the reference (hyperopt/tpe.py:837-964):
  * per-tid best loss, ``from_tid`` aliasing, None -> +inf (tpe.py:874-896);
  * fewer than ``n_startup_jobs`` distinct tids -> random search from the
    priors, drawn on the GPU (rand.suggest_device; tpe.py:909-911);
  * the below set is the best min(ceil(gamma*sqrt(T)), 25) tids (tpe.py:637);
  * every live label gets ``n_EI_candidates`` candidates drawn from its below
    posterior, scored by l(x)/g(x), and the argmax is kept (tpe.py:649-658);
  * one document for ``new_ids[0]`` with ``randint(low, high)`` offsets
    re-applied (tpe.py:945-964).
Differences (documented in DESIGN.md): candidates come from counter-based
Philox streams (the reference's RandomState streams cannot be reproduced),
ties in sorts are stable, and the numeric work runs on the GPU through
``hyperopt_amd.engine`` -- there is no CPU fallback.

Extra keyword arguments: ``linear_forgetting`` (25), ``precision`` (None =
auto: float64 when n_EI_candidates x history is small, float32 otherwise;
or 32 / 64; env HYPEROPT_AMD_PRECISION).  Under torch.distributed each rank
scores its share of the candidates and the winners are combined with an
all-gather + device max-loc (hyperopt_amd/dist.py).
"""
from __future__ import annotations

import functools
import gc
import itertools
import logging
import os
import time

import numpy as np

from . import _lib as _L
from . import dist as hdist
from . import rand
from .base import as_domain, doc_loss, foreign_columnar
from .engine import (DEFAULT_LF, Engine, LabelResult, LabelWork, WorkBatch, _lattice_range,
                     _params)

logger = logging.getLogger(__name__)

EPS = 1e-12
_default_prior_weight = 1.0
_default_n_EI_candidates = 24
_default_gamma = 0.25
_default_n_startup_jobs = 20
_default_linear_forgetting = DEFAULT_LF

_engines = {}
USE_DEVICE_HISTORY = True  # gather observation lists from the HBM mirror (LevelInputs)
SUGGEST_MANY_CHUNKS = 4       # suggest_many: studies per launch = max(MIN_CHUNK, n / CHUNKS)
SUGGEST_MANY_MIN_CHUNK = 64   # (env HYPEROPT_AMD_CHUNK overrides)


def engine(slot=0):
    """The Engine of the current device (created on first use); ``slot`` 1 is a
    second engine with its own buffers, which suggest_many alternates with the
    first so one batch can run while the next is prepared."""
    import torch
    dev = torch.cuda.current_device()
    eng = _engines.get((dev, slot))
    if eng is None:
        eng = _engines[(dev, slot)] = Engine(torch.device("cuda", dev))
    return eng


@functools.lru_cache(maxsize=1 << 16)
def _label_hash(label):
    """FNV-1a of the label (cached: labels repeat on every call)."""
    h = 0xCBF29CE484222325
    for ch in str(label).encode():
        h = ((h ^ ch) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _mix64(h):
    """splitmix64 finaliser."""
    h ^= h >> 30
    h = (h * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    h ^= h >> 27
    h = (h * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return h ^ (h >> 31)


def label_key(seed, label):
    """64-bit Philox key for (suggest seed, label): the label's FNV-1a hash
    xor the mixed seed, through a splitmix finaliser."""
    return _mix64(_label_hash(label) ^ _mix64((int(seed) * 0x9E3779B97F4A7C15 + 1)
                                             & 0xFFFFFFFFFFFFFFFF))


def _mix64_np(h):
    h = h ^ (h >> np.uint64(30))
    h = h * np.uint64(0xBF58476D1CE4E5B9)
    h = h ^ (h >> np.uint64(27))
    h = h * np.uint64(0x94D049BB133111EB)
    return h ^ (h >> np.uint64(31))


@functools.lru_cache(maxsize=4096)
def _label_hashes(labels):
    """FNV-1a hashes of a tuple of labels, as a read-only uint64 array."""
    h = np.fromiter((_label_hash(lab) for lab in labels), np.uint64, len(labels))
    h.flags.writeable = False
    return h


def label_keys_array(seed, labels):
    """label_key(seed, lab) for every label at once, as a uint64 array (uint64
    array arithmetic wraps like the masked Python integers)."""
    s = np.uint64(_mix64((int(seed) * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF))
    try:
        h = _label_hashes(tuple(labels))
    except TypeError:  # unhashable labels
        h = np.fromiter((_label_hash(lab) for lab in labels), np.uint64, len(labels))
    with np.errstate(over="ignore"):
        return _mix64_np(h ^ s)


def label_keys(seed, labels):
    """label_key(seed, lab) for every label at once, as a list of ints."""
    return label_keys_array(seed, labels).tolist()


class History(object):
    """The history tpe.suggest conditions on, one row per distinct tid.

    ``vals`` / ``active`` (T, L) are views or gathers of the trials' columnar
    cache when there is one (``col`` + ``rows``: row i of the history is
    columnar row ``rows[i]``, or row i itself when ``rows`` is None), so the
    device path can gather from the HBM mirror of the same rows instead.
    """

    def __init__(self, tids, losses, obs_tids, vals=None, active=None, col=None, rows=None):
        self.tids = tids          # (T,) loss tids, sorted
        self.losses = losses      # (T,) float64, +inf for unfinished/failed
        self.obs_tids = obs_tids  # (T,) the tid each row's observations are filed under
        self.col = col            # base.Columnar or None
        self.rows = rows          # (T,) int64 columnar rows, or None (= arange(T))
        self._vals, self._active = vals, active

    def _gather(self):
        T = self.tids.size
        if self.rows is None:
            self._vals, self._active = self.col.vals[:T], self.col.active[:T]
        else:
            self._vals, self._active = self.col.vals[self.rows], self.col.active[self.rows]

    @property
    def vals(self):
        if self._vals is None:
            self._gather()
        return self._vals    # (T, L) float64

    @property
    def active(self):
        if self._active is None:
            self._gather()
        return self._active  # (T, L) bool

    def label_counts(self):
        """Active observations per label over the history's rows."""
        if self.col is not None and self.rows is None and self.tids.size == self.col.rows:
            return self.col.n_active
        return self.active.sum(0)


def collect_history(trials, labels):
    """Best document per tid, sorted by tid (tpe.py:874-896), as columns.

    Reference rule, kept exactly: ``best_docs_loss.setdefault(tid, loss)``
    then ``if loss <= best_docs_loss[tid]`` -- so a tid whose first document
    has a NaN loss never gets a document and drops out of the history.
    """
    docs = trials.trials
    if hasattr(trials, "columnar"):
        col = trials.columnar(labels)
    else:  # the reference's Trials (fmin(algo=hyperopt_amd.tpe.suggest)): a cache beside it
        if not isinstance(docs, list):
            docs = list(docs)
        col = foreign_columnar(trials, docs, labels)
    n = len(docs)
    if col is not None and n == col.rows and col.keys_increasing:
        # trials.trials is every cached row (a filtered subsequence of
        # _dynamic_trials of the same length) and each tid has one document;
        # finished documents' losses come from the cache (Columnar.losses)
        losses = col.losses()
        keep = ~np.isnan(losses)
        if keep.all():  # (views: the cache only appends past row n during the call)
            return History(col.key_tid[:n], losses, col.obs_tid[:n], col=col)
        rows = np.flatnonzero(keep)
        return History(col.key_tid[rows], losses[rows], col.obs_tid[rows], col=col, rows=rows)
    tids, losses, obs_tids, bdocs = _best_docs(docs)
    if col is not None and all(id(d) in col.row_of for d in bdocs):
        rows = np.fromiter((col.row_of[id(d)] for d in bdocs), dtype=np.int64, count=len(bdocs))
        return History(tids, losses, obs_tids, col=col, rows=rows)
    return walk_history(docs, labels, (tids, losses, obs_tids, bdocs))


def _best_docs(docs):
    """Per-tid best document, sorted by tid (tpe.py:874-896)."""
    best_loss, best_doc = {}, {}
    for doc in docs:
        tid = doc["misc"].get("from_tid", doc["tid"])
        loss = doc_loss(doc)
        if loss <= best_loss.setdefault(tid, loss):
            best_loss[tid] = loss
            best_doc[tid] = doc
    tids = sorted(best_doc)
    bdocs = [best_doc[t] for t in tids]
    losses = np.array([best_loss[t] for t in tids], dtype=np.float64)
    obs_tids = np.array([d["misc"]["tid"] for d in bdocs], dtype=np.int64)
    return np.asarray(tids, dtype=np.int64), losses, obs_tids, bdocs


def walk_history(docs, labels, best=None):
    """The history by the reference's walk over every document and label
    (tpe.py:874-896 + miscs_to_idxs_vals, base.py:200-214), no cache: the
    fallback of collect_history, and what its cached forms must equal."""
    tids, losses, obs_tids, bdocs = _best_docs(docs) if best is None else best
    L = len(labels)
    index = {lab: j for j, lab in enumerate(labels)}
    vals = np.full((len(bdocs), L), np.nan)
    active = np.zeros((len(bdocs), L), bool)
    for r, d in enumerate(bdocs):
        for lab, vv in d["misc"]["vals"].items():
            j = index.get(lab)
            if j is not None and len(vv):
                vals[r, j] = float(vv[0])
                active[r, j] = True
    return History(tids, losses, obs_tids, vals, active)


def split_masks(hist, gamma, gamma_cap=DEFAULT_LF):
    """Row masks of the below / above sets (ap_split_trials, tpe.py:623-646).

    Membership is decided on loss tids, observations are matched on the tid
    they are filed under -- the reference's behaviour for from_tid documents.
    """
    T = hist.losses.size
    n_below = min(int(np.ceil(gamma * np.sqrt(T))), gamma_cap)
    below_rows = _smallest_rows(hist.losses, n_below)
    # (a columnar history over cached rows without from_tid rows needs no compare)
    same = hist.col is not None and hist.col.n_alias == 0 and hist.tids.size == T and \
        hist.obs_tids.size == T
    if same or (hist.obs_tids.size == T and np.array_equal(hist.obs_tids, hist.tids)):
        isb = np.zeros(T, bool)  # no from_tid aliasing: rows are the tids
        isb[below_rows] = True
        return isb, ~isb
    below = np.zeros(T, bool)
    below[below_rows] = True
    return np.isin(hist.obs_tids, hist.tids[below]), np.isin(hist.obs_tids, hist.tids[~below])


def _smallest_rows(losses, n):
    """Rows of argsort(losses, kind="stable")[:n] in ascending row order, one
    pass in C for the suggest path's small n (tpe_smallest_rows)."""
    T = losses.size
    if n <= 0:
        return np.zeros(0, np.int64)
    if n >= T:
        return np.arange(T)
    losses = np.ascontiguousarray(losses, dtype=np.float64)
    out = np.empty(n, np.int64)
    got = _L.load().tpe_smallest_rows(losses.ctypes.data, T, n, out.ctypes.data)
    if got != n:
        raise _L.TpeHipError("tpe_smallest_rows returned %d" % got)
    return out


FP32_MIN_CAND = 1 << 16  # engine.TABLE_MIN_CAND: the cell-table path's threshold


def _precision(precision, n_ei, T):
    if precision is None:
        env = os.environ.get("HYPEROPT_AMD_PRECISION", "")
        if env:
            precision = int(env)
        else:
            # fp32 only where the table path runs (its argmax is made exact by
            # the band re-score, tpe_band_rescore); every smaller or cheaper
            # level is scored exactly in fp64
            precision = 32 if (n_ei >= FP32_MIN_CAND and n_ei * max(T, 1) > (1 << 24)) else 64
    if precision not in (32, 64):
        raise ValueError("precision must be 32 or 64", precision)
    return precision


def _decode(spec, value):
    """Engine value -> (value used by switches, value stored in the trial)."""
    if spec.kind == "randint":
        k = int(round(value))
        offset = int(spec.args[0]) if spec.args[1] is not None else 0
        return k, k + offset  # tpe.py:945-948
    if spec.kind == "categorical":
        k = int(round(value))
        return k, k
    return float(value), float(value)


def _addr(a):
    """Data address of a numpy array (for ctypes void* arguments)."""
    return a.__array_interface__["data"][0]


class LevelInputs(object):
    """The observation inputs of every label for Engine.run.

    When the trials carry a columnar cache (``History.col``) the lists are
    gathered on the device: the cache is mirrored in HBM
    (``Columnar.device_history``, appended with new rows only) and a suggest
    uploads one split flag per history row (1 below, 0 above, 2 neither --
    from_tid rows outside both sets) plus, when the history is not every cached
    row, the row list; only the <= 25 below rows are read on the host (their
    sizes size the fit).  Without a cache (foreign Trials classes) the lists
    are sliced on the host and uploaded.  Both give bit-identical lists in tid
    order (tests/test_gpu_history.py).
    """

    def __init__(self, hist, isb, isa, eng=None, device=True):
        self.hist, self.isb, self.isa = hist, isb, isa
        self.device = bool(device) and hist.col is not None and eng is not None
        self.run_kwargs = {}
        if not self.device:
            return
        c = hist.col
        T = hist.tids.size
        below_pos = np.flatnonzero(isb)
        every_above = T - below_pos.size == int(np.count_nonzero(isa))
        if every_above:  # every row below (1) or above (0): the mask's bytes are the flags
            flags = np.ascontiguousarray(isb).view(np.uint8)
        else:
            flags = np.full(T, 2, np.uint8)
            flags[isa] = 0
            flags[isb] = 1
        crow = below_pos if hist.rows is None else hist.rows[below_pos]
        self.vb, self.ab = c.vals[crow], c.active[crow]
        self.nb = nb = self.ab.sum(0)
        if every_above:
            self.n_above = hist.label_counts() - nb
        else:
            self.n_above = hist.active[isa].sum(0)
        rows = None if hist.rows is None else hist.rows.astype(np.int32)
        self.run_kwargs = dict(history=c.device_history(eng), rows=rows, is_below=flags)

    @classmethod
    def fast(cls, hist, gamma, eng, gamma_cap=DEFAULT_LF):
        """split_masks + LevelInputs in one C pass (tpe_split_inputs) for the
        common case -- a columnar history over every cached row, no from_tid
        aliasing, device mode -- or None (the caller takes the general path).
        Same split, flags and counts (tests/test_host_api.py)."""
        c = hist.col
        if c is None or hist.rows is not None or c.n_alias or eng is None:
            return None
        T = hist.tids.size
        if T != c.rows or hist.obs_tids.size != T:
            return None
        L = len(c.labels)
        n_below = min(int(np.ceil(gamma * np.sqrt(T))), gamma_cap)
        losses = np.ascontiguousarray(hist.losses, dtype=np.float64)
        act = c.active  # (cap, L) bool, row-major; rows [0, T) are the history
        isb = np.empty(T, np.uint8)
        rows_b = np.empty(max(n_below, 1), np.int64)
        nb = np.empty(L, np.int64)
        na = np.empty(L, np.int64)
        # (raw addresses: numpy's .ctypes builds a helper object per access,
        # ~1 us each -- seven per study add up in suggest_many)
        got = _L.load().tpe_split_inputs(_addr(losses), T, n_below, _addr(act), L,
                                         _addr(c.n_active), _addr(isb), _addr(rows_b), _addr(nb),
                                         _addr(na))
        if got != min(n_below, T):
            raise _L.TpeHipError("tpe_split_inputs returned %d" % got)
        self = cls.__new__(cls)
        self.hist, self.isb, self.isa = hist, isb.view(bool), None
        self.device = True
        rows_b = rows_b[:got]
        self.vb, self.ab = c.vals[rows_b], c.active[rows_b]
        self.nb, self.n_above = nb, na
        self.run_kwargs = dict(history=c.device_history(eng), rows=None, is_below=isb)
        return self

    def work(self, label, spec, j, **kw):
        if self.device:
            return LabelWork(label=label, kind=spec.kind, args=spec.args,
                             obs_below=self.vb[self.ab[:, j], j], obs_above=None, col=j,
                             n_above=int(self.n_above[j]), **kw)
        act, v = self.hist.active[:, j], self.hist.vals[:, j]
        return LabelWork(label=label, kind=spec.kind, args=spec.args,
                         obs_below=v[act & self.isb], obs_above=v[act & self.isa], **kw)


def suggest(new_ids, domain, trials, seed, prior_weight=_default_prior_weight,
            n_startup_jobs=_default_n_startup_jobs, n_EI_candidates=_default_n_EI_candidates,
            gamma=_default_gamma, verbose=True, linear_forgetting=_default_linear_forgetting,
            precision=None):
    """TPE suggest: one new trial document for new_ids[0] (tpe.py:837-964)."""
    t0 = time.time()
    domain = as_domain(domain)  # (hyperopt's own Domain too: fmin(algo=tpe.suggest))
    labels = list(domain.params)
    hist = collect_history(trials, labels)
    if verbose:
        if hist.tids.size:
            logger.info("TPE using %i/%i trials with best loss %f" % (
                hist.tids.size, len(trials), np.nanmin(hist.losses)))
        else:
            logger.info("TPE using 0 trials")
    if hist.tids.size < n_startup_jobs:  # tpe.py:909-911, prior draws on the GPU
        return rand.suggest_device(new_ids, domain, trials, seed)

    first_new_id = new_ids[0]
    prec = _precision(precision, n_EI_candidates, hist.tids.size)
    rank, ws = hdist.world()
    n_ei = max(int(n_EI_candidates), 0)
    col = {lab: j for j, lab in enumerate(labels)}

    walk, stored = {}, {}
    live = []
    if n_ei > 0:
        eng = engine()
        hm = eng.host_marks  # (diagnostic phase marks, Engine.host_marks)
        if hm is not None:
            hm.append(("suggest:split", time.perf_counter()))
        obs = LevelInputs.fast(hist, gamma, eng) if USE_DEVICE_HISTORY else None
        if obs is None:
            isb, isa = split_masks(hist, gamma)
            obs = LevelInputs(hist, isb, isa, eng, device=USE_DEVICE_HISTORY)
        if hm is not None:
            hm.append(("suggest:inputs", time.perf_counter()))
        while True:
            live = domain.reachable(walk)
            level = [lab for lab in live if lab not in walk]
            if not level:
                break
            # under torch.distributed this rank scores its units of the level
            # (whole labels, or candidate ranges when labels < ranks) and the
            # winners are combined across ranks (hyperopt_amd/dist.py)
            if ws == 1:  # every label whole (dist.plan_units' one-rank plan), cached
                units = _whole_units(len(level), n_ei)
            else:
                units = hdist.plan_units([domain.specs[lab].kind for lab in level], n_ei,
                                         ws)[rank]
            if not units:  # more ranks than shards of this level: nothing here, but
                res = []   # the rank still joins the winners' all-gather below
            elif obs.device and _space_sig(domain) is not None:
                res = _level_batch(eng, domain, obs, level, units, seed, n_ei, col,
                                   prior_weight, linear_forgetting, prec, ws == 1)
            else:
                keys = label_keys(seed, level)
                works = [obs.work(level[i], domain.specs[level[i]], col[level[i]], n_cand=count,
                                  key=keys[i], cand_base=start, n_total=n_ei)
                         for i, start, count in units]
                res = eng.run(works, prior_weight=prior_weight, lf=linear_forgetting,
                              precision=prec, **obs.run_kwargs)
            if ws > 1:
                best = hdist.gather_best(len(level), [(u[0], r) for u, r in zip(units, res)])
                values = [b[2] for b in best]
            elif isinstance(res, list) and res and isinstance(res[0], LabelResult):
                values = [r.value for r in res]
            else:  # (_level_batch on one rank: the winners' values in level order)
                values = res
            for lab, v in zip(level, values):
                walk[lab], stored[lab] = _decode(domain.specs[lab], v)
            if hm is not None:
                hm.append(("suggest:decoded", time.perf_counter()))
    live = set(live)
    misc = {"tid": first_new_id, "cmd": domain.cmd, "workdir": domain.workdir,
            "idxs": {lab: ([first_new_id] if lab in live else []) for lab in labels},
            "vals": {lab: ([stored[lab]] if lab in live else []) for lab in labels}}
    if verbose:
        logger.info("tpe.suggest took %f seconds" % (time.time() - t0))
    return trials.new_trial_docs([first_new_id], [None], [domain.new_result()], [misc])


class SuggestRequest(object):
    """One study's suggest call for ``suggest_many``."""

    def __init__(self, new_ids, domain, trials, seed, **kwargs):
        self.new_ids, self.domain, self.trials, self.seed = new_ids, domain, trials, seed
        self.kwargs = kwargs


_SPACE_IDS = {}   # (label, kind, args) tuple of a space -> small int
_LEVELS = {}      # (space id, level labels) -> _Level
_LEVEL_IDS = itertools.count()  # never reused: level ids are part of engine plan keys


def _space_sig(domain):
    """Small int naming a space's (label, kind, prior arguments) list, cached
    on the domain; None when a prior argument is unhashable."""
    d = domain.__dict__
    if "_tpe_space_id" not in d:
        sig = tuple((lab, domain.specs[lab].kind, domain.specs[lab].args) for lab in domain.params)
        try:
            sid = _SPACE_IDS.get(sig)
            if sid is None:
                sid = _SPACE_IDS[sig] = len(_SPACE_IDS)
        except TypeError:
            sid = None
        domain._tpe_space_id = sid
    return d["_tpe_space_id"]


class _Level(object):
    """What a level of a space needs per call, computed once: label columns,
    FNV hashes (label_keys without the per-label Python), and the unbounded
    quantized labels whose lattice range follows the below set."""

    def __init__(self, lid, domain, level):
        self.id = lid
        labels = list(domain.params)
        self.js = np.array([labels.index(lab) for lab in level], np.int64)
        self.h = np.fromiter((_label_hash(lab) for lab in level), np.uint64, len(level))
        self.lat = []
        for i, lab in enumerate(level):
            spec = domain.specs[lab]
            if spec.kind in ("qnormal", "qlognormal"):
                self.lat.append((i, lab, spec))
        # _decode as a plan: (label, 0 continuous / 1 integer, offset)
        self.decode = []
        for lab in level:
            spec = domain.specs[lab]
            off = int(spec.args[0]) if (spec.kind == "randint" and spec.args[1] is not None) \
                else 0
            self.decode.append((lab, 1 if spec.kind in ("randint", "categorical") else 0, off))


def _level_info(domain, level):
    k = (_space_sig(domain), tuple(level))
    lv = _LEVELS.get(k)
    if lv is None:
        if len(_LEVELS) > 4096:
            _LEVELS.clear()
        lv = _LEVELS[k] = _Level(next(_LEVEL_IDS), domain, level)
    return lv


@functools.lru_cache(maxsize=256)
def _whole_units(n, n_ei):
    """dist.plan_units(kinds, n_ei, 1)[0] as a tuple: every label whole."""
    return tuple((i, 0, n_ei) for i in range(n))


@functools.lru_cache(maxsize=256)
def _zero_bases(n):
    z = np.zeros(n, np.int64)
    z.flags.writeable = False
    return z


def _level_batch(eng, domain, obs, level, units, seed, n_ei, col, pw, lf, prec, values=False):
    """One study's level (this rank's units of it) as a WorkBatch on the
    device history: counts from the split, keys from the cached label hashes,
    a structure key of a few small ints -- LabelWork objects only the first
    time the structure is seen.  Returns one LabelResult per unit, or with
    ``values`` (one rank: every unit a whole label, in level order) just the
    winners' values."""
    lv = _level_info(domain, level)
    whole = isinstance(units, tuple) and units is _whole_units(len(level), n_ei)
    if whole:  # (one rank: every label, in level order)
        idx = None
        js = lv.js
    else:
        idx = np.fromiter((u[0] for u in units), np.int64, len(units))
        js = lv.js[idx]
    lat = ()
    if lv.lat:
        lat = tuple(_lattice_range(obs.work(lab, spec, int(lv.js[i])),
                                   _params(spec.kind, spec.args)) for i, lab, spec in lv.lat)
    s = np.uint64(_mix64((int(seed) * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF))
    with np.errstate(over="ignore"):
        keys = _mix64_np((lv.h if whole else lv.h[idx]) ^ s)

    def materialize():
        specs = domain.specs
        return [obs.work(level[i], specs[level[i]], col[level[i]], n_cand=count,
                         key=int(k), cand_base=start, n_total=n_ei)
                for (i, start, count), k in zip(units, keys.tolist())]
    # (the key names the units: a token for the one-rank plan -- tuples do
    # not cache their hash, and this key is hashed a few times per call)
    batch = WorkBatch(("suggest", lv.id, ("whole", len(units)) if whole else tuple(units), n_ei,
                       lat), obs.nb[js],
                      obs.n_above[js], keys,
                      _zero_bases(len(units)) if whole else [u[1] for u in units], materialize)
    r = eng.run(batch, prior_weight=pw, lf=lf, precision=prec, **obs.run_kwargs)
    if values:
        return r.value.tolist()
    return [LabelResult(level[u[0]], ix, v, sc, ns) for u, ix, v, sc, ns in
            zip(units, r.index.tolist(), r.value.tolist(), r.score.tolist(),
                r.n_scored.tolist())]


def _run_columnar(eng, items, pw, lf, prec, defer=False):
    """One engine launch for a batch of studies' levels as a WorkBatch: the
    per-label work is a few array operations per study (counts from the
    LevelInputs, keys from cached hashes); LabelWork objects are only built
    the first time a batch structure is seen.  Returns the winners' values
    per item."""
    hists, struct, nb, na, hh, ss, cb, sizes = [], [], [], [], [], [], [], []
    for st, level in items:
        obs = st["obs"]
        rk = obs.run_kwargs
        hists.append((rk["history"], rk["rows"], rk["is_below"]))
        lv = _level_info(st["rq"].domain, level)
        lat = ()
        if lv.lat:
            lat = tuple(_lattice_range(obs.work(lab, spec, int(lv.js[i])),
                                       _params(spec.kind, spec.args)) for i, lab, spec in lv.lat)
        struct.append((lv.id, st["count"], st["n_ei"], lat))
        nb.append(obs.nb[lv.js])
        na.append(obs.n_above[lv.js])
        hh.append(lv.h)
        ss.append(_mix64((int(st["rq"].seed) * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF))
        cb.append(st["start"])
        sizes.append(len(level))
    sizes = np.asarray(sizes, np.int64)
    with np.errstate(over="ignore"):
        keys = _mix64_np(np.concatenate(hh) ^ np.repeat(np.asarray(ss, np.uint64), sizes))

    def materialize():
        out = []
        for h, (st, level) in enumerate(items):
            specs, col = st["rq"].domain.specs, st["col"]
            for lab, k in zip(level, label_keys(st["rq"].seed, level)):
                w = st["obs"].work(lab, specs[lab], col[lab], n_cand=st["count"], key=k,
                                   cand_base=st["start"], n_total=st["n_ei"])
                w.hist = h
                out.append(w)
        return out
    batch = WorkBatch(tuple(struct), np.concatenate(nb), np.concatenate(na), keys,
                      np.repeat(np.asarray(cb, np.int64), sizes), materialize)
    res = eng.run(batch, prior_weight=pw, lf=lf, precision=prec, histories=hists, defer=defer)
    if defer:
        return res
    vals = res.value.tolist()
    out, a = [], 0
    for n in sizes.tolist():
        out.append(vals[a:a + n])
        a += n
    return out


def _run_works(eng, items, pw, lf, prec, dev, combine):
    """The general path: one LabelWork per label (host lists or histories),
    winners combined across ranks when the candidates are sharded."""
    works, kw_run, hists = [], {}, []
    for h, (st, level) in enumerate(items):
        specs, col = st["rq"].domain.specs, st["col"]
        for lab, k in zip(level, label_keys(st["rq"].seed, level)):
            w = st["obs"].work(lab, specs[lab], col[lab], n_cand=st["count"], key=k,
                               cand_base=st["start"], n_total=st["n_ei"])
            w.hist = h
            works.append(w)
        if dev:  # one history per study of the batch
            rk = st["obs"].run_kwargs
            hists.append((rk["history"], rk["rows"], rk["is_below"]))
    if dev:
        kw_run["histories"] = hists
    res = eng.run(works, prior_weight=pw, lf=lf, precision=prec, **kw_run)
    if combine:
        hdist.allreduce_best(res)
    out, a = [], 0
    for _, level in items:
        out.append([r.value for r in res[a:a + len(level)]])
        a += len(level)
    return out


def suggest_many(requests, shard_studies=False):
    """Batched suggest over many independent studies; see _suggest_many.  The
    cyclic garbage collector is paused for the call: a batch allocates a few
    objects per label and study, and with many studies' trial documents alive
    a full collection triggered mid-call scans them all (tens of ms)."""
    enabled = gc.isenabled()
    gc.disable()
    try:
        return _suggest_many(requests, shard_studies)
    finally:
        if enabled:
            gc.enable()


def _suggest_many(requests, shard_studies=False):
    """Batched suggest over many independent studies.

    Every study runs tpe.suggest's exact logic, but the labels of all studies
    that are live at the same conditional depth are scored in ONE engine launch
    (one fit launch, one scoring launch per label kind).  Studies differ in
    history, space and options; each keeps its own Philox keys.  With
    ``shard_studies`` under torch.distributed, rank r serves studies r::world
    (no collective on the data path) and returns None for the others.
    Returns one list of trial documents per request.

    Studies whose trials carry a columnar cache are gathered on the device:
    each keeps its own HBM mirror (Columnar.device_history) and a batch's lists
    come from one tpe_gather_obs_multi launch over all of them.
    """
    rank, ws = hdist.world()
    out = [None] * len(requests)
    todo = [(qi, rq) for qi, rq in enumerate(requests)
            if not (shard_studies and ws > 1 and qi % ws != rank)]
    columnar = ws == 1 or shard_studies  # no cross-rank combine of the winners
    chunk = int(os.environ.get("HYPEROPT_AMD_CHUNK", "0")) or \
        max(SUGGEST_MANY_MIN_CHUNK, -(-len(todo) // SUGGEST_MANY_CHUNKS))
    states = []
    pend = []  # launched batches not yet decoded: (items, values or _Pending)
    turn = itertools.count()

    def make_state(qi, rq):
        kw = dict(prior_weight=_default_prior_weight, n_startup_jobs=_default_n_startup_jobs,
                  n_EI_candidates=_default_n_EI_candidates, gamma=_default_gamma,
                  linear_forgetting=_default_linear_forgetting, precision=None)
        kw.update({k: v for k, v in rq.kwargs.items() if k != "verbose"})
        rq.domain = as_domain(rq.domain)
        labels = list(rq.domain.params)
        hist = collect_history(rq.trials, labels)
        if hist.tids.size < kw["n_startup_jobs"]:
            out[qi] = rand.suggest_device(rq.new_ids, rq.domain, rq.trials, rq.seed)
            return None
        n_ei = max(int(kw["n_EI_candidates"]), 0)
        start, count = (0, n_ei) if (shard_studies or ws == 1) else hdist.shard(n_ei, rank, ws)
        eng = engine() if n_ei > 0 else None
        obs = LevelInputs.fast(hist, kw["gamma"], eng) if USE_DEVICE_HISTORY else None
        if obs is None:
            isb, isa = split_masks(hist, kw["gamma"])
            obs = LevelInputs(hist, isb, isa, eng, device=USE_DEVICE_HISTORY)
        return dict(qi=qi, rq=rq, kw=kw, labels=labels, hist=hist, obs=obs,
                    col={lab: j for j, lab in enumerate(labels)}, walk={}, stored={},
                    live=[], start=start, count=count, n_ei=n_ei, done=n_ei == 0,
                    prec=_precision(kw["precision"], n_ei, hist.tids.size))

    def finish(items, values):
        if not isinstance(values, list):
            r = values.result().value.tolist()
            values, a = [], 0
            for _, level in items:
                values.append(r[a:a + len(level)])
                a += len(level)
        for (st, level), vals in zip(items, values):
            walk, stored, dom = st["walk"], st["stored"], st["rq"].domain
            if _space_sig(dom) is None:  # (no cached level plan for this space)
                for lab, v in zip(level, vals):
                    walk[lab], stored[lab] = _decode(dom.specs[lab], v)
                continue
            for (lab, mode, off), v in zip(_level_info(dom, level).decode, vals):
                if mode == 0:  # a continuous label: the value itself
                    walk[lab] = stored[lab] = float(v)
                else:  # randint (offset re-applied, tpe.py:945-948) / categorical
                    k = int(round(v))
                    walk[lab], stored[lab] = k, k + off

    # Level by level; within a level the studies go in chunks, each chunk's
    # batches launched without waiting (Engine.run defer=True, two engines
    # taking turns), so the host prepares chunk c+1 while chunk c runs.
    first = True
    while True:
        src = todo if first else [st for st in states if not st["done"]]
        if not src:
            break
        for c0 in range(0, len(src), chunk):
            if first:
                sts = [st for st in (make_state(qi, rq) for qi, rq in src[c0:c0 + chunk])
                       if st is not None]
                states.extend(sts)
            else:
                sts = src[c0:c0 + chunk]
            batches = {}  # (prior_weight, lf, precision, device) -> [(state, level)]
            for st in sts:
                if st["done"]:
                    continue
                live = st["rq"].domain.reachable(st["walk"])
                st["live"] = live
                level = [lab for lab in live if lab not in st["walk"]]
                if not level:
                    st["done"] = True
                    continue
                key = (st["kw"]["prior_weight"], st["kw"]["linear_forgetting"], st["prec"],
                       st["obs"].device)
                batches.setdefault(key, []).append((st, level))
            for (pw, lf, prec, dev), items in batches.items():
                if dev and columnar and all(_space_sig(st["rq"].domain) is not None
                                            for st, _ in items):
                    eng = engine(next(turn) % 2)
                    values = _run_columnar(eng, items, pw, lf, prec, defer=True)
                else:
                    values = _run_works(engine(), items, pw, lf, prec, dev,
                                        ws > 1 and not shard_studies)
                pend.append((items, values))
                while len(pend) > 1:
                    finish(*pend.pop(0))
        while pend:
            finish(*pend.pop(0))
        first = False
    for st in states:
        rq, live = st["rq"], set(st["live"])
        tid = rq.new_ids[0]
        misc = {"tid": tid, "cmd": rq.domain.cmd, "workdir": rq.domain.workdir,
                "idxs": {lab: ([tid] if lab in live else []) for lab in st["labels"]},
                "vals": {lab: ([st["stored"][lab]] if lab in live else [])
                         for lab in st["labels"]}}
        out[st["qi"]] = rq.trials.new_trial_docs([tid], [None], [rq.domain.new_result()], [misc])
    return out

