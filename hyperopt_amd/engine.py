"""GPU engine for one level of TPE labels: Parzen fit, sampling, scoring, argmax.

This is the product path behind ``hyperopt_amd.tpe.suggest``.  One call to
``Engine.run`` takes every label that is active at one level of the search
space (all labels, for a flat space) and runs, on the current torch stream:

    tpe_parzen_fit        adaptive_parzen_normal for every below/above set
    tpe_cat_posterior     randint / categorical pseudocount posteriors
    tpe_table_build       fp32: per-cell Taylor expansions of both mixtures and a
                          cubic of the score per cell
    tpe_score_table_fast  fp32: sample + score cubic lookup + argmax (suggest path)
    tpe_score_table       fp32: sample/read + cell lookup + 2 polynomials + argmax
                          (injected candidates, per-candidate log-densities)
    tpe_score_continuous  unquantized labels: sample + GMM1/LGMM1_lpdf + argmax
    tpe_lattice_*         quantized labels: sample -> distinct values -> score
    tpe_score_categorical categorical labels: sample + lookup + argmax

with one host->device upload of the packed inputs and one device->host copy of
the per-label winners.  Reference: hyperopt/tpe.py:661-757 (build_posterior),
:837-964 (suggest).  There is no CPU fallback: every numeric step above is a
HIP kernel from libtpe_hip.so.
"""
from __future__ import annotations

import ctypes
import functools
import math
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _lib as L
from . import dist as hdist

EPS = 1e-12  # tpe.py:32
DEFAULT_LF = 25  # tpe.py:36
DRAW32_MAX_SLOT = 1 << 12  # fp32 lattice draws only while |k| <= 2^12
LATTICE_CAP = 1 << 22  # max lattice slots per quantized label before the dense fallback
LAT_PACK_MAX = 1 << 16  # lattice slots of a level initialised through the upload (else memset)
TABLE_CAP = 1 << 15  # cells per label in the cell-table path (128 B each)
TABLE_MIN_CAND = 1 << 16  # auto scorer: table path from this many candidates per label
BAND_TILE_CAP = 256  # per scorer tile: band entries kept (tpe_score_table_fast's tile_cap, <= 256)
LAT_PREFIX = 1 << 16  # lattice argmax: candidates drawn before the early decision
LAT_SUGGEST_MAX_SLOTS = 1 << 10  # ... for lattices of at most this many slots (all scored)
PRUNED64_MIN_COMP = 256  # fp64: pruned exact scorer from this many above components
SCORERS = ("auto", "dense", "sorted", "table")
SIDE_KINDS = ("lat", "qfb", "qinj", "cat")  # groups scored on the side stream
HOST_EVENTS = ("result",)  # events the host waits on (system-scope release kept)
_ALIGN = 256

CONTINUOUS = ("uniform", "quniform", "loguniform", "qloguniform",
              "normal", "qnormal", "lognormal", "qlognormal")
CATEGORICAL = ("randint", "categorical")
# unquantized continuous kinds: scored by an fp32 argmax when the candidates
# are injected or per-candidate outputs are asked for (Engine.run re-decides them)
EXACT32_KINDS = ("uniform", "loguniform", "normal", "lognormal")


@dataclass(slots=True)
class LabelWork:
    """One label's inputs for one suggest level."""
    label: str
    kind: str                 # prior distribution name (hp node name)
    args: tuple               # prior arguments, positional
    obs_below: np.ndarray     # below-set observations, tid order (tpe.py:641)
    obs_above: np.ndarray     # above-set observations, tid order (tpe.py:644)
    n_cand: int = 24          # candidates scored on this device
    key: int = 0              # Philox key (seed mixed with the label)
    cand_base: int = 0        # global index of this device's first candidate
    cand: Optional[np.ndarray] = None  # injected candidates (values / category ids)
    # history mode (Engine.run(history=...)): the observation lists are
    # gathered on the device from column `col`; obs_below is still given on
    # the host (it is small) and obs_above is None with its size in n_above
    col: Optional[int] = None
    n_above: int = 0
    hist: int = 0             # Engine.run(histories=...): index of this work's history
    # candidates of the label over all devices (0: n_cand).  The automatic
    # scorer choice follows it, so every shard of a label runs the same
    # kernel and the winner does not depend on the number of ranks
    n_total: int = 0


class WorkBatch(object):
    """The labels of many studies for one Engine.run, as columns -- the
    batched-suggest fast path (tpe.suggest_many).  ``key`` names the
    structure (hashable; equal keys must mean equal kinds, prior arguments,
    candidate counts, history columns and slots, lattice ranges, in order),
    the arrays carry the per-call values in work order, and ``materialize()``
    returns the equivalent LabelWork list, used when the structure is new.
    Requires ``history`` or ``histories``; Engine.run then returns a BatchResult."""
    __slots__ = ("key", "n_below", "n_above", "keys", "cand_base", "materialize")

    def __init__(self, key, n_below, n_above, keys, cand_base, materialize):
        self.key = key
        self.n_below = np.asarray(n_below, np.int64)
        self.n_above = np.asarray(n_above, np.int64)
        self.keys = np.asarray(keys, np.uint64)
        self.cand_base = np.asarray(cand_base, np.int64)
        self.materialize = materialize

    def __len__(self):
        return self.keys.size


@dataclass
class BatchResult:
    """Engine.run's result for a WorkBatch: one entry per work, in work order."""
    index: np.ndarray
    value: np.ndarray
    score: np.ndarray
    n_scored: np.ndarray

    def __len__(self):
        return self.index.size


@dataclass(slots=True)
class LabelResult:
    label: str
    index: int                # global candidate index of the winner (-1: none)
    value: float              # winning candidate value (category id for categorical)
    score: float              # below_llik - above_llik at the winner
    n_scored: int
    below_llik: Optional[np.ndarray] = None
    above_llik: Optional[np.ndarray] = None
    cand: Optional[np.ndarray] = None
    extra: dict = field(default_factory=dict)


def posterior_params(kind, args):
    """Prior -> posterior construction parameters (tpe.py:484-572)."""
    if kind in ("uniform", "quniform", "loguniform", "qloguniform"):
        low, high = float(args[0]), float(args[1])
        q = float(args[2]) if kind.startswith("q") else None
        fam = L.LGMM1 if "log" in kind else L.GMM1
        floor = -math.inf
        if kind == "qloguniform":
            floor = max(EPS, math.exp(low))  # tpe.py:527-532
        return dict(family=fam, transform=L.OBS_LOG if fam == L.LGMM1 else L.OBS_IDENTITY,
                    floor=floor, prior_mu=0.5 * (high + low), prior_sigma=1.0 * (high - low),
                    low=low, high=high, q=q, bounded=True)
    if kind in ("normal", "qnormal", "lognormal", "qlognormal"):
        mu, sigma = float(args[0]), float(args[1])
        q = float(args[2]) if kind.startswith("q") else None
        fam = L.LGMM1 if "log" in kind else L.GMM1
        floor = EPS if kind == "qlognormal" else -math.inf  # tpe.py:567
        return dict(family=fam, transform=L.OBS_LOG if fam == L.LGMM1 else L.OBS_IDENTITY,
                    floor=floor, prior_mu=mu, prior_sigma=sigma, low=0.0, high=0.0, q=q,
                    bounded=False)
    raise ValueError("not a continuous prior: %r" % (kind,))


@functools.lru_cache(maxsize=4096)
def _posterior_params_cached(kind, args):
    return posterior_params(kind, args)


def _params(kind, args):
    try:
        return _posterior_params_cached(kind, tuple(args))
    except TypeError:  # unhashable args
        return posterior_params(kind, args)


def categorical_params(kind, args):
    """(K, offset, mode, prior p) for randint / categorical (tpe.py:578-615)."""
    if kind == "randint":
        if len(args) >= 2 and args[1] is not None:
            low, high = int(args[0]), int(args[1])
            return high - low, low, 0, None
        return int(args[0]), 0, 0, None
    if kind == "categorical":
        p = np.asarray(args[0], dtype=np.float64)
        if p.ndim == 2:
            p = p[0]
        return p.size, 0, 1, p
    raise ValueError("not a categorical prior: %r" % (kind,))


def _align(n):
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


class _Pack:
    """Packs host arrays into one buffer for a single host->device copy."""

    def __init__(self):
        self.parts = []
        self.size = 0

    def add(self, arr):
        arr = np.ascontiguousarray(arr)
        off = _align(self.size)
        self.parts.append((off, arr))
        self.size = off + max(arr.nbytes, 1)
        return off


_KNOBS_WARNED = set()


def _knob(name, default):
    """A level-launcher switch kept for A/B runs: the product
    path takes ``default``; an environment override is read only when
    TPE_DIAG=1 (diagnostic runs).  An override set without TPE_DIAG=1 is
    ignored with a one-time warning, so it is never dropped silently."""
    if os.environ.get("TPE_DIAG") == "1":
        return os.environ.get(name, default)
    if name in os.environ and name not in _KNOBS_WARNED:
        _KNOBS_WARNED.add(name)
        import warnings
        warnings.warn("hyperopt_amd: %s=%s is ignored (engine switches are read only with "
                      "TPE_DIAG=1; the product default %r is used)"
                      % (name, os.environ[name], default), RuntimeWarning, stacklevel=3)
    return default


class DeviceHistory:
    """A trials x labels history resident in HBM, appended in place.

    ``vals[j, r]`` / ``active[j, r]`` (label-major, leading dimension ``ld``)
    hold label j's value in history row r -- the columnar form of the
    reference's per-suggest ``miscs_to_idxs_vals`` (base.py:200-214).  The host
    keeps the active mask and per-label active counts so segment sizes are
    known without a device round trip.
    """

    def __init__(self, engine, n_labels, cap=1024):
        self.torch = engine.torch
        self.device = engine.device
        self.lib = engine.lib
        self.n_labels = int(n_labels)
        self.rows = 0
        self.cap = 0
        self.vals = self.active = None
        # per fitted column: its rows sorted by (transformed value, row)
        # (tpe_history_order; the fit's sort kept across suggests), the
        # (transform, floor) it was sorted with and how many rows it covers
        self.order = None
        self.order_spec = {}
        self.order_rows = {}
        self.active_host = np.zeros((0, self.n_labels), bool)
        self.n_active = np.zeros(self.n_labels, np.int64)
        self._stage = self._stage_ev = None  # pinned staging of appended rows, its upload event
        self._dstage = None  # its device copy (tpe_history_append's input)
        self._grow(max(int(cap), 16))

    @property
    def ld(self):
        return self.cap

    def _grow(self, cap):
        t = self.torch
        v = t.zeros((self.n_labels, cap), dtype=t.float64, device=self.device)
        a = t.zeros((self.n_labels, cap), dtype=t.uint8, device=self.device)
        if self.rows:
            v[:, :self.rows].copy_(self.vals[:, :self.rows])
            a[:, :self.rows].copy_(self.active[:, :self.rows])
        ah = np.zeros((cap, self.n_labels), bool)
        ah[:self.rows] = self.active_host[:self.rows]
        if self.order is not None:
            o = t.zeros((self.n_labels, cap), dtype=t.int32, device=self.device)
            if self.rows:
                o[:, :self.rows].copy_(self.order[:, :self.rows])
            self.order = o
        self.vals, self.active, self.active_host, self.cap = v, a, ah, cap

    def append(self, vals, active=None):
        """Append rows: vals (k, n_labels) float, active (k, n_labels) bool
        (default: finite values)."""
        vals = np.asarray(vals, dtype=np.float64).reshape(-1, self.n_labels)
        active = np.isfinite(vals) if active is None else \
            np.asarray(active, dtype=bool).reshape(vals.shape)
        k = vals.shape[0]
        if k == 0:
            return
        if self.rows + k > self.cap:
            self._grow(max(2 * self.cap, self.rows + k))
        r0, t = self.rows, self.torch
        # the new rows, label-major, through a pinned staging buffer: one
        # async upload on torch's current stream (the level's) into a device
        # stage, then one scatter into columns r0..r0+k (tpe_history_append)
        # -- no host wait, two runtime calls (torch's copies cost ~40 us of
        # host time per suggest; hipMemcpy2DAsync straight into the columns
        # ~0.3 ms more on the GPU, measured)
        nl = self.n_labels
        nv = nl * k * 8
        need = nv + nl * k
        hip = L.hip()
        if self._stage_ev is not None:  # the previous append's upload has read the stage
            L.hip_check(hip.hipEventSynchronize(self._stage_ev), "hipEventSynchronize")
        if self._stage is None or self._stage.numel() < need:
            # grown geometrically; the event is kept (it only orders the stage's reuse)
            old = 0 if self._stage is None else self._stage.numel()
            self._stage = t.empty(max(need, 2 * old, 4096), dtype=t.uint8, pin_memory=True)
        st = self._stage.numpy()
        np.copyto(st[:nv].view(np.float64).reshape(nl, k), np.where(active, vals, 0.0).T)
        np.copyto(st[nv:need].reshape(nl, k), active.T)
        sp = t.cuda.current_stream(self.device).cuda_stream
        if self._dstage is None or self._dstage.numel() < need:
            self._dstage = t.empty(self._stage.numel(), dtype=t.uint8, device=self.device)
        L.hip_check(hip.hipMemcpyAsync(self._dstage.data_ptr(), self._stage.data_ptr(), need, 1,
                                       sp), "hipMemcpyAsync")
        L.check(self.lib.tpe_history_append(self._dstage.data_ptr(), nl, k, self.vals.data_ptr(),
                                             self.active.data_ptr(), self.ld, r0, sp),
                "tpe_history_append")
        if self._stage_ev is None:
            ev = ctypes.c_void_p()
            L.hip_check(hip.hipEventCreateWithFlags(ctypes.byref(ev), L.EVENT_NO_TIMING),
                        "hipEventCreateWithFlags")
            self._stage_ev = ev
        L.hip_check(hip.hipEventRecord(self._stage_ev, sp), "hipEventRecord")
        self.active_host[r0:r0 + k] = active
        self.n_active += active.sum(0)
        self.rows += k


    ORDER_CHUNK = 2048  # new rows merged per tpe_history_order call

    def ensure_order(self, eng, stream, cols, transforms, floors):
        # (stream: the level's torch stream)
        """Bring the sorted orders of columns ``cols`` (with the fit's
        transform / floor per column) up to every row, on ``stream``: new rows
        are merged in (tpe_history_order), a column first seen -- or seen with
        another transform -- is built from scratch the same way."""
        t = self.torch
        if self.order is None:
            self.order = t.zeros((self.n_labels, self.cap), dtype=t.int32, device=self.device)
        sig = (np.asarray(cols).tobytes(), np.asarray(transforms).tobytes(),
               np.asarray(floors, np.float64).tobytes())
        key = (self.rows,) + sig
        if self.__dict__.get("_ordered") == key:
            return  # (the same columns and transforms, nothing appended since)
        # (merging right after each append instead, on the GPU while the host
        # plans the level: same-box A/B 1.050 vs 1.036 ms per drop-in suggest)
        last = self.__dict__.get("_ordered")
        # (sig, specs, columns) of the last slow pass.  When the last pass had
        # this signature no other column set has been ordered since, so the
        # columns still carry these specs (each pass sets _ordered to its key)
        cached = self.__dict__.get("_order_specs_for")
        orows = self.order_rows
        if last is not None and last[1:] == sig and cached is not None and cached[0] == sig \
                and all(orows.get(c) == last[0] for c in cached[2]):
            # (the same columns and specs as last time, every one at its rows)
            todo = {last[0]: cached[1]}
        else:
            todo = {}
            specs_all = []
            for c, tr, fl in zip(np.asarray(cols).tolist(), np.asarray(transforms).tolist(),
                                 np.asarray(floors).tolist()):
                spec = (int(tr), float(fl))
                specs_all.append((c,) + spec)
                if self.order_spec.get(c) != spec:
                    self.order_spec[c] = spec
                    self.order_rows[c] = 0
                if self.order_rows[c] < self.rows:
                    todo.setdefault(self.order_rows[c], []).append((c,) + spec)
            # the spec list is kept with the signature it belongs to, so a
            # later fast pass never merges another column set's specs
            self._order_specs_for = (sig, specs_all, [x[0] for x in specs_all])
        if not todo:
            self._ordered = key
            return
        lib = eng.lib
        sp = ctypes.c_void_p(stream.cuda_stream)
        cache = self.__dict__.setdefault("_spec_dev", {})
        for n_old, specs in todo.items():
            hit = cache.get(tuple(specs))
            if hit is None:  # the column specs on the device (kept: the same every append)
                arr = np.zeros(len(specs), L.COLSPEC_DTYPE)
                arr["col"], arr["transform"], arr["floor"] = zip(*specs)
                with t.cuda.stream(stream):
                    dev = t.from_numpy(arr.view(np.uint8).copy()).to(self.device)
                if len(cache) > 16:
                    cache.clear()
                hit = cache[tuple(specs)] = (arr, dev)
            arr, dev = hit
            scratch = eng._buf("order_scratch",
                               lib.tpe_history_order_scratch_bytes(len(specs), self.rows))
            n = n_old
            while n < self.rows:
                k = min(self.ORDER_CHUNK, self.rows - n)
                L.check(lib.tpe_history_order(self.vals.data_ptr(), self.ld, dev.data_ptr(),
                                              arr.ctypes.data, len(specs), n, k,
                                              self.order.data_ptr(), scratch, sp),
                        "tpe_history_order")
                n += k
            for c, _, _ in specs:
                self.order_rows[c] = self.rows
        self._ordered = key


_LAUNCH_STATE = frozenset(('BS', 'JS', '_hmark', 'band_jobs', 'base', 'cat', 'cnt_off', 'cobs_off', 'csegs', 'd_best', 'd_c32', 'd_c32n', 'd_c64', 'd_ccdf', 'd_cdf', 'd_csegs', 'd_err', 'd_fs', 'd_logp', 'd_mu', 'd_pairs', 'd_pm', 'd_segs', 'd_sig', 'd_sm', 'd_stats', 'd_w', 'd_w32', 'exchange', 'fb_jobs', 'fit_ids', 'g_arr', 'groups', 'h_arr', 'hist_mode', 'histories', 'history', 'inj', 'jobs', 'lat_off', 'lat_ready', 'max_obs', 'n_comp', 'n_jobs', 'n_obs_total', 'n_rows', 'nfs', 'o_cand', 'o_cobs', 'o_fb', 'o_g', 'o_h', 'o_isb', 'o_jobs', 'o_lcnt', 'o_obs', 'o_p', 'o_rows', 'o_slot', 'o_xslot', 'out_off', 'outputs', 'p_pool', 'posteriors', 'precision', 'qfb_off', 'sample_only', 'segs', 'sort_off', 'sorted_fit', 'sp', 'stream', 'table_scores', 'torch', 'works', 'x_comm', 'x_labels', 'x_world'))


class _LevelState:
    """A prepared level's plan, workspace pointers and pack offsets (the locals
    of Engine.run that its launches read; Engine._launch_level)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __getattr__(self, name):  # (pointers of paths the level does not take)
        if name in _LAUNCH_STATE:
            return None
        raise AttributeError(name)


class _LaunchState:
    """Launch-time state of one level shared by its stages (Engine._launch_level:
    the library or recording _OpList, the streams, the output buffers, the side
    stream's fork / join flags), and of one group's launch (its job slice)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class _LaunchCtx:
    """Timer events and cross-stream ordering of one level's launches, issued
    eagerly or appended to the _OpList being recorded (``cap``)."""

    def __init__(self, eng, stream, timers, timer_groups):
        self.eng, self.stream, self.timers, self.timer_groups = eng, stream, timers, timer_groups
        self.cap = None

    def tick(self, name, on=None):
        if self.timers is None or (self.timer_groups is not None and name not in self.timer_groups):
            return None
        if self.cap is not None:
            return self.cap.record(self.eng._hip, self.stream if on is None else on)
        e = self.eng.torch.cuda.Event(enable_timing=True)
        e.record(self.stream if on is None else on)
        return e

    def tock(self, name, e0, on=None):
        if e0 is None:
            return
        if self.cap is not None:
            self.cap.timed.append((name, e0, self.tick(name, on)))
        else:
            self.timers.setdefault(name, []).append((e0, self.tick(name, on)))

    def stream_order(self, name, src, dst):
        if isinstance(self.cap, _OpList):
            self.cap.order(self.eng._event(name), src, dst)
        else:
            self.eng._order(name, src, dst)

    def stream_rec(self, name, src):  # event `name` marks `src`'s work so far
        if isinstance(self.cap, _OpList):
            self.cap.add(L.OP_EVENT_RECORD, self.eng._event(name), src)
        else:
            L.hip_check(self.eng._hip.hipEventRecord(self.eng._event(name), src), "hipEventRecord")

    def stream_wait(self, name, dst):  # `dst` waits for event `name`
        if isinstance(self.cap, _OpList):
            self.cap.add(L.OP_STREAM_WAIT, dst, self.eng._event(name))
        else:
            L.hip_check(self.eng._hip.hipStreamWaitEvent(dst, self.eng._event(name), 0),
                        "hipStreamWaitEvent")


class Engine:
    """Owns the device workspace; one instance per device (kept by tpe.py)."""

    def __init__(self, device=None):
        import torch
        self.torch = torch
        self.lib = L.load()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self._bufs = {}
        self._plans = {}  # level structure -> static descriptor arrays (_plan_record)
        self._retired = []
        self._pinned = {}
        self._res_pin = None   # pinned result block of a level's readback
        self._inflight = None  # a deferred (WorkBatch) run's _Pending until collected
        self._events = {}      # reusable HIP events (no timing) by name
        self._hip = L.hip()
        self.host_marks = None  # set to a list to record host-side phase times (diagnostic)
        # categorical posteriors and quantized / categorical scoring run on a
        # second stream, concurrently with the continuous fit and the
        # cell-table path (they share no buffers): -7% per level on one GPU,
        # -11% at an 8-way label share (tools/rank_share.py).
        # "1": join at the end of the level; "2": the table scorer waits for
        # the side stream; "0": everything on the caller's stream
        self.side_stream = _knob("TPE_SIDE_STREAM", "1")
        self._side = None
        # sampled table jobs without per-candidate outputs: "cubic" scores
        # each candidate by its cell's score cubic (tpe_score_table_fast);
        # "poly" evaluates both cell polynomials (tpe_score_table)
        self.table_scorer = _knob("TPE_TABLE_SCORER", "cubic")
        # fp64 continuous labels: "auto" prunes components (tpe_score_pruned64)
        # once the above mixture has PRUNED64_MIN_COMP components, "dense"
        # always sums every component (tpe_score_continuous), "pruned" always prunes
        self.exact64 = _knob("TPE_EXACT64", "auto")
        # categorical posterior + scoring on the side stream before the fit
        # (TPE_CAT_EARLY=1) or after it with the quantized labels (0)
        self.cat_early = _knob("TPE_CAT_EARLY", "1") == "1"
        # categorical posteriors of a single-history level counted straight
        # from the HBM history (tpe_cat_posterior_hist) instead of a gather
        # of their lists plus tpe_cat_posterior (TPE_CAT_HIST=0)
        self.cat_hist = _knob("TPE_CAT_HIST", "1") == "1"
        # ... over a long history in row chunks by many blocks (the same bits;
        # TPE_CAT_CHUNKED=0: one block per segment and category)
        self.cat_chunked = _knob("TPE_CAT_CHUNKED", "1") == "1"
        # quantized labels on the main stream when it has no scorer of its own
        # (Engine._launch_level); TPE_LAT_MAIN=0: always on the side stream
        self.lat_main = _knob("TPE_LAT_MAIN", "1") == "1"
        # lattices of at most this many slots take the prefix-first argmax
        # (every slot scored); larger ones draw and score their whole stream
        self.lat_max_slots = int(_knob("TPE_LAT_MAX_SLOTS", str(LAT_SUGGEST_MAX_SLOTS)))
        # where the host issues that categorical work: "pre" (before the fit's
        # launches), "post" (after them), "late" (after the table build)
        self.cat_issue = _knob("TPE_CAT_ISSUE", "post")
        # quantized labels of a suggest level: decide the argmax after the first
        # lat_prefix candidates where no unseen lattice value can still win
        # (tpe_lattice_suggest); 0 (TPE_LAT_PREFIX=0): every stream drawn in full
        self.lat_prefix = _lat_prefix(_knob("TPE_LAT_PREFIX", str(LAT_PREFIX)))
        # stream-ordering events (one stream of this device waits for another)
        # without the system-scope fence: a device-scope release is all a
        # consumer on the same GPU needs, and the system-scope one writes back
        # the L2s (~14 us of idle GPU per event on C3 levels).  The host-read
        # "result" event keeps it.  TPE_DEVICE_EVENTS=0: every event system-scope.
        self.device_events = _knob("TPE_DEVICE_EVENTS", "1") == "1"
        # the fit from the history's sorted orders (tpe_fit_sorted) where the
        # level reads one history with its identity row list; "0": the
        # gather + sort + merge fit (tpe_parzen_fit) everywhere
        self.sorted_fit = _knob("TPE_SORTED_FIT", "1") == "1"
        self._last_gkey = None  # launch key of the previous eager level
        self._gen = 0           # bumped whenever a workspace buffer is (re)allocated
        self.graph_stats = {"eager": 0}  # levels issued eagerly / re-issued ("native", "replay")
        # native level launcher (default; TPE_NATIVE_LAUNCH=0: one ctypes call
        # per entry point): a level whose launch key repeats the previous
        # call's is recorded once as tpe_run_ops records -- upload, every
        # launch, stream fork/join, readback and the final synchronise -- and
        # re-issued with one C call per level (hyperopt_amd/csrc/tpe_ops.hip)
        self.native = _knob("TPE_NATIVE_LAUNCH", "1") != "0"
        # TPE_GRAPHS=1 (diagnostic): recorded levels re-issued with the same
        # words replay a hipGraph of their records (_OpList.issue).  Off in the
        # product: on ROCm 7 a replayed C3 level is no faster on the host and
        # slower on the GPU than the records
        self.graphs = _knob("TPE_GRAPHS", "0") == "1"
        # recorded levels are issued by two host threads (the caller: the main
        # stream's records; a worker of the library: the side stream's), so the
        # main chain no longer waits while the host issues the side group
        # (tpe_set_issue_threads); TPE_ISSUE_THREADS=1: one thread
        self.issue_threads = int(_knob("TPE_ISSUE_THREADS", "2"))
        rc = self.lib.tpe_set_issue_threads(self.issue_threads)
        L.check(min(rc, 0), "tpe_set_issue_threads")
        self._cap_stream = None
        self._oplists = {}      # launch key -> _OpList
        self._oplist_once = None
        self._replays = {}      # signature -> _Replay of a recorded WorkBatch level
        self._staged_sig = None  # pack signature of what the pinned staging buffer holds

    # -- memory --------------------------------------------------------------
    def _buf(self, name, nbytes):
        t = self._bufs.get(name)
        nbytes = max(int(nbytes), 16)
        if t is None or t.numel() < nbytes:
            if t is not None:  # may still be in use on the side stream: freed after the run
                self._retired.append(t)
            t = self.torch.empty(_align(int(nbytes * 1.25)), dtype=self.torch.uint8,
                                 device=self.device)
            self._bufs[name] = t
            self._gen += 1  # recorded levels hold the old pointers
        return t.data_ptr()

    def _zbuf(self, name, nbytes):
        """A workspace buffer that is zero when (re)allocated (kernels that use
        it leave it zero again, e.g. the band controls)."""
        t = self._bufs.get(name)
        nbytes = max(int(nbytes), 16)
        if t is None or t.numel() < nbytes:
            if t is not None:
                self._retired.append(t)
            t = self.torch.zeros(_align(int(nbytes * 1.25)), dtype=self.torch.uint8,
                                 device=self.device)
            self._bufs[name] = t
            self._gen += 1
        return t.data_ptr()

    def _presize(self, n_comp, n_obs_total, max_obs, cobs_off, n_seg, tjobs, n_rows):
        """Every workspace buffer whose size follows a level's per-call sizes
        (mixture pools, observation pools, fit / table scratch), grown here,
        before the launch key is formed: a level re-issued from its records
        (which hold the pointers) then finds every buffer large enough, and a
        buffer that had to grow (new pointer, _gen bumped) forces a new
        recording."""
        sizes = (n_comp, n_obs_total, max_obs, cobs_off, n_seg, tjobs, n_rows)
        last = self.__dict__.get("_presized")
        if last is not None and last[0] == self._gen and all(
                a <= b for a, b in zip(sizes, last[1])) and n_seg == last[1][4] and \
                tjobs == last[1][5]:
            return  # every buffer already holds these sizes (buffers only grow)
        lib = self.lib
        if n_comp:
            for name, per in (("w", 8), ("mu", 8), ("sigma", 8), ("wcdf", 8), ("coef64", 32),
                              ("coef32", 16), ("reach_hi", 8), ("reach_lo", 8),
                              ("wide_idx", 4), ("coef32n", 16), ("wide32", 16), ("pm", 4),
                              ("sm", 4)):
                self._buf(name, per * n_comp)
            self._buf("fit_scratch", lib.tpe_fit_scratch_bytes(n_seg, max_obs, n_obs_total))
        self._buf("obs_dev", 8 * max(n_obs_total, 1))
        self._buf("cobs_dev", 8 * max(cobs_off, 1))
        if tjobs:
            self._buf("table_scratch", lib.tpe_table_scratch_bytes(tjobs, max_obs + 1))
        if n_rows:
            self._buf("fit_sorted_scratch", lib.tpe_fit_sorted_scratch_bytes(n_seg, n_rows))
        self._presized = (self._gen, sizes)

    def _capture_stream(self):
        """A stream of this engine's own to capture levels on (the caller's
        stream may be the null stream, which cannot be captured)."""
        if self._cap_stream is None:
            self._cap_stream = self.torch.cuda.Stream(self.device)
        return self._cap_stream.cuda_stream

    def _drop_oplists(self):
        self._replays.clear()
        for o in self._oplists.values():
            o.destroy(self._hip)
        self._oplists.clear()

    def _ones(self, n):
        """n all-ones uint64 words (cached)."""
        a = self.__dict__.get("_ones_arr")
        if a is None or a.size < n:
            a = self._ones_arr = np.full(max(n, 1024), np.uint64(0xFFFFFFFFFFFFFFFF))
        return a[:n]

    def _event(self, name):
        e = self._events.get(name)
        if e is None:
            h = ctypes.c_void_p()
            flags = L.EVENT_NO_TIMING
            if self.device_events and name not in HOST_EVENTS:
                flags |= L.EVENT_NO_SYSTEM_FENCE
            L.hip_check(self._hip.hipEventCreateWithFlags(ctypes.byref(h), flags),
                        "hipEventCreateWithFlags")
            e = self._events[name] = h
        return e

    def _order(self, name, src, dst):
        """`dst` waits for the work queued so far on `src` (raw stream handles)."""
        e = self._event(name)
        L.hip_check(self._hip.hipEventRecord(e, src), "hipEventRecord")
        L.hip_check(self._hip.hipStreamWaitEvent(dst, e, 0), "hipStreamWaitEvent")

    def _res_pinned(self, nbytes):
        pin = self._res_pin
        if pin is None or pin.numel() < nbytes:
            pin = self._res_pin = self.torch.empty(_align(int(nbytes * 1.25)),
                                                   dtype=self.torch.uint8, pin_memory=True)
            self._gen += 1
        return pin

    def _upload(self, pack, stream, slot=0, copy=True):
        """One host->device copy of ``pack`` through pinned buffer / device
        staging area ``slot`` (a level uploads twice: descriptors for the fit,
        then the job table, each into its own slot).  ``copy=False``: stage
        only; the copy (``self._staged`` = dst, src, bytes) is issued later."""
        torch = self.torch
        pinned = self._pinned.get(slot)
        if pinned is None or pinned.numel() < pack.size:
            pinned = torch.empty(_align(int(pack.size * 1.25) + 1), dtype=torch.uint8,
                                 pin_memory=True)
            self._pinned[slot] = pinned
            self._gen += 1
        host = pinned.numpy()
        for off, arr in pack.parts:
            host[off:off + arr.nbytes] = arr.reshape(-1).view(np.uint8)
        name = "stage" if slot == 0 else "stage%d" % slot
        dev = self._buf(name, pack.size)
        self._staged = (dev, pinned.data_ptr(), pack.size)
        self._staged_sig = None  # (a replay may claim it once the level is recorded)
        if copy:
            L.hip_check(self._hip.hipMemcpyAsync(dev, pinned.data_ptr(), pack.size, L.H2D,
                                                 stream.cuda_stream), "hipMemcpyAsync")
        return dev

    # -- level plans -----------------------------------------------------------
    # A level's descriptor arrays (segments, categorical segments, gathers,
    # jobs) depend on the level's structure -- kinds, prior arguments,
    # candidate counts, history columns, lattice ranges, run options -- and,
    # per call, only on the observation counts and the Philox keys.  The first
    # call of a structure builds them in Python; later calls copy the recorded
    # arrays and fill the per-call columns with a few vectorised operations.
    def _plan_key(self, works, prior_weight, lf, precision, scorer, outputs, sample_only,
                  hist_mode, multi):
        if not hist_mode or outputs or sample_only:
            return None
        parts = []
        for w in works:
            if w.cand is not None or w.kind not in CONTINUOUS + CATEGORICAL:
                return None
            lat = None
            if w.kind in CONTINUOUS and w.kind.startswith("q"):
                P = _params(w.kind, w.args)
                if not P["bounded"]:  # the lattice range follows the below set
                    lat = _lattice_range(w, P)
            parts.append((w.kind, w.args, int(w.n_cand), int(w.n_total), w.col, w.hist, lat))
        key = (tuple(parts), float(prior_weight), int(lf), int(precision), scorer, multi)
        try:
            hash(key)
        except TypeError:  # unhashable prior arguments (e.g. a probability list)
            return None
        if len(self._plans) > 64:
            self._plans.clear()
        return key

    def _plan_record(self, works, cont, quant, cat, fit_ids, params, segs, csegs, p_pool,
                     cat_meta, lat_ranges, fallback, modes, groups, order, gathers, jobs,
                     fb_slice, out_off, lat_off, qfb_off, sort_off, cnt_off, tbl_off):
        g = np.zeros(len(gathers), L.GATHER_DTYPE)
        if gathers:
            (g["col"], g["below"], g["dst_off"], g["offset"], g["count"], g["to_int"],
             g["hist"]) = (np.array(c) for c in zip(*gathers))
        return dict(cont=cont, quant=quant, cat=cat, fit_ids=fit_ids, params=params,
                    fit_idx=np.asarray(fit_ids, np.int64), cat_idx=np.asarray(cat, np.int64),
                    order_idx=np.asarray(order, np.int64),
                    segs=segs.copy(), csegs=csegs.copy(), p_pool=p_pool.copy(),
                    cat_meta=cat_meta, lat_ranges=lat_ranges, fallback=fallback, modes=modes,
                    groups=groups, order=order, g=g, jobs=jobs.copy(), fb_slice=fb_slice,
                    counts=(out_off, lat_off, qfb_off, sort_off, cnt_off, tbl_off))

    def _big64(self, precision, n_above):
        """The per-call input of the scorer choice that a plan records: at fp64,
        which labels' above mixtures reach PRUNED64_MIN_COMP (pruned vs dense
        exact scorer) -- part of the plan key, so a cached plan never scores a
        label with the other kernel than an uncached run would."""
        if precision == 32 or self.exact64 != "auto":
            return self.exact64
        return np.packbits(np.asarray(n_above) >= PRUNED64_MIN_COMP).tobytes()

    @staticmethod
    def _columns(works):
        """(n_below, n_above, keys, cand_base) per work of a history-mode list."""
        n = len(works)
        return (np.fromiter((np.size(w.obs_below) for w in works), np.int64, n),
                np.fromiter((w.n_above for w in works), np.int64, n),
                np.fromiter((int(w.key) & 0xFFFFFFFFFFFFFFFF for w in works), np.uint64, n),
                np.fromiter((w.cand_base for w in works), np.int64, n))

    def _plan_fast(self, P, nb, na):
        fit_ids, cat = P["fit_ids"], P["cat"]
        nf = len(fit_ids)
        segs = P["segs"].copy()
        sizes = np.empty(2 * nf, np.int64)
        fi = P["fit_idx"]
        sizes[0::2] = nb[fi]
        sizes[1::2] = na[fi]
        ends = np.cumsum(sizes)
        obs_off = ends - sizes
        segs["obs_off"], segs["n_obs"] = obs_off, sizes
        segs["comp_off"] = np.cumsum(sizes + 1) - (sizes + 1)
        n_obs_total = int(ends[-1]) if nf else 0
        n_comp = n_obs_total + 2 * nf
        max_obs = int(sizes.max()) if nf else 0
        csegs = P["csegs"].copy()
        csizes = np.empty(2 * len(cat), np.int64)
        ci = P["cat_idx"]
        csizes[0::2] = nb[ci]
        csizes[1::2] = na[ci]
        cends = np.cumsum(csizes)
        coff = cends - csizes
        csegs["obs_off"], csegs["n_obs"] = coff, csizes
        cobs_off = int(cends[-1]) if cat else 0
        g_arr = P["g"].copy()
        g_arr["dst_off"] = np.concatenate([obs_off, coff])
        g_arr["count"] = np.concatenate([sizes, csizes])
        return (P["cont"], P["quant"], cat, fit_ids, P["params"], nf, segs, np.zeros(1),
                n_obs_total, n_comp, max_obs, csegs, np.zeros(1, np.int64), P["p_pool"],
                P["cat_meta"], cobs_off, P["lat_ranges"], P["fallback"], P["modes"],
                P["groups"], P["order"], g_arr)

    def _jobs_fast(self, P, keys, cand_base):
        oi = P["order_idx"]
        jobs = P["jobs"].copy()
        jobs["key"] = keys[oi]
        jobs["cand_base"] = cand_base[oi]
        a, b = P["fb_slice"]
        fb_jobs = jobs[a:b].copy()
        fb_jobs["out_off"] = fb_jobs["cand_off"]
        return (jobs, np.zeros(1), fb_jobs, P["fb_slice"]) + tuple(P["counts"])

    def _choose_plan(self, works, batch, prior_weight, lf, precision, scorer, outputs,
                     sample_only, hist_mode, multi, _hmark):
        """A level's plan: replayed from the plan recorded for its structure
        (_plan_fast + _jobs_fast: only the per-call columns -- counts, keys,
        candidate bases -- are filled in) or built from its works (_plan_new,
        which records it when it can be replayed).  A WorkBatch's works are
        materialised only when its structure is new.  Returns (works, plan
        key, recorded plan or None, the plan tuple of _plan_new; a replayed
        plan gives the gather table where _plan_new gives the gather list)."""
        if batch is not None:
            pkey = ("batch", batch.key, float(prior_weight), int(lf), int(precision), scorer,
                    multi, self._big64(precision, batch.n_above))
            cached = self._plans.get(pkey)
            if cached is None:
                works = batch.materialize()
                if len(works) != len(batch):
                    raise ValueError("WorkBatch.materialize() gave %d works for %d rows"
                                     % (len(works), len(batch)))
            elif len(self._plans) > 64:
                self._plans.clear()
        else:
            pkey = self._plan_key(works, prior_weight, lf, precision, scorer, outputs,
                                  sample_only, hist_mode, multi)
            if pkey is not None:
                pkey += (self._big64(precision, np.fromiter(
                    (w.n_above if w.obs_above is None else np.size(w.obs_above) for w in works),
                    np.int64, len(works))),)
            cached = self._plans.get(pkey) if pkey is not None else None
        if cached is None:
            return works, pkey, None, self._plan_new(
                works, pkey, prior_weight, lf, precision, scorer, outputs, sample_only, hist_mode,
                _hmark)
        cols = (batch.n_below, batch.n_above, batch.keys, batch.cand_base) \
            if batch is not None else self._columns(works)
        (cont, quant, cat, fit_ids, params, nf, segs, obs_pool, n_obs_total, n_comp, max_obs,
         csegs, cobs_pool, p_pool, cat_meta, cobs_off, lat_ranges, fallback, modes, groups,
         order, g_arr) = self._plan_fast(cached, cols[0], cols[1])
        if batch is not None:
            inj = lambda i: False  # noqa: E731
        else:
            inj = lambda i: works[i].cand is not None  # noqa: E731
        (jobs, cand_pool, fb_jobs, fb_slice, out_off, lat_off, qfb_off, sort_off, cnt_off,
         tbl_off) = self._jobs_fast(cached, cols[2], cols[3])
        return works, pkey, cached, (
            cont, quant, cat, fit_ids, params, nf, segs, obs_pool, n_obs_total, n_comp, max_obs,
            csegs, cobs_pool, p_pool, cat_meta, cobs_off, lat_ranges, fallback, modes, groups,
            order, g_arr, inj, jobs, cand_pool, fb_jobs, fb_slice, out_off, lat_off, qfb_off,
            sort_off, cnt_off, tbl_off)

    # -- main entry ----------------------------------------------------------
    def _plan_new(self, works, pkey, prior_weight, lf, precision, scorer, outputs, sample_only,
                  hist_mode, _hmark):
        """A level's plan built from its works (the path _plan_fast replays
        from a recorded plan): kernel groups, fit / categorical segments, the
        gather list of a history level, and the job descriptors ordered so
        every kernel call takes a contiguous slice.  Records the plan under
        ``pkey`` when it can be replayed."""
        cont, quant, cat = [], [], []
        for i, w in enumerate(works):
            if w.kind in CONTINUOUS:
                (quant if w.kind.startswith("q") else cont).append(i)
            elif w.kind in CATEGORICAL:
                cat.append(i)
            else:
                raise ValueError("unsupported prior %r for label %r" % (w.kind, w.label))

        _hmark('prep')
        gathers = []  # history mode: (col, below, dst_off, offset, count, to_int, hist)
        # ---- continuous / quantized segments --------------------------------
        fit_ids = cont + quant
        params = {i: _params(works[i].kind, works[i].args) for i in fit_ids}
        nf = len(fit_ids)
        segs = np.zeros(2 * nf, L.SEG_DTYPE)
        obs_pool = None
        n_obs_total = n_comp = max_obs = 0
        if nf:
            if hist_mode:
                sizes = np.empty(2 * nf, np.int64)
                for si, i in enumerate(fit_ids):
                    sizes[2 * si] = np.asarray(works[i].obs_below).size
                    sizes[2 * si + 1] = int(works[i].n_above)
            else:
                parts = [np.asarray(o, dtype=np.float64).reshape(-1) for i in fit_ids
                         for o in (works[i].obs_below, works[i].obs_above)]
                sizes = np.fromiter((o.size for o in parts), np.int64, 2 * nf)
                obs_pool = np.concatenate(parts)
            ends = np.cumsum(sizes)
            obs_off = ends - sizes
            comp_off = np.cumsum(sizes + 1) - (sizes + 1)
            segs["obs_off"], segs["comp_off"], segs["n_obs"] = obs_off, comp_off, sizes
            segs["lf"], segs["prior_weight"] = lf, prior_weight
            pl = [params[i] for i in fit_ids]
            for name in ("transform", "family", "floor", "prior_mu", "prior_sigma", "low", "high"):
                segs[name] = np.repeat([p[name] for p in pl], 2)
            segs["bounded"] = np.repeat([int(p["bounded"]) for p in pl], 2)
            n_obs_total = int(ends[-1])
            n_comp = n_obs_total + 2 * nf
            max_obs = int(sizes.max())
            if hist_mode:
                for si, i in enumerate(fit_ids):
                    for half in (0, 1):
                        k = 2 * si + half
                        gathers.append((works[i].col, 1 - half, int(obs_off[k]), 0, int(sizes[k]),
                                        0, works[i].hist))
        if obs_pool is None:
            obs_pool = np.zeros(1)

        _hmark('segs')
        # ---- categorical segments ------------------------------------------
        csegs = np.zeros(2 * len(cat), L.CAT_SEG_DTYPE)
        cobs_parts, p_init = [], []
        cobs_off = p_off = 0
        cat_meta = {}
        ccols = []
        for ci, i in enumerate(cat):
            w = works[i]
            K, offset, mode, prior_p = categorical_params(w.kind, w.args)
            cat_meta[i] = (K, offset)
            prior_off = -1
            if mode == 1:
                prior_off = p_off
                p_init.append(prior_p)
                p_off += K
            for half in (0, 1):
                if hist_mode:
                    n = np.asarray(w.obs_below).size if half == 0 else int(w.n_above)
                    gathers.append((w.col, 1 - half, cobs_off, offset, n, 1, w.hist))
                else:
                    obs = np.asarray(w.obs_below if half == 0 else w.obs_above).reshape(-1)
                    obs = obs.astype(np.int64) - offset
                    cobs_parts.append(obs)
                    n = obs.size
                ccols.append((cobs_off, p_off, n, K, mode, max(prior_off, 0)))
                p_init.append(np.zeros(K))
                cobs_off += n
                p_off += K
        if cat:  # one column assignment per field instead of per segment
            cc = np.array(ccols, dtype=np.int64)
            (csegs["obs_off"], csegs["p_off"], csegs["n_obs"], csegs["n_cat"], csegs["mode"],
             csegs["prior_p_off"]) = cc.T
            csegs["lf"], csegs["prior_weight"] = lf, prior_weight
        cobs_pool = np.concatenate(cobs_parts) if cobs_parts else np.zeros(1, np.int64)
        p_pool = np.concatenate(p_init) if p_init else np.zeros(1)

        _hmark('cats')
        (inj, lat_ranges, fallback, modes, groups, order, jobs, cand_pool, fb_jobs, fb_slice,
         out_off, lat_off, qfb_off, sort_off, cnt_off, tbl_off) = self._plan_jobs(
            works, cont, quant, cat, fit_ids, params, cat_meta, precision, scorer, outputs,
            sample_only)
        if pkey is not None and not any(k == "sorted" and ids for k, ids in groups):
            self._plans[pkey] = self._plan_record(
                works, cont, quant, cat, fit_ids, params, segs, csegs, p_pool, cat_meta,
                lat_ranges, fallback, modes, groups, order, gathers, jobs, fb_slice, out_off,
                lat_off, qfb_off, sort_off, cnt_off, tbl_off)

        return (cont, quant, cat, fit_ids, params, nf, segs, obs_pool, n_obs_total, n_comp,
                max_obs, csegs, cobs_pool, p_pool, cat_meta, cobs_off, lat_ranges, fallback, modes,
                groups, order, gathers, inj, jobs, cand_pool, fb_jobs, fb_slice, out_off, lat_off,
                qfb_off, sort_off, cnt_off, tbl_off)

    def _plan_jobs(self, works, cont, quant, cat, fit_ids, params, cat_meta, precision, scorer,
                   outputs, sample_only):
        """The job table of a new plan (_plan_new): each label's scorer
        (continuous: table / pruned64 / dense / sorted by precision, size and
        hooks; quantized: lattice or dense fallback; categorical), the kernel
        groups, and one tpe_job per label ordered so every kernel call takes a
        contiguous slice, with its candidate, output, lattice and table offsets."""
        # ---- jobs, ordered so every kernel call takes a contiguous slice -----------
        inj = lambda i: works[i].cand is not None  # noqa: E731
        lat_ranges = {}
        fallback = []
        for i in quant:
            if not inj(i):
                kmin, kmax = _lattice_range(works[i], params[i])
                if kmax - kmin + 1 > LATTICE_CAP:
                    fallback.append(i)
                else:
                    lat_ranges[i] = (kmin, kmax - kmin + 1)
        def cont_mode(i):
            if sample_only:
                return "cont"
            if precision != 32:
                w = works[i]
                m = int(w.n_above) if w.obs_above is None else np.size(w.obs_above)
                return "pruned64" if (self.exact64 == "pruned" or (
                    self.exact64 == "auto" and m >= PRUNED64_MIN_COMP)) else "cont"
            n = int(np.asarray(works[i].cand).size) if inj(i) else \
                int(works[i].n_total or works[i].n_cand)
            mode = scorer
            if mode == "auto":
                mode = "cont"
                if not inj(i):
                    if n >= TABLE_MIN_CAND:
                        mode = "table"  # fp32 scores, exact argmax (the band re-score)
                    elif not outputs:
                        # fp32 draws, exact decision: the fp32 stream scored in
                        # fp64 (tpe_score_pruned64 with TPE_F_DRAW32), so an
                        # explicit precision=32 suggest is exact at every size
                        mode = "pruned64"
            if mode == "sorted" and (inj(i) or outputs):
                mode = "cont"
            return "cont" if mode == "dense" else mode
        modes = {i: cont_mode(i) for i in cont}
        groups = [
            ("cont", [i for i in cont if inj(i) and modes[i] == "cont"]),
            ("cont", [i for i in cont if not inj(i) and modes[i] == "cont"]),
            ("sorted", [i for i in cont if modes[i] == "sorted"]),
            ("pruned64", [i for i in cont if inj(i) and modes[i] == "pruned64"]),
            ("pruned64", [i for i in cont if not inj(i) and modes[i] == "pruned64"]),
            ("table", [i for i in cont if inj(i) and modes[i] == "table"]),
            ("table", [i for i in cont if not inj(i) and modes[i] == "table"]),
            ("lat", [i for i in quant if i in lat_ranges]),
            ("qfb", fallback),
            ("qinj", [i for i in quant if inj(i)]),
            ("cat", [i for i in cat if inj(i)]),
            ("cat", [i for i in cat if not inj(i)]),
        ]
        order = [i for _, ids in groups for i in ids]
        nj_all = len(order)
        jobs = np.zeros(nj_all, L.JOB_DTYPE)
        J = {name: np.zeros(nj_all, L.JOB_DTYPE[name]) for name in L.JOB_DTYPE.names}
        cand_parts, cand_off, out_off, lat_off, qfb_off = [], 0, 0, 0, 0
        sort_off = cnt_off = tbl_off = 0
        seg_of = {i: si for si, i in enumerate(fit_ids)}
        cseg_of = {i: ci for ci, i in enumerate(cat)}
        for pos, i in enumerate(order):
            w = works[i]
            J["key"][pos] = int(w.key) & 0xFFFFFFFFFFFFFFFF
            J["cand_base"][pos] = w.cand_base
            n = int(np.asarray(w.cand).size) if inj(i) else int(w.n_cand)
            J["n_cand"][pos] = n
            J["out_off"][pos] = out_off
            out_off += n
            flags = 0
            if inj(i):
                # categorical candidates are category indices (0..K-1), as the
                # reference's randint_via_categorical samples them (tpe.py:590)
                c = np.asarray(w.cand, dtype=np.float64).reshape(-1)
                J["cand_off"][pos] = cand_off
                cand_parts.append(c)
                cand_off += c.size
                flags |= L.F_INJECTED
            if i in cat_meta:
                J["family"][pos] = L.CAT
                J["lat_n"][pos] = cat_meta[i][0]  # category count (sizes the sampler's path)
                J["below"][pos], J["above"][pos] = 2 * cseg_of[i], 2 * cseg_of[i] + 1
                J["flags"][pos] = flags
                continue
            P = params[i]
            J["family"][pos] = P["family"]
            J["below"][pos], J["above"][pos] = 2 * seg_of[i], 2 * seg_of[i] + 1
            if P["bounded"]:
                flags |= L.F_LOW | L.F_HIGH
                J["low"][pos], J["high"][pos] = P["low"], P["high"]
            if P["q"] is not None:
                flags |= L.F_QUANT
                J["q"][pos] = P["q"]
                if i in lat_ranges:
                    kmin, nk = lat_ranges[i]
                    J["lat_off"][pos], J["lat_kmin"][pos], J["lat_n"][pos] = lat_off, kmin, nk
                    if precision == 32 and max(abs(kmin), abs(kmin + nk - 1)) <= DRAW32_MAX_SLOT:
                        flags |= L.F_DRAW32
                    flags |= L.F_LATTICE_READY  # cleared below for a large level
                    lat_off += nk
                elif i in fallback:
                    J["cand_off"][pos] = qfb_off
                    qfb_off += n
            elif modes[i] == "table":
                J["tbl_off"][pos], J["tbl_cap"][pos] = tbl_off, TABLE_CAP
                tbl_off += TABLE_CAP
                if inj(i):
                    J["bin_lo"][pos], J["bin_hi"][pos] = _injected_range(w, P)
            elif modes[i] == "pruned64" and inj(i):
                J["bin_lo"][pos], J["bin_hi"][pos] = _injected_range(w, P, fp32=False)
            elif modes[i] == "pruned64" and precision == 32:
                flags |= L.F_DRAW32  # the fp32 stream (the table path's draws)
            elif modes[i] == "sorted":
                J["bin_lo"][pos], J["bin_hi"][pos] = _support(w, P)
                J["sort_off"][pos], J["cnt_off"][pos] = sort_off, cnt_off
                slots = ctypes.c_int64(0)
                cnt_off += self.lib.tpe_sort_layout(n, ctypes.byref(slots))
                sort_off += slots.value
            J["flags"][pos] = flags
        if lat_off > LAT_PACK_MAX:  # the slots are set by the library's memset instead
            J["flags"] &= ~L.F_LATTICE_READY
        for name, col in J.items():
            jobs[name] = col
        cand_pool = np.concatenate(cand_parts) if cand_parts else np.zeros(1)
        # the dense fallback first materialises its draws: a job copy whose
        # out_off points into the scratch candidate buffer
        fb_slice = _slice_of(groups, [k for k, _ in groups].index("qfb"))
        fb_jobs = jobs[fb_slice[0]:fb_slice[1]].copy()
        fb_jobs["out_off"] = fb_jobs["cand_off"]
        return (inj, lat_ranges, fallback, modes, groups, order, jobs, cand_pool, fb_jobs,
                fb_slice, out_off, lat_off, qfb_off, sort_off, cnt_off, tbl_off)

    def run(self, works: List[LabelWork], prior_weight=1.0, lf=DEFAULT_LF, precision=32,
            outputs=False, stream=None, timers=None, sample_only=False,
            pruned=True, scorer=None, posteriors=False, history=None, rows=None,
            is_below=None, histories=None, timer_groups=None,
            table_scores=False, defer=False, exchange=None) -> List[LabelResult]:
        """Run one level (``_run_level``); at precision 32 the labels scored by
        an fp32 argmax -- injected candidates, or per-candidate ``outputs`` --
        get the exact decision afterwards (``_exact_decision``), so every
        default precision-32 winner is np.argmax of the exact scores, as the
        suggest path's are.  Arguments: see ``_run_level``."""
        res = self._run_level(works, prior_weight, lf, precision, outputs, stream, timers,
                              sample_only, pruned, scorer, posteriors, history, rows, is_below,
                              histories, timer_groups, table_scores, defer, exchange)
        if precision == 32 and isinstance(works, list) and res and not (
                sample_only or posteriors or table_scores or exchange is not None) and \
                (scorer in (None, "auto") and pruned):
            redo = [i for i, w in enumerate(works) if w.kind in EXACT32_KINDS and
                    (w.cand is not None or outputs)]
            if redo:
                self._exact_decision(works, res, redo, prior_weight, lf, stream, history, rows,
                                     is_below, histories)
        return res

    def _exact_decision(self, works, res, redo, prior_weight, lf, stream, history, rows,
                        is_below, histories):
        """The exact argmax of fp32-decided labels: their candidate values
        (the injected ones, or the drawn ones read back with the outputs)
        scored again in fp64 (tpe_score_pruned64 / the dense fp64 kernel,
        index-exact against the oracle), first maximum, NaN winning
        (np.argmax, tpe.py:649-658).  Patches index / value / score in place;
        the fp32 per-candidate log-densities stay."""
        import dataclasses
        again = []
        for i in redo:
            w, r = works[i], res[i]
            cand = w.cand if w.cand is not None else r.cand
            if cand is None or np.size(cand) == 0:
                continue
            again.append((i, dataclasses.replace(w, cand=np.asarray(cand, np.float64),
                                                 n_cand=int(np.size(cand)), cand_base=0)))
        if not again:
            return
        kw = dict(history=history, rows=rows, is_below=is_below, histories=histories)
        keep = tuple(getattr(self, k, None) for k in ("last_pairs", "last_table_stats",
                                                      "last_plan"))  # the fp32 level's
        exact = self._run_level([w for _, w in again], prior_weight, lf, 64, False, stream, None,
                                False, True, None, False, **kw, timer_groups=None,
                                table_scores=False, defer=False, exchange=None)
        self.last_pairs, self.last_table_stats, self.last_plan = keep
        for (i, w), e in zip(again, exact):
            r = res[i]
            local = int(e.index)
            r.index = local if works[i].cand is not None else \
                (int(works[i].cand_base) + local if local >= 0 else local)
            r.value, r.score = e.value, e.score

    def _run_level(self, works: List[LabelWork], prior_weight=1.0, lf=DEFAULT_LF, precision=32,
                   outputs=False, stream=None, timers=None, sample_only=False,
                   pruned=True, scorer=None, posteriors=False, history=None, rows=None,
                   is_below=None, histories=None, timer_groups=None,
                   table_scores=False, defer=False, exchange=None) -> List[LabelResult]:
        """Run one level.  ``timers`` (optional dict) collects HIP event pairs
        per kernel group ("fit", "cat_fit", "cont", "lat", ...) on ``stream``;
        ``timer_groups`` (optional set) limits them to those groups (each event
        pair costs the stream a ~10 us timestamp barrier).
        ``sample_only``: fit, then only draw the candidates of the continuous
        labels (tpe_sample) into ``LabelResult.cand`` -- the sampler test hook.
        ``scorer`` picks the fp32 kernel for unquantized labels: "dense"
        (k_score32, every component), "sorted" (bucketed candidates +
        component pruning; sampled labels without per-candidate outputs),
        "table" (per-cell expansions, tpe_table_build + tpe_score_table) or
        "auto" (sampled labels: the table path from TABLE_MIN_CAND candidates,
        below it the fp32 stream scored exactly in fp64 by tpe_score_pruned64
        -- so the argmax is exact at every size; with per-candidate outputs or
        injected candidates: dense).
        ``pruned=False`` is the old spelling of scorer="dense".  fp64 always
        runs the exact dense kernel.  ``posteriors``: fit only, and return the
        fitted mixtures in ``LabelResult.extra`` ("below" / "above" as
        (w, mu, sigma) sorted by mu, "p_accept"; categorical: "p_below" /
        "p_above") -- the parity hook for adaptive_parzen_normal.
        ``history`` (DeviceHistory) + ``is_below`` (uint8 per position of
        ``rows``, or of the history rows when ``rows`` is None): every work
        names its label column (``col``) and the observation lists are
        gathered on the device (tpe_gather_obs) instead of being uploaded.
        ``histories``: a list of (DeviceHistory, rows or None, is_below) for
        batches of independent studies; each work names its history by
        ``hist`` (one tpe_gather_obs_multi launch gathers every list).
        ``works`` may be a WorkBatch (with ``histories``): the result is a
        BatchResult, and with ``defer`` a _Pending whose ``result()`` waits
        for it -- the readback is queued behind the launches and the call
        returns at once, so the host can prepare the next batch while this one
        runs (the next run on this engine first collects it).
        ``exchange``: (comm, n_labels, world, slots) -- a label-sharded level
        on one rank of ``world``: after scoring, the works' winners are folded
        into n_labels label slots (``slots``: slot per work; tpe_best_scatter)
        and all-reduced over the RCCL communicator ``comm`` (an ncclComm_t
        address; tpe_maxloc_allreduce), on the level's stream; the combined
        records (BEST_DTYPE, the same on every rank) come back with the level's
        one readback as ``self.last_exchange``."""
        if not works:
            return []
        stream_arg = stream
        if self._inflight is not None:  # its pinned buffers are about to be reused
            self._inflight.result()
        if self._replays and isinstance(works, WorkBatch) and stream is None:
            sig = _Replay.signature(self, works, prior_weight, lf, precision, outputs,
                                    self.torch.cuda.current_stream(self.device).cuda_stream,
                                    sample_only, pruned, scorer, posteriors, history, rows,
                                    is_below, histories, timers, timer_groups, table_scores,
                                    exchange)
            rp = self._replays.get(sig) if sig is not None else None
            # valid while the workspace is unchanged and the staging buffer
            # still holds this level's pack (levels that differ only in their
            # timer events share one)
            if rp is not None and rp.gen == self._gen and self._staged_sig == rp.sig[:-1]:
                out = rp.run(self, works, is_below, timers, defer)
                if out is not None:
                    return out
        if sample_only:
            outputs = True
        if scorer is None:
            scorer = "auto" if pruned else "dense"
        if scorer not in SCORERS:
            raise ValueError("scorer must be one of %s, got %r" % (SCORERS, scorer))
        torch = self.torch
        self._retired.clear()  # every earlier run ended with a synchronising readback / collect
        hp = self.host_marks  # diagnostic: list of (name, perf_counter) or None

        def _hmark(name):
            if hp is not None:
                hp.append((name, time.perf_counter()))
        _hmark("start")

        lib = self.lib
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        sp = ctypes.c_void_p(stream.cuda_stream)
        if history is not None and histories is not None:
            raise ValueError("give either history or histories")
        hist_mode = history is not None or histories is not None
        n_rows = 0  # split flags uploaded (single-history levels)
        if table_scores:  # the fast table path's per-candidate scores (test hook)
            outputs = False
        batch = works if isinstance(works, WorkBatch) else None
        if batch is not None and (not hist_mode or outputs or sample_only or posteriors or
                                  table_scores):
            raise ValueError("a WorkBatch runs with history= / histories= and no output hooks")
        works, pkey, cached, plan = self._choose_plan(
            works, batch, prior_weight, lf, precision, scorer, outputs, sample_only, hist_mode,
            histories is not None, _hmark)
        (cont, quant, cat, fit_ids, params, nf, segs, obs_pool, n_obs_total, n_comp, max_obs,
         csegs, cobs_pool, p_pool, cat_meta, cobs_off, lat_ranges, fallback, modes, groups,
         order, gathers, inj, jobs, cand_pool, fb_jobs, fb_slice, out_off, lat_off, qfb_off,
         sort_off, cnt_off, tbl_off) = plan
        if cached is not None:
            g_arr = gathers  # (a cached plan gives the gather table itself)
        pack = _Pack()
        _hmark('plan')
        # ---- upload (descriptors, jobs, injected candidates: one copy) -----------
        o_segs = pack.add(segs) if segs.size else None
        o_csegs = pack.add(csegs) if csegs.size else None
        o_p = pack.add(p_pool)
        if hist_mode:
            if cached is None:
                g_arr = np.zeros(len(gathers), L.GATHER_DTYPE)
            if cached is None and gathers:
                (g_arr["col"], g_arr["below"], g_arr["dst_off"], g_arr["offset"], g_arr["count"],
                 g_arr["to_int"], g_arr["hist"]) = (np.array(c) for c in zip(*gathers))
            o_g = pack.add(g_arr)
            if histories is None:
                # (the split flags and row list go last in the pack, after the
                # result block: a level whose history grew keeps every other
                # offset, so its records can be re-issued, _Replay)
                isb = np.ascontiguousarray(is_below, dtype=np.uint8)
                n_rows = isb.size
            else:  # row lists / flags at offsets of the staged pack (the `aux` base)
                h_arr = np.zeros(len(histories), L.HISTORY_DTYPE)
                for h, (dh, h_rows, h_isb) in enumerate(histories):
                    h_isb = np.ascontiguousarray(h_isb, dtype=np.uint8)
                    h_arr[h] = (dh.vals.data_ptr(), dh.active.data_ptr(), dh.ld, dh.n_labels,
                                h_isb.size, pack.add(np.ascontiguousarray(h_rows, np.int32))
                                if h_rows is not None else -1, pack.add(h_isb))
                    if h_rows is None and h_isb.size > dh.rows:
                        raise ValueError("history %d: %d split flags for %d rows"
                                         % (h, h_isb.size, dh.rows))
                o_h = pack.add(h_arr)
        else:
            o_obs = pack.add(obs_pool)
            o_cobs = pack.add(cobs_pool)
        # lattice first-index slots (all-ones) and compaction counts (zero) ride
        # in the upload when the level is small (TPE_F_LATTICE_READY): no memsets
        lat_g = _slice_of(groups, [k for k, _ in groups].index("lat"))
        lat_ready = lat_g[1] > lat_g[0] and bool(
            np.all(jobs["flags"][lat_g[0]:lat_g[1]] & L.F_LATTICE_READY))
        if lat_ready:
            o_slot = pack.add(self._ones(lat_off))
            o_lcnt = pack.add(np.zeros(lat_g[1] - lat_g[0], np.int64))
        o_jobs = pack.add(jobs) if jobs.size else None
        o_fb = pack.add(fb_jobs) if fb_jobs.size else None
        o_cand = pack.add(cand_pool)
        # one result block, zeroed by the upload and read back with one copy:
        # [0,16) error bits, [16,40) table stats, [40,48) sorted-path pair
        # count, [64,...) tpe_best per job
        JS, BS = L.JOB_DTYPE.itemsize, L.BEST_DTYPE.itemsize
        n_jobs = len(order)
        xbytes = 0
        if exchange is not None:
            x_comm, x_labels, x_world, x_slots = exchange
            x_slots = np.asarray(x_slots, np.int32).reshape(-1)
            if x_slots.size != len(order):
                raise ValueError("exchange: %d slots for %d works" % (x_slots.size, len(order)))
            o_xslot = pack.add(x_slots[np.asarray(order, np.int64)])
            xbytes = int(x_labels) * BS
        o_res = pack.add(np.zeros(64 + n_jobs * BS + xbytes, np.uint8))
        o_isb = o_rows = None
        if hist_mode and histories is None:
            o_isb = pack.add(isb)
            o_rows = pack.add(np.ascontiguousarray(rows, dtype=np.int32)) \
                if rows is not None else None
        native_ok = self.native and pkey is not None and not (
            outputs or sample_only or posteriors or table_scores)
        base = self._upload(pack, stream, copy=not native_ok)
        d_segs = base + o_segs if o_segs is not None else None
        d_csegs = base + o_csegs if o_csegs is not None else None
        d_res = base + o_res
        d_err, d_stats, d_pairs, d_best = d_res, d_res + 16, d_res + 40, d_res + 64
        # every workspace pointer before the first launch: the launches then
        # follow each other without host work in between
        d_w = d_mu = d_sig = d_cdf = d_c64 = d_c32 = d_logp = d_ccdf = None
        nfs = 2 * len(fit_ids)
        prune = bool(fit_ids) and any(k == "sorted" and ids for k, ids in groups)
        # the fit from the history's sorted orders (tpe_fit_sorted): one kernel
        # instead of gather + sort + merge ranks + three coefficient kernels;
        # needs the single history with its identity row list (row = tid order)
        # (it walks the history's sorted order, a permutation of rows [0, rows):
        # the split flags must cover exactly those rows -- tpe_fit_sorted reads
        # is_below[row] for every one of them)
        sorted_fit = bool(fit_ids) and self.sorted_fit and history is not None and \
            histories is None and rows is None and not prune and n_rows == history.rows
        tjobs = max([b - a for a, b in (_slice_of(groups, g) for g, (k, ids) in enumerate(groups)
                                        if k in ("table", "pruned64") and ids)], default=0)
        self._presize(n_comp, n_obs_total, max_obs, cobs_off, len(segs), tjobs,
                      n_rows if sorted_fit else 0)
        if fit_ids:
            d_w, d_mu, d_sig, d_cdf = (self._bufs[k].data_ptr() for k in ("w", "mu", "sigma",
                                                                            "wcdf"))
            d_c64, d_c32 = self._bufs["coef64"].data_ptr(), self._bufs["coef32"].data_ptr()
            d_fs = self._bufs["fit_scratch"].data_ptr()
            d_c32n = d_w32 = d_pm = d_sm = None
            if prune:
                d_c32n = self._buf("coef32n", 16 * n_comp)
                d_w32 = self._buf("wide32", 16 * n_comp)
                d_pm = self._buf("pm", 4 * n_comp)
                d_sm = self._buf("sm", 4 * n_comp)
        if cat:
            d_logp = self._buf("cat_logp", 8 * p_pool.size)
            d_ccdf = self._buf("cat_cdf", 8 * p_pool.size)
        self.last_plan = (segs, csegs, g_arr if hist_mode else None, jobs, cached is not None)
        if sorted_fit:
            history.ensure_order(self, stream, g_arr["col"][:nfs:2], segs["transform"][::2],
                                 segs["floor"][::2])

        # ---- the level's launches (eager, or recorded and re-issued) ------------
        # Every argument below is a workspace pointer (unchanged while _gen is),
        # an offset into the staged pack, or a size covered by the launch key;
        # the values that change from call to call live in the uploaded pack.
        gkey = None
        if native_ok:
            # (the per-call sizes -- history rows, observation totals, the largest
            # mixture, the pack size -- are size words of the records, rewritten
            # when a recorded level is re-issued: _Replay)
            gkey = (pkey, self._gen, sp.value, tuple(off for off, _ in pack.parts), lat_off,
                    (history.vals.data_ptr(), history.active.data_ptr(), history.ld,
                     history.order.data_ptr() if sorted_fit else None, rows is None)
                    if history is not None else None,
                    None if exchange is None else
                    (int(x_comm), int(x_labels), int(x_world), x_slots.tobytes()),
                    self.side_stream, self.table_scorer, self.exact64, self.lat_prefix,
                    self.cat_early, self.cat_issue, self.cat_hist, self.lat_main,
                    self.lat_max_slots,
                    "off" if timers is None else
                    ("all" if timer_groups is None else frozenset(timer_groups)))
        band_jobs = []  # (first, end) job positions scored by tpe_score_table_fast
        ctx = _LaunchCtx(self, stream, timers, timer_groups)
        here = locals()  # (outside the comprehension: its own scope)
        lv = _LevelState(**{k: v for k, v in here.items() if k in _LAUNCH_STATE})

        nbytes = 64 + n_jobs * BS + xbytes  # the result block read back at the end
        ops, table_calls, band_jobs, post = self._issue_level(
            lv, ctx, gkey, nbytes, d_res, batch is not None,
            dict(n_rows=n_rows, max_obs=max_obs, n_obs_total=n_obs_total, max_comp=max_obs + 1,
                 pack_size=pack.size))
        if post:
            return table_calls
        _hmark('score launches')
        # the exact re-score of a band that overflowed (a plateau of equal fp32
        # scores; tpe_score_table_fast leaves n_scored = -1): after the readback
        fix = None
        if band_jobs:
            fix = functools.partial(self._band_fix, list(band_jobs), d_segs, max_obs + 1, n_comp,
                                    sp.value, exchange is not None)
        xinfo = None
        if exchange is not None:  # (comm, labels, world, slot per job in launch order, stream)
            xinfo = (int(x_comm), int(x_labels), int(x_world),
                     x_slots[np.asarray(order, np.int64)].copy(), sp.value)
        # ---- results: one device->host copy of the result block into pinned memory
        # (issued by the records themselves on the native path)
        pin = self._res_pinned(nbytes)
        if ops is None:
            L.hip_check(self._hip.hipMemcpyAsync(pin.data_ptr(), d_res, nbytes, L.D2H, sp),
                        "hipMemcpyAsync")
        after = None
        if ops is not None and ops.timed and timers is not None:
            after = functools.partial(ops.read_timers, self._hip, timers)
        if batch is not None:  # queued readback (see _Pending)
            ev = self._event("result")
            if ops is None:
                L.hip_check(self._hip.hipEventRecord(ev, sp), "hipEventRecord")
            p = self._inflight = _Pending(self, ev, pin, nbytes, np.asarray(order, np.int64),
                                          64 + n_jobs * BS if xbytes else None,
                                          bool(table_calls), after, fix, jobs, xinfo)
            if ops is not None and self._oplists.get(gkey) is ops and history is not None:
                # a recorded level: the next call with the same signature only
                # rewrites its keys and split flags in the staged pack (_Replay)
                sig = _Replay.signature(self, works, prior_weight, lf, precision, outputs,
                                        (sp.value or 0) if stream_arg is None else None,
                                        sample_only,
                                        pruned, scorer, posteriors,
                                        history, rows, is_below, histories, timers,
                                        timer_groups, table_scores, exchange)
                if sig is not None:
                    if len(self._replays) >= 8:
                        self._replays.clear()
                    self._replays[sig] = _Replay(
                        sig, self._gen, ops, self._pinned[0], pkey, p, pin,
                        dict(segs=o_segs, csegs=o_csegs, g=o_g, jobs=o_jobs, fb=o_fb, isb=o_isb),
                        history if sorted_fit else None, tjobs,
                        (list(band_jobs), d_segs, sp.value, exchange is not None, xinfo))
                    self._staged_sig = sig[:-1]
            return p if defer else p.result()
        return self._read_results(stream, sp, ops is None, after, pin, nbytes, n_jobs, fix, jobs,
                                  xbytes, groups, table_calls, outputs, table_scores, out_off,
                                  works, order, cont, modes, _hmark, xinfo)


    def _issue_level(self, lv, ctx, gkey, nbytes, d_res, queued, sizes):
        """Issue a prepared level's stream work: re-issue its recorded records
        from C (tpe_run_ops); record them first on the second call in a row
        with launch key ``gkey`` (None: the level is not recordable); or launch
        eagerly, the deferred upload first.  ``queued``: the recorded readback
        ends with an event (a WorkBatch, _Pending) instead of a stream sync.
        ``sizes``: this call's size words of the records.
        Returns (ops or None, table_calls, band_jobs, posteriors_done)."""
        sp = lv.sp
        ops = None
        if gkey is not None:
            ops = self._oplists.get(gkey)
            if ops is None and gkey == self._last_gkey:
                # the second call in a row with this launch key: record the
                # level's stream work once, re-issue it from C on later calls
                gen0 = self._gen
                rec = _OpList(self.lib)
                dst, src, nb = self._staged
                rec.add(L.OP_MEMCPY, dst, src, _V("pack_size", nb), L.H2D, sp)
                ctx.cap = rec
                try:
                    rec.table_calls, _ = self._launch_level(lv, ctx, rec)
                    rec.band_jobs = list(lv.band_jobs)
                finally:
                    ctx.cap = None
                pin = self._res_pinned(nbytes)
                rec.add(L.OP_MEMCPY, pin.data_ptr(), d_res, nbytes, L.D2H, sp)
                if queued:
                    rec.add(L.OP_EVENT_RECORD, self._event("result"), sp)
                else:
                    rec.add(L.OP_STREAM_SYNC, sp)
                rec.finish((lv.jobs, lv.fb_jobs, lv.g_arr if lv.hist_mode else None,
                            lv.h_arr if lv.histories is not None else None), sp.value or 0)
                if self._gen == gen0:  # every recorded pointer is still the live one
                    if len(self._oplists) >= 16 or any(
                            k[1] != gen0 for k in self._oplists):
                        self._drop_oplists()
                    self._oplists[gkey] = rec
                else:
                    if self._oplist_once is not None:
                        self._oplist_once.destroy(self._hip)
                    self._oplist_once = rec  # this call's only (its events freed later)
                ops = rec
            if ops is None:  # eager: the deferred upload first
                dst, src, nb = self._staged
                L.hip_check(self._hip.hipMemcpyAsync(dst, src, nb, L.H2D, sp), "hipMemcpyAsync")
        if ops is None:
            table_calls, post = self._launch_level(lv, ctx)
            if not post:
                self._last_gkey = gkey
                self.graph_stats["eager"] += 1
            return None, table_calls, lv.band_jobs, post
        ops.set_sizes(sizes)
        keep = ops.keep  # the host copies the entry points validate: this call's
        keep[0][...] = lv.jobs
        keep[1][...] = lv.fb_jobs
        if keep[2] is not None:
            keep[2][...] = lv.g_arr
        ops.issue(self)
        self.graph_stats["native"] = self.graph_stats.get("native", 0) + 1
        return ops, ops.table_calls, ops.band_jobs, False

    def _launch_level(self, lv, ctx, lib=None):
        """The level's launches, in stream order: the body of run() for a prepared
        level (``lv``: its plan, workspace pointers and pack offsets; ``ctx``: the
        timer / stream-ordering helpers, which follow a recording _OpList).
        ``lib`` is the library, or the _OpList the launches are recorded into.
        Stages: the gather (_launch_gather), the posterior fit (_launch_fit),
        the scorers, one call per group (_launch_group), then the join of the
        side stream and the cross-rank exchange.
        Returns (table_calls, posteriors_done)."""
        if lib is None:
            lib = self.lib
        sp, cat, groups, hist_mode = lv.sp, lv.cat, lv.groups, lv.hist_mode
        # quantized labels on the main stream when it has no scorer of its own
        # (a level of quantized and categorical labels only -- C5's middle
        # level): the lattice work then runs beside the categorical chain on
        # the side stream instead of after it
        has_q = any(ids for k, ids in groups if k in SIDE_KINDS and k != "cat")
        lat_main = self.lat_main and has_q and not any(
            ids for k, ids in groups if k not in SIDE_KINDS)
        side = None
        if self.side_stream != "0" and not lv.sample_only and not lv.posteriors and any(
                ids for k, ids in groups if k in SIDE_KINDS and not (lat_main and k != "cat")):
            if self._side is None:
                self._side = lv.torch.cuda.Stream(self.device)
            side = self._side
        side_p = ctypes.c_void_p(side.cuda_stream) if side is not None else sp
        st = _LaunchState(
            lib=lib, ctx=ctx, side=side, side_p=side_p,
            # with the sorted fit the gather only lists the categorical labels'
            # observations, which only their posterior (side stream) reads: it
            # runs there, behind an event after the upload, and the main
            # stream starts with the fit
            gather_side=hist_mode and lv.histories is None and lv.sorted_fit and
            side is not None and bool(cat) and self.cat_early,
            # the categorical posteriors can count their labels in the history
            # itself (no gathered lists): the gather then lists only the fit's
            # sets, and none with the sorted fit (it reads the history itself)
            cat_hist=hist_mode and lv.histories is None and bool(cat) and self.cat_hist,
            # categorical labels need only the gathered lists: with cat_early
            # the side stream starts their posterior and scoring from an event
            # recorded after the gather, so they run beside the latency-bound
            # fit kernels instead of the VALU-bound table build and scorer
            # (issued on the host after the fit's launches: the fit is not
            # delayed, and the table build still reaches the GPU before the
            # fit ends)
            cat_early=side is not None and bool(cat) and self.cat_early,
            joined=side is None, side_started=side is None, cat_started=False,
            table_calls=[], jobs_ptr=lv.jobs.__array_interface__["data"][0],
            d_obs=None, d_cobs=None, lat_main=lat_main)
        self._launch_gather(lv, st)
        lv._hmark('upload+gather')
        # side stream (TPE_SIDE_STREAM != "0"): quantized and categorical work
        # overlaps the continuous pipeline; the categorical posterior starts on
        # it as soon as the lists are gathered (it needs nothing else)
        # main-stream issue order: gather, fit, table build, scorers; the
        # side stream's launches are issued after the table build (host
        # launches cost a few us each: at a one-eighth label share the main
        # stream would otherwise idle behind them) and start
        # from one event recorded on the main stream after the fit (the
        # categorical posterior could start at the gather, but the side
        # stream has the slack and the fork costs two more host calls)
        st.d_cand = lv.base + lv.o_cand
        st.d_bl = st.d_al = st.d_x = st.d_sc = st.d_eps = None
        if lv.outputs:
            st.d_bl = self._buf("out_bl", 8 * max(lv.out_off, 1))
            st.d_al = self._buf("out_al", 8 * max(lv.out_off, 1))
            st.d_x = self._buf("out_x", 8 * max(lv.out_off, 1))
        elif lv.table_scores:
            st.d_sc = self._buf("out_sc", 8 * max(lv.out_off, 1))
            st.d_x = self._buf("out_x", 8 * max(lv.out_off, 1))
            st.d_eps = self._buf("out_eps", 8 * max(lv.out_off, 1))
        lv.band_jobs.clear()
        if st.cat_early:
            if not st.gather_side:
                ctx.stream_rec("gathered", sp)
            if self.cat_issue == "pre":  # issued before the fit's launches
                for g, (k, ids) in enumerate(groups):
                    if k == "cat" and ids:
                        self._launch_group(lv, st, g, "all")
        self._launch_fit(lv, st)
        if cat and side is None:
            self._cat_fit(lv, st)
        if lv.posteriors:
            return self._read_posteriors(lv.works, lv.fit_ids, cat, lv.segs, lv.csegs,
                                         lv.n_comp, lv.p_pool.size, lv.d_segs, lv.stream,
                                         lv.o_p), True
        lv._hmark('jobs')
        lv._hmark('fit')
        # ---- scoring, one call per group ----------------------------------------
        # quantized and categorical groups go to the side stream (after the job
        # table has landed); continuous groups stay on `stream`
        if side is not None and not lat_main:  # quantized groups need the continuous fit
            ctx.stream_rec("fitted", sp)
        for g, stage in self._group_order(lv, st):
            self._launch_group(lv, st, g, stage)
        if not st.side_started:  # (no side group: only the categorical posterior)
            if cat and not st.cat_early:
                self._cat_fit(lv, st)
        if not st.joined:  # join before the readback
            ctx.stream_order("joined", side_p, sp)
        if lv.exchange is not None:  # label-sharded level: the cross-rank argmax
            BS = lv.BS
            d_xl = self._buf("xchg_local", lv.x_labels * BS)
            d_xg = self._buf("xchg_gathered", lv.x_world * lv.x_labels * BS)
            L.check(lib.tpe_best_scatter(lv.d_best, lv.base + lv.o_xslot, lv.n_jobs, d_xl,
                                         lv.x_labels, sp), "tpe_best_scatter")
            L.check(lib.tpe_maxloc_allreduce(d_xl, d_xg, lv.d_best + lv.n_jobs * BS,
                                             lv.x_labels, lv.x_comm, sp),
                    "tpe_maxloc_allreduce")
        return st.table_calls, False

    def _group_order(self, lv, st):
        """(group, stage) in host issue order.  Without a side stream: group
        order.  With one: the first sampled table group's build (the main
        stream's next kernels after the fit), then the side groups, then the
        main-stream scorers -- the host issues launches at a few us each, and
        at a one-eighth label share the main stream would otherwise sit idle
        behind the side stream's launches."""
        groups, inj = lv.groups, lv.inj
        if st.side is None:
            return [(g, "all") for g in range(len(groups))]
        early = None
        tgroups = [g for g, (k, ids) in enumerate(groups) if k == "table" and ids]
        if len(tgroups) == 1 and not inj(groups[tgroups[0]][1][0]):
            early = tgroups[0]  # (one table group: the workspace tables are its own)
        side_gs = [g for g in range(len(groups)) if groups[g][0] in SIDE_KINDS]
        # categorical groups first, issued right after the fit's launches
        # (they wait for the gather only, so they run beside the fit; the
        # table build is still issued before the fit ends)
        cat_gs = [g for g in side_gs if st.cat_early and groups[g][0] == "cat"]
        pre = [(g, "all") for g in cat_gs] if self.cat_issue == "post" else []
        late = [(g, "all") for g in cat_gs] if self.cat_issue == "late" else []
        return pre + ([(early, "build")] if early is not None else []) + late + \
            [(g, "all") for g in side_gs if g not in cat_gs] + \
            [(g, "score" if g == early else "all") for g in range(len(groups))
             if groups[g][0] not in SIDE_KINDS]

    def _launch_gather(self, lv, st):
        """The observation lists of the level's fit and categorical sets
        (tpe_gather_obs / tpe_gather_obs_multi), or the uploaded lists."""
        lib, ctx, sp = st.lib, st.ctx, lv.sp
        if not lv.hist_mode:
            st.d_obs, st.d_cobs = lv.base + lv.o_obs, lv.base + lv.o_cobs
            return
        nfs, g_arr, base, history = lv.nfs, lv.g_arr, lv.base, lv.history
        g0 = nfs if lv.sorted_fit else 0
        g1 = nfs if st.cat_hist else (len(g_arr) if g_arr is not None else 0)
        # (the categorical descriptors follow the fit's)
        st.d_obs = d_obs = self._buf("obs_dev", 8 * max(lv.n_obs_total, 1))
        st.d_cobs = d_cobs = self._buf("cobs_dev", 8 * max(lv.cobs_off, 1))
        gs, gsp = (st.side, st.side_p) if st.gather_side else (None, sp)
        if st.gather_side:
            ctx.stream_order("uploaded", sp, st.side_p)
        e0 = ctx.tick("gather", gs)
        if lv.histories is None:
            if g1 > g0:
                GI = L.GATHER_DTYPE.itemsize
                L.check(lib.tpe_gather_obs(history.vals.data_ptr(), history.active.data_ptr(),
                                           history.ld,
                                           base + lv.o_rows if lv.o_rows is not None else None,
                                           _V("n_rows", lv.n_rows), base + lv.o_isb,
                                           base + lv.o_g + g0 * GI, g_arr.ctypes.data + g0 * GI,
                                           g1 - g0, d_obs, d_cobs, lv.d_err, gsp),
                        "tpe_gather_obs")
        else:
            h_arr = lv.h_arr
            L.check(lib.tpe_gather_obs_multi(base + lv.o_h, h_arr.ctypes.data_as(ctypes.c_void_p),
                                             len(h_arr), base, base + lv.o_g,
                                             g_arr.ctypes.data_as(ctypes.c_void_p),
                                             len(g_arr), d_obs, d_cobs, lv.d_err, sp),
                    "tpe_gather_obs_multi")
        ctx.tock("gather", e0, gs)

    def _launch_fit(self, lv, st):
        """The continuous labels' posterior fit: tpe_fit_sorted (reads the
        history in its value order) or tpe_parzen_fit (the gathered lists)."""
        if not lv.fit_ids:
            return
        lib, ctx, sp = st.lib, st.ctx, lv.sp
        e0 = ctx.tick("fit")
        if lv.sorted_fit:
            history = lv.history
            d_fss = self._buf("fit_sorted_scratch",
                              lib.tpe_fit_sorted_scratch_bytes(len(lv.segs), lv.n_rows))
            L.check(lib.tpe_fit_sorted(history.vals.data_ptr(), history.active.data_ptr(),
                                       history.ld, history.order.data_ptr(),
                                       _V("n_rows", lv.n_rows),
                                       lv.base + lv.o_isb, lv.base + lv.o_g, lv.g_arr.ctypes.data,
                                       lv.d_segs, len(lv.segs), d_fss, lv.d_w, lv.d_mu, lv.d_sig,
                                       lv.d_cdf, lv.d_c64, lv.d_c32, lv.d_err, sp),
                    "tpe_fit_sorted")
        else:
            L.check(lib.tpe_parzen_fit(st.d_obs, lv.d_fs, lv.d_segs, len(lv.segs),
                                       _V("max_obs", lv.max_obs),
                                       _V("n_obs_total", lv.n_obs_total),
                                       lv.d_w, lv.d_mu, lv.d_sig, lv.d_cdf, lv.d_c64, lv.d_c32,
                                       lv.d_c32n, lv.d_w32, lv.d_pm, lv.d_sm, sp),
                    "tpe_parzen_fit")
        ctx.tock("fit", e0)

    def _cat_fit(self, lv, st):
        """The categorical posteriors (on the side stream, after its fork):
        counted in the history itself (tpe_cat_posterior_hist) or from the
        gathered lists (tpe_cat_posterior)."""
        lib, ctx, side, side_p, csegs = st.lib, st.ctx, st.side, st.side_p, lv.csegs
        e0 = ctx.tick("cat_fit", side)
        d_p = lv.base + lv.o_p  # the posterior is formed in place in the staged pool
        if st.cat_hist:  # (the categorical gather descriptors follow the fit's nfs)
            history = lv.history
            max_cat = int(csegs["n_cat"].max())
            # a long history is counted in row chunks (work sized for the
            # history's capacity: it holds while the history does)
            ws = max(0, int(lib.tpe_cat_hist_scratch_bytes(len(csegs), max_cat, history.ld))) \
                if self.cat_chunked else 0
            d_ws = self._buf("cat_hist_ws", ws) if ws else None
            L.check(lib.tpe_cat_posterior_hist(
                history.vals.data_ptr(), history.active.data_ptr(), history.ld,
                lv.base + lv.o_rows if lv.o_rows is not None else None, _V("n_rows", lv.n_rows),
                lv.base + lv.o_isb, lv.base + lv.o_g + lv.nfs * L.GATHER_DTYPE.itemsize,
                lv.d_csegs, len(csegs), max_cat, d_p, lv.d_logp, lv.d_ccdf, d_ws, ws,
                lv.d_err, side_p), "tpe_cat_posterior_hist")
        else:
            L.check(lib.tpe_cat_posterior(st.d_cobs, lv.d_csegs, len(csegs),
                                          int(csegs["n_cat"].max()), d_p, lv.d_logp, lv.d_ccdf,
                                          side_p), "tpe_cat_posterior")
        ctx.tock("cat_fit", e0, side)

    def _launch_group(self, lv, st, g, stage):
        """One group's scorer launches (``stage``: "all", or "build" / "score"
        -- the two halves of an early-built table group), after the side
        stream's fork where the group is the first to need it."""
        kind, ids = lv.groups[g]
        if not ids:
            return
        ctx = st.ctx
        if st.cat_early and kind == "cat" and not st.cat_started:
            st.cat_started = True  # the categorical work needs only the gather
            if not st.gather_side:  # (else the gather ran on the side stream)
                ctx.stream_wait("gathered", st.side_p)
            self._cat_fit(lv, st)
        side_kind = kind in SIDE_KINDS and not (st.lat_main and kind != "cat")
        if not st.side_started and side_kind and not (st.cat_early and kind == "cat"):
            st.side_started = True  # the side stream's groups that need the fit
            ctx.stream_wait("fitted", st.side_p)
            if lv.cat and not st.cat_early:
                self._cat_fit(lv, st)
        a, b = _slice_of(lv.groups, g)
        if lv.sample_only:
            if kind in ("cont", "lat", "qfb"):
                L.check(st.lib.tpe_sample(lv.base + lv.o_jobs + a * L.JOB_DTYPE.itemsize,
                                          lv.jobs[a:b].ctypes.data_as(ctypes.c_void_p), b - a,
                                          lv.d_segs, lv.d_mu, lv.d_sig, lv.d_cdf, lv.precision,
                                          st.d_x, lv.sp), "tpe_sample")
            return
        on_side = st.side is not None and side_kind
        kst = st.side if on_side else None
        sl = _LaunchState(
            kind=kind, ids=ids, a=a, b=b, nj=b - a, hj=lv.jobs[a:b],
            hjp=st.jobs_ptr + a * lv.JS,  # host copy of the slice (plain int: no ctypes object)
            dj=lv.base + lv.o_jobs + a * lv.JS, db=lv.d_best + a * lv.BS,
            ks=st.side_p if on_side else lv.sp,
            pname="partial_side" if on_side else "partial", stage=stage,
            e0=ctx.tick({"sorted": "sort", "table": "table_build"}.get(kind, kind), kst)
            if stage != "score" else None)
        e0 = _GROUP_LAUNCH[kind](self, lv, st, sl)
        ctx.tock(kind, e0, kst)

    def _score_cont(self, lv, st, sl):
        """Dense scoring of continuous labels (k_score64 / k_score32)."""
        npart = st.lib.tpe_score_partials(sl.hjp, sl.nj)
        d_part = self._buf("partial", 32 * max(npart, 1))
        L.check(st.lib.tpe_score_continuous(sl.dj, sl.hjp, sl.nj, lv.d_segs, lv.d_w, lv.d_mu,
                                            lv.d_sig, lv.d_cdf, lv.d_c64, lv.d_c32, st.d_cand,
                                            lv.precision, st.d_bl, st.d_al, st.d_x, d_part,
                                            npart, sl.db, lv.sp), "tpe_score_continuous")
        return sl.e0

    def _score_sorted(self, lv, st, sl):
        """Bucketed candidates with component pruning (tpe_sort_candidates +
        tpe_score_sorted)."""
        lib, ctx, sp = st.lib, st.ctx, lv.sp
        npart = lib.tpe_score_partials(sl.hjp, sl.nj) * 2
        d_part = self._buf("partial", 32 * max(npart, 1))
        d_cnt = self._buf("sort_cnt", 8 * max(lv.cnt_off, 1))
        d_gen = self._buf("sort_gen", 4 * max(lv.sort_off, 1))
        d_sx = self._buf("sort_x", 4 * max(lv.sort_off, 1))
        d_si = self._buf("sort_i", 4 * max(lv.sort_off, 1))
        L.check(lib.tpe_sort_candidates(sl.dj, sl.hjp, sl.nj, lv.d_segs, lv.d_mu, lv.d_sig,
                                        lv.d_cdf, d_cnt, d_gen, d_sx, d_si, sp),
                "tpe_sort_candidates")
        ctx.tock("sort", sl.e0)
        e0 = ctx.tick("sorted")
        L.check(lib.tpe_score_sorted(sl.dj, sl.hjp, sl.nj, lv.d_segs, lv.d_c32, lv.d_c32n,
                                     lv.d_w32, lv.d_pm, lv.d_sm, d_sx, d_si, d_part, npart,
                                     sl.db, lv.d_pairs, sp), "tpe_score_sorted")
        return e0

    def _score_table(self, lv, st, sl):
        """The cell-table path: tpe_table_build, then tpe_score_table (per-
        candidate outputs, injected candidates) or the suggest path's fp32
        cubic scorer + exact fp64 band re-score (tpe_score_table_fast +
        tpe_band_rescore).  Stage "build" / "score": the two halves of an
        early-built group."""
        lib, ctx, sp = st.lib, st.ctx, lv.sp
        hj, hjp, dj, nj, stage, n_comp = sl.hj, sl.hjp, sl.dj, sl.nj, sl.stage, lv.n_comp
        npart = lib.tpe_table_partials(hjp, nj)
        d_part = self._buf("partial", 32 * max(npart, 1))
        d_tab = self._buf("tables", L.TABLE_DTYPE.itemsize * nj)
        d_cells = self._buf("cells", 128 * int(hj["tbl_off"].max() + TABLE_CAP
                                               - hj["tbl_off"].min()))
        d_cells -= 128 * int(hj["tbl_off"].min())
        d_rh = self._buf("reach_hi", 8 * n_comp)
        d_rl = self._buf("reach_lo", 8 * n_comp)
        d_wide = self._buf("wide_idx", 4 * n_comp)
        max_comp = _V("max_comp", lv.max_obs + 1)
        d_tsc = self._buf("table_scratch", lib.tpe_table_scratch_bytes(nj, max_comp))
        if stage != "score":
            L.check(lib.tpe_table_build(dj, hjp, nj, lv.d_segs, lv.d_mu, lv.d_sig, lv.d_c64,
                                        max_comp, d_rh, d_rl, d_wide, d_tsc, d_tab, d_cells,
                                        lv.d_stats, sp), "tpe_table_build")
            ctx.tock("table_build", sl.e0)
        if stage == "build":
            return None
        if not st.joined and self.side_stream == "2":
            ctx.stream_order("joined", st.side_p, sp)
            st.joined = True
        e0 = ctx.tick("table")
        if lv.outputs or lv.inj(sl.ids[0]) or self.table_scorer == "poly":
            L.check(lib.tpe_score_table(dj, hjp, nj, lv.d_segs, lv.d_mu, lv.d_sig, lv.d_cdf,
                                        lv.d_c32, d_tab, d_cells, st.d_cand, st.d_bl, st.d_al,
                                        st.d_x, d_part, npart, sl.db, lv.d_stats, sp),
                    "tpe_score_table")
        else:  # the suggest path: one score cubic per candidate, exact argmax
            ctl_b, work_b = ctypes.c_int64(0), ctypes.c_int64(0)
            nbb = lib.tpe_band_bytes(hjp, nj, ctypes.byref(ctl_b), ctypes.byref(work_b))
            d_band = self._buf("band", nbb)
            d_bctl = self._buf("band_ctl", ctl_b.value)
            d_bwork = self._zbuf("band_work", work_b.value)
            L.check(lib.tpe_score_table_fast(dj, hjp, nj, lv.d_segs, lv.d_mu, lv.d_sig,
                                             lv.d_cdf, lv.d_c32, d_tab, d_cells, d_band, d_bctl,
                                             st.d_sc, st.d_x, st.d_eps, d_part, npart,
                                             BAND_TILE_CAP, lv.d_stats, sp),
                    "tpe_score_table_fast")
            ctx.tock("table", e0)
            self._tables_slice = (sl.a, sl.b)  # (the test hook reads these tables back)
            e0 = ctx.tick("band")
            L.check(lib.tpe_band_rescore(dj, hjp, nj, lv.d_segs, lv.d_c64, d_tab, d_band, d_bctl,
                                         d_part, npart, sl.db, d_bwork, sp), "tpe_band_rescore")
            ctx.tock("band", e0)
            e0 = None
            lv.band_jobs.append((sl.a, sl.b))
        st.table_calls.append(nj)
        return e0

    def _score_pruned64(self, lv, st, sl):
        """The fp32 candidate stream scored exactly in fp64 with component
        pruning (tpe_score_pruned64; sampled labels below TABLE_MIN_CAND)."""
        lib, n_comp = st.lib, lv.n_comp
        npart = lib.tpe_pruned64_partials(sl.hjp, sl.nj)
        d_part = self._buf("partial", 32 * max(npart, 1))
        d_tab = self._buf("tables", L.TABLE_DTYPE.itemsize * sl.nj)
        d_rh = self._buf("reach_hi", 8 * n_comp)
        d_rl = self._buf("reach_lo", 8 * n_comp)
        d_wide = self._buf("wide_idx", 4 * n_comp)
        max_comp = _V("max_comp", lv.max_obs + 1)
        d_tsc = self._buf("table_scratch", lib.tpe_table_scratch_bytes(sl.nj, max_comp))
        L.check(lib.tpe_score_pruned64(sl.dj, sl.hjp, sl.nj, lv.d_segs, lv.d_mu, lv.d_sig,
                                       lv.d_cdf, lv.d_c64, max_comp, d_rh, d_rl, d_wide, d_tsc,
                                       d_tab, st.d_cand, st.d_bl, st.d_al, st.d_x, d_part, npart,
                                       sl.db, lv.sp), "tpe_score_pruned64")
        return sl.e0

    def _score_lat(self, lv, st, sl):
        """Quantized labels scored on their value lattice: the prefix-first
        tpe_lattice_suggest, or sample + compact + tpe_score_quantized.  The
        lattice values' component windows come from k_qreach, on the quantized
        jobs' own components of the reach arrays."""
        lib, hj, hjp, dj, nj, ks = st.lib, sl.hj, sl.hjp, sl.dj, sl.nj, sl.ks
        d_rh = self._buf("reach_hi", 8 * lv.n_comp)
        d_rl = self._buf("reach_lo", 8 * lv.n_comp)
        d_vals = self._buf("lat_vals", 8 * lv.lat_off)
        d_first = self._buf("lat_first", 8 * lv.lat_off)
        if lv.lat_ready:
            d_slot, d_cnt = lv.base + lv.o_slot, lv.base + lv.o_lcnt
        else:
            d_slot = self._buf("lat_slot", 8 * lv.lat_off)
            d_cnt = self._buf("lat_cnt", 8 * nj)
        max_vals = int(hj["lat_n"].max())
        if self.lat_prefix and max_vals <= self.lat_max_slots and \
                int(hj["n_cand"].max()) > self.lat_prefix:
            # prefix first: the rest of a stream only where an unseen value
            # could still win (tpe_lattice_suggest)
            npart = nj * max_vals
            d_part = self._buf(sl.pname, 32 * npart)
            d_need = self._buf("lat_need", 4 * nj)
            L.check(lib.tpe_lattice_suggest(dj, hjp, nj, lv.d_segs, lv.d_w, lv.d_mu, lv.d_sig,
                                            lv.d_cdf, d_slot, self.lat_prefix, d_part, npart,
                                            d_need, sl.db, lv.d_err, d_rh, d_rl, ks),
                    "tpe_lattice_suggest")
        else:
            L.check(lib.tpe_lattice_sample(dj, hjp, nj, lv.d_segs, lv.d_mu, lv.d_sig, lv.d_cdf,
                                           d_slot, lv.d_err, ks), "tpe_lattice_sample")
            L.check(lib.tpe_lattice_compact(dj, hjp, nj, d_slot, d_vals, d_first, d_cnt, ks),
                    "tpe_lattice_compact")
            npart = lib.tpe_quantized_partials(hjp, nj, max_vals)
            d_part = self._buf(sl.pname, 32 * max(npart, 1))
            L.check(lib.tpe_score_quantized(dj, hjp, nj, lv.d_segs, lv.d_w, lv.d_mu, lv.d_sig,
                                            d_vals, d_first, d_cnt, max_vals, None, None, d_part,
                                            npart, sl.db, lv.d_err, d_rh, d_rl, ks),
                    "tpe_score_quantized")
        return sl.e0

    def _score_quantized(self, lv, st, sl):
        """Quantized labels scored on their candidates: fallback draws
        ("qfb", tpe_sample first) or injected candidates ("qinj")."""
        lib, hjp, nj, ks = st.lib, sl.hjp, sl.nj, sl.ks
        d_rh = self._buf("reach_hi", 8 * lv.n_comp)
        d_rl = self._buf("reach_lo", 8 * lv.n_comp)
        vals = st.d_cand
        if sl.kind == "qfb":
            vals = self._buf("q_cand", 8 * max(lv.qfb_off, 1))
            L.check(lib.tpe_sample(lv.base + lv.o_fb,
                                   lv.fb_jobs.ctypes.data_as(ctypes.c_void_p), nj, lv.d_segs,
                                   lv.d_mu, lv.d_sig, lv.d_cdf, 64, vals, ks), "tpe_sample")
        max_vals = int(sl.hj["n_cand"].max())
        npart = lib.tpe_quantized_partials(hjp, nj, max_vals)
        d_part = self._buf(sl.pname, 32 * max(npart, 1))
        L.check(lib.tpe_score_quantized(sl.dj, hjp, nj, lv.d_segs, lv.d_w, lv.d_mu, lv.d_sig,
                                        vals, None, None, max_vals, st.d_bl, st.d_al, d_part,
                                        npart, sl.db, lv.d_err, d_rh, d_rl, ks),
                "tpe_score_quantized")
        return sl.e0

    def _score_cat(self, lv, st, sl):
        """Categorical labels: the prefix-first tpe_categorical_suggest, or
        tpe_score_categorical (per-candidate outputs, injected candidates)."""
        lib, hj, hjp, nj, ks = st.lib, sl.hj, sl.hjp, sl.nj, sl.ks
        npart = lib.tpe_categorical_partials(hjp, nj)
        d_part = self._buf(sl.pname, 32 * max(npart, 1))
        if self.lat_prefix and not lv.inj(sl.ids[0]) and st.d_bl is None and st.d_x is None \
                and int(hj["n_cand"].max()) > self.lat_prefix:
            # prefix first: the rest of a stream only where an unseen better
            # category could still be drawn (tpe_categorical_suggest)
            d_need = self._buf("cat_need", 4 * nj)
            L.check(lib.tpe_categorical_suggest(sl.dj, hjp, nj, lv.d_csegs, lv.d_logp, lv.d_ccdf,
                                                self.lat_prefix, d_part, npart, d_need, sl.db,
                                                ks), "tpe_categorical_suggest")
        else:
            L.check(lib.tpe_score_categorical(sl.dj, hjp, nj, lv.d_csegs, lv.d_logp, lv.d_ccdf,
                                              st.d_cand, st.d_bl, st.d_al, st.d_x, d_part, npart,
                                              sl.db, ks), "tpe_score_categorical")
        return sl.e0

    def _read_results(self, stream, sp, sync, after, pin, nbytes, n_jobs, fix, jobs, xbytes,
                      groups, table_calls, outputs, table_scores, out_off, works, order, cont,
                      modes, _hmark, xinfo=None):
        """The level's synchronous readback: the result block (error bits, table
        stats, one tpe_best per job, the exchange's label records) from the
        pinned copy, the overflowed bands' exact re-score, per-candidate
        outputs of the test hooks; one LabelResult per work."""
        BS = L.BEST_DTYPE.itemsize
        if sync:
            L.hip_check(self._hip.hipStreamSynchronize(sp), "hipStreamSynchronize")
        if after is not None:
            after()
        res_h = pin[:nbytes].numpy().copy()
        best_h = res_h[64:64 + n_jobs * BS].view(L.BEST_DTYPE)
        if fix is not None:
            fix(best_h, jobs)
        self.last_exchange = res_h[64 + n_jobs * BS:].view(L.BEST_DTYPE).copy() if xbytes \
            else None
        if xbytes:
            self.last_exchange = self._exchange_fix(best_h, self.last_exchange, xinfo)
        with self.torch.cuda.stream(stream):
            err = int(res_h[:4].view(np.int32)[0])
            self.last_pairs = None
            if any(k == "sorted" and ids for k, ids in groups):
                self.last_pairs = int(res_h[40:48].view(np.int64)[0])
            self.last_table_stats = None
            if table_calls:
                st = res_h[16:40].view(np.int64).tolist()
                self.last_table_stats = {"exact_candidates": st[0], "failed_cells": st[1],
                                         "failed_score_cells": st[2]}
            outs = None
            if outputs:
                outs = [self._bufs[k][:8 * max(out_off, 1)].to("cpu").numpy().view(np.float64)
                        for k in ("out_bl", "out_al", "out_x")]
            elif table_scores:
                outs = [self._bufs[k][:8 * max(out_off, 1)].to("cpu").numpy().view(np.float64)
                        for k in ("out_sc", "out_x", "out_eps")]
                ta, tb = self._tables_slice
                tabs = self._bufs["tables"][:L.TABLE_DTYPE.itemsize * (tb - ta)].to("cpu") \
                    .numpy().view(L.TABLE_DTYPE)
        _raise_errors(err)
        _hmark('readback')
        results = [None] * len(works)
        b_idx, b_val = best_h["index"].tolist(), best_h["value"].tolist()
        b_sc, b_ns = best_h["score"].tolist(), best_h["n_scored"].tolist()
        for pos, i in enumerate(order):
            w = works[i]
            r = LabelResult(w.label, b_idx[pos], b_val[pos], b_sc[pos], b_ns[pos])
            if outputs:
                o, n = int(jobs[pos]["out_off"]), int(jobs[pos]["n_cand"])
                r.below_llik = outs[0][o:o + n].copy()
                r.above_llik = outs[1][o:o + n].copy()
                r.cand = outs[2][o:o + n].copy()
            elif table_scores and i in cont and modes[i] == "table":
                o, n = int(jobs[pos]["out_off"]), int(jobs[pos]["n_cand"])
                r.extra["score"] = outs[0][o:o + n].copy()
                r.extra["eps"] = outs[2][o:o + n].copy()  # the band's bound per candidate
                r.extra["table"] = tabs[pos - ta].copy()  # (slope, eps_cubic, eps_mix, ...)
                r.cand = outs[1][o:o + n].copy()
            results[i] = r
        _hmark("results")
        return results

    def _band_fix(self, band_jobs, d_segs, max_comp, n_comp, stream, exchanged, best_h, jobs):
        """Jobs of the table path whose band overflowed (n_scored == -1: more
        than BAND_TILE_CAP candidates of one scorer tile within the fp32 error bound of the maximum --
        a plateau of equal scores) are re-scored exactly: their fp32 candidate
        stream (TPE_F_DRAW32) through tpe_score_pruned64, every candidate in
        fp64.  Patches ``best_h`` (launch order) in place."""
        ns = best_h["n_scored"]  # (one field view: per-element structured access is ~20 us each)
        pos = [p for a, b in band_jobs for p in (a + np.flatnonzero(ns[a:b] < 0)).tolist()]
        if not pos:
            return
        torch, lib = self.torch, self.lib
        hj = np.ascontiguousarray(jobs[np.asarray(pos)].copy())
        hj["flags"] |= L.F_DRAW32
        nj = hj.size
        dj = torch.from_numpy(hj.view(np.uint8).copy()).to(self.device)
        npart = lib.tpe_pruned64_partials(hj.ctypes.data, nj)
        d_part = self._buf("partial_fix", 32 * max(npart, 1))
        out = torch.empty(nj * L.BEST_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        sp = ctypes.c_void_p(stream)
        L.check(lib.tpe_score_pruned64(
            dj.data_ptr(), hj.ctypes.data, nj, d_segs, self._bufs["mu"].data_ptr(),
            self._bufs["sigma"].data_ptr(), self._bufs["wcdf"].data_ptr(),
            self._bufs["coef64"].data_ptr(), max_comp, self._buf("reach_hi", 8 * n_comp),
            self._buf("reach_lo", 8 * n_comp), self._buf("wide_idx", 4 * n_comp),
            self._buf("table_scratch", lib.tpe_table_scratch_bytes(nj, max_comp)),
            self._buf("tables_fix", L.TABLE_DTYPE.itemsize * nj), None, None, None, None,
            d_part, npart, out.data_ptr(), sp), "tpe_score_pruned64 (band overflow)")
        L.hip_check(self._hip.hipStreamSynchronize(sp), "hipStreamSynchronize")
        res = out.cpu().numpy().view(L.BEST_DTYPE)
        for k, p in enumerate(pos):
            best_h[p] = res[k]
        self.band_overflows = getattr(self, "band_overflows", 0) + len(pos)
        self.last_band_overflow = [(int(p), int(jobs[p]["family"]), int(jobs[p]["n_cand"]))
                                   for p in pos]  # (diagnostic: launch position, family, n)

    def _exchange_fix(self, best_h, xrec, xinfo):
        """The exchange of a label-sharded level carries n_scored = -1 for a
        label whose band overflowed on some rank (tpe_best_scatter /
        tpe_best_combine propagate it), and every rank holds the same combined
        records -- so every rank, and only when one is owed, comes here
        together.  By now ``best_h`` holds this rank's exact records (its
        overflowed jobs were re-scored by _band_fix before the exchange was
        read), so the exchange is run once more on them: a second all-gather
        on the same communicator, in the same order on every rank (no rank
        leaves the level early and none takes an inexact winner)."""
        if xinfo is None:
            return xrec
        torch, lib = self.torch, self.lib
        comm, n_labels, world, slots, stream = xinfo
        sp = ctypes.c_void_p(stream)
        BS = L.BEST_DTYPE.itemsize
        dev = self.device

        def exchange(local):
            d_by = torch.from_numpy(np.ascontiguousarray(local).view(np.uint8).copy()).to(dev)
            d_slot = torch.from_numpy(np.ascontiguousarray(slots, np.int32)).to(dev)
            d_xl = torch.empty(n_labels * BS, dtype=torch.uint8, device=dev)
            d_xg = torch.empty(world * n_labels * BS, dtype=torch.uint8, device=dev)
            d_out = torch.empty(n_labels * BS, dtype=torch.uint8, device=dev)
            torch.cuda.current_stream(dev).synchronize()  # (the uploads above, on torch's stream)
            L.check(lib.tpe_best_scatter(d_by.data_ptr(), d_slot.data_ptr(), local.size,
                                         d_xl.data_ptr(), n_labels, sp), "tpe_best_scatter (fix)")
            L.check(lib.tpe_maxloc_allreduce(d_xl.data_ptr(), d_xg.data_ptr(), d_out.data_ptr(),
                                             n_labels, comm, sp), "tpe_maxloc_allreduce (fix)")
            L.hip_check(self._hip.hipStreamSynchronize(sp), "hipStreamSynchronize")
            self.exchange_fixes = getattr(self, "exchange_fixes", 0) + 1
            return d_out.cpu().numpy().view(L.BEST_DTYPE).copy()
        return hdist.settle_exchange(xrec, lambda: best_h, exchange)

    def _read_posteriors(self, works, fit_ids, cat, segs, csegs, n_comp, n_p, d_segs, stream,
                         o_p):
        torch = self.torch
        with torch.cuda.stream(stream):
            host = {}
            if fit_ids:
                for k in ("w", "mu", "sigma"):
                    host[k] = self._bufs[k][:8 * n_comp].to("cpu").numpy().view(np.float64)
                seg_t = self._bufs["stage"]
                # the fit writes prior_pos / p_accept back into the staged segment table
                raw = torch.empty(segs.nbytes, dtype=torch.uint8)
                off = d_segs - seg_t.data_ptr()
                raw.copy_(seg_t[off:off + segs.nbytes])
                dsegs = raw.numpy().view(L.SEG_DTYPE)
            if cat:
                host["p"] = self._bufs["stage"][o_p:o_p + 8 * n_p].to("cpu").numpy() \
                    .view(np.float64)
        results = [LabelResult(w.label, -1, 0.0, 0.0, 0) for w in works]
        for si, i in enumerate(fit_ids):
            post = {}
            for half, name in enumerate(("below", "above")):
                sg = segs[2 * si + half]
                a, n = int(sg["comp_off"]), int(sg["n_obs"]) + 1
                post[name] = tuple(host[k][a:a + n].copy() for k in ("w", "mu", "sigma"))
            post["p_accept"] = (float(dsegs[2 * si]["p_accept"]),
                                float(dsegs[2 * si + 1]["p_accept"]))
            results[i].extra = post
        for ci, i in enumerate(cat):
            post = {}
            for half, name in enumerate(("p_below", "p_above")):
                c = csegs[2 * ci + half]
                a, n = int(c["p_off"]), int(c["n_cat"])
                post[name] = host["p"][a:a + n].copy()
            results[i].extra = post
        return results


class _Pending(object):
    """A WorkBatch run whose result block is being copied back (Engine.run
    with defer=True).  ``result()`` waits for it once, checks the error bits
    and returns the BatchResult (cached)."""

    def __init__(self, eng, event, pin, nbytes, order, xoff, table, after=None, fix=None,
                 jobs=None, xinfo=None):
        self.eng, self.event, self.pin, self.nbytes = eng, event, pin, nbytes
        self.order, self.table, self.after = order, table, after
        self.fix, self.jobs = fix, jobs  # band overflow re-score (Engine._band_fix)
        self.xoff = xoff  # offset of the exchanged label records (Engine.run exchange=)
        self.xinfo = xinfo  # what Engine._exchange_fix needs to redo an owed exchange
        self._res = None

    def result(self):
        if self._res is not None:
            return self._res
        L.hip_check(self.eng._hip.hipEventSynchronize(self.event), "hipEventSynchronize")
        if self.after is not None:
            self.after()
            self.after = None
        eng = self.eng
        if eng._inflight is self:
            eng._inflight = None
        res_h = self.pin[:self.nbytes].numpy().copy()
        err = int(res_h[:4].view(np.int32)[0])
        eng.last_pairs = None
        eng.last_table_stats = None
        if self.table:
            st = res_h[16:40].view(np.int64).tolist()
            eng.last_table_stats = {"exact_candidates": st[0], "failed_cells": st[1],
                                    "failed_score_cells": st[2]}
        n = self.order.size
        best_h = res_h[64:64 + n * L.BEST_DTYPE.itemsize].view(L.BEST_DTYPE)
        # the same order as Engine._read_results: the band fix and the settle
        # exchange first, the error bits after -- a rank whose level set an
        # error bit still takes part in an owed second all-gather, so its
        # peers are not left blocked in it
        if self.fix is not None:
            self.fix(best_h, self.jobs)
        eng.last_exchange = res_h[self.xoff:].view(L.BEST_DTYPE).copy() \
            if self.xoff is not None else None
        if self.xoff is not None:
            eng.last_exchange = eng._exchange_fix(best_h, eng.last_exchange, self.xinfo)
        _raise_errors(err)
        by = np.empty(n, L.BEST_DTYPE)
        by[self.order] = best_h[:n]
        self._res = BatchResult(by["index"].copy(), by["value"].copy(), by["score"].copy(),
                                by["n_scored"].copy())
        return self._res


class _Replay(object):
    """The fast path for a WorkBatch level whose structure repeats the last
    recorded one -- every suggest of an fmin loop (the history grew by a trial:
    new counts, one more split flag) and bench.py's steps: the staged pack
    from that call is still in its pinned buffer with every per-structure part
    in place (prior pools, lattice slots, result block), so the per-call parts
    -- segment sizes, gather counts, the job table's keys and candidate bases,
    the split flags (the pack's last part) -- are rewritten there from the
    cached plan (Engine._plan_fast / _jobs_fast), the records' size words
    (history rows, observation totals, the largest mixture, the pack size) are
    rewritten, and the records are re-issued: no Python planning of the
    level, no packing, no per-launch host calls.  ``signature`` is every other
    input the pack and the records depend on; a workspace buffer that would
    have to grow (a new pointer) sends the call down the full path instead."""

    def __init__(self, sig, gen, ops, pinned, pkey, pending, res_pin, offs, history, tjobs,
                 fix_args):
        self.sig, self.gen, self.ops, self.pkey = sig, gen, ops, pkey
        self.pinned, self.host = pinned, pinned.numpy()
        self.offs, self.history, self.tjobs, self.fix_args = offs, history, tjobs, fix_args
        self.order = pending.order
        self.nbytes, self.xoff, self.table = pending.nbytes, pending.xoff, pending.table
        self.res_pin = res_pin
        n = self.order.size
        o = offs["jobs"]
        self.jobs_view = self.host[o:o + n * L.JOB_DTYPE.itemsize].view(L.JOB_DTYPE)
        self.counts = None  # (n_below, n_above, rows) the staged pack holds
        self.hist_rows = None
        self.fix = None
        self.xinfo = fix_args[4]

    @staticmethod
    def signature(eng, works, prior_weight, lf, precision, outputs, stream, sample_only, pruned,
                  scorer, posteriors, history, rows, is_below, histories, timers, timer_groups,
                  table_scores, exchange):
        if (history is None or rows is not None or histories is not None or outputs
                or sample_only or posteriors or table_scores or stream is None
                or not eng.native):
            return None  # (stream: the caller's current stream handle; None: given explicitly)
        if scorer is None:
            scorer = "auto" if pruned else "dense"
        if exchange is not None:
            exchange = (int(exchange[0]), int(exchange[1]), int(exchange[2]),
                        np.asarray(exchange[3], np.int32).tobytes())
        # (the timer spec last: the rest is the staged pack's signature)
        return (stream, works.key, float(prior_weight), int(lf), int(precision), scorer, pruned,
                history.vals.data_ptr(), history.active.data_ptr(), history.ld,
                exchange, eng.side_stream, eng.table_scorer, eng.exact64, eng.lat_prefix,
                eng.cat_early, eng.cat_issue, eng.cat_hist, eng.lat_main, eng.lat_max_slots,
                eng.device_events,
                eng.sorted_fit, "off" if timers is None else
                ("all" if timer_groups is None else frozenset(timer_groups)))

    def _put(self, name, arr):
        off = self.offs[name]
        if off is not None and arr.size:
            self.host[off:off + arr.nbytes] = arr.reshape(-1).view(np.uint8)

    def run(self, eng, batch, is_below, timers, defer):
        """Re-issue the level for ``batch``; None when it cannot (the caller
        then runs the full path)."""
        hm = eng.host_marks
        if hm is not None:
            hm.append(("start", time.perf_counter()))
        isb = np.ascontiguousarray(is_below, dtype=np.uint8).reshape(-1)
        n_rows = isb.size
        counts = (batch.n_below.tobytes(), batch.n_above.tobytes(), n_rows)
        if counts == self.counts and (self.history is None or
                                      self.history.rows == self.hist_rows):
            # the same counts as the staged pack's: keys, bases and flags only
            oi = self.order
            self.jobs_view["key"] = batch.keys[oi]
            self.jobs_view["cand_base"] = batch.cand_base[oi]
            self._put("isb", isb)
            return self._issue(eng, timers, defer, self.jobs_view, hm)
        P = eng._plans.get(self.pkey)
        if P is None or self.pkey[-1] != eng._big64(self.pkey[4], batch.n_above):
            return None
        (_, _, _, fit_ids, _, nf, segs, _, n_obs_total, n_comp, max_obs, csegs, _, _, _,
         cobs_off, _, _, _, _, _, g_arr) = eng._plan_fast(P, batch.n_below, batch.n_above)
        if hm is not None:
            hm.append(("replay:plan_fast", time.perf_counter()))
        jobs, _, fb_jobs = eng._jobs_fast(P, batch.keys, batch.cand_base)[:3]
        if hm is not None:
            hm.append(("replay:jobs", time.perf_counter()))
        pack_size = self.offs["isb"] + max(n_rows, 1)
        gen0 = eng._gen
        if pack_size > self.pinned.numel():
            return None
        eng._buf("stage", pack_size)
        eng._presize(n_comp, n_obs_total, max_obs, cobs_off, len(segs), self.tjobs,
                     n_rows if self.history is not None else 0)
        if eng._gen != gen0:
            return None
        if hm is not None:
            hm.append(("replay:presize", time.perf_counter()))
        if self.history is not None:  # rows appended since: merged into the sorted orders
            nfs = 2 * nf
            self.history.ensure_order(eng, eng.torch.cuda.current_stream(eng.device),
                                      g_arr["col"][:nfs:2], segs["transform"][::2],
                                      segs["floor"][::2])
        if hm is not None:
            hm.append(("replay:order", time.perf_counter()))
        for name, arr in (("segs", segs), ("csegs", csegs), ("g", g_arr), ("jobs", jobs),
                          ("fb", fb_jobs), ("isb", isb)):
            self._put(name, arr)
        keep = self.ops.keep  # the host copies the entry points validate
        keep[0][...] = jobs
        keep[1][...] = fb_jobs
        if keep[2] is not None:
            keep[2][...] = g_arr
        self.ops.set_sizes(dict(n_rows=n_rows, max_obs=max_obs, n_obs_total=n_obs_total,
                                max_comp=max_obs + 1, pack_size=pack_size))
        self.counts = counts
        self.hist_rows = self.history.rows if self.history is not None else None
        band_jobs, d_segs, stream, exchanged, self.xinfo = self.fix_args
        self.fix = None
        if band_jobs:
            self.fix = functools.partial(eng._band_fix, band_jobs, d_segs, max_obs + 1, n_comp,
                                         stream, exchanged)
        return self._issue(eng, timers, defer, jobs, hm)

    def _issue(self, eng, timers, defer, jobs, hm):
        if hm is not None:
            hm.append(("plan", time.perf_counter()))
        try:
            self.ops.issue(eng)
        except L.TpeHipError:
            eng._replays.clear()
            raise
        if hm is not None:
            hm.append(("score launches", time.perf_counter()))
        eng.graph_stats["native"] = eng.graph_stats.get("native", 0) + 1
        eng.graph_stats["replay"] = eng.graph_stats.get("replay", 0) + 1
        after = None
        if self.ops.timed and timers is not None:
            after = functools.partial(self.ops.read_timers, eng._hip, timers)
        p = eng._inflight = _Pending(eng, eng._event("result"), self.res_pin, self.nbytes,
                                     self.order, self.xoff, self.table, after, self.fix, jobs,
                                     self.xinfo)
        return p if defer else p.result()


class _Timed(object):
    """A kernel-group duration read from a re-issued level's event records,
    in the shape of Engine.run's (start, end) timer pairs:
    ``pair[0].elapsed_time(pair[1])`` gives milliseconds."""
    __slots__ = ("ms",)

    def __init__(self, ms):
        self.ms = ms

    def elapsed_time(self, _end):
        return self.ms


class _V(int):
    """A size argument of a level's launches (history rows, observation totals,
    the largest mixture, the pack size): an int to ctypes, and a named word
    to _OpList, which notes where it sits so a re-issue can rewrite it."""

    def __new__(cls, name, value):
        v = super().__new__(cls, int(value))
        v.name = name
        return v


def _word(a):
    """A tpe_run_ops argument word: pointers / handles as addresses, ints by value."""
    if a is None:
        return 0
    if isinstance(a, ctypes.c_void_p):
        return a.value or 0
    return int(a)


class _Timing(object):
    """Timing events owned by a recorded / captured level (tick/tock groups)."""

    def read_timers(self, hip, timers):
        ms = ctypes.c_float()
        for name, e0, e1 in self.timed:
            L.hip_check(hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1), "hipEventElapsedTime")
            timers.setdefault(name, []).append((_Timed(ms.value), None))

    def _new_event(self, hip):
        h = ctypes.c_void_p()
        L.hip_check(hip.hipEventCreateWithFlags(ctypes.byref(h), 0), "hipEventCreateWithFlags")
        self.events.append(h)
        return h


class _OpList(_Timing):
    """One level's stream work as tpe_run_ops records (Engine.run, native
    launcher).  Stands in for the library while the level is recorded: the
    entry points named in L.OP_CODES append a record (their ctypes-level
    arguments, as words) and return 0; size queries go to the library.
    ``keep`` holds the host arrays the records point to (host job slices,
    gather / history tables) for as long as the records live."""

    def __init__(self, lib):
        self.lib = lib
        self.rows = []
        self.timed = []
        self.events = []
        self.table_calls = []
        self.keep = self.arr = None
        self.ptr = self.n = 0
        # the records as a hipGraph (Engine.graphs): the graph of records
        # [0, cut) and the words it was captured from; the rest (the host's
        # event or stream sync, an RCCL exchange) is issued after it
        self.graph = self.graph_words = self.last_words = None
        self.cut = self.g0 = 0
        self.stream = None
        self.no_graph = False

    def __getattr__(self, name):
        code = L.OP_CODES.get(name)
        if code is None:
            return getattr(self.lib, name)

        def record(*args):
            self.rows.append((code, args))
            return 0
        return record

    def add(self, code, *args):
        self.rows.append((code, args))

    def order(self, ev, src, dst):
        self.add(L.OP_EVENT_RECORD, ev, src)
        self.add(L.OP_STREAM_WAIT, dst, ev)

    def record(self, hip, stream):
        h = self._new_event(hip)
        self.add(L.OP_EVENT_RECORD, h, stream.cuda_stream)
        return h

    def finish(self, keep, stream=None):
        arr = np.zeros(len(self.rows), L.OP_DTYPE)
        self.stream = stream
        codes = [code for code, _ in self.rows]
        # captured: the records between the pack's upload (a plain async copy
        # from pinned memory, issued before the graph) and the first of the
        # readback copy, an RCCL exchange, or the result event / stream sync
        # the host waits on (issued after it): kernels and stream fork / join
        self.g0 = 0
        while self.g0 < len(codes) and codes[self.g0] == L.OP_MEMCPY:
            self.g0 += 1
        tail = [i for i, (c, a) in enumerate(self.rows)
                if i >= self.g0 and (c in (L.OP_MAXLOC_ALLREDUCE, L.OP_STREAM_SYNC) or
                                     (c == L.OP_MEMCPY and len(a) > 3 and a[3] == L.D2H))]
        self.cut = min([len(codes) - 1] + tail)
        self.sizes = []  # (record, argument, size name): the words _Replay rewrites
        for i, (code, args) in enumerate(self.rows):
            if len(args) > L.OP_ARGS:
                raise ValueError("op %d has %d arguments" % (code, len(args)))
            arr["code"][i], arr["n_args"][i] = code, len(args)
            arr["a"][i, :len(args)] = [_word(a) for a in args]
            self.sizes += [(i, j, a.name) for j, a in enumerate(args) if isinstance(a, _V)]
        self.arr, self.keep, self.rows = arr, keep, None
        self.ptr, self.n = arr.ctypes.data, len(arr)

    def set_sizes(self, values):
        """Rewrite the size words of the records (names of _V arguments)."""
        a = self.arr["a"]
        for i, j, name in self.sizes:
            a[i, j] = values[name]

    def issue(self, eng):
        """Issue the records (one tpe_run_ops call), or replay them as a
        hipGraph: captured on the second issue in a row with the same words
        (pointers, sizes, grids -- the per-call inputs are in the uploaded
        pack), replayed while the words stay the same.  A level with timing
        events is never captured.  Raises TpeHipError on failure."""
        lib = self.lib
        failed = ctypes.c_int(-1)
        start = 0
        OPB = L.OP_DTYPE.itemsize
        if eng.graphs and self.cut > self.g0 and not self.timed and not self.no_graph:
            words = self.arr.tobytes()
            if self.graph is not None and words != self.graph_words:
                lib.tpe_graph_destroy(self.graph)
                self.graph = self.graph_words = None
            if self.graph is None and words == self.last_words:
                g = ctypes.c_void_p()
                t0 = time.perf_counter()
                rc = lib.tpe_ops_capture(self.ptr + self.g0 * OPB, self.cut - self.g0,
                                         self.stream, eng._capture_stream(), ctypes.byref(g),
                                         ctypes.byref(failed))
                if rc == 0:
                    self.graph, self.graph_words = g, words
                    eng.graph_stats["captured"] = eng.graph_stats.get("captured", 0) + 1
                    eng.graph_stats["capture_ms"] = eng.graph_stats.get("capture_ms", 0.0) + \
                        (time.perf_counter() - t0) * 1e3
                else:  # this level stays on tpe_run_ops (the reason kept for diagnosis)
                    self.no_graph = True
                    eng.graph_stats["capture_failed"] = lib.tpe_last_error().decode(
                        errors="replace")
            self.last_words = words
            if self.graph is not None:
                if self.g0:  # the upload
                    rc = lib.tpe_run_ops(self.ptr, self.g0, ctypes.byref(failed))
                    if rc != 0:
                        raise L.TpeHipError("tpe_run_ops failed (%d) at record %d: %s" % (
                            rc, failed.value, lib.tpe_last_error().decode(errors="replace")))
                rc = lib.tpe_graph_launch(self.graph, self.stream)
                if rc != 0:
                    raise L.TpeHipError("tpe_graph_launch failed (%d): %s" % (
                        rc, lib.tpe_last_error().decode(errors="replace")))
                eng.graph_stats["graph"] = eng.graph_stats.get("graph", 0) + 1
                start = self.cut
        rc = lib.tpe_run_ops(self.ptr + start * OPB, self.n - start, ctypes.byref(failed))
        if rc != 0:
            raise L.TpeHipError("tpe_run_ops failed (%d) at record %d: %s" % (
                rc, start + failed.value, lib.tpe_last_error().decode(errors="replace")))

    def destroy(self, hip):
        for h in self.events:
            hip.hipEventDestroy(h)
        self.events = []
        if self.graph is not None:
            self.lib.tpe_graph_destroy(self.graph)
            self.graph = self.graph_words = None


def _lat_prefix(text):
    """TPE_LAT_PREFIX: 0 (every stream drawn in full) or a positive multiple
    of 4096 (tpe_lattice_suggest's prefix); anything else is an error here,
    not a failed launch later."""
    try:
        v = int(text)
    except ValueError:
        raise ValueError("TPE_LAT_PREFIX must be an integer, got %r" % (text,))
    if v < 0 or v % 4096:
        raise ValueError("TPE_LAT_PREFIX must be 0 or a positive multiple of 4096, got %d" % v)
    return v


def _raise_errors(err):
    if err & 1:
        raise ValueError("negative arg to lognormal_cdf")  # tpe.py:196-197
    if err & 2:
        raise L.TpeHipError("lattice slot out of range (internal error)")
    if err & 4:
        raise L.TpeHipError("history gather: observation counts do not match the "
                            "segment sizes given by the host")


_GROUP_LAUNCH = {"cont": Engine._score_cont, "sorted": Engine._score_sorted,
                 "table": Engine._score_table, "pruned64": Engine._score_pruned64,
                 "lat": Engine._score_lat, "qfb": Engine._score_quantized,
                 "qinj": Engine._score_quantized, "cat": Engine._score_cat}


def _slice_of(groups, g):
    a = sum(len(ids) for _, ids in groups[:g])
    return a, a + len(groups[g][1])


def _support(w: LabelWork, P):
    """Coordinate range (x for GMM1, log x for LGMM1) every candidate lies in:
    [low, high] when bounded, else the below means +- 9 prior sigmas."""
    if P["bounded"]:
        return P["low"], P["high"]
    obs = np.asarray(w.obs_below, dtype=np.float64)
    if P["transform"] == L.OBS_LOG and obs.size:
        obs = np.log(np.maximum(obs, P["floor"]))
    pts = np.concatenate([obs[np.isfinite(obs)], [P["prior_mu"]]])
    return float(pts.min()) - 9.0 * P["prior_sigma"], float(pts.max()) + 9.0 * P["prior_sigma"]


def _injected_range(w: LabelWork, P, fp32=True):
    """Scoring-coordinate range of injected candidates (finite ones; the table
    grid covers it, anything outside is scored exactly).  fp32: the log of an
    LGMM1 candidate as the fp32 scorer forms it."""
    c = np.asarray(w.cand, dtype=np.float64).reshape(-1)
    if P["family"] == L.LGMM1:
        with np.errstate(all="ignore"):
            c = np.log(c.astype(np.float32)).astype(np.float64) if fp32 else np.log(c)
    c = c[np.isfinite(c)]
    if c.size == 0:
        return P["prior_mu"], P["prior_mu"]
    return float(c.min()), float(c.max())


def _lattice_range(w: LabelWork, P):
    """Inclusive lattice index range [kmin, kmax] covering every possible draw.

    Bounded: draws lie in [low, high) (log space for LGMM1).  Unbounded: every
    component has sigma <= prior_sigma (tpe.py:454-459) and a Box-Muller normal
    from 53-bit uniforms satisfies |z| < 8.6, so mean +- 9 sigma_prior bounds
    every draw.
    """
    q = P["q"]
    if P["bounded"]:
        lo, hi = P["low"], P["high"]
    else:
        obs = np.asarray(w.obs_below, dtype=np.float64)
        if P["transform"] == L.OBS_LOG:
            with np.errstate(all="ignore"):
                obs = np.log(np.maximum(obs, P["floor"])) if obs.size else obs
        # non-finite observations (as _support drops them): the fit places
        # components at them, but the lattice spans the finite draws only --
        # a draw off the lattice is reported (err bit 2), never written
        pts = np.concatenate([obs[np.isfinite(obs)], [P["prior_mu"]]])
        lo = float(pts.min()) - 9.0 * P["prior_sigma"]
        hi = float(pts.max()) + 9.0 * P["prior_sigma"]
    if P["family"] == L.LGMM1:
        lo, hi = math.exp(min(lo, 700.0)), math.exp(min(hi, 700.0))
    kmin = int(math.floor(lo / q)) - 1
    kmax = int(math.ceil(hi / q)) + 1
    return kmin, kmax
