"""Host-side cost of bench.py's C3 step, measured on a machine without a GPU
(diagnostic): the engine runs against stand-ins for the device (CPU tensors
for workspace, a HIP runtime whose calls return success, a library whose
launch entry points do nothing; size queries use the real library), so what
is timed is exactly the Python / numpy / ctypes work of a step -- the part
of a level during which the GPU waits.

    python tools/host_cpu_profile.py [world=1] [rank=0] [--cprofile]
"""
import cProfile
import ctypes
import os
import pstats
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import _lib as L  # noqa: E402
from hyperopt_amd import dist as hdist  # noqa: E402
from hyperopt_amd import engine as E  # noqa: E402


class _Stream(object):
    cuda_stream = 0

    def __init__(self, *a, **k):
        pass


class _Event(object):
    def __init__(self, *a, **k):
        pass

    def record(self, *a):
        pass

    def elapsed_time(self, other):
        return 0.0


def _torch_shim():
    t = types.SimpleNamespace()
    for name in ("uint8", "float64", "int64", "int32", "from_numpy", "device"):
        setattr(t, name, getattr(torch, name))

    def empty(*shape, dtype=None, device=None, pin_memory=False):
        return torch.zeros(*shape, dtype=dtype)

    def zeros(*shape, dtype=None, device=None):
        return torch.zeros(*shape, dtype=dtype)
    t.empty, t.zeros = empty, zeros
    t.cuda = types.SimpleNamespace(Stream=_Stream, Event=_Event,
                                   current_stream=lambda *a: _Stream(),
                                   current_device=lambda: 0,
                                   stream=lambda s: _Null())
    return t


class _Null(object):
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _Hip(object):
    def __getattr__(self, name):
        return lambda *a: 0


class _Lib(object):
    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        if name in L.OP_CODES or name in ("tpe_run_ops", "tpe_history_append", "tpe_ops_capture",
                                          "tpe_graph_launch", "tpe_graph_destroy"):
            return lambda *a: 0
        return getattr(self._lib, name)


def make_engine():
    eng = E.Engine.__new__(E.Engine)
    shim = _torch_shim()
    eng.torch = shim
    eng.lib = _Lib(L.load())
    eng.device = torch.device("cpu")
    eng._bufs, eng._plans, eng._retired, eng._pinned = {}, {}, [], {}
    eng._res_pin = eng._inflight = None
    eng._events = {}
    eng._hip = _Hip()
    eng.host_marks = None
    eng.side_stream = os.environ.get("TPE_SIDE_STREAM", "1")
    eng._side = None
    eng.table_scorer = "cubic"
    eng.exact64 = "auto"
    eng.cat_early = os.environ.get("TPE_CAT_EARLY", "1") == "1"
    eng.cat_issue = os.environ.get("TPE_CAT_ISSUE", "post")
    eng.cat_hist = os.environ.get("TPE_CAT_HIST", "1") == "1"
    eng.cat_chunked = True
    eng.lat_main = os.environ.get("TPE_LAT_MAIN", "1") == "1"
    eng.lat_max_slots = E.LAT_SUGGEST_MAX_SLOTS
    eng.lat_prefix = int(os.environ.get("TPE_LAT_PREFIX", str(E.LAT_PREFIX)))
    eng.device_events = True
    eng.sorted_fit = os.environ.get("TPE_SORTED_FIT", "1") == "1"
    eng._last_gkey, eng._gen = None, 0
    eng.graph_stats = {"eager": 0}
    eng.native = os.environ.get("TPE_NATIVE_LAUNCH", "1") != "0"
    eng.graphs = os.environ.get("TPE_GRAPHS", "0") == "1"
    eng._cap_stream = _Stream()
    eng._oplists, eng._oplist_once, eng._replays, eng._staged_sig = {}, None, {}, None
    E.torch_shim = shim
    L.hip = lambda: eng._hip  # (DeviceHistory.append's event calls)
    return eng


def main(world=1, rank=0, prof=False, append=False):
    """append: one trial appended to the history before every step (as fmin
    does): new counts every level, re-issued records (engine._Replay)."""
    eng = make_engine()
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    mat = bench.c3_matrix(space, vals)
    hist = E.DeviceHistory(eng, len(space), cap=bench.T_HIST)
    hist.append(mat)
    units = hdist.plan_units([k for _, k, _ in space], bench.N_CAND, world)[rank]
    extra = np.random.RandomState(5)
    state = {"mat": mat, "losses": losses}

    def step(k):
        if append:
            row = state["mat"][extra.randint(state["mat"].shape[0])][None]
            hist.append(row)
            state["mat"] = np.concatenate([state["mat"], row])
            state["losses"] = np.append(state["losses"], extra.normal())
        lo, m = state["losses"], state["mat"]
        rb = bench.below_rows(lo)
        isb = np.zeros(lo.size, np.uint8)
        isb[rb] = 1
        works = bench.history_batch(space, m, hist, rb, k, bench.N_CAND, 0, units,
                                    bench.N_CAND)
        return eng.run(works, precision=32, history=hist, is_below=isb)
    for k in range(5):
        step(k)
    n = 300
    t0 = time.perf_counter()
    for k in range(n):
        step(10 + k)
    dt = (time.perf_counter() - t0) / n
    print("world %d rank %d (%d units)%s: host %.1f us per step, stats %s" % (
        world, rank, len(units), " +1 trial per step" if append else "", dt * 1e6,
        eng.graph_stats))
    if prof:
        pr = cProfile.Profile()
        pr.enable()
        for k in range(n):
            step(1000 + k)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)




def marks(world=1, rank=0):
    """Median host time per Engine.run phase (Engine.host_marks)."""
    eng = make_engine()
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    mat = bench.c3_matrix(space, vals)
    hist = E.DeviceHistory(eng, len(space), cap=bench.T_HIST)
    hist.append(mat)
    units = hdist.plan_units([k for _, k, _ in space], bench.N_CAND, world)[rank]
    rows = []
    for k in range(200):
        t0 = time.perf_counter()
        rb = bench.below_rows(losses)
        isb = np.zeros(bench.T_HIST, np.uint8)
        isb[rb] = 1
        t1 = time.perf_counter()
        works = bench.history_batch(space, mat, hist, rb, k, bench.N_CAND, 0, units, bench.N_CAND)
        t2 = time.perf_counter()
        eng.host_marks = [("start", t2)]
        eng.run(works, precision=32, history=hist, is_below=isb)
        eng.host_marks.append(("end", time.perf_counter()))
        hm = eng.host_marks
        rows.append([("below_rows", t1 - t0), ("history_batch", t2 - t1)] +
                    [(b[0], b[1] - a[1]) for a, b in zip(hm[:-1], hm[1:])])
    names = [n for n, _ in rows[-1]]
    med = np.median(np.array([[v for _, v in r] for r in rows[50:] if len(r) == len(names)]), 0)
    print({n: round(v * 1e6, 1) for n, v in zip(names, med)})


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    if "--marks" in sys.argv:
        marks(*(int(a) for a in args))
    else:
        main(*(int(a) for a in args), prof="--cprofile" in sys.argv,
             append="--append" in sys.argv)
