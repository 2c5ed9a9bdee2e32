"""Replayed levels (Engine.run): a level whose launch key repeats is
recorded on its second call and re-issued afterwards by the native level
launcher (tpe_run_ops records, csrc/tpe_ops.hip).

The per-call inputs (split flags, observation counts, Philox keys) travel in
the level's upload, outside the records, so a replayed level must give exactly
what an eager engine gives on the same inputs: every label's winner index,
value, score and n_scored, byte for byte, for every prior kind and scorer
path.  A changed history (new counts), a grown workspace buffer or another
structure must never replay stale records.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SPACE = [("u", "uniform", (-5.0, 5.0)), ("lu", "loguniform", (-5.0, 0.0)),
         ("q", "quniform", (0.0, 20.0, 1.0)), ("n", "normal", (0.0, 2.0)),
         ("qn", "qnormal", (0.0, 3.0, 0.5)), ("ln", "lognormal", (0.0, 1.0)),
         ("c", "randint", (6,)), ("r", "randint", (3, 11)),
         ("k", "categorical", ((0.1, 0.2, 0.3, 0.4),))]


def _history(T, seed):
    rng = np.random.RandomState(seed)
    cols = [rng.uniform(-5, 5, T), np.exp(rng.uniform(-5, 0, T)),
            np.round(rng.uniform(0, 20, T)), rng.normal(0, 2, T),
            np.round(rng.normal(0, 3, T) / 0.5) * 0.5, np.exp(rng.normal(0, 1, T)),
            rng.randint(0, 6, T).astype(float), rng.randint(3, 11, T).astype(float),
            rng.randint(0, 4, T).astype(float)]
    mat = np.stack(cols, axis=1)
    active = rng.uniform(size=mat.shape) >= 0.1
    return mat, active, rng.normal(size=T)


def _works(mat, active, losses, T, step, n_cand):
    from hyperopt_amd.engine import LabelWork
    n_below = min(int(np.ceil(0.25 * np.sqrt(T))), 25)
    isb = np.zeros(T, np.uint8)
    isb[np.argsort(losses[:T], kind="stable")[:n_below]] = 1
    works = []
    for j, (lab, kind, a) in enumerate(SPACE):
        act = active[:T, j]
        below = mat[:T, j][act & (isb == 1)]
        n_above = int((act & (isb == 0)).sum())
        works.append(LabelWork(lab, kind, a, below, None, n_cand=n_cand,
                               key=7919 * step + 31 * j + 5, cand_base=0, col=j,
                               n_above=n_above))
    return works, isb


def _rows(res):
    return [(r.label, r.index, r.value, r.score, r.n_scored) for r in res]


MODES = ["native"]


def _pair(mode):
    from hyperopt_amd.engine import DeviceHistory, Engine
    eager, native = Engine(), Engine()
    eager.native = False
    native.native = True
    return eager, native, DeviceHistory


def _replays(eng):
    """(recorded, re-issued, eager) level counts."""
    st = eng.graph_stats
    return len(eng._oplists), st.get("native", 0), st["eager"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n_cand", [24, 1 << 18])
def test_replayed_level_equals_eager(n_cand, mode):
    eager, native, DeviceHistory = _pair(mode)
    mat, active, losses = _history(3000, 11)
    he = DeviceHistory(eager, len(SPACE), cap=4096)
    hg = DeviceHistory(native, len(SPACE), cap=4096)
    for h in (he, hg):
        h.append(mat, active)
    for step in range(6):  # new Philox keys every call, same counts: recorded, then re-issued
        works, isb = _works(mat, active, losses, 3000, step, n_cand)
        a = eager.run(works, history=he, is_below=isb)
        b = native.run(works, history=hg, is_below=isb)
        assert _rows(a) == _rows(b), step
    # the first call sizes the workspace, a call whose key repeats the previous
    # one's is recorded, every later call replays
    cap, rep, eag = _replays(native)
    assert cap == 1 and rep >= 4 and eag + rep == 6, (cap, rep, eag)
    # the winners moved with the keys (the replay did not reuse old inputs)
    idx = set()
    for s in (10, 11):
        works, isb = _works(mat, active, losses, 3000, s, n_cand)
        idx.add(tuple(r[1] for r in _rows(native.run(works, history=hg, is_below=isb))))
    assert len(idx) == 2


@pytest.mark.parametrize("mode", MODES)
def test_growing_history_never_replays_stale_records(mode):
    eager, native, DeviceHistory = _pair(mode)
    mat, active, losses = _history(2400, 5)
    he = DeviceHistory(eager, len(SPACE), cap=512)
    hg = DeviceHistory(native, len(SPACE), cap=512)
    T = 400
    for h in (he, hg):
        h.append(mat[:T], active[:T])
    for step in range(8):
        works, isb = _works(mat, active, losses, T, step, 1 << 16)
        for _ in range(3):  # three calls per history size: capture, then replay
            a = eager.run(works, history=he, is_below=isb)
            b = native.run(works, history=hg, is_below=isb)
            assert _rows(a) == _rows(b), (step, T)
        # more trials (the history buffers grow past their capacity too)
        for h in (he, hg):
            h.append(mat[T:T + 250], active[T:T + 250])
        T += 250
    cap, rep, eag = _replays(native)
    assert rep >= 8, (cap, rep, eag)


@pytest.mark.parametrize("mode", MODES)
def test_other_structure_between_replays(mode):
    """A larger level in between grows the workspace (new pointers): the
    first structure's records are dropped and re-recorded, never replayed stale."""
    eager, native, DeviceHistory = _pair(mode)
    mat, active, losses = _history(3000, 2)
    he = DeviceHistory(eager, len(SPACE), cap=4096)
    hg = DeviceHistory(native, len(SPACE), cap=4096)
    for h in (he, hg):
        h.append(mat, active)
    for step, n_cand in enumerate([1 << 14, 1 << 14, 1 << 14, 1 << 20, 1 << 20, 1 << 14,
                                   1 << 14, 1 << 14]):
        works, isb = _works(mat, active, losses, 3000, step, n_cand)
        a = eager.run(works, history=he, is_below=isb)
        b = native.run(works, history=hg, is_below=isb)
        assert _rows(a) == _rows(b), step


@pytest.mark.parametrize("mode", MODES)
def test_timers_of_replayed_levels(mode):
    """Timer groups inside a replayed level are event records of its own
    (tpe_run_ops records): their durations are read after the
    level and look like kernel times."""
    _, native, DeviceHistory = _pair(mode)
    mat, active, losses = _history(3000, 4)
    hg = DeviceHistory(native, len(SPACE), cap=4096)
    hg.append(mat, active)
    timers = {}
    for step in range(5):
        works, isb = _works(mat, active, losses, 3000, step, 1 << 20)
        native.run(works, history=hg, is_below=isb, timers=timers, timer_groups={"table"})
    cap, rep, eag = _replays(native)
    assert rep >= 3 and eag + rep == 5, (cap, rep, eag)
    ms = [a.elapsed_time(b) for a, b in timers["table"]]
    assert len(ms) == 5
    assert all(0.0 < m < 50.0 for m in ms), ms
    # replayed durations agree with the eager ones (same kernel, same work)
    assert max(ms[-3:]) < 3.0 * min(ms[:2]) + 0.05


def test_native_batch_deferred_equals_eager():
    """suggest_many's path: WorkBatch levels with deferred readbacks through
    the native launcher equal eager single runs."""
    from hyperopt_amd.engine import WorkBatch
    eager, native, DeviceHistory = _pair("native")
    mat, active, losses = _history(2000, 8)
    hists = []
    for eng in (eager, native):
        h = DeviceHistory(eng, len(SPACE), cap=2048)
        h.append(mat, active)
        hists.append(h)
    for step in range(5):
        works, isb = _works(mat, active, losses, 2000, step, 1 << 12)
        n_b = [np.size(w.obs_below) for w in works]
        n_a = [w.n_above for w in works]
        keys = [w.key for w in works]
        out = []
        for eng, h in zip((eager, native), hists):
            b = WorkBatch(("t",) + tuple(n_b) + tuple(n_a), n_b, n_a, keys, [0] * len(works),
                          lambda works=works: works)
            p = eng.run(b, histories=[(h, None, isb)], defer=True)
            r = p.result()
            out.append((r.index.tolist(), r.value.tolist(), r.score.tolist(),
                        r.n_scored.tolist()))
        assert out[0] == out[1], step
    assert native.graph_stats.get("native", 0) >= 3


def test_level_replay_equals_eager():
    """The WorkBatch level replay (engine._Replay: the staged pack reused,
    only keys / candidate bases / split flags rewritten) gives the eager
    engine's winners when the keys AND the split change from call to call
    (same counts: a different set of below rows each time), and a changed
    count falls back to the full path."""
    from hyperopt_amd.engine import WorkBatch
    eager, native, DeviceHistory = _pair("native")
    T = 3000
    mat, active, losses = _history(T, 9)
    active[:] = True  # every label active: any split of n_below rows keeps the counts
    he = DeviceHistory(eager, len(SPACE), cap=4096)
    hn = DeviceHistory(native, len(SPACE), cap=4096)
    for h in (he, hn):
        h.append(mat, active)
    rng = np.random.RandomState(5)

    # (no unbounded lattice: its range follows the below set, and a WorkBatch
    # key must name it -- a new split would be a new structure)
    space = [(j, e) for j, e in enumerate(SPACE) if e[1] != "qnormal"]

    def batch(works, n_below):
        keys = [w.key for w in works]
        nb = [n_below] * len(works)
        na = [T - n_below] * len(works)
        return WorkBatch(("replay-test", n_below), nb, na, keys, [0] * len(works),
                         lambda works=works: works)
    for step in range(8):
        n_below = 14 if step < 6 else 15  # the last two steps change the counts
        isb = np.zeros(T, np.uint8)
        isb[rng.choice(T, n_below, replace=False)] = 1
        works = []
        from hyperopt_amd.engine import LabelWork
        for j, (lab, kind, a) in space:
            works.append(LabelWork(lab, kind, a, mat[isb == 1, j], None, n_cand=1 << 16,
                                   key=1000 * step + j, cand_base=0, col=j,
                                   n_above=T - n_below))
        out = []
        for eng, h in ((eager, he), (native, hn)):
            r = eng.run(batch(works, n_below), history=h, is_below=isb)
            out.append((r.index.tolist(), r.value.tolist(), r.score.tolist(),
                        r.n_scored.tolist()))
        assert out[0] == out[1], step
    assert native.graph_stats.get("replay", 0) >= 3, native.graph_stats


@pytest.mark.parametrize("variant", ["cat_pre", "cat_late", "cat_off"])
def test_issue_orders_give_the_same_level(variant):
    """The side-stream issue variants (categorical work issued before the fit /
    after it / after the table build / after the fit with the quantized work)
    only move launches between streams and in time: every label's winner
    equals the default engine's."""
    base, other, DeviceHistory = _pair("native")
    if variant == "cat_off":
        other.cat_early = False
    else:
        other.cat_issue = variant.split("_")[1]
    mat, active, losses = _history(2500, 13)
    hb = DeviceHistory(base, len(SPACE), cap=4096)
    ho = DeviceHistory(other, len(SPACE), cap=4096)
    for h in (hb, ho):
        h.append(mat, active)
    for step in range(4):
        works, isb = _works(mat, active, losses, 2500, step, 1 << 17)
        a = base.run(works, history=hb, is_below=isb)
        b = other.run(works, history=ho, is_below=isb)
        assert _rows(a) == _rows(b), (variant, step)


@pytest.mark.parametrize("side", ["1", "0"])
def test_graph_replay_equals_eager(side):
    """A recorded level re-issued with the same words is captured into a
    hipGraph (tpe_ops_capture, on the engine's own stream: the caller's may be
    the null stream) and replayed (tpe_graph_launch): the keys and split flags
    still change per call through the uploaded pack, and the winners equal the
    eager engine's and the records-only engine's (TPE_GRAPHS=0), with and
    without the side stream; a timed level is not captured."""
    from hyperopt_amd.engine import LabelWork, WorkBatch
    eager, native, DeviceHistory = _pair("native")
    _, plain, _ = _pair("native")
    native.graphs, plain.graphs = True, False  # (graphs: a diagnostic switch, off by default)
    for e in (eager, native, plain):
        e.side_stream = side
    T = 3000
    mat, active, losses = _history(T, 21)
    active[:] = True
    hs = [DeviceHistory(e, len(SPACE), cap=4096) for e in (eager, native, plain)]
    for h in hs:
        h.append(mat, active)
    rng = np.random.RandomState(7)
    space = [(j, e) for j, e in enumerate(SPACE) if e[1] != "qnormal"]
    n_below = 14
    for step in range(7):
        isb = np.zeros(T, np.uint8)
        isb[rng.choice(T, n_below, replace=False)] = 1
        works = [LabelWork(lab, kind, a, mat[isb == 1, j], None, n_cand=1 << 16,
                           key=977 * step + j, cand_base=0, col=j, n_above=T - n_below)
                 for j, (lab, kind, a) in space]
        out = []
        for eng, h in zip((eager, native, plain), hs):
            b = WorkBatch(("graph-test", side), [n_below] * len(works),
                          [T - n_below] * len(works), [w.key for w in works],
                          [0] * len(works), lambda works=works: works)
            timers = {} if step == 5 else None  # a timed level: records only
            r = eng.run(b, history=h, is_below=isb, timers=timers)
            out.append((r.index.tolist(), r.value.tolist(), r.score.tolist(),
                        r.n_scored.tolist()))
        assert out[0] == out[1] == out[2], step
    st = native.graph_stats
    assert "capture_failed" not in st, st
    assert st.get("captured", 0) >= 1 and st.get("graph", 0) >= 3, st
    assert plain.graph_stats.get("graph", 0) == 0


def test_quantized_on_idle_main_stream_gives_the_same_level():
    """A level of quantized and categorical labels only (no continuous
    scorer on the main stream): with lat_main the lattice work runs on the
    main stream beside the side stream's categorical chain; the winners equal
    the all-on-the-side-stream engine's, eager and re-issued."""
    base, other, DeviceHistory = _pair("native")
    base.native = True
    base.lat_main, other.lat_main = False, True
    T = 3000
    mat, active, losses = _history(T, 41)
    keep = [j for j, (_, kind, _) in enumerate(SPACE)
            if kind in ("quniform", "qnormal", "randint", "categorical")]
    hb = DeviceHistory(base, len(SPACE), cap=4096)
    ho = DeviceHistory(other, len(SPACE), cap=4096)
    for h in (hb, ho):
        h.append(mat, active)
    for step in range(5):
        works, isb = _works(mat, active, losses, T, step % 2, 1 << 18)
        works = [works[j] for j in keep]
        a = base.run(works, history=hb, is_below=isb)
        b = other.run(works, history=ho, is_below=isb)
        assert _rows(a) == _rows(b), step
    assert other.graph_stats.get("native", 0) >= 2, other.graph_stats
