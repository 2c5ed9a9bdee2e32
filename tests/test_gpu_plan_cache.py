"""Level-plan cache (Engine._plan_key / _plan_fast / _jobs_fast).

The second run of a level structure copies the recorded descriptor arrays and
refills only the per-call columns (observation counts, Philox keys).  Every
descriptor array and every result must be identical to a run that plans from
scratch, while the history grows between calls (counts change), for every
prior kind, unbounded lattices (range in the key) included.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SPACE = [("u", "uniform", (-5.0, 5.0)), ("lu", "loguniform", (-5.0, 0.0)),
         ("q", "quniform", (0.0, 20.0, 1.0)), ("n", "normal", (0.0, 2.0)),
         ("qn", "qnormal", (0.0, 3.0, 0.5)), ("ln", "lognormal", (0.0, 1.0)),
         ("c", "randint", (6,)), ("r", "randint", (3, 11))]


def _history(T, seed):
    rng = np.random.RandomState(seed)
    cols = [rng.uniform(-5, 5, T), np.exp(rng.uniform(-5, 0, T)),
            np.round(rng.uniform(0, 20, T)), rng.normal(0, 2, T),
            np.round(rng.normal(0, 3, T) / 0.5) * 0.5, np.exp(rng.normal(0, 1, T)),
            rng.randint(0, 6, T).astype(float), rng.randint(3, 11, T).astype(float)]
    mat = np.stack(cols, axis=1)
    active = rng.uniform(size=mat.shape) >= 0.1
    return mat, active, rng.normal(size=T)


def _works(hist, mat, active, losses, T, step, n_cand):
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
                               key=1000 * step + j, cand_base=step, col=j, n_above=n_above))
    return works, isb


@pytest.mark.parametrize("n_cand", [24, 1 << 16])
def test_cached_plan_matches_fresh_plan(n_cand):
    from hyperopt_amd.engine import DeviceHistory, Engine
    eng = Engine()
    mat, active, losses = _history(1200, 3)
    hist = DeviceHistory(eng, len(SPACE), cap=256)
    hist.append(mat[:800], active[:800])
    T = 800
    replays = 0
    for step in range(4):
        works, isb = _works(hist, mat, active, losses, T, step, n_cand)
        r_cached = eng.run(works, history=hist, is_below=isb)
        plan_cached = eng.last_plan
        eng._plans.clear()
        r_fresh = eng.run(works, history=hist, is_below=isb)
        plan_fresh = eng.last_plan
        assert not plan_fresh[-1]
        r_replay = eng.run(works, history=hist, is_below=isb)  # same structure: a hit
        plan_replay = eng.last_plan
        assert plan_replay[-1]
        replays += 1
        for cached in (plan_cached, plan_replay):
            for a, b in zip(cached[:4], plan_fresh[:4]):
                assert a.dtype == b.dtype and a.shape == b.shape
                assert a.tobytes() == b.tobytes()
        for rs in (r_cached, r_replay):
            for a, b in zip(rs, r_fresh):
                assert (a.label, a.index, a.value, a.score, a.n_scored) == \
                    (b.label, b.index, b.value, b.score, b.n_scored)
        # the next call sees a longer history: every count changes (the fresh
        # run above recorded the plan the next cached call replays)
        hist.append(mat[T:T + 100], active[T:T + 100])
        T += 100
    assert replays == 4

