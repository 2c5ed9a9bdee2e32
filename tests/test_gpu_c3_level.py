"""bench.py's exact timed level, checked label by label.

The bench times one C3 suggest level (BASELINE configs[2]: 50 labels, a
10k-trial history resident in HBM, 2^22 candidates per label) through
Engine.run with the WorkBatch / history / split-flag path.  Here that same
level (same space, history, split, Philox keys, candidate ranges; first run
and its replay) is run once more and EVERY label's winner is re-derived
exactly from the label's own materialised candidate stream:
  * continuous labels (table path): np.argmax over the fp64 scores of the
    2^22 drawn values (the pruned exact fp64 scorer on the injected stream),
    and the stream's 256 best plus 256 random candidates re-scored by the
    ORACLE (values, and the order of the best);
  * quantized labels (prefix-first lattice path): the ORACLE's fp64 score of
    each distinct drawn value, np.argmax over the stream (first index);
  * categorical labels (prefix-first categorical path): the ORACLE's
    posterior scores of the drawn categories, np.argmax over the stream.
The reference decides each label by np.argmax of its fp64 scores over its
candidates (tpe.py:649-658); north_star asks for bit-exact argmax indices.
"""
import numpy as np
import pytest

import bench
from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def level():
    from hyperopt_amd.engine import DeviceHistory, Engine
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    n = bench.N_CAND
    eng = Engine()
    units = [(j, 0, n) for j in range(len(space))]
    mat = bench.c3_matrix(space, vals)
    hist = DeviceHistory(eng, len(space), cap=bench.T_HIST)
    hist.append(mat)
    rb = bench.below_rows(losses)
    isb = np.zeros(bench.T_HIST, np.uint8)
    isb[rb] = 1
    runs = []
    for _ in range(4):  # the first run, its recording, re-issues
        batch = bench.history_batch(space, mat, hist, rb, 0, n, 0, units, n)
        r = eng.run(batch, precision=32, history=hist, is_below=isb)
        runs.append((r.index.copy(), r.value.copy(), r.score.copy(), r.n_scored.copy()))
    assert eng.graph_stats.get("native", 0) >= 1
    return space, vals, losses, n, runs


def test_replays_equal_the_first_run(level):
    _, _, _, _, runs = level
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            np.testing.assert_array_equal(a, b)


def _stream(eng, w, outputs=False):
    r, = eng.run([w], precision=32, sample_only=not outputs, outputs=outputs)
    return r


@pytest.mark.parametrize("kind", ["uniform", "loguniform", "normal", "quniform", "randint"])
def test_every_label_is_the_exact_argmax_of_its_stream(level, kind):
    from hyperopt_amd.engine import Engine, LabelWork
    space, vals, losses, n, runs = level
    index, value, score, n_scored = runs[0]
    splits = bench.split(vals, losses)
    works = bench.make_works(space, splits, 0, n, 0)
    eng = Engine()
    ex = Engine()
    ex.exact64 = "pruned"
    for j, (lab, k, a) in enumerate(space):
        if k != kind:
            continue
        w = works[j]
        assert n_scored[j] == n
        if kind in ("uniform", "loguniform", "normal"):
            cand = _stream(eng, w).cand
            x, = ex.run([LabelWork(lab, k, a, w.obs_below, w.obs_above, cand=cand)],
                        precision=64, outputs=True)
            assert index[j] == x.index, (lab, index[j], x.index)
            assert value[j] == cand[x.index]
            np.testing.assert_allclose(score[j], x.score, rtol=1e-12, atol=1e-12)
            # pinned to the oracle directly: the stream's 256 best candidates
            # (the whole band the fp32 table could have confused, winner and
            # runner-up first) and 256 drawn at random, re-scored by the numpy
            # restatement (tpe.py:117-180, 265-307): same values, same order
            s64 = x.below_llik - x.above_llik
            best = int(index[j])
            assert best == int(np.argmax(s64))
            top = np.argsort(-s64, kind="stable")[:256]
            assert top[0] == best
            rnd = np.random.RandomState(j).randint(0, n, 256)
            pick = np.concatenate([top, rnd])
            with np.errstate(all="ignore"):
                ref = O.continuous_label_scores(k, a, w.obs_below, w.obs_above, cand[pick])
            rs = ref["below_llik"] - ref["above_llik"]
            np.testing.assert_allclose(rs, s64[pick], rtol=1e-9, atol=1e-9)
            # the oracle's order of the top candidates is the device's wherever
            # two scores differ by more than the two scorers' largest observed
            # disagreement (fp64 summation-order noise)
            err = float(np.max(np.abs(rs - s64[pick])))
            tol = 2 * err + 1e-13 * max(1.0, abs(s64[best]))
            d_dev, d_ref = np.diff(s64[top]), np.diff(rs[:256])
            loud = np.abs(d_dev) > tol
            assert np.all(d_ref[loud] < 0), (lab, np.flatnonzero(loud & (d_ref >= 0))[:5])
            assert rs[0] >= rs.max() - tol, (lab, rs[0], rs.max())
        elif kind == "quniform":
            cand = _stream(eng, w).cand
            u, inv = np.unique(cand, return_inverse=True)
            with np.errstate(all="ignore"):
                ref = O.continuous_label_scores(k, a, w.obs_below, w.obs_above, u)
            s = (ref["below_llik"] - ref["above_llik"])[inv]
            best = int(np.argmax(s))
            assert index[j] == best, (lab, index[j], best)
            assert value[j] == cand[best]
            np.testing.assert_allclose(score[j], s[best], rtol=1e-9, atol=1e-9)
        else:
            r = _stream(eng, w, outputs=True)  # the full categorical stream
            cats = r.cand.astype(np.int64)
            ref = O.categorical_label_scores(k, a, w.obs_below, w.obs_above, cats)
            s = ref["below_llik"] - ref["above_llik"]
            best = int(np.argmax(s))
            assert index[j] == best, (lab, index[j], best)
            assert int(value[j]) == cats[best]
            np.testing.assert_allclose(score[j], s[best], rtol=1e-12, atol=1e-12)
