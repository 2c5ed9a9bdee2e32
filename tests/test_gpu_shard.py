"""Shard invariance on one GPU: a label's candidates split into two ranges
(as two ranks would score them, odd and even split points) and combined on
the device by tpe_best_combine give the unsplit run's winner, byte for byte.

Candidates are keyed by their GLOBAL index (Philox counter), so the split
must not change any candidate's value (tpe_hip.h: tpe_job.cand_base); the
combine applies np.argmax's rule (tpe.py:650-658).  Also covers the multi-GPU
unit plan (hyperopt_amd/dist.py plan_units): every rank count gives the
single-GPU suggestion.
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


def _split(kind, args, n_hist, seed):
    from tests.test_gpu_parity import _mixture_case
    rng = np.random.RandomState(seed)
    gen = _mixture_case(rng, kind, args, 1, n_hist, 1)
    losses = rng.normal(size=n_hist)
    return O.ap_split_trials(np.arange(n_hist), gen.obs_above, np.arange(n_hist), losses, 0.25)


CASES = [("uniform", (-5.0, 5.0)), ("loguniform", (-5.0, 0.0)), ("normal", (0.0, 2.0)),
         ("quniform", (0.0, 100.0, 1.0)), ("randint", (8,))]


@pytest.mark.parametrize("precision", [32, 64])
@pytest.mark.parametrize("kind,args", CASES)
def test_split_equals_unsplit(engine, kind, args, precision):
    from hyperopt_amd import dist as hdist
    from hyperopt_amd import _lib as L
    from hyperopt_amd.engine import LabelWork
    if kind == "randint":
        rng = np.random.RandomState(2)
        below, above = rng.randint(0, 8, 25), rng.randint(0, 8, 3000)
    else:
        below, above = _split(kind, args, 3000, 9)
    n = (1 << 18) if precision == 32 else (1 << 14)

    def run(base, count):
        w = LabelWork("x", kind, args, below, above, n_cand=count, key=4242, cand_base=base,
                      n_total=n)
        r, = engine.run([w], precision=precision)
        return np.array([(r.score, r.index, r.value, r.n_scored)], L.BEST_DTYPE)

    whole = run(0, n)
    assert whole["n_scored"][0] == n
    for cut in (n // 2 + 1, n // 2, 4097, 1):
        parts = np.stack([run(0, cut), run(cut, n - cut)])
        comb = hdist.combine_device(parts)
        assert comb.tobytes() == whole.tobytes(), (kind, cut, comb, whole)
    # three uneven shards, the middle one starting and ending on odd indices
    cuts = [0, 12_345, n - 777, n]
    parts = np.stack([run(a, b - a) for a, b in zip(cuts[:-1], cuts[1:])])
    assert hdist.combine_device(parts).tobytes() == whole.tobytes()


def test_odd_base_draws_equal_even_base_draws(engine):
    """The fp32 pair sampler at an odd first index draws exactly the
    candidates the aligned run draws at those indices."""
    from hyperopt_amd.engine import LabelWork
    below, above = _split("uniform", (-5.0, 5.0), 2000, 3)
    n = 50_000
    w = LabelWork("x", "uniform", (-5.0, 5.0), below, above, n_cand=n, key=99)
    ref, = engine.run([w], precision=32, sample_only=True)
    for base in (1, 3, 4097, 12_345):
        w2 = LabelWork("x", "uniform", (-5.0, 5.0), below, above, n_cand=n - base, key=99,
                       cand_base=base)
        got, = engine.run([w2], precision=32, sample_only=True)
        np.testing.assert_array_equal(got.cand, ref.cand[base:])


def test_plan_units_suggest_invariant_to_rank_count(engine):
    """Every rank count's unit plan, run rank by rank on this GPU and combined,
    gives the single-GPU winners of a mixed 8-label level."""
    from hyperopt_amd import dist as hdist
    from hyperopt_amd.engine import LabelWork
    specs = [("u", "uniform", (-5.0, 5.0)), ("l", "loguniform", (-5.0, 0.0)),
             ("q", "quniform", (0.0, 100.0, 1.0)), ("n", "normal", (0.0, 2.0)),
             ("c", "randint", (8,)), ("u2", "uniform", (0.0, 1.0)),
             ("n2", "normal", (3.0, 1.0)), ("q2", "quniform", (0.0, 10.0, 0.5))]
    rng = np.random.RandomState(0)
    data = {}
    for j, (lab, kind, a) in enumerate(specs):
        if kind == "randint":
            data[lab] = (rng.randint(0, 8, 25), rng.randint(0, 8, 2000))
        else:
            data[lab] = _split(kind, a, 2000, 100 + j)
    n = 1 << 17

    def level(ws):
        plans = hdist.plan_units([k for _, k, _ in specs], n, ws)
        recs = []
        for units in plans:
            works = [LabelWork(specs[i][0], specs[i][1], specs[i][2], *data[specs[i][0]],
                               n_cand=c, key=1000 + i, cand_base=s, n_total=n)
                     for i, s, c in units]
            res = engine.run(works, precision=32)
            rec = hdist.empty_records(len(specs))
            for (i, _, _), r in zip(units, res):
                one = np.array([(r.score, r.index, r.value, r.n_scored)], hdist.L.BEST_DTYPE)
                rec[i] = hdist.combine_host(np.stack([rec[i:i + 1].view(np.uint8),
                                                      one.view(np.uint8)]))[0]
            recs.append(rec)
        return hdist.combine_device(np.stack(recs))

    one = level(1)
    for ws in (2, 3, 8, 16):
        assert level(ws).tobytes() == one.tobytes(), ws
