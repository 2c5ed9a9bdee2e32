"""Categorical labels on the suggest path: tpe_categorical_suggest (the first
`lat_prefix` candidates, the rest of a stream only where an unseen
better-scoring category could still be drawn) gives the full-stream winner
of tpe_score_categorical byte for byte -- np.argmax over the label's own
candidate stream (tpe.py:575-610 sampling, :649-658 argmax), which the
parity tests pin to the oracle.

The rare-best histories make the best-scoring category rare in the below
posterior (a tiny prior weight and no below observations of it): after the
prefix it is usually unseen, the decision stays open, the rest of the stream
is drawn, and some keys' winners lie past the prefix.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1 << 20
T = 10_000


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


def _runs(engine, works, prefixes, **kw):
    out = {}
    old = engine.lat_prefix
    try:
        for p in prefixes:
            engine.lat_prefix = p
            rs = engine.run(works, precision=32, **kw)
            need = engine._bufs["cat_need"][:4 * len(works)].cpu().numpy().view(np.int32).copy() \
                if p and "cat_need" in engine._bufs else None
            out[p] = ([(r.score, r.index, r.value, r.n_scored) for r in rs], need)
    finally:
        engine.lat_prefix = old
    return out


@pytest.mark.parametrize("K", [3, 8, 13, 40])
def test_prefix_equals_full_stream(engine, K):
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(K)
    works = []
    for key in range(6):
        below = rng.randint(0, K, 25).astype(float)
        above = rng.randint(0, K, T - 25).astype(float)
        works.append(LabelWork("c%d" % key, "randint", (K,), below, above, n_cand=N,
                               key=7000 + key))
    out = _runs(engine, works, (0, 4096, 1 << 16))
    assert out[4096][0] == out[0][0]
    assert out[1 << 16][0] == out[0][0]


def test_rare_best_category_draws_the_rest(engine):
    from hyperopt_amd.engine import LabelWork
    K = 8
    rng = np.random.RandomState(11)
    below = rng.randint(0, K - 1, 25).astype(float)  # never category 7
    above = rng.randint(0, K - 1, T - 25).astype(float)
    works = [LabelWork("c", "randint", (K,), below, above, n_cand=N, key=9100 + k)
             for k in range(8)]
    # p_below(7) ~ 1e-5: ~0.04 draws in a 4096 prefix, ~10 in the whole stream
    out = _runs(engine, works, (0, 4096), prior_weight=2e-3)
    full, _ = out[0]
    pre, need = out[4096]
    assert pre == full
    # category 7 scores best: a job stays open unless its prefix drew it
    assert need is not None
    assert need.tolist() == [int(not (r[2] == K - 1 and r[1] < 4096)) for r in full]
    assert need.sum() >= 4
    assert any(r[2] == K - 1 for r in full)
    assert any(r[1] >= 4096 for r in full)  # a winner past the prefix
