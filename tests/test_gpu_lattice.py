"""Quantized labels, sampled: the lattice path's argmax is np.argmax over the
label's own candidate stream.

The lattice path (tpe_lattice_sample -> tpe_lattice_compact ->
tpe_score_quantized) never materialises the N candidates: it keeps the first
global index per lattice value and scores every present value once.  The
reference (tpe.py:81-106 sampling with q, tpe.py:159-174 / 288-305 quantized
lpdf, tpe.py:650-658 argmax) scores all N and takes np.argmax.  Here the same
stream is materialised by ``sample_only`` (tpe_sample: at precision 32 it runs
draw32_pairs, the DRAW32 lattice sampler's own code), every candidate is
scored by the ORACLE (fp64, per distinct value), and the engine's index must
equal np.argmax over that stream exactly -- at C3's size (2^20 candidates,
10k-trial history).
"""
import numpy as np
import pytest
from scipy import stats

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

N = 1 << 20
T = 10_000


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


def _history(kind, args, seed):
    rng = np.random.RandomState(seed)
    if kind == "quniform":
        v = np.round(rng.uniform(args[0], args[1], T) / args[2]) * args[2]
    elif kind == "qloguniform":
        v = np.round(np.exp(rng.uniform(args[0], args[1], T)) / args[2]) * args[2]
    elif kind == "qnormal":
        v = np.round(rng.normal(args[0], args[1], T) / args[2]) * args[2]
    else:  # qlognormal
        v = np.round(np.exp(rng.normal(args[0], args[1], T)) / args[2]) * args[2]
    losses = np.random.RandomState(seed + 1).normal(size=T)
    return O.ap_split_trials(np.arange(T), v, np.arange(T), losses, 0.25)


KINDS = [("quniform", (0.0, 100.0, 1.0)),    # the C3 quantized label
         ("quniform", (-3.0, 7.0, 0.25)),    # power-of-two q (fp32 slot path)
         ("qloguniform", (0.0, 4.0, 1.0)),
         ("qnormal", (0.0, 20.0, 2.0)),
         ("qlognormal", (1.0, 0.7, 0.5))]


def _stream_argmax(w, cand):
    """np.argmax of the oracle's fp64 score over every candidate of the
    stream (each distinct value scored once: equal values score equally)."""
    u, inv = np.unique(cand, return_inverse=True)
    with np.errstate(all="ignore"):
        ref = O.continuous_label_scores(w.kind, w.args, w.obs_below, w.obs_above, u)
    s = (ref["below_llik"] - ref["above_llik"])[inv]
    return int(np.argmax(s)), s


@pytest.mark.parametrize("precision", [32, 64])
@pytest.mark.parametrize("kind,args", KINDS)
def test_lattice_argmax_is_argmax_over_own_stream(engine, kind, args, precision):
    from hyperopt_amd.engine import LabelWork
    below, above = _history(kind, args, 11)
    w = LabelWork("q", kind, args, below, above, n_cand=N, key=0xC3C3 + len(kind))
    timers = {}
    r, = engine.run([w], precision=precision, timers=timers)
    assert "lat" in timers  # the lattice path ran (not the dense fallback)
    draw32 = bool(engine.last_plan[3]["flags"][0] & 16)
    if precision == 32 and kind == "quniform":  # C3's kind draws in fp32 (DRAW32)
        assert draw32
    # the stream the lattice sampler drew: the fp32 pair stream for DRAW32
    # jobs, else the fp64 one (wide lattices draw in fp64 at either precision)
    s, = engine.run([w], precision=32 if draw32 else 64, sample_only=True)
    cand = s.cand
    assert cand.size == N
    k = np.round(cand / args[2])
    assert np.all(k * args[2] == cand)  # every candidate is a lattice value
    best, score = _stream_argmax(w, cand)
    assert r.index == best, (r.index, best, score[r.index], score[best])
    assert r.value == cand[best]
    assert r.n_scored == N
    np.testing.assert_allclose(r.score, score[best], rtol=1e-9, atol=1e-12)


def test_lattice_shard_split_matches_unsplit(engine):
    """Splitting the candidate range (odd and even split points) and combining
    the two winners on the device (tpe_best_combine) gives the unsplit
    winner, byte for byte."""
    from hyperopt_amd import dist as hdist
    from hyperopt_amd.engine import LabelWork
    kind, args = KINDS[0]
    below, above = _history(kind, args, 5)
    n = 1 << 18
    key = 777

    def run(base, count):
        w = LabelWork("q", kind, args, below, above, n_cand=count, key=key, cand_base=base,
                      n_total=n)
        r, = engine.run([w], precision=32)
        return np.array([(r.score, r.index, r.value, r.n_scored)], hdist.L.BEST_DTYPE)

    whole = run(0, n)
    for cut in (100_001, 131_072, 3):
        comb = hdist.combine_device(np.stack([run(0, cut), run(cut, n - cut)]))
        assert comb.tobytes() == whole.tobytes(), (cut, comb, whole)


@pytest.mark.parametrize("kind,args", KINDS[:1] + KINDS[2:])
def test_draw32_quantized_chi2(engine, kind, args):
    """The fp32 pair stream of quantized labels (DRAW32, what C3 uses) against
    reference-style rejection draws: chi-square on the lattice counts."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(4)
    fam, pmu, psig, tf, low, high, q = O.posterior_spec(kind, args)
    below, _ = _history(kind, args, 21)
    obs_b = below[:25]
    w = LabelWork("x", kind, args, obs_b, obs_b[:3], n_cand=200_000, key=31)
    r, = engine.run([w], precision=32, sample_only=True)
    x = r.cand
    ref = (O.gmm1_sample if fam == "GMM1" else O.lgmm1_sample)(
        *O.adaptive_parzen_normal(tf(obs_b), 1.0, pmu, psig), low=low, high=high, q=q,
        rng=rng, size=x.size)
    k = np.round(x / q).astype(np.int64)
    kr = np.round(ref / q).astype(np.int64)
    lo, hi = min(k.min(), kr.min()), max(k.max(), kr.max())
    a = np.bincount(k - lo, minlength=hi - lo + 1)
    b = np.bincount(kr - lo, minlength=hi - lo + 1)
    keep = (a + b) >= 20
    table = np.vstack([np.append(a[keep], a[~keep].sum()), np.append(b[keep], b[~keep].sum())])
    table = table[:, table.sum(0) > 0]
    p = stats.chi2_contingency(table)[1]
    assert p > 1e-4, p


def test_lattice_prefix_decision_equals_full_stream(engine):
    """tpe_lattice_suggest (the suggest path: first `lat_prefix` candidates,
    the rest of a stream only where an unseen lattice value could still win)
    gives the full-stream winner byte for byte, and np.argmax's over the
    stream.  The history makes the best values rare: below and above both sit
    at 50, so the top scores are at the edges of [0, 100], where the below
    mixture has only its prior's mass (~1e-4 per value) -- after 4096 draws
    those values are mostly unseen, the decision stays open and the rest of
    the stream is drawn.  Some key's winner lies past the prefix, which pass
    0 alone cannot produce."""
    from hyperopt_amd.engine import LabelWork
    kind, args = KINDS[0]
    rng = np.random.RandomState(0)
    below = np.clip(np.round(rng.normal(50.0, 1.0, 25)), 0, 100)
    above = np.clip(np.round(rng.normal(50.0, 10.0, T - 25)), 0, 100)
    old = engine.lat_prefix
    late = 0
    try:
        for key in range(4240, 4246):
            out = {}
            for p in (0, 4096, 1 << 16):
                engine.lat_prefix = p
                w = LabelWork("q", kind, args, below, above, n_cand=N, key=key)
                r, = engine.run([w], precision=32)
                out[p] = (r.score, r.index, r.value, r.n_scored)
            assert out[4096] == out[0], (key, out[4096], out[0])
            assert out[1 << 16] == out[0], (key, out[1 << 16], out[0])
            s, = engine.run([w], precision=32, sample_only=True)
            best, score = _stream_argmax(w, s.cand)
            assert out[0][1] == best, (key, out[0], best)
            late += out[0][1] >= 4096
    finally:
        engine.lat_prefix = old
    assert late > 0
