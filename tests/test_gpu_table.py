"""Cell-table scorer (tpe_table_build + tpe_score_table) vs the oracle.

The table path expands each mixture per cell; its
per-candidate log-densities must match GMM1_lpdf / LGMM1_lpdf (tpe.py:117-180,
265-307) within the fp32 tolerance of north_star (rtol 1e-4, atol 1e-4 for
log-densities near 0), on the reference's own injected candidates (goldens),
on injected candidates of random histories, and on its own sampled
candidates.  The argmax must be the dense fp32 kernel's winner or a
candidate whose exact fp64 score ties it within fp32 rounding.
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O
from tests.golden_io import E2E_CASES
from tests.test_gpu_parity import _mixture_case, _works_from_fixture

pytestmark = pytest.mark.gpu

RTOL = ATOL = 1e-4

CONT = [("uniform", (-5.0, 5.0)), ("loguniform", (-5.0, 0.0)), ("normal", (0.0, 2.0)),
        ("lognormal", (0.0, 1.0))]


@pytest.fixture(scope="module")
def engine():
    from hyperopt_amd.engine import Engine
    return Engine()


def _oracle(w, cand=None):
    cand = w.cand if cand is None else cand
    with np.errstate(all="ignore"):
        return O.continuous_label_scores(w.kind, w.args, w.obs_below, w.obs_above, cand)


@pytest.mark.parametrize("case", E2E_CASES)
def test_golden_table(engine, case):
    works, golden, meta = _works_from_fixture(case)
    res = engine.run(works, prior_weight=meta["prior_weight"], precision=32, outputs=True,
                     scorer="table")
    for w, r, (bl, al, best) in zip(works, res, golden):
        np.testing.assert_allclose(r.below_llik, bl, rtol=RTOL, atol=ATOL, equal_nan=True,
                                   err_msg="%s/%s below" % (case, w.label))
        np.testing.assert_allclose(r.above_llik, al, rtol=RTOL, atol=ATOL, equal_nan=True,
                                   err_msg="%s/%s above" % (case, w.label))
        score = bl - al
        if w.kind in ("randint", "categorical") or w.kind.startswith("q"):
            assert r.index == best
        else:
            assert score[r.index] >= np.nanmax(score) - 1e-4 * max(1.0, abs(np.nanmax(score)))


@pytest.mark.parametrize("kind,args", CONT)
@pytest.mark.parametrize("n_above", [0, 1, 2, 30, 3000, 10000])
def test_table_injected_vs_oracle(engine, kind, args, n_above):
    rng = np.random.RandomState(1000 + n_above)
    w = _mixture_case(rng, kind, args, min(n_above, 25), n_above, 4096)
    r, = engine.run([w], precision=32, outputs=True, scorer="table")
    ref = _oracle(w)
    np.testing.assert_allclose(r.below_llik, ref["below_llik"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(r.above_llik, ref["above_llik"], rtol=RTOL, atol=ATOL)
    s = ref["below_llik"] - ref["above_llik"]
    assert s[r.index] >= np.nanmax(s) - 1e-4 * max(1.0, abs(np.nanmax(s)))
    st = engine.last_table_stats
    assert st["failed_cells"] == 0, st
    # every injected candidate inside the sampler's range is on the table
    assert st["exact_candidates"] <= 0.01 * w.cand.size, st


def test_table_far_tails_and_ties(engine):
    """Off-grid candidates (+-1e3, +-60) take the exact path; duplicates tie
    to the first index."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(7)
    obs_b = rng.uniform(-5, 5, 25)
    obs_a = rng.uniform(-5, 5, 4000)
    base = rng.uniform(-5, 5, 300)
    cand = np.concatenate([base, base[::-1], [-1e3, 1e3, 60.0, -60.0]])
    w = LabelWork("x", "uniform", (-5.0, 5.0), obs_b, obs_a, cand=cand)
    ref = _oracle(w)
    r, = engine.run([w], precision=32, outputs=True, scorer="table")
    np.testing.assert_allclose(r.above_llik, ref["above_llik"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(r.below_llik, ref["below_llik"], rtol=RTOL, atol=ATOL)
    assert engine.last_table_stats["exact_candidates"] >= 4
    s = ref["below_llik"] - ref["above_llik"]
    assert s[r.index] >= np.nanmax(s) - 1e-4 * max(1.0, abs(np.nanmax(s)))


@pytest.mark.parametrize("kind,args", CONT)
def test_table_small_budget_falls_back_exactly(engine, kind, args, monkeypatch):
    """A cell budget far below what the error bound needs: failing cells are
    flagged and their candidates scored exactly -- same results."""
    import hyperopt_amd.engine as E
    monkeypatch.setattr(E, "TABLE_CAP", 8)
    rng = np.random.RandomState(3)
    w = _mixture_case(rng, kind, args, 25, 5000, 2048)
    r, = engine.run([w], precision=32, outputs=True, scorer="table")
    ref = _oracle(w)
    np.testing.assert_allclose(r.below_llik, ref["below_llik"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(r.above_llik, ref["above_llik"], rtol=RTOL, atol=ATOL)
    assert engine.last_table_stats["failed_cells"] > 0


@pytest.mark.parametrize("kind,args", CONT)
@pytest.mark.parametrize("n_hist", [3, 40, 2000, 10000])
def test_table_sampled_vs_oracle_and_dense(engine, kind, args, n_hist):
    """Own Philox candidates: per-candidate log-densities vs the oracle at the
    drawn values, and the winner vs the dense fp32 kernel's."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(n_hist + 17)
    gen = _mixture_case(rng, kind, args, 1, n_hist, 1)
    obs = gen.obs_above
    losses = rng.normal(size=n_hist)
    below, above = O.ap_split_trials(np.arange(n_hist), obs, np.arange(n_hist), losses, 0.25)
    n = 1 << 16
    w = LabelWork(kind, kind, args, below, above, n_cand=n, key=424242 + n_hist)
    tab, = engine.run([w], precision=32, outputs=True, scorer="table")
    st = engine.last_table_stats
    assert st["failed_cells"] == 0 and st["exact_candidates"] == 0, st
    dense, = engine.run([w], precision=32, outputs=True, scorer="dense")
    np.testing.assert_array_equal(tab.cand, dense.cand)  # same Philox draws
    pick = np.random.RandomState(0).choice(n, 3000, replace=False)
    ref = _oracle(w, cand=tab.cand[pick])
    np.testing.assert_allclose(tab.below_llik[pick], ref["below_llik"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(tab.above_llik[pick], ref["above_llik"], rtol=RTOL, atol=ATOL)
    assert tab.n_scored == n
    if tab.index != dense.index:
        w2 = LabelWork(kind, kind, args, below, above, cand=np.array([dense.value, tab.value]))
        r, = engine.run([w2], precision=64, outputs=True)
        s = r.below_llik - r.above_llik
        assert abs(s[0] - s[1]) <= 1e-4 * max(1.0, abs(s[0])), (s, dense, tab)


def test_auto_scorer_uses_table_for_large_n(engine):
    from hyperopt_amd.engine import LabelWork, TABLE_MIN_CAND
    rng = np.random.RandomState(5)
    w = LabelWork("x", "uniform", (-5.0, 5.0), rng.uniform(-5, 5, 25), rng.uniform(-5, 5, 5000),
                  n_cand=TABLE_MIN_CAND, key=99)
    timers = {}
    engine.run([w], precision=32, timers=timers)
    assert "table" in timers and "table_build" in timers


C3_KINDS = [("uniform", (-5.0, 5.0), lambda r, n: r.uniform(-5, 5, n)),
            ("loguniform", (-5.0, 0.0), lambda r, n: np.exp(r.uniform(-5, 0, n))),
            ("normal", (0.0, 2.0), lambda r, n: r.normal(0, 2, n)),
            ("lognormal", (0.0, 1.0), lambda r, n: np.exp(r.normal(0, 1, n)))]


def _exact_argmax(kind, args, below, above, cand):
    """np.argmax over the fp64 scores of `cand` (the dense fp64 kernel, whose
    log-densities test_gpu_parity pins to the oracle at rtol 1e-6)."""
    from hyperopt_amd.engine import Engine, LabelWork
    eng = Engine()
    eng.exact64 = "dense"
    x, = eng.run([LabelWork(kind, kind, args, below, above, cand=cand)], precision=64,
                 outputs=True)
    s64 = x.below_llik - x.above_llik
    best = int(np.argmax(s64))
    assert x.index == best
    return s64, best


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("kind,args,gen", C3_KINDS)
def test_table_winner_at_c3_size_is_the_exact_argmax(engine, kind, args, gen, seed):
    """C3's continuous labels at full size (10k-trial history, 2^22 candidates):
    the suggest path's winner (fp32 table scores, then the exact fp64
    re-score of every candidate within the fp32 error bound of the maximum)
    IS np.argmax over the exact fp64 scores of the SAME 2^22 candidates (the
    stream materialised by sample_only) -- index, value and score
    (tpe.py:649-658; north_star: argmax indices bit-exact)."""
    from hyperopt_amd.engine import LabelWork
    T, n = 10_000, 1 << 22
    rng = np.random.RandomState(100 + seed)
    obs = gen(rng, T)
    losses = np.random.RandomState(200 + seed).normal(size=T)
    below, above = O.ap_split_trials(np.arange(T), obs, np.arange(T), losses, 0.25)
    w = LabelWork(kind, kind, args, below, above, n_cand=n, key=0xC3 + seed)
    r, = engine.run([w], precision=32)
    assert engine.last_table_stats is not None  # the table path ran
    s, = engine.run([w], precision=32, sample_only=True)
    cand = s.cand
    s64, best = _exact_argmax(kind, args, below, above, cand)
    assert r.index == best, (r.index, best, s64[r.index], s64[best])
    assert r.value == cand[best] and r.n_scored == n
    np.testing.assert_allclose(r.score, s64[best], rtol=1e-12, atol=1e-12)
    # the winner and the runner-up re-scored by the oracle
    second = int(np.argmax(np.where(np.arange(n) == best, -np.inf, s64)))
    pick = np.array([best, second])
    ref = _oracle(w, cand=cand[pick])
    np.testing.assert_allclose(ref["below_llik"] - ref["above_llik"], s64[pick], rtol=1e-6,
                               atol=1e-9)


@pytest.mark.parametrize("seed", range(2))
@pytest.mark.parametrize("kind,args,gen", C3_KINDS)
def test_table_eps_bounds_every_score_at_c3_size(engine, kind, args, gen, seed):
    """The band's bound is a bound: at C3 size (10k-trial history, 2^22
    candidates) EVERY candidate's fp32 score is within the eps the kernel
    itself used for it (tpe_score_table_fast's out_eps: eps_cubic + 2.0001
    eps_mix + 2^-22 |s| from the job's tpe_table for a cubic-scored
    candidate, its own bound for a two-polynomial one, +inf for a log-sum-exp
    one) of the exact fp64 score of the same value -- no extra slack.  The
    table's fields are the ones the kernel read."""
    from hyperopt_amd.engine import LabelWork
    T, n = 10_000, 1 << 22
    rng = np.random.RandomState(300 + seed)
    obs = gen(rng, T)
    losses = np.random.RandomState(400 + seed).normal(size=T)
    below, above = O.ap_split_trials(np.arange(T), obs, np.arange(T), losses, 0.25)
    w = LabelWork(kind, kind, args, below, above, n_cand=n, key=0xE95 + seed)
    fast, = engine.run([w], precision=32, table_scores=True)
    tab = fast.extra["table"]
    score, eps = fast.extra["score"], fast.extra["eps"]
    s64, best = _exact_argmax(kind, args, below, above, fast.cand)
    err = np.abs(score - s64)
    assert np.all(err <= eps), (np.max(err - eps), int(np.argmax(err - eps)))
    cubic = np.isfinite(eps)
    want = float(tab["eps_cubic"]) + 2.0001 * float(tab["eps_mix"]) + 2.0 ** -22 * np.abs(score)
    # most candidates are cubic-scored, and those carry the table's own eps
    # (plus the outward rounding of s + eps: at most 2^-22 |s| + 1e-6 eps)
    # (a finite eps is the table's for a cubic-scored candidate; the few on a
    # flagged score cell carry their own, larger two-polynomial bound)
    assert cubic.mean() > 0.999
    e, w_ = eps[cubic], want[cubic]
    assert np.all(e >= w_ * (1 - 1e-6)), np.min(e - w_)
    own = e <= w_ * (1 + 1e-5) + 2.0 ** -22 * (np.abs(score[cubic]) + w_) * 1.01 + 1e-12
    assert own.mean() > 0.999, own.mean()
    assert 0 < tab["eps_mix"] < 5e-5 and 0 < tab["eps_cubic"] < 5e-6, tab
    assert fast.index == best


@pytest.mark.parametrize("kind,args,gen", C3_KINDS[:2])
def test_table_band_overflow_rescored_exactly(kind, args, gen, monkeypatch):
    """More band candidates in a scorer tile than it keeps (BAND_TILE_CAP
    shrunk to 0 here; on real histories a plateau of near-equal scores): the
    engine re-scores that label's whole fp32 stream in fp64
    (tpe_score_pruned64 with TPE_F_DRAW32) -- the winner is still the exact
    argmax."""
    import hyperopt_amd.engine as E
    monkeypatch.setattr(E, "BAND_TILE_CAP", 0)
    eng = E.Engine()
    T, n = 10_000, 1 << 20
    rng = np.random.RandomState(41)
    obs = gen(rng, T)
    losses = rng.normal(size=T)
    below, above = O.ap_split_trials(np.arange(T), obs, np.arange(T), losses, 0.25)
    w = E.LabelWork(kind, kind, args, below, above, n_cand=n, key=77)
    r, = eng.run([w], precision=32)
    assert getattr(eng, "band_overflows", 0) == 1
    assert r.n_scored == n
    s, = eng.run([w], precision=32, sample_only=True)
    s64, best = _exact_argmax(kind, args, below, above, s.cand)
    assert r.value == s.cand[r.index]
    assert r.index == best


@pytest.mark.parametrize("kind,args", CONT)
@pytest.mark.parametrize("n_hist", [3, 40, 2000, 10000])
def test_fast_table_scores_vs_oracle(engine, kind, args, n_hist):
    """The suggest path (tpe_score_table_fast: one score cubic per cell):
    per-candidate scores of its own Philox candidates vs the oracle's
    below - above log-density at the same values (fp32 bound of north_star,
    rtol/atol 1e-4), the same candidates as the two-polynomial kernel, and a
    winner whose exact score is the two-polynomial winner's within fp32."""
    from hyperopt_amd.engine import LabelWork
    rng = np.random.RandomState(n_hist + 71)
    gen = _mixture_case(rng, kind, args, 1, n_hist, 1)
    obs = gen.obs_above
    losses = rng.normal(size=n_hist)
    below, above = O.ap_split_trials(np.arange(n_hist), obs, np.arange(n_hist), losses, 0.25)
    n = 1 << 16
    w = LabelWork(kind, kind, args, below, above, n_cand=n, key=515151 + n_hist)
    fast, = engine.run([w], precision=32, table_scores=True)
    st = engine.last_table_stats
    # (cells whose cubic's proven bound exceeds 1e-6 send their candidates to
    # the two-polynomial cell: up to ~a quarter on the few wide cells of a
    # 3- or 40-trial history, none to a few per mille on real ones)
    assert st["exact_candidates"] <= (n // 3 if n_hist < 100 else n // 50), st
    score = fast.extra["score"]
    poly, = engine.run([w], precision=32, outputs=True, scorer="table")
    np.testing.assert_array_equal(fast.cand, poly.cand)  # same Philox draws
    pick = np.random.RandomState(1).choice(n, 3000, replace=False)
    ref = _oracle(w, cand=fast.cand[pick])
    s_ref = ref["below_llik"] - ref["above_llik"]
    np.testing.assert_allclose(score[pick], s_ref, rtol=RTOL, atol=ATOL)
    # against the two-polynomial scores: the cubic adds ~1e-6 at most
    s_poly = poly.below_llik - poly.above_llik
    np.testing.assert_allclose(score, s_poly, rtol=2e-5, atol=2e-5)
    # the winner is decided exactly: np.argmax of the fp64 scores of the stream
    s64, best = _exact_argmax(kind, args, below, above, fast.cand)
    assert fast.index == best, (fast.index, best)
    assert fast.value == fast.cand[fast.index] and fast.n_scored == n
    np.testing.assert_allclose(fast.score, s64[best], rtol=1e-12, atol=1e-12)
    # and every fp32 score is within the bound the band used for it (no slack)
    eps = fast.extra["eps"]
    assert np.all(np.abs(score - s64) <= eps), np.max(np.abs(score - s64) - eps)
