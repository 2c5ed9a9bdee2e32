"""Config C4 (BASELINE configs[3]) shape: many independent 20-dim studies with
2k-trial histories, batched through ``tpe.suggest_many``.

* Every study's suggestion from the batched call equals its own
  ``tpe.suggest`` (same Philox keys, same kernels; the batch only shares
  launches) -- at 256 studies x 20 dims x 2000 trials.
* For a sample of studies, the fitted posteriors and log-densities of every
  label on injected candidates match the oracle (fp64 rtol 1e-6, argmax
  exact, categorical exact) -- the reference's per-label pipeline,
  tpe.py:661-757 and :837-964, at C4's history shape.
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

STUDIES, T, N_EI = 256, 2000, 1 << 12


@pytest.fixture(scope="module")
def studies():
    from hyperopt_amd.base import Domain
    from tools import scale_configs as S
    doms = [Domain(lambda p: 0.0, S.c4_space(s)) for s in range(STUDIES)]
    trs = [S.flat_trials(d, T, s) for s, d in enumerate(doms)]
    return doms, trs


def test_suggest_many_equals_per_study_suggest(studies):
    from hyperopt_amd import tpe
    doms, trs = studies
    reqs = [tpe.SuggestRequest([T], d, t, 1000 + s, n_EI_candidates=N_EI)
            for s, (d, t) in enumerate(zip(doms, trs))]
    many = tpe.suggest_many(reqs)
    assert len(many) == STUDIES
    for s, (d, t) in enumerate(zip(doms, trs)):
        one = tpe.suggest([T], d, t, 1000 + s, n_EI_candidates=N_EI, verbose=False)
        assert many[s][0]["misc"]["vals"] == one[0]["misc"]["vals"], s
        assert many[s][0]["tid"] == one[0]["tid"] == T
        assert set(many[s][0]["misc"]["vals"]) == set(d.params)
    # the studies do not all suggest the same point (independent keys / histories)
    firsts = {tuple(sorted((k, v[0]) for k, v in m[0]["misc"]["vals"].items())) for m in many}
    assert len(firsts) == STUDIES


@pytest.mark.parametrize("s", [0, 17, 255])
def test_c4_study_vs_oracle_on_injected(studies, s):
    from hyperopt_amd.engine import Engine, LabelWork
    doms, trs = studies
    d, t = doms[s], trs[s]
    docs = t.trials
    losses = np.array([x["result"]["loss"] for x in docs])
    tids = np.arange(len(docs))
    rng = np.random.RandomState(s)
    works, refs = [], []
    for lab in d.params:
        spec = d.specs[lab]
        vals = np.array([x["misc"]["vals"][lab][0] for x in docs], dtype=np.float64)
        below, above = O.ap_split_trials(tids, vals, tids, losses, 0.25)
        if spec.kind in ("randint", "categorical"):
            K = len(spec.args[0]) if spec.kind == "categorical" else int(spec.args[0])
            cand = rng.randint(0, K, 512).astype(np.float64)
        else:
            lo, hi = np.percentile(vals, [0.5, 99.5])
            cand = rng.uniform(lo, hi, 512)
            if spec.kind.startswith("q"):
                cand = np.round(cand / spec.args[2]) * spec.args[2]
        works.append(LabelWork(lab, spec.kind, tuple(spec.args), below, above, cand=cand))
    eng = Engine()
    res = eng.run(works, precision=64, outputs=True)
    for w, r in zip(works, res):
        with np.errstate(all="ignore"):
            if w.kind in ("randint", "categorical"):
                ref = O.categorical_label_scores(w.kind, w.args, w.obs_below, w.obs_above,
                                                 w.cand.astype(np.int64))
                np.testing.assert_allclose(r.below_llik, ref["below_llik"], rtol=1e-14)
                np.testing.assert_allclose(r.above_llik, ref["above_llik"], rtol=1e-14)
            else:
                ref = O.continuous_label_scores(w.kind, w.args, w.obs_below, w.obs_above,
                                                w.cand)
                np.testing.assert_allclose(r.below_llik, ref["below_llik"], rtol=1e-6,
                                           err_msg=w.label)
                np.testing.assert_allclose(r.above_llik, ref["above_llik"], rtol=1e-6,
                                           err_msg=w.label)
        s_ref = ref["below_llik"] - ref["above_llik"]
        assert r.index == int(np.argmax(s_ref)), (w.label, r.index, int(np.argmax(s_ref)))


@pytest.mark.parametrize("chunk", ["3", "0"])
def test_suggest_many_chunked_mixed_spaces(monkeypatch, chunk):
    """Pipelined chunks (two engines, deferred readback) over studies of
    different spaces -- nested choices (several levels), a 50-dim mixed space,
    the README space -- one of them still in its startup phase: each study's
    suggestion equals its own tpe.suggest."""
    from hyperopt_amd import hp, tpe
    from hyperopt_amd.base import Domain
    from tests.golden import spaces
    from tools import scale_configs as S
    monkeypatch.setenv("HYPEROPT_AMD_CHUNK", chunk)
    makers = [spaces.nested, spaces.mixed_50d, spaces.readme, spaces.many_dists]
    doms, trs = [], []
    for s in range(11):
        d = Domain(lambda p: 0.0, makers[s % len(makers)](hp))
        doms.append(d)
        trs.append(S.prior_trials(d, 10 if s == 5 else 300 + 37 * s, s))
    reqs = [tpe.SuggestRequest([10_000 + s], d, t, 77 + s,
                               n_EI_candidates=512)
            for s, (d, t) in enumerate(zip(doms, trs))]
    many = tpe.suggest_many(reqs)
    for s, (rq, m) in enumerate(zip(reqs, many)):
        one = tpe.suggest(rq.new_ids, rq.domain, rq.trials, rq.seed, n_EI_candidates=512,
                          verbose=False)
        assert m[0]["misc"]["vals"] == one[0]["misc"]["vals"], s


def test_c4_4096_studies_rank_by_rank(monkeypatch):
    """C4 at its stated size: 4096 studies through suggest_many(shard_studies=
    True), rehearsed rank by rank on one GPU (hdist.world() patched to (r, 8)):
    rank r returns exactly studies r::8, each equal to the unsharded batched
    call's suggestion, and a sample equals its own tpe.suggest.  64 distinct
    20-dim spaces / 2k-trial histories are shared round-robin by the 4096
    studies (each with its own seed, so its own Philox keys)."""
    from hyperopt_amd import dist as hdist
    from hyperopt_amd import tpe
    from hyperopt_amd.base import Domain
    from tools import scale_configs as S
    n_hist, n_studies, world = 64, 4096, 8
    doms = [Domain(lambda p: 0.0, S.c4_space(s)) for s in range(n_hist)]
    trs = [S.flat_trials(d, T, s) for s, d in enumerate(doms)]

    def reqs():
        return [tpe.SuggestRequest([T], doms[q % n_hist], trs[q % n_hist], 5000 + q,
                                   n_EI_candidates=N_EI) for q in range(n_studies)]
    whole = tpe.suggest_many(reqs())
    assert all(w is not None and len(w) == 1 for w in whole)
    for r in range(world):
        monkeypatch.setattr(hdist, "world", lambda r=r: (r, world))
        part = tpe.suggest_many(reqs(), shard_studies=True)
        for q in range(n_studies):
            if q % world == r:
                assert part[q][0]["misc"]["vals"] == whole[q][0]["misc"]["vals"], (r, q)
            else:
                assert part[q] is None
    monkeypatch.undo()
    for q in np.random.RandomState(3).choice(n_studies, 16, replace=False):
        one = tpe.suggest([T], doms[q % n_hist], trs[q % n_hist], 5000 + q,
                          n_EI_candidates=N_EI, verbose=False)
        assert one[0]["misc"]["vals"] == whole[q][0]["misc"]["vals"], q
