"""tpe_maxloc_allreduce (the ABI's cross-GPU max-loc) through a
real RCCL communicator.  One GPU per box here, so the communicator has one
rank: the all-gather is a copy and the combine folds one set -- the call
path, the RCCL binding and the record layout are what is checked; the
multi-rank fold itself is tpe_best_combine's (test_gpu_shard.py) and the
torch path's (tests/test_dist_gloo.py)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_byte * 128)]


def _comm():
    import torch  # noqa: F401  (loads the process's RCCL, which the library binds)
    rccl = ctypes.CDLL("librccl.so.1")
    uid = _UniqueId()
    assert rccl.ncclGetUniqueId(ctypes.byref(uid)) == 0
    comm = ctypes.c_void_p()
    assert rccl.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0
    return rccl, comm


def test_maxloc_allreduce_one_rank():
    import torch
    from hyperopt_amd import _lib as L
    lib = L.load()
    torch.cuda.set_device(0)
    rccl, comm = _comm()
    try:
        rec = np.zeros(5, L.BEST_DTYPE)
        rec["score"] = [0.5, np.nan, -1.0, 2.0, 0.0]
        rec["index"] = [7, 3, -1, 11, 0]
        rec["value"] = [1.5, 2.5, 0.0, -4.0, 9.0]
        rec["n_scored"] = [100, 100, 0, 64, 1]
        dev = torch.device("cuda", 0)
        loc = torch.from_numpy(rec.view(np.uint8).copy()).to(dev)
        gat = torch.empty_like(loc)
        out = torch.zeros_like(loc)
        st = torch.cuda.current_stream(dev)
        rc = lib.tpe_maxloc_allreduce(loc.data_ptr(), gat.data_ptr(), out.data_ptr(), 5, comm,
                                      ctypes.c_void_p(st.cuda_stream))
        assert rc == 0, lib.tpe_last_error()
        got = out.cpu().numpy().view(L.BEST_DTYPE)
        for f in ("index", "n_scored"):
            np.testing.assert_array_equal(got[f], rec[f])
        np.testing.assert_array_equal(got["value"], rec["value"])
        np.testing.assert_array_equal(np.isnan(got["score"]), np.isnan(rec["score"]))
        ok = ~np.isnan(rec["score"])
        np.testing.assert_array_equal(got["score"][ok], rec["score"][ok])
    finally:
        rccl.ncclCommDestroy(comm)


@pytest.mark.parametrize("native", [False, True])
def test_level_exchange_one_rank(native):
    """Engine.run(exchange=...): a label-sharded level's winners folded into
    label slots on the device and all-reduced over the communicator inside
    the level (bench.py's multi-GPU step) equal the host fold of the
    per-work results; replayed levels (native launcher) included."""
    import torch
    from hyperopt_amd import _lib as L
    from hyperopt_amd import dist as hdist
    from hyperopt_amd.engine import DeviceHistory, Engine, LabelWork
    torch.cuda.set_device(0)
    rccl, comm = _comm()
    try:
        eng = Engine()
        eng.native = native
        rng = np.random.RandomState(3)
        T = 1500
        mat = np.stack([rng.uniform(-5, 5, T), rng.normal(0, 2, T),
                        np.round(rng.uniform(0, 20, T)), rng.randint(0, 6, T).astype(float)], 1)
        hist = DeviceHistory(eng, 4, cap=2048)
        hist.append(mat)
        isb = np.zeros(T, np.uint8)
        isb[np.argsort(rng.normal(size=T))[:10]] = 1
        space = [("u", "uniform", (-5.0, 5.0)), ("n", "normal", (0.0, 2.0)),
                 ("q", "quniform", (0.0, 20.0, 1.0)), ("c", "randint", (6,))]
        # this "rank" holds labels 3, 0 and two candidate ranges of label 1 in
        # slots of a 6-label level (slots 2, 4, 5 empty)
        units = [(0, 3, 0, 1 << 16), (1, 0, 0, 1 << 16), (2, 1, 0, 1 << 15), (3, 1, 1 << 15, 1 << 15)]
        for step in range(4):
            works = []
            for col, slot, start, count in units:
                lab, kind, a = space[col]
                below = mat[:, col][isb == 1]
                works.append(LabelWork(lab, kind, a, below, None, n_cand=count,
                                       key=97 * step + col, cand_base=start, col=col,
                                       n_above=int((isb == 0).sum()), n_total=1 << 16))
            res = eng.run(works, history=hist, is_below=isb,
                          exchange=(comm.value, 6, 1, [u[1] for u in units]))
            got = eng.last_exchange
            want = hdist.gather_best(6, [(u[1], r) for u, r in zip(units, res)])
            assert [(float(x["score"]), int(x["index"]), float(x["value"]), int(x["n_scored"]))
                    for x in got] == want
            assert got["index"][2] == -1 and got["n_scored"][1] == 1 << 16
        if native:
            assert eng.graph_stats.get("native", 0) >= 2
    finally:
        rccl.ncclCommDestroy(comm)


@pytest.mark.parametrize("native", [False, True])
def test_level_exchange_settles_band_overflow(native, monkeypatch):
    """A table-path label whose band overflows (BAND_TILE_CAP = 0: every
    scorer tile is full) leaves the level with n_scored = -1; the in-level
    exchange carries the -1 to every rank, and Engine._exchange_fix runs the
    exchange once more on the rank's exact records (after _band_fix re-scored
    the stream in fp64).  On a one-rank communicator: one fix per level, the
    label record holds the full count and the exact argmax of the stream --
    first run and the replayed (re-issued) run alike."""
    import torch
    import hyperopt_amd.engine as E
    from oracle import tpe_oracle as O
    monkeypatch.setattr(E, "BAND_TILE_CAP", 0)
    torch.cuda.set_device(0)
    rccl, comm = _comm()
    try:
        eng = E.Engine()
        eng.native = native
        rng = np.random.RandomState(5)
        T, n = 3000, 1 << 17
        mat = np.stack([rng.uniform(-5, 5, T), np.exp(rng.uniform(-5, 0, T))], 1)
        hist = E.DeviceHistory(eng, 2, cap=4096)
        hist.append(mat)
        isb = np.zeros(T, np.uint8)
        isb[np.argsort(rng.normal(size=T))[:T // 4]] = 1
        space = [("u", "uniform", (-5.0, 5.0)), ("l", "loguniform", (-5.0, 0.0))]
        slots = [1, 0]
        ref = None
        for step in range(3):
            works = []
            for col, (lab, kind, a) in enumerate(space):
                works.append(E.LabelWork(lab, kind, a, mat[:, col][isb == 1], None, n_cand=n,
                                         key=4242 + col, col=col,
                                         n_above=int((isb == 0).sum()), n_total=n))
            before = getattr(eng, "exchange_fixes", 0)
            res = eng.run(works, precision=32, history=hist, is_below=isb,
                          exchange=(comm.value, 2, 1, slots))
            assert getattr(eng, "exchange_fixes", 0) == before + 1
            got = eng.last_exchange
            assert list(got["n_scored"]) == [n, n]
            for col, (lab, kind, a) in enumerate(space):
                r, x = res[col], got[slots[col]]
                assert r.n_scored == n
                assert (int(x["index"]), float(x["value"])) == (r.index, r.value)
            if ref is None:
                ref = [(r.index, r.value) for r in res]
                # the exact argmax of each label's materialised fp32 stream
                for col, (lab, kind, a) in enumerate(space):
                    w = works[col]
                    s, = E.Engine().run([E.LabelWork(lab, kind, a, w.obs_below,
                                                     mat[:, col][isb == 0], n_cand=n,
                                                     key=w.key)],
                                        precision=32, sample_only=True)
                    d, = E.Engine().run([E.LabelWork(lab, kind, a, w.obs_below,
                                                     mat[:, col][isb == 0], cand=s.cand)],
                                        precision=64, outputs=True)
                    best = int(np.argmax(d.below_llik - d.above_llik))
                    assert res[col].index == best and res[col].value == s.cand[best]
                    with np.errstate(all="ignore"):
                        o = O.continuous_label_scores(kind, a, w.obs_below,
                                                      mat[:, col][isb == 0], s.cand[[best]])
                    np.testing.assert_allclose(o["below_llik"] - o["above_llik"],
                                               res[col].score, rtol=1e-9, atol=1e-9)
            else:
                assert [(r.index, r.value) for r in res] == ref
        if native:
            assert eng.graph_stats.get("native", 0) >= 1
    finally:
        rccl.ncclCommDestroy(comm)
