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
