"""Two issuing threads for the level launcher (tpe_set_issue_threads(2),
csrc/tpe_ops.hip): the caller issues the main stream's records, a resident
worker the side stream's, event records in their global list order.

The GPU must see the same work and dependencies as under one-thread issue:
  * a chain of copies bounced between two streams through event records, run
    many times with fresh data, always delivers the source (a wait issued
    before its record would let a copy read stale data);
  * the first failing record in list order is reported, on either thread;
  * whole recorded levels give the eager engine's winners byte for byte with
    one and with two issuing threads, side stream on.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ops(L, records):
    ops = np.zeros(len(records), L.OP_DTYPE)
    for i, (code, args) in enumerate(records):
        ops[i]["code"], ops[i]["n_args"] = code, len(args)
        ops[i]["a"][:len(args)] = [int(a) for a in args]
    return ops


@pytest.fixture
def two_threads():
    from hyperopt_amd import _lib as L
    lib = L.load()
    prev = lib.tpe_set_issue_threads(2)
    assert prev in (1, 2)
    yield lib
    lib.tpe_set_issue_threads(prev)


def _event(L):
    h = ctypes.c_void_p()
    L.hip_check(L.hip().hipEventCreateWithFlags(ctypes.byref(h), L.EVENT_NO_TIMING), "event")
    return h.value


def test_bounced_copies_see_their_records(two_threads):
    import torch
    from hyperopt_amd import _lib as L
    lib = two_threads
    n = 1 << 20
    main = torch.cuda.current_stream().cuda_stream
    side = torch.cuda.Stream().cuda_stream
    a, b, c = (torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3))
    src = torch.empty(n, dtype=torch.float32).pin_memory()
    dst = torch.empty(n, dtype=torch.float32).pin_memory()
    e1, e2, e3 = _event(L), _event(L), _event(L)
    nb = 4 * n
    D2D = 3
    rec = [
        (L.OP_MEMCPY, [a.data_ptr(), src.data_ptr(), nb, L.H2D, main]),
        (L.OP_EVENT_RECORD, [e1, main]),
        (L.OP_STREAM_WAIT, [side, e1]),
        (L.OP_MEMCPY, [b.data_ptr(), a.data_ptr(), nb, D2D, side]),
        (L.OP_MEMCPY, [c.data_ptr(), b.data_ptr(), nb, D2D, side]),
        (L.OP_EVENT_RECORD, [e2, side]),
        (L.OP_STREAM_WAIT, [main, e2]),
        (L.OP_MEMCPY, [a.data_ptr(), c.data_ptr(), nb, D2D, main]),
        (L.OP_EVENT_RECORD, [e3, main]),
        (L.OP_STREAM_WAIT, [side, e3]),
        (L.OP_MEMCPY, [b.data_ptr(), a.data_ptr(), nb, D2D, side]),
        (L.OP_EVENT_RECORD, [e2, side]),   # an event recorded twice in one list
        (L.OP_STREAM_WAIT, [main, e2]),
        (L.OP_MEMCPY, [dst.data_ptr(), b.data_ptr(), nb, L.D2H, main]),
        (L.OP_STREAM_SYNC, [main]),
    ]
    ops = _ops(L, rec)
    failed = ctypes.c_int(5)
    for it in range(60):
        src.fill_(float(it + 1))
        src[it] = -1.0
        rc = lib.tpe_run_ops(ops.ctypes.data_as(ctypes.c_void_p), len(ops), ctypes.byref(failed))
        assert rc == 0 and failed.value == -1, lib.tpe_last_error()
        assert torch.equal(dst, src), it


def test_first_failing_record_is_reported(two_threads):
    import torch
    from hyperopt_amd import _lib as L
    lib = two_threads
    main = torch.cuda.current_stream().cuda_stream
    side = torch.cuda.Stream().cuda_stream
    fit = L.OP_CODES["tpe_parzen_fit"]
    nfit = len(L._SIGNATURES["tpe_parzen_fit"][1])

    def fit_rec(stream, n_seg):  # n_seg = 0: nothing to do; -1: argument error
        args = [0] * nfit
        args[3] = n_seg
        args[-1] = stream
        return (fit, args)
    e = _event(L)
    failed = ctypes.c_int(7)
    cases = [  # (records, failing index)
        ([fit_rec(main, 0), fit_rec(side, 0), fit_rec(side, -1), fit_rec(main, 0)], 2),
        ([fit_rec(main, 0), fit_rec(main, -1), fit_rec(side, 0), fit_rec(side, -1)], 1),
        ([fit_rec(side, 0), (L.OP_EVENT_RECORD, [e, main]), (L.OP_STREAM_WAIT, [side, e]),
          fit_rec(side, -1), fit_rec(main, 0), fit_rec(main, -1)], 3),
        ([fit_rec(main, 0), fit_rec(side, 0), fit_rec(main, 0), fit_rec(side, 0)], -1),
    ]
    for records, want in cases:
        ops = _ops(L, records)
        rc = lib.tpe_run_ops(ops.ctypes.data_as(ctypes.c_void_p), len(ops), ctypes.byref(failed))
        assert failed.value == want, (want, failed.value)
        if want >= 0:
            assert rc == -1 and b"tpe_parzen_fit" in lib.tpe_last_error()
        else:
            assert rc == 0
    torch.cuda.synchronize()


def test_levels_equal_with_one_and_two_threads():
    from hyperopt_amd import _lib as L
    from tests.test_gpu_replay import SPACE, _history, _pair, _rows, _works
    eager, native, DeviceHistory = _pair("native")
    for e in (eager, native):
        e.side_stream = "1"
    lib = L.load()
    T = 2500
    mat, active, losses = _history(T, 17)
    he = DeviceHistory(eager, len(SPACE), cap=4096)
    hn = DeviceHistory(native, len(SPACE), cap=4096)
    for h in (he, hn):
        h.append(mat, active)
    prev = lib.tpe_set_issue_threads(1)
    try:
        for step in range(8):
            works, isb = _works(mat, active, losses, T, step % 3, 1 << 17)
            ref = _rows(eager.run(works, history=he, is_below=isb))
            lib.tpe_set_issue_threads(1 + step % 2)
            got = _rows(native.run(works, history=hn, is_below=isb))
            assert got == ref, step
    finally:
        lib.tpe_set_issue_threads(prev)
    assert native.graph_stats.get("native", 0) >= 4, native.graph_stats
