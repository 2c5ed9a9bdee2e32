"""The C-ABI library loads without a GPU and exports every entry point that
include/tpe_hip.h declares; argument errors are reported, never crash."""
import ctypes
import os
import re

import numpy as np
import pytest

from hyperopt_amd import _lib as L

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "tpe_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+(tpe_\w+)\s*\(", text, flags=re.M)))


def test_header_symbols_exported():
    lib = L.load()
    names = declared_functions()
    assert len(names) >= 15, names
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(L._SIGNATURES), set(names) ^ set(L._SIGNATURES)


def test_struct_sizes_and_abi():
    lib = L.load()
    assert lib.tpe_abi_version() == L.ABI_VERSION == 22
    sizes = (ctypes.c_int32 * 11)()
    assert lib.tpe_struct_sizes(ctypes.cast(sizes, ctypes.c_void_p), 11) == 11
    assert tuple(sizes) == (L.SEG_DTYPE.itemsize, L.CAT_SEG_DTYPE.itemsize,
                            L.JOB_DTYPE.itemsize, L.BEST_DTYPE.itemsize, L.TABLE_DTYPE.itemsize,
                            L.GATHER_DTYPE.itemsize, L.HISTORY_DTYPE.itemsize,
                            L.PRIOR_DTYPE.itemsize, L.OP_DTYPE.itemsize, L.BAND_DTYPE.itemsize,
                            L.COLSPEC_DTYPE.itemsize)
    assert L.BAND_DTYPE.itemsize == 16 and L.COLSPEC_DTYPE.itemsize == 16
    assert L.OP_DTYPE.itemsize == 192


def _ops(*records):
    ops = np.zeros(len(records), L.OP_DTYPE)
    for i, (code, args) in enumerate(records):
        ops[i]["code"], ops[i]["n_args"] = code, len(args)
        ops[i]["a"][:len(args)] = [0 if a is None else a for a in args]
    return ops


def test_run_ops_records():
    """tpe_run_ops (the level launcher): records reach the named entry point
    with their words as its arguments; arity, code and argument errors stop
    the list at the failing record.  Only calls that need no GPU here."""
    lib = L.load()
    failed = ctypes.c_int(7)
    assert lib.tpe_run_ops(None, 0, ctypes.byref(failed)) == 0 and failed.value == -1
    # every record code's arity is its entry point's parameter count
    codes = sorted(L.OP_CODES.values()) + [L.OP_EVENT_RECORD, L.OP_STREAM_WAIT, L.OP_MEMCPY,
                                           L.OP_STREAM_SYNC]
    assert sorted(codes) == list(range(1, len(codes) + 1))
    for name in L.OP_CODES:
        assert name in L._SIGNATURES
    fit = L.OP_CODES["tpe_parzen_fit"]
    nfit = len(L._SIGNATURES["tpe_parzen_fit"][1])
    ok = (fit, [0] * nfit)  # n_seg = 0: nothing to do
    bad_n = (fit, [0, 0, 0, -1] + [0] * (nfit - 4))  # n_seg = -1
    ops = _ops(ok, ok, bad_n, ok)
    rc = lib.tpe_run_ops(ops.ctypes.data_as(ctypes.c_void_p), len(ops), ctypes.byref(failed))
    assert rc == -1 and failed.value == 2 and b"tpe_parzen_fit" in lib.tpe_last_error()
    ops = _ops(ok, (fit, [0] * (nfit - 1)))
    rc = lib.tpe_run_ops(ops.ctypes.data_as(ctypes.c_void_p), len(ops), ctypes.byref(failed))
    assert rc == -1 and failed.value == 1 and b"arguments" in lib.tpe_last_error()
    ops = _ops((99, []))
    rc = lib.tpe_run_ops(ops.ctypes.data_as(ctypes.c_void_p), 1, ctypes.byref(failed))
    assert rc == -1 and failed.value == 0 and b"unknown op" in lib.tpe_last_error()
    ops = _ops((L.OP_MEMCPY, [0, 0, 0, 77, 0]))
    rc = lib.tpe_run_ops(ops.ctypes.data_as(ctypes.c_void_p), 1, ctypes.byref(failed))
    assert rc == -1 and b"memcpy kind" in lib.tpe_last_error()


def test_graph_entry_points_check_arguments():
    """tpe_ops_capture / tpe_graph_launch / tpe_graph_destroy: argument errors
    are reported before any runtime call (no GPU needed here)."""
    lib = L.load()
    failed = ctypes.c_int(3)
    g = ctypes.c_void_p()
    ops = _ops((L.OP_STREAM_SYNC, [0]))
    p = ops.ctypes.data_as(ctypes.c_void_p)
    assert lib.tpe_ops_capture(p, 0, None, 1, ctypes.byref(g), ctypes.byref(failed)) == -1
    assert failed.value == -1 and b"tpe_ops_capture" in lib.tpe_last_error()
    assert lib.tpe_ops_capture(p, 1, None, None, ctypes.byref(g), ctypes.byref(failed)) == -1
    assert lib.tpe_ops_capture(p, 1, None, 1, None, ctypes.byref(failed)) == -1
    assert lib.tpe_graph_launch(None, None) == -1 and b"null graph" in lib.tpe_last_error()
    assert lib.tpe_graph_destroy(None) == 0


def test_argument_errors_are_reported():
    lib = L.load()
    jobs = np.zeros(1, L.JOB_DTYPE)
    jobs["n_cand"] = -5
    hp_ = jobs.ctypes.data_as(ctypes.c_void_p)
    rc = lib.tpe_score_continuous(None, hp_, 1, None, None, None, None, None, None, None, None,
                                  32, None, None, None, None, 0, None, None)
    assert rc == -1
    assert b"n_cand" in lib.tpe_last_error()
    jobs["n_cand"] = 10
    jobs["flags"] = L.F_QUANT
    rc = lib.tpe_score_continuous(None, hp_, 1, None, None, None, None, None, None, None, None,
                                  32, None, None, None, None, 0, None, None)
    assert rc == -1 and b"not an unquantized" in lib.tpe_last_error()
    rc = lib.tpe_score_continuous(None, hp_, 0, None, None, None, None, None, None, None, None,
                                  48, None, None, None, None, 0, None, None)
    assert rc == 0  # nothing to do
    nul = [None] * 11
    assert lib.tpe_parzen_fit(None, None, None, 0, 0, 0, *nul) == 0
    assert lib.tpe_parzen_fit(None, None, None, -1, 0, 0, *nul) == -1
    assert lib.tpe_parzen_fit(None, None, None, 1, 0, 0, *nul) == -1  # null pointers
    assert lib.tpe_fit_scratch_bytes(2, 100, 150) > 150 * 20
    assert lib.tpe_fit_scratch_bytes(-1, 0, 0) == -1
    jobs["flags"] = 0
    jobs["bin_lo"] = jobs["bin_hi"] = 1.0
    rc = lib.tpe_score_sorted(None, hp_, 1, *([None] * 9), 0, None, None, None)
    assert rc == -1 and b"empty bin range" in lib.tpe_last_error()
    rc = lib.tpe_score_table(None, hp_, 1, *([None] * 12), 0, None, None, None)
    assert rc == -1 and b"no cell table" in lib.tpe_last_error()
    jobs["tbl_cap"] = 64
    jobs["flags"] = L.F_INJECTED

    def fast(tile_cap=64, ptr=None, n_partial=1 << 20):
        p = [ptr] * 8
        return lib.tpe_score_table_fast(p[0], hp_, 1, *p[:7], ptr, ptr, None, None, None, ptr,
                                        n_partial, tile_cap, None, None)

    def rescore(ptr=None, n_partial=1 << 20):
        return lib.tpe_band_rescore(ptr, hp_, 1, ptr, ptr, ptr, ptr, ptr, ptr, n_partial, ptr, ptr,
                                    None)
    assert fast() == -1 and b"sampled jobs only" in lib.tpe_last_error()
    assert rescore() == -1 and b"sampled jobs only" in lib.tpe_last_error()
    jobs["flags"] = 0
    assert fast() == -1 and b"null pointer" in lib.tpe_last_error()
    assert rescore() == -1 and b"null pointer" in lib.tpe_last_error()
    eight = ctypes.c_void_p(8)
    assert fast(257, eight) == -1 and b"tile_cap" in lib.tpe_last_error()
    assert fast(-3, eight) == -1 and b"tile_cap" in lib.tpe_last_error()
    assert fast(64, eight, n_partial=0) == -1 and b"partial workspace" in lib.tpe_last_error()
    assert rescore(eight, n_partial=0) == -1 and b"partial workspace" in lib.tpe_last_error()
    ctl, work = ctypes.c_int64(0), ctypes.c_int64(0)
    jobs["n_cand"] = 1 << 22  # 512 tiles of 8192 candidates (256 threads x 32)
    nb = lib.tpe_band_bytes(hp_, 1, ctypes.byref(ctl), ctypes.byref(work))
    assert nb == 512 * 256 * L.BAND_DTYPE.itemsize and ctl.value == 512 * 16 and work.value > 0
    assert lib.tpe_band_bytes(hp_, -1, None, None) == -1
    rc = lib.tpe_table_build(None, hp_, 1, None, None, None, None, 8, *([None] * 8))
    assert rc == -1 and b"null pointer" in lib.tpe_last_error()
    assert lib.tpe_table_scratch_bytes(3, 1000) > 0 and lib.tpe_table_scratch_bytes(-1, 5) == -1
    jobs["flags"] = L.F_QUANT
    rc = lib.tpe_table_build(None, hp_, 1, None, None, None, None, 8, *([None] * 8))
    assert rc == -1 and b"not an unquantized" in lib.tpe_last_error()
    assert lib.tpe_best_combine(None, 0, 1, None, None) == -1
    assert lib.tpe_maxloc_allreduce(None, None, None, 3, None, None) == -1
    assert b"tpe_maxloc_allreduce" in lib.tpe_last_error()
    assert lib.tpe_maxloc_allreduce(None, None, None, 0, None, None) == 0
    pri = np.zeros(1, L.PRIOR_DTYPE)
    pri["kind"] = 9
    pp = pri.ctypes.data_as(ctypes.c_void_p)
    assert lib.tpe_prior_sample(None, pp, 1, None, 4, 0, None, None) == -1
    assert b"kind 9" in lib.tpe_last_error()
    pri["kind"], pri["a"], pri["b"] = L.PRIOR_RANDINT, 3.0, 3.0
    assert lib.tpe_prior_sample(None, pp, 1, None, 4, 0, None, None) == -1
    assert b"high <= low" in lib.tpe_last_error()
    pri["kind"] = L.PRIOR_CATEGORICAL
    assert lib.tpe_prior_sample(None, pp, 1, None, 4, 0, None, None) == -1
    assert lib.tpe_prior_sample(None, None, 0, None, 4, 0, None, None) == 0
    g = np.zeros(1, L.GATHER_DTYPE)
    g["to_int"] = 1
    gp = g.ctypes.data_as(ctypes.c_void_p)
    one = ctypes.c_void_p(1)
    rc = lib.tpe_gather_obs(one, one, 10, None, 0, None, one, gp, 1, one, None, None, None)
    assert rc == -1 and b"output pool" in lib.tpe_last_error()
    assert lib.tpe_gather_obs(None, None, 10, None, 0, None, None, None, 0, None, None, None,
                              None) == 0
    h = np.zeros(1, L.HISTORY_DTYPE)
    h["vals"] = h["active"] = 1
    h["ld"], h["n_cols"], h["n_rows"], h["rows_off"] = 10, 3, 10, -1
    hp2 = h.ctypes.data_as(ctypes.c_void_p)
    g["hist"], g["col"], g["to_int"] = 0, 3, 0
    rc = lib.tpe_gather_obs_multi(one, hp2, 1, one, one, gp, 1, one, None, None, None)
    assert rc == -1 and b"column" in lib.tpe_last_error()
    g["col"], g["hist"] = 2, 1
    rc = lib.tpe_gather_obs_multi(one, hp2, 1, one, one, gp, 1, one, None, None, None)
    assert rc == -1 and b"history" in lib.tpe_last_error()
    h["n_rows"] = 11  # identity rows beyond the leading dimension
    g["hist"] = 0
    rc = lib.tpe_gather_obs_multi(one, hp2, 1, one, one, gp, 1, one, None, None, None)
    assert rc == -1 and b"history 0" in lib.tpe_last_error()
    assert lib.tpe_gather_obs_multi(None, None, 0, None, None, None, 0, None, None, None,
                                    None) == 0
    with pytest.raises(L.TpeHipError):
        L.check(-1, "probe")


def test_lattice_suggest_argument_errors():
    """tpe_lattice_suggest (the prefix-first lattice argmax) validates its
    jobs, pointers, prefix and workspace before any launch."""
    lib = L.load()
    jobs = np.zeros(1, L.JOB_DTYPE)
    jobs["n_cand"] = 1 << 20
    hp_ = jobs.ctypes.data_as(ctypes.c_void_p)
    one = ctypes.c_void_p(8)  # a non-null stand-in: validation fails before any launch
    ptrs = [one] * 6

    def call(prefix, n_partial, need=one, n_jobs=1):
        return lib.tpe_lattice_suggest(one, hp_, n_jobs, *ptrs, prefix, one, n_partial, need, one,
                                       one, None, None, None)
    assert call(1 << 16, 1 << 10, n_jobs=0) == 0  # nothing to do
    assert call(1 << 16, 1 << 10) == -1
    assert b"not a sampled quantized job" in lib.tpe_last_error()
    jobs["flags"] = L.F_QUANT
    jobs["q"] = 1.0
    jobs["lat_n"] = 101
    assert call(1 << 16, 1 << 10, need=None) == -1
    assert b"null pointer" in lib.tpe_last_error()
    assert call(1000, 1 << 10) == -1
    assert b"prefix" in lib.tpe_last_error()
    assert call(1 << 16, 100) == -1
    assert b"partial workspace" in lib.tpe_last_error()
    jobs["flags"] = L.F_QUANT | L.F_INJECTED
    assert call(1 << 16, 1 << 10) == -1
    assert b"not a sampled quantized job" in lib.tpe_last_error()


def test_categorical_suggest_argument_errors():
    """tpe_categorical_suggest (the prefix-first categorical argmax)
    validates its jobs, pointers, prefix and workspace before any launch."""
    lib = L.load()
    jobs = np.zeros(1, L.JOB_DTYPE)
    jobs["n_cand"] = 1 << 20
    jobs["lat_n"] = 8
    hp_ = jobs.ctypes.data_as(ctypes.c_void_p)
    one = ctypes.c_void_p(8)  # a non-null stand-in: validation fails before any launch
    ptrs = [one] * 3

    def call(prefix, n_partial, need=one, n_jobs=1):
        return lib.tpe_categorical_suggest(one, hp_, n_jobs, *ptrs, prefix, one, n_partial,
                                           need, one, None)
    assert call(1 << 16, 1 << 10, n_jobs=0) == 0  # nothing to do
    assert call(1 << 16, 1 << 10) == -1  # family 0: not categorical
    assert b"not a sampled categorical job" in lib.tpe_last_error()
    jobs["family"] = L.CAT
    assert call(1 << 16, 1 << 10, need=None) == -1
    assert b"null pointer" in lib.tpe_last_error()
    assert call(1000, 1 << 10) == -1
    assert b"prefix" in lib.tpe_last_error()
    assert call(1 << 16, 10) == -1
    assert b"partial workspace" in lib.tpe_last_error()
    jobs["flags"] = L.F_INJECTED
    assert call(1 << 16, 1 << 10) == -1
    assert b"not a sampled categorical job" in lib.tpe_last_error()


def test_issue_threads_setting():
    """tpe_set_issue_threads: 1 or 2 (the previous setting is returned), any
    other count is an argument error; records still stop at the first failing
    one whatever the setting (no GPU here: the caller issues them alone)."""
    lib = L.load()
    prev = lib.tpe_set_issue_threads(2)
    try:
        assert prev in (1, 2)
        assert lib.tpe_set_issue_threads(2) == 2
        for bad in (0, 3, -1):
            assert lib.tpe_set_issue_threads(bad) == -1
            assert b"tpe_set_issue_threads" in lib.tpe_last_error()
        fit = L.OP_CODES["tpe_parzen_fit"]
        nfit = len(L._SIGNATURES["tpe_parzen_fit"][1])
        rec = lambda n_seg, stream: (fit, [0, 0, 0, n_seg] + [0] * (nfit - 5) + [stream])
        ops = _ops(rec(0, 0), rec(0, 1234), rec(-1, 1234), rec(-1, 0))
        failed = ctypes.c_int(7)
        rc = lib.tpe_run_ops(ops.ctypes.data_as(ctypes.c_void_p), len(ops), ctypes.byref(failed))
        assert rc == -1 and failed.value == 2 and b"tpe_parzen_fit" in lib.tpe_last_error()
    finally:
        lib.tpe_set_issue_threads(prev)
