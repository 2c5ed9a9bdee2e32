"""ctypes binding of the HIP C-ABI library ``libtpe_hip.so`` (include/tpe_hip.h).

The struct mirrors below are numpy dtypes with C alignment; their sizes are
checked against the library at load time.  The library is REQUIRED: there is
no CPU fallback anywhere on the product path, and loading fails loudly if the
library has not been built (``make`` or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HYPEROPT_AMD_LIB", os.path.join(HERE, "libtpe_hip.so"))

# enums (tpe_hip.h)
GMM1, LGMM1, CAT = 0, 1, 2
OBS_IDENTITY, OBS_LOG = 0, 1
F_LOW, F_HIGH, F_QUANT, F_INJECTED, F_DRAW32, F_LATTICE_READY = 1, 2, 4, 8, 16, 32
ABI_VERSION = 22

SEG_DTYPE = np.dtype([
    ("obs_off", "<i8"), ("comp_off", "<i8"), ("n_obs", "<i4"), ("lf", "<i4"),
    ("transform", "<i4"), ("family", "<i4"), ("floor", "<f8"), ("prior_weight", "<f8"),
    ("prior_mu", "<f8"), ("prior_sigma", "<f8"), ("low", "<f8"), ("high", "<f8"),
    ("bounded", "<i4"), ("prior_pos", "<i4"), ("p_accept", "<f8"), ("cmax", "<f8"),
    ("center", "<f8"), ("lglob", "<f8"), ("n_wide", "<i4"), ("given", "<i4")], align=True)
CAT_SEG_DTYPE = np.dtype([
    ("obs_off", "<i8"), ("p_off", "<i8"), ("n_obs", "<i4"), ("n_cat", "<i4"),
    ("lf", "<i4"), ("mode", "<i4"), ("prior_weight", "<f8"), ("prior_p_off", "<i8")],
    align=True)
JOB_DTYPE = np.dtype([
    ("family", "<i4"), ("flags", "<i4"), ("below", "<i4"), ("above", "<i4"),
    ("low", "<f8"), ("high", "<f8"), ("q", "<f8"), ("n_cand", "<i8"), ("cand_base", "<i8"),
    ("cand_off", "<i8"), ("key", "<u8"), ("lat_off", "<i8"), ("lat_kmin", "<i8"),
    ("lat_n", "<i8"), ("out_off", "<i8"), ("bin_lo", "<f8"), ("bin_hi", "<f8"),
    ("sort_off", "<i8"), ("cnt_off", "<i8"), ("tbl_off", "<i8"), ("tbl_cap", "<i8")],
    align=True)
TABLE_DTYPE = np.dtype([
    ("lo", "<f8"), ("hi", "<f8"), ("h_below", "<f8"), ("h_above", "<f8"), ("origin", "<f8"),
    ("h", "<f8"), ("inv_h", "<f4"), ("inv_w", "<f4"), ("nb", "<i4"), ("n_wide_below", "<i4"),
    ("n_wide_above", "<i4"), ("slope", "<f4"), ("eps_cubic", "<f4"), ("eps_mix", "<f4"),
    ("build_items", "<i4"), ("build_ab", "<f4"), ("T_below", "<f8"), ("T_above", "<f8")],
    align=True)
GATHER_DTYPE = np.dtype([
    ("col", "<i4"), ("below", "<i4"), ("dst_off", "<i8"), ("offset", "<i8"), ("count", "<i8"),
    ("to_int", "<i4"), ("hist", "<i4")], align=True)
HISTORY_DTYPE = np.dtype([
    ("vals", "<u8"), ("active", "<u8"), ("ld", "<i8"), ("n_cols", "<i8"), ("n_rows", "<i8"),
    ("rows_off", "<i8"), ("isb_off", "<i8")], align=True)
BEST_DTYPE = np.dtype([("score", "<f8"), ("index", "<i8"), ("value", "<f8"),
                       ("n_scored", "<i8")], align=True)
BAND_DTYPE = np.dtype([("index", "<i8"), ("y", "<f4"), ("hi", "<f4")], align=True)
COLSPEC_DTYPE = np.dtype([("col", "<i4"), ("transform", "<i4"), ("floor", "<f8")], align=True)
PRIOR_DTYPE = np.dtype([("kind", "<i4"), ("n_cat", "<i4"), ("a", "<f8"), ("b", "<f8"),
                        ("q", "<f8"), ("p_off", "<i8"), ("key", "<u8")], align=True)
OP_ARGS = 23
OP_DTYPE = np.dtype([("code", "<i4"), ("n_args", "<i4"), ("a", "<i8", (OP_ARGS,))], align=True)
# tpe_run_ops record codes (tpe_hip.h TPE_OP_*): entry point -> code
OP_CODES = {name: i + 1 for i, name in enumerate((
    "tpe_gather_obs", "tpe_gather_obs_multi", "tpe_parzen_fit", "tpe_cat_posterior",
    "tpe_table_build", "tpe_score_table", "tpe_score_table_fast", "tpe_score_pruned64",
    "tpe_score_continuous", "tpe_sort_candidates", "tpe_score_sorted", "tpe_lattice_sample",
    "tpe_lattice_compact", "tpe_score_quantized", "tpe_score_categorical", "tpe_sample"))}
OP_EVENT_RECORD, OP_STREAM_WAIT, OP_MEMCPY, OP_STREAM_SYNC = range(len(OP_CODES) + 1,
                                                                  len(OP_CODES) + 5)
OP_CODES["tpe_best_scatter"] = OP_STREAM_SYNC + 1
OP_CODES["tpe_maxloc_allreduce"] = OP_STREAM_SYNC + 2
OP_CODES["tpe_lattice_suggest"] = OP_STREAM_SYNC + 3
OP_CODES["tpe_band_rescore"] = OP_STREAM_SYNC + 4
OP_CODES["tpe_fit_sorted"] = OP_STREAM_SYNC + 5
OP_CODES["tpe_history_order"] = OP_STREAM_SYNC + 6
OP_CODES["tpe_categorical_suggest"] = OP_STREAM_SYNC + 7
OP_CODES["tpe_cat_posterior_hist"] = OP_STREAM_SYNC + 8
OP_MAXLOC_ALLREDUCE = OP_CODES["tpe_maxloc_allreduce"]
PRIOR_UNIFORM, PRIOR_LOGUNIFORM, PRIOR_NORMAL, PRIOR_LOGNORMAL, PRIOR_RANDINT, \
    PRIOR_CATEGORICAL = range(6)


class TpeHipError(RuntimeError):
    """A C-ABI call returned an error status."""


_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64

_SIGNATURES = {
    "tpe_fit_scratch_bytes": (_I64, [_I, _I, _I64]),
    "tpe_parzen_fit": (_I, [_P, _P, _P, _I, _I, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                            _P]),
    "tpe_sort_layout": (_I64, [_I64, _P]),
    "tpe_sort_candidates": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tpe_score_sorted": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _P,
                              _P]),
    "tpe_cat_posterior": (_I, [_P, _P, _I, _I, _P, _P, _P, _P]),
    "tpe_history_append": (_I, [_P, _I, _I64, _P, _P, _I64, _I64, _P]),
    "tpe_cat_posterior_hist": (_I, [_P, _P, _I64, _P, _I64, _P, _P, _P, _I, _I, _P, _P, _P, _P,
                                    _I64, _P, _P]),
    "tpe_cat_hist_scratch_bytes": (_I64, [_I, _I, _I64]),
    "tpe_gather_obs": (_I, [_P, _P, _I64, _P, _I64, _P, _P, _P, _I, _P, _P, _P, _P]),
    "tpe_gather_obs_multi": (_I, [_P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P]),
    "tpe_table_partials": (_I64, [_P, _I]),
    "tpe_table_scratch_bytes": (_I64, [_I, _I]),
    "tpe_table_build": (_I, [_P, _P, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tpe_score_table": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64,
                             _P, _P, _P]),
    "tpe_score_table_fast": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                  _P, _I64, _I, _P, _P]),
    "tpe_band_rescore": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _P]),
    "tpe_band_bytes": (_I64, [_P, _I, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "tpe_categorical_suggest": (_I, [_P, _P, _I, _P, _P, _P, _I64, _P, _I64, _P, _P, _P]),
    "tpe_history_order_scratch_bytes": (_I64, [_I, _I64]),
    "tpe_history_order": (_I, [_P, _I64, _P, _P, _I, _I64, _I64, _P, _P, _P]),
    "tpe_fit_sorted_scratch_bytes": (_I64, [_I, _I64]),
    "tpe_fit_sorted": (_I, [_P, _P, _I64, _P, _I64, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P,
                            _P, _P, _P]),
    "tpe_pruned64_partials": (_I64, [_P, _I]),
    "tpe_score_pruned64": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P,
                                _P, _P, _P, _I64, _P, _P]),
    "tpe_score_partials": (_I64, [_P, _I]),
    "tpe_score_continuous": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P,
                                  _P, _I64, _P, _P]),
    "tpe_lattice_sample": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "tpe_lattice_suggest": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _I64, _P, _I64, _P, _P, _P,
                                 _P, _P, _P]),
    "tpe_lattice_compact": (_I, [_P, _P, _I, _P, _P, _P, _P, _P]),
    "tpe_quantized_partials": (_I64, [_P, _I, _I64]),
    "tpe_score_quantized": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _P, _I64,
                                 _P, _P, _P, _P, _P]),
    "tpe_categorical_partials": (_I64, [_P, _I]),
    "tpe_score_categorical": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _P]),
    "tpe_sample": (_I, [_P, _P, _I, _P, _P, _P, _P, _I, _P, _P]),
    "tpe_best_combine": (_I, [_P, _I, _I, _P, _P]),
    "tpe_maxloc_allreduce": (_I, [_P, _P, _P, _I, _P, _P]),
    "tpe_best_scatter": (_I, [_P, _P, _I, _P, _I, _P]),
    "tpe_prior_sample": (_I, [_P, _P, _I, _P, _I64, _I64, _P, _P]),
    "tpe_run_ops": (_I, [_P, _I, ctypes.POINTER(_I)]),
    "tpe_set_issue_threads": (_I, [_I]),
    "tpe_ops_capture": (_I, [_P, _I, _P, _P, ctypes.POINTER(_P), ctypes.POINTER(_I)]),
    "tpe_graph_launch": (_I, [_P, _P]),
    "tpe_graph_destroy": (_I, [_P]),
    "tpe_check_transcendentals": (_I, [_P, _P]),
    "tpe_mixture_scratch_bytes": (_I64, [_I, _I]),
    "tpe_mixture_prepare": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tpe_smallest_rows": (_I64, [_P, _I64, _I64, _P]),
    "tpe_split_inputs": (_I64, [_P, _I64, _I64, _P, _I64, _P, _P, _P, _P, _P]),
    "tpe_last_error": (ctypes.c_char_p, []),
    "tpe_abi_version": (_I, []),
    "tpe_struct_sizes": (_I, [_P, _I]),
}

_lib = None
_hip = None

H2D, D2H = 1, 2  # hipMemcpyKind
EVENT_NO_TIMING = 0x2  # hipEventDisableTiming
EVENT_NO_SYSTEM_FENCE = 0x20000000  # hipEventDisableSystemFence (device-scope release)


def hip():
    """The HIP runtime the library is bound to (torch's libamdhip64.so.7),
    for the few stream-ordered runtime calls the engine makes per level
    (async copies, events, stream waits) without torch's per-call overhead."""
    global _hip
    if _hip is None:
        load()
        h = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
        for name, args in (("hipMemcpyAsync", [_P, _P, ctypes.c_size_t, _I, _P]),
                           ("hipEventCreateWithFlags", [ctypes.POINTER(_P), ctypes.c_uint]),
                           ("hipEventRecord", [_P, _P]),
                           ("hipStreamWaitEvent", [_P, _P, ctypes.c_uint]),
                           ("hipEventSynchronize", [_P]),
                           ("hipStreamSynchronize", [_P]),
                           ("hipGetLastError", []),
                           ("hipEventElapsedTime", [ctypes.POINTER(ctypes.c_float), _P, _P]),
                           ("hipEventDestroy", [_P])):
            fn = getattr(h, name)
            fn.restype = _I
            fn.argtypes = args
        _hip = h
    return _hip


def hip_check(rc, what):
    if rc != 0:
        raise TpeHipError("%s: hipError %d" % (what, rc))


def load():
    """Load (once) and return the ctypes library; raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "hyperopt_amd: HIP library %s is missing; build it with `make` "
            "(or __graft_entry__.build()). There is no CPU fallback." % LIB_PATH)
    # torch must be loaded first so this library binds torch's HIP runtime
    # (same SONAME libamdhip64.so.7) instead of a second copy.
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    sizes = (ctypes.c_int32 * 11)()
    lib.tpe_struct_sizes(ctypes.cast(sizes, _P), 11)
    want = (SEG_DTYPE.itemsize, CAT_SEG_DTYPE.itemsize, JOB_DTYPE.itemsize, BEST_DTYPE.itemsize,
            TABLE_DTYPE.itemsize, GATHER_DTYPE.itemsize, HISTORY_DTYPE.itemsize,
            PRIOR_DTYPE.itemsize, OP_DTYPE.itemsize, BAND_DTYPE.itemsize,
            COLSPEC_DTYPE.itemsize)
    if lib.tpe_abi_version() != ABI_VERSION:
        raise ImportError("hyperopt_amd: libtpe_hip.so ABI %d, expected %d (rebuild with make)"
                          % (lib.tpe_abi_version(), ABI_VERSION))
    if tuple(sizes) != want:
        raise ImportError("hyperopt_amd: ABI struct size mismatch %s vs %s" % (tuple(sizes), want))
    _lib = lib
    return lib


def check(status, what):
    if status != 0:
        msg = load().tpe_last_error().decode(errors="replace")
        raise TpeHipError("%s failed (%d): %s" % (what, status, msg))
