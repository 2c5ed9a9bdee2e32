"""Band sizes of the C3 table labels (diagnostic): per job the survivors and
listed cells the select kernel leaves (library built with
TPE_DIAG_BAND_KEEP, tools/probes/diag_variants.sh), and the scorer's raw entries.

    TPE_DIAG=1 TPE_NATIVE_LAUNCH=0 HYPEROPT_AMD_LIB=tools/_variants/lib_BAND_KEEP.so python tools/probes/band_probe.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import _lib as L  # noqa: E402
from hyperopt_amd.engine import Engine  # noqa: E402

torch.cuda.set_device(0)
hip = ctypes.CDLL("libamdhip64.so.7")
lib = L.load()
space = [s for s in bench.c3_space() if s[1] in ("uniform", "loguniform", "normal")]
vals, losses = bench.c3_history(bench.c3_space())
sp = bench.split(vals, losses)
seen = {}
orig_fast, orig_res = lib.tpe_score_table_fast, lib.tpe_band_rescore


def ctl_of(ptr, nj):
    torch.cuda.synchronize()
    h = np.zeros(4 * nj, np.uint32)
    assert hip.hipMemcpy(h.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr),
                         ctypes.c_size_t(h.nbytes), 2) == 0
    return h.reshape(nj, 4)


def fast(*a):
    rc = orig_fast(*a)
    seen["entries"] = ctl_of(a[12], a[2])[:, 1].copy()
    return rc


def rescore(*a):
    rc = orig_res(*a)
    c = ctl_of(a[8], a[2])
    seen["surv"], seen["cells"] = c[:, 2].copy(), c[:, 3].copy()
    zero = np.zeros(4 * a[2], np.uint32)
    hip.hipMemcpy(ctypes.c_void_p(a[8]), zero.ctypes.data_as(ctypes.c_void_p),
                  ctypes.c_size_t(zero.nbytes), 1)
    return rc


lib.tpe_score_table_fast, lib.tpe_band_rescore = fast, rescore
eng = Engine()
for step in range(3):
    eng.run(bench.make_works(space, sp, step, 1 << 22, 0), precision=32)
    for j, (lab, kind, _) in enumerate(space):
        print(step, lab, kind, "entries", seen["entries"][j], "survivors", seen["surv"][j],
              "cells", seen["cells"][j])
