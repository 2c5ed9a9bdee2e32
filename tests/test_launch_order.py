"""Host-side launch order of one C3 level (Engine._launch_level and its
stages), checked without a GPU: the engine runs against the stand-ins of
tools/host_cpu_profile.py (CPU tensors for the workspace, a HIP runtime
whose calls return success) with a library that records every launch entry
point it is asked for, and on which stream.  What is pinned is the issue
order DESIGN.md section 5.1 describes -- the stream work the GPU tests run."""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import host_cpu_profile as H  # noqa: E402
from hyperopt_amd import _lib as L  # noqa: E402
from hyperopt_amd import dist as hdist  # noqa: E402
from hyperopt_amd import engine as E  # noqa: E402

SIDE = 7  # the side stream's handle in the stand-in runtime


class _SideStream(object):
    cuda_stream = SIDE

    def __init__(self, *a, **k):
        pass


class _Recorder(object):
    """Launch entry points append (name, stream) and return 0; size queries go
    to the real library."""

    def __init__(self, lib):
        self._lib, self.calls = lib, []

    def __getattr__(self, name):
        if name in L.OP_CODES or name == "tpe_history_append":
            def call(*args):
                s = args[-1]
                s = s.value if isinstance(s, ctypes.c_void_p) else s
                self.calls.append((name, "side" if s == SIDE else "main"))
                return 0
            return call
        return getattr(self._lib, name)


@pytest.fixture(scope="module")
def c3():
    try:
        lib = L.load()
    except Exception as e:  # pragma: no cover - the build check covers this
        pytest.skip("libtpe_hip.so not loadable: %s" % e)
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    mat = bench.c3_matrix(space, vals)
    return lib, space, mat, losses


def _level(c3, side_stream="1", cat_issue="post"):
    lib, space, mat, losses = c3
    eng = H.make_engine()
    eng.torch.cuda.Stream = _SideStream
    eng.native = False  # every call eager: the recorder sees each launch
    eng.side_stream, eng.cat_issue = side_stream, cat_issue
    rec = _Recorder(lib)
    eng.lib = rec
    hist = E.DeviceHistory(eng, len(space), cap=bench.T_HIST)
    hist.append(mat)
    units = hdist.plan_units([k for _, k, _ in space], bench.N_CAND, 1)[0]
    rb = bench.below_rows(losses)
    isb = np.zeros(losses.size, np.uint8)
    isb[rb] = 1
    works = bench.history_batch(space, mat, hist, rb, 0, bench.N_CAND, 0, units, bench.N_CAND)
    del rec.calls[:]
    eng.run(works, precision=32, history=hist, is_below=isb, defer=True)
    return rec.calls


def _first(calls, name):
    return [n for n, _ in calls].index(name)


def test_c3_level_issue_order(c3):
    calls = _level(c3)
    names = [n for n, _ in calls]
    # sorted fit from the history, categorical counts from the history: no gather
    assert "tpe_gather_obs" not in names
    for n in ("tpe_fit_sorted", "tpe_cat_posterior_hist", "tpe_table_build",
              "tpe_score_table_fast", "tpe_band_rescore"):
        assert names.count(n) == 1, (n, names)
    fit, cat = _first(calls, "tpe_fit_sorted"), _first(calls, "tpe_cat_posterior_hist")
    build = _first(calls, "tpe_table_build")
    score, band = _first(calls, "tpe_score_table_fast"), _first(calls, "tpe_band_rescore")
    # main stream: fit, then the early table build, the scorer, the band
    assert fit < build < score < band
    # categorical posterior and scoring issued right after the fit ("post"),
    # before the table build; the quantized side groups after the build
    cat_scores = [i for i, n in enumerate(names) if n in ("tpe_categorical_suggest",
                                                          "tpe_score_categorical")]
    assert cat_scores and fit < cat < min(cat_scores) and max(cat_scores) < build
    lat = [i for i, n in enumerate(names) if n.startswith("tpe_lattice")]
    assert lat and build < min(lat) and max(lat) < score
    # stream placement
    side = {n for n, s in calls if s == "side"}
    main = {n for n, s in calls if s == "main"}
    assert {"tpe_cat_posterior_hist", "tpe_lattice_suggest"} & side
    assert not side & {"tpe_fit_sorted", "tpe_table_build", "tpe_score_table_fast",
                       "tpe_band_rescore"}
    assert {"tpe_fit_sorted", "tpe_table_build", "tpe_score_table_fast",
            "tpe_band_rescore"} <= main
    assert not {n for n in main if n.startswith(("tpe_lattice", "tpe_cat"))}


def test_c3_level_issue_order_variants(c3):
    base = sorted(_level(c3))
    # the categorical issue order moves launches, never adds or drops one
    for mode in ("pre", "late"):
        calls = _level(c3, cat_issue=mode)
        assert sorted(calls) == base, mode
        names = [n for n, _ in calls]
        cat_s = max(i for i, n in enumerate(names) if n.startswith("tpe_categorical") or
                    n == "tpe_score_categorical")
        if mode == "pre":
            assert cat_s < _first(calls, "tpe_fit_sorted")
        else:
            assert _first(calls, "tpe_table_build") < cat_s
    # no side stream: the same launches, all on the main stream
    one = _level(c3, side_stream="0")
    assert sorted(n for n, _ in one) == sorted(n for n, _ in base)
    assert {s for _, s in one} == {"main"}
