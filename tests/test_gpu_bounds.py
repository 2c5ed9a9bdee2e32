"""The hardware facts the fp32 error bounds of the table path assume
(DESIGN.md 3.1), measured exhaustively on the device: v_exp_f32's relative
error over every fp32 input of [-126, 12] (the build's terms: mix_eps takes
2^-22) and v_log_f32's error over every positive normal fp32 input, absolute
or relative to |log2 p| (the two-polynomial fallback's kEtaLog2 = 2^-22)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_transcendentals_within_the_bounds_assumed():
    import torch
    from hyperopt_amd import _lib as L
    lib = L.load()
    out = torch.zeros(2, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream()
    L.check(lib.tpe_check_transcendentals(out.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
            "tpe_check_transcendentals")
    e_exp, e_log = out.cpu().numpy().tolist()
    print("v_exp_f32 max rel err %.3e, v_log_f32 max err %.3e" % (e_exp, e_log))
    assert 0.0 < e_exp <= 2.0 ** -22, e_exp
    assert 0.0 < e_log <= 2.0 ** -22, e_log
