"""cProfile of one suggest_many call on C4's per-GPU share (diagnostic; GPU box).
    python tools/profile_c4.py [studies]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperopt_amd import tpe  # noqa: E402
from hyperopt_amd.base import Domain  # noqa: E402
from tools import scale_configs as S  # noqa: E402

torch.cuda.set_device(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
T = 2000
doms = [Domain(lambda p: 0.0, S.c4_space(s)) for s in range(n)]
trs = [S.flat_trials(d, T, s) for s, d in enumerate(doms)]
import gc  # noqa: E402
gc.collect()
gc.freeze()  # (the documents are long-lived: tools/scale_configs.py c4)


def call(k):
    reqs = [tpe.SuggestRequest([T + k], d, t, s + k, n_EI_candidates=1 << 12)
            for s, (d, t) in enumerate(zip(doms, trs))]
    return tpe.suggest_many(reqs)


for k in range(2):
    call(k)
torch.cuda.synchronize()
t0 = time.perf_counter()
call(2)
print("suggest_many(%d studies): %.1f ms" % (n, (time.perf_counter() - t0) * 1e3))
pr = cProfile.Profile()
pr.enable()
call(3)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats(40)
