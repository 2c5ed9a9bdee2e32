"""C5 strong-scaling projection on one GPU (diagnostic; run on the GPU box).

C5 (BASELINE.json configs[4]): the 3-level nested hp.choice space
(tests/golden/spaces.py:nested), a 100k-trial prior history, 2^24 candidates
per live label.  Its levels hold fewer labels than ranks, so dist.plan_units
deals candidate shards.  For every N and rank r, tpe.suggest runs with
hdist.world() = (r, N) and the winners' all-gather replaced by the N=1 run's
values (the walk -- which branch is live -- is the same on every rank and N),
so each rank's time is its own share of every level: host split + plan +
launches + readback.  Projection = t(N=1) / max_r t_r(N), collective excluded
(its cost: DESIGN.md section 6).

    python tools/c5_share.py [2 4 8]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from hyperopt_amd import dist as hdist  # noqa: E402
from hyperopt_amd import hp, tpe  # noqa: E402
from hyperopt_amd.base import Domain  # noqa: E402
from tests.golden import spaces  # noqa: E402
from tools.scale_configs import prior_trials  # noqa: E402

T, N_EI, SEED, CALLS, WARM = 100_000, 1 << 24, 7, 9, 3


def main(worlds):
    import torch
    torch.cuda.set_device(0)
    domain = Domain(lambda p: 0.0, spaces.nested(hp))
    t0 = time.perf_counter()
    trials = prior_trials(domain, T, 0)
    print(json.dumps({"history_build_s": round(time.perf_counter() - t0, 1)}), flush=True)
    real_world, real_gather, real_decode = hdist.world, hdist.gather_best, tpe._decode
    walk = []  # the N=1 run's (label, value) in level order

    def recording_decode(spec, v):
        walk.append(float(v))
        return real_decode(spec, v)

    def call():
        t0 = time.perf_counter()
        tpe.suggest([T], domain, trials, SEED, n_EI_candidates=N_EI, verbose=False)
        return time.perf_counter() - t0

    tpe._decode = recording_decode
    try:
        call()
    finally:
        tpe._decode = real_decode
    out = {}
    base_units = None
    try:
        for N in [1] + worlds:
            per_rank = []
            for r in range(N):
                pos = [0]

                def fake_gather(n_labels, local, group=None):
                    vals = walk[pos[0]:pos[0] + n_labels]
                    pos[0] += n_labels
                    return [(0.0, 0, v, 0) for v in vals]

                hdist.world = (lambda r=r, N=N: (r, N))
                hdist.gather_best = fake_gather
                ts = []
                for k in range(WARM + CALLS):
                    pos[0] = 0
                    ts.append(call())
                per_rank.append(float(np.median(ts[WARM:])) * 1e3)
                if N == 1:
                    base_units = len(walk)
            out[N] = max(per_rank)
            print(json.dumps({"N": N, "max_rank_ms": round(out[N], 4),
                              "per_rank_ms": [round(x, 4) for x in per_rank]}), flush=True)
    finally:
        hdist.world, hdist.gather_best = real_world, real_gather
    print(json.dumps({"config": "C5", "history": T, "n_EI_candidates": N_EI,
                      "live_label_values": base_units, "seed": SEED}), flush=True)
    for N in worlds:
        print(json.dumps({"N": N, "projected_speedup_no_collective": round(out[1] / out[N], 2)}),
              flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [2, 4, 8])
