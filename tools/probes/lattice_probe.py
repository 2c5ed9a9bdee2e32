"""Lattice sampler cost in isolation (diagnostic): one quantized label, 2^24
candidates, the whole stream drawn (TPE_LAT_PREFIX=0 via the engine's
lat_prefix) -- a narrow quniform lattice vs a wide qlognormal one.

    python tools/probes/lattice_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hyperopt_amd.engine import Engine, LabelWork  # noqa: E402


def run(kind, args, obs_b, n_above, vals_above, label):
    eng = Engine()
    eng.lat_prefix = 0
    w = LabelWork(label, kind, args, obs_b, vals_above, n_cand=1 << 24, key=12345)
    for _ in range(3):
        eng.run([w], precision=32)
    torch.cuda.synchronize()
    ts = []
    for k in range(10):
        t0 = time.perf_counter()
        eng.run([w], precision=32)
        ts.append(time.perf_counter() - t0)
    timers = {}
    eng.run([w], precision=32, timers=timers)
    torch.cuda.synchronize()
    g = {a: round(float(np.mean([e0.elapsed_time(e1) for e0, e1 in v])), 4) for a, v in timers.items()}
    print(label, kind, "p50 ms %.3f" % (np.median(ts) * 1e3), g, flush=True)


def main():
    rng = np.random.RandomState(0)
    a = np.round(rng.uniform(1, 12, 20000))
    run("quniform", (1.0, 12.0, 1.0), a[:25], None, a[25:], "narrow")
    ln = np.round(np.exp(rng.normal(0, 1, 17000)) / 0.5) * 0.5
    run("qlognormal", (0.0, 1.0, 0.5), ln[:25], None, ln[25:], "wide")
    lnn = np.round(np.exp(rng.normal(0, 0.3, 17000)) / 0.5) * 0.5
    run("qlognormal", (0.0, 0.3, 0.5), lnn[:25], None, lnn[25:], "lognarrow")


if __name__ == "__main__":
    main()
