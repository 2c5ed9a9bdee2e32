"""Drop-in C3 suggest (bench.dropin_suggest_p50's loop) on a timeline
(diagnostic; run under rocprofv3 --kernel-trace on the GPU box):

    rocprofv3 --kernel-trace -d gpurun_out/dt -o run -- python3 tools/r04_dropin_timeline.py
    python3 tools/r04_dropin_timeline.py --db gpurun_out/dt

The first form runs 25 calls and prints each call's wall time and host
phase marks (perf_counter around tpe.suggest's steps, Engine.host_marks);
the second splits the kernel trace into calls (GPU idle > 150 us) and prints
the last calls' kernels with start offsets, durations and idle gaps.
"""
import glob
import json
import os
import re
import sqlite3
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run():
    import numpy as np
    import bench
    from hyperopt_amd import tpe
    from hyperopt_amd.base import JOB_STATE_DONE
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    domain, trials = bench.c3_trials(space, vals, losses)
    rng = np.random.RandomState(9)
    eng = tpe.engine()
    out = []
    marks_py = []

    def wrap(name):
        f = getattr(tpe, name)

        def g(*a, **kw):
            marks_py.append((name + ">", time.perf_counter()))
            r = f(*a, **kw)
            marks_py.append((name + "<", time.perf_counter()))
            return r
        setattr(tpe, name, g)
    for name in ("collect_history", "split_masks", "LevelInputs", "_level_batch"):
        wrap(name)
    for k in range(25):
        tid = losses.size + k
        eng.host_marks = []
        del marks_py[:]
        t0 = time.perf_counter()
        docs = tpe.suggest([tid], domain, trials, k, n_EI_candidates=bench.N_CAND, verbose=False)
        t1 = time.perf_counter()
        marks = [(n, round((t - t0) * 1e6, 1))
                 for n, t in sorted(marks_py + list(eng.host_marks), key=lambda m: m[1])]
        docs[0]["state"] = JOB_STATE_DONE
        docs[0]["result"] = {"status": "ok", "loss": float(rng.normal())}
        trials.insert_trial_docs(docs)
        trials.refresh()
        out.append({"call": k, "wall_us": round((t1 - t0) * 1e6, 1), "marks": marks})
        time.sleep(0.002)  # a gap on the GPU timeline between calls
    eng.host_marks = None
    for o in out[-5:]:
        print(json.dumps(o), flush=True)
    print(json.dumps({"wall_p50_us": float(np.median([o["wall_us"] for o in out[5:]]))}))


def short(name):
    m = re.search(r"(k_\w+|__amd_rocclr_\w+|at::native::\w+)", name)
    return m.group(1) if m else name[:40]


def timeline(src, last=3):
    db = sorted(glob.glob(os.path.join(src, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    calls, cur = [], []
    for r in rows:
        if cur and r[1] - max(x[2] for x in cur) > 150e3:
            calls.append(cur)
            cur = []
        cur.append(r)
    calls.append(cur)
    for seg in calls[-last - 1:-1]:
        t0 = seg[0][1]
        span = max(x[2] for x in seg) - t0
        busy = 0.0
        end = t0
        print("call: %d kernels, GPU span %.1f us" % (len(seg), span / 1e3))
        for name, s, e in seg:
            gap = max(0.0, s - end)
            end = max(end, e)
            print("  %8.1f  %7.1f  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3,
                                                   short(name)))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--db"]:
        timeline(sys.argv[2])
    else:
        run()
