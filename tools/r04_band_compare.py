"""Band sizes per table job: bench.py's C3 level vs the drop-in suggest on
the same history (diagnostic; GPU box).  Per job: survivors (ns), listed
cells, overflow, tiles at or above G and the entries walked, from the band
workspace / tile headers the last level left (layout as tools/r04_bandtime.py).
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import hyperopt_amd.engine as E  # noqa: E402
from hyperopt_amd import _lib as L  # noqa: E402


def report(eng, tag):
    lib = L.load()
    a, b = eng._tables_slice
    jobs = eng.last_plan[3][a:b]
    nj = b - a
    ctl_b, work_b = ctypes.c_int64(0), ctypes.c_int64(0)
    lib.tpe_band_bytes(jobs.ctypes.data, nj, ctypes.byref(ctl_b), ctypes.byref(work_b))
    per = work_b.value // nj
    raw = eng._bufs["band_work"][:work_b.value].cpu().numpy()
    nt = ctl_b.value // (nj * 16)
    H = eng._bufs["band_ctl"][:ctl_b.value].cpu().numpy().view(np.uint32).reshape(nj, nt, 4)
    tot_ns = tot_walk = 0
    for j in range(nj):
        w = raw[j * per:(j + 1) * per]
        tail = w[per - (16 + 16 * 24 + 64 + 16):]
        ns, ncell, over, _ = tail[:16].view(np.int32)
        lo = H[j, :, 0].view(np.float32)
        hm = H[j, :, 1].view(np.float32)
        cnt = H[j, :, 2]
        G = lo.max()
        sel = (hm >= G) & (cnt != 0)
        walked = int(cnt[sel & (cnt != 0xFFFFFFFF)].sum())
        tot_ns += ns
        tot_walk += walked
        print("%s job %2d fam %d ns %6d ncell %3d over %d tiles>=G %4d walked %6d full %d" % (
            tag, j, jobs[j]["family"], ns, ncell, over, sel.sum(), walked,
            (cnt == 0xFFFFFFFF).sum()), flush=True)
    print("%s total ns %d walked %d stats %s" % (tag, tot_ns, tot_walk, eng.last_table_stats),
          flush=True)


def main():
    import torch
    torch.cuda.set_device(0)
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    n = bench.N_CAND
    eng = E.Engine()
    units = [(j, 0, n) for j in range(len(space))]
    mat = bench.c3_matrix(space, vals)
    hist = E.DeviceHistory(eng, len(space), cap=bench.T_HIST)
    hist.append(mat)
    rb = bench.below_rows(losses)
    isb = np.zeros(bench.T_HIST, np.uint8)
    isb[rb] = 1
    for it in range(3):
        batch = bench.history_batch(space, mat, hist, rb, it, n, 0, units, n)
        eng.run(batch, precision=32, history=hist, is_below=isb)
        report(eng, "bench%d" % it)
    from hyperopt_amd import tpe
    from hyperopt_amd.base import JOB_STATE_DONE
    domain, trials = bench.c3_trials(space, vals, losses)
    rng = np.random.RandomState(9)
    for k in range(3):
        docs = tpe.suggest([losses.size + k], domain, trials, k, n_EI_candidates=n, verbose=False)
        report(tpe.engine(), "dropin%d" % k)
        docs[0]["state"] = JOB_STATE_DONE
        docs[0]["result"] = {"status": "ok", "loss": float(rng.normal())}
        trials.insert_trial_docs(docs)
        trials.refresh()


if __name__ == "__main__":
    main()
