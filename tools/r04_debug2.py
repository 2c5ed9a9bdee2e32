"""Round-4 diagnostics: bench's C3 level -- which jobs overflow the band and why."""
import numpy as np
import torch
import bench
import hyperopt_amd.engine as E
from hyperopt_amd import _lib as L

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
orig = eng._band_fix
seen = []
def spy(band_jobs, d_segs, max_comp, n_comp, stream, exchanged, best_h, jobs):
    seen.append([int(p) for a, b in band_jobs for p in range(a, b) if best_h["n_scored"][p] < 0])
    return orig(band_jobs, d_segs, max_comp, n_comp, stream, exchanged, best_h, jobs)
eng._band_fix = spy
batch = bench.history_batch(space, mat, hist, rb, 0, n, 0, units, n)
r = eng.run(batch, precision=32, history=hist, is_below=isb)
print("overflowed job positions:", seen)
nt = 1024
ctl = eng._bufs["band_ctl"]
nj = 30
h = ctl[:16 * nt * nj].cpu().numpy().view(np.uint32).reshape(nj, nt, 4)
for j in range(nj):
    lo = h[j, :, 0].view(np.float32)
    hi = h[j, :, 1].view(np.float32)
    cnt = h[j, :, 2]
    G = lo.max()
    rel = ~(hi < G)
    full = cnt == 0xFFFFFFFF
    print(j, "G %.6f rel %d full %d full&rel %d ent(rel) %d maxcnt %d" % (
        G, rel.sum(), full.sum(), (full & rel).sum(), cnt[rel & ~full].sum(), cnt[~full].max()))
tabs = eng._bufs["tables"][:L.TABLE_DTYPE.itemsize * nj].cpu().numpy().view(L.TABLE_DTYPE)
for j in range(nj):
    t = tabs[j]
    print(j, "nb %d items %d eps_mix %.3e eps_cubic %.3e" % (t["nb"], t["build_items"], t["eps_mix"], t["eps_cubic"]))
