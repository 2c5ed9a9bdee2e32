"""Phase timings of k_band (TPE_BAND_TIMING builds), bench's C3 level."""
import numpy as np
import bench
import hyperopt_amd.engine as E
from hyperopt_amd import _lib as L
import ctypes
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
    r = eng.run(batch, precision=32, history=hist, is_below=isb)
lib = L.load()
work_b = ctypes.c_int64(0)
jobs = eng.last_plan[3]
tj = jobs[:30]
lib.tpe_band_bytes(tj.ctypes.data, 30, None, ctypes.byref(work_b))
per = work_b.value // 30
raw = eng._bufs["band_work"][:work_b.value].cpu().numpy()
for j in range(30):
    w = raw[j * per:(j + 1) * per]
    off = per - 16 - 64 * 1 - 64  # locate fields from the end: win[16] BestT (24 B each)...
    # fields: ... ns, ncell, over, pad0, tmark[8], win[16] (24 B), done, pad[3]
    tail = w[per - (16 + 16 * 24 + 64 + 16):]
    ns, ncell, over, _ = tail[:16].view(np.int32)
    tm = tail[16:80].view(np.int64)
    print(j, "ns %5d ncell %3d over %d  k_band phases us: %s  final: start->merged %s ->scored %s ->done %s  gap band->final %.1f" % (
        ns, ncell, over, np.round(np.diff(tm[:4]) / 100.0, 1), round((tm[5] - tm[4]) / 100.0, 1),
        round((tm[6] - tm[5]) / 100.0, 1), round((tm[7] - tm[6]) / 100.0, 1), (tm[4] - tm[3]) / 100.0))
# tile headers: entries walked per job vs survivors
ctl_b = ctypes.c_int64(0)
lib.tpe_band_bytes(tj.ctypes.data, 30, ctypes.byref(ctl_b), None)
nt = ctl_b.value // (30 * 16)
H = eng._bufs["band_ctl"][:ctl_b.value].cpu().numpy().view(np.uint32).reshape(30, nt, 4)
for j in range(30):
    lo = H[j, :, 0].view(np.float32); hm = H[j, :, 1].view(np.float32); cnt = H[j, :, 2]
    G = lo.max()
    sel = (hm >= G) & (cnt != 0)
    print(j, "tiles %d  G %.6g  tiles>=G %d  entries walked %d  full %d" % (
        nt, G, sel.sum(), cnt[sel & (cnt != 0xFFFFFFFF)].sum(), (cnt == 0xFFFFFFFF).sum()))
# slow-component lists of the cell path (BandMix: 21 P + m + n_dir/pad + dir[16] = 248 B)
for j in range(30):
    w = raw[j * per:(j + 1) * per]
    tail = w[per - (16 + 16 * 24 + 64 + 16):]
    ns, ncell, over, _ = tail[:16].view(np.int32)
    if ns <= 128 or over:
        continue
    nch = max(1, 16 // max(ncell, 1))
    nd = [[], []]
    for k in range(ncell):
        for c in range(nch):
            for mix in range(2):
                o = 65536 + ((k * 16 + c) * 2 + mix) * 248 + 176
                nd[mix].append(int(w[o:o + 4].view(np.int32)[0]))
    print(j, "ns %d ncell %d nch %d n_dir per chunk below %s above %s" % (ns, ncell, nch, nd[0], nd[1]))
