"""Table-path stats (fallback candidates, flagged cells) of bench's C3 level."""
import numpy as np
import bench
import hyperopt_amd.engine as E
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
for it in range(2):
    batch = bench.history_batch(space, mat, hist, rb, it, n, 0, units, n)
    r = eng.run(batch, precision=32, history=hist, is_below=isb)
    print("level", it, eng.last_table_stats, flush=True)
print("band overflows (bench level):", getattr(eng, "band_overflows", 0), getattr(eng, "last_band_overflow", None))
