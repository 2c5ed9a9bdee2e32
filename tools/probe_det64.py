"""Determinism of the pruned fp64 scorer: repeated runs and upload vs
history-gather runs of tests/test_gpu_history.py's T=3000 case (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hyperopt_amd.engine import DeviceHistory, Engine  # noqa: E402
from tests import test_gpu_history as H  # noqa: E402

torch.cuda.set_device(0)
eng = Engine()
T = 3000
mat, active, losses = H._history(T, T, 0.0)
rows = np.arange(T)
up, _ = H._works(mat, active, losses, rows)
hist = DeviceHistory(eng, len(H.SPACE), cap=64)
for a in range(0, T, 700):
    hist.append(mat[a:a + 700], active[a:a + 700])
hw, isb = H._works(mat, active, losses, rows, hist=hist)
r1 = eng.run(up, precision=64, outputs=True)
r2 = eng.run(up, precision=64, outputs=True)
p1 = eng.run(up[:1], precision=64, posteriors=True)[0].extra
r3 = eng.run(hw, precision=64, history=hist, is_below=isb)
r4 = eng.run(up, precision=64)
r5 = eng.run(up, precision=64)
for a, b in zip(r1, r2):
    print(a.label, "rep outputs equal:", np.array_equal(a.below_llik, b.below_llik),
          np.array_equal(a.above_llik, b.above_llik), np.array_equal(a.cand, b.cand))
for a, b, c, d in zip(r1, r3, r4, r5):
    print(a.label, (a.index, a.score), (b.index, b.score), (c.index, c.score), (d.index, d.score))
a = r1[0]
s = a.below_llik - a.above_llik
print("argmax", int(np.argmax(s)), s.max())
