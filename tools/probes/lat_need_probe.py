"""Which quantized labels of a C3 level draw the rest of their stream after
the prefix decision (tpe_lattice_suggest's need flags), and the winners'
indices (diagnostic)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    import torch
    from hyperopt_amd.engine import Engine, LabelWork
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    rows = bench.below_rows(losses)
    isb = np.zeros(losses.size, bool)
    isb[rows] = True
    eng = Engine()
    works = [LabelWork(lab, kind, args, vals[lab][isb], vals[lab][~isb], n_cand=bench.N_CAND,
                       key=1000 + j)
             for j, (lab, kind, args) in enumerate(space) if kind == "quniform"]
    res = eng.run(works, precision=32)
    torch.cuda.synchronize()
    need = eng._bufs["lat_need"][:4 * len(works)].cpu().numpy().view(np.int32)
    for w, r, n in zip(works, res, need):
        print("%s need %d index %d value %g score %.6f" % (w.label, n, r.index, r.value, r.score))


if __name__ == "__main__":
    main()
