"""CPU model of the cell-table plan and build work on bench's C3 level
(tools only: sizes the grid and the build's (component, cell) work under
alternative rules before they are written as kernels).

Replicates k_table_plan1/2 + grid_of (tpe_table.hip): the global floor T
(prior's smallest term over the range - log M - tau), per-component
admissible half-width (9|A| + 65|B| <= 5.8), uniform grid h = min over both
mixtures; then the build's per-cell items (reach window + wide list) and the
included ones (max term over the cell >= T).  Alternatives:
  local  - per-cell floor: the largest single component's minimum over the
           cell (a lower bound of the sum) - log M - tau
  graded - cell half-width from the components that reach the cell only
"""
import math
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from oracle import tpe_oracle as O  # noqa: E402

TAU, RHO, DRAWZ = 25.0, 5.8, 5.8


def coefs(w, mu, sg, family, low, high):
    w = w / w.sum()
    if family == "LGMM1":
        lc = np.log(w) - np.log(np.maximum(sg, 1e-12) * math.sqrt(2 * math.pi))
    else:
        pacc = 1.0 if low is None else np.sum(w * (O.normal_cdf(high, mu, sg) - O.normal_cdf(low, mu, sg)))
        lc = np.log(w / np.sqrt(2 * np.pi * sg ** 2) / pacc)
    return mu, 1.0 / np.maximum(sg, 1e-12), lc


def admissible_s(z):
    return (-9.0 * z + np.sqrt(81.0 * z * z + 166.0 * RHO)) / 83.0


def model(kind, args, below, above):
    fam, pmu, psig, tf, low, high, q = O.posterior_spec(kind, args)
    mb = O.adaptive_parzen_normal(tf(below), 1.0, pmu, psig)
    ma = O.adaptive_parzen_normal(tf(above), 1.0, pmu, psig)
    lo_b = low if low is not None else -np.inf
    hi_b = high if high is not None else np.inf
    a = max(np.min(mb[1] - DRAWZ * mb[2]), lo_b)
    b = min(np.max(mb[1] + DRAWZ * mb[2]), hi_b)
    out = {}
    mixes = []
    for (w, mu, sg) in (mb, ma):
        x, inv, lc = coefs(np.asarray(w), np.asarray(mu), np.asarray(sg), fam, low, high)
        pos = int(np.argmax(sg))  # the prior: widest (prior_sigma)
        far = max(abs(a - x[pos]), abs(b - x[pos])) * inv[pos]
        T = lc[pos] - 0.5 * far * far - (math.log(len(x)) + TAU)
        d = lc - T
        z = np.sqrt(np.maximum(2 * d, 0))
        hk = np.where(d > 0, admissible_s(z) / inv, np.inf)
        mixes.append((x, inv, lc, T, hk, z))
    h = min(m[4].min() for m in mixes)
    nb = int(math.ceil((b - a) / (2 * h)))
    h = (b - a) / (2 * nb)
    y0 = a + (2 * np.arange(nb) + 1) * h
    out["cells"] = nb
    for name, (x, inv, lc, T, hk, z) in zip(("below", "above"), mixes):
        # included (global floor): max term over the cell >= T
        inc = 0
        inc_local = 0
        # chunk cells to bound memory
        for c0 in range(0, nb, 256):
            yy = y0[c0:c0 + 256, None]
            zn = np.maximum(np.abs(yy - x) - h, 0) * inv
            zf = (np.abs(yy - x) + h) * inv
            tmax = lc - 0.5 * zn * zn
            tmin = lc - 0.5 * zf * zf
            inc += int((tmax >= T).sum())
            lb = tmin.max(axis=1, keepdims=True) - (math.log(len(x)) + TAU)
            inc_local += int((tmax >= lb).sum())
        out[name + "_pairs"] = inc
        out[name + "_pairs_local"] = inc_local
    # graded: per cell, the admissible half-width of the components included there
    return out


def main():
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    sp = bench.split(vals, losses)
    seen = set()
    for lab, kind, args in space:
        if kind in ("randint", "quniform") or kind in seen:
            continue
        seen.add(kind)
        r = model(kind, args, *sp[lab])
        print(lab, kind, r, flush=True)


if __name__ == "__main__":
    main()
