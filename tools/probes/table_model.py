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


def model_local(kind, args, below, above):
    """Per-component floors from the prior's term across the component's own
    reach: g(y) = prior(y) - term_k(y) >= log M + tau outside [y1, y2]."""
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
        pos = int(np.argmax(sg))
        L = math.log(len(x)) + TAU
        far = max(abs(a - x[pos]), abs(b - x[pos])) * inv[pos]
        Tg = lc[pos] - 0.5 * far * far - L
        wide = inv <= 4.0 / sg[pos]
        y1 = np.full(len(x), -np.inf)
        y2 = np.full(len(x), np.inf)
        zmax = np.zeros(len(x))
        for k in range(len(x)):
            if wide[k]:
                d = lc[k] - Tg
                z = math.sqrt(max(2 * d, 0.0))
                y1[k], y2[k] = x[k] - z / inv[k], x[k] + z / inv[k]
                zmax[k] = z
                continue
            a2 = 0.5 * (inv[k] ** 2 - inv[pos] ** 2)
            a1 = -(x[k] * inv[k] ** 2 - x[pos] * inv[pos] ** 2)
            a0 = (lc[pos] - lc[k]) + 0.5 * (x[k] ** 2 * inv[k] ** 2 - x[pos] ** 2 * inv[pos] ** 2) - L
            disc = a1 * a1 - 4 * a2 * a0
            if disc <= 0:
                y1[k], y2[k] = np.inf, -np.inf  # never above the floor
                continue
            r = math.sqrt(disc)
            y1[k], y2[k] = (-a1 - r) / (2 * a2), (-a1 + r) / (2 * a2)
            y1[k], y2[k] = max(y1[k], a), min(y2[k], b)
            zmax[k] = max(abs(y1[k] - x[k]), abs(y2[k] - x[k])) * inv[k]
        hk = np.where(zmax > 0, admissible_s(zmax) / inv, np.inf)
        mixes.append((x, inv, lc, y1, y2, hk))
    h = min(m[5].min() for m in mixes)
    nb = int(math.ceil((b - a) / (2 * h)))
    h = (b - a) / (2 * nb)
    y0 = a + (2 * np.arange(nb) + 1) * h
    out["cells"] = nb
    for name, (x, inv, lc, y1, y2, hk) in zip(("below", "above"), mixes):
        pairs = 0
        for c0 in range(0, nb, 256):
            yy = y0[c0:c0 + 256, None]
            pairs += int(((yy + h >= y1) & (yy - h <= y2)).sum())
        out[name + "_pairs"] = pairs
    return out


def main_local():
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    sp = bench.split(vals, losses)
    seen = set()
    for lab, kind, args in space:
        if kind in ("randint", "quniform") or kind in seen:
            continue
        seen.add(kind)
        print(lab, kind, "global", model(kind, args, *sp[lab]), flush=True)
        print(lab, kind, "local ", model_local(kind, args, *sp[lab]), flush=True)
