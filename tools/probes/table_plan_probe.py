"""CPU restatement of the cell-table plan (k_table_plan1/2 + grid_of) on
C3's histories: cells per label, components per cell, and the work of a
graded grid (diagnostic for DESIGN.md 3.1's build cost).

    python tools/probes/table_plan_probe.py
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from oracle import tpe_oracle as O  # noqa: E402

RHO = 5.8
TAU = 25.0
CAP = 1 << 15


def adm(z):
    return (-9.0 * z + np.sqrt(81.0 * z * z + 166.0 * RHO)) / 83.0


def mixture(kind, args, obs):
    fam, pmu, psig, tf, low, high, q = O.posterior_spec(kind, args)
    w, mu, sg = O.adaptive_parzen_normal(tf(obs), 1.0, pmu, psig)
    lo = math.log(low) if False else low
    inv = 1.0 / sg
    if fam == "GMM1":
        pacc = 1.0
        if low is not None:
            from scipy.stats import norm
            pacc = np.sum(w * (norm.cdf(high, mu, sg) - norm.cdf(low, mu, sg)))
        lc = np.log(w / np.sqrt(2 * np.pi * sg * sg) / pacc)
    else:
        lc = np.log(w) - np.log(sg * np.sqrt(2 * np.pi))
    return dict(mu=mu, inv=inv, lc=lc, sg=sg, pos=int(np.argmax(sg == psig) if False else
                                                   np.flatnonzero((mu == pmu) & (sg == psig))[0]),
                low=low, high=high, psig=psig)


def plan(B, A):
    a = np.min(B["mu"] - 5.8 * B["sg"])
    b = np.max(B["mu"] + 5.8 * B["sg"])
    if B["low"] is not None:
        a, b = max(a, B["low"]), min(b, B["high"])
    out = {}
    for name, S in (("below", B), ("above", A)):
        p = S["pos"]
        far = max(abs(a - S["mu"][p]), abs(b - S["mu"][p])) * S["inv"][p]
        T = S["lc"][p] - 0.5 * far * far - (math.log(S["mu"].size) + TAU)
        d = S["lc"] - T
        z = np.sqrt(2 * np.maximum(d, 0))
        hk = np.where(d > 0, adm(z) / S["inv"], np.inf)
        out[name] = (T, hk)
    return a, b, out


def included(S, T, y0, h):
    zn = np.maximum(np.abs(y0 - S["mu"]) - h, 0) * S["inv"]
    return np.count_nonzero(S["lc"] - 0.5 * zn * zn >= T)


def main():
    space = bench.c3_space()
    vals, losses = bench.c3_history(space)
    sp = bench.split(vals, losses)
    for lab in ("u0", "lu0", "n0"):
        kind, args = [(k, a) for l_, k, a in space if l_ == lab][0]
        below, above = sp[lab]
        B, A = mixture(kind, args, below), mixture(kind, args, above)
        a, b, P = plan(B, A)
        h = min(P["below"][1].min(), P["above"][1].min())
        span = b - a
        nb = min(CAP, max(1, math.ceil(span / (2 * h))))
        hh = span / (2 * nb)
        ys = a + hh * (2 * np.arange(nb) + 1)
        pick = ys[:: max(1, nb // 200)]
        nbw = np.mean([included(B, P["below"][0], y, hh) for y in pick])
        naw = np.mean([included(A, P["above"][0], y, hh) for y in pick])
        # graded: local admissible h at y = min hk over the components included near y
        loc = []
        for y in pick:
            hl = np.inf
            for name, S in (("below", B), ("above", A)):
                T, hk = P[name]
                zn = np.maximum(np.abs(y - S["mu"]) - 4 * hh, 0) * S["inv"]
                m = S["lc"] - 0.5 * zn * zn >= T
                if m.any():
                    hl = min(hl, hk[m].min())
            loc.append(hl)
        loc = np.array(loc)
        graded = span / len(pick) * np.sum(1.0 / (2 * loc))
        print("%-4s %-10s span %.3f h %.3g nb %d  comps/cell below %.1f above %.1f  "
              "work %.3g  graded cells ~%.0f (local h %.3g..%.3g)"
              % (lab, kind, span, h, nb, nbw, naw, nb * (nbw + naw), graded, loc.min(), loc.max()))


main()
