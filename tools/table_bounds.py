"""Worst-case error bounds of the cell-table expansion (tpe_table.hip header).

For one component, exp(A u + B u^2) = sum_n c_n u^n with |c_n| <= c~_n, the
coefficients of exp(|A| u + |B| u^2) (same recurrence, all terms positive).
On |u| <= 1.05 and over the admissible set 9|A| + 65|B| <= 5.8 this prints
  * the truncation bound  e^{a+b} sum_{n>=P} c~_n 1.05^n   (a = 1.05|A|, b = 1.05^2|B|)
  * the fp16 rounding bound of the stored P_6..P_{P-1}: 2^-11 e^{a+b} sum c~_n 1.05^n
  * the share of the terms P_4..P_{P-1} (summed in fp32 by the build, P_0..P_3
    in fp64): e^{a+b} sum_{4<=n<P} c~_n 1.05^n -- their fp32 sums' rounding is
    at most (depth) 2^-24 times that, relative
  * the fp16 Horner bound of the tail P_6 + u(P_7 + u(P_8 + u P_9)), evaluated
    in fp16 (u rounded to fp16, one rounding per packed FMA): a relative error
    of (k + n - 6) 2^-11 on term n for k = P-6 FMAs, i.e.
    2^-11 e^{a+b} sum_n (n - 6 + P - 6) c~_n 1.05^n
all relative to the mixture density (every term positive, P_0 >= 1).

    python tools/table_bounds.py [P] [n_fp32]
"""
import sys

import numpy as np


def majorant(a, b, n_terms=60):
    c = [1.0, a]
    for n in range(1, n_terms):
        c.append((a * c[n] + 2.0 * b * c[n - 1]) / (n + 1))
    return np.array(c)


def bounds(P=10, n32=6, lim=5.8 * (1 + 2e-5), ulim=1.0501, steps=4001):
    """Maxima over the admissible boundary 9|A| + 65|B| = lim (every bound is
    increasing in |A| and in |B|, so the boundary holds the maximum).  Rigorous
    over the whole boundary, not only at the sample points: on the piece
    between t_i and t_i+1 the bound is at most its value at (A(t_i+1), B(t_i)),
    the piece's largest A and largest B.  lim carries the build's fp32
    admissibility-test slack (5.8 (1 + 1e-5) plus rounding), ulim the scorer's
    |u| range after u's fp32 rounding."""
    trunc = fp16 = horner = tail4 = 0.0
    ts = np.linspace(0.0, 1.0, steps)
    for t0, t1 in zip(ts[:-1], ts[1:]):
        A, B = t1 * lim / 9.0, (1.0 - t0) * lim / 65.0
        a, b = A * ulim, B * ulim * ulim
        c = majorant(a, b)
        e = np.exp(a + b)
        trunc = max(trunc, e * c[P:].sum())
        tail4 = max(tail4, e * c[4:P].sum())
        n = np.arange(n32, P)
        fp16 = max(fp16, e * 2.0 ** -11 * c[n32:P].sum())
        horner = max(horner, e * 2.0 ** -11 * ((n - n32 + P - n32) * c[n32:P]).sum())
    return trunc, fp16, horner, tail4


if __name__ == "__main__":
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    n32 = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    tr, h, hh, t4 = bounds(P, n32)
    print("P=%d (fp32 terms %d): truncation <= %.2e, fp16 storage <= %.2e, fp16 Horner <= %.2e, "
          "total <= %.2e; share of P_4.. (fp32 build sums) <= %.4f" % (P, n32, tr, h, hh,
                                                                       tr + h + hh, t4))
