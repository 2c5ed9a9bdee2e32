"""Worst-case error bounds of the cell-table expansion (tpe_table.hip header).

For one component, exp(A u + B u^2) = sum_n c_n u^n with |c_n| <= c~_n, the
coefficients of exp(|A| u + |B| u^2) (same recurrence, all terms positive).
On |u| <= 1.05 and over the admissible set 9|A| + 65|B| <= 5.8 this prints
  * the truncation bound  e^{a+b} sum_{n>=P} c~_n 1.05^n   (a = 1.05|A|, b = 1.05^2|B|)
  * the fp16 rounding bound of the stored P_6..P_{P-1}: 2^-11 e^{a+b} sum c~_n 1.05^n
both relative to the mixture density (every term positive, P_0 >= 1).

    python tools/table_bounds.py [P] [n_fp32]
"""
import sys

import numpy as np


def majorant(a, b, n_terms=60):
    c = [1.0, a]
    for n in range(1, n_terms):
        c.append((a * c[n] + 2.0 * b * c[n - 1]) / (n + 1))
    return np.array(c)


def bounds(P=10, n32=6, lim=5.8, ulim=1.05, steps=801):
    trunc = fp16 = 0.0
    for t in np.linspace(0.0, 1.0, steps):
        A, B = t * lim / 9.0, (1.0 - t) * lim / 65.0
        a, b = A * ulim, B * ulim * ulim
        c = majorant(a, b)
        e = np.exp(a + b)
        trunc = max(trunc, e * c[P:].sum())
        fp16 = max(fp16, e * 2.0 ** -11 * c[n32:P].sum())
    return trunc, fp16


if __name__ == "__main__":
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n32 = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    tr, h = bounds(P, n32)
    print("P=%d (fp32 terms %d): truncation <= %.2e, fp16 rounding <= %.2e, total <= %.2e"
          % (P, n32, tr, h, tr + h))
