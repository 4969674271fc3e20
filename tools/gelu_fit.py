"""Coefficients of the bf16 epilogues' GELU (csrc/common.h gelu_fast / gelu_fast2): GELU(x) = x Phi(x) =
max(x, 0) - |x| h with h = Phi(-|x|) = 2^q(a), a = min(|x|, A), q a degree-DEG polynomial fit of log2 Phi(-a)
on [0, A] (iteratively reweighted least squares toward the minimax fit on a Chebyshev grid). Prints the
float32 coefficients (highest power first) and the error of the float32 evaluation against the exact
erf GELU in float64.
    python tools/gelu_fit.py [A] [DEG]"""
import sys

import numpy as np
from scipy.special import log_ndtr, ndtr


def fit(A, deg):
    a = np.cos(np.linspace(0, np.pi, 20000)) * A / 2 + A / 2
    q = log_ndtr(-a) / np.log(2)
    w = np.ones_like(a)
    best = None
    for _ in range(200):
        c = np.polyfit(a, q, deg, w=w)
        err = np.abs(np.polyval(c, a) - q)
        if best is None or err.max() < best[0]:
            best = (err.max(), c)
        w = w * (1 + 0.5 * err / err.max())
        w /= w.mean()
    return best[1].astype(np.float32)


def gelu_f32(x, c, A):
    a = np.minimum(np.abs(x), np.float32(A))
    p = np.full_like(a, c[0])
    for k in c[1:]:
        p = (p * a + k).astype(np.float32)
    h = np.exp2(p.astype(np.float64)).astype(np.float32)
    return (np.maximum(x, 0) - np.abs(x) * h).astype(np.float32)


def main():
    A = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
    deg = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    c = fit(A, deg)
    x = np.linspace(-12, 12, 2000001).astype(np.float32)
    y = gelu_f32(x, c, A)
    yt = x.astype(np.float64) * ndtr(x.astype(np.float64))
    rel = np.abs(y - yt) / np.maximum(np.abs(yt), 1e-30)
    print("coefficients:", ", ".join("%.9ef" % v for v in c))
    print("max relative error |x| <= A: %.2e; max abs error: %.2e; max abs error x < -A: %.2e"
          % (rel[np.abs(x) <= A].max(), np.abs(y - yt).max(), np.abs(y - yt)[x < -A].max()))


if __name__ == "__main__":
    main()
