"""Accuracy of the E-step's fp32 digamma (stc_internal.h digamma_fast) against scipy, in numpy fp32.

    python tools/dg_check.py
"""
import numpy as np
from scipy.special import digamma

F = np.float32


def series(y):
    iy = F(1) / y
    f = iy * iy
    t = f * (F(-1 / 12) + f * (F(1 / 120) + f * (F(-1 / 252) + f * (F(1 / 240) + f * F(-1 / 132)))))
    return np.log(y) - F(0.5) * iy + t


def dg_shift4(x):
    """ψ(x) = ψ(x+4) − 1/x − (3x²+12x+11)/((x+1)(x+2)(x+3)): three reciprocals and one log."""
    x = F(x)
    num = (F(3) * x + F(12)) * x + F(11)
    den = ((x + F(6)) * x + F(11)) * x + F(6)
    return series(x + F(4)) - (F(1) / x + num * (F(1) / den))


def dg_shift6(x):
    """ψ(x) = ψ(x+6) − Σ_{i<6} 1/(x+i): seven reciprocals and one log (the previous form)."""
    x = F(x)
    r = sum(F(1) / (x + F(i)) for i in range(6))
    return series(x + F(6)) - r


if __name__ == "__main__":
    xs = np.logspace(-4, 7, 40000).astype(np.float32)
    ref = digamma(xs.astype(np.float64))
    for name, fn in [("shift6", dg_shift6), ("shift4", dg_shift4)]:
        with np.errstate(all="ignore"):
            v = fn(xs).astype(np.float64)
        err = np.abs(v - ref)
        print(f"{name}: max abs err {err.max():.3e}, max err/max(|psi|,1) {(err / np.maximum(np.abs(ref), 1)).max():.3e}")
