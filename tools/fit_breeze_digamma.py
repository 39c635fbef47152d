"""Generates the coefficients of E(y) = ψ(y) − S8(y), the truncation error of the 8-term asymptotic
digamma series S8 that Breeze 0.13.2's digamma evaluates at y ∈ (5, 6] ([U] breeze.numerics.digamma:
recurrence while x ≤ 5, then S8).  The device digamma evaluates S8 at x + 6 (one rational for the six
recurrence terms); adding E(x + 6) − E(y_B) at y_B = x + ⌊5 − x⌋ + 1 reproduces Breeze's value to
~1e-16 instead of differing from it by up to 8e-13 (which a slowly-dying topic of a long E-step
amplifies past 1e-7).  E(y)·y^18 is fitted as a polynomial in f = 1/y² over y ∈ [5, 11.5] with
mpmath at 50 digits.  Prints the C initialiser for csrc/stc_internal.h."""
import mpmath as mp
import numpy as np

mp.mp.dps = 50


def s8(y):
    f = 1 / (y * y)
    t = f * (mp.mpf(-1) / 12 + f * (mp.mpf(1) / 120 + f * (mp.mpf(-1) / 252 + f * (mp.mpf(1) / 240 + f * (
        mp.mpf(-1) / 132 + f * (mp.mpf(691) / 32760 + f * (mp.mpf(-1) / 12 + f * mp.mpf(3617) / 8160)))))))
    return mp.log(y) - mp.mpf(1) / 2 / y + t


def main(deg=4):
    ys = [mp.mpf(5) + (mp.mpf(13) / 2) * mp.mpf(i) / 400 for i in range(401)]
    f = np.array([float(1 / (y * y)) for y in ys])
    g = np.array([float((mp.digamma(y) - s8(y)) * y ** 18) for y in ys])
    # Chebyshev-like conditioning: fit in u = (f − f_mid)/f_half, then expand
    c = np.polynomial.polynomial.polyfit(f, g, deg)
    fit = np.polynomial.polynomial.polyval(f, c)
    err = np.max(np.abs(fit - g) * f ** 9)
    print(f"// max |E_fit − E| = {err:.2e} over y in [5, 11.5]")
    print("static constexpr double kBreezeE[%d] = {%s};" % (deg + 1, ", ".join(repr(float(x)) for x in c)))


if __name__ == "__main__":
    main()
