"""Fit the float32 polynomial coefficients used by include/cvr_detmath.h.

The renderer needs transcendental functions (log, sin/cos, acos, atan) whose
float32 results are *identical* on the CPU oracle (gcc) and on gfx950 (hipcc),
so that one path traced on both sides consumes the same random numbers and
takes the same branches.  Vendor libm/ocml differ in the last ulp, so both
sides use these hand-rolled polynomials instead (evaluated with explicit fmaf,
which is correctly rounded on x86-64 and on CDNA4).

Method: weighted least squares on Chebyshev nodes in float64, coefficients
rounded to float32.  Accuracy is then validated in C against double-precision
libm by tests/test_detmath.py (max ulp error is asserted there).

Run: python tools/fit_detmath.py   (prints the coefficient tables)
"""
import numpy as np


def cheb_nodes(a, b, n):
    k = np.arange(n)
    return 0.5 * (a + b) + 0.5 * (b - a) * np.cos((2 * k + 1) * np.pi / (2 * n))


def fit(basis_fn, target, xs, weight):
    A = np.stack([basis_fn(xs, i) for i in range(basis_fn.n)], axis=1)
    w = weight(xs)
    c, *_ = np.linalg.lstsq(A * w[:, None], target(xs) * w, rcond=None)
    return c.astype(np.float32)


class Basis:
    def __init__(self, n, fn):
        self.n = n
        self.fn = fn

    def __call__(self, x, i):
        return self.fn(x, i)


def show(name, c):
    print(name)
    for v in c:
        print(f"  {float(v)!r}f  /* {np.float32(v).view(np.uint32):#010x} */")


def main():
    # log1p(f) = f - f^2/2 + f^3 * P(f), f in [sqrt(.5)-1, sqrt(2)-1]
    lo, hi = np.sqrt(0.5) - 1, np.sqrt(2.0) - 1
    xs = cheb_nodes(lo, hi, 4000)
    deg = 8
    b = Basis(deg, lambda x, i: x ** i)
    c = fit(b, lambda x: np.where(np.abs(x) < 1e-8, 1.0 / 3.0,
                                  (np.log1p(x) - x + 0.5 * x * x) / np.where(x == 0, 1, x ** 3)),
            xs, lambda x: np.abs(x) ** 3 / np.abs(np.log1p(x) + 1e-300))
    show("LOG P (f^0..)", c)

    # sin(r) = r + r^3 * S(r^2), cos(r) = 1 - r^2/2 + r^4 * C(r^2), |r| <= pi/4
    zs = cheb_nodes(0.0, (np.pi / 4) ** 2, 2000)
    r = np.sqrt(zs)
    bs = Basis(4, lambda z, i: z ** i)
    s = fit(bs, lambda z: (np.sin(np.sqrt(z)) - np.sqrt(z)) / (np.sqrt(z) ** 3),
            zs, lambda z: np.sqrt(z) ** 3 / np.sin(np.sqrt(z)))
    show("SIN S (z^0..)", s)
    cc = fit(bs, lambda z: (np.cos(np.sqrt(z)) - 1 + 0.5 * z) / (z * z),
             zs, lambda z: z * z / np.cos(np.sqrt(z)))
    show("COS C (z^0..)", cc)

    # asin(x) = x + x^3 * A(x^2), |x| <= 0.5
    zs = cheb_nodes(0.0, 0.25, 2000)
    ba = Basis(6, lambda z, i: z ** i)
    a = fit(ba, lambda z: (np.arcsin(np.sqrt(z)) - np.sqrt(z)) / (np.sqrt(z) ** 3),
            zs, lambda z: np.sqrt(z) ** 3 / np.arcsin(np.sqrt(z)))
    show("ASIN A (z^0..)", a)

    # atan(x) = x + x^3 * T(x^2), 0 <= x <= 1
    zs = cheb_nodes(0.0, 1.0, 4000)
    bt = Basis(10, lambda z, i: z ** i)
    t = fit(bt, lambda z: (np.arctan(np.sqrt(z)) - np.sqrt(z)) / (np.sqrt(z) ** 3),
            zs, lambda z: np.sqrt(z) ** 3 / np.arctan(np.sqrt(z)))
    show("ATAN T (z^0..)", t)


if __name__ == "__main__":
    main()
