"""Fit the bf16-output GELU used in the GEMM / conv epilogues: GELU(x) ~= x / (1 + 2^-(a1 x + a3 x^3 + a5 x^5)),
minimax on the absolute error of y over [-8, 8]; reports how often the bf16-rounded result differs from the
bf16-rounded exact (erf) GELU on N(0, 2^2) inputs, next to the A&S 7.1.26 erf form used in fp32 mode.

  python tools/fit_gelu.py
"""
import numpy as np
from scipy.optimize import minimize
from scipy.special import erf


def bf16(v):
    u = np.asarray(v, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def approx(c, x):
    a1, a3, a5 = c
    w = x * (a1 + x * x * (a3 + x * x * a5))
    return x / (1 + np.exp2(-w))


def as_gelu(x):
    ax = np.abs(x / np.sqrt(2))
    t = 1 / (1 + 0.3275911 * ax)
    p = 1.061405429
    for cc in [-1.453152027, 1.421413741, -0.284496736, 0.254829592]:
        p = p * t + cc
    r = 1 - p * t * np.exp(-ax * ax)
    return 0.5 * x * (1 + np.sign(x) * r)


def main():
    x = np.linspace(-8, 8, 200001)
    y = x * 0.5 * (1 + erf(x / np.sqrt(2)))
    L = np.log2(np.e)
    c0 = np.array([1.5976 * L, 0.070566 * L, 0.0])
    err = lambda c: np.max(np.abs(approx(c, x) - y))  # noqa: E731
    print("sigmoid-cubic (Bowling) max |err|", err(c0))
    best = None
    for a5 in [0, 1e-4, -1e-4, 3e-4, -3e-4]:
        r = minimize(err, c0 + np.array([0, 0, a5]), method="Nelder-Mead",
                     options={"xatol": 1e-12, "fatol": 1e-14, "maxiter": 40000})
        if best is None or r.fun < best.fun:
            best = r
    c = best.x
    print("fit a1 a3 a5 =", repr(c.astype(np.float32).tolist()), "max |err|", best.fun)
    xs = (np.random.default_rng(0).standard_normal(2000000) * 2).astype(np.float32)
    ye = bf16(xs * 0.5 * (1 + erf(xs.astype(np.float64) / np.sqrt(2))))
    ya = bf16(approx(c.astype(np.float32), xs.astype(np.float64)))
    yb = bf16(as_gelu(xs.astype(np.float64)))
    print("bf16 outputs differing from exact: fit %.4f%% (max %.3g), A&S %.4f%% (max %.3g)" %
          (100 * np.mean(ye != ya), np.max(np.abs(ye - ya)), 100 * np.mean(ye != yb), np.max(np.abs(ye - yb))))


if __name__ == "__main__":
    main()
