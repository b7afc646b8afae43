"""Second, independent restatement of the four ChF kernels in vectorised
numpy (test infrastructure).  Used to cross-check the C oracle bit for bit
on small boxes, so an indexing slip in either restatement shows up.

Arrays carry one ghost layer: shape (nz+2, ny+2, nx+2), [k, j, i].
Each expression keeps the Fortran evaluation order of
Source/VariableCoeffPoissonOperatorF.ChF.
"""
import numpy as np


def lap7(u):
    c = u[1:-1, 1:-1, 1:-1]
    tx = (u[1:-1, 1:-1, 2:] + u[1:-1, 1:-1, :-2]) - 2.0 * c
    ty = (u[1:-1, 2:, 1:-1] + u[1:-1, :-2, 1:-1]) - 2.0 * c
    tz = (u[2:, 1:-1, 1:-1] + u[:-2, 1:-1, 1:-1]) - 2.0 * c
    return (tx + ty) + tz


def colour_mask(shape, lo, rb):
    nz, ny, nx = shape
    k, j, i = np.meshgrid(np.arange(nz) + lo[2], np.arange(ny) + lo[1], np.arange(nx) + lo[0],
                          indexing="ij")
    return ((i + j + k) % 2) == rb


def gsrb(u, rhs, a, b, lam, dx, alpha, beta, rb, lo=(0, 0, 0)):
    """GSRBHELMHOLTZVC3D (.ChF:56-139) on the interior; returns new u."""
    dxinv = 1.0 / (dx * dx)
    c = u[1:-1, 1:-1, 1:-1]
    lof = alpha * a * c
    ld = lap7(u)
    ld = ld * dxinv * b
    lof = lof - beta * ld
    new = c - lam * (lof - rhs)
    out = u.copy()
    m = colour_mask(c.shape, lo, rb)
    out[1:-1, 1:-1, 1:-1][m] = new[m]
    return out


def apply_op(u, a, b, dx, alpha, beta):
    """VCCOMPUTEOP3D (.ChF:181-237)."""
    dxinv = 1.0 / (dx * dx)
    lof = alpha * a * u[1:-1, 1:-1, 1:-1]
    ld = lap7(u) * dxinv * beta * b
    return lof - ld


def residual(u, rhs, a, b, dx, alpha, beta):
    """VCCOMPUTERES3D (.ChF:283-339)."""
    dxinv = 1.0 / (dx * dx)
    r = rhs - alpha * a * u[1:-1, 1:-1, 1:-1]
    ld = lap7(u) * dxinv * beta * b
    return r + ld


def restrict(u, rhs, a, b, dx, alpha, beta):
    """RESTRICTRESVC3D (.ChF:379-437) after res.setVal(0): children summed
    in k, j, i order."""
    dxinv = 1.0 / (dx * dx)
    lof = alpha * a * u[1:-1, 1:-1, 1:-1]
    ld = lap7(u) * dxinv * beta * b
    lof = lof - ld
    t = (rhs - lof) / 8.0
    nz, ny, nx = t.shape
    s = np.zeros((nz // 2, ny // 2, nx // 2))
    for kk in range(2):
        for jj in range(2):
            for ii in range(2):
                s = s + t[kk::2, jj::2, ii::2]
    return s


def lam(a, dx, alpha, beta):
    shift = 2.0 * 3 * beta / (dx * dx)
    v = a * alpha
    v = v + shift
    return 1.0 / v


def average(fine, ratio, harmonic):
    nz, ny, nx = fine.shape
    s = np.zeros((nz // ratio, ny // ratio, nx // ratio))
    for kk in range(ratio):
        for jj in range(ratio):
            for ii in range(ratio):
                f = fine[kk::ratio, jj::ratio, ii::ratio]
                s = s + (1.0 / f if harmonic else f)
    rs = 1.0 / (ratio ** 3)
    return 1.0 / (s * rs) if harmonic else s * rs
