"""Independent numpy restatement of the COLMAP 3.4/3.5 estimator arithmetic the
reference op reaches through TwoViewGeometry::Estimate
(reference integration/op_cpp/sequential_matching.cc:98-99; upstream, un-vendored
estimators/fundamental_matrix.cc, estimators/homography_matrix.cc,
estimators/utils.cc, util/polynomial.cc) in COLMAP's own formulation:

* 7-point F: the 7 x 9 constraint matrix, its SVD (Eigen::JacobiSVD, full V):
  f1 = V[:, 7], f2 = V[:, 8], f1 -= f2; the closed-form det(l f1 + f2) cubic;
  roots as companion-matrix eigenvalues (FindPolynomialRootsCompanionMatrix ->
  np.roots), kept when |imag| <= 1e-10; F = l f1 + f2 (column-major reshape,
  transposed on return), skipped when |F(2,2)| < 1e-10, divided by F(2,2).
* 8-point F: CenterAndNormalizeImagePoints, N x 9 constraint matrix, null vector
  = last right singular vector, rank-2 projection by SVD with sigma_3 = 0,
  F = T2^T F T1.
* Homography DLT: normalised 2N x 9 system, last right singular vector,
  H = T2^-1 H T1.
* Residuals: ComputeSquaredSampsonError, HomographyMatrixEstimator::Residuals.

Test infrastructure only (tests/test_estimators_independent.py): the product
and the CPU oracle share geom_solvers.h (Householder QR null spaces, bracketed
Newton cubic roots, inverse-squaring least-squares null vectors); this module
checks that arithmetic against the SVD / eigenvalue formulation without sharing
any code with it.
"""
from __future__ import annotations

import numpy as np


def normalize(pts: np.ndarray):
    """CenterAndNormalizeImagePoints: centroid, RMS distance, sqrt(2) scale."""
    c = pts.mean(axis=0)
    rms = np.sqrt(((pts - c) ** 2).sum(axis=1).mean())
    s = np.sqrt(2.0) / rms
    T = np.array([[s, 0.0, -s * c[0]], [0.0, s, -s * c[1]], [0.0, 0.0, 1.0]])
    h = np.c_[pts, np.ones(len(pts))] @ T.T
    return h[:, :2] / h[:, 2:3], T


def f_rows(x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    """Rows [x2 x1, x2 y1, x2, y2 x1, y2 y1, y2, x1, y1, 1] (x2' F x1 = 0)."""
    x0, y0 = x1[:, 0], x1[:, 1]
    xx, yy = x2[:, 0], x2[:, 1]
    one = np.ones(len(x1))
    return np.stack([xx * x0, xx * y0, xx, yy * x0, yy * y0, yy, x0, y0, one], axis=1)


def fundamental_7pt(x1: np.ndarray, x2: np.ndarray) -> list[np.ndarray]:
    A = f_rows(x1, x2)
    _, _, vt = np.linalg.svd(A, full_matrices=True)
    f1 = vt[7].copy()
    f2 = vt[8].copy()
    f1 -= f2
    t0 = f1[4] * f1[8] - f1[5] * f1[7]
    t1 = f1[3] * f1[8] - f1[5] * f1[6]
    t2 = f1[3] * f1[7] - f1[4] * f1[6]
    t3 = f2[4] * f2[8] - f2[5] * f2[7]
    t4 = f2[3] * f2[8] - f2[5] * f2[6]
    t5 = f2[3] * f2[7] - f2[4] * f2[6]
    c = np.zeros(4)
    c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2
    c[1] = (f2[0] * t0 - f2[1] * t1 + f2[2] * t2
            - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7])
            + f2[4] * (f1[0] * f1[8] - f1[2] * f1[6])
            - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6])
            + f2[6] * (f1[1] * f1[5] - f1[2] * f1[4])
            - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3])
            + f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]))
    c[2] = (f1[0] * t3 - f1[1] * t4 + f1[2] * t5
            - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7])
            + f1[4] * (f2[0] * f2[8] - f2[2] * f2[6])
            - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6])
            + f1[6] * (f2[1] * f2[5] - f2[2] * f2[4])
            - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3])
            + f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]))
    c[3] = f2[0] * t3 - f2[1] * t4 + f2[2] * t5
    roots = np.roots(c)  # companion-matrix eigenvalues (leading zeros removed)
    out = []
    for r in roots:
        if abs(r.imag) > 1e-10:
            continue
        F = r.real * f1 + f2  # row-major = Eigen's column-major reshape, transposed
        if abs(F[8]) < 1e-10:
            continue
        out.append((F / F[8]).reshape(3, 3))
    return out


def fundamental_8pt(x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    n1, T1 = normalize(x1)
    n2, T2 = normalize(x2)
    _, _, vt = np.linalg.svd(f_rows(n1, n2), full_matrices=True)
    F0 = vt[8].reshape(3, 3)
    u, s, wt = np.linalg.svd(F0)
    s[2] = 0.0
    return T2.T @ (u @ np.diag(s) @ wt) @ T1


def homography_dlt(x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    s, T1 = normalize(x1)
    d, T2 = normalize(x2)
    N = len(x1)
    A = np.zeros((2 * N, 9))
    A[:N, 0] = -s[:, 0]
    A[:N, 1] = -s[:, 1]
    A[:N, 2] = -1.0
    A[:N, 6] = s[:, 0] * d[:, 0]
    A[:N, 7] = s[:, 1] * d[:, 0]
    A[:N, 8] = d[:, 0]
    A[N:, 3] = -s[:, 0]
    A[N:, 4] = -s[:, 1]
    A[N:, 5] = -1.0
    A[N:, 6] = s[:, 0] * d[:, 1]
    A[N:, 7] = s[:, 1] * d[:, 1]
    A[N:, 8] = d[:, 1]
    _, _, vt = np.linalg.svd(A, full_matrices=True)
    return np.linalg.inv(T2) @ vt[8].reshape(3, 3) @ T1


def sampson_sq(F: np.ndarray, x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    h1 = np.c_[x1, np.ones(len(x1))]
    h2 = np.c_[x2, np.ones(len(x2))]
    Fx1 = h1 @ F.T
    Ftx2 = h2 @ F
    num = (h2 * Fx1).sum(axis=1)
    return num * num / (Fx1[:, 0] ** 2 + Fx1[:, 1] ** 2 + Ftx2[:, 0] ** 2 + Ftx2[:, 1] ** 2)


def transfer_sq(H: np.ndarray, x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    p = np.c_[x1, np.ones(len(x1))] @ H.T
    d = x2 - p[:, :2] / p[:, 2:3]
    return (d * d).sum(axis=1)


def fundamental_7pt_mp(x1: np.ndarray, x2: np.ndarray, dps: int = 60) -> list[np.ndarray]:
    """The 7-point models at `dps` decimal digits (mpmath SVD null space and
    polynomial roots): the numerical truth the two double-precision
    formulations are measured against on ill-conditioned samples.  The model
    set {F : F in the null space, det F = 0, F(2,2) = 1} does not depend on
    the null-space basis."""
    import mpmath as mp
    with mp.workdps(dps):
        A = mp.matrix(f_rows(x1, x2).tolist())
        _, _, V = mp.svd_r(A, full_matrices=True)
        f2 = [V[8, k] for k in range(9)]
        f1 = [V[7, k] - f2[k] for k in range(9)]

        def det(l):
            F = [l * f1[k] + f2[k] for k in range(9)]
            return (F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6])
                    + F[2] * (F[3] * F[7] - F[4] * F[6]))
        # det(l f1 + f2) is a cubic in l: interpolate it exactly at 4 points.
        xs = [mp.mpf(v) for v in (-1, 0, 1, 2)]
        ys = [det(x) for x in xs]
        M = mp.matrix([[x ** 3, x ** 2, x, 1] for x in xs])
        c = mp.lu_solve(M, mp.matrix(ys))
        coeffs = [c[i] for i in range(4)]
        while coeffs and abs(coeffs[0]) == 0:
            coeffs.pop(0)
        roots = mp.polyroots(coeffs, maxsteps=200, extraprec=200) if len(coeffs) > 1 else []
        out = []
        for r in roots:
            if abs(mp.im(r)) > mp.mpf(10) ** (-dps // 2):
                continue
            F = [mp.re(r) * f1[k] + f2[k] for k in range(9)]
            if abs(F[8]) < 1e-10:
                continue
            out.append(np.array([float(v / F[8]) for v in F]).reshape(3, 3))
        return out
