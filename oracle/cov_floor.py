"""Covariance floors of the stage fixtures (TEST INFRASTRUCTURE; numpy only, no reference
import: it reads the reference's own normal matrices recorded in tests/golden/<name>_stage.npz
by oracle/refgen/gen_stage.py).  Writes tests/golden/cov_floor.json.

For an ill-conditioned GLS system (J0740: cond 7e12; B1855: 1e16 with its ECORR block) the
fitted uncertainties and correlations of two correct evaluations differ by far more than the
FP64 rounding of either solve, because the normal matrix itself is only reproducible to the
precision of its design matrix: the device's Gram matches the reference's mtcm to ~1e-13
relative to the diagonal (tests/test_gpu_stage.py, bar 1e-12).  This script measures, on the
reference's own matrix A = mtcm (timing + red-noise block, normalised):

* solver:  the reference's recorded cho_solve inverse (xvar) against A^-1 formed in numpy
           longdouble (Cholesky + triangular inverse at 64-bit mantissa);
* gram:    the spread of A^-1 when A moves by a symmetric perturbation of 1e-13 x
           sqrt(A_ii A_jj) per entry (N(0, 1) draws, seeds 1..NREP), inverted in longdouble;

each as max |sigma / sigma_exact - 1| (uncertainties, sqrt of the diagonal) and max
|corr - corr_exact| (correlation matrix).  The GPU tests bar the device's uncertainties and
correlations against the reference's at 2x (solver + gram).

Usage: python oracle/cov_floor.py [name ...]
"""
import json
import os
import sys

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
LD = np.longdouble
NREP = 4
REL = 1e-13


def chol_inv(A):
    """A^-1 of a symmetric positive-definite longdouble matrix (Cholesky, triangular inverse)."""
    K = A.shape[0]
    L = np.zeros_like(A)
    for j in range(K):
        L[j, j] = np.sqrt(A[j, j] - np.dot(L[j, :j], L[j, :j]))
        L[j + 1:, j] = (A[j + 1:, j] - L[j + 1:, :j] @ L[j, :j]) / L[j, j]
    Li = np.zeros_like(A)
    for j in range(K):
        x = np.zeros(K, dtype=LD)
        x[j] = 1 / L[j, j]
        for i in range(j + 1, K):
            x[i] = -np.dot(L[i, j:i], x[j:i]) / L[i, i]
        Li[:, j] = x
    return Li.T @ Li


def stats(X, X0):
    d, d0 = np.sqrt(np.diag(X)), np.sqrt(np.diag(X0))
    C, C0 = X / np.outer(d, d), X0 / np.outer(d0, d0)
    return float(np.max(np.abs(d / d0 - 1))), float(np.max(np.abs(C - C0)))


def floor(name):
    st = dict(np.load(os.path.join(GOLDEN, name + "_stage.npz"), allow_pickle=False))
    tri = st["mtcm_tr_triu"]
    K = int(round((np.sqrt(8 * len(tri) + 1) - 1) / 2))
    A = np.zeros((K, K), dtype=LD)
    A[np.triu_indices(K)] = tri
    A = A + A.T - np.diag(np.diag(A))
    if "mtcm_te" in st:  # ECORR block (B1855): the full system; xvar_tr is its timing+red block
        te = st["mtcm_te"].astype(LD)
        A = np.block([[A, te], [te.T, np.diag(st["mtcm_ee_diag"].astype(LD))]])
    Kf = A.shape[0]
    X0 = chol_inv(A)[:K, :K]
    Xr = st["xvar_tr"].astype(LD).reshape(K, K)
    e_s, c_s = stats(Xr, X0)
    dg = np.sqrt(np.diag(A))
    e_g = c_g = 0.0
    for rep in range(1, NREP + 1):
        g = np.random.default_rng(rep).normal(size=(Kf, Kf))
        g = np.triu(g) + np.triu(g, 1).T
        X = chol_inv(A + LD(REL) * g.astype(LD) * np.outer(dg, dg))[:K, :K]
        e, c = stats(X, X0)
        e_g, c_g = max(e_g, e), max(c_g, c)
    return {"K": K, "solver_err_rel": e_s, "solver_corr_abs": c_s, "gram_err_rel": e_g, "gram_corr_abs": c_g,
            "gram_rel": REL, "nrep": NREP}


if __name__ == "__main__":
    path = os.path.join(GOLDEN, "cov_floor.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for n in sys.argv[1:] or ["j0740", "b1855", "pta_iso", "pta_ell1", "pta_dd"]:
        out[n] = floor(n)
        print(n, out[n], flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
