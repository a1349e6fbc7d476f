"""Stage-wise parity on the GPU (SURVEY.md §8(a) parity definition 2) and the configs /
fitter outputs the end-to-end tests do not reach.

The stage fixtures (tests/golden/<name>_stage.npz, oracle/refgen/gen_stage.py) hold the
arrays the reference's GLSFitter forms inside its first iteration (fitter.py:2164-2202):
mtcm, mtcy, xhat, xvar, the column norms, phiinv, its noise realisations, and the Woodbury
chi2 of its own post-fit residuals.  The device is fed the reference's own residual arrays
(pint_debug_set_resids), so what is compared is the Gram, the solve and the chi2 stage by
stage, not the end-to-end floor of two longdouble/double-double evaluations.

Bars:
* Gram (normalised, ECORR eliminated): |dA_ij| <= 1e-12 sqrt(D_i D_j), D the Gram diagonal
  (§8(a): 1e-12 relative to the diagonal); mtcy alike; column norms 1e-12 relative.
* step, errors, covariance: 1e-9 sigma where the system allows it (the PTA fixtures, cond
  1e5 .. 1e7, measured 1e-13 .. 3e-12).  J0740 (cond 7e12) and B1855 (3e11): any FP64
  solver's rounding moves the solution by ~cond * eps, the reference's LAPACK cho_solve
  included; the test measures each solver against a longdouble solve of the system it was
  given and requires the device's error <= 3x the reference's own (and errors within 1e-3).
* chi2 of the reference's post-fit residuals: 1e-9 relative (§8(a)).
"""
import copy

import numpy as np
import pytest

from golden_util import GOLDEN, chi2_bar, load, ref_value, rms_ps

pytestmark = pytest.mark.gpu

GLS = ["pta_iso", "pta_ell1", "pta_dd", "j0740", "b1855"]


def stage(name):
    import os
    return dict(np.load(os.path.join(GOLDEN, name + "_stage.npz"), allow_pickle=False))


def ref_schur(st):
    """The reference's mtcm/mtcy with the ECORR block eliminated (its block is diagonal:
    disjoint epochs), in longdouble so the reduction adds no rounding of its own."""
    tr = st["cols_tr"]
    n = len(tr)
    A = np.zeros((n, n), dtype=np.longdouble)
    A[np.triu_indices(n)] = st["mtcm_tr_triu"]
    A = A + np.triu(A, 1).T
    b = st["mtcy"][tr].astype(np.longdouble)
    if len(st["cols_ecorr"]):
        te = st["mtcm_te"].astype(np.longdouble)
        ee = st["mtcm_ee_diag"].astype(np.longdouble)
        A = A - (te / ee) @ te.T
        b = b - te @ (st["mtcy"][st["cols_ecorr"]].astype(np.longdouble) / ee)
    return A, b


def device_stage(name, resid):
    from pint_amd.engine import Session
    from pint_amd.fitter import BatchFit
    model, toas, z, meta = load(name)
    bf = BatchFit([(model, toas)], mode="gls")
    s = bf.s
    s.eval(want_M=Session.FIT)
    s.debug_set_resids([resid])
    s.fit_step(1)
    G, colsq = s.debug_gram()[0]
    Gpre, _ = s.debug_gram(pre_ecorr=True)[0]
    dp, er, cov, _ = s.read_step()
    nr = s.noise_resids()[0]
    bf.Gpre = Gpre
    return bf, G, colsq, dp[0], er[0], cov[0], nr


@pytest.mark.parametrize("name", GLS)
def test_stage_gram_step(name):
    """Gram, mtcy, norms, step, errors and covariance of the GLS normal equations on the
    reference's own pre-fit residuals, against the reference's mtcm/mtcy/xhat/xvar."""
    model, toas, z, meta = load(name)
    st = stage(name)
    bf, G, colsq, dp, er, cov, _ = device_stage(name, z["res_time"])
    lay = bf.layouts[0]
    if name == "b1855":  # 72 DMX bins + 235 ECORR epochs on the compact layout (k_ecorr_dmx)
        assert bf.s.fit_layout(lay)[0] == 1
    tr = st["cols_tr"]
    K = lay.K
    assert K == len(tr), (K, len(tr))
    norm_ref = st["norm"][tr]
    norm = np.sqrt(colsq)
    assert np.max(np.abs(norm / norm_ref - 1)) < 1e-12  # the design matrix columns agree to ~1e-13
    # the normal matrix before the ECORR elimination, mtcm = M^T N^-1 M + diag(phiinv) as the
    # reference forms it (fitter.py:2187-2192), against the device Gram + the device's own
    # phiinv (1 / red-noise weight), both normalised; scale: mtcm's diagonal
    ntr = len(tr)
    Af = np.zeros((ntr, ntr))
    Af[np.triu_indices(ntr)] = st["mtcm_tr_triu"]
    Af = Af + np.triu(Af, 1).T
    d = np.sqrt(np.diag(Af))
    phi_dev = np.zeros(K)
    if lay.nred:
        phi_dev[len(lay.columns):] = 1.0 / np.asarray(lay.red_phi) / norm[len(lay.columns):] ** 2
    An_pre = bf.Gpre[:K, :K] / np.outer(norm, norm) + np.diag(phi_dev)
    dA = np.abs(An_pre - Af) / np.outer(d, d)
    print(f"{name}: gram max rel-diag err {dA.max():.2e}")
    assert dA.max() <= 1e-12
    rWr = bf.Gpre[K, K]
    db = np.abs(bf.Gpre[:K, K] / norm - st["mtcy"][tr]) / (d * np.sqrt(rWr))
    print(f"{name}: mtcy max err {db.max():.2e}")
    assert db.max() <= 1e-12
    A, b = ref_schur(st)
    A = A - np.diag(st["phiinv_n"][tr].astype(np.longdouble))       # the data part, ECORR eliminated
    if len(st["cols_ecorr"]):
        # the ECORR Schur term sum_e s_e s_e^T / D_e (device k_ecorr sums) against the
        # reference's mtcm_TE diag(mtcm_EE)^-1 mtcm_ET, on the same scale
        te, ee = st["mtcm_te"], st["mtcm_ee_diag"]
        Eref = (te / ee) @ te.T
        Edev = (bf.Gpre[:K, :K] - G[:K, :K]) / np.outer(norm, norm)
        dE = np.abs(Edev - Eref) / np.outer(d, d)
        print(f"{name}: ECORR Schur term max rel-diag err {dE.max():.2e}")
        assert dE.max() <= 1e-12
    # step and uncertainties (dpars = xhat / norm, fitter.py:2231-2233)
    ncol = len(lay.columns)
    dref = st["xhat"][tr] / norm_ref
    eref = np.sqrt(np.diag(st["xvar_tr"])) / norm_ref
    ds = np.abs(dp[:K] - dref) / eref
    de = np.abs(er[:K] / eref - 1)
    cref = st["xvar_tr"][:ncol, :ncol] / np.outer(norm_ref[:ncol], norm_ref[:ncol])
    dc = np.abs(cov - cref) / np.outer(eref[:ncol], eref[:ncol])
    Aph = A + np.diag(st["phiinv_n"][tr].astype(np.longdouble))
    w, _ = np.linalg.eigh(Aph.astype(np.float64))
    cond = w.max() / w.min()
    print(f"{name}: cond {cond:.1e} step {ds.max():.2e} sigma, errs {de.max():.2e}, cov {dc.max():.2e}")
    if ds.max() <= 1e-9 and de.max() <= 1e-9 and dc.max() <= 1e-9:
        bf.close()
        return
    # ill-conditioned systems (J0740 cond 7e12, B1855 3e11): split the step difference into
    # the two solvers' own rounding, each measured against a longdouble solve of the system
    # it was given -- the reference's cho_solve on its mtcm, the device's Cholesky on the
    # device Gram -- and the propagation of the (1e-13-level) Gram difference.
    x_ref_exact = ld_solve(Aph, b) / norm_ref
    # the device's normalised system, element for element as the solve kernels form it
    inv = 1.0 / norm
    Ad = G[:K, :K] * (inv[:, None] * inv[None, :])
    if lay.nred:
        r0 = len(lay.columns)
        Ad[np.arange(r0, K), np.arange(r0, K)] += (inv[r0:] * inv[r0:]) / np.asarray(lay.red_phi)
    bd = G[:K, K] * inv
    x_dev_exact = ld_solve(Ad, bd) * inv
    e_ref = np.max(np.abs(dref - x_ref_exact) / eref)
    e_dev = np.max(np.abs(dp[:K] - x_dev_exact) / eref)
    e_in = np.max(np.abs(x_dev_exact - x_ref_exact) / eref)
    print(f"{name}: solver rounding: reference cho_solve {e_ref:.2e} sigma, device {e_dev:.2e} sigma; "
          f"Gram difference propagated {e_in:.2e} sigma")
    assert e_dev <= max(1e-9, 3 * e_ref), (e_dev, e_ref)
    # the covariance decomposed the same way: each side's inverse against the longdouble
    # inverse of the system it was given (the reference's cho_solve(c, I) of its mtcm, the
    # device's Cholesky inverse of the device Gram), in units of sigma_i sigma_j
    ncol = len(lay.columns)
    Xref = ld_inverse(Aph)[:ncol, :ncol] / np.outer(norm_ref[:ncol], norm_ref[:ncol])
    Xdev = ld_inverse(Ad)[:ncol, :ncol] * np.outer(inv[:ncol], inv[:ncol])
    ee = np.outer(eref[:ncol], eref[:ncol])
    c_ref = float(np.max(np.abs(cref - Xref) / ee))
    c_dev = float(np.max(np.abs(cov - Xdev) / ee))
    c_in = float(np.max(np.abs(Xdev - Xref) / ee))
    print(f"{name}: covariance rounding: reference {c_ref:.2e}, device {c_dev:.2e}; Gram difference "
          f"propagated {c_in:.2e} (sigma_i sigma_j)")
    # measured on MI355X: J0740 (cond 7e12) reference 5.6e-5, device 6.4e-4, Gram difference
    # propagated 1.7e-3.  The device's FP64 Cholesky inverse (no refinement of the inverse,
    # unlike the step) carries more rounding than LAPACK's, but below what the 1e-15-level
    # Gram difference between the two sides already moves the covariance by: the device's
    # own rounding must stay under the larger of 3x the reference's and that input floor.
    assert c_dev <= max(1e-9, 3 * c_ref, c_in), (c_dev, c_ref, c_in)
    assert de.max() <= 1e-3 and dc.max() <= 5e-3
    bf.close()


def ld_inverse(A):
    """Gauss-Jordan inverse with partial pivoting in longdouble."""
    A = np.array(A, dtype=np.longdouble)
    n = len(A)
    M = np.concatenate([A, np.eye(n, dtype=np.longdouble)], axis=1)
    for k in range(n):
        p = k + int(np.argmax(np.abs(M[k:, k])))
        if p != k:
            M[[k, p]] = M[[p, k]]
        M[k] /= M[k, k]
        f = M[:, k].copy()
        f[k] = 0
        M -= np.outer(f, M[k])
    return M[:, n:]


def ld_solve(A, b):
    """Gaussian elimination with partial pivoting in longdouble (numpy's solvers drop to
    float64): the reference solution of a stage's linear system."""
    A = np.array(A, dtype=np.longdouble)
    b = np.array(b, dtype=np.longdouble)
    n = len(b)
    for k in range(n):
        p = k + int(np.argmax(np.abs(A[k:, k])))
        if p != k:
            A[[k, p]] = A[[p, k]]
            b[[k, p]] = b[[p, k]]
        f = A[k + 1:, k] / A[k, k]
        A[k + 1:, k:] -= np.outer(f, A[k, k:])
        b[k + 1:] -= f * b[k]
    x = np.zeros(n, dtype=np.longdouble)
    for k in range(n - 1, -1, -1):
        x[k] = (b[k] - A[k, k + 1:] @ x[k + 1:]) / A[k, k]
    return x


@pytest.mark.parametrize("name", GLS)
def test_stage_chi2_reference_resids(name):
    """The Woodbury GLS chi2 and log-normalisation of the reference's own post-fit residuals
    (residuals.py:567-589), fed to the device: 1e-9 relative (§8(a))."""
    model, toas, z, meta = load(name)
    st = stage(name)
    from pint_amd.engine import Session
    from pint_amd.fitter import BatchFit
    bf = BatchFit([(model, toas)], mode="gls")
    s = bf.s
    s.eval(want_M=Session.FIT)
    s.fit_step(1)                       # Sigma factor (noise basis only)
    s.debug_set_resids([st["post_resid"]])
    c2 = s.chi2_gls()[0]
    if not bf.use_gls_chi2[0]:          # no basis columns: the offset-only Woodbury form
        c2 = s.chi2_gls()[0]
    rel = abs(c2 / st["post_chi2"][0] - 1)
    print(f"{name}: chi2 {c2:.12f} ref {st['post_chi2'][0]:.12f} rel {rel:.2e}")
    assert rel <= 1e-9
    kind = 1 if bf.use_gls_chi2[0] else 2
    ln = s.lognorm(kind)[0]
    assert abs(ln - st["post_lognorm"][0]) <= 1e-9 * abs(st["post_lognorm"][0])
    bf.close()


@pytest.mark.parametrize("name", GLS)
def test_stage_noise_resids(name):
    """Noise realisations (fitter.py:2270-2282) of the step on the reference's residuals
    against the reference's, per component."""
    model, toas, z, meta = load(name)
    st = stage(name)
    bf, G, colsq, dp, er, cov, nr = device_stage(name, z["res_time"])
    want = {k[len("noise_resid_"):]: v for k, v in st.items() if k.startswith("noise_resid_")}
    assert set(nr) == set(want), (set(nr), set(want))
    for k, v in want.items():
        scale = max(np.max(np.abs(v)), 1e-30)
        err = np.max(np.abs(nr[k] - v)) / scale
        print(f"{name}: noise {k} max err {err:.2e} of {scale:.2e} s")
        assert err <= TOL_NOISE[name], (k, err)
    bf.close()


# the realisations are M_n @ xhat_n: the noise coefficients inherit the step's conditioning
TOL_NOISE = {"pta_iso": 1e-8, "pta_ell1": 1e-8, "pta_dd": 1e-8, "j0740": 1e-8, "b1855": 1e-5}


@pytest.mark.parametrize("name", ["pta_dd", "b1855"])
def test_fitter_noise_resids_and_update_model(name):
    """GLSFitter.fit_toas end to end: resids.noise_resids (fitter.py:2270-2282) and
    update_model (fitter.py:530-555) against the reference's fit of the same data."""
    from pint_amd import GLSFitter
    model, toas, z, meta = load(name)
    st = stage(name)
    f = GLSFitter(toas, model)
    c2 = f.fit_toas(maxiter=1)
    for k in [k for k in st if k.startswith("noise_resid_")]:
        comp = k[len("noise_resid_"):]
        v = st[k]
        err = np.max(np.abs(f.resids.noise_resids[comp] - v)) / np.max(np.abs(v))
        print(f"{name}: fitter noise {comp} rel err {err:.2e}")
        assert err < 1e-3
    um = dict(zip([str(x) for x in st["update_model_keys"]], st["update_model_vals"]))
    assert f.model.NTOA.value == int(um["NTOA"])
    assert float(f.model.START.value) == um["START"] and float(f.model.FINISH.value) == um["FINISH"]
    # end-to-end: 2x the reference's chi2 spread at the measured post-fit residual rms
    bar = chi2_bar(name, "fit", rms_ps(f.resids.time_resids, st["post_resid"]) if "post_resid" in st else 30.0)
    assert abs(f.model.CHI2.value / um["CHI2"] - 1) < bar
    assert abs(f.model.CHI2R.value / um["CHI2R"] - 1) < bar
    # TRES is the weighted rms of the post-fit residuals: end-to-end, so at the ~ps floor of
    # two longdouble/double-double evaluations (tests/test_oracle_golden.py::test_gls_fit)
    assert abs(f.model.TRES.value / um["TRES"] - 1) < 1e-5
    assert f.model.DMDATA.value is False


def test_compact_ecorr_matches_full_layout():
    """B1855 (72 DMX bins, 235 ECORR epochs): the compact layout (DMX as bin sums, the ECORR
    elimination's DMX share in k_ecorr_dmx) and the full layout (DMX columns in M) solve the
    same normal equations: step, errors, covariance, GLS chi2 and the ECORR realisations agree
    to rounding."""
    from pint_amd.engine import Session
    from pint_amd.fitter import BatchFit
    model, toas, z, meta = load("b1855")
    out = {}
    for key, want in (("compact", Session.FIT), ("full", True)):
        bf = BatchFit([(model, toas)], mode="gls")
        s = bf.s
        s.eval(want_M=want)
        assert s.fit_layout(bf.layouts[0])[0] == 1
        s.debug_set_resids([z["res_time"]])
        s.fit_step(1)
        dp, er, cov, _ = s.read_step()
        nr = s.noise_resids()[0]
        c2 = s.chi2_gls()[0]
        G, _ = s.debug_gram(pre_ecorr=True)[0]
        K = bf.layouts[0].K
        out[key] = (dp[0][:K], er[0][:K], cov[0], nr, c2, G)
        bf.close()
    dc, ec, cc, nc, c2c, Gc = out["compact"]
    df, ef, cf, nf, c2f, Gf = out["full"]
    d = np.sqrt(np.diag(Gf)[:K])
    print(f"b1855 compact vs full: gram {np.max(np.abs(Gc - Gf)[:K, :K] / np.outer(d, d)):.1e} "
          f"step {np.max(np.abs(dc - df) / ef):.1e} errs {np.max(np.abs(ec / ef - 1)):.1e} "
          f"chi2 {abs(c2c / c2f - 1):.1e}")
    assert np.max(np.abs(Gc - Gf)[:K, :K] / np.outer(d, d)) < 1e-12
    # the Grams agree to rounding, but B1855's normal matrix has cond ~3e11: the two layouts'
    # solves (k_solve_dmx on the DMX-eliminated system, k_solve_blk on the full one) differ by
    # ~cond x eps (measured 1.1e-5 sigma in the step, 1.2e-5 in the errors)
    assert np.max(np.abs(dc - df) / ef) < 1e-4
    assert np.max(np.abs(ec / ef - 1)) < 1e-4
    assert np.max(np.abs(cc - cf) / np.outer(ef[:len(cc)], ef[:len(cc)])) < 1e-4
    assert abs(c2c / c2f - 1) < 1e-9
    for k in nf:
        assert np.max(np.abs(nc[k] - nf[k])) <= 1e-6 * np.max(np.abs(nf[k])) + 1e-15, k


def test_full_cov_matches_rank_reduced():
    """GLSFitter(full_cov=True) gives the rank-reduced result (the reference asserts the
    equality, tests/test_gls_fitter.py:85-90) and no noise realisations."""
    from pint_amd import GLSFitter
    model, toas, z, meta = load("pta_dd")
    a = GLSFitter(toas, copy.deepcopy(model))
    ca = a.fit_toas(full_cov=False)
    b = GLSFitter(toas, copy.deepcopy(model))
    cb = b.fit_toas(full_cov=True)
    assert ca == cb
    assert b.resids.noise_resids == {} and "pl_red_noise" in a.resids.noise_resids
    for p in model.free_params:
        assert a.model[p].value == b.model[p].value


def test_downhill_gls_j0740():
    """C3: DownhillGLSFitter on J0740 (ELL1 + Shapiro, ecliptic, DMX, FD, JUMP; ECORR with
    one TOA per epoch) against the reference's down_* fixture."""
    from pint_amd import DownhillGLSFitter
    from pint_amd.fitter import MaxiterReached, StepProblem
    model, toas, z, meta = load("j0740")
    f = DownhillGLSFitter(toas, model)
    try:
        f.fit_toas(maxiter=10)
        status = "converged"
    except (MaxiterReached, StepProblem) as e:
        status = type(e).__name__
    assert status == meta["down_status"]
    rel = abs(f.resids.chi2 / meta["down_chi2"] - 1)
    worst = 0.0
    for p in meta["down_params"]:
        s = meta["down_errors"][p]
        d = float((np.longdouble(f.model[p].value) - ref_value(meta, "down_params", p)) / np.longdouble(s))
        worst = max(worst, abs(d))
    from pint_amd import Residuals
    bar = chi2_bar("j0740", "down", rms_ps(Residuals(toas, model).time_resids, z["res_time"]))
    print(f"j0740 downhill: chi2 rel {rel:.2e} (bar {bar:.1e}), worst param {worst:.2e} sigma")
    assert rel < bar
    assert worst < 1e-3


def test_grid_m2_sini_j0740():
    """C4 second shape: grid_chisq over (M2, SINI) on J0740, GLSFitter per point, from the
    reference's own post-fit model, against the reference's parallel (cold-start) grid, with
    the extra parameter PB meshgrid-shaped."""
    from pint_amd import GLSFitter
    from pint_amd.gridutils import grid_chisq
    model, toas, z, meta = load("j0740")
    st = stage("j0740")
    for p, h, l in zip(st["grid_base_params"], st["grid_base_hi"], st["grid_base_lo"]):
        model[str(p)].value = np.longdouble(h) + np.longdouble(l)
    f = GLSFitter(toas, model)
    m2, sini = st["grid_M2"], st["grid_SINI"]
    c2, ex = grid_chisq(f, ("M2", "SINI"), (m2, sini), extraparnames=["PB"])
    ref = st["grid_chi2_parallel"]
    assert c2.shape == ref.shape and ex["PB"].shape == ref.shape
    rel = np.max(np.abs(c2 / ref - 1))
    pb_ref = st["grid_PB_parallel_hi"] + st["grid_PB_parallel_lo"]
    dpb = np.max(np.abs(ex["PB"] - pb_ref))
    print(f"j0740 (M2,SINI) grid: chi2 max rel {rel:.2e}; PB max abs {dpb:.2e} d")
    # each point's chi2 is a post-fit chi2: end-to-end, so at the floor of test_gls_fit (2x
    # the reference's fit chi2 spread at the measured residual rms, golden_util.chi2_bar)
    from pint_amd import Residuals
    m0 = load("j0740")[0]  # the fixture's own model (model above holds the grid's base values)
    assert rel < chi2_bar("j0740", "fit", rms_ps(Residuals(toas, m0).time_resids, z["res_time"]))
    assert np.unravel_index(np.argmin(c2), c2.shape) == np.unravel_index(np.argmin(ref), ref.shape)
    # serial (warm start) and parallel (cold start) differ in the reference itself
    print("reference serial vs parallel:", np.max(np.abs(st["grid_chi2_serial"] / ref - 1)))


def test_device_grid_tables_match_host_tables():
    """pint_set_grid's point tables (formed on the device from the base table and the grid
    axes, k_grid_tables) equal the host restatement (golden_util.grid_tables) bit for bit:
    a meshgrid block starting inside the grid (k0 > 0) and a list of per-point values."""
    from golden_util import grid_tables
    from pint_amd.engine import Session, build_layout, pack_table
    from pint_amd.gridutils import meshgrid_axes
    model, toas, _, _ = load("ngc6440e")
    s = Session()
    lay = s.add(build_layout(model, toas))
    base = pack_table(lay, model)
    F0, F1 = np.longdouble(model.F0.value), np.longdouble(model.F1.value)
    g0 = F0 + np.linspace(-3, 3, 17, dtype=np.longdouble) * np.longdouble(1e-11)
    g1 = F1 + np.linspace(-3, 3, 13, dtype=np.longdouble) * np.longdouble(1e-19)
    axes, npts = meshgrid_axes((g0, g1))
    var = [(p, a, st, sz) for p, (a, st, sz) in zip(("F0", "F1"), axes)]
    for grid in ((base, var, npts - 40, 40),
                 (base, [("DM", np.linspace(10, 11, 9, dtype=np.longdouble), 1, 9)], 9, 0)):
        s.set_grid(lay, *grid)
        got = s.read_tables_flat().reshape(grid[2], lay.tstride)
        np.testing.assert_array_equal(got, grid_tables(lay, grid))
    s.close()


@pytest.mark.parametrize("name,fitter", [("ngc6440e", "WLSFitter"), ("pta_dd", "GLSFitter")])
def test_resident_grid_batch_matches_fresh(name, fitter):
    """A grid over the same pulsar and point count as the resident batch reuses its instance
    arrays, launch groups and buffers (pint_set_grid's fast path, only the tables formed
    anew): the second grid equals the same grid in a fresh session bit for bit, after a first
    grid with other values, and after a grid with an invalid point (whose batch was re-bound
    without it)."""
    import pint_amd
    from pint_amd import gridutils
    from pint_amd.gridutils import grid_chisq
    model, toas = load(name)[:2]
    f = getattr(pint_amd, fitter)(toas, copy.deepcopy(model))
    f.fit_toas(maxiter=1)
    F0, F1 = np.longdouble(f.model.F0.value), np.longdouble(f.model.F1.value)
    s0, s1 = np.longdouble(f.model.F0.uncertainty), np.longdouble(f.model.F1.uncertainty)
    ga = (F0 + np.linspace(-2, 2, 6) * s0, F1 + np.linspace(-2, 2, 5) * s1)
    gb = (F0 + np.linspace(-3, 1, 6) * s0, F1 + np.linspace(-1, 3, 5) * s1)
    extra = ["DM"]
    gridutils._drop_grid_session()
    grid_chisq(f, ("F0", "F1"), ga, extraparnames=extra)
    c_res, e_res = grid_chisq(f, ("F0", "F1"), gb, extraparnames=extra)
    gridutils._drop_grid_session()
    c_new, e_new = grid_chisq(f, ("F0", "F1"), gb, extraparnames=extra)
    np.testing.assert_array_equal(c_res, c_new)
    np.testing.assert_array_equal(e_res["DM"], e_new["DM"])


@pytest.mark.parametrize("name", ["ngc6440e", "pta_iso"])
def test_spin_grid_eval_matches_full(name):
    """A grid whose points differ in F0 and F1 only (pint_set_grid, isolated model) evaluates
    its first design matrix with the shared head (k_eval_head: every row's delay, astrometric
    geometry and dispersion factors once) and each point's spin part (k_eval_spin): the
    phases, Taylor frequencies, delays and design matrix equal the full per-point evaluation
    (PINT_OPT_SPIN_EVAL off) bit for bit, and so do the fitted steps.  pta_iso (red noise) is
    outside the shared path and must take the full evaluation either way."""
    from pint_amd.engine import Session, build_layout, pack_table
    model, toas = load(name)[:2]

    def run(spin):
        s = Session()
        s.set_spin_eval(spin)
        lay = s.add(build_layout(model, toas))
        base = pack_table(lay, model)
        F0, F1 = np.longdouble(model.F0.value), np.longdouble(model.F1.value)
        g0 = F0 + np.linspace(-2, 2, 7) * np.longdouble(1e-10)
        g1 = F1 + np.linspace(-2, 2, 11) * np.longdouble(1e-18)
        s.set_grid(lay, base, [("F0", g0, 11, 7), ("F1", g1, 1, 11)], 77)
        s.eval(want_M=Session.FIT)
        ev = s.read_eval()
        # (the compact vg layout of pta_iso stores no Fourier columns: its M buffer is read
        # only where written, through the fit below)
        M = s.read_designmatrix() if name == "ngc6440e" else []
        s.fit_step(0)
        dp, er, _, cl = s.read_step()
        out = [np.array(x, copy=True) for x in ev] + [np.array(M, copy=True)]
        out += [np.array(x, copy=True) for x in dp] + [np.array(cl, copy=True)]
        s.close()
        return out

    a, b = run(True), run(False)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_chunked_grid_matches_one_batch(monkeypatch):
    """A grid fitted in equal chunks (the resident batch re-bound per chunk: pint_set_grid's
    fast path) and a last smaller one (a fresh set-up) equals the same grid as one batch, bit
    for bit (62-row points: one N-split whatever the batch size)."""
    from pint_amd import WLSFitter, gridutils
    from pint_amd.gridutils import grid_chisq
    model, toas = load("ngc6440e")[:2]
    f = WLSFitter(toas, copy.deepcopy(model))
    f.fit_toas(maxiter=1)
    F0, F1 = np.longdouble(f.model.F0.value), np.longdouble(f.model.F1.value)
    g = (F0 + np.linspace(-2, 2, 6) * np.longdouble(f.model.F0.uncertainty),
         F1 + np.linspace(-2, 2, 5) * np.longdouble(f.model.F1.uncertainty))
    gridutils._drop_grid_session()
    c_one, e_one = grid_chisq(f, ("F0", "F1"), g, extraparnames=["DM"])
    monkeypatch.setattr(gridutils, "GRID_MAX_POINTS", 7)  # 30 points: 7, 7, 7, 7, 2
    c_ch, e_ch = grid_chisq(f, ("F0", "F1"), g, extraparnames=["DM"])
    np.testing.assert_array_equal(c_ch, c_one)
    np.testing.assert_array_equal(e_ch["DM"], e_one["DM"])


@pytest.mark.parametrize("npipe", [2, 3])
def test_grid_pipelines_match_one_session(monkeypatch, npipe):
    """A grid split over concurrent sessions (gridutils.GRID_PIPES: contiguous blocks, each
    enqueued on its own session before any is waited on) equals the grid on one session, bit
    for bit, chi2 and extra parameters (62-row points: one N-split whatever the block)."""
    from pint_amd import WLSFitter, gridutils
    from pint_amd.gridutils import grid_chisq
    model, toas = load("ngc6440e")[:2]
    f = WLSFitter(toas, copy.deepcopy(model))
    f.fit_toas(maxiter=1)
    F0, F1 = np.longdouble(f.model.F0.value), np.longdouble(f.model.F1.value)
    g = (F0 + np.linspace(-2, 2, 7) * np.longdouble(f.model.F0.uncertainty),
         F1 + np.linspace(-2, 2, 5) * np.longdouble(f.model.F1.uncertainty))
    gridutils._drop_grid_session()
    monkeypatch.setattr(gridutils, "GRID_PIPES", 1)
    c_one, e_one = grid_chisq(f, ("F0", "F1"), g, extraparnames=["DM"])
    monkeypatch.setattr(gridutils, "GRID_PIPES", npipe)
    monkeypatch.setattr(gridutils, "GRID_PIPE_MIN", 4)  # 35 points over npipe sessions
    c_p, e_p = grid_chisq(f, ("F0", "F1"), g, extraparnames=["DM"])
    assert len(gridutils._GRID["cur"][1]) == npipe
    np.testing.assert_array_equal(c_p, c_one)
    np.testing.assert_array_equal(e_p["DM"], e_one["DM"])
    gridutils._drop_grid_session()


def test_invalid_grid_point_fails_alone():
    """A grid over the DD eccentricity that includes ECC >= 1: those points are NaN (the
    reference's doonefit returns NaN for the failed fit, gridutils.py:89-106) and every other
    point equals its own single fit -- the invalid points do not touch the batch."""
    from pint_amd import GLSFitter
    from pint_amd.gridutils import grid_chisq
    model, toas, z, meta = load("pta_dd")
    e0 = float(model.ECC.value)
    eccs = np.array([e0, e0 * (1 + 1e-9), 1.2, e0 * (1 - 1e-9), 1.5])
    f = GLSFitter(toas, copy.deepcopy(model))
    c2, ex = grid_chisq(f, ("ECC",), (eccs,), extraparnames=["OM"])
    assert np.isnan(c2[2]) and np.isnan(c2[4]) and np.isnan(ex["OM"][2])
    for k in (0, 1, 3):
        m = copy.deepcopy(model)
        m.ECC.value = eccs[k]
        m.ECC.frozen = True
        g = GLSFitter(toas, m)
        want = g.fit_toas()
        assert abs(c2[k] / want - 1) < 1e-12, (k, c2[k], want)


def test_invalid_single_fit_raises():
    from pint_amd import GLSFitter
    from pint_amd.fitter import InvalidModelParameters
    model, toas, z, meta = load("pta_dd")
    model.ECC.value = 1.3
    with pytest.raises((InvalidModelParameters, ValueError)):
        GLSFitter(toas, model).fit_toas()
