"""C3 / C4 at 10,000 TOAs against the reference (tests/golden/j0740_10k, made by
oracle/refgen/gen_j0740_10k.py from the reference itself).

J0740+6620 (ELL1 + Shapiro, 68 DMX, FD, JUMP, EFAC/EQUAD/ECORR) on 10k synthetic TOAs -- ten
times the j0740 fixture -- fitted by the reference's GLSFitter and DownhillGLSFitter, and a
16 x 16 patch of the bench's 256 x 256 (M2, SINI) grid (indices 120..135 of each axis) by its
grid_chisq.  Bars are per fixture: 2x the reference's own spread when every one of its time
residuals is shifted by a fixed N(0, 5 ps) draw (the floor two longdouble / double-double
evaluations of the same model differ by; meta["spread"]), with 1e-3 sigma as the parameter
floor.  The fixture is checked to take the bench C3 pulsar's device path.
"""
import copy

import numpy as np
import pytest

from golden_util import load, ref_value

pytestmark = pytest.mark.gpu

NAME = "j0740_10k"


@pytest.fixture(scope="module")
def fx():
    return load(NAME)


def _bar(meta, key, floor):
    return max(floor, 2.0 * meta["spread"][key])


def test_fixture_takes_the_bench_c3_path(fx):
    """Same compact layout, vg path, binned-tile choice and k_gram_v instantiation <NTR, NTC>
    as the bench's 50k-TOA C3 pulsar (bench.py j0740_data), in one session (one N-split for
    both).  The column counts differ by the empty masks each TOA set freezes (the 10k
    reference TOAs leave 50 DMX bins and one more timing column free, the 50k ones 54)."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import j0740_data
    from pint_amd.engine import Session, build_layout, pack_table
    model, toas, z, meta = fx
    bm, bt, _ = j0740_data()
    s = Session()
    try:
        lf = s.add(build_layout(model, toas))
        lb = s.add(build_layout(bm, bt))
        s.set_instances([(lf, pack_table(lf, model)), (lb, pack_table(lb, bm))])
        ff, fb = s.fit_layout(lf), s.fit_layout(lb)
        vf, vb = s.vgram_layout(lf), s.vgram_layout(lb)
    finally:
        s.close()
    print(f"fixture fit_layout {ff} vgram {vf}; bench {fb} {vb}")
    assert ff[0] == fb[0] == 1                    # compact fit layout
    assert vf[0] == vb[0] and vf[0] & 1           # vg path, binned-tile flag
    inst = [((v[3] + 1 + v[1]) // 16, v[2] // 16) for v in (vf, vb)]
    assert inst[0] == inst[1], inst               # the same k_gram_v<NTR, NTC, VB> instantiation


def test_gls_fit_10k(fx):
    from pint_amd import GLSFitter
    model, toas, z, meta = fx
    f = GLSFitter(toas, copy.deepcopy(model))
    c2 = f.fit_toas(maxiter=1)
    worst = 0.0
    for p in meta["gls_params"]:
        s = meta["gls_errors"][p]
        d = float((np.longdouble(f.model[p].value) - ref_value(meta, "gls_params", p)) / np.longdouble(s))
        worst = max(worst, abs(d))
        assert abs(d) < max(1e-3, 2 * meta["spread"]["gls_param_sigma"][p]), (p, d)
    bar = _bar(meta, "gls_chi2_rel", 1e-8)
    print(f"GLS chi2 {c2!r} ref {meta['gls_chi2']!r} rel {c2 / meta['gls_chi2'] - 1:.2e} (bar {bar:.1e}); "
          f"worst parameter {worst:.2e} sigma")
    assert abs(c2 / meta["gls_chi2"] - 1) < bar


def test_downhill_gls_10k(fx):
    """C3's fitter (DownhillGLSFitter.fit_toas(maxiter=10), fitter.py:1015-1105) on 10k TOAs."""
    from pint_amd import DownhillGLSFitter
    from pint_amd.fitter import MaxiterReached, StepProblem
    model, toas, z, meta = fx
    f = DownhillGLSFitter(toas, copy.deepcopy(model))
    try:
        f.fit_toas(maxiter=10)
        status = "converged"
    except (MaxiterReached, StepProblem) as e:
        status = type(e).__name__
    assert status == meta["down_status"]
    bar = _bar(meta, "down_chi2_rel", 1e-8)
    rel = f.resids.chi2 / meta["down_chi2"] - 1
    worst = 0.0
    for p in meta["down_params"]:
        s = meta["down_errors"][p]
        d = float((np.longdouble(f.model[p].value) - ref_value(meta, "down_params", p)) / np.longdouble(s))
        worst = max(worst, abs(d))
        assert abs(d) < max(1e-3, 2 * meta["spread"]["down_param_sigma"][p]), (p, d)
    print(f"Downhill {status} chi2 rel {rel:.2e} (bar {bar:.1e}); worst parameter {worst:.2e} sigma")
    assert abs(rel) < bar


def test_grid_patch_10k(fx):
    """C4: the 16 x 16 (M2, SINI) patch of the bench grid, GLSFitter per point from the
    GLS-fitted model (gridutils.py:72 parallel semantics), chi2 and the extra parameter PB."""
    from pint_amd import GLSFitter
    from pint_amd.gridutils import grid_chisq
    model, toas, z, meta = fx
    g = GLSFitter(toas, copy.deepcopy(model))
    g.fit_toas(maxiter=1)
    c2, ex = grid_chisq(g, ("M2", "SINI"), (z["grid_M2"], z["grid_SINI"]), extraparnames=["PB"])
    ref = z["grid_chi2"]
    assert c2.shape == ref.shape == (16, 16)
    rel = np.abs(c2 / ref - 1)
    bar = _bar(meta, "gls_chi2_rel", 1e-8)
    print(f"grid: max chi2 rel {np.max(rel):.2e} (bar {bar:.1e}); argmin {np.unravel_index(np.argmin(c2), c2.shape)} "
          f"ref {np.unravel_index(np.argmin(ref), ref.shape)}")
    assert np.max(rel) < bar
    assert np.argmin(c2) == np.argmin(ref)
    pb_ref = z["grid_PB_hi"].astype(np.longdouble) + z["grid_PB_lo"]
    dpb = np.abs((np.asarray(ex["PB"], dtype=np.longdouble) - pb_ref) / np.longdouble(meta["gls_errors"]["PB"]))
    assert float(np.max(dpb)) < 1e-3
