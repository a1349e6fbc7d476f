"""Golden fixtures for the synthetic configs (reference run; container only).

* j0740  : profiling/J0740+6620.par (ELL1, ecliptic+PM, FD1, DMX, EFAC/EQUAD/ECORR, JUMP),
           EPHEM->builtin, CLK->TT(TAI), TZRSITE->geocenter, make_fake_toas_uniform
           (N=1000, 820/1400 MHz alternating, geocenter), receivers assigned by freq,
           re-zeroed (simulation.py:125 make_fake_toas). DownhillGLS + GLS. (C3 shape)
* pta_*  : the C5 per-pulsar template: equatorial + PM + PX, F0/F1,
           DM/DM1/DM2, DMX bins, PLRedNoise, EFAC/EQUAD; isolated / ELL1 / DD variants,
           N=1000, 4 frequencies alternating, geocenter, add_noise + add_correlated_noise.
Usage: run_ref.sh gen_synth.py [name ...]
"""
import copy
import io
import sys

import numpy as np
import astropy.units as u

from refcommon import (REFPROF, register_clockless_sites, pack_toas, export_model, mask_table,
                       component_delays, phase_outputs, residual_outputs, designmatrix_outputs,
                       noise_outputs, split_ld, save)
import pint.simulation as sim
from pint.models import get_model
from pint.fitter import GLSFitter, DownhillGLSFitter, DownhillWLSFitter, WLSFitter


def j0740_model():
    lines = []
    for line in open(f"{REFPROF}/J0740+6620.par"):
        k = line.split()[0] if line.split() else ""
        if k in ("EPHEM",):
            line = "EPHEM builtin\n"
        elif k == "CLK":
            line = "CLK TT(TAI)\n"
        elif k == "TZRSITE":
            line = "TZRSITE geocenter\n"
        lines.append(line)
    return get_model(io.StringIO("".join(lines)))


def pta_par(seed, binary, ndmx=20):
    rng = np.random.default_rng(1000 + seed)
    ra = rng.uniform(0, 2 * np.pi)
    dec = np.arcsin(rng.uniform(-1, 1))
    rah = ra * 12 / np.pi
    h = int(rah); m = int((rah - h) * 60); s = ((rah - h) * 60 - m) * 60
    dd = np.degrees(abs(dec)); dg = int(dd); dm_ = int((dd - dg) * 60); ds = ((dd - dg) * 60 - dm_) * 60
    sign = "-" if dec < 0 else "+"
    F0 = rng.uniform(100, 700)
    F1 = -1e-15 * F0 / 300
    DM = rng.uniform(5, 100)
    par = f"""PSR J{seed:04d}+SYN
RAJ {h:02d}:{m:02d}:{s:011.8f} 1
DECJ {sign}{dg:02d}:{dm_:02d}:{ds:010.7f} 1
PMRA {rng.normal(0, 5):.4f} 1
PMDEC {rng.normal(0, 5):.4f} 1
PX 1.0 1
POSEPOCH 54800
F0 {F0:.15f} 1
F1 {F1:.6e} 1
PEPOCH 54800
DM {DM:.6f}
DM1 0.0001 1
DM2 0.00001 1
DMEPOCH 54800
EPHEM builtin
CLK TT(TAI)
UNITS TDB
TZRMJD 54800.1234
TZRFRQ 1400
TZRSITE geocenter
EFAC -f fake 1.1
EQUAD -f fake 0.1
TNRedAmp {rng.uniform(-14.5, -13.5):.4f}
TNRedGam {rng.uniform(3, 5):.4f}
TNRedC 30
"""
    edges = np.linspace(53000, 56652.01, ndmx + 1)
    par += "DMX 14.0\n"
    for i in range(ndmx):
        par += f"DMX_{i+1:04d} {rng.normal(0, 1e-3):.6e} 1\nDMXR1_{i+1:04d} {edges[i]:.5f}\nDMXR2_{i+1:04d} {edges[i+1]:.5f}\n"
    if binary == "ELL1":
        par += f"""BINARY ELL1
A1 {rng.uniform(1, 20):.9f} 1
PB {rng.uniform(1, 30):.12f} 1
TASC 54801.123456789 1
EPS1 {rng.normal(0, 1e-5):.6e} 1
EPS2 {rng.normal(0, 1e-5):.6e} 1
M2 0.25
SINI 0.95
"""
    elif binary.startswith("ELL1H"):
        # binary_ell1.py:312-417 (Freire & Wex 2010): H3 alone, H3 + H4, or H3 + STIGMA
        extra = {"ELL1H_H3": "NHARMS 3\n", "ELL1H_H4": "H4 3.1e-7 1\nNHARMS 8\n",
                 "ELL1H_STIG": "STIGMA 0.6 1\n"}[binary]
        par += f"""BINARY ELL1H
A1 {rng.uniform(1, 20):.9f} 1
PB {rng.uniform(1, 30):.12f} 1
TASC 54801.123456789 1
EPS1 {rng.normal(0, 1e-5):.6e} 1
EPS2 {rng.normal(0, 1e-5):.6e} 1
H3 5.2e-7 1
""" + extra
    elif binary == "BT":
        par += f"""BINARY BT
A1 {rng.uniform(5, 30):.9f} 1
PB {rng.uniform(5, 60):.12f} 1
T0 54801.987654321 1
ECC {rng.uniform(0.05, 0.4):.8f} 1
OM {rng.uniform(0, 360):.6f} 1
OMDOT 0.01 1
GAMMA 0.0004 1
PBDOT 1e-12 1
"""
    elif binary.startswith("DDK"):
        # binary_ddk.py / DDK_model.py: KIN/KOM replace SINI; Kopeikin (1995) annual-orbital
        # parallax and (1996) proper-motion terms on a1, omega and i; K96 N drops the latter
        par += f"""BINARY DDK
A1 {rng.uniform(5, 30):.9f} 1
PB {rng.uniform(5, 60):.12f} 1
T0 54801.987654321 1
ECC {rng.uniform(0.05, 0.4):.8f} 1
OM {rng.uniform(0, 360):.6f} 1
OMDOT 0.01 1
M2 0.3 1
KIN {rng.uniform(50, 80):.6f} 1
KOM {rng.uniform(0, 360):.6f} 1
""" + ("K96 N\n" if binary == "DDK_NK" else "")
    elif binary == "DD":
        par += f"""BINARY DD
A1 {rng.uniform(5, 30):.9f} 1
PB {rng.uniform(5, 60):.12f} 1
T0 54801.987654321 1
ECC {rng.uniform(0.05, 0.4):.8f} 1
OM {rng.uniform(0, 360):.6f} 1
OMDOT 0.01 1
M2 0.3 1
SINI 0.9 1
GAMMA 0.0
"""
    return par


def capture(name, model, toas, fit="gls", n_dm_rows=None):
    arr, flags = pack_toas(toas)
    tz = model.get_TZR_toa(toas)
    tza, _ = pack_toas(tz)
    arrays = dict(arr)
    arrays.update({"tzr_" + k: v for k, v in tza.items()})
    arrays.update(mask_table(model, toas))
    arrays.update(component_delays(model, toas))
    arrays.update(phase_outputs(model, toas))
    r, ra, rm = residual_outputs(model, toas)
    arrays.update(ra)
    dm, dmm = designmatrix_outputs(model, toas)
    arrays.update(dm)
    no, nm = noise_outputs(model, toas)
    arrays.update(no)
    meta = {"name": name, "model": export_model(model), "flags": flags}
    obs = [str(o) for o in toas.get_obss()]
    meta["obs_names"] = sorted(set(obs))
    arrays["obs_index"] = np.array([meta["obs_names"].index(o) for o in obs], dtype=np.int16)
    from pint.observatory import get_observatory
    meta["obs_aliases"] = {o: list(get_observatory(o).aliases) for o in meta["obs_names"]}
    meta.update(rm)
    meta.update(dmm)
    meta.update(nm)
    # ssb->psb direction vectors (erfa pmsafe / SkyCoord path) at the TOA epochs
    arrays["psr_dir_icrs"] = np.asarray(model.ssb_to_psb_xyz_ICRS(
        epoch=toas.table["tdbld"].astype(np.float64)), dtype=np.float64)
    if fit == "gls":
        f = GLSFitter(toas, copy.deepcopy(model))
        chi2 = f.fit_toas(maxiter=1)
        meta["gls_chi2"] = float(chi2)
        meta["gls_params"] = {p: list(map(float, split_ld(getattr(f.model, p).value)))
                              for p in f.model.free_params}
        meta["gls_errors"] = {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}
        arrays["gls_cov"] = np.asarray(f.parameter_covariance_matrix.matrix, dtype=np.float64)
        arrays["gls_fac"] = np.asarray(f.fac, dtype=np.float64)
        arrays["gls_post_resid"] = np.asarray(f.resids.time_resids.to_value(u.s))
        for k, v in f.resids.noise_resids.items():
            arrays["gls_noise_" + k] = np.asarray(v.to_value(u.s))
        fd = DownhillGLSFitter(toas, copy.deepcopy(model))
    else:
        f = WLSFitter(toas, copy.deepcopy(model))
        chi2 = f.fit_toas(maxiter=1)
        meta["wls_chi2"] = float(chi2)
        meta["wls_params"] = {p: list(map(float, split_ld(getattr(f.model, p).value)))
                              for p in f.model.free_params}
        meta["wls_errors"] = {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}
        fd = DownhillWLSFitter(toas, copy.deepcopy(model))
    try:
        fd.fit_toas(maxiter=10)
        meta["down_status"] = "converged"
    except Exception as e:  # MaxiterReached / StepProblem: record like grid_chisq does
        meta["down_status"] = type(e).__name__
    meta["down_chi2"] = float(fd.resids.chi2)
    meta["down_converged"] = bool(fd.converged)
    meta["down_params"] = {p: list(map(float, split_ld(getattr(fd.model, p).value)))
                           for p in fd.model.free_params}
    meta["down_errors"] = {p: float(getattr(fd.model, p).uncertainty_value) for p in fd.model.free_params}
    save(name, arrays, meta)


def gen_j0740(n=1000):
    np.random.seed(0)
    model = j0740_model()
    ts = sim.make_fake_toas_uniform(56640, 58461, n, model, freq=np.array([820, 1400]) * u.MHz,
                                    obs="geocenter", error=1 * u.us, add_noise=False,
                                    include_bipm=False, multi_freqs_in_epoch=False,
                                    flags={"f": "Rcvr1_2_GUPPI", "fe": "Rcvr1_2"})
    for fl, fr in zip(ts.table["flags"], ts.table["freq"]):
        if fr < 1000:
            fl["f"] = "Rcvr_800_GUPPI"
            fl["fe"] = "Rcvr_800"
    ts = sim.make_fake_toas(ts, model, add_noise=True)
    model.find_empty_masks(ts, freeze=True)
    capture("j0740", model, ts, fit="gls")


extra_name = None


def _par(seed, binary, extra):
    par = pta_par(seed, binary)
    if "TNDMAMP" in extra:  # PLDMNoise models DM variations in place of DMX (noise_model.py:443)
        par = "\n".join(l for l in par.splitlines() if not l.startswith("DMX")) + "\n"
    return par + extra


def gen_pta(seed, binary, n=1000, extra=""):
    np.random.seed(seed)
    model = get_model(io.StringIO(_par(seed, binary, extra)))
    ts = sim.make_fake_toas_uniform(53000, 56652, n, model,
                                    freq=np.array([800, 1200, 1600, 2000]) * u.MHz,
                                    obs="geocenter", error=0.5 * u.us, add_noise=True,
                                    add_correlated_noise=True, include_bipm=False,
                                    multi_freqs_in_epoch=False)
    model.find_empty_masks(ts, freeze=True)
    name = {"": "pta_iso", "ELL1": "pta_ell1", "DD": "pta_dd", "ELL1H_H3": "ell1h_h3", "ELL1H_H4": "ell1h_h4",
            "ELL1H_STIG": "ell1h_stig", "BT": "pta_bt",
            "DDK": "pta_ddk", "DDK_NK": "pta_ddk_nk"}[binary] if not extra else extra_name
    with open(__import__("os").path.join(__import__("refcommon").GOLDEN, name + ".par"), "w") as f:
        f.write(_par(seed, binary, extra))
    capture(name, model, ts, fit="gls")


if __name__ == "__main__":
    register_clockless_sites()
    which = sys.argv[1:] or ["j0740", "pta_iso", "pta_ell1", "pta_dd"]
    if "j0740" in which:
        gen_j0740()
    if "pta_iso" in which:
        gen_pta(1, "")
    if "pta_ell1" in which:
        gen_pta(2, "ELL1")
    if "pta_dd" in which:
        gen_pta(3, "DD")
    if "pta_bt" in which:
        gen_pta(14, "BT")
    if "pta_ddk" in which:
        gen_pta(16, "DDK")
    if "pta_ddk_nk" in which:
        gen_pta(17, "DDK_NK")
    if "pta_dmn" in which:  # PLDMNoise (noise_model.py:443) beside PLRedNoise
        extra_name = "pta_dmn"
        gen_pta(15, "ELL1", extra="TNDMAMP -13.2\nTNDMGAM 2.8\nTNDMC 20\n")
        extra_name = None
    for i, b in enumerate(("ELL1H_H3", "ELL1H_H4", "ELL1H_STIG")):
        if b.lower() in which:
            gen_pta(11 + i, b)
