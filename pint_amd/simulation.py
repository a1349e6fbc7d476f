"""Synthetic TOAs (reference simulation.py:218 make_fake_toas_uniform, :125 make_fake_toas,
:29 zero_residuals) generated with the GPU model itself, for benchmarks on the GPU box.

Host-side TOA preparation is outside the path (north star), and the GPU box has no
astropy/erfa, so observatory positions for geocentric TOAs come from a committed daily
table of the reference's offline ephemeris (erfa epv00 via astropy "builtin";
``oracle/refgen/gen_ephem.py``) with cubic-Hermite interpolation.  Simplifications vs the
reference, documented in DESIGN.md: the requested MJDs are taken as TDB directly (no
UTC->TT->TDB chain: geocentric fake TOAs need no clock file), and ``mjd_float`` = TDB MJD.
Zeroing the residuals, pulse numbers, white and correlated noise follow the reference.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np

from .parameter import LD
from .toa import TOAs

_EPH = None


def _ephem():
    global _EPH
    if _EPH is None:
        z = np.load(os.path.join(os.path.dirname(__file__), "data", "earth_ephem.npz"), allow_pickle=False)
        _EPH = {k: z[k] for k in ("mjd", "earth_pos_km", "earth_vel_kms", "sun_pos_km")}
    return _EPH


def earth_posvel(tdb_mjd: np.ndarray):
    """Earth SSB position (km), velocity (km/s) and observatory->Sun vector (km) for a
    geocentric observer at TDB MJDs (cubic Hermite on the daily table)."""
    E = _ephem()
    t = np.asarray(tdb_mjd, dtype=np.float64)
    t0 = E["mjd"][0]
    if t.min() < t0 or t.max() > E["mjd"][-1] - 1:
        raise ValueError("synthetic ephemeris covers MJD 52900-58699 only")
    i = np.floor(t - t0).astype(int)
    u = (t - t0) - i
    p0, p1 = E["earth_pos_km"][i], E["earth_pos_km"][i + 1]
    v0, v1 = E["earth_vel_kms"][i] * 86400.0, E["earth_vel_kms"][i + 1] * 86400.0
    u = u[:, None]
    h00 = 2 * u ** 3 - 3 * u ** 2 + 1
    h10 = u ** 3 - 2 * u ** 2 + u
    h01 = -2 * u ** 3 + 3 * u ** 2
    h11 = u ** 3 - u ** 2
    pos = h00 * p0 + h10 * v0 + h01 * p1 + h11 * v1
    dh00 = 6 * u ** 2 - 6 * u
    dh10 = 3 * u ** 2 - 4 * u + 1
    dh01 = -6 * u ** 2 + 6 * u
    dh11 = 3 * u ** 2 - 2 * u
    vel = (dh00 * p0 + dh10 * v0 + dh01 * p1 + dh11 * v1) / 86400.0
    s0, s1 = E["sun_pos_km"][i], E["sun_pos_km"][i + 1]
    sun = s0 + u * (s1 - s0) - pos
    return pos, vel, sun


def _split(v):
    v = np.asarray(v, dtype=np.longdouble)
    hi = v.astype(np.float64)
    lo = (v - hi.astype(np.longdouble)).astype(np.float64)
    return hi, lo


def _row_arrays(tdb: np.ndarray, freqs, err_us, obs: str):
    hi, lo = _split(tdb)
    n = len(tdb)
    if obs.lower() in ("@", "ssb", "barycenter", "bary"):
        pos = vel = sun = np.zeros((n, 3))
        bary = np.ones(n, dtype=np.uint8)
    elif obs.lower() in ("geocenter", "geo", "coe", "0"):
        pos, vel, sun = earth_posvel(hi)
        bary = np.zeros(n, dtype=np.uint8)
    else:
        raise NotImplementedError("synthetic TOAs support geocenter or barycenter observers")
    return {"tdb_hi": hi, "tdb_lo": lo, "freq_mhz": np.asarray(freqs, dtype=np.float64),
            "err_us": np.broadcast_to(np.asarray(err_us, dtype=np.float64), (n,)).copy(),
            "ssb_obs_pos_km": pos, "ssb_obs_vel_kms": vel, "obs_sun_pos_km": sun,
            "mjd_float": hi.copy(), "is_bary": bary, "delta_pulse_number": np.zeros(n)}


def _times_freqs(start, end, ntoas, freqs, multi):
    """simulation.py:662 _get_freqs_and_times."""
    freqs = np.atleast_1d(np.asarray(freqs, dtype=np.float64))
    nf = len(freqs)
    if multi:
        nep = ntoas // nf + 1
        ep = np.linspace(LD(start), LD(end), nep, dtype=np.longdouble)
        return np.repeat(ep, nf)[:ntoas], np.tile(freqs, nep)[:ntoas]
    t = np.linspace(LD(start), LD(end), ntoas, dtype=np.longdouble)
    return t, np.tile(freqs, ntoas // nf + 1)[:ntoas]


def _tzr(model, obs):
    if "AbsPhase" not in model.components or model.TZRMJD.value is None:
        return None
    site = str(model.TZRSITE.value or "@")
    t = np.array([LD(model.TZRMJD.value)])
    f = float(model.TZRFRQ.value) if model.TZRFRQ.value else np.inf
    r = _row_arrays(t, [f], [1.0], site if site.lower() in ("geocenter", "@", "ssb", "barycenter", "coe") else obs)
    r["flags"] = {}
    return r


def make_fake_toas_batch(specs: Sequence[dict], seed: Optional[int] = None, maxiter: int = 10,
                         tolerance_s: float = 1e-9):
    """Generate several pulsars' fake TOAs at once (one GPU batch per zeroing iteration).

    specs: dicts with model, start, end, ntoas, freq, obs, error_us, add_noise,
    add_correlated_noise, multi_freqs_in_epoch, flags, seed.
    """
    from .engine import Session, pack_table
    from .noise import fourier_basis, red_noise_freqs_weights, scaled_sigma_us

    toas_list = []
    for sp in specs:
        t, f = _times_freqs(sp["start"], sp["end"], sp["ntoas"], sp.get("freq", 1400.0),
                            sp.get("multi_freqs_in_epoch", False))
        arr = _row_arrays(t, f, sp.get("error_us", 1.0), sp.get("obs", "geocenter"))
        fl = {"name": ["fake"] * len(t)}
        for k, v in (sp.get("flags") or {}).items():
            fl[k] = [v] * len(t)
        toas_list.append(TOAs(arr, fl, _tzr(sp["model"], sp.get("obs", "geocenter")), "fake"))
    models = [sp["model"] for sp in specs]

    def residuals(track_pn):
        s = Session()
        try:
            lays = s.add_all(zip(models, toas_list), track_mode="use_pulse_numbers" if track_pn else "nearest",
                             use_gls_basis=False)
            s.set_instances([(l, pack_table(l)) for l in lays])
            s.eval(False)
            tr, pr, _ = s.read_resids()
            hi, lo, ft, dl = s.read_eval()
            return tr, hi, lo
        finally:
            s.close()

    # pulse numbers from the model phase (toa.py:1984 compute_pulse_numbers)
    _, hi, lo = residuals(False)
    for t, h, l in zip(toas_list, hi, lo):
        ph = (np.longdouble(h) + np.longdouble(l))
        rel = ph[:-1] - ph[-1]
        t.arrays["pulse_number"] = np.floor(rel + LD(0.5)).astype(np.float64)
    # zero_residuals (simulation.py:29): iterate TOA adjustments until |r| < 1 ns
    for it in range(maxiter):
        tr, _, _ = residuals(True)
        worst = max(np.abs(r).max() for r in tr)
        if worst < tolerance_s:
            break
        for t, r in zip(toas_list, tr):
            tdb = t.tdbld - np.asarray(r, dtype=np.longdouble) / LD(86400)
            new = _row_arrays(tdb, t.arrays["freq_mhz"], t.arrays["err_us"],
                              "barycenter" if t.arrays["is_bary"][0] else "geocenter")
            for k in ("tdb_hi", "tdb_lo", "ssb_obs_pos_km", "ssb_obs_vel_kms", "obs_sun_pos_km"):
                t.arrays[k] = new[k]
    else:
        raise ValueError(f"Unable to make fake residuals - left over errors are {worst}")
    rng = np.random.default_rng(seed)
    for sp, m, t in zip(specs, models, toas_list):
        r = np.random.default_rng(sp.get("seed", None)) if sp.get("seed") is not None else rng
        shift = np.zeros(t.ntoas, dtype=np.longdouble)
        if sp.get("add_correlated_noise") and "PLRedNoise" in m.components:
            F = fourier_basis(m, t)
            _, phi = red_noise_freqs_weights(m, t)
            shift += np.asarray(F @ (np.sqrt(phi) * r.normal(size=len(phi))), dtype=np.longdouble)
        if sp.get("add_noise"):
            shift += np.asarray(scaled_sigma_us(m, t) * 1e-6 * r.normal(size=t.ntoas), dtype=np.longdouble)
        if np.any(shift != 0):
            tdb = t.tdbld + shift / LD(86400)
            new = _row_arrays(tdb, t.arrays["freq_mhz"], t.arrays["err_us"],
                              "barycenter" if t.arrays["is_bary"][0] else "geocenter")
            for k in ("tdb_hi", "tdb_lo", "ssb_obs_pos_km", "ssb_obs_vel_kms", "obs_sun_pos_km"):
                t.arrays[k] = new[k]
    return toas_list


def make_fake_toas_uniform(startMJD, endMJD, ntoas, model, freq=1400.0, obs="geocenter", error=1.0,
                           add_noise=False, add_correlated_noise=False, multi_freqs_in_epoch=False,
                           flags=None, seed=None):
    """simulation.py:218 (error in microseconds, freq in MHz)."""
    return make_fake_toas_batch([dict(model=model, start=startMJD, end=endMJD, ntoas=ntoas, freq=freq, obs=obs,
                                      error_us=error, add_noise=add_noise,
                                      add_correlated_noise=add_correlated_noise,
                                      multi_freqs_in_epoch=multi_freqs_in_epoch, flags=flags, seed=seed)])[0]


def pta_par(seed: int, binary: str = "", ndmx: int = 100, nmodes: int = 30) -> str:
    """Synthetic PTA pulsar template of SURVEY.md §8(d) C5 (pulsar i uses seed i):
    sky position uniform on the sphere, PM ~ N(0, 5 mas/yr), PX 1 mas, F0 ~ U[100, 700] Hz,
    F1 = -1e-15 F0/300, DM ~ U[5, 100] (frozen: DMX covers every TOA), DM1/DM2 free,
    `ndmx` DMX bins over MJD 53000-56652, PLRedNoise (TNRedAmp ~ U[-14.5,-13.5],
    TNRedGam ~ U[3,5], TNRedC 30), EFAC 1.1, EQUAD 0.1 us; ELL1 or DD binaries."""
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
TNRedC {nmodes}
"""
    edges = np.linspace(53000, 56652.01, ndmx + 1)
    par += "DMX 14.0\n"
    for i in range(ndmx):
        par += (f"DMX_{i+1:04d} {rng.normal(0, 1e-3):.6e} 1\nDMXR1_{i+1:04d} {edges[i]:.5f}\n"
                f"DMXR2_{i+1:04d} {edges[i+1]:.5f}\n")
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


def pta_kind(i: int) -> str:
    """Binary model of PTA pulsar i: about 1/3 ELL1 and 1/6 DD."""
    return "ELL1" if i % 6 in (1, 4) else ("DD" if i % 6 == 2 else "")


def pta_model(i: int, ndmx: int = 100):
    from .timing_model import get_model
    return get_model(pta_par(i, pta_kind(i), ndmx=ndmx))


def make_pta(npsr: int = 68, ntoas: int = 10000, ndmx: int = 100, seed0: int = 0, indices=None, models=None):
    """The C5 synthetic PTA (pulsar i uses seed i), or the pulsars `indices` of it (a rank's
    shard): every pulsar's data depends on its own index only."""
    idx = list(indices) if indices is not None else list(range(seed0, seed0 + npsr))
    specs = []
    for k, i in enumerate(idx):
        m = models[k] if models is not None else pta_model(i, ndmx)
        specs.append(dict(model=m, start=53000, end=56652, ntoas=ntoas, freq=[800, 1200, 1600, 2000],
                          obs="geocenter", error_us=0.5, add_noise=True, add_correlated_noise=True, seed=i))
    if not specs:
        return []
    toas = make_fake_toas_batch(specs)
    return [(sp["model"], t) for sp, t in zip(specs, toas)]
