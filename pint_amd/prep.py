"""Host TOA preparation without PINT/astropy: clock corrections, TT,
TDB and the observatory/Earth/Sun vectors the device path consumes, for tim-file TOAs.

The reference does this once per TOA load with astropy/erfa (toa.py:109-330 get_TOAs;
:2184 apply_clock_corrections; :2251 compute_TDBs -> Time.tdb; :2323 compute_posvels ->
observatory posvel + solar_system_ephemerides.objPosVel_wrt_SSB; erfautils.py
gcrs_posvel_from_itrf -> EarthLocation.get_gcrs_posvel).  The same quantities here:

* UTC -> TAI -> TT: TAI-UTC from the leap-second steps (erfa.dat), TT = TAI + 32.184 s;
* TT -> TDB: TDB - TT = erfa.dtdb(TT, ut, elong, u, v), evaluated from its exact
  decomposition G(t) + u [sin(tsol) C(t) + cos(tsol) S(t)] + v B(t), tsol = 2 pi ut + elong,
  with G, C, S, B tabulated (astropy passes the UTC fraction of day as ut and the site's
  longitude, axis distance and z in km; geocentric for a Time without location);
* the site's GCRS position/velocity (astropy 4.3 EarthLocation.get_gcrs_posvel): ITRS ->
  CIRS by the Earth rotation angle (era00 of UT1 = UTC + dUT1) and polar motion (pom00 of
  x_p, y_p and s' = sp00), CIRS -> GCRS by c2ixys of the IAU 2006/2000A CIP X, Y, s
  (tabulated), velocity = (Earth rotation vector) x position, at the TDB time converted
  back to TT with the geocentric TDB - TT (the reference builds that Time without a
  location);
* the Earth's and the Sun's barycentric vectors from the "builtin" ephemeris (erfa.epv00,
  tabulated; 6-point Lagrange interpolation).

The tables (pint_amd/data/prep_tables.npz) are data sampled from the reference's own
environment (astropy 4.3.1 / pyerfa 2.0.0 / bundled IERS-B) by
oracle/refgen/gen_prep_tables.py; the rotations and interpolations are restated here.
IERS values are interpolated as astropy's IERS._interpolate does (linear in UTC MJD; the
UT1-UTC difference corrected for leap-second jumps).  Outside the tables' span
(MJD 49900-60600; IERS-B to 59406) preparation raises.
"""
from __future__ import annotations

import os
from functools import lru_cache
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from .observatory import sites

LD = np.longdouble
DAYSEC = 86400.0
DJM0 = 2400000.5
DJ00 = 2451545.0
TT_TAI = 32.184
OMEGA_EARTH = 1.00273781191135448 * 2.0 * np.pi / DAYSEC  # astropy coordinates.earth
ASEC2RAD = np.pi / 648000.0
_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "prep_tables.npz")


@lru_cache(maxsize=1)
def tables() -> Dict[str, np.ndarray]:
    z = np.load(_DATA, allow_pickle=False)
    return {k: z[k] for k in z.files}


# ---------------------------------------------------------------------------------------
# time scales
# ---------------------------------------------------------------------------------------
def tai_minus_utc(mjd_day: np.ndarray) -> np.ndarray:
    """erfa.dat at 0h UTC of the day (leap-second era, >= 1972)."""
    lp = tables()["leap"]
    idx = np.searchsorted(lp[:, 0], np.asarray(mjd_day, dtype=np.float64), side="right") - 1
    if np.any(idx < 0):
        raise ValueError("UTC before 1972 is outside the leap-second table")
    return lp[idx, 1]


def utc_to_tt(day: np.ndarray, frac: np.ndarray) -> np.ndarray:
    """TT MJD (longdouble) of UTC (day, fraction): TAI = UTC + dat, TT = TAI + 32.184 s
    (erfa utctai/taitt; days are 86400 s as in the pulsar_mjd convention)."""
    day = np.asarray(day, dtype=np.float64)
    return LD(day) + (LD(frac) + (LD(tai_minus_utc(day)) + LD(TT_TAI)) / LD(DAYSEC))


def tt_to_utc_parts(tt: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """UTC (day, fraction) of a TT MJD (longdouble), for the IERS lookups (taiutc)."""
    tt = np.asarray(tt, dtype=LD)
    approx = tt - LD(TT_TAI + 37.0) / LD(DAYSEC)
    day = np.floor(approx.astype(np.float64))
    dat = tai_minus_utc(day)
    utc = tt - (LD(dat) + LD(TT_TAI)) / LD(DAYSEC)
    day = np.floor(utc.astype(np.float64))
    return day, (utc - LD(day)).astype(np.float64)


def _grid(name: str, t: np.ndarray):
    tb = tables()
    t0, dt = float(tb[name + "_t0"]), float(tb[name + "_dt"])
    y = tb[name]
    x = (np.asarray(t, dtype=np.float64) - t0) / dt
    i = np.floor(x).astype(np.int64)
    if np.any(i < 1) or np.any(i >= len(y) - 2):
        raise ValueError(f"time outside the {name} table (MJD {t0 + dt:.1f}-{t0 + (len(y) - 3) * dt:.1f})")
    return y, i, x - i, dt


def _lagrange4(name: str, t: np.ndarray) -> np.ndarray:
    """Cubic (4-point Lagrange) interpolation on a uniform grid."""
    y, i, u, _ = _grid(name, t)
    um, u1, u2 = u + 1.0, u - 1.0, u - 2.0
    w0 = -u * u1 * u2 / 6.0
    w1 = um * u1 * u2 / 2.0
    w2 = -um * u * u2 / 2.0
    w3 = um * u * u1 / 6.0
    sh = (-1,) + (1,) * (y.ndim - 1)
    return (w0.reshape(sh) * y[i - 1] + w1.reshape(sh) * y[i] + w2.reshape(sh) * y[i + 1]
            + w3.reshape(sh) * y[i + 2])


def tdb_minus_tt(tt: np.ndarray, ut_frac: np.ndarray, elong: float, u_km: float, v_km: float) -> np.ndarray:
    """erfa.dtdb (s) through its tabulated decomposition (see module doc)."""
    g = _lagrange4("dtdb", tt)
    tsol = np.mod(np.asarray(ut_frac, dtype=np.float64), 1.0) * 2.0 * np.pi + elong
    return g[:, 0] + u_km * (np.sin(tsol) * g[:, 1] + np.cos(tsol) * g[:, 2]) + v_km * g[:, 3]


# ---------------------------------------------------------------------------------------
# ephemeris (builtin = erfa.epv00)
# ---------------------------------------------------------------------------------------
def _lagrange6(name: str, t: np.ndarray) -> np.ndarray:
    """6-point Lagrange interpolation on a uniform grid (nodes i-2 .. i+3): for the Earth
    at 0.25-day spacing the lunar-monthly term leaves < 1 cm."""
    y, i, u, _ = _grid(name, t)
    if np.any(i < 2) or np.any(i >= len(y) - 3):
        raise ValueError(f"time outside the {name} table")
    nodes = np.arange(-2, 4)
    out = 0.0
    for k in nodes:
        w = np.ones_like(u)
        for m in nodes:
            if m != k:
                w = w * (u - m) / (k - m)
        out = out + w[:, None] * y[i + k]
    return out


def _posvel(name: str, t: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Position (km) and velocity (km/s) at t from the tabulated samples."""
    v = _lagrange6(name, t)
    return v[:, :3], v[:, 3:]


def earth_posvel(tdb: np.ndarray):
    """objPosVel_wrt_SSB("earth", tdb, "builtin"): km, km/s."""
    return _posvel("earth", tdb)


def sun_posvel(tdb: np.ndarray):
    return _posvel("sun", tdb)


PLANETS = ("jupiter", "saturn", "venus", "uranus", "neptune")   # solar_system_shapiro.py:112


def planet_pos(name: str, tdb: np.ndarray) -> np.ndarray:
    """objPosVel_wrt_SSB(name, tdb, "builtin").pos (km): astropy's builtin planets (erfa.plan94
    heliocentric + the Sun's barycentric vector), tabulated."""
    return _lagrange6(name, tdb)


# ---------------------------------------------------------------------------------------
# Earth orientation (astropy 4.3 EarthLocation.get_gcrs_posvel via CIRS)
# ---------------------------------------------------------------------------------------
def _iers(utc_day: np.ndarray, utc_frac: np.ndarray):
    """(x_p, y_p [rad], UT1-UTC [s]) -- astropy IERS._interpolate: linear in MJD between the
    table's integer days, the UT1-UTC step corrected by its rounded value (leap seconds)."""
    tab = tables()["iers"]
    mjd = np.asarray(utc_day, dtype=np.float64)
    if np.any(mjd < tab[0, 0]) or np.any(mjd >= tab[-1, 0]):
        raise ValueError(f"UTC MJD outside the IERS-B table ({tab[0, 0]:.0f}-{tab[-1, 0]:.0f})")
    i = np.searchsorted(tab[:, 0], mjd, side="right")
    i1 = np.clip(i, 1, len(tab) - 1)
    i0 = i1 - 1
    f = mjd - tab[i0, 0] + np.asarray(utc_frac, dtype=np.float64)
    out = []
    for col in (1, 2, 3):
        v0, v1 = tab[i0, col], tab[i1, col]
        d = v1 - v0
        if col == 3:
            d = d - np.round(d)
        out.append(v0 + f * d)
    return out[0] * ASEC2RAD, out[1] * ASEC2RAD, out[2]


def _rx(a):
    c, s = np.cos(a), np.sin(a)
    o, z = np.ones_like(a), np.zeros_like(a)
    return np.stack([np.stack([o, z, z], -1), np.stack([z, c, s], -1), np.stack([z, -s, c], -1)], -2)


def _ry(a):
    c, s = np.cos(a), np.sin(a)
    o, z = np.ones_like(a), np.zeros_like(a)
    return np.stack([np.stack([c, z, -s], -1), np.stack([z, o, z], -1), np.stack([s, z, c], -1)], -2)


def _rz(a):
    c, s = np.cos(a), np.sin(a)
    o, z = np.ones_like(a), np.zeros_like(a)
    return np.stack([np.stack([c, s, z], -1), np.stack([-s, c, z], -1), np.stack([z, z, o], -1)], -2)


def c2ixys(x, y, s):
    """Celestial-to-intermediate matrix from the CIP X, Y and the CIO locator s (SOFA
    c2ixys): Rz(-(E+s)) Ry(d) Rz(E), E = atan2(Y, X), d = atan(sqrt(r2 / (1 - r2)))."""
    r2 = x * x + y * y
    e = np.where(r2 > 0, np.arctan2(y, x), 0.0)
    d = np.arctan(np.sqrt(r2 / (1.0 - r2)))
    return _rz(-(e + s)) @ _ry(d) @ _rz(e)


def era00(ut1_day: np.ndarray, ut1_frac: np.ndarray) -> np.ndarray:
    """Earth rotation angle (IAU 2000, SOFA era00) of UT1 = MJD day + fraction."""
    d1 = np.asarray(ut1_day, dtype=np.float64) + DJM0
    d2 = np.asarray(ut1_frac, dtype=np.float64)
    t = d2 + (d1 - DJ00)
    f = np.fmod(d1, 1.0) + np.fmod(d2, 1.0)
    return np.mod(2.0 * np.pi * (f + 0.7790572732640 + 0.00273781191135448 * t), 2.0 * np.pi)


def pom00(xp, yp, sp):
    """Polar-motion matrix (SOFA pom00): Rx(-yp) Ry(-xp) Rz(sp)."""
    return _rx(-yp) @ _ry(-xp) @ _rz(sp)


def sp00(tt: np.ndarray) -> np.ndarray:
    """The TIO locator s' (SOFA sp00): -47 uas per Julian century of TT."""
    t = (np.asarray(tt, dtype=np.float64) + (DJM0 - DJ00)) / 36525.0
    return -47e-6 * t * ASEC2RAD


def site_gcrs_posvel(itrf_m: Sequence[float], tdb: np.ndarray):
    """EarthLocation.get_gcrs_posvel at TDB times (km, km/s): see the module doc."""
    tdb = np.asarray(tdb, dtype=LD)
    # the TDB Time carries no location: TT = TDB - dtdb(geocentric)
    tt = tdb - LD(tdb_minus_tt(tdb.astype(np.float64), 0.0, 0.0, 0.0, 0.0)) / LD(DAYSEC)
    ttf = tt.astype(np.float64)
    uday, ufrac = tt_to_utc_parts(tt)
    xp, yp, dut1 = _iers(uday, ufrac)
    ut1 = LD(uday) + LD(ufrac) + LD(dut1) / LD(DAYSEC)
    u1day = np.floor(ut1.astype(np.float64))
    era = era00(u1day, (ut1 - LD(u1day)).astype(np.float64))
    cip = _lagrange4("cip", ttf)
    c2i = c2ixys(cip[:, 0], cip[:, 1], cip[:, 2])               # GCRS -> CIRS
    cirs_to_itrs = pom00(xp, yp, sp00(ttf)) @ _rz(era)            # c2tcio(I, era, rpom)
    itrs_to_gcrs = np.swapaxes(c2i, -1, -2) @ np.swapaxes(cirs_to_itrs, -1, -2)
    pos = itrs_to_gcrs @ (np.asarray(itrf_m, dtype=np.float64) / 1000.0)
    rot = np.swapaxes(c2i, -1, -2)[..., 2] * OMEGA_EARTH
    vel = np.cross(rot, pos)
    return pos, vel


# ---------------------------------------------------------------------------------------
# sites
# ---------------------------------------------------------------------------------------
def site_info(name: str) -> dict:
    s = sites()[name]
    kind = s.get("special") or "topo"
    if kind == "topo" and not s.get("itrf_xyz"):
        raise NotImplementedError(f"site {name} has no ITRF position")
    return {"kind": kind, "itrf": s.get("itrf_xyz")}


def _geodetic_args(itrf_m):
    """(elong [rad], u = distance from the spin axis [km], v = z [km]) as astropy passes
    them to dtdb (time/core.py _get_delta_tdb_tt)."""
    x, y, z = (float(c) / 1000.0 for c in itrf_m)
    return float(np.arctan2(y, x)), float(np.hypot(x, y)), z


# ---------------------------------------------------------------------------------------
# the whole preparation
# ---------------------------------------------------------------------------------------
def prepare(day: np.ndarray, frac: np.ndarray, obs: Sequence[str], corr_s: Optional[np.ndarray] = None,
            planets: bool = False) -> Dict[str, np.ndarray]:
    """Per-TOA boundary columns (pint_amd.toa FIELDS) for MJD (day, fraction) in each site's
    time scale (UTC for observatories and the geocenter, TDB for the barycenter), after
    adding clock corrections corr_s (s): tdb_hi/lo, mjd_float, ssb_obs_pos/vel, obs_sun_pos,
    is_bary; with planets=True also obs_<planet>_pos for the Shapiro planets and the Earth
    (toa.py:2403-2433: the body's barycentric position minus the observatory's)."""
    n = len(day)
    day = np.asarray(day, dtype=np.float64)
    frac = np.asarray(frac, dtype=np.float64)
    corr = np.zeros(n) if corr_s is None else np.asarray(corr_s, dtype=np.float64)
    t = LD(day) + LD(frac) + LD(corr) / LD(DAYSEC)   # the clock-corrected time in the site scale
    mjd_float = (day + frac) + corr / DAYSEC      # toa.py:2242 mjd_float += corrections
    tdb = np.zeros(n, dtype=LD)
    pos = np.zeros((n, 3))
    vel = np.zeros((n, 3))
    is_bary = np.zeros(n, dtype=np.uint8)
    obs = np.asarray(obs, dtype=object)
    for name in dict.fromkeys(obs.tolist()):
        g = np.nonzero(obs == name)[0]
        info = site_info(name)
        if info["kind"] == "barycenter":
            tdb[g] = t[g]
            is_bary[g] = 1
            continue
        if info["kind"] != "topo" and info["kind"] != "geocenter":
            raise NotImplementedError(f"site kind {info['kind']} ({name})")
        tg = t[g]
        uday = np.floor(tg.astype(np.float64))
        ufrac = (tg - LD(uday)).astype(np.float64)
        tt = utc_to_tt(uday, ufrac)
        if info["kind"] == "topo":
            el, uu, vv = _geodetic_args(info["itrf"])
        else:
            el, uu, vv = 0.0, 0.0, 0.0
        tdb[g] = tt + LD(tdb_minus_tt(tt.astype(np.float64), ufrac, el, uu, vv)) / LD(DAYSEC)
        ep, ev = earth_posvel(tdb[g].astype(np.float64))
        if info["kind"] == "topo":
            gp, gv = site_gcrs_posvel(info["itrf"], tdb[g])
            ep, ev = ep + gp, ev + gv
        pos[g], vel[g] = ep, ev
    sp, _ = sun_posvel(tdb.astype(np.float64))
    hi = tdb.astype(np.float64)
    lo = (tdb - LD(hi)).astype(np.float64)
    out = {"tdb_hi": hi, "tdb_lo": lo, "mjd_float": mjd_float, "ssb_obs_pos_km": pos, "ssb_obs_vel_kms": vel,
           "obs_sun_pos_km": sp - pos, "is_bary": is_bary}
    if planets:
        tf = tdb.astype(np.float64)
        for pl in PLANETS:
            out[f"obs_{pl}_pos_km"] = planet_pos(pl, tf) - pos
        out["obs_earth_pos_km"] = earth_posvel(tf)[0] - pos
    return out
