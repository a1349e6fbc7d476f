"""pint_oracle — CPU restatement of PINT's fit-and-residual hot path (TEST INFRASTRUCTURE).

This module is the *checker*: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it.  The product (``pint_amd``) never
does; it computes on the GPU or fails.

It restates the reference algorithms in numpy (longdouble where the reference uses
longdouble), function by function, citing the reference file:line followed.  It is
*pinned* by ``tests/test_oracle_golden.py`` against golden vectors captured from the real
reference (``oracle/refgen``, run in the build container via ``oracle/refenv``): delays,
phases, residuals, design matrices, chi2 and WLS/GLS fit steps of the C1-C5 fixtures.

Third-party arithmetic the reference calls and this file restates from the published
algorithm: erfa/SOFA ``pmsafe``/``starpm``/``starpv`` (pyerfa 2.0.0, via astrometry.py:513
and astropy 4.3.1 ``SkyCoord.apply_space_motion``); numpy/scipy linear algebra (svd,
cho_factor) is used directly.

Inputs are plain containers (see ``OModel``) so the oracle does not depend on the
product's par parser: ``from_fixture(meta)`` builds one from a golden fixture's exported
parameter table; ``from_product_model`` converts a pint_amd model (for seeded tests).
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import scipy.linalg

LD = np.longdouble

# constants (reference pint/__init__.py:67-102 and astropy/erfa values captured by
# oracle/refgen: c, au, Tsun, DMconst, obliquities)
C_KMS = 299792.458
AU_KM = 149597870.7
KPC_KM = 3.0856775814913674e16
TSUN = 4.92549094830932e-06
# M_sun / M_planet of the PLANET_SHAPIRO planets (pint/__init__.py:84-90), summation order of
# solar_system_shapiro.py:112
PLANETS = (("jupiter", 1047.3486), ("saturn", 3497.898), ("venus", 408523.71), ("uranus", 22902.98),
           ("neptune", 19412.24))
DMCONST = 4149.377593360996
DAYSEC = 86400.0
DJY = 365.25
ERFA_DC = 173.1446326742403
DR2AS = 206264.80624709636
MAS_RAD = 4.84813681109536e-09
HA_RAD = 0.2617993877991494
DEG_RAD = 0.017453292519943295
MASYR_RADS = 1.5362818500441604e-16
YR_S = 31557600.0
OBL = {"IERS2010": 0.4090926006005829, "IERS2003": 0.40909260011576914, "DEFAULT": 84381.406 / DR2AS}


@dataclass
class OModel:
    values: Dict[str, object]                 # numeric params (np.longdouble / float) in par units
    free: List[str]                           # free params in model.params order
    comps: set
    masks: Dict[str, tuple] = field(default_factory=dict)  # name -> (key, [key_value...])
    binary: Optional[str] = None
    ecl: str = "IERS2010"

    def v(self, name, default=0.0):
        x = self.values.get(name)
        return default if x is None else x

    def has(self, name):
        return self.values.get(name) is not None

    def prefix(self, rx):
        out = []
        for n in self.values:
            m = re.match(rx, n)
            if m and self.values[n] is not None:
                out.append((int(m.group(1)), n))
        return [n for _, n in sorted(out)]


def from_fixture(meta) -> OModel:
    vals = {}
    masks = {}
    mm = meta["model"]
    for name, d in mm["values"].items():
        val = d.get("value")
        if isinstance(val, list):
            vals[name] = LD(val[0]) + LD(val[1])
        elif d.get("kind") == "boolParameter" and val is not None:  # e.g. DDK's K96
            vals[name] = 1.0 if str(val).strip().upper() in ("TRUE", "1", "Y", "T") else 0.0
        if d.get("key"):
            masks[name] = (d["key"], d.get("key_value") or [])
    comps = set(mm["components"])
    binary = next((b for b in ("ELL1H", "ELL1", "DD", "DDK", "BT") if "Binary" + b in comps), None)
    ecl = mm["values"].get("ECL", {}).get("value") or "IERS2010"
    return OModel(vals, list(mm["free_params"]), comps, masks, binary, ecl)


def from_product_model(model) -> OModel:
    vals, masks = {}, {}
    for n in model.params:
        p = model[n]
        if p.kind == "bool":  # e.g. DDK's K96 (unset: the binary's default True)
            if p.value is not None:
                vals[n] = 1.0 if p.value else 0.0
            continue
        if p.kind == "str":
            continue
        if p.value is not None:
            vals[n] = LD(p.value) if (p.long_double or p.kind == "mjd") else float(p.value)
        if p.kind == "mask":
            masks[n] = (p.key, list(p.key_value))
    comps = set(model.components)
    if model.binary:
        comps.add("Binary" + model.binary)
    return OModel(vals, list(model.free_params), comps, masks, model.binary,
                  str(model.ECL.value) if "ECL" in model and model.ECL.value else "IERS2010")


# ----------------------------------------------------------------------------------
# TOA helpers
# ----------------------------------------------------------------------------------
def _rows(toas: dict, tzr: bool):
    """Concatenate TOA rows and the TZR row (as the product does) -> dict of arrays."""
    keys = ["tdb_hi", "tdb_lo", "freq_mhz", "ssb_obs_pos_km", "ssb_obs_vel_kms", "obs_sun_pos_km", "mjd_float",
            "is_bary", "delta_pulse_number"]
    keys = keys + [f"obs_{pl}_pos_km" for pl, _ in PLANETS if f"obs_{pl}_pos_km" in toas]
    out = {}
    for k in keys:
        a = np.asarray(toas[k])
        if tzr and k not in toas["tzr"] and k.startswith("obs_") and k != "obs_sun_pos_km":
            a = np.concatenate([a, np.zeros((1, 3))])   # a barycentric TZR TOA carries no planets
        elif tzr:
            b = np.asarray(toas["tzr"][k], dtype=a.dtype).reshape((1,) + a.shape[1:])
            a = np.concatenate([a, b])
        out[k] = a
    return out


def select_mask(toas: dict, key: str, key_value, tzr=False) -> np.ndarray:
    """maskParameter.select_toa_mask (parameter.py:2124): flag equality or inclusive
    mjd/freq ranges (toa_select.py:101).  tzr=True evaluates it on the TZR TOA (no flags)."""
    src = toas["tzr"] if tzr else toas
    n = len(np.atleast_1d(src["tdb_hi"]))
    kl = key.lower()
    if kl in ("mjd", "freq"):
        col = np.atleast_1d(np.asarray(src["mjd_float" if kl == "mjd" else "freq_mhz"], dtype=float))
        if len(key_value) == 2:
            return (col >= float(key_value[0])) & (col <= float(key_value[1]))
        return col == float(key_value[0])
    if kl == "tel":  # parameter.py:1868, :2156: canonical site names (fixture obs_names)
        if tzr or "obs" not in toas:
            return np.zeros(n, dtype=bool)
        want = str(key_value[0]).lower()
        return np.array([o == want or want in toas["obs_alias"].get(o, ()) for o in toas["obs"]], dtype=bool)
    k = key[1:] if key.startswith("-") else key
    fl = {} if tzr else toas.get("flags", {})
    if k not in fl:
        return np.zeros(n, dtype=bool)
    return np.array([f == key_value[0] for f in fl[k]], dtype=bool)


def select_rows(toas: dict, key, key_value, with_tzr=True):
    sel = select_mask(toas, key, key_value)
    if with_tzr:
        sel = np.concatenate([sel, select_mask(toas, key, key_value, tzr=True)])
    return sel


def toas_from_fixture(z: dict, meta: dict) -> dict:
    """Golden fixture arrays -> oracle TOA dict (TOA rows, flags, TZR row)."""
    d = {k: np.asarray(z[k]) for k in ("tdb_hi", "tdb_lo", "freq_mhz", "err_us", "ssb_obs_pos_km",
                                       "ssb_obs_vel_kms", "obs_sun_pos_km", "mjd_float", "is_bary",
                                       "delta_pulse_number")}
    for pl, _ in PLANETS:
        if f"obs_{pl}_pos_km" in z:
            d[f"obs_{pl}_pos_km"] = np.asarray(z[f"obs_{pl}_pos_km"])
    if "pulse_number" in z:
        d["pulse_number"] = np.asarray(z["pulse_number"])
    d["flags"] = meta.get("flag_columns", {})
    if "obs_index" in z and meta.get("obs_names"):
        d["obs"] = [meta["obs_names"][i] for i in np.asarray(z["obs_index"])]
        d["obs_alias"] = {k: [a.lower() for a in v] for k, v in meta.get("obs_aliases", {}).items()}
    d["tzr"] = {k[4:]: np.asarray(z[k]) for k in z if k.startswith("tzr_")}
    if "wb_pp_dm" in z:  # wideband DM measurements (-pp_dm / -pp_dme flags)
        d["pp_dm"], d["pp_dme"] = np.asarray(z["wb_pp_dm"]), np.asarray(z["wb_pp_dme"])
    return d


# ----------------------------------------------------------------------------------
# astrometry (astrometry.py)
# ----------------------------------------------------------------------------------
def _starpm_dir(ra, dec, pmr, pmd, px, dt):
    """erfa pmsafe -> starpm -> starpv (SOFA), rv = 0; returns unit vectors (N,3)."""
    a = np.array([np.cos(ra) * np.cos(dec), np.sin(ra) * np.cos(dec), np.sin(dec)])
    b = np.array([np.cos(ra + pmr) * np.cos(dec + pmd), np.sin(ra + pmr) * np.cos(dec + pmd), np.sin(dec + pmd)])
    pm = np.arctan2(np.linalg.norm(np.cross(a, b)), np.dot(a, b))
    px1 = max(px, pm * 326.0, 5e-7)
    r = DR2AS / max(px1, 1e-7)
    rad, decd = pmr / DJY, pmd / DJY
    st, ct, sp, cp = np.sin(ra), np.cos(ra), np.sin(dec), np.cos(dec)
    x, y = r * cp * ct, r * cp * st
    rpd = r * decd
    w = rpd * sp
    p = np.array([x, y, r * sp])
    v = np.array([-y * rad - w * ct, x * rad - w * st, rpd * cp])
    if np.linalg.norm(v) / ERFA_DC > 0.5:
        v = np.zeros(3)
    pm_ = np.linalg.norm(p)
    xu = p / pm_
    vsr = xu @ v
    usr = vsr * xu
    ust = v - usr
    vst = np.linalg.norm(ust)
    betsr, betst = vsr / ERFA_DC, vst / ERFA_DC
    bett, betr = betst, betsr
    d = 1.0
    dl = 0.0
    od = odel = odd = oddel = 0.0
    for i in range(100):
        d = 1.0 + betr
        w2 = betr * betr + bett * bett
        dl = -w2 / (np.sqrt(1.0 - w2) + 1.0)
        betr = d * betsr + dl
        bett = d * betst
        if i > 0:
            dd, ddel = abs(d - od), abs(dl - odel)
            if i > 1 and dd >= odd and ddel >= oddel:
                break
            odd, oddel = dd, ddel
        od, odel = d, dl
    wr = d + dl / betsr if betsr != 0 else 1.0
    v1 = wr * usr + d * ust
    tl1 = pm_ / ERFA_DC
    dt = np.asarray(dt, dtype=float)
    q = p[None, :] + (dt + tl1)[:, None] * v1[None, :]
    r2 = (q * q).sum(1)
    rdv = q @ v1
    v2 = v1 @ v1
    c2 = ERFA_DC ** 2 - v2
    tl2 = (-rdv + np.sqrt(rdv * rdv + c2 * r2)) / c2
    p2 = p[None, :] + (dt + (tl1 - tl2))[:, None] * v1[None, :]
    th = np.arctan2(p2[:, 1], p2[:, 0])
    ph = np.arctan2(p2[:, 2], np.hypot(p2[:, 0], p2[:, 1]))
    return np.stack([np.cos(th) * np.cos(ph), np.sin(th) * np.cos(ph), np.sin(ph)], axis=1)


def _rot_ecl_to_icrs(obl, v):
    c, s = np.cos(obl), np.sin(obl)
    v = np.atleast_2d(v)
    return np.stack([v[:, 0], c * v[:, 1] - s * v[:, 2], s * v[:, 1] + c * v[:, 2]], axis=1)


def _rot_icrs_to_ecl(obl, v):
    c, s = np.cos(obl), np.sin(obl)
    v = np.atleast_2d(v)
    return np.stack([v[:, 0], c * v[:, 1] + s * v[:, 2], -s * v[:, 1] + c * v[:, 2]], axis=1)


def psr_dir_icrs(om: OModel, epoch_mjd: np.ndarray) -> np.ndarray:
    """ssb_to_psb_xyz_ICRS (astrometry.py:469-528 equatorial; :71 base path for ecliptic,
    SkyCoord apply_space_motion with a 1-kpc dummy distance, utils.py:2171)."""
    n = len(epoch_mjd)
    pep = float(om.v("POSEPOCH", 0.0))
    if "AstrometryEquatorial" in om.comps:
        ra, dec = float(om.v("RAJ")) * HA_RAD, float(om.v("DECJ")) * DEG_RAD
        pml, pmb = float(om.v("PMRA")), float(om.v("PMDEC"))
        if pml == 0 and pmb == 0:
            return np.tile([np.cos(ra) * np.cos(dec), np.sin(ra) * np.cos(dec), np.sin(dec)], (n, 1))
        return _starpm_dir(ra, dec, pml * MAS_RAD / np.cos(dec), pmb * MAS_RAD, float(om.v("PX")) * 1e-3,
                           np.asarray(epoch_mjd, dtype=float) - pep)
    obl = OBL[om.ecl]
    l, b = float(om.v("ELONG")) * DEG_RAD, float(om.v("ELAT")) * DEG_RAD
    pml, pmb = float(om.v("PMELONG")), float(om.v("PMELAT"))
    ue = np.array([np.cos(l) * np.cos(b), np.sin(l) * np.cos(b), np.sin(b)])
    if pml == 0 and pmb == 0:
        return np.tile(_rot_ecl_to_icrs(obl, ue)[0], (n, 1))
    el = np.array([-np.sin(l), np.cos(l), 0.0])
    eb = np.array([-np.sin(b) * np.cos(l), -np.sin(b) * np.sin(l), np.cos(b)])
    u = _rot_ecl_to_icrs(obl, ue)[0]
    vv = _rot_ecl_to_icrs(obl, pml * MAS_RAD * el + pmb * MAS_RAD * eb)[0]
    ra = np.arctan2(u[1], u[0])
    dec = np.arctan2(u[2], np.hypot(u[0], u[1]))
    era = np.array([-np.sin(ra), np.cos(ra), 0.0])
    edec = np.array([-np.sin(dec) * np.cos(ra), -np.sin(dec) * np.sin(ra), np.cos(dec)])
    return _starpm_dir(ra, dec, (vv @ era) / np.cos(dec), vv @ edec, 1e-3, np.asarray(epoch_mjd, dtype=float) - pep)


# ----------------------------------------------------------------------------------
# binary models (stand_alone_psr_binaries) in longdouble
# ----------------------------------------------------------------------------------
def _orbits(om, tt0):
    """binary_orbits.py:98 OrbitPB.orbits and :25 orbit_phase."""
    PB = LD(om.v("PB")) * LD(DAYSEC)
    x = tt0 / PB
    orbits = x - LD(0.5) * (LD(om.v("PBDOT")) + LD(om.v("XPBDOT"))) * x * x
    norb = np.floor(orbits)
    return orbits, norb, (orbits - norb) * LD(2 * np.pi)


class _ELL1:
    """ELL1_model.py (ELL1model, 3rd-order Roemer, delayI, delayS) and derivatives."""

    def __init__(self, om, bt_days, acc):
        self.om = om
        self.tt0 = (bt_days - LD(om.v("TASC"))) * LD(DAYSEC) - LD(0) if acc is None else \
            (bt_days - LD(om.v("TASC"))) * LD(DAYSEC) - np.asarray(acc, dtype=LD)
        tt0 = self.tt0
        self.PBs = LD(om.v("PB")) * LD(DAYSEC)
        self.PBDOT, self.XPBDOT = LD(om.v("PBDOT")), LD(om.v("XPBDOT"))
        self.orbits, _, self.Phi = _orbits(om, tt0)
        self.pb = self.PBs + self.PBDOT * tt0
        self.A1DOT = LD(om.v("A1DOT"))
        self.a1 = LD(om.v("A1")) + tt0 * self.A1DOT
        self.E1DOT, self.E2DOT = LD(om.v("EPS1DOT")) * LD(1e-12), LD(om.v("EPS2DOT")) * LD(1e-12)
        self.e1 = LD(om.v("EPS1")) + tt0 * self.E1DOT
        self.e2 = LD(om.v("EPS2")) + tt0 * self.E2DOT
        self.TM2 = LD(om.v("M2")) * LD(TSUN)
        self.SINI = LD(om.v("SINI"))
        P, e1, e2 = self.Phi, self.e1, self.e2
        s = [None] + [np.sin(k * P) for k in range(1, 5)]
        c = [None] + [np.cos(k * P) for k in range(1, 5)]
        self.s, self.c = s, c
        self.R0 = (s[1] + 0.5 * (e2 * s[2] - e1 * c[2])
                   - (1.0 / 8) * (5 * e2 ** 2 * s[1] - 3 * e2 ** 2 * s[3] - 2 * e2 * e1 * c[1] + 6 * e2 * e1 * c[3]
                                  + 3 * e1 ** 2 * s[1] + 3 * e1 ** 2 * s[3])
                   - (1.0 / 12) * (5 * e2 ** 3 * s[2] + 3 * e1 ** 2 * e2 * s[2] - 6 * e1 * e2 ** 2 * c[2]
                                   - 4 * e1 ** 3 * c[2] - 4 * e2 ** 3 * s[4] + 12 * e1 ** 2 * e2 * s[4]
                                   + 12 * e1 * e2 ** 2 * c[4] - 4 * e1 ** 3 * c[4]))
        self.R1 = (c[1] + e1 * s[2] + e2 * c[2]
                   - (1.0 / 8) * (5 * e2 ** 2 * c[1] - 9 * e2 ** 2 * c[3] + 2 * e1 * e2 * s[1] - 18 * e1 * e2 * s[3]
                                  + 3 * e1 ** 2 * c[1] + 9 * e1 ** 2 * c[3])
                   - (1.0 / 12) * (10 * e2 ** 3 * c[2] + 6 * e1 ** 2 * e2 * c[2] + 12 * e1 * e2 ** 2 * s[2]
                                   + 8 * e1 ** 3 * s[2] - 16 * e2 ** 3 * c[4] + 48 * e1 ** 2 * e2 * c[4]
                                   - 48 * e1 * e2 ** 2 * s[4] + 16 * e1 ** 3 * s[4]))
        self.R2 = (-s[1] + 2 * e1 * c[2] - 2 * e2 * s[2]
                   - (1.0 / 8) * (-5 * e2 ** 2 * s[1] + 27 * e2 ** 2 * s[3] + 2 * e1 * e2 * c[1]
                                  - 54 * e1 * e2 * c[3] - 3 * e1 ** 2 * s[1] - 27 * e1 ** 2 * s[3])
                   - (1.0 / 12) * (-20 * e2 ** 3 * s[2] - 12 * e1 ** 2 * e2 * s[2] + 24 * e1 * e2 ** 2 * c[2]
                                   + 16 * e1 ** 3 * c[2] + 64 * e2 ** 3 * s[4] - 192 * e1 ** 2 * e2 * s[4]
                                   - 192 * e1 * e2 ** 2 * c[4] + 64 * e1 ** 3 * c[4]))
        self.Dre, self.Drep, self.Drepp = self.a1 * self.R0, self.a1 * self.R1, self.a1 * self.R2
        self.nhat = LD(2 * np.pi) / self.pb
        nD = self.nhat * self.Drep
        self.delayI = self.Dre * (1 - nD + nD ** 2 + 0.5 * self.nhat ** 2 * self.Dre * self.Drepp)
        self.delayS = -2 * self.TM2 * np.log(1 - self.SINI * s[1])
        self.delay = self.delayI + self.delayS

    def deriv(self, par):
        """d_ELL1delay_d_par (ELL1_model.py:637) per SI unit of par."""
        tt0, PBs = self.tt0, self.PBs
        z = np.zeros_like(tt0)
        d_a1 = d_Phi = d_e1 = d_e2 = d_pb = d_TM2 = d_SINI = z
        if par == "A1": d_a1 = z + 1
        elif par == "A1DOT": d_a1 = tt0
        elif par == "EPS1": d_e1 = z + 1
        elif par == "EPS1DOT": d_e1 = tt0
        elif par == "EPS2": d_e2 = z + 1
        elif par == "EPS2DOT": d_e2 = tt0
        elif par == "TASC":
            d_e1, d_e2 = z - self.E1DOT, z - self.E2DOT
            d_Phi = (self.PBDOT * tt0 / self.pb - 1.0) * LD(2 * np.pi) / self.pb
        elif par == "PB":
            d_Phi = LD(2 * np.pi) * ((self.PBDOT + self.XPBDOT) * tt0 ** 2 / PBs ** 3 - tt0 / PBs ** 2)
            d_pb = z + 1
        elif par == "PBDOT":
            d_Phi = -LD(np.pi) * tt0 ** 2 / PBs ** 2
            d_pb = tt0
        elif par == "XPBDOT": d_Phi = -LD(np.pi) * tt0 ** 2 / PBs ** 2
        elif par == "M2": d_TM2 = z + LD(TSUN)
        elif par == "SINI": d_SINI = z + 1
        else: return z
        s, c, e1, e2, a1 = self.s, self.c, self.e1, self.e2, self.a1
        nhat, Dre, Drep, Drepp = self.nhat, self.Dre, self.Drep, self.Drepp
        d_nhat = -LD(2 * np.pi) / self.pb ** 2 * d_pb
        dDre_de1 = a1 * (-0.5 * c[2] - (1.0 / 8) * (-2 * e2 * c[1] + 6 * e2 * c[3] + 6 * e1 * s[1] + 6 * e1 * s[3])
                         - (1.0 / 12) * (6 * e1 * e2 * s[2] - 6 * e2 ** 2 * c[2] - 12 * e1 ** 2 * c[2]
                                         + 24 * e1 * e2 * s[4] + 12 * e2 ** 2 * c[4] - 12 * e1 ** 2 * c[4]))
        dDre_de2 = a1 * (0.5 * s[2] - (1.0 / 8) * (-2 * e1 * c[1] + 6 * e1 * c[3] + 10 * e2 * s[1] - 6 * e2 * s[3])
                         - (1.0 / 12) * (15 * e2 ** 2 * s[2] + 3 * e1 ** 2 * s[2] - 12 * e1 * e2 * c[2]
                                         - 12 * e2 ** 2 * s[4] + 12 * e1 ** 2 * s[4] + 24 * e1 * e2 * c[4]))
        dDre = d_a1 * self.R0 + Drep * d_Phi + dDre_de1 * d_e1 + dDre_de2 * d_e2
        dDrep_de1 = a1 * (s[2] - (1.0 / 8) * (6 * e1 * c[1] + 18 * e1 * c[3] + 2 * e2 * s[1] - 18 * e2 * s[3])
                          - (1.0 / 12) * (12 * e1 * e2 * c[2] + 12 * e2 ** 2 * s[2] + 16 * e1 ** 2 * s[2]
                                          + 96 * e1 * e2 * c[4] - 48 * e2 ** 2 * s[4] + 48 * e1 ** 2 * s[4]))
        dDrep_de2 = a1 * (c[2] - (1.0 / 8) * (2 * e1 * s[1] - 18 * e1 * s[3] + 10 * e2 * c[1] - 18 * e2 * c[3])
                          - (1.0 / 12) * (30 * e2 ** 2 * c[2] + 6 * e1 ** 2 * c[2] + 24 * e1 * e2 * s[2]
                                          - 48 * e2 ** 2 * c[4] + 48 * e1 ** 2 * c[4] - 96 * e1 * e2 * s[4]))
        dDrep = d_a1 * self.R1 + Drepp * d_Phi + dDrep_de1 * d_e1 + dDrep_de2 * d_e2
        dDrepp_dPhi = a1 * (-c[1] - 4.0 * (e1 * s[2] + e2 * c[2])
                            - (1.0 / 8) * (-5 * e2 ** 2 * c[1] + 81 * e2 ** 2 * c[3] - 2 * e1 * e2 * s[1]
                                           + 162 * e1 * e2 * s[3] - 3 * e1 ** 2 * c[1] - 81 * e1 ** 2 * c[3])
                            - (1.0 / 12) * (-40 * e2 ** 3 * c[2] - 24 * e1 ** 2 * e2 * c[2] - 48 * e1 * e2 ** 2 * s[2]
                                            - 32 * e1 ** 3 * s[2] + 256 * e2 ** 3 * c[4] - 768 * e1 ** 2 * e2 * c[4]
                                            + 768 * e1 * e2 ** 2 * s[4] - 256 * e1 ** 3 * s[4]))
        dDrepp_de1 = a1 * (2.0 * c[2] - (1.0 / 8) * (-6 * e1 * s[1] - 54 * e1 * s[3] + 2 * e2 * c[1] - 54 * e2 * c[3])
                           - (1.0 / 12) * (-24 * e1 * e2 * s[2] + 24 * e2 ** 2 * c[2] + 48 * e1 ** 2 * c[2]
                                           - 384 * e1 * e2 * s[4] - 192 * e2 ** 2 * c[4] + 192 * e1 ** 2 * c[4]))
        dDrepp_de2 = a1 * (-2.0 * s[2] - (1.0 / 8) * (2 * e1 * c[1] - 54 * e1 * c[3] - 10 * e2 * s[1] + 54 * e2 * s[3])
                           - (1.0 / 12) * (-60 * e2 ** 2 * s[2] - 12 * e1 ** 2 * s[2] + 48 * e1 * e2 * c[2]
                                           + 192 * e2 ** 2 * s[4] - 192 * e1 ** 2 * s[4] - 384 * e1 * e2 * c[4]))
        dDrepp = d_a1 * self.R2 + dDrepp_dPhi * d_Phi + dDrepp_de1 * d_e1 + dDrepp_de2 * d_e2
        nD = nhat * Drep
        dI = ((1 - nD + nD ** 2 + 0.5 * nhat ** 2 * Dre * Drepp) + Dre * 0.5 * nhat ** 2 * Drepp) * dDre \
            + (-Dre * nhat + 2 * nD * nhat * Dre) * dDrep + 0.5 * (nhat * Dre) ** 2 * dDrepp \
            + Dre * (-Drep + 2 * nD * Drep + nhat * Dre * Drepp) * d_nhat
        lg = 1 - self.SINI * s[1]
        # ELL1_model.py:620 d_delayS_d_Phi without cos(Phi) -- reproduced as in the reference
        dS = -2 * np.log(lg) * d_TM2 + (-2 * self.TM2 / lg * (-s[1])) * d_SINI + (-2 * self.TM2 / lg * (-self.SINI)) * d_Phi
        return dI + dS


class _ELL1H(_ELL1):
    """ELL1H_model.py (Freire & Wex 2010) on binary_ell1.py:312-417's setup: ELL1's delayI
    plus the H3 Shapiro delay, no M2/SINI.  Modes (binary_ell1.py:383-405): H3 alone -> the
    approximate 3rd-and-higher harmonics (Eq. 19) with stigma = 0; H3 + H4 -> the same with
    stigma = H4/H3 and NHARMS = max(NHARMS, 7); H3 + STIGMA -> the exact form (Eq. 29)."""

    def __init__(self, om, bt_days, acc):
        super().__init__(om, bt_days, acc)  # M2 = SINI = 0: ELL1's delayS vanishes
        H3 = LD(om.v("H3"))
        self.H3 = H3
        P = self.Phi
        if om.has("H4"):
            self.mode = 2
            H4 = LD(om.v("H4"))
            self.sig = LD(0) if H3 == 0 else H4 / H3
            self.dsig_dH3 = LD(0) if H3 == 0 else -H4 / H3 / H3
            self.dsig_dH4 = LD(0) if H3 == 0 else 1 / H3
            self.N = max(int(om.v("NHARMS", 7) or 7), 7)
        elif om.has("STIGMA"):
            self.mode = 3
            self.sig = LD(om.v("STIGMA"))
            self.dsig_dH3, self.dsig_dH4 = LD(0), LD(0)
        else:
            self.mode = 1
            self.sig = LD(0)
            self.dsig_dH3, self.dsig_dH4 = LD(0), LD(0)
            self.N = int(om.v("NHARMS", 3) or 3)
        sg = self.sig
        if self.mode == 3:
            lg = 1 + sg * sg - 2 * sg * np.sin(P)
            self.dS = -2 * H3 / sg ** 3 * np.log(lg)
            self.dS_dH3 = -2 / sg ** 3 * np.log(lg)
            self.dS_dsig = -2 * H3 / sg ** 4 * (-3 * np.log(lg) + 2 * sg * (sg - np.sin(P)) / lg)
            self.dS_dPhi = 4 * H3 / sg ** 2 * (np.cos(P) / lg)
        else:
            # Eq. (19): -2 H3 sum_{k=3}^{N} c_k stigma^(k-3) basis_k(k Phi), c_k = (-1)^pwr 2/k,
            # odd k: sin, pwr = (k+1)/2; even k: cos, pwr = (k+2)/2 (ELL1H_model.py:90-140)
            f = np.zeros_like(P)
            fs = np.zeros_like(P)
            fp = np.zeros_like(P)
            for k in range(3, self.N + 1):
                pwr = (k + 1) // 2 if k % 2 else (k + 2) // 2
                ck = LD((-1) ** pwr * 2.0 / k)
                b = np.sin(k * P) if k % 2 else np.cos(k * P)
                db = k * np.cos(k * P) if k % 2 else -k * np.sin(k * P)
                f = f + ck * sg ** (k - 3) * b
                fp = fp + ck * sg ** (k - 3) * db
                if k > 3:
                    fs = fs + ck * (k - 3) * sg ** (k - 4) * b
            self.dS = -2 * H3 * f
            self.dS_dH3 = -2 * f
            self.dS_dsig = -2 * H3 * fs
            self.dS_dPhi = -2 * H3 * fp
        self.delayS = self.dS
        self.delay = self.delayI + self.dS

    def deriv(self, par):
        """d_ELL1Hdelay_d_par: d_delayI_d_par + d_delayS_d_par (ELL1H_model.py:326-359)."""
        base = super().deriv(par) if par not in ("H3", "H4", "STIGMA") else np.zeros_like(self.tt0)
        tt0, PBs = self.tt0, self.PBs
        d_Phi = LD(0)
        if par == "TASC":
            d_Phi = (self.PBDOT * tt0 / self.pb - 1.0) * LD(2 * np.pi) / self.pb
        elif par == "PB":
            d_Phi = LD(2 * np.pi) * ((self.PBDOT + self.XPBDOT) * tt0 ** 2 / PBs ** 3 - tt0 / PBs ** 2)
        elif par in ("PBDOT", "XPBDOT"):
            d_Phi = -LD(np.pi) * tt0 ** 2 / PBs ** 2
        d_sig = {"H3": self.dsig_dH3, "H4": self.dsig_dH4, "STIGMA": LD(1)}.get(par, LD(0))
        d_H3 = LD(1) if par == "H3" else LD(0)
        return base + self.dS_dH3 * d_H3 + self.dS_dPhi * d_Phi + self.dS_dsig * d_sig


class _BT:
    """BT_model.py (Blandford & Teukolsky 1976): (delayL1 + delayL2) * delayR with
    omega = OM + OMDOT tt0 (binary_generic.py:631), and the reference's derivative chain
    d_BTdelay_d_par = delayR (dL1 + dL2) (:258; delayR's derivatives ignored, d_delayL1_d_ECC
    with +a1 sin(omega) as written at :189, T0 through E only)."""

    def __init__(self, om, bt_days, acc):
        tt0 = (bt_days - LD(om.v("T0"))) * LD(DAYSEC) - np.asarray(acc, dtype=LD)
        self.tt0 = tt0
        self.PBs = LD(om.v("PB")) * LD(DAYSEC)
        self.PBDOT, self.XPBDOT = LD(om.v("PBDOT")), LD(om.v("XPBDOT"))
        orbits, _, M = _orbits(om, tt0)
        self.pb = self.PBs + self.PBDOT * tt0
        self.EDOT = LD(om.v("EDOT"))
        self.ecc = LD(om.v("ECC")) + tt0 * self.EDOT
        self.A1DOT = LD(om.v("A1DOT"))
        self.a1 = LD(om.v("A1")) + tt0 * self.A1DOT
        self.GAMMA = LD(om.v("GAMMA"))
        e = self.ecc
        E = M.copy()
        for _ in range(100):  # compute_eccentric_anomaly (binary_generic.py:337)
            dE = (E - e * np.sin(E) - M) / (1 - e * np.cos(E))
            E = E - dE
            if np.all(np.abs(E - e * np.sin(E) - M) < 5e-15):
                break
        self.E = E
        self.omega = LD(om.v("OM")) * LD(DEG_RAD) + LD(om.v("OMDOT")) * LD(DEG_RAD / YR_S) * tt0
        sw, cw = np.sin(self.omega), np.cos(self.omega)
        sE, cE = np.sin(E), np.cos(E)
        sq = np.sqrt(1 - e * e)
        a1 = self.a1
        self.L1 = a1 * sw * (cE - e)
        self.L2 = (a1 * cw * sq + self.GAMMA) * sE
        num = a1 * cw * sq * cE - a1 * sw * sE
        self.R = 1.0 - LD(2 * np.pi) * num / ((1.0 - e * cE) * self.pb)
        self.delay = (self.L1 + self.L2) * self.R
        self.sw, self.cw, self.sE, self.cE, self.sq = sw, cw, sE, cE, sq

    def deriv(self, par):
        e, a1, tt0 = self.ecc, self.a1, self.tt0
        sw, cw, sE, cE, sq = self.sw, self.cw, self.sE, self.cE, self.sq
        iom = 1.0 / (1.0 - e * cE)
        dL1_dE = -a1 * sw * sE
        dL2_dE = (a1 * cw * sq + self.GAMMA) * cE
        z = np.zeros_like(tt0)
        PBs = self.PBs
        f = tt0 if par in ("A1DOT", "OMDOT", "EDOT") else z + 1
        if par in ("A1", "A1DOT"):
            dL1, dL2 = f * sw * (cE - e), f * cw * sq * sE
        elif par in ("OM", "OMDOT"):
            dL1, dL2 = f * a1 * cw * (cE - e), -f * a1 * sw * sq * sE
        elif par in ("ECC", "EDOT"):
            dEe = sE * iom
            dL1 = f * (a1 * sw + dL1_dE * dEe)
            dL2 = f * (-a1 * cw * e * sE / sq + dL2_dE * dEe)
        elif par == "GAMMA":
            dL1, dL2 = z, sE
        elif par in ("T0", "PB", "PBDOT", "XPBDOT"):
            if par == "T0":
                dM = ((self.PBDOT - self.XPBDOT) * tt0 / PBs - 1.0) * LD(2 * np.pi) / PBs
                dE = (dM - self.EDOT * sE) * iom
            elif par == "PB":
                dE = LD(2 * np.pi) * ((self.PBDOT + self.XPBDOT) * tt0 ** 2 / PBs ** 3 - tt0 / PBs ** 2) * iom
            else:
                dE = -LD(np.pi) * tt0 ** 2 / PBs ** 2 * iom
            dL1, dL2 = dL1_dE * dE, dL2_dE * dE
        else:
            return z
        return self.R * (dL1 + dL2)


class _DD:
    """DD_model.py + binary_generic.py (Kepler Newton, nu, omega, er/eTheta, alpha/beta,
    delayInverse, delayS, delayA) and the reference's prtl_der chain."""

    def __init__(self, om, bt_days, acc):
        self.om = om
        tt0 = (bt_days - LD(om.v("T0"))) * LD(DAYSEC) - np.asarray(acc, dtype=LD)
        self.tt0 = tt0
        self.PBs = LD(om.v("PB")) * LD(DAYSEC)
        self.PBDOT, self.XPBDOT = LD(om.v("PBDOT")), LD(om.v("XPBDOT"))
        self.orbits, self.norb, self.M = _orbits(om, tt0)
        self.pb = self.PBs + self.PBDOT * tt0
        self.A1DOT, self.EDOT = LD(om.v("A1DOT")), LD(om.v("EDOT"))
        self.a1 = LD(om.v("A1")) + tt0 * self.A1DOT
        self.ecc = LD(om.v("ECC")) + tt0 * self.EDOT
        e, M = self.ecc, self.M
        U = M.copy()
        for _ in range(100):  # binary_generic.py:337-370, global tolerance 5e-15
            k = U - e * np.sin(U) - M
            if np.max(np.abs(k)) <= 5e-15:
                break
            U = U - k / (1 - e * np.cos(U))
        self.E = U
        self.sE, self.cE = np.sin(U), np.cos(U)
        nu = 2 * np.arctan(np.sqrt((1.0 + e) / (1.0 - e)) * np.tan(U / 2.0))
        nu = np.where(nu < 0, nu + LD(2 * np.pi), nu)
        self.nu = LD(2 * np.pi) * self.orbits + nu - M  # unwrapped (binary_generic.py:538-549)
        self.OMDOT = LD(om.v("OMDOT")) * LD(DEG_RAD) / LD(YR_S)
        self.k = self.OMDOT / (LD(2 * np.pi) / self.pb)
        self.omega = LD(om.v("OM")) * LD(DEG_RAD) + self.nu * self.k
        self.SINI = LD(om.v("SINI"))
        self._kopeikin()
        self.DR, self.DTH = LD(om.v("DR")), LD(om.v("DTH"))
        self.er, self.eTh = e * (1 + self.DR), e * (1 + self.DTH)
        self.sw, self.cw = np.sin(self.omega), np.cos(self.omega)
        self.alpha = self.a1 * self.sw
        self.beta = self.a1 * np.sqrt(1 - self.eTh ** 2) * self.cw
        self.GAMMA = LD(om.v("GAMMA"))
        sE, cE = self.sE, self.cE
        self.Dre = self.alpha * (cE - self.er) + self.beta * sE + self.GAMMA * sE
        self.Drep = -self.alpha * sE + (self.beta + self.GAMMA) * cE
        self.Drepp = -self.alpha * cE - (self.beta + self.GAMMA) * sE
        self.nhat = LD(2 * np.pi) / self.pb / (1 - e * cE)
        nH = self.nhat
        dI = self.Dre * (1 - nH * self.Drep + (nH * self.Drep) ** 2 + 0.5 * nH ** 2 * self.Dre * self.Drepp
                         - 0.5 * e * sE / (1 - e * cE) * nH ** 2 * self.Dre * self.Drep)
        self.TM2 = LD(om.v("M2")) * LD(TSUN)
        self.logNum = 1 - e * cE - self.SINI * (self.sw * (cE - e) + np.sqrt(1 - e ** 2) * self.cw * sE)
        dS = -2 * self.TM2 * np.log(self.logNum)
        self.A0, self.B0 = LD(om.v("A0")), LD(om.v("B0"))
        oPn = self.omega + self.nu
        dA = self.A0 * (np.sin(oPn) + e * self.sw) + self.B0 * (np.cos(oPn) + e * self.cw)
        self.delay = dI + dS + dA

    def _kopeikin(self):
        """DDK's corrections to a1, omega and SINI (none for DD)."""

    def _kop_deriv(self, par):
        """DDK's extra d(a1)/d(par), d(omega)/d(par) (SI) and prtl_der('SINI', par)."""
        return 0.0, 0.0, (1.0 if par == "SINI" else 0.0)

    def deriv(self, par):
        """d_DDdelay_d_par (DD_model.py:855) per SI unit of par."""
        e, sE, cE, tt0, PBs = self.ecc, self.sE, self.cE, self.tt0, self.PBs
        z = np.zeros_like(tt0)
        orbit = par in ("PB", "PBDOT", "XPBDOT", "T0")
        d_ecc = d_a1 = d_M = d_pb = z
        if par == "T0":
            d_ecc, d_a1 = z - self.EDOT, z - self.A1DOT
            d_M = ((self.PBDOT - self.XPBDOT) * tt0 / PBs - 1.0) * LD(2 * np.pi) / PBs
            d_pb = z - self.PBDOT
        elif par == "ECC": d_ecc = z + 1
        elif par == "EDOT": d_ecc = tt0
        elif par == "A1": d_a1 = z + 1
        elif par == "A1DOT": d_a1 = tt0
        elif par == "PB":
            d_M = LD(2 * np.pi) * ((self.PBDOT + self.XPBDOT) * tt0 ** 2 / PBs ** 3 - tt0 / PBs ** 2)
            d_pb = z + 1
        elif par == "PBDOT": d_M, d_pb = -LD(np.pi) * tt0 ** 2 / PBs ** 2, tt0
        elif par == "XPBDOT": d_M = -LD(np.pi) * tt0 ** 2 / PBs ** 2
        ka1, kom, d_SI = self._kop_deriv(par)
        omeE = 1 - e * cE
        dEdECC = sE / (1.0 - e * cE)
        if par == "T0": d_E = (d_M - self.EDOT * sE) / (1.0 - cE * e)
        elif par == "ECC": d_E = dEdECC
        elif par == "EDOT": d_E = tt0 * dEdECC
        elif orbit: d_E = d_M / (1.0 - cE * e)
        else: d_E = z
        snu, cnu = np.sin(self.nu), np.cos(self.nu)
        dnu_dE = (1 + e * cnu) / (1 - e * cE) * (sE / snu)
        dnu_de = sE ** 2 / (e * cE - 1) ** 2 / snu
        if par == "T0": d_nu = dnu_de * (-self.EDOT) + dnu_dE * d_E
        elif par == "ECC": d_nu = dnu_de + dnu_dE * dEdECC
        elif par == "EDOT": d_nu = tt0 * (dnu_de + dnu_dE * dEdECC)
        elif orbit: d_nu = dnu_dE * d_E
        else: d_nu = z
        if par == "OM": d_om = z + 1
        elif par == "OMDOT": d_om = self.pb / LD(2 * np.pi) * self.nu
        elif orbit: d_om = d_nu * self.k + d_pb * self.nu * self.OMDOT / LD(2 * np.pi)
        else: d_om = self.k * d_nu
        d_om = d_om + kom
        d_a1 = d_a1 + ka1  # alpha and d_beta_d_par; DD's d_beta_d_T0 keeps d_a1_d_T0 (DD_model.py:352)
        d_er = e if par == "DR" else d_ecc
        d_eTh = e if par == "DTH" else d_ecc
        sw, cw, eTh = self.sw, self.cw, self.eTh
        sq = np.sqrt(1 - eTh ** 2)
        d_alpha = d_a1 * sw + self.a1 * cw * d_om
        if par == "A1": d_beta = sq * cw
        elif par == "A1DOT": d_beta = tt0 * sq * cw
        elif par == "T0": d_beta = -self.A1DOT * sq * cw
        elif par in ("ECC", "EDOT"):
            f = tt0 if par == "EDOT" else 1.0
            d_beta = self.a1 * ((-eTh) / sq * cw * f - sq * sw * d_om)
        elif par == "DTH": d_beta = self.a1 * (-eTh) / sq * cw
        else: d_beta = sq * cw * d_a1 + (-self.a1 * sq * sw) * d_om + (self.a1 * (-eTh) / sq * cw) * d_eTh
        d_g = z + (1.0 if par == "GAMMA" else 0.0)
        al, be, G = self.alpha, self.beta, self.GAMMA
        dDre = al * (-d_er - d_E * sE) + (cE - self.er) * d_alpha + (d_beta + d_g) * sE + (be + G) * cE * d_E
        dDrep = -sE * d_alpha - (al * cE + (be + G) * sE) * d_E + cE * (d_beta + d_g)
        dDrepp = -cE * d_alpha + (al * sE - (be + G) * cE) * d_E - sE * (d_beta + d_g)
        dPB = 1.0 if par == "PB" else 0.0
        d_nhat = -LD(2 * np.pi) / self.pb / omeE * (dPB / self.pb - (cE * d_ecc - e * sE * d_E) / omeE)
        Dre, Drep, Drepp, nH = self.Dre, self.Drep, self.Drepp, self.nhat
        x = -0.5 * e * sE / omeE
        dx = -sE / (2 * omeE ** 2) * d_ecc + e * (e - cE) / (2 * omeE ** 2) * d_E
        dI = (dDre * (1 + (Drep * nH) ** 2 + Dre * Drepp * nH ** 2 + Drep * nH * (2 * Dre * nH * x - 1))
              + dDrep * (Dre * nH * (2 * Drep * nH + Dre * nH * x - 1))
              + dDrepp * ((Dre * nH) ** 2 / 2) + dx * ((Dre * nH) ** 2 * Drep)
              + d_nhat * (Dre * (-Drep + 2 * Drep ** 2 * nH + nH * Dre * Drepp + 2 * x * nH * Dre * Drep)))
        sq1 = np.sqrt(1 - e ** 2)
        ln, TM2, SI = self.logNum, self.TM2, self.SINI
        d_TM2 = LD(TSUN) if par == "M2" else 0.0
        dS = (d_TM2 * (-2 * np.log(ln)) + d_ecc * (-2 * TM2 / ln * (-cE - SI * (-e * cw * sE / sq1 - sw)))
              + d_E * (-2 * TM2 / ln * (e * sE - SI * (sq1 * cE * cw - sE * sw)))
              + d_om * (2 * TM2 / ln * SI * ((cE - e) * cw - sq1 * sE * sw))
              + d_SI * (-2 * TM2 / ln * (-sq1 * cw * sE - (cE - e) * sw)))
        oPn = self.omega + self.nu
        if par == "A0": dA = e * sw + np.sin(oPn)
        elif par == "B0": dA = e * cw + np.cos(oPn)
        else:
            dA = (d_om * (self.A0 * (np.cos(oPn) + e * cw) - self.B0 * (np.sin(oPn) + e * sw))
                  + d_nu * (self.A0 * np.cos(oPn) - self.B0 * np.sin(oPn)) + d_ecc * (self.A0 * sw + self.B0 * cw))
        return dI + dS + dA


class _DDK(_DD):
    """DDK_model.py: DD with Kopeikin (1995) annual-orbital parallax terms on a1 and omega
    (:355-524, Eqs. 15-19) and, with K96, the Kopeikin (1996) proper-motion terms on a1,
    omega and the inclination (:157-349); SINI = sin(kin) (:140).  obs_pos and psr_pos are
    in the astrometry's frame (pulsar_binary.py:398-416).  Derivatives follow the
    reference's prtl_der chain: d_a1_d_par / d_omega_d_par gain d_delta_*_d_{KIN,KOM,T0}
    (:547-602), d_SINI_d_{KIN,KOM,T0} as written (:176-195, incl. its T0 and non-K96 forms),
    and DD's d_beta_d_T0 still uses binary_generic's d_a1_d_T0."""

    def __init__(self, om, bt_days, acc, obs_pos, psr_pos):
        self.obs_pos = np.asarray(obs_pos, dtype=float)
        self.psr_pos = np.asarray(psr_pos, dtype=float)
        super().__init__(om, bt_days, acc)

    def _kopeikin(self):
        om = self.om
        self.K96 = bool(om.v("K96", 1.0))
        ecl = "AstrometryEcliptic" in om.comps
        pml = LD(om.v("PMELONG" if ecl else "PMRA")) * LD(MASYR_RADS)
        pmb = LD(om.v("PMELAT" if ecl else "PMDEC")) * LD(MASYR_RADS)
        KIN, KOM = LD(om.v("KIN")) * LD(DEG_RAD), LD(om.v("KOM")) * LD(DEG_RAD)
        sK, cK = np.sin(KOM), np.cos(KOM)
        tt0 = self.tt0
        A = -pml * sK + pmb * cK           # d kin / dt (delta_kin_proper_motion)
        Bv = pml * cK + pmb * sK
        dkin = A * tt0 if self.K96 else 0 * tt0
        kin = KIN + dkin
        sk, ck = np.sin(kin), np.cos(kin)
        tk = sk / ck
        # psr_pos setter (:106-121), delta_I0 / delta_J0 (:355-373)
        sl = self.psr_pos[:, 2].astype(LD)
        cl = np.cos(np.arcsin(sl))
        slo, clo = self.psr_pos[:, 1] / cl, self.psr_pos[:, 0] / cl
        ox, oy, oz = (self.obs_pos[:, i].astype(LD) for i in range(3))
        dI0 = -ox * slo + oy * clo
        dJ0 = -ox * sl * clo - oy * sl * slo + oz * cl
        ipx = LD(om.v("PX")) / LD(KPC_KM)  # 1/PX_kpc per km
        P1 = (dI0 * sK - dJ0 * cK) * ipx
        P2 = (dI0 * cK + dJ0 * sK) * ipx
        P3 = (-dI0 * sK + dJ0 * cK) * ipx
        a1b = self.a1
        a1pm = a1b * dkin / tk if self.K96 else 0 * tt0
        a1p = a1b + a1pm
        self.a1 = a1p + a1p / tk * P1
        wpm = Bv / sk * tt0 if self.K96 else 0 * tt0
        self.omega = self.omega + wpm - P2 / sk
        self.SINI = sk
        # derivative pieces per (KIN, KOM, T0), SI units
        z = 0 * tt0
        dk = {"KIN": z + 1, "KOM": -Bv * tt0 if self.K96 else z, "T0": z - A if self.K96 else z}
        dpm_a1 = {"KIN": -a1b * dkin / sk ** 2,
                  "KOM": a1b * (-Bv * tt0) * (-dkin / sk ** 2 + 1 / tk),
                  "T0": a1b * (-A) * (-dkin / sk ** 2 + 1 / tk)} if self.K96 else {k: z for k in dk}
        base_a1 = {"KIN": z, "KOM": z, "T0": z - self.A1DOT}
        out = {}
        for p in ("KIN", "KOM", "T0"):
            da1p = base_a1[p] + dpm_a1[p]   # d_a1_k_d_par(p, pm=K96, px=False)
            dpx = (da1p / tk - a1p * dk[p] / sk ** 2) * P1
            if p == "KOM":
                dpx = dpx + a1p / tk * P2
            ka1 = dpm_a1[p] + dpx
            if self.K96:
                if p == "KIN":
                    dwpm = -ck / sk ** 2 * Bv * tt0
                elif p == "KOM":
                    dwpm = (-ck / sk ** 2 * (-Bv * tt0) * Bv + A / sk) * tt0
                else:
                    dwpm = (-ck / sk ** 2 * (-A) * tt0 - 1 / sk) * Bv
            else:
                dwpm = z
            dwpx = ck / sk ** 2 * dk[p] * P2
            if p == "KOM":
                dwpx = dwpx - P3 / sk
            if p == "KIN":
                dsi = ck
            elif p == "KOM":  # non-K96: cos(kin) per degree, 1 per day (:180-195)
                dsi = -Bv * tt0 * ck if self.K96 else ck / LD(DEG_RAD)
            else:
                dsi = z - A if self.K96 else z + 1 / LD(DAYSEC)
            out[p] = (ka1, dwpm + dwpx, dsi)
        self._kd = out

    def _kop_deriv(self, par):
        return self._kd.get(par, (0.0, 0.0, 0.0))


BIN_UNIT = {"PB": DAYSEC, "T0": DAYSEC, "TASC": DAYSEC, "OM": DEG_RAD, "OMDOT": DEG_RAD / YR_S,
            "EPS1DOT": 1e-12, "EPS2DOT": 1e-12, "KIN": DEG_RAD, "KOM": DEG_RAD}
BIN_PARAMS = {"PB", "PBDOT", "XPBDOT", "A1", "A1DOT", "ECC", "EDOT", "T0", "OM", "OMDOT", "M2", "SINI", "GAMMA",
              "DR", "DTH", "A0", "B0", "TASC", "EPS1", "EPS2", "EPS1DOT", "EPS2DOT", "H3", "H4", "STIGMA",
              "KIN", "KOM"}


# ----------------------------------------------------------------------------------
# delays, phase (timing_model.py:1515, :1548)
# ----------------------------------------------------------------------------------
def _dmx_bins(om, mjd):
    out = []
    for n in om.prefix(r"^DMX_(\d+)$"):
        tag = n.split("_")[1]
        r1, r2 = float(om.v("DMXR1_" + tag)), float(om.v("DMXR2_" + tag))
        out.append((n, (mjd >= r1) & (mjd <= r2)))
    return out


def evaluate(om: OModel, toas: dict, with_tzr=True):
    """Per-component delays (float64 accumulation, timing_model.py:1531-1545), phase in
    longdouble, and intermediates for the design matrix.  Row order: TOAs then TZR."""
    R = _rows(toas, with_tzr)
    n = len(R["tdb_hi"])
    tdb = R["tdb_hi"].astype(LD) + R["tdb_lo"].astype(LD)
    tdb_f = tdb.astype(float)
    pos, vel, sun = R["ssb_obs_pos_km"], R["ssb_obs_vel_kms"], R["obs_sun_pos_km"]
    out = {"tdb": tdb}
    delay = np.zeros(n)
    L = np.tile([0.0, 0.0, 1.0], (n, 1))
    astro = "AstrometryEquatorial" in om.comps or "AstrometryEcliptic" in om.comps
    if astro:
        L = psr_dir_icrs(om, tdb_f)
        c = np.all(pos != 0, axis=1)
        rdl = (pos * L).sum(1)
        d = np.where(c, -rdl / C_KMS, 0.0)
        px = float(om.v("PX"))
        if px != 0:
            rr = (pos * pos).sum(1)
            Lkm = KPC_KM / px
            d = d + np.where(c, 0.5 * (rr / Lkm) * (1 - rdl ** 2 / rr) / C_KMS, 0.0)
        out["geometric"] = d
        delay += d
    if "SolarSystemShapiro" in om.comps and astro:
        nb = R["is_bary"] == 0
        r = np.linalg.norm(sun, axis=1)
        rct = (sun * L).sum(1)
        d = np.where(nb, -2.0 * TSUN * np.log((r - rct) / AU_KM), 0.0)
        if om.v("PLANET_SHAPIRO"):
            # solar_system_shapiro.py:110-117: each planet's term added in this order
            for pl, ratio in PLANETS:
                pp = R[f"obs_{pl}_pos_km"]
                rp = np.linalg.norm(pp, axis=1)
                d = d + np.where(nb, -2.0 * (TSUN / ratio) * np.log((rp - (pp * L).sum(1)) / AU_KM), 0.0)
        out["shapiro"] = d
        delay += d
    bfreq = R["freq_mhz"] * (1.0 - (vel * L).sum(1) / C_KMS) if astro else R["freq_mhz"]
    out["bfreq"] = bfreq
    dm_terms = ["DM"] + om.prefix(r"^DM(\d+)$") if om.has("DM") else []
    # dispersion_model.py:266-274: DMEPOCH unset -> 0
    dt_yr = (tdb - LD(om.v("DMEPOCH", 0.0))) / LD(DJY)
    out["dt_yr"] = dt_yr
    if dm_terms:
        x = dt_yr if any(LD(om.v(t)) != 0 for t in dm_terms[1:]) else np.zeros(n, dtype=LD)
        dm = np.zeros(n, dtype=LD)
        fact = len(dm_terms)
        for t in dm_terms[::-1]:  # utils.py:449 taylor_horner_deriv
            dm = dm * x / fact + LD(om.v(t))
            fact -= 1
        d = (dm * LD(DMCONST) / bfreq.astype(LD) ** 2).astype(float)
        out["dm"] = d
        delay += d
    dmx = _dmx_bins(om, R["mjd_float"])
    out["dmx_bins"] = dmx
    if dmx:
        v = np.zeros(n)
        for name, sel in dmx:
            v[sel] += float(om.v(name))
        d = v * DMCONST / bfreq ** 2
        out["dmx"] = d
        delay += d
    out["binary_obj"] = None
    if om.binary:
        bt = tdb  # barycentric days; acc_delay = delay so far (pulsar_binary.py:398)
        if om.binary == "DDK":  # obs_pos / psr_pos in the astrometry's frame (pulsar_binary.py:398-416)
            op, pp = pos, L
            if "AstrometryEcliptic" in om.comps:
                op, pp = _rot_icrs_to_ecl(OBL[om.ecl], pos), _rot_icrs_to_ecl(OBL[om.ecl], L)
            B = _DDK(om, bt, delay.astype(LD), op, pp)
        else:
            B = {"ELL1": _ELL1, "ELL1H": _ELL1H, "DD": _DD, "BT": _BT}[om.binary](om, bt, delay.astype(LD))
        d = B.delay.astype(float)
        out["binary"] = d
        out["binary_obj"] = B
        delay += d
    fds = om.prefix(r"^FD(\d+)$")
    logf = np.log(bfreq / 1000.0)
    logf = np.where(np.isfinite(logf), logf, 0.0)
    out["logf"] = logf
    if fds:
        d = np.polyval([float(om.v(f)) for f in fds[::-1]] + [0.0], logf)
        out["fd"] = d
        delay += d
    out["delay"] = delay
    # spindown phase (spindown.py:124-155): dt in longdouble seconds
    F = [LD(om.v(f)) for f in om.prefix(r"^F(\d+)$")]
    dt = (tdb - LD(om.v("PEPOCH"))) * LD(DAYSEC) - delay.astype(LD)
    ph = np.zeros(n, dtype=LD)
    coeffs = [LD(0)] + F
    fact = len(coeffs)
    for cf in coeffs[::-1]:
        ph = ph * dt / fact + cf
        fact -= 1
    # jumps (jump.py:119): JUMP * F0 on selected TOAs
    for name in sorted((k for k in om.masks if re.match(r"^JUMP\d+$", k)), key=lambda x: int(x[4:])):
        sel = select_rows(toas, *om.masks[name], with_tzr=with_tzr)
        ph = ph + np.where(sel, LD(om.v(name)) * F[0], LD(0))
    # PhaseOffset.offset_phase (phase_offset.py): -PHOFF on the TOAs, 0 on the TZR TOA
    if "PhaseOffset" in om.comps:
        off = np.full(n, -LD(om.v("PHOFF")), dtype=LD)
        if with_tzr:
            off[-1] = LD(0)
        ph = ph + off
    out["phase"] = ph
    out["dt"] = dt
    out["dt0"] = (tdb - LD(om.v("PEPOCH"))) * LD(DAYSEC)
    out["L"] = L
    return out


def _taylor_freq(F, dt):
    r = np.zeros_like(dt) + F[-1]
    for j in range(len(F) - 1, 0, -1):
        r = r * dt / j + F[j - 1]
    return r


def scaled_sigma_us(om, toas):
    """ScaleToaError.scale_toa_sigma (noise_model.py:159): EQUADs then EFACs."""
    s = np.array(toas["err_us"], dtype=float)
    for n in sorted((k for k in om.masks if re.match(r"^EQUAD\d+$", k)), key=lambda x: int(x[5:])):
        sel = select_mask(toas, *om.masks[n])
        s[sel] = np.hypot(s[sel], float(om.v(n)))
    for n in sorted((k for k in om.masks if re.match(r"^EFAC\d+$", k)), key=lambda x: int(x[4:])):
        sel = select_mask(toas, *om.masks[n])
        s[sel] *= float(om.v(n))
    return s


def residuals(om: OModel, toas: dict, track_mode=None, subtract_mean=True, use_weighted_mean=True):
    """Residuals.calc_phase_resids / calc_time_resids (residuals.py:314-538); no implicit
    mean subtraction with a PhaseOffset (residuals.py:124-128, :348-352)."""
    subtract_mean = subtract_mean and "PhaseOffset" not in om.comps
    ev = evaluate(om, toas, True)
    ph = ev["phase"]
    n = len(toas["tdb_hi"])
    dpn = np.asarray(toas.get("delta_pulse_number", np.zeros(n)), dtype=LD)
    rel = ph[:n] - ph[n] + dpn
    if track_mode is None:
        pn = toas.get("pulse_number")
        track_mode = "use_pulse_numbers" if pn is not None and not np.any(np.isnan(pn)) else "nearest"
    if track_mode == "use_pulse_numbers":
        full = rel - np.asarray(toas["pulse_number"], dtype=LD)
    else:
        x = rel - rel[0] if subtract_mean else rel
        full = x - np.floor(x + LD(0.5))
    sig = scaled_sigma_us(om, toas)
    if subtract_mean:
        w = 1.0 / sig ** 2 if use_weighted_mean else np.ones(n)
        full = full - (w * full).sum() / w.sum()
    F = [LD(om.v(f)) for f in om.prefix(r"^F(\d+)$")]
    ft = _taylor_freq(F, ev["dt0"][:n])
    tr = (full / ft).astype(float)
    return {"time": tr, "phase": full.astype(float), "sigma_us": sig, "track_mode": track_mode, "eval": ev}


def chi2_wls(r, sigma_us):
    """residuals.py:638."""
    return float(((r / (sigma_us * 1e-6)) ** 2).sum())


# ----------------------------------------------------------------------------------
# design matrix (timing_model.py:2073-2175)
# ----------------------------------------------------------------------------------
def designmatrix(om: OModel, toas: dict):
    ev = evaluate(om, toas, True)
    n = len(toas["tdb_hi"])
    F = [LD(om.v(f)) for f in om.prefix(r"^F(\d+)$")]
    F0 = float(F[0])
    dt = ev["dt"][:n]
    fdt = _taylor_freq(F, dt).astype(float)
    chain = fdt / F0  # -(d_phase_d_delay * d_delay_d_p)/F0 with d_phase_d_delay = -F(dt)
    pos = np.asarray(toas["ssb_obs_pos_km"])
    rr = (pos * pos).sum(1)
    r_km = np.sqrt(rr)
    edec = np.arctan2(pos[:, 2], np.hypot(pos[:, 0], pos[:, 1]))
    era = np.arctan2(pos[:, 1], pos[:, 0])
    ecl = "AstrometryEcliptic" in om.comps
    if ecl:
        obl = OBL[om.ecl]
        c, s = np.cos(obl), np.sin(obl)
        u = np.stack([np.cos(era) * np.cos(edec), np.sin(era) * np.cos(edec), np.sin(edec)], 1)
        ue = np.stack([u[:, 0], c * u[:, 1] + s * u[:, 2], -s * u[:, 1] + c * u[:, 2]], 1)
        era = np.arctan2(ue[:, 1], ue[:, 0])
        edec = np.arctan2(ue[:, 2], np.hypot(ue[:, 0], ue[:, 1]))
        plon, plat = float(om.v("ELONG")) * DEG_RAD, float(om.v("ELAT")) * DEG_RAD
        lonf = DEG_RAD
    else:
        plon, plat = float(om.v("RAJ", 0)) * HA_RAD, float(om.v("DECJ", 0)) * DEG_RAD
        lonf = HA_RAD
    te = ((ev["tdb"][:n] - LD(om.v("POSEPOCH", 0))) * LD(DAYSEC)).astype(float)
    L = ev["L"][:n]
    rdl = (pos * L).sum(1)
    bf = ev["bfreq"][:n]
    dt_yr = ev["dt_yr"][:n].astype(float)
    logf = ev["logf"][:n]
    dmx = {name: sel[:n] for name, sel in ev["dmx_bins"]}
    dm_terms = ["DM"] + om.prefix(r"^DM(\d+)$") if om.has("DM") else []
    fds = om.prefix(r"^FD(\d+)$")
    B = ev["binary_obj"]
    # the implicit Offset column unless a PhaseOffset is present (timing_model.py:2145)
    cols, names = ([], []) if "PhaseOffset" in om.comps else ([np.full(n, 1.0 / F0)], ["Offset"])
    for p in om.free:
        m = re.match(r"^F(\d+)$", p)
        if p == "PHOFF":  # -d_offset_phase_d_PHOFF / F0 (phase_offset.py)
            col = np.full(n, 1.0 / F0)
        elif m:
            k = int(m.group(1))
            col = -(dt ** (k + 1) / LD(math.factorial(k + 1))).astype(float) / F0
        elif p in ("RAJ", "ELONG"):
            col = chain * r_km * np.cos(edec) * np.cos(plat) * np.sin(plon - era) / C_KMS * lonf
        elif p in ("DECJ", "ELAT"):
            g = np.cos(edec) * np.sin(plat) * np.cos(plon - era) - np.sin(edec) * np.cos(plat)
            col = chain * r_km * g / C_KMS * DEG_RAD
        elif p in ("PMRA", "PMELONG"):
            col = chain * r_km * np.cos(edec) * np.sin(plon - era) * te / C_KMS * MASYR_RADS
        elif p in ("PMDEC", "PMELAT"):
            g = np.cos(edec) * np.sin(plat) * np.cos(plon - era) - np.cos(plat) * np.sin(edec)
            col = chain * r_km * g * te / C_KMS * MASYR_RADS
        elif p == "PX":
            col = chain * 0.5 * (rr - rdl ** 2) / (AU_KM * C_KMS) * MAS_RAD
        elif p in dm_terms:
            k = dm_terms.index(p)
            col = chain * DMCONST * dt_yr ** k / math.factorial(k) / bf ** 2
        elif p in dmx:
            col = chain * DMCONST * dmx[p].astype(float) / bf ** 2
        elif p in fds:
            col = chain * logf ** (fds.index(p) + 1)
        elif re.match(r"^JUMP\d+$", p):
            col = np.where(select_mask(toas, *om.masks[p]), -1.0, 0.0)
        elif re.match(r"^DMJUMP\d+$", p):  # DMJUMPs leave the delay alone (dispersion_model.py:797)
            col = np.zeros(n)
        elif p in BIN_PARAMS and B is not None:
            d = B.deriv(p)[:n].astype(float)
            col = chain * d * BIN_UNIT.get(p, 1.0)
        elif re.match(r"^(EFAC|EQUAD|ECORR|TNEQ|DMEFAC|DMEQUAD)\d+$", p) or p.startswith(("TNRED", "RN")):
            continue
        else:
            raise ValueError(f"unfittable {p}")
        cols.append(np.asarray(col, dtype=float))
        names.append(p)
    return np.stack(cols, axis=1), names


# ----------------------------------------------------------------------------------
# noise bases and fitters
# ----------------------------------------------------------------------------------
def red_noise(om, toas):
    """PLRedNoise basis and weights (noise_model.py:761-892)."""
    nf = int(om.v("TNREDC", 30)) if om.has("TNREDC") else 30
    if om.has("TNREDAMP") and om.has("TNREDGAM"):
        amp, gam = 10 ** float(om.v("TNREDAMP")), float(om.v("TNREDGAM"))
    else:
        fac = (86400.0 * 365.24 * 1e6) / (2.0 * np.pi * np.sqrt(3.0))
        amp, gam = float(om.v("RNAMP")) / fac, -float(om.v("RNIDX"))
    t = (np.asarray(toas["tdb_hi"], dtype=LD) + np.asarray(toas["tdb_lo"], dtype=LD)) * LD(86400)
    T = t.max() - t.min()
    f = np.linspace(1 / T, nf / T, nf)
    ff = np.zeros(2 * nf)
    ff[::2] = f
    ff[1::2] = f
    Fm = np.zeros((len(t), 2 * nf))
    Fm[:, ::2] = np.sin(2 * np.pi * t[:, None] * ff[::2])
    Fm[:, 1::2] = np.cos(2 * np.pi * t[:, None] * ff[1::2])
    phi = amp ** 2 / 12.0 / np.pi ** 2 * (1 / 3.16e7) ** (gam - 3) * ff ** (-gam)
    return Fm, phi * ff[0]


def ecorr_basis(om, toas):
    """EcorrNoise quantization matrix and weights (noise_model.py:385-427, :808-844)."""
    t = ((np.asarray(toas["tdb_hi"], dtype=LD) + np.asarray(toas["tdb_lo"], dtype=LD)) * LD(86400)).astype(float)
    mats, wts = [], []
    for n in sorted((k for k in om.masks if re.match(r"^ECORR\d+$", k)), key=lambda x: int(x[5:])):
        sel = np.where(select_mask(toas, *om.masks[n]))[0]
        ts = t[sel]
        isort = np.argsort(ts)
        buckets, ref = [], []
        for i in isort:
            if ref and ts[i] - ref[-1] < 1.0:
                buckets[-1].append(i)
            else:
                ref.append(ts[i])
                buckets.append([i])
        eps = [b for b in buckets if len(b) >= 2]
        U = np.zeros((len(t), len(eps)))
        for j, b in enumerate(eps):
            U[sel[b], j] = 1.0
        mats.append(U)
        wts.append(np.full(len(eps), (float(om.v(n)) * 1e-6) ** 2))
    return mats, wts


def dm_noise(om, toas):
    """PLDMNoise basis and weights (noise_model.py:443-540): the Fourier basis of TNDMC modes
    scaled by (1400 MHz / f_bary)^2 per TOA, weights powerlaw(f, 10^TNDMAMP, TNDMGAM) f_1."""
    nf = int(om.v("TNDMC", 30)) if om.has("TNDMC") else 30
    amp, gam = 10 ** float(om.v("TNDMAMP")), float(om.v("TNDMGAM"))
    t = (np.asarray(toas["tdb_hi"], dtype=LD) + np.asarray(toas["tdb_lo"], dtype=LD)) * LD(86400)
    T = t.max() - t.min()
    f = np.linspace(1 / T, nf / T, nf)
    ff = np.zeros(2 * nf)
    ff[::2] = f
    ff[1::2] = f
    n = len(t)
    bf = np.asarray(evaluate(om, toas, True)["bfreq"][:n], dtype=float)
    D = (1400.0 / bf) ** 2
    Fm = np.zeros((n, 2 * nf))
    Fm[:, ::2] = np.sin(2 * np.pi * t[:, None] * ff[::2])
    Fm[:, 1::2] = np.cos(2 * np.pi * t[:, None] * ff[1::2])
    phi = amp ** 2 / 12.0 / np.pi ** 2 * (1 / 3.16e7) ** (gam - 3) * ff ** (-gam)
    return Fm * D[:, None], phi * ff[0]


def noise_basis(om, toas):
    """noise_model_designmatrix / noise_model_basis_weight (timing_model.py:1631-1660):
    PLRedNoise, then PLDMNoise, then ECORR (the reference's order of the three follows its
    component order, which is not fixed: tests compare blocks through noise_dims)."""
    mats, wts = [], []
    if "PLRedNoise" in om.comps:
        Fm, phi = red_noise(om, toas)
        mats.append(Fm)
        wts.append(phi)
    if "PLDMNoise" in om.comps:
        Fm, phi = dm_noise(om, toas)
        mats.append(Fm)
        wts.append(phi)
    em, ew = ecorr_basis(om, toas)
    mats += em
    wts += ew
    if not mats:
        return None, None
    return np.hstack(mats), np.concatenate(wts)


def ecorr_only(om):
    """calc_chi2's Sherman-Morrison branch (residuals.py:705-709): ECORR without
    time-correlated noise and with a PhaseOffset."""
    return "PhaseOffset" in om.comps and "PLRedNoise" not in om.comps and \
        any(re.match(r"^ECORR\d+$", k) for k in om.masks)


def chi2_ecorr(om, toas, r, sigma_us, lognorm=False):
    """_calc_ecorr_chi2 (residuals.py:591-636): TOAs outside every epoch by r^2/N, each
    ECORR epoch by sherman_morrison_dot (utils.py:3024-3071) with v = 1, w = ECORR^2."""
    if "PHOFF" not in om.free:
        raise AssertionError("the ECORR-only chi2 needs a free PHOFF (residuals.py:595-599)")
    mats, wts = ecorr_basis(om, toas)
    N = (sigma_us * 1e-6) ** 2
    U = np.hstack(mats) if mats else np.zeros((len(r), 0))
    w = np.concatenate(wts) if wts else np.zeros(0)
    noec = ~np.any(U.astype(bool), axis=1)
    chi2 = float(np.dot(r[noec], r[noec] / N[noec]))
    ld = float(np.sum(np.log(N[noec])))
    for j in range(U.shape[1]):
        m = U[:, j].astype(bool)
        Ninv = 1 / N[m]
        denom = 1 + w[j] * Ninv.sum()
        s = np.dot(r[m], Ninv)
        chi2 += float(np.dot(r[m], Ninv * r[m]) - w[j] * s * s / denom)
        ld += float(np.sum(np.log(N[m])) + np.log(denom))
    return (chi2, 0.5 * ld) if lognorm else chi2


def chi2_gls(om, toas, r, sigma_us):
    """_calc_gls_chi2 via woodbury_dot (residuals.py:567-589, utils.py:3074); the offset
    column of ones only without a free PHOFF (:583-585)."""
    if ecorr_only(om):
        return chi2_ecorr(om, toas, r, sigma_us)
    U, phi = noise_basis(om, toas)
    N = (sigma_us * 1e-6) ** 2
    if U is None:
        return chi2_wls(r, sigma_us)
    # a correlated-noise model takes the Woodbury form even when its basis has no columns
    # (ECORR without multi-TOA epochs): the offset column alone, unless PHOFF is free
    if "PHOFF" not in om.free:
        U = np.append(U, np.ones((len(r), 1)), axis=1)
        phi = np.append(phi, [1e40])
    if U.shape[1] == 0:
        return chi2_wls(r, sigma_us)
    xNy = np.sum(r * r / N)
    xNU = (r / N) @ U
    Sigma = np.diag(1 / phi) + (U.T / N) @ U
    cf = scipy.linalg.cho_factor(Sigma)
    return float(xNy - xNU @ scipy.linalg.cho_solve(cf, xNU))


# ----------------------------------------------------------------------------------
# wideband DM residuals (residuals.py:908-1071, :1146-1271)
# ----------------------------------------------------------------------------------
def total_dm(om: OModel, toas: dict) -> np.ndarray:
    """TimingModel.total_dm (timing_model.py:1593): DispersionDM.base_dm (Taylor series in
    years from DMEPOCH, dispersion_model.py:217-234) + DispersionDMX.dmx_dm (:659-678) +
    DispersionJump.jump_dm (-DMJUMP on the selected TOAs, :773-785); pc/cm^3."""
    n = len(toas["tdb_hi"])
    tdb = np.asarray(toas["tdb_hi"], dtype=LD) + np.asarray(toas["tdb_lo"], dtype=LD)
    out = np.zeros(n)
    dm_terms = ["DM"] + om.prefix(r"^DM(\d+)$") if om.has("DM") else []
    if dm_terms:
        if any(LD(om.v(t)) != 0 for t in dm_terms[1:]):
            x = ((tdb - LD(om.v("DMEPOCH", 0.0))) / LD(DJY)).astype(float)
        else:
            x = np.zeros(n)
        dm = np.zeros(n)
        fact = len(dm_terms)
        for t in dm_terms[::-1]:  # utils.py:449 taylor_horner
            dm = dm * x / fact + float(om.v(t))
            fact -= 1
        out = out + dm
    for name, sel in _dmx_bins(om, np.asarray(toas["mjd_float"], dtype=float)):
        out = out + np.where(sel, float(om.v(name)), 0.0)
    for name in sorted((k for k in om.masks if re.match(r"^DMJUMP\d+$", k)), key=lambda x: int(x[6:])):
        out = out + np.where(select_mask(toas, *om.masks[name]), -float(om.v(name)), 0.0)
    return out


def scaled_dm_sigma(om: OModel, toas: dict) -> np.ndarray:
    """ScaleDmError.scale_dm_sigma (noise_model.py:291-315): DMEQUADs (hypot), then DMEFACs."""
    s = np.array(toas["pp_dme"], dtype=float)
    for n in sorted((k for k in om.masks if re.match(r"^DMEQUAD\d+$", k)), key=lambda x: int(x[7:])):
        sel = select_mask(toas, *om.masks[n])
        s[sel] = np.hypot(s[sel], float(om.v(n)))
    for n in sorted((k for k in om.masks if re.match(r"^DMEFAC\d+$", k)), key=lambda x: int(x[6:])):
        sel = select_mask(toas, *om.masks[n])
        s[sel] *= float(om.v(n))
    return s


def dm_residuals(om: OModel, toas: dict, subtract_mean=False, use_weighted_mean=True):
    """WidebandDMResiduals.calc_resids / calc_chi2 (residuals.py:1000-1031): pp_dm - total_dm,
    the mean (weighted by the unscaled DM errors) removed only with subtract_mean; chi2 with
    the scaled errors."""
    r = np.asarray(toas["pp_dm"], dtype=float) - total_dm(om, toas)
    if subtract_mean:
        if use_weighted_mean:
            w = 1.0 / np.asarray(toas["pp_dme"], dtype=float) ** 2
            r = r - np.sum(r * w) / np.sum(w)
        else:
            r = r - r.mean()
    sig = scaled_dm_sigma(om, toas)
    return {"resids": r, "sigma": sig, "chi2": float(np.sum((r / sig) ** 2))}


def wideband_chi2(om: OModel, toas: dict) -> float:
    """WidebandTOAResiduals.calc_chi2 (residuals.py:1206-1246): a WidebandTOAFitter pass with
    no free parameters, i.e. GLS over [TOA rows; DM rows] with the Offset column (zero on the
    DM rows) and the TOA noise basis: the TOA residuals' GLS (offset-marginalised) chi2 plus
    the DM rows' white chi2."""
    rr = residuals(om, toas)
    c2 = chi2_gls(om, toas, rr["time"], rr["sigma_us"]) if noise_basis(om, toas)[0] is not None else \
        chi2_wls(rr["time"] - np.sum(rr["time"] / rr["sigma_us"] ** 2) / np.sum(1 / rr["sigma_us"] ** 2),
                 rr["sigma_us"])
    return c2 + dm_residuals(om, toas)["chi2"]


def dm_designmatrix(om: OModel, names, toas: dict) -> np.ndarray:
    """The DM rows' design matrix (TimingModel.d_dm_d_param, timing_model.py:2039, through
    DesignMatrixMaker("dm"), pint_matrix.py:395-439): Offset 0; DMk: dt^k/k! (dt in Julian
    years from DMEPOCH, dispersion_model.py:253-275); DMX_i: 1 in its bin (:684-708);
    DMJUMP: -1 on its TOAs (:787-795); every other parameter 0."""
    n = len(toas["tdb_hi"])
    tdb = np.asarray(toas["tdb_hi"], dtype=LD) + np.asarray(toas["tdb_lo"], dtype=LD)
    dm_terms = ["DM"] + om.prefix(r"^DM(\d+)$") if om.has("DM") else []
    x = ((tdb - LD(om.v("DMEPOCH", 0.0))) / LD(DJY)).astype(float)
    dmx = dict(_dmx_bins(om, np.asarray(toas["mjd_float"], dtype=float)))
    out = np.zeros((n, len(names)))
    for j, p in enumerate(names):
        if p in dm_terms:
            k = dm_terms.index(p)
            out[:, j] = x ** k / math.factorial(k)
        elif p in dmx:
            out[:, j] = dmx[p].astype(float)
        elif re.match(r"^DMJUMP\d+$", p):
            out[:, j] = np.where(select_mask(toas, *om.masks[p]), -1.0, 0.0)
    return out


def wideband_gls_step(om: OModel, toas: dict):
    """WidebandTOAFitter.fit_toas, one iteration (fitter.py:2465-2637, full_cov=False): the TOA
    design matrix + noise basis over the TOA rows, the DM design matrix (noise columns 0)
    over the DM rows, residuals [TOA residuals (s); DM residuals (pc/cm^3)] with errors [scaled
    TOA errors; scaled DM errors]; normalised columns; GLS with the noise priors; Cholesky
    (SVD fallback).  Returns the step, errors, covariance and the linearised chi2."""
    res = residuals(om, toas)
    M, names = designmatrix(om, toas)
    ntm = M.shape[1]
    Md = dm_designmatrix(om, names, toas)
    dr = dm_residuals(om, toas)
    U, phi = noise_basis(om, toas)
    phiinv = np.zeros(ntm)
    if U is not None:
        phiinv = np.concatenate((phiinv, 1 / phi))
        M = np.hstack((M, U))
        Md = np.hstack((Md, np.zeros((Md.shape[0], U.shape[1]))))
    M = np.vstack((M, Md))
    M, norm = _normalize(M)
    phiinv = phiinv / norm ** 2
    y = np.concatenate((res["time"], dr["resids"]))
    Nvec = np.concatenate(((res["sigma_us"] * 1e-6) ** 2, dr["sigma"] ** 2))
    cinv = 1 / Nvec
    mtcm = M.T @ (cinv[:, None] * M) + np.diag(phiinv)
    mtcy = M.T @ (cinv * y)
    try:
        c = scipy.linalg.cho_factor(mtcm)
        xhat = scipy.linalg.cho_solve(c, mtcy)
        xvar = scipy.linalg.cho_solve(c, np.eye(len(mtcy)))
    except scipy.linalg.LinAlgError:
        Uu, s, Vt = scipy.linalg.svd(mtcm, full_matrices=False)
        s = np.where(s <= 0, np.inf, s)
        xvar = (Vt.T / s) @ Vt
        xhat = Vt.T @ ((Uu.T @ mtcy) / s)
    newres = y - M @ xhat
    chi2 = float(newres @ (cinv * newres) + xhat @ (phiinv * xhat))
    dpars = xhat / norm
    errs = np.sqrt(np.diag(xvar)) / norm
    cov = (xvar / norm).T / norm
    return dict(dpars=dpars[:ntm], errs=errs[:ntm], cov=cov[:ntm, :ntm], names=names, chi2=chi2)


def lognorm(om, toas, r, sigma_us, gls=True):
    """Residuals.calc_chi2(lognorm=True)'s log_norm: sum log sigma_s (_calc_wls_chi2,
    residuals.py:638-667) or logdet(C)/2 (_calc_gls_chi2 :567-589 via woodbury_dot
    utils.py:3074-3126: logdet N + logdet Phi + slogdet Sigma, U = [noise basis, 1],
    Phi = [phi, 1e40])."""
    sig = sigma_us * 1e-6
    U, phi = noise_basis(om, toas) if gls else (None, None)
    if U is None:
        return float(np.sum(np.log(sig)))
    if ecorr_only(om):
        return chi2_ecorr(om, toas, r, sigma_us, lognorm=True)[1]
    # a correlated-noise model always takes the Woodbury form, with the offset column even
    # when its basis has no columns (ECORR without multi-TOA epochs), unless PHOFF is free
    N = sig ** 2
    if "PHOFF" not in om.free:
        U = np.append(U, np.ones((len(r), 1)), axis=1)
        phi = np.append(phi, [1e40])
    Sigma = np.diag(1 / phi) + (U.T / N) @ U
    _, ld_sigma = np.linalg.slogdet(Sigma)
    return float(0.5 * (np.sum(np.log(N)) + np.sum(np.log(phi)) + ld_sigma))


def lnlikelihood(om, toas, gls=True):
    """Residuals.lnlikelihood (residuals.py:713-716): -(chi2/2 + log_norm)."""
    r = residuals(om, toas)
    corr = gls and noise_basis(om, toas)[0] is not None
    c2 = chi2_gls(om, toas, r["time"], r["sigma_us"]) if corr else chi2_wls(r["time"], r["sigma_us"])
    return -(c2 / 2 + lognorm(om, toas, r["time"], r["sigma_us"], corr))


def lnlikelihood_of(om, toas, r):
    """Residuals.lnlikelihood (residuals.py:713) of FIXED time residuals r at om's noise
    values -- the objective DownhillFitter._fit_noise evaluates (fitter.py:1239-1247: one
    Residuals object, only its model's noise values change)."""
    sig = scaled_sigma_us(om, toas)
    corr = noise_basis(om, toas)[0] is not None
    c2 = chi2_gls(om, toas, r, sig) if corr else chi2_wls(r, sig)
    return -(c2 / 2 + lognorm(om, toas, r, sig, corr))


def d_lnlikelihood_d_param(om, toas, r, name):
    """Residuals.d_lnlikelihood_d_param (residuals.py:809-828) for EFAC/EQUAD without
    correlated noise: sum_i dlnL/dN_i dN_i/dp, dlnL/dN_i = -(-r^2/N^2 + 1/N)/2
    (residuals.py:718-728), dN_i/dp = 2 sigma_i dsigma_i/dp (:772-777) with
    dsigma/dEFAC = sigma/EFAC and dsigma/dEQUAD = sigma EQUAD / (sigma0^2 + sum EQUAD^2)
    on the parameter's mask (noise_model.py:183-214).  In s, us and 1/us as the reference."""
    if noise_basis(om, toas)[0] is not None:
        raise NotImplementedError("restated for white noise only")
    sig = scaled_sigma_us(om, toas)
    N = (sig * 1e-6) ** 2
    dl_dN = -0.5 * (-(r ** 2) / N ** 2 + 1 / N)
    sel = select_mask(toas, *om.masks[name])
    ds = np.zeros(len(r))
    if name.startswith("EFAC"):
        ds[sel] = sig[sel] * 1e-6 / float(om.v(name))
    elif name.startswith("EQUAD"):
        s2 = np.array(toas["err_us"], dtype=float) ** 2
        for n in (k for k in om.masks if re.match(r"^EQUAD\d+$", k)):
            m = select_mask(toas, *om.masks[n])
            s2[m] += float(om.v(n)) ** 2
        ds[sel] = sig[sel] * float(om.v(name)) / s2[sel] * 1e-6  # s per us
    else:
        raise NotImplementedError(name)
    return float(np.sum(dl_dN * 2 * sig * 1e-6 * ds))


def _normalize(M):
    norm = np.sqrt((M ** 2).sum(0))
    norm[norm == 0] = 1
    return M / norm, norm


def wls_step(om, toas, res=None):
    """WLSFitter.fit_toas one iteration (fitter.py:1965-2080): SVD of the whitened,
    normalised design matrix; threshold 1e-14 max(shape)."""
    res = res or residuals(om, toas)
    M, names = designmatrix(om, toas)
    Nvec = res["sigma_us"] * 1e-6
    Mw = M / Nvec[:, None]
    r = res["time"] / Nvec
    Mw, fac = _normalize(Mw)
    U, s, Vt = scipy.linalg.svd(Mw, full_matrices=False)
    thr = 1e-14 * max(Mw.shape)
    s = np.where(s <= thr * s[0], np.inf, s)
    dpars = (Vt.T @ ((U.T @ r) / s)) / fac
    Sigma = (Vt.T / s ** 2) @ Vt
    cov = (Sigma / fac).T / fac
    return dict(dpars=dpars, errs=np.sqrt(np.diag(cov)), cov=cov, names=names)


def gls_step(om, toas, res=None, svd=False):
    """GLSFitter.fit_toas one iteration (fitter.py:2104-2263), rank-reduced (full_cov=False),
    Cholesky with SVD fallback (threshold 0); svd=True is GLSState.step (fitter.py:1425-1500)."""
    res = res or residuals(om, toas)
    M, names = designmatrix(om, toas)
    ntm = M.shape[1]
    U, phi = noise_basis(om, toas)
    phiinv = np.zeros(M.shape[1])
    if U is not None:
        phiinv = np.concatenate((phiinv, 1 / phi))
        M = np.hstack((M, U))
    M, norm = _normalize(M)
    phiinv = phiinv / norm ** 2
    Nvec = (res["sigma_us"] * 1e-6) ** 2
    cinv = 1 / Nvec
    mtcm = M.T @ (cinv[:, None] * M) + np.diag(phiinv)
    mtcy = M.T @ (cinv * res["time"])
    try:
        if svd:
            raise scipy.linalg.LinAlgError
        c = scipy.linalg.cho_factor(mtcm)
        xhat = scipy.linalg.cho_solve(c, mtcy)
        xvar = scipy.linalg.cho_solve(c, np.eye(len(mtcy)))
    except scipy.linalg.LinAlgError:
        Uu, s, Vt = scipy.linalg.svd(mtcm, full_matrices=False)
        s = np.where(s <= 0, np.inf, s)
        xvar = (Vt.T / s) @ Vt
        xhat = Vt.T @ ((Uu.T @ mtcy) / s)
    dpars = xhat / norm
    errs = np.sqrt(np.diag(xvar)) / norm
    cov = (xvar / norm).T / norm
    return dict(dpars=dpars[:ntm], errs=errs[:ntm], cov=cov[:ntm, :ntm], names=names, xhat=xhat, norm=norm)


def apply_step(om: OModel, names, dpars, lam=1.0) -> OModel:
    """pv + dpv in longdouble (fitter.py:2073-2080 / :957 take_step_model)."""
    vals = dict(om.values)
    for n, d in zip(names, dpars):
        if n == "Offset":
            continue
        vals[n] = LD(vals[n]) + LD(lam * d)
    return OModel(vals, om.free, om.comps, om.masks, om.binary, om.ecl)


def fit_once(om, toas, gls=True):
    """One WLS/GLS iteration + post-fit chi2 (fitter.py:2104-2289 with maxiter=1)."""
    res = residuals(om, toas)
    st = gls_step(om, toas, res) if gls else wls_step(om, toas, res)
    om2 = apply_step(om, st["names"], st["dpars"])
    r2 = residuals(om2, toas)
    chi2 = chi2_gls(om2, toas, r2["time"], r2["sigma_us"]) if gls else chi2_wls(r2["time"], r2["sigma_us"])
    return om2, st, chi2


def chi2_of(om, toas, gls):
    """Residuals.chi2 (residuals.py:~620): Woodbury GLS chi2 with correlated noise."""
    r = residuals(om, toas)
    if gls and noise_basis(om, toas)[0] is not None:
        return chi2_gls(om, toas, r["time"], r["sigma_us"])
    return chi2_wls(r["time"], r["sigma_us"])


def downhill_fit(om, toas, gls=False, maxiter=10, required_chi2_decrease=1e-2):
    """DownhillFitter._fit_toas (fitter.py:999-1105) as called by fit_toas without free noise
    parameters (fitter.py:1168-1175: max_chi2_increase = min_lambda = required_chi2_decrease).
    Returns (best model, status, step-record of the best state, chi2)."""
    max_inc = min_lambda = required_chi2_decrease
    stepf = (lambda m: gls_step(m, toas, svd=True)) if gls else (lambda m: wls_step(m, toas))
    cur, cur_c2 = om, chi2_of(om, toas, gls)
    best, best_c2 = cur, cur_c2
    status = "MaxiterReached"
    for _ in range(maxiter):
        st = stepf(cur)
        lam, dec, exc = 1.0, 0.0, False
        while True:
            new = apply_step(cur, st["names"], st["dpars"], lam)
            c2 = chi2_of(new, toas, gls)
            dec = cur_c2 - c2
            if c2 < best_c2:
                best, best_c2 = new, c2
            if dec < -max_inc:
                lam /= 2
                if lam < min_lambda:
                    exc = True
                    break
                continue
            cur, cur_c2 = new, c2
            break
        if -max_inc <= dec < required_chi2_decrease and lam == 1:
            status = "converged"
            break
        if exc:
            status = "StepProblem"
            break
    return best, status, stepf(best), best_c2


def grid_chisq(om_fit, toas, names, values, gls=False):
    """gridutils.py:166 grid_chisq: for every grid point set the grid parameters (frozen), fit
    the remaining free ones with one WLS/GLS iteration (doonefit, gridutils.py:55), record
    the post-fit chi2."""
    free = [p for p in om_fit.free if p not in names]
    grid = np.meshgrid(*[np.asarray(v, dtype=LD) for v in values])  # gridutils.py:331
    out = np.zeros(grid[0].shape)
    for idx in np.ndindex(*out.shape):
        vals = dict(om_fit.values)
        for n, g in zip(names, grid):
            vals[n] = LD(g[idx])
        m = OModel(vals, free, om_fit.comps, om_fit.masks, om_fit.binary, om_fit.ecl)
        out[idx] = fit_once(m, toas, gls=gls)[2]
    return out


def toas_from_product(toas) -> dict:
    d = {k: np.asarray(v) for k, v in toas.arrays.items()}
    d["flags"] = toas.flag_columns
    d["tzr"] = dict(toas.tzr) if toas.tzr is not None else None
    return d


def gls_fit_from_product_inputs(model, toas):
    """cpu_baseline entry (bench.py): one GLS fit on product-side inputs."""
    om = from_product_model(model)
    return fit_once(om, toas_from_product(toas), gls=True)
