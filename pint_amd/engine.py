"""GPU engine: packs (TimingModel, TOAs) into the C-ABI structures and drives the HIP
launch sequence through ctypes.  One ``Session`` = one pint_ctx (one HIP stream on one
device) holding any number of pulsars and a batch of parameter-table instances.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib as L
from .noise import red_noise_freqs_weights, scaled_sigma_us
from .parameter import LD
from .timing_model import BIN_IDS, OBLIQUITY, TimingModel

UNITS = {  # design-matrix column units as the reference prints them (per par unit / F0)
    "RAJ": "1 / (hourangle Hz)", "DECJ": "1 / (deg Hz)", "ELONG": "1 / (deg Hz)", "ELAT": "1 / (deg Hz)",
}


def split_ld(v) -> tuple:
    v = LD(v)
    hi = float(v)
    lo = float(v - LD(hi))
    return hi, lo


@dataclass
class PulsarLayout:
    """Host record of one uploaded pulsar: table layout, columns, sizes."""
    model: TimingModel
    toas: object
    n: int
    offsets: Dict[str, int]
    tstride: int
    columns: List[str]
    spec: L.SpecT
    nred: int
    K: int
    red_freq: Optional[np.ndarray] = None
    red_phi: Optional[np.ndarray] = None
    sigma_us: Optional[np.ndarray] = None
    psr_id: int = -1
    track_mode: str = "nearest"
    keep: list = field(default_factory=list)
    # ECORR epochs (noise_model.py:385-427): CSR TOA lists + prior variances (s^2)
    nep: int = 0
    ep_ptr: Optional[np.ndarray] = None
    ep_idx: Optional[np.ndarray] = None
    ep_phi: Optional[np.ndarray] = None
    ep_param: Optional[list] = None  # the ECORR parameter of each epoch


def _track_mode(model, toas, track_mode):
    """residuals.py:133-149 auto-selection."""
    if track_mode is not None:
        return track_mode
    tr = model["TRACK"].value if "TRACK" in model else None
    if tr == "-2":
        return "use_pulse_numbers"
    if tr == "0":
        return "nearest"
    pn = toas.get_pulse_numbers()
    if pn is not None and not np.any(np.isnan(pn)):
        return "use_pulse_numbers"
    return "nearest"


def build_layout(model: TimingModel, toas, track_mode=None, subtract_mean=True, use_weighted_mean=True,
                 use_gls_basis=True) -> PulsarLayout:
    model.validate()
    spec = L.SpecT()
    offs: Dict[str, int] = {}
    pos = 0

    def place(name):
        nonlocal pos
        offs[name] = pos
        pos += 2
        return offs[name]

    for s in ("o_F", "o_PEPOCH", "o_lon", "o_lat", "o_pmlon", "o_pmlat", "o_px", "o_POSEPOCH", "o_DM",
              "o_DMEPOCH", "o_DMX", "o_FD", "o_JUMP", "o_PHOFF", "o_DMJUMP"):
        setattr(spec, s, -1)
    for i in range(L.B_NPAR):
        spec.o_bin[i] = -1
    F = model.spin_terms()
    spec.nf = len(F)
    spec.o_F = pos
    for n in F:
        place(n)
    spec.o_PEPOCH = place("PEPOCH")
    has_phoff = "PhaseOffset" in model.components
    if has_phoff:
        if model.PHOFF.value is None:
            model.PHOFF.value = 0.0
        spec.o_PHOFF = place("PHOFF")
    free = model.free_params
    phoff_free = has_phoff and "PHOFF" in free
    spec.wb_noones = 1 if phoff_free else 0
    # (a frozen PHOFF with correlated noise: the Woodbury chi2 appends a column of ones the fit
    # layout does not carry; k_onesrow forms its row of Sigma -- PLRedNoise from the weighted
    # trig sums, PLDMNoise from the stored basis columns, ECORR from the epoch sums)
    ak = model.astrometry_kind
    spec.astrometry = ak
    if ak:
        names = ["RAJ", "DECJ", "PMRA", "PMDEC"] if ak == 1 else ["ELONG", "ELAT", "PMELONG", "PMELAT"]
        spec.o_lon, spec.o_lat, spec.o_pmlon, spec.o_pmlat = [place(n) for n in names]
        spec.o_px = place("PX")
        if model.POSEPOCH.value is not None:
            spec.o_POSEPOCH = place("POSEPOCH")
        spec.shapiro = 0
        if "SolarSystemShapiro" in model.components:
            spec.shapiro = 2 if ("PLANET_SHAPIRO" in model and model.PLANET_SHAPIRO.value) else 1
        if ak == 2:
            spec.obliquity = OBLIQUITY[str(model.ECL.value or "IERS2010")]
    dms = model.dm_terms()
    spec.ndm = len(dms)
    if dms:
        spec.o_DM = pos
        for n in dms:
            place(n)
        if model.DMEPOCH.value is not None:
            spec.o_DMEPOCH = place("DMEPOCH")
    dmx = model.dmx_params()
    spec.ndmx = len(dmx)
    if dmx:
        spec.o_DMX = pos
        for n in dmx:
            place(n)
    fds = model.fd_terms()
    spec.nfd = len(fds)
    if fds:
        spec.o_FD = pos
        for n in fds:
            place(n)
    jumps = model.mask_params("JUMP")
    spec.njump = len(jumps)
    if len(jumps) > 64:
        raise NotImplementedError("more than 64 JUMPs")
    if jumps:
        spec.o_JUMP = pos
        for n in jumps:
            place(n)
    spec.binary = {None: L.BIN_NONE, "ELL1": L.BIN_ELL1, "DD": L.BIN_DD, "ELL1H": L.BIN_ELL1H, "BT": L.BIN_BT,
                   "DDK": L.BIN_DDK}[model.binary]
    spec.k96 = 0 if (model.binary == "DDK" and "K96" in model and model.K96.value is False) else 1
    if model.binary:
        for n, pid in BIN_IDS.items():
            if n in model:
                spec.o_bin[pid] = place(n)
        if model.binary == "ELL1H":
            # BinaryELL1H.setup (binary_ell1.py:383-405)
            has4 = model.H4.value is not None
            hasst = model.STIGMA.value is not None
            nh = model.NHARMS.value
            if has4 and hasst:
                raise ValueError("ELL1H can use H4 or STIGMA but not both")
            if hasst and not float(model.STIGMA.value) > 0:
                raise ValueError("STIGMA must be greater than zero.")
            if has4 and float(model.H3.value or 0.0) == 0.0 and float(model.H4.value) != 0.0:
                raise ValueError("To use H4, H3 needs to be significant(H3 != 0).")
            spec.ell1h = 2 if has4 else (3 if hasst else 1)
            spec.nharms = max(int(nh), 7) if (has4 and nh is not None) else (7 if has4 else int(nh or 3))
        need = ["PB", "A1", "TASC" if model.binary in ("ELL1", "ELL1H") else "T0"]
        for n in need:
            if n not in model or model[n].value is None:
                raise ValueError(f"binary parameter {n} missing")
    tstride = pos
    spec.tstride = tstride
    # ---- columns: Offset (unless a PhaseOffset is present, timing_model.py:2145) + free
    # params in params order (timing_model.py:2141-2173)
    cols, kinds, idxs, toffs = ([], [], [], []) if has_phoff else (["Offset"], [L.COL_OFFSET], [0], [-1])
    dmjumps = model.mask_params("DMJUMP")
    spec.ndmjump = len(dmjumps)
    if len(dmjumps) > 64:
        raise NotImplementedError("more than 64 DMJUMPs")
    if dmjumps:
        spec.o_DMJUMP = pos
        for n in dmjumps:
            place(n)
        tstride = pos
        spec.tstride = tstride
    noise_like = {"EFAC", "EQUAD", "ECORR", "TNEQ", "DMEFAC", "DMEQUAD"}
    noise_amp = {"TNREDAMP", "TNREDGAM", "TNREDC", "RNAMP", "RNIDX", "TNDMAMP", "TNDMGAM", "TNDMC"}
    # parameter -> (column kind, index), built once per layout (a PTA pulsar has ~115 free
    # parameters, 100 of them DMX: list.index per parameter was a quadratic scan)
    kind_of = {"PHOFF": (L.COL_OFFSET, 0), "PX": (L.COL_PX, 0)}  # (PHOFF: -d_offset_phase_d_PHOFF / F0 = 1/F0)
    for names, kk in ((("RAJ", "ELONG"), L.COL_LON), (("DECJ", "ELAT"), L.COL_LAT), (("PMRA", "PMELONG"), L.COL_PMLON),
                      (("PMDEC", "PMELAT"), L.COL_PMLAT)):
        for nm in names:
            kind_of[nm] = (kk, 0)
    # (later groups first, so that an earlier group wins a shared name, as the if-chain did)
    for group, kk in ((dmjumps, L.COL_ZERO), (jumps, L.COL_JUMP), (fds, L.COL_FD), (dmx, L.COL_DMX),
                      (dms, L.COL_DM), (F, L.COL_F)):
        for j, nm in enumerate(group):
            kind_of[nm] = (kk, j)
    for n in free:
        p = model[n]
        if p.kind == "mask" and "".join(ch for ch in n if not ch.isdigit()) in noise_like:
            continue
        if n in noise_amp:
            continue
        ki = kind_of.get(n)
        if ki is not None:
            k, i = ki
        elif model.binary and n in BIN_IDS and n in offs:
            k, i = L.COL_BIN, BIN_IDS[n]
        else:
            raise ValueError(f"Cannot compute the design matrix because parameter {n} is unfittable "
                             f"(timing_model.py:2118-2131)")
        if n not in offs:
            raise ValueError(f"parameter {n} has no table slot")
        cols.append(n)
        kinds.append(k)
        idxs.append(i)
        toffs.append(offs[n])
    if len(cols) > L.MAX_COLS:
        raise NotImplementedError("too many design-matrix columns")
    spec.ncol = nc = len(cols)
    spec.col_kind[:nc] = kinds
    spec.col_index[:nc] = idxs
    spec.col_toff[:nc] = toffs
    tm = _track_mode(model, toas, track_mode)
    spec.track_pn = 1 if tm == "use_pulse_numbers" else 0
    spec.subtract_mean = 1 if (subtract_mean and not has_phoff) else 0
    spec.weighted_mean = 1 if use_weighted_mean else 0
    nred = 0
    rf = rp = None
    dmn0 = 0
    if use_gls_basis and ("PLRedNoise" in model.components or "PLDMNoise" in model.components):
        from .noise import fourier_modes
        rf, rp, dmn0 = fourier_modes(model, toas)
        nred = len(rf)
    ep_lists, ep_phi, ep_param = [], [], []
    if model.mask_params("ECORR") and use_gls_basis:
        from .noise import ecorr_epochs
        t = np.asarray(toas.tdbld * LD(86400))
        for name in model.mask_params("ECORR"):
            p = model[name]
            idx = toas.select_mask(p.key, p.key_value)
            for b in ecorr_epochs(t[idx]):
                ep_lists.append(np.sort(idx[b]))
                ep_phi.append((float(p.value) * 1e-6) ** 2)
                ep_param.append(name)
    spec.nred = nred
    spec.dmn0 = dmn0 if (use_gls_basis and "PLDMNoise" in model.components) else nred
    lay = PulsarLayout(model=model, toas=toas, n=toas.ntoas, offsets=offs, tstride=tstride, columns=cols,
                       spec=spec, nred=nred, K=len(cols) + 2 * nred, red_freq=rf, red_phi=rp, track_mode=tm)
    if ep_lists:
        lay.nep = len(ep_lists)
        lay.ep_ptr = np.concatenate([[0], np.cumsum([len(e) for e in ep_lists])]).astype(np.int32)
        lay.ep_idx = np.concatenate(ep_lists).astype(np.int32)
        lay.ep_phi = np.asarray(ep_phi, dtype=np.float64)
        lay.ep_param = ep_param
    return lay


def pack_table(lay: PulsarLayout, model: Optional[TimingModel] = None) -> np.ndarray:
    """The device parameter table of `model` in `lay`'s layout: every parameter as its
    (hi, lo) double-double split (split_ld's operations, on all parameters at once)."""
    model = model or lay.model
    tab = np.zeros(lay.tstride)
    offs = lay.__dict__.get("_offs_np")
    if offs is None or offs[0] is not lay.offsets or len(offs[1]) != len(lay.offsets):
        offs = (lay.offsets, list(lay.offsets), np.fromiter(lay.offsets.values(), dtype=np.int64, count=len(lay.offsets)))
        lay.__dict__["_offs_np"] = offs
    names, o = offs[1], offs[2]
    p = model._params
    v = np.array([0.0 if p[n].value is None else p[n].value for n in names], dtype=np.longdouble)
    hi = v.astype(np.float64)
    tab[o] = hi
    tab[o + 1] = (v - hi.astype(np.longdouble)).astype(np.float64)
    return tab


def unpack_table(lay: PulsarLayout, tab: np.ndarray, model: TimingModel):
    """Write device table values back into a model (longdouble where the reference keeps it)."""
    for n, o in lay.offsets.items():
        p = model[n]
        if p.value is None and tab[o] == 0.0 and tab[o + 1] == 0.0:
            continue
        v = LD(tab[o]) + LD(tab[o + 1])
        p.value = v if (p.long_double or p.kind == "mjd") else float(v)


def pack_toas(lay: PulsarLayout):
    """Per-TOA boundary arrays (n+1 rows; the last is the TZR TOA) + masks."""
    model, toas = lay.model, lay.toas
    n = toas.ntoas
    A = toas.arrays
    tz = (toas.tzr_for(model) if hasattr(toas, "tzr_for") else toas.tzr) if "AbsPhase" in model.components else None
    if tz is None:
        tz = make_tzr_row(model, toas)

    def cat(name, default=0.0, width=None):
        a = np.asarray(A[name], dtype=np.float64)
        b = np.asarray(tz.get(name, np.full((1,) + a.shape[1:], default)), dtype=np.float64).reshape((1,) + a.shape[1:])
        return np.ascontiguousarray(np.concatenate([a, b]))

    tdb_hi, tdb_lo = cat("tdb_hi"), cat("tdb_lo")
    freq = cat("freq_mhz", np.inf)
    pos, vel, sun = cat("ssb_obs_pos_km"), cat("ssb_obs_vel_kms"), cat("obs_sun_pos_km")
    dpn = cat("delta_pulse_number")
    is_bary = np.concatenate([np.asarray(A["is_bary"]), np.asarray(tz.get("is_bary", [0])).reshape(1)]).astype(bool)
    allpos = (pos[:, 0] != 0) & (pos[:, 1] != 0) & (pos[:, 2] != 0)
    flags = (is_bary.astype(np.uint32) | (allpos.astype(np.uint32) << 1)).astype(np.uint32)
    sigma = scaled_sigma_us(model, toas)
    lay.sigma_us = sigma
    sigma_s = np.ascontiguousarray(sigma * 1e-6)
    pn = toas.get_pulse_numbers()
    pn = np.ascontiguousarray(pn if pn is not None else np.zeros(n), dtype=np.float64)
    jm = np.zeros(n + 1, dtype=np.uint64)
    for k, name in enumerate(model.mask_params("JUMP")):
        p = model[name]
        idx = toas.select_mask(p.key, p.key_value)
        jm[idx] |= np.uint64(1) << np.uint64(k)
        if len(toas.select_mask(p.key, p.key_value, tzr=True)) if toas.tzr else False:
            jm[n] |= np.uint64(1) << np.uint64(k)
    da = np.full(n + 1, -1, dtype=np.int32)
    db = np.full(n + 1, -1, dtype=np.int32)
    extra = {}
    mjdf = np.concatenate([np.asarray(A["mjd_float"], dtype=np.float64),
                           np.asarray(tz.get("mjd_float", [0.0]), dtype=np.float64).reshape(1)])
    dmxn = model.dmx_params()
    if dmxn:
        tags = [name.split("_")[1] for name in dmxn]
        r1 = np.array([float(model["DMXR1_" + t].value) for t in tags])
        r2 = np.array([float(model["DMXR2_" + t].value) for t in tags])
        order = np.argsort(r1, kind="stable")
        s1, s2 = r1[order], r2[order]
        vec = bool(np.all(s1 <= s2) and np.all(np.diff(s2) >= 0))
        if vec:
            # ranges sorted by start with non-decreasing ends (consecutive bins, possibly
            # sharing an endpoint): the bins holding MJD t (toa_select.py:101, inclusive) are
            # the sorted positions lo..hi, lo = #(ends < t), hi = #(starts <= t) - 1 -- two
            # sorted searches instead of a pass over the TOAs per bin
            if n > 1 and np.all(mjdf[1:n] >= mjdf[:n - 1]):  # time-ordered TOAs (the TZR row apart):
                # the bins' edges located among the TOAs (2 x bins searches, not 2 x TOAs)
                lo, hi = np.empty(n + 1, dtype=np.int64), np.empty(n + 1, dtype=np.int64)
                lo[:n] = np.repeat(np.arange(len(s2) + 1), np.diff(np.concatenate(
                    [[0], np.searchsorted(mjdf[:n], s2, side="right"), [n]])))
                hi[:n] = np.repeat(np.arange(len(s1) + 1), np.diff(np.concatenate(
                    [[0], np.searchsorted(mjdf[:n], s1, side="left"), [n]]))) - 1
                lo[n] = np.searchsorted(s2, mjdf[n], side="left")
                hi[n] = np.searchsorted(s1, mjdf[n], side="right") - 1
            else:
                lo = np.searchsorted(s2, mjdf, side="left")
                hi = np.searchsorted(s1, mjdf, side="right") - 1
            cnt = hi - lo + 1
            vec = bool(cnt.max(initial=0) <= 2)
        if vec:
            one, two = cnt >= 1, cnt == 2
            a, b = order[np.clip(lo, 0, len(order) - 1)], order[np.clip(hi, 0, len(order) - 1)]
            da[one] = np.minimum(a, b)[one].astype(np.int32)     # a TOA's first slot: the bin
            db[two] = np.maximum(a, b)[two].astype(np.int32)     # first in parameter order
        else:
            for j in range(len(dmxn)):
                sel = np.where((mjdf >= r1[j]) & (mjdf <= r2[j]))[0]  # toa_select.py:101 inclusive
                fa = da[sel] < 0            # (bins in parameter order: a TOA's first free slot)
                da[sel[fa]] = j
                rest = sel[~fa]
                fb = db[rest] < 0
                db[rest[fb]] = j
                for i in rest[~fb]:         # a third (fourth, ...) overlapping bin: the CSR overflow below
                    extra.setdefault(int(i), []).append(j)
    dmx_x = None
    if extra:
        # n+2 offsets into the same array, then the bin indices in parameter order (the
        # reference sums every selecting bin, dispersion_model.py:672-677)
        cnt = np.zeros(n + 1, dtype=np.int64)
        for i, js in extra.items():
            cnt[i] = len(js)
        off = (n + 2) + np.concatenate([[0], np.cumsum(cnt)])
        dmx_x = np.empty(int(off[-1]), dtype=np.int32)
        dmx_x[:n + 2] = off
        for i, js in extra.items():
            dmx_x[off[i]:off[i + 1]] = js
    planet = None
    if lay.spec.shapiro == 2:
        planet = planet_rows(toas, tz, is_bary)
    keep = [tdb_hi, tdb_lo, freq, sigma_s, pos, vel, sun, pn, dpn, flags, jm, da, db, planet, dmx_x]
    t = L.ToasT(n, L.ptr(tdb_hi), L.ptr(tdb_lo), L.ptr(freq), L.ptr(sigma_s), L.ptr(pos), L.ptr(vel), L.ptr(sun),
                L.ptr(pn), L.ptr(dpn), L.ptr(flags, C.c_uint32), L.ptr(jm, C.c_uint64), L.ptr(da, C.c_int32),
                L.ptr(db, C.c_int32), L.ptr(planet) if planet is not None else None,
                L.ptr(dmx_x, C.c_int32) if dmx_x is not None else None)
    return t, keep


def pack_cols(lay: PulsarLayout):
    """The TOA table's own columns for pint_add_pulsar_cols / pint_pack_toas: the library
    forms the n+1-row boundary arrays (pack_toas) itself.  Returns (ToaColsT, keep)."""
    model, toas = lay.model, lay.toas
    n = toas.ntoas
    A = toas.arrays
    tz = (toas.tzr_for(model) if hasattr(toas, "tzr_for") else toas.tzr) if "AbsPhase" in model.components else None
    if tz is None:
        tz = make_tzr_row(model, toas)

    def col(name, w=1):
        a = np.ascontiguousarray(A[name], dtype=np.float64)
        if a.size != w * n:
            raise ValueError(f"TOA column {name}: {a.shape}, expected {n} x {w}")
        return a

    def tzv(name, default, w=1):
        return np.asarray(tz[name], dtype=np.float64).reshape(w) if name in tz else np.full(w, default)

    cols = [col("tdb_hi"), col("tdb_lo"), col("freq_mhz"), col("ssb_obs_pos_km", 3), col("ssb_obs_vel_kms", 3),
            col("obs_sun_pos_km", 3), col("delta_pulse_number"), col("mjd_float")]
    is_bary = np.ascontiguousarray(np.asarray(A["is_bary"]).astype(bool).astype(np.uint8))
    tzr = np.concatenate([tzv("tdb_hi", 0.0), tzv("tdb_lo", 0.0), tzv("freq_mhz", np.inf),
                          tzv("ssb_obs_pos_km", 0.0, 3), tzv("ssb_obs_vel_kms", 0.0, 3), tzv("obs_sun_pos_km", 0.0, 3),
                          tzv("delta_pulse_number", 0.0), tzv("mjd_float", 0.0),
                          [float(bool(np.asarray(tz.get("is_bary", [0])).reshape(1)[0]))]])
    sigma = scaled_sigma_us(model, toas)
    lay.sigma_us = sigma
    sigma = np.ascontiguousarray(sigma, dtype=np.float64)
    pn = toas.get_pulse_numbers()
    pn = np.ascontiguousarray(pn, dtype=np.float64) if pn is not None else None
    jm = None
    jumps = model.mask_params("JUMP")
    if jumps:
        jm = np.zeros(n + 1, dtype=np.uint64)
        for k, name in enumerate(jumps):
            p = model[name]
            jm[toas.select_mask(p.key, p.key_value)] |= np.uint64(1) << np.uint64(k)
            if len(toas.select_mask(p.key, p.key_value, tzr=True)) if toas.tzr else False:
                jm[n] |= np.uint64(1) << np.uint64(k)
    P = model._params
    tags = [name[4:] for name in model.dmx_params()]  # DMX_<tag>
    r = tuple(np.array([P[k + t].value for t in tags], dtype=np.longdouble).astype(np.float64)
              for k in ("DMXR1_", "DMXR2_"))
    planet = planet_rows(toas, tz, np.concatenate([is_bary, [int(tzr[14])]]).astype(bool)) \
        if lay.spec.shapiro == 2 else None
    c = L.ToaColsT(n, *[L.ptr(a) for a in cols[:7]], L.ptr(cols[7]), L.ptr(is_bary, C.c_uint8), L.ptr(sigma),
                   L.ptr(pn), L.ptr(jm, C.c_uint64), L.ptr(planet), (C.c_double * 15)(*tzr), len(r[0]),
                   L.ptr(r[0]), L.ptr(r[1]))
    return c, [cols, is_bary, sigma, pn, jm, r, planet]


SHAPIRO_PLANETS = ("jupiter", "saturn", "venus", "uranus", "neptune")   # solar_system_shapiro.py:112


def planet_rows(toas, tz, is_bary) -> np.ndarray:
    """(n+1, 15) observatory -> planet vectors (km) of the TOAs and the TZR TOA for
    PLANET_SHAPIRO; like the reference (solar_system_shapiro.py:118-122) missing columns are
    a KeyError naming planets=True.  A barycentric TZR TOA needs none (its Shapiro delay is
    not evaluated, :100)."""
    cols = []
    for pl in SHAPIRO_PLANETS:
        k = f"obs_{pl}_pos_km"
        if k not in toas.arrays:
            raise KeyError("Planet positions not found when trying to compute Solar System Shapiro delay. "
                           "Make sure that you include `planets=True` in your `get_TOAs()` call, or use "
                           "`get_model_and_toas()`.")
        if k in tz:
            b = np.asarray(tz[k], dtype=np.float64).reshape(1, 3)
        elif is_bary[-1]:
            b = np.zeros((1, 3))
        else:
            raise KeyError(f"the TZR TOA has no {k} (prepare it with planets=True)")
        cols.append(np.concatenate([np.asarray(toas.arrays[k], dtype=np.float64), b]))
    return np.ascontiguousarray(np.concatenate(cols, axis=1))


def make_tzr_row(model, toas) -> dict:
    """No TZRMJD in the model: the reference adds AbsPhase with TZRMJD = first TOA after
    PEPOCH at the barycenter, infinite frequency (timing_model.py:1584, absolute_phase.py:129)."""
    mjds = toas.get_mjds()
    pe = float(model.PEPOCH.value)
    later = mjds[mjds > pe]
    tz = later.min() if len(later) else mjds[mjds <= pe].max()
    hi, lo = split_ld(LD(tz))
    return {"tdb_hi": np.array([hi]), "tdb_lo": np.array([lo]), "freq_mhz": np.array([np.inf]),
            "ssb_obs_pos_km": np.zeros((1, 3)), "ssb_obs_vel_kms": np.zeros((1, 3)),
            "obs_sun_pos_km": np.zeros((1, 3)), "mjd_float": np.array([tz]), "is_bary": np.array([1]),
            "delta_pulse_number": np.zeros(1), "flags": {}}


class SplitView:
    """Per-instance views of one flat output buffer (list-like: len, indexing, iteration),
    formed on access: a batched step hands out its outputs without building one array
    object per instance (host time per step), and the pinned buffer behind it is filled by
    the device copies."""

    def __init__(self, flat, offsets, shapes=None):
        self.flat, self.off, self.shapes = flat, offsets, shapes

    def __len__(self):
        return len(self.off) - 1

    def __getitem__(self, k):
        if isinstance(k, slice):
            return [self[i] for i in range(*k.indices(len(self)))]
        if k < 0:
            k += len(self)
        v = self.flat[self.off[k]:self.off[k + 1]]
        return v.reshape(self.shapes[k]) if self.shapes is not None else v

    def __iter__(self):
        return (self[k] for k in range(len(self)))


class Session:
    """A pint_ctx with uploaded pulsars and a batch of instances."""

    def __init__(self, device: Optional[int] = None):
        self.L = L.lib()
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        if self.L.pint_device_count() <= 0:
            raise RuntimeError("no HIP device visible: the pint_amd compute path needs an MI355X GPU")
        self.ctx = self.L.pint_ctx_create(device)
        if not self.ctx:
            raise RuntimeError("pint_ctx_create failed")
        err = self.L.pint_last_error(self.ctx)
        if err:
            raise RuntimeError(err.decode())
        self.layouts: List[PulsarLayout] = []
        self.inst_psr: List[int] = []
        self.inst_layout: List[PulsarLayout] = []
        self._uniform, self._offs = False, None
        self.lazy = False
        self._pinned: Dict[str, tuple] = {}
        self._inflight = set()  # pinned staging buffers with a copy still enqueued (lazy)
        self._keep = []         # host arrays of enqueued copies (lazy)
        self._slot = 0          # pipelined steps: the slot the next launches belong to
        self._slot_state = {0: (self._inflight, self._keep)}
        self._slot_state.update({k: (set(), []) for k in range(1, L.NSLOT)})
        self._pending = set()   # slots of ended, not yet checked steps

    def close(self):
        if self.ctx:
            self.L.pint_ctx_destroy(self.ctx)
            self.ctx = None
        for ptr_, _ in self._pinned.values():
            self.L.pint_host_free(ptr_)
        self._pinned = {}

    def _pin(self, name, n):
        """Page-locked host buffer of n doubles (reused across calls, grown on demand), so
        device->host copies of the fit outputs can run asynchronously.  One per pipeline
        slot (step_end/check_step), so step k+1's copies never touch step k's buffers."""
        n = max(1, int(n))
        if self._slot in self._pending:
            raise RuntimeError("pipelined steps: enqueueing into a slot whose step was never checked")
        name = f"{name}@{self._slot}"
        cur = self._pinned.get(name)
        if cur is not None and cur[1].size >= n:
            return cur[1][:n]
        if cur is not None:
            self.L.pint_host_free(cur[0])
        p = self.L.pint_host_alloc(8 * n)
        if not p:
            raise MemoryError("pint_host_alloc failed")
        arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_double)), shape=(n,))
        self._pinned[name] = (p, arr)
        return arr

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise L.PintError(rc, self.L.pint_last_error(self.ctx).decode())

    def add(self, lay: PulsarLayout, packed=None) -> PulsarLayout:
        """Upload a pulsar: pint_add_pulsar_cols (the library packs the TOA table's columns;
        packed: pack_cols(lay) when already formed), or pint_add_pulsar when packed is
        pack_toas(lay) (the numpy packing)."""
        if packed is None:  # the table's columns, packed by the library (pint_add_pulsar_cols)
            packed = pack_cols(lay)
        native = isinstance(packed[0], L.ToaColsT)
        t, keep = packed
        if lay.red_freq is not None:  # double-double frequencies: hi[nred] then lo[nred]
            f = np.asarray(lay.red_freq, dtype=np.longdouble)
            fh = f.astype(np.float64)
            rf = np.ascontiguousarray(np.concatenate([fh, (f - fh.astype(np.longdouble)).astype(np.float64)]))
        else:
            rf = np.zeros(2)
        rp = np.ascontiguousarray(lay.red_phi if lay.red_phi is not None else np.zeros(1))
        if native:
            pid = self.L.pint_add_pulsar_cols(self.ctx, C.byref(t), C.byref(lay.spec), L.ptr(rf), L.ptr(rp))
        else:
            pid = self.L.pint_add_pulsar(self.ctx, C.byref(t), C.byref(lay.spec), L.ptr(rf), L.ptr(rp))
        if pid < 0:
            self._check(-pid)
        lay.psr_id = pid
        if lay.nep > 0:
            self._check(self.L.pint_set_ecorr(self.ctx, pid, lay.nep, L.ptr(lay.ep_ptr, C.c_int32),
                                              L.ptr(lay.ep_idx, C.c_int32), L.ptr(lay.ep_phi)))
        self.layouts.append(lay)
        return lay

    def add_all(self, items, **layout_kw) -> List[PulsarLayout]:
        """Add many pulsars ((model, toas) pairs), in order: each pulsar's host layout and
        TOA columns (build_layout, pack_cols) are formed on this thread while one worker thread
        uploads the previous ones (pint_add_pulsar_cols runs without the GIL), so the Python
        host work and the library's packing and staging overlap.  self.add_timing: the
        caller thread's host ms and the ms it then waited for the uploads."""
        from concurrent.futures import ThreadPoolExecutor
        import time
        t0 = time.perf_counter()
        futs, lays, failed = [], [], []

        def upload(lay, packed):
            if failed:  # (nothing after a rejected pulsar, as a loop of add() would stop there)
                return None
            try:
                return self.add(lay, packed)
            except BaseException as e:
                failed.append(e)
                raise

        with ThreadPoolExecutor(1, thread_name_prefix="pint-upload") as ex:
            try:
                for m, t in items:
                    if failed:
                        break
                    lay = build_layout(m, t, **layout_kw)
                    futs.append(ex.submit(upload, lay, pack_cols(lay)))
                    lays.append(lay)
            finally:
                t1 = time.perf_counter()
                for f in futs:  # in order; the first failure raises (after every upload ended)
                    f.exception()
        t2 = time.perf_counter()
        for f in futs:
            f.result()
        self.add_timing = {"host_ms": (t1 - t0) * 1e3, "upload_wait_ms": (t2 - t1) * 1e3}
        return lays

    def set_instances(self, insts: Sequence[tuple]):
        """insts: sequence of (layout, table ndarray)."""
        ids = np.array([lay.psr_id for lay, _ in insts], dtype=np.int32)
        tabs = np.ascontiguousarray(np.concatenate([np.asarray(t, dtype=np.float64) for _, t in insts]))
        self._set(ids, tabs, [lay for lay, _ in insts])

    def set_instances_of(self, lay: PulsarLayout, tables: np.ndarray):
        """Many instances of one pulsar (grid points): tables is (ninst, tstride)."""
        tables = np.ascontiguousarray(tables, dtype=np.float64)
        if tables.ndim != 2 or tables.shape[1] != lay.tstride:
            raise ValueError(f"tables must be (ninst, {lay.tstride}), got {tables.shape}")
        ids = np.full(tables.shape[0], lay.psr_id, dtype=np.int32)
        self._set(ids, tables.ravel(), [lay] * tables.shape[0], uniform=True)

    def set_grid(self, lay: PulsarLayout, base_table: np.ndarray, variables, npts: int, k0: int = 0):
        """npts grid points of one pulsar as instances (pint_set_grid): every point's table is
        base_table with each variable's entry replaced, formed on the device.  variables:
        [(parameter name, longdouble values, stride, size)] -- point k takes
        values[((k0 + k) // stride) % size] (a meshgrid axis; stride 1, size npts for every
        point's own value)."""
        base = np.ascontiguousarray(base_table, dtype=np.float64)
        if base.shape != (lay.tstride,):
            raise ValueError(f"base table must have {lay.tstride} entries, got {base.shape}")
        toff = np.array([lay.offsets[p] for p, _, _, _ in variables], dtype=np.int32)
        stride = np.array([int(st) for _, _, st, _ in variables], dtype=np.int64)
        size = np.array([int(sz) for _, _, _, sz in variables], dtype=np.int64)
        pairs = []
        for (_, v, _, sz) in variables:
            v = np.asarray(v, dtype=np.longdouble).reshape(-1)
            if v.size != sz:
                raise ValueError("grid variable: values and size differ")
            h = v.astype(np.float64)
            lo = (v - h.astype(np.longdouble)).astype(np.float64)
            pairs.append(np.stack([h, lo], axis=1).reshape(-1))
        vals = np.ascontiguousarray(np.concatenate(pairs) if pairs else np.zeros(2))
        self._check(self.L.pint_set_grid(self.ctx, lay.psr_id, int(npts), L.ptr(base), len(variables),
                                         L.ptr(toff, C.c_int32), L.ptr(stride, C.c_int64), L.ptr(size, C.c_int64),
                                         L.ptr(vals), int(k0)))
        self._after_set([lay] * int(npts), int(npts) * lay.tstride, uniform=True)

    def _set(self, ids, tabs, lays, uniform=False):
        self._check(self.L.pint_set_instances(self.ctx, len(ids), L.ptr(ids, C.c_int32), L.ptr(tabs)))
        self._after_set(lays, len(tabs), uniform)

    def _after_set(self, lays, ntab, uniform=False):
        self.inst_layout = lays
        self.ntab = ntab
        self._uniform = uniform
        self._offs = None  # (formed at the first read that needs them: a grid's points never do)

    def _offsets(self):
        """Per-instance output offsets (read_step, noise_resids), formed once per batch (one
        layout for every instance -- grid points -- without a Python loop over them: a
        256 x 256 grid's loops took ~15 ms of its ~25 ms)."""
        if self._offs is None:
            lays = self.inst_layout
            if self._uniform and lays:
                n = len(lays)
                kk = np.full(n, lays[0].K + 1, dtype=np.int64)
                nc = np.full(n, len(lays[0].columns), dtype=np.int64)
                nn = np.full(n, lays[0].n, dtype=np.int64)
                shapes = [(int(nc[0]), int(nc[0]))] * n
            else:
                kk = np.array([l.K + 1 for l in lays], dtype=np.int64)
                nc = np.array([len(l.columns) for l in lays], dtype=np.int64)
                nn = np.array([l.n for l in lays], dtype=np.int64)
                shapes = [(int(c), int(c)) for c in nc]
            self._offs = (np.concatenate([[0], np.cumsum(kk)]), np.concatenate([[0], np.cumsum(nc * nc)]),
                          np.concatenate([[0], np.cumsum(nn)]), shapes)
        return self._offs

    @property
    def _off_k(self):
        return self._offsets()[0]

    @property
    def _off_cov(self):
        return self._offsets()[1]

    @property
    def _off_n(self):
        return self._offsets()[2]

    @property
    def _cov_shapes(self):
        return self._offsets()[3]

    # -- launches -------------------------------------------------------------------
    FIT = 2  # want_M for a fit step: compact layout (DMX columns as bin sums)

    def eval(self, want_M=False):
        """want_M: False (phases/residuals only), True (full design matrix, as
        TimingModel.designmatrix returns it) or Session.FIT (fit layout for fit_step)."""
        self._check(self.L.pint_eval(self.ctx, 2 if want_M == self.FIT else (1 if want_M else 0)))

    def fit_step(self, mode):
        self._check(self.L.pint_fit_step(self.ctx, int(mode)))

    def fit_step_apply(self, mode, lam=1.0):
        """fit_step(mode) then apply_step_uniform(lam) (pint_fit_step_apply: fused into the
        solve kernel when every instance allows it).  read_step / noise_resids may follow:
        they read the step, not the tables."""
        self._check(self.L.pint_fit_step_apply(self.ctx, int(mode), float(lam)))

    def apply_step(self, lam):
        lam = np.broadcast_to(np.asarray(lam, dtype=np.float64), (len(self.inst_layout),))
        if self.lazy and "lambda" not in self._inflight:
            buf = self._pin("lambda", lam.size)  # pinned (fixed for graph replays); reused after check()
            buf[:] = lam
            lam = buf
            self._inflight.add("lambda")
        else:
            lam = np.array(lam, dtype=np.float64)
            self._keep.append(lam)
        self._check(self.L.pint_apply_step(self.ctx, L.ptr(lam)))

    def apply_step_uniform(self, lam=1.0):
        """tables += lam * step for every instance (one lambda: a kernel argument)."""
        self._check(self.L.pint_apply_step_uniform(self.ctx, float(lam)))

    def save_tables(self):
        """Snapshot the batch's parameter tables on the device (pint_save_tables)."""
        self._check(self.L.pint_save_tables(self.ctx))

    def restore_tables(self):
        """Put the device snapshot back (a device->device copy, pint_restore_tables)."""
        self._check(self.L.pint_restore_tables(self.ctx))

    # -- HIP graphs ---------------------------------------------------------------------
    def capture(self, fn):
        """Capture the launches fn() enqueues (lazy mode) into a HIP graph; returns fn()'s
        result (pinned output buffers that every replay refills)."""
        self._check(self.L.pint_capture_begin(self.ctx))
        try:
            out = fn()
        except Exception:
            self.L.pint_capture_end(self.ctx)
            raise
        self._check(self.L.pint_capture_end(self.ctx))
        return out

    def replay(self):
        """Launch the captured graph (complete after check())."""
        self._check(self.L.pint_graph_launch(self.ctx))

    def set_tables(self, tabs):
        tabs = np.asarray(tabs, dtype=np.float64).ravel()
        if self.lazy and "tables" not in self._inflight:
            # pinned staging buffer (fixed for graph replays); reused only after check()
            buf = self._pin("tables", tabs.size)
            buf[:] = tabs
            tabs = buf
            self._inflight.add("tables")
        else:
            tabs = np.array(tabs, dtype=np.float64)
            self._keep.append(tabs)  # lazy: must outlive the enqueued copy
        self._check(self.L.pint_set_tables(self.ctx, L.ptr(tabs)))

    # -- reads ----------------------------------------------------------------------
    def _split(self, flat, sizes):
        out, o = [], 0
        for s in sizes:
            out.append(flat[o:o + s])
            o += s
        return out

    def read_resids(self):
        n = [l.n for l in self.inst_layout]
        tr = np.empty(sum(n))
        pr = np.empty(sum(n))
        c2 = np.empty(len(n))
        self._check(self.L.pint_read_resids(self.ctx, L.ptr(tr), L.ptr(pr), L.ptr(c2)))
        return self._split(tr, n), self._split(pr, n), c2

    def set_wideband(self, lay):
        """Upload a pulsar's wideband DM data (pint_set_wideband): -pp_dm / -pp_dme, the errors
        scaled by DMEFAC/DMEQUAD (host preparation, noise_model.py:291) and the DMJUMP masks
        (bit k: the k-th DMJUMP, the layout's table order)."""
        from .noise import scaled_dm_sigma
        model, toas = lay.model, lay.toas
        try:
            dm, dme = toas.get_dms(), toas.get_dm_errors()
        except AttributeError:
            raise ValueError("Input TOA object does not have wideband DM values")
        if len(dm) != lay.n or len(dme) != lay.n:
            raise ValueError("Input TOA object' DM data and DM errors do not match.")
        sig = scaled_dm_sigma(model, toas)
        jm = np.zeros(lay.n, dtype=np.uint64)
        for k, name in enumerate(model.mask_params("DMJUMP")):
            p = model[name]
            jm[toas.select_mask(p.key, p.key_value)] |= np.uint64(1) << np.uint64(k)
        dm, dme = np.ascontiguousarray(dm, dtype=np.float64), np.ascontiguousarray(dme, dtype=np.float64)
        self._check(self.L.pint_set_wideband(self.ctx, lay.psr_id, L.ptr(dm), L.ptr(dme), L.ptr(sig),
                                             L.ptr(jm, C.c_uint64)))
        lay.keep += [dm, dme, sig, jm]
        lay.dm_data, lay.dm_error, lay.dm_sigma = dm, dme, sig

    def dm_resids(self, subtract_mean=False, use_weighted_mean=True):
        """WidebandDMResiduals of every instance (pint_dm_resids): (residual rows per
        instance, chi2 per instance), pc/cm^3."""
        n = [l.n for l in self.inst_layout]
        r = np.empty(sum(n))
        c2 = np.empty(len(n))
        self._check(self.L.pint_dm_resids(self.ctx, 1 if subtract_mean else 0, 1 if use_weighted_mean else 0,
                                          L.ptr(r), L.ptr(c2)))
        return self._split(r, n), c2

    def read_chi2(self):
        """WLS chi2 per instance only (no residual rows copied back); lazy: a pinned buffer
        that is complete after check()."""
        # (pinned either way: a copy into pageable memory left the host ~1 ms behind the
        # device at 65,536 grid points)
        c2 = self._pin("chi2r", len(self.inst_layout))
        self._check(self.L.pint_read_resids(self.ctx, None, None, L.ptr(c2)))
        return c2 if self.lazy else c2.copy()

    def read_eval(self):
        rows = [l.n + 1 for l in self.inst_layout]
        a = [np.empty(sum(rows)) for _ in range(4)]
        self._check(self.L.pint_read_eval(self.ctx, *[L.ptr(x) for x in a]))
        return [self._split(x, rows) for x in a]

    def read_designmatrix(self):
        sizes = [l.n * l.K for l in self.inst_layout]
        M = np.empty(sum(sizes))
        self._check(self.L.pint_read_designmatrix(self.ctx, L.ptr(M)))
        return [m.reshape(l.K, l.n).T for m, l in zip(self._split(M, sizes), self.inst_layout)]

    def set_lazy(self, lazy=True):
        """Lazy mode: launches and output copies are only enqueued; read_step/chi2_gls return
        pinned buffers that are complete after check()."""
        self._check(self.L.pint_set_lazy(self.ctx, 1 if lazy else 0))
        self.lazy = bool(lazy)

    def fit_layout(self, lay):
        """(compact, Gram columns, sparse DMX columns, padded Gram width) of a pulsar."""
        out = np.zeros(4, dtype=np.int32)
        self._check(self.L.pint_fit_layout(self.ctx, lay.psr_id, L.ptr(out, C.c_int32)))
        return tuple(int(x) for x in out)

    def vgram_layout(self, lay):
        """(on the vg path (bit 1: with the binned DMX x F tile), DMX slots, k_gram_v LDS
        width, compact timing columns)."""
        out = np.zeros(4, dtype=np.int32)
        self._check(self.L.pint_vgram_layout(self.ctx, lay.psr_id, L.ptr(out, C.c_int32)))
        return tuple(int(x) for x in out)

    def set_blocked_solve(self, on=True):
        self._check(self.L.pint_set_option(self.ctx, 1, 1 if on else 0))

    def set_timing_mask(self, mask=0xFF):
        """Timing slots of timing() whose HIP events are recorded (each costs device time)."""
        self._check(self.L.pint_set_option(self.ctx, 3, int(mask)))

    def set_timing_every(self, k=1):
        """Gram timing events on every k-th fit step only (PINT_OPT_TIMING_EVERY); timing()
        then reads 0 in slot 6 after an unsampled step."""
        self._check(self.L.pint_set_option(self.ctx, 8, int(k)))

    def set_refine(self, on=True):
        """Iterative refinement of ill-conditioned solves (PINT_OPT_REFINE, default on)."""
        self._check(self.L.pint_set_option(self.ctx, 4, 1 if on else 0))

    def set_vgram(self, on=True):
        """Generated-Fourier compact fit path (k_gram_v); applies from the next set_instances."""
        self._check(self.L.pint_set_option(self.ctx, 2, 1 if on else 0))

    def set_wbfit(self, on=True):
        """Wideband DM rows in the fit steps (PINT_OPT_WBFIT, WidebandTOAFitter)."""
        self._check(self.L.pint_set_option(self.ctx, 6, 1 if on else 0))

    def set_cov_defer(self, mode=1):
        """Covariance of the DMX-eliminated solve formed at the read (PINT_OPT_COV_DEFER: 0
        never, 1 batches of >= 16 instances, 2 always)."""
        self._check(self.L.pint_set_option(self.ctx, 7, int(mode)))

    def set_schur(self, on=True):
        """The DMX-eliminated solve's build phase in k_schur (PINT_OPT_SCHUR, default on)."""
        self._check(self.L.pint_set_option(self.ctx, 9, 1 if on else 0))

    def set_small(self, on=True):
        """Small-instance kernels (PINT_OPT_SMALL, default on): k_gram_s from the next
        set_instances, the one-wave solve from the next fit step."""
        self._check(self.L.pint_set_option(self.ctx, 10, 1 if on else 0))

    def set_la_chol(self, on=True):
        """Look-ahead blocked Cholesky in the DMX-eliminated solve (PINT_OPT_LA_CHOL, default on)."""
        self._check(self.L.pint_set_option(self.ctx, 11, 1 if on else 0))

    def set_efuse(self, on=True):
        """The residual pass's first half fused into the evaluation (PINT_OPT_EFUSE, default
        on); applies from the next set_instances."""
        self._check(self.L.pint_set_option(self.ctx, 12, 1 if on else 0))

    def set_lane_solve(self, on=True):
        """A lane per instance for small-instance solves of <= 8 columns (PINT_OPT_LANE_SOLVE, default on)."""
        self._check(self.L.pint_set_option(self.ctx, 13, 1 if on else 0))

    def set_spin_eval(self, on=True):
        """Shared evaluation head for spin-only grids (PINT_OPT_SPIN_EVAL, default on)."""
        self._check(self.L.pint_set_option(self.ctx, 14, 1 if on else 0))

    def set_solve_w8(self, on=True):
        """8 waves per instance in the DMX-eliminated solve when its dense block fits (PINT_OPT_SOLVE_W8)."""
        self._check(self.L.pint_set_option(self.ctx, 15, 1 if on else 0))

    def set_vbin(self, on=True):
        """k_gram_v's binned DMX x Fourier tile (PINT_OPT_VBIN); applies from the next set_instances."""
        self._check(self.L.pint_set_option(self.ctx, 5, 1 if on else 0))

    def n_vgram(self):
        """Instances of the current batch on the generated-Fourier compact path."""
        return int(self.L.pint_query(self.ctx, 1))

    def nsplit(self):
        """The Gram's N-split count of the current batch (row blocks per instance)."""
        return int(self.L.pint_query(self.ctx, 2))

    def check(self):
        try:
            self._check(self.L.pint_check(self.ctx))
        finally:  # synchronised either way: the staging buffers are free again
            self._inflight.clear()
            self._keep.clear()

    # -- pipelined steps (lazy mode) ------------------------------------------------
    def step_end(self) -> int:
        """Close the step enqueued since the previous step_end; later launches, pinned
        buffers and status go to the next slot.  Returns the closed step's slot for
        check_step().  At most L.NSLOT steps in flight."""
        sl = C.c_int(-1)
        self._check(self.L.pint_step_end(self.ctx, C.byref(sl)))
        self._closed(sl.value)
        return sl.value

    def _closed(self, sl):
        self._slot_state[sl] = (self._inflight, self._keep)
        self._pending.add(sl)
        self._slot = (sl + 1) % L.NSLOT
        self._inflight, self._keep = self._slot_state[self._slot]

    def fit_step_enqueue(self, restore=True, lam=1.0, want_cov=True, noise=True):
        """One GLSFitter.fit_toas(maxiter=1) step of every instance enqueued by one C call
        (pint_fit_step_enqueue: [restore_tables], eval(FIT), fit_step_apply(1, lam),
        read_step, noise_resids, eval, chi2_gls, step_end).  Lazy mode.  Returns (slot,
        (steps, errors, covariances, linearised chi2), noise views or None, chi2); the
        pinned arrays are complete after check_step(slot)."""
        if not self.lazy:
            raise RuntimeError("fit_step_enqueue needs lazy mode (set_lazy(True))")
        lays = self.inst_layout
        ok = self._off_k
        dp, er = self._pin("dp", ok[-1]), self._pin("er", ok[-1])
        cov = self._pin("cov", self._off_cov[-1]) if want_cov else None
        cl = self._pin("cl", len(ok) - 1)
        n = int(self._off_n[-1])
        red = ec = dm = None
        if noise:
            if any(l.spec.dmn0 > 0 for l in lays):
                red = self._pin("noise_red", n)
            if any("EcorrNoise" in l.model.components for l in lays):
                ec = self._pin("noise_ec", n)
            if any(l.spec.dmn0 < l.nred for l in lays):
                dm = self._pin("noise_dm", n)
        c2 = self._pin("chi2g", len(lays))
        sl = C.c_int(-1)
        self._check(self.L.pint_fit_step_enqueue(self.ctx, 1 if restore else 0, 1, float(lam), L.ptr(dp), L.ptr(er),
                                                 L.ptr(cov), L.ptr(cl), L.ptr(red), L.ptr(ec), L.ptr(dm), L.ptr(c2),
                                                 C.byref(sl)))
        self._closed(sl.value)
        covs = SplitView(cov, self._off_cov, self._cov_shapes) if want_cov else []
        nz = _NoiseViews(lays, self._off_n, red, ec, dm) if noise else None
        return sl.value, (SplitView(dp, ok), SplitView(er, ok), covs, cl), nz, c2

    def check_step(self, slot: int):
        """Wait for the step closed as `slot`; its outputs (pinned buffers handed out while
        it was enqueued) and timing() are then complete."""
        rc = self.L.pint_check_step(self.ctx, int(slot))
        self._pending.discard(int(slot))
        inflight, keep = self._slot_state[slot]
        inflight.clear()
        keep.clear()
        self._check(rc)

    def read_step(self, want_cov=True):
        """(steps, errors, covariances, linearised chi2) of the last fit_step: per-instance
        views (SplitView) of the K+1 step / error vectors and the timing covariance."""
        ok = self._off_k
        # lazy: pinned per-slot buffers the copy stream fills; synchronous: fresh pageable
        # arrays (a first synchronous fit pays no page-locked allocation of its outputs)
        get = self._pin if self.lazy else (lambda name, n: np.empty(max(1, int(n))))
        dp = get("dp", ok[-1])
        er = get("er", ok[-1])
        cov = get("cov", self._off_cov[-1]) if want_cov else None
        cl = get("cl", len(ok) - 1)
        self._check(self.L.pint_read_step(self.ctx, L.ptr(dp), L.ptr(er), L.ptr(cov), L.ptr(cl)))
        covs = SplitView(cov, self._off_cov, self._cov_shapes) if want_cov else []
        return SplitView(dp, ok), SplitView(er, ok), covs, cl

    def read_tables(self):
        return self._split(self.read_tables_flat(), [l.tstride for l in self.inst_layout])

    def read_tables_flat(self):
        """All instances' parameter tables, concatenated."""
        t = np.empty(self.ntab)
        self._check(self.L.pint_get_tables(self.ctx, L.ptr(t)))
        return t

    def chi2_gls(self):
        c = self._pin("chi2g", len(self.inst_layout)) if self.lazy else np.empty(len(self.inst_layout))
        self._check(self.L.pint_chi2_gls(self.ctx, L.ptr(c)))
        return c

    def chi2_wls(self):
        """WLS chi2 of the current residuals per instance (pint_chi2_wls)."""
        c = self._pin("chi2w", len(self.inst_layout)) if self.lazy else np.empty(len(self.inst_layout))
        self._check(self.L.pint_chi2_wls(self.ctx, L.ptr(c)))
        return c

    def solve_eig(self, mode, thresholds):
        """SVD path of the fitters on the last fit_step's Gram (k_eig): replaces the step
        outputs; returns, per instance, the dropped directions (list of arrays over the
        instance's fit columns, smallest singular value first)."""
        n = len(self.inst_layout)
        th = np.ascontiguousarray(np.broadcast_to(np.asarray(thresholds, dtype=np.float64), (n,)))
        kmax = max((len(l.columns) if mode == 0 else l.K) for l in self.inst_layout)
        nd = np.zeros(n, dtype=np.int32)
        dv = np.zeros(n * L.EIG_MAXDEG * kmax)
        self._check(self.L.pint_solve_eig(self.ctx, int(mode), L.ptr(th), L.ptr(nd, C.c_int32), L.ptr(dv), kmax))
        dv = dv.reshape(n, L.EIG_MAXDEG, kmax)
        out = []
        for k, lay in enumerate(self.inst_layout):
            kk = len(lay.columns) if mode == 0 else lay.K
            out.append([dv[k, d, :kk].copy() for d in range(nd[k])])
        return out

    def lognorm(self, gls):
        """Per-instance likelihood normalisation: logdet(C)/2 of the last chi2_gls (gls=1), of
        C = N + 1e40 11^T (gls=2: correlated model, no basis columns) or sum log sigma (gls=0)
        (residuals.py:567-589, :638-667)."""
        out = np.zeros(len(self.inst_layout))
        self._check(self.L.pint_lognorm(self.ctx, int(gls), L.ptr(out)))
        return out

    def timing(self):
        ms = np.zeros(8)
        self.L.pint_last_timing(self.ctx, L.ptr(ms))
        return ms

    def inst_status(self):
        """Per-instance status bits (1 << PINT_E_*) raised since the last read (cleared)."""
        out = np.zeros(len(self.inst_layout), dtype=np.int32)
        self._check(self.L.pint_inst_status(self.ctx, L.ptr(out, C.c_int32)))
        return out

    def noise_resids(self):
        """Noise realisations of the last GLS fit_step: per instance {component: n-array}
        with the reference's component names (fitter.py:2270-2282, noise_model_dimensions)."""
        n = [l.n for l in self.inst_layout]
        anyred = any(l.spec.dmn0 > 0 for l in self.inst_layout)
        anyec = any("EcorrNoise" in l.model.components for l in self.inst_layout)
        anydm = any(l.spec.dmn0 < l.nred for l in self.inst_layout)
        if self.lazy:
            # enqueued (kernels after the solve, copies on the copy stream into pinned
            # buffers): the arrays handed out are complete after check()/check_step()
            red = self._pin("noise_red", sum(n)) if anyred else None
            ec = self._pin("noise_ec", sum(n)) if anyec else None
        else:
            red = np.empty(sum(n)) if anyred else None
            ec = np.empty(sum(n)) if anyec else None
        self._check(self.L.pint_noise_resids(self.ctx, L.ptr(red), L.ptr(ec)))
        if self.lazy:
            dm = None
            if anydm:  # PLDMNoise: enqueued on the copy stream as well (pint_noise_resids_dm)
                dm = self._pin("noise_dm", sum(n))
                self._check(self.L.pint_noise_resids_dm(self.ctx, L.ptr(dm)))
            return _NoiseViews(self.inst_layout, self._off_n, red if anyred else None, ec if anyec else None, dm)
        red = red if red is not None else np.zeros(sum(n))
        ec = ec if ec is not None else np.zeros(sum(n))
        dm = np.zeros(sum(n))
        if anydm:
            self._check(self.L.pint_noise_resids_dm(self.ctx, L.ptr(dm)))
        out = []
        for lay, r, e, m in zip(self.inst_layout, self._split(red, n), self._split(ec, n), self._split(dm, n)):
            d = {}
            if "EcorrNoise" in lay.model.components:
                d["ecorr_noise"] = e.copy()
            if lay.spec.dmn0 > 0:
                d["pl_red_noise"] = r.copy()
            if lay.spec.dmn0 < lay.nred:
                d["pl_DM_noise"] = m.copy()
            out.append(d)
        return out

    def read_norms(self, mode):
        """Per instance the K squared column norms of the last fit_step's design matrix
        (pint_read_norms): mode 1 the unweighted sums of squares of [M | F], mode 0 the
        whitened Gram's diagonal."""
        kk = [l.K + 1 for l in self.inst_layout]
        out = np.empty(sum(kk))
        self._check(self.L.pint_read_norms(self.ctx, int(mode), L.ptr(out)))
        return [x[:l.K] for x, l in zip(self._split(out, kk), self.inst_layout)]

    def debug_gram(self, pre_ecorr=False):
        """Stage-wise parity introspection: per instance (G, colsq) of the last fit_step, G the
        unnormalised (K+1)^2 normal matrix [M | r]^T N^-1 [M | r] (ECORR eliminated, or
        before the elimination with pre_ecorr), colsq M's unweighted column sums of squares."""
        sizes = [(l.K + 1) ** 2 + l.K for l in self.inst_layout]
        buf = np.empty(sum(sizes))
        self._check(self.L.pint_debug_gram(self.ctx, 1 if pre_ecorr else 0, L.ptr(buf)))
        out = []
        for lay, b in zip(self.inst_layout, self._split(buf, sizes)):
            w = lay.K + 1
            out.append((b[:w * w].reshape(w, w).copy(), b[w * w:].copy()))
        return out

    # -- noise-parameter fits (fitter.py:1230-1273) -----------------------------------
    def set_resids(self, resids):
        """Replace every instance's time residuals (list of n-arrays, seconds)."""
        self.debug_set_resids(resids)

    def set_sigma(self, lay, sigma_s):
        """Replace a pulsar's scaled TOA uncertainties (seconds) in place."""
        sg = np.ascontiguousarray(sigma_s, dtype=np.float64)
        if sg.shape != (lay.n,):
            raise ValueError(f"sigma must have {lay.n} entries")
        self._check(self.L.pint_set_sigma(self.ctx, lay.psr_id, L.ptr(sg)))

    def set_noise_weights(self, lay, red_phi=None, ep_phi=None):
        """Replace a pulsar's PLRedNoise (2 nred) and/or ECORR (nep) prior variances (s^2)."""
        rp = None if red_phi is None else np.ascontiguousarray(red_phi, dtype=np.float64)
        ep = None if ep_phi is None else np.ascontiguousarray(ep_phi, dtype=np.float64)
        if rp is not None and rp.shape != (2 * lay.nred,):
            raise ValueError(f"red_phi must have {2 * lay.nred} entries")
        if ep is not None and ep.shape != (lay.nep,):
            raise ValueError(f"ep_phi must have {lay.nep} entries")
        self._check(self.L.pint_set_noise_weights(self.ctx, lay.psr_id, L.ptr(rp), L.ptr(ep)))

    def set_noise_classes(self, lay, cls_ptr, cls_idx, sigma0_us):
        cp = np.ascontiguousarray(cls_ptr, dtype=np.int32)
        ci = np.ascontiguousarray(cls_idx, dtype=np.int32)
        s0 = np.ascontiguousarray(sigma0_us, dtype=np.float64)
        self._check(self.L.pint_set_noise_classes(self.ctx, lay.psr_id, len(cp) - 1, L.ptr(cp, C.c_int32),
                                                  L.ptr(ci, C.c_int32), L.ptr(s0)))

    def noise_lnlike(self, kinds, cls_qf, ep_w=None, grad=True):
        """k_noise_lnl over the batch: (out [ninst, 3] = (lnL, chi2, logdet C / 2),
        cls_g [sum ncls, 2], ep_g [sum nep]) -- see include/pint_amd.h pint_noise_lnlike."""
        kd = np.ascontiguousarray(kinds, dtype=np.int32)
        q = np.ascontiguousarray(cls_qf, dtype=np.float64).ravel()
        w = None if ep_w is None else np.ascontiguousarray(ep_w, dtype=np.float64)
        out = np.empty(3 * len(kd))
        g = np.empty(q.size) if grad else None
        nep = sum(l.nep for l in self.inst_layout)
        eg = np.empty(max(nep, 1)) if grad else None
        self._check(self.L.pint_noise_lnlike(self.ctx, L.ptr(kd, C.c_int32), L.ptr(q), L.ptr(w), L.ptr(out),
                                             L.ptr(g), L.ptr(eg)))
        return out.reshape(-1, 3), (g.reshape(-1, 2) if grad else None), (eg[:nep] if grad else None)

    def debug_set_resids(self, resids):
        """Replace every instance's time residuals (list of n-arrays, seconds)."""
        flat = np.ascontiguousarray(np.concatenate([np.asarray(r, dtype=np.float64) for r in resids]))
        if flat.size != sum(l.n for l in self.inst_layout):
            raise ValueError("residual arrays do not match the batch's TOA counts")
        self._check(self.L.pint_debug_set_resids(self.ctx, L.ptr(flat)))


def release_cache():
    """Hand the device-buffer cache back to the HIP runtime (pint_release_cache)."""
    L.lib().pint_release_cache()


class _NoiseViews(SplitView):
    """Per-instance {component: n-array} views of the noise realisations (lazy sessions)."""

    def __init__(self, lays, off, red, ec, dm=None):
        super().__init__(None, off)
        self.lays, self.red, self.ec, self.dm = lays, red, ec, dm

    def __getitem__(self, k):
        if isinstance(k, slice):
            return [self[i] for i in range(*k.indices(len(self)))]
        if k < 0:
            k += len(self)
        lay, a, b = self.lays[k], self.off[k], self.off[k + 1]
        d = {}
        if self.ec is not None and "EcorrNoise" in lay.model.components:
            d["ecorr_noise"] = self.ec[a:b]
        if self.red is not None and lay.spec.dmn0 > 0:
            d["pl_red_noise"] = self.red[a:b]
        if self.dm is not None and lay.spec.dmn0 < lay.nred:
            d["pl_DM_noise"] = self.dm[a:b]
        return d


# -- resident uploads (reference-API single fits and residuals) ------------------------
# The last few (TOAs, model structure) uploads stay on the device with their Session, like
# the TOAs of a serving process: a fit or Residuals of the same TOAs and model structure
# re-binds one parameter table instead of packing and uploading the TOAs again.  An entry is
# reused only when every parameter outside the device table (noise values, DMX ranges,
# masks, TZR, ...) is unchanged, the frozen set and the components are the same and the
# TOA object is the same object; anything else re-uploads.
RESIDENT_MAX = 4
_RESIDENT: "Dict[tuple, tuple]" = {}


def _structure_sig(model, lay):
    # the values themselves (scalars compared with ==; a NaN never matches, so it re-uploads)
    # (the parameter dict's insertion order and the components fix the column order); mask
    # parameters also by their selector (key, key_value), which build_layout/pack_toas turn
    # into the per-TOA JUMP/EFAC/EQUAD/ECORR/DMJUMP masks
    offs = lay.offsets
    return (tuple(model.components), model.binary,
            tuple((n, (p.value is None) if n in offs else p.value, p.frozen, p.key,
                   tuple(str(v) for v in (p.key_value or ()))) for n, p in model._params.items()))


def _toas_fingerprint(toas):
    """What the upload of `toas` was built from, by object identity: every TOA column (numpy
    arrays are read-only views and flag columns tuples, pint_amd.toa._Columns, so a column
    changes only by being replaced), the observatory column and the TZR TOA's values.  The
    objects themselves are held (not their ids), so a freed column's address cannot be
    reused by a new one while the entry lives.  O(columns), not O(TOAs): hashing every
    column's bytes per fit cost ~1.3-2.7 ms on C3's 50k TOAs."""
    tz = getattr(toas, "tzr", None) or {}

    def val(v):  # the TZR row's values (an array's bytes: numpy's repr costs ~30 us each)
        if isinstance(v, np.ndarray):
            return (v.dtype.str, v.shape, v.tobytes() if v.dtype != object else repr(v.tolist()))
        if isinstance(v, dict):
            return tuple(sorted((k, repr(x)) for k, x in v.items()))
        return repr(v)
    return (tuple(sorted(toas.arrays.items())), tuple(sorted(toas.flag_columns.items())), getattr(toas, "obs", None),
            tuple((k, val(tz[k])) for k in sorted(tz)))


def _same_fingerprint(a, b):
    def same_cols(x, y):
        return len(x) == len(y) and all(kx == ky and vx is vy for (kx, vx), (ky, vy) in zip(x, y))
    return same_cols(a[0], b[0]) and same_cols(a[1], b[1]) and a[2] is b[2] and a[3] == b[3]


def resident(model, toas, tag=None, track_mode=None, subtract_mean=True, use_weighted_mean=True,
             use_gls_basis=True):
    """(Session, PulsarLayout) of the resident upload of (model structure, toas), creating
    it (and evicting the least recently used entry beyond RESIDENT_MAX) when needed.  The
    Session belongs to the cache: callers must not close it."""
    key = (id(toas), toas.ntoas, tag, track_mode, bool(subtract_mean), bool(use_weighted_mean), bool(use_gls_basis))
    ent = _RESIDENT.pop(key, None)
    fp = _toas_fingerprint(toas)
    if ent is not None:
        s, lay, t0, sig, fp0 = ent
        if t0 is toas and _same_fingerprint(fp, fp0) and model.binary != "ELL1H" and _structure_sig(model, lay) == sig:
            model.validate()
            _RESIDENT[key] = ent  # most recently used last
            return s, lay
        s.close()
    s = Session()
    try:
        lay = s.add(build_layout(model, toas, track_mode=track_mode, subtract_mean=subtract_mean,
                                 use_weighted_mean=use_weighted_mean, use_gls_basis=use_gls_basis))
    except Exception:
        s.close()
        raise
    _RESIDENT[key] = (s, lay, toas, _structure_sig(model, lay), fp)
    while len(_RESIDENT) > RESIDENT_MAX:
        old = next(iter(_RESIDENT))
        _RESIDENT.pop(old)[0].close()
    return s, lay


def drop_resident():
    """Close every resident upload's Session."""
    while _RESIDENT:
        _RESIDENT.pop(next(iter(_RESIDENT)))[0].close()


# -- convenience single-model evaluations (used by TimingModel methods) ----------------
def _single(model, toas, **kw):
    s = Session()
    lay = s.add(build_layout(model, toas, **kw))
    s.set_instances([(lay, pack_table(lay))])
    return s, lay


def evaluate_delay_phase(model, toas):
    s, lay = _single(model, toas)
    s.eval(False)
    hi, lo, ft, dl = [x[0] for x in s.read_eval()]
    s.close()
    return {"delay": dl[:-1], "phase_hi": hi, "phase_lo": lo, "tzr_delay": dl[-1], "phase": (hi, lo)}


def evaluate_designmatrix(model, toas):
    s, lay = _single(model, toas, use_gls_basis=False)
    s.eval(True)
    M = s.read_designmatrix()[0]
    s.close()
    return M[:, :len(lay.columns)].copy(), list(lay.columns), [UNITS.get(c, "") for c in lay.columns]
