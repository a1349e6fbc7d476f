"""Packed TOA container (host side).

TOA loading, clock corrections, TDB and ephemeris lookup stay on the host (north star);
this module holds the *result* of that preparation in the boundary schema of SURVEY.md
Appendix C -- the same columns the reference keeps in ``TOAs.table`` (toa.py:2320 tdbld,
:2385-2439 ssb_obs_pos / ssb_obs_vel / obs_sun_pos, freq, error, mjd_float,
pulse_number, delta_pulse_number, flags) -- plus the TZR TOA (absolute_phase.py:79).

Loaders: ``get_TOAs(path)`` reads a packed ``.npz`` (+ ``.json`` sidecar with flag
columns), as written by ``oracle/refgen`` from the reference's own TOAs or by
``pint_amd.simulation``.  Ingesting raw ``.tim`` files (TDB, ephemeris, clocks) on the GPU
host is SURVEY.md §8(f) item 1 and is not part of this round.
"""
from __future__ import annotations

import json
import os
import warnings
from typing import Dict, List, Optional

import numpy as np

FIELDS = ["tdb_hi", "tdb_lo", "freq_mhz", "err_us", "ssb_obs_pos_km", "ssb_obs_vel_kms", "obs_sun_pos_km",
          "mjd_float", "is_bary", "delta_pulse_number"]
# compute_posvels(planets=True) columns (toa.py:96 all_planets, :2403-2433)
PLANET_FIELDS = [f"obs_{p}_pos_km" for p in ("jupiter", "saturn", "venus", "uranus", "neptune", "earth")]


def _ro_array(v):
    """A read-only view of v (the caller's array keeps its own flags)."""
    a = np.asarray(v).view()
    a.setflags(write=False)
    return a


class _Columns(dict):
    """TOA columns whose values cannot be edited in place: a column changes only by being
    replaced (``toas.arrays[k] = new``), which the resident-upload cache
    (engine.resident) sees by object identity instead of hashing every column per fit."""
    @staticmethod
    def _conv(v):
        raise NotImplementedError

    def __init__(self, items=()):
        super().__init__()
        self.update(items)

    def __setitem__(self, k, v):
        super().__setitem__(k, self._conv(v))

    def update(self, items=(), **kw):
        for k, v in (items.items() if hasattr(items, "items") else items):
            self[k] = v
        for k, v in kw.items():
            self[k] = v

    def setdefault(self, k, v=None):
        if k not in self:
            self[k] = v
        return self[k]


class _ArrayColumns(_Columns):
    _conv = staticmethod(_ro_array)


class _FlagColumns(_Columns):
    _conv = staticmethod(tuple)


class TOAs:
    def __init__(self, arrays: Dict[str, np.ndarray], flag_columns: Optional[Dict[str, List[str]]] = None,
                 tzr: Optional[Dict[str, np.ndarray]] = None, name: str = "", obs: Optional[List[str]] = None):
        self.arrays = arrays
        n = len(self.arrays["tdb_hi"])
        self.flag_columns = flag_columns or {}
        for k, v in self.flag_columns.items():
            if len(v) != n:
                raise ValueError(f"flag column {k} has {len(v)} rows, expected {n}")
        if "delta_pulse_number" not in self.arrays:
            self.arrays["delta_pulse_number"] = np.zeros(n)
        if "is_bary" not in self.arrays:
            self.arrays["is_bary"] = np.zeros(n, dtype=np.uint8)
        self.tzr = tzr
        self.name = name
        self.prepared = None  # tim-file TOAs: the preparation options (TZR TOAs are prepared alike)
        self.commands = []
        # observatory (canonical site name) of each TOA, when known: TEL masks select on it
        self.obs = obs
        if self.obs is not None and len(self.obs) != n:
            raise ValueError(f"obs has {len(self.obs)} rows, expected {n}")
        self.ephem = None   # the host preparation's ephemeris / clock chain, when known
        self.clock = None   # (update_model writes them into the model as EPHEM / CLOCK)
        self._uid = id(self)

    # read-only columns (numpy arrays as read-only views, flag columns as tuples): assigning
    # a new dict or a new column replaces objects, an in-place edit raises
    @property
    def arrays(self):
        return self._arrays

    @arrays.setter
    def arrays(self, v):
        self._arrays = _ArrayColumns(v)

    @property
    def flag_columns(self):
        return self._flags

    @flag_columns.setter
    def flag_columns(self, v):
        self._flags = _FlagColumns(v)

    @property
    def obs(self):
        """Observatory (canonical site name) of each TOA, when known (TEL masks select on it)."""
        return self._obs

    @obs.setter
    def obs(self, v):
        self._obs = None if v is None else _ro_array(np.asarray([str(o) for o in v], dtype=object))

    # -- reference-like accessors ------------------------------------------------------
    @property
    def planets(self) -> bool:
        """Planet positions present (toa.py:1336 TOAs.planets / compute_posvels(planets=True))."""
        return all(k in self.arrays for k in PLANET_FIELDS)

    @property
    def ntoas(self) -> int:
        return len(self.arrays["tdb_hi"])

    def __len__(self):
        return self.ntoas

    @property
    def tdbld(self) -> np.ndarray:
        return self.arrays["tdb_hi"].astype(np.longdouble) + self.arrays["tdb_lo"].astype(np.longdouble)

    def tdbld_extent(self):
        """(min, max) of tdbld, equal to tdbld.min() / .max(), from the few TOAs whose hi part
        is extreme (with lo within half an ulp of hi the order of hi decides but for ties):
        the red-noise span T needs only these, not a longdouble pass over every TOA."""
        hi, lo = self.arrays["tdb_hi"], self.arrays["tdb_lo"]
        if len(hi) == 0:
            t = self.tdbld
            return t.min(), t.max()
        hmin, hmax = hi.min(), hi.max()
        # every |lo| within half an ulp of its hi: at once when the largest |lo| is within half
        # an ulp of the smallest positive hi (the ulp only grows with |hi|), else row by row
        if not (hmin > 0 and max(lo.max(), -lo.min()) <= 0.5 * np.spacing(hmin)) and \
                not np.all(np.abs(lo) <= 0.5 * np.spacing(np.abs(hi))):
            t = self.tdbld
            return t.min(), t.max()
        out = []
        for ext in (hmin, hmax):
            k = np.flatnonzero(hi == ext)
            v = hi[k].astype(np.longdouble) + lo[k].astype(np.longdouble)
            out.append(v.min() if ext == hmin and len(out) == 0 else v.max())
        return out[0], out[1]

    def get_mjds(self) -> np.ndarray:
        return self.arrays["mjd_float"]

    def get_errors(self) -> np.ndarray:
        """TOA uncertainties in microseconds (toa.py:1697)."""
        return self.arrays["err_us"]

    def get_freqs(self) -> np.ndarray:
        return self.arrays["freq_mhz"]

    def get_pulse_numbers(self) -> Optional[np.ndarray]:
        return self.arrays.get("pulse_number")

    def get_flag_value(self, flag: str, fill_value=None):
        col = self.flag_columns.get(flag)
        if col is None:
            return [fill_value] * self.ntoas, []
        return [c if c != "" else fill_value for c in col], [i for i, c in enumerate(col) if c != ""]

    def is_wideband(self) -> bool:
        """toa.py:1656: every TOA carries a -pp_dm measurement."""
        col = self.flag_columns.get("pp_dm")
        return col is not None and all(c != "" for c in col)

    @property
    def wideband(self) -> bool:
        return self.is_wideband()

    def get_dms(self) -> np.ndarray:
        """The wideband DM measurements, pc/cm^3 (toa.py:1767, the -pp_dm flags)."""
        v, valid = self.get_flag_value("pp_dm")
        if valid == []:
            raise AttributeError("No DM is provided.")
        return np.array([float(v[i]) for i in valid])

    def get_dm_errors(self) -> np.ndarray:
        """Their uncertainties, pc/cm^3 (toa.py:1780, the -pp_dme flags)."""
        v, valid = self.get_flag_value("pp_dme")
        if valid == []:
            raise AttributeError("No DM error is provided.")
        return np.array([float(v[i]) for i in valid])

    def get_Tspan(self) -> float:
        m = self.get_mjds()
        return float(m.max() - m.min())

    def __getitem__(self, idx):
        idx = np.arange(self.ntoas)[idx]
        arr = {k: v[idx] for k, v in self.arrays.items()}
        fl = {k: [v[i] for i in idx] for k, v in self.flag_columns.items()}
        return TOAs(arr, fl, self.tzr, self.name, None if self.obs is None else self.obs[idx])

    def tzr_for(self, model):
        """The TZR TOA row of ``model`` (absolute_phase.py:79-127 get_TZR_toa): the stored one
        (packed fixtures), else -- for TOAs prepared from a tim file -- TZRMJD at TZRSITE with
        TZRFRQ prepared with the same options, cached on (TZRMJD, TZRSITE, TZRFRQ)."""
        if self.tzr is not None or self.prepared is None or "TZRMJD" not in model or model.TZRMJD.value is None:
            return self.tzr
        key = (str(model.TZRMJD.value), str(model.TZRSITE.value) if "TZRSITE" in model else None,
               None if "TZRFRQ" not in model or model.TZRFRQ.value is None else float(model.TZRFRQ.value))
        cache = self.prepared.setdefault("tzr_cache", {})
        if key not in cache:
            cache[key] = tzr_row(model, self.prepared)
        return cache[key]

    def get_obss(self):
        """Site name of each TOA (toa.py get_obss)."""
        if self.obs is None:
            raise ValueError("these TOAs carry no observatory names")
        return self.obs

    # -- mask selection (parameter.py:2124 select_toa_mask, toa_select.py:101) ----------
    def select_mask(self, key: str, key_value: List[str], tzr: bool = False) -> np.ndarray:
        """Indices selected by a mask parameter key; with tzr=True evaluate it on the TZR
        TOA instead (returns [0] or [])."""
        k = key[1:] if key.startswith("-") else key
        kl = key.lower()
        if kl == "tel":  # parameter.py:1868 / :2156: the canonical site name vs the obs column
            from .observatory import get_observatory_name
            site = get_observatory_name(key_value[0])
            if tzr:
                o = (self.tzr or {}).get("obs")
                return np.array([0]) if o is not None and get_observatory_name(str(np.atleast_1d(o)[0])) == site \
                    else np.array([], dtype=int)
            if self.obs is None:
                raise NotImplementedError("TEL masks need the TOAs' observatory names")
            return np.where(self.obs == site)[0]
        if kl in ("mjd", "freq"):
            col = {"mjd": "mjd_float", "freq": "freq_mhz"}[kl]
            src = (self.tzr or {}).get(col, np.zeros(0)) if tzr else self.arrays[col]
            src = np.asarray(src, dtype=float)
            if len(key_value) == 2:
                lo, hi = float(key_value[0]), float(key_value[1])
                return np.where((src >= lo) & (src <= hi))[0]
            return np.where(src == float(key_value[0]))[0]
        if tzr:
            fl = (self.tzr or {}).get("flags", {})
            return np.array([0]) if fl.get(k) == key_value[0] else np.array([], dtype=int)
        col = self.flag_columns.get(k)
        if col is None:
            return np.array([], dtype=int)
        if len(key_value) == 2:
            raise NotImplementedError("range selection on a flag column")
        # each entry compared with == as the reference's selector does (an object array keeps
        # None and non-string values as they are); the column's object array and the
        # selections are cached per column object (flag columns are tuples: an edit replaces
        # the column, and the cache entry with it) -- EFAC, EQUAD and JUMP masks on one flag
        # share them at upload
        cache = self.__dict__.setdefault("_sel_cache", {})
        ent = cache.get(k)
        if ent is None or ent[0] is not col:
            arr = np.empty(len(col), dtype=object)
            arr[:] = col
            ent = cache[k] = (col, arr, {})
        sel = ent[2]
        v = key_value[0]
        key_ = (type(v), v) if isinstance(v, (str, int, float)) else None
        hit = sel.get(key_) if key_ is not None else None
        if hit is None:
            hit = np.where(ent[1] == v)[0]
            hit.setflags(write=False)
            if key_ is not None:
                sel[key_] = hit
        return hit

    # -- persistence -----------------------------------------------------------------
    def save(self, path: str):
        base = path[:-4] if path.endswith(".npz") else path
        arr = dict(self.arrays)
        names = None
        if self.obs is not None:
            names = sorted(set(self.obs.tolist()))
            arr["obs_index"] = np.array([names.index(o) for o in self.obs], dtype=np.int16)
        if self.tzr:
            arr.update({"tzr_" + k: np.atleast_1d(v) for k, v in self.tzr.items() if k != "flags"})
        np.savez_compressed(base + ".npz", **arr)
        with open(base + ".json", "w") as f:
            json.dump({"flag_columns": {k: list(v) for k, v in self.flag_columns.items()}, "name": self.name,
                       "obs_names": names}, f)


def from_arrays_with_tzr(z: Dict[str, np.ndarray], flag_columns=None, name="", obs_names=None) -> TOAs:
    arrays = {k: np.asarray(z[k]) for k in z if not k.startswith("tzr_") and (k in FIELDS or k in PLANET_FIELDS or k in (
        "pulse_number", "ssb_obs_vel_ecl_kms"))}
    tzr = None
    if "tzr_tdb_hi" in z:
        tzr = {k[4:]: np.asarray(z[k]) for k in z if k.startswith("tzr_")}
        tzr["flags"] = {}
    obs = None
    if obs_names is not None and "obs_index" in z:
        obs = [obs_names[i] for i in np.asarray(z["obs_index"])]
    return TOAs(arrays, flag_columns, tzr, name, obs)


def _is_tim(path) -> bool:
    if hasattr(path, "readlines"):
        return True
    p = str(path)
    return not (p.endswith(".npz") or os.path.exists(p + ".npz"))


def _ephem_choice(ephem, model):
    if ephem is None and model is not None and "EPHEM" in model and model.EPHEM.value:
        ephem = str(model.EPHEM.value)
    ephem = "builtin" if ephem is None else ephem
    if str(ephem).lower() != "builtin":
        raise NotImplementedError(
            f"ephemeris {ephem!r} is not available offline: only the 'builtin' (erfa epv00) table is bundled "
            "(pass ephem='builtin')")
    return "builtin"


def _bipm_choice(include_bipm, model):
    """toa.py:196-225: CLOCK = TT(TAI) or UNCORR -> no BIPM correction."""
    if include_bipm is None and model is not None and "CLOCK" in model and model.CLOCK.value:
        clk = str(model.CLOCK.value)
        if clk in ("TT(TAI)", "UNCORR"):
            include_bipm = False
    if include_bipm is None:
        include_bipm = True
    if include_bipm:
        raise NotImplementedError("the TT(BIPM) clock table is not bundled: pass include_bipm=False "
                                  "(TT(TAI)), as the model's CLOCK = TT(TAI) does")
    return False


_NO_CLOCK_SITES = {"barycenter", "geocenter", "spacecraft", "ssb", "stl_geo"}


def _warn_missing_clocks(obs, clock_files):
    """The reference applies each topocentric site's clock files by default and warns when
    they are missing (observatory/topo_obs.py clock_corrections); here clock files are only
    applied when passed, so topocentric TOAs without any for their site warn the same way
    (residuals of real observatory data then differ from the reference's at the us level)."""
    from .observatory import get_observatory_name
    have = set()
    for k in (clock_files or {}):
        try:
            have.add(get_observatory_name(k))
        except KeyError:
            have.add(str(k))
    for site in sorted(set(obs)):
        try:
            canon = get_observatory_name(site)
        except KeyError:
            canon = str(site)
        if canon.lower() in _NO_CLOCK_SITES or canon in have:
            continue
        warnings.warn(f"No clock corrections found for observatory {canon}: topocentric TOAs are prepared "
                      "without site clock corrections (pass clock_files={site: path} to apply them)",
                      UserWarning)


def load_tim(timfile, model=None, ephem=None, include_bipm=None, planets=None, include_pn=True,
             clock_files=None) -> TOAs:
    """get_TOAs for a tim file (toa.py:109-330) without PINT/astropy: read (pint_amd.tim),
    clock corrections (TIME statements as -to flags, plus optional per-site clock files,
    pint_amd.clock), TDB and posvels (pint_amd.prep), pulse numbers and PHASE/-padd
    (toa.py:1959-1983).  Options follow the reference (EPHEM/CLOCK from the model); only the
    builtin ephemeris is available offline, and BIPM corrections are not bundled."""
    from . import prep
    from .tim import read_tim
    ephem = _ephem_choice(ephem, model)
    _bipm_choice(include_bipm, model)
    if planets is None:   # toa.py:226-231: the model's PLANET_SHAPIRO decides
        planets = bool(model is not None and "PLANET_SHAPIRO" in model and model.PLANET_SHAPIRO.value)
    recs, commands = read_tim(timfile)
    if not recs:
        raise ValueError("No TOAs found!")
    n = len(recs)
    day = np.array([r.imjd for r in recs], dtype=np.float64)
    frac = np.array([r.fmjd for r in recs], dtype=np.float64)
    obs = [r.obs for r in recs]
    flags = [dict(r.flags) for r in recs]
    corr = np.array([float(f.get("to", 0.0)) for f in flags])
    _warn_missing_clocks(obs, clock_files)
    if clock_files:
        from .clock import site_corrections
        corr = corr + site_corrections(clock_files, obs, day + frac)
    for f, c in zip(flags, corr):
        if c != 0:
            f["clkcorr"] = str(c)
    cols = prep.prepare(day, frac, obs, corr, planets=bool(planets))
    cols["freq_mhz"] = np.array([r.freq_mhz for r in recs], dtype=np.float64)
    cols["err_us"] = np.array([r.error_us for r in recs], dtype=np.float64)
    # phase_columns_from_flags (toa.py:1959-1983)
    dph = np.array([float(f.get("phase", 0)) + float(f.get("padd", 0)) for f in flags])
    cols["delta_pulse_number"] = dph
    pns = np.array([float(f.get("pn", np.nan)) for f in flags])
    if include_pn and not np.all(np.isnan(pns)):
        cols["pulse_number"] = pns
    for f in flags:
        f.pop("pn", None)
        f.pop("padd", None)
    keys = list(dict.fromkeys(k for f in flags for k in f))
    fc = {k: [f.get(k, "") for f in flags] for k in keys}
    name = getattr(timfile, "name", None) or os.path.basename(str(timfile))
    t = TOAs(cols, fc, None, name, obs)
    t.ephem = ephem
    t.clock = "TT(TAI)"
    t.commands = commands
    t.prepared = {"ephem": ephem, "include_bipm": False, "clock_files": clock_files, "planets": bool(planets)}
    return t


def tzr_row(model, prepared) -> dict:
    """get_TZR_toa (absolute_phase.py:79-127) prepared like the TOAs: TZRMJD (its parsed
    day + fraction) at TZRSITE (default barycenter) with TZRFRQ (none/0 -> infinite)."""
    from . import prep
    from .observatory import get_observatory_name
    p = model.TZRMJD
    day, frac = p.mjd_pair if p.mjd_pair is not None else (float(np.floor(p.value)), float(p.value - np.floor(p.value)))
    site = get_observatory_name(model.TZRSITE.value if "TZRSITE" in model and model.TZRSITE.value else "ssb")
    fr = float(model.TZRFRQ.value) if "TZRFRQ" in model and model.TZRFRQ.value is not None else np.inf
    if fr == 0.0:
        fr = np.inf
    corr = None
    if prepared.get("clock_files"):
        from .clock import site_corrections
        corr = site_corrections(prepared["clock_files"], [site], np.array([day + frac]))
    # the TZR TOA is prepared with the TOAs' planets choice (absolute_phase.py:118)
    cols = prep.prepare(np.array([day]), np.array([frac]), [site], corr, planets=prepared.get("planets", False))
    cols["freq_mhz"] = np.array([fr])
    cols["delta_pulse_number"] = np.zeros(1)
    cols["flags"] = {}
    cols["obs"] = np.array([site])
    return cols


def get_TOAs(path, ephem=None, include_bipm=None, planets=None, include_pn=True, model=None, **kwargs) -> TOAs:
    """Load TOAs (toa.py:109 get_TOAs): a tim file is read and prepared on the host
    (load_tim); a packed ``.npz`` (+ optional ``.json`` with ``flag_columns``) is loaded as is."""
    if _is_tim(path):
        return load_tim(path, model=model, ephem=ephem, include_bipm=include_bipm, planets=planets,
                        include_pn=include_pn, clock_files=kwargs.get("clock_files"))
    base = path[:-4] if path.endswith(".npz") else path
    z = dict(np.load(base + ".npz", allow_pickle=False))
    fl, name, obs = None, os.path.basename(base), None
    if os.path.exists(base + ".json"):
        with open(base + ".json") as f:
            meta = json.load(f)
        fl = meta.get("flag_columns")
        name = meta.get("name", name)
        obs = meta.get("obs_names")
    return from_arrays_with_tzr(z, fl, name, obs)


def get_model_and_toas(parfile: str, timfile: str, ephem=None, include_bipm=None, planets=None,
                       include_pn=True, **kwargs):
    """Reference API (model_builder.py:859): the model, then its TOAs prepared with the
    model's EPHEM/CLOCK/PLANET_SHAPIRO (a tim file) or loaded packed (``.npz``)."""
    from .timing_model import get_model
    m = get_model(parfile)
    return m, get_TOAs(timfile, ephem=ephem, include_bipm=include_bipm, planets=planets, include_pn=include_pn,
                       model=m, **kwargs)
