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
from typing import Dict, List, Optional

import numpy as np

FIELDS = ["tdb_hi", "tdb_lo", "freq_mhz", "err_us", "ssb_obs_pos_km", "ssb_obs_vel_kms", "obs_sun_pos_km",
          "mjd_float", "is_bary", "delta_pulse_number"]


class TOAs:
    def __init__(self, arrays: Dict[str, np.ndarray], flag_columns: Optional[Dict[str, List[str]]] = None,
                 tzr: Optional[Dict[str, np.ndarray]] = None, name: str = "", obs: Optional[List[str]] = None):
        self.arrays = {k: np.asarray(v) for k, v in arrays.items()}
        n = len(self.arrays["tdb_hi"])
        self.flag_columns = {k: list(v) for k, v in (flag_columns or {}).items()}
        for k, v in self.flag_columns.items():
            if len(v) != n:
                raise ValueError(f"flag column {k} has {len(v)} rows, expected {n}")
        if "delta_pulse_number" not in self.arrays:
            self.arrays["delta_pulse_number"] = np.zeros(n)
        if "is_bary" not in self.arrays:
            self.arrays["is_bary"] = np.zeros(n, dtype=np.uint8)
        self.tzr = tzr
        self.name = name
        # observatory (canonical site name) of each TOA, when known: TEL masks select on it
        self.obs = None if obs is None else np.asarray([str(o) for o in obs], dtype=object)
        if self.obs is not None and len(self.obs) != n:
            raise ValueError(f"obs has {len(self.obs)} rows, expected {n}")
        self.ephem = None   # the host preparation's ephemeris / clock chain, when known
        self.clock = None   # (update_model writes them into the model as EPHEM / CLOCK)
        self._uid = id(self)

    # -- reference-like accessors ------------------------------------------------------
    @property
    def ntoas(self) -> int:
        return len(self.arrays["tdb_hi"])

    def __len__(self):
        return self.ntoas

    @property
    def tdbld(self) -> np.ndarray:
        return self.arrays["tdb_hi"].astype(np.longdouble) + self.arrays["tdb_lo"].astype(np.longdouble)

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

    def get_Tspan(self) -> float:
        m = self.get_mjds()
        return float(m.max() - m.min())

    def __getitem__(self, idx):
        idx = np.arange(self.ntoas)[idx]
        arr = {k: v[idx] for k, v in self.arrays.items()}
        fl = {k: [v[i] for i in idx] for k, v in self.flag_columns.items()}
        return TOAs(arr, fl, self.tzr, self.name, None if self.obs is None else self.obs[idx])

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
        return np.array([i for i, c in enumerate(col) if c == key_value[0]], dtype=int)

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
            json.dump({"flag_columns": self.flag_columns, "name": self.name, "obs_names": names}, f)


def from_arrays_with_tzr(z: Dict[str, np.ndarray], flag_columns=None, name="", obs_names=None) -> TOAs:
    arrays = {k: np.asarray(z[k]) for k in z if not k.startswith("tzr_") and (k in FIELDS or k in (
        "pulse_number", "ssb_obs_vel_ecl_kms"))}
    tzr = None
    if "tzr_tdb_hi" in z:
        tzr = {k[4:]: np.asarray(z[k]) for k in z if k.startswith("tzr_")}
        tzr["flags"] = {}
    obs = None
    if obs_names is not None and "obs_index" in z:
        obs = [obs_names[i] for i in np.asarray(z["obs_index"])]
    return TOAs(arrays, flag_columns, tzr, name, obs)


def get_TOAs(path: str, **kwargs) -> TOAs:
    """Load packed TOAs (``.npz`` + optional ``.json`` with ``flag_columns``)."""
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


def get_model_and_toas(parfile: str, timfile: str, **kwargs):
    """Reference API (model_builder.py:859).  ``timfile`` must be a packed TOA file."""
    from .timing_model import get_model
    return get_model(parfile), get_TOAs(timfile)
