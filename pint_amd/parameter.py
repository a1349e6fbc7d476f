"""Timing-model parameters and par-file parsing (host side).

Mirrors the behaviour of the reference's parameter classes for the parameters on the hot
path (reference ``src/pint/models/parameter.py``): values keep the precision the reference
keeps -- numpy longdouble for ``long_double=True`` parameters and all MJD parameters
(``parameter.py:1064`` MJDParameter, ``:1143`` time_to_longdouble), float64 otherwise
(``fortran_float``) -- and unit-scaled binary rates follow ``parameter.py:765-800``
(``PBDOT 7.2`` means 7.2e-12 when ``|value| > 1e-7``).

Values are held in the reference's par-file units (``.value``); the device code converts
to SI where it evaluates (``pint_amd/csrc/physics.hpp``).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

LD = np.longdouble


def fortran_float(s: str) -> float:
    """Parse a par-file float allowing Fortran ``D`` exponents (parameter.py fortran_float)."""
    return float(s.replace("D", "E").replace("d", "e"))


def data2longdouble(s: str) -> np.longdouble:
    return np.longdouble(s.replace("D", "E").replace("d", "e"))


def mjd_string_to_longdouble(s: str) -> np.longdouble:
    """MJD string -> longdouble as the reference does it: integer day plus the fractional
    part parsed as float64 (pulsar_mjd.py _str_to_mjds + time_to_longdouble)."""
    s = s.strip().replace("D", "E").replace("d", "e")
    if "e" in s.lower():
        return np.longdouble(s)
    neg = s.startswith("-")
    s = s.lstrip("+-")
    if "." in s:
        ip, fp = s.split(".", 1)
    else:
        ip, fp = s, "0"
    v = np.longdouble(int(ip or "0")) + np.longdouble(float("0." + (fp or "0")))
    return -v if neg else v


def parse_sexagesimal(s: str) -> float:
    """``hh:mm:ss.s`` / ``dd:mm:ss.s`` -> float hours/degrees (astropy hms_to_hours /
    dms_to_degrees: sign * (|h| + m/60 + s/3600))."""
    s = s.strip()
    sign = -1.0 if s.startswith("-") else 1.0
    parts = s.lstrip("+-").split(":")
    h = float(parts[0])
    m = float(parts[1]) if len(parts) > 1 else 0.0
    sec = float(parts[2]) if len(parts) > 2 else 0.0
    return sign * (abs(h) + abs(m) / 60.0 + abs(sec) / 3600.0)


@dataclass
class Param:
    """One timing-model parameter (subset of the reference Parameter API)."""

    name: str
    kind: str = "float"  # float | mjd | hourangle | degangle | str | bool | int | mask
    units: str = ""
    long_double: bool = False
    value: object = None
    frozen: bool = True
    uncertainty_value: Optional[float] = None
    key: Optional[str] = None
    key_value: List[str] = field(default_factory=list)
    index: Optional[int] = None
    scale: Optional[tuple] = None  # (scale_factor, threshold) unit_scale params
    component: str = ""
    description: str = ""
    alias: Optional[str] = None       # the par-file spelling when it was an alias (use_alias)
    mjd_pair: Optional[tuple] = None  # MJDs: the parsed (day, fraction) float64 pair
    implicit: bool = False            # a 0 default standing in for the reference's unset value

    # -- value handling ---------------------------------------------------------------
    def set_from_string(self, s: str):
        k = self.kind
        if k in ("str",):
            self.value = s
        elif k == "bool":
            self.value = s.upper() in ("Y", "YES", "T", "TRUE", "1")
        elif k == "int":
            self.value = int(float(s))
        elif k == "hourangle" or k == "degangle":
            self.value = parse_sexagesimal(s) if ":" in s else fortran_float(s)
        elif k == "mjd":
            from .parfile import str_to_mjds
            self.value = mjd_string_to_longdouble(s)
            self.mjd_pair = str_to_mjds(s)
        else:
            v = data2longdouble(s) if self.long_double else fortran_float(s)
            if self.scale is not None and abs(float(v)) > abs(self.scale[1]):
                v = v * (LD(self.scale[0]) if self.long_double else self.scale[0])
            self.value = v

    def set_uncertainty_from_string(self, s: str):
        try:
            # long-double parameters keep a longdouble uncertainty (parameter.py
            # _set_uncertainty parses it like the value)
            u = data2longdouble(s) if (self.long_double and self.kind in ("float", "mjd")) else fortran_float(s)
        except ValueError:
            return
        if self.kind == "hourangle":  # uncertainty in seconds of time (parameter.py AngleParameter)
            u = u / 3600.0
        elif self.kind == "degangle" and self.name in ("DECJ",):
            u = u / 3600.0
        if self.scale is not None and abs(u) > abs(self.scale[1]):
            u *= self.scale[0]
        self.uncertainty_value = u

    @property
    def quantity(self):
        return self.value

    @property
    def uncertainty(self):
        return self.uncertainty_value

    @uncertainty.setter
    def uncertainty(self, v):
        self.uncertainty_value = None if v is None else float(v)

    def __repr__(self):
        return f"{self.name} ({self.units}) {self.value} frozen={self.frozen}"


# ---- parameter definitions -----------------------------------------------------------
# name -> (component, kind, units, long_double, scale)
_DEFS = {
    # top level
    "PSR": ("", "str", "", False, None), "EPHEM": ("", "str", "", False, None),
    "CLOCK": ("", "str", "", False, None), "CLK": ("", "str", "", False, None),
    "UNITS": ("", "str", "", False, None), "START": ("", "mjd", "d", True, None),
    "FINISH": ("", "mjd", "d", True, None), "TRACK": ("", "str", "", False, None),
    "BINARY": ("", "str", "", False, None), "NTOA": ("", "int", "", False, None),
    "CHI2": ("", "float", "", False, None), "CHI2R": ("", "float", "", False, None),
    "TRES": ("", "float", "us", False, None), "DMDATA": ("", "bool", "", False, None),
    "DMRES": ("", "float", "pc / cm3", False, None),
    "INFO": ("", "str", "", False, None), "TIMEEPH": ("", "str", "", False, None),
    "T2CMETHOD": ("", "str", "", False, None), "DILATEFREQ": ("", "bool", "", False, None),
    "TZRMJD": ("AbsPhase", "mjd", "d", True, None), "TZRSITE": ("AbsPhase", "str", "", False, None),
    "TZRFRQ": ("AbsPhase", "float", "MHz", False, None),
    # astrometry (astrometry.py)
    "POSEPOCH": ("Astrometry", "mjd", "d", True, None), "PX": ("Astrometry", "float", "mas", False, None),
    "PHOFF": ("PhaseOffset", "float", "", False, None),
    "RAJ": ("AstrometryEquatorial", "hourangle", "hourangle", False, None),
    "DECJ": ("AstrometryEquatorial", "degangle", "deg", False, None),
    "PMRA": ("AstrometryEquatorial", "float", "mas / yr", False, None),
    "PMDEC": ("AstrometryEquatorial", "float", "mas / yr", False, None),
    "ELONG": ("AstrometryEcliptic", "degangle", "deg", False, None),
    "ELAT": ("AstrometryEcliptic", "degangle", "deg", False, None),
    "PMELONG": ("AstrometryEcliptic", "float", "mas / yr", False, None),
    "PMELAT": ("AstrometryEcliptic", "float", "mas / yr", False, None),
    "ECL": ("AstrometryEcliptic", "str", "", False, None),
    # spindown (spindown.py)
    "PEPOCH": ("Spindown", "mjd", "d", True, None),
    # dispersion (dispersion_model.py)
    "DM": ("DispersionDM", "float", "pc / cm3", True, None),
    "DMEPOCH": ("DispersionDM", "mjd", "d", True, None),
    "DMX": ("DispersionDMX", "float", "pc / cm3", False, None),
    # solar system / misc zero components
    "PLANET_SHAPIRO": ("SolarSystemShapiro", "bool", "", False, None),
    "CORRECT_TROPOSPHERE": ("TroposphereDelay", "bool", "", False, None),
    "NE_SW": ("SolarWindDispersion", "float", "1 / cm3", False, None),
    "SWM": ("SolarWindDispersion", "int", "", False, None),
    # binaries (pulsar_binary.py, binary_ell1.py, binary_dd.py)
    "PB": ("Binary", "float", "d", True, None),
    "PBDOT": ("Binary", "float", "", False, (1e-12, 1e-7)),
    "XPBDOT": ("Binary", "float", "", False, (1e-12, 1e-7)),
    "A1": ("Binary", "float", "ls", False, None),
    "A1DOT": ("Binary", "float", "ls / s", False, (1e-12, 1e-7)),
    "ECC": ("Binary", "float", "", False, None),
    "EDOT": ("Binary", "float", "1 / s", False, (1e-12, 1e-7)),
    "T0": ("Binary", "mjd", "d", True, None),
    "OM": ("Binary", "float", "deg", True, None),
    "OMDOT": ("Binary", "float", "deg / yr", True, None),
    "M2": ("Binary", "float", "solMass", False, None),
    # ELL1H (binary_ell1.py:345-378): H3/H4 (s) and STIGMA longdouble, NHARMS an int
    "H3": ("Binary", "float", "s", True, None), "H4": ("Binary", "float", "s", True, None),
    "STIGMA": ("Binary", "float", "", True, None), "NHARMS": ("Binary", "int", "", False, None),
    "SINI": ("Binary", "float", "", False, None),
    "GAMMA": ("Binary", "float", "s", False, None),
    "DR": ("Binary", "float", "", False, None), "DTH": ("Binary", "float", "", False, None),
    # DDK (binary_ddk.py:120-145): inclination and node longitude (deg), the K96 flag
    "KIN": ("Binary", "float", "deg", False, None), "KOM": ("Binary", "float", "deg", False, None),
    "K96": ("Binary", "bool", "", False, None),
    "A0": ("Binary", "float", "s", False, None), "B0": ("Binary", "float", "s", False, None),
    "TASC": ("Binary", "mjd", "d", True, None),
    "EPS1": ("Binary", "float", "", True, None), "EPS2": ("Binary", "float", "", True, None),
    "EPS1DOT": ("Binary", "float", "1e-12 / s", True, None),
    "EPS2DOT": ("Binary", "float", "1e-12 / s", True, None),
    # red noise (noise_model.py:679-805)
    "TNREDAMP": ("PLRedNoise", "float", "", False, None), "TNREDGAM": ("PLRedNoise", "float", "", False, None),
    "TNREDC": ("PLRedNoise", "float", "", False, None), "RNAMP": ("PLRedNoise", "float", "", False, None),
    "RNIDX": ("PLRedNoise", "float", "", False, None),
    "TNDMAMP": ("PLDMNoise", "float", "", False, None), "TNDMGAM": ("PLDMNoise", "float", "", False, None),
    "TNDMC": ("PLDMNoise", "float", "", False, None),
}

_ALIASES = {
    "RA": "RAJ", "DEC": "DECJ", "LAMBDA": "ELONG", "BETA": "ELAT", "PMLAMBDA": "PMELONG",
    "PMBETA": "PMELAT", "E": "ECC", "ECCDOT": "EDOT", "XDOT": "A1DOT", "T2EFAC": "EFAC",
    "T2EQUAD": "EQUAD", "TNECORR": "ECORR", "SOLARN0": "NE_SW", "CLK": "CLOCK", "PSRJ": "PSR", "PSRB": "PSR", "VARSIGMA": "STIGMA", "STIG": "STIGMA",
}

_PREFIX = {  # prefix params: regex -> (component, units template, long_double)
    r"^F(\d+)$": ("Spindown", "Hz / s^{n}", True),
    r"^DM(\d+)$": ("DispersionDM", "pc / (cm3 yr^{n})", True),
    r"^DMX_(\d+)$": ("DispersionDMX", "pc / cm3", False),
    r"^DMXR1_(\d+)$": ("DispersionDMX", "d", True),
    r"^DMXR2_(\d+)$": ("DispersionDMX", "d", True),
    r"^FD(\d+)$": ("FD", "s", False),
}

MASK_PARAMS = {"JUMP": ("PhaseJump", "s"), "EFAC": ("ScaleToaError", ""),
               "EQUAD": ("ScaleToaError", "us"), "TNEQ": ("ScaleToaError", "log10(s)"),
               "ECORR": ("EcorrNoise", "us"),
               # wideband DM data (dispersion_model.py:724 DispersionJump; noise_model.py:228
               # ScaleDmError): DM offsets and DM-error scaling, pc/cm^3
               "DMJUMP": ("DispersionJump", "pc / cm3"), "DMEFAC": ("ScaleDmError", ""),
               "DMEQUAD": ("ScaleDmError", "pc / cm3")}

IGNORED = {"MODE", "NITS", "IBOOT", "RM", "SWP", "DMXEP", "DMXF1", "DMXF2"}


def make_param(name: str) -> Optional[Param]:
    if name in _DEFS:
        comp, kind, units, ld, scale = _DEFS[name]
        return Param(name=name, kind=kind, units=units, long_double=ld, scale=scale, component=comp)
    for rx, (comp, units, ld) in _PREFIX.items():
        m = re.match(rx, name)
        if m:
            idx = int(m.group(1))
            kind = "mjd" if name.startswith("DMXR") else "float"
            u = units.replace("{n}", str(idx))
            if name == "F0":
                u = "Hz"
            if name.startswith("DM") and not name.startswith("DMX") and idx == 0:
                return None
            return Param(name=name, kind=kind, units=u, long_double=ld, component=comp, index=idx)
    return None


@dataclass
class ParLine:
    name: str
    fields: List[str]


def read_parfile(path_or_text) -> List[ParLine]:
    """Tokenise a par file (model_builder.py:102-250 parse semantics: '#' / 'C ' comments)."""
    if hasattr(path_or_text, "read"):
        text = path_or_text.read()
    elif "\n" in str(path_or_text):
        text = str(path_or_text)
    else:
        with open(path_or_text) as f:
            text = f.read()
    out = []
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#") or line.startswith("C ") or line == "C":
            continue
        toks = line.split()
        out.append(ParLine(toks[0].upper() if not toks[0].startswith("TN") else toks[0].upper(), toks[1:]))
    return out
