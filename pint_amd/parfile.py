"""Par-file writer: ``TimingModel.as_parfile`` / ``write_parfile`` (reference
``timing_model.py:2747-2862``) for the models this path holds.

Each line follows the reference's per-parameter format (``parameter.py:441-522``
``as_parfile_line``):

* ``"%-15s %25s" % (name, value)``, then ``" %d %s" % (fit flag, uncertainty)`` when an
  uncertainty is set, else ``" 1"`` for a free parameter;
* mask parameters (``parameter.py:2039``): ``"%-15s %s " % (name, key)``, the key values
  each followed by a space, ``"%25s" % value`` and the same suffix;
* values: ``str()`` of the float64 or longdouble value (``parameter.py:805``); booleans
  ``Y``/``N``; MJDs as ``imjd`` + the day fraction to 16 decimals (``pulsar_mjd.py:506``
  ``_mjds_to_str`` over astropy's exact ``day_frac``); TZRMJD (UTC) through the
  nanosecond time of day as ``pulsar_mjd_string`` does (``pulsar_mjd.py:399-421``);
  RAJ/DECJ sexagesimal to 8 decimals of seconds, ELONG/ELAT decimal to 15 places
  (``parameter.py:1382-1398``, astropy ``hours_to_string`` / ``degrees_to_string``);
* names as the par file spelled them (``use_alias``: LAMBDA, E, T2EFAC, ...).

Order: the top-level parameters, astrometry, spindown, then the other components in the
order the reference most often prints them (``timing_model.py:2789-2823``: its middle
categories follow its component-type insertion order, a set iteration in ``model_builder``,
so the reference itself does not fix it), each component's parameters in the reference
component's own order.

Defaults the reference's components carry but this path does not model (SOLARN0, SWM,
CORRECT_TROPOSPHERE, PLANET_SHAPIRO N, DILATEFREQ, TIMEEPH, T2CMETHOD, ...) are not
written; reading the file back with the reference gives them their default values, the
same values the reference would have written.
"""
from __future__ import annotations

import math
from typing import Iterable, List, Tuple

import numpy as np

from .parameter import LD, Param

DJM0 = 2400000.5
UTC_MJD_PARAMS = {"TZRMJD"}  # + DMXR1_/DMXR2_ (dispersion_model.py:411-428)
TOP_LEVEL = ["PSR", "EPHEM", "CLOCK", "CLK", "UNITS", "START", "FINISH", "INFO", "TIMEEPH", "T2CMETHOD", "TRACK",
             "DILATEFREQ", "DMDATA", "NTOA", "CHI2", "CHI2R", "TRES", "DMRES"]


# ---- exact float64 day + fraction (astropy time.utils.day_frac / two_sum, restated) ----
def two_sum(a: float, b: float) -> Tuple[float, float]:
    x = a + b
    eb = x - a
    ea = x - eb
    eb = b - eb
    ea = a - ea
    return x, ea + eb


def day_frac(v1: float, v2: float) -> Tuple[float, float]:
    s, e = two_sum(float(v1), float(v2))
    day = float(np.round(s))
    extra, frac = two_sum(s, -day)
    frac += extra + e
    excess = float(np.round(frac))
    day += excess
    extra, frac = two_sum(s, -day)
    frac += extra + e
    return day, frac


def str_to_mjds(s: str) -> Tuple[float, float]:
    """pulsar_mjd.py:455 _str_to_mjds for plain decimal strings: integer day + float64
    fraction, through day_frac."""
    ss = s.lower().strip().replace("d", "e")
    if "e" in ss:
        v = np.longdouble(ss)
        i = float(np.floor(v))
        return day_frac(i, float(v - LD(i)))
    parts = ss.split(".")
    if len(parts) == 1:
        parts.append("0")
    imjd = int(parts[0])
    fmjd = float(f"0.{parts[1]}")
    if ss.startswith("-"):
        fmjd = -fmjd
    return day_frac(imjd, fmjd)


def _mjds_to_str(d: float, f: float) -> str:
    imjd, fmjd = day_frac(d, f)
    imjd = int(imjd)
    while fmjd < 0.0:
        imjd -= 1
        fmjd += 1.0
    return str(imjd) + "{:.16f}".format(fmjd)[1:]


def _pair_from_ld(v) -> Tuple[float, float]:
    """time_from_longdouble (pulsar_mjd.py:262): i = floor(t), f = float(t - i)."""
    t = LD(v)
    i = float(np.floor(t))
    return i, float(t - LD(i))


def _utc_roundtrip(d: float, f: float) -> Tuple[float, float]:
    """pulsar_mjd.py:399-445: UTC MJD -> calendar day + h/m/s (86400-s day) -> jd pair ->
    erfa d2dtf to 9 digits of seconds -> h/24 + m/1440 + s/86400 + ns/86400e9."""
    v1, v2 = day_frac(d, f)
    imjd = v1
    frac = v2
    if frac < 0:
        imjd -= 1.0
        frac += 1.0
    x = frac * 24
    h = math.floor(x)
    x = (x - h) * 60
    m = math.floor(x)
    s = (x - m) * 60
    ns = int(round((h * 3600 + m * 60 + s) * 1e9))
    h2, r = divmod(ns, 3600 * 10 ** 9)
    m2, r = divmod(r, 60 * 10 ** 9)
    s2, f2 = divmod(r, 10 ** 9)
    fr = h2 / 24.0 + m2 / 1440.0 + s2 / 86400.0 + f2 / 86400.0 / 10 ** 9
    return day_frac(imjd, fr)


def mjd_string(p: Param) -> str:
    """The value as the reference's Time would print it: the (day, fraction) pair the par
    file gave (or time_from_longdouble's pair after a change), stored by astropy as
    (jd1, jd2) = day_frac(day + DJM0, frac) and read back through day_frac(jd1 - DJM0, jd2)
    (pulsar_mjd.py:386-394) -- each step re-rounds the float64 fraction, which is what puts
    the last of the 16 decimals where the reference puts it."""
    pair = getattr(p, "mjd_pair", None)
    if pair is None or LD(pair[0]) + LD(pair[1]) != LD(p.value):
        pair = _pair_from_ld(p.value)
    if p.name in UTC_MJD_PARAMS or p.name.startswith(("DMXR1_", "DMXR2_")):  # time_scale utc
        return _mjds_to_str(*_utc_roundtrip(*pair))
    jd1, jd2 = day_frac(pair[0] + DJM0, pair[1])
    return _mjds_to_str(*day_frac(jd1 - DJM0, jd2))


# ---- angles (astropy angle_formats.hours_to_string / degrees_to_string, restated) -------
def _sexagesimal(x: float, precision: int = 8) -> str:
    sign = math.copysign(1.0, x)
    a = abs(x)
    hf, h = math.modf(a)
    mf, m = math.modf(hf * 60.0)
    s = mf * 60.0
    h, m, s = math.floor(sign * h), sign * math.floor(m), sign * s
    vals = [abs(h), abs(m), abs(s)]
    if vals[2] >= 60.0 - 10.0 ** -precision:
        vals[2] = 0.0
        vals[1] += 1.0
    if vals[1] >= 60.0:
        vals[1] = 0.0
        vals[0] += 1.0
    last = "{0:.{p}f}".format(vals[2], p=precision)
    if len(last) == 1 or last[1] == ".":
        last = "0" + last
    return "{0:0{pad}.0f}:{1:02d}:{2}".format(math.copysign(vals[0], sign), int(vals[1]), last, pad=0)


def value_string(p: Param) -> str:
    v = p.value
    if p.kind == "str":
        return str(v)
    if p.kind == "bool":
        return "Y" if v else "N"
    if p.kind == "int":
        return str(int(v))
    if p.kind == "mjd":
        return mjd_string(p)
    if p.kind == "hourangle":
        return _sexagesimal(float(v))
    if p.kind == "degangle":
        if p.name == "DECJ":
            return _sexagesimal(float(v))
        return "{0:0.15f}".format(float(v))
    if p.long_double:
        return str(LD(v))
    return str(float(v))


def uncertainty_string(p: Param) -> str:
    u = p.uncertainty_value
    if p.kind == "hourangle":  # arcsec / 15: seconds of time (parameter.py:1389-1398)
        return "{0:0.20f}".format(float(u) * 3600.0)
    if p.kind == "degangle":
        return "{0:0.20f}".format(float(u) * (3600.0 if p.name == "DECJ" else 1.0))
    if p.long_double:
        return str(LD(u))
    return str(float(u))


def _display_name(p: Param) -> str:
    return getattr(p, "alias", None) or (p.name.rstrip("0123456789") if p.kind == "mask" else p.name)


def parfile_line(p: Param) -> str:
    """The reference's as_parfile_line (parameter.py:441, :2039) for one parameter; "" when
    unset."""
    if p.value is None:
        return ""
    if getattr(p, "implicit", False) and p.frozen and p.value == 0:
        return ""  # a default the reference leaves unset (None): not written
    name = _display_name(p)
    if p.kind == "mask":
        line = "%-15s %s " % (name, p.key)
        kl = p.key.lower()
        for kv in p.key_value:
            # parameter.py:1864-1869 key_identifier: mjd/freq keys are floats (MHz), tel the
            # canonical site name
            if kl in ("mjd", "freq"):
                kv = str(float(kv))
            elif kl == "tel":
                from .observatory import get_observatory_name
                kv = get_observatory_name(kv)
            line += f"{kv} "
        line += "%25s" % value_string(p)
    else:
        line = "%-15s %25s" % (name, value_string(p))
    if p.uncertainty_value is not None:
        line += " %d %s" % (0 if p.frozen else 1, uncertainty_string(p))
    elif not p.frozen:
        line += " 1"
    return line + "\n"


# within-component orders of the reference's components (their add_param order)
_ORDER = {
    "astrometry_eq": ["RAJ", "DECJ", "PMRA", "PMDEC", "PX", "POSEPOCH"],
    "astrometry_ecl": ["ELONG", "ELAT", "PMELONG", "PMELAT", "PX", "ECL", "POSEPOCH"],
    "AbsPhase": ["TZRMJD", "TZRSITE", "TZRFRQ"],
    "SolarWindDispersion": ["NE_SW", "SWM"],
    "DD": ["PB", "PBDOT", "A1", "A1DOT", "ECC", "EDOT", "T0", "OM", "OMDOT", "M2", "SINI", "A0", "B0", "GAMMA",
           "DR", "DTH"],
    "ELL1": ["PB", "PBDOT", "A1", "A1DOT", "M2", "SINI", "TASC", "EPS1", "EPS2", "EPS1DOT", "EPS2DOT"],
    "DDK": ["PB", "PBDOT", "A1", "A1DOT", "ECC", "EDOT", "T0", "OM", "OMDOT", "M2", "A0", "B0", "GAMMA",
            "DR", "DTH", "KIN", "KOM", "K96"],
    "BT": ["PB", "PBDOT", "A1", "A1DOT", "ECC", "EDOT", "T0", "OM", "OMDOT", "GAMMA"],
    "ELL1H": ["PB", "PBDOT", "A1", "A1DOT", "TASC", "EPS1", "EPS2", "EPS1DOT", "EPS2DOT", "H3", "H4", "STIGMA",
              "NHARMS"],
    "PLRedNoise": ["RNAMP", "RNIDX", "TNREDAMP", "TNREDGAM", "TNREDC"],
    "PLDMNoise": ["TNDMAMP", "TNDMGAM", "TNDMC"],
}
MIDDLE = ["TroposphereDelay", "SolarSystemShapiro", "SolarWindDispersion", "DispersionDM", "DispersionDMX",
          "Binary", "FD", "AbsPhase", "PhaseOffset", "PhaseJump", "EcorrNoise", "ScaleToaError", "PLRedNoise",
          "PLDMNoise"]


def _by_index(names, prefix):
    return sorted([n for n in names if n.startswith(prefix) and n[len(prefix):].isdigit()],
                  key=lambda n: int(n[len(prefix):]))


def _component_params(model, comp: str) -> List[str]:
    P = model._params
    names = [n for n, p in P.items() if (p.component or "TimingModel") == comp]
    if comp == "Spindown":
        return _by_index(names, "F") + [n for n in names if not (n[1:].isdigit() and n.startswith("F"))]
    if comp == "DispersionDM":
        return [n for n in ["DM"] if n in names] + _by_index(names, "DM") + \
            [n for n in names if n != "DM" and not (n.startswith("DM") and n[2:].isdigit())]
    if comp == "DispersionDMX":  # DMX, then DMX_i, DMXR1_i, DMXR2_i per bin (dispersion_model.py)
        head = [n for n in names if n == "DMX"]
        idx = sorted({int(n.split("_")[1]) for n in names if "_" in n})
        body = [f"{pre}{i:04d}" for i in idx for pre in ("DMX_", "DMXR1_", "DMXR2_") if f"{pre}{i:04d}" in P]
        return head + body + [n for n in names if n not in head and n not in body]
    if comp == "Binary":
        order = _ORDER.get(model.binary or "", [])
        return [n for n in order if n in names] + [n for n in names if n not in order]
    if comp == "ScaleToaError":  # EFAC1, EQUAD1 exist with the component, the rest are added
        ef, eq = _by_index(names, "EFAC"), _by_index(names, "EQUAD")
        head = [n for n in ("EFAC1", "EQUAD1") if n in names]
        return head + [n for n in ef if n not in head] + [n for n in eq if n not in head]
    if comp in _ORDER:
        return [n for n in _ORDER[comp] if n in names] + [n for n in names if n not in _ORDER[comp]]
    return names


def _astrometry_params(model) -> List[str]:
    P = model._params
    names = [n for n, p in P.items() if p.component.startswith("Astrometry")]
    order = _ORDER["astrometry_ecl" if "AstrometryEcliptic" in model.components else "astrometry_eq"]
    return [n for n in order if n in names] + [n for n in names if n not in order]


def _ell1_comments(model) -> str:
    """ELL1's derived ECC and OM (binary_ell1.py:25-33 _eps_to_e / _eps_to_om, funcParameter
    lines written commented out, parameter.py:2593-2598)."""
    if model.binary not in ("ELL1", "ELL1H") or "EPS1" not in model or "EPS2" not in model:
        return ""
    e1, e2 = model["EPS1"].value, model["EPS2"].value
    if e1 is None or e2 is None:
        return ""
    a, b = LD(e1), LD(e2)
    ecc = np.sqrt(a ** 2 + b ** 2)
    om = np.arctan2(a, b)
    if om < 0:
        om = om + LD(360 * math.pi / 180)
    om = om * LD(180 / math.pi)
    return "# " + "%-15s %25s" % ("ECC", str(ecc)) + "\n" + "# " + "%-15s %25s" % ("OM", str(om)) + "\n"


def _ddk_comments(model) -> str:
    """DDK's funcParameters KINIAU = 180 deg - KIN, KOMIAU = 90 deg - KOM and SINI = sin(KIN)
    (binary_ddk.py:14-41, :148-174), written commented out like ELL1's."""
    if model.binary != "DDK" or model["KIN"].value is None or model["KOM"].value is None:
        return ""
    kin, kom = float(model["KIN"].value), float(model["KOM"].value)
    out = ""
    for n, v in (("KINIAU", 180.0 - kin), ("KOMIAU", 90.0 - kom), ("SINI", np.sin(kin * (math.pi / 180)))):
        out += "# " + "%-15s %25s" % (n, str(v)) + "\n"
    return out


def ordered_params(model) -> List[str]:
    top = [n for n in TOP_LEVEL if n in model._params and model[n].component in ("", "TimingModel")]
    top += [n for n, p in model._params.items() if p.component in ("", "TimingModel") and n not in top
            and n != "BINARY"]
    out = list(top) + _astrometry_params(model) + _component_params(model, "Spindown")
    comps = list(MIDDLE)
    comps += [c for c in dict.fromkeys(p.component for p in model._params.values())
              if c and c not in comps and c != "TimingModel" and not c.startswith("Astrometry")
              and c != "Spindown"]
    for c in comps:
        ns = _component_params(model, c)
        if c == "Binary" and ns and "BINARY" in model._params:
            ns = ["BINARY"] + ns
        out += [n for n in ns if n not in out]
    return out


def as_parfile(model, include_info: bool = True, comment: str = None) -> str:
    """TimingModel.as_parfile (timing_model.py:2747), format "pint"."""
    head = ""
    if include_info:
        head = "# Created by pint_amd (MI355X fit-and-residual path)\n"
        if comment:
            head += "".join(f"# {c}\n" for c in str(comment).splitlines())
        head += "# Format: pint\n"
    body = ""
    names = ordered_params(model)
    # ELL1's ECC/OM comment lines follow the ELL1 parameters (ELL1H's own come after them)
    h_own = ("H3", "H4", "STIGMA", "NHARMS") if model.binary == "ELL1H" else ()
    last_bin = max((i for i, n in enumerate(names) if model[n].component == "Binary" and n not in h_own
                    and (model[n].value is not None or n == "BINARY")), default=None)
    for i, n in enumerate(names):
        body += parfile_line(model[n])
        if i == last_bin:
            body += _ell1_comments(model) + _ddk_comments(model)
    return head + body


def write_parfile(model, filename, include_info: bool = True, comment: str = None):
    """TimingModel.write_parfile (timing_model.py:2823)."""
    text = as_parfile(model, include_info=include_info, comment=comment)
    if hasattr(filename, "write"):
        filename.write(text)
    else:
        with open(filename, "w") as f:
            f.write(text)
