"""TimingModel host mirror: par file -> components/parameters -> device spec + table.

Reference API kept: ``get_model`` (model_builder.py:777), ``TimingModel`` attribute access
to parameters (``model.F0.value``), ``params``/``free_params`` (timing_model.py:614/655),
``components``, ``has_correlated_errors``, ``designmatrix`` (:2073), ``delay`` (:1515),
``phase`` (:1548), ``scaled_toa_uncertainty`` (:1644), ``noise_model_designmatrix`` /
``noise_model_basis_weight`` (:1704-1716).  Evaluation runs on the GPU through
``pint_amd.engine``; this module only builds the structure and parameter tables.
"""
from __future__ import annotations

import copy
import re
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np

from . import parameter as P
from .parameter import LD, Param

# components supported on the hot path
DELAY_ORDER = ["AstrometryEquatorial", "AstrometryEcliptic", "TroposphereDelay", "SolarSystemShapiro",
               "SolarWindDispersion", "DispersionDM", "DispersionDMX", "BinaryELL1", "BinaryDD", "FD"]
PHASE_ORDER = ["AbsPhase", "Spindown", "PhaseOffset", "PhaseJump"]
NOISE = ["ScaleToaError", "EcorrNoise", "PLRedNoise", "PLDMNoise"]

ELL1_PARAMS = ["PB", "PBDOT", "A1", "A1DOT", "EDOT", "OMDOT", "M2", "SINI", "TASC", "EPS1", "EPS2",
               "EPS1DOT", "EPS2DOT"]
DD_PARAMS = ["PB", "PBDOT", "A1", "A1DOT", "ECC", "EDOT", "T0", "OM", "OMDOT", "M2", "SINI", "A0", "B0",
             "GAMMA", "DR", "DTH"]
DDK_PARAMS = [n for n in DD_PARAMS if n != "SINI"] + ["KIN", "KOM"]  # binary_ddk.py:120-145
BT_PARAMS = ["PB", "PBDOT", "A1", "A1DOT", "ECC", "EDOT", "T0", "OM", "OMDOT", "GAMMA"]
BIN_IDS = {"PB": 0, "PBDOT": 1, "XPBDOT": 2, "A1": 3, "A1DOT": 4, "ECC": 5, "EDOT": 6, "T0": 7, "OM": 8,
           "OMDOT": 9, "M2": 10, "SINI": 11, "GAMMA": 12, "DR": 13, "DTH": 14, "A0": 15, "B0": 16,
           "TASC": 17, "EPS1": 18, "EPS2": 19, "EPS1DOT": 20, "EPS2DOT": 21, "H3": 22, "H4": 23, "STIGMA": 24,
           "KIN": 25, "KOM": 26}
# obliquity values (rad) from the reference's runtime ecliptic.dat (pulsar_ecliptic.py:29)
OBLIQUITY = {"IERS2010": 0.4090926006005829, "IERS2003": 0.40909260011576914,
             "DEFAULT": 84381.406 / 206264.80624709636}


class MissingParameter(ValueError):
    pass


class TimingModelError(ValueError):
    """timing_model.py TimingModelError (an invalid model structure)."""


class TimingModel:
    """Host-side model: ordered parameters grouped by component."""

    def __init__(self, name: str = ""):
        object.__setattr__(self, "_params", OrderedDict())
        self.name = name
        self.components: "OrderedDict[str, list]" = OrderedDict()
        self.binary: Optional[str] = None

    # -- parameter access -------------------------------------------------------------
    def __getattr__(self, name):
        params = object.__getattribute__(self, "_params")
        if name in params:
            return params[name]
        raise AttributeError(name)

    def __getitem__(self, name):
        return self._params[name]

    def __contains__(self, name):
        return name in self._params

    def add_param(self, p: Param):
        self._params[p.name] = p
        self.components.setdefault(p.component or "TimingModel", []).append(p.name)
        object.__setattr__(self, "_order", None)
        object.__setattr__(self, "_names", {})

    @property
    def params(self) -> List[str]:
        """Parameter order: top level, astrometry, spindown, remaining components
        (timing_model.py:614-652).  Cached until the next add_param (the fitters ask for
        it, and for free_params, several times per fit)."""
        cached = self.__dict__.get("_order")
        if cached is not None and cached[0] == len(self._params):
            return list(cached[1])
        order = self._params_order()
        object.__setattr__(self, "_order", (len(self._params), tuple(order)))
        return order

    def _params_order(self) -> List[str]:
        # one stable sort by group rank (dict order within a group): top level, astrometry,
        # spindown, the delay/phase/noise components in order, the rest
        order = [("Binary" if c.startswith("Binary") else c) for c in DELAY_ORDER]
        rest = {}
        for comp in dict.fromkeys(order + ["AbsPhase", "PhaseJump"] + NOISE):
            if not comp.startswith("Astrometry"):
                rest.setdefault(comp, 3 + len(rest))
        big = 3 + len(rest)

        def rank(c):
            if c in ("", "TimingModel"):
                return 0
            if c.startswith("Astrometry"):
                return 1
            if c == "Spindown":
                return 2
            return rest.get(c, big)
        ranks = {c: rank(c) for c in {p.component for p in self._params.values()}}
        return sorted(self._params, key=lambda n: ranks[self._params[n].component])

    def as_parfile(self, include_info: bool = True, comment: str = None) -> str:
        """The model as par-file text (timing_model.py:2747 as_parfile, format "pint")."""
        from .parfile import as_parfile
        return as_parfile(self, include_info=include_info, comment=comment)

    def write_parfile(self, filename, include_info: bool = True, comment: str = None):
        """timing_model.py:2823 write_parfile."""
        from .parfile import write_parfile
        write_parfile(self, filename, include_info=include_info, comment=comment)

    @property
    def free_params(self) -> List[str]:
        return [p for p in self.params if not self._params[p].frozen]

    @free_params.setter
    def free_params(self, names):
        want = set(names)
        for n, p in self._params.items():
            p.frozen = n not in want
            want.discard(n)
        if want:
            raise ValueError(f"Parameter(s) not in the model: {sorted(want)}")

    def get_params_dict(self, which="free", kind="value"):
        names = self.free_params if which == "free" else self.params
        return OrderedDict((n, self._params[n].value) for n in names)

    # -- component queries ------------------------------------------------------------
    @property
    def component_names(self) -> List[str]:
        return [c for c in DELAY_ORDER + PHASE_ORDER + NOISE if c in self.components]

    @property
    def has_correlated_errors(self) -> bool:
        return any(c in self.components for c in ("PLRedNoise", "PLDMNoise", "EcorrNoise"))

    @property
    def has_time_correlated_errors(self) -> bool:
        return "PLRedNoise" in self.components or "PLDMNoise" in self.components

    @property
    def astrometry_kind(self) -> int:
        if "AstrometryEquatorial" in self.components:
            return 1
        if "AstrometryEcliptic" in self.components:
            return 2
        return 0

    def _names_of(self, key, build):
        """Name lists derived from the parameter set alone, cached until the next add_param
        (parameters are never removed): build_layout / validate ask for them many times per
        upload, and a regex pass over ~250 parameters each time dominated the host layout."""
        cache = self.__dict__.get("_names")
        if cache is None or cache.get("_n") != len(self._params):  # (a shallow copy shares _params)
            cache = {"_n": len(self._params)}
            object.__setattr__(self, "_names", cache)
        hit = cache.get(key)
        if hit is None:
            hit = cache[key] = tuple(build())
        return list(hit)

    def prefix_list(self, prefix_rx: str) -> List[str]:
        def build():
            rx = re.compile(prefix_rx)
            out = []
            for n in self._params:
                m = rx.match(n)
                if m:
                    out.append((int(m.group(1)), n))
            return [n for _, n in sorted(out)]
        return self._names_of(("prefix", prefix_rx), build)

    def spin_terms(self) -> List[str]:
        return self.prefix_list(r"^F(\d+)$")

    def dm_terms(self) -> List[str]:
        return ["DM"] + self.prefix_list(r"^DM(\d+)$") if "DM" in self._params else []

    def dmx_params(self) -> List[str]:
        return self.prefix_list(r"^DMX_(\d+)$")

    def fd_terms(self) -> List[str]:
        return self.prefix_list(r"^FD(\d+)$")

    def mask_params(self, base: str) -> List[str]:
        def build():
            rx = re.compile(rf"^{base}\d+$")
            return [n for n, p in self._params.items() if p.kind == "mask" and rx.match(n)]
        return self._names_of(("mask", base), build)

    # -- validation (the parts of Component.validate that matter on the hot path) -----
    def validate(self):
        for n in self.spin_terms():
            if self._params[n].value is None:
                raise MissingParameter(n)
        if "F0" not in self._params:
            raise MissingParameter("Spindown requires F0")
        if self.PEPOCH.value is None:
            raise MissingParameter("PEPOCH is required (spindown.py:104)")
        if self.astrometry_kind:
            pml = "PMRA" if self.astrometry_kind == 1 else "PMELONG"
            pmb = "PMDEC" if self.astrometry_kind == 1 else "PMELAT"
            if (self[pml].value or self[pmb].value) and self.POSEPOCH.value is None:
                self.POSEPOCH.value = LD(self.PEPOCH.value)  # astrometry.py:339-349
        if "DispersionDM" in self.components:
            if len(self.dm_terms()) > 1 and any(self[n].value for n in self.dm_terms()[1:]):
                if self.DMEPOCH.value is None:
                    self.DMEPOCH.value = LD(self.PEPOCH.value)  # dispersion_model.py:197
        if "NE_SW" in self and self.NE_SW.value:
            raise NotImplementedError("solar-wind dispersion (NE_SW != 0) is outside the supported hot path")
        if "CORRECT_TROPOSPHERE" in self and self.CORRECT_TROPOSPHERE.value:
            raise NotImplementedError("troposphere delay is outside the supported hot path")
        if self.binary in ("DD", "BT", "DDK"):
            e = float(self.ECC.value or 0.0)
            if not (0 <= e < 1):
                raise ValueError("Eccentricity should be in the range of [0,1).")
        if self.binary == "DDK":  # BinaryDDK.validate (binary_ddk.py:200-231)
            if not self.astrometry_kind:
                raise TimingModelError("No valid AstrometryEcliptic or AstrometryEquatorial component found")
            if "PX" not in self or self.PX.value is None or self.PX.value <= 0.0:
                raise TimingModelError("DDK model needs a valid `PX` value.")

    # -- noise ------------------------------------------------------------------------
    def red_noise_params(self):
        """(amp, gamma, nmodes) — noise_model.py:761-768 get_pl_vals."""
        nf = int(self.TNREDC.value) if "TNREDC" in self and self.TNREDC.value is not None else 30
        if "TNREDAMP" in self and self.TNREDAMP.value is not None and self.TNREDGAM.value is not None:
            return 10.0 ** float(self.TNREDAMP.value), float(self.TNREDGAM.value), nf
        fac = (86400.0 * 365.24 * 1e6) / (2.0 * np.pi * np.sqrt(3.0))
        return float(self.RNAMP.value) / fac, -1.0 * float(self.RNIDX.value), nf

    def dm_noise_params(self):
        """(amp, gamma, nmodes) of PLDMNoise (noise_model.py:508-511 get_pl_vals)."""
        nf = int(self.TNDMC.value) if "TNDMC" in self and self.TNDMC.value is not None else 30
        return 10.0 ** float(self.TNDMAMP.value), float(self.TNDMGAM.value), nf

    def find_empty_masks(self, toas, freeze=False):
        """Free mask/DMX parameters that select no TOAs (timing_model.py:2895)."""
        bad = []
        for n in self.free_params:
            p = self[n]
            if p.kind == "mask" and len(toas.select_mask(p.key, p.key_value)) == 0:
                bad.append(n)
        mj = toas.get_mjds()
        for n in self.dmx_params():
            tag = n.split("_")[1]
            r1, r2 = float(self["DMXR1_" + tag].value), float(self["DMXR2_" + tag].value)
            if not np.any((mj >= r1) & (mj <= r2)):
                bad.append(n)
        if freeze:
            for n in bad:
                self[n].frozen = True
        return bad

    def copy(self):
        return copy.deepcopy(self)

    # -- device-side evaluation (delegated to the GPU engine) ---------------------------
    def designmatrix(self, toas, incfrozen=False, incoffset=True):
        from .engine import evaluate_designmatrix
        return evaluate_designmatrix(self, toas)

    def delay(self, toas):
        from .engine import evaluate_delay_phase
        return evaluate_delay_phase(self, toas)["delay"]

    def phase(self, toas, abs_phase=True):
        from .engine import evaluate_delay_phase
        return evaluate_delay_phase(self, toas)["phase"]

    def scaled_toa_uncertainty(self, toas):
        from .noise import scaled_sigma_us
        return scaled_sigma_us(self, toas)

    def noise_model_designmatrix(self, toas):
        from .noise import noise_basis
        return noise_basis(self, toas)[0]

    def noise_model_basis_weight(self, toas):
        """timing_model.py:1716: the prior variances, PLRedNoise, PLDMNoise, then ECORR."""
        from .noise import fourier_modes, noise_basis
        if "PLDMNoise" not in self.components:
            return noise_basis(self, toas)[1]
        _, phi, _ = fourier_modes(self, toas)
        ec = noise_basis(_without(self, "PLRedNoise", "PLDMNoise"), toas)[1] if self.mask_params("ECORR") else None
        return phi if ec is None else np.concatenate([phi, ec])

    def __repr__(self):
        return f"<TimingModel {self.name}: {', '.join(self.component_names)}>"


def _without(model, *comps):
    """A shallow view of model without the named components (for the ECORR weights)."""
    import copy as _copy
    m = _copy.copy(model)
    m.components = {k: v for k, v in model.components.items() if k not in comps}
    return m


def _parse_mask_line(model: TimingModel, base: str, fields: List[str], counters: Dict[str, int]):
    comp, units = P.MASK_PARAMS[base]
    key = fields[0]
    klow = key.lower().lstrip("-") if key.startswith("-") else key.lower()
    nkv = 2 if klow in ("mjd", "freq") and not key.startswith("-") else 1
    key_value = fields[1:1 + nkv]
    rest = fields[1 + nkv:]
    counters[base] = counters.get(base, 0) + 1
    idx = counters[base]
    name = "EQUAD" if base == "TNEQ" else base
    p = Param(name=f"{name}{idx}", kind="mask", units=units if base != "TNEQ" else "us",
              component=comp, key=key, key_value=key_value, index=idx,
              long_double=False)
    v = P.fortran_float(rest[0])
    if base == "TNEQ":  # TNEQ is log10(seconds) (noise_model.py:95-128)
        v = 10.0 ** v * 1e6
    p.value = v
    if len(rest) > 1:
        p.frozen = rest[1] != "1"
        p.uncertainty_value = 0.0
    if len(rest) > 2:
        p.set_uncertainty_from_string(rest[2])
    model.add_param(p)
    return p


def get_model(parfile) -> TimingModel:
    """Build a TimingModel from a par file (model_builder.py:777 get_model)."""
    lines = P.read_parfile(parfile)
    names = [l.name for l in lines]
    model = TimingModel()
    counters: Dict[str, int] = {}
    binary = None
    for l in lines:
        if l.name == "BINARY" and l.fields:
            binary = l.fields[0].upper()
    if binary not in (None, "ELL1", "DD", "ELL1H", "BT", "DDK"):
        raise NotImplementedError(f"BINARY {binary} is outside the supported hot path (ELL1, ELL1H, DD, DDK, BT)")
    model.binary = binary
    has_eq = any(n in ("RAJ", "RA") for n in names)
    has_ecl = any(n in ("ELONG", "LAMBDA") for n in names)
    # defaults the reference components create (values 0 / None)
    defaults = []
    if has_eq:
        defaults += [("POSEPOCH", None), ("PX", 0.0), ("RAJ", None), ("DECJ", None), ("PMRA", 0.0), ("PMDEC", 0.0)]
    if has_ecl:
        defaults += [("POSEPOCH", None), ("PX", 0.0), ("ELONG", None), ("ELAT", None), ("PMELONG", 0.0),
                     ("PMELAT", 0.0), ("ECL", "IERS2010")]
    defaults += [("F0", None), ("PEPOCH", None)]
    # top-level parameters every reference model carries (timing_model.py:330-350)
    defaults += [("DILATEFREQ", False), ("DMDATA", False), ("NTOA", 0), ("UNITS", "TDB")]
    if has_eq or has_ecl:
        defaults += [("PLANET_SHAPIRO", False)]
    if any(n in ("NE_SW", "SOLARN0") for n in names):
        defaults += [("SWM", 0)]
    if any(n == "DM" or re.match(r"^DM\d+$", n) for n in names):
        defaults += [("DM", LD(0)), ("DMEPOCH", None)]
    if binary in ("ELL1", "ELL1H"):
        defaults += [(n, 0.0) for n in ELL1_PARAMS if not (binary == "ELL1H" and n in ("M2", "SINI"))]
        defaults += [("TASC", None)]
        if binary == "ELL1H":  # binary_ell1.py:345-378 (no values by default)
            defaults += [("H3", None), ("H4", None), ("STIGMA", None), ("NHARMS", None)]
    elif binary == "DD":
        defaults += [(n, 0.0) for n in DD_PARAMS]
        defaults += [("T0", None)]
    elif binary == "DDK":  # DD's parameters less SINI, KIN/KOM 0, K96 unset (default True)
        defaults += [(n, 0.0) for n in DDK_PARAMS]
        defaults += [("T0", None), ("K96", None)]
    elif binary == "BT":  # binary_bt.py:38-69: no M2/SINI, GAMMA 0, rates 0
        defaults += [(n, 0.0) for n in BT_PARAMS if n != "T0"]
        defaults += [("T0", None)]
    for n, v in defaults:
        if n in model:
            continue
        p = P.make_param(n)
        if p is None:
            continue
        if n in ("PB", "OM", "OMDOT", "EPS1", "EPS2", "EPS1DOT", "EPS2DOT", "DM") and v is not None:
            v = LD(v)
        p.value = v
        # ELL1's rates are unset (None) in the reference (binary_ell1.py), 0 here
        p.implicit = binary in ("ELL1", "ELL1H") and n in ("PBDOT", "A1DOT", "EDOT", "OMDOT", "EPS1DOT", "EPS2DOT")
        if p.component == "Binary":
            p.component = "Binary"
        model.add_param(p)
    for l in lines:
        raw = l.name
        name = P._ALIASES.get(raw, raw)
        if name in P.IGNORED or re.match(r"^DMX(EP|F1|F2)_\d+$", name):
            continue
        if name in P.MASK_PARAMS or raw in ("T2EFAC", "T2EQUAD", "TNECORR"):
            base = P._ALIASES.get(raw, raw)
            mp = _parse_mask_line(model, base, l.fields, counters)
            if raw != base and mp is not None:
                mp.alias = raw
            continue
        if name == "BINARY":
            p = model._params.get("BINARY") or P.make_param("BINARY")
            p.value = l.fields[0] if l.fields else None
            if "BINARY" not in model:
                model.add_param(p)
            continue
        if name not in model:
            p = P.make_param(name)
            if p is None:
                if name in ("FB0", "SWP", "H3", "STIGMA"):
                    continue
                raise NotImplementedError(f"parameter {raw} is outside the supported hot path")
            model.add_param(p)
        p = model[name]
        if raw != name:
            p.alias = raw
        if not l.fields:
            continue
        p.set_from_string(l.fields[0])
        # TimingModel.validate (timing_model.py:405-413): the only values PINT supports
        if name == "TIMEEPH" and p.value not in (None, "FB90"):
            p.value = "FB90"
        elif name == "T2CMETHOD" and p.value not in (None, "IAU2000B"):
            p.value = "IAU2000B"
        elif name == "DILATEFREQ" and p.value:
            p.value = False
        if len(l.fields) > 1 and p.kind not in ("str", "bool"):
            # parameter.py:551-576: a third field is a fit flag (uncertainty 0 unless a
            # fourth field gives it) or an uncertainty
            fl = l.fields[1]
            if fl in ("0", "1"):
                p.frozen = fl != "1"
                p.uncertainty_value = 0.0
                if len(l.fields) > 2:
                    p.set_uncertainty_from_string(l.fields[2])
            else:
                p.set_uncertainty_from_string(fl)
    # components present
    comps = set()
    for n, p in model._params.items():
        comps.add(p.component)
    if has_eq:
        model.components.setdefault("AstrometryEquatorial", [])
    if has_ecl:
        model.components.setdefault("AstrometryEcliptic", [])
    if has_eq or has_ecl:
        model.components.setdefault("SolarSystemShapiro", [])
    if binary:
        model.components["Binary" + binary] = model.components.pop("Binary", [])
    if model.mask_params("JUMP"):
        model.components.setdefault("PhaseJump", [])
    if "DMX" in model and not model.dmx_params():
        pass
    for noise in ("TNREDAMP", "RNAMP"):
        if noise in model and model[noise].value is not None:
            model.components.setdefault("PLRedNoise", [])
    if "TNDMAMP" in model and model.TNDMAMP.value is not None:
        model.components.setdefault("PLDMNoise", [])
    # normalise the components dict keys used above for the binary
    for n, p in model._params.items():
        if p.component == "Binary":
            p.component = "Binary"
    if "PSR" in model:
        model.name = str(model.PSR.value)
    model.validate()
    return model
