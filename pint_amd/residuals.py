"""Residuals (host mirror of reference residuals.py:40-906), WidebandDMResiduals (:908) and
WidebandTOAResiduals (:1146).

All arithmetic runs on the GPU (k_eval + k_resid + k_gram/k_solve/k_woodbury); this class
holds the results.  Values are plain float64 arrays in seconds / cycles (the reference
returns astropy Quantities with the same numbers).
"""
from __future__ import annotations

import collections

import numpy as np

from . import _lib as L
from .engine import Session, build_layout, pack_table, resident


class Residuals:
    def __new__(cls, toas=None, model=None, residual_type="toa", *args, **kwargs):
        # residual_map (residuals.py:1076): "dm" -> WidebandDMResiduals
        if cls is Residuals and residual_type == "dm":
            return super().__new__(WidebandDMResiduals)
        return super().__new__(cls)

    def __init__(self, toas=None, model=None, residual_type="toa", unit="s", subtract_mean=True,
                 use_weighted_mean=True, track_mode=None, use_abs_phase=True, _session=None):
        if residual_type != "toa":
            raise ValueError(f"unknown residual_type {residual_type!r} (residuals.py:1076 residual_map)")
        self.residual_type = "toa"
        self._is_combined = False
        self.toas = toas
        self.model = model
        self.subtract_mean = subtract_mean and "PhaseOffset" not in model.components
        self.use_weighted_mean = use_weighted_mean
        self.use_abs_phase = use_abs_phase
        self._chi2 = None
        self.noise_resids = {}
        self._track_mode_arg = track_mode
        self.phase_resids = None
        self.time_resids = None
        if toas is not None and model is not None:
            self.update()

    def update(self):
        # the resident upload of these TOAs and this model structure (engine.resident): a
        # Residuals of a fitted model re-binds one parameter table
        s, lay = resident(self.model, self.toas, track_mode=self._track_mode_arg,
                          subtract_mean=self.subtract_mean, use_weighted_mean=self.use_weighted_mean)
        self.track_mode = lay.track_mode
        s.set_instances([(lay, pack_table(lay, self.model))])
        corr = self.model.has_correlated_errors and (lay.nred > 0 or lay.nep > 0)
        s.eval(want_M=Session.FIT if corr else False)
        tr, pr, c2 = s.read_resids()
        self.time_resids = tr[0]
        self.phase_resids = pr[0]
        self._sigma_us = lay.sigma_us
        if corr:
            try:  # the step only provides the Woodbury factor; a degenerate timing solve is irrelevant
                s.fit_step(1)
            except L.PintError as e:
                if e.code != L.PINT_E_NOT_PD:
                    raise
            self._chi2 = float(s.chi2_gls()[0])
        else:
            self._chi2 = float(c2[0])
        ln_kind = 1 if corr else (2 if self.model.has_correlated_errors else 0)
        self._lognorm = float(s.lognorm(ln_kind)[0])

    @classmethod
    def _from_batch(cls, toas, model, bf, d, chi2, track_mode=None):
        """The residuals of device instance `d` of a BatchFit after its last evaluation
        (the fit's final state): read from the fit's session, no re-upload."""
        r = cls.__new__(cls)
        r.toas, r.model = toas, model
        r.subtract_mean = "PhaseOffset" not in model.components
        r.use_weighted_mean = True
        r.use_abs_phase = True
        r.noise_resids = {}
        r._track_mode_arg = track_mode
        lay = bf.layouts[d]
        tr, pr, _ = bf.s.read_resids()
        r.time_resids, r.phase_resids = tr[d].copy(), pr[d].copy()
        r.track_mode = lay.track_mode
        r._sigma_us = lay.sigma_us
        r._chi2 = float(chi2)
        corr = model.has_correlated_errors and (lay.nred > 0 or lay.nep > 0)
        kind = 1 if (corr and bf.gls) else (2 if model.has_correlated_errors else 0)
        r._lognorm = float(bf.s.lognorm(kind)[d])
        return r

    @property
    def resids(self):
        return self.time_resids

    @property
    def resids_value(self):
        return self.time_resids

    @property
    def chi2(self) -> float:
        return self._chi2

    def calc_chi2(self, lognorm=False):
        """residuals.py:669-711: (chi2, log_norm) with lognorm=True, log_norm = logdet(C)/2
        (Woodbury, correlated noise) or sum log sigma (white noise), from the GPU."""
        return (self._chi2, self._lognorm) if lognorm else self._chi2

    def lnlikelihood(self) -> float:
        """residuals.py:713-716: -(chi2/2 + log_norm)."""
        chi2, log_norm = self.calc_chi2(lognorm=True)
        return -(chi2 / 2 + log_norm)

    @property
    def dof(self) -> int:
        return self.toas.ntoas - (len(self.model.free_params) + 1)

    @property
    def reduced_chi2(self) -> float:
        return self.chi2 / self.dof

    def get_data_error(self, scaled=True):
        return self._sigma_us if scaled else self.toas.get_errors()

    def rms_weighted(self):
        """Weighted RMS in microseconds (residuals.py:252 via utils.py:2002)."""
        w = 1.0 / (self._sigma_us * 1e-6) ** 2
        r = self.time_resids
        m = (w * r).sum() / w.sum()
        return float(np.sqrt((w * (r - m) ** 2).sum() / w.sum()) * 1e6)


class WidebandDMResiduals(Residuals):
    """residuals.py:908-1071: the wideband DM measurements (-pp_dm / -pp_dme TOA flags) minus
    the model's total DM (DispersionDM + DMX + DMJUMP), in pc/cm^3, computed on the GPU
    (k_dm_resid through pint_dm_resids); chi2 with the DMEFAC/DMEQUAD-scaled errors."""

    def __init__(self, toas=None, model=None, residual_type="dm", unit="pc / cm3", subtract_mean=False,
                 use_weighted_mean=True):
        self.toas = toas
        self.model = model
        self.residual_type = residual_type
        self.unit = unit
        self.base_unit = "pc / cm3"
        self.subtract_mean = subtract_mean
        self.use_weighted_mean = use_weighted_mean
        self._is_combined = False
        self.debug_info = {}
        self.dm_data, self.dm_error, self.relevant_toas = self.get_dm_data()
        self._chi2 = None
        self._resids = None
        if toas is not None and model is not None:
            self.update()

    def get_dm_data(self):
        """(dm_data, dm_error, valid TOA indices) from the TOA flags (residuals.py:1044-1071)."""
        dm, valid = self.toas.get_flag_value("pp_dm")
        dme, valid_e = self.toas.get_flag_value("pp_dme")
        if valid == []:
            raise ValueError("Input TOA object does not have wideband DM values")
        if valid != valid_e:
            raise ValueError("Input TOA object' DM data and DM errors do not match.")
        return (np.array([float(dm[i]) for i in valid]), np.array([float(dme[i]) for i in valid]), valid)

    def update(self):
        if len(self.relevant_toas) != self.toas.ntoas:
            raise NotImplementedError("wideband DMs on only some TOAs (toa.py:1767-1791 does not handle them "
                                      "either)")
        s = Session()
        try:
            lay = s.add(build_layout(self.model, self.toas))
            s.set_instances([(lay, pack_table(lay))])
            s.set_wideband(lay)
            r, c2 = s.dm_resids(self.subtract_mean, self.use_weighted_mean)
            self._resids = r[0]
            self._chi2 = float(c2[0])
            self._sigma = lay.dm_sigma
        finally:
            s.close()

    @property
    def resids(self):
        return self._resids

    @property
    def resids_value(self):
        return self._resids

    def calc_resids(self):
        return self._resids

    @property
    def chi2(self) -> float:
        return self._chi2

    def calc_chi2(self, lognorm=False) -> float:
        if np.any(self._sigma == 0.0):
            return np.inf
        return self._chi2

    @property
    def dof(self) -> int:
        """len(DM data) - the free parameters of the Dispersion components - 1 (residuals.py:967)."""
        if self._is_combined:
            raise AttributeError("Please use the `.dof` in the CombinedResidual class. The individual residual's "
                                 "dof is not calculated correctly in the combined residuals.")
        disp = ("DispersionDM", "DispersionDMX", "DispersionJump")
        return len(self.dm_data) - sum(1 for n in self.model.free_params if self.model[n].component in disp) - 1

    def get_data_error(self, scaled=True):
        return self._sigma if scaled else self.dm_error

    def rms_weighted(self):
        """Weighted standard deviation of the DM residuals, weights 1/scaled error^2
        (residuals.py:1033 via utils.py:2002 weighted_mean)."""
        if np.any(self._sigma == 0):
            raise ValueError("Some DM errors are zero - cannot calculate weighted RMS of residuals")
        w = 1.0 / self._sigma ** 2
        r = self._resids
        m = (w * r).sum() / w.sum()
        return float(np.sqrt((w * (r - m) ** 2).sum() / w.sum()))

    def update_model(self, new_model, **kwargs):
        self.model = new_model
        self.update()


class CombinedResiduals:
    """residuals.py:1079-1144: results of several residual types (units differ, so the
    combined arrays are unitless)."""

    def __init__(self, residuals):
        self.residual_objs = collections.OrderedDict()
        for res in residuals:
            res._is_combined = True
            self.residual_objs[res.residual_type] = res
        self.debug_info = {}

    @property
    def _combined_resids(self) -> np.ndarray:
        return np.hstack([res.resids_value for res in self.residual_objs.values()])

    @property
    def _combined_data_error(self) -> np.ndarray:
        return np.hstack(list(self.data_error.values()))

    @property
    def unit(self) -> dict:
        return {k: ("s" if k == "toa" else "pc / cm3") for k in self.residual_objs}

    @property
    def chi2(self) -> float:
        return sum(res.chi2 for res in self.residual_objs.values())

    @property
    def data_error(self):
        """The scaled errors per type (TOAs in us, DMs in pc/cm^3, as the reference's .value)."""
        return collections.OrderedDict((k, np.asarray(rs.get_data_error())) for k, rs in self.residual_objs.items())

    def rms_weighted(self) -> dict:
        if np.any(self._combined_data_error == 0):
            raise ValueError("Some data errors are zero - cannot calculate weighted RMS of residuals")
        return {k: rs.rms_weighted() for k, rs in self.residual_objs.items()}


class WidebandTOAResiduals(CombinedResiduals):
    """residuals.py:1146-1271: TOA residuals and wideband DM residuals of one model.  Its chi2
    is the reference's WidebandTOAFitter pass with no free parameters (:1206-1246): a GLS over
    [TOA rows; DM rows] whose design matrix is the Offset column (zero on the DM rows) plus
    the TOA noise basis, i.e. the TOA residuals' GLS chi2 (offset marginalised, Woodbury on
    the device) plus the DM rows' chi2."""

    def __init__(self, toas, model, toa_resid_args: dict = {}, dm_resid_args: dict = {}):
        self.toas = toas
        self._model = model
        toa_resid = Residuals(self.toas, self.model, residual_type="toa", **toa_resid_args)
        dm_resid = Residuals(self.toas, self.model, residual_type="dm", **dm_resid_args)
        self._chi2 = None
        super().__init__([toa_resid, dm_resid])

    @property
    def toa(self) -> Residuals:
        return self.residual_objs["toa"]

    @property
    def dm(self) -> WidebandDMResiduals:
        return self.residual_objs["dm"]

    @property
    def chi2(self) -> float:
        if self._chi2 is None:
            self._chi2 = self.calc_chi2()
        return self._chi2

    def calc_chi2(self, full_cov=False) -> float:
        return float(self.toa.chi2 + self.dm.chi2)

    @property
    def model(self):
        return self._model

    @property
    def dof(self) -> int:
        return len(self._combined_resids) - (len(self.model.free_params) + 1)

    @property
    def reduced_chi2(self) -> float:
        return self.chi2 / self.dof
