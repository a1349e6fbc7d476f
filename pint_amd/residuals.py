"""Residuals (host mirror of reference residuals.py:40-906, TOA residuals only).

All arithmetic runs on the GPU (k_eval + k_resid + k_gram/k_solve/k_woodbury); this class
holds the results.  Values are plain float64 arrays in seconds / cycles (the reference
returns astropy Quantities with the same numbers).
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .engine import Session, build_layout, pack_table


class Residuals:
    def __init__(self, toas=None, model=None, residual_type="toa", unit="s", subtract_mean=True,
                 use_weighted_mean=True, track_mode=None, use_abs_phase=True, _session=None):
        if residual_type != "toa":
            raise NotImplementedError("only TOA residuals are on this hot path (wideband is out of scope)")
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
        s = Session()
        try:
            lay = s.add(build_layout(self.model, self.toas, track_mode=self._track_mode_arg,
                                     subtract_mean=self.subtract_mean, use_weighted_mean=self.use_weighted_mean))
            self.track_mode = lay.track_mode
            s.set_instances([(lay, pack_table(lay))])
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
        finally:
            s.close()

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
