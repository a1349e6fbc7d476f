"""Noise-model host preparation: scaled TOA uncertainties, PLRedNoise frequencies/weights,
ECORR epochs.  These are parameter-independent during a timing fit (noise parameters are
not fitted on this path) and are computed once per (model, TOAs) at upload, like the
DMX/JUMP index tables.  Reference: noise_model.py:159-177 (scale_toa_sigma), :761-789
(PLRedNoise weights), :808-880 (ECORR epochs, Fourier basis), :883 (powerlaw).
"""
from __future__ import annotations

import numpy as np


def scaled_sigma_us(model, toas) -> np.ndarray:
    """ScaleToaError.scale_toa_sigma (noise_model.py:159): EQUADs in quadrature, then EFACs."""
    sigma = np.array(toas.get_errors(), dtype=np.float64, copy=True)
    for name in model.mask_params("EQUAD"):
        p = model[name]
        if p.value is None:
            continue
        idx = toas.select_mask(p.key, p.key_value)
        if len(idx):
            sigma[idx] = np.hypot(sigma[idx], float(p.value))
    for name in model.mask_params("EFAC"):
        p = model[name]
        idx = toas.select_mask(p.key, p.key_value)
        if len(idx):
            sigma[idx] *= float(p.value)
    return sigma


def scaled_dm_sigma(model, toas) -> np.ndarray:
    """ScaleDmError.scale_dm_sigma (noise_model.py:291-315): DMEQUADs in quadrature, then
    DMEFACs, on the -pp_dme errors (pc/cm^3); host preparation at upload like the TOA errors."""
    sigma = np.array(toas.get_dm_errors(), dtype=np.float64, copy=True)
    for name in model.mask_params("DMEQUAD"):
        p = model[name]
        if p.value is None:
            continue
        idx = toas.select_mask(p.key, p.key_value)
        if len(idx):
            sigma[idx] = np.hypot(sigma[idx], float(p.value))
    for name in model.mask_params("DMEFAC"):
        p = model[name]
        idx = toas.select_mask(p.key, p.key_value)
        if len(idx):
            sigma[idx] *= float(p.value)
    return sigma


def red_noise_freqs_weights(model, toas):
    """(f_k [nmodes], phi [2 nmodes]) — get_rednoise_freqs (noise_model.py:847) with
    T = max(t) - min(t) of t = tdbld*86400 in longdouble, powerlaw(f) * f[0] (:780-789).
    f_k stays longdouble, as the reference builds its basis sin(2 pi t f_k) with it
    (noise_model.py:861-880); the device receives it as a double-double pair."""
    amp, gam, nf = model.red_noise_params()
    lo, hi = toas.tdbld_extent()  # (== tdbld.min(), .max(): T as (tdbld * 86400).max() - .min())
    T = hi * np.longdouble(86400) - lo * np.longdouble(86400)
    f = np.linspace(1 / T, nf / T, nf)
    ff = np.zeros(2 * nf)
    ff[::2] = f
    ff[1::2] = f
    fyr = 1 / 3.16e7
    phi = amp ** 2 / 12.0 / np.pi ** 2 * fyr ** (gam - 3) * ff ** (-gam)
    return f, phi * ff[0]


def dm_noise_freqs_weights(model, toas):
    """PLDMNoise (noise_model.py:443-540): (f_k [nmodes], phi [2 nmodes]) as for PLRedNoise
    with TNDMAMP/TNDMGAM/TNDMC; its basis is the Fourier basis times (1400 MHz / f_bary)^2 per
    TOA, formed on the device (the barycentric frequency depends on the model)."""
    amp, gam, nf = model.dm_noise_params()
    lo, hi = toas.tdbld_extent()  # (== tdbld.min(), .max(): T as (tdbld * 86400).max() - .min())
    T = hi * np.longdouble(86400) - lo * np.longdouble(86400)
    f = np.linspace(1 / T, nf / T, nf)
    ff = np.zeros(2 * nf)
    ff[::2] = f
    ff[1::2] = f
    fyr = 1 / 3.16e7
    phi = amp ** 2 / 12.0 / np.pi ** 2 * fyr ** (gam - 3) * ff ** (-gam)
    return f, phi * ff[0]


def fourier_modes(model, toas):
    """All Fourier noise modes of the model in the device's order: PLRedNoise, then
    PLDMNoise.  Returns (f [nmodes], phi [2 nmodes], first DM mode)."""
    fs, ph = [], []
    if "PLRedNoise" in model.components:
        f, p = red_noise_freqs_weights(model, toas)
        fs.append(f)
        ph.append(p)
    n_red = sum(len(f) for f in fs)
    if "PLDMNoise" in model.components:
        f, p = dm_noise_freqs_weights(model, toas)
        fs.append(f)
        ph.append(p)
    if not fs:
        return None, None, 0
    return np.concatenate(fs), np.concatenate(ph), n_red


def fourier_basis(model, toas) -> np.ndarray:
    """Host copy of the red-noise basis for API/parity use (noise_model.py:861).  The device
    generates the same columns inside k_eval."""
    f, _ = red_noise_freqs_weights(model, toas)
    t = toas.tdbld * np.longdouble(86400)
    F = np.zeros((toas.ntoas, 2 * len(f)))
    F[:, ::2] = np.sin(2 * np.pi * t[:, None] * f)
    F[:, 1::2] = np.cos(2 * np.pi * t[:, None] * f)
    return F


def ecorr_epochs(t_sec: np.ndarray, dt: float = 1.0, nmin: int = 2):
    """get_ecorr_epochs (noise_model.py:808): 1-s buckets on sorted times, >= nmin TOAs."""
    if len(t_sec) == 0:
        return []
    isort = np.argsort(t_sec, kind="stable")
    ts = t_sec[isort]
    # a gap >= dt to the previous TOA always opens a bucket (the bucket reference time is
    # <= the previous TOA); only clusters spanning >= dt need the sequential scan
    cut = np.concatenate([[0], np.nonzero(np.diff(ts) >= dt)[0] + 1, [len(ts)]])
    keep = np.nonzero(np.diff(cut) >= nmin)[0]
    out = []
    for a, b in zip(cut[keep].tolist(), cut[keep + 1].tolist()):
        if ts[b - 1] - ts[a] < dt:
            out.append(isort[a:b])
            continue
        s = a
        for i in range(a + 1, b):
            if ts[i] - ts[s] >= dt:
                if i - s >= nmin:
                    out.append(isort[s:i])
                s = i
        if b - s >= nmin:
            out.append(isort[s:b])
    return out


def noise_basis(model, toas):
    """(U, weights) in the reference's NoiseComponent_list order (timing_model.py:1133,
    :1690): PLRedNoise before EcorrNoise (pinned by the B1855 fixture's noise_dims)."""
    mats, wts = [], []
    if "PLRedNoise" in model.components:
        mats.append(fourier_basis(model, toas))
        wts.append(red_noise_freqs_weights(model, toas)[1])
    if "PLDMNoise" in model.components:
        raise NotImplementedError("the PLDMNoise basis depends on the barycentric frequency: it is formed on the "
                                  "device (use noise_model_basis_weight for its weights)")
    if "EcorrNoise" in model.components or model.mask_params("ECORR"):
        t = np.asarray(toas.tdbld * np.longdouble(86400))
        for name in model.mask_params("ECORR"):
            p = model[name]
            idx = toas.select_mask(p.key, p.key_value)
            eps = ecorr_epochs(t[idx])
            U = np.zeros((toas.ntoas, len(eps)))
            for j, b in enumerate(eps):
                U[idx[b], j] = 1.0
            mats.append(U)
            wts.append(np.full(len(eps), (float(p.value) * 1e-6) ** 2))
    if not mats:
        return None, None
    return np.hstack(mats), np.concatenate(wts)
