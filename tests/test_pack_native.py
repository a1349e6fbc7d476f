"""pint_pack_toas (the library's host packer behind pint_add_pulsar_cols, the default upload
path of Session.add) against engine.pack_toas (numpy): the n+1-row boundary arrays, flags,
JUMP masks and DMX bins bit for bit.  Host only: no device is touched."""
import ctypes as C

import numpy as np
import pytest

from golden_util import load

LD = np.longdouble


def _native(lay):
    from pint_amd import _lib as L
    from pint_amd.engine import pack_cols
    lib = L.lib()
    c, keep = pack_cols(lay)
    n = lay.toas.ntoas
    bufs = dict(tdb_hi=np.zeros(n + 1), tdb_lo=np.zeros(n + 1), freq_mhz=np.zeros(n + 1), sigma_s=np.zeros(n),
                pos_km=np.zeros((n + 1, 3)), vel_kms=np.zeros((n + 1, 3)), sun_km=np.zeros((n + 1, 3)),
                pulse_number=np.zeros(n), delta_pn=np.zeros(n + 1), flags=np.zeros(n + 1, np.uint32),
                jump_mask=np.zeros(n + 1, np.uint64), dmx_a=np.zeros(n + 1, np.int32),
                dmx_b=np.zeros(n + 1, np.int32))
    ct = {np.dtype(np.uint32): C.c_uint32, np.dtype(np.uint64): C.c_uint64, np.dtype(np.int32): C.c_int32}
    t = L.ToasT()
    t.n = n
    for k, a in bufs.items():
        setattr(t, k, L.ptr(a, ct.get(a.dtype, C.c_double)))
    need = lib.pint_pack_toas(C.byref(c), C.byref(t), None, 0)
    assert need >= 0
    x = None
    if need > 0:
        assert not t.dmx_x
        x = np.full(need, -7, dtype=np.int32)
        assert lib.pint_pack_toas(C.byref(c), C.byref(t), L.ptr(x, C.c_int32), need) == need
        assert t.dmx_x
    return bufs, x


def _check(lay):
    from pint_amd.engine import pack_toas
    _, keep = pack_toas(lay)
    sig = lay.sigma_us.copy()
    got, x = _native(lay)
    want = dict(zip(["tdb_hi", "tdb_lo", "freq_mhz", "sigma_s", "pos_km", "vel_kms", "sun_km", "pulse_number",
                     "delta_pn", "flags", "jump_mask", "dmx_a", "dmx_b"], keep[:13]))
    for k, w in want.items():
        g = got[k]
        assert g.dtype == w.dtype, k
        np.testing.assert_array_equal(g.reshape(w.shape).view(np.uint8), w.view(np.uint8), err_msg=k)  # bits
    if keep[14] is None:
        assert x is None
    else:
        np.testing.assert_array_equal(x, keep[14])
    np.testing.assert_array_equal(lay.sigma_us, sig)
    return got, x


@pytest.mark.parametrize("name", ["ngc6440e", "b1855", "j0740", "pta_dd", "pta_ell1", "pta_iso", "pta_ddk", "wb_dd",
                                  "dmx_overlap", "planet_ngc", "ecorr_fit", "white_mjd",
                                  "pta_bt", "phoff_red"])
def test_native_pack_matches_pack_toas(name):
    from pint_amd.engine import build_layout
    model, toas = load(name)[:2]
    _check(build_layout(model, toas))


@pytest.mark.parametrize("par,tim", [("NGC6440E.par", "NGC6440E.tim"), ("planet_b1855.par",
                                                                          "B1855+09_NANOGrav_9yv1.tim.gz")])
def test_native_pack_from_tim(par, tim):
    """TOAs prepared from a tim file (the TZR TOA prepared on demand; PLANET_SHAPIRO rows)."""
    import os
    from golden_util import GOLDEN
    from pint_amd.engine import build_layout
    from pint_amd.toa import get_model_and_toas
    model, toas = get_model_and_toas(os.path.join(GOLDEN, par), os.path.join(GOLDEN, tim), ephem="builtin",
                                     include_bipm=False)
    _check(build_layout(model, toas))


@pytest.mark.parametrize("name", ["b1855", "dmx_overlap"])
def test_native_pack_unordered_toas(name):
    """TOAs out of time order (the binary-search form of the sorted-range bins)."""
    from pint_amd.engine import build_layout
    model, toas = load(name)[:2]
    p = np.random.default_rng(3).permutation(toas.ntoas)
    _check(build_layout(model, toas[p]))


@pytest.mark.parametrize("case", ["touching", "shuffled", "nested", "triple", "nan_range"])
def test_native_pack_bin_cases(case):
    """Shared endpoints, parameter order != time order, nested ranges (the per-range pass),
    three ranges over one TOA (the dmx_x CSR), and a NaN range end (selects nothing)."""
    from pint_amd.engine import build_layout
    model, toas = load("dmx_overlap")[:2]
    names = model.dmx_params()
    mjd = toas.get_mjds().astype(np.float64)
    m = len(names)
    edges = np.linspace(mjd.min() - 1, mjd.max() + 1, m + 1)
    r1, r2 = edges[:-1].copy(), edges[1:].copy()
    if case == "touching":
        k = np.arange(1, m)
        r2[k - 1] = r1[k] = np.sort(mjd[np.argmin(np.abs(mjd[:, None] - edges[None, k]), axis=0)])
    elif case == "shuffled":
        p = np.random.default_rng(5).permutation(m)
        r1, r2 = r1[p], r2[p]
    elif case == "nested":
        r1[1], r2[1] = r1[0] + 0.1, r2[0] - 0.1
    elif case == "triple":
        r1[1], r2[1] = r1[0], r2[0]
        r1[2], r2[2] = r1[0] - 0.5, r2[0] + 0.5
    else:
        r2[0] = np.nan
    for nm, a, b in zip(names, r1, r2):
        model["DMXR1_" + nm[4:]].value = LD(a)
        model["DMXR2_" + nm[4:]].value = LD(b)
    got, x = _check(build_layout(model, toas))
    if case == "triple":
        assert x is not None


def test_native_pack_rejects_missing_columns():
    from pint_amd import _lib as L
    lib = L.lib()
    c = L.ToaColsT()
    c.n = 4
    t = L.ToasT()
    t.n = 4
    assert lib.pint_pack_toas(C.byref(c), C.byref(t), None, 0) < 0


@pytest.mark.parametrize("case", ["fixture", "unnormalised_lo", "negative"])
def test_tdbld_extent_equals_longdouble_min_max(case):
    """TOAs.tdbld_extent (the red-noise span's ends, from the extreme hi parts) equals
    tdbld.min() / .max(), whichever form of the half-ulp guard it takes."""
    model, toas = load("b1855")[:2]
    if case == "unnormalised_lo":  # a lo beyond half an ulp of its hi: the longdouble pass
        lo = np.array(toas.arrays["tdb_lo"])
        lo[5] = 3.0
        toas.arrays["tdb_lo"] = lo
    elif case == "negative":
        toas.arrays["tdb_hi"] = -toas.arrays["tdb_hi"]
        toas.arrays["tdb_lo"] = -toas.arrays["tdb_lo"]
    lo, hi = toas.tdbld_extent()
    t = toas.tdbld
    assert lo == t.min() and hi == t.max()
