"""Par-file writer/reader parity: pint_amd's as_parfile against the
reference's own as_parfile text of the same models (tests/golden/parfile_*.txt by
oracle/refgen/gen_parfile.py), round trips through pint_amd's reader, and (in the build
container) the reference reading pint_amd's output back.  CPU only."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from golden_util import GOLDEN, PARS

NAMES = [n for n in PARS if n != "j0740_10k"]  # j0740_10k shares j0740's par file
REFENV = os.path.join(os.path.dirname(__file__), "..", "oracle", "refenv", "run_ref.sh")
REFGEN = os.path.join(os.path.dirname(__file__), "..", "oracle", "refgen")


def _model(name):
    from pint_amd import get_model
    return get_model(os.path.join(GOLDEN, PARS[name]))


def _fitted(name):
    """The model with the reference GLS fit's values and uncertainties (fixture meta)."""
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    m = _model(name)
    m.free_params = [p for p in meta["model"]["free_params"] if p in m]
    for p, v in meta["gls_params"].items():
        par = m[p]
        val = np.longdouble(v[0]) + np.longdouble(v[1])
        par.value = val if (par.long_double or par.kind == "mjd") else float(val)
        par.uncertainty = meta["gls_errors"][p]
    return m


def _ref_lines(fname):
    return open(os.path.join(GOLDEN, fname)).read().splitlines()


@pytest.mark.parametrize("name", NAMES)
def test_parfile_lines_match_reference(name):
    """Every line the reference writes for the model -- values (longdouble / float64 str,
    MJD day + 16 decimals through astropy's day_frac, UTC MJDs through the ns time of day,
    sexagesimal angles), fit flags, uncertainties, mask keys, aliases, defaults, ELL1's
    derived ECC/OM comments -- and no other.  (The reference orders its middle component
    categories by a set iteration, so the comparison is of the lines, not their order.)"""
    ours = _model(name).as_parfile(include_info=False).splitlines()
    ref = _ref_lines(f"parfile_{name}.txt")
    assert sorted(ours) == sorted(ref), (sorted(set(ref) - set(ours))[:5], sorted(set(ours) - set(ref))[:5])


@pytest.mark.parametrize("name", ["pta_dd", "j0740"])
def test_fitted_parfile_lines_match_reference(name):
    """The same after a fit: longdouble values from fit arithmetic, MJDs set from longdouble
    (time_from_longdouble), uncertainties in each parameter's print convention."""
    ours = _fitted(name).as_parfile(include_info=False).splitlines()
    ref = _ref_lines(f"parfile_{name}_fit.txt")
    assert sorted(ours) == sorted(ref), (sorted(set(ref) - set(ours))[:5], sorted(set(ours) - set(ref))[:5])


@pytest.mark.parametrize("name", NAMES + ["pta_dd_fit", "j0740_fit"])
def test_roundtrip(name, tmp_path):
    """write_parfile -> get_model gives back every value bit for bit, the fit flags and the
    uncertainties, and writing again reproduces the same text."""
    from pint_amd import get_model
    m = _fitted(name[:-4]) if name in ("pta_dd_fit", "j0740_fit") else _model(name)
    path = tmp_path / "out.par"
    m.write_parfile(str(path), include_info=True, comment="round trip")
    m2 = get_model(str(path))
    assert list(m2.free_params) == list(m.free_params)
    for n in m.params:
        a, b = m[n], m2[n] if n in m2 else None
        if a.value is None or getattr(a, "implicit", False):
            continue
        assert b is not None, n
        if a.kind in ("str", "bool", "int"):
            assert a.value == b.value, n
        elif a.kind in ("hourangle", "degangle"):
            # sexagesimal to 8 decimals of seconds: 1e-8 s of time / 1e-8 arcsec
            tol = 1e-8 / 3600 * (1 if a.kind == "hourangle" else 1) + 1e-15 * abs(float(a.value))
            assert abs(float(a.value) - float(b.value)) <= tol, (n, a.value, b.value)
        elif a.kind == "mjd":
            # 16 decimals of a day, re-read as integer day + float64 fraction: one longdouble
            # ulp at MJD 5e4 (7e-15 d = 0.6 ns), as with the reference's own files
            assert abs(float(np.longdouble(a.value) - np.longdouble(b.value))) <= 8e-15, n
        else:
            assert np.longdouble(a.value) == np.longdouble(b.value), (n, a.value, b.value)
        if a.uncertainty_value is not None and a.kind not in ("hourangle", "degangle"):
            assert b.uncertainty_value is not None and \
                abs(float(a.uncertainty_value) - float(b.uncertainty_value)) <= 1e-15 * abs(float(a.uncertainty_value)), n
    assert m2.as_parfile(include_info=False) == m.as_parfile(include_info=False)


@pytest.mark.skipif(not (os.path.isdir("/root/reference") and shutil.which("bash")
                         and os.path.exists("/opt/conda/bin/python3.9")),
                    reason="needs the reference in the build container")
@pytest.mark.parametrize("name", NAMES)
def test_reference_reads_our_parfile(name, tmp_path):
    """The reference's get_model on pint_amd's output gives the model whose own as_parfile
    is the reference's text of the original par file (the file round-trips into a PINT
    workflow)."""
    path = tmp_path / f"{name}.par"
    _model(name).write_parfile(str(path))
    out = subprocess.run(["bash", REFENV, "check_parfile.py", str(path)], cwd=REFGEN, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    assert sorted(out.stdout.splitlines()) == sorted(_ref_lines(f"parfile_{name}.txt"))
