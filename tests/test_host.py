"""CPU tests of the host side: par parsing, TOA masks, noise preparation, the C-ABI library
(load + exported symbols + struct layout), multi-rank grid sharding over gloo.  No GPU."""
import ctypes as C
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from golden_util import GOLDEN, load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["ngc6440e", "b1855", "j0740", "pta_iso", "pta_ell1", "pta_dd"]


def _meta(name):
    return json.load(open(os.path.join(GOLDEN, name + ".json")))


# ---- par parsing (model_builder.py:777, parameter.py) -------------------------------
@pytest.mark.parametrize("name", NAMES)
def test_parfile_values(name):
    model, toas, z, meta = load(name)
    vals = meta["model"]["values"]
    checked = 0
    for n, d in vals.items():
        v = d.get("value")
        if not isinstance(v, list) or n not in model or n in ("NTOA", "TRES", "SWM", "SWP"):
            continue
        ref = np.longdouble(v[0]) + np.longdouble(v[1])
        got = model[n].value
        assert got is not None, n
        if re.match(r"^DMXR[12]_", n):
            # bin edges: the reference keeps an MJD (jd1, jd2) pair; used as float64 only
            assert float(got) == float(ref), n
        else:
            tol = 2 * abs(float(np.spacing(ref))) if model[n].kind == "mjd" or model[n].long_double else \
                4 * abs(np.spacing(float(ref)))
            assert abs(float(np.longdouble(got) - ref)) <= tol, (n, got, ref)
        checked += 1
    assert checked > 5


@pytest.mark.parametrize("name", NAMES)
def test_free_params_and_components(name):
    model, toas, z, meta = load(name)
    assert model.free_params == meta["model"]["free_params"]
    for c in ("AstrometryEquatorial", "AstrometryEcliptic", "BinaryELL1", "BinaryDD", "PLRedNoise"):
        assert (c in meta["model"]["components"]) == (c in model.components), c


@pytest.mark.parametrize("name", [n for n in NAMES if n != "ngc6440e"])
def test_mask_selection(name):
    model, toas, z, meta = load(name)
    for k in z:
        if not k.startswith("mask_"):
            continue
        p = model[k[5:]]
        idx = toas.select_mask(p.key, p.key_value)
        assert np.array_equal(np.sort(idx), np.where(z[k].astype(bool))[0]), k


@pytest.mark.parametrize("name", NAMES)
def test_scaled_sigma(name):
    from pint_amd.noise import scaled_sigma_us
    model, toas, z, meta = load(name)
    assert np.allclose(scaled_sigma_us(model, toas), z["res_sigma_us"], rtol=1e-15, atol=0)


@pytest.mark.parametrize("name", ["pta_iso", "pta_ell1", "pta_dd", "b1855"])
def test_noise_weights(name):
    from pint_amd.noise import noise_basis
    model, toas, z, meta = load(name)
    nb = noise_basis(model, toas)
    w = nb[1] if isinstance(nb, tuple) else nb["weights"]
    assert np.allclose(w, z["noise_weights"], rtol=1e-12, atol=0)


def test_track_mode():
    from pint_amd.engine import _track_mode
    for name in NAMES:
        model, toas, z, meta = load(name)
        assert _track_mode(model, toas, None) == meta["res_track_mode"], name


# ---- the C-ABI library ----------------------------------------------------------------
def _lib_path():
    from pint_amd import _lib
    if not os.path.exists(_lib.LIBPATH):
        sys.path.insert(0, ROOT)
        import __graft_entry__
        __graft_entry__.build()
    return _lib.LIBPATH


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "pint_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pint_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    from pint_amd import _lib
    lib = C.CDLL(_lib_path())
    decl = _header_functions()
    assert len(decl) >= 20
    for f in decl:
        assert hasattr(lib, f), f
    assert sorted(_lib.EXPORTED) == decl
    assert lib.pint_device_count() >= 0 or True  # callable without a GPU (returns 0 / error)


@pytest.mark.parametrize("dims", [(7,), (5, 3), (4, 3, 2), (2, 3, 4, 5)])
def test_meshgrid_axes_reproduce_the_flattened_meshgrid(dims):
    """gridutils.meshgrid_axes (what pint_set_grid expands on the device) gives every flat
    point of np.meshgrid(*parvalues) ('xy' indexing, C-order flatten) -- the reference's
    point order (gridutils.py:331, :366) -- including a rank's block starting at k0."""
    from golden_util import grid_tables
    from pint_amd.gridutils import grid_points, meshgrid_axes

    class Lay:
        offsets = {f"P{j}": 2 * j for j in range(len(dims))}
    vals = [np.longdouble(10 * j + 1) + np.arange(n, dtype=np.longdouble) / 3 for j, n in enumerate(dims)]
    _, flat = grid_points(vals)
    axes, npts = meshgrid_axes(vals)
    assert npts == flat[0].size
    var = [(f"P{j}", a, st, sz) for j, (a, st, sz) in enumerate(axes)]
    for k0, cnt in ((0, npts), (npts // 3, npts - npts // 3)):
        t = grid_tables(Lay, (np.zeros(2 * len(dims)), var, cnt, k0))
        for j, f in enumerate(flat):
            got = t[:, 2 * j].astype(np.longdouble) + t[:, 2 * j + 1]
            np.testing.assert_array_equal(got, f[k0:k0 + cnt])


def test_one_hip_runtime_whatever_loads_first():
    """libpint_hip.so loaded before `import torch` must not leave two HIP/HSA runtimes in the
    process (torch's would then see no device and the RCCL gathers could not start)."""
    _lib_path()
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from pint_amd import _lib; _lib.lib()\n"
            "import torch\n"
            "m = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}\n"
            "h = {l.split()[-1] for l in open('/proc/self/maps') if 'libhsa-runtime64' in l}\n"
            "print(len(m), len(h))\n") % ROOT
    env = dict(os.environ)
    env.pop("PINT_HIP_RUNTIME", None)
    out = subprocess.run([sys.executable, "-c", code], check=True, capture_output=True, text=True, env=env)
    assert out.stdout.split() == ["1", "1"], out.stdout
    # ... and it is the system ROCm's (torch's copies never mapped)
    code2 = code.replace("print(len(m), len(h))", "print(all('/torch/' not in x for x in m | h))")
    out = subprocess.run([sys.executable, "-c", code2], check=True, capture_output=True, text=True, env=env)
    assert out.stdout.split() == ["True"], out.stdout


def test_struct_layout_matches_header():
    """ctypes mirrors (pint_amd/_lib.py) == the C header layout (compiled with gcc)."""
    from pint_amd import _lib
    fields = {"pint_toas_t": _lib.ToasT, "pint_spec_t": _lib.SpecT, "pint_toa_cols_t": _lib.ToaColsT}
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "pint_amd.h"', 'int main(void){']
    for st, cls in fields.items():
        src.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for fname, _ in cls._fields_:
            src.append(f'printf("{st}.{fname} %zu\\n", offsetof({st}, {fname}));')
    src.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write("\n".join(src))
        exe = os.path.join(d, "l")
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(l.split() for l in out if l)
    for st, cls in fields.items():
        assert int(got[st]) == C.sizeof(cls), st
        for fname, _ in cls._fields_:
            assert int(got[f"{st}.{fname}"]) == getattr(cls, fname).offset, (st, fname)


def test_no_gpu_compute_fails_loudly():
    """Without a GPU the product raises; it never falls back to a CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pint_amd import Residuals
    model, toas, z, meta = load("ngc6440e")
    with pytest.raises(Exception):
        Residuals(toas, model).time_resids


# ---- multi-rank sharding (gloo, world size 2) ---------------------------------------------
def _gloo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from pint_amd.gridutils import gather_blocks, shard_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        for npts in (1, 7, 64, 65):
            per, lo, hi = shard_range(npts, rank, world)
            local = np.arange(lo, hi, dtype=np.float64) ** 2  # stand-in for chi2 of my block
            res[npts] = gather_blocks(local, per, npts, dist).tolist()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_grid_sharding_gloo():
    import torch.multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out:
        for npts, arr in res.items():
            assert arr == (np.arange(npts, dtype=np.float64) ** 2).tolist(), (rank, npts)


def test_shard_range_covers():
    from pint_amd.gridutils import shard_range
    for npts in (0, 1, 5, 100, 101):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                per, lo, hi = shard_range(npts, r, world)
                got += list(range(lo, max(lo, hi)))
            assert got == list(range(npts))


@pytest.mark.parametrize("name", ["ngc6440e", "b1855", "j0740", "pta_dd", "pta_ell1", "pta_iso", "pta_ddk", "wb_dd"])
def test_pack_table_matches_per_parameter_split(name):
    """engine.pack_table (all parameters converted at once) equals split_ld parameter by
    parameter: the same (hi, lo) double-double split, bit for bit."""
    from pint_amd.engine import build_layout, pack_table, split_ld
    model, toas = load(name)[:2]
    lay = build_layout(model, toas)
    ref = np.zeros(lay.tstride)
    for n, o in lay.offsets.items():
        v = model[n].value
        ref[o], ref[o + 1] = split_ld(0.0 if v is None else v)
    np.testing.assert_array_equal(pack_table(lay, model), ref)
    np.testing.assert_array_equal(pack_table(lay, model), ref)  # (the cached offset arrays)
