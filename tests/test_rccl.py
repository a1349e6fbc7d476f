"""The RCCL branch of the result gathers, executed on one GPU.

pint_amd.pta.gather_rows and pint_amd.gridutils.gather_blocks return early at world size 1;
with pta.FORCE_COLLECTIVE they run the all-gather through the process group anyway.  Here
the group is a one-rank nccl (RCCL) group on cuda:0, so the device placement of the gather
buffers (cuda:LOCAL_RANK) and the all_gather itself execute before an 8-GPU node sees them:
the gathered arrays, a PTA fit and a chi2 grid through the group equal the ones without it.
"""
import copy
import os
import socket

import numpy as np
import pytest

from golden_util import load

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_group():
    from pint_amd import _lib
    ndev = _lib.lib().pint_device_count()  # (before torch: the process's HIP runtime is chosen here)
    import torch
    import torch.distributed as dist
    from pint_amd import pta
    if ndev <= 0:
        pytest.skip("no GPU visible to libpint_hip")
    # the library sees a device, so torch must too: a False here is a second HIP runtime in
    # the process (pint_amd._lib._one_hip_runtime), never a reason to skip
    maps = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln})
    assert torch.cuda.is_available(), (f"libpint_hip sees {ndev} device(s) but torch sees "
                                       f"{torch.cuda.device_count()}; HIP runtimes mapped: {maps}")
    os.environ.setdefault("LOCAL_RANK", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", world_size=1, rank=0)
    pta.FORCE_COLLECTIVE = True
    try:
        yield dist
    finally:
        pta.FORCE_COLLECTIVE = False
        dist.destroy_process_group()


def test_gathers_through_rccl(nccl_group):
    from pint_amd.gridutils import gather_blocks
    from pint_amd.pta import gather_rows
    assert nccl_group.get_backend() == "nccl"
    rows = np.arange(12.0).reshape(3, 4)
    np.testing.assert_array_equal(gather_rows(rows, [3], nccl_group), rows)
    blk = np.array([1.5, np.nan, -2.0, 7.25, 3.0])
    np.testing.assert_array_equal(gather_blocks(blk, 5, 5, nccl_group), blk)


def test_pta_fit_through_rccl(nccl_group):
    import pint_amd.pta as pta
    from pint_amd.pta import fit_pta
    items = [load(n)[:2] for n in ("pta_iso", "pta_ell1")]
    pta.FORCE_COLLECTIVE = False  # the same fit without the collective
    ref, _ = fit_pta([(copy.deepcopy(m), t) for m, t in items], mode="gls", dist=nccl_group)
    pta.FORCE_COLLECTIVE = True
    got_items = [(copy.deepcopy(m), t) for m, t in items]
    got, shards = fit_pta(got_items, mode="gls", dist=nccl_group)
    assert shards == [[0, 1]]
    for r, g, (m, _) in zip(ref, got, got_items):
        assert g.status == r.status
        assert g.chi2 == r.chi2
        np.testing.assert_array_equal(g.errors, r.errors)


def test_grid_through_rccl(nccl_group):
    from pint_amd import WLSFitter
    from pint_amd.gridutils import grid_chisq
    import pint_amd.pta as pta
    model, toas, _, _ = load("ngc6440e")
    f = WLSFitter(toas, model)
    f.fit_toas(maxiter=1)
    g0 = np.longdouble(f.model.F0.value) + np.linspace(-2, 2, 4) * np.longdouble(f.model.F0.uncertainty)
    g1 = np.longdouble(f.model.F1.value) + np.linspace(-2, 2, 3) * np.longdouble(f.model.F1.uncertainty)
    c_rccl, ex_rccl = grid_chisq(f, ("F0", "F1"), (g0, g1), extraparnames=["DM"])
    pta.FORCE_COLLECTIVE = False  # the same grid without the collective
    c_one, ex_one = grid_chisq(f, ("F0", "F1"), (g0, g1), extraparnames=["DM"])
    pta.FORCE_COLLECTIVE = True
    np.testing.assert_array_equal(c_rccl, c_one)
    np.testing.assert_array_equal(ex_rccl["DM"], ex_one["DM"])
