"""The bench's exact hot path pinned to the reference at full C5 shape.

Fixtures (oracle/refgen/gen_fullshape.py, the reference in the build container): the par
files of the bench's PTA pulsars 0 (isolated), 1 (ELL1) and 2 (DD) -- 100 DMX bins,
PLRedNoise with 30 modes, EFAC/EQUAD -- on 10,000 TOAs from the reference's own
make_fake_toas_uniform, with the arrays its GLSFitter.fit_toas forms (mtcm, mtcy, xhat, xvar,
norm, noise realisations, post-fit residuals and chi2, fitted values).

The GPU test fits them inside the bench's own batch: the 68-pulsar PTA of bench.py with
pulsars 0-2 replaced by the fixtures, so the N-split, the k_gram_v instantiation and the
per-instance path flags (vg + VB for the isolated and ELL1 pulsars, the slot tiles for DD)
are the ones that produce the headline number; it asserts those flags equal the bench
pulsars' and then applies the §8(a) stage bars: Gram 1e-12 relative to its diagonal, mtcy
1e-12, norms 1e-12, step / errors / covariance 1e-9 sigma, chi2 of the reference's post-fit
residuals 1e-9, noise realisations 1e-13 s.
"""
import os

import numpy as np
import pytest

from golden_util import GOLDEN, chi2_bar, load, ref_value, rms_ps

NAMES = ["c5_iso", "c5_ell1", "c5_dd"]
KIND = {"c5_iso": (0, ""), "c5_ell1": (1, "ELL1"), "c5_dd": (2, "DD")}


@pytest.mark.parametrize("name", NAMES)
def test_fixture_is_bench_pulsar(name):
    """The fixture's model is the bench's pulsar i (pint_amd.simulation.pta_par text)."""
    from pint_amd import simulation as sim
    i, kind = KIND[name]
    assert sim.pta_kind(i) == kind
    assert open(os.path.join(GOLDEN, name + ".par")).read() == sim.pta_par(i, kind, ndmx=100)
    model, toas, z, meta = load(name)
    assert toas.ntoas == 10000
    assert sum(1 for p in model.free_params if p.startswith("DMX_")) == 100
    assert model.TNREDC.value == 30


@pytest.mark.parametrize("name", NAMES)
def test_oracle_fullshape_residuals(name):
    """The CPU oracle's residuals of the full-shape fixture vs the reference's: 1 ns bar."""
    import pint_oracle as O
    model, toas, z, meta = load(name)
    r = O.residuals(O.from_product_model(model), O.toas_from_product(toas))
    err = np.max(np.abs(r["time"] - z["res_time"]))
    print(f"{name}: oracle residuals max |dr| {err:.2e} s")
    assert err < 1e-9


def _stage(z):
    return {k[len("stage_"):]: v for k, v in z.items() if k.startswith("stage_")}


@pytest.fixture(scope="module")
def bench_batch():
    """The bench's 68-pulsar batch with pulsars 0-2 replaced by the fixtures, one fit step on
    the reference's own pre-fit residuals (fixtures) / the device's (the rest)."""
    from pint_amd import simulation as sim
    from pint_amd.engine import Session, build_layout, pack_table
    fx = [load(n) for n in NAMES]
    bench_items = sim.make_pta(ntoas=10000, indices=list(range(68)))
    s = Session()
    # the bench's own pulsars 0-2 alone at the bench's batch shape: their path flags
    lays_b = [s.add(build_layout(m, t)) for m, t in bench_items]
    s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays_b, bench_items)])
    bench_flags = [s.vgram_layout(l) for l in lays_b[:3]]
    nsplit_bench = s.nsplit()
    items = [(m, t) for m, t, _, _ in fx] + bench_items[3:]
    lays = [s.add(build_layout(m, t)) for m, t in items[:3]] + lays_b[3:]
    s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
    out = {"s": s, "lays": lays, "fx": fx, "bench_flags": bench_flags, "nsplit_bench": nsplit_bench,
           "nsplit": s.nsplit(), "flags": [s.vgram_layout(l) for l in lays[:3]]}
    s.eval(want_M=Session.FIT)
    tr, _, _ = s.read_resids()
    s.debug_set_resids([z["res_time"] for _, _, z, _ in fx] + tr[3:])
    s.fit_step(1)
    out["gram"] = s.debug_gram()[:3]
    out["gram_pre"] = s.debug_gram(pre_ecorr=True)[:3]
    dp, er, cov, _ = s.read_step()
    out["step"] = (dp[:3], er[:3], cov[:3])
    out["noise"] = s.noise_resids()[:3]
    s.debug_set_resids([z["gls_post_resid"] for _, _, z, _ in fx] + tr[3:])
    out["chi2"] = s.chi2_gls()[:3].copy()
    yield out
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(3), ids=NAMES)
def test_fullshape_path_is_the_benchs(bench_batch, k):
    """The fixture takes the bench pulsar's path at the bench's N-split: k_gram_v with the
    same [T | r | slots] x [F] tile shape (NTR, NTC) and binned flag (isolated/ELL1: vg + VB,
    the k_gram_v<2,6,true> instantiation; DD: the slot tiles)."""
    b = bench_batch
    assert b["nsplit"] == b["nsplit_bench"]
    vg, ns, kpv, r0 = b["flags"][k]
    assert b["flags"][k] == b["bench_flags"][k], (b["flags"][k], b["bench_flags"][k])
    ntr, ntc, vb = (r0 + 1 + ns) // 16, kpv // 16, bool(vg & 2)
    print(f"{NAMES[k]}: vg {vg} NTR {ntr} NTC {ntc} VB {vb} nsplit {b['nsplit']}")
    assert vg & 1
    if k < 2:
        assert (ntr, ntc, vb) == (2, 6, True)
    else:
        assert not vb


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(3), ids=NAMES)
def test_fullshape_stage(bench_batch, k):
    """Gram, mtcy, norms, step, errors, covariance, noise realisations and the chi2 of the
    reference's post-fit residuals against the reference's GLSFitter arrays."""
    b = bench_batch
    name = NAMES[k]
    model, toas, z, meta = b["fx"][k]
    st = _stage(z)
    lay = b["lays"][k]
    K = lay.K
    assert K == int(st["K"][0]), (K, st["K"])
    G, colsq = b["gram"][k]
    Gpre, _ = b["gram_pre"][k]
    norm = np.sqrt(colsq)
    nref = st["norm"]
    assert np.max(np.abs(norm / nref - 1)) < 1e-12
    Af = np.zeros((K, K))
    Af[np.triu_indices(K)] = st["mtcm_tr_triu"]
    Af = Af + np.triu(Af, 1).T
    d = np.sqrt(np.diag(Af))
    phi_dev = np.zeros(K)
    nc = len(lay.columns)
    phi_dev[nc:] = 1.0 / np.asarray(lay.red_phi) / norm[nc:] ** 2
    An = Gpre[:K, :K] / np.outer(norm, norm) + np.diag(phi_dev)
    dA = np.max(np.abs(An - Af) / np.outer(d, d))
    db = np.max(np.abs(Gpre[:K, K] / norm - st["mtcy"]) / (d * np.sqrt(Gpre[K, K])))
    dp, er, cov = (x[k] for x in b["step"])
    eref = np.sqrt(np.diag(st["xvar_tr"])) / nref
    ds = np.max(np.abs(dp[:K] - st["xhat"] / nref) / eref)
    de = np.max(np.abs(er[:K] / eref - 1))
    cref = st["xvar_tr"][:nc, :nc] / np.outer(nref[:nc], nref[:nc])
    dc = np.max(np.abs(cov - cref) / np.outer(eref[:nc], eref[:nc]))
    nz = b["noise"][k]["pl_red_noise"]
    dn = np.max(np.abs(nz - z["gls_noise_pl_red_noise"]))
    c2 = b["chi2"][k]
    dchi = abs(c2 / meta["post_chi2"] - 1)
    print(f"{name}: K {K} gram {dA:.2e} mtcy {db:.2e} step {ds:.2e} sigma errs {de:.2e} cov {dc:.2e} "
          f"noise {dn:.2e} s chi2 {dchi:.2e}")
    assert dA <= 1e-12 and db <= 1e-12
    assert ds <= 1e-9 and de <= 1e-9 and dc <= 1e-9
    assert dn <= 1e-13
    assert dchi <= 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_fullshape_gls_fit(name):
    """GLSFitter.fit_toas(maxiter=1) end to end vs the reference's fit: parameters 1e-3 sigma,
    uncertainties 1e-6, chi2 within 2x the reference's own spread at the measured post-fit
    residual rms (golden_util.chi2_bar)."""
    from pint_amd import GLSFitter
    model, toas, z, meta = load(name)
    f = GLSFitter(toas, model)
    c2 = f.fit_toas(maxiter=1)
    worst = max(abs(float((np.longdouble(f.model[p].value) - ref_value(meta, "gls_params", p))
                          / np.longdouble(meta["gls_errors"][p]))) for p in meta["gls_params"])
    eu = max(abs(f.model[p].uncertainty / meta["gls_errors"][p] - 1) for p in meta["gls_params"])
    print(f"{name}: params {worst:.2e} sigma, errors {eu:.2e}, chi2 {c2 / meta['gls_chi2'] - 1:.2e}")
    assert worst < 1e-3 and eu < 1e-6
    bar = chi2_bar(name, "fit", rms_ps(f.resids.time_resids, z["gls_post_resid"]))
    assert abs(c2 / meta["gls_chi2"] - 1) < bar, (c2 / meta["gls_chi2"] - 1, bar)
