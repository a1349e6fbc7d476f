"""Reference CPU timings in this container (TEST/BENCH INFRASTRUCTURE; container only).

Times the reference (PINT at /root/reference, offline recipe of SURVEY.md §8(c)) on the
configs of BASELINE.json and writes bench/reference_cpu.json.  The reference cannot travel
to the GPU box, so this row is measured here and committed; bench.py reports it beside the
GPU numbers and the port's CPU rate measured on the GPU box's own host cores.

Usage: oracle/refenv/run_ref.sh oracle/refgen/bench_ref.py
"""
import copy
import io
import json
import os
import platform
import time

import numpy as np
import astropy.units as u

from refcommon import REPO, REFDATA, register_clockless_sites
import pint.simulation as sim
import pint.toa as toa
from pint.models import get_model
from pint.fitter import GLSFitter, WLSFitter, DownhillGLSFitter
from pint.gridutils import grid_chisq

import gen_synth


def timed(fn, reps=1):
    ts = []
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), out


def cpu_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    register_clockless_sites()
    rows = []
    ncores = len(os.sched_getaffinity(0))

    # C1: NGC6440E WLS fit and (F0, F1) grids, serial and ProcessPoolExecutor(ncores)
    model = get_model(f"{REFDATA}/NGC6440E.par")
    toas = toa.get_TOAs(f"{REFDATA}/NGC6440E.tim", ephem="builtin", include_bipm=False, planets=False,
                        model=model)
    t, _ = timed(lambda: WLSFitter(toas, copy.deepcopy(model)).fit_toas(maxiter=1), reps=5)
    rows.append(dict(config="C1", workload="NGC6440E WLSFitter.fit_toas (62 TOAs)", seconds=t,
                     rate=1 / t, unit="fits/s", cores=1))
    f = WLSFitter(toas, copy.deepcopy(model))
    f.fit_toas()
    side = 8
    g0 = f.model.F0.quantity + np.linspace(-3, 3, side) * f.model.F0.uncertainty
    g1 = f.model.F1.quantity + np.linspace(-3, 3, side) * f.model.F1.uncertainty
    for ncpu in (1, ncores):
        ff = WLSFitter(toas, copy.deepcopy(f.model))
        t, _ = timed(lambda: grid_chisq(ff, ("F0", "F1"), (g0, g1), ncpu=ncpu, printprogress=False))
        rows.append(dict(config="C1/C4", workload=f"NGC6440E grid_chisq {side}x{side} (F0,F1) WLSFitter, ncpu={ncpu}",
                         seconds=t, rate=side * side / t, unit="points/s", cores=ncpu))

    # C2: B1855+09 9-yr GLS fit
    model = get_model(f"{REFDATA}/B1855+09_NANOGrav_9yv1.gls.par")
    toas = toa.get_TOAs(f"{REFDATA}/B1855+09_NANOGrav_9yv1.tim", ephem="builtin", include_bipm=False,
                        planets=False, model=model)
    t, _ = timed(lambda: GLSFitter(toas, copy.deepcopy(model)).fit_toas(maxiter=1))
    rows.append(dict(config="C2", workload="B1855+09 9-yr GLSFitter.fit_toas (4005 TOAs, ECORR + PLRedNoise)",
                     seconds=t, rate=1 / t, unit="fits/s", cores=1))

    # C5 unit: one synthetic PTA pulsar, 10k TOAs, red noise + 20 DMX (gen_synth template)
    np.random.seed(0)
    model = get_model(io.StringIO(gen_synth.pta_par(0, "")))
    t_gen, ts = timed(lambda: sim.make_fake_toas_uniform(
        53000, 56652, 10000, model, freq=np.array([800, 1200, 1600, 2000]) * u.MHz, obs="geocenter",
        error=0.5 * u.us, add_noise=True, add_correlated_noise=True, include_bipm=False,
        multi_freqs_in_epoch=False))
    t, _ = timed(lambda: GLSFitter(ts, copy.deepcopy(model)).fit_toas(maxiter=1))
    rows.append(dict(config="C5 unit", workload="synthetic PTA pulsar, 10k TOAs, GLSFitter.fit_toas (maxiter=1)",
                     seconds=t, rate=1 / t, unit="fits/s", cores=1,
                     note=f"x68 pulsars = {68 * t:.0f} s per PTA sweep on one core; make_fake_toas took {t_gen:.1f} s"))

    # C3/C4: J0740 synthetic 10k TOAs (the 50k of C3 is out of reach of the CPU path's memory/time)
    np.random.seed(0)
    model = gen_synth.j0740_model()
    tj = sim.make_fake_toas_uniform(56640, 58461, 10000, model, freq=np.array([820, 1400]) * u.MHz,
                                    obs="geocenter", error=1 * u.us, add_noise=True, include_bipm=False,
                                    multi_freqs_in_epoch=False, flags={"f": "Rcvr1_2_GUPPI", "fe": "Rcvr1_2"})
    model.find_empty_masks(tj, freeze=True)
    def down():
        fd = DownhillGLSFitter(tj, copy.deepcopy(model))
        try:
            fd.fit_toas(maxiter=10)
        except Exception:
            pass
    t, _ = timed(down)
    rows.append(dict(config="C3", workload="J0740 synthetic 10k TOAs DownhillGLSFitter.fit_toas (maxiter=10)",
                     seconds=t, rate=1 / t, unit="fits/s", cores=1))
    g = GLSFitter(tj, copy.deepcopy(model))
    g.fit_toas()
    m2 = np.linspace(0.2, 0.3, 2) * u.Msun
    sini = np.sin(np.deg2rad(np.linspace(86.25, 88.5, 2))) * u.dimensionless_unscaled
    t, _ = timed(lambda: grid_chisq(g, ("M2", "SINI"), (m2, sini), ncpu=1, printprogress=False))
    rows.append(dict(config="C3/C4", workload="J0740 synthetic 10k TOAs grid_chisq 2x2 (M2,SINI) GLSFitter, ncpu=1",
                     seconds=t, rate=4 / t, unit="points/s", cores=1))

    out = dict(host=dict(cpu=cpu_name(), cores=ncores, python=platform.python_version(), numpy=np.__version__,
                         note="reference PINT (pure Python) on the offline recipe: ephem=builtin, no clock files"),
               rows=rows)
    os.makedirs(os.path.join(REPO, "bench"), exist_ok=True)
    with open(os.path.join(REPO, "bench", "reference_cpu.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for r in rows:
        print(f"{r['config']:8s} {r['rate']:10.4f} {r['unit']:9s} {r['seconds']:8.2f} s  {r['workload']}")


if __name__ == "__main__":
    main()
