"""Single-fit legs A/B (VERDICT r5 ask 2): C3 DownhillGLSFitter(maxiter=10) on the J0740
50k-TOA data and the C2 single GLSFitter fit of B1855, wall per fit, then a cProfile of one
Downhill fit (the host functions that own the time).  Runs unchanged in an older tree (it
uses only the public fitter API and bench.j0740_data):

    python3 scripts/diag/ab_single.py [--prof]
"""
import copy
import cProfile
import os
import pstats
import sys
import time

ROOT = os.environ.get("AB_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from bench import j0740_data
    from pint_amd import DownhillGLSFitter, GLSFitter
    from pint_amd.toa import get_model_and_toas
    model, toas, _ = j0740_data()
    dts = []
    for rep in range(6):
        f = DownhillGLSFitter(toas, copy.deepcopy(model))
        t0 = time.perf_counter()
        try:
            f.fit_toas(maxiter=10)
        except Exception as e:
            print("status", type(e).__name__, flush=True)
        dts.append((time.perf_counter() - t0) * 1e3)
    print(f"[{ROOT}] C3 downhill ms: {[round(x, 2) for x in dts]}", flush=True)
    g = os.path.join(ROOT, "tests", "golden")
    m2, t2 = get_model_and_toas(os.path.join(g, "B1855+09_NANOGrav_9yv1.gls.par"),
                                os.path.join(g, "B1855+09_NANOGrav_9yv1.tim.gz"), ephem="builtin",
                                include_bipm=False)
    dts = []
    for rep in range(6):
        f = GLSFitter(t2, copy.deepcopy(m2))
        t0 = time.perf_counter()
        f.fit_toas(maxiter=1)
        dts.append((time.perf_counter() - t0) * 1e3)
    print(f"[{ROOT}] C2 single ms: {[round(x, 2) for x in dts]}", flush=True)
    if "--prof" in sys.argv:
        f = DownhillGLSFitter(toas, copy.deepcopy(model))
        pr = cProfile.Profile()
        pr.enable()
        f.fit_toas(maxiter=10)
        pr.disable()
        st = pstats.Stats(pr)
        st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
