"""Host profile of the reference-API single fits (C3 DownhillGLSFitter on J0740 50k TOAs,
C2 GLSFitter on B1855): one warm-up fit, then 3 fits under cProfile; prints the wall time
per fit and the top functions by total and cumulative time."""
import copy
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def prof(name, make, fit, n=3):
    f = make()
    fit(f)
    walls = []
    pr = cProfile.Profile()
    for _ in range(n):
        f = make()
        t0 = time.perf_counter()
        pr.enable()
        fit(f)
        pr.disable()
        walls.append(time.perf_counter() - t0)
    print(f"== {name}: wall per fit {[round(w * 1e3, 2) for w in walls]} ms", flush=True)
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


def main():
    from bench import j0740_data
    from pint_amd import DownhillGLSFitter, GLSFitter
    from pint_amd.fitter import MaxiterReached
    from pint_amd.toa import get_model_and_toas
    model, toas, _ = j0740_data()

    def dfit(f):
        try:
            f.fit_toas(maxiter=10)
        except MaxiterReached:
            pass
    prof("C3 DownhillGLSFitter J0740 50k", lambda: DownhillGLSFitter(toas, copy.deepcopy(model)), dfit)
    g = os.path.join(ROOT, "tests", "golden")
    m2, t2 = get_model_and_toas(os.path.join(g, "B1855+09_NANOGrav_9yv1.gls.par"),
                                os.path.join(g, "B1855+09_NANOGrav_9yv1.tim.gz"), ephem="builtin", include_bipm=False)
    prof("C2 GLSFitter B1855", lambda: GLSFitter(t2, copy.deepcopy(m2)), lambda f: f.fit_toas(maxiter=1))


if __name__ == "__main__":
    main()
