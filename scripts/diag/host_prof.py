"""Host profile of the single-fit legs: cProfile over K C3 DownhillGLSFitter(maxiter=10)
fits (J0740 50k TOAs) and K C2 GLSFitter(maxiter=1) fits of B1855, printed per fit in us
(tottime includes the ctypes calls a function makes: they are not profiled entries).

    python3 scripts/diag/host_prof.py [K]
"""
import copy
import cProfile
import os
import pstats
import sys
import time

ROOT = os.environ.get("AB_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def show(pr, k, title):
    st = pstats.Stats(pr)
    rows = []
    for (f, ln, fn), (cc, nc, tt, ct, _) in st.stats.items():
        rows.append((tt, ct, nc, f"{os.path.basename(f)}:{ln}({fn})"))
    print(f"== {title}: top tottime (us per fit), calls per fit, cumtime")
    for tt, ct, nc, name in sorted(rows, reverse=True)[:30]:
        print(f"  {tt / k * 1e6:9.1f} {nc / k:7.1f} {ct / k * 1e6:9.1f}  {name}")


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    from bench import j0740_data
    from pint_amd import DownhillGLSFitter, GLSFitter
    from pint_amd.toa import get_model_and_toas
    model, toas, _ = j0740_data()
    for _ in range(2):
        DownhillGLSFitter(toas, copy.deepcopy(model)).fit_toas(maxiter=10)
    fs = [DownhillGLSFitter(toas, copy.deepcopy(model)) for _ in range(k)]
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for f in fs:
        f.fit_toas(maxiter=10)
    pr.disable()
    print(f"C3 downhill: {(time.perf_counter() - t0) / k * 1e3:.2f} ms per fit (profiled)")
    show(pr, k, "C3")
    g = os.path.join(ROOT, "tests", "golden")
    m2, t2 = get_model_and_toas(os.path.join(g, "B1855+09_NANOGrav_9yv1.gls.par"),
                                os.path.join(g, "B1855+09_NANOGrav_9yv1.tim.gz"), ephem="builtin",
                                include_bipm=False)
    for _ in range(2):
        GLSFitter(t2, copy.deepcopy(m2)).fit_toas(maxiter=1)
    fs = [GLSFitter(t2, copy.deepcopy(m2)) for _ in range(k)]
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for f in fs:
        f.fit_toas(maxiter=1)
    pr.disable()
    print(f"C2 single: {(time.perf_counter() - t0) / k * 1e3:.2f} ms per fit (profiled)")
    show(pr, k, "C2")


if __name__ == "__main__":
    main()
