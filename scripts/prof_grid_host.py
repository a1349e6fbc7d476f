"""Host-side profile of the NGC6440E 256x256 (F0, F1) grid leg (bench.py grid_leg)."""
import cProfile, pstats, sys, os, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from golden_util import load
from pint_amd import WLSFitter
from pint_amd.gridutils import grid_chisq
side = int(sys.argv[1]) if len(sys.argv) > 1 else 256
model, toas, _, _ = load("ngc6440e")
f = WLSFitter(toas, model)
f.fit_toas(maxiter=1)
F0, F1 = np.longdouble(f.model.F0.value), np.longdouble(f.model.F1.value)
g0 = F0 + np.linspace(-3, 3, side) * np.longdouble(f.model.F0.uncertainty)
g1 = F1 + np.linspace(-3, 3, side) * np.longdouble(f.model.F1.uncertainty)
for rep in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    t0 = time.perf_counter()
    grid_chisq(f, ("F0", "F1"), (g0, g1))
    print("grid", side, "rep", rep, round(time.perf_counter() - t0, 4), flush=True)
pr = cProfile.Profile()
pr.enable()
grid_chisq(f, ("F0", "F1"), (g0, g1))
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
