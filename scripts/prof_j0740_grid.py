"""Host/device time split of the J0740 (M2,SINI) grid leg (bench.py j0740_legs)."""
import cProfile, pstats, sys, time, os, copy
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pint_amd import GLSFitter
from pint_amd.gridutils import grid_chisq
from bench import j0740_data
side = int(sys.argv[1]) if len(sys.argv) > 1 else 16
model, toas, _ = j0740_data()
g = GLSFitter(toas, copy.deepcopy(model))
g.fit_toas(maxiter=1)
m2 = np.linspace(0.2, 0.3, side)
sini = np.sin(np.deg2rad(np.linspace(86.25, 88.5, side)))
for rep in range(3):
    t0 = time.perf_counter()
    grid_chisq(g, ("M2", "SINI"), (m2, sini))
    print("grid", side, "rep", rep, time.perf_counter() - t0, flush=True)
pr = cProfile.Profile()
pr.enable()
grid_chisq(g, ("M2", "SINI"), (m2, sini))
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
