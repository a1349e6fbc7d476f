"""Python-side profile of grid_chisq on the 256 x 256 NGC6440E (F0, F1) grid (the bench's
grid leg): cProfile over 20 grids after warm-up, by own time; the device wait is check()."""
import copy
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from golden_util import load
from pint_amd import WLSFitter
from pint_amd.gridutils import grid_chisq

model, toas, _, _ = load("ngc6440e")
f = WLSFitter(toas, copy.deepcopy(model))
f.fit_toas(maxiter=1)
F0, F1 = np.longdouble(f.model.F0.value), np.longdouble(f.model.F1.value)
g0 = F0 + np.linspace(-3, 3, 256) * np.longdouble(f.model.F0.uncertainty)
g1 = F1 + np.linspace(-3, 3, 256) * np.longdouble(f.model.F1.uncertainty)
for _ in range(3):
    grid_chisq(f, ("F0", "F1"), (g0, g1))
ts = []
for _ in range(20):
    t = time.perf_counter()
    grid_chisq(f, ("F0", "F1"), (g0, g1))
    ts.append(time.perf_counter() - t)
print(f"grid wall median {np.median(ts) * 1e3:.3f} ms")
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    grid_chisq(f, ("F0", "F1"), (g0, g1))
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
