"""Host time of the stages of one NGC6440E 256 x 256 grid_chisq call (wrappers around the
gridutils / BatchFit / Session entry points), averaged over 20 grids after 3 warm-ups."""
import functools
import os
import sys
import time
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pint_amd import _lib
_lib.lib()
from golden_util import load
from pint_amd import WLSFitter, gridutils, fitter, engine
from pint_amd.gridutils import grid_chisq

acc = defaultdict(float)


def wrap(obj, name, label):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[label] += time.perf_counter() - t0
    setattr(obj, name, g)


for obj, name in [(gridutils, "_grid_session"), (gridutils, "meshgrid_axes"), (gridutils, "_fit_block"),
                  (gridutils, "gather_blocks"), (engine, "pack_table"),
                  (fitter.BatchFit, "__init__"), (fitter.BatchFit, "fit_plain"), (fitter.BatchFit, "_step"),
                  (fitter.BatchFit, "_eval"), (fitter.BatchFit, "_chi2_now"),
                  (engine.Session, "set_grid"), (engine.Session, "eval"), (engine.Session, "fit_step"),
                  (engine.Session, "apply_step_uniform"), (engine.Session, "read_chi2"),
                  (engine.Session, "_after_set")]:
    wrap(obj, name, f"{getattr(obj, '__name__', '')}.{name}")
gridutils.pack_table = engine.pack_table
model, toas, _, _ = load("ngc6440e")
f = WLSFitter(toas, model)
f.fit_toas(maxiter=1)
F0, F1 = np.longdouble(f.model.F0.value), np.longdouble(f.model.F1.value)
g0 = F0 + np.linspace(-3, 3, 256) * np.longdouble(f.model.F0.uncertainty)
g1 = F1 + np.linspace(-3, 3, 256) * np.longdouble(f.model.F1.uncertainty)
for _ in range(3):
    grid_chisq(f, ("F0", "F1"), (g0, g1))
acc.clear()
N = 20
t0 = time.perf_counter()
for _ in range(N):
    grid_chisq(f, ("F0", "F1"), (g0, g1))
tot = (time.perf_counter() - t0) / N
print(f"grid_chisq {tot * 1e6:.0f} us per grid")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:40s} {v / N * 1e6:8.0f} us")
