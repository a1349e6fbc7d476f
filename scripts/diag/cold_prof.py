"""Host profile of the cold-start packing (build_layout + pack_toas) of the bench PTA."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pint_amd import _lib
_lib.lib()
from pint_amd import simulation as sim
from pint_amd.engine import build_layout, pack_toas

models = [sim.pta_model(i) for i in range(68)]
items = sim.make_pta(ntoas=10000, indices=list(range(68)), models=models)
for rep in range(2):
    t0 = time.perf_counter()
    lays = [build_layout(m, t) for m, t in items]
    t1 = time.perf_counter()
    pk = [pack_toas(l) for l in lays]
    t2 = time.perf_counter()
    print(f"layout {1e3 * (t1 - t0):.1f} ms  pack {1e3 * (t2 - t1):.1f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
lays = [build_layout(m, t) for m, t in items]
pk = [pack_toas(l) for l in lays]
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
