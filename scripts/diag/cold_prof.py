"""Cold-start host profile of the 68-pulsar PTA: layouts, pack_toas, the session's uploads
(cProfile of pack_toas and of the upload calls, top entries by own time)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.getcwd())
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table, pack_toas

items = sim.make_pta(ntoas=10000, indices=list(range(68)))
for rep in range(2):
    t0 = time.perf_counter()
    s = Session(0)
    ts = time.perf_counter()
    lays = [build_layout(m, t) for m, t in items]
    t1 = time.perf_counter()
    pk = [pack_toas(l) for l in lays]
    t2 = time.perf_counter()
    for l, p in zip(lays, pk):
        s.add(l, p)
    t3 = time.perf_counter()
    tb = [pack_table(l, m) for l, (m, _) in zip(lays, items)]
    t4 = time.perf_counter()
    s.set_instances(list(zip(lays, tb)))
    s.check()
    t5 = time.perf_counter()
    print(f"rep {rep}: session {1e3 * (ts - t0):.1f} layout {1e3 * (t1 - ts):.1f} pack_toas {1e3 * (t2 - t1):.1f} "
          f"add {1e3 * (t3 - t2):.1f} pack_table {1e3 * (t4 - t3):.1f} set_instances {1e3 * (t5 - t4):.1f} ms")
    s.close()
lays = [build_layout(m, t) for m, t in items]
pr = cProfile.Profile()
pr.enable()
pk = [pack_toas(l) for l in lays]
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
s = Session(0)
pr = cProfile.Profile()
pr.enable()
for l, p in zip(lays, pk):
    s.add(l, p)
s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
s.check()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
s.close()
