"""The first synchronous fit of a fresh 68-pulsar session, call by call (ms), in three
sessions made one after another in one process (bench.cold_start's sequence).
    python3 scripts/diag/cold_after.py [nogc] [nohuge] [pinout]
(nohuge: numpy's hugepage madvise off; pinout: read_step into page-locked buffers, not fresh
pageable arrays)"""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table

items = sim.make_pta(ntoas=10000, indices=list(range(68)))
if "nohuge" in sys.argv[1:]:
    import numpy as np
    np._core.multiarray._set_madvise_hugepage(False)
    print("numpy hugepage madvise off")
if "nogc" in sys.argv[1:]:
    import gc
    gc.collect()
    gc.disable()
    print("garbage collector off")
for rep in range(3):
    s = Session(0)
    lays = [s.add(build_layout(m, t)) for m, t in items]
    s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
    s.check()
    T = [time.perf_counter()]
    s.eval(want_M=Session.FIT); T.append(time.perf_counter())
    s.fit_step_apply(1, 1.0); T.append(time.perf_counter())
    if "pinout" in sys.argv[1:]:
        s.lazy = True  # (Python side only: read_step's outputs from the pinned per-name pool)
        s.read_step()
        s.lazy = False
    else:
        s.read_step()
    T.append(time.perf_counter())
    s.noise_resids(); T.append(time.perf_counter())
    s.eval(want_M=False); T.append(time.perf_counter())
    s.chi2_gls(); T.append(time.perf_counter())
    s.check(); T.append(time.perf_counter())
    d = [round((b - a) * 1e3, 2) for a, b in zip(T, T[1:])]
    print(f"session {rep}: eval(FIT) {d[0]} step+apply {d[1]} read_step {d[2]} noise {d[3]} eval {d[4]} chi2 {d[5]} check {d[6]}  total {sum(d):.2f} ms")
    s.close()
