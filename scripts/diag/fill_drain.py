"""Fill/drain of the timed region: bench.timed_steps' wall time T(K) for K steps of the
68-pulsar step (1 and 2 pipelines, direct launches), so T(K) = a + b K separates the
per-run constant a from the per-step time b."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import bench
from pint_amd import simulation as sim

NPSR = int(sys.argv[1]) if len(sys.argv) > 1 else 68
items = sim.make_pta(ntoas=10000, indices=list(range(NPSR)))
ss, _ = bench.pipelines(items, 2)
for p in (1, 2):
    ks, ts = [], []
    for K in (10, 20, 40, 100, 200):
        r = []
        for _ in range(3):
            dt, _, _, _, mode, pp = bench.timed_steps(ss, K, 5, lambda: None, lambda v: v, graph="0", gram_pass=False,
                                                      pipes=p)
            r.append(dt)
        ks.append(K)
        ts.append(float(np.median(r)))
        print(f"{NPSR} psr x{p}: K {K:4d}  T {ts[-1] * 1e3:8.3f} ms  per step {ts[-1] / K * 1e3:.4f} ms")
    b, a = np.polyfit(ks, ts, 1)
    print(f"   fit T = {a * 1e3:.3f} ms + K x {b * 1e3:.4f} ms")
for s in ss:
    s.close()
