"""bench.timed_steps with 1..3 pipelines on the 9-pulsar PTA (pulsars 0..8), beside the
plain round-robin loop of two_pipes.py, in one process."""
import os
import sys
import time
from collections import deque

import numpy as np

sys.path.insert(0, os.getcwd())
# (GPU_MAX_HW_QUEUES as the environment has it)
import bench
from pint_amd import _lib as L
from pint_amd import simulation as sim

PRE = int(sys.argv[1]) if len(sys.argv) > 1 else 0  # 68-pulsar sessions run and closed first
PRE_P = int(sys.argv[2]) if len(sys.argv) > 2 else PRE  # ... of which this many pipelines are run
PRE_N = int(sys.argv[3]) if len(sys.argv) > 3 else 68
if PRE:
    big = sim.make_pta(ntoas=10000, indices=list(range(PRE_N)))
    pre, _ = bench.pipelines(big, PRE)
    dt, _, _, _, mode, pp = bench.timed_steps(pre, 50, 5, lambda: None, lambda v: v, graph="0", gram_pass=False,
                                              pipes=PRE_P)
    print(f"prelude: {PRE} x {PRE_N} pulsars, {PRE_P} run, {dt / 50 * 1e3:.4f} ms per step")
    for s in pre:
        s.close()
    if os.environ.get("RELEASE_CACHE") == "1":
        L.lib().pint_release_cache()
        print("device buffer cache released")
items = sim.make_pta(ntoas=10000, indices=list(range(9)))
ss, _ = bench.pipelines(items, 3)
for p in (1, 2, 3):
    r = []
    for _ in range(3):
        dt, _, _, _, mode, pp = bench.timed_steps(ss, 200, 5, lambda: None, lambda v: v, graph="0", gram_pass=False,
                                                  pipes=p)
        r.append(dt / 200 * 1e3)
    print(f"timed_steps pipes={p} ({mode} x{pp}): ms per step {[round(x, 4) for x in r]}")
for _ in range(2):
    dt, _, _, _, mode, pp = bench.timed_steps(ss, 50, 5, lambda: None, lambda v: v, graph="0", gram_pass=False,
                                              pipes="auto")
    print(f"timed_steps auto -> {mode} x{pp}: {dt / 50 * 1e3:.4f} ms per step")
for s in ss:
    s.close()
