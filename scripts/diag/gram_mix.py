"""Gram time of the bench PTA against the same PTA with its DD pulsars made isolated: how
much of k_gram_v's time is the DD workgroups' makespan (12 MFMAs per k-step against 8)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pint_amd import simulation as sim  # noqa: E402
from pint_amd.engine import Session, build_layout, pack_table  # noqa: E402


def gram_ms(items):
    s = Session()
    lays = [s.add(build_layout(m, t)) for m, t in items]
    s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
    s.set_timing_mask(1 << 6)
    ts = []
    for _ in range(8):
        s.eval(want_M=Session.FIT)
        s.fit_step(1)
        s.check()
        ts.append(s.timing()[6])
    flags = sorted(set(tuple(s.vgram_layout(l)) for l in lays))
    s.close()
    return np.median(ts[2:]), flags


kind0 = sim.pta_kind
print("default mix: %.4f ms  layouts %s" % gram_ms(sim.make_pta(ntoas=10000, indices=list(range(68)))))
sim.pta_kind = lambda i: "" if kind0(i) == "DD" else kind0(i)
print("no DD:       %.4f ms  layouts %s" % gram_ms(sim.make_pta(ntoas=10000, indices=list(range(68)))))
