"""The k_gram_v layouts of the bench PTA: (r0 = timing columns, vns DMX slots, kpv, nred) per pulsar."""
import sys, os
from collections import Counter
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table

models = [sim.pta_model(i) for i in range(68)]
items = sim.make_pta(ntoas=10000, indices=list(range(68)), models=models)
s = Session(device=0)
lays = [s.add(build_layout(m, t)) for m, t in items]
s.set_instances(list(zip(lays, [pack_table(l, m) for l, (m, _) in zip(lays, items)])))
c = Counter()
for l in lays:
    vg, ns, kpv, r0 = s.vgram_layout(l)
    c[(vg, r0, ns, kpv, l.nred, l.K)] += 1
print("nsplit", s.nsplit())
for k, v in sorted(c.items()):
    print("vg %d r0 %d ns %d kpv %d nred %d K %d : %d pulsars" % (k + (v,)))
s.close()
