"""Diagnostic: batch vs single GLS chi2 with the blocked / column solves."""
import copy, sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(__file__)); sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
from golden_util import load
from pint_amd.fitter import BatchFit
a = load("pta_dd"); b = load("pta_ell1")
for blocked in (True, False):
    single = BatchFit([(copy.deepcopy(a[0]), a[1])], mode="gls"); single.s.set_blocked_solve(blocked)
    r1 = single.fit_plain(1)
    items = [((copy.deepcopy((a if k % 3 == 1 else b)[0])), (a if k % 3 == 1 else b)[1]) for k in range(37)]
    batch = BatchFit(items, mode="gls"); batch.s.set_blocked_solve(blocked)
    rs = batch.fit_plain(1)
    print("blocked", blocked, "single", r1[0].chi2, "batch", [rs[k].chi2 for k in (1, 4, 7)], "ell1", [rs[k].chi2 for k in (0, 2)])
    # sigma factors
    for bf, name in ((single, "single"), (batch, "batch")):
        bf.s.eval(want_M=2); bf.s.fit_step(1)
        import pint_amd._lib as L
        n = bf.s.L.pint_debug_read(bf.s.ctx, 2, None) if False else None
    single.close(); batch.close()
