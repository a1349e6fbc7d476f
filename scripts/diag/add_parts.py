"""pint_add_pulsar_cols of the 68-pulsar PTA split: the library's host packer alone
(pint_pack_toas into reused buffers) vs the whole add (packer + staging + per-pulsar set-up),
and the staged upload's commit (check).  Two fresh sessions; ms for 68 pulsars."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
from pint_amd import _lib as L
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_cols

items = sim.make_pta(ntoas=10000, indices=list(range(68)))
lib = L.lib()
for rep in range(2):
    lays = [build_layout(m, t) for m, t in items]
    cols = [pack_cols(l) for l in lays]
    n = max(l.n for l in lays)
    D = np.zeros(15 * (n + 1))
    F, J, I = np.zeros(n + 1, np.uint32), np.zeros(n + 1, np.uint64), np.zeros(2 * (n + 1), np.int32)
    t0 = time.perf_counter()
    for (c, _), l in zip(cols, lays):
        m = l.n + 1
        t = L.ToasT(l.n, *[L.ptr(D[k * m:]) for k in range(4)], L.ptr(D[6 * m:]), L.ptr(D[9 * m:]),
                    L.ptr(D[12 * m:]), L.ptr(D[4 * m:]), L.ptr(D[5 * m:]), L.ptr(F, C.c_uint32),
                    L.ptr(J, C.c_uint64), L.ptr(I, C.c_int32), L.ptr(I[m:], C.c_int32), None, None)
        lib.pint_pack_toas(C.byref(c), C.byref(t), None, 0)
    t1 = time.perf_counter()
    s = Session(0)
    t2 = time.perf_counter()
    for l, pk in zip(lays, cols):
        s.add(l, pk)
    t3 = time.perf_counter()
    s.check()
    t4 = time.perf_counter()
    print(f"rep {rep}: packer alone {1e3 * (t1 - t0):.2f}  add (packer + staging + set-up) {1e3 * (t3 - t2):.2f}  "
          f"check {1e3 * (t4 - t3):.2f} ms")
    s.close()
