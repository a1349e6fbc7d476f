"""Concurrent step pipelines on one GPU (DESIGN.md §3 "Round 6").

One batch of pulsars held by several Sessions -- each with its own HIP streams and device
buffers -- whose GLSFitter.fit_toas(maxiter=1) steps (Session.fit_step_enqueue: restore,
evaluation, Gram, solve with the update, outputs, noise realisations, post-fit chi2) are
enqueued round-robin, each session pipelined L.NSLOT steps deep.  Steps of different
sessions are independent and overlap on the device: a small batch's step is a chain of
latency-bound kernels that leaves most of the chip idle (two 9-pulsar pipelines 0.10 ms per
step against 0.17 for one; bench.py --pipes measures it).  Every step is a full fit of the
batch from its initial models, with the same kernels and bits as a lone session's.

Streams are pooled per device and role (libpint_hip.so), so sessions made and closed in
turn keep the first sessions' hardware-queue mapping; leave GPU_MAX_HW_QUEUES at its default
(4): with more queues than the scheduler maps at once, concurrent sessions run slower than
one.
"""
from collections import deque
from typing import Callable, Optional, Sequence

import numpy as np

from . import _lib as L
from .engine import Session, pack_table


class StepPipelines:
    """items: [(model, toas)] -- the batch, uploaded once per pipeline; n: pipelines.

    enqueue() puts one step on the next pipeline and returns its step number; a step's
    outputs (pinned views that the step's slot reuses) are handed to on_done(step, outputs)
    when the step is retired -- when its slot comes round again, or at drain() -- so the
    callback copies what it keeps.  outputs = (steps, errors, covariances, linearised chi2,
    noise views or None, post-fit chi2), per instance in `items` order."""

    def __init__(self, items: Sequence[tuple], n: int = 2, device: int = 0,
                 on_done: Optional[Callable] = None):
        if n < 1:
            raise ValueError("StepPipelines needs at least one pipeline")
        self.sessions = []
        try:
            for _ in range(n):
                s = Session(device)
                lays = s.add_all(items)
                s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
                s.save_tables()  # every step fits from these initial models
                s.set_lazy(True)
                s.set_timing_mask(0)
                self.sessions.append(s)
        except Exception:
            self.close()
            raise
        self.on_done = on_done
        self._pend = [deque() for _ in self.sessions]
        self._next = 0
        self._count = 0

    def enqueue(self, lam: float = 1.0) -> int:
        k = self._next
        self._next = (k + 1) % len(self.sessions)
        if len(self._pend[k]) >= L.NSLOT:
            self._retire(k)
        slot, (dp, er, cov, cl), nz, c2 = self.sessions[k].fit_step_enqueue(restore=True, lam=lam)
        step = self._count
        self._count += 1
        self._pend[k].append((step, slot, (dp, er, cov, cl, nz, c2)))
        return step

    def _retire(self, k: int):
        step, slot, out = self._pend[k].popleft()
        self.sessions[k].check_step(slot)
        if self.on_done is not None:
            self.on_done(step, out)

    def drain(self):
        """Retire every step in flight, oldest first across the pipelines."""
        while any(self._pend):
            k = min((q[0][0], i) for i, q in enumerate(self._pend) if q)[1]
            self._retire(k)

    def close(self):
        for s in self.sessions:
            s.close()
        self.sessions = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        try:
            if self.sessions and not any(exc):
                self.drain()
        finally:
            self.close()
