"""bench.timed_steps' pipeline logic on the host (no GPU): a stand-in session records the
order of enqueues and retirements.  Checks that steps go round-robin over the pipelines, that
a pipeline's slot is retired before it is reused and every step is retired by the end, that
the trial times each candidate twice and keeps the fastest, and that a fixed count is used
as given."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class FakeSession:
    """The Session calls timed_steps makes; each 'step' costs `cost` seconds of host sleep
    divided by the number of pipelines the run uses (a stand-in for overlap)."""

    log = []

    def __init__(self, name, nslot):
        self.name, self.nslot = name, nslot
        self.next, self.pending = 0, []
        self.enqueued = self.retired = 0

    def save_tables(self):
        pass

    def set_lazy(self, on):
        assert on

    def set_timing_mask(self, m):
        pass

    def set_timing_every(self, k):
        pass

    def timing(self):
        return [0.0] * 8

    def fit_step_enqueue(self, restore=True, lam=1.0):
        assert len(self.pending) < self.nslot, "enqueue into a slot whose step was never checked"
        sl = self.next
        self.next = (sl + 1) % self.nslot
        self.pending.append(sl)
        self.enqueued += 1
        FakeSession.log.append(("enq", self.name))
        return sl, None, None, None

    def check_step(self, sl):
        assert self.pending and self.pending[0] == sl, "steps retired out of order"
        self.pending.pop(0)
        self.retired += 1


@pytest.fixture
def bench_mod(monkeypatch):
    import bench
    from pint_amd import _lib as L
    from pint_amd import engine
    monkeypatch.setattr(engine, "Session", FakeSession)  # (timed_steps' isinstance check)
    FakeSession.log = []
    return bench, L.NSLOT


def test_round_robin_and_every_step_retired(bench_mod):
    bench, nslot = bench_mod
    ss = [FakeSession("a", nslot), FakeSession("b", nslot)]
    dt, _, _, _, mode, p = bench.timed_steps(ss, 21, 3, lambda: None, lambda v: v, graph="0", gram_pass=False,
                                             pipes=2)
    assert (mode, p) == ("direct", 2)
    for s in ss:
        assert s.enqueued == s.retired and not s.pending
    timed = [n for k, n in FakeSession.log[-21:]]
    assert timed == [("a", "b")[i % 2] for i in range(21)]


def test_fixed_pipeline_count_uses_the_first_sessions(bench_mod):
    bench, nslot = bench_mod
    ss = [FakeSession("a", nslot), FakeSession("b", nslot)]
    _, _, _, _, _, p = bench.timed_steps(ss, 10, 2, lambda: None, lambda v: v, graph="0", gram_pass=False, pipes=1)
    assert p == 1
    assert [n for _, n in FakeSession.log[-10:]] == ["a"] * 10


def test_trial_keeps_the_fastest_candidate(bench_mod, monkeypatch):
    bench, nslot = bench_mod
    ss = [FakeSession("a", nslot), FakeSession("b", nslot)]
    clock = {"t": 0.0}

    def fake_clock():
        return clock["t"]

    orig = FakeSession.fit_step_enqueue

    def enq(self, restore=True, lam=1.0):
        # two pipelines: half the cost per step
        npipe = 2 if any(s.pending for s in ss if s is not self) else 1
        clock["t"] += 1.0 / npipe
        return orig(self, restore, lam)

    monkeypatch.setattr(FakeSession, "fit_step_enqueue", enq)
    monkeypatch.setattr(bench.time, "perf_counter", fake_clock)
    _, _, _, _, mode, p = bench.timed_steps(ss, 40, 2, lambda: None, lambda v: v, graph="0", gram_pass=False,
                                            pipes="auto")
    assert (mode, p) == ("direct", 2)
