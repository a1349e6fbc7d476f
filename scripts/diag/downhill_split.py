"""Host/device time split of the C3 leg: DownhillGLSFitter.fit_toas(maxiter=10) on the
J0740 50k-TOA data (bench.py j0740_data).  Run under a kernel trace:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/profdh -o run -- \\
        python3 scripts/diag/downhill_split.py > gpurun_out/downhill_split.txt

then on the host:  python3 scripts/diag/downhill_split.py --trace gpurun_out/profdh/run_kernel_trace.csv
gpurun_out/downhill_split.txt -- the device-busy time (union of the kernel intervals) inside
each timed fit's [start, end] window (CLOCK_MONOTONIC ns, the trace's clock), and the rest
(host work and launch gaps)."""
import copy
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def run():
    from bench import j0740_data
    from pint_amd import DownhillGLSFitter
    model, toas, _ = j0740_data()
    for rep in range(4):
        f = DownhillGLSFitter(toas, copy.deepcopy(model))
        t0 = time.monotonic_ns()
        try:
            f.fit_toas(maxiter=10)
        except Exception as e:  # (the status is part of the record, not an error here)
            print("status", type(e).__name__, flush=True)
        t1 = time.monotonic_ns()
        print(f"fit {rep} {t0} {t1} {(t1 - t0) / 1e6:.2f} ms", flush=True)


def analyse(trace, log):
    ks = []
    for r in csv.DictReader(open(trace)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    ks.sort()
    agg = {}
    for line in open(log):
        if not line.startswith("fit "):
            continue
        _, rep, t0, t1, _, _ = line.split()
        t0, t1 = int(t0), int(t1)
        busy, cur_s, cur_e, n = 0, None, None, 0
        for s, e, _ in ks:
            if e <= t0 or s >= t1:
                continue
            s, e = max(s, t0), min(e, t1)
            n += 1
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        if int(rep) >= 1:
            for s, e, nm in ks:
                if s >= t0 and e <= t1:
                    agg.setdefault(nm, [0, 0])
                    agg[nm][0] += 1
                    agg[nm][1] += e - s
        print(f"fit {rep}: wall {(t1 - t0) / 1e6:.2f} ms, device busy {busy / 1e6:.2f} ms "
              f"({100.0 * busy / (t1 - t0):.0f} %), {n} kernels; host + gaps {(t1 - t0 - busy) / 1e6:.2f} ms")
    print("per fit (fits 1..), by kernel: launches, device ms")
    nf = 3
    for nm, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {nm[:60]:60s} {c / nf:6.1f} {t / nf / 1e6:8.3f}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--trace":
        analyse(sys.argv[2], sys.argv[3])
    else:
        run()
