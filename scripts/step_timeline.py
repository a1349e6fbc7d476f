"""Per-step kernel timeline from a rocprofv3 kernel trace of the bench (PTA leg only):
    python scripts/step_timeline.py gpurun_out/profq/run_kernel_trace.csv
Finds the steady-state steps (one k_gram_v group launch per step), and prints for the median
step each dispatch's start offset, duration and the idle gap before it (queue 0 = the main
stream; the copy-stream kernels are listed with their stream)."""
import csv
import sys
from collections import defaultdict

import numpy as np


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "")[:40]


rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
               r.get("Queue_Id", r.get("Stream_Id", "?"))))
ks.sort()
# steps start at the table reset (k_prep) or, when the restore is folded into it (round 4),
# at the evaluation with M
def _is_start(name):
    return name.startswith("k_prep") or name.startswith("k_eval_mix_w<1") or name.startswith("k_eval_mix<1")


starts = []
for i, k in enumerate(ks):
    if _is_start(k[2]) and not (starts and ks[starts[-1]][2].startswith("k_prep") and i == starts[-1] + 1):
        starts.append(i)
steps = []
for a, b in zip(starts, starts[1:]):
    seg = ks[a:b]
    if any(k[2].startswith("k_gram_v") for k in seg):
        steps.append(seg)
steps = steps[len(steps) // 3:]  # steady state
dur = [s[-1][1] - s[0][0] for s in steps]
med = steps[int(np.argsort(dur)[len(dur) // 2])]
print(f"{len(steps)} steady steps; span median {np.median(dur) / 1e3:.1f} us (min {min(dur) / 1e3:.1f})")
# the device's step interval: consecutive steps' first dispatches (with several pipelines
# the steps of the sessions interleave, and a step's span is its latency, not the interval)
st0 = np.array(sorted(s[0][0] for s in steps), dtype=np.float64)
if len(st0) > 2:
    print(f"step interval (start to start): median {np.median(np.diff(st0)) / 1e3:.1f} us, "
          f"mean {(st0[-1] - st0[0]) / (len(st0) - 1) / 1e3:.1f} us over {len(st0)} steps")
t0 = med[0][0]
prev_end = defaultdict(lambda: t0)
tot = defaultdict(float)
for s, e, n, q in med:
    gap = s - prev_end[q]
    print(f"  q{q:>3} +{(s - t0) / 1e3:7.1f} us  {(e - s) / 1e3:6.1f} us  gap {gap / 1e3:5.1f}  {n}")
    prev_end[q] = e
# per-kernel average over the steady steps
for st in steps:
    for s, e, n, q in st:
        tot[n] += (e - s) / 1e3 / len(steps)
print("per-step kernel time (avg over steady steps):")
for n, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {v:7.1f} us  {n}")
