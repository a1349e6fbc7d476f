"""Largest idle gaps and longest kernels on each queue of a rocprofv3 kernel trace (bench
runs): python scripts/trace_gaps.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
q = defaultdict(list)
for r in rows:
    q[r.get("Queue_Id", r.get("Stream_Id", "?"))].append(
        (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40]))
t_end = max(e for v in q.values() for _, e, _ in v)
for k, v in sorted(q.items()):
    v.sort()
    gaps = sorted(((v[i + 1][0] - v[i][1], i) for i in range(len(v) - 1)), reverse=True)[:5]
    longk = sorted(((e - s, n) for s, e, n in v), reverse=True)[:3]
    print(f"queue {k}: {len(v)} kernels; largest gaps (us, before, after, t_from_end_ms): "
          + "; ".join(f"{g / 1e3:.1f} {v[i][2]} -> {v[i + 1][2]} @{(t_end - v[i][1]) / 1e6:.2f}" for g, i in gaps))
    print(f"   longest kernels (us): " + "; ".join(f"{d / 1e3:.1f} {n}" for d, n in longk))

# per-step spans on the main queue (a step starts at the evaluation with the design matrix)
main = max(q.items(), key=lambda kv: len(kv[1]))[1]
starts = [i for i, (_, _, n) in enumerate(main) if n.startswith("void k_eval_mix_w<1") or n.startswith("void k_eval_mix<1")]
print("steps (span us, k_gram_v us, gap before us):")
line = []
for a, b in zip(starts, starts[1:]):
    span = (main[b][0] - main[a][0]) / 1e3
    g = [(e - s) / 1e3 for s, e, n in main[a:b] if "k_gram_v" in n]
    gap = (main[a][0] - main[a - 1][1]) / 1e3 if a > 0 else 0.0
    line.append(f"{span:.0f}/{(g[0] if g else 0):.0f}/{gap:.0f}")
print(" ".join(line[-80:]))
