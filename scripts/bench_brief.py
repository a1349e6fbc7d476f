"""One-screen summary of a bench.py JSON line (headline, predicted strong scaling, grid, cold start)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"value {d['value']:.0f} fits/s  {d['ms_per_step']:.4f} ms/step  {d['config'].get('launch')} x{d['config'].get('pipelines')}  gram frac {r.get('frac')}  "
      f"kernel_ms {json.dumps(r.get('kernel_ms'))}")
print("per_kernel", json.dumps(r.get("per_kernel")))
ps = d.get("predicted_strong") or {}
for k in ("n2", "n4", "n8"):
    if k in ps:
        print(k, ps[k]["ms_per_step"], "ms", ps[k]["speedup_vs_n1"], "x", ps[k]["ms_per_shard"], ps[k].get("launch"))
if d.get("grid"):
    print("grid", d["grid"]["value"], d["grid"].get("seconds_all"), d["grid"].get("roofline"))
    print("grid predicted", json.dumps(d["grid"].get("predicted_strong")))
print("cold", json.dumps(d.get("cold_start")))
for k in ("j0740", "c2"):
    if d.get(k):
        print(k, json.dumps(d[k])[:600])
