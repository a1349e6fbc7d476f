"""profiles/pmc_gram_rNN.json from scripts/gpu_prof.sh's rocprofv3 --pmc passes: per-kernel
counters per *step*, where a kernel's step value is the sum over its template
instantiations of the per-dispatch mean (a fit step launches k_gram_v once per layout
group), plus derived MFMA figures:

  mfma_gflop      SQ_INSTS_MFMA x 2048 flop (v_mfma_f64_16x16x4f64) / 1e9, per step
  mfma_busy_frac  SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles), kernel cycles =
                  GRBM_GUI_ACTIVE / XCDs (GRBM_GUI_ACTIVE is summed over the 8 XCDs)

usage: pmc_gram_summary.py OUT WORKLOAD DIR...
"""
import collections
import csv
import json
import re
import sys

SIMDS, XCDS = 1024, 8


def main(out, workload, *dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
    for d in dirs:
        for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
            full = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            if full.startswith("__amd"):
                continue
            base = re.sub(r"<.*", "", full)
            agg[base][full][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for base, inst in agg.items():
        m = collections.defaultdict(float)
        for full, cnt in inst.items():
            for c, x in cnt.items():
                m[c] += sum(x) / len(x)
        m = dict(m)
        m["instantiations"] = sorted(inst)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            cyc = m["GRBM_GUI_ACTIVE"] / XCDS
            m["kernel_cycles"] = cyc
            m["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc)
        if "SQ_INSTS_MFMA" in m:
            m["mfma_gflop"] = m["SQ_INSTS_MFMA"] * 2048.0 / 1e9
        if "SQ_INSTS_VALU" in m and m.get("SQ_INSTS_MFMA"):
            m["valu_per_mfma"] = m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"]
        res[base] = m
    json.dump({"workload": workload, "workload_key": workload.split(" ")[0], "note": __doc__, "kernels": res},
              open(out, "w"), indent=1)
    for k, m in res.items():
        if m.get("mfma_busy_frac"):
            print(f"{k:24s} MFMA busy {m['mfma_busy_frac']:.3f}  MFMA {m.get('mfma_gflop', 0):.4g} GFLOP/step")


if __name__ == "__main__":
    main(*sys.argv[1:])
