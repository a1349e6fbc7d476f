"""profiles/pmc_gram_rNN.json from scripts/pmc_gram.sh's three rocprofv3 --pmc passes:
per-kernel averages of the MFMA / LDS / activity counters, plus derived MFMA utilisation.

mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles), kernel cycles =
GRBM_GUI_ACTIVE / XCDs (GRBM_GUI_ACTIVE is summed over the 8 XCDs)."""
import collections
import csv
import json
import sys

SIMDS, XCDS = 1024, 8


def main(out, *dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k.startswith("__amd"):
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, v in agg.items():
        m = {c: sum(x) / len(x) for c, x in v.items()}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            cyc = m["GRBM_GUI_ACTIVE"] / XCDS
            m["kernel_cycles"] = cyc
            m["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc)
            m["mfma_f64_flops"] = m.get("SQ_INSTS_MFMA", 0.0) * 2048.0
        res[k] = m
    json.dump({"note": __doc__, "kernels": res}, open(out, "w"), indent=1)
    for k, m in res.items():
        if m.get("mfma_busy_frac"):
            print(f"{k:24s} MFMA busy {m['mfma_busy_frac']:.3f}  MFMA insts {m.get('SQ_INSTS_MFMA', 0):.3g}")


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:])
