"""Per-kernel averages of rocprofv3 --pmc passes: python scripts/pmc_table.py DIR [DIR...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:24]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:24s} " + " ".join(f"{c.replace('SQ_', '')}={sum(x) / len(x):.4g}" for c, x in sorted(v.items())))
