"""Print a rocprofv3 kernel_stats.csv as a short table: python scripts/kstats.py DIR"""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")):
    print(f"{r['Name'][:64]:64s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:9.1f} us {float(r['Percentage']):6.2f}%")
