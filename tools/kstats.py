"""Print a rocprofv3 run_kernel_stats.csv compactly: python tools/kstats.py <dir>"""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1].rstrip("/") + "/run_kernel_stats.csv")):
    print(f"{r['Name'][:64]:64s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.1f} us {float(r['Percentage']):6.2f}%")
