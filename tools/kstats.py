"""Print a rocprofv3 --stats kernel_stats.csv compactly: short name, calls, average us.
Usage: python3 tools/kstats.py <csv or dir> [min_us]"""
import csv
import glob
import os
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = sorted(glob.glob(path + "/**/*kernel_stats.csv", recursive=True))[-1]
lim = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
for r in csv.DictReader(open(path)):
    n = r["Name"]
    n = n.split("(anonymous namespace)::", 1)[1] if "(anonymous namespace)::" in n else n.split("::")[-1]
    us = float(r["AverageNs"]) / 1e3
    if us >= lim:
        print("%-48s %5s %9.1f" % (n.split("(")[0][:48], r["Calls"], us))
