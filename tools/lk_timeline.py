"""Timeline of one lookup-columns call from a rocprofv3 --kernel-trace CSV (diagnostics): the
last call's kernels (from its lk_table_kernel on, plus those still running when it started), start / end in microseconds from the call's
first kernel start, with the stream (queue) each ran on.
Usage: python3 tools/lk_timeline.py <kernel_trace.csv or its directory>"""
import csv
import glob
import os
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[-1]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "lk_table_kernel" in r["Kernel_Name"]]
t0 = int(rows[starts[-1]]["Start_Timestamp"])
# the call's kernels, and those queued before its table pass that were still running at its start
# (the count pass on the main stream)
call = [r for i, r in enumerate(rows) if i >= starts[-1] or
        (i >= starts[-1] - 8 and int(r["End_Timestamp"]) > t0)]
for r in call:
    n = r["Kernel_Name"]
    n = n.split("::")[-1] if "(anonymous namespace)::" not in n else n.split("(anonymous namespace)::", 1)[1]
    n = n.split("(")[0]
    print("%-44s q%-3s %9.1f %9.1f %8.1f" % (n[:44], r["Queue_Id"], (int(r["Start_Timestamp"]) - t0) / 1e3,
                                              (int(r["End_Timestamp"]) - t0) / 1e3,
                                              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
