"""Effective shader clock per kernel (MI355X_MICROARCH.md 'DVFS give-back'): GRBM_GUI_ACTIVE
(summed over the 8 XCDs) / 8 / the dispatch's wall time, from one rocprofv3 run with
--kernel-trace --pmc GRBM_GUI_ACTIVE. Diagnostics.
    python tools/pmc_clock.py <rocprof output dir> [name-substring ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if want and not any(w in k for w in want):
                continue
            ns = dur.get(r["Dispatch_Id"])
            if ns and ns > 300000:
                per[k].append((float(r["Counter_Value"]) / 8 / ns, ns / 1e6))
    for k, v in sorted(per.items()):
        ghz = sorted(x for x, _ in v)
        ms = sorted(y for _, y in v)
        print("%-50s n=%3d  clock %.2f GHz (min %.2f max %.2f)  ms median %.3f" % (
            k[-50:], len(v), ghz[len(ghz) // 2], ghz[0], ghz[-1], ms[len(ms) // 2]))


if __name__ == "__main__":
    main()
