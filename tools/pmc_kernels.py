"""Summarise rocprofv3 --pmc CSVs for the kernels whose names contain any of the given
substrings: per kernel, the counters summed over its dispatches, the dispatch count and the
average kernel-trace duration (diagnostics).
Usage: python3 tools/pmc_kernels.py <rocprof dir> <substr[,substr...]> [--json]"""
import collections
import csv
import glob
import json
import sys


def short(k):
    if "(anonymous namespace)::" in k:
        k = k.split("(anonymous namespace)::", 1)[1]
    return k.split("(")[0].split(" ")[-1]


def main():
    root, subs = sys.argv[1], sys.argv[2].split(",")
    agg = collections.OrderedDict()
    for f in sorted(glob.glob(root + "/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not any(s in k for s in subs):
                continue
            name = short(k)
            d = agg.setdefault(name, {"dispatches": set(), "counters": collections.Counter()})
            d["dispatches"].add((f, r["Dispatch_Id"]))
            d["counters"][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(root + "/**/*kernel_trace.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if any(s in k for s in subs):
                dur[short(k)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for name, d in agg.items():
        n = len(d["dispatches"])
        c = {k: v / n for k, v in sorted(d["counters"].items())}
        us = dur.get(name)
        out[name] = {"dispatches": n, "avg_us": round(sum(us) / len(us), 2) if us else None,
                     "per_dispatch": {k: round(v, 1) for k, v in c.items()}}
    if "--json" in sys.argv:
        print(json.dumps(out, indent=1))
    else:
        for name, o in out.items():
            print(name, "dispatches=%d avg_us=%s" % (o["dispatches"], o["avg_us"]),
                  " ".join("%s=%.4g" % kv for kv in o["per_dispatch"].items()))


if __name__ == "__main__":
    main()
