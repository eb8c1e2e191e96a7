"""Summarise rocprofv3 --pmc CSVs per kernel dispatch (diagnostics)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.OrderedDict()
for f in sorted(glob.glob(root + "/*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "fill_kernel" not in k and "eval_kernel" not in k and "fused_kernel" not in k:
            continue
        name = k.split("(")[0].split("::")[-1]
        mode = k.split("<")[1].split(">")[0] if "<" in k else ""
        key = (name + "<" + mode + ">", f.split("/")[-2], r["Dispatch_Id"])
        agg.setdefault(key, {})[r["Counter_Name"]] = agg.get(key, {}).get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for (name, run, disp), c in agg.items():
    print(name, run, disp, " ".join("%s=%.3g" % (k, v) for k, v in sorted(c.items())))
