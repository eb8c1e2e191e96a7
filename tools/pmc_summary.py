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
        if not any(t in k for t in ("fill_kernel", "eval_kernel", "eval_hr_kernel", "eval_edge_kernel",
                                    "fused_kernel", "fused_hr_kernel", "fused_edge_kernel")):
            continue
        name = k.split("(anonymous namespace)::")[1].split("<")[0].split("(")[0]
        head = k.split("(anonymous namespace)::")[1].split("(")[0]
        mode = head.split("<")[1].split(">")[0] if "<" in head else ""
        key = (name + "<" + mode + ">", f.split("/")[-2], r["Dispatch_Id"])
        agg.setdefault(key, {})[r["Counter_Name"]] = agg.get(key, {}).get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for (name, run, disp), c in agg.items():
    print(name, run, disp, " ".join("%s=%.3g" % (k, v) for k, v in sorted(c.items())))
