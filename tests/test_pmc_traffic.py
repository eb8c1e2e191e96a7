"""CPU check of tools/pmc_traffic.py, the summariser behind profiles/pmc_traffic.json (the bench
line's roofline.traffic): per kind, each kernel's average per dispatch, summed over the kind's
kernels (the eval fast pass -- one launch since round 6 -- plus the gated exact kernel), the
gfx950 FETCH_SIZE correction (x2) and the source stamp."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def write_pass(d, counter, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "p_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=FIELDS)
        w.writeheader()
        for disp, name, v in rows:
            w.writerow({"Dispatch_Id": disp, "Kernel_Name": name, "Counter_Name": counter, "Counter_Value": v})


def test_traffic_per_kind(tmp_path):
    hr = "void (anonymous namespace)::eval_hr_kernel<27>(unsigned int const*)"
    ex = "void (anonymous namespace)::eval_kernel<7>(unsigned int const*)"
    fu = "void (anonymous namespace)::fused_hr_kernel<27>(b2f_input const*)"
    fi = "void (anonymous namespace)::fill_kernel<3>(b2f_input const*)"
    # two eval calls (fast pass 1000 / 1010 KiB, exact kernel 2 / 4 KiB), two fused, one fill;
    # a dispatch's value may come in several rows (per XCD), which add up
    fetch = [(1, hr, 600), (1, hr, 400), (2, ex, 2), (3, hr, 1010), (4, ex, 4), (5, fu, 10), (6, fu, 30),
             (7, fi, 8), (8, "void other_kernel(int)", 99999)]
    write = [(1, hr, 0), (2, ex, 0), (3, hr, 0), (4, ex, 0), (5, fu, 5000), (6, fu, 5200), (7, fi, 4000)]
    write_pass(str(tmp_path / "fetch"), "FETCH_SIZE", fetch)
    write_pass(str(tmp_path / "write"), "WRITE_SIZE", write)
    out = tmp_path / "traffic.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path / "fetch"),
                    str(tmp_path / "write"), "8_1", str(out)], check=True, capture_output=True)
    res = json.load(open(out))
    from b2f import _lib

    ev = res["eval_8_1"]
    assert ev["fetch_size_kib_raw"] == 1005 + 3  # fast pass average + exact kernel average
    assert ev["fetch_bytes_corrected"] == 2 * 1008 * 1024
    assert ev["hbm_bytes_per_launch"] == 2 * 1008 * 1024
    assert ev["kernels"] == ["eval_hr_kernel<27>", "eval_kernel<7>"]
    fe = res["fill_eval_8_1"]
    assert fe["fetch_size_kib_raw"] == 20 and fe["write_size_kib"] == 5100
    assert fe["hbm_bytes_per_launch"] == 2 * 20 * 1024 + 5100 * 1024
    assert res["fill_8_1"]["hbm_bytes_per_launch"] == 2 * 8 * 1024 + 4000 * 1024
    assert {v["source_stamp"] for v in res.values()} == {_lib.source_stamp()}
