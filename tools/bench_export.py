"""Fp export throughput A/B (b2f_export_fp_dev): 2^25 rows of a filled 12-round trace exported
in pasta Montgomery and BN254 Montgomery form by each library given, interleaved rep by rep in
one process (HIP-event kernel time). Diagnostic only:
    python tools/bench_export.py [--libs a.so,b.so] [--rows N] [--pads 0,256]
--pads: output column strides of rows + pad (out_rows; the bench's [10, 2^25, 4] tensor puts the
columns exactly 2^30 bytes apart)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="", help="variant libraries besides the product")
    ap.add_argument("--rows", type=int, default=1 << 25)
    ap.add_argument("--instances", type=int, default=1 << 13)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--pads", default="0", help="comma-separated out_rows - rows values")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    batch = b2f.DeviceBatch(synth.batch(args.instances, rounds=12))
    prod = b2f.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    batch.fill(prod, s)
    prod.sync(s)
    nr = min(args.rows, batch.total_rows)
    engines = [("product", prod)] + [(os.path.basename(p), b2f.Engine(0, lib_path=os.path.join(ROOT, p)))
                                     for p in args.libs.split(",") if p]
    pads = [int(p) for p in args.pads.split(",")]  # a pad may repeat: allocations in this order
    outs = [torch.empty((10, nr + p, 4), dtype=torch.int64, device=batch.advice.device) for p in pads]
    res = {}
    for rep in range(args.reps):
        for name, eng in engines:
            for ip, p in enumerate(pads):
                for form in (b2f.FP_MONTGOMERY, b2f.FP_BN254_MONTGOMERY):
                    eng.set_timing(True)
                    batch.export_fp(eng, nrows=nr, out=outs[ip], form=form, stream=s)
                    eng.sync(s)
                    tot, cnt = eng.kernel_times()["export"]
                    res.setdefault((name, ip, p, form), []).append(tot / max(cnt, 1))
    nbytes = nr * 10 * 36
    for (name, ip, p, form), v in res.items():
        best = min(v[1:]) if len(v) > 1 else v[0]
        print(json.dumps({"lib": name, "alloc": ip, "base_mod_1GiB": outs[ip].data_ptr() % (1 << 30),
                          "pad_rows": p, "form": form, "ms": round(best, 4),
                          "GBs": round(nbytes / best / 1e6, 1), "all": [round(x, 3) for x in v]}))


if __name__ == "__main__":
    main()
