"""Probe: does the eval read a freshly filled slice from the 256 MB Infinity Cache (MALL)?
Splits N 12-round instances into slices of S instances (separate buffers, so every slice
writes fresh addresses like one pass over a large trace), then runs fill(slice) + eval(slice)
back to back on one stream for every slice. Prints per-slice-size kernel sums and wall time
next to the same N in one batch."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "zk-odst_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--instances", type=int, default=1 << 16)
    ap.add_argument("--slices", default="1,16,64,128,256")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    eng = b2f.Engine(0)
    x = synth.batch(args.instances, rounds=12)
    s = torch.cuda.current_stream().cuda_stream
    for ns in [int(v) for v in args.slices.split(",")]:
        per = args.instances // ns
        batches = [b2f.DeviceBatch(x[i * per:(i + 1) * per]) for i in range(ns)]
        for b in batches:  # warm-up (also first-touch of the buffers)
            b.fill(eng)
            b.evaluate(eng)
        eng.sync(s)
        res = []
        for _ in range(2):
            eng.set_timing(True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for b in batches:
                b.fill(eng)
                b.evaluate(eng)
            eng.sync(s)
            wall = (time.perf_counter() - t0) * 1e3
            kt = eng.kernel_times()
            res.append((wall, kt["fill"][0], kt["eval"][0], kt["record"][0]))
        wall, f, e, r = min(res)
        ok = all(b.report_dict()["first_failure"] == 2**64 - 1 for b in batches)
        print(json.dumps({"slices": ns, "instances_per_slice": per,
                          "slice_trace_MB": round(batches[0].total_rows * 44 / 2**20, 1),
                          "wall_ms": round(wall, 3), "fill_ms": round(f, 3), "eval_ms": round(e, 3),
                          "record_ms": round(r, 3), "clean": ok}), flush=True)
        del batches
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
