"""Eval fast clean-check pass ablation (diagnostics library): B2F_DIAG_EVALFAST = check mode of
the fast pass (0 loads + staging only, 1 + lookups, 8 + gates, 16 + copies, 27 all), the exact
eval kernel skipped; 27 = the product path (fast pass, exact kernel gated). One process,
interleaved reps. python tools/ev_ablate.py [--modes 27,0,1,8,16]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 18)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="27,0,1,8,16")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    batch = b2f.DeviceBatch(synth.batch(args.batch, rounds=args.rounds))
    eng = b2f.Engine(0, diag=True)
    s = torch.cuda.current_stream().cuda_stream
    batch.fill(eng, s)
    eng.sync(s)
    res = {}
    for rep in range(args.reps):
        for m in args.modes.split(","):
            os.environ["B2F_DIAG_EVALFAST"] = m
            eng.set_timing(True)
            batch.evaluate(eng, s)
            res.setdefault("evalfast%s" % m, []).append(eng.kernel_times()["eval"][0])
            eng.sync(s)
        os.environ.pop("B2F_DIAG_EVALFAST")
        eng.set_timing(True)
        batch.evaluate(eng, s)
        os.environ["B2F_DIAG_EVAL"] = "7"  # the exact kernel alone (a diagnostics mode number)
        res.setdefault("product_eval", []).append(eng.kernel_times()["eval"][0])
        os.environ.pop("B2F_DIAG_EVAL")
    for k, v in res.items():
        print("%-16s min %8.3f ms  all %s" % (k, min(v), ["%.2f" % t for t in v]))
    rep = batch.report_dict()
    print("last verdict clean:", rep["first_failure"] == 2**64 - 1)


if __name__ == "__main__":
    main()
