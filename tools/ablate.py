"""Ablation timings of the fill/eval kernel variants (B2F_DIAG_FILL / B2F_DIAG_EVAL), one
process, interleaved rounds. Diagnostic only: python tools/ablate.py [--batch N]."""
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
    ap.add_argument("--fill-modes", default="3,2,1,0")
    ap.add_argument("--eval-modes", default="7,8,2,4")
    ap.add_argument("--bands", default="", help="fused fill+eval band sizes to time (B2F_BAND)")
    ap.add_argument("--fused-modes", default="", help="fused kernel variants (B2F_DIAG_FUSED)")
    ap.add_argument("--lib", default=None, help="an explicit build of the ABI (A/B runs); "
                    "default: the diagnostics library libb2f_diag.so")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    x = synth.batch(args.batch, rounds=args.rounds)
    batch = b2f.DeviceBatch(x)
    eng = b2f.Engine(0, diag=True, lib_path=args.lib)
    s = torch.cuda.current_stream().cuda_stream
    nbytes = batch.used_rows * 44
    batch.fill(eng, s)
    batch.evaluate(eng, s)
    eng.sync(s)
    res = {}
    for rep in range(args.reps):
        for m in args.fill_modes.split(","):
            os.environ["B2F_DIAG_FILL"] = m
            eng.set_timing(True)
            batch.fill(eng, s)
            t = eng.kernel_times()["fill"][0]
            res.setdefault("fill%s" % m, []).append(t)
        os.environ.pop("B2F_DIAG_FILL")
        batch.fill(eng, s)
        for m in args.eval_modes.split(","):
            os.environ["B2F_DIAG_EVAL"] = m
            eng.set_timing(True)
            batch.evaluate(eng, s)
            t = eng.kernel_times()["eval"][0]
            res.setdefault("eval%s" % m, []).append(t)
        os.environ.pop("B2F_DIAG_EVAL")
        for b in [v for v in args.bands.split(",") if v]:
            os.environ["B2F_BAND"] = b
            eng.set_timing(True)
            batch.fill_evaluate(eng, s)
            t = eng.kernel_times()["fill_eval"][0]
            res.setdefault("fused%s" % b, []).append(t)
        os.environ.pop("B2F_BAND", None)
        for m in [v for v in args.fused_modes.split(",") if v]:
            os.environ["B2F_DIAG_FUSED"] = m
            eng.set_timing(True)
            batch.fill_evaluate(eng, s)
            t = eng.kernel_times()["fill_eval"][0]
            res.setdefault("fmode%s" % m, []).append(t)
        os.environ.pop("B2F_DIAG_FUSED", None)
    for k, v in res.items():
        best = min(v)
        print("%-6s min %8.3f ms  (%6.0f GB/s)  all %s" % (k, best, nbytes / best / 1e6,
                                                        ["%.2f" % t for t in v]))
    eng.sync(s)


if __name__ == "__main__":
    main()
