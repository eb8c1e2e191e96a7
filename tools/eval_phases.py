"""Eval-kernel phase breakdown (diagnostics): runs the EVAL_CLOCK variant (B2F_DIAG_EVAL=23)
on a 2^18 x 12-round batch and prints, per wave of the workgroup, the share of s_memtime
cycles spent in each phase of the tile loop. python tools/eval_phases.py [--batch N]
--fused M: the fused kernel's clocked variant instead; --fill: the split fill's (FILL_CLOCK,
B2F_DIAG_FILL=11), so the two can be compared on one box."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))
PHASES = ["stage+lookup", "barrier1", "prefetch", "gtable", "gpass", "copies", "perquad", "barrier2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 18)
    ap.add_argument("--fused", type=int, default=0,
                    help="the fused kernel's clocked variant: 155 (full), 130 (stores only), 128")
    ap.add_argument("--fill", action="store_true", help="the split fill's clocked variant")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    x = synth.batch(args.batch, rounds=12)
    batch = b2f.DeviceBatch(x)
    eng = b2f.Engine(0, diag=True)  # EVAL_CLOCK / FZ_CLOCK variants: diagnostics build only
    s = torch.cuda.current_stream().cuda_stream
    batch.fill(eng, s)
    run = batch.fill_evaluate if args.fused else batch.evaluate
    os.environ["B2F_DIAG_FUSED" if args.fused else "B2F_DIAG_EVAL"] = str(args.fused) if args.fused else "23"
    kname = "fill_eval" if args.fused else "eval"
    global PHASES
    if args.fill:
        os.environ.pop("B2F_DIAG_EVAL", None)
        os.environ["B2F_DIAG_FILL"] = "11"
        run = batch.fill
        kname = "fill"
        PHASES = ["next-ops", "cells", "stores", "loop", "drain", "-", "-", "-"]
    if args.fused:
        # fused_hr_kernel (the half-round launch, second form) tick points
        PHASES = ["load+words", "chains+publish", "operands+cells", "stage-wait", "stores",
                  "fast-checks", "exact+end", "vmcnt"]
    run(eng, s)
    eng.sync(s)
    out = (ctypes.c_uint64 * 32)()
    eng._check(eng.lib.b2f_debug_clock(eng.ctx, out))  # clear
    eng.set_timing(True)
    run(eng, s)
    eng.sync(s)
    ms = eng.kernel_times()[kname][0]
    eng._check(eng.lib.b2f_debug_clock(eng.ctx, out))
    if args.fill:
        print("fill (clocked variant) %.3f ms" % ms)
    else:
        rep = batch.report_dict()
        print(kname + " (clocked variant) %.3f ms, verdict clean: %s" % (ms, rep["first_failure"] == 2**64 - 1))
    for w in range(4):
        row = [out[8 * w + k] for k in range(8)]
        tot = sum(row) or 1
        print("wave %d: " % w + "  ".join("%s %4.1f%%" % (PHASES[k], 100.0 * row[k] / tot) for k in range(8)))


if __name__ == "__main__":
    main()
