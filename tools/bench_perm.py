"""Throughput of the permutation-argument prover columns: a circuit of 2^k rows filled with
12-round instances; the per-proof z call (b2f_permutation_columns_dev without sigma) and the
keygen sigma call (b2f_permutation_sigma_dev) timed with HIP events (b2f_kernel_times). One
JSON line per form."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "zk-odst_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=22)
    ap.add_argument("--chunk", type=int, default=3)
    ap.add_argument("--forms", default="1,3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default=None, help="a variant library (A/B), default the product")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    eng = b2f.Engine(0) if not args.lib else b2f.Engine(0, lib_path=args.lib)
    n_rows = 1 << args.k
    usable = n_rows - 7
    n_inst = usable // 5220
    batch = b2f.DeviceBatch(synth.batch(n_inst, rounds=12))
    batch.fill(eng)
    s = torch.cuda.current_stream().cuda_stream
    eng.sync(s)
    for form in [int(f) for f in args.forms.split(",")]:
        batch.permutation_columns(eng, args.k, usable, 3, 5, chunk_len=args.chunk, form=form, sigma=False)
        sig = batch.permutation_sigma(eng, args.k, form=form)
        eng.sync(s)
        eng.set_timing(True)
        for _ in range(args.reps):
            _, z = batch.permutation_columns(eng, args.k, usable, 3, 5, chunk_len=args.chunk,
                                             form=form, sigma=False)
            sig = batch.permutation_sigma(eng, args.k, form=form)
        eng.sync(s)
        kt = eng.kernel_times()
        ms, cnt = kt["perm"]
        sms, scnt = kt["perm_sigma"]
        per, sper = ms / cnt, sms / scnt
        sets = (8 + args.chunk - 1) // args.chunk
        print(json.dumps({"lib": args.lib or "product", "k": args.k, "instances": n_inst, "form": form,
                          "chunk_len": args.chunk, "z_ms_per_call": round(per, 3),
                          "sigma_ms_per_call": round(sper, 3), "rows_per_s": round(n_rows / per * 1e3),
                          "z_written_GBps": round(usable * 32 * sets / per / 1e6, 1)}))
        del sig, z


if __name__ == "__main__":
    main()
