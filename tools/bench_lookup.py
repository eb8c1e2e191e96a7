"""Throughput of the lookup-argument prover columns (b2f_lookup_columns_dev): a filled trace
of N 12-round instances cut into circuits of `usable` rows, columns built for `--circuits`
circuits per call into one preallocated output (HIP-event kernel time via b2f_kernel_times).
Prints one JSON line: rows/s and the algorithmic bytes per row (16 B of lookup cells read,
5 x 32 B of columns written)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "zk-odst_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--instances", type=int, default=1 << 13)
    ap.add_argument("--usable", type=int, default=(1 << 17) - 7)
    ap.add_argument("--circuits", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--form", type=int, default=1)
    ap.add_argument("--lib", default=None, help="a variant library (A/B), default the product")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    eng = b2f.Engine(0) if not args.lib else b2f.Engine(0, lib_path=args.lib)
    batch = b2f.DeviceBatch(synth.batch(args.instances, rounds=12))
    batch.fill(eng)
    s = torch.cuda.current_stream().cuda_stream
    eng.sync(s)
    nc = min(args.circuits, batch.total_rows // args.usable)
    dev = batch.advice.device
    rb = torch.arange(nc, dtype=torch.int64, device=dev) * args.usable
    out = torch.empty((nc, 5, args.usable + 1, 4), dtype=torch.int64, device=dev)
    bad = torch.empty(nc, dtype=torch.int64, device=dev)
    th, be, ga = 0x1234567 << 200, 0x89abcdef << 180, 0x13579bdf << 190
    call = lambda: eng.lookup_columns_dev(batch.advice.data_ptr(), batch.total_rows,  # noqa
                                          rb.data_ptr(), nc, args.usable, th, be, ga, args.form,
                                          out.data_ptr(), args.usable + 1, bad.data_ptr(), s)
    def sync():
        try:
            eng.sync(s)
        except b2f.B2FError as e:  # a diagnostics variant whose columns are wrong by design
            if not args.lib or e.code != b2f._lib.ERR_CHECK:
                raise

    call()
    sync()
    assert (bad.cpu() == -1).all()
    eng.set_timing(True)
    for _ in range(args.reps):
        call()
    sync()
    ms, cnt = eng.kernel_times()["lookup"]
    per = ms / cnt
    rows = nc * args.usable
    print(json.dumps({"lib": args.lib or "product", "circuits": nc, "usable_rows": args.usable, "rows": rows,
                      "ms_per_call": round(per, 3), "rows_per_s": round(rows / per * 1e3),
                      "algorithmic_GBps": round(rows * 176 / per / 1e6, 1),
                      "note": "176 B/row algorithmic (16 B read, 160 B written)"}))


if __name__ == "__main__":
    main()
