"""Diagnostics: does a kernel's store rate depend on WHICH device allocation it writes? (round 6:
the Fp export of 2^25 rows ran 2.45 ms into the first two 10.7 GB outputs a process allocated and
2.19 into the later ones, whatever their column stride, profiles/r06e_export_alloc.txt).
Allocates --n outputs of [10, rows, 4] int64 one after another and times, per output, the pasta
export (HIP events, best of --reps) and a plain torch fill_ (memset, CUDA events); prints one
JSON line per output with its device address."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 25)
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--instances", type=int, default=1 << 13)
    ap.add_argument("--libs", default="", help="variant libraries timed beside the product (export)")
    ap.add_argument("--fused", type=int, default=0,
                    help="instead: this many 2^18 x 12 batches (60 GB each), the fused pass timed on each")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    eng = b2f.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    if args.fused:
        x = synth.batch(1 << 18, rounds=12)
        bs = [b2f.DeviceBatch(x) for _ in range(args.fused)]
        t = {i: [] for i in range(args.fused)}
        for _ in range(args.reps):
            for i, b in enumerate(bs):
                eng.set_timing(True)
                b.fill_evaluate(eng, s)
                eng.sync(s)
                t[i].append(eng.kernel_times()["fill_eval"][0])
        for i, b in enumerate(bs):
            assert b.report_dict()["first_failure"] == 2**64 - 1
            print(json.dumps({"batch": i, "addr_GiB": round(b.advice.data_ptr() / 2**30, 3),
                              "fused_ms": round(min(t[i]), 4), "all": [round(v, 3) for v in t[i]]}))
        return
    batch = b2f.DeviceBatch(synth.batch(args.instances, rounds=12))
    batch.fill(eng, s)
    eng.sync(s)
    nr = min(args.rows, batch.total_rows)
    outs = [torch.empty((10, nr, 4), dtype=torch.int64, device="cuda:0") for _ in range(args.n)]
    engines = [("product", eng)] + [(os.path.basename(p)[6:-3], b2f.Engine(0, lib_path=os.path.join(ROOT, p)))
                                    for p in args.libs.split(",") if p]
    res = {i: {"fill": []} for i in range(args.n)}
    for _ in range(args.reps):
        for i, o in enumerate(outs):
            for name, e in engines:
                for form in (b2f.FP_MONTGOMERY, b2f.FP_BN254_MONTGOMERY):
                    e.set_timing(True)
                    batch.export_fp(e, nrows=nr, out=o, form=form, stream=s)
                    e.sync(s)
                    tot, cnt = e.kernel_times()["export"]
                    res[i].setdefault("%s/%d" % (name, form), []).append(tot / max(cnt, 1))
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            o.fill_(0)
            b.record()
            torch.cuda.synchronize()
            res[i]["fill"].append(a.elapsed_time(b))
    nbytes = nr * 10 * 32
    for i, o in enumerate(outs):
        line = {"alloc": i, "addr_GiB": round(o.data_ptr() / 2**30, 3),
                "fill_ms": round(min(res[i]["fill"]), 4), "fill_TBs": round(nbytes / min(res[i]["fill"]) / 1e9, 3)}
        line.update({k: round(min(v), 4) for k, v in res[i].items() if k != "fill"})
        print(json.dumps(line))


if __name__ == "__main__":
    main()
