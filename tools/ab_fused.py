"""A/B of fused fill+eval library variants in ONE process, interleaved rep by rep (boxes and
even consecutive runs on one box differ by up to ~25 % in store rate, so variants are only
compared inside one process). Diagnostic only:
    python tools/ab_fused.py --libs zk-odst_amd/variants/libb2f_a.so,... [--modes 27,2,0]
The product library's split path (fill + eval) is timed in the same loop as the reference."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="", help="comma-separated variant libraries (diag builds)")
    ap.add_argument("--modes", default="27", help="B2F_DIAG_FUSED modes to time per variant")
    ap.add_argument("--batch", type=int, default=1 << 18)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--mix", action="store_true", help="rounds uniform in {1,4,12} (config 5)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--eval", action="store_true", help="also time each variant's eval kernel")
    ap.add_argument("--fill", action="store_true", help="also time each variant's split fill")
    args = ap.parse_args()
    import torch

    import b2f
    from b2f import synth

    x = synth.batch(args.batch, rounds=args.rounds, rounds_mix=[1, 4, 12] if args.mix else None)
    batch = b2f.DeviceBatch(x)
    s = torch.cuda.current_stream().cuda_stream
    prod = b2f.Engine(0)
    engines = [("product", prod)]
    envs = {}
    for spec in [v for v in args.libs.split(",") if v]:
        # path[@K=V[;K=V]]: environment set around that variant's fused calls (diag builds)
        p, _, env = spec.partition("@")
        name = os.path.basename(p)[6:-3] + ("@" + env if env else "")
        engines.append((name, b2f.Engine(0, lib_path=os.path.join(ROOT, p))))
        envs[name] = dict(kv.split("=", 1) for kv in env.split(";") if kv)
    nbytes = batch.used_rows * 44
    batch.fill(prod, s)
    batch.evaluate(prod, s)
    prod.sync(s)
    res = {}
    modes = [m for m in args.modes.split(",") if m]
    for rep in range(args.reps):
        prod.set_timing(True)
        batch.fill(prod, s)
        batch.evaluate(prod, s)
        kt = prod.kernel_times()
        res.setdefault("split(fill+eval)", []).append(kt["fill"][0] + kt["eval"][0] + kt["record"][0])
        for name, eng in engines:
            for k, v in envs.get(name, {}).items():
                os.environ[k] = v
            if args.fill:
                eng.set_timing(True)
                batch.fill(eng, s)
                kt = eng.kernel_times()
                res.setdefault("%s/fill" % name, []).append(kt["fill"][0])
                eng.sync(s)
            if args.eval:
                eng.set_timing(True)
                batch.evaluate(eng, s)
                kt = eng.kernel_times()
                res.setdefault("%s/eval" % name, []).append(kt["eval"][0])
                eng.sync(s)
            for m in modes if name != "product" else ["27"]:
                os.environ["B2F_DIAG_FUSED"] = m
                eng.set_timing(True)
                batch.fill_evaluate(eng, s)
                kt = eng.kernel_times()
                res.setdefault("%s/fused%s" % (name, m), []).append(kt["fill_eval"][0] + kt["record"][0])
                eng.sync(s)
            for k in envs.get(name, {}):
                os.environ.pop(k, None)
        os.environ.pop("B2F_DIAG_FUSED", None)
    for k, v in res.items():
        best = min(v)
        print("%-28s min %8.3f ms  (%6.0f GB/s)  all %s" % (k, best, nbytes / best / 1e6,
                                                         ["%.2f" % t for t in v]))
    rep = batch.report_dict()
    print("last verdict clean:", rep["first_failure"] == 2**64 - 1)


if __name__ == "__main__":
    main()
