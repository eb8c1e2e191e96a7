"""Headline benchmark: BLAKE2f compressions/s, witness fill + constraint eval, 2^18 batch of
12-round compressions per GPU (BASELINE.json configs[2]; configs[4] with --mix).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

One step = fill (record + fill kernels) then eval of the whole per-GPU batch (--path split, the
headline; --path fused runs b2f_fill_eval_dev instead; the other path is timed beside it as
"other_path"); inputs and the trace stay resident in HBM. N > 1: every rank runs its own 2^18 shard (weak scaling); the
step ends with one all_reduce of the verdict counters and one RCCL all_gather of the h'
outputs. Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
ADVICE_COLS = 10
ROW_BYTES = 4 * (ADVICE_COLS + 1)  # 10 advice u32 + 1 fixed u32
INPUT_BYTES = 216


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(rounds, mix, target_s):
    """Time the CPU oracle (oracle/, a C port of the same fill + eval) on a bounded sample of
    the same workload, all host threads it is given. Test infrastructure: the checker."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from b2f import synth

    threads = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))

    chunk = 2048  # ~0.5 GB of trace per chunk at 12 rounds: memory stays bounded

    def run(seed):
        x = synth.batch(chunk, rounds=rounds, rounds_mix=mix, seed=seed)
        ox = np.frombuffer(x.tobytes(), dtype=oracle.INPUT_DTYPE).copy()
        t0 = time.perf_counter()
        adv, fixed, h_out, off = oracle.fill(ox, nthreads=threads)
        rep = oracle.evaluate(adv, fixed, off, nthreads=threads)
        dt = time.perf_counter() - t0
        assert rep["first_failure"] == 2**64 - 1
        return dt

    run(1)  # warm the thread pool and the allocator
    n2, dt2, seed = 0, 0.0, 2
    while dt2 < target_s:
        dt2 += run(seed)
        n2 += chunk
        seed += 1
    # one thread, one chunk of 256: the per-core rate
    x1 = synth.batch(256, rounds=rounds, rounds_mix=mix, seed=99)
    o1 = np.frombuffer(x1.tobytes(), dtype=oracle.INPUT_DTYPE).copy()
    t1 = time.perf_counter()
    a1, f1, _, off1 = oracle.fill(o1, nthreads=1)
    oracle.evaluate(a1, f1, off1, nthreads=1)
    single = 256 / (time.perf_counter() - t1)
    return {"value": n2 / dt2, "unit": "compressions/s", "cores": threads, "kind": "port",
            "single_thread": round(single, 1), "host_cpus": os.cpu_count(),
            "sample": "%d x %s-round compressions in chunks of %d, oracle fill + eval "
                      "(%.1f s timed, %d threads)"
                      % (n2, "mixed" if mix else rounds, chunk, dt2, threads)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 18, help="instances per GPU")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--mix", action="store_true", help="rounds uniform in {1,4,12} (config 5)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--export-rows", type=int, default=1 << 25,
                    help="rows of the Fp export timed after the headline loop (0 = skip)")
    ap.add_argument("--path", choices=["split", "fused"], default="split",
                    help="split: fill kernel then eval kernel (the headline); fused: "
                         "b2f_fill_eval_dev, one kernel that checks each tile as it assigns it")
    ap.add_argument("--lookup-circuits", type=int, default=64,
                    help="lookup-argument columns for this many 2^17-row circuits of the trace "
                         "(reported beside the headline; 0 skips)")
    ap.add_argument("--hasher-messages", type=int, default=1 << 16,
                    help="multi-block BLAKE2b over the chip: this many 1 KiB messages "
                         "(reported beside the headline; 0 skips)")
    ap.add_argument("--witness-gather", type=int, default=1 << 13,
                    help="N > 1: instances per rank of a separate batch whose whole witness "
                         "table is all-gathered to every rank (timed apart; 0 skips)")
    ap.add_argument("--aux-steps", type=int, default=5,
                    help="steps of the other path timed after the headline loop (0 = skip)")
    ap.add_argument("--floor-reps", type=int, default=3,
                    help="launches of each diagnostic floor variant (0 = skip)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py output)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import b2f
    from b2f import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    # rehearsal of the N > 1 code path on a one-GPU box (never for measurements): every rank
    # on cuda:0, collectives over gloo
    rehearse = os.environ.get("B2F_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    mix = [1, 4, 12] if args.mix else None
    n = args.batch
    x = synth.batch(n, rounds=args.rounds, rounds_mix=mix, first=rank * n)
    batch = b2f.DeviceBatch(x, device="cuda:%d" % local)
    eng = b2f.Engine(local)
    stream = torch.cuda.current_stream().cuda_stream
    rows = batch.used_rows
    log("rank %d: %d instances, %d rows, trace %.1f GB" % (rank, n, rows, rows * ROW_BYTES / 1e9))

    if world > 1:
        gathered = torch.empty((world * n, 8), dtype=torch.int64, device=batch.h_out.device)
        verdict = torch.empty(20, dtype=torch.int64, device=batch.h_out.device)

    def run_path(path):
        if path == "fused":
            batch.fill_evaluate(eng, stream)
        else:
            batch.fill(eng, stream)
            batch.evaluate(eng, stream)

    def step():
        run_path(args.path)
        if world > 1:
            r = batch.report.view(torch.int64)
            verdict[:18].copy_(r[:18])
            first = r[18]
            verdict[18] = torch.where(first == -1, torch.iinfo(torch.int64).max, first)
            dist.all_reduce(verdict[:18], op=dist.ReduceOp.SUM)
            dist.all_reduce(verdict[18:19], op=dist.ReduceOp.MIN)
            dist.all_gather_into_tensor(gathered, batch.h_out)

    for _ in range(args.warmup):
        step()
    eng.sync(stream)
    rep = batch.report_dict()
    if rep["first_failure"] != 2**64 - 1:
        raise SystemExit("eval flagged the trace: %s" % rep)

    eng.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ktimes = eng.kernel_times()
    eng.sync(stream)
    rep = batch.report_dict()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=batch.h_out.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if int(verdict[18].item()) != torch.iinfo(torch.int64).max or int(verdict[:18].sum()) != 0:
            raise SystemExit("eval flagged a shard")
    if rep["first_failure"] != 2**64 - 1:
        raise SystemExit("eval flagged the trace: %s" % rep)

    # the step's collectives alone (all-gather time reported separately)
    collectives = None
    if world > 1:
        def exchange():
            dist.all_reduce(verdict[:18], op=dist.ReduceOp.SUM)
            dist.all_reduce(verdict[18:19], op=dist.ReduceOp.MIN)
            dist.all_gather_into_tensor(gathered, batch.h_out)
        verdict.zero_()
        dist.barrier()
        torch.cuda.synchronize()
        tc = time.perf_counter()
        for _ in range(args.steps):
            exchange()
        torch.cuda.synchronize()
        ct = torch.tensor([time.perf_counter() - tc], dtype=torch.float64,
                          device=batch.h_out.device)
        dist.all_reduce(ct, op=dist.ReduceOp.MAX)
        collectives = {"ms_per_step": round(1e3 * float(ct.item()) / args.steps, 4),
                       "all_gather_bytes_per_rank": n * 64,
                       "note": "2 all_reduce (verdict) + 1 all_gather (h'), timed alone"}

    # optional: reassemble a (smaller) batch's whole witness table on every rank, the
    # north_star's all-gather, for a batch that fits; timed apart
    witness_gather = None
    if world > 1 and args.witness_gather > 0:
        try:
            from b2f import dist as bdist
            xw = synth.batch(args.witness_gather, rounds=args.rounds, rounds_mix=mix,
                             seed=1000 + rank)
            wb = b2f.DeviceBatch(xw, device="cuda:%d" % local)
            wb.fill(eng, stream)
            eng.sync(stream)
            rows_w = torch.tensor([wb.total_rows], dtype=torch.int64, device=wb.advice.device)
            all_rows = [torch.zeros_like(rows_w) for _ in range(world)]
            dist.all_gather(all_rows, rows_w)
            srows = [int(r.item()) for r in all_rows]
            bdist.gather_trace(wb.advice, wb.fixed, srows, dist, torch)  # warm-up
            dist.barrier()
            torch.cuda.synchronize()
            tw = time.perf_counter()
            ga, gf = bdist.gather_trace(wb.advice, wb.fixed, srows, dist, torch)
            torch.cuda.synchronize()
            wt = torch.tensor([time.perf_counter() - tw], dtype=torch.float64,
                              device=wb.advice.device)
            dist.all_reduce(wt, op=dist.ReduceOp.MAX)
            gathered_bytes = sum(srows) * ROW_BYTES
            witness_gather = {"instances_per_rank": args.witness_gather,
                              "trace_bytes_per_rank": wb.total_rows * ROW_BYTES,
                              "gathered_bytes_per_rank": gathered_bytes,
                              "ms": round(float(wt.item()) * 1e3, 3),
                              "GBs_received_per_rank": round(
                                  (gathered_bytes - wb.total_rows * ROW_BYTES)
                                  / float(wt.item()) / 1e9, 1),
                              "note": "one all_gather of the 11 columns + reassembly copy"}
            del ga, gf, wb
        except Exception as e:
            witness_gather = {"error": repr(e)}

    value = world * n * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # roofline: algorithmic bytes per launch / average launch duration (HIP events)
    fill_bytes = n * INPUT_BYTES + rows * ROW_BYTES      # inputs read + trace written
    eval_bytes = rows * ROW_BYTES + 8 * (n + 1)          # trace + offsets read

    def kernel_table(ktimes):
        kern = {}
        for name, nbytes in (("fill", fill_bytes), ("eval", eval_bytes),
                             ("fill_eval", fill_bytes), ("record", None)):
            tot, cnt = ktimes[name]
            if not cnt:
                continue
            avg = tot / cnt
            kern[name] = {"avg_ms": round(avg, 4), "launches": cnt}
            if nbytes:
                gbs = nbytes / (avg * 1e-3) / 1e9
                kern[name].update({"bytes_per_launch": nbytes, "achieved_GBs": round(gbs, 1),
                                   "frac": round(gbs / HBM_PEAK_GBS, 4)})
        return kern

    kern = kernel_table(ktimes)
    big = [k for k in kern if k != "record"]
    dom = max(big, key=lambda k: kern[k]["avg_ms"])
    traffic = None
    try:
        with open(args.traffic) as fh:
            tr = json.load(fh)
        key = "%s_%d_%s" % (dom, n, "mix" if mix else args.rounds)
        traffic = tr.get(key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    roof = {"bound": "hbm", "achieved": kern[dom]["achieved_GBs"], "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": kern[dom]["frac"], "traffic": traffic, "kernel": dom}

    # same-box floors (diagnostic kernel variants, reported beside the headline): the fill with
    # its stores but no cell computation (B2F_DIAG_FILL=2) and the eval with its loads, staging
    # and lookups but no gates or copies (B2F_DIAG_EVAL=1). Boxes differ by up to ~25 % on the
    # store-bound fill, so the achieved/floor ratio is the comparable number.
    floors = None
    if world == 1 and args.floor_reps > 0:
        floors = {}
        for var, val, kname in (("B2F_DIAG_FILL", "2", "fill"), ("B2F_DIAG_EVAL", "1", "eval")):
            os.environ[var] = val
            try:
                eng.set_timing(True)
                for _ in range(args.floor_reps):
                    if kname == "fill":
                        batch.fill(eng, stream)
                    else:
                        batch.evaluate(eng, stream)
                tot, cnt = eng.kernel_times()[kname]
            finally:
                os.environ.pop(var, None)
            floors[kname + "_floor_ms"] = round(tot / max(cnt, 1), 4)
            floors[kname + "_over_floor"] = round(kern[kname]["avg_ms"] / (tot / max(cnt, 1)), 4) \
                if kname in kern else None
        batch.fill(eng, stream)  # leave a real trace behind
        eng.sync(stream)

    # the other path, timed the same way (reported beside the headline, not part of it)
    aux = None
    other = "fused" if args.path == "split" else "split"
    if args.aux_steps > 0 and world == 1:
        run_path(other)
        eng.sync(stream)
        eng.set_timing(True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.aux_steps):
            run_path(other)
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        k2 = kernel_table(eng.kernel_times())
        eng.sync(stream)
        r2 = batch.report_dict()
        aux = {"path": other, "value": round(n * args.aux_steps / el, 1),
               "ms_per_step": round(1e3 * el / args.aux_steps, 4), "kernels": k2,
               "verdict_clean": r2["first_failure"] == 2**64 - 1}

    # Fp export, reported beside the headline, not part of it:
    # Montgomery pallas limbs for a chunk of the resident trace (4 B read, 32 B written/cell)
    fp_export = None
    if args.export_rows > 0:
        nr = min(args.export_rows, batch.total_rows)
        out = torch.empty((10, nr, 4), dtype=torch.int64, device=batch.advice.device)
        batch.export_fp(eng, nrows=nr, out=out, stream=stream)
        eng.sync(stream)
        eng.set_timing(True)
        reps = 5
        for _ in range(reps):
            batch.export_fp(eng, nrows=nr, out=out, stream=stream)
        tot, cnt = eng.kernel_times()["export"]
        avg = tot / max(cnt, 1)
        nbytes = nr * 10 * (4 + 32)
        fp_export = {"rows": nr, "form": "montgomery", "avg_ms": round(avg, 4),
                     "bytes_per_launch": nbytes,
                     "achieved_GBs": round(nbytes / (avg * 1e-3) / 1e9, 1),
                     "frac": round(nbytes / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        del out

    # Lookup-argument prover columns for circuits cut from the resident
    # trace, and the multi-block hasher (row 3): reported beside the headline, not part of it
    lookup = None
    if world == 1 and args.lookup_circuits > 0:
        try:
            usable = (1 << 17) - 7
            nc = min(args.lookup_circuits, batch.total_rows // usable)
            dev = batch.advice.device
            rb = torch.arange(nc, dtype=torch.int64, device=dev) * usable
            lout = torch.empty((nc, 5, usable + 1, 4), dtype=torch.int64, device=dev)
            lbad = torch.empty(nc, dtype=torch.int64, device=dev)
            chal = (0x1234567 << 200, 0x89ABCDEF << 180, 0x13579BDF << 190)

            def lk_call():
                eng.lookup_columns_dev(batch.advice.data_ptr(), batch.total_rows, rb.data_ptr(), nc,
                                       usable, *chal, 1, lout.data_ptr(), usable + 1,
                                       lbad.data_ptr(), stream)
            lk_call()
            eng.sync(stream)
            eng.set_timing(True)
            for _ in range(3):
                lk_call()
            tot, cnt = eng.kernel_times()["lookup"]
            avg = tot / max(cnt, 1)
            lrows = nc * usable
            lookup = {"circuits": nc, "usable_rows": usable, "avg_ms": round(avg, 4),
                      "rows_per_s": round(lrows / (avg * 1e-3)),
                      "algorithmic_GBs": round(lrows * 176 / (avg * 1e-3) / 1e9, 1),
                      "all_rows_in_table": bool((lbad == -1).all().item())}
            del lout
        except Exception as e:  # reported, never masks the headline
            lookup = {"error": repr(e)}
    hasher_aux = None
    if world == 1 and args.hasher_messages > 0:
        try:
            import hashlib

            from b2f import hasher
            hm = args.hasher_messages
            buf = np.random.default_rng(3).integers(0, 256, (hm, 1024), dtype=np.uint8)
            msgs = [bytes(r) for r in buf]
            plan = hasher.Plan(msgs)
            hasher.run_plan(eng, plan)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res = hasher.run_plan(eng, plan)
            el2 = time.perf_counter() - t2
            ok = res.verified and all(res.digests[i] == hashlib.blake2b(msgs[i]).digest()
                                      for i in range(0, hm, max(1, hm // 64)))
            hasher_aux = {"messages": hm, "bytes_each": 1024, "block_steps": plan.steps,
                          "compressions": int(plan.start[-1]), "ms": round(el2 * 1e3, 3),
                          "compressions_per_s": round(int(plan.start[-1]) / el2),
                          "digests_match_hashlib": ok,
                          "note": "wall clock incl. block upload and h' download"}
        except Exception as e:
            hasher_aux = {"error": repr(e)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.rounds, mix, args.cpu_seconds)

    if rank == 0:
        workload = ("%d x %s-round BLAKE2f compressions per GPU: Table16 witness fill + "
                    "constraint eval (LAYOUT v1)" % (n, "{1,4,12}-mixed" if mix else args.rounds))
        out = {"metric": "BLAKE2f compressions/sec (witness+constraint eval), 2^18 batch, "
                         "1/2/4/8 GPU",
               "value": round(value, 1), "unit": "compressions/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
               "data": "synthetic (seeded splitmix64 h/m/t/f)",
               "config": {"workload": workload, "batch_per_gpu": n,
                          "rounds": "mix{1,4,12}" if mix else args.rounds,
                          "rows_per_gpu": rows, "trace_bytes_per_gpu": rows * ROW_BYTES,
                          "path": args.path,
                          "parallelism": "dp%d (instance shards)" % world},
               "roofline": roof, "cpu_baseline": cpu, "kernels": kern, "floors": floors,
               "other_path": aux,
               "collectives": collectives, "witness_gather": witness_gather,
               "fp_export": fp_export, "lookup_columns": lookup, "hasher": hasher_aux,
               "gpu_vs_cpu": round(value / cpu["value"], 1) if cpu else None}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
