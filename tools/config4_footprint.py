"""BASELINE configs[3] (2^20 x 12-round compressions sharded over 8 GPUs) per-rank memory plan,
run on ONE MI355X without RCCL: allocate a rank's footprint at full size --
its 2^17-instance shard (30.1 GB), the [11, 8 W] gathered table (240.8 GB) and the compaction
staging (0.74 GB) -- fill + evaluate the shard (fused path) in its window, place it into two
slots of the table as the all-gather would (slot 0 and slot 7; a single process cannot receive
the other ranks' rows), and run dist.compact_windows over the last two windows as if slot 6's
shard were one instance short (the unequal-shard path, 30 GB moved through the staging buffer).
Prints one JSON line with the byte budget, free HBM at the peak, times and checks."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    import torch

    import b2f
    from b2f import dist as bdist
    from b2f import synth

    world, global_n, rounds = 8, 1 << 20, 12
    dev = "cuda:0"
    xr = synth.rounds_of(global_n, rounds=rounds)
    shards = bdist.plan_shards(xr, world)
    srows, sbase = bdist.shard_rows(xr, shards)
    w = bdist.trace_window(srows)
    lo, hi = shards[0]
    res = {"config": "2^20 x 12-round over 8 ranks (rank 0's footprint)", "window_rows": w,
           "shard_instances": hi - lo}
    free0, total = torch.cuda.mem_get_info(0)
    res["hbm_total_gb"] = round(total / 1e9, 1)
    res["free_at_start_gb"] = round(free0 / 1e9, 1)
    eng = b2f.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    t0 = time.perf_counter()
    batch = b2f.DeviceBatch(synth.batch(hi - lo, rounds=rounds, first=lo), device=dev, total_rows=w)
    log("shard allocated: %.1f GB" % (w * 44 / 1e9))
    batch.fill_evaluate(eng, s)
    eng.sync(s)
    rep = batch.report_dict()
    torch.cuda.synchronize()
    eng.set_timing(True)
    batch.fill_evaluate(eng, s)
    eng.sync(s)
    res["fill_eval_ms"] = round(eng.kernel_times()["fill_eval"][0], 3)
    res["shard_verdict_clean"] = rep["first_failure"] == 2**64 - 1 and batch.report_dict()["first_failure"] == 2**64 - 1
    res["shard_gb"] = round((w * 44 + (hi - lo) * (216 + 64 + 8)) / 1e9, 2)
    log("shard filled + evaluated", res["fill_eval_ms"], "ms")
    gather_bytes = bdist.gather_trace_bytes(srows)
    out = torch.empty((11, world * w), dtype=torch.int32, device=dev)
    stage = torch.empty((11, min(bdist.STAGE_ROWS, w)), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    free_peak = torch.cuda.mem_get_info(0)[0]
    res["gather_buffers_gb"] = round(gather_bytes / 1e9, 2)
    res["free_at_peak_gb"] = round(free_peak / 1e9, 2)
    res["torch_reserved_gb"] = round(torch.cuda.memory_reserved(0) / 1e9, 2)
    log("gather buffers allocated; free %.2f GB" % (free_peak / 1e9))
    # the all-gather's placement of this rank's window into slots 0 and 7
    tg = time.perf_counter()
    for slot in (0, world - 1):
        out[:10, slot * w:(slot + 1) * w].copy_(batch.advice)
        out[10, slot * w:(slot + 1) * w].copy_(batch.fixed)
        torch.cuda.synchronize()
        log("slot %d placed" % slot)
    res["place_two_slots_s"] = round(time.perf_counter() - tg, 2)
    # slot 6 <- slot 7's copy of the shard so windows 6, 7 both hold it; then compact as if
    # shard 6 were one instance (5,220 rows) short: window 7 moves down by 5,220 rows
    out[:, 6 * w:7 * w].copy_(out[:, 7 * w:8 * w])
    torch.cuda.synchronize()
    short = w - b2f.layout.rows(rounds)
    view = out[:, 6 * w:]
    tc = time.perf_counter()
    bdist.compact_windows(view, [short, w], w, torch, stage=stage)
    torch.cuda.synchronize()
    res["compaction_s"] = round(time.perf_counter() - tc, 2)
    res["compaction_moved_gb"] = round(w * 44 / 1e9, 1)
    log("compacted in %.2f s" % res["compaction_s"])
    # checks: slot 0 == the shard; the moved window starts at row `short` of slot 6 and equals
    # the shard; the tail after it is zero (sampled columns and rows)
    ok0 = bool(torch.equal(out[:10, :w], batch.advice)) and bool(torch.equal(out[10, :w], batch.fixed))
    ok7 = True
    for c in (0, 1, 5, 9):
        ok7 &= bool(torch.equal(view[c, short:short + w], batch.advice[c]))
    ok7 &= bool(torch.equal(view[10, short:short + w], batch.fixed))
    ok7 &= bool((view[:, short + w:] == 0).all().item())
    res["slot0_equals_shard"] = ok0
    res["compacted_window_equals_shard"] = ok7
    res["total_plan_gb"] = round(res["shard_gb"] + res["gather_buffers_gb"], 2)
    res["wall_s"] = round(time.perf_counter() - t0, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
