"""Multi-GPU sharding of a batch of independent compressions.

Instances are independent: each rank fills and evaluates a contiguous shard with no
data-path collective. The only exchanges are the results: the verdict counters
(all_reduce) and the 64-byte h' per instance (one all_gather). RCCL has no all_gather_v, so
unequal shards are padded to the largest shard. Reassembling the whole witness table on every
rank (gather_trace, one all_gather of the 11 columns) is an optional step for batches that
fit one GPU (2^18 x 12 rounds x 8 ranks would be 480 GB).
"""
import numpy as np

from .layout import as_inputs, offsets

REPORT_WORDS = 20  # 16 gates, lookup, copy, first_failure, rows_checked
NONE = np.iinfo(np.int64).max


def plan_shards(inputs, world):
    """Contiguous instance ranges [(lo, hi)] per rank, balanced by rows (prefix sum of
    R(rounds_i)) so mixed-rounds batches balance."""
    off = offsets(as_inputs(inputs)).astype(np.float64)
    n = len(off) - 1
    total = off[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(off, total * r / world, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.minimum(np.array(cuts), n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def report_to_tensor(rep, torch, device):
    """Verdict dict -> int64[20] with first_failure = INT64_MAX when clean (for MIN)."""
    v = list(rep["gate_failures"]) + [rep["lookup_failures"], rep["copy_failures"]]
    first = rep["first_failure"]
    v += [NONE if first == 2**64 - 1 else first, rep["rows_checked"]]
    return torch.tensor(v, dtype=torch.int64, device=device)


def reduce_report(rep, dist, torch, device, group=None):
    """Combine the ranks' verdicts: counters and rows summed, first failure = min.
    Row numbers stay rank-local (each rank owns its own trace)."""
    t = report_to_tensor(rep, torch, device)
    counts = t[:18].clone()
    dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    first = t[18:19].clone()
    dist.all_reduce(first, op=dist.ReduceOp.MIN, group=group)
    rows = t[19:20].clone()
    dist.all_reduce(rows, op=dist.ReduceOp.SUM, group=group)
    f = int(first.item())
    return {"gate_failures": [int(x) for x in counts[:16].tolist()],
            "lookup_failures": int(counts[16].item()), "copy_failures": int(counts[17].item()),
            "first_failure": 2**64 - 1 if f == NONE else f, "rows_checked": int(rows.item())}


def gather_h_out(h_local, shards, dist, torch, group=None):
    """All ranks' h' [n_r, 8] (int64 bit patterns) -> the whole batch [n, 8] in instance
    order, by one all_gather of shards padded to the largest."""
    world = len(shards)
    width = max(hi - lo for lo, hi in shards)
    pad = torch.zeros((width, 8), dtype=h_local.dtype, device=h_local.device)
    pad[: h_local.shape[0]] = h_local
    out = torch.empty((world * width, 8), dtype=h_local.dtype, device=h_local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    parts = [out[r * width: r * width + (hi - lo)] for r, (lo, hi) in enumerate(shards)]
    return torch.cat(parts, dim=0)


def gather_trace(adv_local, fixed_local, shard_rows, dist, torch, group=None):
    """The whole batch's trace on every rank: adv_local [10, rows_r] and fixed_local
    [rows_r] (int32 bit patterns, rows_r = shard_rows[rank]) -> (advice [10, total],
    fixed [total]) with the ranks' rows in order, by one all_gather of the 11 columns padded
    to the largest shard, then one device copy into the column-major layout."""
    world = len(shard_rows)
    width = max(shard_rows)
    rows = adv_local.shape[1]
    pad = torch.zeros((11, width), dtype=adv_local.dtype, device=adv_local.device)
    pad[:10, :rows] = adv_local
    pad[10, :rows] = fixed_local
    out = torch.empty((world, 11, width), dtype=adv_local.dtype, device=adv_local.device)
    dist.all_gather_into_tensor(out.view(world * 11, width), pad, group=group)
    cols = torch.cat([out[r, :, :n] for r, n in enumerate(shard_rows)], dim=1)  # [11, total]
    return cols[:10].contiguous(), cols[10].contiguous()
