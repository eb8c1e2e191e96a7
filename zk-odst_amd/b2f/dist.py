"""Multi-GPU sharding of a batch of independent compressions.

Instances are independent: each rank fills and evaluates a contiguous shard with no
data-path collective. The exchanges are the results: the verdict counters (all_reduce), the
64-byte h' per instance (one all_gather) and, when the caller wants the whole witness table on
every rank, one all-gather per column straight into the final column-major buffers
(gather_trace). RCCL has no all_gather_v, so unequal shards are gathered in windows padded to
the widest shard and compacted in place afterwards.

Memory at BASELINE config 4 (2^20 x 12-round compressions over 8 ranks, R = 5,220 rows,
44 B per row): each rank's shard is 2^17 x 5,220 rows = 30.1 GB; the gathered table is
[11][8 W] u32 with W = the widest shard's rows, 241 GB; the compaction staging buffer is
11 x 2^24 x 4 B = 0.74 GB. Total ~272 GB of the 288 GB HBM3E per GPU.
"""
import numpy as np

from .layout import as_inputs, offsets

# int64 words of b2f_eval_report: 16 gates, lookup, copy, first_failure, rows_checked, fixed
REPORT_WORDS = 21
W_LOOKUP, W_COPY, W_FIRST, W_ROWS, W_FIXED = 16, 17, 18, 19, 20
NONE = np.iinfo(np.int64).max
STAGE_ROWS = 1 << 24  # compaction staging rows per pass (x 11 columns x 4 B = 0.74 GB)


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


def shard_rows(inputs, shards):
    """(rows of each shard, global row offset of each shard) for plan_shards' ranges."""
    off = offsets(as_inputs(inputs))
    rows = [int(off[hi] - off[lo]) for lo, hi in shards]
    return rows, [int(off[lo]) for lo, _ in shards]


def verdict_words(report, row_offset, torch):
    """A rank's report (int64 [21] device tensor, b2f_eval_report bit patterns) -> int64 [20]:
    [0:16] gate, 16 lookup, 17 copy, 18 fixed counters, 19 first failure made global
    ((row + row_offset) << 8 | code; INT64_MAX when clean) -- ready for SUM over [0:19] and MIN
    over [19]. No host synchronisation."""
    r = report.view(torch.int64)
    out = torch.empty(20, dtype=torch.int64, device=r.device)
    out[:18].copy_(r[:18])
    out[18] = r[W_FIXED]
    first = r[W_FIRST]
    out[19] = torch.where(first == -1, torch.full_like(first, NONE), first + (int(row_offset) << 8))
    return out


def all_reduce_verdict(words, dist, group=None):
    """Combine verdict_words over the ranks in place (counters summed, first failure min)."""
    dist.all_reduce(words[:19], op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(words[19:20], op=dist.ReduceOp.MIN, group=group)
    return words


def reduce_report(rep, dist, torch, device, row_offset=0, group=None):
    """Combine the ranks' verdict dicts: counters and rows summed, first failure = the minimum
    over ranks of the GLOBAL row key ((rank-local row + the shard's first global row) << 8 |
    code), so it names the failing row of the whole batch's trace."""
    v = list(rep["gate_failures"]) + [rep["lookup_failures"], rep["copy_failures"],
                                      rep.get("fixed_failures", 0)]
    first = rep["first_failure"]
    first = NONE if first == 2**64 - 1 else first + (int(row_offset) << 8)
    t = torch.tensor(v + [first, rep["rows_checked"]], dtype=torch.int64, device=device)
    counts = t[:19].clone()
    dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    fmin = t[19:20].clone()
    dist.all_reduce(fmin, op=dist.ReduceOp.MIN, group=group)
    rows = t[20:21].clone()
    dist.all_reduce(rows, op=dist.ReduceOp.SUM, group=group)
    f = int(fmin.item())
    return {"gate_failures": [int(x) for x in counts[:16].tolist()],
            "lookup_failures": int(counts[16].item()), "copy_failures": int(counts[17].item()),
            "first_failure": 2**64 - 1 if f == NONE else f, "rows_checked": int(rows.item()),
            "fixed_failures": int(counts[18].item())}


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


def trace_window(rows_per_rank):
    """W: the per-rank window every rank's trace buffers are allocated with (the widest
    shard's rows; a multiple of 4 as every R(rounds) is)."""
    w = max(rows_per_rank)
    return w + (-w) % 4


def gather_trace_bytes(rows_per_rank):
    """HBM bytes gather_trace allocates on every rank (result + staging)."""
    world, w = len(rows_per_rank), trace_window(rows_per_rank)
    return 11 * 4 * (world * w + min(STAGE_ROWS, w))


def _gather_coalesced(out, cols, dist, group, dev):
    """The eleven column all-gathers as one coalesced group (torch's private
    _coalescing_manager; RCCL issues them between one group start/end). Returns False, having
    issued nothing, when this torch or backend cannot coalesce (no such API, another signature,
    or a backend without startCoalescing, as gloo): the caller then runs the plain loop. The
    manager registers the group in its pending-op table before it starts coalescing, so a start
    that raises would leave every later collective of the group queued there; that entry is
    removed on the way out."""
    coalesce = getattr(dist, "_coalescing_manager", None)
    if coalesce is None:
        return False
    issued = []
    try:
        with coalesce(group=group, device=dev):
            for c in range(11):
                dist.all_gather_into_tensor(out[c], cols[c], group=group)
                issued.append(c)
        return True
    except (RuntimeError, TypeError, ValueError, NotImplementedError):
        if issued:  # a failure after ops were queued is not a capability problem
            raise
        c10d = getattr(dist, "distributed_c10d", None)
        state = getattr(getattr(c10d, "_world", None), "pg_coalesce_state", None)
        if state is not None:
            state.pop(group if group is not None else c10d._get_default_group(), None)
        return False


def gather_trace(adv_local, fixed_local, rows_per_rank, dist, torch, group=None, out=None,
                 coalesce=None):
    """The whole batch's witness table on every rank.

    adv_local [10, W] and fixed_local [W] (int32 bit patterns): this rank's trace, allocated
    with the common window W = trace_window(rows_per_rank) rows (b2f_fill_dev writes zeros past
    the shard's used rows). Returns (advice [10, world * W], fixed [world * W]) -- views of one
    [11, world * W] buffer (`out`, allocated when None) -- holding every rank's used rows back
    to back from row 0, in rank order, and zeros after: exactly the trace one process would
    fill for the whole batch with total_rows = world * W.

    One all_gather_into_tensor per column, straight into that column of the result (no
    pad-and-cat copies; on RCCL the eleven calls are issued in one coalesced group, falling back
    to the plain loop where this torch cannot coalesce; `coalesce` forces the attempt (True) or
    the loop (False), default: RCCL only), then an
    in-place compaction of the padded windows through a bounded staging buffer: rank k's rows
    move from k * W down to the prefix sum of the shards before it, in increasing row order, so
    a staged chunk never overwrites rows that still have to move."""
    world = len(rows_per_rank)
    w = adv_local.shape[1]
    if w != trace_window(rows_per_rank) or fixed_local.shape[0] != w:
        raise ValueError("gather_trace: local trace has %d rows, window is %d"
                         % (w, trace_window(rows_per_rank)))
    dev = adv_local.device
    if out is None:
        out = torch.empty((11, world * w), dtype=adv_local.dtype, device=dev)
    cols = [adv_local[c] for c in range(10)] + [fixed_local]
    if coalesce is None:
        coalesce = dist.get_backend(group) == "nccl"
    if not (coalesce and _gather_coalesced(out, cols, dist, group, dev)):
        for c in range(11):
            dist.all_gather_into_tensor(out[c], cols[c], group=group)
    compact_windows(out, rows_per_rank, w, torch)
    return out[:10], out[10]


def compact_windows(out, rows_per_rank, w, torch, stage=None):
    """In place: the padded windows of `out` [cols, world * w] (rank k's rows at k * w) moved
    back to back from row 0 in rank order through a staging buffer of at most STAGE_ROWS rows
    (allocated here unless given), zeros after. Rank k's rows move down, chunk by chunk in
    increasing row order, so a staged chunk never overwrites rows still to move. No-op (no
    staging) when every shard fills its window."""
    dst = 0
    for k, r in enumerate(rows_per_rank):
        src = k * w
        if src != dst and r:
            if stage is None:
                stage = torch.empty((out.shape[0], min(STAGE_ROWS, w)), dtype=out.dtype,
                                    device=out.device)
            for o in range(0, r, stage.shape[1]):
                t = min(stage.shape[1], r - o)
                stage[:, :t].copy_(out[:, src + o: src + o + t])
                out[:, dst + o: dst + o + t].copy_(stage[:, :t])
        dst += r
    out[:, dst:].zero_()
