"""GPU parity of the fused fill + eval path (b2f_fill_eval_dev, csrc/b2f_fused.hip).

The fused kernel must produce exactly what b2f_fill_dev followed by b2f_eval_dev produce --
the trace, h' and the MockProver verdict -- and therefore what the CPU oracle produces. Fault
injection (b2f_debug_inject) flips one cell as the fused kernel assigns it; the trace it writes
then differs from the clean one in exactly that cell, and its verdict must equal the verdict
of b2f_eval_dev and of the oracle on that written trace. Faults are placed where the fused
kernel's wave tiles make things special: both sides of every init / half-round / final tile
boundary (copy sources recomputed from the producer side, gates whose rows run past the tile
and are deferred to the written trace), the zero tail and the last rows of the trace. Every
test here needs an MI355X (`-m gpu`)."""
import os

import numpy as np
import pytest

from conftest import random_inputs

pytestmark = pytest.mark.gpu

NONE = 2**64 - 1


def _as_oracle(x, orc):
    return np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()


def _stream():
    import torch

    return torch.cuda.current_stream().cuda_stream


def _fused(engine, x, total_rows=None, inject=None):
    """One b2f_fill_eval_dev call on a fresh DeviceBatch (buffers poisoned first)."""
    import b2f

    batch = b2f.DeviceBatch(x, total_rows=total_rows)
    batch.advice.fill_(-1)
    batch.fixed.fill_(-1)
    try:
        if inject is not None:
            engine.debug_inject(*inject)
        batch.fill_evaluate(engine)
        engine.sync(_stream())
    finally:
        engine.debug_inject(None)
    return batch


@pytest.mark.parametrize("rounds_choices,n,seed", [((12,), 23, 31), ((0, 1, 4, 12, 13), 71, 32),
                                                   ((1,), 200, 33), ((0,), 9, 35),
                                                   ((2, 3), 1000, 36), ((12,), 1, 37), ((1,), 1, 38),
                                                   ((25, 0), 50, 39), ((100,), 2, 40)])
def test_fused_equals_oracle(engine, orc, rounds_choices, n, seed):
    """Single instances and runs of zero-round instances included: the half-round launch walks
    whole instances (a wave skips instances without half-rounds and carries the state from tile
    to tile)."""
    x = random_inputs(n, rounds_choices, seed)
    batch = _fused(engine, x)
    adv, fixed = batch.host_trace()
    oadv, ofixed, oh, ooff = orc.fill(_as_oracle(x, orc))
    for c in range(10):
        bad = np.nonzero(adv[c] != oadv[c])[0]
        assert bad.size == 0, "a_%d differs at rows %s" % (c, bad[:10])
    assert np.array_equal(fixed, ofixed)
    assert np.array_equal(batch.host_h_out(), oh)
    rep = batch.report_dict()
    assert rep == orc.evaluate(adv, fixed, ooff)
    assert rep["first_failure"] == NONE and rep["rows_checked"] == int(ooff[-1])


@pytest.mark.parametrize("pad", [4, 252, 256, 1028])
def test_fused_padded_tail(engine, orc, pad):
    """total_rows past the batch (zero tail tiles of 64 quads, the last one partial): zero
    rows, clean."""
    import b2f

    x = random_inputs(9, (1, 4), 34)
    total = int(b2f.offsets(x)[-1]) + pad
    batch = _fused(engine, x, total_rows=total)
    adv, fixed = batch.host_trace()
    used = batch.used_rows
    assert not adv[:, used:].any() and not fixed[used:].any()
    rep = batch.report_dict()
    assert rep == orc.evaluate(adv, fixed, batch.offsets_host) and rep["first_failure"] == NONE


@pytest.mark.parametrize("pad", [0, 4, 8, 12, 16, 20, 24, 28])
def test_fused_every_line_offset(engine, orc, pad):
    """The half-round tiles store whole 128-byte lines: each tile also writes the previous
    tile's last quads that share its first line (recomputed from the producer chain) and leaves
    its own last quads to the next tile. Column c's line offset at a tile is (c total_rows +
    row) mod 32 rows, so total_rows = used + pad over pad = 0 .. 28 puts every column at every
    offset; the trace must equal the oracle's at each."""
    import b2f

    x = random_inputs(11, (1, 2, 5), 40 + pad)
    total = int(b2f.offsets(x)[-1]) + pad
    batch = _fused(engine, x, total_rows=total)
    adv, fixed = batch.host_trace()
    oadv, ofixed, oh, ooff = orc.fill(_as_oracle(x, orc))
    used = batch.used_rows
    for c in range(10):
        bad = np.nonzero(adv[c, :used] != oadv[c])[0]
        assert bad.size == 0, "pad %d: a_%d differs at rows %s" % (pad, c, bad[:10])
    assert np.array_equal(fixed[:used], ofixed)
    assert not adv[:, used:].any() and not fixed[used:].any()
    rep = batch.report_dict()
    assert rep == orc.evaluate(adv, fixed, batch.offsets_host) and rep["first_failure"] == NONE


def _boundary_rows(total, starts, rng, k):
    """Rows on both sides of the given tile starts, the first/last rows, and random rows."""
    rows = set()
    for t in starts:
        for d in (-16, -13, -12, -9, -5, -4, -1, 0, 1, 3, 4, 11, 15, 29, 45, 51):
            r = t + d
            if 0 <= r < total:
                rows.add(r)
    rows.update([0, 1, 2, 3, total - 1, total - 2, total - 4, total - 8, total - 12])
    rows = sorted(rows)
    pick = list(rng.choice(rows, size=min(k, len(rows)), replace=False))
    pick += list(rng.integers(0, total, k // 4))
    return [int(r) for r in pick]


def _tile_rows(x):
    """First rows of the fused kernel's tiles (init, every half-round, final) and of the zero
    tail's 64-quad tiles."""
    import b2f

    off = b2f.offsets(x)
    out = []
    for i, r in enumerate(x["rounds"]):
        o = int(off[i])
        out += [o, o + 164] + [o + 164 + 208 * h for h in range(1, 2 * int(r))] + \
            [o + 164 + 416 * int(r)]
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fused_injection_matches_eval(engine, orc, seed):
    """Fused verdict == b2f_eval_dev verdict on the trace the fused kernel wrote, for single
    cell faults in every column (advice and fixed) on both sides of the fused kernel's tile
    boundaries (init / half-round / final tiles: copy sources recomputed from the producer
    side, gates deferred past the tile end) and at random rows; the written trace differs from
    the clean one in exactly the injected cell; a subset is checked against the oracle too."""
    import torch

    rng = np.random.default_rng(40 + seed)
    x = random_inputs(24, (0, 1, 4, 12), 41 + seed)
    clean = _fused(engine, x)
    cadv, cfix = clean.advice.clone(), clean.fixed.clone()
    total = clean.total_rows
    flagged = 0
    cases = 0
    for r in _boundary_rows(total, _tile_rows(x), rng, 96):
        for col in rng.choice(11, size=2, replace=False):
            col = int(col)
            bit = int(rng.integers(0, 16 if col == 10 and rng.random() < 0.7 else 32))
            batch = _fused(engine, x, inject=(r, col, 1 << bit))
            dadv = (batch.advice != cadv).nonzero().cpu().numpy()
            dfix = (batch.fixed != cfix).nonzero().cpu().numpy()
            if col < 10:
                assert dadv.tolist() == [[col, r]] and dfix.size == 0, (r, col, bit)
            else:
                assert dadv.size == 0 and dfix.reshape(-1).tolist() == [r], (r, col, bit)
            got = batch.report_dict()
            batch.evaluate(engine)  # the standalone eval on the written trace
            engine.sync(_stream())
            ref = batch.report_dict()
            assert got == ref, (r, col, bit, got, ref)
            if cases % 8 == 0:
                adv, fixed = batch.host_trace()
                assert got == orc.evaluate(adv, fixed, batch.offsets_host), (r, col, bit)
            flagged += got["first_failure"] != NONE
            cases += 1
            del batch
            torch.cuda.empty_cache()
    assert flagged > cases // 3


def test_fused_injection_last_rows(engine, orc):
    """Selector bits injected into the last rows of the trace: gates that run past the end
    read zero rows (the eval's out-of-trace rule) -- through the fused kernel's zero halo."""
    import b2f

    x = random_inputs(5, (1,), 42)
    total = int(b2f.offsets(x)[-1])
    total_p = ((total + 1023) // 1024) * 1024  # trace ends exactly on a tile boundary
    for total_rows in (total, total_p):
        for r in (total_rows - 1, total_rows - 3, total_rows - 7, total_rows - 12):
            for bit in (0, 1, 4, 6, 8, 11, 13, 15):
                batch = _fused(engine, x, total_rows=total_rows, inject=(r, 10, 1 << bit))
                got = batch.report_dict()
                adv, fixed = batch.host_trace()
                assert got == orc.evaluate(adv, fixed, batch.offsets_host), (total_rows, r, bit)


def test_fused_2p16_equals_fill_eval(engine):
    """BASELINE config 2 size: the fused trace, h' and verdict equal fill_dev + eval_dev's
    (compared on the device; fill_dev itself is diffed against the oracle at this size in
    test_gpu_parity.test_device_batch_2p16_bitexact)."""
    import b2f
    import torch

    from b2f import synth

    x = synth.batch(1 << 16, rounds=12)
    a = b2f.DeviceBatch(x)
    a.fill(engine)
    a.evaluate(engine)
    engine.sync(_stream())
    ra = a.report_dict()
    b = _fused(engine, x)
    assert torch.equal(a.advice, b.advice) and torch.equal(a.fixed, b.fixed)
    assert torch.equal(a.h_out, b.h_out)
    assert b.report_dict() == ra and ra["first_failure"] == NONE


def test_fused_mixed_rounds_2p14(engine, orc):
    """BASELINE config 5 shape (rounds in {1, 4, 12}) at 2^14, oracle-checked in chunks."""
    import b2f
    from b2f import synth

    n = 1 << 14
    x = synth.batch(n, rounds_mix=[1, 4, 12])
    batch = _fused(engine, x)
    rep = batch.report_dict()
    assert rep["first_failure"] == NONE and sum(rep["gate_failures"]) == 0
    off = batch.offsets_host
    h_out = batch.host_h_out()
    for s in range(0, n, 4096):
        e = min(n, s + 4096)
        oadv, ofixed, oh, _ = orc.fill(_as_oracle(x[s:e], orc))
        r0, r1 = int(off[s]), int(off[e])
        assert np.array_equal(batch.advice[:, r0:r1].cpu().numpy().view(np.uint32), oadv)
        assert np.array_equal(batch.fixed[r0:r1].cpu().numpy().view(np.uint32), ofixed)
        assert np.array_equal(h_out[s:e], oh)
    del b2f


def test_2p18_mixed_split_equals_fused(engine, orc):
    """BASELINE config 5 at full size (2^18, rounds in {1, 4, 12}) through size-independent
    properties: both paths' verdicts are clean, the fused trace and h' equal the split path's
    bit for bit (compared on the device), and h' of a sample of instances equals the oracle's
    BLAKE2f compression."""
    import b2f
    import torch

    from b2f import synth

    n = 1 << 18
    x = synth.batch(n, rounds_mix=[1, 4, 12])
    a = b2f.DeviceBatch(x)
    a.fill(engine)
    a.evaluate(engine)
    engine.sync(_stream())
    ra = a.report_dict()
    assert ra["first_failure"] == NONE and sum(ra["gate_failures"]) == 0
    adv, fx, h = a.advice.clone(), a.fixed.clone(), a.h_out.clone()
    a.fill_evaluate(engine)
    engine.sync(_stream())
    assert a.report_dict() == ra
    assert torch.equal(a.advice, adv) and torch.equal(a.fixed, fx) and torch.equal(a.h_out, h)
    del adv, fx
    rng = np.random.default_rng(50)
    h_host = h.cpu().numpy().view(np.uint64)
    for i in rng.integers(0, n, 256):
        r = x[int(i)]
        ref = orc.compress(int(r["rounds"]), r["h"], r["m"], r["t"], int(r["f"]))
        assert np.array_equal(h_host[int(i)], ref), int(i)


def test_2p18x12_fused_equals_split_past_2p30(engine, orc):
    """BASELINE config 3 at full size, on the headline path itself: 2^18 uniform 12-round
    instances = 1.368 G rows, so every column runs past row 2^30 and past 4 GiB of bytes.
    The fused kernel's verdict reads its wave's LDS staging, not HBM, so it cannot see a
    store-address error; this test can. (1) The fused trace, fixed column and h' written over
    poisoned buffers equal the split path's (fill_dev + eval_dev) bit for bit on the device,
    with the same clean verdict. (2) Instances whose rows lie past 2^30 (a random sample plus
    the first and last of them) equal the oracle's fill of those instances. (3) Single-cell
    faults injected past row 2^30 as the fused kernel assigns them change exactly that cell of
    the written trace, and the fused verdict equals b2f_eval_dev's on the written trace and
    the oracle's on the faulted instance (re-based to the global row)."""
    import b2f
    import torch

    from b2f import synth

    n = 1 << 18
    x = synth.batch(n, rounds=12)
    a = b2f.DeviceBatch(x)
    a.fill(engine)
    a.evaluate(engine)
    engine.sync(_stream())
    ra = a.report_dict()
    assert ra["first_failure"] == NONE and ra["rows_checked"] == a.used_rows
    assert a.used_rows > 1 << 30 and a.used_rows * 4 > 1 << 32
    adv, fx, h = a.advice.clone(), a.fixed.clone(), a.h_out.clone()
    a.advice.fill_(-1)
    a.fixed.fill_(-1)
    a.h_out.fill_(-1)
    a.fill_evaluate(engine)
    engine.sync(_stream())
    assert a.report_dict() == ra
    for c in range(10):
        assert torch.equal(a.advice[c], adv[c]), "fused a_%d != split a_%d" % (c, c)
    assert torch.equal(a.fixed, fx) and torch.equal(a.h_out, h)

    off = a.offsets_host
    first_past = int(np.searchsorted(off, 1 << 30, side="right")) - 1  # holds row 2^30
    assert 200000 < first_past < n - 40000
    rng = np.random.default_rng(60)
    sample = sorted({first_past, first_past + 1, n - 1}
                    | {int(i) for i in rng.integers(first_past, n, 45)})
    h_host = a.host_h_out()
    for i in sample:
        oadv, ofixed, oh, _ = orc.fill(_as_oracle(x[i:i + 1], orc))
        r0, r1 = int(off[i]), int(off[i + 1])
        assert np.array_equal(a.advice[:, r0:r1].cpu().numpy().view(np.uint32), oadv), i
        assert np.array_equal(a.fixed[r0:r1].cpu().numpy().view(np.uint32), ofixed), i
        assert np.array_equal(h_host[i], oh[0]), i

    # (instance, column (10 = fixed), row inside the instance, bit): a half-round a1 limb, an
    # XOR63 cell, a selector bit, an XOR3 operand (a copy) of the last instance, the lookup
    # cell of the first row past 2^30
    cross = (1 << 30) - int(off[first_past])
    faults = [(n - 3, 1, 164 + 416 * 7 + 52 * 2 + 3, 5), (230001, 8, 164 + 416 * 4 + 46, 0),
              (250000, 10, 164 + 416 * 10 + 52 * 1 + 4, 2), (n - 1, 5, 164 + 416 * 12 + 8, 9),
              (first_past, 1, cross, 11)]
    for i, c, r, b in faults:
        r0, r1 = int(off[i]), int(off[i + 1])
        row = r0 + r
        assert row >= 1 << 30 and row < r1
        try:
            engine.debug_inject(row, c, 1 << b)
            a.fill_evaluate(engine)
            engine.sync(_stream())
        finally:
            engine.debug_inject(None)
        got = a.report_dict()
        if c < 10:
            for cc in range(10):
                d = (a.advice[cc] != adv[cc]).nonzero().reshape(-1).tolist()
                assert d == ([row] if cc == c else []), (i, c, r, cc, d[:4])
            assert torch.equal(a.fixed, fx)
        else:
            for cc in range(10):
                assert torch.equal(a.advice[cc], adv[cc])
            assert (a.fixed != fx).nonzero().reshape(-1).tolist() == [row]
        assert torch.equal(a.h_out, h)
        a.evaluate(engine)  # the standalone eval on the trace the fused kernel wrote
        engine.sync(_stream())
        assert a.report_dict() == got, (i, c, r, b)
        iadv = a.advice[:, r0:r1].cpu().numpy().view(np.uint32)
        ifx = a.fixed[r0:r1].cpu().numpy().view(np.uint32)
        o = orc.evaluate(iadv, ifx, np.array([0, r1 - r0], dtype=np.uint64))
        assert o["first_failure"] != NONE, (i, c, r, b)
        want = dict(o, rows_checked=a.used_rows, first_failure=o["first_failure"] + (r0 << 8))
        assert got == want, (i, c, r, b, got, want)
    del adv, fx, h
    torch.cuda.empty_cache()


def test_fused_long_instance_is_segmented(engine, orc):
    """an instance far longer than the rest (10^4 rounds, 20,000 half-round tiles) in
    a batch of 12-round ones. The half-round launch walks it in segments of SEG_HR half-rounds,
    the later ones from recorded states on whichever waves are free, so it no longer runs at one
    wave's speed: fused trace == split trace column by column, h' and verdict equal, oracle
    samples at segment starts, and the pass takes a few ms (one wave alone took ~100 ms)."""
    import time

    import torch

    import b2f

    x = random_inputs(4096, (12,), 91)
    x["rounds"][1777] = 10000
    fused = _fused(engine, x)
    split = b2f.DeviceBatch(x)
    split.fill(engine)
    split.evaluate(engine)
    engine.sync(_stream())
    for c in range(10):
        assert torch.equal(fused.advice[c], split.advice[c]), "a_%d" % c
    assert torch.equal(fused.fixed, split.fixed)
    assert torch.equal(fused.h_out, split.h_out)
    rep = fused.report_dict()
    assert rep == split.report_dict() and rep["first_failure"] == NONE
    # oracle on the long instance alone, compared at its segment starts (rows of half-rounds
    # 24 m - 1 .. 24 m)
    one = x[1777:1778].copy()
    oadv, ofixed, oh, _ = orc.fill(_as_oracle(one, orc))
    base = int(fused.offsets_host[1777])
    adv = fused.advice[:, base: base + oadv.shape[1]].cpu().numpy().view(np.uint32)
    for m in (1, 2, 417, 833):
        lo = 164 + 208 * (24 * m - 1)
        assert np.array_equal(adv[:, lo: lo + 416], oadv[:, lo: lo + 416]), m
    assert np.array_equal(fused.host_h_out()[1777], oh[0])
    # time: the pass with the long instance vs without it
    s = _stream()
    engine.set_timing(True)
    for _ in range(3):
        fused.fill_evaluate(engine, s)
    t_long = engine.kernel_times()["fill_eval"][0] / 3
    x2 = x.copy()
    x2["rounds"][1777] = 12
    b2 = b2f.DeviceBatch(x2)
    b2.fill_evaluate(engine, s)
    engine.sync(s)
    engine.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(3):
        b2.fill_evaluate(engine, s)
    t_base = engine.kernel_times()["fill_eval"][0] / 3
    print("fused fill+eval: %.3f ms with the 10^4-round instance, %.3f ms without (%.1f s wall)"
          % (t_long, t_base, time.perf_counter() - t0))
    assert t_long < 30.0


def test_fused_injection_at_segment_starts(engine, orc):
    """Faults on both sides of the segment boundaries of 25-round instances (half-round 24 starts
    a listed segment on another wave): fused verdict == b2f_eval_dev verdict == oracle."""
    x = random_inputs(6, (25,), 92)
    clean = _fused(engine, x)
    off = clean.offsets_host
    cases = 0
    for i in (0, 3, 5):
        b = int(off[i]) + 164 + 208 * 24  # first row of half-round 24
        for r in (b - 29, b - 4, b - 1, b, b + 3, b + 51):
            for col in (1, 3, 10):
                batch = _fused(engine, x, inject=(r, col, 1 << (cases % 13)))
                got = batch.report_dict()
                batch.evaluate(engine)
                engine.sync(_stream())
                assert got == batch.report_dict(), (i, r, col)
                adv, fixed = batch.host_trace()
                assert got == orc.evaluate(adv, fixed, off), (i, r, col)
                cases += 1


def test_max_rounds_instance(engine, orc):
    """An instance at B2F_MAX_ROUNDS (2^20 rounds: 436 M rows, 19 GB of trace, 87,381 listed
    segments of the fused launch) among 12-round ones: h' equals the oracle's compression
    (oracle.compress, the same rounds), the fused and split traces are equal column by column,
    both verdicts are clean, and a fault near the instance's end is reported at the same row by
    the fused pass and by b2f_eval_dev (the eval's exact kernel then runs over 436 M rows)."""
    import torch

    import b2f

    x = random_inputs(8, (12,), 95)
    i = 5
    x["rounds"][i] = b2f._lib.MAX_ROUNDS
    fused = _fused(engine, x)
    rep = fused.report_dict()
    assert rep["first_failure"] == NONE and rep["rows_checked"] >= fused.used_rows
    want = orc.compress(int(x["rounds"][i]), x["h"][i], x["m"][i], x["t"][i], int(x["f"][i]))
    assert np.array_equal(fused.host_h_out()[i], np.asarray(want, dtype=np.uint64))
    split = b2f.DeviceBatch(x)
    split.fill(engine)
    split.evaluate(engine)
    engine.sync(_stream())
    assert split.report_dict() == rep
    for c in range(10):
        assert torch.equal(fused.advice[c], split.advice[c]), "a_%d" % c
    assert torch.equal(fused.fixed, split.fixed) and torch.equal(fused.h_out, split.h_out)
    del split
    torch.cuda.empty_cache()
    # a fault in the instance's last half-round: fused verdict == split eval's
    r = int(fused.offsets_host[i + 1]) - 64 - 100
    bad = _fused(engine, x, inject=(r, 3, 1 << 5))
    got = bad.report_dict()
    assert got["first_failure"] != NONE and (got["first_failure"] >> 8) <= r + 2
    bad.evaluate(engine)
    engine.sync(_stream())
    assert bad.report_dict() == got
