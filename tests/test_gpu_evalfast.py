"""The eval's fast clean-check pass (eval_hr_kernel / eval_edge_kernel, csrc/b2f_fused.hip) in
front of the exact eval kernel: a clean trace must cost the fast pass only (the exact kernel is
skipped by its device-side gate), and any corruption the pass sees must hand the trace to the exact
kernel, whose report then equals the oracle's. The fast pass checks a wave's band of consecutive
half-round tiles with the limb table (the state words' canonical cells as the half-round starts)
carried from the previous tile's staging; the cases below put faults in those carried cells, at band
and instance boundaries, on mixed rounds (bands that cross instances). Needs an MI355X (`-m gpu`)."""
import numpy as np
import pytest

from conftest import random_inputs

pytestmark = pytest.mark.gpu

NONE = 2**64 - 1
INIT_ROWS, ROUND_ROWS, G_ROWS = 164, 416, 52


def _dev_eval(engine, batch, adv, fixed):
    import torch

    batch.advice.copy_(torch.from_numpy(adv.view(np.int32)).to(batch.advice.device))
    batch.fixed.copy_(torch.from_numpy(fixed.view(np.int32)).to(batch.fixed.device))
    batch.evaluate(engine)
    path = engine.debug_eval_path()
    return path, batch.report_dict()


def _canon_rows(off, rounds, hr):
    """Instance-local rows of the canonical state cells as half-round hr (>= 1) starts (a2 / b2 /
    c2 / d2 blocks of the G's of half-round hr - 1; LAYOUT.md, b2f_layout.h canon_state)."""
    hp = hr - 1
    rp = hp >> 1
    rows = []
    for g4 in range(4):
        g = g4 + 4 * (hp & 1)
        gb = INIT_ROWS + ROUND_ROWS * rp + G_ROWS * g
        rows += [(1, gb + 28), (2, gb + 28 + 3), (7, gb + 44), (8, gb + 46), (1, gb + 40 + 1),
                 (2, gb + 32 + 2), (1, gb + 32 + 6)]
    return [(c, off + r) for c, r in rows]


@pytest.mark.parametrize("rounds_choices,n,seed", [((12,), 600, 41), ((1, 4, 12, 13), 700, 42),
                                                   ((2, 3), 900, 43)])
def test_fast_pass_clean_and_carried_faults(engine, orc, rounds_choices, n, seed):
    import b2f

    x = random_inputs(n, rounds_choices, seed)
    batch = b2f.DeviceBatch(x)
    batch.fill(engine)
    engine.sync(0)
    adv, fixed = batch.host_trace()
    adv, fixed = adv.copy(), fixed.copy()
    off = batch.offsets_host.astype(np.uint64)
    path, rep = _dev_eval(engine, batch, adv, fixed)
    assert path == 0, "the fast pass flagged a clean trace"
    assert rep["first_failure"] == NONE and rep["rows_checked"] == int(off[-1])
    rng = np.random.default_rng(seed)
    # canonical cells of half-rounds inside bands (carried) and at band starts (gathered): the
    # tiles of instance i are numbered from sum(2 rounds) over earlier instances
    insts = rng.choice(n, 6, replace=False)
    for i in insts:
        r_i = int((off[i + 1] - off[i] - 228) // ROUND_ROWS)
        if r_i < 1:
            continue
        for hr in sorted({1, 2, int(rng.integers(1, 2 * r_i + 1)), 2 * r_i}):
            cells = _canon_rows(int(off[i]), r_i, hr)
            c, r = cells[int(rng.integers(0, len(cells)))]
            a2 = adv.copy()
            a2[c, r] ^= np.uint32(1 << int(rng.integers(0, 16)))
            path, g = _dev_eval(engine, batch, a2, fixed)
            o = orc.evaluate(a2, fixed, off)
            assert g == o, (i, hr, c, r)
            if o["first_failure"] != NONE:
                assert path == 1, "a corruption the oracle sees was not handed to the exact kernel"
    # the batch restored: clean again, fast pass only
    path, rep = _dev_eval(engine, batch, adv, fixed)
    assert path == 0 and rep["first_failure"] == NONE


def test_fast_pass_tile_map_across_zero_round_runs(engine, orc):
    """The fast pass's tile descriptors (eval_desc_kernel: a wave searches the row map for its
    first tile, its lanes then search the next 64 instances and fall back to their own search
    past them) on a batch with runs of 0-round instances -- which own no half-round tile -- of
    1, 63, 64, 65 and 300 instances between 1-, 2- and 12-round ones: clean, then a fault in a
    half-round cell of the instance right after each run is handed to the exact kernel and
    reported where the oracle reports it."""
    import b2f

    x = random_inputs(1200, (1, 2, 12), 44)
    runs = [(10, 1), (40, 63), (200, 64), (400, 65), (700, 300)]
    for a, k in runs:
        x["rounds"][a:a + k] = 0
    batch = b2f.DeviceBatch(x)
    batch.fill(engine)
    engine.sync(0)
    adv, fixed = batch.host_trace()
    adv, fixed = adv.copy(), fixed.copy()
    off = batch.offsets_host.astype(np.uint64)
    path, rep = _dev_eval(engine, batch, adv, fixed)
    assert path == 0 and rep["first_failure"] == NONE and rep["rows_checked"] == int(off[-1])
    for a, k in runs:
        i = a + k  # the first instance after the run
        r = int(off[i]) + INIT_ROWS + 30  # a cell of its first half-round tile
        a2 = adv.copy()
        a2[4, r] ^= np.uint32(1 << 3)
        path, g = _dev_eval(engine, batch, a2, fixed)
        o = orc.evaluate(a2, fixed, off)
        assert o["first_failure"] != NONE and g == o and path == 1, (a, k)
