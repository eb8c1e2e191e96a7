"""CPU check of the lookup z pass's row-run logic (zk-odst_amd/csrc/b2f_lookup.hip): the
rank-order scan's arrays (lk_scan_write: pos, dcnt, the compacted leftover ranks), the per-block
windows (lk_block_kernel: J(p) = p - dcnt[ra(p)] + [p starts a run], the pos-rank and leftover
windows) and the z pass's scatter of those windows into per-row and per-leftover-index tables,
restated in numpy and compared with the definition of halo2's permute_expression_pair
(oracle/lookup.py's restatement): row p's A' rank is the run holding p, a run start takes its
own rank as S', the j-th repeated row takes leftover item n_left - 1 - j.

The kernel's tables hold x_of_rank[r] where this restatement holds r (a relabelling: the z pass
gathers the table in table order). Host logic only; the GPU tests (tests/test_gpu_lookup.py)
compare the kernels' columns with the oracle end to end, including the distributions below."""
import numpy as np
import pytest

TROWS = 1 << 16
LB = 1024


def _scan(count, usable):
    """pos, dcnt, leftover multiplicity per rank, compacted leftover ranks and their starts."""
    mult = np.ones(TROWS, dtype=np.int64)
    # table row 0's multiplicity (it fills the rows past the table); the kernel gives it to the
    # rank holding table row 0, here rank 0 -- the window logic does not depend on which rank
    mult[0] = usable - TROWS + 1
    pos = np.concatenate([[0], np.cumsum(count)[:-1]])
    dcnt = np.cumsum(count > 0)
    m = mult - (count > 0)
    lrank = np.nonzero(m)[0]
    lstart = np.concatenate([[0], np.cumsum(m[lrank])[:-1]]) if len(lrank) else np.zeros(0, dtype=np.int64)
    return pos, dcnt, m, lrank, lstart


def _last_le(a, v, lim=None):
    a = a if lim is None else a[:lim]
    return int(np.searchsorted(a, v, side="right")) - 1


def _windows(pos, dcnt, lstart, nr, usable, b):
    """lk_block_kernel for block b: (r0, r1, J0, J1, k0, k1)."""
    n_left = usable - int(dcnt[-1])
    base, end = b * LB, min(b * LB + LB, usable)

    def J(p):
        r = _last_le(pos, p)
        return p - int(dcnt[r]) + (1 if pos[r] == p else 0)

    r0, r1 = _last_le(pos, base), _last_le(pos, end - 1)
    J0 = J(base)
    J1 = n_left if end == usable else J(end)
    k0, k1 = 1, 0
    if J1 > J0:
        k0 = _last_le(lstart, n_left - J1, nr)
        k1 = _last_le(lstart, n_left - 1 - J0, nr)
    return r0, r1, J0, J1, k0, k1


def _scatter(pos, dcnt, lrank, lstart, usable, b, win):
    """The z pass's step 1 for block b: (A' rank, S' rank) of every row of the block."""
    r0, r1, J0, J1, k0, k1 = win
    n_left = usable - int(dcnt[-1])
    nr = len(lrank)
    base, end = b * LB, min(b * LB + LB, usable)
    ent = np.full(end - base, -1, dtype=np.int64)
    start = np.zeros(end - base, dtype=bool)
    jrel = np.zeros(end - base, dtype=np.int64)
    for r in range(r0, r1 + 1):
        s0, s1 = int(pos[r]), int(pos[r + 1]) if r + 1 < TROWS else usable
        for q in range(max(s0, base), min(s1, end)):
            ent[q - base] = r
            start[q - base] = q == s0
            jrel[q - base] = q - int(dcnt[r]) - J0
    ylo, yhi = n_left - J1, n_left - J0
    yl = np.full(max(yhi - ylo, 0), -1, dtype=np.int64)
    for kk in range(k0, k1 + 1):
        y0, y1 = int(lstart[kk]), int(lstart[kk + 1]) if kk + 1 < nr else n_left
        for y in range(max(y0, ylo), min(y1, yhi)):
            yl[y - ylo] = lrank[kk]
    assert (ent >= 0).all(), "a row of the block outside its pos window"
    rs = np.where(start, ent, -1)
    for i in np.nonzero(~start)[0]:
        y = yhi - 1 - jrel[i]
        assert 0 <= jrel[i] < J1 - J0 and yl[y - ylo] >= 0, "a leftover index outside its window"
        rs[i] = yl[y - ylo]
    return ent, rs


def _reference(count, usable):
    """A' / S' ranks of every row by the definition (run holding the row; run start; the j-th
    repeated row takes leftover item n_left - 1 - j, leftover items in rank order)."""
    a_rank = np.repeat(np.arange(TROWS), count)
    starts = np.zeros(usable, dtype=bool)
    starts[np.concatenate([[0], np.cumsum(count)[:-1]])[count > 0]] = True
    m = np.ones(TROWS, dtype=np.int64)
    m[0] = usable - TROWS + 1
    m -= count > 0
    items = np.repeat(np.arange(TROWS), m)  # leftover items, ascending
    s_rank = a_rank.copy()
    rep = np.nonzero(~starts)[0]
    s_rank[rep] = items[len(items) - 1 - np.arange(len(rep))]
    return a_rank, s_rank


def _counts(kind, usable, rng):
    if kind == "uniform":
        x = rng.integers(0, TROWS, usable)
    elif kind == "three_values":
        x = rng.choice(np.array([5, 40000, 65535]), usable, p=[0.8, 0.15, 0.05])
    elif kind == "two_runs":
        x = np.where(np.arange(usable) < 100000, 7, 60000)
    else:  # every value once, then repeats of the last
        x = np.concatenate([np.arange(TROWS), np.full(usable - TROWS, TROWS - 1)])
    # ranks: a random order of the table values (the compressed values' sort order)
    rank_of = rng.permutation(TROWS)
    return np.bincount(rank_of[x], minlength=TROWS)


@pytest.mark.parametrize("kind", ["uniform", "three_values", "two_runs", "every_value_once"])
def test_block_windows_equal_definition(kind):
    rng = np.random.default_rng(53)
    usable = (1 << 17) - 7
    count = _counts(kind, usable, rng)
    assert count.sum() == usable
    pos, dcnt, m, lrank, lstart = _scan(count, usable)
    assert int(m.sum()) == usable - int(dcnt[-1])  # leftover items = repeated rows
    a_ref, s_ref = _reference(count, usable)
    nb = (usable + LB - 1) // LB
    # every block of a sample (first, last and some inside), scattered and compared
    for b in sorted({0, 1, nb // 3, nb // 2, nb - 2, nb - 1}):
        win = _windows(pos, dcnt, lstart, len(lrank), usable, b)
        a, s = _scatter(pos, dcnt, lrank, lstart, usable, b, win)
        lo = b * LB
        assert np.array_equal(a, a_ref[lo:lo + len(a)]), (kind, b)
        assert np.array_equal(s, s_ref[lo:lo + len(s)]), (kind, b)
