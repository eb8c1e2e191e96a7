"""GPU parity of the lookup-argument prover columns (b2f_lookup_columns_dev, SURVEY.md §8(f)
row 4) with the CPU restatement of halo2_proofs 0.3.0's lookup prover (oracle/lookup.py):
A, S, A', S' and z bit-exact, in Montgomery and canonical form, for circuits inside the trace,
straddling its end and almost entirely past it; a corrupted lookup cell is reported at its
row. Needs an MI355X (`-m gpu`)."""
import numpy as np
import pytest

from conftest import random_inputs

pytestmark = pytest.mark.gpu

R256 = 1 << 256


def _mod(form):
    import lookup as lk

    return lk.P_BN254 if form & 2 else lk.P


def _chal(seed, form=1):
    r = np.random.default_rng(seed)
    return [int.from_bytes(r.bytes(32), "little") % _mod(form) for _ in range(3)]


def _col_ints(t):
    """int64 [rows, 4] limbs -> list of Python ints."""
    a = t.cpu().numpy().view(np.uint64).astype(object)
    return [int(v) for v in (a[:, 0] | (a[:, 1] << 64) | (a[:, 2] << 128) | (a[:, 3] << 192))]


def _circuit_rows(adv, total, begin, usable):
    a = np.zeros((3, usable), dtype=np.uint32)
    n = max(0, min(usable, total - begin))
    a[:, :n] = adv[:3, begin:begin + n]
    return a


@pytest.fixture(scope="module")
def trace(engine):
    import b2f
    import torch

    x = random_inputs(26, (12,), 61)
    batch = b2f.DeviceBatch(x)
    batch.fill(engine)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    return batch


@pytest.mark.parametrize("form", [1, 0, 3, 2])
def test_lookup_columns_equal_oracle(engine, trace, form):
    """Forms 0/1 pasta Fp, 2/3 BN254 Fr (the reference circuit's field)."""
    import lookup as lk
    import torch

    usable = (1 << 17) - 7
    total = trace.total_rows
    begins = [0, total - 20000, total - 5]
    p = _mod(form)
    theta, beta, gamma = _chal(7 + form, form)
    out, bad = trace.lookup_columns(engine, begins, usable, theta, beta, gamma, form=form)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    assert (bad.cpu().numpy().view(np.uint64) == np.uint64(2**64 - 1)).all()
    adv, _ = trace.host_trace()
    for c, b in enumerate(begins):
        a = _circuit_rows(adv, total, b, usable)
        ref = lk.columns(a[0], a[1], a[2], usable, theta, beta, gamma, p)
        assert ref[4][-1] == 1  # a valid lookup closes
        for j, name in enumerate(["A", "S", "A'", "S'", "z"]):
            n = usable + 1 if j == 4 else usable
            got = _col_ints(out[c, j, :n])
            want = ref[j] if form in (0, 2) else [v * R256 % p for v in ref[j]]
            if got != want:
                i = next(i for i in range(n) if got[i] != want[i])
                pytest.fail("circuit %d column %s differs first at row %d" % (c, name, i))


@pytest.mark.parametrize("which", ["small", "minus", "mid"])
def test_lookup_structured_theta(engine, trace, which):
    """Challenges whose table values share their top 64-bit limb in long runs (round 6): theta =
    3 puts all 2^16 values below 2^192 (one run, already in order), theta = -2^40 puts 65,281 of
    them below 2^192 in descending order of x (a long run out of order), theta = 2^100 + 1 leaves
    runs by tag. The rank order is the order of the full values in every case
    (lk_tie_fix_kernel), so the columns equal the oracle's. (Each theta keeps the 2^16 table
    values distinct; a theta that makes two of them equal -- theta = -3: T[1] = T[2] -- is not
    covered: the kernels treat equal values of two table rows as two runs where halo2 makes one,
    which moves a leftover in S'; for a transcript challenge that has probability ~2^-222.)"""
    import lookup as lk
    import torch

    usable = 1 << 16
    theta = {"small": 3, "minus": lk.P - (1 << 40), "mid": (1 << 100) + 1}[which]
    _, beta, gamma = _chal(13)
    out, bad = trace.lookup_columns(engine, [5000], usable, theta, beta, gamma)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    assert (bad.cpu().numpy().view(np.uint64) == np.uint64(2**64 - 1)).all()
    adv, _ = trace.host_trace()
    a = _circuit_rows(adv, trace.total_rows, 5000, usable)
    ref = lk.columns(a[0], a[1], a[2], usable, theta, beta, gamma)
    for j, name in enumerate(["A", "S", "A'", "S'", "z"]):
        n = usable + 1 if j == 4 else usable
        got = _col_ints(out[0, j, :n])
        want = [v * R256 % lk.P for v in ref[j]]
        if got != want:
            i = next(i for i in range(n) if got[i] != want[i])
            pytest.fail("theta %s column %s differs first at row %d" % (which, name, i))


def test_lookup_min_usable_and_bad_row(engine, trace):
    """usable = 2^16 (the table exactly fills the circuit); a flipped spread cell in the trace
    is reported at its circuit row (and only for the circuits holding it)."""
    import lookup as lk
    import torch

    usable = 1 << 16
    theta, beta, gamma = _chal(11)
    out, bad = trace.lookup_columns(engine, [3 * usable], usable, theta, beta, gamma)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    adv, _ = trace.host_trace()
    a = _circuit_rows(adv, trace.total_rows, 3 * usable, usable)
    ref = lk.columns(a[0], a[1], a[2], usable, theta, beta, gamma)
    assert _col_ints(out[0, 3, :usable]) == [v * R256 % lk.P for v in ref[3]]
    assert _col_ints(out[0, 4, :usable + 1]) == [v * R256 % lk.P for v in ref[4]]
    row = 70000
    saved = trace.advice[2, row].item()
    trace.advice[2, row] = saved ^ 0x10
    try:
        out, bad = trace.lookup_columns(engine, [0, 60000, 71000], usable, theta, beta, gamma)
        engine.sync(torch.cuda.current_stream().cuda_stream)
        b = bad.cpu().numpy().view(np.uint64)
        assert int(b[0]) == 2**64 - 1 and int(b[1]) == row - 60000 and int(b[2]) == 2**64 - 1
    finally:
        trace.advice[2, row] = saved


def test_lookup_argument_errors(engine, trace):
    """Argument checks of b2f_lookup_columns_dev (all before any launch)."""
    import lookup as lk
    import torch

    import b2f

    dev = trace.advice.device
    rb = torch.zeros(1, dtype=torch.int64, device=dev)
    bad = torch.empty(1, dtype=torch.int64, device=dev)
    u = 1 << 16
    out = torch.empty((1, 5, u + 1, 4), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def call(usable=u, theta=3, form=1, out_rows=u + 1):  # noqa: E306
        engine.lookup_columns_dev(trace.advice.data_ptr(), trace.total_rows, rb.data_ptr(), 1,
                                  usable, theta, 5, 7, form, out.data_ptr(), out_rows,
                                  bad.data_ptr(), s)

    for kw, code in [({"usable": u - 1}, b2f._lib.ERR_ROWS), ({"out_rows": u}, b2f._lib.ERR_ROWS),
                     ({"theta": lk.P}, b2f._lib.ERR_ARG), ({"form": 4}, b2f._lib.ERR_ARG),
                     ({"theta": lk.P_BN254, "form": 3}, b2f._lib.ERR_ARG)]:
        with pytest.raises(b2f.B2FError) as e:
            call(**kw)
        assert e.value.code == code, kw
    call()  # valid arguments still run
    engine.sync(s)


@pytest.mark.parametrize("form", [1, 0, 3, 2])
def test_spread_table_columns(engine, form):
    """VERDICT r1 missing 5: the spread table as the prover's three table columns
    (SpreadTableChip::load), rows past 2^16 the row-0 default, in every field form; the
    table side S of the lookup columns is its theta-compression."""
    import lookup as lk
    import torch

    usable = (1 << 16) + 300
    out = engine.spread_table(usable, form)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    p = _mod(form)
    got = out.cpu().numpy().view(np.uint64)
    tag = [lk.tag(x) for x in range(1 << 16)] + [0] * 300
    dense = list(range(1 << 16)) + [0] * 300
    spread = [lk.spread(x) for x in range(1 << 16)] + [0] * 300
    for c, col in enumerate((tag, dense, spread)):
        if form & 1:
            want = np.array([lk.to_limbs(v * R256 % p) for v in col], dtype=np.uint64)
        else:
            want = np.zeros((usable, 4), dtype=np.uint64)
            want[:, 0] = col
        assert np.array_equal(got[c], want), c


@pytest.mark.parametrize("form,which", [(1, "beta"), (3, "beta"), (1, "gamma")])
def test_lookup_zero_factor_reported_then_clean(engine, trace, form, which):
    """beta = -A[row] makes (A + beta) and (A' + beta) zero for that row's value, and
    gamma = -T[x] makes (S + gamma) and (S' + gamma) zero for table row x, so the den total is
    zero: the call reports B2F_ERR_FIELD at b2f_sync (D = the num side's product, lk_nscan_kernel
    on the side stream), and the next call with sound challenges syncs clean -- with no
    B2F_ERR_CHECK, i.e. the permuted columns' den product equals the num side's D -- and its z
    ends at one (N / D by construction; the sync is the check that matters)."""
    import lookup as lk
    import torch

    import b2f

    s = torch.cuda.current_stream().cuda_stream
    usable = (1 << 17) - 7
    p = _mod(form)
    theta, _, gamma = _chal(19, form)
    adv, _ = trace.host_trace()
    row = 1234
    a = lk.compress(theta, int(adv[0, row]), int(adv[1, row]), int(adv[2, row]), p)
    beta = (p - a) % p
    if which == "gamma":  # table row 40,000 (not necessarily among the inputs)
        _, beta, _ = _chal(19, form)
        x = 40000
        gamma = (p - lk.compress(theta, lk.tag(x), x, lk.spread(x), p)) % p
    out, bad = trace.lookup_columns(engine, [0], usable, theta, beta, gamma, form=form)
    with pytest.raises(b2f.B2FError) as e:
        engine.sync(s)
    assert e.value.code == b2f._lib.ERR_FIELD
    if which == "gamma":
        gamma = (gamma + 1) % p
    else:
        beta = (beta + 1) % p
    out, bad = trace.lookup_columns(engine, [0], usable, theta, beta, gamma, form=form)
    engine.sync(s)
    z = _col_ints(out[0, 4, usable:usable + 1])[0]
    one = 1 if form in (0, 2) else R256 % p
    assert z == one  # a valid lookup closes to 1


def test_lookup_group_of_circuits_equal_oracle(engine, trace):
    """Five circuits in one call, one group: each circuit's num block products, their prefix and
    D^-1 come from the trace on the side stream (lk_npart_kernel, lk_nscan_kernel) while the count
    and rank-scan passes run, and one z pass (lk_zpass_kernel, a den-side look-back per circuit)
    covers the group. Every circuit's five columns equal the restatement, BN254 Montgomery form."""
    import lookup as lk
    import torch

    form = 3
    usable = (1 << 16) + 100
    total = trace.total_rows
    begins = [0, 70001, 2 * usable, total - 40000, total - 3]
    p = _mod(form)
    theta, beta, gamma = _chal(23, form)
    out, bad = trace.lookup_columns(engine, begins, usable, theta, beta, gamma, form=form)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    assert (bad.cpu().numpy().view(np.uint64) == np.uint64(2**64 - 1)).all()
    adv, _ = trace.host_trace()
    for c, b in enumerate(begins):
        a = _circuit_rows(adv, total, b, usable)
        ref = lk.columns(a[0], a[1], a[2], usable, theta, beta, gamma, p)
        for j in (2, 3, 4):  # A', S' and z (A and S are per-row maps, covered above)
            n = usable + 1 if j == 4 else usable
            got = _col_ints(out[c, j, :n])
            want = [v * R256 % p for v in ref[j]]
            assert got == want, (c, j)


def test_lookup_two_groups_equal_within_call(engine, trace):
    """More circuits than one group holds (at most 2^24 rows per group: 16 circuits of 2^20
    rows), so the call loops over two groups, each forking its own num-side chain (block
    products, prefix, D^-1) to the side stream at its start and reusing the count / NK /
    look-back scratch of the group before (the S part of the block products is computed once, by
    the first group). Circuit 16 (group 2) repeats circuit 5's rows (group 1): all five columns
    bit-identical, the sync clean (no B2F_ERR_CHECK) and every z ends at one (Montgomery form). A
    group that read the previous group's counts, NK or look-back state would differ."""
    import torch

    form = 1
    usable = 1 << 20
    begins = [i * 8000 for i in range(16)] + [5 * 8000]  # inside the 135,720-row trace
    theta, beta, gamma = _chal(31, form)
    out, bad = trace.lookup_columns(engine, begins, usable, theta, beta, gamma, form=form)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    assert (bad.cpu().numpy().view(np.uint64) == np.uint64(2**64 - 1)).all()
    one = R256 % _mod(form)
    for c in range(len(begins)):
        assert _col_ints(out[c, 4, usable:usable + 1])[0] == one, c
    # columns A .. S' hold `usable` rows, z usable + 1 (the row after A .. S' is never written)
    assert torch.equal(out[16, :4, :usable], out[5, :4, :usable])
    assert torch.equal(out[16, 4, :usable + 1], out[5, 4, :usable + 1])
    assert not torch.equal(out[16, 2, :usable], out[4, 2, :usable])


def _spread16(x):
    x = x.astype(np.uint32)
    x = (x | (x << 8)) & np.uint32(0x00FF00FF)
    x = (x | (x << 4)) & np.uint32(0x0F0F0F0F)
    x = (x | (x << 2)) & np.uint32(0x33333333)
    x = (x | (x << 1)) & np.uint32(0x55555555)
    return x


def test_lookup_sparse_values_wide_windows(engine):
    """Dense-cell distributions that stretch the z pass's per-block windows (lk_block_kernel):
    three distinct values (a block's rows then span thousands of unused table ranks in rank
    order, the scatter's loops past their first four ranks per thread), two runs of 100,000 and
    31,065 rows (one rank covers every row of many blocks), and every table value once followed
    by 65,529 repeats of 65,535 (leftover items of nearly every rank, the leftover windows at
    their widest). All five columns equal the restatement."""
    import b2f
    import lookup as lk
    import torch

    usable = (1 << 17) - 7
    rng = np.random.default_rng(41)
    xs = [rng.choice(np.array([5, 40000, 65535], dtype=np.uint32), usable, p=[0.8, 0.15, 0.05]),
          np.where(np.arange(usable) < 100000, 7, 60000).astype(np.uint32),
          np.concatenate([rng.permutation(65536).astype(np.uint32),
                          np.full(usable - 65536, 65535, dtype=np.uint32)])]
    rows = (3 * usable + 3) // 4 * 4  # a trace holds a multiple of 4 rows
    adv = rng.integers(0, 2**32, (10, rows), dtype=np.uint64).astype(np.uint32)
    x = np.concatenate(xs + [np.zeros(rows - 3 * usable, dtype=np.uint32)])
    adv[0] = np.where(x < 256, 0, np.where(x < 32768, 1, 2)).astype(np.uint32)
    adv[1] = x
    adv[2] = _spread16(x)
    batch = b2f.DeviceBatch(random_inputs(1, (0,), 1), device="cuda:0", total_rows=rows)
    batch.advice.copy_(torch.from_numpy(adv.view(np.int32)))
    theta, beta, gamma = _chal(43)
    out, bad = batch.lookup_columns(engine, [0, usable, 2 * usable], usable, theta, beta, gamma)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    assert (bad.cpu().numpy().view(np.uint64) == np.uint64(2**64 - 1)).all()
    for c in range(3):
        a = adv[:3, c * usable:(c + 1) * usable]
        ref = lk.columns(a[0], a[1], a[2], usable, theta, beta, gamma)
        for j in range(5):
            n = usable + 1 if j == 4 else usable
            got = _col_ints(out[c, j, :n])
            want = [v * R256 % lk.P for v in ref[j]]
            if got != want:
                i = next(i for i in range(n) if got[i] != want[i])
                pytest.fail("circuit %d column %d differs first at row %d" % (c, j, i))
