"""GPU parity of the permutation-argument prover columns (b2f_permutation_columns_dev, VERDICT
r1 item 9) with the CPU restatement of halo2_proofs 0.3.0's keygen + prover
(oracle/permutation.py): sigma and every z bit-exact in all four field forms and several
column-set sizes, for circuits made of all or part of a batch; z closes to 1 on the valid
trace and not on a broken copy. Needs an MI355X (`-m gpu`)."""
import numpy as np
import pytest

import permutation as pm

from conftest import random_inputs

pytestmark = pytest.mark.gpu

R256 = 1 << 256


def _ints(t):
    a = t.cpu().numpy().view(np.uint64).astype(object)
    return [int(v) for v in (a[:, 0] | (a[:, 1] << 64) | (a[:, 2] << 128) | (a[:, 3] << 192))]


def _p(form):
    return pm.P_BN254 if form & 2 else pm.P_PALLAS


@pytest.fixture(scope="module")
def batch(engine):
    import b2f
    import torch

    x = random_inputs(5, (0, 1, 2), 91)
    b = b2f.DeviceBatch(x)
    b.fill(engine)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    return b


def _check(engine, batch, orc, k, usable, form, chunk, instances):
    import torch

    p = _p(form)
    rng = np.random.default_rng(92 + form + 10 * chunk)
    beta = int.from_bytes(rng.bytes(32), "little") % p
    gamma = int.from_bytes(rng.bytes(32), "little") % p
    sig, z = batch.permutation_columns(engine, k, usable, beta, gamma, chunk_len=chunk, form=form,
                                       instances=instances)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    i0, i1 = instances
    off = batch.offsets_host[i0:i1 + 1].astype(np.int64)
    adv, _ = batch.host_trace()
    cadv = adv[:, int(off[0]):int(off[-1])]
    rel = off - off[0]
    sigma, zs = pm.columns(cadv, rel, k, usable, beta, gamma, chunk, p, orc.copies)
    conv = (lambda v: v) if form in (0, 2) else (lambda v: v * R256 % p)
    for j in range(8):
        got = _ints(sig[j])
        want = [conv(v) for v in sigma[j]]
        if got != want:
            i = next(i for i in range(len(got)) if got[i] != want[i])
            pytest.fail("sigma column %d differs first at row %d" % (j, i))
    assert z.shape[0] == len(zs)
    for c, zc in enumerate(zs):
        got = _ints(z[c, :usable + 1])
        want = [conv(v) for v in zc]
        if got != want:
            i = next(i for i in range(len(got)) if got[i] != want[i])
            pytest.fail("z set %d differs first at row %d" % (c, i))
    return zs


@pytest.mark.parametrize("form,chunk", [(1, 3), (0, 3), (3, 1), (2, 8), (1, 8), (3, 5)])
def test_permutation_columns_equal_oracle(engine, batch, orc, form, chunk):
    k = 12
    zs = _check(engine, batch, orc, k, (1 << k) - 7, form, chunk, (0, batch.n))
    assert zs[-1][-1] == 1  # a valid trace closes


def test_permutation_circuit_inside_batch(engine, batch, orc):
    """A circuit of instances 1..3 (its first trace row is not 0), a looser usable count."""
    _check(engine, batch, orc, 12, 4000, 1, 3, (1, 4))


def test_permutation_closes_and_broken_copy(engine, orc):
    import b2f
    import torch

    x = random_inputs(6, (1, 4), 93)
    b = b2f.DeviceBatch(x)
    b.fill(engine)
    s = torch.cuda.current_stream().cuda_stream
    k, usable = 14, (1 << 14) - 9
    one = (1 << 256) % pm.P_PALLAS
    _, z = b.permutation_columns(engine, k, usable, 12345, 67890, chunk_len=3)
    engine.sync(s)
    assert _ints(z[-1, usable:usable + 1]) == [one]
    dr, dc, sr, sc = (int(v) for v in orc.copies(4)[100])
    row = int(b.offsets_host[1]) + dr
    b.advice[dc, row] ^= 1 << 3
    _, z = b.permutation_columns(engine, k, usable, 12345, 67890, chunk_len=3)
    engine.sync(s)
    assert _ints(z[-1, usable:usable + 1]) != [one]


def test_permutation_argument_errors(engine, batch):
    import b2f
    import torch

    s = torch.cuda.current_stream().cuda_stream
    dev = batch.advice.device
    z = torch.empty((8, 1 << 12, 4), dtype=torch.int64, device=dev)
    off = batch.offsets_host
    w, d = pm.domain(pm.P_PALLAS, 12)

    def call(k=12, usable=4089, beta=3, chunk=3, form=1, offs=off, out_rows=1 << 12):
        engine.permutation_columns_dev(batch.advice.data_ptr(), batch.total_rows, offs, k, usable,
                                       w, d, beta, 5, chunk, form, 0, z.data_ptr(), out_rows, s)

    bad_off = off.copy()
    bad_off[2] += 4
    for kw, code in [({"k": 9}, b2f._lib.ERR_ARG), ({"chunk": 0}, b2f._lib.ERR_ARG),
                     ({"chunk": 9}, b2f._lib.ERR_ARG), ({"beta": pm.P_PALLAS}, b2f._lib.ERR_ARG),
                     ({"form": 4}, b2f._lib.ERR_ARG), ({"usable": 100}, b2f._lib.ERR_ROWS),
                     ({"usable": 4096}, b2f._lib.ERR_ROWS), ({"out_rows": 100}, b2f._lib.ERR_ROWS),
                     ({"offs": bad_off}, b2f._lib.ERR_LAYOUT)]:
        with pytest.raises(b2f.B2FError) as e:
            call(**kw)
        assert e.value.code == code, kw
    call()
    engine.sync(s)


def test_permutation_scratch_scales_with_column_sets(engine, batch):
    """The scratch holds one num / den / product slice per column SET (ceil(8 / chunk_len)),
    not per column: measured as the device memory a fresh context takes on its first call,
    chunk_len 1 (8 sets) against chunk_len 8 (1 set) at a 2^20-row domain."""
    import b2f
    import torch

    k, usable = 20, (1 << 20) - 7
    dev = batch.advice.device
    w, d = pm.domain(pm.P_PALLAS, k)
    s = torch.cuda.current_stream().cuda_stream
    taken = {}
    for chunk in (8, 1, 3):
        sets = (8 + chunk - 1) // chunk
        z = torch.empty((sets, 1 << k, 4), dtype=torch.int64, device=dev)
        eng = b2f.Engine(0)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info(dev)[0]
        eng.permutation_columns_dev(batch.advice.data_ptr(), batch.total_rows, batch.offsets_host,
                                    k, usable, w, d, 3, 5, chunk, 1, 0, z.data_ptr(), 1 << k, s)
        eng.sync(s)
        taken[sets] = free0 - torch.cuda.mem_get_info(dev)[0]
        eng.close()
        del z
        torch.cuda.empty_cache()
    per_set = (taken[8] - taken[1]) / 7
    # num + den (2 x 32 B per row) + the grand product's chunk totals (~4 B per row)
    assert 60 * usable < per_set < 80 * usable, taken
    assert abs((taken[3] - taken[1]) - 2 * per_set) < 0.1 * per_set, taken


def test_zero_denominator_is_reported(engine, batch):
    """A challenge that makes a den factor zero (beta = gamma = 0 against a zero cell) cannot
    give a meaningful z (halo2's batch_invert would leave a zero and the proof fail): the call
    reports B2F_ERR_FIELD at b2f_sync, and the sticky word is clear after that."""
    import b2f
    import torch

    s = torch.cuda.current_stream().cuda_stream
    k = 12
    sig, z = batch.permutation_columns(engine, k, (1 << k) - 7, 0, 0, chunk_len=3, form=1,
                                       sigma=False)
    with pytest.raises(b2f.B2FError) as e:
        engine.sync(s)
    assert e.value.code == b2f._lib.ERR_FIELD
    engine.sync(s)  # cleared
    # the lookup argument: (A' + beta) is zero for the zero row's compressed value when beta = 0
    usable = (1 << 16) + 100
    out, bad = batch.lookup_columns(engine, [0], usable, 7, 0, 11, form=1)
    with pytest.raises(b2f.B2FError) as e:
        engine.sync(s)
    assert e.value.code == b2f._lib.ERR_FIELD
    # non-degenerate challenges: clean
    batch.permutation_columns(engine, k, (1 << k) - 7, 3, 5, chunk_len=3, form=1, sigma=False)
    batch.lookup_columns(engine, [0], usable, 7, 3, 11, form=1)
    engine.sync(s)


@pytest.mark.parametrize("form", [1, 2])
def test_permutation_sigma_keygen_equals_columns_call(engine, batch, form):
    """sigma is keygen (build_pk), so b2f_permutation_sigma_dev computes it
    alone, once per circuit shape; it equals the sigma columns the full call writes (which the
    oracle pins above), and the per-proof call without sigma writes the same z."""
    import torch

    k, usable = 12, (1 << 12) - 7
    p = _p(form)
    sig, z = batch.permutation_columns(engine, k, usable, 7, 11, chunk_len=3, form=form,
                                       instances=(1, 4))
    sk = batch.permutation_sigma(engine, k, form=form, instances=(1, 4))
    _, z2 = batch.permutation_columns(engine, k, usable, 7, 11, chunk_len=3, form=form,
                                      instances=(1, 4), sigma=False)
    engine.sync(torch.cuda.current_stream().cuda_stream)
    assert torch.equal(sk, sig)
    assert torch.equal(z2[:, :usable + 1], z[:, :usable + 1])
    assert p  # the field of the form


def test_permutation_sigma_argument_errors(engine, batch):
    import b2f
    import torch

    s = torch.cuda.current_stream().cuda_stream
    sig = torch.empty((8, 1 << 12, 4), dtype=torch.int64, device=batch.advice.device)
    off = batch.offsets_host
    w, d = pm.domain(pm.P_PALLAS, 12)
    bad_off = off.copy()
    bad_off[2] += 4
    for kw, code in [({"k": 9}, b2f._lib.ERR_ARG), ({"k": 31}, b2f._lib.ERR_ARG),
                     ({"form": 4}, b2f._lib.ERR_ARG), ({"delta": pm.P_PALLAS}, b2f._lib.ERR_ARG),
                     ({"out_rows": 100}, b2f._lib.ERR_ROWS), ({"k": 10}, b2f._lib.ERR_ROWS),
                     ({"offs": bad_off}, b2f._lib.ERR_LAYOUT)]:
        a = dict(k=12, form=1, delta=d, out_rows=1 << 12, offs=off)
        a.update(kw)
        with pytest.raises(b2f.B2FError) as e:
            engine.permutation_sigma_dev(a["offs"], a["k"], w, a["delta"], a["form"], sig.data_ptr(),
                                         a["out_rows"], s)
        assert e.value.code == code, kw
    engine.permutation_sigma_dev(off, 12, w, d, 1, sig.data_ptr(), 1 << 12, s)
    engine.sync(s)
