"""GPU tests of the keygen structure (b2f_fill_fixed_dev, the fixed-column check of the eval
and fused kernels), sticky device errors and the product library's independence from the
environment. Every test here needs an MI355X (`-m gpu`)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, random_inputs

pytestmark = pytest.mark.gpu

NONE = 2**64 - 1


def _stream():
    import torch

    return torch.cuda.current_stream().cuda_stream


def _as_oracle(x, orc):
    return np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()


@pytest.mark.parametrize("rounds_choices,n,pad", [((0, 1, 4, 12), 37, 0), ((12,), 5, 1028),
                                                  ((1, 13), 300, 4)])
def test_fill_fixed_dev_equals_fill_and_oracle(engine, orc, rounds_choices, n, pad):
    """The fixed column from the row map alone == the fill's fixed column == the oracle's
    structure-mode synthesis (zeros past the last instance)."""
    import b2f
    import torch

    x = random_inputs(n, rounds_choices, 70 + n)
    total = int(b2f.offsets(x)[-1]) + pad
    batch = b2f.DeviceBatch(x, total_rows=total)
    batch.fill(engine)
    fx = torch.full_like(batch.fixed, -1)
    engine.fill_fixed_dev(batch.offsets.data_ptr(), n, total, fx.data_ptr(), _stream())
    engine.sync(_stream())
    assert torch.equal(fx, batch.fixed)
    want = orc.fixed_structure(batch.offsets_host, total_rows=total)
    assert np.array_equal(fx.cpu().numpy().view(np.uint32), want)


def test_fill_fixed_dev_rejects_bad_layout(engine):
    import b2f

    x = random_inputs(4, (1,), 71)
    batch = b2f.DeviceBatch(x)
    batch.offsets[2] += 4
    engine.fill_fixed_dev(batch.offsets.data_ptr(), 4, batch.total_rows, batch.fixed.data_ptr(),
                          _stream())
    with pytest.raises(b2f.B2FError) as ei:
        engine.sync(_stream())
    assert ei.value.code == 5


@pytest.mark.parametrize("kind,row,delta", [
    (1, 164 + 416 * 2 + 52 * 3 + 0, 1 << 40),      # a1 (ADD3) of round 2, G 3
    (1, 164 + 416 * 3 + 52 * 7 + 28, 12345),       # the last a2 of the instance
    (1, 164 + 416 * 0 + 52 * 5 + 40, 7),           # c2 (ADD2)
    (2, 108 + 4 * 5, 1 << 32),                     # IV5 in advice and k_0
    (2, 108 + 4 * 7, 0xffff_0000_0000_0001),       # IV7 (v15)
])
def test_tampered_trace_flagged_by_fixed_check(engine, orc, kind, row, delta):
    """a trace consistent with an altered fixed column (cleared s_spread_a1/a2/c2
    with the wrong sum propagated downstream; a wrong IV in advice and k_0 alike) passes every
    gate, lookup and copy; the GPU eval flags it through fixed_failures (code 18), exactly as
    the oracle does."""
    x = random_inputs(5, (4,), 72)
    ox = _as_oracle(x, orc)
    adv, fixed, h_out, off = orc.fill_tampered(ox, 2, kind, row, delta)
    got = engine.eval_host(adv, fixed, off)
    want = orc.evaluate(adv, fixed, off)
    assert got == want
    assert sum(got["gate_failures"]) == got["lookup_failures"] == got["copy_failures"] == 0
    assert got["fixed_failures"] >= 1 and (got["first_failure"] & 0xff) == 18
    assert int(off[2]) + row <= got["first_failure"] >> 8 < int(off[2]) + row + 4


def test_fused_fixed_injection_flagged(engine, orc):
    """A selector bit cleared (or a k_0 bit flipped) as the fused kernel assigns it: the
    written trace's verdict carries the fixed-column failure, equal to the eval's and the
    oracle's on that trace."""
    import b2f

    x = random_inputs(6, (1, 4), 73)
    off = b2f.offsets(x)
    cases = [(int(off[1]) + 164 + 52 * 2 + 0, 1 << 3),      # s_spread_a1 of an a1 block
             (int(off[3]) + 164 + 416 + 52 * 4 + 44, 1 << 8),  # s_spread_b2 of an XOR63 block
             (int(off[4]) + 108 + 4 * 2 + 1, 1 << 20),          # a k_0 bit of an IV limb
             (int(off[0]) + 50, 1 << 14)]                       # s_const on a non-CONST row
    for r, mask in cases:
        batch = b2f.DeviceBatch(x)
        engine.debug_inject(r, 10, mask)
        try:
            batch.fill_evaluate(engine)
            engine.sync(_stream())
        finally:
            engine.debug_inject(None)
        got = batch.report_dict()
        assert got["fixed_failures"] >= 1, (r, mask, got)
        adv, fixed = batch.host_trace()
        assert got == orc.evaluate(adv, fixed, batch.offsets_host), (r, mask)
        batch.evaluate(engine)
        engine.sync(_stream())
        assert batch.report_dict() == got


def test_errors_are_sticky_until_sync(engine):
    """fill_evaluate(bad) then fill_evaluate(good) then ONE sync must raise, and
    the bad batch's report reads 'not checked' (rows_checked 0, first failure code 19), never
    clean. The same for eval_dev. The error is cleared by the sync that reported it."""
    import b2f

    x = random_inputs(4, (1, 4), 74)
    bad = b2f.DeviceBatch(x)
    bad.offsets[2] += 4
    good = b2f.DeviceBatch(x)
    bad.fill_evaluate(engine)
    good.fill_evaluate(engine)
    with pytest.raises(b2f.B2FError) as ei:
        engine.sync(_stream())
    assert ei.value.code == 5
    rb = bad.report_dict()
    assert rb["rows_checked"] == 0 and rb["first_failure"] == 19
    assert good.report_dict()["first_failure"] == NONE
    engine.sync(_stream())  # cleared
    good.fill(engine)
    bad.evaluate(engine)
    good.evaluate(engine)
    with pytest.raises(b2f.B2FError) as ei:
        engine.sync(_stream())
    assert ei.value.code == 5
    assert bad.report_dict()["rows_checked"] == 0
    assert good.report_dict()["first_failure"] == NONE
    engine.sync(_stream())


def test_product_library_ignores_diagnostic_environment():
    """with B2F_DIAG_EVAL=1 (the variant that skips gates and copies) and
    B2F_DIAG_FUSED=2 (assignment only) set BEFORE libb2f.so loads, in a fresh interpreter, a
    corrupted trace is still flagged by the eval and by the fused path."""
    code = r"""
import sys
sys.path.insert(0, %r)
import torch, numpy as np, b2f
from b2f import synth
eng = b2f.Engine(0)
s = torch.cuda.current_stream().cuda_stream
b = b2f.DeviceBatch(synth.batch(64, rounds=2))
b.fill(eng)
b.advice[4, 3000] ^= 1 << 5          # an operand cell: a copy and a gate fail
b.evaluate(eng); eng.sync(s)
r1 = b.report_dict()
eng.debug_inject(2000, 3, 1 << 7)
b.fill_evaluate(eng); eng.sync(s)
eng.debug_inject(None)
r2 = b.report_dict()
print("FLAGGED", r1["first_failure"] != 2**64 - 1 and r1["copy_failures"] > 0,
      r2["first_failure"] != 2**64 - 1)
""" % (ROOT + "/zk-odst_amd")
    env = dict(os.environ, B2F_DIAG_EVAL="1", B2F_DIAG_FUSED="2", B2F_DIAG_FILL="0")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=300)
    assert "FLAGGED True True" in out.stdout, out.stdout + out.stderr
