"""The library's internal cross-checks fire: B2F_ERR_CHECK at b2f_sync is a library
defect, never a witness verdict, so each check is shown raising it once, on the diagnostics
build (libb2f_diag.so), whose hooks break one internal invariant on request:

* B2F_DIAG_LK_CORRUPT=1: one permuted cell (row 0's A') of the lookup columns is read from the
  wrong table row, so block 0's den product from the permuted columns differs from the num
  side's D (lk_zpass_kernel's cross-check);
* B2F_DIAG_SEG_CAP=n: the fused launch's long-instance segment list holds only n entries, so
  the record kernel's overflow check fires and the report reads "not checked" with
  first_failure = B2F_CODE_CHECK (not B2F_CODE_LAYOUT: it is not the caller's row map).

After each, the same call without the hook syncs clean. Needs an MI355X (`-m gpu`)."""
import os

import pytest

from conftest import random_inputs

pytestmark = pytest.mark.gpu


def _stream():
    import torch

    return torch.cuda.current_stream().cuda_stream


def test_lookup_den_crosscheck_fires_on_a_wrong_permuted_cell(diag_engine):
    import b2f

    x = random_inputs(26, (12,), 61)
    batch = b2f.DeviceBatch(x)
    batch.fill(diag_engine)
    diag_engine.sync(_stream())
    usable = (1 << 17) - 7
    chal = (0x1234567 << 200, 0x89ABCDEF << 180, 0x13579BDF << 190)
    os.environ["B2F_DIAG_LK_CORRUPT"] = "1"
    try:
        batch.lookup_columns(diag_engine, [0, 5000], usable, *chal, form=1)
        with pytest.raises(b2f.B2FError) as e:
            diag_engine.sync(_stream())
        assert e.value.code == b2f._lib.ERR_CHECK
    finally:
        os.environ.pop("B2F_DIAG_LK_CORRUPT", None)
    batch.lookup_columns(diag_engine, [0, 5000], usable, *chal, form=1)
    diag_engine.sync(_stream())  # clean again


def test_fused_segment_overflow_reads_as_check_not_layout(diag_engine):
    import b2f

    x = random_inputs(64, (12,), 7)
    x["rounds"][5] = 100  # (200 - 1) // 24 = 8 later segments
    batch = b2f.DeviceBatch(x)
    os.environ["B2F_DIAG_SEG_CAP"] = "3"
    try:
        batch.fill_evaluate(diag_engine, _stream())
        with pytest.raises(b2f.B2FError) as e:
            diag_engine.sync(_stream())
        assert e.value.code == b2f._lib.ERR_CHECK
    finally:
        os.environ.pop("B2F_DIAG_SEG_CAP", None)
    rep = batch.report_dict()
    assert rep["rows_checked"] == 0 and rep["first_failure"] == b2f._lib.CODE_CHECK
    batch.fill_evaluate(diag_engine, _stream())
    diag_engine.sync(_stream())
    rep = batch.report_dict()
    assert rep["first_failure"] == 2**64 - 1 and rep["rows_checked"] >= batch.used_rows
