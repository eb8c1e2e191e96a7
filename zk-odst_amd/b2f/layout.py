"""Host-side view of LAYOUT v1 (docs/LAYOUT.md): the input record, row map and column map.

Row counts and offsets come from the C ABI (b2f_layout_rows / b2f_layout_offsets), so the
host and the kernels cannot disagree about where an instance's region starts.
"""
import ctypes

import numpy as np

from . import _lib

# b2f_input (include/b2f.h): the reference's Blake2fWitness{rounds, h, m, t, f}
INPUT_DTYPE = np.dtype([("h", "<u8", (8,)), ("m", "<u8", (16,)), ("t", "<u8", (2,)),
                        ("rounds", "<u4"), ("f", "<u4")])
assert INPUT_DTYPE.itemsize == 216

INIT_ROWS, ROUND_ROWS, FINAL_ROWS = 164, 416, 64
COLUMNS = ["a_%d" % i for i in range(_lib.NUM_ADVICE)]
# selector bit -> name (bits 0..11 are the reference's compression.rs:561-577 selectors)
SELECTORS = ["s_decompose_abcd", "s_decompose_efgh", "s_decompose_ijkl", "s_spread_a1",
             "s_spread_b1", "s_spread_c1", "s_spread_d1", "s_spread_a2", "s_spread_b2",
             "s_spread_c2", "s_spread_d2", "s_digest", "s_xor", "s_xor3", "s_const", "s_fmask"]


def rows(rounds):
    """R(rounds) = 228 + 416*rounds; raises for rounds > B2F_MAX_ROUNDS."""
    r = int(_lib.load().b2f_layout_rows(int(rounds)))
    if r == 0:
        raise _lib.B2FError(_lib.ERR_ROUNDS, "rounds %d > %d" % (rounds, _lib.MAX_ROUNDS))
    return r


def as_inputs(inputs):
    return np.ascontiguousarray(inputs, dtype=INPUT_DTYPE)


def offsets(inputs):
    """Row offset of every instance region, n+1 entries (b2f_layout_offsets)."""
    inputs = as_inputs(inputs)
    off = np.zeros(len(inputs) + 1, dtype=np.uint64)
    rc = _lib.load().b2f_layout_offsets(ctypes.c_void_p(inputs.ctypes.data), len(inputs),
                                        ctypes.c_void_p(off.ctypes.data))
    if rc != _lib.OK:
        raise _lib.B2FError(rc, "layout offsets")
    return off


def halo2_column_index(a_i):
    """halo2 advice-column index of a_i (table16.rs:281-294 allocation order)."""
    return int(_lib.load().b2f_halo2_column_index(int(a_i)))


def parse_eip152(raw):
    """213-byte EIP-152 input -> one INPUT_DTYPE record (B2F_ERR_INPUT if malformed)."""
    raw = bytes(raw)
    buf = ctypes.create_string_buffer(raw, len(raw))
    out = np.zeros(1, dtype=INPUT_DTYPE)
    rc = _lib.load().b2f_parse_eip152(buf, len(raw), ctypes.c_void_p(out.ctypes.data))
    if rc != _lib.OK:
        raise _lib.B2FError(rc, "malformed EIP-152 input (%d bytes)" % len(raw))
    return out[0]


def split_fixed(fixed):
    """Unpack the fixed column into (selector bool matrix [16, rows], constant column)."""
    fixed = np.asarray(fixed, dtype=np.uint32)
    sel = ((fixed[None, :] >> np.arange(16, dtype=np.uint32)[:, None]) & 1).astype(bool)
    return sel, (fixed >> 16).astype(np.uint32)
