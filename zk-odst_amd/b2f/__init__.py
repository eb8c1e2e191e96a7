"""b2f: MI355X-native BLAKE2f Table16 witness fill + constraint eval (host side).

The compute is the HIP library libb2f.so (include/b2f.h); this package is the host-side
mirror of the reference's gadget API (blake2f-circuit/src/blake2f.rs) over that C ABI.
"""
from ._lib import (FP_BN254_CANONICAL, FP_BN254_MONTGOMERY, FP_CANONICAL, FP_MONTGOMERY,  # noqa: F401
                   B2FError, EvalReport, load)
from .layout import (INPUT_DTYPE, SELECTORS, as_inputs, halo2_column_index, offsets,  # noqa: F401
                     parse_eip152, rows, split_fixed)
from .engine import DeviceBatch, Engine, copy_constraints, permutation_mapping  # noqa: F401
from . import field  # noqa: F401
