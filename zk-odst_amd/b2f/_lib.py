"""ctypes binding of the C ABI in include/b2f.h (libb2f.so, built in-tree by
__graft_entry__.build() / `make -C zk-odst_amd`).

There is no fallback: if the HIP library is missing or fails to load, every entry point
raises. The product path never touches oracle/.

libb2f.so is the product library: it reads no environment and launches only the full
kernels. libb2f_diag.so is the same ABI built with -DB2F_DIAG, whose diagnostic kernel
variants (floors, ablations, phase clocks) are selected by B2F_DIAG_* variables; it is loaded
only on explicit request (load(diag=True) / Engine(diag=True)) by bench floors and tools/.
"""
import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # zk-odst_amd/
LIB_PATH = os.path.join(PKG_ROOT, "libb2f.so")
DIAG_LIB_PATH = os.path.join(PKG_ROOT, "libb2f_diag.so")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "b2f.h")

NUM_ADVICE = 10
NUM_GATES = 16
CODE_LOOKUP = 16
CODE_COPY = 17
CODE_FIXED = 18
CODE_LAYOUT = 19
CODE_CHECK = 20  # an internal cross-check failed (B2F_ERR_CHECK): a library defect
MAX_ROUNDS = 1 << 20
KERNEL_NAMES = ["record", "fill", "eval", "export", "fill_eval", "lookup", "perm",
                "perm_sigma"]  # B2F_KERNEL_*
FP_CANONICAL, FP_MONTGOMERY, FP_BN254_CANONICAL, FP_BN254_MONTGOMERY = 0, 1, 2, 3  # B2F_FP_*

OK, ERR_ARG, ERR_ROUNDS, ERR_ROWS, ERR_HIP, ERR_LAYOUT, ERR_INPUT, ERR_FIELD, ERR_CHECK = range(9)
STATUS_NAMES = {OK: "OK", ERR_ARG: "B2F_ERR_ARG", ERR_ROUNDS: "B2F_ERR_ROUNDS",
                ERR_ROWS: "B2F_ERR_ROWS", ERR_HIP: "B2F_ERR_HIP", ERR_LAYOUT: "B2F_ERR_LAYOUT",
                ERR_INPUT: "B2F_ERR_INPUT", ERR_FIELD: "B2F_ERR_FIELD",
                ERR_CHECK: "B2F_ERR_CHECK"}


def source_stamp():
    """A 16-hex-digit hash of the sources libb2f.so is built from (zk-odst_amd/csrc/*, the
    Makefile, include/b2f.h): measurement records (PMC traffic) carry it, so bench.py can tell
    whether a record describes the kernels it is running. Reads files only; the GPU box has no
    .git, so a commit id would not do."""
    import glob
    import hashlib

    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(PKG_ROOT, "csrc", "*"))) + [os.path.join(PKG_ROOT, "Makefile"),
                                                                       HEADER]
    for f in files:
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


class B2FError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (STATUS_NAMES.get(code, code), msg))
        self.code = code


class EvalReport(ctypes.Structure):
    _fields_ = [("gate_failures", ctypes.c_uint64 * NUM_GATES),
                ("lookup_failures", ctypes.c_uint64),
                ("copy_failures", ctypes.c_uint64),
                ("first_failure", ctypes.c_uint64),
                ("rows_checked", ctypes.c_uint64),
                ("fixed_failures", ctypes.c_uint64)]

    def as_dict(self):
        return {"gate_failures": list(self.gate_failures),
                "lookup_failures": self.lookup_failures,
                "copy_failures": self.copy_failures,
                "first_failure": self.first_failure,
                "rows_checked": self.rows_checked,
                "fixed_failures": self.fixed_failures}


REPORT_BYTES = ctypes.sizeof(EvalReport)

# (name, restype, argtypes) for every function include/b2f.h declares.
P = ctypes.c_void_p
U64 = ctypes.c_uint64
SIZE = ctypes.c_size_t
I32 = ctypes.c_int
SIGNATURES = [
    ("b2f_version", I32, []),
    ("b2f_layout_rows", U64, [ctypes.c_uint32]),
    ("b2f_layout_offsets", I32, [P, SIZE, P]),
    ("b2f_halo2_column_index", I32, [I32]),
    ("b2f_parse_eip152", I32, [P, SIZE, P]),
    ("b2f_create", P, [I32]),
    ("b2f_destroy", None, [P]),
    ("b2f_last_error", ctypes.c_char_p, [P]),
    ("b2f_fill_dev", I32, [P, P, SIZE, P, U64, P, P, P, P]),
    ("b2f_eval_dev", I32, [P, P, P, P, SIZE, U64, P, P]),
    ("b2f_fill_eval_dev", I32, [P, P, SIZE, P, U64, P, P, P, P, P]),
    ("b2f_debug_inject", I32, [P, U64, ctypes.c_uint32, ctypes.c_uint32]),
    ("b2f_debug_clock", I32, [P, P]),
    ("b2f_debug_eval_path", I32, [P, P]),
    ("b2f_fill_fixed_dev", I32, [P, P, SIZE, U64, P, P]),
    ("b2f_copy_constraints", U64, [ctypes.c_uint32, P, U64]),
    ("b2f_chain_inputs_dev", I32, [P, P, P, P, P, ctypes.c_uint32, SIZE, P, P]),
    ("b2f_export_fp_dev", I32, [P, P, U64, U64, U64, ctypes.c_uint32, P, U64, P]),
    ("b2f_lookup_columns_dev", I32, [P, P, U64, P, ctypes.c_uint32, U64, P, P, P,
                                     ctypes.c_uint32, P, U64, P, P]),
    ("b2f_spread_table_dev", I32, [P, U64, ctypes.c_uint32, P, U64, P]),
    ("b2f_permutation_mapping", U64, [ctypes.c_uint32, P, U64]),
    ("b2f_permutation_columns_dev", I32, [P, P, U64, P, SIZE, ctypes.c_uint32, U64, P, P, P, P,
                                          ctypes.c_uint32, ctypes.c_uint32, P, P, U64, P]),
    ("b2f_permutation_sigma_dev", I32, [P, P, SIZE, ctypes.c_uint32, P, P, ctypes.c_uint32, P, U64, P]),
    ("b2f_sync", I32, [P, P]),
    ("b2f_fill", I32, [P, P, SIZE, P, P, P]),
    ("b2f_eval", I32, [P, P, P, P, SIZE, U64, P]),
    ("b2f_num_kernels", I32, []),
    ("b2f_set_timing", I32, [P, I32]),
    ("b2f_kernel_times", I32, [P, P, P]),
]

_libs = {}


def _share_hip_runtime_with_torch():
    """One HIP runtime per process. PyTorch-ROCm ships its own libamdhip64 (soname
    libamdhip64.so.7, the same soname /opt/rocm's has); if libb2f.so is loaded first, torch
    later maps its own copy as a second runtime and then sees no GPUs. Importing torch
    first makes the dynamic linker satisfy libb2f.so's libamdhip64.so.7 with torch's copy, so
    torch tensors, torch streams and the b2f kernels share one runtime. Without torch in the
    process, /opt/rocm's runtime is used."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(diag=False, path=None):
    """Load libb2f.so (diag=True: libb2f_diag.so; path: an explicit build of the same ABI,
    for A/B runs in tools/). Raises OSError with a build hint when the file is absent."""
    path = path or (DIAG_LIB_PATH if diag else LIB_PATH)
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise OSError("%s not found: build it with "
                      "`python -c 'import __graft_entry__ as g; g.build()'` or "
                      "`make -C zk-odst_amd`" % path)
    _share_hip_runtime_with_torch()
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        if path != LIB_PATH and path != DIAG_LIB_PATH and not hasattr(lib, name):
            continue  # an older A/B build (tools/) without a later entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _libs[path] = lib
    return lib


def check(ctx, rc, lib=None):
    if rc != OK:
        msg = (lib or load()).b2f_last_error(ctx)
        raise B2FError(rc, msg.decode() if msg else "")
