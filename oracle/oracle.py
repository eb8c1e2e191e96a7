"""ctypes wrapper of the CPU oracle (oracle/liboracle_b2f.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker or the timed CPU baseline. The product package
(zk-odst_amd/b2f) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_b2f.so")

NCOLS = 10
NGATES = 16
CODE_LOOKUP = 16
CODE_COPY = 17
CODE_FIXED = 18

# orc_input (b2f_oracle.h) as a numpy record: 216 bytes
INPUT_DTYPE = np.dtype([("h", "<u8", (8,)), ("m", "<u8", (16,)), ("t", "<u8", (2,)),
                        ("rounds", "<u4"), ("f", "<u4")])
assert INPUT_DTYPE.itemsize == 216


class Report(ctypes.Structure):
    _fields_ = [("gate_failures", ctypes.c_uint64 * NGATES),
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


_lib = None
V4_PATH = os.path.join(HERE, "liboracle_b2f_v4.so")
V4_FLAGS = "-O3 -march=x86-64-v4 -mtune=znver3 -fopenmp"
V2_FLAGS = "-O3 -march=x86-64-v2 -mtune=generic -fopenmp"


def host_has_avx512():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("flags"):
                    f = set(line.split(":", 1)[1].split())
                    return {"avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"} <= f
    except OSError:
        pass
    return False


def use_fastest_build():
    """Bind the x86-64-v4 build when the host has AVX-512 (before the first call); returns the
    compiler flags of the build in use. For bench.py's CPU baseline only."""
    global LIB_PATH
    if _lib is None and host_has_avx512() and os.path.exists(V4_PATH):
        LIB_PATH = V4_PATH
    return V4_FLAGS if LIB_PATH == V4_PATH else V2_FLAGS


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.orc_rows.argtypes = [ctypes.c_uint32]
        L.orc_rows.restype = ctypes.c_uint64
        L.orc_offsets.argtypes = [P, ctypes.c_size_t, P]
        L.orc_copies.argtypes = [ctypes.c_uint32, P, ctypes.c_size_t]
        L.orc_copies.restype = ctypes.c_size_t
        L.orc_compress.argtypes = [ctypes.c_uint32, P, P, P, ctypes.c_uint32, P]
        L.orc_fill.argtypes = [P, ctypes.c_size_t, P, ctypes.c_uint64, P, P, P, ctypes.c_int]
        L.orc_fill.restype = ctypes.c_int
        L.orc_eval.argtypes = [P, P, P, ctypes.c_size_t, ctypes.c_uint64, P, ctypes.c_int]
        L.orc_eval.restype = ctypes.c_int
        L.orc_max_threads.restype = ctypes.c_int
        L.orc_export_fp.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                    ctypes.c_uint32, P, ctypes.c_uint64]
        L.orc_fp_mont.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P]
        L.orc_fixed.argtypes = [P, ctypes.c_size_t, ctypes.c_uint64, P]
        L.orc_fill_tampered.argtypes = [P, ctypes.c_size_t, P, ctypes.c_uint64, P, P, P,
                                        ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32,
                                        ctypes.c_uint64]
        L.orc_fixed.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def rows(rounds):
    return int(lib().orc_rows(rounds))


def offsets(inputs):
    inputs = np.ascontiguousarray(inputs, dtype=INPUT_DTYPE)
    off = np.zeros(len(inputs) + 1, dtype=np.uint64)
    lib().orc_offsets(_p(inputs), len(inputs), _p(off))
    return off


def copies(rounds):
    n = lib().orc_copies(rounds, None, 0)
    out = np.zeros((n, 4), dtype=np.uint32)
    lib().orc_copies(rounds, _p(out), n)
    return out


def compress(rounds, h, m, t, f):
    h = np.ascontiguousarray(h, dtype=np.uint64)
    m = np.ascontiguousarray(m, dtype=np.uint64)
    t = np.ascontiguousarray(t, dtype=np.uint64)
    out = np.zeros(8, dtype=np.uint64)
    lib().orc_compress(rounds, _p(h), _p(m), _p(t), int(bool(f)), _p(out))
    return out


def fill(inputs, total_rows=None, nthreads=0):
    """Returns (advice [10, total_rows] u32, fixed [total_rows] u32, h_out [n, 8] u64, offsets)."""
    inputs = np.ascontiguousarray(inputs, dtype=INPUT_DTYPE)
    off = offsets(inputs)
    total = int(off[-1]) if total_rows is None else int(total_rows)
    adv = np.empty((NCOLS, total), dtype=np.uint32)
    fixed = np.empty(total, dtype=np.uint32)
    h_out = np.zeros((len(inputs), 8), dtype=np.uint64)
    rc = lib().orc_fill(_p(inputs), len(inputs), _p(off), total, _p(adv), _p(fixed), _p(h_out),
                        nthreads)
    if rc != 0:
        raise ValueError("orc_fill: inconsistent offsets")
    return adv, fixed, h_out, off


TAMPER_ADD, TAMPER_CONST = 1, 2


def fill_tampered(inputs, inst, kind, row, delta):
    """A trace consistent with an altered fixed column (see orc_fill_tampered)."""
    inputs = np.ascontiguousarray(inputs, dtype=INPUT_DTYPE)
    off = offsets(inputs)
    total = int(off[-1])
    adv = np.empty((NCOLS, total), dtype=np.uint32)
    fixed = np.empty(total, dtype=np.uint32)
    h_out = np.zeros((len(inputs), 8), dtype=np.uint64)
    rc = lib().orc_fill_tampered(_p(inputs), len(inputs), _p(off), total, _p(adv), _p(fixed),
                                 _p(h_out), int(inst), int(kind), int(row), int(delta))
    if rc != 0:
        raise ValueError("orc_fill_tampered: inconsistent offsets")
    return adv, fixed, h_out, off


def evaluate(adv, fixed, off, nthreads=0):
    adv = np.ascontiguousarray(adv, dtype=np.uint32)
    fixed = np.ascontiguousarray(fixed, dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    rep = Report()
    rc = lib().orc_eval(_p(adv), _p(fixed), _p(off), len(off) - 1, adv.shape[1],
                        ctypes.byref(rep), nthreads)
    if rc != 0:
        raise ValueError("orc_eval: offsets are not a LAYOUT v1 row map")
    return rep.as_dict()


def fixed_structure(off, total_rows=None):
    """Keygen fixed column of a row map (structure-mode synthesis, zeros past off[-1])."""
    off = np.ascontiguousarray(off, dtype=np.uint64)
    total = int(off[-1]) if total_rows is None else int(total_rows)
    fx = np.empty(total, dtype=np.uint32)
    if lib().orc_fixed(_p(off), len(off) - 1, total, _p(fx)) != 0:
        raise ValueError("orc_fixed: offsets are not a LAYOUT v1 row map")
    return fx


FP_CANONICAL, FP_MONTGOMERY, FP_BN254_CANONICAL, FP_BN254_MONTGOMERY = 0, 1, 2, 3
PALLAS, BN254 = 0, 1
MODULI = {PALLAS: 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001,
          BN254: 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001}


def export_fp(adv, row_begin=0, nrows=None, form=FP_MONTGOMERY, out_rows=None):
    """Fp export restatement: returns u64 [10 (halo2 order), out_rows, 4] (rows past nrows
    zero)."""
    adv = np.ascontiguousarray(adv, dtype=np.uint32)
    total = adv.shape[1]
    nrows = total - row_begin if nrows is None else int(nrows)
    out_rows = nrows if out_rows is None else int(out_rows)
    out = np.zeros((NCOLS, out_rows, 4), dtype=np.uint64)
    lib().orc_export_fp(_p(adv), total, int(row_begin), nrows, int(form), _p(out), out_rows)
    return out


def fp_mont(x, field=PALLAS):
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_fp_mont(int(field), int(x), _p(out))
    return out


def max_threads():
    return int(lib().orc_max_threads())
