"""Engine: one b2f_ctx on one HIP device, plus torch-allocated device trace buffers.

PyTorch is plumbing here (device memory, the stream handle); the work is the HIP kernels
behind include/b2f.h.
"""
import ctypes
import os

import numpy as np

from . import _lib
from .layout import INPUT_DTYPE, as_inputs, offsets as layout_offsets


def _vp(x):
    return ctypes.c_void_p(int(x))


def _np_ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


_hip = None


def hip_runtime():
    """The HIP runtime this process (torch and libb2f.so) uses, for the one call torch does not
    order for us (copy_h2d_async)."""
    global _hip
    if _hip is None:
        import torch

        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        _hip = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        _hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_int, ctypes.c_void_p]
        _hip.hipMemcpyAsync.restype = ctypes.c_int
    return _hip


def copy_h2d_async(dst, src, stream):
    """dst (device tensor) <- src (page-locked host tensor, same bytes) as hipMemcpyAsync on
    `stream`, the stream the library's launches go to: ordered before them. torch's own
    non_blocking copy (dst.copy_(src, non_blocking=True) under that stream) was measured NOT to
    be: tools/hasher_race.py (profiles/r03f_hasher_race.txt) -- 3 of 4 runs of 2^14 messages read
    a stale t counter in every step-0 input (49,152 wrong digests), 0 with this call, 0 with a
    host synchronize, 0 with blocking copies. The caller keeps src alive until the copy is done
    (the HIP call is invisible to torch's host allocator)."""
    nbytes = src.numel() * src.element_size()
    if nbytes != dst.numel() * dst.element_size():
        raise _lib.B2FError(_lib.ERR_ARG, "copy_h2d_async: %d bytes into %d"
                            % (nbytes, dst.numel() * dst.element_size()))
    rc = hip_runtime().hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), nbytes, 1, stream)
    if rc:
        raise _lib.B2FError(_lib.ERR_HIP, "hipMemcpyAsync returned %d" % rc)


class Engine:
    """Wraps b2f_create/b2f_destroy and the fill/eval entry points."""

    def __init__(self, device=0, diag=False, lib_path=None):
        """diag=True binds the diagnostics build (libb2f_diag.so); lib_path an explicit build
        of the same ABI (A/B runs). The default is the product library."""
        self.lib = _lib.load(diag=diag, path=lib_path)
        self.diag = bool(diag or lib_path)
        self.device = int(device)
        self.ctx = self.lib.b2f_create(self.device)
        if not self.ctx:
            raise _lib.B2FError(_lib.ERR_HIP, "b2f_create(%d) failed (no such HIP device?)" % device)

    def close(self):
        if self.ctx:
            self.lib.b2f_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        _lib.check(self.ctx, rc, self.lib)

    # ---------------------------------------------------------------- host-pointer calls
    def fill_host(self, inputs):
        """inputs: INPUT_DTYPE records. Returns (advice[10, R] u32, fixed[R] u32,
        h_out[n, 8] u64, offsets[n+1])."""
        inputs = as_inputs(inputs)
        off = layout_offsets(inputs)
        total = int(off[-1])
        adv = np.empty((_lib.NUM_ADVICE, total), dtype=np.uint32)
        fixed = np.empty(total, dtype=np.uint32)
        h_out = np.empty((len(inputs), 8), dtype=np.uint64)
        self._check(self.lib.b2f_fill(self.ctx, _np_ptr(inputs), len(inputs), _np_ptr(adv),
                                      _np_ptr(fixed), _np_ptr(h_out)))
        return adv, fixed, h_out, off

    def eval_host(self, adv, fixed, off):
        adv = np.ascontiguousarray(adv, dtype=np.uint32)
        fixed = np.ascontiguousarray(fixed, dtype=np.uint32)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        rep = _lib.EvalReport()
        self._check(self.lib.b2f_eval(self.ctx, _np_ptr(adv), _np_ptr(fixed), _np_ptr(off),
                                      len(off) - 1, adv.shape[1], ctypes.byref(rep)))
        return rep.as_dict()

    # ---------------------------------------------------------------- device-pointer calls
    def fill_dev(self, d_in, n, d_off, total_rows, d_adv, d_fixed, d_h_out, stream=0):
        self._check(self.lib.b2f_fill_dev(self.ctx, _vp(d_in), n, _vp(d_off), int(total_rows),
                                          _vp(d_adv), _vp(d_fixed),
                                          _vp(d_h_out) if d_h_out else None, _vp(stream)))

    def eval_dev(self, d_adv, d_fixed, d_off, n, total_rows, d_report, stream=0):
        self._check(self.lib.b2f_eval_dev(self.ctx, _vp(d_adv), _vp(d_fixed), _vp(d_off), n,
                                          int(total_rows), _vp(d_report), _vp(stream)))

    def fill_eval_dev(self, d_in, n, d_off, total_rows, d_adv, d_fixed, d_h_out, d_report,
                      stream=0):
        self._check(self.lib.b2f_fill_eval_dev(self.ctx, _vp(d_in), n, _vp(d_off),
                                               int(total_rows), _vp(d_adv), _vp(d_fixed),
                                               _vp(d_h_out) if d_h_out else None,
                                               _vp(d_report), _vp(stream)))

    def fill_fixed_dev(self, d_off, n, total_rows, d_fixed, stream=0):
        """Keygen structure: the fixed column from the row map alone (b2f_fill_fixed_dev)."""
        self._check(self.lib.b2f_fill_fixed_dev(self.ctx, _vp(d_off), int(n), int(total_rows),
                                                _vp(d_fixed), _vp(stream)))

    def debug_inject(self, row=None, col=0, mask=0):
        """Test hook: XOR `mask` into cell (row, col) (col 10 = fixed) as the fused path assigns
        it; row=None turns it off."""
        r = 2**64 - 1 if row is None else int(row)
        self._check(self.lib.b2f_debug_inject(self.ctx, r, int(col), int(mask) & 0xffffffff))

    def chain_inputs_dev(self, d_h_prev, d_blocks, d_t, d_f, rounds, n, d_out, stream=0):
        self._check(self.lib.b2f_chain_inputs_dev(self.ctx, _vp(d_h_prev), _vp(d_blocks), _vp(d_t),
                                                  _vp(d_f), int(rounds), int(n), _vp(d_out),
                                                  _vp(stream)))

    def export_fp_dev(self, d_adv, total_rows, row_begin, nrows, form, d_out, out_rows,
                      stream=0):
        self._check(self.lib.b2f_export_fp_dev(self.ctx, _vp(d_adv), int(total_rows),
                                               int(row_begin), int(nrows), int(form),
                                               _vp(d_out), int(out_rows), _vp(stream)))

    def lookup_columns_dev(self, d_adv, total_rows, d_row_begin, n_circuits, usable_rows, theta,
                           beta, gamma, form, d_out, out_rows, d_first_bad, stream=0):
        """b2f_lookup_columns_dev; theta/beta/gamma are Python ints (canonical Fp)."""
        lim = [(ctypes.c_uint64 * 4)(*[(int(v) >> (64 * k)) & (2**64 - 1) for k in range(4)])
               for v in (theta, beta, gamma)]
        self._check(self.lib.b2f_lookup_columns_dev(
            self.ctx, _vp(d_adv), int(total_rows), _vp(d_row_begin), int(n_circuits),
            int(usable_rows), lim[0], lim[1], lim[2], int(form), _vp(d_out), int(out_rows),
            _vp(d_first_bad), _vp(stream)))

    def spread_table_dev(self, usable_rows, form, d_out, out_rows, stream=0):
        self._check(self.lib.b2f_spread_table_dev(self.ctx, int(usable_rows), int(form), _vp(d_out),
                                                  int(out_rows), _vp(stream)))

    def spread_table(self, usable_rows, form=_lib.FP_MONTGOMERY, device="cuda:0", stream=None):
        """The spread table's three prover columns (tag, dense, spread): int64 tensor
        [3, usable_rows, 4] of field elements in `form` (b2f_spread_table_dev)."""
        import torch

        out = torch.empty((3, int(usable_rows), 4), dtype=torch.int64, device=device)
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self.spread_table_dev(usable_rows, form, out.data_ptr(), int(usable_rows), s)
        return out

    def permutation_columns_dev(self, d_adv, total_rows, h_offsets, k, usable_rows, omega, delta,
                                beta, gamma, chunk_len, form, d_sigma, d_z, out_rows, stream=0):
        """b2f_permutation_columns_dev; h_offsets: host u64 row map of the circuit's instances,
        omega/delta/beta/gamma Python ints (canonical)."""
        off = np.ascontiguousarray(h_offsets, dtype=np.uint64)
        lim = [(ctypes.c_uint64 * 4)(*[(int(v) >> (64 * i)) & (2**64 - 1) for i in range(4)])
               for v in (omega, delta, beta, gamma)]
        self._check(self.lib.b2f_permutation_columns_dev(
            self.ctx, _vp(d_adv), int(total_rows), _np_ptr(off), len(off) - 1, int(k),
            int(usable_rows), lim[0], lim[1], lim[2], lim[3], int(chunk_len), int(form),
            _vp(d_sigma) if d_sigma else None, _vp(d_z), int(out_rows), _vp(stream)))

    def permutation_sigma_dev(self, h_offsets, k, omega, delta, form, d_sigma, out_rows, stream=0):
        """b2f_permutation_sigma_dev (keygen: the sigma columns alone); omega/delta Python ints."""
        off = np.ascontiguousarray(h_offsets, dtype=np.uint64)
        lim = [(ctypes.c_uint64 * 4)(*[(int(v) >> (64 * i)) & (2**64 - 1) for i in range(4)])
               for v in (omega, delta)]
        self._check(self.lib.b2f_permutation_sigma_dev(
            self.ctx, _np_ptr(off), len(off) - 1, int(k), lim[0], lim[1], int(form), _vp(d_sigma),
            int(out_rows), _vp(stream)))

    def debug_eval_path(self):
        """Path of the last eval_dev call (device-synchronizing): 0 the fast clean-check pass
        found the trace clean, 1 it flagged something and the exact eval kernel reported, 2 no
        fast pass ran."""
        out = ctypes.c_uint32(0)
        self._check(self.lib.b2f_debug_eval_path(self.ctx, ctypes.byref(out)))
        return int(out.value)

    def sync(self, stream=0):
        self._check(self.lib.b2f_sync(self.ctx, _vp(stream)))

    def set_timing(self, enable=True):
        self._check(self.lib.b2f_set_timing(self.ctx, 1 if enable else 0))

    def kernel_times(self):
        """{kernel: (total_ms, launches)} since set_timing(True) / the previous call."""
        k = int(self.lib.b2f_num_kernels())  # the library's count sizes the buffers
        if k != len(_lib.KERNEL_NAMES):
            raise _lib.B2FError(_lib.ERR_ARG, "library reports %d kernel kinds, binding knows %d"
                                % (k, len(_lib.KERNEL_NAMES)))
        tot = (ctypes.c_double * k)()
        cnt = (ctypes.c_uint32 * k)()
        self._check(self.lib.b2f_kernel_times(self.ctx, tot, cnt))
        return {name: (float(tot[i]), int(cnt[i])) for i, name in enumerate(_lib.KERNEL_NAMES)}


def permutation_mapping(rounds):
    """Keygen's permutation mapping of one instance: u32 [8, R] entries (c' << 29) | r'
    (b2f_permutation_mapping)."""
    lib = _lib.load()
    n = int(lib.b2f_permutation_mapping(int(rounds), None, 0))
    out = np.zeros(n, dtype=np.uint32)
    lib.b2f_permutation_mapping(int(rounds), _np_ptr(out), n)
    return out.reshape(8, -1)


def copy_constraints(rounds):
    """The copy constraints of one instance: u32 [count, 4] (dst_row, dst_col, src_row,
    src_col), instance-relative rows (b2f_copy_constraints)."""
    lib = _lib.load()
    n = int(lib.b2f_copy_constraints(int(rounds), None, 0))
    out = np.zeros((n, 4), dtype=np.uint32)
    lib.b2f_copy_constraints(int(rounds), _np_ptr(out), n)
    return out


class DeviceBatch:
    """A batch resident on one GPU: inputs, offsets, the trace and the outputs, as torch
    tensors (int32/int64 storage holding u32/u64 bit patterns)."""

    def __init__(self, inputs, device="cuda:0", total_rows=None):
        import torch

        self.torch = torch
        inputs = as_inputs(inputs)
        self.n = len(inputs)
        off = layout_offsets(inputs)
        self.offsets_host = off
        self.used_rows = int(off[-1])
        self.total_rows = int(total_rows) if total_rows is not None else self.used_rows
        if self.total_rows < self.used_rows or self.total_rows % 4:
            raise _lib.B2FError(_lib.ERR_ROWS, "total_rows %d (need >= %d, multiple of 4)"
                                % (self.total_rows, self.used_rows))
        dev = torch.device(device)
        raw = np.frombuffer(inputs.tobytes(), dtype=np.uint8)
        # synchronous (pageable) uploads: construction is not the hot path, and a later launch
        # on any stream sees them (see copy_h2d_async for the asynchronous form)
        self.inputs = torch.from_numpy(raw.copy()).to(dev)
        self.offsets = torch.from_numpy(off.view(np.int64).copy()).to(dev)
        self.advice = torch.empty((_lib.NUM_ADVICE, self.total_rows), dtype=torch.int32, device=dev)
        self.fixed = torch.empty(self.total_rows, dtype=torch.int32, device=dev)
        self.h_out = torch.empty((self.n, 8), dtype=torch.int64, device=dev)
        self.report = torch.empty(_lib.REPORT_BYTES // 8, dtype=torch.int64, device=dev)

    def fill(self, eng, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream().cuda_stream
        eng.fill_dev(self.inputs.data_ptr(), self.n, self.offsets.data_ptr(), self.total_rows,
                     self.advice.data_ptr(), self.fixed.data_ptr(), self.h_out.data_ptr(), s)

    def evaluate(self, eng, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream().cuda_stream
        eng.eval_dev(self.advice.data_ptr(), self.fixed.data_ptr(), self.offsets.data_ptr(),
                     self.n, self.total_rows, self.report.data_ptr(), s)

    def fill_evaluate(self, eng, stream=None):
        """Fused fill + eval (b2f_fill_eval_dev): trace, h' and report in one pass."""
        s = stream if stream is not None else self.torch.cuda.current_stream().cuda_stream
        eng.fill_eval_dev(self.inputs.data_ptr(), self.n, self.offsets.data_ptr(),
                          self.total_rows, self.advice.data_ptr(), self.fixed.data_ptr(),
                          self.h_out.data_ptr(), self.report.data_ptr(), s)

    def export_fp(self, eng, row_begin=0, nrows=None, form=_lib.FP_MONTGOMERY, out=None,
                  stream=None):
        """Advice rows [row_begin, row_begin + nrows) as pallas Fp elements: int64 tensor
        [10 (halo2 column order), out_rows, 4] (u64 limb bit patterns). `out` may be a
        preallocated tensor of that shape (out_rows >= nrows)."""
        torch = self.torch
        nrows = self.total_rows - row_begin if nrows is None else int(nrows)
        if out is None:
            out = torch.empty((_lib.NUM_ADVICE, nrows, 4), dtype=torch.int64,
                              device=self.advice.device)
        if out.dim() != 3 or out.shape[0] != _lib.NUM_ADVICE or out.shape[2] != 4 \
                or out.dtype != torch.int64 or not out.is_contiguous():
            raise _lib.B2FError(_lib.ERR_ARG, "export_fp: out must be contiguous int64 [10, rows, 4]")
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        eng.export_fp_dev(self.advice.data_ptr(), self.total_rows, row_begin, nrows, form,
                          out.data_ptr(), out.shape[1], s)
        return out

    def lookup_columns(self, eng, row_begin, usable_rows, theta, beta, gamma,
                       form=_lib.FP_MONTGOMERY, stream=None):
        """Lookup-argument prover columns for circuits starting at trace rows `row_begin`:
        (out int64 [n_circuits, 5 (A, S, A', S', z), usable_rows + 1, 4], first_bad int64
        [n_circuits]) -- see b2f_lookup_columns_dev."""
        torch = self.torch
        dev = self.advice.device
        rb = torch.tensor([int(r) for r in row_begin], dtype=torch.int64, device=dev)
        nc = len(row_begin)
        out = torch.empty((nc, 5, usable_rows + 1, 4), dtype=torch.int64, device=dev)
        bad = torch.empty(nc, dtype=torch.int64, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        eng.lookup_columns_dev(self.advice.data_ptr(), self.total_rows, rb.data_ptr(), nc,
                               usable_rows, theta, beta, gamma, form, out.data_ptr(),
                               usable_rows + 1, bad.data_ptr(), s)
        return out, bad

    def permutation_columns(self, eng, k, usable_rows, beta, gamma, chunk_len=3,
                            form=_lib.FP_MONTGOMERY, instances=None, sigma=True, stream=None):
        """Permutation-argument prover columns of the circuit holding instances
        [i0, i1) = `instances` (default: all) in a 2^k-row domain: (sigma int64 [8, 2^k, 4] or
        None, z int64 [sets, 2^k, 4] with rows 0..usable_rows written) -- see
        b2f_permutation_columns_dev. omega and delta come from the field of `form`."""
        from . import field

        torch = self.torch
        dev = self.advice.device
        i0, i1 = (0, self.n) if instances is None else instances
        off = self.offsets_host[i0:i1 + 1]
        f = field.of_form(form)
        n_rows = 1 << int(k)
        sets = (8 + chunk_len - 1) // chunk_len
        sig = torch.empty((8, n_rows, 4), dtype=torch.int64, device=dev) if sigma else None
        z = torch.empty((sets, n_rows, 4), dtype=torch.int64, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        eng.permutation_columns_dev(self.advice.data_ptr(), self.total_rows, off, k, usable_rows,
                                    field.omega(f, int(k)), field.delta(f), beta, gamma,
                                    chunk_len, form, sig.data_ptr() if sigma else 0,
                                    z.data_ptr(), n_rows, s)
        return sig, z

    def permutation_sigma(self, eng, k, form=_lib.FP_MONTGOMERY, instances=None, stream=None):
        """Keygen's sigma columns (int64 [8, 2^k, 4]) of the circuit holding instances
        [i0, i1) = `instances` (default: all): b2f_permutation_sigma_dev, the same columns
        permutation_columns returns, without a witness."""
        from . import field

        torch = self.torch
        i0, i1 = (0, self.n) if instances is None else instances
        off = self.offsets_host[i0:i1 + 1]
        f = field.of_form(form)
        n_rows = 1 << int(k)
        sig = torch.empty((8, n_rows, 4), dtype=torch.int64, device=self.advice.device)
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        eng.permutation_sigma_dev(off, k, field.omega(f, int(k)), field.delta(f), form, sig.data_ptr(),
                                  n_rows, s)
        return sig

    def report_dict(self):
        raw = self.report.cpu().numpy().view(np.uint64)
        rep = _lib.EvalReport.from_buffer_copy(raw.tobytes())
        return rep.as_dict()

    def host_trace(self):
        adv = self.advice.cpu().numpy().view(np.uint32)
        fixed = self.fixed.cpu().numpy().view(np.uint32)
        return adv, fixed

    def host_h_out(self):
        return self.h_out.cpu().numpy().view(np.uint64)
