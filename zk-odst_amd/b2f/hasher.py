"""Multi-block BLAKE2b over the chip (the chaining half).

Mirrors the reference gadget's hasher API, blake2f-circuit/src/blake2f.rs:81-180:
`Blake2f::new` (state from the chip's IV, :90-98), `update` (absorb data, compress each full
block, :101-147), `finalize` (pad and compress the last block, take the digest, :150-168) and
the one-shot `digest` (:172-179). The reference's gadget is unfinished -- it is the SHA-256
gadget's shape (32-bit BlockWords, `length += len * 32`, no byte counter, no final-block flag),
so its chaining would not compute BLAKE2b. The hasher here follows RFC 7693 BLAKE2b instead
(parameter block in h[0], byte counter t, final flag f, optional key block, digest truncation)
and is pinned to `hashlib.blake2b` by tests/test_hasher.py and tests/test_gpu_hasher.py.

A batch of messages runs one block step at a time: every step is one fill (+ eval) of the
chip over the messages that still have blocks, with their compression inputs built on the
device from the previous step's outputs (b2f_chain_inputs_dev). Messages are ordered by block
count, longest first, so the messages still running at step j are a prefix 0 .. active[j] - 1
and every step's trace, offsets and outputs are prefixes of one allocation.
"""
import numpy as np

from . import _lib
from .engine import copy_h2d_async
from .layout import rows

BLOCK_BYTES = 128
BLAKE2B_ROUNDS = 12
IV = np.array([0x6A09E667F3BCC908, 0xBB67AE8584CAA73B, 0x3C6EF372FE94F82B, 0xA54FF53A5F1D36F1,
               0x510E527FADE682D1, 0x9B05688C2B3E6C1F, 0x1F83D9ABFB41BD6B, 0x5BE0CD19137E2179],
              dtype=np.uint64)


def param_state(digest_size=64, key_len=0):
    """h0 = IV ^ parameter block (RFC 7693 §3.3: fanout 1, depth 1, key length, digest
    length; the rest zero)."""
    if not 1 <= digest_size <= 64:
        raise _lib.B2FError(_lib.ERR_ARG, "digest_size %d not in 1..64" % digest_size)
    if not 0 <= key_len <= 64:
        raise _lib.B2FError(_lib.ERR_ARG, "key length %d > 64" % key_len)
    h = IV.copy()
    h[0] ^= np.uint64(0x01010000 | (key_len << 8) | digest_size)
    return h


class Plan:
    """Host side of a batch: every compression's message words, byte counter and final flag,
    step-major (step j's messages at rows start[j] .. start[j] + active[j] - 1, in `order`)."""

    def __init__(self, messages, digest_size=64, key=b""):
        key = bytes(key)
        self.digest_size = int(digest_size)
        self.h0 = param_state(self.digest_size, len(key))
        prefix = key.ljust(BLOCK_BYTES, b"\0") if key else b""
        datas = [prefix + bytes(m) for m in messages]
        self.n = len(datas)
        nblocks = np.array([max(1, -(-len(d) // BLOCK_BYTES)) for d in datas], dtype=np.int64)
        self.order = np.argsort(-nblocks, kind="stable")
        nb_sorted = nblocks[self.order]
        self.steps = int(nb_sorted[0]) if self.n else 0
        self.active = np.array([int((nb_sorted > j).sum()) for j in range(self.steps)],
                               dtype=np.int64)
        self.start = np.concatenate([[0], np.cumsum(self.active)]).astype(np.int64)
        total = int(self.start[-1])
        self.blocks = np.zeros((total, 16), dtype=np.uint64)
        self.t = np.zeros((total, 2), dtype=np.uint64)
        self.f = np.zeros(total, dtype=np.uint32)
        for pos, i in enumerate(self.order):
            d = datas[i]
            nb = int(nblocks[i])
            idx = self.start[:nb] + pos
            self.blocks[idx] = np.frombuffer(d.ljust(nb * BLOCK_BYTES, b"\0"),
                                             dtype="<u8").reshape(nb, 16)
            self.t[idx, 0] = np.minimum(np.arange(1, nb + 1, dtype=np.uint64) * BLOCK_BYTES,
                                        np.uint64(len(d)))
            self.f[idx[-1]] = 1

    def pinned(self):
        """The plan's blocks, counters, flags, initial states and the row of every message's
        final h' (step-major), as page-locked host tensors (built once and cached), so every
        upload is an asynchronous DMA ordered on the stream (engine.upload explains why a
        pageable copy is not)."""
        if not hasattr(self, "_pinned"):
            import torch

            def pin(a):
                a = np.array(a, order="C")  # a writable copy (h0 is a broadcast view)
                return torch.from_numpy(a.view(np.int64 if a.dtype in (np.uint64, np.int64)
                                               else np.int32)).pin_memory()

            h0 = np.broadcast_to(self.h0, (self.n, 8))
            # message at sorted position p ends at step nblocks - 1, i.e. at row start[nb - 1] + p
            last = (self.active[None, :] > np.arange(self.n)[:, None]).sum(1) - 1
            fin = (self.start[last] + np.arange(self.n)).astype(np.int64)
            self._pinned = (pin(self.blocks), pin(self.t), pin(self.f), pin(h0), pin(fin))
        return self._pinned

    def step(self, j):
        """(blocks, t, f) of step j: arrays over messages 0 .. active[j] - 1 (sorted order)."""
        s, e = int(self.start[j]), int(self.start[j + 1])
        return self.blocks[s:e], self.t[s:e], self.f[s:e]

    def digests(self, final_h):
        """final_h: [n, 8] u64 in sorted order -> digests (bytes) in the callers' order."""
        out = [b""] * self.n
        raw = np.ascontiguousarray(final_h, dtype="<u8")
        for pos, i in enumerate(self.order):
            out[int(i)] = raw[pos].tobytes()[:self.digest_size]
        return out


class ChainResult:
    def __init__(self, plan, reports, final_sorted):
        self.plan = plan
        self.reports = reports  # one MockProver report per block step
        self._final_sorted = final_sorted  # [n, 8] u64, sorted order

    @property
    def final_h(self):
        """[n, 8] u64 final chaining values, callers' order."""
        fin = np.empty_like(self._final_sorted)
        fin[self.plan.order] = self._final_sorted
        return fin

    @property
    def digests(self):
        """Digest bytes per message, callers' order (built on first access)."""
        if not hasattr(self, "_digests"):
            self._digests = self.plan.digests(self._final_sorted)
        return self._digests

    @property
    def verified(self):
        return all(r["first_failure"] == 2**64 - 1 for r in self.reports)


def blake2b_batch(engine, messages, digest_size=64, key=b"", path="fused", device="cuda:0",
                  stream=None):
    """BLAKE2b digests of `messages` (a list of bytes-like) through the chip on one GPU, every
    block step witnessed and checked: path "fused" (b2f_fill_eval_dev, the default) or "split"
    (b2f_fill_dev + b2f_eval_dev)."""
    return run_plan(engine, Plan(messages, digest_size, key), path, device, stream)


class Workspace:
    """Device buffers of a hasher batch: blocks, counters, flags, initial states, every step's
    h', the step's compression inputs, the trace (advice + fixed) and the per-step reports.
    Allocated once and reused by every run_plan call whose plan fits (no
    allocation inside the fill hot calls). A plan keeps the workspace its first run made
    (Plan.workspace); a caller running many plans can pass one sized for the largest."""

    def __init__(self, n, compressions, steps, device="cuda:0", keep_inputs=False):
        import torch

        dev = torch.device(device)
        R = rows(BLAKE2B_ROUNDS)
        self.device, self.n, self.compressions, self.steps = dev, int(n), int(compressions), int(steps)
        self.keep_inputs = bool(keep_inputs)
        self.blocks = torch.empty((self.compressions, 16), dtype=torch.int64, device=dev)
        self.t = torch.empty((self.compressions, 2), dtype=torch.int64, device=dev)
        self.f = torch.empty(self.compressions, dtype=torch.int32, device=dev)
        self.h0 = torch.empty((self.n, 8), dtype=torch.int64, device=dev)
        self.fin_idx = torch.empty(self.n, dtype=torch.int64, device=dev)
        self.offsets = torch.arange(self.n + 1, dtype=torch.int64, device=dev) * R
        # h' of every compression, step-major like the plan: step j's outputs are rows
        # start[j] .. start[j] + active[j] - 1, and step j + 1 reads its h from that prefix
        self.hs = torch.empty((self.compressions, 8), dtype=torch.int64, device=dev)
        self.inputs = torch.empty((self.compressions if keep_inputs else self.n) * 216,
                                  dtype=torch.uint8, device=dev)
        # one flat trace buffer: a step over `a` messages uses its first 10 * R * a words as
        # advice[10][R * a] (column stride R * a) and the fixed column beside it
        self.advice = torch.empty(_lib.NUM_ADVICE * R * self.n, dtype=torch.int32, device=dev)
        self.fixed = torch.empty(R * self.n, dtype=torch.int32, device=dev)
        self.report = torch.empty((self.steps, _lib.REPORT_BYTES // 8), dtype=torch.int64,
                                  device=dev)

    @classmethod
    def for_plan(cls, plan, device="cuda:0", keep_inputs=False):
        return cls(plan.n, int(plan.start[-1]), plan.steps, device, keep_inputs)

    def fits(self, plan, device, keep_inputs=False):
        import torch

        return (torch.device(device) == self.device and plan.n <= self.n
                and int(plan.start[-1]) <= self.compressions and plan.steps <= self.steps
                and (self.keep_inputs or not keep_inputs))


def run_plan(engine, plan, path="fused", device="cuda:0", stream=None, workspace=None,
             phases=None, _diag=None):
    """The device half of blake2b_batch for a prebuilt Plan. The blocks go up in one
    asynchronous copy from page-locked memory (Plan.pinned), every block step runs on the
    stream, and only the final chaining values come back to the host. Buffers come from
    `workspace` (a Workspace that fits the plan) or the plan's own, made by its first run.
    `phases`, a dict, receives the call's phase times in ms (host wall clock, the stream
    synchronized between phases -- only when asked for): workspace (allocation, ~0 when reused),
    upload, steps, download."""
    import time

    import torch

    if path not in ("split", "fused"):
        raise _lib.B2FError(_lib.ERR_ARG, "path must be 'split' or 'fused'")
    n = plan.n
    if n == 0:
        return ChainResult(plan, [], np.zeros((0, 8), dtype=np.uint64))
    dev = torch.device(device)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    compute = torch.cuda.ExternalStream(s, device=dev)
    p_blocks, p_t, p_f, p_h0, p_fin = plan.pinned()
    R = rows(BLAKE2B_ROUNDS)
    keep = _diag is not None and _diag.get("keep_inputs")
    tw = time.perf_counter()
    ws = workspace
    if ws is None:
        ws = getattr(plan, "workspace", None)
        if ws is None or not ws.fits(plan, dev, keep):
            # allocated on the stream `s` so its memory is ordered with the launches below
            with torch.cuda.stream(compute):
                ws = Workspace.for_plan(plan, dev, keep)
            plan.workspace = ws
    elif not ws.fits(plan, dev, keep):
        raise _lib.B2FError(_lib.ERR_ARG, "run_plan: workspace too small for the plan")
    alloc_ms = 1e3 * (time.perf_counter() - tw)
    total_c = int(plan.start[-1])
    d_blocks, d_t, d_f = ws.blocks[:total_c], ws.t[:total_c], ws.f[:total_c]
    h0, fin_idx, hs = ws.h0[:n], ws.fin_idx[:n], ws.hs
    offsets, inputs_all, advice, fixed, report = ws.offsets, ws.inputs, ws.advice, ws.fixed, ws.report
    if phases is not None:
        compute.synchronize()
        tp = [time.perf_counter()]
    # Every host -> device copy is hipMemcpyAsync from page-locked memory on `s` itself
    # (engine.copy_h2d_async: torch's non_blocking copy is not ordered before the library's
    # launches), so no host synchronize is needed (tests/test_gpu_hasher.py runs batches back
    # to back on alternating paths, without one).
    how = _diag.get("upload", "hip") if _diag is not None else "hip"
    if how == "hip":
        for d, p in ((d_blocks, p_blocks), (d_t, p_t), (d_f, p_f), (h0, p_h0), (fin_idx, p_fin)):
            copy_h2d_async(d, p, s)
    else:  # diagnostics (tools/hasher_race.py): torch's copy, non-blocking or blocking
        nb = how != "blocking"
        with torch.cuda.stream(compute):
            for d, p in ((d_blocks, p_blocks), (d_t, p_t), (d_f, p_f), (h0, p_h0), (fin_idx, p_fin)):
                d.copy_(p, non_blocking=nb)
    if _diag is not None and _diag.get("sync_upload"):  # diagnostics (tools/hasher_race.py)
        if _diag["sync_upload"] == "stream":
            compute.synchronize()
        else:
            torch.cuda.synchronize(dev)
    if phases is not None:
        compute.synchronize()
        tp.append(time.perf_counter())
    for j in range(plan.steps):
        a = int(plan.active[j])
        s0 = int(plan.start[j])
        h_prev = h0 if j == 0 else hs[int(plan.start[j - 1])]
        inputs = inputs_all[s0 * 216:] if keep else inputs_all
        engine.chain_inputs_dev(h_prev.data_ptr(), d_blocks[s0].data_ptr(), d_t[s0].data_ptr(),
                                d_f[s0:].data_ptr(), BLAKE2B_ROUNDS, a, inputs.data_ptr(), s)
        total = R * a
        h_out = hs[s0].data_ptr()
        if path == "fused":
            engine.fill_eval_dev(inputs.data_ptr(), a, offsets.data_ptr(), total,
                                 advice.data_ptr(), fixed.data_ptr(), h_out,
                                 report[j].data_ptr(), s)
        else:
            engine.fill_dev(inputs.data_ptr(), a, offsets.data_ptr(), total, advice.data_ptr(),
                            fixed.data_ptr(), h_out, s)
            engine.eval_dev(advice.data_ptr(), fixed.data_ptr(), offsets.data_ptr(), a, total,
                            report[j].data_ptr(), s)
    engine.sync(s)
    if phases is not None:
        tp.append(time.perf_counter())
    td = time.perf_counter()
    with torch.cuda.stream(compute):
        fin_host = hs.index_select(0, fin_idx).cpu().numpy().view(np.uint64)
        raw = report[:plan.steps].cpu().numpy().view(np.uint64)
    if phases is not None:
        phases.update({"workspace_ms": round(alloc_ms, 3),
                       "upload_ms": round(1e3 * (tp[1] - tp[0]), 3),
                       "steps_ms": round(1e3 * (tp[2] - tp[1]), 3),
                       "download_ms": round(1e3 * (time.perf_counter() - td), 3)})
    reps = [_lib.EvalReport.from_buffer_copy(raw[j].tobytes()).as_dict()
            for j in range(plan.steps)]
    res = ChainResult(plan, reps, fin_host)
    if _diag is not None:  # diagnostics: every step's h' (step-major, sorted order)
        res.all_h = hs[:total_c].cpu().numpy().view(np.uint64)
        res.stream = int(s)
        if keep:  # every step's b2f_input records as chain_inputs built them
            res.all_inputs = inputs_all[:total_c * 216].cpu().numpy()
    return res


class Blake2f:
    """The reference gadget's hasher (blake2f.rs:81-180) over the GPU chip, for one message:
    new -> update* -> finalize, or the one-shot digest. Data is buffered until finalize (BLAKE2b
    cannot compress a full block before it knows whether it is the last one); finalize runs
    every block step through the chip and raises B2FError if any step's trace fails its
    constraints."""

    def __init__(self, engine, digest_size=64, key=b"", device="cuda:0", path="fused"):
        param_state(digest_size, len(key))  # validates
        self.engine, self.digest_size, self.key = engine, digest_size, bytes(key)
        self.device, self.path = device, path
        self._buf = bytearray()
        self.length = 0

    @classmethod
    def new(cls, engine, **kw):
        return cls(engine, **kw)

    def update(self, data):
        data = bytes(data)
        self._buf += data
        self.length += len(data)
        return self

    def finalize(self):
        res = blake2b_batch(self.engine, [bytes(self._buf)], self.digest_size, self.key,
                            self.path, self.device)
        if not res.verified:
            bad = next(r for r in res.reports if r["first_failure"] != 2**64 - 1)
            raise _lib.B2FError(_lib.ERR_INPUT, "chip constraints failed at row %d"
                                % bad["first_failure"])
        return res.digests[0]

    @classmethod
    def digest(cls, engine, data, **kw):
        return cls(engine, **kw).update(data).finalize()
