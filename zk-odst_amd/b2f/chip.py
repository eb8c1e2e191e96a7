"""Host-side mirror of the reference's gadget API over the C ABI.

Names, argument meaning and error behaviour follow the reference's intended batch API
(blake2f-circuit/src/blake2f.rs:184-304, commented out there; the names come from
zkevm-circuits): `Blake2fWitness{rounds, h, m, t, f}`, `Blake2fTable::construct`,
`Blake2fConfig::configure(meta, table)`, `Blake2fChip::construct(config, witnesses)` +
`chip.load(&mut layouter)`, checked by `MockProver::run(k, &circuit, vec![]).verify()`.
halo2 itself is not available here; `DeviceLayouter` stands in for the Layouter (it owns the
trace in HBM) and `MockProver` returns the verdict of the eval kernel.
"""
import numpy as np

from . import _lib
from .layout import (INPUT_DTYPE, SELECTORS, as_inputs, halo2_column_index, offsets,
                     parse_eip152)

# halo2's MockProver keeps the last rows of the 2^k domain for blinding; mirror its
# NotEnoughRowsAvailable check with the usual reserve (blinding factors + 1).
BLINDING_ROWS = 6
SPREAD_TABLE_ROWS = 1 << 16  # spread_table.rs:480 (forces k >= 17, spread_table.rs:759)


class Error(Exception):
    """plonk::Error"""


class NotEnoughRowsAvailable(Error):
    def __init__(self, current_k):
        super().__init__("NotEnoughRowsAvailable { current_k: %d }" % current_k)
        self.current_k = current_k


class Synthesis(Error):
    pass


class VerifyFailure(Exception):
    """Summary of MockProver::verify failures (VerifyFailure::{ConstraintNotSatisfied,
    Lookup, Permutation}); `first` locates the first failing row."""

    def __init__(self, report, first):
        self.report = report
        self.first = first
        parts = ["%s: %d" % (SELECTORS[g], c) for g, c in enumerate(report["gate_failures"]) if c]
        if report["lookup_failures"]:
            parts.append("lookup: %d" % report["lookup_failures"])
        if report["copy_failures"]:
            parts.append("permutation: %d" % report["copy_failures"])
        super().__init__("constraint system not satisfied (%s); first: %s"
                         % (", ".join(parts), first))


class Blake2fWitness:
    """One EIP-152 compression input (blake2f.rs:208-239)."""

    __slots__ = ("rounds", "h", "m", "t", "f")

    def __init__(self, rounds, h, m, t, f):
        self.rounds = int(rounds)
        self.h = [int(v) for v in h]
        self.m = [int(v) for v in m]
        self.t = [int(v) for v in t]
        self.f = bool(f)
        if len(self.h) != 8 or len(self.m) != 16 or len(self.t) != 2:
            raise Synthesis("Blake2fWitness needs h[8], m[16], t[2]")

    @classmethod
    def from_eip152(cls, raw):
        r = parse_eip152(raw)
        return cls(r["rounds"], r["h"], r["m"], r["t"], r["f"])

    def record(self):
        x = np.zeros((), dtype=INPUT_DTYPE)
        x["h"], x["m"], x["t"] = self.h, self.m, self.t
        x["rounds"], x["f"] = self.rounds, int(self.f)
        return x


class Blake2fTable:
    """The (tag, dense, spread) lookup table (spread_table.rs:331-335, generated as in
    spread_table.rs:574-600)."""

    rows = SPREAD_TABLE_ROWS

    @staticmethod
    def construct(meta=None):
        return Blake2fTable()

    @staticmethod
    def generate():
        dense = np.arange(SPREAD_TABLE_ROWS, dtype=np.uint32)
        tag = np.where(dense < 256, 0, np.where(dense < 32768, 1, 2)).astype(np.uint32)
        spread = np.zeros_like(dense)
        for b in range(16):
            spread |= ((dense >> b) & 1) << (2 * b)
        return tag, dense, spread


class Blake2fConfig:
    """Columns, selectors and the lookup of the chip (table16.rs:277-327,
    compression.rs:555-1074 as re-derived in docs/LAYOUT.md)."""

    def __init__(self, table):
        self.table = table
        self.advice = ["a_%d" % i for i in range(_lib.NUM_ADVICE)]
        self.halo2_index = {a: halo2_column_index(i) for i, a in enumerate(self.advice)}
        self.equality = ["a_%d" % i for i in range(1, 9)]  # table16.rs:312-314
        self.selectors = list(SELECTORS)
        self.lookup = (("a_0", "tag"), ("a_1", "dense"), ("a_2", "spread"))

    @staticmethod
    def configure(meta=None, table=None):
        return Blake2fConfig(table if table is not None else Blake2fTable.construct(meta))


class DeviceLayouter:
    """Stand-in for halo2's Layouter: regions are assigned into a trace kept in HBM."""

    def __init__(self, k, device="cuda:0"):
        self.k = int(k)
        self.device = device
        self.batch = None

    @property
    def usable_rows(self):
        return (1 << self.k) - BLINDING_ROWS

    def assign_batch(self, records, engine):
        from .engine import DeviceBatch

        records = as_inputs(records)
        if len(records) == 0:
            return None
        try:
            off = offsets(records)
        except _lib.B2FError as e:
            raise Synthesis(str(e))
        used = int(off[-1])
        if used > self.usable_rows or SPREAD_TABLE_ROWS > self.usable_rows:
            raise NotEnoughRowsAvailable(self.k)
        total = (used + 3) & ~3
        self.batch = DeviceBatch(records, device=self.device, total_rows=total)
        try:
            self.batch.fill(engine)
        except _lib.B2FError as e:
            if e.code == _lib.ERR_ROWS:
                raise NotEnoughRowsAvailable(self.k)
            raise Synthesis(str(e))
        return self.batch


class Blake2fChip:
    """`Blake2fChip::construct(config, Vec<Blake2fWitness>)` + `chip.load(&mut layouter)`."""

    def __init__(self, config, witnesses):
        self.config = config
        self.witnesses = list(witnesses)

    @staticmethod
    def construct(config, witnesses):
        return Blake2fChip(config, witnesses)

    def load(self, layouter, engine):
        recs = np.array([w.record() for w in self.witnesses], dtype=INPUT_DTYPE)
        return layouter.assign_batch(recs, engine)


class Blake2fCircuit:
    """`Blake2fTestCircuit { inputs }` (blake2f.rs:251-278)."""

    def __init__(self, inputs):
        self.inputs = list(inputs)

    def configure(self):
        return Blake2fConfig.configure(None, Blake2fTable.construct())

    def synthesize(self, config, layouter, engine):
        return Blake2fChip.construct(config, self.inputs).load(layouter, engine)


class MockProver:
    """`MockProver::run(k, &circuit, vec![])` then `.verify()` on the GPU."""

    def __init__(self, k, batch, engine):
        self.k = k
        self.batch = batch
        self.engine = engine

    @staticmethod
    def run(k, circuit, instances=(), engine=None, device="cuda:0"):
        from .engine import Engine

        if instances:
            raise Synthesis("the BLAKE2f chip has no instance columns")
        eng = engine or Engine(int(str(device).split(":")[-1]) if ":" in str(device) else 0)
        config = circuit.configure()
        layouter = DeviceLayouter(k, device)
        batch = circuit.synthesize(config, layouter, eng)
        return MockProver(k, batch, eng)

    def verify(self):
        """Ok(()) -> None; otherwise raises VerifyFailure."""
        if self.batch is None:
            return None
        import torch

        self.batch.evaluate(self.engine)
        self.engine.sync(torch.cuda.current_stream().cuda_stream)
        rep = self.batch.report_dict()
        if rep["first_failure"] == 2**64 - 1:
            return None
        key = rep["first_failure"]
        row, code = key >> 8, key & 0xff
        off = self.batch.offsets_host
        inst = int(np.searchsorted(off, row, side="right") - 1)
        what = (SELECTORS[code] if code < 16 else
                {_lib.CODE_LOOKUP: "lookup", _lib.CODE_COPY: "permutation",
                 _lib.CODE_FIXED: "fixed column (differs from keygen)",
                 _lib.CODE_LAYOUT: "row map rejected",
                 _lib.CODE_CHECK: "internal cross-check failed"}.get(code, "code %d" % code))
        raise VerifyFailure(rep, {"row": int(row), "instance": inst,
                                  "local_row": int(row - off[inst]), "constraint": what})

    def h_out(self):
        return self.batch.host_h_out()
