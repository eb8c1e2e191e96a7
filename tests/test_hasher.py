"""Host logic of the multi-block hasher (b2f/hasher.py): the Plan's
block words, byte counters, final flags and step prefixes, chained through the CPU oracle's
BLAKE2f compression, must give hashlib.blake2b's digests (RFC 7693) -- for empty, exact-block,
ragged and multi-block messages, keyed and unkeyed, every digest size class. No GPU."""
import hashlib

import numpy as np
import pytest

from b2f import hasher


def _chain_oracle(plan, orc):
    h = np.broadcast_to(plan.h0, (plan.n, 8)).copy()
    final = np.zeros((plan.n, 8), dtype=np.uint64)
    for j in range(plan.steps):
        blocks, t, f = plan.step(j)
        a = int(plan.active[j])
        nh = np.stack([orc.compress(12, h[i], blocks[i], t[i], int(f[i])) for i in range(a)])
        h[:a] = nh
        final[f.astype(bool).nonzero()[0]] = nh[f.astype(bool)]
    return plan.digests(final)


LENGTHS = [0, 1, 3, 64, 127, 128, 129, 255, 256, 257, 383, 500, 640]


@pytest.mark.parametrize("key", [b"", b"k", bytes(range(64))])
@pytest.mark.parametrize("digest_size", [1, 20, 32, 64])
def test_plan_chain_equals_hashlib(orc, key, digest_size):
    rng = np.random.default_rng(len(key) * 100 + digest_size)
    msgs = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in LENGTHS]
    rng.shuffle(msgs)
    plan = hasher.Plan(msgs, digest_size, key)
    got = _chain_oracle(plan, orc)
    for m, d in zip(msgs, got):
        assert d == hashlib.blake2b(m, digest_size=digest_size, key=key).digest(), len(m)


def test_plan_layout():
    msgs = [b"a" * 300, b"", b"b" * 128, b"c" * 129, b"d" * 1000]
    plan = hasher.Plan(msgs)
    # block counts 3, 1, 1, 2, 8 -> order by count, longest first (stable)
    assert list(plan.order) == [4, 0, 3, 1, 2]
    assert list(plan.active) == [5, 3, 2, 1, 1, 1, 1, 1]
    assert list(plan.start) == [0, 5, 8, 10, 11, 12, 13, 14, 15]
    # the active messages of every step are a prefix; flags mark each message's last block once
    assert int(plan.f.sum()) == 5
    b, t, f = plan.step(0)
    assert list(t[:, 0]) == [128, 128, 128, 0, 128] and list(f) == [0, 0, 0, 1, 1]
    b, t, f = plan.step(2)
    assert list(t[:, 0]) == [384, 300] and list(f) == [0, 1]
    b, t, f = plan.step(7)
    assert list(t[:, 0]) == [1000] and list(f) == [1]
    assert not plan.t[:, 1].any()


def test_param_state_errors():
    from b2f import B2FError

    with pytest.raises(B2FError):
        hasher.param_state(0)
    with pytest.raises(B2FError):
        hasher.param_state(65)
    with pytest.raises(B2FError):
        hasher.Plan([b"x"], 32, bytes(65))
    assert hasher.Plan([], 64).steps == 0


def test_workspace_reuse_rules():
    """hasher.Workspace (no allocation inside the timed hasher call): a plan's
    workspace is sized from the plan and reused by every plan that fits it (device, messages,
    compressions, steps, kept inputs). Built on the CPU device here: sizes only."""
    from b2f import hasher

    big = hasher.Plan([bytes(300), bytes(1000), b"x"])
    small = hasher.Plan([bytes(200), b"y"])
    ws = hasher.Workspace.for_plan(big, device="cpu")
    assert (ws.n, ws.compressions, ws.steps) == (3, int(big.start[-1]), big.steps)
    assert ws.advice.numel() == 10 * hasher.rows(12) * 3 and ws.inputs.numel() == 3 * 216
    assert ws.fits(big, "cpu") and ws.fits(small, "cpu")
    assert not ws.fits(big, "cpu", keep_inputs=True)  # kept inputs need a step-major buffer
    assert not hasher.Workspace.for_plan(small, device="cpu").fits(big, "cpu")
    kept = hasher.Workspace.for_plan(big, device="cpu", keep_inputs=True)
    assert kept.inputs.numel() == int(big.start[-1]) * 216 and kept.fits(small, "cpu", keep_inputs=True)
