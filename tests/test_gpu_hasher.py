"""Multi-block BLAKE2b through the chip on the GPU (b2f/hasher.py + b2f_chain_inputs_dev,
SURVEY.md §8(f) row 3): digests equal hashlib.blake2b, every block step's trace passes the
MockProver check, on both the split and the fused path. Needs an MI355X (`-m gpu`)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _msgs(rng, n, max_len):
    lens = rng.integers(0, max_len, n)
    lens[: min(n, 6)] = [0, 1, 127, 128, 129, 256][: min(n, 6)]
    return [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]


@pytest.mark.parametrize("path", ["split", "fused"])
@pytest.mark.parametrize("key,digest_size", [(b"", 64), (b"secret key", 32), (bytes(64), 7)])
def test_batch_equals_hashlib(engine, path, key, digest_size):
    from b2f import hasher

    rng = np.random.default_rng(digest_size + len(key))
    msgs = _msgs(rng, 300, 1200)
    res = hasher.blake2b_batch(engine, msgs, digest_size, key, path=path)
    assert res.verified, [r for r in res.reports if r["first_failure"] != 2**64 - 1][:1]
    assert len(res.reports) == max(1, -(-(max(map(len, msgs)) + (128 if key else 0)) // 128))
    for m, d in zip(msgs, res.digests):
        assert d == hashlib.blake2b(m, digest_size=digest_size, key=key).digest(), len(m)


def test_blake2f_api(engine):
    """new / update / finalize and the one-shot digest (blake2f.rs:90-179)."""
    from b2f.hasher import Blake2f

    data = bytes(range(256)) * 3
    h = Blake2f.new(engine)
    for i in range(0, len(data), 100):
        h.update(data[i:i + 100])
    assert h.finalize() == hashlib.blake2b(data).digest()
    assert Blake2f.digest(engine, b"abc", digest_size=32) == \
        hashlib.blake2b(b"abc", digest_size=32).digest()
    assert Blake2f.digest(engine, b"") == hashlib.blake2b(b"").digest()


def test_many_equal_messages(engine):
    """2^14 messages of 1 KiB (8 block steps, every step full width)."""
    from b2f import hasher

    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, (1 << 14, 1024), dtype=np.uint8)
    msgs = [bytes(r) for r in buf]
    res = hasher.blake2b_batch(engine, msgs)
    assert res.verified and len(res.reports) == 8
    for i in rng.integers(0, len(msgs), 64):
        assert res.digests[int(i)] == hashlib.blake2b(msgs[int(i)]).digest()


def test_chain_inputs_errors(engine):
    import torch

    import b2f

    dev = torch.device("cuda:0")
    h = torch.zeros((4, 8), dtype=torch.int64, device=dev)
    m = torch.zeros((4, 16), dtype=torch.int64, device=dev)
    t = torch.zeros((4, 2), dtype=torch.int64, device=dev)
    f = torch.zeros(4, dtype=torch.int32, device=dev)
    out = torch.empty(4 * 216, dtype=torch.uint8, device=dev)
    with pytest.raises(b2f.B2FError) as e:
        engine.chain_inputs_dev(h.data_ptr(), m.data_ptr(), t.data_ptr(), f.data_ptr(),
                                b2f._lib.MAX_ROUNDS + 1, 4, out.data_ptr())
    assert e.value.code == b2f._lib.ERR_ROUNDS
    with pytest.raises(b2f.B2FError):
        engine.chain_inputs_dev(0, m.data_ptr(), t.data_ptr(), f.data_ptr(), 12, 4, out.data_ptr())
    engine.chain_inputs_dev(h.data_ptr(), m.data_ptr(), t.data_ptr(), f.data_ptr(), 12, 0,
                            out.data_ptr())  # n = 0: nothing to do


@pytest.mark.parametrize("use_side_stream", [False, True])
def test_split_right_after_fused_without_host_sync(engine, use_side_stream):
    """run_plan once needed a host synchronize between torch's copies/allocations
    and the library's launches. Back-to-back batches on alternating paths, on the current
    stream or on a side stream, with nothing between them but stream order, must all give
    hashlib's digests."""
    import torch

    from b2f import hasher

    rng = np.random.default_rng(11)
    side = torch.cuda.Stream() if use_side_stream else None
    s = side.cuda_stream if side is not None else None
    batches = [_msgs(rng, n, L) for n, L in ((700, 2000), (400, 900), (900, 2600), (300, 400))]
    plans = [hasher.Plan(m) for m in batches]
    results = []
    for i, plan in enumerate(plans):  # fused, split, fused, split; no synchronize between
        results.append(hasher.run_plan(engine, plan, "fused" if i % 2 == 0 else "split", stream=s))
    for msgs, res in zip(batches, results):
        assert res.verified
        for m, d in zip(msgs, res.digests):
            assert d == hashlib.blake2b(m).digest(), len(m)
