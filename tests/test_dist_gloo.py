"""Multi-process sharding path on CPU (gloo, world_size 2): shard planning, verdict
reduction and the h' all_gather reproduce the single-process batch. The per-shard compute
here is the oracle (test infrastructure); on the GPU box it is the HIP engine."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, random_inputs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, inputs_bytes, q, coalesce=None):
    import sys

    for p in (os.path.join(ROOT, "zk-odst_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import oracle
    from b2f import INPUT_DTYPE, dist as bdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = np.frombuffer(inputs_bytes, dtype=INPUT_DTYPE)
    shards = bdist.plan_shards(x, world)
    srows, sbase = bdist.shard_rows(x, shards)
    w = bdist.trace_window(srows)
    lo, hi = shards[rank]
    ox = np.frombuffer(x[lo:hi].tobytes(), dtype=oracle.INPUT_DTYPE).copy()
    adv, fixed, h_out, off = oracle.fill(ox, total_rows=w)  # the common window, zero tail
    if rank == 1:  # a corruption on one rank must show in the combined verdict
        adv[1, 5] += 1
    rep = oracle.evaluate(adv, fixed, off)
    combined = bdist.reduce_report(rep, dist, torch, "cpu", row_offset=sbase[rank])
    # the device-tensor form bench.py uses (no host round trip)
    raw = np.array([*rep["gate_failures"], rep["lookup_failures"], rep["copy_failures"],
                    rep["first_failure"], rep["rows_checked"], rep["fixed_failures"]],
                   dtype=np.uint64)
    words = bdist.all_reduce_verdict(
        bdist.verdict_words(torch.from_numpy(raw.view(np.int64)), sbase[rank], torch), dist)
    h = bdist.gather_h_out(torch.from_numpy(h_out.view(np.int64)), shards, dist, torch)
    ga, gf = bdist.gather_trace(torch.from_numpy(adv.view(np.int32)),
                                torch.from_numpy(fixed.view(np.int32)), srows, dist, torch,
                                coalesce=coalesce)
    # a refused coalescing attempt must leave the group usable: this collective runs now
    probe = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(probe)
    assert int(probe.item()) == world * (world + 1) // 2
    q.put((rank, combined, words.tolist(), h.numpy().view(np.uint64).tobytes(), shards, sbase,
           ga.numpy().view(np.uint32).tobytes(), gf.numpy().view(np.uint32).tobytes()))
    dist.destroy_process_group()


def test_plan_shards_balances_rows():
    from b2f import dist as bdist, offsets

    x = random_inputs(101, (1, 4, 12), 41)
    for world in (1, 2, 3, 8):
        sh = bdist.plan_shards(x, world)
        assert sh[0][0] == 0 and sh[-1][1] == 101
        assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        off = offsets(x)
        rows = [int(off[hi] - off[lo]) for lo, hi in sh]
        assert max(rows) - min(rows) <= 2 * 5220  # within two instances of even


@pytest.mark.parametrize("n,rounds,seed,coalesce", [(37, (0, 1, 4, 12), 42, None),
                                                    (23, (1, 4, 12), 43, None),
                                                    (23, (1, 4, 12), 44, True)])
def test_gloo_world2_matches_single_process(orc, n, rounds, seed, coalesce):
    """Unequal mixed-rounds shards: the all-gathered witness table is the single-process
    trace (total_rows = world x window), h' is the batch's, and the combined verdict equals the
    oracle's verdict on the reassembled table, first failure at its global row. coalesce=True
    forces gather_trace's RCCL-style coalesced attempt, which gloo refuses (no
    startCoalescing): the guarded fallback must gather the same table and leave the group
    usable."""
    import multiprocessing as mp

    from b2f import dist as bdist

    x = random_inputs(n, rounds, seed)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, x.tobytes(), q, coalesce))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ox = np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()
    shards = res[0][4]
    srows, _ = bdist.shard_rows(x, shards)
    assert srows[0] != srows[1], "the shards must be unequal for this test"
    total = 2 * bdist.trace_window(srows)
    adv_ref, fixed_ref, h_ref, off_ref = orc.fill(ox, total_rows=total)
    want = adv_ref.copy()
    want[1, int(off_ref[shards[1][0]]) + 5] += 1  # rank 1's corrupted cell at its global row
    want_rep = orc.evaluate(want, fixed_ref, off_ref)
    # the INW gate of that word fails on its block row, 4 rows into rank 1's shard
    assert want_rep["first_failure"] >> 8 == int(off_ref[shards[1][0]]) + 4
    for rank, combined, words, hbytes, sh, sbase, abytes, fbytes in res:
        assert np.array_equal(np.frombuffer(hbytes, dtype=np.uint64).reshape(-1, 8), h_ref)
        ga = np.frombuffer(abytes, dtype=np.uint32).reshape(10, -1)
        assert np.array_equal(ga, want)
        assert np.array_equal(np.frombuffer(fbytes, dtype=np.uint32), fixed_ref)
        assert combined == want_rep
        assert words[:16] == want_rep["gate_failures"]
        assert words[16:20] == [want_rep["lookup_failures"], want_rep["copy_failures"],
                                want_rep["fixed_failures"], want_rep["first_failure"]]
