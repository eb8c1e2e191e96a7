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


def _worker(rank, world, port, inputs_bytes, q):
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
    lo, hi = shards[rank]
    ox = np.frombuffer(x[lo:hi].tobytes(), dtype=oracle.INPUT_DTYPE).copy()
    adv, fixed, h_out, off = oracle.fill(ox)
    if rank == 1:  # a corruption on one rank must show in the combined verdict
        adv[1, 5] += 1
    rep = oracle.evaluate(adv, fixed, off)
    combined = bdist.reduce_report(rep, dist, torch, "cpu")
    h = bdist.gather_h_out(torch.from_numpy(h_out.view(np.int64)), shards, dist, torch)
    srows = [int(bdist.offsets(x[a:b])[-1]) for a, b in shards]
    ga, gf = bdist.gather_trace(torch.from_numpy(adv.view(np.int32)),
                                torch.from_numpy(fixed.view(np.int32)), srows, dist, torch)
    q.put((rank, combined, h.numpy().view(np.uint64).tobytes(), shards,
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


def test_gloo_world2_matches_single_process(orc):
    import multiprocessing as mp

    x = random_inputs(37, (0, 1, 4, 12), 42)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, x.tobytes(), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ox = np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()
    adv_ref, fixed_ref, h_ref, off_ref = orc.fill(ox)
    adv_ref = adv_ref.copy()
    for rank, combined, hbytes, shards, abytes, fbytes in res:
        assert np.array_equal(np.frombuffer(hbytes, dtype=np.uint64).reshape(-1, 8), h_ref)
        # the reassembled witness table is the single-process trace (with rank 1's corrupted
        # cell at its global row)
        ga = np.frombuffer(abytes, dtype=np.uint32).reshape(10, -1)
        want = adv_ref.copy()
        want[1, int(off_ref[shards[1][0]]) + 5] += 1
        assert np.array_equal(ga, want)
        assert np.array_equal(np.frombuffer(fbytes, dtype=np.uint32), fixed_ref)
        assert combined["lookup_failures"] >= 1 and combined["first_failure"] != 2**64 - 1
        assert combined["rows_checked"] == int(orc.offsets(ox)[-1])
