"""Diagnostics for the hasher's stream-order race: run the hashlib-test batches
(split and fused, three key configurations) many times in one process, with and without a
host synchronize after the block upload, and for every wrong digest find the first block step
whose h' differs from a CPU recomputation (oracle.compress) -- which says whether the device
read stale blocks / h0 (step 0 wrong) or a later input. Prints one line per case."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def msgs_for(rng, n, max_len):
    lens = rng.integers(0, max_len, n)
    lens[:6] = [0, 1, 127, 128, 129, 256]
    return [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]


def first_bad_step(plan, all_h, pos, orc):
    h = plan.h0.copy()
    for j in range(plan.steps):
        if pos >= plan.active[j]:
            break
        r = int(plan.start[j]) + pos
        want = orc.compress(12, h, plan.blocks[r], plan.t[r], int(plan.f[r]))
        if not np.array_equal(all_h[r], want):
            return j, int(plan.active[j])
        h = want
    return None, None


def input_diff(plan, res, orc, pos, j):
    """Which fields of step j's input record for sorted position pos differ from the CPU's."""
    r = int(plan.start[j]) + pos
    got = np.frombuffer(res.all_inputs[216 * r:216 * (r + 1)].tobytes(), dtype=orc.INPUT_DTYPE)[0]
    h = plan.h0.copy()
    for k in range(j):
        rr = int(plan.start[k]) + pos
        h = orc.compress(12, h, plan.blocks[rr], plan.t[rr], int(plan.f[rr]))
    bad = []
    if not np.array_equal(got["h"], h):
        bad.append("h(%d words)" % int((got["h"] != h).sum()))
    if not np.array_equal(got["m"], plan.blocks[r]):
        bad.append("m(%d words)" % int((got["m"] != plan.blocks[r]).sum()))
    if not np.array_equal(got["t"], plan.t[r]):
        bad.append("t")
    if int(got["f"]) != int(plan.f[r]) or int(got["rounds"]) != 12:
        bad.append("f/rounds")
    return bad or ["inputs ok: the compression itself is wrong"]


def big_case(eng, hasher, orc, reps):
    """test_many_equal_messages' shape: 2^14 messages of 1 KiB, 8 block steps."""
    import hashlib as hl
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, (1 << 14, 1024), dtype=np.uint8)
    msgs = [bytes(r) for r in buf]
    variants = [("torch", False), ("torch", "stream"), ("torch", True), ("hip", False),
                ("blocking", False)]
    for how, sync in variants:
        nb = 0
        for rep in range(reps):
            plan = hasher.Plan(msgs)
            res = hasher.run_plan(eng, plan, "fused",
                                  _diag={"sync_upload": sync, "keep_inputs": True, "upload": how})
            bad = [i for i in range(len(msgs)) if res.digests[i] != hl.blake2b(msgs[i]).digest()]
            nb += len(bad)
            if bad:
                pos = [int(np.nonzero(plan.order == i)[0][0]) for i in bad[:3]]
                steps = [first_bad_step(plan, res.all_h, p, orc) for p in pos]
                why = [input_diff(plan, res, orc, p, st[0]) for p, st in zip(pos, steps)
                       if st[0] is not None]
                print("big upload=%s sync=%s rep=%d stream=%#x: %d bad, pos %s, first bad %s, %s"
                      % (how, sync, rep, res.stream, len(bad), pos, steps, why), flush=True)
        print("big upload=%s sync=%s total bad digests %d" % (how, sync, nb), flush=True)


def main():
    import torch

    import b2f
    import oracle as orc
    from b2f import hasher

    eng = b2f.Engine(0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    big_case(eng, hasher, orc, reps)
    if os.environ.get("B2F_RACE_BIG_ONLY"):
        return
    for sync in (False, True):
        nbad_total = 0
        for rep in range(reps):
            for path in ("split", "fused"):
                for key, ds in ((b"", 64), (b"secret key", 32), (bytes(64), 7)):
                    rng = np.random.default_rng(ds + len(key))
                    msgs = msgs_for(rng, 300, 1200)
                    plan = hasher.Plan(msgs, ds, key)
                    res = hasher.run_plan(eng, plan, path, _diag={"sync_upload": sync})
                    bad = [i for i, (m, d) in enumerate(zip(msgs, res.digests))
                           if d != hashlib.blake2b(m, digest_size=ds, key=key).digest()]
                    nbad_total += len(bad)
                    if bad:
                        pos = [int(np.nonzero(plan.order == i)[0][0]) for i in bad[:4]]
                        steps = [first_bad_step(plan, res.all_h, p, orc) for p in pos]
                        print("sync=%d rep=%d %s key=%d ds=%d: %d bad, sorted pos %s, first bad "
                              "(step, active) %s, steps %d" % (sync, rep, path, len(key), ds,
                                                               len(bad), pos, steps, plan.steps),
                              flush=True)
        print("sync=%d total bad digests %d" % (sync, nbad_total), flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
