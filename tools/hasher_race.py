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


def main():
    import torch

    import b2f
    import oracle as orc
    from b2f import hasher

    eng = b2f.Engine(0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
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
