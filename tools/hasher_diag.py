import sys, hashlib, numpy as np
sys.path.insert(0, "zk-odst_amd")
import torch, b2f
from b2f import hasher
eng = b2f.Engine(0)
def _msgs(rng, n, maxlen):
    return [rng.integers(0, 256, int(rng.integers(0, maxlen)), dtype=np.uint8).tobytes() for _ in range(n)]
for key, ds in [(b"", 64), (b"secret key", 32), (bytes(64), 7)]:
    for path in ["split", "fused"]:
        rng = np.random.default_rng(ds + len(key))
        msgs = _msgs(rng, 300, 1200)
        for rep in range(2):
            res = hasher.blake2b_batch(eng, msgs, ds, key, path=path)
            bad = [i for i, (m, d) in enumerate(zip(msgs, res.digests)) if d != hashlib.blake2b(m, digest_size=ds, key=key).digest()]
            print(len(key), ds, path, rep, "verified", res.verified, "bad", len(bad), bad[:5], flush=True)
