"""The permutation-argument restatement (oracle/permutation.py, halo2_proofs 0.3.0 keygen +
prover) pinned by the argument's properties, and the product's keygen mapping
(b2f_permutation_mapping, host code) bit-exact against it. No GPU."""
import numpy as np
import pytest

import permutation as pm

from conftest import random_inputs


def _orc_inputs(x, orc):
    return np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()


@pytest.mark.parametrize("rounds", [0, 1, 2, 12])
def test_mapping_matches_oracle(orc, rounds):
    import b2f

    got = b2f.permutation_mapping(rounds)
    want = np.array(pm.instance_mapping(rounds, orc.copies(rounds)), dtype=np.uint32)
    assert got.shape == want.shape == (8, 228 + 416 * rounds)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("rounds", [1, 3])
def test_cycles_are_copy_classes(orc, rounds):
    """sigma is a permutation whose cycles are exactly the equivalence classes of the copy
    graph (union-find over the copies, independent of halo2's merge order)."""
    R = 228 + 416 * rounds
    m = pm.instance_mapping(rounds, orc.copies(rounds))
    nxt = [((m[j][i] >> 29) * R + (m[j][i] & ((1 << 29) - 1))) for j in range(8) for i in range(R)]
    assert sorted(nxt) == list(range(8 * R))  # a permutation
    parent = list(range(8 * R))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for dr, dc, sr, sc in orc.copies(rounds).tolist():
        parent[find((dc - 1) * R + dr)] = find((sc - 1) * R + sr)
    seen = [False] * (8 * R)
    for x in range(8 * R):
        if seen[x]:
            continue
        cyc = []
        y = x
        while not seen[y]:
            seen[y] = True
            cyc.append(y)
            y = nxt[y]
        roots = {find(c) for c in cyc}
        assert len(roots) == 1
        assert sum(1 for c in range(8 * R) if find(c) in roots) == len(cyc)


def test_domain_constants():
    """The crates' ROOT_OF_UNITY (pasta_curves 0.5.1 Fp, halo2curves 0.3.2 bn256::Fr) as
    published, and omega of order exactly 2^k; delta = g^(2^S) has order dividing t."""
    assert pm.domain(pm.P_PALLAS, 32)[0] == \
        0x2bce74deac30ebda362120830561f81aea322bf2b7bb7584bdad6fabd87ea32f
    assert pm.domain(pm.P_BN254, 28)[0] == \
        0x03ddb9f5166d18b798865ea93dd31f743215cf6dd39329c8d34f1ed960c37c9c
    for p in (pm.P_PALLAS, pm.P_BN254):
        for k in (10, 12, 17):
            w, d = pm.domain(p, k)
            assert pow(w, 1 << k, p) == 1 and pow(w, 1 << (k - 1), p) == p - 1
            g, s = pm.GEN[p]
            assert pow(d, (p - 1) >> s, p) == 1


def test_host_field_constants_match_restatement():
    from b2f import field

    for f, p in ((field.PALLAS, pm.P_PALLAS), (field.BN254, pm.P_BN254)):
        assert field.MODULUS[f] == p
        for k in (12, 20):
            assert (field.omega(f, k), field.delta(f)) == pm.domain(p, k)


@pytest.mark.parametrize("p,chunk", [(pm.P_PALLAS, 3), (pm.P_BN254, 8), (pm.P_PALLAS, 1)])
def test_z_closes_on_valid_trace_and_not_on_broken_copy(orc, p, chunk):
    x = random_inputs(3, (0, 1, 2), 81)
    adv, fixed, h_out, off = orc.fill(_orc_inputs(x, orc))
    k, usable = 12, (1 << 12) - 7
    rng = np.random.default_rng(82)
    beta, gamma = (int(rng.integers(1, 2**62)) << 180) % p, int(rng.integers(1, 2**62)) * 7
    sigma, zs = pm.columns(adv, off, k, usable, beta, gamma, chunk, p, orc.copies)
    assert len(zs) == -(-8 // chunk) and zs[0][0] == 1
    assert zs[-1][usable] == 1
    assert all(zs[c][0] == zs[c - 1][usable] for c in range(1, len(zs)))
    w, d = pm.domain(p, k)
    ident = sorted(pow(d, j, p) * pow(w, i, p) % p for j in range(8) for i in range(1 << k))
    assert sorted(v for col in sigma for v in col) == ident  # sigma permutes the identity values
    # a copied cell (the destination of the first copy) corrupted: the product no longer closes
    dr, dc, sr, sc = (int(v) for v in orc.copies(1)[5])
    bad = adv.copy()
    bad[dc, int(off[1]) + dr] ^= 1
    _, zb = pm.columns(bad, off, k, usable, beta, gamma, chunk, p, orc.copies)
    assert zb[-1][usable] != 1
