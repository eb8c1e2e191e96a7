"""The lookup-argument restatement (oracle/lookup.py, halo2_proofs 0.3.0 lookup prover) checked
by the argument's defining properties -- halo2 itself is not buildable here, so these pin the
restatement: A' is A sorted, S' is a permutation of S, every A' row either starts a run with
S' equal to it or repeats the row above, and the grand product closes (z[usable] = 1). No GPU."""
import numpy as np
import pytest

import lookup as lk

rng = np.random.default_rng(5)


def _rows(n, zero_frac=0.3):
    x = rng.integers(0, 1 << 16, n)
    x[rng.random(n) < zero_frac] = 0
    a0 = np.array([lk.tag(int(v)) for v in x])
    a2 = np.array([lk.spread(int(v)) for v in x])
    return a0, x, a2


def _chal(p=lk.P):
    return [int(rng.integers(0, 2**63)) * 2**190 % p + int(rng.integers(1, 2**63))
            for _ in range(3)]


@pytest.mark.parametrize("usable,p", [(1 << 16, lk.P), ((1 << 16) + 777, lk.P),
                                      ((1 << 16) + 333, lk.P_BN254)])
def test_permutation_properties(usable, p):
    a0, a1, a2 = _rows(usable)
    theta, beta, gamma = _chal(p)
    A, S, Ap, Sp, z = lk.columns(a0, a1, a2, usable, theta, beta, gamma, p)
    assert Ap == sorted(A)
    assert sorted(Sp) == sorted(S)
    assert Ap[0] == Sp[0]
    for i in range(1, usable):
        assert Ap[i] == Sp[i] or Ap[i] == Ap[i - 1], i
    assert len(z) == usable + 1 and z[0] == 1 and z[-1] == 1
    assert A[5] == lk.compress(theta, int(a0[5]), int(a1[5]), int(a2[5]), p)
    assert S[0] == 0 and all(v == 0 for v in S[1 << 16:])
    # halo2 hands leftovers out ascending, each to the last open repeated row: the leftover
    # values sit on repeated rows in descending order
    rep = [i for i in range(1, usable) if Ap[i] == Ap[i - 1]]
    vals = [Sp[i] for i in rep]
    assert vals == sorted(vals, reverse=True)


def test_rejects_non_table_rows():
    a0, a1, a2 = _rows(1 << 16)
    a2 = a2.copy()
    a2[1234] ^= 4
    assert lk.first_bad_row(a0, a1, a2) == 1234
    with pytest.raises(ValueError):
        lk.columns(a0, a1, a2, 1 << 16, *_chal())
    a1b = a1.copy()
    a1b[99] = 1 << 16
    assert lk.first_bad_row(a0, a1b, a2) == 99


def test_batch_invert():
    vals = [int(v) + 1 for v in rng.integers(0, 2**62, 50)]
    inv = lk.batch_invert(vals)
    assert all(v * w % lk.P == 1 for v, w in zip(vals, inv))


@pytest.mark.parametrize("p", [lk.P, lk.P_BN254])
def test_den_total_equals_num_total(p):
    """The identity the GPU's lk_dtot_kernel rests on (lookup columns): A' is a
    permutation of A and S' one of S, so prod_p (A'_p + beta)(S'_p + gamma) = prod_p (A_p + beta)
    * prod_p (S_p + gamma) -- the grand product's den total is known from the rows and the table
    alone, before any permuted column exists. Also z[p + 1] = N_p / D_p with that D."""
    usable = (1 << 16) + 501
    a0, a1, a2 = _rows(usable, zero_frac=0.5)
    theta, beta, gamma = _chal(p)
    A, S, Ap, Sp, z = lk.columns(a0, a1, a2, usable, theta, beta, gamma, p)
    den = num_a = num_s = 1
    for i in range(usable):
        den = den * (Ap[i] + beta) % p * (Sp[i] + gamma) % p
        num_a = num_a * (A[i] + beta) % p
        num_s = num_s * (S[i] + gamma) % p
    assert den == num_a * num_s % p
    # the S part is the same for every circuit: the table once, then row 0's value
    tv = lk.table_values(theta, p)
    s_part = 1
    for x in range(1 << 16):
        s_part = s_part * (tv[x] + gamma) % p
    s_part = s_part * pow(tv[0] + gamma, usable - (1 << 16), p) % p
    assert s_part == num_s
