"""CPU restatement of the permutation argument's prover columns for the equality columns.

TEST INFRASTRUCTURE ONLY: tests/ use this as the checker for b2f_permutation_mapping and
b2f_permutation_columns_dev (the widening of SURVEY.md §8(f) row 2);
nothing in the product path imports it. Pure-Python big integers: small circuits only.

The algorithm lives in halo2_proofs 0.3.0 (crates.io, /root/reference/Cargo.lock:841-855),
which is not in /root/reference; restated from its published source:

* Columns: the permutation argument's columns in `enable_equality` order, here
  [a_1 .. a_8] (table16.rs:312-314); column j is a_{j+1}.
* keygen.rs `Assembly`: mapping[j][i] = aux[j][i] = (j, i), sizes all 1. `copy(left, right)`:
  if aux[left] == aux[right] nothing; otherwise the larger cycle (by sizes of the
  representatives; ties keep left) absorbs the other: sizes add, every cell of the absorbed
  cycle gets aux = the absorbing representative (walking mapping from the absorbed
  representative back to itself), then mapping[left] and mapping[right] swap.
  The copies are the instance's copy constraints in synthesis order (oracle's own
  restatement, b2f_oracle.c orc_copies), each `copy_advice` calling
  constrain_equal(new cell, source) = copy(left = destination, right = source).
* build_pk: sigma_j(w^i) = delta^c' w^r' with (c', r') = mapping[j][i]; the identity column
  j is delta^j w^i. delta = F::DELTA = g^(2^S), w the 2^k-th root of unity (ROOT_OF_UNITY =
  g^t squared S - k times); pasta Fp g = 5, S = 32; BN254 Fr (halo2curves 0.3.2) g = 7,
  S = 28.
* prover.rs `commit`: for each chunk of chunk_len = cs.degree() - 2 columns,
  modified[i] = prod_j (v_j(i) + beta sigma_j(w^i) + gamma), batch-inverted, times
  prod_j (v_j(i) + beta delta^j w^i + gamma) (delta^j running over all columns, across
  chunks); z[0] = last_z (1 for the first chunk), z[i] = z[i - 1] modified[i - 1]; the last
  blinding_factors rows are random and last_z = z[n - blinding_factors - 1] = z[usable].
  Only rows i <= usable are restated (they depend on rows < usable alone).

Parity against halo2 itself is unpinned (halo2 cannot be built here): the tests pin this
restatement by the argument's properties (sigma is a permutation of the identity values whose
cycles are exactly the copy classes; z closes to 1 on a valid trace and not on a broken
copy) and the GPU path to this restatement bit for bit.
"""
P_PALLAS = 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001
P_BN254 = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
GEN = {P_PALLAS: (5, 32), P_BN254: (7, 28)}
NCOL = 8


def domain(p, k):
    """(omega of the 2^k-row domain, delta) by the crates' definitions."""
    g, s = GEN[p]
    t = (p - 1) >> s
    root = pow(g, t, p)
    omega = root
    for _ in range(s - k):
        omega = omega * omega % p
    return omega, pow(g, 1 << s, p)


class Assembly:
    """keygen.rs Assembly over NCOL columns x n rows; cells are j * n + i."""

    def __init__(self, n):
        self.n = n
        self.mapping = list(range(NCOL * n))
        self.aux = list(range(NCOL * n))
        self.sizes = [1] * (NCOL * n)

    def copy(self, lc, lr, rc, rr):
        left, right = lc * self.n + lr, rc * self.n + rr
        lcyc, rcyc = self.aux[left], self.aux[right]
        if lcyc == rcyc:
            return
        if self.sizes[lcyc] < self.sizes[rcyc]:
            lcyc, rcyc = rcyc, lcyc
        self.sizes[lcyc] += self.sizes[rcyc]
        i = rcyc
        while True:
            self.aux[i] = lcyc
            i = self.mapping[i]
            if i == rcyc:
                break
        self.mapping[left], self.mapping[right] = self.mapping[right], self.mapping[left]


def instance_mapping(rounds, copies):
    """Mapping of one instance (copies: the oracle's [count, 4] list): [8][R] entries
    (c' << 29) | r' -- the layout b2f_permutation_mapping returns."""
    R = 228 + 416 * rounds
    a = Assembly(R)
    for dr, dc, sr, sc in copies.tolist():
        assert 1 <= dc <= 8 and 1 <= sc <= 8
        a.copy(dc - 1, dr, sc - 1, sr)
    return [[((a.mapping[j * R + i] // R) << 29) | (a.mapping[j * R + i] % R) for i in range(R)]
            for j in range(NCOL)]


def circuit_mapping(offsets, copies_of):
    """The whole circuit's Assembly after every instance's copies (instances in order;
    offsets relative to the circuit, copies_of(rounds) the oracle's list)."""
    n = int(offsets[-1])
    a = Assembly(max(n, 1))
    for i in range(len(offsets) - 1):
        s = int(offsets[i])
        rounds = (int(offsets[i + 1]) - s - 228) // 416
        for dr, dc, sr, sc in copies_of(rounds).tolist():
            a.copy(dc - 1, s + dr, sc - 1, s + sr)
    return a


def columns(adv, offsets, k, usable, beta, gamma, chunk_len, p, copies_of):
    """adv: advice [10, >= used] (the circuit's rows from 0), offsets: circuit row map.
    Returns (sigma [8][2^k] canonical ints, z: list over column sets of usable + 1 ints)."""
    n_rows = 1 << k
    used = int(offsets[-1])
    omega, delta = domain(p, k)
    a = circuit_mapping(offsets, copies_of)
    wp = [1] * n_rows
    for i in range(1, n_rows):
        wp[i] = wp[i - 1] * omega % p
    dp = [pow(delta, j, p) for j in range(NCOL)]

    def sig(j, i):
        if i >= used:
            return dp[j] * wp[i] % p
        m = a.mapping[j * a.n + i]
        return dp[m // a.n] * wp[m % a.n] % p

    sigma = [[sig(j, i) for i in range(n_rows)] for j in range(NCOL)]

    def v(j, i):
        return int(adv[j + 1][i]) if i < used else 0

    zs = []
    last = 1
    for j0 in range(0, NCOL, chunk_len):
        cols = range(j0, min(j0 + chunk_len, NCOL))
        den = [1] * usable
        num = [1] * usable
        for i in range(usable):
            for j in cols:
                den[i] = den[i] * (v(j, i) + beta * sigma[j][i] + gamma) % p
                num[i] = num[i] * (v(j, i) + beta * dp[j] * wp[i] + gamma) % p
        inv = _batch_invert(den, p)
        z = [last]
        for i in range(usable):
            z.append(z[-1] * inv[i] % p * num[i] % p)
        zs.append(z)
        last = z[usable]
    return sigma, zs


def _batch_invert(vals, p):
    pre, acc = [], 1
    for x in vals:
        acc = acc * x % p
        pre.append(acc)
    inv = pow(acc, p - 2, p)
    out = [0] * len(vals)
    for i in range(len(vals) - 1, -1, -1):
        out[i] = inv * (pre[i - 1] if i else 1) % p
        inv = inv * vals[i] % p
    return out
