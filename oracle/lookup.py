"""CPU restatement of the lookup argument's prover columns for the spread lookup.

TEST INFRASTRUCTURE ONLY: tests/ use this as the checker for b2f_lookup_columns_dev
(SURVEY.md §8(f) rank 4); nothing in the product path imports it.

The algorithm lives in third-party crates that are not in /root/reference:
halo2_proofs 0.3.0 (crates.io, /root/reference/Cargo.lock:841-855) and its field
pasta_curves 0.5.1 (Cargo.lock:1334-1337). Restated from their published source:

* `Argument::commit_permuted` (halo2_proofs src/plonk/lookup/prover.rs): each side's
  expressions are compressed with the challenge theta as `fold(0, |acc, e| acc * theta + e)`
  over the lookup's expression list. For this chip the list is (tag, dense, spread)
  (spread_table.rs:443-453), so a row compresses to theta^2 tag + theta dense + spread.
* The table side is the three table columns over the usable rows: the 2^16 rows written by
  `SpreadTableChip::load` (spread_table.rs:470-508, values from `generate`, :574-600), then
  the layouter's `fill_from_row` default (the value at row 0, i.e. (0, 0, 0)) up to the last
  usable row.
* `permute_expression_pair` (same file): sort the compressed inputs (pasta's `Ord` on Fp is
  the order of canonical integers); count the compressed table values in a BTreeMap; at the
  first row of each run of equal inputs put that value into the permuted table column and
  take one from its count; give the remaining table values, in ascending order, to the
  repeated-input rows, each to the LAST row still open (`repeated_input_rows.pop()`).
* Fields: pasta Fp (halo2_proofs' own) and BN254 Fr (halo2curves 0.3.2 bn256::Fr,
  Cargo.lock:859-861, the reference circuit's field, blake2f.rs:283,293); `Ord` on both is
  the order of canonical integers. Every function takes the modulus `p` (default pasta).
* `Permuted::commit_product`: z[0] = 1, z[i + 1] = z[i] (A[i] + beta)(S[i] + gamma) /
  ((A'[i] + beta)(S'[i] + gamma)) over the usable rows, so z has usable + 1 known entries
  and z[usable] = 1 for a valid lookup.

Blinding rows (random) are the prover's and not restated. Parity against halo2 itself is
unpinned (halo2 cannot be built here); the tests pin this restatement by the argument's
defining properties and pin the GPU path to this restatement bit for bit.
"""
P = 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001
P_BN254 = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
TABLE_ROWS = 1 << 16


def spread(x):
    s = 0
    for b in range(16):
        if (x >> b) & 1:
            s |= 1 << (2 * b)
    return s


def tag(x):
    # get_tag thresholds as generate() increments the tag (spread_table.rs:213-222, :583-586)
    return 0 if x < (1 << 8) else (1 if x < (1 << 15) else 2)


def compress(theta, t, d, s, p=P):
    acc = 0
    for e in (t, d, s):
        acc = (acc * theta + e) % p
    return acc


def table_values(theta, p=P):
    """Compressed table value of every dense x < 2^16 (the table row x)."""
    th2 = theta * theta % p
    return [(th2 * tag(x) + theta * x + spread(x)) % p for x in range(TABLE_ROWS)]


def batch_invert(vals, p=P):
    pre = []
    acc = 1
    for v in vals:
        acc = acc * v % p
        pre.append(acc)
    inv = pow(acc, p - 2, p)
    out = [0] * len(vals)
    for i in range(len(vals) - 1, -1, -1):
        out[i] = inv * (pre[i - 1] if i else 1) % p
        inv = inv * vals[i] % p
    return out


def columns(a0, a1, a2, usable, theta, beta, gamma, p=P):
    """The five prover columns over `usable` rows whose lookup inputs are a0/a1/a2 (sequences
    of row values, length `usable`): (A, S, A', S', z) as lists of canonical integers, z with
    usable + 1 entries. Raises ValueError at the first input row not in the table."""
    if usable < TABLE_ROWS:
        raise ValueError("usable rows %d < table size" % usable)
    P = p  # noqa: N806 (the field of this call)
    A = [compress(theta, int(a0[i]), int(a1[i]), int(a2[i]), P) for i in range(usable)]
    T = table_values(theta, P)
    S = T + [T[0]] * (usable - TABLE_ROWS)
    # permute_expression_pair
    Ap = sorted(A)
    leftover = {}
    for v in S:
        leftover[v] = leftover.get(v, 0) + 1
    Sp = [0] * usable
    repeated = []
    for row, v in enumerate(Ap):
        if row == 0 or v != Ap[row - 1]:
            Sp[row] = v
            if leftover.get(v, 0) == 0:
                raise ValueError("input value %#x not in the table" % v)
            leftover[v] -= 1
        else:
            repeated.append(row)
    for v in sorted(leftover):
        for _ in range(leftover[v]):
            Sp[repeated.pop()] = v
    assert not repeated
    # commit_product
    den = [(Ap[i] + beta) * (Sp[i] + gamma) % P for i in range(usable)]
    inv = batch_invert(den, P)
    z = [1]
    for i in range(usable):
        z.append(z[-1] * inv[i] % P * ((A[i] + beta) % P) % P * ((S[i] + gamma) % P) % P)
    return A, S, Ap, Sp, z


def first_bad_row(a0, a1, a2):
    """Index of the first row whose (tag, dense, spread) is not a table row, or None."""
    for i in range(len(a1)):
        x = int(a1[i])
        if x >= TABLE_ROWS or int(a0[i]) != tag(x) or int(a2[i]) != spread(x):
            return i
    return None


def to_limbs(v):
    return [(v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)]


def to_mont(v, p=P):
    return v * (1 << 256) % p
