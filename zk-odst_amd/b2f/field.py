"""Host-side constants of the two prover fields (the values a halo2 prover passes to
b2f_lookup_columns_dev / b2f_permutation_columns_dev as plain integers).

pasta_curves 0.5.1 Fp (halo2_proofs 0.3.0's field) and halo2curves 0.3.2 bn256::Fr (the
reference circuit's field, blake2f.rs:283,293): p - 1 = t 2^S with t odd, a multiplicative
generator g; ROOT_OF_UNITY = g^t (a primitive 2^S-th root of unity), DELTA = g^(2^S) (the
coset shift of the permutation argument's identity columns), and the 2^k-row domain's
generator is ROOT_OF_UNITY squared S - k times (halo2 EvaluationDomain::new).
"""
from . import _lib

PALLAS, BN254 = 0, 1
MODULUS = {PALLAS: 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001,
           BN254: 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001}
GENERATOR = {PALLAS: 5, BN254: 7}
S = {PALLAS: 32, BN254: 28}


def of_form(form):
    """The field a B2F_FP_* form selects."""
    return BN254 if int(form) & 2 else PALLAS


def root_of_unity(field):
    p = MODULUS[field]
    return pow(GENERATOR[field], (p - 1) >> S[field], p)


def delta(field):
    p = MODULUS[field]
    return pow(GENERATOR[field], 1 << S[field], p)


def omega(field, k):
    """Generator of the 2^k-row evaluation domain."""
    if not 0 <= k <= S[field]:
        raise _lib.B2FError(_lib.ERR_ARG, "k = %d exceeds the field's 2-adicity" % k)
    p = MODULUS[field]
    return pow(root_of_unity(field), 1 << (S[field] - k), p)


def limbs(v):
    """A field element as the 4 little-endian u64 limbs the ABI takes."""
    return [(int(v) >> (64 * i)) & (2**64 - 1) for i in range(4)]
