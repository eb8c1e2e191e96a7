"""The CPU oracle against the golden vectors (pinning it), and its own verdict logic.

CPU only. The oracle is test infrastructure (oracle/b2f_oracle.h)."""
import numpy as np
import pytest

from conftest import ROOT, random_inputs, words


def _orc_inputs(x, orc):
    return np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()


def test_reference_kat(orc, golden):
    """blake2f.rs:193-247: rounds 12, "abc" -> ba80a53f..."""
    k = golden["kat"]
    out = orc.compress(k["rounds"], words(k["h"]), words(k["m"]), words(k["t"]), k["f"])
    assert out.astype("<u8").tobytes().hex() == k["expected"]


def test_rounds0_vectors(orc, golden):
    for c in golden["rounds0"]:
        out = orc.compress(0, words(c["h"]), words(c["m"]), words(c["t"]), c["f"])
        assert out.astype("<u8").tobytes().hex() == c["expected"], c["name"]


def test_hashlib_chains(orc, golden):
    for c in golden["hash_cases"]:
        h = words(c["h"])
        for blk in c["chain"]:
            h = orc.compress(blk["rounds"], h, words(blk["m"]), words(blk["t"]), blk["f"])
        assert h.astype("<u8").tobytes()[: c["digest_size"]].hex() == c["digest"], c["name"]


def test_fill_h_out_equals_compress(orc):
    x = random_inputs(40, (0, 1, 2, 4, 10, 11, 12, 13), 11)
    ox = _orc_inputs(x, orc)
    adv, fixed, h_out, off = orc.fill(ox)
    for i in range(len(x)):
        ref = orc.compress(int(x["rounds"][i]), x["h"][i], x["m"][i], x["t"][i], int(x["f"][i]))
        assert np.array_equal(h_out[i], ref)
    # the digest cells (a_7, a_8 of each final XOR3 block) hold h' as u32 halves
    for i in range(len(x)):
        fb = int(off[i]) + 164 + 416 * int(x["rounds"][i])
        for w in range(8):
            lo, hi = int(adv[7, fb + 8 * w]), int(adv[8, fb + 8 * w])
            assert lo | (hi << 32) == int(h_out[i][w])


def test_row_and_copy_counts(orc):
    for r in (0, 1, 4, 12, 25):
        assert orc.rows(r) == 228 + 416 * r
        assert len(orc.copies(r)) == 24 + 576 * r + 96
    cp = orc.copies(2)
    # every copy pair: destination is an operand column, source precedes it
    assert set(cp[:, 1]) <= {3, 4, 5}
    assert np.all(cp[:, 2] < cp[:, 0])
    assert len({(int(a), int(b)) for a, b, _, _ in cp}) == len(cp)  # one source per cell


def test_clean_trace_and_tail(orc):
    x = random_inputs(10, (0, 1, 3), 12)
    ox = _orc_inputs(x, orc)
    adv, fixed, h_out, off = orc.fill(ox, total_rows=int(orc.offsets(ox)[-1]) + 8)
    assert not adv[:, -8:].any() and not fixed[-8:].any()
    rep = orc.evaluate(adv, fixed, off)
    assert rep["first_failure"] == 2**64 - 1 and rep["rows_checked"] == adv.shape[1]


def test_every_used_cell_is_constrained(orc):
    """Flipping any non-zero cell of a one-round instance is flagged; the only cells that
    are never flagged are the ones the layout leaves at 0."""
    x = random_inputs(1, (1,), 13)
    adv, fixed, h_out, off = orc.fill(_orc_inputs(x, orc))
    for c in range(10):
        for r in range(adv.shape[1]):
            if adv[c, r] == 0:
                continue
            a2 = adv.copy()
            a2[c, r] ^= 1
            assert orc.evaluate(a2, fixed, off, nthreads=1)["first_failure"] != 2**64 - 1, (c, r)


@pytest.mark.parametrize("col,row,code", [
    (9, 164, 3),        # carry of the first a1 ADD3 -> s_spread_a1
    (1, 0, 16),         # h_0 limb 0 dense -> lookup (reported before s_decompose_abcd, same row)
    (3, 168, 17),       # d1 operand spread(d_0) -> copy
    (7, 0, 0),          # input binding cell -> s_decompose_abcd
])
def test_first_failure_codes(orc, col, row, code):
    x = random_inputs(1, (1,), 14)
    adv, fixed, h_out, off = orc.fill(_orc_inputs(x, orc))
    adv[col, row] += 1
    rep = orc.evaluate(adv, fixed, off)
    first = rep["first_failure"]
    assert first >> 8 <= row
    codes_at_row = first & 0xff
    if code < 16:
        assert rep["gate_failures"][code] >= 1
    elif code == 16:
        assert rep["lookup_failures"] >= 1
    else:
        assert rep["copy_failures"] >= 1
    assert codes_at_row in range(18)


def test_spread_table_rows(orc, golden):
    """The reference's spread-table fixture rows (spread_table.rs:684-724) are table rows;
    perturbing tag, dense or spread makes them non-members."""
    rows = np.array(golden["spread_rows"], dtype=np.uint32)
    n = (len(rows) + 3) & ~3
    adv = np.zeros((10, n), dtype=np.uint32)
    adv[0, :len(rows)], adv[1, :len(rows)], adv[2, :len(rows)] = rows.T
    fixed = np.zeros(n, dtype=np.uint32)
    off = np.zeros(1, dtype=np.uint64)
    assert orc.evaluate(adv, fixed, off)["lookup_failures"] == 0
    for col in (0, 1, 2):
        bad = adv.copy()
        bad[col, 3] += 1
        assert orc.evaluate(bad, fixed, off)["lookup_failures"] == 1
    bad = adv.copy()
    bad[1, 0] = 1 << 16  # dense outside the table
    assert orc.evaluate(bad, fixed, off)["lookup_failures"] == 1


def test_bad_offsets_rejected(orc):
    x = random_inputs(3, (1,), 15)
    adv, fixed, h_out, off = orc.fill(_orc_inputs(x, orc))
    off2 = off.copy()
    off2[1] += 4
    with pytest.raises(ValueError):
        orc.evaluate(adv, fixed, off2)


P_PALLAS = 0x40000000000000000000000000000000224698fc094cf91b992d30ed00000001  # pasta Fp modulus
# BN254 scalar field modulus r (halo2curves 0.3.2 bn256::Fr, the reference's circuit field:
# blake2f.rs:283,293, blake2f_circuit_bench.rs:10): the group order of alt_bn128 (EIP-196)
R_BN254 = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def _limbs_to_int(v):
    return sum(int(v[i]) << (64 * i) for i in range(4))


def test_fp_montgomery_vs_bigint(orc):
    """Fp export restatement pinned to the definition
    mont(x) = x * 2^256 mod p, with p the pallas base modulus."""
    rng = np.random.default_rng(21)
    xs = [0, 1, 2, 3, 255, 256, 0x7fff, 0xffff, 0x55555555, 0xaaaaaaaa, 0xfffffffe, 0xffffffff]
    xs += [int(v) for v in rng.integers(0, 2**32, 2000, dtype=np.uint64)]
    for x in xs:
        assert _limbs_to_int(orc.fp_mont(x)) == (x << 256) % P_PALLAS, x
    # mont(1) is pasta's R = 2^256 mod p
    assert _limbs_to_int(orc.fp_mont(1)) == 0x3fffffffffffffffffffffffffffffff992c350be41914ad34786d38fffffffd


def test_fp_bn254_montgomery_vs_bigint(orc):
    """the BN254 Fr form pinned to mont(x) = x * 2^256 mod r, r the
    alt_bn128 group order (decimal, as EIP-196 publishes it)."""
    assert orc.MODULI[orc.BN254] == R_BN254
    rng = np.random.default_rng(26)
    xs = [0, 1, 2, 3, 255, 256, 0x7fff, 0xffff, 0x55555555, 0xaaaaaaaa, 0xfffffffe, 0xffffffff]
    xs += [int(v) for v in rng.integers(0, 2**32, 2000, dtype=np.uint64)]
    for x in xs:
        assert _limbs_to_int(orc.fp_mont(x, orc.BN254)) == (x << 256) % R_BN254, x
    # mont(1) = R mod r: halo2curves' bn256::Fr one() in memory
    assert _limbs_to_int(orc.fp_mont(1, orc.BN254)) == \
        0x0e0a77c19a07df2f666ea36f7879462e36fc76959f60cd29ac96341c4ffffffb


def test_fp_export_layout(orc):
    x = random_inputs(3, (1, 2), 22)
    adv, fixed, h_out, off = orc.fill(_orc_inputs(x, orc))
    order = [5, 3, 4, 6, 7, 8, 9, 0, 1, 2]  # halo2 column h -> a_i (table16.rs:281-294)
    can = orc.export_fp(adv, form=orc.FP_CANONICAL)
    for h, a in enumerate(order):
        assert np.array_equal(can[h, :, 0], adv[a].astype(np.uint64))
        assert not can[h, :, 1:].any()
    r0, nr = 37, 501
    mont = orc.export_fp(adv, row_begin=r0, nrows=nr, form=orc.FP_MONTGOMERY, out_rows=nr + 3)
    assert not mont[:, nr:].any()
    rng = np.random.default_rng(23)
    for h, a in enumerate(order):
        for r in rng.integers(0, nr, 40):
            v = int(adv[a, r0 + r])
            assert _limbs_to_int(mont[h, r]) == (v << 256) % P_PALLAS
    bn = orc.export_fp(adv, row_begin=r0, nrows=nr, form=orc.FP_BN254_MONTGOMERY)
    bc = orc.export_fp(adv, row_begin=r0, nrows=nr, form=orc.FP_BN254_CANONICAL)
    assert np.array_equal(bc, can[:, r0:r0 + nr])
    for h, a in enumerate(order):
        for r in rng.integers(0, nr, 40):
            v = int(adv[a, r0 + r])
            assert _limbs_to_int(bn[h, r]) == (v << 256) % R_BN254


def test_keygen_fixed_structure_equals_fill(orc):
    """The fixed column from the row map alone (keygen) is the fill's fixed column."""
    x = random_inputs(9, (0, 1, 4, 12), 61)
    ox = np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()
    adv, fixed, _, off = orc.fill(ox, total_rows=int(orc.offsets(ox)[-1]) + 40)
    assert np.array_equal(orc.fixed_structure(off, total_rows=fixed.shape[0]), fixed)


@pytest.mark.parametrize("kind,row,delta", [
    (1, 164 + 416 * 1 + 52 * 3 + 0, 1 << 40),       # an a1 add, round 1, G 3
    (1, 164 + 416 * 3 + 52 * 7 + 28, 12345),        # the last a2 add of the last round
    (1, 164 + 416 * 0 + 52 * 0 + 12, 1),            # a c1 add (ADD2)
    (2, 108 + 4 * 5, 0x0000_0001_0000_0000),        # IV5 (feeds v13 = IV5 ^ t1)
    (2, 108 + 4 * 0, 0xffff),                       # IV0 (v8)
])
def test_tampered_trace_caught_only_by_the_fixed_check(orc, kind, row, delta):
    """a trace whose advice is consistent with an altered fixed column (a
    cleared ADD selector with a wrong sum propagated downstream, or a wrong IV constant in both
    the advice and k_0) passes every gate, lookup and copy constraint; only the check of the
    fixed column against the keygen structure flags it."""
    x = random_inputs(3, (4,), 62)
    ox = np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()
    adv, fixed, h_out, off = orc.fill_tampered(ox, 1, kind, row, delta)
    _, good_fixed, good_h, _ = orc.fill(ox)
    assert not np.array_equal(h_out[1], good_h[1])  # the compression output is wrong
    rep = orc.evaluate(adv, fixed, off)
    assert sum(rep["gate_failures"]) == rep["lookup_failures"] == rep["copy_failures"] == 0
    bad_rows = np.nonzero(fixed != good_fixed)[0]
    assert rep["fixed_failures"] == len(bad_rows) >= 1
    assert rep["first_failure"] == (int(bad_rows[0]) << 8) | orc.CODE_FIXED
    assert int(off[1]) + row <= int(bad_rows[0]) < int(off[1]) + row + 4  # the altered block


def test_oracle_under_host_sanitizers():
    """The oracle's every entry point under AddressSanitizer + UndefinedBehaviorSanitizer
    (`make -C oracle asan`, driver oracle/asan_check.c): mixed rounds, a padded tail, single-cell
    corruptions, a tampered fill, the Fp export. Host code only (GPU sanitizers are not available
    on the pool). Found and fixed: a left shift of a negative 128-bit sum in the ADD gates."""
    import os
    import shutil
    import subprocess

    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    b = subprocess.run(["make", "-s", "-C", root, "asan"], capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "sanitize" in (b.stderr or ""):
        pytest.skip("sanitizer runtime unavailable: " + b.stderr[-200:])
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(root, "_asan", "asan_check")], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-2000:])
    assert "asan_check ok" in r.stdout


def test_v4_build_matches_the_checker_build(orc):
    """bench.py's CPU baseline may run the x86-64-v4 (AVX-512) build of the same source; it must
    compute what the x86-64-v2 checker build computes (run in a fresh interpreter so it binds
    the other library)."""
    import hashlib
    import subprocess
    import sys

    if not orc.host_has_avx512():
        pytest.skip("host without AVX-512")
    x = random_inputs(40, (0, 1, 4, 12), 77)
    ox = np.frombuffer(x.tobytes(), dtype=orc.INPUT_DTYPE).copy()
    adv, fixed, h, off = orc.fill(ox)
    want = hashlib.sha256(adv.tobytes() + fixed.tobytes() + h.tobytes()).hexdigest()
    code = ("import sys, hashlib, numpy as np; sys.path.insert(0, %r); import oracle\n"
            "print(oracle.use_fastest_build())\n"
            "x = np.frombuffer(bytes.fromhex(sys.stdin.read()), dtype=oracle.INPUT_DTYPE).copy()\n"
            "a, f, h, o = oracle.fill(x)\n"
            "print(oracle.LIB_PATH); print(hashlib.sha256(a.tobytes() + f.tobytes() + h.tobytes()).hexdigest())"
            ) % (ROOT + "/oracle")
    out = subprocess.run([sys.executable, "-c", code], input=ox.tobytes().hex(), capture_output=True,
                         text=True, timeout=120)
    lines = out.stdout.split()
    assert "x86-64-v4" in out.stdout and lines[-2].endswith("liboracle_b2f_v4.so"), out.stdout + out.stderr
    assert lines[-1] == want
