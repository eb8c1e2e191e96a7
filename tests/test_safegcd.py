"""The one-lane inversion of the grand products (zk-odst_amd/csrc/b2f_safegcd.h: Bernstein-Yang
divsteps) built for the host with g++ and checked against Python's big-integer inverse for both
prover fields: edge values and 4,000 random elements each (CPU; the GPU tests pin the same code
through the lookup and permutation z columns)."""
import os
import random
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P_PALLAS = 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001
P_BN254 = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("sgcd") / "check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "zk-odst_amd", "csrc"),
                    "-o", exe, os.path.join(ROOT, "tools", "safegcd", "check.cpp")], check=True)
    return exe


@pytest.mark.parametrize("p", [P_PALLAS, P_BN254])
def test_safegcd_inverse_equals_big_integer_inverse(checker, p):
    rng = random.Random(p & 0xffff)
    xs = [0, 1, 2, 3, p - 1, p - 2, (1 << 255) % p, 1 << 128, (1 << 254) + 1] + \
         [rng.randrange(1, p) for _ in range(4000)]
    inp = "".join("%x %x\n" % (p, x) for x in xs)
    out = subprocess.run([checker], input=inp, capture_output=True, text=True, check=True).stdout.split()
    assert len(out) == len(xs)
    for x, o in zip(xs, out):
        assert int(o, 16) == (pow(x, -1, p) if x else 0), hex(x)


def test_safegcd_reports_no_inverse(checker):
    """inverse() says when the divsteps did not end at a unit (no silent wrong D^-1):
    a non-invertible x (odd composite moduli) and x = p are reported; x = 0 is the documented 0."""
    cases = [(15, 5), (15, 3), (21, 14), (P_PALLAS, P_PALLAS), (15, 0), (15, 7)]
    inp = "".join("%x %x\n" % c for c in cases)
    out = subprocess.run([checker], input=inp, capture_output=True, text=True, check=True).stdout.split()
    assert out[:4] == ["nonconverged"] * 4, out
    assert int(out[4], 16) == 0 and int(out[5], 16) == pow(7, -1, 15)
