"""CPU checks of the generated Montgomery product (zk-odst_amd/csrc/b2f_mont_asm.h).

* the committed header is exactly what tools/gen_mont_asm.py writes;
* the instruction streams it emits, run by a small interpreter of the VALU instructions they use
  (one lane, vcc as a bit), give a b / 2^256 mod p for random and edge operands of both fields,
  checked against Python integers. The GPU check of the same code is tools/mulbench.hip's
  mismatch count and every field test of tests/test_gpu_*.py.
"""
import importlib.util
import os
import random
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "tools", "gen_mont_asm.py")


def _gen():
    spec = importlib.util.spec_from_file_location("gen_mont_asm", GEN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


M32 = 0xffffffff


def _run(lines, ops):
    """Interpret asm lines on one lane. ops: operand index -> value (32-bit); physical v0..v3."""
    v = {"v0": 0, "v1": 0, "v2": 0, "v3": 0}
    vcc = [0]

    def rd(x):
        x = x.strip()
        if x.startswith("%"):
            return ops[int(x[1:])]
        if x in v:
            return v[x]
        if x.startswith("v["):
            lo = int(x[2:x.index(":")])
            return v["v%d" % lo] | (v["v%d" % (lo + 1)] << 32)
        return int(x, 0)

    def wr(x, val, bits=32):
        x = x.strip()
        if x.startswith("%"):
            ops[int(x[1:])] = val & M32
        elif x.startswith("v["):
            lo = int(x[2:x.index(":")])
            v["v%d" % lo] = val & M32
            v["v%d" % (lo + 1)] = (val >> 32) & M32
        else:
            v[x] = val & M32

    for ln in lines:
        op, rest = ln.split(" ", 1)
        args = [t.strip() for t in re.split(r",(?![^\[]*\])", rest)]
        if op == "v_mad_u64_u32":
            r = rd(args[2]) * rd(args[3]) + rd(args[4])
            vcc[0] = r >> 64
            wr(args[0], r & ((1 << 64) - 1))
        elif op == "v_addc_co_u32_e32":
            r = rd(args[2]) + rd(args[3]) + vcc[0]
            vcc[0] = r >> 32
            wr(args[0], r)
        elif op == "v_add_co_u32_e32":
            r = rd(args[2]) + rd(args[3])
            vcc[0] = r >> 32
            wr(args[0], r)
        elif op == "v_cndmask_b32_e64":
            wr(args[0], rd(args[2]) if vcc[0] else rd(args[1]))
        elif op == "v_cndmask_b32_e32":
            wr(args[0], rd(args[2]) if vcc[0] else rd(args[1]))
        elif op == "v_sub_co_u32_e32":
            r = rd(args[2]) - rd(args[3])
            vcc[0] = 1 if r < 0 else 0
            wr(args[0], r)
        elif op == "v_sub_u32_e32":
            wr(args[0], rd(args[1]) - rd(args[2]))
        elif op == "v_subrev_co_u32_e32":
            r = rd(args[3]) - rd(args[2])
            vcc[0] = 1 if r < 0 else 0
            wr(args[0], r)
        elif op == "v_subbrev_co_u32_e32":
            r = rd(args[3]) - rd(args[2]) - vcc[0]
            vcc[0] = 1 if r < 0 else 0
            wr(args[0], r)
        elif op == "v_mul_lo_u32":
            wr(args[0], rd(args[1]) * rd(args[2]))
        elif op == "v_mov_b32":
            wr(args[0], rd(args[1]))
        elif op == "v_alignbit_b32":
            wr(args[0], ((rd(args[1]) << 32) | rd(args[2])) >> rd(args[3]))
        elif op == "v_lshlrev_b32":
            wr(args[0], rd(args[2]) << rd(args[1]))
        elif op == "v_lshrrev_b32":
            wr(args[0], rd(args[2]) >> rd(args[1]))
        elif op == "v_add_u32_e32":
            wr(args[0], rd(args[1]) + rd(args[2]))
        else:
            raise AssertionError("interpreter lacks " + op)
    return ops


def _words(x):
    return [(x >> (32 * i)) & M32 for i in range(8)]


def _val(w):
    return sum(x << (32 * i) for i, x in enumerate(w))


def _mont(g, p_words, np_, a, b):
    p = _val(p_words)
    pl, psp, has_np = g.product_asm(p_words, np_)
    ops = {i: 0 for i in range(8)}
    for i, x in enumerate(_words(a)):
        ops[8 + i] = x
    for i, x in enumerate(_words(b)):
        ops[16 + i] = x
    n = 24
    for i in psp:
        ops[n] = p_words[i]
        n += 1
    if has_np:
        ops[n] = np_
    _run(pl, ops)
    t = [ops[1], ops[2], ops[3], ops[4], ops[5], ops[6], ops[7], ops[0]]
    assert _val(t) < 2 * p
    rl, rsp = g.reduce_asm(p_words)
    rops = {i: 0 for i in range(8)}
    for i, x in enumerate(t):
        rops[8 + i] = x
    for n, i in enumerate(rsp):
        rops[16 + n] = p_words[i]
    _run(rl, rops)
    return _val([rops[i] for i in range(8)])


def test_header_is_generated():
    g = _gen()
    with open(g.OUT) as f:
        assert f.read() == g.generate(), "run python tools/gen_mont_asm.py"


def test_generated_product_matches_integers():
    g = _gen()
    rng = random.Random(5)
    for pw, np_ in ((g.PALLAS_P, g.PALLAS_NP), (g.BN254_P, g.BN254_NP)):
        p = _val(pw)
        rinv = pow(1 << 256, -1, p)
        cases = [(0, 0), (1, 1), (p - 1, p - 1), (p - 1, 1), (0, p - 1)]
        cases += [(rng.randrange(p), rng.randrange(p)) for _ in range(300)]
        for a, b in cases:
            assert _mont(g, pw, np_, a, b) == a * b * rinv % p, (hex(a), hex(b))
