"""Generate zk-odst_amd/csrc/b2f_mont_asm.h: the Montgomery product of b2f_field.h as ONE inline
asm block per field (gfx950), so the column accumulator never leaves two fixed VGPR pairs.

Why: the per-step asm of b2f_field.h's Comba product (acc_madd2) leaves the column shift
(acc = acc >> 32 | carry << 32), the carry re-initialisation and the words m_k to the compiler,
which spends ~68 v_mov and a wait state per asm block on them (disassembly of
lk_zpass_kernel, r05); v_mad_u64_u32 itself is ~4 wave cycles and everything else 2, so the
glue costs about as much as the multiplies.

Scheme (product scanning, 8 x 32-bit words, R = 2^256):
  * the column sum lives in a 64-bit pair ACC (v[0:1] = X or v[2:3] = Y, clobbered registers:
    inline asm has no way to name one half of a 64-bit operand), its carry word in the high
    VGPR of the other pair;
  * every word product is v_mad_u64_u32 ACC, vcc, x, y, ACC then v_addc (the first of a column
    v_cndmask from vcc: it initialises the carry word);
  * at a column's end the next accumulator is (ACC.hi, carry): one v_mov into the low half of
    the other pair (whose high half already is the carry), and the roles swap;
  * m_k = ACC.lo * (-p^-1 mod 2^32) (pallas: 0 - ACC.lo) goes to the k-th output register; the
    output registers of the m words take the result words as the m words die (m_j is last used
    in column j + 7), so the block needs no extra outputs: r_j = m_(j+1), r_7 = m_0;
  * zero words of p are skipped (pallas: p_4..p_6); p_0 = 1 (pallas) is the inline constant 1.
The result is < 2p (both moduli have a top word below 2^31 - 1) and reduce_once_asm finishes it
by a borrow chain and v_cndmask.

Run: python tools/gen_mont_asm.py  (writes the header; tests/test_mont_asm_gen.py checks the
committed header is what this script writes).
"""
import os
import sys

PALLAS_P = [0x00000001, 0x992d30ed, 0x094cf91b, 0x224698fc, 0, 0, 0, 0x40000000]
PALLAS_NP = 0xffffffff
BN254_P = [0xf0000001, 0x43e1f593, 0x79b97091, 0x2833e848, 0x8181585d, 0xb85045b6, 0xe131a029,
           0x30644e72]
BN254_NP = 0xefffffff

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "zk-odst_amd", "csrc", "b2f_mont_asm.h")


def product_asm(p, np_):
    """Return (lines, sgpr_p_indices, has_np): the asm text of a b / R (< 2p). Operands: %0..%7
    m/result words (=&v), %8..%15 a, %16..%23 b, then the SGPR p words in index order, then NP
    (unless it is -1).

    pallas (p = 1 + p1 2^32 + p2 2^64 + p3 2^96 + 2^254, NP = -1) takes two shortcuts:
      * m_k p_0 = m_k: m_k = 0 - ACC.lo, so ACC + m_k = (ACC.hi + (ACC.lo != 0)) 2^32, and
        v_sub_co's borrow is that bit: it goes into the shift's v_addc, no multiply;
      * m_i 2^254 (p_7 = 2^30) puts (m_i << 30) mod 2^32 into column i + 7 and m_i >> 2 into
        column i + 8: column j gets w_j = v_alignbit(m_(j-7), m_(j-8), 2), added at the shift
        into column j (2 instructions and an add instead of 2 multiplies).
    """
    pallas = p[0] == 1 and np_ == 0xffffffff and p[7] == 1 << 30 and p[4:7] == [0, 0, 0]
    sp = [i for i in range(8) if p[i] not in (0, 1) and not (pallas and i == 7)]
    nop = 24
    pop = {}
    for i in sp:
        pop[i] = "%%%d" % nop
        nop += 1
    np_op = None
    if np_ != 0xffffffff:
        np_op = "%%%d" % nop
        nop += 1

    def pw(j):
        return "1" if p[j] == 1 else pop[j]

    m = ["%%%d" % i for i in range(8)]
    a = ["%%%d" % (8 + i) for i in range(8)]
    b = ["%%%d" % (16 + i) for i in range(8)]
    X, Y = ("v[0:1]", "v0", "v1"), ("v[2:3]", "v2", "v3")
    lines = []
    acc, other = X, Y  # the column accumulates in acc; its carry word is other's high half
    fresh_acc = True  # acc is zero (column 0 only)

    def madd(x, y, live):
        nonlocal fresh_acc
        if fresh_acc:
            lines.append("v_mad_u64_u32 %s, vcc, %s, %s, 0" % (acc[0], x, y))
            fresh_acc = False  # 0 + x y < 2^64: no carry
            return live
        lines.append("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (acc[0], x, y, acc[0]))
        carry_in(live)
        return True

    def carry_in(live):  # other.hi += vcc (initialised when not yet live)
        if live:
            lines.append("v_addc_co_u32_e32 %s, vcc, 0, %s, vcc" % (other[2], other[2]))
        else:
            lines.append("v_cndmask_b32_e64 %s, 0, 1, vcc" % other[2])

    for k in range(15):
        terms = []
        for i in range(max(0, k - 7), min(k, 7) + 1):
            if i == k:
                continue  # a_k b_0 goes last (before m_k)
            terms.append((a[i], b[k - i]))
            if p[k - i] != 0 and not (pallas and k - i == 7):  # k - i >= 1: m_i is known
                terms.append((m[i], pw(k - i)))
        if k < 8:
            terms.append((a[k], b[0]))
        live = False
        for (x, y) in terms:
            live = madd(x, y, live)
        if k < 8:
            if pallas:
                lines.append("v_sub_co_u32_e32 %s, vcc, 0, %s" % (m[k], acc[1]))  # borrow pending
            else:
                lines.append("v_mul_lo_u32 %s, %s, %s" % (m[k], acc[1], np_op))
                live = madd(m[k], pw(0), live)
        if k == 14:
            if pallas:  # r_7 = acc.hi + (m_7 >> 2); m_7 takes r_6 after its last read
                lines.append("v_lshrrev_b32 %s, 2, %s" % (other[1], m[7]))
                lines.append("v_mov_b32 %s, %s" % (m[7], acc[1]))
                lines.append("v_add_u32_e32 %s, %s, %s" % (m[0], acc[2], other[1]))
            else:  # r_7 = the column's high word (its carry is zero: the result is < 2^256)
                lines.append("v_mov_b32 %s, %s" % (m[7], acc[1]))
                lines.append("v_mov_b32 %s, %s" % (m[0], acc[2]))
            break
        # shift into column k + 1: the next accumulator is (acc.hi [+ borrow], carry) in other
        j = k + 1
        if pallas and k < 8:
            lines.append("v_addc_co_u32_e32 %s, vcc, 0, %s, vcc" % (other[1], acc[2]))
            carry_in(live)
        elif pallas and j >= 8:
            # w_j reads m_(k-7), whose register takes r_(k-8): w first
            lines.append("v_alignbit_b32 %s, %s, %s, 2" % (other[1], m[j - 7], m[j - 8]))
            lines.append("v_mov_b32 %s, %s" % (m[k - 7], acc[1]))
            lines.append("v_add_co_u32_e32 %s, vcc, %s, %s" % (other[1], acc[2], other[1]))
            lines.append("v_addc_co_u32_e32 %s, vcc, 0, %s, vcc" % (other[2], other[2]))
        else:
            if k >= 8:
                lines.append("v_mov_b32 %s, %s" % (m[k - 7], acc[1]))
            lines.append("v_mov_b32 %s, %s" % (other[1], acc[2]))
        if pallas and j in (7, 8):  # w_7 = m_0 << 30, w_8 = alignbit(m_1, m_0, 2) (acc.lo is 0)
            if j == 7:
                lines.append("v_lshlrev_b32 %s, 30, %s" % (acc[1], m[0]))
            else:
                lines.append("v_alignbit_b32 %s, %s, %s, 2" % (acc[1], m[1], m[0]))
            lines.append("v_add_co_u32_e32 %s, vcc, %s, %s" % (other[1], other[1], acc[1]))
            lines.append("v_addc_co_u32_e32 %s, vcc, 0, %s, vcc" % (other[2], other[2]))
        acc, other = other, acc
    return lines, sp, np_op is not None


def reduce_asm(p):
    """t (< 2p) - p by a borrow chain into %0..%7, kept only when it did not borrow.
    Operands: %0..%7 result (=&v), %8..%15 t, then the p words that are not inline constants
    (0, 1), as VGPRs: with the borrow in vcc an SGPR source would be a second constant-bus read."""
    sp = [i for i in range(8) if p[i] not in (0, 1)]
    pop = {i: "%%%d" % (16 + n) for n, i in enumerate(sp)}
    lines = []
    for i in range(8):
        src = str(p[i]) if p[i] in (0, 1) else pop[i]
        if i == 0:
            lines.append("v_subrev_co_u32_e32 %%%d, vcc, %s, %%%d" % (i, src, 8 + i))
        else:
            lines.append("v_subbrev_co_u32_e32 %%%d, vcc, %s, %%%d, vcc" % (i, src, 8 + i))
    for i in range(8):
        lines.append("v_cndmask_b32_e32 %%%d, %%%d, %%%d, vcc" % (i, i, 8 + i))
    return lines, sp


def emit(name, p, np_):
    pl, psp, has_np = product_asm(p, np_)
    rl, rsp = reduce_asm(p)
    out = []
    nmad = sum(1 for ln in pl if ln.startswith("v_mad"))
    out.append("// %s: %d v_mad_u64_u32, %d instructions in the product block, %d in the reduction"
               % (name, nmad, len(pl), len(rl)))
    out.append("template <>")
    out.append("__device__ __forceinline__ Fe mul_asm<%s>(const Fe& a, const Fe& b) {" % name)
    out.append("  uint32_t m0, m1, m2, m3, m4, m5, m6, m7;")
    out.append("  asm(")
    for ln in pl:
        out.append('      "%s\\n\\t"' % ln)
    out[-1] = out[-1][:-5] + '"'
    outs = ", ".join('"=&v"(m%d)' % i for i in range(8))
    ins = ['"v"(a.w[%d])' % i for i in range(8)] + ['"v"(b.w[%d])' % i for i in range(8)]
    ins += ['"s"(%s::P[%d])' % (name, i) for i in psp]
    if has_np:
        ins.append('"s"(%s::NP)' % name)
    out.append("      : %s" % outs)
    out.append("      : %s" % ", ".join(ins[:8]))
    out.append("        , %s" % ", ".join(ins[8:16]))
    if ins[16:]:
        out.append("        , %s" % ", ".join(ins[16:]))
    out.append('      : "v0", "v1", "v2", "v3", "vcc");')
    out.append("  Fe t, r;")
    out.append("  t.w[0] = m1; t.w[1] = m2; t.w[2] = m3; t.w[3] = m4;")
    out.append("  t.w[4] = m5; t.w[5] = m6; t.w[6] = m7; t.w[7] = m0;")
    out.append("  asm(")
    for ln in rl:
        out.append('      "%s\\n\\t"' % ln)
    out[-1] = out[-1][:-5] + '"'
    outs = ", ".join('"=&v"(r.w[%d])' % i for i in range(8))
    tin = ", ".join('"v"(t.w[%d])' % i for i in range(8))
    # VGPR p words: a carry-in (vcc) and an SGPR source exceed gfx9's one constant-bus read
    pin = ", ".join('"v"(%s::P[%d])' % (name, i) for i in rsp)
    out.append("      : %s" % outs)
    out.append("      : %s%s" % (tin, (", " + pin) if pin else ""))
    out.append('      : "vcc");')
    out.append("  return r;")
    out.append("}")
    return out


def generate():
    hdr = [
        "// b2f_mont_asm.h -- GENERATED by tools/gen_mont_asm.py (do not edit): the Montgomery",
        "// product of b2f_field.h (mul) as one inline asm block per field, its column accumulator",
        "// in two fixed VGPR pairs (v[0:1], v[2:3], declared clobbered). See the generator's",
        "// docstring for the scheme; tools/mulbench.hip checks it against mul_cios.",
        "#pragma once",
        "",
        "template <class F>",
        "__device__ __forceinline__ Fe mul_asm(const Fe& a, const Fe& b);",
        "",
    ]
    hdr += emit("Pallas", PALLAS_P, PALLAS_NP)
    hdr.append("")
    hdr += emit("Bn254", BN254_P, BN254_NP)
    return "\n".join(hdr) + "\n"


if __name__ == "__main__":
    text = generate()
    if len(sys.argv) > 1 and sys.argv[1] == "--check":
        with open(OUT) as f:
            sys.exit(0 if f.read() == text else 1)
    with open(OUT, "w") as f:
        f.write(text)
    print("wrote", OUT)
