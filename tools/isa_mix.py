"""Instruction mix of one kernel in a gfx950 assembly listing (hipcc --cuda-device-only -S).

Per basic block: instruction counts by class (VALU, SALU, VMEM load/store, LDS, SMEM, branch,
waitcnt). Loops are found from backward branches; `--loop` prints the blocks inside each.

  hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -o /tmp/f.s csrc/b2f_fused.hip
  python3 tools/isa_mix.py /tmp/f.s fused_kernelILi27ELi1E --loop
"""
import argparse
import re
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("buffer_store", "global_store", "flat_store")):
        return "vstore"
    if op.startswith(("buffer_load", "global_load", "flat_load", "buffer_atomic", "global_atomic")):
        return "vload"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def blocks_of(lines, sym):
    start = None
    for i, l in enumerate(lines):
        if start is None and l.startswith("_Z") and sym in l.split(":")[0]:
            start = i
        elif start is not None and (l.startswith("_Z") or l.strip().startswith(".Lfunc_end")):
            end = i
            break
    else:
        end = len(lines)
    body = lines[start:end]
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    for l in body[1:]:
        s = l.strip()
        m = re.match(r"^(\.LBB[\w_]+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        blocks[cur].append(s.split()[0])
    return blocks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="substring of the mangled kernel name")
    ap.add_argument("--loop", action="store_true", help="per-loop totals")
    ap.add_argument("--blocks", action="store_true", help="every block")
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    B = blocks_of(lines, a.kernel)
    names = list(B)
    tot = Counter()
    for n in names:
        tot.update(classify(o) for o in B[n])
    print("kernel total:", dict(tot), "instructions", sum(tot.values()))
    if a.blocks:
        for n in names:
            c = Counter(classify(o) for o in B[n])
            print(f"{n:28s} {sum(c.values()):5d} {dict(c)}")
    if a.loop:
        idx = {n: i for i, n in enumerate(names)}
        for i, n in enumerate(names):
            for o_i, o in enumerate(B[n]):
                pass
        # backward branches: a branch in block i whose target block j <= i
        raw = "\n".join(lines)
        for i, n in enumerate(names):
            pass
        seen = set()
        for i, n in enumerate(names):
            # re-scan the source lines of block n for branch targets
            pass
        body_targets = []
        cur = None
        for l in lines:
            s = l.strip()
            m = re.match(r"^(\.LBB[\w_]+):", s)
            if m:
                cur = m.group(1)
                continue
            m = re.match(r"^s_(?:cbranch_\w+|branch)\s+(\.LBB[\w_]+)", s)
            if m and cur in idx and m.group(1) in idx and idx[m.group(1)] <= idx[cur]:
                body_targets.append((m.group(1), cur))
        for head, tail in body_targets:
            if (head, tail) in seen:
                continue
            seen.add((head, tail))
            c = Counter()
            for n in names[idx[head]: idx[tail] + 1]:
                c.update(classify(o) for o in B[n])
            print(f"loop {head} .. {tail}: {idx[tail] - idx[head] + 1} blocks, {sum(c.values())} instr {dict(c)}")


if __name__ == "__main__":
    main()
