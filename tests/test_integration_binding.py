"""The Rust binding INTEGRATION.md gives a maintainer must match include/b2f.h exactly.

No Rust toolchain exists here, so the binding is text; this test is its compiler's type
check. It parses the `#[repr(C)]` structs and the `extern "C"` blocks of every ```rust block
in INTEGRATION.md and checks them against the C header: every B2F_API entry point declared,
with the same argument count, order and types and the same return type; every struct with the
same fields in the same order and the same size (a Rust caller of b2f_eval writes into its own
struct, so a missing field is a buffer overrun). It also checks that the chip's `load` sketch
constrains what the reference's region drivers constrain (fixed constants, copy constraints)
and that the ctypes table of the Python binding agrees with the header too."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "b2f.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")

C_SCALARS = {"uint64_t": ("u64", 8), "uint32_t": ("u32", 4), "uint8_t": ("u8", 1),
             "size_t": ("usize", 8), "int": ("i32", 4), "double": ("f64", 8),
             "char": ("c_char", 1), "void": ("void", 0),
             "b2f_input": ("B2fInput", 216), "b2f_eval_report": ("B2fEvalReport", 168),
             "b2f_ctx": ("B2fCtx", None)}
RUST_ALIASES = {"c_int": "i32", "c_void": "void", "c_char": "c_char"}
RUST_SIZES = {"u64": 8, "u32": 4, "u8": 1, "usize": 8, "i32": 4, "f64": 8}


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", "", s, flags=re.S)


def _c_type(decl):
    """'const uint64_t* d_offsets' / 'const uint64_t theta[4]' / 'int' -> canonical
    ('ptr_const'|'ptr_mut'|'val', base) in Rust vocabulary."""
    decl = decl.strip()
    arr = re.search(r"\[\s*\d*\s*\]\s*$", decl)
    is_const = bool(re.match(r"const\b", decl))
    decl = re.sub(r"\bconst\b", "", decl)
    stars = decl.count("*") + (1 if arr else 0)
    decl = re.sub(r"\[.*?\]", "", decl).replace("*", " ")
    words = decl.split()
    base = words[0]
    assert base in C_SCALARS, "unmapped C type %r" % base
    rb = C_SCALARS[base][0]
    if stars == 0:
        return ("val", rb)
    assert stars == 1, decl
    return ("ptr_const" if is_const else "ptr_mut", rb)


def _rust_type(t):
    t = t.strip()
    m = re.match(r"\*(const|mut)\s+(.+)$", t)
    if m:
        inner = m.group(2).strip()
        if inner.startswith("*"):  # a pointer to a pointer (hipMalloc's out argument)
            return ("ptr_" + m.group(1), _rust_type(inner))
        return ("ptr_" + m.group(1), RUST_ALIASES.get(inner, inner))
    return ("val", RUST_ALIASES.get(t, t))


def header_functions():
    s = _strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"B2F_API\s+([^;(]*?)\b(b2f_\w+)\s*\(([^;]*?)\)\s*;", s, re.S):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        rtype = _c_type(ret + " x") if ret != "void" else ("val", "void")
        argl = [] if args in ("", "void") else [_c_type(a) for a in args.split(",")]
        out[name] = (rtype, argl)
    return out


def header_structs():
    s = _strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"typedef struct\s*\{(.*?)\}\s*(\w+)\s*;", s, re.S):
        fields = []
        for line in m.group(1).split(";"):
            line = line.strip()
            if not line:
                continue
            fm = re.match(r"(\w+)\s+(\w+)\s*(?:\[\s*(\w+)\s*\])?$", line)
            assert fm, line
            typ, name, n = fm.groups()
            count = 1
            if n:
                count = int(n) if n.isdigit() else int(re.search(r"#define %s (\d+)" % n,
                                                                  open(HEADER).read()).group(1))
            fields.append((name, C_SCALARS[typ][0], count))
        out[m.group(2)] = fields
    return out


def rust_blocks():
    doc = open(DOC).read()
    return re.findall(r"```rust\n(.*?)```", doc, re.S)


def rust_externs():
    """{name: (ret, [args])} of every `fn` inside an `extern "C" { ... }` block, and the
    library each block links."""
    fns, links = {}, {}
    for blk in rust_blocks():
        for m in re.finditer(r'(?:#\[link\(name = "(\w+)"\)\]\s*)?extern "C" \{(.*?)\n\}', blk, re.S):
            lib = m.group(1)
            for fm in re.finditer(r"(?:pub\s+)?fn\s+(\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;",
                                  m.group(2), re.S):
                name, args, ret = fm.group(1), fm.group(2), fm.group(3)
                argl = []
                for a in [a for a in args.split(",") if a.strip()]:
                    _, t = a.split(":", 1)
                    argl.append(_rust_type(t))
                rtype = _rust_type(ret) if ret else ("val", "void")
                assert name not in fns, "%s declared twice in INTEGRATION.md" % name
                fns[name] = (rtype, argl)
                links[name] = lib
    return fns, links


def rust_structs():
    out = {}
    for blk in rust_blocks():
        for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive\([^)]*\)\]\s*)?pub struct (\w+)\s*\{(.*?)\}",
                             blk, re.S):
            fields = []
            for f in m.group(2).split(","):
                f = f.strip()
                if not f:
                    continue
                fm = re.match(r"pub\s+(\w+)\s*:\s*(?:\[\s*(\w+)\s*;\s*(\d+)\s*\]|(\w+))$", f)
                assert fm, f
                name, at, an, st = fm.groups()
                fields.append((name, at or st, int(an) if an else 1))
            out[m.group(1)] = fields
    return out


def test_every_header_entry_point_is_bound_with_the_same_signature():
    hdr = header_functions()
    assert len(hdr) >= 27
    fns, links = rust_externs()
    missing = sorted(set(hdr) - set(fns))
    assert not missing, "INTEGRATION.md does not bind %s" % missing
    for name, (ret, args) in hdr.items():
        rret, rargs = fns[name]
        assert links[name] == "b2f", name
        assert rret == ret, "%s returns %s in Rust, %s in C" % (name, rret, ret)
        assert len(rargs) == len(args), "%s: %d args in Rust, %d in C" % (name, len(rargs), len(args))
        for i, (ra, ca) in enumerate(zip(rargs, args)):
            assert ra == ca, "%s arg %d: Rust %s, C %s" % (name, i, ra, ca)
    extra = sorted(n for n in fns if n.startswith("b2f_") and n not in hdr)
    assert not extra, "INTEGRATION.md binds functions the header does not declare: %s" % extra


def test_structs_match_field_for_field():
    hs = header_structs()
    rs = rust_structs()
    for cname, rname, size in (("b2f_input", "B2fInput", 216),
                               ("b2f_eval_report", "B2fEvalReport", 168)):
        assert hs[cname] == rs[rname], (cname, hs[cname], rs[rname])
        assert sum(RUST_SIZES[t] * n for _, t, n in rs[rname]) == size
        doc = open(DOC).read()
        assert "size_of::<%s>() == %d" % (rname, size) in doc
    # the Python (ctypes) binding agrees too
    import sys

    sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))
    from b2f import _lib

    assert ctypes.sizeof(_lib.EvalReport) == 168 and _lib.REPORT_BYTES == 168
    assert [f[0] for f in _lib.EvalReport._fields_] == [f[0] for f in hs["b2f_eval_report"]]


def test_hip_calls_exist_in_the_hip_runtime_header():
    fns, links = rust_externs()
    hip = [n for n, lib in links.items() if lib == "amdhip64"]
    assert set(hip) >= {"hipMalloc", "hipFree", "hipMemcpy"}
    api = "/opt/rocm/include/hip/hip_runtime_api.h"
    if not os.path.exists(api):
        pytest.skip("no ROCm headers")
    text = open(api).read()
    for n in hip:
        assert re.search(r"hipError_t\s+%s\s*\(" % n, text), n
    # hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2 in the enum the binding hardcodes
    kinds = open(os.path.join(os.path.dirname(api), "driver_types.h")).read()
    assert re.search(r"hipMemcpyHostToDevice\s*=\s*1", kinds)
    assert re.search(r"hipMemcpyDeviceToHost\s*=\s*2", kinds)


def test_load_sketch_constrains_what_the_region_drivers_constrain():
    """The chip's load must put the fixed constants and every copy constraint into the
    circuit (the region drivers' assign_fixed / copy_advice), not just the advice cells."""
    load = [b for b in rust_blocks() if "fn load" in b]
    assert len(load) == 1
    body = load[0]
    for needle in ("b2f_fill_eval_dev", "b2f_fill_fixed_dev", "assign_fixed", "self.config.k_0",
                   "b2f_copy_constraints", "constrain_equal", "selectors[s].enable",
                   "assign_advice", "Value::unknown()", "NotEnoughRowsAvailable",
                   "first_failure != u64::MAX"):
        assert needle in body, needle
    # the copy quadruples are (dst_row, dst_col, src_row, src_col) instance-relative
    assert re.search(r"constrain_equal\(cell\[dc\]\[dr\], cell\[sc\]\[sr\]\)", body)
