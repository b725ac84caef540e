"""INTEGRATION.md's Rust FFI module (qf_sys.rs) against include/qf_fec.h,
mechanically: every function the header declares is
declared in the `extern "C"` block with the same name, the same number of
arguments and the same C types (Rust `*const T` / `*mut T` / integer widths
mapped to their C spelling), and every `#[repr(C)]` struct has the header's
fields in the header's order and types.  No Rust toolchain is needed: both
sides are parsed as text.  CPU only."""
from __future__ import annotations

import re
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
HEADER = REPO / "include" / "qf_fec.h"
DOC = REPO / "INTEGRATION.md"

C_BASE = {"int": "int", "char": "char", "void": "void", "float": "float", "double": "double",
          "size_t": "size_t", "uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64",
          "int32_t": "i32", "int64_t": "i64"}
RUST_BASE = {"c_int": "int", "c_char": "char", "c_void": "void", "f32": "float", "f64": "double",
             "usize": "size_t", "u8": "u8", "u16": "u16", "u32": "u32", "u64": "u64", "i32": "i32", "i64": "i64"}


def _strip_c_comments(text: str) -> str:
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", " ", text)


def c_type(decl: str) -> tuple:
    """'const uint8_t *const *data' -> ('u8', ('const', 'const')): the base and,
    from the outermost pointer inwards, whether each pointee is const."""
    toks = re.findall(r"[A-Za-z_][A-Za-z0-9_]*|\*", decl.strip())
    if toks and toks[-1] not in ("*", "const") and len([t for t in toks if t not in ("*", "const")]) > 1:
        toks = toks[:-1]                         # the parameter name
    base_const = False
    base = None
    quals = []                                   # qualifier after each '*', innermost first
    for t in toks:
        if t == "const":
            if quals:
                quals[-1] = True                 # 'T *const': that pointer is const
            else:
                base_const = True                # 'const T' / 'T const'
        elif t == "*":
            quals.append(False)
        elif t not in ("struct", "unsigned", "signed"):
            base = C_BASE.get(t, t)
    # pointee constness, outermost pointer first: level i (outermost = last)
    # points at level i-1 (qualifier quals[i-1]) or at the base
    pointee = []
    for i in range(len(quals) - 1, -1, -1):
        pointee.append("const" if (quals[i - 1] if i > 0 else base_const) else "mut")
    return base, tuple(pointee)


def rust_type(t: str) -> tuple:
    t = t.strip()
    pointee = []
    while t.startswith("*"):
        m = re.match(r"\*(const|mut)\s+", t)
        assert m, t
        pointee.append(m.group(1))
        t = t[m.end():].strip()
    return RUST_BASE.get(t, t), tuple(pointee)


def header_functions() -> dict[str, tuple]:
    text = _strip_c_comments(HEADER.read_text())
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(qf_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        ret = re.sub(r"\b(extern|static|inline)\b", "", ret).strip()
        params = [] if args.strip() in ("", "void") else [a.strip() for a in args.split(",")]
        out[name] = (c_type(ret + " x") if ret else None, [c_type(p) for p in params])
    return out


def rust_block() -> str:
    text = DOC.read_text()
    m = re.search(r'extern "C" \{(.*?)\n\}', text, flags=re.S)
    assert m, "INTEGRATION.md has no extern \"C\" block"
    return m.group(1)


def rust_functions() -> dict[str, tuple]:
    body = re.sub(r"//[^\n]*", " ", rust_block())
    out = {}
    for m in re.finditer(r"pub fn (qf_[a-z0-9_]+)\s*\((.*?)\)\s*(->\s*([^;]+))?;", body, flags=re.S):
        name, args, ret = m.group(1), m.group(2), m.group(4)
        params = [a.strip() for a in args.split(",") if a.strip()]
        types = [rust_type(p.split(":", 1)[1]) for p in params]
        out[name] = (rust_type(ret) if ret else ("void", ()), types)
    return out


def test_every_header_function_is_declared_in_the_rust_binding():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 70
    missing = sorted(set(h) - set(r))
    assert missing == [], f"declared in qf_fec.h, missing from INTEGRATION.md qf_sys.rs: {missing}"
    extra = sorted(set(r) - set(h))
    assert extra == [], f"declared in qf_sys.rs but not in qf_fec.h: {extra}"


def test_rust_signatures_match_the_header():
    h, r = header_functions(), rust_functions()
    bad = []
    for name, (cret, cargs) in h.items():
        rret, rargs = r[name]
        if len(cargs) != len(rargs):
            bad.append(f"{name}: {len(cargs)} args in C, {len(rargs)} in Rust")
            continue
        if (cret or ("void", ())) != rret:
            bad.append(f"{name}: returns {cret} in C, {rret} in Rust")
        for i, (ca, ra) in enumerate(zip(cargs, rargs)):
            if ca != ra:
                bad.append(f"{name} arg {i}: {ca} in C, {ra} in Rust")
    assert bad == [], "\n".join(bad)


def _c_structs() -> dict[str, list[tuple]]:
    text = _strip_c_comments(HEADER.read_text())
    out = {}
    for m in re.finditer(r"typedef struct (qf_[a-z0-9_]+)\s*\{(.*?)\}\s*(qf_[a-z0-9_]+)\s*;", text, flags=re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = decl.strip()
            if not decl:
                continue
            arr = re.search(r"\[(\w+)\]$", decl)
            n = None
            if arr:
                n = arr.group(1)
                decl = decl[: arr.start()].strip()
            tm = re.match(r"((?:const\s+)?[A-Za-z_]\w*)\s+(.*)$", decl, flags=re.S)
            head, names = tm.group(1), tm.group(2)
            for nm in names.split(","):
                stars = nm.count("*")
                fields.append((nm.strip("* "), c_type(head + " *" * stars + " x"), n))
        out[m.group(3)] = fields
    return out


def _rust_structs() -> dict[str, list[tuple]]:
    text = re.sub(r"//[^\n]*", " ", DOC.read_text())
    out = {}
    for m in re.finditer(r"pub struct (qf_[a-z0-9_]+)\s*\{(.*?)\}", text, flags=re.S):
        body = m.group(2)
        if "_p:" in body:            # opaque handle
            continue
        fields = []
        for f in re.finditer(r"pub (\w+):\s*(\[[^\]]+\]|[^,\n]+)", body):
            nm, ty = f.group(1), f.group(2).strip()
            arr = re.match(r"\[(.+);\s*(\w+)\]", ty)
            n = None
            if arr:
                ty, n = arr.group(1), arr.group(2)
            fields.append((nm, rust_type(ty), n))
        out[m.group(1)] = fields
    return out


def test_rust_structs_match_the_header():
    c, r = _c_structs(), _rust_structs()
    assert {"qf_encode_shape", "qf_decode_shape", "qf_packet_desc", "qf_fec_config"} <= set(r)
    bad = []
    for name, rf in r.items():
        assert name in c, f"{name} is not a typedef struct of qf_fec.h"
        cf = c[name]
        if [f[0] for f in cf] != [f[0] for f in rf]:
            bad.append(f"{name}: fields {[f[0] for f in cf]} in C, {[f[0] for f in rf]} in Rust")
            continue
        for (n, ct, ca), (_, rt, ra) in zip(cf, rf):
            if ct != rt:
                bad.append(f"{name}.{n}: {ct} in C, {rt} in Rust")
            if ca is not None and ra is not None and ca != ra and not (ca.isdigit() is False):
                bad.append(f"{name}.{n}: array [{ca}] in C, [{ra}] in Rust")
    assert bad == [], "\n".join(bad)


def test_c_type_parser():
    assert c_type("const uint8_t *const *data") == ("u8", ("const", "const"))
    assert c_type("qf_adaptive *const *conns") == ("qf_adaptive", ("const", "mut"))
    assert c_type("qf_ctx **out") == ("qf_ctx", ("mut", "mut"))
    assert c_type("const char **name") == ("char", ("mut", "const"))
    assert c_type("uint32_t G") == ("u32", ())
    assert c_type("void *stream") == ("void", ("mut",))
    assert rust_type("*const *mut qf_adaptive") == ("qf_adaptive", ("const", "mut"))
    assert rust_type("*mut *const c_char") == ("char", ("mut", "const"))
