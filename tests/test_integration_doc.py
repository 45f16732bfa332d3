"""INTEGRATION.md's Rust binding must match the C ABI it binds.

A vortex maintainer pastes that `extern "C"` block into bittorrent/src; a
signature that drifted from include/vx_hash.h would be undefined behaviour at
the FFI boundary with no compiler to catch it.  No Rust toolchain exists here,
so this test parses both texts and checks every Rust declaration against the C
prototype of the same name (argument count, each argument's type, return type)
and the `#[repr(C)]` structs against the C structs (field names and types, in
order).  CPU only.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Rust FFI scalar and handle types -> C base types
RUST_TO_C = {
    "u8": "uint8_t", "u32": "uint32_t", "u64": "uint64_t", "i32": "int32_t", "i64": "int64_t",
    "usize": "size_t", "c_int": "int", "c_char": "char", "c_void": "void", "f64": "double",
    "VxCtx": "vx_ctx", "VxConfig": "vx_config", "VxCompletion": "vx_completion", "VxPlan": "vx_plan",
    "VxStats": "vx_stats", "VxVerifyTrace": "vx_verify_trace", "VxVerifyRound": "vx_verify_round",
    "VxSplit": "vx_split",
}


def rust_type_to_c(t: str) -> str:
    """Canonical form: innermost type then one entry per pointer level, each
    entry suffixed with "c" when that object is const (Rust `*const T` makes
    T const; C `const T* const*` makes T and the first pointer const)."""
    t = t.strip()
    m = re.fullmatch(r"\[(\w+);\s*(\d+)\]", t)
    if m:
        return f"{rust_type_to_c(m.group(1))}[{m.group(2)}]"
    m = re.fullmatch(r"\*(const|mut)\s+(.+)", t)
    if m:
        inner = rust_type_to_c(m.group(2)).split(" ")
        if m.group(1) == "const":
            inner[-1] += "c"
        return " ".join(inner + ["*"])
    return RUST_TO_C[t]


def norm_c(t: str) -> str:
    out = []
    for tok in re.findall(r"\w+|\*", t):
        if tok == "const":
            if out:
                out[-1] += "c"
            else:
                out.append(None)  # leading const: applies to the base type
        elif tok == "*":
            out.append("*")
        elif out and out[0] is None:
            out[0] = tok + "c"
        else:
            out.append(tok)
    return " ".join(out)


def c_prototypes():
    text = open(os.path.join(ROOT, "include", "vx_hash.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    protos = {}
    for m in re.finditer(r"([\w\s\*]+?)\b(vx_\w+)\s*\(([^;{]*?)\)\s*;", text):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        ret = ret.strip().split("\n")[-1]
        params = [] if args.strip() in ("", "void") else [a.strip() for a in args.split(",")]
        types = []
        for p in params:
            pm = re.fullmatch(r"(.+?)\s*\b(\w+)", re.sub(r"\s+", " ", p))
            types.append(norm_c(pm.group(1)))
        protos[name] = (norm_c(ret), types)
    return protos


def c_structs():
    text = open(os.path.join(ROOT, "include", "vx_hash.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"typedef struct (\w+) \{(.*?)\}", text, flags=re.S):
        fields = []
        for line in m.group(2).split(";"):
            line = line.strip()
            if not line:
                continue
            fm = re.fullmatch(r"(\w+)\s+(\w+)(?:\[(\w+)\])?", line)
            ctype, fname, dim = fm.group(1), fm.group(2), fm.group(3)
            dim = {"VX_DIGEST_LEN": "20", "VX_STATS_HIST": "24"}.get(dim, dim)
            fields.append((fname, ctype + (f"[{dim}]" if dim else "")))
        out[m.group(1)] = fields
    return out


def rust_block():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"```rust\n(.*?)```", text, flags=re.S)
    assert m, "INTEGRATION.md has no rust block"
    return m.group(1)


def rust_externs():
    block = rust_block()
    ext = re.search(r'extern "C" \{(.*?)\n\}', block, flags=re.S).group(1)
    out = {}
    for m in re.finditer(r"fn (vx_\w+)\((.*?)\)\s*(?:->\s*([\w:]+))?\s*;", ext, flags=re.S):
        name, args, ret = m.group(1), m.group(2), m.group(3)
        types = []
        for a in [a for a in re.split(r",\s*(?![^\[]*\])", args) if a.strip()]:
            _, t = a.split(":", 1)
            types.append(rust_type_to_c(t))
        out[name] = (RUST_TO_C[ret] if ret else "void", types)
    return out


def rust_structs():
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*pub struct (\w+)\s*\{(.*?)\}", rust_block(), flags=re.S):
        fields = []
        for f in re.split(r",\s*(?![^\[]*\])", m.group(2)):
            f = f.strip()
            if not f:
                continue
            f = re.sub(r"^pub\s+", "", f)
            fname, t = f.split(":", 1)
            fields.append((fname.strip(), rust_type_to_c(t)))
        out[m.group(1)] = fields
    return out


def test_rust_externs_match_header():
    c = c_prototypes()
    r = rust_externs()
    assert len(r) >= 10, r.keys()
    for name, (ret, args) in r.items():
        assert name in c, f"{name} is bound in INTEGRATION.md but not declared in include/vx_hash.h"
        cret, cargs = c[name]
        assert ret == cret, f"{name}: return {ret} (Rust) vs {cret} (C)"
        assert args == cargs, f"{name}: args {args} (Rust) vs {cargs} (C)"


def test_rust_structs_match_header():
    c = c_structs()
    r = rust_structs()
    pairs = {"VxCompletion": "vx_completion", "VxConfig": "vx_config", "VxPlan": "vx_plan", "VxStats": "vx_stats",
             "VxVerifyTrace": "vx_verify_trace", "VxVerifyRound": "vx_verify_round", "VxSplit": "vx_split"}
    for rname, cname in pairs.items():
        assert r[rname] == c[cname], f"{rname} vs {cname}: {r[rname]} / {c[cname]}"
    assert r["VxCtx"] == [("_private", "uint8_t[0]")]  # opaque handle
