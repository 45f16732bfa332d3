"""INTEGRATION.md's Rust call sites must type-check against the binding.

No Rust toolchain exists here, so this is a small checker in
its place.  It reads every ```rust block of INTEGRATION.md and, for every call
of a `vx_*` function and of a `GpuHasher` method, checks the argument count
and each argument's type against the declaration (the `extern "C"` block,
itself checked against include/vx_hash.h by test_integration_doc.py, and the
`impl GpuHasher` signatures).  Argument types come from the snippets' own
`let name: Type` annotations and function parameters, and from the types
vortex and lava_torrent give the names the snippets use at their call sites:

* `metadata`: lava_torrent 0.11.1 `Torrent` — `pieces: Vec<Piece>` with
  `Piece = Vec<u8>` (indexed as `&Vec<u8>` at peer_connection.rs:1146 and
  iterated as `&Vec<u8>` at torrent.rs:724-726), `piece_length: i64`,
  `length: i64`, `name: String`, `files: Option<Vec<File>>`;
* `index: i32`, `conn_id: ConnectionId`, `buffer: Buffer`, `piece_len: u32`
  at peer_connection.rs:1122-1144 (`PieceSelector::piece_len -> u32`,
  piece_selector.rs:292);
* `Buffer::raw_slice(&self) -> &[u8]` (buf_pool.rs:51).

Rust's coercions that matter at an FFI call are modelled: `&T`/`&mut T` to
`*const T`/`*mut T`, `*mut T` to `*const T`, `&Vec<T>`/`&[T; N]` to `&[T]`,
and `as` casts.  Anything the checker cannot type fails the test, so the
snippets stay checkable.  CPU only.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INTS = {"u8", "u16", "u32", "u64", "usize", "i8", "i16", "i32", "i64", "isize", "c_int"}

REF_NAMES = {"metadata": "Torrent", "index": "i32", "conn_id": "ConnectionId", "buffer": "Buffer",
             "piece_len": "u32", "root": "PathBuf", "num_gpus": "usize", "initialized_state": "InitializedState",
             "torrent_state": "InitializedState", "file_store": "FileStore",
             # rayon::Scope opened at event_loop.rs:385, passed down to handle_message (peer_connection.rs:631-637)
             "scope": "Scope"}
REF_FIELDS = {("Torrent", "pieces"): "Vec<Vec<u8>>", ("Torrent", "piece_length"): "i64",
              ("Torrent", "length"): "i64", ("Torrent", "name"): "String",
              ("Torrent", "files"): "Option<Vec<File>>",
              ("InitializedState", "hasher"): "GpuHasher"}  # the field this integration adds


class Untyped(Exception):
    pass


def split_top(s: str, sep: str = ","):
    out, depth, cur, i = [], 0, "", 0
    while i < len(s):
        ch = s[i]
        if ch in "([{<" and not (ch == "<" and s[i - 1:i] == " "):
            depth += 1
        elif ch in ")]}>" and not (ch == ">" and s[i - 1:i] in ("-", " ")):
            depth -= 1
        if depth == 0 and s.startswith(sep, i):
            out.append(cur)
            cur = ""
            i += len(sep)
            continue
        cur += ch
        i += 1
    if cur.strip():
        out.append(cur)
    return [x.strip() for x in out]


def matching(s: str, open_at: int) -> int:
    pairs = {"(": ")", "[": "]", "{": "}"}
    want, depth = pairs[s[open_at]], 0
    for j in range(open_at, len(s)):
        if s[j] == s[open_at]:
            depth += 1
        elif s[j] == want:
            depth -= 1
            if depth == 0:
                return j
    raise ValueError("unbalanced")


def norm(t: str) -> str:
    t = re.sub(r"\s+", " ", t.strip())
    t = re.sub(r"&\s*mut\s+", "&mut ", t)
    t = re.sub(r"&\s+", "&", t)
    return t.replace("< ", "<").replace(" >", ">")


def deref(t: str) -> str:
    t = norm(t)
    while t.startswith("&"):
        t = t[5:] if t.startswith("&mut ") else t[1:]
    return t


def elem_of(t: str):
    t = deref(t)
    m = re.fullmatch(r"Vec<(.+)>", t) or re.fullmatch(r"\[(.+?)(?:; *\w+)?\]", t)
    return norm(m.group(1)) if m else None


class Checker:
    def __init__(self, blocks):
        self.blocks = blocks
        ext = re.search(r'extern "C" \{(.*?)\n\}', blocks[0], flags=re.S).group(1)
        self.externs = {}
        for m in re.finditer(r"fn (vx_\w+)\((.*?)\)\s*(?:->\s*([\w:]+))?\s*;", ext, flags=re.S):
            params = [norm(a.split(":", 1)[1]) for a in split_top(m.group(2)) if a]
            self.externs[m.group(1)] = (params, m.group(3) or "()")
        self.structs = {}
        for m in re.finditer(r"pub struct (\w+)\s*\{(.*?)\}", "\n".join(blocks), flags=re.S):
            fields = {}
            for f in split_top(m.group(2)):
                f = re.sub(r"^pub\s+", "", f.strip())
                if ":" in f:
                    n, t = f.split(":", 1)
                    fields[n.strip()] = norm(t)
            self.structs[m.group(1)] = fields
        impl = re.search(r"impl GpuHasher \{(.*?)\n\}", blocks[0], flags=re.S).group(1)
        self.methods = {}
        for m in re.finditer(r"pub fn (\w+)\((.*?)\)", impl, flags=re.S):
            params = [norm(a.split(":", 1)[1]) for a in split_top(m.group(2)) if ":" in a]
            self.methods[m.group(1)] = params

    # ---- types of expressions -------------------------------------------
    def env_of(self, bi: int) -> dict:
        """Names in scope in block bi: the reference's names, the block's
        parameters and `let` bindings, and (call-site blocks) the bindings of
        the call-site blocks before it, which the prose says they reuse."""
        env = dict(REF_NAMES)
        env["self"] = "GpuHasher" if bi == 0 else "InitializedState"
        block = "\n".join(self.blocks[1:bi + 1]) if bi else self.blocks[0]
        for m in re.finditer(r"\bfn \w+\((.*?)\)", block, flags=re.S):
            for a in split_top(m.group(1)):
                if ":" in a and not a.strip().startswith("&"):
                    n, t = a.split(":", 1)
                    env[n.strip()] = norm(t)
        for m in re.finditer(r"\blet\s+(?:mut\s+)?(\w+)\s*:\s*(.+?)\s*=", block):
            env[m.group(1)] = norm(m.group(2))
        for m in re.finditer(r"\(\w+\.\.(\w+)\)\.map\(\|(\w+)\|", block):  # (0..n).map(|d| ..): d has n's type
            if m.group(1) in env:
                env[m.group(2)] = env[m.group(1)]
        return env

    def field(self, t: str, f: str) -> str:
        t = deref(t)
        if (t, f) in REF_FIELDS:
            return REF_FIELDS[(t, f)]
        if t in self.structs and f in self.structs[t]:
            return self.structs[t][f]
        raise Untyped(f"no field {f} on {t}")

    def method(self, t: str, m: str, args) -> str:
        d = deref(t)
        if m == "raw_slice" and d == "Buffer":
            return "&[u8]"
        if m == "as_ptr" and d == "CString":
            return "*const c_char"
        e = elem_of(d)
        if m in ("as_ptr", "as_mut_ptr") and e:
            return ("*const " if m == "as_ptr" else "*mut ") + e
        if m == "len" and e:
            return "usize"
        if m == "concat" and e and elem_of(e):
            return f"Vec<{elem_of(e)}>"
        if m == "as_flattened" and e and re.fullmatch(r"\[.+; *\w+\]", e):
            return f"&[{elem_of(e)}]"
        raise Untyped(f"no method {m}() on {d}")

    def ty(self, e: str, env: dict) -> str:
        e = e.strip()
        parts = split_top(e, " as ")
        if len(parts) > 1:
            self.ty(" as ".join(parts[:-1]), env)  # the cast operand must type too
            return norm(parts[-1])
        if re.fullmatch(r"\d+(u8|u32|u64|usize|i32|i64)?", e):
            return "{int}"
        if re.fullmatch(r"\d+\.\d*(f64)?", e):
            return "{float}"
        if e == "std::ptr::null_mut()":
            return "*mut _"
        if e == "rayon::current_num_threads()":
            return "usize"
        if e.startswith("&mut "):
            return "&mut " + self.ty(e[5:], env)
        if e.startswith("&"):
            return "&" + self.ty(e[1:], env)
        if e.endswith(")"):
            depth, j = 0, len(e) - 1
            for j in range(len(e) - 1, -1, -1):  # the '(' matching the final ')'
                depth += {")": 1, "(": -1}.get(e[j], 0)
                if depth == 0:
                    break
            head, args = e[:j], split_top(e[j + 1:-1])
            if "." in head:
                k = head.rfind(".")
                return self.method(self.ty(head[:k], env), head[k + 1:], args)
            raise Untyped(e)
        if e.endswith("]"):
            k = e.rfind("[")
            el = elem_of(self.ty(e[:k], env))
            if el is None:
                raise Untyped(e)
            return el
        if "." in e:
            k = e.rfind(".")
            return self.field(self.ty(e[:k], env), e[k + 1:])
        if e in env:
            return env[e]
        raise Untyped(e)

    @staticmethod
    def compat(a: str, p: str) -> bool:
        a, p = norm(a), norm(p)
        if a == p:
            return True
        if a == "{int}":
            return p in INTS
        if a == "{float}":
            return p in ("f32", "f64")
        if a == "*mut _":
            return p.startswith("*mut ")
        if p.startswith("*const ") and a.startswith("*mut ") and a[5:] == p[7:]:
            return True
        if a.startswith("&mut ") and p.startswith(("*mut ", "*const ")):
            return Checker.compat("*mut " + a[5:], p)
        if a.startswith("&") and not a.startswith("&mut ") and p.startswith("*const "):
            return a[1:] == p[7:]
        if p.startswith("&") and a.startswith("&") and re.fullmatch(r"&(mut )?\[.+\]", p):
            mut = p.startswith("&mut ")
            if mut and not a.startswith("&mut "):
                return False
            return elem_of(a) == elem_of(p) and elem_of(a) is not None
        return False

    # ---- the check ----------------------------------------------------------
    def calls(self):
        """(block index, callee, kind, args) of every vx_* call and GpuHasher
        method call outside the extern declarations."""
        out = []
        for bi, block in enumerate(self.blocks):
            text = re.sub(r'extern "C" \{.*?\n\}', "", block, flags=re.S)
            text = re.sub(r"//[^\n]*", "", text)
            for m in re.finditer(r"(?<![\w.])(vx_\w+)\s*\(|\.(spawn|spawn_indexed|drain_into|register|"
                                 r"set_piece_table)\s*\(|\b(GpuHasher::new)\s*\(", text):
                name = m.group(1) or m.group(2) or m.group(3)
                start = m.end() - 1
                if re.search(r"\bfn\s+$", text[:m.start()]):  # a declaration, not a call
                    continue
                args = split_top(text[start + 1:matching(text, start)])
                recv = None
                if m.group(2):
                    k = m.start()
                    r = re.search(r"([\w.]+)$", text[:k])
                    recv = r.group(1) if r else None
                out.append((bi, name, recv, args))
        return out

    def check(self):
        problems, n = [], 0
        for bi, name, recv, args in self.calls():
            env = self.env_of(bi)
            if name.startswith("vx_"):
                if name not in self.externs:
                    problems.append(f"{name}: not declared in the extern block")
                    continue
                params = self.externs[name][0]
            else:
                if recv is not None:
                    try:
                        rt = deref(self.ty(recv, env))
                    except Untyped as e:
                        problems.append(f"{recv}.{name}: receiver untyped ({e})")
                        continue
                    if rt == "Scope" and name == "spawn":
                        continue  # rayon's Scope::spawn: the reference's own closure, not the binding
                    if rt != "GpuHasher":
                        problems.append(f"{recv}.{name}: receiver is {rt}, not GpuHasher")
                        continue
                params = self.methods["new" if name == "GpuHasher::new" else name]
            n += 1
            if len(args) != len(params):
                problems.append(f"{name}: {len(args)} arguments, declared {len(params)}")
                continue
            for a, p in zip(args, params):
                try:
                    t = self.ty(a, env)
                except Untyped as e:
                    problems.append(f"{name}: cannot type argument `{a}` ({e})")
                    continue
                if not self.compat(t, p):
                    problems.append(f"{name}: argument `{a}` is {t}, parameter is {p}")
        return n, problems

    def let_results(self):
        """`let x: T = unsafe { vx_f(..) }` must declare vx_f's return type."""
        out = []
        for block in self.blocks:
            for m in re.finditer(r"let\s+(?:mut\s+)?\w+\s*:\s*([^=]+?)\s*=\s*unsafe\s*\{\s*(vx_\w+)\s*\(", block):
                out.append((m.group(2), norm(m.group(1)), self.externs[m.group(2)][1]))
        return out


def rust_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.findall(r"```rust\n(.*?)```", text, flags=re.S)


def test_call_sites_type_check():
    blocks = rust_blocks()
    assert len(blocks) >= 4
    ck = Checker(blocks)
    n, problems = ck.check()
    assert not problems, "\n".join(problems)
    called = {name for _, name, _, _ in ck.calls()}
    for must in ("vx_create", "vx_submit", "vx_submit_piece", "vx_set_piece_table", "vx_flush", "vx_poll",
                 "vx_verify_files", "vx_verify_files_multi", "vx_plan_verify", "vx_verify_files_split",
                 "vx_split_init", "vx_split_claim", "vx_split_done", "vx_split_boundary",
                 "vx_register_host_buffer",
                 "vx_destroy", "spawn", "drain_into"):
        assert must in called, must
    assert n >= 15


def test_let_bound_results_have_the_declared_type():
    ck = Checker(rust_blocks())
    res = ck.let_results()
    assert len(res) >= 8
    for name, declared, ret in res:
        assert declared == norm(ret), f"{name} returns {ret}, bound as {declared}"


@pytest.mark.parametrize("bad,needle", [
    # round 1's bug: lava_torrent's pieces is Vec<Vec<u8>>; as_flattened exists only on [[T; N]]
    ("let io_errors: i64 = unsafe { vx_verify_files(hasher.ctx, path_ptrs.as_ptr(), lens.as_ptr(), "
     "path_ptrs.len(), metadata.piece_length as u32, metadata.pieces.as_flattened().as_ptr(), matched.len(), "
     "matched.as_mut_ptr(), 0) };", "as_flattened"),
    ("let rc: c_int = unsafe { vx_set_piece_table(self.ctx, metadata.pieces, 3) };", "vx_set_piece_table"),
    ("let rc: c_int = unsafe { vx_submit(self.ctx, 1, buffer.raw_slice().as_ptr(), 5) };", "arguments"),
    ("let rc: c_int = unsafe { vx_flush(&self.ctx) };", "vx_flush"),
])
def test_checker_rejects_known_mistakes(bad, needle):
    blocks = rust_blocks()
    extra = ("let hasher: &GpuHasher = &initialized_state.hasher;\nlet path_ptrs: Vec<*const c_char> = x;\n"
             "let lens: Vec<u64> = x;\nlet mut matched: Vec<u8> = x;\n" + bad)
    _, problems = Checker(blocks + [extra]).check()
    assert any(needle in p for p in problems), problems


def test_refused_spawn_hands_the_buffer_back():
    """vx_hash.h's ownership rule at the Rust boundary: a submit that returns
    non-zero did not take the piece, so GpuHasher::spawn / spawn_indexed must
    return the Buffer in the Err (and insert into `inflight` only on success),
    and every call site must bind that Buffer and hash the piece itself — a
    dropped Err would strand a piece vortex already marked downloaded
    (peer_connection.rs:1140) and trip BufferPool's leak check (buf_pool.rs:21-30)."""
    blocks = rust_blocks()
    impl = re.search(r"impl GpuHasher \{(.*?)\n\}", blocks[0], flags=re.S).group(1)
    for name in ("spawn", "spawn_indexed"):
        m = re.search(rf"pub fn {name}\(.*?\)\s*->\s*([^{{]+?)\s*\{{(.*?)\n    \}}", impl, flags=re.S)
        assert m, name
        assert norm(m.group(1)) == "Result<(), (i64, usize, ConnectionId, Buffer)>", (name, m.group(1))
        body = m.group(2)
        ret = body.find("return Err((rc as i64, index, conn_id, buffer))")
        ins = body.find("self.inflight.insert(")
        assert 0 <= ret < ins, f"{name}: the refused piece must return before it enters inflight"
    sites = 0
    for block in blocks[1:]:
        code = re.sub(r"//[^\n]*", "", block)
        for m in re.finditer(r"\.(spawn|spawn_indexed)\s*\(", code):
            recv = re.search(r"([\w.]+)$", code[:m.start()]).group(1)
            if not recv.endswith("hasher"):
                continue
            sites += 1
            head = code[:m.start()]
            b = re.search(r"if let Err\(\((\w+), (\w+), (\w+), (\w+)\)\) =\s*[\w.]+$", head)
            assert b, f"{recv}.{m.group(1)}: the Err (with the Buffer) must be bound"
            rest = code[matching(code, m.end() - 1):]
            body = rest[rest.index("{"):]
            body = body[:matching(body, 0) + 1]
            assert re.search(rf"\b{b.group(4)}\b", body), "the returned Buffer must be used (hashed and handed on)"
            assert "complete_tx.send(" in body, "a refused piece must still produce its DownloadedPiece"
    assert sites >= 1
