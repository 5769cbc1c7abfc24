"""Static check of the Julia binding (julia-ocean-modelling_amd/julia/QGMI355.jl) against the
C-ABI it calls (include/qg_mi355.h).  No Julia toolchain exists in this image, so the binding
cannot run here; this reads both files and checks what a wrong `ccall` would get wrong
silently: every `ccall`ed symbol is declared, the argument count matches, every argument and
return type is the Julia type of the C type (scalars by width and signedness, pointers as
`Ptr{..}` / `Ref{..}` / `Cstring` of a compatible element), and the Julia mirrors of the
structs passed by pointer (`qg_params`, `qg_stats`, `qg_diag`) list the C fields in the same
order with the same types, so their layouts agree field for field."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "qg_mi355.h")
JL = os.path.join(ROOT, "julia-ocean-modelling_amd", "julia", "QGMI355.jl")


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", " ", s, flags=re.S)


def _c_param(p):
    """'const double alpha[2]' -> ('double', 1 pointer level); names dropped."""
    p = " ".join(p.replace("const", " ").split())
    arr = re.search(r"\[\s*\d*\s*\]\s*$", p)
    ptr = p.count("*") + (1 if arr else 0)
    p = re.sub(r"\[.*?\]", "", p).replace("*", " ")
    words = p.split()
    base = " ".join(words[:-1]) if len(words) > 1 else words[0]
    return base, ptr


def c_prototypes():
    text = _strip_c_comments(open(HEADER).read())
    protos = {}
    for m in re.finditer(r"\b(int|const\s+char\s*\*)\s*(qg_\w+)\s*\(([^;]*?)\)\s*;", text, re.S):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        plist = [] if params in ("", "void") else [_c_param(x) for x in params.split(",")]
        protos[name] = ("cstring" if "char" in ret else "int", plist)
    return protos


def c_struct(name):
    text = _strip_c_comments(open(HEADER).read())
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), text, re.S).group(1)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        typ, rest = decl.split(None, 1)
        for d in rest.split(","):
            d = d.strip()
            n = re.search(r"\[(\d+)\]", d)
            fields.append((re.sub(r"\[.*\]", "", d).strip(), typ, int(n.group(1)) if n else 0))
    return fields


def jl_struct(name):
    text = open(JL).read()
    body = re.search(r"\nstruct %s\n(.*?)\nend" % name, text, re.S).group(1)
    body = re.sub(r"#.*", "", body)
    return [tuple(x.strip().split("::")) for x in re.split(r"[;\n]", body) if "::" in x]


def jl_ccalls():
    text = open(JL).read()
    loops = dict(re.findall(r"\(:(\w+), :(qg_\w+)\)", text))  # @eval loop: (:jl, :qg_sym)
    calls = []
    for m in re.finditer(r"ccall\(\((:\w+|\$\(QuoteNode\(c\)\)), libqg\),\s*(\w+),\s*\(([^()]*)\)", text, re.S):
        sym, ret, args = m.group(1), m.group(2), m.group(3)
        names = [sym[1:]] if sym.startswith(":") else sorted(loops.values())
        argt = [a.strip() for a in re.split(r",(?![^{]*\})", args) if a.strip()]
        for n in names:
            calls.append((n, ret, argt))
    return calls


SCALAR = {"int": {"Cint", "Int32"}, "int32_t": {"Cint", "Int32"}, "int64_t": {"Int64"},
          "uint64_t": {"UInt64"}, "double": {"Float64", "Cdouble"}}
ELEM = {"double": {"Float64", "Cdouble", "Cvoid"}, "int": {"Cint", "Int32"}, "int64_t": {"Int64"},
        "char": {"UInt8", "Cchar"}, "void": {"Cvoid"}, "qg_params": {"QGParams"},
        "qg_stats": {"QGStats"}, "qg_diag": {"QGDiag"}, "qg_ctx": {"Cvoid"}, "qg_solver": {"Cvoid"}}


def _jl_ok(ctype, julia):
    base, ptr = ctype
    if ptr == 0:
        if base.endswith("_fn"):
            return False
        return julia in SCALAR.get(base, ())
    if base.endswith("_fn"):  # function-pointer typedefs are passed as plain pointers
        return julia == "Ptr{Cvoid}"
    if base == "char" and julia == "Cstring":
        return True
    m = re.fullmatch(r"(Ptr|Ref)\{(.*)\}", julia)
    if not m:
        return False
    inner = m.group(2)
    if ptr >= 2:
        return inner in ("Ptr{Cvoid}",) and base in ("qg_ctx", "qg_solver")
    tup = re.fullmatch(r"NTuple\{\d+,\s*(\w+)\}", inner)
    if tup:
        inner = tup.group(1)
    return inner in ELEM.get(base, ()) or inner == "Cvoid"


def test_every_ccall_matches_the_header():
    protos = c_prototypes()
    calls = jl_ccalls()
    assert len(calls) >= 25, "parser found too few ccalls"
    for name, ret, args in calls:
        assert name in protos, f"{name}: ccall'ed by QGMI355.jl but not declared in qg_mi355.h"
        cret, cparams = protos[name]
        assert (ret == "Cstring") if cret == "cstring" else (ret == "Cint"), (name, ret)
        assert len(args) == len(cparams), (name, args, cparams)
        for k, (j, c) in enumerate(zip(args, cparams)):
            assert _jl_ok(c, j), f"{name} argument {k + 1}: Julia {j} for C {c}"


def test_the_binding_covers_the_drop_in_surface():
    """The entry points the reference's loop needs are all bound."""
    bound = {n for n, _, _ in jl_ccalls()}
    for n in ("qg_create", "qg_destroy", "qg_bind_state", "qg_initialise", "qg_evolve_zeta", "qg_evolve_psi",
              "qg_run", "qg_canonicalize", "qg_set_keep_order", "qg_solver_create", "qg_solver_solve",
              "qg_laplace_5p", "qg_cd", "qg_arakawa_J", "qg_fill_ghosts", "qg_comm_unique_id", "qg_comm_init",
              "qg_snapshot", "qg_diagnostics", "qg_strerror"):
        assert n in bound, n
    # everything else in the header is bound too, except: the schedule helper the CPU tests
    # call, the host-transport attach (a Julia caller would pass @cfunction pointers; RCCL is
    # the Julia path) and the flattened duplicate of qg_get_stats
    assert set(c_prototypes()) - bound == {"qg_comm_exchange_plan", "qg_comm_init_host", "qg_solver_stats"}


JL_OF_C = {"double": "Float64", "int64_t": "Int64", "int32_t": "Int32"}


@pytest.mark.parametrize("cname,jname", [("qg_params", "QGParams"), ("qg_stats", "QGStats"), ("qg_diag", "QGDiag")])
def test_struct_mirrors_match(cname, jname):
    c = c_struct(cname)
    j = jl_struct(jname)
    assert [f[0] for f in c] == [f[0] for f in j], (cname, c, j)
    for (n, ct, cnt), (_, jt) in zip(c, j):
        want = JL_OF_C[ct] if cnt == 0 else f"NTuple{{{cnt},{JL_OF_C[ct]}}}"
        assert jt.replace(" ", "") == want, (cname, n, ct, cnt, jt)


def test_dropin_slot_modes_match_the_header():
    """set_dropin_slots! (Julia) and set_dropin_slots (Python) pass the header's keep-order
    codes: :slot1 = QG_KEEP_ORDER_SLOT1 (slot 1 newest after every call), :slot1_deferred =
    QG_KEEP_ORDER_SLOT1_DEFERRED (slot 1 of zeta stale between evolve_zeta! and evolve_psi!),
    and the Julia docstring states that contract."""
    hdr = open(HEADER).read()
    code = {k: int(v) for k, v in re.findall(r"#define (QG_KEEP_ORDER_\w+) (\d+)", hdr)}
    assert code == {"QG_KEEP_ORDER_SLOT1": 2, "QG_KEEP_ORDER_SLOT1_DEFERRED": 3}
    text = open(JL).read()
    m = re.search(r"_DROPIN_SLOTS\[\] = mode === :slot1 \? Cint\((\d)\) : mode === :slot1_deferred \? Cint\((\d)\)",
                  text)
    assert m and (int(m.group(1)), int(m.group(2))) == (2, 3)
    doc = re.search(r'"""`set_dropin_slots!(.*?)"""', text, re.S).group(1)
    assert "must not be" in doc and "evolve_psi!" in doc
    import sys
    sys.path.insert(0, os.path.join(ROOT, "julia-ocean-modelling_amd"))
    from qgamd import _lib
    assert (_lib.QG_KEEP_ORDER_SLOT1, _lib.QG_KEEP_ORDER_SLOT1_DEFERRED) == (2, 3)


def test_preconditioner_codes_match_the_header():
    """QG_PRECOND_* (header enum) = the Julia PRECOND_* constants = qgamd._lib's."""
    hdr = open(HEADER).read()
    code = {k: int(v) for k, v in re.findall(r"(QG_PRECOND_\w+) = (\d+)", hdr)}
    assert code == {"QG_PRECOND_NONE": 0, "QG_PRECOND_SPECTRAL": 1, "QG_PRECOND_MULTIGRID": 2}
    text = open(JL).read()
    jl = {k: int(v) for k, v in re.findall(r"const (PRECOND_\w+) = Int32\((\d+)\)", text)}
    assert {"QG_" + k: v for k, v in jl.items()} == code
    import sys
    sys.path.insert(0, os.path.join(ROOT, "julia-ocean-modelling_amd"))
    from qgamd import _lib
    assert {k: getattr(_lib, k) for k in code} == code


_JL_OPEN = {"module", "baremodule", "function", "struct", "if", "for", "while", "let", "begin", "do", "try",
            "macro", "quote"}


def _jl_strip(src):
    """Julia source without comments, strings and character literals (for the block check)."""
    out, i, n = [], 0, len(src)
    while i < n:
        if src.startswith('"""', i):
            i = src.index('"""', i + 3) + 3
            out.append(" ")
            continue
        c = src[i]
        if c == '"':
            j = i + 1
            while src[j] != '"':
                j += 2 if src[j] == "\\" else 1
            out.append(" ")
            i = j + 1
            continue
        m = re.match(r"'(\\.|[^\\'])'", src[i:i + 4]) if c == "'" else None
        if m:
            out.append(" ")
            i += m.end()
            continue
        if src.startswith("#=", i):
            i = src.index("=#", i) + 2
            continue
        if c == "#":
            j = src.find("\n", i)
            i = n if j < 0 else j
            continue
        out.append(c)
        i += 1
    return "".join(out)


def jl_block_balance(src):
    """None if every block keyword of the Julia source has its `end` (keywords and `end`
    inside brackets -- comprehensions, `x[end]` -- do not count), else the first problem."""
    s = _jl_strip(src)
    stack, brack = [], 0
    for m in re.finditer(r"[A-Za-z_][A-Za-z_0-9!]*|[\[\]\(\)\{\}]|:\w+", s):
        t = m.group(0)
        if t in "([{":
            brack += 1
        elif t in ")]}":
            brack -= 1
        elif brack == 0 and not t.startswith(":"):
            if t in _JL_OPEN:
                stack.append((t, s.count("\n", 0, m.start()) + 1))
            elif t == "end":
                if not stack:
                    return f"unmatched end at line {s.count(chr(10), 0, m.start()) + 1}"
                stack.pop()
    if stack:
        return f"unclosed {stack[-1][0]} from line {stack[-1][1]}"
    return f"bracket imbalance {brack}" if brack else None


def test_julia_blocks_are_balanced():
    """No Julia parser here: a block-structure check of QGMI355.jl (every function / struct /
    if / for / let / begin / do / try / module has its `end`, brackets balance), validated on a
    copy with one `end` removed."""
    src = open(JL).read()
    assert jl_block_balance(src) is None
    lines = src.split("\n")
    ends = [i for i, l in enumerate(lines) if l.strip() == "end"]
    assert len(ends) > 10
    broken = "\n".join(lines[:ends[5]] + lines[ends[5] + 1:])
    assert jl_block_balance(broken) is not None
