"""Static checks of the Go plugin source (go/pkg/gpuagg) for a box without a Go toolchain.

The image has no `go` binary, so nothing here can compile the plugin.  These checks
catch, from the source text alone, the classes of compile error that a cgo package of
this shape can carry and that no Python transcription would see:

* two top-level declarations of one name across the files that build together (same
  package, same `//go:build` expression) -- "redeclared in this block";
* a method declared twice on one receiver type;
* an import a file never uses, or a well-known package a file uses without importing;
* a `C.name` that include/gpuagg.h (or cgo / libc) does not define;
* `Record` drifting from `struct gpuagg_record` (field order, types, offsets, size);
* an unexported identifier called from a Go snippet of INTEGRATION.md (the snippets are
  pasted into other packages), and `gpuagg.X` names the package does not export.

Test infrastructure only: the product never imports this module.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_PKG = os.path.join(ROOT, "go", "pkg", "gpuagg")
HEADER = os.path.join(ROOT, "include", "gpuagg.h")

GO_BUILTINS = {
    "append", "cap", "clear", "close", "complex", "copy", "delete", "imag", "len", "make", "max", "min",
    "new", "panic", "print", "println", "real", "recover",
    # conversions to predeclared types
    "bool", "byte", "complex64", "complex128", "error", "float32", "float64", "int", "int8", "int16",
    "int32", "int64", "rune", "string", "uint", "uint8", "uint16", "uint32", "uint64", "uintptr", "any",
}
GO_KEYWORDS = {
    "break", "case", "chan", "const", "continue", "default", "defer", "else", "fallthrough", "for", "func",
    "go", "goto", "if", "import", "interface", "map", "package", "range", "return", "select", "struct",
    "switch", "type", "var",
}
# cgo pseudo-package members that are not declared by the C preamble's headers
CGO_BUILTINS = {"CString", "GoString", "GoStringN", "GoBytes", "CBytes"}
C_TYPES = {
    "char", "schar", "uchar", "short", "ushort", "int", "uint", "long", "ulong", "longlong", "ulonglong",
    "float", "double", "size_t", "int8_t", "int16_t", "int32_t", "int64_t", "uint8_t", "uint16_t",
    "uint32_t", "uint64_t", "uintptr_t",
}
LIBC = {"free", "malloc", "calloc", "memcpy", "memset"}  # <stdlib.h> / <string.h> of the preamble


def strip_go(src: str) -> str:
    """Comments removed and string / rune literals blanked (kept as `""`), lines kept."""
    out = []
    i, n = 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append("\n" * src.count("\n", i, j))
            i = j
        elif c == "`":
            j = src.find("`", i + 1)
            j = n if j < 0 else j + 1
            out.append('""' + "\n" * src.count("\n", i, j))
            i = j
        elif c in "\"'":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if src[j] == "\\" else 1
            out.append('""' if c == '"' else "0")
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


@dataclass
class GoFile:
    path: str
    raw: str
    code: str  # stripped
    package: str = ""
    build: str = ""
    imports: dict = field(default_factory=dict)  # local name -> path ("C" for cgo)
    funcs: list = field(default_factory=list)  # (name, line)
    methods: list = field(default_factory=list)  # (receiver type, name, line)
    names: list = field(default_factory=list)  # top-level type / var / const names, (name, line)
    preamble: str = ""  # the cgo comment before import "C"


def _line(code: str, pos: int) -> int:
    return code.count("\n", 0, pos) + 1


def parse_go(path: str) -> GoFile:
    raw = open(path, encoding="utf-8").read()
    code = strip_go(raw)
    f = GoFile(path=path, raw=raw, code=code)
    m = re.search(r"^//go:build (.+)$", raw, re.M)
    f.build = " ".join(m.group(1).split()) if m else ""
    m = re.search(r"^package\s+(\w+)", code, re.M)
    f.package = m.group(1) if m else ""
    m = re.search(r"/\*(.*?)\*/\s*import\s+\"C\"", raw, re.S)
    f.preamble = m.group(1) if m else ""
    # imports: import "C" is blanked to import "" by strip_go, so read the raw text
    for blk in re.finditer(r"^import\s*\((.*?)^\)", raw, re.M | re.S):
        for ln in blk.group(1).splitlines():
            ln = ln.split("//")[0].strip()
            mm = re.match(r'(?:(\w+|\.|_)\s+)?"([^"]+)"', ln)
            if mm:
                alias, p = mm.group(1), mm.group(2)
                f.imports[alias or _pkg_name(p)] = p
    for mm in re.finditer(r'^import\s+(?:(\w+)\s+)?"([^"]+)"', raw, re.M):
        f.imports[mm.group(1) or _pkg_name(mm.group(2))] = mm.group(2)
    # top-level declarations: depth-0 lines of the stripped code
    depth = 0
    lines = code.split("\n")
    in_group = None  # "type" / "var" / "const" while inside a ( ... ) group at depth 1
    for ln_no, ln in enumerate(lines, 1):
        s = ln.strip()
        if depth == 0:
            mm = re.match(r"func\s+\(\s*\w*\s*\*?\s*(\w+)(?:\[[^\]]*\])?\s*\)\s*(\w+)", s)
            if mm:
                f.methods.append((mm.group(1), mm.group(2), ln_no))
            else:
                mm = re.match(r"func\s+(\w+)", s)
                if mm:
                    f.funcs.append((mm.group(1), ln_no))
            mm = re.match(r"(type|var|const)\s*\($", s)
            if mm:
                in_group = mm.group(1)
            else:
                mm = re.match(r"(type|var|const)\s+(\w+(?:\s*,\s*\w+)*)", s)
                if mm:
                    for nm in re.split(r"\s*,\s*", mm.group(2)):
                        f.names.append((nm, ln_no))
        elif depth == 1 and in_group and s and not s.startswith(")"):
            mm = re.match(r"(\w+(?:\s*,\s*\w+)*)", s)
            if mm and not s.startswith("}"):
                for nm in re.split(r"\s*,\s*", mm.group(1)):
                    f.names.append((nm, ln_no))
        for ch in ln:
            if ch in "({[":
                depth += 1
            elif ch in ")}]":
                depth -= 1
        if depth == 0:
            in_group = None
    return f


def _pkg_name(path: str) -> str:
    last = path.rstrip("/").split("/")[-1]
    if re.fullmatch(r"v\d+", last):  # a major-version suffix: the package is the element before
        last = path.rstrip("/").split("/")[-2]
    return last.replace("-", "_")


def load_package(d: str = GO_PKG) -> list:
    return [parse_go(os.path.join(d, n)) for n in sorted(os.listdir(d)) if n.endswith(".go")]


def build_sets(files: list) -> dict:
    """Files that compile together: same package and same //go:build expression."""
    sets: dict = {}
    for f in files:
        sets.setdefault((f.package, f.build), []).append(f)
    return sets


def duplicate_declarations(files: list) -> list:
    errs = []
    for (pkg, build), fs in build_sets(files).items():
        seen: dict = {}
        mseen: dict = {}
        for f in fs:
            for nm, ln in f.funcs + f.names:
                if nm in ("_", "init"):
                    continue
                where = f"{os.path.basename(f.path)}:{ln}"
                if nm in seen:
                    errs.append(f"{nm} redeclared in package {pkg} [{build}]: {seen[nm]} and {where}")
                else:
                    seen[nm] = where
            for rt, nm, ln in f.methods:
                where = f"{os.path.basename(f.path)}:{ln}"
                if (rt, nm) in mseen:
                    errs.append(f"method {rt}.{nm} redeclared: {mseen[(rt, nm)]} and {where}")
                else:
                    mseen[(rt, nm)] = where
        # a method and a field / func of the same name on one type is rarer; skip
    return errs


# package names this repository's Go files use; a selector on one of them needs its import
KNOWN_PACKAGES = {
    "binary", "context", "errors", "fmt", "io", "net", "os", "runtime", "sort", "strconv", "strings", "sync",
    "atomic", "time", "unsafe", "flow", "v1", "api", "validations", "common", "kcfg", "cache", "exporter",
    "ktime", "pubsub", "log", "metrics", "registry", "utils", "prometheus", "zap", "wrapperspb", "container",
}


def _locals(code: str) -> set:
    """Identifiers the file declares anywhere (params, :=, var, range), to tell a local
    `x.` from a package selector."""
    out = set()
    for mm in re.finditer(r"([\w\s,]+?):=", code):
        for nm in re.split(r"[\s,]+", mm.group(1).strip()):
            if re.fullmatch(r"\w+", nm):
                out.add(nm)
    for mm in re.finditer(r"\bvar\s+(\w+)", code):
        out.add(mm.group(1))
    # parameters and results: "name Type" / "a, b Type" inside func signatures
    for mm in re.finditer(r"\bfunc\b\s*(?:\([^()]*\)\s*)?\w*\s*\(([^()]*(?:\([^()]*\)[^()]*)*)\)", code):
        for part in mm.group(1).split(","):
            toks = part.strip().split()
            if toks and re.fullmatch(r"\w+", toks[0]):
                out.add(toks[0])
    for mm in re.finditer(r"\bfunc\s*\(\s*(\w+)\s", code):
        out.add(mm.group(1))
    return out


def import_errors(files: list) -> list:
    errs = []
    for f in files:
        name = os.path.basename(f.path)
        body = re.sub(r"^import\s*\(.*?^\)", "", f.code, flags=re.M | re.S)
        body = re.sub(r'^import\s+(\w+\s+)?""\s*$', "", body, flags=re.M)
        locs = _locals(body)
        for alias, path in f.imports.items():
            if alias in ("_", ".") or path == "C":
                continue
            if not re.search(r"(?<![\w.])" + re.escape(alias) + r"\.", body):
                errs.append(f'{name}: "{path}" imported and not used')
        for pk in KNOWN_PACKAGES:
            if pk in f.imports or pk in locs:
                continue
            mm = re.search(r"(?<![\w.])" + pk + r"\.[A-Za-z_]", body)
            if mm:
                errs.append(f"{name}:{_line(body, mm.start())}: undefined: {pk} (package used without import)")
    return errs


def header_names(path: str = HEADER) -> set:
    txt = open(path, encoding="utf-8").read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    names = set(re.findall(r"#define\s+(\w+)", txt))
    names |= set(re.findall(r"\b(gpuagg_\w+)\s*\(", txt))  # functions
    names |= set(re.findall(r"typedef\s+struct\s+\w+(?:\s*\{[^}]*\})?\s*(\w+)\s*;", txt, flags=re.S))
    names |= set(re.findall(r"\bstruct\s+(\w+)", txt))
    names |= set(re.findall(r"typedef\s+[\w\s\*]+?\b(\w+)\s*;", txt))
    return names


def cgo_errors(files: list, header: str = HEADER) -> list:
    hdr = header_names(header)
    errs = []
    for f in files:
        if "C" not in f.imports:
            if re.search(r"(?<![\w.])C\.\w", f.code):
                errs.append(f"{os.path.basename(f.path)}: C.* used without import \"C\"")
            continue
        for mm in re.finditer(r"(?<![\w.])C\.(\w+)", f.code):
            nm = mm.group(1)
            if nm in CGO_BUILTINS or nm in C_TYPES or nm in LIBC or nm in hdr:
                continue
            if nm.startswith("sizeof_") and nm[len("sizeof_"):] in hdr | C_TYPES:
                continue
            if nm.startswith("struct_") and nm[len("struct_"):] in hdr:
                continue
            errs.append(f"{os.path.basename(f.path)}:{_line(f.code, mm.start())}: C.{nm} is not in gpuagg.h")
    return errs


# ---- Record vs struct gpuagg_record ---------------------------------------------------
_GO_SIZES = {"uint8": 1, "int8": 1, "uint16": 2, "int16": 2, "uint32": 4, "int32": 4, "float32": 4,
             "uint64": 8, "int64": 8, "float64": 8}
_C_TO_GO = {"uint8_t": "uint8", "int8_t": "int8", "uint16_t": "uint16", "int16_t": "int16", "uint32_t": "uint32",
            "int32_t": "int32", "uint64_t": "uint64", "int64_t": "int64", "float": "float32", "double": "float64"}


def _layout(fields: list) -> tuple:
    """(name, type, offset) with natural alignment, and the padded size."""
    off, out, align = 0, [], 1
    for nm, ty in fields:
        sz = _GO_SIZES[ty]
        off = (off + sz - 1) // sz * sz
        out.append((nm, ty, off))
        off += sz
        align = max(align, sz)
    return out, (off + align - 1) // align * align


def go_struct_fields(files: list, name: str) -> list:
    for f in files:
        mm = re.search(r"^type\s+" + name + r"\s+struct\s*\{(.*?)^\}", f.code, re.M | re.S)
        if not mm:
            continue
        fields = []
        for ln in mm.group(1).splitlines():
            ln = ln.strip()
            if not ln:
                continue
            m2 = re.match(r"([\w\s,]+?)\s+(\w+)$", ln)
            if not m2:
                raise ValueError(f"unparsed field line in {name}: {ln!r}")
            for nm in re.split(r"\s*,\s*", m2.group(1).strip()):
                fields.append((nm, m2.group(2)))
        return fields
    raise KeyError(name)


def c_struct_fields(name: str, header: str = HEADER) -> list:
    txt = re.sub(r"/\*.*?\*/", " ", open(header, encoding="utf-8").read(), flags=re.S)
    mm = re.search(r"typedef\s+struct\s+" + name + r"\s*\{(.*?)\}\s*" + name + r"\s*;", txt, re.S)
    if not mm:
        raise KeyError(name)
    fields = []
    for decl in mm.group(1).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        m2 = re.match(r"(\w+)\s+(.*)", decl, re.S)
        ty = _C_TO_GO[m2.group(1)]
        for nm in re.split(r"\s*,\s*", m2.group(2).strip()):
            fields.append((nm, ty))
    return fields


def _norm(nm: str) -> str:
    return nm.replace("_", "").lower()


def record_layout_errors(files: list, header: str = HEADER) -> list:
    go = _layout(go_struct_fields(files, "Record"))
    cf = c_struct_fields("gpuagg_record", header)
    cl = _layout(cf)
    errs = []
    c_named = [(n, t, o) for n, t, o in cl[0] if not n.endswith("_")]  # pad_ has no Go field
    if [(_norm(n), t, o) for n, t, o in go[0]] != [(_norm(n), t, o) for n, t, o in c_named]:
        errs.append(f"Record fields {go[0]} != gpuagg_record {c_named}")
    if go[1] != cl[1]:
        errs.append(f"Record is {go[1]} bytes, gpuagg_record {cl[1]}")
    return errs


# ---- INTEGRATION.md snippets ----------------------------------------------------------
def exported_names(files: list) -> set:
    out = set()
    for f in files:
        for nm, _ in f.funcs + f.names:
            if nm[:1].isupper():
                out.add(nm)
    return out


def snippet_errors(md_path: str, files: list) -> list:
    txt = open(md_path, encoding="utf-8").read()
    exported = exported_names(files)
    errs = []
    for blk in re.finditer(r"```go\n(.*?)```", txt, re.S):
        code = strip_go(blk.group(1))
        start = _line(txt, blk.start())
        defined = _locals(code) | {m.group(1) for m in re.finditer(r"\bfunc\s+(\w+)", code)}
        for mm in re.finditer(r"(?<![\w.])([a-z_]\w*)\s*\(", code):
            nm = mm.group(1)
            if nm in GO_BUILTINS or nm in GO_KEYWORDS or nm in defined:
                continue
            errs.append(f"INTEGRATION.md:{start + _line(code, mm.start())}: {nm}() is not callable from the "
                        f"producer's package (unexported or undefined)")
        for mm in re.finditer(r"(?<![\w.])gpuagg\.(\w+)", code):
            if mm.group(1) not in exported:
                errs.append(f"INTEGRATION.md:{start + _line(code, mm.start())}: gpuagg.{mm.group(1)} is not "
                            f"exported by go/pkg/gpuagg")
    return errs


def undefined_calls(files: list) -> list:
    """Calls of unexported names the package does not declare: a bare `name(` must be a
    builtin, a local, an import or a package-level declaration of the same build set; a
    selector `.name(` (lowercase: only this package's methods can be unexported) must be
    a method some file of the set declares."""
    errs = []
    for (_, _), fs in build_sets(files).items():
        pkg = {n for f in fs for n, _ in f.funcs + f.names}
        meths = {n for f in fs for _, n, _ in f.methods}
        for f in fs:
            loc = _locals(f.code)
            own = {n for _, n, _ in f.methods}
            for mm in re.finditer(r"(\.?)\b([a-z_]\w*)\s*\(", f.code):
                dot, nm = mm.group(1), mm.group(2)
                if dot:
                    recv = re.search(r"(\w+)\s*$", f.code[:mm.start()])
                    if recv and recv.group(1) == "C":  # cgo names: cgo_errors checks them
                        continue
                    if nm not in meths:
                        errs.append(f"{os.path.basename(f.path)}:{_line(f.code, mm.start())}: .{nm}() is no "
                                    f"method of package {f.package}")
                    continue
                if f.code[max(0, mm.start() - 1):mm.start()] in (".",) or re.search(r"\w$", f.code[:mm.start()]):
                    continue
                if (nm in GO_BUILTINS or nm in GO_KEYWORDS or nm in loc or nm in pkg or nm in f.imports
                        or nm in own):
                    continue
                errs.append(f"{os.path.basename(f.path)}:{_line(f.code, mm.start())}: undefined: {nm}")
    return errs


def struct_fields(files: list) -> dict:
    """type name -> field names (embedded fields by their type name) of the package's structs."""
    out = {}
    for f in files:
        for mm in re.finditer(r"^type\s+(\w+)\s+struct\s*\{(.*?)^\}", f.code, re.M | re.S):
            names = set()
            depth = 0
            for ln in mm.group(2).splitlines():
                t = ln.strip()
                if depth == 0 and t:
                    m2 = re.match(r"([A-Za-z_]\w*(?:\s*,\s*[A-Za-z_]\w*)*)\s+\S", t)
                    if m2:
                        names.update(re.split(r"\s*,\s*", m2.group(1)))
                    else:  # embedded: *pkg.Type or Type
                        m3 = re.match(r"\*?(?:\w+\.)?(\w+)\s*$", t)
                        if m3:
                            names.add(m3.group(1))
                depth += ln.count("{") - ln.count("}")
            out[mm.group(1)] = names
    return out


def selector_errors(files: list) -> list:
    """Inside a method of struct T, `recv.x` must be a field or method of T."""
    errs = []
    fields = struct_fields(files)
    meths: dict = {}
    for f in files:
        for rt, nm, _ in f.methods:
            meths.setdefault(rt, set()).add(nm)
    for f in files:
        heads = [(m.start(), m) for m in re.finditer(r"^func\s+\(\s*(\w+)\s+\*?\s*(\w+)\s*\)", f.code, re.M)]
        starts = sorted([m.start() for m in re.finditer(r"^func\b", f.code, re.M)] + [len(f.code)])
        for pos, m in heads:
            recv, typ = m.group(1), m.group(2)
            if typ not in fields:
                continue
            end = next(x for x in starts if x > pos)
            body = f.code[pos:end]
            allowed = fields[typ] | meths.get(typ, set())
            for sm in re.finditer(r"(?<![\w.])" + recv + r"\.(\w+)", body):
                if sm.group(1) not in allowed:
                    errs.append(f"{os.path.basename(f.path)}:{_line(f.code, pos + sm.start())}: {recv}.{sm.group(1)} "
                                f"undefined (type *{typ} has no field or method {sm.group(1)})")
    return errs


def all_errors() -> list:
    files = load_package()
    return (duplicate_declarations(files) + import_errors(files) + cgo_errors(files) + record_layout_errors(files)
            + undefined_calls(files) + selector_errors(files)
            + snippet_errors(os.path.join(ROOT, "INTEGRATION.md"), files))
