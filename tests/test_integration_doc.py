"""The cgo shim in INTEGRATION.md cannot be compiled here (no Go toolchain),
so this checks what can be checked without one: every C function the Go
text calls is declared in include/xrs_hip.h with the same number of
arguments, and every C type it names is a type the header defines."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _go_code():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return "\n".join(re.findall(r"```go\n(.*?)```", text, re.S))


def _header():
    text = open(os.path.join(ROOT, "include", "xrs_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def _split_args(s):
    """Top-level comma split of a call's or prototype's argument text."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out]


def _calls(go):
    """(name, argument count) of every C.xrs_* call in the Go text."""
    calls = []
    for m in re.finditer(r"\bC\.(xrs_\w+)\(", go):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(go[i], 0)
            i += 1
        calls.append((m.group(1), len(_split_args(go[m.end():i - 1]))))
    return calls


def _prototypes(h):
    protos = {}
    for m in re.finditer(r"\b(xrs_\w+)\s*\(([^;{}]*?)\)\s*;", h):
        args = m.group(2).strip()
        protos[m.group(1)] = 0 if args in ("", "void") else len(_split_args(args))
    return protos


def test_go_shim_calls_match_the_header():
    go, protos = _go_code(), _prototypes(_header())
    calls = _calls(go)
    assert len({n for n, _ in calls}) >= 15, calls  # the shim binds the whole method set
    for name, n in calls:
        assert name in protos, f"INTEGRATION.md calls C.{name}, which xrs_hip.h does not declare"
        assert n == protos[name], f"C.{name}: {n} arguments in the Go text, {protos[name]} in xrs_hip.h"


def test_go_shim_types_exist_in_the_header():
    go, h = _go_code(), _header()
    for t in set(re.findall(r"\bC\.(xrs_\w+)\b(?!\()", go)):
        assert re.search(rf"\b(struct\s+{t}\b|typedef\b[^;]*\b{t}\s*;)", h), f"C.{t} is not a header type"
