#!/usr/bin/env python3
"""Source lint for the repo (the CI `lint` job; analogue of the reference's
`make test_lint test_fmt`, Makefile + .travis.yml:6): stdlib only, so it runs
in the offline image.

Python (drynx_amd/, tests/, tools/, top-level scripts):
  * syntax (compile), no tabs, no trailing whitespace, lines <= 120 chars;
  * unused imports (a name bound by `import` that the module never reads,
    ignoring `__init__` re-exports, `noqa` lines and `__future__`).
HIP/C++ (csrc/): no tabs, no trailing whitespace, lines <= 150 chars, and no
CUDA spellings (this is a gfx950-only code base: no cuda* API, no
__HIP_PLATFORM_* dual paths).

Exit status 1 when anything is found; `--quiet` prints only the count."""
from __future__ import annotations

import ast
import os
import re
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
MAX_LEN = 120       # Python
MAX_LEN_CPP = 150   # HIP/C++ (kernel launch lines)
PY_DIRS = ("drynx_amd", "tests", "tools")
PY_TOP = ("bench.py", "__graft_entry__.py")
CUDA_RE = re.compile(r"\bcuda[A-Z]\w*\(|__HIP_PLATFORM_|#include\s*<cuda")


def _py_files():
    for d in PY_DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            if "__pycache__" in dp:
                continue
            for f in sorted(fs):
                if f.endswith(".py"):
                    yield os.path.join(dp, f)
    for f in PY_TOP:
        yield os.path.join(ROOT, f)


def _cpp_files():
    for dp, _, fs in os.walk(os.path.join(ROOT, "csrc")):
        for f in sorted(fs):
            if f.endswith((".h", ".hip", ".cpp")) and f != "constants.h":  # constants.h is generated
                yield os.path.join(dp, f)


def _text_checks(path, text, out, max_len=MAX_LEN):
    for i, line in enumerate(text.splitlines(), 1):
        if "\t" in line:
            out.append(f"{path}:{i}: tab")
        if line != line.rstrip():
            out.append(f"{path}:{i}: trailing whitespace")
        if len(line) > max_len:
            out.append(f"{path}:{i}: line longer than {max_len}")


def _unused_imports(path, tree, text, out):
    if os.path.basename(path) == "__init__.py":
        return
    lines = text.splitlines()
    bound = {}
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            if "noqa" in lines[node.lineno - 1]:
                continue
            for a in node.names:
                name = (a.asname or a.name).split(".")[0]
                bound.setdefault(name, node.lineno)
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            base = node
            while isinstance(base, ast.Attribute):
                base = base.value
            if isinstance(base, ast.Name):
                used.add(base.id)
    dunder_all = re.search(r"__all__\s*=", text) is not None
    for name, ln in bound.items():
        if name not in used and not (dunder_all and f'"{name}"' in text):
            out.append(f"{os.path.relpath(path, ROOT)}:{ln}: unused import {name}")


def main() -> int:
    out: list = []
    for p in _py_files():
        text = open(p, encoding="utf-8").read()
        rel = os.path.relpath(p, ROOT)
        try:
            tree = ast.parse(text, p)
        except SyntaxError as e:
            out.append(f"{rel}:{e.lineno}: syntax error {e.msg}")
            continue
        _text_checks(rel, text, out)
        _unused_imports(p, tree, text, out)
    for p in _cpp_files():
        text = open(p, encoding="utf-8").read()
        rel = os.path.relpath(p, ROOT)
        _text_checks(rel, text, out, MAX_LEN_CPP)
        for i, line in enumerate(text.splitlines(), 1):
            if CUDA_RE.search(line):
                out.append(f"{rel}:{i}: CUDA spelling in gfx950 code")
    if "--quiet" not in sys.argv:
        for o in out:
            print(o)
    print(f"lint: {len(out)} finding(s)")
    return 1 if out else 0


if __name__ == "__main__":
    sys.exit(main())
