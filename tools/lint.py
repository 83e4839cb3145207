#!/usr/bin/env python3
"""Minimal, dependency-free lint of the Python sources (the CI lint step).

The reference runs flake8 in CI (/root/reference/tox.ini:4-5, peteris.yaml:1-16).
flake8 is not installed in this image, so this checker implements the subset of
its rules the project relies on, with flake8's codes, on the stdlib ``ast`` /
``tokenize`` modules.  ``tox.ini`` carries the equivalent ``[flake8]`` section for
environments that have flake8.

  E999  syntax error
  F401  module imported but unused (module scope; ``__init__.py`` exempt)
  F811  redefinition of an unused import
  E722  bare ``except:``
  E501  line longer than max-line-length (120)
  W291  trailing whitespace
  W191  indentation contains tabs
  W292  no newline at end of file

``# noqa`` (optionally ``# noqa: CODE``) on a line silences it.

Usage:  python tools/lint.py [paths...]   (default: the package, tests, tools, top-level *.py)
Exit status 1 when anything is reported.
"""

from __future__ import annotations

import ast
import io
import os
import re
import sys
import tokenize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_LINE = 120
DEFAULT_PATHS = ["fast_tffm_amd", "tests", "tools", "bench.py", "run.py", "run_tffm.py", "setup.py",
                 "__graft_entry__.py"]
_NOQA = re.compile(r"#\s*noqa(?::\s*([A-Z0-9, ]+))?", re.I)


def _noqa(line: str, code: str) -> bool:
    m = _NOQA.search(line)
    if not m:
        return False
    codes = m.group(1)
    return codes is None or code in {c.strip().upper() for c in codes.split(",")}


class _Imports(ast.NodeVisitor):
    """Module-level imports and every name / attribute root used anywhere."""

    def __init__(self):
        self.imported: dict[str, int] = {}   # bound name -> line
        self.redef: list[tuple[str, int]] = []
        self.used: set[str] = set()
        self.exported: set[str] = set()

    def bind(self, name: str, line: int) -> None:
        if name in self.imported and name.split(".")[0] not in self.used:
            self.redef.append((name, line))
        self.imported[name] = line

    def visit_Module(self, node):
        for stmt in node.body:
            if isinstance(stmt, ast.Import):
                for a in stmt.names:  # `import a.b` binds `a`; keyed by the dotted name (a.b, a.c differ)
                    self.bind(a.asname or a.name, stmt.lineno)
            elif isinstance(stmt, ast.ImportFrom) and stmt.module != "__future__":
                for a in stmt.names:
                    if a.name != "*":
                        self.bind(a.asname or a.name, stmt.lineno)
            elif isinstance(stmt, ast.Assign):
                for t in stmt.targets:
                    if isinstance(t, ast.Name) and t.id == "__all__" and isinstance(stmt.value, (ast.List, ast.Tuple)):
                        self.exported |= {e.value for e in stmt.value.elts if isinstance(e, ast.Constant)}
        self.generic_visit(node)

    def visit_Name(self, node):
        self.used.add(node.id)

    def visit_Attribute(self, node):
        self.generic_visit(node)

    def visit_Constant(self, node):  # names used in string annotations
        if isinstance(node.value, str) and node.value.isidentifier():
            self.used.add(node.value)
        elif isinstance(node.value, str) and re.fullmatch(r"[\w.\[\], |]+", node.value or ""):
            self.used |= set(re.findall(r"[A-Za-z_]\w*", node.value))


def lint_file(path: str) -> list[str]:
    out = []
    with open(path, "rb") as f:
        raw = f.read()
    text = raw.decode("utf-8", "replace")
    lines = text.splitlines()
    try:
        tree = ast.parse(text, filename=path)
    except SyntaxError as e:
        return [f"{path}:{e.lineno}:{e.offset}: E999 {e.msg}"]
    for i, ln in enumerate(lines, 1):
        if len(ln) > MAX_LINE and not _noqa(ln, "E501"):
            out.append(f"{path}:{i}:{MAX_LINE + 1}: E501 line too long ({len(ln)} > {MAX_LINE} characters)")
        if ln.rstrip() != ln and not _noqa(ln, "W291"):
            out.append(f"{path}:{i}:{len(ln.rstrip()) + 1}: W291 trailing whitespace")
        if ln[: len(ln) - len(ln.lstrip())].count("\t") and not _noqa(ln, "W191"):
            out.append(f"{path}:{i}:1: W191 indentation contains tabs")
    if raw and not raw.endswith(b"\n"):
        out.append(f"{path}:{len(lines)}:1: W292 no newline at end of file")
    # docstrings / strings spanning lines are not code: tokenize to find comment lines for noqa only
    try:
        list(tokenize.generate_tokens(io.StringIO(text).readline))
    except (tokenize.TokenError, IndentationError) as e:
        out.append(f"{path}:1:1: E902 {e}")
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            if not _noqa(lines[node.lineno - 1], "E722"):
                out.append(f"{path}:{node.lineno}:1: E722 do not use bare 'except'")
    if os.path.basename(path) != "__init__.py":
        v = _Imports()
        v.visit(tree)
        for name, line in sorted(v.imported.items(), key=lambda kv: kv[1]):
            if name.split(".")[0] not in v.used and name not in v.exported and not _noqa(lines[line - 1], "F401"):
                out.append(f"{path}:{line}:1: F401 '{name}' imported but unused")
        for name, line in v.redef:
            if not _noqa(lines[line - 1], "F811"):
                out.append(f"{path}:{line}:1: F811 redefinition of unused '{name}'")
    return out


def iter_files(paths: list[str]):
    for p in paths:
        p = os.path.join(ROOT, p) if not os.path.isabs(p) else p
        if os.path.isfile(p) and p.endswith(".py"):
            yield p
        elif os.path.isdir(p):
            for d, dirs, files in os.walk(p):
                dirs[:] = [x for x in dirs if not x.startswith(".") and x != "__pycache__"]
                for f in sorted(files):
                    if f.endswith(".py"):
                        yield os.path.join(d, f)


def main(argv: list[str] | None = None) -> int:
    paths = (argv if argv is not None else sys.argv[1:]) or DEFAULT_PATHS
    problems = []
    for f in iter_files(paths):
        problems += lint_file(f)
    for p in problems:
        print(os.path.relpath(p, ROOT) if p.startswith(ROOT) else p)
    return 1 if problems else 0


if __name__ == "__main__":
    sys.exit(main())
