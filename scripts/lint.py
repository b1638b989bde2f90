"""Repository lint (stdlib only, so it runs in the offline image and in CI before any install).

Checks (reference counterpart: .pre-commit-config.yaml + .github/workflows/ci.yml "Quick Lint"):

  * every Python file under tilelang/, tests/, examples/, scripts/, benchmarks/ and the top-level
    entry points parses (``compile``);
  * no tabs, no trailing whitespace, lines <= 120 columns in Python / C++ / HIP sources (the
    column limit is not applied to scripts/: one-off measurement and probe drivers);
  * HIP/C++ sources are gfx950-native: no ``__HIP_PLATFORM_*`` / ``__CUDA_ARCH__`` dual paths, no
    CUDA headers or ``cuda*`` runtime calls, no hipify markers;
  * unused ``import x`` at module top level (names never referenced again; ``__init__`` re-exports
    and ``# noqa`` lines are exempt).

    python scripts/lint.py [paths...]      # exit status 1 on findings
"""
import ast
import os
import re
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
PY_DIRS = ("tilelang", "tests", "examples", "scripts", "benchmarks")
TOP = ("bench.py", "__graft_entry__.py", "setup.py")
CPP_EXT = (".h", ".hpp", ".cpp", ".cc", ".hip")
MAX_COLS = 120
_CUDA = re.compile(r"__HIP_PLATFORM_|__CUDA_ARCH__|#\s*include\s*[<\"]cuda|"
                   r"\bcuda(Malloc|Memcpy|Stream|Launch|Device)\w*\(|hipify|HIPIFY")


def _files(paths):
    if paths:
        for p in paths:
            if os.path.isdir(p):
                for d, _, fs in os.walk(p):
                    for f in fs:
                        yield os.path.join(d, f)
            else:
                yield p
        return
    for t in TOP:
        yield os.path.join(ROOT, t)
    for top in PY_DIRS + ("csrc", ):
        for d, dirs, fs in os.walk(os.path.join(ROOT, top)):
            dirs[:] = [x for x in dirs if x not in ("__pycache__", "build")]
            for f in fs:
                yield os.path.join(d, f)


def _unused_imports(tree, src_lines):
    names = {}
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if "noqa" in src_lines[node.lineno - 1] or getattr(node, "module", None) == "__future__":
                continue
            for a in node.names:
                n = (a.asname or a.name).split(".")[0]
                if n != "*":
                    names[n] = node.lineno
    if not names:
        return []
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            b = node
            while isinstance(b, ast.Attribute):
                b = b.value
            if isinstance(b, ast.Name):
                used.add(b.id)
    allv = set()
    for node in tree.body:  # __all__ re-exports
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            try:
                allv |= set(ast.literal_eval(node.value))
            except ValueError:
                pass
    text = "\n".join(src_lines)
    out = []
    for n, ln in names.items():
        if n in used or n in allv:
            continue
        if re.search(r"[\"']%s[\"']" % re.escape(n), text):  # string references (getattr / __all__)
            continue
        out.append((ln, f"unused import {n!r}"))
    return out


def lint(paths=None):
    problems = []
    for f in _files(paths):
        if not os.path.isfile(f):
            continue
        py = f.endswith(".py")
        cpp = f.endswith(CPP_EXT)
        if not (py or cpp):
            continue
        rel = os.path.relpath(f, ROOT)
        try:
            src = open(f, encoding="utf-8").read()
        except UnicodeDecodeError:
            problems.append((rel, 0, "not UTF-8"))
            continue
        lines = src.splitlines()
        for i, l in enumerate(lines, 1):
            if "\t" in l and py:
                problems.append((rel, i, "tab character"))
            if l != l.rstrip():
                problems.append((rel, i, "trailing whitespace"))
            if len(l) > MAX_COLS and not rel.startswith("scripts" + os.sep):
                problems.append((rel, i, f"line longer than {MAX_COLS} columns ({len(l)})"))
        if py:
            try:
                tree = ast.parse(src, filename=f)
            except SyntaxError as e:
                problems.append((rel, e.lineno or 0, f"syntax error: {e.msg}"))
                continue
            if not f.endswith("__init__.py"):
                problems += [(rel, ln, msg) for ln, msg in _unused_imports(tree, lines)]
        else:
            for i, l in enumerate(lines, 1):
                if _CUDA.search(l):
                    problems.append((rel, i, "CUDA / dual-platform construct in gfx950 source"))
    return problems


def main():
    probs = lint(sys.argv[1:])
    for rel, ln, msg in probs:
        print(f"{rel}:{ln}: {msg}")
    print(f"{len(probs)} problem(s)")
    return 1 if probs else 0


if __name__ == "__main__":
    sys.exit(main())
