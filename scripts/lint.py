"""Self-contained linter (no third-party tools in the build image; reference .golangci.yml, SURVEY.md
§2.1 R29). Python: compiles, no unused imports (ast), no tabs / trailing whitespace, <= 140 columns.
HIP/C++ (csrc/): no tabs / trailing whitespace, <= 140 columns, and the MI355X-only policy:
  * no CUDA compatibility layers (cuda_runtime, __CUDA_ARCH__, __HIP_PLATFORM_* dual paths, hipify).
The scalar-memory policy is enforced on the *built* ISA by an allow-list (scripts/isa_check.py), so
no source file needs to spell out the instructions it rejects.
Usage: python scripts/lint.py [paths...]   (exit 1 on findings)"""
from __future__ import annotations

import ast
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP_DIRS = {".git", "build", "gpurun_out", "__pycache__", ".pytest_cache", ".hypothesis", "node_modules"}
MAX_COL = 140
NATIVE_EXT = (".hip", ".cpp", ".h", ".hpp", ".s")
FORBIDDEN_NATIVE = [
    (re.compile(r"#\s*include\s*[<\"]cuda"), "CUDA header"),
    (re.compile(r"__CUDA_ARCH__|__NVCC__"), "CUDA dual path"),
    (re.compile(r"#\s*if(def)?\s+.*__HIP_PLATFORM_(AMD|NVIDIA)__"), "HIP platform dual path"),
    (re.compile(r"hipify", re.I), "hipify output"),
]


def iter_files(paths):
    for p in paths:
        if os.path.isfile(p):
            yield p
            continue
        for d, subdirs, files in os.walk(p):
            subdirs[:] = [s for s in subdirs if s not in SKIP_DIRS]
            for f in files:
                if f.endswith(".py") or f.endswith(NATIVE_EXT):
                    yield os.path.join(d, f)


def unused_imports(tree: ast.AST, src: str) -> list[tuple[int, str]]:
    imported: dict[str, int] = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            for a in node.names:
                imported[(a.asname or a.name).split(".")[0]] = node.lineno
        elif isinstance(node, ast.ImportFrom) and node.module != "__future__":
            for a in node.names:
                if a.name != "*":
                    imported[a.asname or a.name] = node.lineno
    used = {n.id for n in ast.walk(tree) if isinstance(n, ast.Name)}
    used |= {n.value.id for n in ast.walk(tree) if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name)}
    exported = set()
    for node in ast.walk(tree):  # __all__ = [...] re-exports
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            if isinstance(node.value, (ast.List, ast.Tuple)):
                exported |= {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
    lines = src.splitlines()
    out = []
    for name, ln in imported.items():
        if name in used or name in exported or "noqa" in lines[ln - 1]:
            continue
        if name in src.replace(f"import {name}", ""):  # string annotations / doctest mentions
            if re.search(rf"[\"'][^\"']*\b{re.escape(name)}\b", src):
                continue
        out.append((ln, f"unused import '{name}'"))
    return out


def lint_file(path: str) -> list[str]:
    rel = os.path.relpath(path, ROOT)
    try:
        src = open(path, encoding="utf-8").read()
    except UnicodeDecodeError:
        return [f"{rel}: not UTF-8"]
    msgs = []
    for i, line in enumerate(src.splitlines(), 1):
        if "\t" in line and not path.endswith(".s"):
            msgs.append(f"{rel}:{i}: tab character")
        if line != line.rstrip():
            msgs.append(f"{rel}:{i}: trailing whitespace")
        if len(line) > MAX_COL:
            msgs.append(f"{rel}:{i}: line longer than {MAX_COL} columns ({len(line)})")
    if path.endswith(".py"):
        try:
            tree = ast.parse(src, filename=path)
        except SyntaxError as e:
            return msgs + [f"{rel}:{e.lineno}: syntax error: {e.msg}"]
        if not path.endswith("__init__.py"):
            msgs += [f"{rel}:{ln}: {m}" for ln, m in unused_imports(tree, src)]
    elif path.endswith(NATIVE_EXT):
        for i, line in enumerate(src.splitlines(), 1):
            code = line.split("//")[0]
            for rx, what in FORBIDDEN_NATIVE:
                if rx.search(code if "hipify" not in what else line):
                    msgs.append(f"{rel}:{i}: forbidden ({what})")
    return msgs


def main(argv: list[str]) -> int:
    paths = argv or [os.path.join(ROOT, d) for d in ("ollama_operator_amd", "csrc", "scripts", "tests")] + \
        [os.path.join(ROOT, f) for f in ("bench.py", "build_native.py", "__graft_entry__.py")]
    msgs = [m for f in iter_files(paths) for m in lint_file(f)]
    for m in msgs:
        print(m)
    print(f"lint: {len(msgs)} finding(s)")
    return 1 if msgs else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
