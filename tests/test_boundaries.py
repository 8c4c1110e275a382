"""Repository rules that keep the oracle a checker only ("No CPU fallback"):
outside tests/ and oracle/ itself, the only code that may import oracle/ is bench.py's
``cpu_baseline`` (the timed reference CPU leg) and ``__graft_entry__.smoke`` (the checker)."""

import ast
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
ALLOWED = {("bench.py", "cpu_baseline"), ("__graft_entry__.py", "smoke")}


def _oracle_imports(tree):
    """(enclosing top-level function name or None, lineno) of every import of ``oracle``."""
    found = []

    def visit(node, func):
        for child in ast.iter_child_nodes(node):
            f = func
            if isinstance(child, (ast.FunctionDef, ast.AsyncFunctionDef)) and func is None:
                f = child.name
            if isinstance(child, ast.Import) and any(a.name.split(".")[0] == "oracle" for a in child.names):
                found.append((f, child.lineno))
            elif isinstance(child, ast.ImportFrom) and (child.module or "").split(".")[0] == "oracle":
                found.append((f, child.lineno))
            visit(child, f)

    visit(tree, None)
    return found


def test_oracle_imported_only_by_checkers():
    offenders = []
    for path in ROOT.rglob("*.py"):
        rel = path.relative_to(ROOT)
        if rel.parts[0] in ("tests", "oracle") or any(p.startswith(".") for p in rel.parts):
            continue
        for func, line in _oracle_imports(ast.parse(path.read_text())):
            if (str(rel), func) not in ALLOWED:
                offenders.append(f"{rel}:{line} (in {func})")
    assert not offenders, "oracle/ imported outside its checkers: " + ", ".join(offenders)

