"""Static check for names a function reads as globals that its module never defines.

GPU-only branches do not run in the CPU suite.  One of them (bench.py's per-rank memory report)
once read ``torch`` in a module-level helper, while bench.py imports torch inside ``main()``.  That
is a NameError only a GPU run would hit.  ``symtable`` lists every function's global reads, and each
must be a module-level import / assignment / def / class or a builtin."""
import ast
import builtins
import glob
import os
import symtable

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(["bench.py", "__graft_entry__.py"]
               + [os.path.relpath(p, ROOT) for p in glob.glob(os.path.join(ROOT, "distributed_llm_amd", "**", "*.py"),
                                                              recursive=True)])


def _module_names(tree):
    names = set()

    def bind(node):
        for n in ast.walk(node):
            if isinstance(n, (ast.Import, ast.ImportFrom)):
                names.update((a.asname or a.name).split(".")[0] for a in n.names)
            elif isinstance(n, ast.Name) and isinstance(n.ctx, ast.Store):
                names.add(n.id)
            elif isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
                names.add(n.name)

    for node in tree.body:   # module level, including imports under if / try / with / for
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            names.add(node.name)
        else:
            bind(node)
    return names


def _unbound_globals(path):
    src = open(os.path.join(ROOT, path)).read()
    known = _module_names(ast.parse(src)) | set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__"}
    bad = []

    def walk(t):
        if t.get_type() == "function":
            for s in t.get_symbols():
                if s.is_referenced() and s.is_global() and not s.is_declared_global() and s.get_name() not in known:
                    bad.append(f"{path}:{t.get_lineno()} {t.get_name()}() reads undefined global {s.get_name()!r}")
        for c in t.get_children():
            walk(c)

    walk(symtable.symtable(src, path, "exec"))
    return bad


@pytest.mark.parametrize("path", FILES)
def test_functions_read_only_defined_globals(path):
    assert not _unbound_globals(path)


def test_the_check_catches_a_deferred_import():
    import tempfile
    src = "def f():\n    return torch.zeros(1)\n\ndef main():\n    import torch\n    return f()\n"
    with tempfile.NamedTemporaryFile("w", suffix=".py", dir=ROOT, delete=False) as fh:
        fh.write(src)
    try:
        assert _unbound_globals(os.path.relpath(fh.name, ROOT))
    finally:
        os.unlink(fh.name)
