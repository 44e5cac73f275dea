"""Static checks standing in for the reference CI's `pyflakes .` / `pycodestyle` steps
(.travis.yml:25, 36-38; neither tool is installed in this image): every Python file compiles
and no module-level import is unused; package, entry points and tests stay within 110 columns
(scripts/ are one-off measurement tools and exempt from the length rule)."""
import ast
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIRS = ["distributed_char_rnn_amd", "scripts", "tests"]
TOP = ["bench.py", "train.py", "sample.py", "data_splitter.py", "__graft_entry__.py"]


def _files():
    out = [os.path.join(ROOT, f) for f in TOP if os.path.exists(os.path.join(ROOT, f))]
    for d in DIRS:
        for dp, _, fns in os.walk(os.path.join(ROOT, d)):
            if "__pycache__" in dp:
                continue
            out += [os.path.join(dp, f) for f in fns if f.endswith(".py")]
    return sorted(out)


FILES = _files()


def _rel(p):
    return os.path.relpath(p, ROOT)


@pytest.mark.parametrize("path", FILES, ids=_rel)
def test_compiles_and_no_unused_imports(path):
    src = open(path, encoding="utf-8").read()
    tree = ast.parse(src, filename=path)
    compile(tree, path, "exec")
    if os.path.basename(path) == "__init__.py":
        return  # re-exports
    lines = src.splitlines()
    imported = {}
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if "noqa" in lines[node.lineno - 1]:
                continue
            for a in node.names:
                future = isinstance(node, ast.ImportFrom) and node.module == "__future__"
                if a.name == "*" or future:
                    continue
                name = (a.asname or a.name).split(".")[0]
                imported[name] = node.lineno
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
    unused = [f"{n} (line {ln})" for n, ln in imported.items() if n not in used]
    assert not unused, f"{_rel(path)}: unused imports: {unused}"


@pytest.mark.parametrize("path", [f for f in FILES if not _rel(f).startswith("scripts")],
                         ids=_rel)
def test_line_length(path):
    long = [i + 1 for i, line in enumerate(open(path, encoding="utf-8").read().splitlines())
            if len(line) > 110]
    assert not long, f"{_rel(path)}: lines over 110 columns: {long[:10]}"
