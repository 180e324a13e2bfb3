"""Undefined-name check of the Python entry points (bench.py's GPU-only branches never run on the
CPU suite, so a misspelt name there would first show up on the GPU box)."""
import builtins
import pathlib
import symtable

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
FILES = ["bench.py", "__graft_entry__.py"] + sorted(
    str(p.relative_to(ROOT)) for p in (ROOT / "cryptmpi_2022_amd").glob("*.py"))


def undefined_globals(path: pathlib.Path):
    top = symtable.symtable(path.read_text(), str(path), "exec")
    module_names = set(top.get_identifiers())
    bad = []

    def walk(t):
        for s in t.get_symbols():
            n = s.get_name()
            if s.is_global() and s.is_referenced() and n not in module_names and not hasattr(builtins, n):
                bad.append(f"{path.name}:{t.get_lineno()} {t.get_name()}: {n}")
        for c in t.get_children():
            walk(c)

    walk(top)
    return bad


@pytest.mark.parametrize("rel", FILES)
def test_no_undefined_globals(rel):
    assert undefined_globals(ROOT / rel) == []
