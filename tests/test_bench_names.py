"""bench.py is only executed on the GPU box; catch undefined names in any of
its functions here, on CPU (symtable: every free/global name a function
reads must be a module-level binding or a builtin)."""
import builtins
import os
import symtable

ROOT = os.path.join(os.path.dirname(__file__), "..")


def _walk(tab, out):
    for ch in tab.get_children():
        if ch.get_type() == "function":
            for sym in ch.get_symbols():
                if sym.is_global() and sym.is_referenced():
                    out.append((ch.get_name(), sym.get_name()))
        _walk(ch, out)


def test_bench_has_no_undefined_names():
    path = os.path.join(ROOT, "bench.py")
    top = symtable.symtable(open(path).read(), path, "exec")
    defined = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    defined |= set(dir(builtins))
    refs = []
    _walk(top, refs)
    missing = sorted({(f, n) for f, n in refs if n not in defined})
    assert not missing, "undefined names in bench.py: %s" % missing
