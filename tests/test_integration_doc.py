"""INTEGRATION.md's Option B -- the ctypes stub a maintainer of the reference
adds to bind pg_eval_population from ga.py:83 (``toolbox.register("map", ...)``)
-- tested as written: the code block is extracted from the document, its
structures are checked against the C header's offsetof/sizeof (gcc), and its
schedule loop (evaluate()'s six games, main.py:33-53, with
create_model_from_hall_of_fame's in-place shuffles, utils.py:90-101) is run on
a stand-in hall of fame against pong_amd.schedule.  No GPU needed."""
import ast
import ctypes
import os
import random
import re
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = os.path.join(REPO, "INTEGRATION.md")
HEADER = os.path.join(REPO, "include", "pong_ga.h")


def stub_source():
    text = open(DOC).read()
    m = re.search(r"```python\n(# pong_ga_binding\.py.*?)```", text, flags=re.S)
    assert m, "INTEGRATION.md has no pong_ga_binding.py block"
    return m.group(1)


def stub_tree():
    return ast.parse(stub_source())


def stub_structs():
    """Execute the block's constants and class definitions (not its CDLL load)."""
    tree = stub_tree()
    keep = [n for n in tree.body if isinstance(n, ast.ClassDef) or (
        isinstance(n, ast.Assign) and all(isinstance(t, ast.Name) and t.id.startswith("PG_") for t in n.targets))]
    ns = {"ctypes": ctypes}
    exec(compile(ast.Module(body=keep, type_ignores=[]), DOC, "exec"), ns)
    return ns


def test_stub_abi_version_matches_header():
    ns = stub_structs()
    want = int(re.search(r"#define PG_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert ns["PG_ABI_VERSION"] == want
    assert ns["PG_MAX_NODES"] == int(re.search(r"#define PG_MAX_NODES (\d+)", open(HEADER).read()).group(1))


def test_stub_layout_matches_c(tmp_path):
    """Every field of the stub's PgNet / PgEvalArgs at the header's offset, the
    same sizeof, and the same field list as the package's binding."""
    from pong_amd import _lib
    ns = stub_structs()
    structs = {"pg_net": ns["PgNet"], "pg_eval_args": ns["PgEvalArgs"]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(src)])
    c = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        s, f, v = line.split()
        c[(s, f)] = int(v)
    for cname, cls in structs.items():
        assert c[(cname, "size")] == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert c[(cname, fname)] == getattr(cls, fname).offset, f"{cname}.{fname}"
    assert [f for f, _ in ns["PgEvalArgs"]._fields_] == [f for f, _ in _lib.PgEvalArgs._fields_]
    a = ns["PgEvalArgs"]()
    assert a.struct_size == c[("pg_eval_args", "size")], "the stub must fill struct_size (ABI 10)"


def test_stub_struct_is_accepted_by_the_library():
    """The library takes the stub's struct (struct_size matches) and refuses it
    once the size is wrong: argument validation, no device touched."""
    from pong_amd import _lib
    from pong_amd import build as B
    B.build()
    L = _lib.lib()
    ns = stub_structs()
    a = ns["PgEvalArgs"]()
    a.net.n_nodes = 3
    a.net.nodes[:3] = (6, 2, 2)
    a.net.bias, a.net.dtype = 1, 1
    a.n_genomes, a.n_games = 0, 6
    p = ctypes.cast(ctypes.byref(a), ctypes.POINTER(_lib.PgEvalArgs))
    assert L.pg_eval_population(p, None) == _lib.PG_OK
    a.struct_size -= 4
    assert L.pg_eval_population(p, None) == _lib.PG_ERR_INVALID


class _Fitness:
    def __init__(self, v):
        self.valid = v is not None
        self.values = (v,) if v is not None else ()


class _Member(list):
    def __init__(self, genes, fit):
        super().__init__(genes)
        self.fitness = _Fitness(fit)


class _Hof:
    def __init__(self, items):
        self.items = items


def _schedule_from_stub(inds, hof):
    """gpu_map's statements up to the first device call, run on the host."""
    fn = next(n for n in stub_tree().body if isinstance(n, ast.FunctionDef) and n.name == "gpu_map")
    body = []
    for stmt in fn.body:
        if isinstance(stmt, ast.Assign) and "torch" in ast.unparse(stmt.value):
            break
        if isinstance(stmt, ast.Import) or isinstance(stmt, ast.Expr):
            continue  # `import ga` (the stand-in below) and the docstring
        body.append(stmt)
    ns = {"np": np, "random": random, "individuals": inds, "ga": type("ga", (), {"hall_of_fame": hof})}
    exec(compile(ast.Module(body=body, type_ignores=[]), DOC, "exec"), ns)
    return ns["kind"], ns["opp"], ns["mult"], ns["members"]


def test_stub_schedule_equals_package_schedule():
    """The stub's six-game schedule draws the hall-of-fame opponents exactly as
    the package's (and, through utils.pick_hall_of_famer, the reference's
    create_model_from_hall_of_fame): same kinds, rows, multipliers, members."""
    import utils
    from pong_amd import schedule as S
    rng = np.random.default_rng(3)
    inds = [list(rng.standard_normal(20)) for _ in range(9)]
    for items in ([], [(rng.standard_normal(20), f) for f in (0.5, None, -2.0, 3.25, None)],
                  [(rng.standard_normal(20), None)]):
        members_a = [_Member(g, f) for g, f in items]
        members_b = [_Member(g, f) for g, f in items]
        random.seed(11)
        k1, o1, m1, mem1 = _schedule_from_stub(inds, _Hof(members_a))
        random.seed(11)
        k2, o2, m2, mem2 = S.reference_schedule(len(inds), 6, _Hof(members_b), utils.pick_hall_of_famer)
        assert np.array_equal(k1, k2) and np.array_equal(o1, o2) and np.array_equal(m1, m2)
        assert [list(m) for m in mem1] == [list(m) for m in mem2]
