"""Extract the expected arrays of the reference's own unit tests.

Run in the development container (needs /root/reference):

    python tests/golden/make_reference_test_goldens.py

For every test method of the listed reference test modules, every
``np.array(<literal>)`` passed as the EXPECTED argument of
``np.testing.assert_almost_equal`` / ``assert_array_equal`` / ``assert_allclose``
is evaluated (literals only: numbers, nested lists, ``nan``/``np.nan``) and
written in order to reference_test_goldens.json.  Only data is kept — the
expected values and the assertion precision (``decimal=``) — no test code.
Our tests (tests/test_reference_goldens_*.py) re-create each test's inputs and
calls with the engine's API and compare against these arrays.
"""

from __future__ import annotations

import ast
import json
import math
import os

import numpy as np

REF = os.environ.get("XRS_REFERENCE_ROOT", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
MODULES = ["tests/test_affine.py", "tests/test_rectify.py", "tests/test_reproject.py",
           "tests/test_spatial.py", "tests/test_coarsen.py", "tests/gridmapping/test_bboxes.py"]
ASSERTS = {"assert_almost_equal", "assert_array_equal", "assert_allclose",
           "assert_array_almost_equal"}


def _literal(node, consts):
    """Evaluate an expected-value expression made of literals only."""
    if isinstance(node, ast.Call) and getattr(node.func, "attr", None) == "array":
        return _literal(node.args[0], consts)
    if isinstance(node, (ast.List, ast.Tuple)):
        return [_literal(e, consts) for e in node.elts]
    if isinstance(node, ast.Constant) and isinstance(node.value, (int, float)):
        return node.value
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
        return -_literal(node.operand, consts)
    if isinstance(node, ast.Name) and node.id in consts:
        return consts[node.id]
    if isinstance(node, ast.Attribute) and node.attr == "nan":
        return math.nan
    if isinstance(node, ast.Name) and node.id == "nan":
        return math.nan
    raise ValueError(ast.dump(node)[:80])


def _jsonable(v):
    if isinstance(v, list):
        return [_jsonable(x) for x in v]
    if isinstance(v, float) and math.isnan(v):
        return None
    return v


def main():
    out = {}
    for rel in MODULES:
        path = os.path.join(REF, rel)
        tree = ast.parse(open(path).read())
        consts = {}
        for node in tree.body:  # module-level literal arrays, e.g. expected_rad_13x13
            if isinstance(node, ast.Assign) and len(node.targets) == 1 and \
                    isinstance(node.targets[0], ast.Name):
                try:
                    consts[node.targets[0].id] = _literal(node.value, consts)
                except ValueError:
                    pass
        mod = {}
        for cls in [n for n in tree.body if isinstance(n, ast.ClassDef)]:
            for fn in [n for n in cls.body if isinstance(n, ast.FunctionDef)]:
                if fn.name.startswith("expected_"):  # helper returning a literal golden
                    for node in ast.walk(fn):
                        if isinstance(node, ast.Return) and node.value is not None:
                            try:
                                val = _literal(node.value, consts)
                            except ValueError:
                                continue
                            mod.setdefault("__helpers__", {})[fn.name] = _jsonable(
                                np.asarray(val, dtype=float).tolist())
                if not fn.name.startswith("test_"):
                    continue
                local = dict(consts)
                found = []
                for node in ast.walk(fn):
                    if isinstance(node, ast.Assign) and len(node.targets) == 1 and \
                            isinstance(node.targets[0], ast.Name):
                        try:
                            local[node.targets[0].id] = _literal(node.value, local)
                        except ValueError:
                            pass
                calls = [n for n in ast.walk(fn) if isinstance(n, ast.Call)
                         and getattr(n.func, "attr", None) in ASSERTS and len(n.args) >= 2]
                calls.sort(key=lambda n: (n.lineno, n.col_offset))
                for c in calls:
                    try:
                        val = _literal(c.args[1], local)
                    except ValueError:
                        continue
                    dec = next((k.value.value for k in c.keywords if k.arg == "decimal"), 7)
                    found.append({"line": c.lineno, "decimal": dec,
                                  "expected": _jsonable(np.asarray(val, dtype=float).tolist())})
                if found:
                    mod[fn.name] = found
        out[rel] = mod
    with open(os.path.join(HERE, "reference_test_goldens.json"), "w") as f:
        json.dump(out, f, indent=0)
    for k, v in out.items():
        print(k, len(v), "tests,", sum(len(x) for x in v.values()), "expected arrays")


if __name__ == "__main__":
    main()
