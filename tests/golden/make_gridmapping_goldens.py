"""Extract the EXPECTED VALUES of the reference's GridMapping / helper unit
tests into reference_gridmapping_goldens.json (data only, no test code).

Run in the development container (needs /root/reference):

    python tests/golden/make_gridmapping_goldens.py

For every test method of the modules below, in source order:

* every assertion with a literal on one side —
  ``self.assertEqual / assertAlmostEqual / assertTrue / assertFalse`` and
  ``np.testing.assert_almost_equal / assert_array_equal / assert_allclose`` —
  becomes ``{"what": <label>, "expected": <literal>, "almost": bool, "n": k}``
  where <label> names the checked quantity as the test writes it (e.g.
  ``gm.size``, ``gm1.ij_transform_to(gm2)``) and k counts earlier entries with
  the same label in that method (a label re-checked after a reassignment);
* calls of the test class's own helpers with literal arguments
  (``_assert_coord_vars``, ``assertMatrixPoint``, ``_assert_values``) record
  the literal arguments; ``values = [...]`` tables handed to
  ``_assert_values`` and the literal arguments of ``round_to_fraction``
  inside an inner ``def f(value)`` are recorded with them.

Literals: numbers, strings, bools, None, tuples / lists, ``np.array(...)``,
``Fraction(n, d)`` (stored as {"fraction": [n, d]}), ``nan``, and +,-,*,/ of
number literals.  Our tests (tests/test_gridmapping_goldens_cpu.py) build the
same inputs with the engine's API and compare every recorded value.
"""

from __future__ import annotations

import ast
import json
import math
import os

REF = os.environ.get("XRS_REFERENCE_ROOT", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
MODULES = ["tests/gridmapping/test_helpers.py", "tests/gridmapping/test_coords.py",
           "tests/gridmapping/test_regular.py", "tests/gridmapping/test_base.py",
           "tests/gridmapping/test_transform.py"]
SELF_ASSERTS = {"assertEqual": False, "assertAlmostEqual": True, "assertTupleEqual": False}
NP_ASSERTS = {"assert_almost_equal": True, "assert_array_equal": False, "assert_allclose": True,
              "assert_equal": False,
              "assert_array_almost_equal": True}
HELPERS = {"_assert_coord_vars", "assertMatrixPoint", "_assert_values"}


class NotLiteral(ValueError):
    pass


def lit(node, env):
    if isinstance(node, ast.Constant) and isinstance(node.value, (int, float, str, bool,
                                                                  type(None))):
        return node.value
    if isinstance(node, (ast.Tuple, ast.List)):
        return [lit(e, env) for e in node.elts]
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, (ast.USub, ast.UAdd)):
        v = lit(node.operand, env)
        return -v if isinstance(node.op, ast.USub) else v
    if isinstance(node, ast.BinOp) and isinstance(node.op, (ast.Add, ast.Sub, ast.Mult,
                                                            ast.Div)):
        a, b = lit(node.left, env), lit(node.right, env)
        if not all(isinstance(v, (int, float)) and not isinstance(v, bool) for v in (a, b)):
            raise NotLiteral()
        return {ast.Add: a + b, ast.Sub: a - b, ast.Mult: a * b,
                ast.Div: a / b if b else math.nan}[type(node.op)]
    if isinstance(node, ast.Call):
        fn = node.func
        name = fn.attr if isinstance(fn, ast.Attribute) else getattr(fn, "id", None)
        if name == "array" and node.args:
            return lit(node.args[0], env)
        if name == "Fraction" and len(node.args) == 2:
            return {"fraction": [lit(node.args[0], env), lit(node.args[1], env)]}
        if name == "dict" and not node.args:
            return {k.arg: lit(k.value, env) for k in node.keywords}
        if name == "float" and len(node.args) == 1 and \
                isinstance(node.args[0], ast.Constant) and node.args[0].value == "nan":
            return math.nan
    if isinstance(node, ast.Attribute) and node.attr == "nan":
        return math.nan
    if isinstance(node, ast.Name) and node.id in env:
        return env[node.id]
    raise NotLiteral()


def try_lit(node, env):
    try:
        return True, lit(node, env)
    except NotLiteral:
        return False, None


def jsonable(v):
    if isinstance(v, float) and math.isnan(v):
        return {"nan": True}
    if isinstance(v, list):
        return [jsonable(x) for x in v]
    if isinstance(v, dict):
        return {k: jsonable(x) for k, x in v.items()}
    return v


def extract_method(fn):
    env, out, counts = {}, [], {}

    def add(entry):
        key = entry["what"]
        entry["n"] = counts.get(key, 0)
        counts[key] = entry["n"] + 1
        entry["expected"] = jsonable(entry.get("expected"))
        out.append(entry)

    inner_args = {}
    for node in fn.body:
        if isinstance(node, ast.FunctionDef):   # def f(value): return float(round_to_fraction(value, D, R))
            for c in ast.walk(node):
                if isinstance(c, ast.Call) and getattr(c.func, "id", None) == "round_to_fraction":
                    ok, args = try_lit(ast.Tuple(elts=c.args[1:], ctx=ast.Load()), env)
                    if ok:
                        inner_args[node.name] = args
    if inner_args:
        out.append({"what": "__inner_fn_args__", "expected": inner_args, "n": 0, "line": fn.lineno})

    for node in ast.walk(fn):
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and \
                isinstance(node.targets[0], ast.Name):
            ok, v = try_lit(node.value, env)
            if ok:
                env[node.targets[0].id] = v
    calls = sorted((n for n in ast.walk(fn) if isinstance(n, ast.Call)),
                   key=lambda n: (n.lineno, n.col_offset))
    for c in calls:
        f = c.func
        name = f.attr if isinstance(f, ast.Attribute) else None
        owner = f.value if isinstance(f, ast.Attribute) else None
        is_self = isinstance(owner, ast.Name) and owner.id == "self"
        if is_self and name in SELF_ASSERTS and len(c.args) >= 2:
            ok0, v0 = try_lit(c.args[0], env)
            ok1, v1 = try_lit(c.args[1], env)
            if ok0 == ok1:
                continue
            exp, other = (v0, c.args[1]) if ok0 else (v1, c.args[0])
            add({"what": ast.unparse(other), "expected": exp, "almost": SELF_ASSERTS[name],
                 "line": c.lineno})
        elif is_self and name in ("assertTrue", "assertFalse") and c.args:
            add({"what": ast.unparse(c.args[0]), "expected": name == "assertTrue",
                 "almost": False, "line": c.lineno})
        elif name in NP_ASSERTS and len(c.args) >= 2:
            ok0, v0 = try_lit(c.args[0], env)
            ok1, v1 = try_lit(c.args[1], env)
            if ok0 == ok1:
                continue
            exp, other = (v0, c.args[1]) if ok0 else (v1, c.args[0])
            add({"what": ast.unparse(other), "expected": exp, "almost": NP_ASSERTS[name],
                 "line": c.lineno})
        elif is_self and name in HELPERS:
            args = []
            for a in c.args:
                ok, v = try_lit(a, env)
                args.append(v if ok else {"expr": ast.unparse(a)})
            add({"what": name, "expected": args, "almost": True, "line": c.lineno})
    return out


def main():
    out = {}
    for rel in MODULES:
        tree = ast.parse(open(os.path.join(REF, rel)).read())
        mod = {}
        for cls in [n for n in tree.body if isinstance(n, ast.ClassDef)]:
            for fn in [n for n in cls.body if isinstance(n, ast.FunctionDef)
                       and n.name.startswith("test_")]:
                entries = extract_method(fn)
                if entries:
                    mod[f"{cls.name}.{fn.name}"] = entries
        out[rel] = mod
    path = os.path.join(HERE, "reference_gridmapping_goldens.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    for k, v in out.items():
        print(k, len(v), "tests,", sum(len(x) for x in v.values()), "expected values")


if __name__ == "__main__":
    main()
