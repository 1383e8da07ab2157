"""Extract the INPUTS and EXPECTED VALUES of the reference's CF grid-mapping
discovery tests into reference_cf_goldens.json (data only, no test code).

Run in the development container (needs /root/reference):

    python tests/golden/make_cf_goldens.py

Sources: tests/gridmapping/test_cfconv.py (GetDatasetGridMappingsTest,
lines 54-330) and tests/gridmapping/test_dataset.py (DatasetGridMappingTest,
lines 38-142, plus tests/sampledata.py:create_s2plus_dataset, which one of
them builds its input with).  For every test method, in source order:

* "inputs": the datasets / arrays the test constructs, as data —
  ``{"Dataset": {"data_vars": {...}, "coords": {...}, "attrs": {...}}}`` with
  every variable ``{"dims": [...], "values": <values>, "attrs": {...}}``;
  values are literals, ``{"linspace": [a, b, n]}``, ``{"zeros": shape}``,
  ``{"random": shape}`` (any seeded values will do) or
  ``{"array": literal, "dtype": name}``; a CRS is ``{"crs": "EPSG:4326"}``,
  ``{"crs_string": s}`` or ``{"crs_cf": attrs}``, its CF encoding
  ``{"to_cf": <crs>}``; attribute assignments after construction are listed
  under "set_attrs";
* "steps", in source order: the discovery calls the test makes on its
  inputs, with literal keyword arguments (``get_dataset_grid_mapping_proxies``,
  ``_find_potential_coord_vars``, ``_is_potential_coord_var``,
  ``GridMapping.from_dataset``) and the name the result is bound to, and every
  assertion as ``{"op": "eq" | "in" | "not_in" | "isinstance" | "true" |
  "false" | "raises", "what": <label>, "value": <literal or spec>}`` where
  <label> names the checked quantity as the test writes it
  (``len(grid_mappings)``, ``grid_mapping.coords.x.name``, ...).

Tests that need data the container lacks (test_from_real_olci's zarr
archive is not in the snapshot; ``XarrayDecodeCfTest`` and
``TestAddSpatialRef`` exercise xarray's and zarr's own behaviour, neither is
installed) are listed under "skipped" with the reason.
"""

from __future__ import annotations

import ast
import json
import math
import os

REF = os.environ.get("XRS_REFERENCE_ROOT", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
MODULES = {"tests/gridmapping/test_cfconv.py": "GetDatasetGridMappingsTest",
           "tests/gridmapping/test_dataset.py": "DatasetGridMappingTest"}
CALLS = {"get_dataset_grid_mapping_proxies", "_find_potential_coord_vars",
         "_is_potential_coord_var", "from_dataset", "to_regular", "create_s2plus_dataset"}


class Unsupported(ValueError):
    pass


def dotted(node) -> str:
    if isinstance(node, ast.Name):
        return node.id
    if isinstance(node, ast.Attribute):
        return dotted(node.value) + "." + node.attr
    raise Unsupported(ast.dump(node))


def spec(node, env):
    """JSON spec of an input expression (see the module docstring)."""
    if isinstance(node, ast.Constant):
        v = node.value
        if isinstance(v, float) and math.isnan(v):
            return {"nan": True}
        return v
    if isinstance(node, (ast.Tuple, ast.List)):
        return [spec(e, env) for e in node.elts]
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
        v = spec(node.operand, env)
        if isinstance(v, (int, float)):
            return -v
    if isinstance(node, ast.BinOp) and isinstance(node.op, ast.Mult):
        a, b = spec(node.left, env), spec(node.right, env)
        if isinstance(a, int) and isinstance(b, int):
            return a * b
    if isinstance(node, ast.Name):
        if node.id in env:
            return env[node.id]
        raise Unsupported(node.id)
    if isinstance(node, ast.Dict):
        return {"dict": [[spec(k, env), spec(v, env)] for k, v in zip(node.keys, node.values)]}
    if isinstance(node, ast.Call):
        f = node.func
        name = f.attr if isinstance(f, ast.Attribute) else getattr(f, "id", None)
        kw = {k.arg: spec(k.value, env) for k in node.keywords}
        args = node.args
        if name == "dict" and not args:
            return {"dict": [[k, v] for k, v in kw.items()]}
        if name == "set" and not args and not kw:
            return {"set": []}
        if name == "linspace":
            return {"linspace": [spec(a, env) for a in args]}
        if name == "zeros":
            return {"zeros": spec(args[0], env)}
        if name in ("random", "rand"):
            return {"random": [spec(a, env) for a in args] if name == "rand"
                    else spec(args[0], env)}
        if name == "reshape" and isinstance(f, ast.Attribute):
            inner = spec(f.value, env)
            shape = spec(args[0], env) if len(args) == 1 else [spec(a, env) for a in args]
            if isinstance(inner, dict) and "random" in inner:
                return {"random": shape}
        if name == "array":
            out = {"array": spec(args[0], env)}
            if "dtype" in kw:
                out["dtype"] = kw["dtype"]
            return out
        if name == "DataArray":
            return {"DataArray": {"values": spec(args[0], env) if args else kw.get("data"),
                                  "dims": kw.get("dims"), "attrs": kw.get("attrs", {"dict": []})}}
        if name == "Dataset":
            return {"Dataset": {"data_vars": spec(args[0], env) if args else kw.get("data_vars"),
                                "coords": kw.get("coords"), "attrs": kw.get("attrs")}}
        if name == "CRS" and len(args) == 1:
            return {"crs": f"EPSG:{spec(args[0], env)}"}
        if name == "from_string":
            return {"crs_string": spec(args[0], env)}
        if name == "from_cf":
            return {"crs_cf": spec(args[0], env)}
        if name == "to_cf" and isinstance(f, ast.Attribute):
            return {"to_cf": spec(f.value, env)}
        if name == "create_s2plus_dataset":
            return env["__s2plus__"]
    if isinstance(node, ast.Attribute):
        if node.attr in ("float32", "float64", "uint32", "int32"):
            return node.attr
    raise Unsupported(ast.unparse(node))


def module_env(tree) -> dict:
    env = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and \
                isinstance(node.targets[0], ast.Name):
            try:
                env[node.targets[0].id] = spec(node.value, env)
            except Unsupported:
                pass
    return env


def s2plus_spec() -> dict:
    tree = ast.parse(open(os.path.join(REF, "tests/sampledata.py")).read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef)
              and n.name == "create_s2plus_dataset")
    env = {}
    for node in fn.body:
        if isinstance(node, ast.Assign):
            env[node.targets[0].id] = spec(node.value, env)
        elif isinstance(node, ast.Return):
            return spec(node.value, env)
    raise Unsupported("create_s2plus_dataset")


def call_entry(target, call, env):
    f = call.func
    name = f.attr if isinstance(f, ast.Attribute) else f.id
    owner = dotted(f.value) if isinstance(f, ast.Attribute) else None
    args = []
    for a in call.args:
        if isinstance(a, ast.Name) and a.id not in env.get("__consts__", ()):
            args.append({"ref": a.id})
        else:
            args.append(spec(a, env))
    kwargs = {k.arg: spec(k.value, env) for k in call.keywords}
    return {"bind": target, "call": name, "on": owner, "args": args, "kwargs": kwargs}


def extract_method(fn, menv):
    env = dict(menv)
    inputs, steps = {}, []
    calls = expect = steps   # one ordered list: calls and the assertions after them
    body = list(fn.body)
    # flatten `with ...:` blocks in source order
    flat = []
    for node in body:
        if isinstance(node, ast.With):
            items = [ast.unparse(i.context_expr) for i in node.items]
            flat.append(("with", items, node))
            flat.extend(("stmt", None, n) for n in node.body)
        else:
            flat.append(("stmt", None, node))
    for kind, items, node in flat:
        if kind == "with":
            if any("assertRaises" in i for i in items):
                exc = node.items[0].context_expr.args[0]
                expect.append({"op": "raises", "what": "the next call", "value": dotted(exc)})
            if any("catch_warnings" in i for i in items):
                calls.append({"capture_warnings": node.items[0].optional_vars.id})
            continue
        if isinstance(node, ast.Assign) and len(node.targets) == 1:
            t = node.targets[0]
            if isinstance(t, ast.Name) and isinstance(node.value, ast.Call):
                f = node.value.func
                name = f.attr if isinstance(f, ast.Attribute) else getattr(f, "id", None)
                if name in CALLS and name != "create_s2plus_dataset":
                    calls.append(call_entry(t.id, node.value, env))
                    continue
                if name == "get" and isinstance(f, ast.Attribute):
                    calls.append({"bind": t.id, "get": {"ref": dotted(f.value)},
                                  "key": spec(node.value.args[0], env)})
                    continue
            if isinstance(t, ast.Name):
                try:
                    env[t.id] = spec(node.value, env)
                    inputs[t.id] = env[t.id]
                except Unsupported:
                    pass
                continue
            if isinstance(t, ast.Tuple):   # lat, lon = xr.broadcast(lat, lon): not needed here
                continue
            if isinstance(t, ast.Subscript) and isinstance(t.value, ast.Attribute) and \
                    t.value.attr == "attrs":   # dataset["lat"].attrs["bounds"] = "lat_bounds"
                var = t.value.value
                inputs.setdefault("__set_attrs__", []).append(
                    [dotted(var.value), spec(var.slice, env), spec(t.slice, env),
                     spec(node.value, env)])
                continue
        if isinstance(node, ast.Expr) and isinstance(node.value, ast.Call):
            c = node.value
            f = c.func
            name = f.attr if isinstance(f, ast.Attribute) else getattr(f, "id", None)
            owner = f.value.id if isinstance(f, ast.Attribute) and \
                isinstance(f.value, ast.Name) else None
            if owner == "self" and name in ("assertEqual", "assertIn", "assertNotIn",
                                            "assertIsInstance", "assertTrue", "assertFalse"):
                a = c.args
                if name == "assertEqual":
                    try:
                        v, what = spec(a[0], env), a[1]
                    except Unsupported:
                        v, what = spec(a[1], env), a[0]
                    expect.append({"op": "eq", "what": ast.unparse(what), "value": v})
                elif name in ("assertIn", "assertNotIn"):
                    expect.append({"op": "in" if name == "assertIn" else "not_in",
                                   "what": ast.unparse(a[1]), "value": spec(a[0], env)})
                elif name == "assertIsInstance":
                    expect.append({"op": "isinstance", "what": ast.unparse(a[0]),
                                   "value": dotted(a[1])})
                elif name in ("assertTrue", "assertFalse"):
                    inner = a[0]
                    if isinstance(inner, ast.Call) and \
                            getattr(inner.func, "id", getattr(inner.func, "attr", "")) in CALLS:
                        calls.append(call_entry("__value__", inner, env))
                        what = "__value__"
                    else:
                        what = ast.unparse(inner)
                    expect.append({"op": "true" if name == "assertTrue" else "false",
                                   "what": what, "value": None})
                continue
            if name in CALLS:   # a call whose result is discarded (inside assertRaises)
                calls.append(call_entry(None, c, env))
                continue
    return {"inputs": inputs, "steps": steps}


def main():
    out = {"skipped": {}}
    s2 = s2plus_spec()
    for rel, cls_name in MODULES.items():
        tree = ast.parse(open(os.path.join(REF, rel)).read())
        menv = module_env(tree)
        menv["__s2plus__"] = s2
        menv["__consts__"] = [k for k in menv if k.isupper()]
        cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls_name)
        mod = {}
        for fn in [n for n in cls.body if isinstance(n, ast.FunctionDef)
                   and n.name.startswith("test_")]:
            if fn.name == "test_from_real_olci":
                out["skipped"][f"{rel}::{fn.name}"] = (
                    "its input, examples/inputdata/S3-OLCI-L2A.zarr.zip, is not in the "
                    "reference snapshot (and zarr is not installed)")
                continue
            try:
                mod[fn.name] = dict(line=fn.lineno, **extract_method(fn, menv))
            except (Unsupported, KeyError, AttributeError, IndexError) as e:
                out["skipped"][f"{rel}::{fn.name}"] = f"not expressible as data: {e}"
        out[rel] = {"constants": {k: v for k, v in menv.items()
                                  if k.isupper() and not k.startswith("__")},
                    "tests": mod}
    out["skipped"]["tests/gridmapping/test_cfconv.py::XarrayDecodeCfTest"] = \
        "checks xarray's own decode_cf behaviour on a zarr store (xarray, zarr absent)"
    out["skipped"]["tests/gridmapping/test_cfconv.py::TestAddSpatialRef"] = \
        "add_spatial_ref writes a zarr store (zarr absent; not on the hot path)"
    path = os.path.join(HERE, "reference_cf_goldens.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    for rel in MODULES:
        t = out[rel]["tests"]
        print(rel, len(t), "tests,", sum(1 for v in t.values() for e in v["steps"] if "op" in e),
              "expectations")
    print("skipped:", json.dumps(out["skipped"], indent=1))


if __name__ == "__main__":
    main()
