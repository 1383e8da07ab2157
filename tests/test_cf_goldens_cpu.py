"""CF grid-mapping discovery pinned to the reference's own tests (SURVEY §8
(f3); reference gridmapping/cfconv.py:66-305, dataset.py:31-102).

tests/golden/reference_cf_goldens.json holds, as data, the inputs every test
of tests/gridmapping/test_cfconv.py (GetDatasetGridMappingsTest) and
tests/gridmapping/test_dataset.py (DatasetGridMappingTest) builds, the
discovery calls it makes and every value it asserts (make_cf_goldens.py).
Here the same inputs are built with the engine's Dataset / DataArray / CRS,
the engine's functions are called the same way, and every recorded assertion
is checked.  CRS CF attributes the reference takes from pyproj's
``CRS.to_cf()`` come from the engine's own CRS registry (pyproj is absent);
the discovery logic under test is what reads them.  Labels are evaluated by
a small attribute / len / str / subscript / to_string() interpreter
(no eval)."""

from __future__ import annotations

import ast
import json
import os
import warnings

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_cf_goldens.json")


def _load():
    with open(GOLDEN) as f:
        return json.load(f)


def _cases():
    g = _load()
    out = []
    for rel in ("tests/gridmapping/test_cfconv.py", "tests/gridmapping/test_dataset.py"):
        for name, case in g[rel]["tests"].items():
            out.append(pytest.param(rel, name, case, id=f"{os.path.basename(rel)}::{name}"))
    return out


# ---- building inputs from their specs ---------------------------------------------
def _crs(spec):
    from xcube_resampling_amd.crs import CRS

    if "crs" in spec:
        return CRS.from_string(spec["crs"])
    if "crs_string" in spec:
        return CRS.from_string(spec["crs_string"])
    if "crs_cf" in spec:
        return CRS.from_cf(build(spec["crs_cf"]))
    raise KeyError(spec)


def build(spec, rng=None):
    """numpy / engine objects for a JSON input spec."""
    import xcube_resampling_amd as xrs

    rng = rng or np.random.default_rng(1)
    if isinstance(spec, list):
        return [build(s, rng) for s in spec]
    if not isinstance(spec, dict):
        return spec
    if "dict" in spec:
        return {k: build(v, rng) for k, v in spec["dict"]}
    if "set" in spec:
        return set(build(spec["set"], rng))
    if "nan" in spec:
        return float("nan")
    if "linspace" in spec:
        return np.linspace(*spec["linspace"])
    if "zeros" in spec:
        return np.zeros(tuple(spec["zeros"]))
    if "random" in spec:
        shape = spec["random"]
        return rng.random(tuple(shape) if isinstance(shape, list) else (shape,))
    if "array" in spec:
        return np.array(build(spec["array"], rng), dtype=spec.get("dtype"))
    if "to_cf" in spec:
        return _crs(spec["to_cf"]).to_cf()
    if any(k in spec for k in ("crs", "crs_string", "crs_cf")):
        return _crs(spec)
    if "DataArray" in spec:
        d = spec["DataArray"]
        values = np.asarray(build(d["values"], rng))
        dims = d["dims"]
        if dims is None:
            dims = tuple(f"dim_{i}" for i in range(values.ndim))
        return xrs.DataArray(values, dims, build(d["attrs"], rng) or {})
    if "Dataset" in spec:
        d = spec["Dataset"]

        def var(v):
            v = build(v, rng)
            if isinstance(v, list):   # ("dims", values) tuple form
                return (v[0], np.asarray(v[1]))
            return v

        dv = {k: var(v) for k, v in (build_items(d["data_vars"]))}
        co = {k: var(v) for k, v in (build_items(d["coords"]))}
        return xrs.Dataset(data_vars=dv, coords=co, attrs=build(d["attrs"], rng) or {})
    raise KeyError(f"unknown spec {list(spec)}")


def build_items(spec):
    if spec is None:
        return []
    return spec["dict"]


# ---- the label interpreter ----------------------------------------------------------
def evaluate(label: str, ns: dict):
    node = ast.parse(label, mode="eval").body

    def ev(n):
        if isinstance(n, ast.Name):
            return ns[n.id]
        if isinstance(n, ast.Constant):
            return n.value
        if isinstance(n, ast.Attribute):
            return getattr(ev(n.value), n.attr)
        if isinstance(n, ast.Subscript):
            return ev(n.value)[ev(n.slice)]
        if isinstance(n, ast.Call) and isinstance(n.func, ast.Name) and \
                n.func.id in ("len", "str") and len(n.args) == 1 and not n.keywords:
            return {"len": len, "str": str}[n.func.id](ev(n.args[0]))
        if isinstance(n, ast.Call) and isinstance(n.func, ast.Attribute) and \
                n.func.attr in ("to_string",) and not n.args and not n.keywords:
            return getattr(ev(n.func.value), n.func.attr)()
        if isinstance(n, ast.JoinedStr):
            return "".join(str(ev(v.value)) if isinstance(v, ast.FormattedValue) else v.value
                           for v in n.values)
        raise ValueError(f"label form not supported: {ast.dump(n)}")

    return ev(node)


def _isinstance(obj, name: str) -> bool:
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd.gridmapping import dataset as D

    types = {"GridMappingProxy": D._GridMappingProxy, "GridCoords": D._GridCoords,
             "xr.DataArray": xrs.DataArray}
    return isinstance(obj, types[name])


def _same(actual, expected) -> bool:
    if isinstance(expected, list) and isinstance(actual, tuple):
        return tuple(_same_norm(e) for e in expected) == tuple(_same_norm(a) for a in actual)
    return actual == expected


def _same_norm(v):
    return tuple(v) if isinstance(v, list) else v


def _call(step, ns):
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd.gridmapping import dataset as D

    fn = {"get_dataset_grid_mapping_proxies": D.get_dataset_grid_mapping_proxies,
          "_find_potential_coord_vars": D._find_potential_coord_vars,
          "_is_potential_coord_var": D._is_potential_coord_var}.get(step["call"])
    if step["call"] == "from_dataset":
        assert step["on"] == "GridMapping"
        fn = xrs.GridMapping.from_dataset
    elif step["call"] == "to_regular":
        return ns[step["on"]].to_regular(**{k: build(v) for k, v in step["kwargs"].items()})
    args = [ns[a["ref"]] if isinstance(a, dict) and "ref" in a else build(a)
            for a in step["args"]]
    return fn(*args, **{k: build(v) for k, v in step["kwargs"].items()})


@pytest.mark.parametrize("rel,name,case", _cases())
def test_reference_cf_discovery(rel, name, case):
    g = _load()
    if f"{rel}::{name}" in g["skipped"]:
        pytest.skip(g["skipped"][f"{rel}::{name}"])
    ns = {k: build(v) for k, v in case["inputs"].items() if not k.startswith("__")}
    for var, key, attr, value in case["inputs"].get("__set_attrs__", []):
        ns[var][key].attrs[attr] = value
    n_checked = 0
    pending_raise = None
    capture = None
    for step in case["steps"]:
        if "capture_warnings" in step:
            capture = step["capture_warnings"]
            continue
        if step.get("op") == "raises":
            pending_raise = step["value"]
            continue
        if "call" in step:
            if pending_raise is not None:
                exc_type = {"ValueError": ValueError}[pending_raise]
                with pytest.raises(exc_type) as info:
                    _call(step, ns)
                ns["cm"] = type("cm", (), {"exception": info.value})
                pending_raise = None
            elif capture is not None:
                with warnings.catch_warnings(record=True) as w:
                    warnings.simplefilter("always")
                    result = _call(step, ns)
                ns[capture] = w
                capture = None
                if step["bind"]:
                    ns[step["bind"]] = result
            else:
                result = _call(step, ns)
                if step["bind"]:
                    ns[step["bind"]] = result
            continue
        if "get" in step:
            ns[step["bind"]] = ns[step["get"]["ref"]].get(step["key"])
            continue
        op, what = step["op"], step["what"]
        actual = evaluate(what, ns)
        msg = f"{name}: {what}"
        if op == "eq":
            exp = build(step["value"])
            assert _same(actual, exp), f"{msg}: {actual!r} != {exp!r}"
        elif op == "in":
            assert build(step["value"]) in actual, f"{msg}: {step['value']!r} not in {actual!r}"
        elif op == "not_in":
            assert build(step["value"]) not in actual, f"{msg}: {step['value']!r} in {actual!r}"
        elif op == "isinstance":
            assert _isinstance(actual, step["value"]), f"{msg}: {type(actual)}"
        elif op in ("true", "false"):
            assert bool(actual) == (op == "true"), msg
        n_checked += 1
    assert n_checked > 0


def test_goldens_cover_the_reference_tests():
    """Every GetDatasetGridMappingsTest / DatasetGridMappingTest method is
    either recorded or listed as skipped with its reason."""
    g = _load()
    cf = g["tests/gridmapping/test_cfconv.py"]["tests"]
    ds = g["tests/gridmapping/test_dataset.py"]["tests"]
    assert len(cf) == 12 and len(ds) == 4
    assert "tests/gridmapping/test_dataset.py::test_from_real_olci" in g["skipped"]
    n = sum(1 for t in list(cf.values()) + list(ds.values()) for s in t["steps"] if "op" in s)
    assert n >= 100
