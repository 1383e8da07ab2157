"""Grid-mapping discovery in a dataset (gridmapping/dataset.py:31-102 and the
CF parsing of gridmapping/cfconv.py:66-317, restated for the engine's CRS
registry)."""

from __future__ import annotations

import warnings
from dataclasses import dataclass

from ..crs import CRS, CRS_WGS84, normalize_crs
from .base import DEFAULT_TOLERANCE, GridMapping
from .coords import new_grid_mapping_from_coords


@dataclass
class _GridCoords:
    x: object = None
    y: object = None


@dataclass
class _GridMappingProxy:
    crs: CRS
    name: str | None
    coords: _GridCoords | None = None
    tile_size: tuple[int, int] | None = None


def _parse_crs_from_attrs(attrs) -> _GridMappingProxy | None:
    """cfconv.py:215-221."""
    try:
        crs = CRS.from_cf(dict(attrs))
    except (ValueError, TypeError):
        return None
    return _GridMappingProxy(crs=crs, name=attrs.get("grid_mapping_name"))


def _get_dataset_chunks(dataset) -> dict:
    """helpers.py:113-161 — most common (max) chunk size per dimension."""
    counts: dict = {}
    for var in dataset.data_vars.values():
        if getattr(var, "chunks", None):
            for d, c in zip(var.dims, var.chunks):
                max_c = max(0, *c)
                counts.setdefault(d, {}).setdefault(max_c, 0)
                counts[d][max_c] += 1
    out = {}
    for d, size_counts in counts.items():
        best, best_n = 0, 0
        for max_c, n in size_counts.items():
            if n > best_n:
                best, best_n = max_c, n
        out[d] = best
    return out


def _is_potential_coord_var(dataset, bounds_var_names, var_name) -> bool:
    """cfconv.py:299-305."""
    if var_name in dataset:
        return dataset[var_name].ndim in (1, 2) and var_name not in bounds_var_names
    return False


def _find_potential_coord_vars(dataset) -> list:
    """cfconv.py:254-296: 1-D / 2-D variables that are not bounds variables
    (CF ``bounds`` attribute or a ``<name>_bnds`` / ``<name>_bounds`` name),
    those of the global ``coordinates`` attribute first."""
    bounds_vars = set()
    for k in dataset.variables:
        var = dataset[k]
        bk = var.attrs.get("bounds")
        if bk is not None and bk in dataset:
            bounds_vars.add(bk)
        parts = str(k).rsplit("_", maxsplit=1)
        if len(parts) == 2 and parts[1] in ("bnds", "bounds") and parts[0] in dataset:
            bounds_vars.add(k)
    out = []
    coordinates = dataset.attrs.get("coordinates")
    if coordinates is not None:
        for name in coordinates.split():
            if _is_potential_coord_var(dataset, bounds_vars, name):
                out.append(name)
    for name in dataset.variables:
        if name not in out and _is_potential_coord_var(dataset, bounds_vars, name):
            out.append(name)
    return out


def _complement(coords: _GridCoords, gm_name, missing_crs, proxies: dict):
    """cfconv.py:224-253."""
    if coords.x is None and coords.y is None:
        return
    gm = next((g for g in proxies.values() if gm_name is None or gm_name == g.name), None)
    if gm is None and missing_crs is not None:
        gm = _GridMappingProxy(crs=missing_crs, name=gm_name)
        proxies[None] = gm
    if gm is not None:
        if gm.coords is None:
            gm.coords = coords
        if gm.coords.x is None:
            gm.coords.x = coords.x
        if gm.coords.y is None:
            gm.coords.y = coords.y


def get_dataset_grid_mapping_proxies(dataset, *, missing_latitude_longitude_crs=None,
                                     missing_rotated_latitude_longitude_crs=None,
                                     missing_projected_crs=None, emit_warnings=False) -> dict:
    """cfconv.py:66-212.  Rotated-pole grids are discovered (their CRS is
    recognised from the CF attributes) but cannot be resampled."""
    proxies: dict = {}
    for var in dataset.variables.values():
        gm_var_name = var.attrs.get("grid_mapping")
        if gm_var_name and gm_var_name not in proxies and gm_var_name in dataset:
            gmp = _parse_crs_from_attrs(dataset[gm_var_name].attrs)
            proxies[gm_var_name] = gmp
    proxies = {k: v for k, v in proxies.items() if v is not None}
    if not proxies:
        for name, var in dataset.variables.items():
            gmp = _parse_crs_from_attrs(var.attrs)
            if gmp is not None:
                proxies[name] = gmp
                break
    if not proxies:
        gmp = _parse_crs_from_attrs(dataset.attrs)
        if gmp is not None:
            proxies[None] = gmp

    latlon, rotated, projected = _GridCoords(), _GridCoords(), _GridCoords()
    candidates = _find_potential_coord_vars(dataset)
    by_standard_name = ((latlon, "longitude", "latitude"),
                        (rotated, "grid_longitude", "grid_latitude"),
                        (projected, "projection_x_coordinate", "projection_y_coordinate"))
    for name in candidates:
        var = dataset[name]
        sn = var.attrs.get("standard_name")
        for coords, xn, yn in by_standard_name:
            if coords.x is None and sn == xn:
                coords.x = var
            if coords.y is None and sn == yn:
                coords.y = var
    by_name = ((latlon, ("lon", "longitude"), ("lat", "latitude")),
               (rotated, ("rlon", "rlongitude"), ("rlat", "rlatitude")),
               (projected, ("x", "xc", "transformed_x"), ("y", "yc", "transformed_y")))
    for name in candidates:
        var = dataset[name]
        for coords, xns, yns in by_name:
            if coords.x is None and name in xns:
                coords.x = var
            if coords.y is None and name in yns:
                coords.y = var
    for gmp in proxies.values():
        gmp.coords = (latlon if gmp.name == "latitude_longitude" else
                      rotated if gmp.name == "rotated_latitude_longitude" else projected)
    _complement(latlon, "latitude_longitude", missing_latitude_longitude_crs or CRS_WGS84, proxies)
    _complement(rotated, "rotated_latitude_longitude", missing_rotated_latitude_longitude_crs,
                proxies)
    _complement(projected, None, missing_projected_crs, proxies)

    complete = {}
    chunks = _get_dataset_chunks(dataset)
    for name, gmp in proxies.items():
        c = gmp.coords
        if (c is not None and c.x is not None and c.y is not None and c.x.size >= 2
                and c.y.size >= 2 and c.x.ndim == c.y.ndim):
            if c.x.ndim == 1:
                xd, yd = c.x.dims[0], c.y.dims[0]
            elif c.x.dims == c.y.dims:
                xd, yd = c.x.dims[1], c.x.dims[0]
            else:
                continue
            tw, th = chunks.get(xd), chunks.get(yd)
            gmp.tile_size = (tw, th) if tw is not None and th is not None else None
            complete[name] = gmp
        elif emit_warnings:
            warnings.warn(f'CRS "{gmp.name}": missing x- and/or y-coordinates '
                          f'(grid mapping variable "{name}": grid_mapping_name="{gmp.name}")')
    return complete


def new_grid_mapping_from_dataset(dataset, *, crs=None, tile_size=None, prefer_crs=None,
                                  prefer_is_regular=None, emit_warnings: bool = False,
                                  tolerance: float = DEFAULT_TOLERANCE) -> GridMapping:
    """dataset.py:31-102."""
    if crs is not None:
        crs = normalize_crs(crs)
    prefer_crs = normalize_crs(prefer_crs) if prefer_crs is not None else crs
    proxies = get_dataset_grid_mapping_proxies(
        dataset, emit_warnings=emit_warnings, missing_projected_crs=crs,
        missing_rotated_latitude_longitude_crs=crs,
        missing_latitude_longitude_crs=crs).values()
    gms = [new_grid_mapping_from_coords(x_coords=g.coords.x, y_coords=g.coords.y, crs=g.crs,
                                        tile_size=tile_size or g.tile_size, tolerance=tolerance)
           for g in proxies]
    if len(gms) > 1:
        if prefer_crs is not None and prefer_is_regular is not None:
            for gm in gms:
                if gm.crs == prefer_crs and bool(gm.is_regular) == prefer_is_regular:
                    return gm
            for gm in gms:
                if (gm.crs.is_geographic and prefer_crs.is_geographic
                        and bool(gm.is_regular) == prefer_is_regular):
                    return gm
        if prefer_crs is not None:
            for gm in gms:
                if gm.crs == prefer_crs:
                    return gm
            for gm in gms:
                if gm.crs.is_geographic and prefer_crs.is_geographic:
                    return gm
        if prefer_is_regular is not None:
            for gm in gms:
                if bool(gm.is_regular) == prefer_is_regular:
                    return gm
    if gms:
        return gms[0]
    raise ValueError("cannot find any grid mapping in dataset")
