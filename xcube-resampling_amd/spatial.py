"""resample_in_space — the reference's dispatcher (spatial.py:40-168)."""

from __future__ import annotations

from collections.abc import Iterable

from . import multidevice
from .affine import affine_transform_dataset
from .constants import LOG
from .gridmapping import GridMapping
from .rectify import rectify_dataset
from .reproject import reproject_dataset
from .utils import _can_apply_affine_transform, as_dataset


def resample_in_space(source_ds, target_gm: GridMapping | None = None,
                      source_gm: GridMapping | None = None,
                      variables: str | Iterable[str] | None = None, interp_methods=None,
                      agg_methods=None, recover_nans=False, fill_values=None, tile_size=None,
                      devices=None):
    """Irregular source -> rectify; regular + same CRS (or both geographic) ->
    affine; otherwise -> reproject; close grid mappings -> the input.
    ``devices`` (engine extension): the GPUs each variable's partitions are
    spread over (``multidevice``)."""
    with multidevice.use_devices(devices):
        return _resample_in_space(source_ds, target_gm, source_gm, variables, interp_methods,
                                  agg_methods, recover_nans, fill_values, tile_size)


def _resample_in_space(source_ds, target_gm, source_gm, variables, interp_methods, agg_methods,
                       recover_nans, fill_values, tile_size):
    source_ds = as_dataset(source_ds)
    if source_gm is None:
        source_gm = GridMapping.from_dataset(source_ds)
    if not source_gm.is_regular:
        return rectify_dataset(source_ds, target_gm=target_gm, source_gm=source_gm,
                               variables=variables, interp_methods=interp_methods,
                               agg_methods=agg_methods, recover_nans=recover_nans,
                               fill_values=fill_values, tile_size=tile_size)
    if target_gm is None:
        LOG.warning("If source grid mapping is regular `target_gm` must be given. "
                    "Source dataset is returned.")
        return source_ds
    GridMapping.assert_regular(target_gm, name="target_gm")
    if source_gm.is_close(target_gm):
        return source_ds
    if _can_apply_affine_transform(source_gm, target_gm):
        return affine_transform_dataset(source_ds, target_gm, source_gm=source_gm,
                                        variables=variables, interp_methods=interp_methods,
                                        agg_methods=agg_methods, recover_nans=recover_nans,
                                        fill_values=fill_values)
    return reproject_dataset(source_ds, target_gm, source_gm=source_gm, variables=variables,
                             interp_methods=interp_methods, agg_methods=agg_methods,
                             recover_nans=recover_nans, fill_values=fill_values)
