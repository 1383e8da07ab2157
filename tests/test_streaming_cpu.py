"""Host logic of the streamed path (no GPU): band split and the source rows
each band needs before its kernel may run."""

from __future__ import annotations

import pytest

from helpers import load_golden, reproject_golden_inputs


def _plan(g):
    import xcube_resampling_amd as xrs

    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    return xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                  always_xy=True))


@pytest.mark.parametrize("height,rows", [(36, 1), (36, 5), (36, 36), (36, 100), (1, 7)])
def test_band_ranges_cover_rows_once(height, rows):
    from xcube_resampling_amd.streaming import band_ranges

    bands = band_ranges(height, rows)
    assert [r for a, b in bands for r in range(a, b)] == list(range(height))
    assert all(0 < b - a <= rows for a, b in bands)


def test_band_ranges_rejects_empty_bands():
    from xcube_resampling_amd.streaming import band_ranges

    with pytest.raises(ValueError):
        band_ranges(10, 0)


@pytest.mark.parametrize("rows", [1, 5, 13, 64])
def test_band_source_rows_cover_every_read(rows):
    """Band b runs once rows [0, j1_b) are resident: j1 never decreases and
    covers every source row the band's tiles read."""
    from xcube_resampling_amd.streaming import band_ranges, band_source_rows

    plan = _plan(load_golden("reproject_f32.npz"))
    bands = band_ranges(plan.dst_height, rows)
    src_rows = band_source_rows(plan, bands)
    his = [j1 for _, j1 in src_rows]
    assert his == sorted(his) and his[-1] <= plan.src_height
    for (r0, r1), (_, j1) in zip(bands, src_rows):
        assert plan.source_rows_for(r0, r1)[1] <= j1
