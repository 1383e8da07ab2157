"""GPU tests of ``resample_in_space`` (reference spatial.py:40-168) against the
reference's tests/test_spatial.py goldens: dispatch to affine, to rectify with
a downscaling pre-step (4x4 irregular -> 2x2), and to rectify with upscaling.
The reproject cases (UTM source) are in test_crs_gpu.py."""

from __future__ import annotations

import numpy as np
import pytest

from fixtures import (
    dataset_2x2_irregular,
    dataset_4x4_irregular,
    dataset_8x6_regular,
    reference_goldens,
)

pytestmark = pytest.mark.gpu
GOLD = reference_goldens("tests/test_spatial.py")


def test_resample_in_space_affine():
    import xcube_resampling_amd as xrs

    src = dataset_8x6_regular()
    sgm = xrs.GridMapping.from_dataset(src)
    out = xrs.resample_in_space(src, xrs.GridMapping.regular((3, 3), (50.0, 10.0), 0.1,
                                                             sgm.crs), interp_methods=1)
    assert set(out.variables) == set(src.variables) | {"spatial_ref"}
    exp, dec = GOLD["test_affine_transform_dataset"][0]
    np.testing.assert_almost_equal(out["refl"].values, exp, decimal=dec)


@pytest.mark.parametrize("interp,idx", [(0, 0), (1, 1)])
def test_resample_in_space_rectify_and_downscale(interp, idx):
    import xcube_resampling_amd as xrs

    tgm = xrs.GridMapping.regular((2, 2), (-1, 51), 2, "EPSG:4326")
    out = xrs.resample_in_space(dataset_4x4_irregular(), target_gm=tgm, interp_methods=interp)
    exp, dec = GOLD["test_rectify_and_downscale_dataset"][idx]
    np.testing.assert_almost_equal(out["rad"].values, exp, decimal=dec)


def test_resample_in_space_rectify_and_upscale():
    import xcube_resampling_amd as xrs

    tgm = xrs.GridMapping.regular((4, 4), (-1, 49), 2, "EPSG:4326")
    out = xrs.resample_in_space(dataset_2x2_irregular(), target_gm=tgm, interp_methods=0)
    exp, dec = GOLD["test_rectify_and_upscale_dataset"][0]
    np.testing.assert_almost_equal(out["rad"].values, exp, decimal=dec)
