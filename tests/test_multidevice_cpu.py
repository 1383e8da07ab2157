"""Host logic of the one-process multi-GPU path (xcube_resampling_amd.multidevice):
device-list resolution, its thread-local scope, the part runner (one thread
per part, results in part order, errors re-raised after every part ended)
and the partitioned reproject / affine / rectify assembly — every target
pixel written by exactly one part from exactly the source rows its shard
names.  The kernels are replaced by host stand-ins here (no GPU); the GPU
suite (test_multidevice_gpu.py) runs the real ones against the oracle."""

from __future__ import annotations

import contextlib
import threading

import numpy as np
import pytest


@pytest.fixture
def no_hip(monkeypatch):
    """Parts run without a HIP stream (the per-part context is a no-op) and
    'upload' by copying host rows."""
    from xcube_resampling_amd import multidevice

    monkeypatch.setattr(multidevice, "_part_context", lambda dev: contextlib.nullcontext())
    monkeypatch.setattr(multidevice, "rows_to_device",
                        lambda arr, j0, j1, dev: np.ascontiguousarray(arr[:, j0:j1]))
    return multidevice


def test_devices_option_and_keyword_scope():
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import multidevice

    assert multidevice.active_devices() is None
    with xrs.set_options(devices=[0, "cuda:1", 0]):
        assert multidevice.active_devices() == [torch.device("cuda", 0), torch.device("cuda", 1),
                                                torch.device("cuda", 0)]
        with multidevice.use_devices(["cuda:3"]):   # the keyword wins over the option
            assert multidevice.active_devices() == [torch.device("cuda", 3)]
        assert len(multidevice.active_devices()) == 3
    # an index-less "cuda" is the current device when normalised
    monkey = pytest.MonkeyPatch()
    monkey.setattr(torch.cuda, "current_device", lambda: 5)
    try:
        assert multidevice.normalize(["cuda", 2]) == [torch.device("cuda", 5),
                                                      torch.device("cuda", 2)]
    finally:
        monkey.undo()
    for bad in ([], [-1], ["cpu"], "cuda:0", [True], [1.5]):
        with pytest.raises(ValueError):
            with xrs.set_options(devices=bad):
                pass
        if bad != "cuda:0":
            with pytest.raises(ValueError):
                multidevice.normalize(bad)


def test_use_devices_is_local_to_its_thread():
    """A chunk scheduler's threads each pass their own list: one thread's
    keyword is invisible to another."""
    import torch

    from xcube_resampling_amd import multidevice

    seen = {}
    gate = threading.Barrier(2, timeout=30)

    def worker(k):
        with multidevice.use_devices([k]):
            gate.wait()
            seen[k] = multidevice.active_devices()

    ts = [threading.Thread(target=worker, args=(k,)) for k in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert seen == {1: [torch.device("cuda", 1)], 2: [torch.device("cuda", 2)]}
    assert multidevice.active_devices() is None


def test_run_parts_threads_order_and_errors(no_hip):
    multidevice = no_hip
    names = {}
    gate = threading.Barrier(4, timeout=30)   # all four parts are in flight together

    def fn(i, dev):
        gate.wait()
        names[i] = threading.current_thread().name
        return i * 10

    assert multidevice.run_parts(["a", "b", "c", "d"], fn) == [0, 10, 20, 30]
    assert len(set(names.values())) == 4
    ended = []

    def bad(i, dev):
        if i == 1:
            raise RuntimeError("part 1")
        ended.append(i)

    with pytest.raises(RuntimeError, match="part 1"):
        multidevice.run_parts(["a", "b", "c"], bad)
    assert sorted(ended) == [0, 2]          # the other parts still ran to the end


def _plan_case():
    import xcube_resampling_amd as xrs

    h, w = 300, 400
    lon = -5.0 + (np.arange(w) + 0.5) * 0.0075
    lat = 55.0 - (np.arange(h) + 0.5) * 0.005
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                      xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    tgm = xrs.GridMapping.regular((350, 260), (-540000.0, 6500000.0), (800.0, 840.0),
                                  "EPSG:3857", tile_size=(64, 48))
    return xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                  always_xy=True))


@pytest.mark.parametrize("world", [1, 2, 3, 7])
def test_reproject_partitioned_assembles_every_row_once(no_hip, monkeypatch, world):
    """Each part gets exactly its shard's source rows and writes exactly its
    target rows: a stand-in kernel stamps (part, row) and checks the band it
    was handed; the assembled output holds every row once."""
    from xcube_resampling_amd import kernels, reproject
    from xcube_resampling_amd.sharding import band_shard

    plan = _plan_case()
    src = np.arange(2 * plan.src_height * plan.src_width, dtype=np.float32).reshape(
        2, plan.src_height, plan.src_width)
    shards = [band_shard(plan, world, i, "cost", 8) for i in range(world)]

    def fake(band, p, interp, fill, out_dtype=None, rows=None, src_row0=0, **kw):
        i = next(k for k, s in enumerate(shards) if s.rows == rows)
        j0, j1 = shards[i].src_rows
        assert src_row0 == j0 and np.array_equal(band, src[:, j0:j1])
        r0, r1 = rows
        return np.broadcast_to((i * 100000 + np.arange(r0, r1))[None, :, None],
                               (2, r1 - r0, p.dst_width)).astype(out_dtype)

    monkeypatch.setattr(kernels, "reproject", fake)
    out = reproject._reproject_partitioned(src, plan, "bilinear", np.nan, None,
                                           ["d"] * world)
    assert out.dtype == np.float64 and out.shape == (2, plan.dst_height, plan.dst_width)
    rows = out[0, :, 0]
    cuts = [s.row0 for s in shards] + [plan.dst_height]
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        assert np.array_equal(rows[a:b], i * 100000 + np.arange(a, b))
    assert (out == out[:, :, :1]).all()


def test_rectify_put_tiles_takes_only_the_parts_tiles():
    """A part's band covers whole target rows, but only its own tiles'
    pixels are copied; the tiles of all parts together cover the raster."""
    from xcube_resampling_amd import kernels, multidevice
    from xcube_resampling_amd.sharding import rectify_shard

    th, tw, H, W = 5, 7, 23, 30
    ys = [th] * (H // th) + [H % th]
    xs = [tw] * (W // tw) + [W % tw]
    tiles = np.zeros(len(ys) * len(xs), dtype=kernels.TILE_INFO_DTYPE)
    tiles["r0"] = np.repeat(np.cumsum([0] + ys[:-1]), len(xs))
    tiles["c0"] = np.tile(np.cumsum([0] + xs[:-1]), len(ys))
    tiles["th"], tiles["tw"] = np.repeat(ys, len(xs)), np.tile(xs, len(ys))
    tiles["si0"], tiles["swin"], tiles["shin"] = 0, 9, 9
    out = np.full((1, H, W), -1.0)
    for world in (3,):
        for i in range(world):
            sh = rectify_shard(tiles, world, i)
            band = np.full((1, sh.row1 - sh.row0, W), float(i))
            multidevice.put_tiles(out, band, tiles[sh.tile0:sh.tile1], sh.row0)
    assert (out >= 0).all()
    owner = np.empty((H, W))
    for i in range(3):
        sh = rectify_shard(tiles, 3, i)
        for t in tiles[sh.tile0:sh.tile1]:
            owner[t["r0"]:t["r0"] + t["th"], t["c0"]:t["c0"] + t["tw"]] = i
    assert np.array_equal(out[0], owner)
