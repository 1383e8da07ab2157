"""Host logic of the streamed path (no GPU): band split and the source rows
each band needs before its kernel may run."""

from __future__ import annotations

import numpy as np
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


def test_source_rows_copies_only_missing_runs():
    """_SourceRows copies each needed row once, in contiguous runs, whatever
    the order of the requests."""
    from xcube_resampling_amd import streaming

    calls = []

    class _Dev:   # stand-in device buffer: only data_ptr() is used
        def __getitem__(self, idx):
            return type("R", (), {"data_ptr": lambda self: 0})()

    class _Stage:  # stand-in staging: records the host runs handed to it
        def h2d(self, dst_ptr, src, stream):
            assert src.flags.c_contiguous
            calls.append(src.nbytes)

    src = np.zeros((2, 100, 8), np.float32)
    rows = streaming._SourceRows(src, _Dev(), None, _Stage())
    rows.need(40, 60)
    rows.need(10, 50)        # rows 10..39 missing -> one run
    rows.need(55, 70)        # rows 60..69
    rows.need(-5, 5)         # clipped to 0..4
    rows.need(30, 20)        # empty
    row = 8 * 4
    assert calls == [20 * row] * 2 + [30 * row] * 2 + [10 * row] * 2 + [5 * row] * 2
    assert rows.resident[0:5].all() and rows.resident[10:70].all()
    assert not rows.resident[5:10].any() and not rows.resident[70:].any()


def test_host_copy_parts_cover_the_array():
    """The staging copies split large arrays over a thread pool in parts:
    every byte lands once, sizes above and below one part, odd lengths."""
    from xcube_resampling_amd import streaming

    rng = np.random.default_rng(0)
    for n in (0, 7, streaming._COPY_PART, 3 * streaming._COPY_PART + 12345):
        src = rng.integers(0, 256, n, dtype=np.uint8)
        dst = np.zeros(n, np.uint8)
        streaming._host_copy(dst, src)
        assert np.array_equal(dst, src)


def test_band_rows_multiple_of_unit():
    from xcube_resampling_amd.streaming import _band_rows

    assert _band_rows(1000, 1 << 20, 8) % 8 == 0
    assert _band_rows(10, 1, 8) == 16     # whole (rounded-up) height in one band
    assert _band_rows(5000, 64 << 20, 7) == 7


def test_staging_pool_is_bounded_and_exclusive(monkeypatch):
    """staging pairs are borrowed from a process-wide pool of at
    most _POOL_MAX, one thread at a time each, and returned drained — not one
    pinned pair per thread for the thread's life."""
    import threading
    import time

    from xcube_resampling_amd import streaming

    made, in_use, peak = [], set(), [0]
    lock = threading.Lock()

    class FakeStaging:
        def __init__(self):
            made.append(self)
            self.drained = 0

        def drain(self):
            self.drained += 1

    monkeypatch.setattr(streaming, "_Staging", FakeStaging)
    monkeypatch.setattr(streaming, "_POOL_FREE", [])
    monkeypatch.setattr(streaming, "_POOL_MADE", 0)
    monkeypatch.setattr(streaming, "_POOL_MAX", 3)

    def work(_):
        for _ in range(5):
            with streaming._staging() as st:
                with lock:
                    assert st not in in_use          # never shared by two threads
                    in_use.add(st)
                    peak[0] = max(peak[0], len(in_use))
                time.sleep(0.002)
                with lock:
                    in_use.discard(st)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(12)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(made) <= 3 and peak[0] <= 3
    assert sorted(map(id, streaming._POOL_FREE)) == sorted(map(id, made))
    assert sum(s.drained for s in made) == 12 * 5
