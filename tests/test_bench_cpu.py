"""CPU checks of bench.py's host logic (no GPU): algorithmic byte counts,
the bounded CPU baseline, the PMC traffic reduction."""

from __future__ import annotations

import csv
import os

import numpy as np


def test_source_pixels_read_matches_band_sum():
    """S_read of the whole raster == the plan's rows x columns read, and the
    row bands of a split never read fewer rows than the whole."""
    import bench
    from xcube_resampling_amd.sharding import band_shard

    _, _, plan, _, _ = bench.workload(4096, 512)
    total = bench.source_pixels_read(plan)
    lo, hi = plan.row_source_extent()
    rows = int(hi.max() - lo.min() + 1)
    assert total == rows * plan.source_cols_read()
    parts = [bench.source_pixels_read(plan, band_shard(plan, 4, r).rows) for r in range(4)]
    assert total <= sum(parts) <= total + 4 * 2 * plan.source_cols_read()


def test_cpu_baseline_runs_on_all_cores():
    import bench

    _, tgm, plan, _, _ = bench.workload(2048, 512)
    cpu = bench.cpu_baseline(plan, tgm, seconds=0.5)
    assert cpu["cores"] == len(os.sched_getaffinity(0))
    assert cpu["value"] > 0 and cpu["kind"] == "port"


def test_pmc_traffic_reduce(tmp_path):
    """Two gather dispatches per pass (calibration, bench); FETCH_SIZE is
    scaled by the identity launch's known 4*S bytes."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "scripts"))
    import pmc_traffic

    size = 1000
    for name, counter, vals in (("fetch", "FETCH_SIZE", (4 * size * size / 2 / 1024, 3000.0)),
                                ("write", "WRITE_SIZE", (4 * size * size / 1024, 3906.25))):
        d = tmp_path / name
        d.mkdir()
        with open(d / f"{name}_counter_collection.csv", "w", newline="") as f:
            w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for did, v in enumerate(vals, start=1):
                for half in (0.5, 0.5):   # two instances per dispatch are summed
                    w.writerow(dict(Dispatch_Id=did, Kernel_Name="gather_separable_kernel<...>",
                                    Counter_Name=counter, Counter_Value=v * half))
                w.writerow(dict(Dispatch_Id=did + 10, Kernel_Name="axis_tables_kernel<1>",
                                Counter_Name=counter, Counter_Value=1e9))
    r = pmc_traffic.reduce(str(tmp_path), size, "f32", write=False)
    assert np.isclose(r["calibration"]["fetch_factor"], 2.0)
    assert r["read_bytes"] == int(3000.0 * 1024 * 2.0)
    assert r["write_bytes"] == int(3906.25 * 1024)
