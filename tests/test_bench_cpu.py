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


def test_cpu_baseline_thread_sweep():
    """The CPU baseline runs all cores plus a thread sweep; `value` is the best
    point and `cores` the thread count it used."""
    import bench

    _, tgm, plan, _, _ = bench.workload(2048, 512)
    cpu = bench.cpu_baseline(plan, tgm, seconds=0.5, sweep=(1, 2), sweep_seconds=0.3)
    allc = len(os.sched_getaffinity(0))
    sweep = {int(k): v for k, v in cpu["threads_sweep"].items()}
    assert allc in sweep and all(v > 0 for v in sweep.values())
    assert cpu["value"] == max(sweep.values()) and sweep[cpu["cores"]] == cpu["value"]
    assert cpu["kind"] == "port" and "GIL" in cpu["sample"]
    assert cpu["per_thread_Mpx_s"] == round(cpu["value"] / cpu["cores"], 3)


def test_split_predictions_report_every_model():
    """For N > 1 the bench line carries every balance model's prediction of
    the split it ran; each model's own split is the one it rates balanced."""
    import bench
    from xcube_resampling_amd.sharding import BALANCE_MODELS, band_splits, split_predictions

    _, _, plan, _, _ = bench.workload(4096, 512)
    for m in BALANCE_MODELS:
        cuts = band_splits(plan, 8, m)
        pred = split_predictions(plan, cuts)
        assert set(pred) == set(BALANCE_MODELS)
        assert pred[m]["max_over_mean"] < 1.01
        assert abs(sum(pred[m]["relative"]) - 8) < 1e-3


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


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys

    from conftest import ROOT

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", **(env_extra or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                       cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_gpus_flag_launches_the_ranks_itself():
    """`python bench.py --gpus 2` outside torchrun starts 2 ranks itself
    (torch.distributed.run child of the untouched parent); host-only
    rehearsal (--dry-run, gloo): ONE JSON line from rank 0 with n_gpus 2, the
    ranks block (both ranks' times, the cuts, every balance model's
    prediction) and no measured value."""
    r, line = _run_bench(["--gpus", "2", "--dry-run", "--size", "2048", "--tile", "512",
                          "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert sum(ln.startswith("{") for ln in r.stdout.splitlines()) == 1
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "bands2"
    assert len(line["ranks"]["kernel_ms"]) == 2
    cuts = line["ranks"]["cuts"]
    assert cuts[0] == 0 and cuts[-1] == 2048 and len(cuts) == 3
    assert set(line["ranks"]["predicted"]) == {"rows", "bytes", "cost"}
    assert line["value"] is None and line["roofline"] is None and "dry_run" in line


def test_gpus_flag_refuses_more_ranks_than_gpus():
    """Without enough visible GPUs (none here) `--gpus 4` exits non-zero with
    the exact torchrun command instead of measuring one GPU."""
    r, line = _run_bench(["--gpus", "4", "--steps", "1", "--warmup", "0"], timeout=120)
    assert r.returncode == 2 and line is None
    assert "--nproc-per-node 4" in r.stderr and "--master-addr 127.0.0.1" in r.stderr
