"""CPU checks of bench.py's host logic (no GPU): algorithmic byte counts,
the bounded CPU baseline, the PMC traffic reduction."""

from __future__ import annotations

import csv
import os

import numpy as np
import pytest


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
    """Read / write bytes from the size-resolved request counters, per launch
    (two copies, then two gather dispatches: identity calibration, bench),
    instances summed; the calibration launches are reported as measured /
    known bytes, without any correction of the bench numbers."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "scripts"))
    import pmc_traffic

    size = 1000
    nb = 4 * size * size
    # per launch (copy16, copy4, ident, bench): (n32, n64, n128), (wr, wr64), dram
    rd = {"copy16": (0, 0, nb // 128), "copy4": (0, 10, nb // 128 - 5),
          "ident": (0, 2, nb // 128 - 1), "bench": (4, 100, 40000)}
    wr = {"copy16": (nb // 64, nb // 64), "copy4": (nb // 64, nb // 64),
          "ident": (nb // 64, nb // 64), "bench": (nb // 64 + 8, nb // 64)}
    kname = {"copy16": "copy_unrolled_kernel<1, false>", "copy4": "copy_b32_kernel<8>",
             "ident": "gather_separable_kernel<...>", "bench": "gather_separable_kernel<...>"}
    for p, counters in pmc_traffic.PASSES.items():
        d = tmp_path / p
        d.mkdir()
        with open(d / f"{p}_counter_collection.csv", "w", newline="") as f:
            w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for did, launch in enumerate(pmc_traffic.LAUNCHES, start=1):
                n32, n64, n128 = rd[launch]
                vals = {"TCC_EA0_RDREQ_sum": n32 + n64 + n128, "TCC_EA0_RDREQ_32B_sum": n32,
                        "TCC_EA0_RDREQ_64B_sum": n64, "TCC_EA0_RDREQ_128B_sum": n128,
                        "TCC_EA0_WRREQ_sum": wr[launch][0], "TCC_EA0_WRREQ_64B_sum": wr[launch][1],
                        "TCC_EA0_RDREQ_DRAM_sum": 7}
                for c in counters:
                    for half in (0.5, 0.5):   # two instances per dispatch are summed
                        w.writerow(dict(Dispatch_Id=did, Kernel_Name=kname[launch],
                                        Counter_Name=c, Counter_Value=vals[c] * half))
                w.writerow(dict(Dispatch_Id=did + 10, Kernel_Name="axis_tables_kernel<1>",
                                Counter_Name=counters[0], Counter_Value=1e9))
    r = pmc_traffic.reduce(str(tmp_path), size, "f32", write=False)
    assert r["read_bytes"] == 4 * 32 + 100 * 64 + 40000 * 128
    assert r["write_bytes"] == (nb // 64) * 64 + 8 * 32
    assert r["launches"]["copy16"]["read_over_known"] == 1.0
    assert r["launches"]["copy4"]["read_over_known"] == round((640 + nb - 640) / nb, 4)
    assert r["launches"]["bench"]["rdreq_dram"] == 7
    assert r["hbm_bytes_per_launch"] == r["read_bytes"] + r["write_bytes"]


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


def _fake_kfd(tmp_path, simds):
    nodes = tmp_path / "nodes"
    for i, n in enumerate(simds):
        d = nodes / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {n}\nmax_waves_per_simd 8\n")
    return str(nodes)


def test_visible_gpu_count_reads_kfd_topology_and_visibility(tmp_path):
    """The launcher's GPU count comes from the KFD topology (nodes with
    SIMDs; the CPU node has none), narrowed by the *_VISIBLE_DEVICES lists as
    the runtime narrows them."""
    import bench

    nodes = _fake_kfd(tmp_path, [0] + [1024] * 8)     # one CPU node + 8 GPUs
    assert bench.visible_gpu_count(nodes, env={}) == 8
    assert bench.visible_gpu_count(nodes, env={"HIP_VISIBLE_DEVICES": "0,3"}) == 2
    assert bench.visible_gpu_count(nodes, env={"ROCR_VISIBLE_DEVICES": "1,2,3",
                                               "HIP_VISIBLE_DEVICES": "0"}) == 1
    assert bench.visible_gpu_count(nodes, env={"CUDA_VISIBLE_DEVICES": "-1"}) == 0
    assert bench.visible_gpu_count(nodes, env={"HIP_VISIBLE_DEVICES": "0,9,1"}) == 1
    assert bench.visible_gpu_count(nodes, env={"HIP_VISIBLE_DEVICES": ""}) == 0
    with pytest.raises(OSError):
        bench.visible_gpu_count(str(tmp_path / "missing"), env={})


def test_launcher_count_does_not_initialise_hip():
    """Counting GPUs for `--gpus N` leaves torch's HIP runtime untouched in
    the parent (torch.cuda.device_count() may fall back to
    hipGetDeviceCount)."""
    import subprocess
    import sys

    from conftest import ROOT

    code = ("import sys, torch; sys.path.insert(0, %r); import bench\n"
            "try:\n    bench.visible_gpu_count()\nexcept OSError:\n    pass\n"
            "assert not torch.cuda.is_initialized()\nprint('ok')\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]
