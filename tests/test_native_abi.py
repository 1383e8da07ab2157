"""CPU checks of the C-ABI library: it loads and exports every symbol that
include/xrs.h declares (no compute calls: there is no GPU here)."""

import ast
import os

import pytest

from conftest import ROOT


def test_library_exports_every_declared_symbol():
    from xcube_resampling_amd import _native

    names = _native.declared_symbols()
    assert "xrs_reproject" in names and "xrs_last_error" in names
    lib = _native.load_library()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared in include/xrs.h but not exported: {missing}"
    assert lib.xrs_version().decode().startswith("xrs ")
    # every declared symbol has a ctypes signature in the binding
    assert set(names) <= set(_native._SIGNATURES), set(names) - set(_native._SIGNATURES)


def test_product_package_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "xcube-resampling_amd")
    offenders = []
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if not f.endswith(".py"):
                continue
            path = os.path.join(dirpath, f)
            tree = ast.parse(open(path).read())
            for node in ast.walk(tree):
                mods = []
                if isinstance(node, ast.Import):
                    mods = [a.name for a in node.names]
                elif isinstance(node, ast.ImportFrom) and node.module:
                    mods = [node.module]
                if any(m == "oracle" or m.startswith("oracle.") for m in mods):
                    offenders.append(path)
    assert not offenders, offenders


def test_compute_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from xcube_resampling_amd.device import require_device
    from xcube_resampling_amd._native import NativeLibraryError

    with pytest.raises(NativeLibraryError, match="no HIP device"):
        require_device()


def test_product_library_reads_no_environment():
    """The product's numerics cannot depend on an environment variable: the
    library imports no getenv (the test-only path knobs are an explicit ABI,
    xrs_testing_set)."""
    import subprocess

    from xcube_resampling_amd import _native

    syms = subprocess.run(["nm", "-D", "--undefined-only", _native.LIB_PATH],
                          capture_output=True, text=True, check=True).stdout
    assert "getenv" not in syms
    assert "secure_getenv" not in syms


def test_argument_errors_are_reported_before_any_device_work():
    """xrs_reproject / xrs_reproject_proj / xrs_ij_bboxes_fill validate their
    arguments on the host and return XRS_ERR_ARG with a message (no HIP call
    is made): a float64 source row above 2 GiB (K1 addresses rows as buffer
    resources), an unsupported projection pipeline, a fill scratch that is
    missing or not 16-byte aligned."""
    import ctypes

    from xcube_resampling_amd import _native

    lib = _native.load_library()
    fake = ctypes.c_void_p(4096)   # never dereferenced: validation fails first
    w = 300_000_000                # 2.4 GB per float64 row
    rc = lib.xrs_reproject(fake, 11, 1, 4, w, 0, 4, 4 * w, w, fake, 11, 4, 4, 0, 4, 16, 4,
                           4, 4, fake, fake, 0, fake, fake, fake, 4, 4, 1.0, 1.0, 0, 0.0,
                           fake, 1 << 20, fake, None)
    assert rc == _native.XRS_ERR_ARG
    assert b"2 GiB" in lib.xrs_last_error()
    steps = (_native.ProjStep * 2)()
    steps[0].kind, steps[1].kind = 1, 3   # forward then forward: not a pipeline
    rc = lib.xrs_reproject_proj(fake, 10, 1, 4, 4, 0, 4, 16, 4, fake, 10, 4, 4, 0, 4, 16, 4,
                                4, 4, fake, fake, ctypes.cast(steps, ctypes.c_void_p), 2,
                                fake, fake, fake, 4, 4, 1.0, 1.0, 0, 0.0, fake, None)
    assert rc == _native.XRS_ERR_ARG
    assert b"pipeline" in lib.xrs_last_error()
    # K4's claim-key fill needs a 16-byte aligned scratch (non-temporal
    # 16-byte stores)
    rc = lib.xrs_ij_bboxes_fill(fake, fake, 4, 4, 4, 1, 0, 0, fake, fake, fake,
                                ctypes.c_void_p(4096 + 4), 16, None)
    assert rc == _native.XRS_ERR_ARG
    rc = lib.xrs_ij_bboxes_fill(fake, fake, 4, 4, 4, 1, 0, 0, fake, fake, fake, None, 16, None)
    assert rc == _native.XRS_ERR_ARG


def test_library_override_limited_to_probe_arms(tmp_path):
    """XRS_LIBRARY (A/B timing scripts) may name the product library or an arm
    under probe/; any other path is refused, so the environment cannot put a
    different binary behind the product API."""
    import os
    import subprocess
    import sys

    code = ("import xcube_resampling_amd._native as N\n"
            "try:\n    N.load_library()\n    print('loaded', N.LIB_PATH)\n"
            "except N.NativeLibraryError as e:\n    print('refused', e)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fake = tmp_path / "libxrs.so"
    fake.write_bytes(b"")
    for value, expect in ((str(fake), "refused"),
                          (os.path.join(root, "xcube-resampling_amd", "lib", "libxrs.so"),
                           "loaded")):
        env = dict(os.environ, XRS_LIBRARY=value)
        out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root,
                             capture_output=True, text=True, timeout=120).stdout
        assert out.startswith(expect), out


def test_host_register_refuses_partial_pages():
    """xrs_host_register accepts whole pages only: an array
    that starts inside a page (numpy's malloc'd buffers do) or a size that is
    not a page multiple is refused with XRS_ERR_ARG before any HIP call."""
    import ctypes
    import mmap

    from xcube_resampling_amd import _native

    lib = _native.load_library()
    page = mmap.PAGESIZE
    buf = mmap.mmap(-1, 4 * page)
    base = ctypes.addressof(ctypes.c_char.from_buffer(buf))
    try:
        assert base % page == 0
        for ptr, size in [(base + 16, page), (base, page + 8), (base, 100)]:
            assert lib.xrs_host_register(ctypes.c_void_p(ptr), size) == _native.XRS_ERR_ARG
            assert "page" in _native.last_error()
        assert lib.xrs_host_register(None, page) == _native.XRS_ERR_ARG
        one = (ctypes.c_void_p * 1)(None)
        assert lib.xrs_host_unregister(None, one, 1) == _native.XRS_ERR_ARG
        # the caller must name the streams that used the range (no device drain)
        assert lib.xrs_host_unregister(ctypes.c_void_p(base), None, 1) == _native.XRS_ERR_ARG
        assert lib.xrs_host_unregister(ctypes.c_void_p(base), one, 0) == _native.XRS_ERR_ARG
        assert lib.xrs_host_unregister(ctypes.c_void_p(base), one, 65) == _native.XRS_ERR_ARG
    finally:
        del base
        buf.close()
