"""ORACLE — CPU restatement of xcube-resampling's hot path (TEST INFRASTRUCTURE).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import anything in this package, and only as the
checker / the timed CPU baseline — never as part of the product path
(``xcube_resampling_amd`` must not import it; a test enforces that).

Each function restates one reference function (xcube-dev/xcube-resampling @
2025-09-05, cited as file:line) in plain numpy (or plain C for the numba
kernels, see rectify_ref.c), operation by operation, so its outputs are the
reference's outputs.  Pinning (see DESIGN.md "Oracle"):

* reproject_ref / gridmapping_ref: against fixtures produced by executing the
  reference's own ``_reproject_block``, ``_get_scr_bboxes_indices`` and
  ``_reorganize_data_array_slice`` (AST-extracted from /root/reference with
  numpy stand-ins for dask; tests/golden/make_goldens.py) and the reference's
  GridMapping test goldens.  The PROJ step (EPSG:3857 -> 4326) is restated from
  PROJ's published formulas; no reference test pins it -> that step is
  "parity unpinned" (documented in DESIGN.md).
"""
