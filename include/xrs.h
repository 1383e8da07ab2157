/*
 * xrs.h — C-ABI of libxrs, the MI355X (gfx950) engine for xcube-resampling's
 * per-chunk inner loops.
 *
 * Every compute entry point replaces one per-chunk seam of the reference
 * (xcube-dev/xcube-resampling @ 2025-09-05, paths relative to its repo root):
 * the dask block callables / numba kernels that do the pixel work.  Host code
 * (the Python package `xcube_resampling_amd`, or any FFI: ctypes, cgo, JNI)
 * keeps the reference's orchestration semantics and calls these functions on
 * device buffers.
 *
 * Conventions
 *  - All data pointers are DEVICE pointers (hipMalloc / torch CUDA tensors),
 *    unless a parameter is documented as host memory.
 *  - Shapes, strides and indices are int64_t; strides are in ELEMENTS.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).  Every
 *    call is asynchronous and stream-ordered; no hidden allocation, no host
 *    synchronisation inside (safe to capture in a hipGraph).
 *  - Return value: XRS_OK (0) or a negative XRS_ERR_* code; the message is in
 *    xrs_last_error() (thread-local).
 *  - Data-dependent errors the reference raises from inside a block (e.g. the
 *    IndexError of numpy fancy indexing in reproject.py:284) are reported by
 *    OR-ing a bit into the caller-provided device word `err_flags`; the host
 *    reads it after the stream is synchronised and raises the same exception.
 */
#ifndef XRS_H_
#define XRS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define XRS_OK 0
#define XRS_ERR_ARG (-1)      /* invalid argument (shape/dtype/method)       */
#define XRS_ERR_HIP (-2)      /* HIP runtime error (launch failed, ...)      */
#define XRS_ERR_NOTIMPL (-3)  /* method not implemented (reference: NotImplementedError) */

/* ---- dtype codes ------------------------------------------------------- */
#define XRS_DTYPE_U8 1
#define XRS_DTYPE_I8 2
#define XRS_DTYPE_U16 3
#define XRS_DTYPE_I16 4
#define XRS_DTYPE_U32 5
#define XRS_DTYPE_I32 6
#define XRS_DTYPE_I64 7
#define XRS_DTYPE_F32 10
#define XRS_DTYPE_F64 11

/* ---- interpolation codes (constants.py:66-70) --------------------------- */
#define XRS_INTERP_NEAREST 0
#define XRS_INTERP_BILINEAR 1
#define XRS_INTERP_TRIANGULAR 2

/* ---- err_flags bits ------------------------------------------------------ */
#define XRS_EFLAG_INDEX 1     /* numpy IndexError (window index out of range) */
#define XRS_EFLAG_BAND 2      /* read outside the source band held on device  */
#define XRS_EFLAG_NAN_TO_INT 4  /* int(nan): coarsen mode on a float chunk with NaN (ValueError) */
#define XRS_EFLAG_INF_TO_INT 8  /* int(+-inf): coarsen mode, infinite values (OverflowError)   */
#define XRS_EFLAG_STATE 16    /* rectify: a tile record, claim key or source position outside
                                 its raster (inconsistent inputs); the access was skipped  */

/* library identification */
const char* xrs_version(void);
/* thread-local message of the last failing call ("" if none) */
const char* xrs_last_error(void);

/* -------------------------------------------------------------------------
 * Host-resident rasters (the reference's numpy-in / numpy-out contract,
 * reproject.py:254-255, affine.py:227-228): page-lock a caller-owned host
 * buffer in place so band-wise H2D / D2H copies run as DMA on their own
 * streams, overlapped with the kernels (xcube_resampling_amd/streaming.py).
 * The engine itself stages through its own page-locked buffers; these two
 * are for bindings that own long-lived, page-aligned buffers (mmap /
 * posix_memalign).  xrs_host_register accepts only whole pages: `ptr` on a
 * page boundary and `bytes` a multiple of the page size (else XRS_ERR_ARG —
 * a malloc'd numpy array shares its edge pages with its neighbours); returns
 * XRS_OK, 1 when the range was already registered (the caller must then NOT
 * unregister it), or XRS_ERR_HIP.  xrs_host_unregister synchronises the
 * `nstreams` (1..64) streams the caller names — every stream that copied
 * to or from the range (a null entry is the current device's null stream)
 * — then unpins; no other stream or device waits, so one host thread per
 * device may unregister while the others keep their queues busy.  A stream
 * still queueing copies of the range after the call is the caller's error.
 * ------------------------------------------------------------------------- */
int xrs_host_register(void* ptr, int64_t bytes);
int xrs_host_unregister(void* ptr, void* const* streams, int64_t nstreams);
/* stream-ordered copy of `bytes` between any two of host / device memory
 * (hipMemcpyAsync, direction from unified addressing) */
int xrs_copy_async(void* dst, const void* src, int64_t bytes, void* stream);

/* -------------------------------------------------------------------------
 * xrs_reproject — replaces `_reproject_block` (reproject.py:268-335) for ALL
 * target tiles of one variable in one launch, and the per-tile source-window
 * materialisation it depends on (`_reorganize_data_array_slice`,
 * reproject.py:499-530: da.pad + copy) by bounds-checked reads that return
 * `fill` outside the source (equivalent to the constant padding).
 *
 * Per target pixel (global row r, col c; tile t = (r/tile_h, c/tile_w)):
 *   sx, sy = coordinate of the pixel centre in the source CRS
 *            coord_mode 0 (separable): sx = src_x[c], sy = src_y[r]
 *            coord_mode 1 (2-D):       sx = src_x[r*dst_w+c], sy = src_y[...]
 *            coord_mode 2 (separable, column generators): sy = src_y[r];
 *              src_x = ntiles_x records {start, stop, step, n} (f64 x 4) and
 *              then (m1, m2); for c in tile column tx, k = c - tx*tile_w:
 *              v = k == n-1 ? stop : k*step + start, sx = (v*m1)*m2 — dask's
 *              blockwise linspace of the target pixel centres and the
 *              separable transformation's scalings, evaluated with the
 *              host's operation order.  The caller must have checked that
 *              these values equal its src_x bit for bit (0 B/column read).
 *   ix = (sx - (double)tile_x0[t]) / x_res           (reproject.py:278)
 *   iy = (sy - (double)tile_y0[t]) / -y_res          (reproject.py:279)
 *   window index -> int16 as numpy, python-style negative wrap in
 *   [-win, win), else IndexError (err_flags |= XRS_EFLAG_INDEX);
 *   source row/col = tile_win[2t+1] + wy, tile_win[2t] + wx (unpadded);
 *   outside [0,src_h) x [0,src_w) -> fill (the da.pad constant).
 *   nearest: rint (half-even); bilinear: f64 lerps, source differences in the
 *   source dtype; triangular: two-triangle plane, stored in the source dtype.
 *
 * src: (n, src_rows, src_w) with element strides (src_sn, src_sy, 1); row 0
 *      of the buffer is global source row `src_row0` (a device may hold a band).
 * dst: (n, row_end-row_begin, dst_w) with strides (dst_sn, dst_sy, 1); only
 *      target rows [row_begin, row_end) are computed (multi-GPU row bands).
 * tile_x0/tile_y0 (float32, ntiles), tile_win (int64, 2*ntiles: i0, j0 of
 *      each tile's window in unpadded source indices): device memory,
 *      ntiles = ceil(dst_h/tile_h) * ceil(dst_w/tile_w), row-major.
 * dst_dtype: = src_dtype for nearest/triangular; float32 or float64 for
 *      bilinear (the reference yields float64 there; float32 = declared dtype).
 * workspace: device scratch of xrs_reproject_workspace_size(...) bytes; 0
 *      since round 5 (K1's work items resolve their own axis entries), so
 *      NULL / 0 may be passed.
 * A source row may span at most 2 GiB (src_w * element size), else XRS_ERR_ARG.
 * ------------------------------------------------------------------------- */
int64_t xrs_reproject_workspace_size(int64_t dst_h, int64_t dst_w, int64_t tile_h,
                                     int64_t tile_w, int coord_mode);

int xrs_reproject(const void* src, int src_dtype, int64_t n, int64_t src_h,
                  int64_t src_w, int64_t src_row0, int64_t src_rows,
                  int64_t src_sn, int64_t src_sy, void* dst, int dst_dtype,
                  int64_t dst_h, int64_t dst_w, int64_t row_begin,
                  int64_t row_end, int64_t dst_sn, int64_t dst_sy,
                  int64_t tile_h, int64_t tile_w, const double* src_x,
                  const double* src_y, int coord_mode, const float* tile_x0,
                  const float* tile_y0, const int64_t* tile_win,
                  int64_t win_h, int64_t win_w, double x_res, double y_res,
                  int interp, double fill, void* workspace,
                  int64_t workspace_bytes, int32_t* err_flags, void* stream);

/* ---- aggregation codes (constants.py:51-65, coarsen.py) ------------------ */
#define XRS_AGG_NONE 0
#define XRS_AGG_MEAN 1
#define XRS_AGG_SUM 2
#define XRS_AGG_MAX 3
#define XRS_AGG_MIN 4
#define XRS_AGG_PROD 5
#define XRS_AGG_COUNT 6
#define XRS_AGG_FIRST 7
#define XRS_AGG_LAST 8
#define XRS_AGG_CENTER 9
#define XRS_AGG_MEDIAN 10     /* xrs_coarsen only (the fused xrs_affine path: 1..9) */
#define XRS_AGG_MODE 11
#define XRS_AGG_STD 12
#define XRS_AGG_VAR 13

/* -------------------------------------------------------------------------
 * xrs_affine — replaces affine._upscale (affine.py:316-362), i.e.
 * dask_image.ndinterp.affine_transform -> scipy.ndimage.affine_transform
 * (diagonal matrix, order 0/1, mode "constant", cval) evaluated per dask-image
 * output chunk, and — with div_y/div_x > 1 — affine._downscale
 * (affine.py:277-313): the div-x upscale fused with da.coarsen(agg).
 *
 * src: (nt, src_h, src_w) strides (src_st, src_sy, 1); dst: (nt, out_h,
 *   out_w) strides (dst_st, dst_sy, 1) with dst_dtype = the reducer's numpy
 *   result dtype (agg NONE: the scipy output dtype = src dtype, or float64
 *   with recover_nan).
 * Per axis (y, x) of the div-x intermediate (out_h*div_y, out_w*div_x):
 *   scale, chunk = dask-image output chunk size, and per chunk k (device
 *   arrays): rel[k] = first input index of the chunk's input slice, len[k] =
 *   slice length, off[k] = offset + scale*chunk_offset - rel[k] (float64).
 * t_next (device, nt entries, or NULL for 2-D data): index of the time slice
 *   scipy multiplies by a zero weight (order 1), mirrored inside the time
 *   chunk's input slice; -1 = none.
 * recover_nan: affine.py:344-360 (NaN -> 0 image / (1 - mask) image ratio;
 *   the host decides it with xrs_any_nan as the reference does with da.any).
 * run_weights: a speed hint for square 2/4/8 float coarsens of order 1 —
 *   nonzero when the div-x grid has scale 1 but offsets off the integral
 *   layout (a target grid not aligned to the source): the contiguous-run
 *   kernel with fractional weights (K3w) instead of the integral-run one
 *   (K3i).  Results are identical either way (each falls back to the exact
 *   path wherever its runs break).
 * workspace: xrs_affine_workspace_size(out_h*div_y, out_w*div_x) bytes.
 * ------------------------------------------------------------------------- */
int64_t xrs_affine_workspace_size(int64_t inter_h, int64_t inter_w);

int xrs_affine(const void* src, int src_dtype, int64_t nt, int64_t src_h, int64_t src_w,
               int64_t src_st, int64_t src_sy, void* dst, int dst_dtype, int64_t out_h,
               int64_t out_w, int64_t dst_st, int64_t dst_sy, int64_t div_y, int64_t div_x,
               int agg, int order, double scale_y, double scale_x, int64_t chunk_y,
               const int64_t* rel_y, const int64_t* len_y, const double* off_y,
               int64_t chunk_x, const int64_t* rel_x, const int64_t* len_x,
               const double* off_x, const int64_t* t_next, double cval, int recover_nan,
               int run_weights, void* workspace, int64_t workspace_bytes, void* stream);

/* -------------------------------------------------------------------------
 * xrs_coarsen — replaces da.coarsen(agg, array, {ndim-2: div_y, ndim-1:
 * div_x}) (affine.py:308-310 -> dask chunk.coarsen -> coarsen.py:50-155),
 * SURVEY §8(b) seam 3, for every AGG_METHODS key (constants.py:51-65):
 * mean, sum, max, min, prod, count, first, last, center, median, mode, std,
 * var.  Float blocks use numpy's nan-reducers; integer blocks the plain
 * reducers with float results rint-ed and cast back (coarsen.py:91-111).
 * src: (nt, src_h, src_w) strides (src_st, src_sy, 1), src_h % div_y == 0 and
 *   src_w % div_x == 0 (dask's alignment check).
 * dst: (nt, src_h/div_y, src_w/div_x) strides (dst_st, dst_sy, 1); dst_dtype
 *   = the reducer's numpy result dtype (count, mode: int64; sum/prod of
 *   integers: int64 bits, uint64 for unsigned sources).
 * The dask chunking (after da.coarsen's aligned rechunk) is passed as the
 *   chunk id of every slice / row / column: chunk_t (nt), chunk_y (src_h),
 *   chunk_x (src_w), device int32, ids < n_chunks_*.  It matters twice:
 *   - a window that is a whole chunk wide (chunk width == div_x) is summed as
 *     ONE pairwise loop over its div_y*div_x values (numpy coalesces the
 *     window axes of such a block), other windows row by row; chunk_x NULL
 *     = the whole width is one chunk;
 *   - mode on float sources (coarsen.py:133-139): the offset is int(min) of
 *     the chunk holding the window, so all three id arrays, a workspace of
 *     xrs_coarsen_workspace_size(n_chunks_t*n_chunks_y*n_chunks_x) bytes and
 *     err_flags (NaN -> XRS_EFLAG_NAN_TO_INT, +-inf -> XRS_EFLAG_INF_TO_INT)
 *     are required; otherwise chunk_t / chunk_y / workspace may be NULL / 0.
 * ------------------------------------------------------------------------- */
int64_t xrs_coarsen_workspace_size(int64_t n_chunks);

int xrs_coarsen(const void* src, int src_dtype, int64_t nt, int64_t src_h, int64_t src_w,
                int64_t src_st, int64_t src_sy, void* dst, int dst_dtype, int64_t dst_st,
                int64_t dst_sy, int64_t div_y, int64_t div_x, int agg, const int32_t* chunk_t,
                const int32_t* chunk_y, const int32_t* chunk_x, int64_t n_chunks_t,
                int64_t n_chunks_y, int64_t n_chunks_x, void* workspace,
                int64_t workspace_bytes, int32_t* err_flags, void* stream);

/* *flag = 1 if any of the n elements of a float32/float64 device array is NaN
 * (da.any(da.isnan(array)), affine.py:347-349); integer dtypes -> 0. */
int xrs_any_nan(const void* src, int src_dtype, int64_t n, int32_t* flag, void* stream);

/* -------------------------------------------------------------------------
 * xrs_ij_bboxes — replaces compute_ij_bboxes (gridmapping/bboxes.py:28-106;
 * caller GridMapping.ij_bboxes_from_xy_bboxes, base.py:565-629): for every box
 * the min/max source pixel (i, j) whose (x, y) lies inside the box (borders
 * already applied by the caller: [x_min-b, x_max+b] etc., inclusive).
 * x, y: (h, w) float64 device images, row stride sy.
 * Grid mode (ntx > 0, ntx*nty == nboxes, box k = ty*ntx + tx): bx = (ntx, 2)
 *   [x_min, x_max] per tile column, by = (nty, 2) [y_min, y_max] per tile row.
 * Otherwise (ntx == 0): bx = (nboxes, 4) [x_min, y_min, x_max, y_max].
 * acc: (nboxes, 4) int32 device accumulators, initialised by the caller to
 *   {INT32_MAX, INT32_MAX, -1, -1}; receives {min i, min j, max i, max j}
 *   (max i == -1: no pixel).  The ij_border expansion is host-side.
 * ------------------------------------------------------------------------- */
int xrs_ij_bboxes(const double* x, const double* y, int64_t h, int64_t w, int64_t sy,
                  int64_t nboxes, int64_t ntx, int64_t nty, const double* bx,
                  const double* by, int32_t* acc, void* stream);

/* xrs_ij_bboxes_fill — xrs_ij_bboxes whose grid also sets fill_words 32-bit
 * words at `fill` (16-byte aligned) to 0xFFFFFFFF: the claim-key scratch of
 * the xrs_rectify_ij / _ij_var call that follows on the same stream
 * (keys_ready = 1), filled while K4 streams the coordinates instead of in a
 * pass of its own.  fill_words = 0: exactly xrs_ij_bboxes. */
int xrs_ij_bboxes_fill(const double* x, const double* y, int64_t h, int64_t w, int64_t sy,
                       int64_t nboxes, int64_t ntx, int64_t nty, const double* bx,
                       const double* by, int32_t* acc, uint32_t* fill, int64_t fill_words,
                       void* stream);

/* -------------------------------------------------------------------------
 * xrs_rectify_ij — replaces _compute_target_source_ij_block and the numba
 * kernels _compute_target_source_ij_sequential/_line (rectify.py:373-576):
 * for every target pixel the fractional source pixel (i, j) of the FIRST
 * source quad (raster order within the target tile's source bbox) whose
 * triangle A or B contains the target pixel centre (tolerance uv_delta).
 * x, y: (h, w) float64 source coordinates in the target CRS (row stride sy).
 * tiles: device array of ntiles records {int32 r0, c0, th, tw, si0, sj0,
 *   swin, shin; float64 x_off, y_off} (row-major, ntiles_x per row): target
 *   tile origin/size, source window origin (si0 = -1: no source) and size,
 *   and the reference's per-tile dst_x/y_offset.
 * chunk_offsets (device, ntiles + 1): the work list of quad strips (16
 *   quad rows x 63 quads, one wave each) as an exclusive prefix sum of each
 *   tile's strip count (ceil((swin-1)/63) * ceil((shin-1)/16), 0 for a tile
 *   without source); chunk_offsets[ntiles] = total.  Produced by xrs_rectify_tiles on
 *   the device, so no host round trip is needed between K4 and K5.
 * max_chunks: the total if the caller knows it (one strip per wave), else 0
 *   (a persistent grid reads the total on the device).
 * x_scale = dst_x_res; y_scale = dst_y_res (j-axis up) or -dst_y_res.
 * keys: (dst_h, dst_w) uint32 scratch; ij: (2, dst_h, dst_w) float64 output
 *   (NaN where no quad hits).
 * keys_ready: 0 — the call sets keys to 0xFFFFFFFF first (on `stream`);
 *   1 — keys already hold 0xFFFFFFFF everywhere, ordered before this call
 *   (xrs_ij_bboxes_fill).  A claim pass consumes the fill.
 * ------------------------------------------------------------------------- */
int xrs_rectify_ij(const double* x, const double* y, int64_t h, int64_t w, int64_t sy,
                   const void* tiles, int64_t ntiles, int64_t ntiles_x,
                   const int64_t* chunk_offsets, int64_t max_chunks,
                   int64_t dst_h, int64_t dst_w, double x_scale, double y_scale,
                   double uv_delta, uint32_t* keys, int keys_ready, double* ij,
                   int32_t* err_flags, void* stream);

/* -------------------------------------------------------------------------
 * xrs_rectify_ij_var — xrs_rectify_ij with the first variable sampled by the
 * resolve pass itself (xrs_rectify_var's per-pixel sampling, rectify.py:
 * 605-734, fused into K5b): the variable (n, src_h, src_w) of dtype
 * src_dtype is written to dst (n, dst_h, dst_w) as xrs_rectify_var would
 * write it from the ij image.  ij may be NULL when no other variable needs
 * the positions (the ij image is then never written); else it is written as
 * by xrs_rectify_ij.  (xrs_rectify_ij's ntiles_x, unused, is omitted.)
 * ------------------------------------------------------------------------- */
int xrs_rectify_ij_var(const double* x, const double* y, int64_t h, int64_t w, int64_t sy,
                       const void* tiles, int64_t ntiles, const int64_t* chunk_offsets,
                       int64_t max_chunks, int64_t dst_h, int64_t dst_w, double x_scale,
                       double y_scale, double uv_delta, uint32_t* keys, int keys_ready,
                       double* ij, const void* src, int src_dtype, int64_t n, int64_t src_h, int64_t src_w,
                       int64_t src_sn, int64_t src_sy, void* dst, int64_t dst_sn, int interp,
                       double fill, int32_t* err_flags, void* stream);

/* -------------------------------------------------------------------------
 * xrs_rectify_tiles — the host-side tiling of _compute_target_source_ij
 * (rectify.py:312-419: per target tile its source ij bbox, via
 * ij_bboxes_from_xy_bboxes base.py:565-629 + bboxes.py:90-106, the source
 * window it scans and the tile's dst_x/y offsets) done on the device from the
 * raw K4 accumulators `acc` (xrs_ij_bboxes grid mode, ntiles_x*ntiles_y
 * boxes), so K4 -> K5 needs no host synchronisation.
 * tiles (device, ntiles records as in xrs_rectify_ij) and chunk_offsets
 * (device, ntiles + 1) are written.  j_axis_up selects y_off = dst_y_min +
 * r0*res (else dst_y_max - r0*res).
 * ------------------------------------------------------------------------- */
int xrs_rectify_tiles(const int32_t* acc, int64_t ntiles_x, int64_t ntiles_y, int64_t tile_w,
                      int64_t tile_h, int64_t dst_w, int64_t dst_h, int64_t src_w,
                      int64_t src_h, int64_t ij_border, double dst_x_min, double dst_y_min,
                      double dst_y_max, double dst_x_res, double dst_y_res, int j_axis_up,
                      void* tiles, int64_t* chunk_offsets, void* stream);

/* -------------------------------------------------------------------------
 * xrs_rectify_var — replaces _compute_var_image_block / _sequential /
 * _for_dest_line (rectify.py:605-734): sample a (n, src_h, src_w) variable
 * at the fractional source positions ij (2, dst_h, dst_w): i plane at ij, j
 * plane at ij + ij_sn (a row band of a larger ij image: ij points at the
 * band's first row, ij_sn = the whole image's plane size); nearest (u > 0.5
 * rounds up), triangular or bilinear in float64, stored in the variable
 * dtype; NaN positions -> fill.  dst: (n, dst_h, dst_w), slice stride dst_sn.
 * ------------------------------------------------------------------------- */
int xrs_rectify_var(const double* ij, int64_t ij_sn, int64_t dst_h, int64_t dst_w, const void* src,
                    int src_dtype, int64_t n, int64_t src_h, int64_t src_w, int64_t src_sn,
                    int64_t src_sy, void* dst, int64_t dst_sn, int interp, double fill,
                    int32_t* err_flags, void* stream);

/* -------------------------------------------------------------------------
 * Test-only path selection.  Every kernel has ONE schedule per case; these
 * knobs only force alternative, bit-identical code paths (or work shapes) so
 * that the parity tests can cover them.  Nothing reads the environment: a
 * process that never calls xrs_testing_set() runs the product paths.
 *   XRS_TESTING_REPROJECT_BAND            target rows per K1 work item (0 = 32)
 *   XRS_TESTING_REPROJECT_BLOCKS_PER_CU   cap K1's grid (grid-stride loop; 0 = none)
 *   XRS_TESTING_AFFINE_GENERIC            1: aligned integer coarsens take the
 *                                         generic K3 instead of K3i
 *   XRS_TESTING_RECTIFY_EXACT             1: K5 decides every triangle test and
 *                                         pixel floor by the exact division
 *   XRS_TESTING_RECTIFY_MARGIN            k > 1: K5 widens its float32 form margin
 *                                         k-fold (more pixels take the exact test)
 *   (6: retired in round 5 — K1's column-group deal, measured slower, left
 *    the product; setting it is accepted and changes nothing)
 *   XRS_TESTING_RECTIFY_PLAIN_KEYS        1: K5 claims with plain raster keys and
 *                                         the resolve tests both triangles (the
 *                                         path of swaths of 2^31 points or more)
 *   XRS_TESTING_PROJ_TWO_STEP             1: LAEA inverse -> tmerc forward runs as
 *                                         two library-transcendental steps instead
 *                                         of the fused sine / cosine pipeline
 *   XRS_TESTING_RECTIFY_COMPACT           1 / 2: K5's claim walks every tile's
 *                                         windows compacted across the wave / per
 *                                         lane (0: chosen per tile)
 * Returns the previous value (or XRS_ERR_ARG for an unknown knob).
 * ------------------------------------------------------------------------- */
#define XRS_TESTING_REPROJECT_BAND 1
#define XRS_TESTING_REPROJECT_BLOCKS_PER_CU 2
#define XRS_TESTING_AFFINE_GENERIC 3
#define XRS_TESTING_RECTIFY_EXACT 4
#define XRS_TESTING_RECTIFY_MARGIN 5
#define XRS_TESTING_RECTIFY_PLAIN_KEYS 7
#define XRS_TESTING_PROJ_TWO_STEP 8
#define XRS_TESTING_RECTIFY_COMPACT 9
#define XRS_TESTING_NUM_KNOBS 10
int64_t xrs_testing_set(int knob, int64_t value);

/* ---- coordinate transformation (reproject.py:472-496, rectify.py:182-231) --
 * xrs_transform — the reference's per-point pyproj transformation for CRS
 *   pairs that are not separable, as a pipeline of up to XRS_MAX_PROJ_STEPS
 *   PROJ operations (source -> geographic -> target: [inverse], [forward] or
 *   [inverse, forward]; degrees for geographic,
 *   metres for projected CRSs, always_xy order).  Each step restates PROJ's
 *   operation as xcube_resampling_amd/projections.py does (results agree with
 *   that numpy restatement to a few ulps: device libm).
 *   grid != 0: x (w,), y (h,) are a grid's axes, point (r, c) = (x[c], y[r]);
 *   grid == 0: x, y are (h, w) row-major images.  out_x, out_y: (h, w).
 *   steps: HOST array of nsteps records (copied at the call).
 */
#define XRS_MAX_PROJ_STEPS 4
#define XRS_PROJ_WEBMERC_FWD 1   /* degrees -> EPSG:3857 metres (merc_s, webmerc) */
#define XRS_PROJ_WEBMERC_INV 2
#define XRS_PROJ_TMERC_FWD 3     /* tmerc, poder_engsager (UTM: k0 0.9996, ...)   */
#define XRS_PROJ_TMERC_INV 4
#define XRS_PROJ_LAEA_FWD 5      /* laea, ellipsoidal                              */
#define XRS_PROJ_LAEA_INV 6

typedef struct XrsProjStep {
  int32_t kind;      /* XRS_PROJ_* */
  int32_t mode;      /* laea aspect: 0 north pole, 1 south pole, 2 equatorial, 3 oblique */
  double a, ra;      /* semi-major axis, 1 / a */
  double x0, y0;     /* false easting / northing (metres) */
  double lam0, phi0; /* central meridian / latitude of origin (radians) */
  double e, es, one_es;
  double c[24];      /* tmerc: cgb[6], cbg[6], utg[6], gtu[6] */
  double Qn, Zb;     /* tmerc */
  double qp, mmf, apa[3], rq, dd, xmf, ymf, sinb1, cosb1;   /* laea */
} XrsProjStep;

int xrs_transform(const double* x, const double* y, int64_t w, int64_t h, int grid,
                  const XrsProjStep* steps, int nsteps, double* out_x, double* out_y,
                  void* stream);

/* -------------------------------------------------------------------------
 * xrs_reproject_proj — xrs_reproject for non-separable CRS pairs with the
 * coordinate transformation fused: replaces reproject.py:472-496
 * (_transform_gridpoints: every target pixel centre -> source CRS through
 * pyproj) together with 268-335 / 499-530 (_reproject_block on the padded
 * window), per target pixel, without 2-D coordinate tables.
 * grid_x (dst_w,), grid_y (dst_h,): the target grid's pixel-centre axes
 *   (device memory); point (r, c) = (grid_x[c], grid_y[r]) is transformed by
 *   the pipeline `steps` (HOST array, as xrs_transform; the same device code,
 *   so the result equals xrs_transform + xrs_reproject(coord_mode 1) bit for
 *   bit).  Every other argument as xrs_reproject; no workspace.
 * ------------------------------------------------------------------------- */
int xrs_reproject_proj(const void* src, int src_dtype, int64_t n, int64_t src_h,
                       int64_t src_w, int64_t src_row0, int64_t src_rows,
                       int64_t src_sn, int64_t src_sy, void* dst, int dst_dtype,
                       int64_t dst_h, int64_t dst_w, int64_t row_begin,
                       int64_t row_end, int64_t dst_sn, int64_t dst_sy,
                       int64_t tile_h, int64_t tile_w, const double* grid_x,
                       const double* grid_y, const XrsProjStep* steps, int nsteps,
                       const float* tile_x0, const float* tile_y0,
                       const int64_t* tile_win, int64_t win_h, int64_t win_w,
                       double x_res, double y_res, int interp, double fill,
                       int32_t* err_flags, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* XRS_H_ */
