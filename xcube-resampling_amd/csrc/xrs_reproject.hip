// xrs_reproject.hip — K1: regular->regular reprojection gather for gfx950.
//
// Replaces, for all target tiles of one variable in ONE call:
//   * reproject._reproject_block            (reproject.py:268-335)  per-tile gather/lerp
//   * reproject._reorganize_data_array_slice (reproject.py:499-530)  pad + window copy
// The per-tile window geometry (reproject._get_scr_bboxes_indices,
// reproject.py:385-469) is computed by the host and passed as small tables.
//
// Separable CRS pairs (coord_mode 0: target x -> source x only, y -> y only,
// e.g. EPSG:3857 -> EPSG:4326) run ONE launch, K1b, the HBM-bound gather.
// One work item = one tile x one 512-column segment x one band of kBand rows,
// so the tile (and every row entry) is block-uniform: row pointers are scalar,
// lane offsets 32-bit.  The item resolves the reference's per-pixel index math
// itself — ix = (sx-x0)/res, floor/ceil/rint, int16 cast, python-style window
// wrap, window -> source index, pad -> "outside" — for its own columns (one
// per lane and column, from the source-CRS column coordinate src_x[c]) and its
// own rows (lane q of every wave resolves row r0 + q; the batch reads the
// entries back by readlane).  Bit-exact because for separable transforms the
// per-pixel ix only depends on the column (iy on the row).  Lanes take
// consecutive columns (each wave-load touches ~256 contiguous source bytes);
// the loads of kRows target rows are issued before any is consumed
// (memory-level parallelism); stores are non-temporal.  The ceil/floor overlap
// between neighbouring rows and columns is served by L1/L2.
// (Rounds 1-4 resolved the entries in a separate K1a launch into 16-byte
// tables; every item re-fetched its 512 x entries through the fabric: reads
// 1.154x the algorithmic bytes.  DESIGN.md §3 "K1, round 5".)
// Non-separable pairs (coord_mode 1: 2-D coordinate tables) run K1c, the same
// work decomposition with the index math done per pixel.
//
// Index and weight math is float64 without contraction (-ffp-contract=off) so
// nearest picks and lerp weights are bit-identical to numpy's.
//
// The product library holds exactly one schedule per path.  The alternative
// schedules measured in round 1 (carried rows, LDS-staged footprints,
// wave-private LDS rings, 16-byte tap runs, transposed stores, two-phase row
// loads, ...) are documented in DESIGN.md §3 with their timings; experiments
// live in probes/ and are never linked into libxrs.so.

#include <cstdlib>
#include <type_traits>

#include "xrs_common.hpp"
#include "xrs_proj.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;
constexpr int kPx = 2;                       // columns per thread
constexpr int kSegW = kThreads * kPx;        // columns per work item
constexpr int kBand = 32;                    // target rows per work item
constexpr int kRows = 8;                     // target rows whose loads are in flight together

// K1b's work shape per output width.  float32 out: 512 columns x 32 rows,
// 8 rows in flight.  float64 out (the reference's bilinear dtype, twice the
// store bytes): 1024 columns x 12 rows, 4 rows in flight — with the round-5
// prologue 2 % faster than the 8-row bands of rounds 3-4 (3.533 vs 3.603-3.615
// ms at config 5, profiles/r05_k1_f64out_shapes_ab.jsonl; 512 x 16 3.56,
// 1024 x 16 3.58, 512 x 32 3.60); each output width takes its own shape
// (profiles/r03_k1_shapes_ab.jsonl).
template <typename O>
struct K1Shape {
  static constexpr int px = sizeof(O) == 8 ? 4 : kPx;
  static constexpr int band = sizeof(O) == 8 ? 12 : kBand;
  static constexpr int rows = sizeof(O) == 8 ? 4 : kRows;
  static constexpr int segw = kThreads * px;
};
constexpr int kRows2D = 2;                   // K1c: target rows per step (2-D tables; 4: slower)

struct AxisEntry {   // one resolved column (or row) of one tile
  int32_t f;         // source index of floor(ix) (nearest: of rint(ix)); -1 = outside source
  int32_t c;         // source index of ceil(ix); -1 = outside source
  double d;          // ix - (double)(int16)floor(ix)
};
static_assert(sizeof(AxisEntry) == 16, "AxisEntry layout");

// coord_mode 2: the source-CRS x of target column c in tile column tx, as the
// host computes it (dask's blockwise linspace of the pixel centres,
// regular.py:44-52, then the separable transformation's scalings,
// reproject.py:472-496): v = k == n-1 ? stop : k * step + start (k = c - tx *
// tile_w), x = (v * m1) * m2.  src_x then holds ntiles_x records followed by
// (m1, m2); the host uses this mode only after checking it bit for bit.
struct ColumnGen {
  double start, stop, step, n;
};
static_assert(sizeof(ColumnGen) == 32, "ColumnGen layout");

struct Geometry {
  int64_t src_h, src_w, src_row0, src_rows;
  int64_t dst_h, dst_w, row_begin, row_end;
  int64_t tile_h, tile_w, ntiles_x, ntiles_y;
  const double* src_x;
  const double* src_y;
  const float* tile_x0;
  const float* tile_y0;
  const int64_t* tile_win;
  int64_t win_h, win_w;
  double x_res, neg_y_res;
  int32_t* err_flags;
  int64_t band;   // target rows per work item of the gathers
  int64_t segw;   // target columns per work item (kThreads x columns per thread)
  int64_t band_first;   // bands of tile row ty0 above row_begin (not in the work list)
  int64_t xgen;         // K1b: src_x holds column generators (coord_mode 2, ColumnGen)
};

// numpy fancy index on a window axis of length `win` with an int16 index:
// negative indices wrap once (python semantics), anything else outside
// [0, win) is an IndexError (reproject.py:284,292-295,322-325).
__device__ inline bool window_index(int16_t idx16, int64_t win, int64_t& out) {
  int64_t i = idx16;
  if (i < 0) i += win;
  out = i;
  return i >= 0 && i < win;
}

// Window position -> source index along one axis; -1 when the window position
// lies in the constant-padded region (outside the source).  Rows are returned
// relative to the band held on this device.
__device__ inline int32_t to_source(int64_t w0, int64_t widx, int64_t size, int64_t band0,
                                    int64_t band_len, int32_t& eflags) {
  const int64_t g = w0 + widx;
  if (g < 0 || g >= size) return -1;
  const int64_t l = g - band0;
  if (l < 0 || l >= band_len) {
    eflags |= XRS_EFLAG_BAND;
    return -1;
  }
  return (int32_t)l;
}

// The reference's index math for one coordinate along one axis
// (reproject.py:278-283 nearest, 286-291 / 316-321 floor/ceil/diff).
template <int INTERP>
__device__ inline AxisEntry resolve_axis(double coord, float origin, double res, int64_t win,
                                         int64_t w0, int64_t size, int64_t band0,
                                         int64_t band_len, int32_t& eflags) {
  const double i = (coord - (double)origin) / res;
  AxisEntry e;
  if (INTERP == XRS_INTERP_NEAREST) {
    int64_t wi;
    if (window_index(f64_to_i16_np(rint(i)), win, wi)) {
      e.f = to_source(w0, wi, size, band0, band_len, eflags);
    } else {
      eflags |= XRS_EFLAG_INDEX;
      e.f = -1;
    }
    e.c = e.f;
    e.d = 0.0;
  } else {
    const int16_t fi = f64_to_i16_np(floor(i)), ci = f64_to_i16_np(ceil(i));
    e.d = i - (double)fi;
    int64_t wf, wc;
    const bool okf = window_index(fi, win, wf);
    const bool okc = window_index(ci, win, wc);
    if (!okf || !okc) eflags |= XRS_EFLAG_INDEX;
    e.f = okf ? to_source(w0, wf, size, band0, band_len, eflags) : -1;
    e.c = okc ? to_source(w0, wc, size, band0, band_len, eflags) : -1;
  }
  return e;
}

// resolve_axis for the per-pixel gathers (K1c, K1p): the same entries with
// 32-bit index arithmetic whenever every quantity fits (window and band
// bounds below 2^30, |window origin| <= 2^30: no sum or difference below can
// leave int32); otherwise resolve_axis itself.
template <int INTERP>
__device__ inline AxisEntry resolve_axis_px(double coord, float origin, double res, int64_t win,
                                            int64_t w0, int64_t size, int64_t band0,
                                            int64_t band_len, int32_t& eflags) {
  constexpr int64_t kLim = int64_t(1) << 30;
  if (!(win <= kLim && size <= INT32_MAX && band0 >= 0 && band0 <= kLim && band_len <= INT32_MAX &&
        w0 >= -kLim && w0 <= kLim))
    return resolve_axis<INTERP>(coord, origin, res, win, w0, size, band0, band_len, eflags);
  const int32_t win32 = (int32_t)win, w032 = (int32_t)w0, size32 = (int32_t)size;
  const int32_t b032 = (int32_t)band0, bl32 = (int32_t)band_len;
  auto window32 = [&](int16_t idx16, int32_t& out) {
    int32_t i = idx16;
    if (i < 0) i += win32;
    out = i;
    return i >= 0 && i < win32;
  };
  auto source32 = [&](int32_t widx) -> int32_t {
    const int32_t g = w032 + widx;
    if (g < 0 || g >= size32) return -1;
    const int32_t l = g - b032;
    if (l < 0 || l >= bl32) {
      eflags |= XRS_EFLAG_BAND;
      return -1;
    }
    return l;
  };
  const double i = (coord - (double)origin) / res;
  AxisEntry e;
  if (INTERP == XRS_INTERP_NEAREST) {
    int32_t wi;
    if (window32(f64_to_i16_np(rint(i)), wi)) {
      e.f = source32(wi);
    } else {
      eflags |= XRS_EFLAG_INDEX;
      e.f = -1;
    }
    e.c = e.f;
    e.d = 0.0;
  } else {
    const int16_t fi = f64_to_i16_np(floor(i)), ci = f64_to_i16_np(ceil(i));
    e.d = i - (double)fi;
    int32_t wf, wc;
    const bool okf = window32(fi, wf);
    const bool okc = window32(ci, wc);
    if (!okf || !okc) eflags |= XRS_EFLAG_INDEX;
    e.f = okf ? source32(wf) : -1;
    e.c = okc ? source32(wc) : -1;
  }
  return e;
}

// ---- interpolation of one pixel (reproject.py:304-314, 326-328) ------------
template <typename T, int INTERP>
__device__ inline double interp4(T v00, T v01, T v10, T v11, double dx, double dy) {
  if (INTERP == XRS_INTERP_BILINEAR) {
    const double u0 = Conv<T>::to_f64(v00) + dx * Conv<T>::to_f64(Conv<T>::diff(v01, v00));
    const double u1 = Conv<T>::to_f64(v10) + dx * Conv<T>::to_f64(Conv<T>::diff(v11, v10));
    return u0 + dy * (u1 - u0);
  }
  if (dx + dy < 1.0)  // closest triangle
    return Conv<T>::to_f64(v00) + dx * Conv<T>::to_f64(Conv<T>::diff(v01, v00)) +
           dy * Conv<T>::to_f64(Conv<T>::diff(v10, v00));
  return Conv<T>::to_f64(v11) + (1.0 - dx) * Conv<T>::to_f64(Conv<T>::diff(v10, v11)) +
         (1.0 - dy) * Conv<T>::to_f64(Conv<T>::diff(v01, v11));
}

// A wave-uniform source row as a buffer resource (4 SGPRs): its taps are
// buffer loads with a 32-bit lane byte offset — no 64-bit address per lane
// (VALU and VGPRs the 16 tap rows of a batch no longer pay)
__device__ inline __amdgpu_buffer_rsrc_t row_rsrc(const void* row, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(row), 0, (int)bytes, 0x00020000);
}
template <typename T>
__device__ inline T row_at(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  if constexpr (sizeof(T) == 1) {
    return __builtin_bit_cast(T, (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rs, off, 0, 0));
  } else if constexpr (sizeof(T) == 2) {
    return __builtin_bit_cast(T, (uint16_t)__builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0));
  } else if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
  }
}

struct GatherArgs {
  Geometry g;
  const void* src;
  int64_t n, src_sn, src_sy;
  void* dst;
  int64_t dst_sn, dst_sy;
  double fill;
};

// Work decomposition shared by K1b/K1c: bands of kBand rows inside one tile row
// x segments of kSegW columns inside one tile column, band-major; the XCDs
// take whole bands in turn (XCD x: bands x, x + 8, ...).  The list starts at
// the band holding row_begin and ends at the band holding row_end - 1, so a
// row band of the raster (a rank's share) has no empty items (blocks are dealt
// to XCDs round-robin whatever their cost: empty items would idle an XCD).
// Returns false for empty items (partial edge tiles).
struct WorkItem {
  int64_t t, ty, tx, r0, r1, c0, c1;
};
__device__ inline bool work_item(const Geometry& g, int64_t w, int64_t ty0, int64_t nsegs,
                                 int64_t bands_per_tile, int64_t segs_per_tile, WorkItem& it) {
  const int64_t bw = w / nsegs, s = w - bw * nsegs;
  const int64_t b = bw + g.band_first;
  const int64_t tyi = b / bands_per_tile;
  it.ty = ty0 + tyi;
  const int64_t bi = b - tyi * bands_per_tile;
  const int64_t tr0 = it.ty * g.tile_h;
  it.r0 = max(g.row_begin, tr0 + bi * g.band);
  it.r1 = min(min(g.row_end, tr0 + g.tile_h), tr0 + bi * g.band + g.band);
  it.tx = s / segs_per_tile;
  const int64_t si = s - it.tx * segs_per_tile;
  it.c0 = it.tx * g.tile_w + si * g.segw;
  it.c1 = min(min(g.dst_w, it.tx * g.tile_w + g.tile_w), it.c0 + g.segw);
  it.t = it.ty * g.ntiles_x + it.tx;
  return it.r0 < it.r1 && it.c0 < it.c1;
}

// ---- K1b: separable gather --------------------------------------------------
// No rows are carried between target rows: every target row loads its two
// source rows (their overlap with the neighbouring rows is served by L1/L2),
// but the loads of kRows target rows are independent and in flight together.
// The item's axis entries are resolved in the item (header): its columns'
// from src_x (8 B per column, L2-resident: the whole raster's column
// coordinates are 320 KB), its rows' by lane, 64 rows per resolve.
template <typename T, typename O, int INTERP>
__global__ void __launch_bounds__(kThreads)
gather_separable_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                        int64_t segs_per_tile, int64_t nwork) {
  const Geometry& g = a.g;
  constexpr int kPx = K1Shape<O>::px, kRows = K1Shape<O>::rows;
  static_assert(64 % kRows == 0, "a 64-row entry chunk holds whole batches");
  const T fill = Conv<T>::from_f64(a.fill);
  const int lane = (int)(threadIdx.x & 63);
  int32_t eflags = 0;
  // the XCDs take whole bands in turn (XCD x: bands x, x + 8, ...)
  const int64_t xcd = blockIdx.x & 7;
  for (int64_t i = blockIdx.x >> 3;; i += gridDim.x >> 3) {
    const int64_t m = i / nsegs;
    const int64_t w = (m * 8 + xcd) * nsegs + (i - m * nsegs);
    if (w >= nwork) break;
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const int ncols = (int)(it.c1 - it.c0);
    // this item's columns and its first 64 rows: the source-CRS coordinates
    // are requested together (one memory round trip before the taps), then
    // resolved
    const float x0 = g.tile_x0[it.t];
    const int64_t wi0 = g.tile_win[2 * it.t];
    const float y0 = g.tile_y0[it.t];
    const int64_t wj0 = g.tile_win[2 * it.t + 1];
    double sx[kPx];
    if (g.xgen) {
      // coord_mode 2: the column coordinates from the tile column's
      // generator — the host checked it reproduces src_x bit for bit
      const ColumnGen cg = reinterpret_cast<const ColumnGen*>(g.src_x)[it.tx];
      const double m1 = g.src_x[4 * g.ntiles_x], m2 = g.src_x[4 * g.ntiles_x + 1];
      const int last = (int)cg.n - 1, k0 = (int)(it.c0 - it.tx * g.tile_w);
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const int kk = k0 + min((int)threadIdx.x + k * kThreads, ncols - 1);
        const double v = kk == last ? cg.stop : (double)kk * cg.step + cg.start;
        sx[k] = (v * m1) * m2;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const int lc = (int)threadIdx.x + k * kThreads;
        sx[k] = g.src_x[it.c0 + min(lc, ncols - 1)];
      }
    }
    const int64_t ry0 = it.r0 + lane;
    const double sy0 = g.src_y[min(ry0, it.r1 - 1)];
    int32_t cf[kPx], cc[kPx];
    double dx[kPx];
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      const int lc = (int)threadIdx.x + k * kThreads;
      AxisEntry e{-1, -1, 0.0};
      if (lc < ncols)
        e = resolve_axis<INTERP>(sx[k], x0, g.x_res, g.win_w, wi0, g.src_w, 0, g.src_w, eflags);
      cf[k] = e.f;
      cc[k] = e.c;
      dx[k] = e.d;
    }
    const uint32_t row_bytes = (uint32_t)(g.src_w * (int64_t)sizeof(T));
    // byte offsets of the tap columns in a row (< 2^31: checked at launch)
    uint32_t fo[kPx], co[kPx];
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      fo[k] = (uint32_t)max(cf[k], 0) * (uint32_t)sizeof(T);
      co[k] = (uint32_t)max(cc[k], 0) * (uint32_t)sizeof(T);
    }
    // this item's rows: lane q holds the entry of row ybase + q (rows past
    // r1 hold "outside", as the batches expect); one resolve per 64 rows
    int32_t yf = -1, yc = -1;
    double yd = 0.0;
    int64_t ybase = it.r0;
    if (ry0 < it.r1) {
      const AxisEntry e = resolve_axis<INTERP>(sy0, y0, g.neg_y_res, g.win_h, wj0, g.src_h,
                                               g.src_row0, g.src_rows, eflags);
      yf = e.f;
      yc = e.c;
      yd = e.d;
    }
    for (int64_t sn = 0; sn < a.n; ++sn) {
      const T* __restrict__ src = static_cast<const T*>(a.src) + sn * a.src_sn;
      O* __restrict__ dst = static_cast<O*>(a.dst) + sn * a.dst_sn - g.row_begin * a.dst_sy + it.c0;
      // stores are deferred by one batch: a store's data register stays
      // busy until the store completes, so the previous batch's stores are
      // issued after this batch's loads (they no longer hold the loads back)
      O outv[kRows][kPx];
      int64_t rprev = -1;
      auto flush = [&](int64_t rp) {
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
          if (rp + q >= it.r1) break;
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            const int lc = (int)threadIdx.x + k * kThreads;
            if (lc < ncols) __builtin_nontemporal_store(outv[q][k], &dst[(rp + q) * a.dst_sy + lc]);
          }
        }
      };
      for (int64_t r = it.r0; r < it.r1; r += kRows) {
        if (r < ybase || r >= ybase + 64) {   // wave-uniform; once per item for bands <= 64
          ybase = r;
          const int64_t ry = r + lane;
          AxisEntry e{-1, -1, 0.0};
          if (ry < it.r1)
            e = resolve_axis<INTERP>(g.src_y[ry], y0, g.neg_y_res, g.win_h, wj0, g.src_h,
                                     g.src_row0, g.src_rows, eflags);
          yf = e.f;
          yc = e.c;
          yd = e.d;
        }
        const int j0 = (int)(r - ybase);
        AxisEntry ye[kRows];
        T v[kRows][4][kPx];
        // all taps of kRows target rows requested before any is used; entries
        // outside the source (-1) read element 0 of the band (a valid address)
        // and are replaced by the fill value below
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
          ye[q].f = __builtin_amdgcn_readlane(yf, j0 + q);
          ye[q].c = __builtin_amdgcn_readlane(yc, j0 + q);
          const uint64_t db = __builtin_bit_cast(uint64_t, yd);
          const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)db, j0 + q);
          const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(db >> 32), j0 + q);
          ye[q].d = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
          const __amdgpu_buffer_rsrc_t rf =
              row_rsrc(src + (int64_t)max(ye[q].f, 0) * a.src_sy, row_bytes);
          const __amdgpu_buffer_rsrc_t rc =
              row_rsrc(src + (int64_t)max(ye[q].c, 0) * a.src_sy, row_bytes);
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            v[q][0][k] = row_at<T>(rf, fo[k]);
            if (INTERP != XRS_INTERP_NEAREST) {
              v[q][1][k] = row_at<T>(rf, co[k]);
              v[q][2][k] = row_at<T>(rc, fo[k]);
              v[q][3][k] = row_at<T>(rc, co[k]);
            }
          }
        }
        if (rprev >= 0) flush(rprev);
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
          const bool okf = ye[q].f >= 0, okc = ye[q].c >= 0;
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            const bool xf = cf[k] >= 0, xc = cc[k] >= 0;
            const T v00 = (okf && xf) ? v[q][0][k] : fill;
            if (INTERP == XRS_INTERP_NEAREST) {
              outv[q][k] = (O)v00;
            } else {
              const T v01 = (okf && xc) ? v[q][1][k] : fill;
              const T v10 = (okc && xf) ? v[q][2][k] : fill;
              const T v11 = (okc && xc) ? v[q][3][k] : fill;
              outv[q][k] = Conv<O>::from_f64(interp4<T, INTERP>(v00, v01, v10, v11, dx[k], ye[q].d));
            }
          }
        }
        rprev = r;
      }
      if (rprev >= 0) flush(rprev);
    }
  }
  if (eflags) atomicOr(g.err_flags, eflags);
}

// ---- one target pixel of every dim-0 slice, from its resolved entries -------
template <typename T, typename O, int INTERP>
__device__ inline void gather_pixel(const GatherArgs& a, int64_t r, int64_t col,
                                    const AxisEntry& ex, const AxisEntry& ey) {
  const T fill = Conv<T>::from_f64(a.fill);
  for (int64_t sn = 0; sn < a.n; ++sn) {
    const T* src = static_cast<const T*>(a.src) + sn * a.src_sn;
    O* dst = static_cast<O*>(a.dst) + sn * a.dst_sn + (r - a.g.row_begin) * a.dst_sy;
    auto at = [&](int32_t row, int32_t c) -> T {
      return (row >= 0 && c >= 0) ? src[(int64_t)row * a.src_sy + c] : fill;
    };
    if (INTERP == XRS_INTERP_NEAREST) {
      dst[col] = (O)at(ey.f, ex.f);
    } else {
      const double v = interp4<T, INTERP>(at(ey.f, ex.f), at(ey.f, ex.c), at(ey.c, ex.f),
                                          at(ey.c, ex.c), ex.d, ey.d);
      dst[col] = Conv<O>::from_f64(v);
    }
  }
}

// ---- K1c: per-pixel gather (2-D coordinate tables) --------------------------
template <typename T, typename O, int INTERP>
__global__ void __launch_bounds__(kThreads)
gather_2d_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                 int64_t segs_per_tile, int64_t nwork) {
  const Geometry& g = a.g;
  int32_t eflags = 0;
  for (XcdGroups sl = xcd_groups(nwork, nsegs);; sl.i += sl.step) {
    const int64_t w = sl.item();
    if (w >= nwork) break;
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const int ncols = (int)(it.c1 - it.c0);
    const float x0 = g.tile_x0[it.t], y0 = g.tile_y0[it.t];
    const int64_t wi0 = g.tile_win[2 * it.t], wj0 = g.tile_win[2 * it.t + 1];
    // kRows2D rows x kPx columns per step: their table entries, then every
    // tap of a slice, are requested together (one dependent chain per step
    // instead of per pixel)
    for (int64_t r = it.r0; r < it.r1; r += kRows2D) {
      bool ok[kRows2D][kPx];
      double sx[kRows2D][kPx], sy[kRows2D][kPx];
#pragma unroll
      for (int q = 0; q < kRows2D; ++q)
#pragma unroll
        for (int k = 0; k < kPx; ++k) {
          const int lc = (int)threadIdx.x + k * kThreads;
          ok[q][k] = r + q < it.r1 && lc < ncols;
          const int64_t p = ok[q][k] ? (r + q) * g.dst_w + it.c0 + lc : it.r0 * g.dst_w + it.c0;
          sx[q][k] = g.src_x[p];
          sy[q][k] = g.src_y[p];
        }
      AxisEntry ex[kRows2D][kPx], ey[kRows2D][kPx];
#pragma unroll
      for (int q = 0; q < kRows2D; ++q)
#pragma unroll
        for (int k = 0; k < kPx; ++k) {
          ex[q][k] = ey[q][k] = AxisEntry{-1, -1, 0.0};
          if (ok[q][k]) {
            ex[q][k] = resolve_axis_px<INTERP>(sx[q][k], x0, g.x_res, g.win_w, wi0, g.src_w, 0,
                                            g.src_w, eflags);
            ey[q][k] = resolve_axis_px<INTERP>(sy[q][k], y0, g.neg_y_res, g.win_h, wj0, g.src_h,
                                            g.src_row0, g.src_rows, eflags);
          }
        }
      // the tap phase's arguments re-read here (kernel_arg_after: SGPR spills)
      const GatherArgs ga = kernel_arg_after<GatherArgs>(ex[0][0].d);
      const T fill = Conv<T>::from_f64(ga.fill);
      for (int64_t sn = 0; sn < ga.n; ++sn) {
        const T* src = static_cast<const T*>(ga.src) + sn * ga.src_sn;
        O* dst = static_cast<O*>(ga.dst) + sn * ga.dst_sn + (r - ga.g.row_begin) * ga.dst_sy + it.c0;
        auto at = [&](int32_t row, int32_t c) -> T {
          return src[(int64_t)max(row, 0) * ga.src_sy + max(c, 0)];
        };
        T t[kRows2D][kPx][4];
#pragma unroll
        for (int q = 0; q < kRows2D; ++q)
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            t[q][k][0] = at(ey[q][k].f, ex[q][k].f);
            if (INTERP != XRS_INTERP_NEAREST) {
              t[q][k][1] = at(ey[q][k].f, ex[q][k].c);
              t[q][k][2] = at(ey[q][k].c, ex[q][k].f);
              t[q][k][3] = at(ey[q][k].c, ex[q][k].c);
            }
          }
#pragma unroll
        for (int q = 0; q < kRows2D; ++q)
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            if (!ok[q][k]) continue;
            const AxisEntry& fx = ex[q][k];
            const AxisEntry& fy = ey[q][k];
            const T v00 = (fy.f >= 0 && fx.f >= 0) ? t[q][k][0] : fill;
            O out;
            if (INTERP == XRS_INTERP_NEAREST) {
              out = (O)v00;
            } else {
              const T v01 = (fy.f >= 0 && fx.c >= 0) ? t[q][k][1] : fill;
              const T v10 = (fy.c >= 0 && fx.f >= 0) ? t[q][k][2] : fill;
              const T v11 = (fy.c >= 0 && fx.c >= 0) ? t[q][k][3] : fill;
              out = Conv<O>::from_f64(interp4<T, INTERP>(v00, v01, v10, v11, fx.d, fy.d));
            }
            dst[q * ga.dst_sy + (int)threadIdx.x + k * kThreads] = out;
          }
      }
    }
  }
  if (eflags) atomicOr(g.err_flags, eflags);
}

// ---- K1p: per-pixel gather with the projection fused (non-separable pairs) --
constexpr int kModeAny = -1;
constexpr int kModeF32Nearest = XRS_DTYPE_F32 * 4 + 0;
constexpr int kModeF32BilinearF64 = XRS_DTYPE_F32 * 4 + 3;
constexpr int kModeF64BilinearF64 = XRS_DTYPE_F64 * 4 + 3;
// reproject.py:472-496 + 268-335 for one target pixel: its centre
// (grid_x[c], grid_y[r]) goes through the pipeline (xrs_proj.hpp, the code
// xrs_transform runs), then the index math and the taps of every dim-0 slice.
// No coordinate tables: 32 B/px less HBM traffic than xrs_transform + K1c (a
// plan reused by several variables keeps the tables; the host decides).  The
// pipeline is the template (its registers dominate); source / output dtype
// and interpolation are a wave-uniform switch (`mode` = dtype code x 4 +
// variant: 0 nearest, 1 triangular, 2 bilinear -> f32, 3 bilinear -> f64).
__device__ inline void gather_pixel_any(int mode, const GatherArgs& a, int64_t r, int64_t col,
                                        const AxisEntry& ex, const AxisEntry& ey) {
  const int v = mode & 3;
  switch (mode >> 2) {
#define XRS_GP(CODE, T)                                                              \
  case CODE:                                                                         \
    if (v == 0) gather_pixel<T, T, XRS_INTERP_NEAREST>(a, r, col, ex, ey);           \
    else if (v == 1) gather_pixel<T, T, XRS_INTERP_TRIANGULAR>(a, r, col, ex, ey);   \
    else if (v == 2) gather_pixel<T, float, XRS_INTERP_BILINEAR>(a, r, col, ex, ey); \
    else gather_pixel<T, double, XRS_INTERP_BILINEAR>(a, r, col, ex, ey);            \
    break;
    XRS_GP(XRS_DTYPE_U8, uint8_t)
    XRS_GP(XRS_DTYPE_I8, int8_t)
    XRS_GP(XRS_DTYPE_U16, uint16_t)
    XRS_GP(XRS_DTYPE_I16, int16_t)
    XRS_GP(XRS_DTYPE_U32, uint32_t)
    XRS_GP(XRS_DTYPE_I32, int32_t)
    XRS_GP(XRS_DTYPE_I64, int64_t)
    XRS_GP(XRS_DTYPE_F32, float)
    XRS_GP(XRS_DTYPE_F64, double)
#undef XRS_GP
    default: break;
  }
}

// one (dtype, variant) as a template: the hot modes get kernels of their own
// (the switch keeps every case's arguments live, and those SGPRs spilled into
// VGPR lanes and were read back inside the projection)
template <int MODE>
__device__ inline void gather_pixel_mode(const GatherArgs& a, int64_t r, int64_t col,
                                         const AxisEntry& ex, const AxisEntry& ey) {
  if constexpr (MODE == kModeF32Nearest)
    gather_pixel<float, float, XRS_INTERP_NEAREST>(a, r, col, ex, ey);
  else if constexpr (MODE == kModeF32BilinearF64)
    gather_pixel<float, double, XRS_INTERP_BILINEAR>(a, r, col, ex, ey);
  else if constexpr (MODE == kModeF64BilinearF64)
    gather_pixel<double, double, XRS_INTERP_BILINEAR>(a, r, col, ex, ey);
}

// n / d for n < 2^31 by a multiply-high (the round-up method: m = floor(2^32
// (2^l - d) / d) + 1, l = ceil(log2 d); exact for every such n and d >= 1)
struct DivU32 {
  uint32_t m, l;
  static DivU32 make(uint32_t d) {
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    return DivU32{(uint32_t)((((1ull << l) - d) << 32) / d + 1), l};
  }
  __device__ uint32_t div(uint32_t n) const { return (__umulhi(n, m) + n) >> l; }
};

template <int K0, int K1, int FAST, int MODE>
__global__ void __launch_bounds__(kThreads)
gather_proj_kernel(GatherArgs a, XrsProjStep s0, XrsProjStep s1, int mode, DivU32 div_th,
                   DivU32 div_tw) {
  const proj::Pipeline<K0, K1, FAST> pipe(s0, s1);
  // one target pixel per thread and step, grid-stride over the rows of the
  // launch (lanes on consecutive columns): the loop carries almost no state
  // beside the projection's registers (a tile-item loop cost it one wave per
  // SIMD of occupancy)
  const Geometry& g = a.g;
  const bool nearest = MODE >= 0 ? (MODE & 3) == 0 : (mode & 3) == 0;
  const uint32_t w32 = (uint32_t)g.dst_w;
  const int64_t np = (g.row_end - g.row_begin) * g.dst_w;
  // the pixel's row and column step by (S / W, S % W) per grid stride S (no
  // 64-bit division per pixel); rows and columns are < 2^31 (checked at launch)
  const int64_t q0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int64_t S = (int64_t)gridDim.x * kThreads;
  const uint32_t sr = (uint32_t)(S / g.dst_w), sc = (uint32_t)(S - (int64_t)sr * g.dst_w);
  uint32_t r = (uint32_t)(g.row_begin + q0 / g.dst_w), c = (uint32_t)(q0 % g.dst_w);
  int32_t eflags = 0;
  for (int64_t q = q0; q < np; q += S) {
    double px = g.src_x[c], py = g.src_y[r];   // the target pixel centre
    pipe(s0, s1, px, py);
    // the gather's arguments re-read after the projection (kernel_arg_after:
    // kept live through it, they spilled ~110 SGPRs' reads into the projection)
    const GatherArgs ga = kernel_arg_after<GatherArgs>(px);
    const Geometry& gg = ga.g;
    const uint32_t t = div_th.div(r) * (uint32_t)gg.ntiles_x + div_tw.div(c);
    const float x0 = gg.tile_x0[t], y0 = gg.tile_y0[t];
    const int64_t wi0 = gg.tile_win[2 * t], wj0 = gg.tile_win[2 * t + 1];
    AxisEntry ex, ey;
    if (nearest) {
      ex = resolve_axis_px<XRS_INTERP_NEAREST>(px, x0, gg.x_res, gg.win_w, wi0, gg.src_w, 0, gg.src_w,
                                            eflags);
      ey = resolve_axis_px<XRS_INTERP_NEAREST>(py, y0, gg.neg_y_res, gg.win_h, wj0, gg.src_h,
                                            gg.src_row0, gg.src_rows, eflags);
    } else {
      ex = resolve_axis_px<XRS_INTERP_BILINEAR>(px, x0, gg.x_res, gg.win_w, wi0, gg.src_w, 0, gg.src_w,
                                             eflags);
      ey = resolve_axis_px<XRS_INTERP_BILINEAR>(py, y0, gg.neg_y_res, gg.win_h, wj0, gg.src_h,
                                             gg.src_row0, gg.src_rows, eflags);
    }
    if constexpr (MODE >= 0)
      gather_pixel_mode<MODE>(ga, r, c, ex, ey);
    else
      gather_pixel_any(mode, ga, r, c, ex, ey);
    c += sc;
    r += sr;
    if (c >= w32) {
      c -= w32;
      ++r;
    }
  }
  if (eflags) atomicOr(g.err_flags, eflags);
}

// Work decomposition of the gathers (K1b/K1c/K1p): bands from the one holding
// row_begin to the one holding row_end - 1, all segments of a band together.
struct Work {
  GatherArgs args;
  int64_t ty0, ty1, nsegs, bands_per_tile, segs_per_tile, nwork;
  int nb;
};
inline Work work_of(const GatherArgs& a, int64_t band = kBand, int64_t segw = kSegW) {
  const Geometry& g = a.g;
  Work k;
  k.args = a;
  k.ty0 = g.row_begin / g.tile_h;
  k.ty1 = (g.row_end - 1) / g.tile_h + 1;
  // band height / grid cap: fixed in the product; xrs_testing_set() can change
  // them so the tests cover items that split tiles and the grid-stride loop
  const int64_t band_knob = xrs_testing_value(XRS_TESTING_REPROJECT_BAND);
  k.args.g.band = band_knob > 0 ? band_knob : band;
  k.args.g.segw = segw;
  k.bands_per_tile = (g.tile_h + k.args.g.band - 1) / k.args.g.band;
  k.segs_per_tile = (g.tile_w + k.args.g.segw - 1) / k.args.g.segw;
  k.nsegs = g.ntiles_x * k.segs_per_tile;
  k.args.g.band_first = (g.row_begin - k.ty0 * g.tile_h) / k.args.g.band;
  const int64_t band_last = (k.ty1 - 1 - k.ty0) * k.bands_per_tile +
                            (g.row_end - 1 - (k.ty1 - 1) * g.tile_h) / k.args.g.band;
  k.nwork = (band_last - k.args.g.band_first + 1) * k.nsegs;
  // One work item per block (measured fastest: short blocks let the dispatcher
  // balance the CUs and keep each XCD's concurrent row set L2-sized; a
  // persistent grid of 8 blocks/CU was 12 % slower).
  const int64_t bpc = xrs_testing_value(XRS_TESTING_REPROJECT_BLOCKS_PER_CU);
  k.nb = grid_blocks(k.nwork, 1, bpc > 0 ? (int)(256 * bpc) : (1 << 24));
  return k;
}

template <typename T, typename O, int INTERP>
int launch(const GatherArgs& a, int coord_mode, hipStream_t stream) {
  Work k = coord_mode != 1 ? work_of(a, K1Shape<O>::band, K1Shape<O>::segw) : work_of(a);
  if (coord_mode != 1) {
    hipLaunchKernelGGL((gather_separable_kernel<T, O, INTERP>), dim3(k.nb), dim3(kThreads), 0,
                       stream, k.args, k.ty0, k.nsegs, k.bands_per_tile, k.segs_per_tile, k.nwork);
  } else {
    hipLaunchKernelGGL((gather_2d_kernel<T, O, INTERP>), dim3(k.nb), dim3(kThreads), 0, stream,
                       k.args, k.ty0, k.nsegs, k.bands_per_tile, k.segs_per_tile, k.nwork);
  }
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

template <int K0, int K1, int FAST>
void launch_proj_mode(int nb, const GatherArgs& a, const XrsProjStep& s0, const XrsProjStep& s1,
                      int mode, hipStream_t stream) {
  const DivU32 dh = DivU32::make((uint32_t)a.g.tile_h), dw = DivU32::make((uint32_t)a.g.tile_w);
  switch (mode) {
#define XRS_KP(M)                                                                          \
  case M:                                                                                  \
    hipLaunchKernelGGL((gather_proj_kernel<K0, K1, FAST, M>), dim3(nb), dim3(kThreads), 0, \
                       stream, a, s0, s1, mode, dh, dw);                                   \
    break;
    XRS_KP(kModeF32Nearest)
    XRS_KP(kModeF32BilinearF64)
    XRS_KP(kModeF64BilinearF64)
#undef XRS_KP
    default:
      hipLaunchKernelGGL((gather_proj_kernel<K0, K1, FAST, kModeAny>), dim3(nb), dim3(kThreads),
                         0, stream, a, s0, s1, mode, dh, dw);
  }
}

template <int K0, int K1>
int launch_proj(const GatherArgs& a, const XrsProjStep& s0, const XrsProjStep& s1, int mode,
                hipStream_t stream) {
  const int64_t np = (a.g.row_end - a.g.row_begin) * a.g.dst_w;
  const int nb = grid_blocks(np, kThreads, 256 * 16);
  // the same pipeline code as xrs_transform (proj::fast_kind picks it there too)
  int fast = proj::kFastNone;
  if constexpr (K0 == XRS_PROJ_LAEA_INV && K1 == XRS_PROJ_TMERC_FWD)
    fast = xrs_testing_value(XRS_TESTING_PROJ_TWO_STEP) ? proj::kFastNone
                                                        : proj::fast_kind(K0, K1, s0);
  if (fast == proj::kFastObliq)
    launch_proj_mode<K0, K1, proj::kFastObliq>(nb, a, s0, s1, mode, stream);
  else if (fast == proj::kFastEquit)
    launch_proj_mode<K0, K1, proj::kFastEquit>(nb, a, s0, s1, mode, stream);
  else
    launch_proj_mode<K0, K1, proj::kFastNone>(nb, a, s0, s1, mode, stream);
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

// pipelines of crs.Transformer: [inverse], [forward], [inverse, forward]
template <int K0>
int launch_proj_second(int k1, const GatherArgs& a, const XrsProjStep& s0,
                       const XrsProjStep& s1, int mode, hipStream_t st) {
  switch (k1) {
    case 0: return launch_proj<K0, 0>(a, s0, s1, mode, st);
    case XRS_PROJ_WEBMERC_FWD: return launch_proj<K0, XRS_PROJ_WEBMERC_FWD>(a, s0, s1, mode, st);
    case XRS_PROJ_TMERC_FWD: return launch_proj<K0, XRS_PROJ_TMERC_FWD>(a, s0, s1, mode, st);
    case XRS_PROJ_LAEA_FWD: return launch_proj<K0, XRS_PROJ_LAEA_FWD>(a, s0, s1, mode, st);
    default: return XRS_ERR_ARG;
  }
}

}  // namespace
}  // namespace xrs

// K1 needs no scratch since round 5 (each work item resolves its own axis
// entries); the entry point stays so a binding sized by it keeps working.
extern "C" int64_t xrs_reproject_workspace_size(int64_t dst_h, int64_t dst_w, int64_t tile_h,
                                                int64_t tile_w, int coord_mode) {
  (void)dst_h; (void)dst_w; (void)tile_h; (void)tile_w; (void)coord_mode;
  return 0;
}

extern "C" int xrs_reproject(const void* src, int src_dtype, int64_t n, int64_t src_h,
                             int64_t src_w, int64_t src_row0, int64_t src_rows,
                             int64_t src_sn, int64_t src_sy, void* dst, int dst_dtype,
                             int64_t dst_h, int64_t dst_w, int64_t row_begin,
                             int64_t row_end, int64_t dst_sn, int64_t dst_sy,
                             int64_t tile_h, int64_t tile_w, const double* src_x,
                             const double* src_y, int coord_mode, const float* tile_x0,
                             const float* tile_y0, const int64_t* tile_win,
                             int64_t win_h, int64_t win_w, double x_res, double y_res,
                             int interp, double fill, void* workspace,
                             int64_t workspace_bytes, int32_t* err_flags, void* stream) {
  using namespace xrs;
  if (interp != XRS_INTERP_NEAREST && interp != XRS_INTERP_BILINEAR &&
      interp != XRS_INTERP_TRIANGULAR) {
    xrs_set_error("interp must be nearest(0), bilinear(1) or triangular(2), was %d", interp);
    return XRS_ERR_NOTIMPL;
  }
  if (!src || !dst || !src_x || !src_y || !tile_x0 || !tile_y0 || !tile_win || !err_flags ||
      n < 1 || src_h < 1 || src_w < 1 || dst_h < 1 || dst_w < 1 || tile_h < 1 || tile_w < 1 ||
      win_h < 1 || win_w < 1 || row_begin < 0 || row_end > dst_h || row_begin > row_end ||
      src_rows < 0 || src_sy < src_w || src_w > INT32_MAX || src_rows > INT32_MAX ||
      coord_mode < 0 || coord_mode > 2) {
    xrs_set_error("xrs_reproject: invalid argument");
    return XRS_ERR_ARG;
  }
  const int64_t need = xrs_reproject_workspace_size(dst_h, dst_w, tile_h, tile_w, coord_mode);
  if (workspace_bytes < need || (need > 0 && !workspace)) {
    xrs_set_error("xrs_reproject: workspace of %lld bytes required, %lld given",
                  (long long)need, (long long)workspace_bytes);
    return XRS_ERR_ARG;
  }
  if (row_begin == row_end) return XRS_OK;
  // K1b addresses a source row through a buffer resource (byte extent < 2^31)
  const int64_t esz = dispatch_dtype(src_dtype, [](auto tag) -> int { return (int)sizeof(tag); });
  if (esz > 0 && src_w * esz > INT32_MAX) {
    xrs_set_error("xrs_reproject: source rows above 2 GiB are not supported");
    return XRS_ERR_ARG;
  }
  if ((interp == XRS_INTERP_NEAREST || interp == XRS_INTERP_TRIANGULAR) && dst_dtype != src_dtype) {
    xrs_set_error("xrs_reproject: nearest/triangular output dtype must equal the source dtype");
    return XRS_ERR_ARG;
  }
  if (interp == XRS_INTERP_BILINEAR && dst_dtype != XRS_DTYPE_F32 && dst_dtype != XRS_DTYPE_F64) {
    xrs_set_error("xrs_reproject: bilinear output dtype must be float32 or float64");
    return XRS_ERR_ARG;
  }
  GatherArgs a;
  Geometry& g = a.g;
  g.src_h = src_h; g.src_w = src_w; g.src_row0 = src_row0; g.src_rows = src_rows;
  g.dst_h = dst_h; g.dst_w = dst_w; g.row_begin = row_begin; g.row_end = row_end;
  g.tile_h = tile_h; g.tile_w = tile_w;
  g.ntiles_x = (dst_w + tile_w - 1) / tile_w;
  g.ntiles_y = (dst_h + tile_h - 1) / tile_h;
  g.src_x = src_x; g.src_y = src_y; g.tile_x0 = tile_x0; g.tile_y0 = tile_y0;
  g.tile_win = tile_win; g.win_h = win_h; g.win_w = win_w;
  g.x_res = x_res; g.neg_y_res = -y_res; g.err_flags = err_flags; g.band = kBand; g.segw = kSegW; g.band_first = 0;
  g.xgen = coord_mode == 2;
  a.src = src; a.n = n; a.src_sn = src_sn; a.src_sy = src_sy;
  a.dst = dst; a.dst_sn = dst_sn; a.dst_sy = dst_sy; a.fill = fill;
  hipStream_t st = static_cast<hipStream_t>(stream);

  return dispatch_dtype(src_dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    if (interp == XRS_INTERP_NEAREST)
      return launch<T, T, XRS_INTERP_NEAREST>(a, coord_mode, st);
    if (interp == XRS_INTERP_TRIANGULAR)
      return launch<T, T, XRS_INTERP_TRIANGULAR>(a, coord_mode, st);
    if (dst_dtype == XRS_DTYPE_F32)
      return launch<T, float, XRS_INTERP_BILINEAR>(a, coord_mode, st);
    return launch<T, double, XRS_INTERP_BILINEAR>(a, coord_mode, st);
  });
}

extern "C" int xrs_reproject_proj(const void* src, int src_dtype, int64_t n, int64_t src_h,
                                  int64_t src_w, int64_t src_row0, int64_t src_rows,
                                  int64_t src_sn, int64_t src_sy, void* dst, int dst_dtype,
                                  int64_t dst_h, int64_t dst_w, int64_t row_begin,
                                  int64_t row_end, int64_t dst_sn, int64_t dst_sy,
                                  int64_t tile_h, int64_t tile_w, const double* grid_x,
                                  const double* grid_y, const XrsProjStep* steps, int nsteps,
                                  const float* tile_x0, const float* tile_y0,
                                  const int64_t* tile_win, int64_t win_h, int64_t win_w,
                                  double x_res, double y_res, int interp, double fill,
                                  int32_t* err_flags, void* stream) {
  using namespace xrs;
  if (interp != XRS_INTERP_NEAREST && interp != XRS_INTERP_BILINEAR &&
      interp != XRS_INTERP_TRIANGULAR) {
    xrs_set_error("interp must be nearest(0), bilinear(1) or triangular(2), was %d", interp);
    return XRS_ERR_NOTIMPL;
  }
  if (!src || !dst || !grid_x || !grid_y || !tile_x0 || !tile_y0 || !tile_win || !err_flags ||
      n < 1 || src_h < 1 || src_w < 1 || dst_h < 1 || dst_w < 1 || tile_h < 1 || tile_w < 1 ||
      win_h < 1 || win_w < 1 || row_begin < 0 || row_end > dst_h || row_begin > row_end ||
      src_rows < 0 || src_sy < src_w || src_w > INT32_MAX || src_rows > INT32_MAX ||
      nsteps < 0 || nsteps > 2 || (nsteps > 0 && !steps) || dst_h > INT32_MAX ||
      dst_w > INT32_MAX) {
    xrs_set_error("xrs_reproject_proj: invalid argument");
    return XRS_ERR_ARG;
  }
  const int k0 = nsteps > 0 ? steps[0].kind : 0, k1 = nsteps > 1 ? steps[1].kind : 0;
  const bool fwd0 = k0 == XRS_PROJ_WEBMERC_FWD || k0 == XRS_PROJ_TMERC_FWD ||
                    k0 == XRS_PROJ_LAEA_FWD;
  if ((nsteps > 0 && (k0 < XRS_PROJ_WEBMERC_FWD || k0 > XRS_PROJ_LAEA_INV)) ||
      (nsteps > 1 && (fwd0 || !(k1 == XRS_PROJ_WEBMERC_FWD || k1 == XRS_PROJ_TMERC_FWD ||
                                k1 == XRS_PROJ_LAEA_FWD)))) {
    xrs_set_error("xrs_reproject_proj: unsupported projection pipeline");
    return XRS_ERR_ARG;
  }
  if (row_begin == row_end) return XRS_OK;
  int variant;
  if (interp == XRS_INTERP_BILINEAR) {
    if (dst_dtype != XRS_DTYPE_F32 && dst_dtype != XRS_DTYPE_F64) {
      xrs_set_error("xrs_reproject_proj: bilinear output dtype must be float32 or float64");
      return XRS_ERR_ARG;
    }
    variant = dst_dtype == XRS_DTYPE_F32 ? 2 : 3;
  } else {
    if (dst_dtype != src_dtype) {
      xrs_set_error("xrs_reproject_proj: nearest/triangular output dtype must equal the source dtype");
      return XRS_ERR_ARG;
    }
    variant = interp == XRS_INTERP_NEAREST ? 0 : 1;
  }
  if (dispatch_dtype(src_dtype, [](auto) { return XRS_OK; }) != XRS_OK) {
    xrs_set_error("xrs_reproject_proj: unsupported source dtype %d", src_dtype);
    return XRS_ERR_ARG;
  }
  GatherArgs a;
  Geometry& g = a.g;
  g.src_h = src_h; g.src_w = src_w; g.src_row0 = src_row0; g.src_rows = src_rows;
  g.dst_h = dst_h; g.dst_w = dst_w; g.row_begin = row_begin; g.row_end = row_end;
  g.tile_h = tile_h; g.tile_w = tile_w;
  g.ntiles_x = (dst_w + tile_w - 1) / tile_w;
  g.ntiles_y = (dst_h + tile_h - 1) / tile_h;
  g.src_x = grid_x; g.src_y = grid_y; g.tile_x0 = tile_x0; g.tile_y0 = tile_y0;
  g.tile_win = tile_win; g.win_h = win_h; g.win_w = win_w;
  g.x_res = x_res; g.neg_y_res = -y_res; g.err_flags = err_flags; g.band = kBand; g.segw = kSegW; g.band_first = 0;
  g.xgen = 0;
  a.src = src; a.n = n; a.src_sn = src_sn; a.src_sy = src_sy;
  a.dst = dst; a.dst_sn = dst_sn; a.dst_sy = dst_sy; a.fill = fill;
  XrsProjStep s0{}, s1{};
  if (nsteps > 0) s0 = steps[0];
  if (nsteps > 1) s1 = steps[1];
  const int mode = src_dtype * 4 + variant;
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (k0) {
    case 0: return launch_proj<0, 0>(a, s0, s1, mode, st);
    case XRS_PROJ_WEBMERC_FWD: return launch_proj<XRS_PROJ_WEBMERC_FWD, 0>(a, s0, s1, mode, st);
    case XRS_PROJ_TMERC_FWD: return launch_proj<XRS_PROJ_TMERC_FWD, 0>(a, s0, s1, mode, st);
    case XRS_PROJ_LAEA_FWD: return launch_proj<XRS_PROJ_LAEA_FWD, 0>(a, s0, s1, mode, st);
    case XRS_PROJ_WEBMERC_INV:
      return launch_proj_second<XRS_PROJ_WEBMERC_INV>(k1, a, s0, s1, mode, st);
    case XRS_PROJ_TMERC_INV:
      return launch_proj_second<XRS_PROJ_TMERC_INV>(k1, a, s0, s1, mode, st);
    default:
      return launch_proj_second<XRS_PROJ_LAEA_INV>(k1, a, s0, s1, mode, st);
  }
}
