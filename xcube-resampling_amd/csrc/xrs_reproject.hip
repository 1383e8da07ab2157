// xrs_reproject.hip — K1: regular->regular reprojection gather for gfx950.
//
// Replaces, for all target tiles of one variable in ONE call:
//   * reproject._reproject_block            (reproject.py:268-335)  per-tile gather/lerp
//   * reproject._reorganize_data_array_slice (reproject.py:499-530)  pad + window copy
// The per-tile window geometry (reproject._get_scr_bboxes_indices,
// reproject.py:385-469) is computed by the host and passed as small tables.
//
// Separable CRS pairs (coord_mode 0: target x -> source x only, y -> y only,
// e.g. EPSG:3857 -> EPSG:4326) run in two launches:
//   K1a axis_tables   : for every (tile, column) and (tile, row) resolve the
//                       reference's per-pixel index math ONCE — ix = (sx-x0)/res,
//                       floor/ceil/rint, int16 cast, python-style window wrap,
//                       window -> source index, pad -> "outside" — into
//                       {idx_floor, idx_ceil, frac} entries (16 B).  Bit-exact
//                       because for separable transforms the per-pixel ix only
//                       depends on the column (iy on the row).
//   K1b gather_sep    : the HBM-bound part.  One work item = one tile x one
//                       1024-column segment x one band of kBand rows, so the tile
//                       (and every row entry) is block-uniform: row pointers are
//                       scalar, lane offsets 32-bit.  Lanes take consecutive
//                       columns (each wave-load touches ~256 contiguous source
//                       bytes, each store writes 256 contiguous bytes).  The
//                       loads of 4 target rows are issued together (memory-level
//                       parallelism: the loop was latency-bound with one source
//                       row in flight per block); the ceil/floor overlap between
//                       neighbouring rows and columns is served by L1/L2.
// Non-separable pairs (coord_mode 1: 2-D coordinate tables) run K1c, the same
// work decomposition with the index math done per pixel.
//
// Index and weight math is float64 without contraction (-ffp-contract=off) so
// nearest picks and lerp weights are bit-identical to numpy's.

#include <cstdlib>
#include <type_traits>

#include "xrs_common.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;
constexpr int kPx = 4;                       // columns per thread
constexpr int kSegW = kThreads * kPx;        // columns per work item
constexpr int kBand = 32;                    // target rows per work item

struct AxisEntry {   // one resolved column (or row) of one tile
  int32_t f;         // source index of floor(ix) (nearest: of rint(ix)); -1 = outside source
  int32_t c;         // source index of ceil(ix); -1 = outside source
  double d;          // ix - (double)(int16)floor(ix)
};
static_assert(sizeof(AxisEntry) == 16, "AxisEntry layout");

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

// ---- K1a: axis tables ------------------------------------------------------
template <int INTERP>
__global__ void __launch_bounds__(kThreads)
axis_tables_kernel(Geometry g, AxisEntry* __restrict__ xtab, AxisEntry* __restrict__ ytab) {
  const int64_t ntiles = g.ntiles_x * g.ntiles_y;
  const int64_t nx = ntiles * g.tile_w, total = nx + ntiles * g.tile_h;
  int32_t eflags = 0;
  for (int64_t idx = (int64_t)blockIdx.x * kThreads + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * kThreads) {
    if (idx < nx) {
      const int64_t t = idx / g.tile_w, k = idx - t * g.tile_w;
      const int64_t c = (t % g.ntiles_x) * g.tile_w + k;
      const int64_t r0 = (t / g.ntiles_x) * g.tile_h;
      AxisEntry e{-1, -1, 0.0};
      // tiles outside the computed rows [row_begin, row_end) are never read
      if (c < g.dst_w && r0 < g.row_end && r0 + g.tile_h > g.row_begin)
        e = resolve_axis<INTERP>(g.src_x[c], g.tile_x0[t], g.x_res, g.win_w, g.tile_win[2 * t],
                                 g.src_w, 0, g.src_w, eflags);
      xtab[idx] = e;
    } else {
      const int64_t j = idx - nx;
      const int64_t t = j / g.tile_h, k = j - t * g.tile_h;
      const int64_t r = (t / g.ntiles_x) * g.tile_h + k;
      AxisEntry e{-1, -1, 0.0};
      if (r >= g.row_begin && r < g.row_end)
        e = resolve_axis<INTERP>(g.src_y[r], g.tile_y0[t], g.neg_y_res, g.win_h,
                                 g.tile_win[2 * t + 1], g.src_h, g.src_row0, g.src_rows, eflags);
      ytab[j] = e;
    }
  }
  if (eflags) atomicOr(g.err_flags, eflags);
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

struct GatherArgs {
  Geometry g;
  const void* src;
  int64_t n, src_sn, src_sy;
  void* dst;
  int64_t dst_sn, dst_sy;
  double fill;
  const AxisEntry* xtab;
  const AxisEntry* ytab;
};

// Work decomposition shared by K1b/K1c: bands of kBand rows inside one tile row
// x segments of kSegW columns inside one tile column.  Returns false for empty
// items (partial edge tiles, rows outside [row_begin, row_end)).
struct WorkItem {
  int64_t t, ty, tx, r0, r1, c0, c1;
};
__device__ inline bool work_item(const Geometry& g, int64_t w, int64_t ty0, int64_t nsegs,
                                 int64_t bands_per_tile, int64_t segs_per_tile, WorkItem& it) {
  const int64_t b = w / nsegs, s = w - b * nsegs;
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
template <typename T, typename O, int INTERP>
__global__ void __launch_bounds__(kThreads)
gather_separable_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                        int64_t segs_per_tile, int64_t nwork) {
  const Geometry& g = a.g;
  const T fill = Conv<T>::from_f64(a.fill);
  const XcdSlice sl = xcd_slice(nwork);
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;

    // per-lane columns: entries resolved by K1a
    const AxisEntry* xt = a.xtab + it.t * g.tile_w + (it.c0 - it.tx * g.tile_w);
    const int ncols = (int)(it.c1 - it.c0);
    int32_t cf[kPx], cc[kPx];
    double dx[kPx];
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      const int lc = (int)threadIdx.x + k * kThreads;
      AxisEntry e{-1, -1, 0.0};
      if (lc < ncols) e = xt[lc];
      cf[k] = e.f;
      cc[k] = e.c;
      dx[k] = e.d;
    }
    const AxisEntry* yt = a.ytab + it.t * g.tile_h - it.ty * g.tile_h;

    for (int64_t sn = 0; sn < a.n; ++sn) {
      const T* __restrict__ src = static_cast<const T*>(a.src) + sn * a.src_sn;
      O* __restrict__ dst = static_cast<O*>(a.dst) + sn * a.dst_sn - g.row_begin * a.dst_sy + it.c0;
      // source rows carried from one target row to the next
      T vf0[kPx], vf1[kPx], vc0[kPx], vc1[kPx];
      int32_t rowf = INT32_MIN, rowc = INT32_MIN;
#pragma unroll
      for (int k = 0; k < kPx; ++k) vf0[k] = vf1[k] = vc0[k] = vc1[k] = fill;

      for (int64_t r = it.r0; r < it.r1; ++r) {
        const AxisEntry ye = yt[r];  // block-uniform
        T nf0[kPx], nf1[kPx];
        // ---- floor row
        if (ye.f == rowf) {
#pragma unroll
          for (int k = 0; k < kPx; ++k) { nf0[k] = vf0[k]; nf1[k] = vf1[k]; }
        } else if (ye.f == rowc) {
#pragma unroll
          for (int k = 0; k < kPx; ++k) { nf0[k] = vc0[k]; nf1[k] = vc1[k]; }
        } else if (ye.f < 0) {
#pragma unroll
          for (int k = 0; k < kPx; ++k) { nf0[k] = fill; nf1[k] = fill; }
        } else {
          const T* row = src + (int64_t)ye.f * a.src_sy;
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            nf0[k] = cf[k] >= 0 ? row[max(cf[k], 0)] : fill;
            nf1[k] = fill;
            if (INTERP != XRS_INTERP_NEAREST) nf1[k] = cc[k] >= 0 ? row[max(cc[k], 0)] : fill;
          }
        }
        if (INTERP == XRS_INTERP_NEAREST) {
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            const int lc = (int)threadIdx.x + k * kThreads;
            if (lc < ncols) dst[r * a.dst_sy + lc] = (O)nf0[k];
            vf0[k] = nf0[k];
          }
          rowf = ye.f;
          continue;
        }
        // ---- ceil row
        T nc0[kPx], nc1[kPx];
        if (ye.c == ye.f) {
#pragma unroll
          for (int k = 0; k < kPx; ++k) { nc0[k] = nf0[k]; nc1[k] = nf1[k]; }
        } else if (ye.c == rowc) {
#pragma unroll
          for (int k = 0; k < kPx; ++k) { nc0[k] = vc0[k]; nc1[k] = vc1[k]; }
        } else if (ye.c == rowf) {
#pragma unroll
          for (int k = 0; k < kPx; ++k) { nc0[k] = vf0[k]; nc1[k] = vf1[k]; }
        } else if (ye.c < 0) {
#pragma unroll
          for (int k = 0; k < kPx; ++k) { nc0[k] = fill; nc1[k] = fill; }
        } else {
          const T* row = src + (int64_t)ye.c * a.src_sy;
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            nc0[k] = cf[k] >= 0 ? row[max(cf[k], 0)] : fill;
            nc1[k] = cc[k] >= 0 ? row[max(cc[k], 0)] : fill;
          }
        }
#pragma unroll
        for (int k = 0; k < kPx; ++k) {
          const int lc = (int)threadIdx.x + k * kThreads;
          const double v = interp4<T, INTERP>(nf0[k], nf1[k], nc0[k], nc1[k], dx[k], ye.d);
          if (lc < ncols) dst[r * a.dst_sy + lc] = Conv<O>::from_f64(v);
          vf0[k] = nf0[k]; vf1[k] = nf1[k]; vc0[k] = nc0[k]; vc1[k] = nc1[k];
        }
        rowf = ye.f;
        rowc = ye.c;
      }
    }
  }
}

// ---- K1b': separable gather, loads of kRowsB target rows issued up front ----
// No carried rows: every target row loads its two source rows (the ceil/floor
// overlap of neighbouring rows is served by L1/L2), but the loads of kRowsB
// rows are independent and in flight together (memory-level parallelism).
template <typename T, typename O, int INTERP, int kRowsB, bool NT = false, int PX = kPx,
          int DBG = 0>
__global__ void __launch_bounds__(kThreads)
gather_separable_mlp_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                            int64_t segs_per_tile, int64_t nwork) {
  const Geometry& g = a.g;
  const T fill = Conv<T>::from_f64(a.fill);
  const XcdSlice sl = xcd_slice(nwork);
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const AxisEntry* xt = a.xtab + it.t * g.tile_w + (it.c0 - it.tx * g.tile_w);
    const int ncols = (int)(it.c1 - it.c0);
    int32_t cf[PX], cc[PX];
    double dx[PX];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int lc = (int)threadIdx.x + k * kThreads;
      AxisEntry e{-1, -1, 0.0};
      if (lc < ncols) e = xt[lc];
      cf[k] = e.f;
      cc[k] = e.c;
      dx[k] = e.d;
    }
    const AxisEntry* yt = a.ytab + it.t * g.tile_h - it.ty * g.tile_h;
    for (int64_t sn = 0; sn < a.n; ++sn) {
      const T* __restrict__ src = static_cast<const T*>(a.src) + sn * a.src_sn;
      O* __restrict__ dst = static_cast<O*>(a.dst) + sn * a.dst_sn - g.row_begin * a.dst_sy + it.c0;
      for (int64_t r = it.r0; r < it.r1; r += kRowsB) {
        AxisEntry ye[kRowsB];
        T v[kRowsB][4][PX];
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          ye[q] = (r + q < it.r1) ? yt[r + q] : AxisEntry{-1, -1, 0.0};
          const T* rf = src + (int64_t)max(ye[q].f, 0) * a.src_sy;
          const T* rc = src + (int64_t)max(ye[q].c, 0) * a.src_sy;
#pragma unroll
          for (int k = 0; k < PX; ++k) {
            const int32_t f = max(cf[k], 0), c = max(cc[k], 0);
            v[q][0][k] = rf[f];
            if (INTERP != XRS_INTERP_NEAREST) {
              if (DBG != 2) v[q][1][k] = rf[c];
              if (DBG != 3 && DBG != 4 && DBG != 5) v[q][2][k] = rc[f];
              if (DBG != 2 && DBG != 3 && DBG != 4 && DBG != 5) v[q][3][k] = rc[c];
              if (DBG == 3) { v[q][2][k] = v[q][0][k]; v[q][3][k] = v[q][1][k]; }
            }
          }
        }
        // DBG 5: a ceil row that is the next target row's floor row is not
        // fetched again: the taps come from that row's registers (uniform
        // test; the loads of the other ceil rows sit in uniform branches)
        bool share[kRowsB];
#pragma unroll
        for (int q = 0; q < kRowsB; ++q)
          share[q] = DBG == 5 && q + 1 < kRowsB && ye[q].c == ye[q + 1].f;
        if (DBG == 5 && INTERP != XRS_INTERP_NEAREST) {
#pragma unroll
          for (int q = 0; q < kRowsB; ++q) {
            if (share[q]) continue;
            const T* rc = src + (int64_t)max(ye[q].c, 0) * a.src_sy;
#pragma unroll
            for (int k = 0; k < PX; ++k) {
              v[q][2][k] = rc[max(cf[k], 0)];
              v[q][3][k] = rc[max(cc[k], 0)];
            }
          }
        }
        if (DBG == 4 && INTERP != XRS_INTERP_NEAREST) {
          // two phases: the ceil rows are requested only once the floor rows
          // have landed, so a ceil row that is the next target row's floor row
          // hits L1 instead of sending a second request to L2 for the same
          // lines (in flight together, the two requests do not merge).  The
          // opaque zero makes the ceil addresses depend on the last floor load.
          int32_t z;
          asm volatile("v_and_b32 %0, 0, %1" : "=v"(z)
                       : "v"(__float_as_int((float)v[kRowsB - 1][1][PX - 1])));
#pragma unroll
          for (int q = 0; q < kRowsB; ++q) {
            const T* rc = src + (int64_t)max(ye[q].c, 0) * a.src_sy + z;
#pragma unroll
            for (int k = 0; k < PX; ++k) {
              v[q][2][k] = rc[max(cf[k], 0)];
              v[q][3][k] = rc[max(cc[k], 0)];
            }
          }
        }
        if (DBG == 2) {   // timing probe: ceil taps from the next lane (wrong values)
#pragma unroll
          for (int q = 0; q < kRowsB; ++q)
#pragma unroll
            for (int k = 0; k < PX; ++k) {
              v[q][1][k] = __shfl_down(v[q][0][k], 1);
              v[q][3][k] = __shfl_down(v[q][2][k], 1);
            }
        }
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          if (r + q >= it.r1) break;
          const bool okf = ye[q].f >= 0, okc = ye[q].c >= 0;
#pragma unroll
          for (int k = 0; k < PX; ++k) {
            const int lc = (int)threadIdx.x + k * kThreads;
            const bool xf = cf[k] >= 0, xc = cc[k] >= 0;
            const T v00 = (okf && xf) ? v[q][0][k] : fill;
            O out;
            if (INTERP == XRS_INTERP_NEAREST) {
              out = (O)v00;
            } else {
              const T v01 = (okf && xc) ? v[q][1][k] : fill;
              const T c0 = share[q] ? v[q + 1 < kRowsB ? q + 1 : q][0][k] : v[q][2][k];
              const T c1 = share[q] ? v[q + 1 < kRowsB ? q + 1 : q][1][k] : v[q][3][k];
              const T v10 = (okc && xf) ? c0 : fill;
              const T v11 = (okc && xc) ? c1 : fill;
              if (DBG == 1) out = (O)(v00 + v01 + v10 + v11);
              else out = Conv<O>::from_f64(interp4<T, INTERP>(v00, v01, v10, v11, dx[k], ye[q].d));
            }
            if (lc < ncols) {
              if (NT) __builtin_nontemporal_store(out, &dst[(r + q) * a.dst_sy + lc]);
              else dst[(r + q) * a.dst_sy + lc] = out;
            }
          }
        }
      }
    }
  }
}

// ---- K1b'': bilinear with source-row reuse --------------------------------
// reproject.py:315-328 computes per target pixel u0 = lerp(row floor),
// u1 = lerp(row ceil), out = u0 + dy*(u1 - u0).  The horizontal lerp of a
// source row only depends on (row, column), so when consecutive target rows
// share a source row (ceil of row r == floor of row r+1, or the same floor)
// the value is reused bit for bit instead of recomputed — one third fewer
// float64 operations; the decisions are block-uniform (row entries are).
// COND_LOADS additionally skips the loads of reused rows.
template <typename T, typename O, int kRowsB, bool NT, bool COND_LOADS, int PX = kPx>
__global__ void __launch_bounds__(kThreads)
gather_bilinear_reuse_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                             int64_t segs_per_tile, int64_t nwork) {
  const Geometry& g = a.g;
  const T fill = Conv<T>::from_f64(a.fill);
  const XcdSlice sl = xcd_slice(nwork);
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const AxisEntry* xt = a.xtab + it.t * g.tile_w + (it.c0 - it.tx * g.tile_w);
    const int ncols = (int)(it.c1 - it.c0);
    int32_t cf[PX], cc[PX];
    double dx[PX];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int lc = (int)threadIdx.x + k * kThreads;
      AxisEntry e{-1, -1, 0.0};
      if (lc < ncols) e = xt[lc];
      cf[k] = e.f;
      cc[k] = e.c;
      dx[k] = e.d;
    }
    const AxisEntry* yt = a.ytab + it.t * g.tile_h - it.ty * g.tile_h;
    for (int64_t sn = 0; sn < a.n; ++sn) {
      const T* __restrict__ src = static_cast<const T*>(a.src) + sn * a.src_sn;
      O* __restrict__ dst = static_cast<O*>(a.dst) + sn * a.dst_sn - g.row_begin * a.dst_sy + it.c0;
      // carried: source rows of the previous target row and their lerps
      int32_t pf = INT32_MIN, pc = INT32_MIN;
      double ptop[PX], pbot[PX];
#pragma unroll
      for (int k = 0; k < PX; ++k) ptop[k] = pbot[k] = 0.0;
      for (int64_t r = it.r0; r < it.r1; r += kRowsB) {
        AxisEntry ye[kRowsB];
        bool need_f[kRowsB], need_c[kRowsB];
        T v[kRowsB][4][PX];
        {
          int32_t qf = pf, qc = pc;
#pragma unroll
          for (int q = 0; q < kRowsB; ++q) {
            ye[q] = (r + q < it.r1) ? yt[r + q] : AxisEntry{-1, -1, 0.0};
            // which rows' lerps can be taken from the previous target row
            need_f[q] = !(ye[q].f == qf || ye[q].f == qc);
            need_c[q] = !(ye[q].c == ye[q].f || ye[q].c == qc);
            qf = ye[q].f;
            qc = ye[q].c;
          }
        }
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          const T* rf = src + (int64_t)max(ye[q].f, 0) * a.src_sy;
          const T* rc = src + (int64_t)max(ye[q].c, 0) * a.src_sy;
          if (!COND_LOADS || need_f[q]) {
#pragma unroll
            for (int k = 0; k < PX; ++k) {
              v[q][0][k] = rf[max(cf[k], 0)];
              v[q][1][k] = rf[max(cc[k], 0)];
            }
          }
          if (!COND_LOADS || need_c[q]) {
#pragma unroll
            for (int k = 0; k < PX; ++k) {
              v[q][2][k] = rc[max(cf[k], 0)];
              v[q][3][k] = rc[max(cc[k], 0)];
            }
          }
        }
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          if (r + q >= it.r1) break;
          const bool okf = ye[q].f >= 0, okc = ye[q].c >= 0;
          double top[PX], bot[PX];
#pragma unroll
          for (int k = 0; k < PX; ++k) {
            const bool xf = cf[k] >= 0, xc = cc[k] >= 0;
            if (need_f[q]) {
              const T v00 = (okf && xf) ? v[q][0][k] : fill;
              const T v01 = (okf && xc) ? v[q][1][k] : fill;
              top[k] = Conv<T>::to_f64(v00) + dx[k] * Conv<T>::to_f64(Conv<T>::diff(v01, v00));
            } else {
              top[k] = ye[q].f == pf ? ptop[k] : pbot[k];
            }
            if (ye[q].c == ye[q].f) {
              bot[k] = top[k];
            } else if (need_c[q]) {
              const T v10 = (okc && xf) ? v[q][2][k] : fill;
              const T v11 = (okc && xc) ? v[q][3][k] : fill;
              bot[k] = Conv<T>::to_f64(v10) + dx[k] * Conv<T>::to_f64(Conv<T>::diff(v11, v10));
            } else {
              bot[k] = pbot[k];
            }
            const O out = Conv<O>::from_f64(top[k] + ye[q].d * (bot[k] - top[k]));
            const int lc = (int)threadIdx.x + k * kThreads;
            if (lc < ncols) {
              if (NT) __builtin_nontemporal_store(out, &dst[(r + q) * a.dst_sy + lc]);
              else dst[(r + q) * a.dst_sy + lc] = out;
            }
            ptop[k] = top[k];
            pbot[k] = bot[k];
          }
          pf = ye[q].f;
          pc = ye[q].c;
        }
      }
    }
  }
}

// ---- K1b-run (variant 23): 4 consecutive columns per lane, 8-element runs ----
// At x scales near 1 (config 5: 0.994) pixel k of a lane's 4 consecutive
// target columns has its floor column at cf[0] + k + {-1, 0, +1} and its ceil
// column at floor + 1, so ONE run of 8 source elements starting at cf[0] - 1
// holds every horizontal tap of the lane's 4 pixels: per source row two
// 16-byte loads instead of 8 scalar gathers, per target row one 16-byte store
// instead of 4.  Lanes whose columns do not fit (window / source edges,
// exact-integer positions, other scales, a partial last lane) gather tap by
// tap; the run loads stay unconditional (column 0 for such lanes) so no
// branch separates the loads of a batch.
template <typename T, typename O, int INTERP, int kRowsB>
__global__ void __launch_bounds__(kThreads)
gather_run_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                  int64_t segs_per_tile, int64_t nwork, int vec_store) {
  constexpr int RW = 8;
  const Geometry& g = a.g;
  const T fill = Conv<T>::from_f64(a.fill);
  const XcdSlice sl = xcd_slice(nwork);
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const AxisEntry* xt = a.xtab + it.t * g.tile_w + (it.c0 - it.tx * g.tile_w);
    const int ncols = (int)(it.c1 - it.c0);
    const int lc0 = 4 * (int)threadIdx.x;
    int32_t cf[4], cc[4], sel[4];
    double dx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      AxisEntry e{-1, -1, 0.0};
      if (lc0 + k < ncols) e = xt[lc0 + k];
      cf[k] = e.f;
      cc[k] = e.c;
      dx[k] = e.d;
    }
    const int32_t ws = cf[0] - 1;
    bool run = lc0 + 3 < ncols && ws >= 0 && (int64_t)ws + RW <= g.src_w;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sel[k] = cf[k] - ws - k;   // run index of pixel k's floor tap, minus k: 0, 1 or 2
      run = run && cf[k] >= 0 && cc[k] == cf[k] + 1 && sel[k] >= 0 && sel[k] <= 2;
    }
    const int32_t wsr = run ? ws : 0;
    const bool vst = vec_store && lc0 + 3 < ncols;
    const AxisEntry* yt = a.ytab + it.t * g.tile_h - it.ty * g.tile_h;
    for (int64_t sn = 0; sn < a.n; ++sn) {
      const T* __restrict__ src = static_cast<const T*>(a.src) + sn * a.src_sn;
      O* __restrict__ dst =
          static_cast<O*>(a.dst) + sn * a.dst_sn - g.row_begin * a.dst_sy + it.c0 + lc0;
      for (int64_t r = it.r0; r < it.r1; r += kRowsB) {
        AxisEntry ye[kRowsB];
        T wf[kRowsB][RW], wc[kRowsB][RW];
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          ye[q] = (r + q < it.r1) ? yt[r + q] : AxisEntry{-1, -1, 0.0};
          const T* rf = src + (int64_t)max(ye[q].f, 0) * a.src_sy + wsr;
          const T* rc = src + (int64_t)max(ye[q].c, 0) * a.src_sy + wsr;
#pragma unroll
          for (int e = 0; e < RW; ++e) {
            wf[q][e] = rf[e];
            wc[q][e] = rc[e];
          }
        }
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          if (r + q >= it.r1) break;
          const bool okf = ye[q].f >= 0, okc = ye[q].c >= 0;
          O out[4];
          if (run) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int s = sel[k];
              const T a0 = s == 0 ? wf[q][k] : (s == 1 ? wf[q][k + 1] : wf[q][k + 2]);
              const T a1 = s == 0 ? wf[q][k + 1] : (s == 1 ? wf[q][k + 2] : wf[q][k + 3]);
              const T b0 = s == 0 ? wc[q][k] : (s == 1 ? wc[q][k + 1] : wc[q][k + 2]);
              const T b1 = s == 0 ? wc[q][k + 1] : (s == 1 ? wc[q][k + 2] : wc[q][k + 3]);
              out[k] = Conv<O>::from_f64(interp4<T, INTERP>(okf ? a0 : fill, okf ? a1 : fill,
                                                            okc ? b0 : fill, okc ? b1 : fill,
                                                            dx[k], ye[q].d));
            }
          } else {   // tap by tap (edges)
            const T* rf = src + (int64_t)max(ye[q].f, 0) * a.src_sy;
            const T* rc = src + (int64_t)max(ye[q].c, 0) * a.src_sy;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const bool xf = cf[k] >= 0, xc = cc[k] >= 0;
              const int32_t f = max(cf[k], 0), c = max(cc[k], 0);
              const T v00 = (okf && xf) ? rf[f] : fill;
              const T v01 = (okf && xc) ? rf[c] : fill;
              const T v10 = (okc && xf) ? rc[f] : fill;
              const T v11 = (okc && xc) ? rc[c] : fill;
              out[k] = Conv<O>::from_f64(interp4<T, INTERP>(v00, v01, v10, v11, dx[k], ye[q].d));
            }
          }
          O* drow = dst + (r + q) * a.dst_sy;
          if (vst) {
            typedef O O2 __attribute__((ext_vector_type(2)));
            if (sizeof(O) == 4) {
              typedef O O4 __attribute__((ext_vector_type(4)));
              const O4 o4 = {out[0], out[1], out[2], out[3]};
              __builtin_nontemporal_store(o4, reinterpret_cast<O4*>(drow));
            } else {
              const O2 lo = {out[0], out[1]}, hi = {out[2], out[3]};
              __builtin_nontemporal_store(lo, reinterpret_cast<O2*>(drow));
              __builtin_nontemporal_store(hi, reinterpret_cast<O2*>(drow) + 1);
            }
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (lc0 + k < ncols) __builtin_nontemporal_store(out[k], drow + k);
          }
        }
      }
    }
  }
}

// ---- K1b-T (variant 24): variant-12 gathers, LDS-transposed 16-byte stores ----
// Each wave owns 256 consecutive target columns; lane L gathers columns
// L + 64k (k < 4: every tap load of the wave is 256 contiguous-ish bytes, as
// in variant 12), then the wave transposes its row through a wave-private LDS
// row (4 conflict-free dword writes, one ds_read_b128) so that lane L stores
// columns 4L .. 4L+3 with ONE 16-byte non-temporal store instead of four
// 4-byte ones.
template <typename T, typename O, int INTERP, int kRowsB>
__global__ void __launch_bounds__(kThreads)
gather_transpose_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                        int64_t segs_per_tile, int64_t nwork, int vec_store) {
  __shared__ __align__(16) O lds[kThreads / 64][kRowsB][256];
  const Geometry& g = a.g;
  const T fill = Conv<T>::from_f64(a.fill);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const XcdSlice sl = xcd_slice(nwork);
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const int64_t wc0 = it.c0 + 256 * wv;   // this wave's first target column
    const int ncols = (int)max((int64_t)0, min((int64_t)256, it.c1 - wc0));
    if (ncols == 0) continue;
    const AxisEntry* xt = a.xtab + it.t * g.tile_w + (wc0 - it.tx * g.tile_w);
    int32_t cf[4], cc[4];
    double dx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int lc = lane + 64 * k;
      AxisEntry e{-1, -1, 0.0};
      if (lc < ncols) e = xt[lc];
      cf[k] = e.f;
      cc[k] = e.c;
      dx[k] = e.d;
    }
    const bool vst = vec_store && 4 * lane + 3 < ncols;
    const AxisEntry* yt = a.ytab + it.t * g.tile_h - it.ty * g.tile_h;
    for (int64_t sn = 0; sn < a.n; ++sn) {
      const T* __restrict__ src = static_cast<const T*>(a.src) + sn * a.src_sn;
      O* __restrict__ dst = static_cast<O*>(a.dst) + sn * a.dst_sn - g.row_begin * a.dst_sy + wc0;
      for (int64_t r = it.r0; r < it.r1; r += kRowsB) {
        AxisEntry ye[kRowsB];
        T v[kRowsB][4][4];
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          ye[q] = (r + q < it.r1) ? yt[r + q] : AxisEntry{-1, -1, 0.0};
          const T* rf = src + (int64_t)max(ye[q].f, 0) * a.src_sy;
          const T* rc = src + (int64_t)max(ye[q].c, 0) * a.src_sy;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int32_t f = max(cf[k], 0), c = max(cc[k], 0);
            v[q][0][k] = rf[f];
            if (INTERP != XRS_INTERP_NEAREST) {
              v[q][1][k] = rf[c];
              v[q][2][k] = rc[f];
              v[q][3][k] = rc[c];
            }
          }
        }
        // the previous batch's LDS reads are done before this batch's writes
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          const bool okf = ye[q].f >= 0, okc = ye[q].c >= 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const bool xf = cf[k] >= 0, xc = cc[k] >= 0;
            const T v00 = (okf && xf) ? v[q][0][k] : fill;
            O out;
            if (INTERP == XRS_INTERP_NEAREST) {
              out = (O)v00;
            } else {
              const T v01 = (okf && xc) ? v[q][1][k] : fill;
              const T v10 = (okc && xf) ? v[q][2][k] : fill;
              const T v11 = (okc && xc) ? v[q][3][k] : fill;
              out = Conv<O>::from_f64(interp4<T, INTERP>(v00, v01, v10, v11, dx[k], ye[q].d));
            }
            lds[wv][q][lane + 64 * k] = out;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
        for (int q = 0; q < kRowsB; ++q) {
          if (r + q >= it.r1) break;
          O* drow = dst + (r + q) * a.dst_sy;
          if (vst) {
            typedef O O2 __attribute__((ext_vector_type(2)));
            if (sizeof(O) == 4) {
              typedef O O4 __attribute__((ext_vector_type(4)));
              const O4 o4 = *reinterpret_cast<const O4*>(&lds[wv][q][4 * lane]);
              __builtin_nontemporal_store(o4, reinterpret_cast<O4*>(drow + 4 * lane));
            } else {
              const O2 lo = *reinterpret_cast<const O2*>(&lds[wv][q][4 * lane]);
              const O2 hi = *reinterpret_cast<const O2*>(&lds[wv][q][4 * lane + 2]);
              __builtin_nontemporal_store(lo, reinterpret_cast<O2*>(drow + 4 * lane));
              __builtin_nontemporal_store(hi, reinterpret_cast<O2*>(drow + 4 * lane) + 1);
            }
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (4 * lane + k < ncols)
                __builtin_nontemporal_store(lds[wv][q][4 * lane + k], drow + 4 * lane + k);
          }
        }
      }
    }
  }
}

// ---- K1c: per-pixel gather (2-D coordinate tables) --------------------------
template <typename T, typename O, int INTERP>
__global__ void __launch_bounds__(kThreads)
gather_2d_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                 int64_t segs_per_tile, int64_t nwork) {
  const Geometry& g = a.g;
  const T fill = Conv<T>::from_f64(a.fill);
  const XcdSlice sl = xcd_slice(nwork);
  int32_t eflags = 0;
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const int ncols = (int)(it.c1 - it.c0);
    const float x0 = g.tile_x0[it.t], y0 = g.tile_y0[it.t];
    const int64_t wi0 = g.tile_win[2 * it.t], wj0 = g.tile_win[2 * it.t + 1];
    for (int64_t r = it.r0; r < it.r1; ++r) {
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const int lc = (int)threadIdx.x + k * kThreads;
        if (lc >= ncols) continue;
        const int64_t p = r * g.dst_w + it.c0 + lc;
        const AxisEntry ex = resolve_axis<INTERP>(g.src_x[p], x0, g.x_res, g.win_w, wi0, g.src_w,
                                                  0, g.src_w, eflags);
        const AxisEntry ey = resolve_axis<INTERP>(g.src_y[p], y0, g.neg_y_res, g.win_h, wj0,
                                                  g.src_h, g.src_row0, g.src_rows, eflags);
        for (int64_t sn = 0; sn < a.n; ++sn) {
          const T* src = static_cast<const T*>(a.src) + sn * a.src_sn;
          O* dst = static_cast<O*>(a.dst) + sn * a.dst_sn + (r - g.row_begin) * a.dst_sy;
          auto at = [&](int32_t row, int32_t col) -> T {
            return (row >= 0 && col >= 0) ? src[(int64_t)row * a.src_sy + col] : fill;
          };
          if (INTERP == XRS_INTERP_NEAREST) {
            dst[it.c0 + lc] = (O)at(ey.f, ex.f);
          } else {
            const double v = interp4<T, INTERP>(at(ey.f, ex.f), at(ey.f, ex.c), at(ey.c, ex.f),
                                                at(ey.c, ex.c), ex.d, ey.d);
            dst[it.c0 + lc] = Conv<O>::from_f64(v);
          }
        }
      }
    }
  }
  if (eflags) atomicOr(g.err_flags, eflags);
}

// ---- K1s: LDS-staged separable gather ------------------------------------
// The source footprint of a work item (rows [rmin, rmax] x columns [cmin,
// cmax] of every valid tap) is read ONCE with 16-byte loads per lane — the
// access shape of a streaming copy, ≈ 2 KB contiguous per row — and parked in
// LDS; the per-pixel taps (irregular, 4 per bilinear pixel) are then gathered
// from LDS instead of as 4-byte global loads.  Spans come from the entries
// already in registers (wave shuffles + one LDS exchange).  Items whose span
// does not fit (window wrap-around, extreme scales) take the direct path.
template <typename T>
__device__ inline int32_t wave_min(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ inline int32_t wave_max_i(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

template <typename T, typename O, int INTERP, bool VEC, int PX = 2>
__global__ void __launch_bounds__(kThreads)
gather_staged_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                     int64_t segs_per_tile, int64_t nwork, int lds_cap) {
  extern __shared__ __align__(16) unsigned char smem[];
  T* stage = reinterpret_cast<T*>(smem);
  __shared__ int32_t part[4][4];
  __shared__ AxisEntry rows_s[64];   // the band's row entries (band <= 64)
  constexpr int E = VEC ? 16 / (int)sizeof(T) : 1;   // elements per staging load
  const Geometry& g = a.g;
  const T fill = Conv<T>::from_f64(a.fill);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = threadIdx.x % 64;
  const XcdSlice sl = xcd_slice(nwork);
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const AxisEntry* xt = a.xtab + it.t * g.tile_w + (it.c0 - it.tx * g.tile_w);
    const int ncols = (int)(it.c1 - it.c0);
    int32_t cf[PX], cc[PX];
    double dx[PX];
    int32_t lo = INT32_MAX, hi = -1;
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int lc = (int)threadIdx.x + k * kThreads;
      AxisEntry e{-1, -1, 0.0};
      if (lc < ncols) e = xt[lc];
      cf[k] = e.f;
      cc[k] = e.c;
      dx[k] = e.d;
      if (e.f >= 0) { lo = min(lo, e.f); hi = max(hi, e.f); }
      if (INTERP != XRS_INTERP_NEAREST && e.c >= 0) { lo = min(lo, e.c); hi = max(hi, e.c); }
    }
    const AxisEntry* yt = a.ytab + it.t * g.tile_h - it.ty * g.tile_h;
    const int nrows = (int)(it.r1 - it.r0);
    int32_t rlo = INT32_MAX, rhi = -1;
    for (int q = lane; q < nrows; q += 64) {   // rows: every wave, same answer
      const AxisEntry e = yt[it.r0 + q];
      if (wave == 0) rows_s[q] = e;
      if (e.f >= 0) { rlo = min(rlo, e.f); rhi = max(rhi, e.f); }
      if (INTERP != XRS_INTERP_NEAREST && e.c >= 0) { rlo = min(rlo, e.c); rhi = max(rhi, e.c); }
    }
    lo = wave_min<T>(lo);
    hi = wave_max_i(hi);
    if (lane == 0) { part[wave][0] = lo; part[wave][1] = hi; }
    __syncthreads();   // also: the previous item's gathers from `stage` are done
    lo = min(min(part[0][0], part[1][0]), min(part[2][0], part[3][0]));
    hi = max(max(part[0][1], part[1][1]), max(part[2][1], part[3][1]));
    rlo = wave_min<T>(rlo);
    rhi = wave_max_i(rhi);
    const int cs = lo - lo % E;                             // 16-byte aligned start
    const int ce = hi < 0 ? cs : ((hi + 1 + E - 1) / E) * E;   // exclusive, aligned
    const int pitch = max(ce - cs, 0);
    const int nr = rhi - rlo + 1;
    const bool staged = hi >= 0 && rhi >= 0 && (int64_t)nr * pitch * (int64_t)sizeof(T) <= lds_cap;
    __syncthreads();   // everyone has read `part` before the next item rewrites it
    if (staged) {
      // wave-uniform (row, pass) schedule: 8 loads per lane in flight, then stores
      const int nvec = pitch / E;
      const int passes = (nvec + 63) / 64;
      const int rows_w = (nr - wave + 3) / 4;            // rows of this wave
      const int nitems = rows_w * passes;
      for (int i0 = 0; i0 < nitems; i0 += 8) {
        using V = typename std::conditional<VEC, uint4, T>::type;
        V tmp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u;
          const int r = wave + 4 * (i / passes), vi = (i % passes) * 64 + lane;
          if (i < nitems && vi < nvec) {
            const T* gp = static_cast<const T*>(a.src) + (int64_t)(rlo + r) * a.src_sy + cs + vi * E;
            tmp[u] = *reinterpret_cast<const V*>(gp);
          }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u;
          const int r = wave + 4 * (i / passes), vi = (i % passes) * 64 + lane;
          if (i < nitems && vi < nvec)
            *reinterpret_cast<V*>(stage + r * pitch + vi * E) = tmp[u];
        }
      }
      __syncthreads();
    }
    // (a.n > 1 re-stages per slice below; the bench and configs use n = 1)
    for (int64_t sn = 0; sn < a.n; ++sn) {
      const T* __restrict__ src = static_cast<const T*>(a.src) + sn * a.src_sn;
      O* __restrict__ dst = static_cast<O*>(a.dst) + sn * a.dst_sn - g.row_begin * a.dst_sy + it.c0;
      if (sn > 0 && staged) {
        __syncthreads();
        const int nvec = pitch / E;
        for (int e = threadIdx.x; e < nr * nvec; e += kThreads) {
          const int r = e / nvec, vi = e - r * nvec;
          using V = typename std::conditional<VEC, uint4, T>::type;
          *reinterpret_cast<V*>(stage + r * pitch + vi * E) =
              *reinterpret_cast<const V*>(src + (int64_t)(rlo + r) * a.src_sy + cs + vi * E);
        }
        __syncthreads();
      }
      for (int64_t r = it.r0; r < it.r1; ++r) {
        const AxisEntry ye = rows_s[r - it.r0];   // LDS broadcast, no global round trip
        const bool okf = ye.f >= 0, okc = ye.c >= 0;
        T v[4][PX];
        if (staged) {
          const T* lf = stage + (okf ? ye.f - rlo : 0) * pitch - cs;
          const T* lcr = stage + (okc ? ye.c - rlo : 0) * pitch - cs;
#pragma unroll
          for (int k = 0; k < PX; ++k) {
            const int32_t f = cf[k] >= 0 ? cf[k] : cs, c = cc[k] >= 0 ? cc[k] : cs;
            v[0][k] = lf[f];
            if (INTERP != XRS_INTERP_NEAREST) { v[1][k] = lf[c]; v[2][k] = lcr[f]; v[3][k] = lcr[c]; }
          }
        } else {
          const T* rf = src + (int64_t)max(ye.f, 0) * a.src_sy;
          const T* rc = src + (int64_t)max(ye.c, 0) * a.src_sy;
#pragma unroll
          for (int k = 0; k < PX; ++k) {
            const int32_t f = max(cf[k], 0), c = max(cc[k], 0);
            v[0][k] = rf[f];
            if (INTERP != XRS_INTERP_NEAREST) { v[1][k] = rf[c]; v[2][k] = rc[f]; v[3][k] = rc[c]; }
          }
        }
#pragma unroll
        for (int k = 0; k < PX; ++k) {
          const int lc = (int)threadIdx.x + k * kThreads;
          const bool xf = cf[k] >= 0, xc = cc[k] >= 0;
          const T v00 = (okf && xf) ? v[0][k] : fill;
          O out;
          if (INTERP == XRS_INTERP_NEAREST) {
            out = (O)v00;
          } else {
            const T v01 = (okf && xc) ? v[1][k] : fill;
            const T v10 = (okc && xf) ? v[2][k] : fill;
            const T v11 = (okc && xc) ? v[3][k] : fill;
            out = Conv<O>::from_f64(interp4<T, INTERP>(v00, v01, v10, v11, dx[k], ye.d));
          }
          if (lc < ncols) __builtin_nontemporal_store(out, &dst[r * a.dst_sy + lc]);
        }
      }
    }
  }
}

// ---- K1w: wave-staged separable gather -------------------------------------
// bilinear from 4-byte gathers issues 4 vector-memory instructions per target
// pixel and is bound by that issue rate (PMC: WAIT_INST dominates; nearest,
// 1 tap, streams at 6.4 TB/s).  Here each wave owns 256 consecutive target
// columns (4 per lane) of a band of rows.  The source rows the band needs are
// staged ONCE per wave into a private LDS ring with aligned 16-byte loads —
// one vector-memory instruction moves 256 source elements — in bursts of the
// rows needed by G target rows (all loads of a burst in flight together);
// the taps are then LDS reads and each lane writes its 4 pixels with one
// vector store.  No block-level synchronisation: the ring is wave-private.
// Falls back to 4-byte global taps (same arithmetic) for a burst whose rows
// are not increasing or do not fit the ring, and for a wave whose column
// span exceeds the stage width.
constexpr int kWsW = 320;     // staged elements per source row and wave
constexpr int kWsR = 8;       // ring rows per wave
constexpr int kWsG = 4;       // target rows per staging burst

template <typename T, typename O, int INTERP, bool VEC_ST>
__global__ void __launch_bounds__(kThreads)
gather_wave_staged_kernel(GatherArgs a, int64_t ty0, int64_t nsegs, int64_t bands_per_tile,
                          int64_t segs_per_tile, int64_t nwork) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr int E = 16 / (int)sizeof(T);       // elements per 16-byte load
  constexpr int NV = kWsW / E;                 // 16-byte vectors per staged row
  const Geometry& g = a.g;
  const T fill = Conv<T>::from_f64(a.fill);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  T* ring = reinterpret_cast<T*>(smem) + wv * (kWsR * kWsW);
  const XcdSlice sl = xcd_slice(nwork);
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    WorkItem it;
    if (!work_item(g, w, ty0, nsegs, bands_per_tile, segs_per_tile, it)) continue;
    const int64_t wc0 = it.c0 + 256 * wv;          // this wave's first target column
    if (wc0 >= it.c1) continue;
    const int ncols = (int)min((int64_t)256, it.c1 - wc0);
    const AxisEntry* xt = a.xtab + it.t * g.tile_w + (wc0 - it.tx * g.tile_w);
    int32_t cf[4], cc[4];
    double dx[4];
    int32_t lo = INT32_MAX, hi = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int lc = 4 * lane + k;
      AxisEntry e{-1, -1, 0.0};
      if (lc < ncols) e = xt[lc];
      cf[k] = e.f; cc[k] = e.c; dx[k] = e.d;
      if (e.f >= 0) { lo = min(lo, e.f); hi = max(hi, e.f); }
      if (INTERP != XRS_INTERP_NEAREST && e.c >= 0) { lo = min(lo, e.c); hi = max(hi, e.c); }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o, 64));
      hi = max(hi, __shfl_xor(hi, o, 64));
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    const int32_t base = hi >= 0 ? lo - lo % E : 0;
    const bool cols_fit = hi < 0 || hi - base < kWsW;
    const int nvec = hi >= 0 ? (hi - base) / E + 1 : 0;
    int32_t of[4], oc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      of[k] = cf[k] >= 0 ? cf[k] - base : 0;
      oc[k] = cc[k] >= 0 ? cc[k] - base : 0;
    }
    const AxisEntry* yt = a.ytab + it.t * g.tile_h - it.ty * g.tile_h;
    for (int64_t sn = 0; sn < a.n; ++sn) {
      const T* __restrict__ src = static_cast<const T*>(a.src) + sn * a.src_sn;
      O* __restrict__ dst = static_cast<O*>(a.dst) + sn * a.dst_sn - g.row_begin * a.dst_sy + wc0;
      // ring contents: every source row in [ring_lo, staged_hi] (at most the
      // last kWsR of them) is staged; rows are only ever appended upwards.
      // Software pipeline: the loads of burst b+1's new rows are issued before
      // burst b is computed and land in LDS after it.
      typedef unsigned int V __attribute__((ext_vector_type(4)));   // SROA-friendly
      constexpr int NJ = (NV + 63) / 64;
      int32_t staged_hi = INT32_MIN, ring_lo = 0;
      AxisEntry ye[kWsG];
      int nr = 0;
      int32_t rlo = INT32_MAX, rhi = -1;
      auto burst = [&](int64_t rb, AxisEntry (&e)[kWsG], int& n, int32_t& l, int32_t& h) {
        n = (int)min((int64_t)kWsG, it.r1 - rb);
        l = INT32_MAX; h = -1;
#pragma unroll
        for (int q = 0; q < kWsG; ++q) {
          e[q] = q < n ? yt[rb + q] : AxisEntry{-1, -1, 0.0};
          const int32_t f = e[q].f, c = INTERP != XRS_INTERP_NEAREST ? e[q].c : e[q].f;
          if (f >= 0) { l = min(l, f); h = max(h, f); }
          if (c >= 0) { l = min(l, c); h = max(h, c); }
        }
      };
      // can rows [l, h] be served by the ring after appending (staged_hi, h]?
      auto plan = [&](int32_t l, int32_t h, bool& cont) -> bool {
        cont = staged_hi != INT32_MIN && l <= staged_hi + 1 &&
               l >= max(ring_lo, staged_hi - (kWsR - 1));
        return cols_fit && h >= 0 && h - l < kWsR && (cont || staged_hi == INT32_MIN || l > staged_hi);
      };
      auto load_rows = [&](int32_t s0, int nnew, V (&buf)[kWsR][NJ]) {
#pragma unroll
        for (int i = 0; i < kWsR; ++i) {
          if (i < nnew) {
            const T* row = src + (int64_t)(s0 + i) * a.src_sy + base;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              const int v = lane + 64 * j;
              if (v < nvec) buf[i][j] = *reinterpret_cast<const V*>(row + v * E);
            }
          }
        }
      };
      auto store_rows = [&](int32_t s0, int nnew, const V (&buf)[kWsR][NJ]) {
#pragma unroll
        for (int i = 0; i < kWsR; ++i) {
          if (i < nnew) {
            T* lrow = ring + ((s0 + i) % kWsR) * kWsW;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              const int v = lane + 64 * j;
              if (v < nvec) *reinterpret_cast<V*>(lrow + v * E) = buf[i][j];
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      };
      V buf[kWsR][NJ];
      burst(it.r0, ye, nr, rlo, rhi);
      bool use_ring;
      {
        bool cont;
        use_ring = plan(rlo, rhi, cont);
        if (use_ring) {
          const int32_t s0 = cont ? staged_hi + 1 : rlo;
          load_rows(s0, rhi - s0 + 1, buf);
          store_rows(s0, rhi - s0 + 1, buf);
          ring_lo = rlo; staged_hi = rhi;
        }
      }
      for (int64_t r = it.r0; r < it.r1; r += kWsG) {
        // next burst: entries, plan, loads in flight
        AxisEntry yn[kWsG];
        int nrn = 0;
        int32_t rlon = INT32_MAX, rhin = -1;
        const bool has_next = r + kWsG < it.r1;
        bool next_ring = false, next_cont = false;
        int32_t ns0 = 0;
        int nnew = 0;
        if (has_next) {
          burst(r + kWsG, yn, nrn, rlon, rhin);
          next_ring = plan(rlon, rhin, next_cont);
          if (next_ring) {
            ns0 = next_cont ? staged_hi + 1 : rlon;
            nnew = rhin - ns0 + 1;
            load_rows(ns0, nnew, buf);
          }
        }
#pragma unroll
        for (int q = 0; q < kWsG; ++q) {
          if (q >= nr) break;
          const bool okf = ye[q].f >= 0, okc = ye[q].c >= 0;
          T v[4][4];
          if (use_ring) {
            const T* lf = ring + ((okf ? ye[q].f : 0) % kWsR) * kWsW;
            const T* lc = ring + ((okc ? ye[q].c : 0) % kWsR) * kWsW;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              v[0][k] = lf[of[k]];
              if (INTERP != XRS_INTERP_NEAREST) { v[1][k] = lf[oc[k]]; v[2][k] = lc[of[k]]; v[3][k] = lc[oc[k]]; }
            }
          } else {
            const T* rf = src + (int64_t)max(ye[q].f, 0) * a.src_sy;
            const T* rc = src + (int64_t)max(ye[q].c, 0) * a.src_sy;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int32_t f = max(cf[k], 0), c = max(cc[k], 0);
              v[0][k] = rf[f];
              if (INTERP != XRS_INTERP_NEAREST) { v[1][k] = rf[c]; v[2][k] = rc[f]; v[3][k] = rc[c]; }
            }
          }
          O out[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const bool xf = cf[k] >= 0, xc = cc[k] >= 0;
            const T v00 = (okf && xf) ? v[0][k] : fill;
            if (INTERP == XRS_INTERP_NEAREST) {
              out[k] = (O)v00;
            } else {
              const T v01 = (okf && xc) ? v[1][k] : fill;
              const T v10 = (okc && xf) ? v[2][k] : fill;
              const T v11 = (okc && xc) ? v[3][k] : fill;
              out[k] = Conv<O>::from_f64(interp4<T, INTERP>(v00, v01, v10, v11, dx[k], ye[q].d));
            }
          }
          O* drow = dst + (r + q) * a.dst_sy + 4 * lane;
          if (VEC_ST && 4 * lane + 3 < ncols) {
            typedef O O4 __attribute__((ext_vector_type(4)));
            O4 o4 = {out[0], out[1], out[2], out[3]};
            __builtin_nontemporal_store(o4, reinterpret_cast<O4*>(drow));
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (4 * lane + k < ncols) __builtin_nontemporal_store(out[k], drow + k);
          }
        }
        if (has_next) {
          if (next_ring) {
            store_rows(ns0, nnew, buf);
            if (!next_cont) ring_lo = rlon;
            if (nnew > 0) staged_hi = rhin;
          }
#pragma unroll
          for (int q = 0; q < kWsG; ++q) ye[q] = yn[q];
          nr = nrn;
          use_ring = next_ring;
        }
      }
    }
  }
}

// Separable gather variant (XRS_REPROJECT_VARIANT, for A/B measurements; all
// variants are bit-identical, only the load schedule differs):
//   0      rows carried in registers (fewest loads, one source row in flight)
//   1/3/2  loads of 2/3/4 target rows issued together
//   5/4/8  the same for 2/4/8 rows with non-temporal (streaming) output stores
//   6/7    bilinear with source-row lerp reuse (7: also skips reused loads)
//   9/10/11  as 4 with 2/8/1 columns per thread (512/2048/256-column items)
//   12/13  8/16 rows in flight, 2 columns per thread, non-temporal stores
//   14     LDS-staged footprint (16-byte staging loads, taps gathered from LDS)
// Default 12.  Interleaved A/B on one MI355X, 40960^2 bilinear, one work item
// per block: 12 = 2.51 ms, 9 = 2.57, 4 = 2.76, 11 = 2.96, 13 = 3.69
// (scripts/ab_reproject.py; absolute times vary ~10 % between boxes).
// 14 (unpipelined: entries -> stage -> gather are dependent round trips per
// item, 40 KB of LDS caps residency at 3 blocks/CU) = 7.9-11 ms for bands of
// 6-16 rows vs 2.73 ms for 12 in the same run: kept for reference, a
// double-buffered stage is the way to make it pay.
// Also measured and dropped: the two horizontal taps as one dword-aligned
// 8-byte load (global_load_dwordx2 at odd addresses): 4.08 ms vs 2.69 ms.
// Reference point on the same box: nearest (1 tap) 2.08 ms = 6.4 TB/s, a
// torch copy_ of the raster 2.8 ms — bilinear is tap-issue bound, not HBM
// (PMC: SQ_WAIT_INST_ANY > SQ_WAIT_ANY; dropping the f64 lerps, keeping the 4
// taps, changes nothing: 2.63 vs 2.68 ms).
//   20     wave-staged: 256 columns per wave, source rows staged once into a
//          wave-private LDS ring by 16-byte loads, software-pipelined bursts
//          of 4 target rows, one 16-byte store per lane and row: 3.48 ms
//          (12: 2.56 ms) — the LDS round trip and 168 VGPRs cost more than the
//          saved gathers; lane-strided pixels with dword stores: 3.85 ms.
//   23     4 consecutive columns per lane, taps from one 8-element run per
//          source row (two 16-byte loads) and 16-byte stores: 2.97 ms vs 2.66
//          (8192^2: 0.145 vs 0.110 ms) — fewer, wider memory instructions do
//          not pay: K1 is not VMEM-issue bound
//   24     variant-12 gathers (4 rows x 4 columns per lane) with the output
//          row transposed through LDS into 16-byte stores: 2.88 vs 2.66 ms
//          (8192^2: 0.125 vs 0.110) — the dword stores are not the limit either
//   90/91  timing probes (wrong values): 90 drops the float64 lerps (2.49 vs
//          2.65 ms), 91 takes the two ceil-column taps from the next lane by
//          shuffle instead of loading them (2.67 ms: no gain).  Nearest in the
//          same run: 2.33 ms.  So bilinear costs the nearest gather (~copy rate)
//          plus ~0.16 ms of float64 lerp (required for bit-exact parity) plus
//          ~0.16 ms for the second source row — not tap-issue bound.
//   92     probe: the ceil row's taps not loaded (floor row reused): 2.21-2.37
//          vs 2.45-2.65 ms — the second row fetch (the same lines requested
//          again while the first request is in flight) is the cost.  Fixes
//          tried, all bit-identical and slower: 25 (ceil rows requested after
//          the floor rows landed, so they hit L1): 4.20 ms; each source row of
//          a batch loaded once into register vectors and picked by a
//          wave-uniform index (GPR indexing mode, 10/13-row windows): 5.1 ms;
//          28 (a ceil row equal to the next target row's floor row taken from
//          that row's registers, the other ceil rows loaded in uniform
//          branches): 2.63 vs 2.51 ms — the branches and the partial waits they
//          bring cost more than the saved fetches.
inline int variant() {
  const char* v = getenv("XRS_REPROJECT_VARIANT");
  return v ? atoi(v) : 12;
}

template <typename T, typename O, int INTERP>
int launch(const GatherArgs& a, int coord_mode, AxisEntry* xtab, AxisEntry* ytab,
           hipStream_t stream) {
  const Geometry& g = a.g;
  const int64_t ty0 = g.row_begin / g.tile_h, ty1 = (g.row_end - 1) / g.tile_h + 1;
  const char* band_env = getenv("XRS_REPROJECT_BAND");  // A/B knob (target rows per item)
  GatherArgs args = a;
  args.g.band = band_env && atoi(band_env) > 0 ? atoi(band_env) : (variant() == 14 ? 8 : kBand);
  if (variant() == 14 && args.g.band > 64) args.g.band = 64;   // rows_s capacity
  const int64_t bands_per_tile = (g.tile_h + args.g.band - 1) / args.g.band;
  const int v = variant();
  args.g.segw = kThreads * (v == 9 || v == 12 || v == 13 || v == 14 || v == 90 || v == 91 || v == 92 || v == 25 || v == 28 || v == 21 || v == 22 ? 2 : v == 10 ? 8 : (v == 20 || v == 23 || v == 24) ? 4 : v == 11 ? 1 : kPx);
  const int64_t segs_per_tile = (g.tile_w + args.g.segw - 1) / args.g.segw;
  const int64_t nsegs = g.ntiles_x * segs_per_tile;
  const int64_t nwork = (ty1 - ty0) * bands_per_tile * nsegs;
  // One work item per block (measured fastest: short blocks let the dispatcher
  // balance the CUs and keep each XCD's concurrent row set L2-sized; a
  // persistent grid of 8 blocks/CU was 12 % slower).  A/B knob: blocks per CU.
  const char* bpc_env = getenv("XRS_REPROJECT_BLOCKS_PER_CU");
  const int bpc = bpc_env ? atoi(bpc_env) : 0;
  const int nb = grid_blocks(nwork, 1, bpc > 0 ? 256 * bpc : (1 << 24));
  if (coord_mode == 0) {
    const int64_t ntab = g.ntiles_x * g.ntiles_y * (g.tile_w + g.tile_h);
    const int nbt = grid_blocks(ntab, kThreads, 256 * 8);
    hipLaunchKernelGGL((axis_tables_kernel<INTERP>), dim3(nbt), dim3(kThreads), 0, stream, g,
                       xtab, ytab);
    XRS_HIP_CHECK(hipGetLastError());
    args.xtab = xtab;
    args.ytab = ytab;
    if (v == 1)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 2>), dim3(nb), dim3(kThreads),
                         0, stream, args, ty0, nsegs, bands_per_tile, segs_per_tile, nwork);
    else if (v == 2)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 4>), dim3(nb), dim3(kThreads),
                         0, stream, args, ty0, nsegs, bands_per_tile, segs_per_tile, nwork);
    else if (v == 3)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 3>), dim3(nb), dim3(kThreads),
                         0, stream, args, ty0, nsegs, bands_per_tile, segs_per_tile, nwork);
    else if (v == 4)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 4, true>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 5)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 2, true>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 8)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 8, true>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 9)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 4, true, 2>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 10)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 4, true, 8>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 11)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 4, true, 1>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 12)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 8, true, 2>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 13)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 16, true, 2>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 20) {
      // wave-staged: 16-byte staging loads need 16-byte aligned source rows
      const int esz = (int)sizeof(T);
      const bool aligned = (16 % esz == 0) && ((uintptr_t)a.src % 16 == 0) &&
                           ((a.src_sy * esz) % 16 == 0) && ((a.src_sn * esz) % 16 == 0);
      const bool vst = ((uintptr_t)a.dst % (4 * sizeof(O)) == 0) && (a.dst_sy % 4 == 0) &&
                       (a.dst_sn % 4 == 0) && (g.tile_w % 4 == 0);
      const size_t lds = (size_t)4 * kWsR * kWsW * sizeof(T);
      if (!aligned)
        hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 8, true, 2>), dim3(nb),
                           dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                           segs_per_tile, nwork);
      else if (vst)
        hipLaunchKernelGGL((gather_wave_staged_kernel<T, O, INTERP, true>), dim3(nb),
                           dim3(kThreads), lds, stream, args, ty0, nsegs, bands_per_tile,
                           segs_per_tile, nwork);
      else
        hipLaunchKernelGGL((gather_wave_staged_kernel<T, O, INTERP, false>), dim3(nb),
                           dim3(kThreads), lds, stream, args, ty0, nsegs, bands_per_tile,
                           segs_per_tile, nwork);
    } else if (v == 28)   // ceil rows shared with the next target row's floor row
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 8, true, 2, 5>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 25)   // two-phase row loads (floor rows, then ceil rows)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 8, true, 2, 4>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 92)   // timing probe only: the ceil row's taps not loaded (floor row reused)
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 8, true, 2, 3>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 91)   // timing probe only: 2 of the 4 taps by cross-lane shuffle
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 8, true, 2, 2>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 90)   // timing probe only: bilinear loads, f32 sum instead of the f64 lerps
      hipLaunchKernelGGL((gather_separable_mlp_kernel<T, O, INTERP, 8, true, 2, 1>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 14) {
      // LDS stage: 16-byte staging loads when every row start is 16-byte aligned
      const int esz = (int)sizeof(T);
      const bool vec = (16 % esz == 0) && ((uintptr_t)a.src % 16 == 0) &&
                       ((a.src_sy * esz) % 16 == 0) && ((a.src_sn * esz) % 16 == 0) &&
                       ((g.src_w * esz) % 16 == 0);
      const char* cap_env = getenv("XRS_REPROJECT_LDS");
      const int cap = cap_env ? atoi(cap_env) : 40 * 1024;
      if (vec)
        hipLaunchKernelGGL((gather_staged_kernel<T, O, INTERP, true>), dim3(nb), dim3(kThreads),
                           (size_t)cap, stream, args, ty0, nsegs, bands_per_tile, segs_per_tile,
                           nwork, cap);
      else
        hipLaunchKernelGGL((gather_staged_kernel<T, O, INTERP, false>), dim3(nb), dim3(kThreads),
                           (size_t)cap, stream, args, ty0, nsegs, bands_per_tile, segs_per_tile,
                           nwork, cap);
    } else if (v == 6 && INTERP == XRS_INTERP_BILINEAR)
      hipLaunchKernelGGL((gather_bilinear_reuse_kernel<T, O, 4, true, false>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if ((v == 23 || v == 24) && std::is_same<T, float>::value) {
      // 16-byte output stores need 4-element aligned output runs
      const bool vst = ((uintptr_t)a.dst % (4 * sizeof(O)) == 0 || sizeof(O) == 8) &&
                       ((uintptr_t)a.dst % 16 == 0) && (a.dst_sy % 4 == 0) &&
                       (a.dst_sn % 4 == 0) && (g.tile_w % 4 == 0);
      if constexpr (std::is_same<T, float>::value) {
        if (v == 23 && INTERP != XRS_INTERP_NEAREST)
          hipLaunchKernelGGL((gather_run_kernel<T, O, INTERP, 4>), dim3(nb), dim3(kThreads), 0,
                             stream, args, ty0, nsegs, bands_per_tile, segs_per_tile, nwork,
                             (int)vst);
        else
          hipLaunchKernelGGL((gather_transpose_kernel<T, O, INTERP, 4>), dim3(nb),
                             dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                             segs_per_tile, nwork, (int)vst);
      }
    } else if (v == 21 && INTERP == XRS_INTERP_BILINEAR)
      hipLaunchKernelGGL((gather_bilinear_reuse_kernel<T, O, 8, true, true, 2>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 22 && INTERP == XRS_INTERP_BILINEAR)
      hipLaunchKernelGGL((gather_bilinear_reuse_kernel<T, O, 4, true, true, 2>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else if (v == 7 && INTERP == XRS_INTERP_BILINEAR)
      hipLaunchKernelGGL((gather_bilinear_reuse_kernel<T, O, 4, true, true>), dim3(nb),
                         dim3(kThreads), 0, stream, args, ty0, nsegs, bands_per_tile,
                         segs_per_tile, nwork);
    else
      hipLaunchKernelGGL((gather_separable_kernel<T, O, INTERP>), dim3(nb), dim3(kThreads), 0,
                         stream, args, ty0, nsegs, bands_per_tile, segs_per_tile, nwork);
  } else {
    hipLaunchKernelGGL((gather_2d_kernel<T, O, INTERP>), dim3(nb), dim3(kThreads), 0, stream,
                       args, ty0, nsegs, bands_per_tile, segs_per_tile, nwork);
  }
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

}  // namespace
}  // namespace xrs

extern "C" int64_t xrs_reproject_workspace_size(int64_t dst_h, int64_t dst_w, int64_t tile_h,
                                                int64_t tile_w, int coord_mode) {
  if (coord_mode != 0 || dst_h < 1 || dst_w < 1 || tile_h < 1 || tile_w < 1) return 0;
  const int64_t ntiles = ((dst_h + tile_h - 1) / tile_h) * ((dst_w + tile_w - 1) / tile_w);
  return ntiles * (tile_w + tile_h) * (int64_t)sizeof(xrs::AxisEntry);
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
      (coord_mode != 0 && coord_mode != 1)) {
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
  g.x_res = x_res; g.neg_y_res = -y_res; g.err_flags = err_flags; g.band = kBand; g.segw = kSegW;
  a.src = src; a.n = n; a.src_sn = src_sn; a.src_sy = src_sy;
  a.dst = dst; a.dst_sn = dst_sn; a.dst_sy = dst_sy; a.fill = fill;
  a.xtab = a.ytab = nullptr;
  AxisEntry* xtab = static_cast<AxisEntry*>(workspace);
  AxisEntry* ytab = xtab ? xtab + g.ntiles_x * g.ntiles_y * tile_w : nullptr;
  hipStream_t st = static_cast<hipStream_t>(stream);

  return dispatch_dtype(src_dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    if (interp == XRS_INTERP_NEAREST)
      return launch<T, T, XRS_INTERP_NEAREST>(a, coord_mode, xtab, ytab, st);
    if (interp == XRS_INTERP_TRIANGULAR)
      return launch<T, T, XRS_INTERP_TRIANGULAR>(a, coord_mode, xtab, ytab, st);
    if (dst_dtype == XRS_DTYPE_F32)
      return launch<T, float, XRS_INTERP_BILINEAR>(a, coord_mode, xtab, ytab, st);
    return launch<T, double, XRS_INTERP_BILINEAR>(a, coord_mode, xtab, ytab, st);
  });
}
