// xrs_reproject.hip — K1: regular->regular reprojection gather for gfx950.
//
// Replaces, for all target tiles of one variable in ONE launch:
//   * reproject._reproject_block            (reproject.py:268-335)  per-tile gather/lerp
//   * reproject._reorganize_data_array_slice (reproject.py:499-530)  pad + window copy
// The per-tile window geometry (reproject._get_scr_bboxes_indices,
// reproject.py:385-469) is computed by the host and passed as tables.
//
// Memory-bound gather: one thread = 4 consecutive target pixels of one row;
// one workgroup = 1024 pixels of one row; each XCD walks a contiguous band of
// rows so the source rows it pulls into its 4 MiB L2 serve the next target rows
// (scale ~1 => every source row is read by ~2 target rows).  Output stores are
// 16-byte vectors where aligned.  Index math is float64 without contraction
// (library built with -ffp-contract=off) so nearest-neighbour picks and lerp
// weights are bit-identical to numpy's.

#include "xrs_common.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;
constexpr int kPx = 4;                      // pixels per thread (one row)
constexpr int kBlockPx = kThreads * kPx;    // pixels per work item

struct ReprojectArgs {
  const void* src;
  int64_t n, src_h, src_w, src_row0, src_rows, src_sn, src_sy;
  void* dst;
  int64_t dst_h, dst_w, row_begin, row_end, dst_sn, dst_sy;
  int64_t tile_h, tile_w, ntiles_x;
  const double* src_x;
  const double* src_y;
  const float* tile_x0;
  const float* tile_y0;
  const int64_t* tile_win;
  int64_t win_h, win_w;
  double x_res, neg_y_res;
  double fill;
  int32_t* err_flags;
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

// A tap offset < 0 means "outside the source" -> the da.pad constant fill.
template <typename T>
__device__ inline T fetch(const T* __restrict__ src, int64_t off, int64_t slice_off, T fill) {
  return off >= 0 ? src[slice_off + off] : fill;
}

template <typename O>
__device__ inline void store_px(O* __restrict__ row, int64_t c0, int nvalid, const O (&v)[kPx]) {
#pragma unroll
  for (int k = 0; k < kPx; ++k)
    if (k < nvalid) row[c0 + k] = v[k];
}
template <>
__device__ inline void store_px<float>(float* __restrict__ row, int64_t c0, int nvalid,
                                       const float (&v)[kPx]) {
  float* p = row + c0;
  if (nvalid == kPx && (((uintptr_t)p) & 15) == 0) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int k = 0; k < kPx; ++k)
      if (k < nvalid) p[k] = v[k];
  }
}
template <>
__device__ inline void store_px<double>(double* __restrict__ row, int64_t c0, int nvalid,
                                        const double (&v)[kPx]) {
  double* p = row + c0;
  if (nvalid == kPx && (((uintptr_t)p) & 15) == 0) {
    reinterpret_cast<double2*>(p)[0] = make_double2(v[0], v[1]);
    reinterpret_cast<double2*>(p)[1] = make_double2(v[2], v[3]);
  } else {
#pragma unroll
    for (int k = 0; k < kPx; ++k)
      if (k < nvalid) p[k] = v[k];
  }
}

// Resolve window indices (wy, wx) of tile t to a source offset within a slice.
__device__ inline int64_t resolve(const ReprojectArgs& a, int64_t j0, int64_t i0,
                                  int64_t wy, int64_t wx, int32_t& eflags) {
  const int64_t gj = j0 + wy, gi = i0 + wx;
  if (gj < 0 || gj >= a.src_h || gi < 0 || gi >= a.src_w) return -1;  // pad region
  const int64_t lj = gj - a.src_row0;
  if (lj < 0 || lj >= a.src_rows) {  // host plan did not give this device the band
    eflags |= XRS_EFLAG_BAND;
    return -1;
  }
  return lj * a.src_sy + gi;
}

template <typename T, typename O, int INTERP, int COORD>
__global__ void __launch_bounds__(kThreads)
reproject_kernel(ReprojectArgs a) {
  const T* __restrict__ src = static_cast<const T*>(a.src);
  O* __restrict__ dst = static_cast<O*>(a.dst);
  const T fill = Conv<T>::from_f64(a.fill);
  const int64_t nrows = a.row_end - a.row_begin;
  const int64_t nbcol = (a.dst_w + kBlockPx - 1) / kBlockPx;
  const XcdSlice s = xcd_slice(nrows * nbcol);
  int32_t eflags = 0;

  for (int64_t w = s.first; w < s.end; w += s.step) {
    const int64_t lr = w / nbcol;            // local target row
    const int64_t r = a.row_begin + lr;      // global target row
    const int64_t c0 = (w - lr * nbcol) * kBlockPx + (int64_t)threadIdx.x * kPx;
    if (c0 >= a.dst_w) continue;
    const int nvalid = (int)min((int64_t)kPx, a.dst_w - c0);
    const int64_t ty = r / a.tile_h;

    // ---- per-pixel geometry (independent of the slice index n) ----------
    int64_t off[kPx][4];
    double dx[kPx], dy[kPx];
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      off[k][0] = off[k][1] = off[k][2] = off[k][3] = -1;
      dx[k] = dy[k] = 0.0;
      if (k >= nvalid) continue;
      const int64_t c = c0 + k;
      const int64_t t = ty * a.ntiles_x + c / a.tile_w;
      double sx, sy;
      if (COORD == 0) {
        sx = a.src_x[c];
        sy = a.src_y[r];
      } else {
        sx = a.src_x[r * a.dst_w + c];
        sy = a.src_y[r * a.dst_w + c];
      }
      const double ix = (sx - (double)a.tile_x0[t]) / a.x_res;      // reproject.py:278
      const double iy = (sy - (double)a.tile_y0[t]) / a.neg_y_res;  // reproject.py:279
      const int64_t wi0 = a.tile_win[2 * t], wj0 = a.tile_win[2 * t + 1];
      if (INTERP == XRS_INTERP_NEAREST) {                            // reproject.py:281-284
        int64_t wx, wy;
        const bool okx = window_index(f64_to_i16_np(rint(ix)), a.win_w, wx);
        const bool oky = window_index(f64_to_i16_np(rint(iy)), a.win_h, wy);
        if (okx && oky) off[k][0] = resolve(a, wj0, wi0, wy, wx, eflags);
        else eflags |= XRS_EFLAG_INDEX;
      } else {                                                       // reproject.py:286-289,316-321
        const int16_t ixc = f64_to_i16_np(ceil(ix)), ixf = f64_to_i16_np(floor(ix));
        const int16_t iyc = f64_to_i16_np(ceil(iy)), iyf = f64_to_i16_np(floor(iy));
        dx[k] = ix - (double)ixf;
        dy[k] = iy - (double)iyf;
        int64_t wxf, wxc, wyf, wyc;
        // all four resolved (no short-circuit): each IndexError is flagged
        const int ok = (int)window_index(ixf, a.win_w, wxf) & (int)window_index(ixc, a.win_w, wxc) &
                       (int)window_index(iyf, a.win_h, wyf) & (int)window_index(iyc, a.win_h, wyc);
        if (ok) {
          off[k][0] = resolve(a, wj0, wi0, wyf, wxf, eflags);  // value_00
          off[k][1] = resolve(a, wj0, wi0, wyf, wxc, eflags);  // value_01
          off[k][2] = resolve(a, wj0, wi0, wyc, wxf, eflags);  // value_10
          off[k][3] = resolve(a, wj0, wi0, wyc, wxc, eflags);  // value_11
        } else {
          eflags |= XRS_EFLAG_INDEX;
        }
      }
    }

    // ---- gather + interpolate every slice of dim 0 ----------------------
    for (int64_t sn = 0; sn < a.n; ++sn) {
      const int64_t so = sn * a.src_sn;
      O out[kPx];
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        if (INTERP == XRS_INTERP_NEAREST) {
          out[k] = (O)fetch(src, off[k][0], so, fill);
        } else {
          const T v00 = fetch(src, off[k][0], so, fill);
          const T v01 = fetch(src, off[k][1], so, fill);
          const T v10 = fetch(src, off[k][2], so, fill);
          const T v11 = fetch(src, off[k][3], so, fill);
          double res;
          if (INTERP == XRS_INTERP_BILINEAR) {               // reproject.py:326-328
            const double u0 = Conv<T>::to_f64(v00) + dx[k] * Conv<T>::to_f64(Conv<T>::diff(v01, v00));
            const double u1 = Conv<T>::to_f64(v10) + dx[k] * Conv<T>::to_f64(Conv<T>::diff(v11, v10));
            res = u0 + dy[k] * (u1 - u0);
          } else if (dx[k] + dy[k] < 1.0) {                   // reproject.py:296,304-308
            res = Conv<T>::to_f64(v00) + dx[k] * Conv<T>::to_f64(Conv<T>::diff(v01, v00)) +
                  dy[k] * Conv<T>::to_f64(Conv<T>::diff(v10, v00));
          } else {                                            // reproject.py:310-314
            res = Conv<T>::to_f64(v11) + (1.0 - dx[k]) * Conv<T>::to_f64(Conv<T>::diff(v10, v11)) +
                  (1.0 - dy[k]) * Conv<T>::to_f64(Conv<T>::diff(v01, v11));
          }
          out[k] = Conv<O>::from_f64(res);
        }
      }
      store_px<O>(dst + sn * a.dst_sn + lr * a.dst_sy, c0, nvalid, out);
    }
  }
  if (eflags) atomicOr(a.err_flags, eflags);
}

template <typename T, typename O, int INTERP>
int launch_coord(const ReprojectArgs& a, int coord_mode, hipStream_t stream) {
  const int64_t nwork = (a.row_end - a.row_begin) * ((a.dst_w + kBlockPx - 1) / kBlockPx);
  const int nb = grid_blocks(nwork, 1, 256 * 16);
  if (coord_mode == 0)
    hipLaunchKernelGGL((reproject_kernel<T, O, INTERP, 0>), dim3(nb), dim3(kThreads), 0, stream, a);
  else
    hipLaunchKernelGGL((reproject_kernel<T, O, INTERP, 1>), dim3(nb), dim3(kThreads), 0, stream, a);
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

}  // namespace
}  // namespace xrs

extern "C" int xrs_reproject(const void* src, int src_dtype, int64_t n, int64_t src_h,
                             int64_t src_w, int64_t src_row0, int64_t src_rows,
                             int64_t src_sn, int64_t src_sy, void* dst, int dst_dtype,
                             int64_t dst_h, int64_t dst_w, int64_t row_begin,
                             int64_t row_end, int64_t dst_sn, int64_t dst_sy,
                             int64_t tile_h, int64_t tile_w, const double* src_x,
                             const double* src_y, int coord_mode, const float* tile_x0,
                             const float* tile_y0, const int64_t* tile_win,
                             int64_t win_h, int64_t win_w, double x_res, double y_res,
                             int interp, double fill, int32_t* err_flags, void* stream) {
  using namespace xrs;
  if (interp != XRS_INTERP_NEAREST && interp != XRS_INTERP_BILINEAR &&
      interp != XRS_INTERP_TRIANGULAR) {
    xrs_set_error("interp must be nearest(0), bilinear(1) or triangular(2), was %d", interp);
    return XRS_ERR_NOTIMPL;
  }
  if (!src || !dst || !src_x || !src_y || !tile_x0 || !tile_y0 || !tile_win || !err_flags ||
      n < 1 || src_h < 1 || src_w < 1 || dst_h < 1 || dst_w < 1 || tile_h < 1 || tile_w < 1 ||
      win_h < 1 || win_w < 1 || row_begin < 0 || row_end > dst_h || row_begin > row_end ||
      src_rows < 0 || src_sy < src_w || (coord_mode != 0 && coord_mode != 1)) {
    xrs_set_error("xrs_reproject: invalid argument");
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
  ReprojectArgs a;
  a.src = src; a.n = n; a.src_h = src_h; a.src_w = src_w; a.src_row0 = src_row0;
  a.src_rows = src_rows; a.src_sn = src_sn; a.src_sy = src_sy;
  a.dst = dst; a.dst_h = dst_h; a.dst_w = dst_w; a.row_begin = row_begin; a.row_end = row_end;
  a.dst_sn = dst_sn; a.dst_sy = dst_sy; a.tile_h = tile_h; a.tile_w = tile_w;
  a.ntiles_x = (dst_w + tile_w - 1) / tile_w;
  a.src_x = src_x; a.src_y = src_y; a.tile_x0 = tile_x0; a.tile_y0 = tile_y0;
  a.tile_win = tile_win; a.win_h = win_h; a.win_w = win_w;
  a.x_res = x_res; a.neg_y_res = -y_res; a.fill = fill; a.err_flags = err_flags;
  hipStream_t st = static_cast<hipStream_t>(stream);

  return dispatch_dtype(src_dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    if (interp == XRS_INTERP_NEAREST) return launch_coord<T, T, XRS_INTERP_NEAREST>(a, coord_mode, st);
    if (interp == XRS_INTERP_TRIANGULAR) return launch_coord<T, T, XRS_INTERP_TRIANGULAR>(a, coord_mode, st);
    if (dst_dtype == XRS_DTYPE_F32) return launch_coord<T, float, XRS_INTERP_BILINEAR>(a, coord_mode, st);
    return launch_coord<T, double, XRS_INTERP_BILINEAR>(a, coord_mode, st);
  });
}
