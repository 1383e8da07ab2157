// xrs_transform.hip — coordinate transformation pipelines on the device (gfx950).
//
// Replaces the per-pixel pyproj calls of the reference for the CRS pairs that
// are not separable (x' depends on x AND y):
//   * reproject.py:472-496 (_transform_gridpoints): every target pixel centre
//     of a tile -> source CRS, before _reproject_block;
//   * rectify.py:182-231 (_transform_coords): every source coordinate ->
//     target CRS.
// A pipeline is one or two steps (source -> geographic -> target, crs.py
// Transformer), each a template parameter of the kernel; the steps are the
// PROJ restatements of xrs_proj.hpp (a few ulps from the numpy restatement,
// tests/test_transform_gpu.py).
//
// Launch: one thread per point, grid-stride; compute bound (f64 VALU and the
// transcendental sequences), 16 B in (image mode) and 16 B out per point.

#include <cmath>

#include "xrs_common.hpp"
#include "xrs_proj.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;

// grid mode: point (r, c) = (x[c], y[r]) (a regular grid's pixel centres,
// np.meshgrid order); image mode: point p = (x[p], y[p]).  Out row-major.
// Pipeline = step K0 then step K1 (0: none), proj::Pipeline.
template <int K0, int K1, bool GRID, int FAST>
__global__ void __launch_bounds__(kThreads)
transform_kernel(const double* __restrict__ x, const double* __restrict__ y, int64_t w,
                 int64_t h, XrsProjStep s0, XrsProjStep s1, double* __restrict__ out_x,
                 double* __restrict__ out_y) {
  const proj::Pipeline<K0, K1, FAST> pipe(s0, s1);
  const int64_t n = w * h;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * kThreads) {
    double px, py;
    if (GRID) {
      const int64_t r = p / w;
      px = x[p - r * w];
      py = y[r];
    } else {
      px = x[p];
      py = y[p];
    }
    pipe(s0, s1, px, py);
    out_x[p] = px;
    out_y[p] = py;
  }
}

template <int K0, int K1, int FAST>
void launch_fast(bool grid, int nb, hipStream_t st, const double* x, const double* y, int64_t w,
                 int64_t h, const XrsProjStep& s0, const XrsProjStep& s1, double* ox,
                 double* oy) {
  if (grid)
    hipLaunchKernelGGL((transform_kernel<K0, K1, true, FAST>), dim3(nb), dim3(kThreads), 0, st,
                       x, y, w, h, s0, s1, ox, oy);
  else
    hipLaunchKernelGGL((transform_kernel<K0, K1, false, FAST>), dim3(nb), dim3(kThreads), 0, st,
                       x, y, w, h, s0, s1, ox, oy);
}

template <int K0, int K1>
int launch_pipeline(bool grid, int nb, hipStream_t st, const double* x, const double* y,
                    int64_t w, int64_t h, const XrsProjStep& s0, const XrsProjStep& s1,
                    double* ox, double* oy) {
  if constexpr (K0 == XRS_PROJ_LAEA_INV && K1 == XRS_PROJ_TMERC_FWD) {
    const int fast = xrs_testing_value(XRS_TESTING_PROJ_TWO_STEP) ? proj::kFastNone
                                                                  : proj::fast_kind(K0, K1, s0);
    if (fast == proj::kFastObliq) {
      launch_fast<K0, K1, proj::kFastObliq>(grid, nb, st, x, y, w, h, s0, s1, ox, oy);
      return XRS_OK;
    }
    if (fast == proj::kFastEquit) {
      launch_fast<K0, K1, proj::kFastEquit>(grid, nb, st, x, y, w, h, s0, s1, ox, oy);
      return XRS_OK;
    }
  }
  launch_fast<K0, K1, proj::kFastNone>(grid, nb, st, x, y, w, h, s0, s1, ox, oy);
  return XRS_OK;
}

// second step: a forward projection (geographic -> target) or none
template <int K0>
int launch_second(int k1, bool grid, int nb, hipStream_t st, const double* x, const double* y,
                  int64_t w, int64_t h, const XrsProjStep& s0, const XrsProjStep& s1,
                  double* ox, double* oy) {
  switch (k1) {
    case 0: return launch_pipeline<K0, 0>(grid, nb, st, x, y, w, h, s0, s1, ox, oy);
    case XRS_PROJ_WEBMERC_FWD:
      return launch_pipeline<K0, XRS_PROJ_WEBMERC_FWD>(grid, nb, st, x, y, w, h, s0, s1, ox, oy);
    case XRS_PROJ_TMERC_FWD:
      return launch_pipeline<K0, XRS_PROJ_TMERC_FWD>(grid, nb, st, x, y, w, h, s0, s1, ox, oy);
    case XRS_PROJ_LAEA_FWD:
      return launch_pipeline<K0, XRS_PROJ_LAEA_FWD>(grid, nb, st, x, y, w, h, s0, s1, ox, oy);
    default: return XRS_ERR_ARG;
  }
}

}  // namespace
}  // namespace xrs

extern "C" int xrs_transform(const double* x, const double* y, int64_t w, int64_t h, int grid,
                             const XrsProjStep* steps, int nsteps, double* out_x, double* out_y,
                             void* stream) {
  using namespace xrs;
  if (!x || !y || !out_x || !out_y || w < 0 || h < 0 || nsteps < 0 || nsteps > 2 ||
      (nsteps > 0 && !steps)) {
    xrs_set_error("xrs_transform: invalid argument");
    return XRS_ERR_ARG;
  }
  // pipelines of crs.Transformer: [inverse], [forward], [inverse, forward] or none
  XrsProjStep s0{}, s1{};
  const int k0 = nsteps > 0 ? steps[0].kind : 0, k1 = nsteps > 1 ? steps[1].kind : 0;
  if (nsteps > 0) s0 = steps[0];
  if (nsteps > 1) s1 = steps[1];
  const bool fwd0 = k0 == XRS_PROJ_WEBMERC_FWD || k0 == XRS_PROJ_TMERC_FWD ||
                    k0 == XRS_PROJ_LAEA_FWD;
  if ((nsteps > 0 && (k0 < XRS_PROJ_WEBMERC_FWD || k0 > XRS_PROJ_LAEA_INV)) ||
      (nsteps > 1 && (fwd0 || !(k1 == XRS_PROJ_WEBMERC_FWD || k1 == XRS_PROJ_TMERC_FWD ||
                                k1 == XRS_PROJ_LAEA_FWD)))) {
    xrs_set_error("xrs_transform: unsupported projection pipeline");
    return XRS_ERR_ARG;
  }
  if (w * h == 0) return XRS_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nb = grid_blocks(w * h, kThreads, 256 * 16);
  const bool g = grid != 0;
  int rc;
  switch (k0) {
    case 0: rc = launch_pipeline<0, 0>(g, nb, st, x, y, w, h, s0, s1, out_x, out_y); break;
    case XRS_PROJ_WEBMERC_FWD:
      rc = launch_pipeline<XRS_PROJ_WEBMERC_FWD, 0>(g, nb, st, x, y, w, h, s0, s1, out_x, out_y);
      break;
    case XRS_PROJ_TMERC_FWD:
      rc = launch_pipeline<XRS_PROJ_TMERC_FWD, 0>(g, nb, st, x, y, w, h, s0, s1, out_x, out_y);
      break;
    case XRS_PROJ_LAEA_FWD:
      rc = launch_pipeline<XRS_PROJ_LAEA_FWD, 0>(g, nb, st, x, y, w, h, s0, s1, out_x, out_y);
      break;
    case XRS_PROJ_WEBMERC_INV:
      rc = launch_second<XRS_PROJ_WEBMERC_INV>(k1, g, nb, st, x, y, w, h, s0, s1, out_x, out_y);
      break;
    case XRS_PROJ_TMERC_INV:
      rc = launch_second<XRS_PROJ_TMERC_INV>(k1, g, nb, st, x, y, w, h, s0, s1, out_x, out_y);
      break;
    default:
      rc = launch_second<XRS_PROJ_LAEA_INV>(k1, g, nb, st, x, y, w, h, s0, s1, out_x, out_y);
      break;
  }
  if (rc != XRS_OK) return rc;
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}
