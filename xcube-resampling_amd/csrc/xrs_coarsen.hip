// xrs_coarsen.hip — K7: da.coarsen(agg, array, {-2: div_y, -1: div_x}) for gfx950.
//
// Replaces the third per-chunk seam of the affine downscale:
// dask's chunk.coarsen (reshape (h/dy, dy, w/dx, dx), reduce over the window
// axes) with the reducers of coarsen.py:50-155 — every AGG_METHODS key of
// constants.py:51-65.  The fused K3 in xrs_affine.hip covers the streaming
// reducers without materialising the intermediate; K7 is the general seam and
// the path for the reducers that need the whole window at once (median, mode)
// or two passes over it (std, var), exactly as the reference, which
// materialises the div-x intermediate before da.coarsen.
//
// One output pixel per thread, 64 x 4 output tiles, lanes on consecutive
// output columns: each lane reads its window's dx contiguous values per row,
// so a wave streams 64*dx contiguous elements of each window row.  The
// window re-reads of median/mode (O(n^2) rank / multiplicity counting —
// order-free, so results do not depend on a device sort) hit L1/L2.
//
// Numerics mirror numpy on the window (coarsen.py:78-111 via _reduce):
//   float: nanmean/nansum (window_sum: pairwise row sums, rows sequential —
//     the order numpy's add.reduce walks the contiguous (h/d, d, w/d, d) copy
//     — or one pairwise loop when the chunk is one window wide), nanvar
//     = sum((v - mean)^2) / count with the mean rounded to the dtype (numpy
//     nanvar), nanstd = sqrt(nanvar) in the dtype, nanmedian = (lo + hi) / 2
//     in the dtype (np.ma.median), all-NaN -> NaN;
//   int: mean/var/std/median in float64 then rint and cast back (_reduce);
//   mode (coarsen.py:114-155): key = int64(x - m) + m with m = int(chunk min),
//     most frequent key, ties -> smallest key, int64 result.  For floats m is
//     the min of the dask chunk that holds the window (device pre-pass);
//     NaN / +-inf in the array raise in the reference (int(nan), int(inf)) and
//     set XRS_EFLAG_NAN_TO_INT / XRS_EFLAG_INF_TO_INT here.

#include <cmath>
#include <limits>
#include <type_traits>

#include "xrs_common.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;
constexpr int kTileW = 64;
constexpr int kTileH = kThreads / kTileW;

enum Agg : int {
  AGG_MEAN = 1, AGG_SUM = 2, AGG_MAX = 3, AGG_MIN = 4, AGG_PROD = 5, AGG_COUNT = 6,
  AGG_FIRST = 7, AGG_LAST = 8, AGG_CENTER = 9, AGG_MEDIAN = 10, AGG_MODE = 11, AGG_STD = 12,
  AGG_VAR = 13,
};

struct CoarsenArgs {
  const void* src;
  int64_t nt, src_w, src_st, src_sy;
  void* dst;
  int dst_dtype;
  int64_t out_h, out_w, dst_st, dst_sy;
  int dy, dx, agg;
  const int32_t* chunk_t;   // dask chunk id per slice / row (mode on floats)
  const int32_t* chunk_y;
  const int32_t* chunk_x;   // per column (window == whole chunk test; NULL = one chunk)
  int64_t ncy, ncx;
  unsigned long long* cmin;  // per chunk: ordered key of the chunk minimum
  int32_t* err;
};

// total order of doubles as unsigned keys (for atomicMin)
__device__ inline unsigned long long order_key(double d) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ inline double order_val(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

__device__ inline int64_t chunk_of(const CoarsenArgs& a, int64_t t, int64_t r, int64_t c) {
  return ((int64_t)a.chunk_t[t] * a.ncy + a.chunk_y[r]) * a.ncx + a.chunk_x[c];
}

// mode pre-pass over the array (floats): per dask chunk the minimum, and the
// error bits of int(flat.min()) / int(flat.max()) (coarsen.py:133-134).
template <typename T>
__global__ void __launch_bounds__(kThreads)
chunk_min_kernel(CoarsenArgs a, int64_t h, int64_t w) {
  const T* src = static_cast<const T*>(a.src);
  const int64_t n = a.nt * h * w;
  bool nan = false, inf = false;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads) {
    const int64_t t = i / (h * w), rem = i - t * h * w, r = rem / w, c = rem - r * w;
    const T v = src[t * a.src_st + r * a.src_sy + c];
    nan |= is_nan(v);
    inf |= !is_nan(v) && !is_finite(v);
    if (!is_nan(v)) atomicMin(a.cmin + chunk_of(a, t, r, c), order_key((double)v));
  }
  if (__any(nan) && (threadIdx.x & 63) == 0) atomicOr(a.err, XRS_EFLAG_NAN_TO_INT);
  if (__any(inf) && (threadIdx.x & 63) == 0) atomicOr(a.err, XRS_EFLAG_INF_TO_INT);
}

// rank selection: the values of sorted order positions lo_k and hi_k among the
// window values that pass `keep` (O(n^2), order-free)
template <typename T, typename V, typename K>
__device__ inline void select2(int n, V&& val, K&& keep, int lo_k, int hi_k, T& lo, T& hi) {
  for (int i = 0; i < n; ++i) {
    const T vi = val(i);
    if (!keep(vi)) continue;
    int lt = 0, eq = 0;
    for (int j = 0; j < n; ++j) {
      const T vj = val(j);
      if (!keep(vj)) continue;
      lt += vj < vi ? 1 : 0;
      eq += vj == vi ? 1 : 0;
    }
    if (lt <= lo_k && lo_k < lt + eq) lo = vi;
    if (lt <= hi_k && hi_k < lt + eq) hi = vi;
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) coarsen_kernel(CoarsenArgs a) {
  constexpr bool kFloat = std::is_floating_point<T>::value;
  const int tx = threadIdx.x % kTileW;
  const int ty = __builtin_amdgcn_readfirstlane(threadIdx.x / kTileW);
  const int64_t ntx = (a.out_w + kTileW - 1) / kTileW, nty = (a.out_h + kTileH - 1) / kTileH;
  const XcdSlice sl = xcd_slice(ntx * nty * a.nt);
  const int ny = a.dy, nx = a.dx, nwin = ny * nx;
  for (int64_t wk = sl.first; wk < sl.end; wk += sl.step) {
    const int64_t t = wk / (ntx * nty);
    const int64_t rem = wk - t * ntx * nty;
    const int64_t tj = rem / ntx, ti = rem - tj * ntx;
    const int64_t oj = tj * kTileH + ty, oi = ti * kTileW + tx;
    if (oj >= a.out_h || oi >= a.out_w) continue;
    const T* base = static_cast<const T*>(a.src) + t * a.src_st + (oj * ny) * a.src_sy + oi * nx;
    auto at = [&](int r, int c) -> T { return base[(int64_t)r * a.src_sy + c]; };
    auto flat = [&](int i) -> T { return at(i / nx, i % nx); };
    const int64_t didx = t * a.dst_st + oj * a.dst_sy + oi;
    const int64_t c0 = oi * nx;
    const bool whole = a.chunk_x ? ((c0 == 0 || a.chunk_x[c0 - 1] != a.chunk_x[c0]) &&
                                    (c0 + nx == a.src_w || a.chunk_x[c0 + nx] != a.chunk_x[c0]))
                                 : a.src_w == nx;

    switch (a.agg) {
      case AGG_FIRST: store_any(a.dst, didx, a.dst_dtype, (double)at(0, 0), (int64_t)at(0, 0), !kFloat); continue;
      case AGG_LAST: {
        const T v = at(ny - 1, nx - 1);
        store_any(a.dst, didx, a.dst_dtype, (double)v, (int64_t)v, !kFloat);
        continue;
      }
      case AGG_CENTER: {
        const T v = at(ny / 2, nx / 2);
        store_any(a.dst, didx, a.dst_dtype, (double)v, (int64_t)v, !kFloat);
        continue;
      }
      case AGG_COUNT: {  // np.count_nonzero (NaN is non-zero)
        int64_t c = 0;
        for (int i = 0; i < nwin; ++i) c += flat(i) != (T)0 ? 1 : 0;
        store_any(a.dst, didx, a.dst_dtype, 0.0, c, true);
        continue;
      }
      default: break;
    }

    if (a.agg == AGG_MODE) {
      int64_t m = 0;
      if (kFloat) {  // m = int(flat.min()) of the window's dask chunk
        const double cm = order_val(a.cmin[chunk_of(a, t, oj * ny, oi * nx)]);
        m = (cm == cm && cm - cm == 0.0) ? (int64_t)cm : 0;
      }
      auto key = [&](int i) -> int64_t {
        const T v = flat(i);
        if (kFloat) return f64_to_i64_x86((double)(T)(v - (T)m)) + m;
        return (int64_t)v;
      };
      int64_t best = 0;
      int best_n = -1;
      for (int i = 0; i < nwin; ++i) {
        const int64_t ki = key(i);
        int c = 0;
        for (int j = 0; j < nwin; ++j) c += key(j) == ki ? 1 : 0;
        if (c > best_n || (c == best_n && ki < best)) { best = ki; best_n = c; }
      }
      store_any(a.dst, didx, a.dst_dtype, 0.0, best, true);
      continue;
    }

    if constexpr (kFloat) {
      if (a.agg == AGG_MEDIAN) {  // np.nanmedian (masked median for windows < 600)
        int c = 0;
        for (int i = 0; i < nwin; ++i) c += is_nan(flat(i)) ? 0 : 1;
        T res = (T)NAN;
        if (c > 0) {
          const int h = c / 2, l = (c % 2 == 1) ? h : h - 1;
          T lo = (T)0, hi = (T)0;
          select2<T>(nwin, flat, [](T v) { return !is_nan(v); }, l, h, lo, hi);
          res = (T)(lo + hi) / (T)2;
        }
        store_any(a.dst, didx, a.dst_dtype, (double)res, 0, false);
        continue;
      }
      // streaming reducers, first pass (numpy nan-reducer semantics)
      T prod = (T)1.0, mx = (T)0.0;
      int64_t cnt = 0;
      bool have = false;
      const T total = window_sum<T>(whole, ny, nx, [&](int r, int c) -> T {
          const T v = at(r, c);
          const bool nan = v != v;
          cnt += nan ? 0 : 1;
          prod = prod * (nan ? (T)1.0 : v);
          if (a.agg == AGG_MAX) {  // np.fmax.reduce
            if (!have) { mx = v; have = true; }
            else mx = (mx >= v || nan) ? mx : v;
          } else if (a.agg == AGG_MIN) {
            if (!have) { mx = v; have = true; }
            else mx = (mx <= v || nan) ? mx : v;
          }
          return nan ? (T)0.0 : v;
      });
      double res;
      if (a.agg == AGG_SUM) res = (double)total;
      else if (a.agg == AGG_PROD) res = (double)prod;
      else if (a.agg == AGG_MAX || a.agg == AGG_MIN) res = (double)mx;
      else {
        const T avg = (T)((double)total / (double)cnt);
        if (a.agg == AGG_MEAN) {
          res = (double)avg;
        } else {  // nanvar / nanstd: second pass over the NaN-zeroed deviations
          const T sq = window_sum<T>(whole, ny, nx, [&](int r, int c) -> T {
            const T v = at(r, c);
            if (v != v) return (T)0.0;
            const T d = v - avg;
            return d * d;
          });
          T var = cnt > 0 ? (T)((double)sq / (double)cnt) : (T)NAN;
          if (a.agg == AGG_STD) var = sqrt(var);
          res = (double)var;
        }
      }
      store_any(a.dst, didx, a.dst_dtype, res, 0, false);
    } else {
      // integer blocks: np.<reducer> (not the nan-variant), float results
      // rounded with rint and cast back (coarsen.py:104-110)
      double dres = 0.0;
      bool as_float = true;
      int64_t ires = 0;
      if (a.agg == AGG_MEDIAN) {  // np.median: mean of the middle one / two, in float64
        const int h = nwin / 2, l = (nwin % 2 == 1) ? h : h - 1;
        T lo = (T)0, hi = (T)0;
        select2<T>(nwin, flat, [](T) { return true; }, l, h, lo, hi);
        dres = (nwin % 2 == 1) ? (double)lo : ((double)lo + (double)hi) / 2.0;
      } else {
        int64_t isum = 0, iprod = 1, imx = 0;
        bool have = false;
        const double dtotal = window_sum<double>(whole, ny, nx, [&](int r, int c) -> double {
            const T v = at(r, c);
            isum += (int64_t)v;
            iprod *= (int64_t)v;
            if (!have) { imx = (int64_t)v; have = true; }
            else if (a.agg == AGG_MAX) imx = max(imx, (int64_t)v);
            else if (a.agg == AGG_MIN) imx = min(imx, (int64_t)v);
            return (double)v;
        });
        const double mean = dtotal / (double)nwin;
        if (a.agg == AGG_SUM) { as_float = false; ires = isum; }
        else if (a.agg == AGG_PROD) { as_float = false; ires = iprod; }
        else if (a.agg == AGG_MAX || a.agg == AGG_MIN) { as_float = false; ires = imx; }
        else if (a.agg == AGG_MEAN) dres = mean;
        else {  // np.var / np.std: float64 deviations
          const double sq = window_sum<double>(whole, ny, nx, [&](int r, int c) -> double {
            const double d = (double)at(r, c) - mean;
            return d * d;
          });
          dres = sq / (double)nwin;
          if (a.agg == AGG_STD) dres = sqrt(dres);
        }
      }
      if (as_float) ires = (int64_t)Conv<T>::from_f64(rint(dres));
      store_any(a.dst, didx, a.dst_dtype, 0.0, ires, true);
    }
  }
}

}  // namespace
}  // namespace xrs

extern "C" int64_t xrs_coarsen_workspace_size(int64_t n_chunks) {
  return n_chunks > 0 ? n_chunks * (int64_t)sizeof(unsigned long long) : 0;
}

extern "C" int xrs_coarsen(const void* src, int src_dtype, int64_t nt, int64_t src_h,
                           int64_t src_w, int64_t src_st, int64_t src_sy, void* dst,
                           int dst_dtype, int64_t dst_st, int64_t dst_sy, int64_t div_y,
                           int64_t div_x, int agg, const int32_t* chunk_t,
                           const int32_t* chunk_y, const int32_t* chunk_x, int64_t n_chunks_t,
                           int64_t n_chunks_y, int64_t n_chunks_x, void* workspace,
                           int64_t workspace_bytes, int32_t* err_flags, void* stream) {
  using namespace xrs;
  if (!src || !dst || nt < 1 || src_h < 1 || src_w < 1 || div_y < 1 || div_x < 1 ||
      div_y * div_x > (1 << 20) || src_h % div_y || src_w % div_x || src_sy < src_w ||
      agg < AGG_MEAN || agg > AGG_VAR) {
    xrs_set_error("xrs_coarsen: invalid argument");
    return XRS_ERR_ARG;
  }
  const bool is_float = src_dtype == XRS_DTYPE_F32 || src_dtype == XRS_DTYPE_F64;
  const bool need_min = agg == AGG_MODE && is_float;
  const int64_t nchunks = n_chunks_t * n_chunks_y * n_chunks_x;
  if (need_min && (!chunk_t || !chunk_y || !chunk_x || nchunks < 1 || !err_flags ||
                   !workspace || workspace_bytes < xrs_coarsen_workspace_size(nchunks))) {
    xrs_set_error("xrs_coarsen: float mode needs the chunk tables, a workspace and err_flags");
    return XRS_ERR_ARG;
  }
  CoarsenArgs a;
  a.src = src; a.nt = nt; a.src_w = src_w; a.src_st = src_st; a.src_sy = src_sy;
  a.dst = dst; a.dst_dtype = dst_dtype; a.out_h = src_h / div_y; a.out_w = src_w / div_x;
  a.dst_st = dst_st; a.dst_sy = dst_sy; a.dy = (int)div_y; a.dx = (int)div_x; a.agg = agg;
  a.chunk_t = chunk_t; a.chunk_y = chunk_y; a.chunk_x = chunk_x;
  a.ncy = n_chunks_y; a.ncx = n_chunks_x;
  a.cmin = static_cast<unsigned long long*>(workspace);
  a.err = err_flags;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (need_min)
    XRS_HIP_CHECK(hipMemsetAsync(workspace, 0xff, nchunks * sizeof(unsigned long long), st));
  const int64_t ntiles = ((a.out_w + kTileW - 1) / kTileW) * ((a.out_h + kTileH - 1) / kTileH) * nt;
  const int nb = grid_blocks(ntiles, 1, 256 * 64);
  return dispatch_dtype(src_dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    if (need_min) {
      hipLaunchKernelGGL((chunk_min_kernel<T>), dim3(grid_blocks(nt * src_h * src_w, kThreads, 2048)),
                         dim3(kThreads), 0, st, a, src_h, src_w);
      XRS_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL((coarsen_kernel<T>), dim3(nb), dim3(kThreads), 0, st, a);
    XRS_HIP_CHECK(hipGetLastError());
    return XRS_OK;
  });
}
