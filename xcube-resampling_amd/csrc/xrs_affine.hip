// xrs_affine.hip — K2/K3: same-CRS affine resampling (+ fused coarsen) for gfx950.
//
// Replaces, for one variable in one call:
//   * affine._upscale (affine.py:316-362): dask_image.ndinterp.affine_transform
//     -> scipy.ndimage.affine_transform, order 0/1, mode "constant", with the
//     per-output-chunk input slicing of dask-image (its footprint rules make
//     the edge/mirror behaviour depend on the chunk), incl. recover_nans;
//   * affine._downscale (affine.py:277-313): the div-x upscale followed by
//     da.coarsen(agg) (coarsen.py reducers), FUSED: the div-x intermediate is
//     never written to HBM — each output pixel computes its dj x di sub-samples
//     and reduces them in registers.
//
// K2a axis_tables: per intermediate row / column, the scipy footprint on that
//   axis — chunk-local coordinate c = offset' + o*scale (dask-image re-based
//   offset of the output chunk), OOB iff c < 0 or c > len-1 (-> cval), order 1:
//   start = floor(c), w0 = 1-(c-start), w1 = 1-w0, neighbours mirrored inside
//   the chunk's input slice; order 0: floor(c+0.5).  Stored as global source
//   indices + float64 weights.  Exact: the matrix is diagonal, so every
//   per-pixel coordinate depends on one output index only.
// K2b/K3 affine_kernel: one 256-thread block = a 64x4 tile of output pixels.
//   The source patch the tile needs (bounded by the monotone axis tables) is
//   staged in LDS with coalesced loads (two slices when the zero-weight time
//   neighbour of order-1 3-D transforms must be read), then each thread
//   evaluates scipy's corner sum ((v*wy)*wx accumulated from +0.0 in corner
//   order, last dim fastest) for its sub-samples and reduces them exactly like
//   numpy's nan-reducers under dask's chunk.coarsen (row sums pairwise, rows
//   accumulated sequentially, mean divided in float64).  Tiles whose patch
//   does not fit the LDS budget read the corners from global memory instead.

#include <cmath>
#include <limits>
#include <type_traits>

#include "xrs_common.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;
constexpr int kTileW = 64;                 // output pixels per tile row
constexpr int kTileH = kThreads / kTileW;  // output rows per tile
constexpr int kLdsBytes = 40 * 1024;       // patch budget per block (4 blocks / CU)

struct AxisTab {   // scipy footprint of one intermediate row / column
  int32_t g0;      // global source index of the first tap; -1 = out of bounds (cval)
  int32_t g1;      // second tap (order 1; mirrored); == g0 for order 0
  double w0, w1;   // order-1 spline weights (1 - x, 1 - w0)
};

struct AxisChunks {
  int64_t n;             // intermediate length along the axis
  int64_t chunk;         // dask-image output chunk size (uniform, last may be short)
  const int64_t* rel;    // per chunk: first index of the input slice
  const int64_t* len;    // per chunk: input slice length
  const double* off;     // per chunk: re-based offset (offset + M*chunk_off - rel)
  double scale;
};

// scipy map_coordinate, NI_EXTEND_MIRROR (spline footprint of mode "constant")
__device__ inline int64_t mirror(int64_t idx, int64_t n) {
  if (n <= 1) return 0;
  const int64_t s2 = 2 * n - 2;
  if (idx < 0) {
    idx = s2 * (int64_t)(-idx / s2) + idx;
    return idx <= 1 - n ? idx + s2 : -idx;
  }
  if (idx >= n) {
    idx -= s2 * (int64_t)(idx / s2);
    if (idx >= n) idx = s2 - idx;
  }
  return idx;
}

template <int ORDER>
__device__ inline AxisTab axis_entry(const AxisChunks& a, int64_t o) {
  const int64_t k = o / a.chunk, ol = o - k * a.chunk;
  const int64_t n = a.len[k];
  const double c = a.off[k] + (double)ol * a.scale;
  AxisTab e{-1, -1, 0.0, 0.0};
  if (c < 0.0 || c > (double)(n - 1)) return e;
  if (ORDER == 1) {
    const double s = floor(c);
    const double x = c - s;
    e.w0 = 1.0 - x;
    e.w1 = 1.0 - e.w0;
    e.g0 = (int32_t)(a.rel[k] + mirror((int64_t)s, n));
    e.g1 = (int32_t)(a.rel[k] + mirror((int64_t)s + 1, n));
  } else {
    e.g0 = e.g1 = (int32_t)(a.rel[k] + (int64_t)floor(c + 0.5));
    e.w0 = 1.0;
  }
  return e;
}

template <int ORDER>
__global__ void __launch_bounds__(kThreads)
affine_tables_kernel(AxisChunks ay, AxisChunks ax, AxisTab* __restrict__ ytab,
                     AxisTab* __restrict__ xtab) {
  const int64_t total = ay.n + ax.n;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    if (i < ay.n) ytab[i] = axis_entry<ORDER>(ay, i);
    else xtab[i - ay.n] = axis_entry<ORDER>(ax, i - ay.n);
  }
}

// ---- scipy output casts ----------------------------------------------------
template <typename T> struct ScipyOut {
  // integer outputs: round half away from zero, clamp to the type range
  __device__ static inline T cast(double t) {
    t = t > 0 ? t + 0.5 : t - 0.5;
    const double lo = (double)std::numeric_limits<T>::min();
    const double hi = (double)std::numeric_limits<T>::max();
    t = t > hi ? hi : t;
    t = t < lo ? lo : t;
    return (T)t;
  }
};
template <> struct ScipyOut<float> {
  __device__ static inline float cast(double t) { return (float)t; }
};
template <> struct ScipyOut<double> {
  __device__ static inline double cast(double t) { return t; }
};

template <typename T> __device__ inline bool is_nan(T v) { return false; }
template <> __device__ inline bool is_nan<float>(float v) { return v != v; }
template <> __device__ inline bool is_nan<double>(double v) { return v != v; }

enum Agg : int {
  AGG_NONE = 0, AGG_MEAN = 1, AGG_SUM = 2, AGG_MAX = 3, AGG_MIN = 4, AGG_PROD = 5,
  AGG_COUNT = 6, AGG_FIRST = 7, AGG_LAST = 8, AGG_CENTER = 9,
};

struct AffineArgs {
  const void* src;
  int64_t nt, src_h, src_w, src_st, src_sy;
  void* dst;
  int dst_dtype;
  int64_t out_h, out_w, dst_st, dst_sy;
  int64_t dy, dx;          // coarsen factors (1 = none)
  int agg;
  const int64_t* t_next;   // zero-weight time neighbour per slice, -1 = none
  double cval;
  const AxisTab* ytab;     // (out_h*dy) entries
  const AxisTab* xtab;     // (out_w*dx) entries
};

// numpy's float add.reduce of one contiguous window row (pairwise_sum):
// n < 8 sequential from -0.0; 8 <= n <= 128 eight accumulators (static
// indices: the blocks of 8 are unrolled), combined pairwise, then the tail.
// `val(i)` returns element i (already NaN-replaced by the caller).
template <typename A, typename F>
__device__ inline A pairwise_row(int n, F&& val) {
  if (n < 8) {
    A s = (A)-0.0;
    for (int i = 0; i < n; ++i) s = s + val(i);
    return s;
  }
  A r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = val(j);
  const int full = n - (n % 8);
  int i = 8;
  for (; i < full; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + val(i + j);
  }
  A s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) s = s + val(i);
  return s;
}

__device__ inline void store_any(void* dst, int64_t idx, int dtype, double fv, int64_t iv,
                                 bool is_int) {
  switch (dtype) {
    case XRS_DTYPE_F32: static_cast<float*>(dst)[idx] = (float)fv; break;
    case XRS_DTYPE_F64: static_cast<double*>(dst)[idx] = fv; break;
    case XRS_DTYPE_I64: static_cast<int64_t*>(dst)[idx] = is_int ? iv : (int64_t)fv; break;
    case XRS_DTYPE_U8: static_cast<uint8_t*>(dst)[idx] = (uint8_t)iv; break;
    case XRS_DTYPE_I8: static_cast<int8_t*>(dst)[idx] = (int8_t)iv; break;
    case XRS_DTYPE_U16: static_cast<uint16_t*>(dst)[idx] = (uint16_t)iv; break;
    case XRS_DTYPE_I16: static_cast<int16_t*>(dst)[idx] = (int16_t)iv; break;
    case XRS_DTYPE_U32: static_cast<uint32_t*>(dst)[idx] = (uint32_t)iv; break;
    case XRS_DTYPE_I32: static_cast<int32_t*>(dst)[idx] = (int32_t)iv; break;
    default: break;
  }
}

// Source access: LDS patch or global memory.
template <typename T>
struct Patch {
  const T* lds0;     // slice t
  const T* lds1;     // zero-weight time neighbour slice
  int32_t r0, c0, w; // patch origin and row length
  bool use_lds;
  const T* g0;       // global slice t
  const T* g1;       // global neighbour slice
  int64_t sy;
  __device__ inline T at0(int32_t r, int32_t c) const {
    return use_lds ? lds0[(r - r0) * w + (c - c0)] : g0[(int64_t)r * sy + c];
  }
  __device__ inline T at1(int32_t r, int32_t c) const {
    return use_lds ? lds1[(r - r0) * w + (c - c0)] : g1[(int64_t)r * sy + c];
  }
};

// One sub-sample: scipy's value (intermediate dtype I) — recover_nans handled
// by the caller passing RECOVER.
template <typename T, typename I, int ORDER, bool RECOVER>
__device__ inline I subsample(const Patch<T>& p, const AxisTab& ey, const AxisTab& ex,
                              bool has_t1, double cval) {
  if (ey.g0 < 0 || ex.g0 < 0) {
    if (RECOVER) {  // im = cval cast to T, norm = cval (float64)
      const double im = (double)ScipyOut<T>::cast(cval);
      const double norm = cval;
      return (fabs(norm) <= 1e-8) ? (I)NAN : (I)(im / norm);
    }
    return (I)ScipyOut<T>::cast(cval);
  }
  if (ORDER == 0) return (I)p.at0(ey.g0, ex.g0);
  const int32_t rr[2] = {ey.g0, ey.g1}, cc[2] = {ex.g0, ex.g1};
  const double wy[2] = {ey.w0, ey.w1}, wx[2] = {ex.w0, ex.w1};
  double t = 0.0, tn = 0.0;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const T v = p.at0(rr[a], cc[b]);
      if (RECOVER) {
        const double fv = is_nan(v) ? 0.0 : (double)v;
        const double mv = is_nan(v) ? 0.0 : 1.0;
        t += (fv * wy[a]) * wx[b];
        tn += (mv * wy[a]) * wx[b];
      } else {
        t += ((double)v * wy[a]) * wx[b];
      }
    }
  if (has_t1) {  // the zero-weight neighbour slice: contributes ((v*0)*wy)*wx
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const T v = p.at1(rr[a], cc[b]);
        if (RECOVER) {
          const double fv = is_nan(v) ? 0.0 : (double)v;
          t += ((fv * 0.0) * wy[a]) * wx[b];
          tn += ((is_nan(v) ? 0.0 : 0.0) * wy[a]) * wx[b];
        } else {
          t += (((double)v * 0.0) * wy[a]) * wx[b];
        }
      }
  }
  if (RECOVER) {
    const double im = (double)ScipyOut<T>::cast(t);
    return (fabs(tn) <= 1e-8) ? (I)NAN : (I)(im / tn);
  }
  return (I)ScipyOut<T>::cast(t);
}

template <typename T, typename I, int ORDER, bool RECOVER>
__global__ void __launch_bounds__(kThreads)
affine_kernel(AffineArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  T* lds = reinterpret_cast<T*>(smem);
  __shared__ int32_t s_bounds[4];

  const int tx = threadIdx.x % kTileW, ty = threadIdx.x / kTileW;
  const int64_t ntx = (a.out_w + kTileW - 1) / kTileW, nty = (a.out_h + kTileH - 1) / kTileH;
  const int64_t nwork = ntx * nty * a.nt;
  const XcdSlice sl = xcd_slice(nwork);
  const int64_t cap = kLdsBytes / (int64_t)sizeof(T);

  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    const int64_t t = w / (ntx * nty);
    const int64_t rem = w - t * ntx * nty;
    const int64_t tj = rem / ntx, ti = rem - tj * ntx;
    const int64_t oj0 = tj * kTileH, oi0 = ti * kTileW;
    const int64_t t1 = a.t_next ? a.t_next[t] : -1;
    const bool has_t1 = ORDER == 1 && t1 >= 0;

    // ---- patch bounds of the tile (rows/cols of all in-bounds taps)
    if (threadIdx.x < 4) s_bounds[threadIdx.x] = (threadIdx.x & 1) ? -1 : INT32_MAX;
    __syncthreads();
    {
      int32_t rmin = INT32_MAX, rmax = -1, cmin = INT32_MAX, cmax = -1;
      const int64_t ry0 = oj0 * a.dy, ry1 = min(a.out_h, oj0 + kTileH) * a.dy;
      for (int64_t r = ry0 + threadIdx.x; r < ry1; r += kThreads) {
        const AxisTab e = a.ytab[r];
        if (e.g0 >= 0) {
          rmin = min(rmin, min(e.g0, e.g1));
          rmax = max(rmax, max(e.g0, e.g1));
        }
      }
      const int64_t cx0 = oi0 * a.dx, cx1 = min(a.out_w, oi0 + kTileW) * a.dx;
      for (int64_t c = cx0 + threadIdx.x; c < cx1; c += kThreads) {
        const AxisTab e = a.xtab[c];
        if (e.g0 >= 0) {
          cmin = min(cmin, min(e.g0, e.g1));
          cmax = max(cmax, max(e.g0, e.g1));
        }
      }
      if (rmax >= 0) { atomicMin(&s_bounds[0], rmin); atomicMax(&s_bounds[1], rmax); }
      if (cmax >= 0) { atomicMin(&s_bounds[2], cmin); atomicMax(&s_bounds[3], cmax); }
    }
    __syncthreads();
    const int32_t pr0 = s_bounds[0], pr1 = s_bounds[1], pc0 = s_bounds[2], pc1 = s_bounds[3];
    const bool any = pr1 >= 0 && pc1 >= 0;
    const int64_t ph = any ? (int64_t)(pr1 - pr0 + 1) : 0, pw = any ? (int64_t)(pc1 - pc0 + 1) : 0;
    const int64_t need = ph * pw * (has_t1 ? 2 : 1);

    Patch<T> p;
    p.g0 = static_cast<const T*>(a.src) + t * a.src_st;
    p.g1 = has_t1 ? static_cast<const T*>(a.src) + t1 * a.src_st : p.g0;
    p.sy = a.src_sy;
    p.r0 = pr0; p.c0 = pc0; p.w = (int32_t)pw;
    p.use_lds = any && need <= cap;
    p.lds0 = lds;
    p.lds1 = lds + ph * pw;
    if (p.use_lds) {  // coalesced staging: consecutive threads -> consecutive columns
      const int64_t n1 = ph * pw;
      for (int64_t i = threadIdx.x; i < n1; i += kThreads) {
        const int64_t r = i / pw, c = i - r * pw;
        lds[i] = p.g0[(int64_t)(pr0 + r) * a.src_sy + pc0 + c];
        if (has_t1) lds[n1 + i] = p.g1[(int64_t)(pr0 + r) * a.src_sy + pc0 + c];
      }
    }
    __syncthreads();

    // ---- one output pixel per thread
    const int64_t oj = oj0 + ty, oi = oi0 + tx;
    if (oj < a.out_h && oi < a.out_w) {
      const int64_t didx = t * a.dst_st + oj * a.dst_sy + oi;
      const int ny = (int)a.dy, nx = (int)a.dx;
      if (a.agg == AGG_NONE || a.agg == AGG_FIRST || a.agg == AGG_LAST || a.agg == AGG_CENTER) {
        int sj = 0, si = 0;
        if (a.agg == AGG_LAST) { sj = ny - 1; si = nx - 1; }
        if (a.agg == AGG_CENTER) { sj = ny / 2; si = nx / 2; }
        const I v = subsample<T, I, ORDER, RECOVER>(p, a.ytab[oj * a.dy + sj],
                                                    a.xtab[oi * a.dx + si], has_t1, a.cval);
        if (std::is_floating_point<I>::value) store_any(a.dst, didx, a.dst_dtype, (double)v, 0, false);
        else store_any(a.dst, didx, a.dst_dtype, 0.0, (int64_t)v, true);
      } else if (std::is_floating_point<I>::value) {
        // float reducers (nanmean / nansum / nanmax / nanmin / nanprod / count)
        I total = (I)0.0, prod = (I)1.0, mx = (I)0.0;
        int64_t cnt = 0, nonzero = 0;
        bool have = false;
        for (int sj = 0; sj < ny; ++sj) {
          const AxisTab ey = a.ytab[oj * a.dy + sj];
          auto val = [&](int si) -> I {
            const I v = subsample<T, I, ORDER, RECOVER>(p, ey, a.xtab[oi * a.dx + si], has_t1,
                                                        a.cval);
            const bool nan = v != v;
            cnt += nan ? 0 : 1;
            nonzero += (v != (I)0.0) ? 1 : 0;
            prod = prod * (nan ? (I)1.0 : v);
            if (a.agg == AGG_MAX) {  // np.fmax.reduce: (acc >= v || isnan(v)) ? acc : v
              if (!have) { mx = v; have = true; }
              else mx = (mx >= v || nan) ? mx : v;
            } else if (a.agg == AGG_MIN) {
              if (!have) { mx = v; have = true; }
              else mx = (mx <= v || nan) ? mx : v;
            }
            return nan ? (I)0.0 : v;
          };
          total = total + pairwise_row<I>(nx, val);
        }
        double res;
        if (a.agg == AGG_MEAN) res = (double)(I)((double)total / (double)cnt);
        else if (a.agg == AGG_SUM) res = (double)total;
        else if (a.agg == AGG_PROD) res = (double)prod;
        else if (a.agg == AGG_COUNT) res = 0.0;
        else res = (double)mx;
        if (a.agg == AGG_COUNT) store_any(a.dst, didx, a.dst_dtype, 0.0, nonzero, true);
        else store_any(a.dst, didx, a.dst_dtype, res, 0, false);
      } else {
        // integer reducers: mean via float64 (np.mean) + rint; sum/prod in int64
        double total = 0.0;
        int64_t isum = 0, iprod = 1, nonzero = 0, mx = 0;
        bool have = false;
        for (int sj = 0; sj < ny; ++sj) {
          const AxisTab ey = a.ytab[oj * a.dy + sj];
          auto val = [&](int si) -> double {
            const I v = subsample<T, I, ORDER, RECOVER>(p, ey, a.xtab[oi * a.dx + si], has_t1,
                                                        a.cval);
            isum += (int64_t)v;
            iprod *= (int64_t)v;
            nonzero += v != 0 ? 1 : 0;
            if (!have) { mx = (int64_t)v; have = true; }
            else if (a.agg == AGG_MAX) mx = max(mx, (int64_t)v);
            else if (a.agg == AGG_MIN) mx = min(mx, (int64_t)v);
            return (double)v;
          };
          total = total + pairwise_row<double>(nx, val);
        }
        if (a.agg == AGG_MEAN) {
          const double m = rint(total / (double)(ny * nx));
          store_any(a.dst, didx, a.dst_dtype, 0.0, (int64_t)Conv<T>::from_f64(m), true);
        } else if (a.agg == AGG_SUM) {
          store_any(a.dst, didx, a.dst_dtype, 0.0, isum, true);
        } else if (a.agg == AGG_PROD) {
          store_any(a.dst, didx, a.dst_dtype, 0.0, iprod, true);
        } else if (a.agg == AGG_COUNT) {
          store_any(a.dst, didx, a.dst_dtype, 0.0, nonzero, true);
        } else {
          store_any(a.dst, didx, a.dst_dtype, 0.0, mx, true);
        }
      }
    }
    __syncthreads();  // the next tile overwrites the patch
  }
}

template <typename T, typename I, int ORDER, bool RECOVER>
int launch(const AffineArgs& a, const AxisChunks& ay, const AxisChunks& ax, AxisTab* ytab,
           AxisTab* xtab, hipStream_t st) {
  const int nbt = grid_blocks(ay.n + ax.n, kThreads, 1024);
  hipLaunchKernelGGL((affine_tables_kernel<ORDER>), dim3(nbt), dim3(kThreads), 0, st, ay, ax,
                     ytab, xtab);
  XRS_HIP_CHECK(hipGetLastError());
  AffineArgs args = a;
  args.ytab = ytab;
  args.xtab = xtab;
  const int64_t ntiles = ((a.out_w + kTileW - 1) / kTileW) * ((a.out_h + kTileH - 1) / kTileH) * a.nt;
  const int nb = grid_blocks(ntiles, 1, 256 * 4);
  hipLaunchKernelGGL((affine_kernel<T, I, ORDER, RECOVER>), dim3(nb), dim3(kThreads), kLdsBytes,
                     st, args);
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
any_nan_kernel(const T* __restrict__ src, int64_t n, int32_t* __restrict__ flag) {
  bool found = false;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads)
    found |= is_nan(src[i]);
  if (__any(found) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

}  // namespace
}  // namespace xrs

extern "C" int xrs_any_nan(const void* src, int src_dtype, int64_t n, int32_t* flag,
                           void* stream) {
  using namespace xrs;
  if (!src || !flag || n < 0) {
    xrs_set_error("xrs_any_nan: invalid argument");
    return XRS_ERR_ARG;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  XRS_HIP_CHECK(hipMemsetAsync(flag, 0, sizeof(int32_t), st));
  if (n == 0 || (src_dtype != XRS_DTYPE_F32 && src_dtype != XRS_DTYPE_F64)) return XRS_OK;
  const int nb = grid_blocks(n, kThreads, 1024);
  if (src_dtype == XRS_DTYPE_F32)
    hipLaunchKernelGGL((any_nan_kernel<float>), dim3(nb), dim3(kThreads), 0, st,
                       static_cast<const float*>(src), n, flag);
  else
    hipLaunchKernelGGL((any_nan_kernel<double>), dim3(nb), dim3(kThreads), 0, st,
                       static_cast<const double*>(src), n, flag);
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

extern "C" int64_t xrs_affine_workspace_size(int64_t inter_h, int64_t inter_w) {
  if (inter_h < 0 || inter_w < 0) return 0;
  return (inter_h + inter_w) * (int64_t)sizeof(xrs::AxisTab);
}

extern "C" int xrs_affine(const void* src, int src_dtype, int64_t nt, int64_t src_h,
                          int64_t src_w, int64_t src_st, int64_t src_sy, void* dst,
                          int dst_dtype, int64_t out_h, int64_t out_w, int64_t dst_st,
                          int64_t dst_sy, int64_t div_y, int64_t div_x, int agg, int order,
                          double scale_y, double scale_x, int64_t chunk_y,
                          const int64_t* rel_y, const int64_t* len_y, const double* off_y,
                          int64_t chunk_x, const int64_t* rel_x, const int64_t* len_x,
                          const double* off_x, const int64_t* t_next, double cval,
                          int recover_nan, void* workspace, int64_t workspace_bytes,
                          void* stream) {
  using namespace xrs;
  if (order != 0 && order != 1) {
    xrs_set_error("interp_methods must be one of 0, 1, 'nearest', 'bilinear'. Higher order is "
                  "not supported for 3D arrays in affine transforms, as it causes unintended "
                  "blending across the non-spatial (e.g., time) dimension.");
    return XRS_ERR_ARG;
  }
  if (!src || !dst || !rel_y || !len_y || !off_y || !rel_x || !len_x || !off_x || nt < 1 ||
      src_h < 1 || src_w < 1 || out_h < 1 || out_w < 1 || div_y < 1 || div_x < 1 ||
      div_x > 128 || chunk_y < 1 || chunk_x < 1 || src_sy < src_w || src_h > INT32_MAX ||
      src_w > INT32_MAX || agg < AGG_NONE || agg > AGG_CENTER ||
      (agg == AGG_NONE && (div_y != 1 || div_x != 1))) {
    xrs_set_error("xrs_affine: invalid argument");
    return XRS_ERR_ARG;
  }
  const bool is_float = src_dtype == XRS_DTYPE_F32 || src_dtype == XRS_DTYPE_F64;
  if (recover_nan && !is_float) {
    xrs_set_error("xrs_affine: recover_nan requires a floating-point source");
    return XRS_ERR_ARG;
  }
  const int64_t ih = out_h * div_y, iw = out_w * div_x;
  if (workspace_bytes < xrs_affine_workspace_size(ih, iw) || !workspace) {
    xrs_set_error("xrs_affine: workspace too small");
    return XRS_ERR_ARG;
  }
  AxisChunks ay{ih, chunk_y, rel_y, len_y, off_y, scale_y};
  AxisChunks ax{iw, chunk_x, rel_x, len_x, off_x, scale_x};
  AffineArgs a;
  a.src = src; a.nt = nt; a.src_h = src_h; a.src_w = src_w; a.src_st = src_st; a.src_sy = src_sy;
  a.dst = dst; a.dst_dtype = dst_dtype; a.out_h = out_h; a.out_w = out_w; a.dst_st = dst_st;
  a.dst_sy = dst_sy; a.dy = div_y; a.dx = div_x; a.agg = agg; a.t_next = t_next; a.cval = cval;
  a.ytab = a.xtab = nullptr;
  AxisTab* ytab = static_cast<AxisTab*>(workspace);
  AxisTab* xtab = ytab + ih;
  hipStream_t st = static_cast<hipStream_t>(stream);
  return dispatch_dtype(src_dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    if constexpr (std::is_floating_point<T>::value) {
      if (recover_nan)
        return order ? launch<T, double, 1, true>(a, ay, ax, ytab, xtab, st)
                     : launch<T, double, 0, true>(a, ay, ax, ytab, xtab, st);
    }
    return order ? launch<T, T, 1, false>(a, ay, ax, ytab, xtab, st)
                 : launch<T, T, 0, false>(a, ay, ax, ytab, xtab, st);
  });
}
