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
// K2b affine_direct_kernel (plain affine; coarsen first/last/center pick one
//   sub-sample): one output pixel per thread, lanes on consecutive columns,
//   scipy's corner sum ((v*wy)*wx accumulated from +0.0 in corner order, last
//   dim fastest; the zero-weight time neighbour of order-1 3-D transforms
//   included, as it propagates NaN) evaluated from global memory.  Its two
//   table entries are evaluated inline (the same axis_entry), so plain
//   affine is ONE launch (config 1 is launch-latency bound).
// K3 affine_reduce_kernel (mean/sum/max/min/prod/count): per 64x4 output
//   tile, the intermediate band of a group of sub-sample rows is evaluated
//   into LDS with lanes on consecutive intermediate columns (coalesced), then
//   each thread folds its pixel's values exactly like numpy's nan-reducers
//   under dask's chunk.coarsen (row sums pairwise, rows accumulated
//   sequentially, mean divided in float64).

#include <cmath>
#include <cstdlib>
#include <limits>
#include <type_traits>

#include "xrs_common.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;
constexpr int kTileW = 64;                 // output pixels per tile row
constexpr int kTileH = kThreads / kTileW;  // output rows per tile

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

// o / chunk: a 32-bit division while both fit (the usual case; a 64-bit
// division is a long software sequence on the critical path of K2)
__device__ inline int64_t chunk_of(int64_t o, int64_t chunk) {
  if (((uint64_t)o | (uint64_t)chunk) <= 0x7FFFFFFFull) return (int64_t)((uint32_t)o / (uint32_t)chunk);
  return o / chunk;
}

template <int ORDER>
__device__ inline AxisTab axis_entry(const AxisChunks& a, int64_t o) {
  const int64_t k = chunk_of(o, a.chunk), ol = o - k * a.chunk;
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
__device__ inline bool integral_entry(const AxisTab& e, int32_t g_first, int k) {
  return e.g0 >= 0 && e.g0 == g_first + k &&
         (ORDER == 0 || (e.w1 == 0.0 && e.g1 == e.g0 + 1));
}

// K3w's run entries: contiguous source taps (g0 = first + k, order 1: the
// second tap at g0 + 1, not mirrored) with any weights
template <int ORDER>
__device__ inline bool run_entry(const AxisTab& e, int32_t g_first, int k, bool weighted) {
  if (!weighted) return integral_entry<ORDER>(e, g_first, k);
  return e.g0 >= 0 && e.g0 == g_first + k && (ORDER == 0 || e.g1 == e.g0 + 1);
}

// With `runs` (K3i candidates, div dy x dx): also K3i's run records — per
// output row / column the first source index of its integral-contiguous run
// of entries (entry k of a pixel's run = first entry + k, order 1: weight 0
// and the next tap at +1), -1 where the layout breaks (the image's last row /
// column, where scipy mirrors the tap, always breaks it: K3i serves such
// pixels through its exact path).  `weighted` (K3w): the records of contiguous
// runs with any weights (run_entry).  Block 0 also sets K3i's counters: the
// slow-pixel count to 0 and — with time neighbours — whether any slice's
// zero-weight neighbour is another slice (plain stores: no memset before
// this launch; K3i and its finish run after it on the same stream).
template <int ORDER>
__global__ void __launch_bounds__(kThreads)
affine_tables_kernel(AxisChunks ay, AxisChunks ax, AxisTab* __restrict__ ytab,
                     AxisTab* __restrict__ xtab, int64_t dy, int64_t dx,
                     int32_t* __restrict__ counters, const int64_t* __restrict__ t_next,
                     int64_t nt, bool check_self, int32_t* __restrict__ yrun,
                     int32_t* __restrict__ xrun, bool wave_runs, bool weighted) {
  if (counters && blockIdx.x == 0) {
    bool other = false;   // K3i: a zero-weight time neighbour other than the slice?
    if (check_self)
      for (int64_t t = threadIdx.x; t < nt; t += kThreads) other = other || t_next[t] != t;
    const int any = __syncthreads_or(other);
    if (threadIdx.x == 0) {
      counters[1] = any ? 1 : 0;
      counters[2] = 0;   // K3i's slow-pixel count
    }
  }
  const int64_t total = ay.n + ax.n;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const bool is_y = i < ay.n;
    const int64_t o = is_y ? i : i - ay.n;
    const AxisChunks& ac = is_y ? ay : ax;
    const AxisTab e = axis_entry<ORDER>(ac, o);
    (is_y ? ytab : xtab)[o] = e;
    const int64_t d = is_y ? dy : dx;
    if (wave_runs) {
      // a run's d entries sit on consecutive lanes of one wave (d divides 64,
      // runs start at multiples of d on both axes: checked at launch): each
      // lane tests its own entry against the run's first, a ballot ANDs them
      const int lane = (int)(threadIdx.x & 63);
      const int k = (int)(o % d);
      const int32_t g_first = __shfl(e.g0, lane - k);
      const uint64_t bad = __ballot(!run_entry<ORDER>(e, g_first, k, weighted));
      if (k == 0)
        (is_y ? yrun : xrun)[o / d] = ((bad >> lane) & ((1ull << d) - 1)) == 0 ? e.g0 : -1;
    } else if (counters && o % d == 0) {   // K3i's run record of row / column o / d
      bool ok = e.g0 >= 0 && run_entry<ORDER>(e, e.g0, 0, weighted);
      for (int64_t j = 1; j < d && ok; ++j)
        ok = run_entry<ORDER>(axis_entry<ORDER>(ac, o + j), e.g0, (int)j, weighted);
      (is_y ? yrun : xrun)[o / d] = ok ? e.g0 : -1;
    }
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

// Source access: global memory (slice t and its zero-weight time neighbour
// t1).  The out-of-bounds marker (-1) is clamped to a valid element; eval()
// returns cval there.
template <typename T>
struct Src {
  const T* g0;       // slice t
  const T* g1;       // zero-weight time neighbour slice
  int64_t sy;
  __device__ inline int32_t crow(int32_t g) const { return max(g, 0); }
  __device__ inline int32_t ccol(int32_t g) const { return max(g, 0); }
  __device__ inline const T* row0(int32_t r) const { return g0 + (int64_t)r * sy; }
  __device__ inline const T* row1(int32_t r) const { return g1 + (int64_t)r * sy; }
};

// The source taps of one sub-sample (loaded first, evaluated later, so that
// several sub-samples' loads are in flight together).
template <typename T>
struct Taps {
  T v0[2][2], v1[2][2];
  // Branch-free: out-of-bounds entries (g0 == -1) read element 0 of the row /
  // column instead (a valid address); eval() then returns cval.
  template <int ORDER, bool HAS_T1, typename R>
  __device__ inline void load(const R& p, const AxisTab& ey, const AxisTab& ex) {
    const int32_t ra = p.crow(ey.g0), ca = p.ccol(ex.g0);
    const T* r0 = p.row0(ra);
    if (ORDER == 0) { v0[0][0] = r0[ca]; return; }
    const int32_t rb = p.crow(ey.g1), cb = p.ccol(ex.g1);
    const T* r1 = p.row0(rb);
    v0[0][0] = r0[ca]; v0[0][1] = r0[cb];
    v0[1][0] = r1[ca]; v0[1][1] = r1[cb];
    if (HAS_T1) {
      const T* q0 = p.row1(ra);
      const T* q1 = p.row1(rb);
      v1[0][0] = q0[ca]; v1[0][1] = q0[cb];
      v1[1][0] = q1[ca]; v1[1][1] = q1[cb];
    }
  }
  // scipy's value (intermediate dtype I); recover_nans when RECOVER
  template <typename I, int ORDER, bool RECOVER, bool HAS_T1>
  __device__ inline I eval(const AxisTab& ey, const AxisTab& ex, double cval) const {
    if (ey.g0 < 0 || ex.g0 < 0) {
      if (RECOVER) {  // im = cval cast to T, norm = cval (float64)
        const double im = (double)ScipyOut<T>::cast(cval);
        const double norm = cval;
        return (fabs(norm) <= 1e-8) ? (I)NAN : (I)(im / norm);
      }
      return (I)ScipyOut<T>::cast(cval);
    }
    if (ORDER == 0) {   // scipy's t = 0.0 + v*1.0: the value itself, -0 -> +0
      const T a = v0[0][0];
      return (I)(a == (T)0 ? (T)0 : a);
    }
    if (!RECOVER && ey.w1 == 0.0 && ex.w1 == 0.0) {
      // Integral position (w0 = 1, w1 = 0 on both axes; every integer-factor
      // coarsen of aligned grids): scipy's sum below reduces EXACTLY to
      //   t = ((((+0 + v00) + (v01*1)*0) + (v10*0)*1) + (v11*0)*0) [+ t1 terms]
      // where each zero-weight term is a signed zero, or NaN when its tap is
      // +-inf/NaN; adding signed zeros to +0 + v00 leaves v00 except -0 -> +0.
      bool bad = !is_finite(v0[0][1]) || !is_finite(v0[1][0]) || !is_finite(v0[1][1]);
      if (HAS_T1)
        bad = bad || !is_finite(v1[0][0]) || !is_finite(v1[0][1]) || !is_finite(v1[1][0]) ||
              !is_finite(v1[1][1]);
      const T a = v0[0][0];
      if (bad) return (I)ScipyOut<T>::cast(NAN);
      return (I)(a == (T)0 ? (T)0 : a);
    }
    const double wy[2] = {ey.w0, ey.w1}, wx[2] = {ex.w0, ex.w1};
    double t = 0.0, tn = 0.0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const T v = v0[a][b];
        if (RECOVER) {
          const double fv = is_nan(v) ? 0.0 : (double)v;
          const double mv = is_nan(v) ? 0.0 : 1.0;
          t += (fv * wy[a]) * wx[b];
          tn += (mv * wy[a]) * wx[b];
        } else {
          t += ((double)v * wy[a]) * wx[b];
        }
      }
    if (HAS_T1) {  // the zero-weight neighbour slice: contributes ((v*0)*wy)*wx
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const T v = v1[a][b];
          if (RECOVER) {
            const double fv = is_nan(v) ? 0.0 : (double)v;
            t += ((fv * 0.0) * wy[a]) * wx[b];
            tn += (0.0 * wy[a]) * wx[b];
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
};

template <typename T, typename I, int ORDER, bool RECOVER, bool HAS_T1>
__device__ inline I subsample(const Src<T>& p, const AxisTab& ey, const AxisTab& ex,
                              double cval) {
  Taps<T> tp;
  tp.template load<ORDER, HAS_T1>(p, ey, ex);
  return tp.template eval<I, ORDER, RECOVER, HAS_T1>(ey, ex, cval);
}

template <typename I>
__device__ inline void store_value(const AffineArgs& a, int64_t didx, I v) {
  if (std::is_floating_point<I>::value) store_any(a.dst, didx, a.dst_dtype, (double)v, 0, false);
  else store_any(a.dst, didx, a.dst_dtype, 0.0, (int64_t)v, true);
}

// The output dtype code of an intermediate type (K2's output dtype is its
// intermediate dtype for every plan the host makes: plain affine and the
// first / last / center picks keep it; anything else takes store_any).
template <typename I> constexpr int dtype_code() {
  return std::is_same<I, float>::value ? XRS_DTYPE_F32 : std::is_same<I, double>::value ? XRS_DTYPE_F64
       : std::is_same<I, uint8_t>::value ? XRS_DTYPE_U8 : std::is_same<I, int8_t>::value ? XRS_DTYPE_I8
       : std::is_same<I, uint16_t>::value ? XRS_DTYPE_U16 : std::is_same<I, int16_t>::value ? XRS_DTYPE_I16
       : std::is_same<I, uint32_t>::value ? XRS_DTYPE_U32 : std::is_same<I, int32_t>::value ? XRS_DTYPE_I32
       : std::is_same<I, int64_t>::value ? XRS_DTYPE_I64 : 0;
}

template <typename I>
__device__ inline void store_typed(const AffineArgs& a, int64_t didx, I v) {
  if (a.dst_dtype == dtype_code<I>()) {   // wave-uniform
    I* d = static_cast<I*>(a.dst) + didx;
    if (std::is_floating_point<I>::value) __builtin_nontemporal_store(v, d);
    else *d = v;
  } else {
    store_value<I>(a, didx, v);
  }
}

__device__ inline int32_t wave_uniform(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// K2 (no reduction: plain affine, or coarsen first/last/center which pick ONE
// sub-sample): lanes on consecutive output columns (coalesced xtab reads,
// stores and — for scales near 1 — source reads), a 64 x (4 x kDirectRows)
// tile per block: each wave takes kDirectRows consecutive output rows whose
// row entries are wave-uniform (scalar) and whose taps are all requested
// before the first is used, so a thread pays the entry -> tap -> store chain
// once for kDirectRows pixels (config 1: one resident round of blocks).
constexpr int kDirectRows = 4;
constexpr int kDirectSlices0 = 4;   // slices per grouped K2 item, order 0 (taps in flight: 16)
constexpr int kDirectSlices1 = 2;   // order 1 (4 taps per pixel: 32)

template <typename T, typename I, int ORDER, bool RECOVER, bool HAS_T1>
__device__ inline void direct_rows(const AffineArgs& a, const AxisChunks& ay, const Src<T>& p,
                                   int64_t t, int64_t oj0, int64_t oi, int sj,
                                   const AxisTab& ex) {
  AxisTab ey[kDirectRows];
  Taps<T> tp[kDirectRows];
#pragma unroll
  for (int q = 0; q < kDirectRows; ++q) {
    ey[q] = oj0 + q < a.out_h ? axis_entry<ORDER>(ay, (oj0 + q) * a.dy + sj)
                              : AxisTab{-1, -1, 0.0, 0.0};   // wave-uniform
    tp[q].template load<ORDER, HAS_T1>(p, ey[q], ex);
  }
#pragma unroll
  for (int q = 0; q < kDirectRows; ++q) {
    if (oj0 + q >= a.out_h) break;
    const I v = tp[q].template eval<I, ORDER, RECOVER, HAS_T1>(ey[q], ex, a.cval);
    store_typed<I>(a, t * a.dst_st + (oj0 + q) * a.dst_sy + oi, v);
  }
}

// K2 for slices that share one geometry — order 0, or order 1 without a
// zero-weight time neighbour (the dask shape: many chunks of one grid stacked
// on dim 0).  A work item is S consecutive slices x kItemH output rows x 64
// columns: the column entry and the kDirectRows row entries of a wave are
// evaluated once for all S slices, and the taps of S x kDirectRows pixels
// are in flight together per lane.  Items are listed band by band (a band =
// every 64-column tile of one slice group's kItemH rows) and the XCDs take
// whole bands in turn (K1 / K3i's deal: the items in flight cover one
// contiguous run of source rows; xcd_slice's eight contiguous eighths were
// slower for both).  Stores are typed (no per-pixel dtype switch).
template <typename T, typename I, int ORDER, bool RECOVER, int S>
__global__ void __launch_bounds__(kThreads)
affine_direct_group_kernel(AffineArgs a, AxisChunks ay, AxisChunks ax) {
  constexpr int64_t kItemH = kTileH * kDirectRows;
  const int tx = threadIdx.x % kTileW;
  const int ty = wave_uniform(threadIdx.x / kTileW);
  const int64_t ntx = (a.out_w + kTileW - 1) / kTileW, nty = (a.out_h + kItemH - 1) / kItemH;
  const int64_t ngroups = (a.nt + S - 1) / S;
  const int64_t nwork = ntx * nty * ngroups;
  int sj = 0, si = 0;
  if (a.agg == AGG_LAST) { sj = (int)a.dy - 1; si = (int)a.dx - 1; }
  if (a.agg == AGG_CENTER) { sj = (int)a.dy / 2; si = (int)a.dx / 2; }
  for (XcdGroups sg = xcd_groups(nwork, ntx);; sg.i += sg.step) {
    const int64_t w = sg.item();
    if (w >= nwork) break;
    const int64_t band = w / ntx, ti = w - band * ntx;
    const int64_t grp = band / nty, tj = band - grp * nty;
    const int64_t oj0 = tj * kItemH + ty * kDirectRows, oi = ti * kTileW + tx;
    if (oj0 >= a.out_h || oi >= a.out_w) continue;
    const AxisTab ex = axis_entry<ORDER>(ax, oi * a.dx + si);
    AxisTab ey[kDirectRows];
#pragma unroll
    for (int q = 0; q < kDirectRows; ++q)
      ey[q] = oj0 + q < a.out_h ? axis_entry<ORDER>(ay, (oj0 + q) * a.dy + sj)
                                : AxisTab{-1, -1, 0.0, 0.0};   // wave-uniform
    const int64_t t0 = grp * S;
    Taps<T> tp[S][kDirectRows];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      Src<T> p;   // a slice past nt (the last group) reads slice t0: a valid address
      p.g0 = p.g1 = static_cast<const T*>(a.src) + (t0 + k < a.nt ? t0 + k : t0) * a.src_st;
      p.sy = a.src_sy;
#pragma unroll
      for (int q = 0; q < kDirectRows; ++q) tp[k][q].template load<ORDER, false>(p, ey[q], ex);
    }
#pragma unroll
    for (int k = 0; k < S; ++k) {
      if (t0 + k >= a.nt) break;
#pragma unroll
      for (int q = 0; q < kDirectRows; ++q) {
        if (oj0 + q >= a.out_h) break;
        const I v = tp[k][q].template eval<I, ORDER, RECOVER, false>(ey[q], ex, a.cval);
        store_typed<I>(a, (t0 + k) * a.dst_st + (oj0 + q) * a.dst_sy + oi, v);
      }
    }
  }
}

template <typename T, typename I, int ORDER, bool RECOVER>
__global__ void __launch_bounds__(kThreads)
affine_direct_kernel(AffineArgs a, AxisChunks ay, AxisChunks ax) {
  constexpr int64_t kItemH = kTileH * kDirectRows;
  const int tx = threadIdx.x % kTileW;
  const int ty = wave_uniform(threadIdx.x / kTileW);
  const int64_t ntx = (a.out_w + kTileW - 1) / kTileW, nty = (a.out_h + kItemH - 1) / kItemH;
  const int64_t nwork = ntx * nty * a.nt;
  const XcdSlice sl = xcd_slice(nwork);
  int sj = 0, si = 0;
  if (a.agg == AGG_LAST) { sj = (int)a.dy - 1; si = (int)a.dx - 1; }
  if (a.agg == AGG_CENTER) { sj = (int)a.dy / 2; si = (int)a.dx / 2; }
  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    const int64_t t = w / (ntx * nty);
    const int64_t rem = w - t * ntx * nty;
    const int64_t tj = rem / ntx, ti = rem - tj * ntx;
    const int64_t oj0 = tj * kItemH + ty * kDirectRows, oi = ti * kTileW + tx;
    if (oj0 >= a.out_h || oi >= a.out_w) continue;
    const int64_t t1 = a.t_next ? a.t_next[t] : -1;
    Src<T> p;
    p.g0 = static_cast<const T*>(a.src) + t * a.src_st;
    p.g1 = t1 >= 0 ? static_cast<const T*>(a.src) + t1 * a.src_st : p.g0;
    p.sy = a.src_sy;
    const AxisTab ex = axis_entry<ORDER>(ax, oi * a.dx + si);
    if (ORDER == 1 && t1 >= 0) direct_rows<T, I, ORDER, RECOVER, true>(a, ay, p, t, oj0, oi, sj, ex);
    else direct_rows<T, I, ORDER, RECOVER, false>(a, ay, p, t, oj0, oi, sj, ex);
  }
}

// LDS position of intermediate column k of a tile row: one pad word every 32
// so the reduce pass (lane tx reads k = tx*dx + si) is bank-conflict free.
__device__ inline int lds_pos(int k) { return k + (k >> 5); }

// K3 (coarsen reducers): a block owns 64 output columns x kRedRows output
// rows.  For each group of G sub-sample rows it (A) evaluates the scipy
// sub-samples of the whole intermediate band — lanes on consecutive
// intermediate columns, so source reads and xtab reads coalesce and the row
// entry is block-uniform — into LDS, then (B) every thread folds its output
// pixel's dx values of each row exactly as numpy (pairwise row sum, rows
// accumulated sequentially).  The dy*dx intermediate never reaches HBM.
constexpr int kRedRows = kThreads / kTileW;  // 4 output rows per block

// (A) of K3: sub-samples of rows s0 .. s0+g_n-1 of every output row of the
// tile into the LDS band.  The column entry is the same for all rows
// (hoisted), the row entries are block-uniform (scalar loads), and the taps of
// KB rows are loaded before any is consumed (memory-level parallelism).
template <typename T, typename I, int ORDER, bool RECOVER, bool HAS_T1, int KB>
__device__ inline void fill_band(const AffineArgs& a, const Src<T>& p,
                                 const AxisTab* __restrict__ ytab,
                                 const AxisTab* __restrict__ xtab, I* buf, int64_t oj0,
                                 int64_t ic0, int rows, int s0, int g_n, int kmax,
                                 int row_stride) {
  for (int k = threadIdx.x; k < kmax; k += kThreads) {
    const AxisTab ex = xtab[ic0 + k];
    for (int r = 0; r < rows; ++r) {
      const AxisTab* yrow = ytab + (oj0 + r) * a.dy + s0;
      I* bcol = buf + (r * g_n) * row_stride + lds_pos(k);
      for (int g0 = 0; g0 < g_n; g0 += KB) {
        Taps<T> tp[KB];
        AxisTab ey[KB];
#pragma unroll
        for (int q = 0; q < KB; ++q) {
          ey[q] = yrow[min(g0 + q, g_n - 1)];
          tp[q].template load<ORDER, HAS_T1>(p, ey[q], ex);
        }
#pragma unroll
        for (int q = 0; q < KB; ++q)
          if (g0 + q < g_n)
            bcol[(g0 + q) * row_stride] =
                tp[q].template eval<I, ORDER, RECOVER, HAS_T1>(ey[q], ex, a.cval);
      }
    }
  }
}

// numpy's nan-reducers over one output pixel's dy x dx sub-samples in dask
// chunk.coarsen order (coarsen.py:72-111): each sub-sample row is one pairwise
// add.reduce, rows accumulated sequentially; integers accumulate in int64 /
// float64 and the mean is rint-ed back (coarsen.py:104-110).
template <typename I, bool FLOAT = std::is_floating_point<I>::value>
struct Fold {
  I total = (I)0.0, prod = (I)1.0, mx = (I)0.0;
  int64_t cnt = 0, nonzero = 0;
  bool have = false;
  template <typename F>
  __device__ inline void add_row(int agg, int nx, F&& get) {
    auto val = [&](int si) -> I {
      const I v = get(si);
      const bool nan = v != v;
      cnt += nan ? 0 : 1;
      nonzero += (v != (I)0.0) ? 1 : 0;
      prod = prod * (nan ? (I)1.0 : v);
      if (agg == AGG_MAX) {  // np.fmax.reduce
        if (!have) { mx = v; have = true; }
        else mx = (mx >= v || nan) ? mx : v;
      } else if (agg == AGG_MIN) {
        if (!have) { mx = v; have = true; }
        else mx = (mx <= v || nan) ? mx : v;
      }
      return nan ? (I)0.0 : v;
    };
    total = total + pairwise_row<I>(nx, val);
  }
  __device__ inline void store(const AffineArgs& a, int64_t didx) const {
    double res;
    if (a.agg == AGG_MEAN) res = (double)(I)((double)total / (double)cnt);
    else if (a.agg == AGG_SUM) res = (double)total;
    else if (a.agg == AGG_PROD) res = (double)prod;
    else res = (double)mx;
    if (a.agg == AGG_COUNT) store_any(a.dst, didx, a.dst_dtype, 0.0, nonzero, true);
    else store_any(a.dst, didx, a.dst_dtype, res, 0, false);
  }
};
template <typename I>
struct Fold<I, false> {
  double dtotal = 0.0;
  int64_t nonzero = 0, isum = 0, iprod = 1, imx = 0, n = 0;
  bool have = false;
  template <typename F>
  __device__ inline void add_row(int agg, int nx, F&& get) {
    auto val = [&](int si) -> double {
      const I v = get(si);
      isum += (int64_t)v;
      iprod *= (int64_t)v;
      nonzero += v != 0 ? 1 : 0;
      if (!have) { imx = (int64_t)v; have = true; }
      else if (agg == AGG_MAX) imx = max(imx, (int64_t)v);
      else if (agg == AGG_MIN) imx = min(imx, (int64_t)v);
      return (double)v;
    };
    dtotal = dtotal + pairwise_row<double>(nx, val);
    n += nx;
  }
  __device__ inline void store(const AffineArgs& a, int64_t didx) const {
    if (a.agg == AGG_MEAN) {
      const double m = rint(dtotal / (double)n);
      store_any(a.dst, didx, a.dst_dtype, 0.0, (int64_t)Conv<I>::from_f64(m), true);
    } else if (a.agg == AGG_SUM) {
      store_any(a.dst, didx, a.dst_dtype, 0.0, isum, true);
    } else if (a.agg == AGG_PROD) {
      store_any(a.dst, didx, a.dst_dtype, 0.0, iprod, true);
    } else if (a.agg == AGG_COUNT) {
      store_any(a.dst, didx, a.dst_dtype, 0.0, nonzero, true);
    } else {
      store_any(a.dst, didx, a.dst_dtype, 0.0, imx, true);
    }
  }
};

// sub-sample rows whose taps are loaded together (2 measured fastest of 2/4/8)
constexpr int kReduceBatch = 2;

template <typename T, typename I, int ORDER, bool RECOVER>
__device__ inline void reduce_body(const AffineArgs& a, const AxisTab* __restrict__ ytab,
                                   const AxisTab* __restrict__ xtab, int group) {
  constexpr int KB = kReduceBatch;
  extern __shared__ __align__(16) unsigned char smem[];
  I* buf = reinterpret_cast<I*>(smem);
  const int tx = threadIdx.x % kTileW;
  const int ty = wave_uniform(threadIdx.x / kTileW);
  const int ny = (int)a.dy, nx = (int)a.dx;
  const int band_w = kTileW * nx;                 // intermediate columns per tile row
  const int row_stride = lds_pos(band_w - 1) + 1;
  const int64_t ntx = (a.out_w + kTileW - 1) / kTileW;
  const int64_t nty = (a.out_h + kRedRows - 1) / kRedRows;
  const int64_t nwork = ntx * nty * a.nt;
  const XcdSlice sl = xcd_slice(nwork);
  const int64_t iw = a.out_w * a.dx;

  for (int64_t w = sl.first; w < sl.end; w += sl.step) {
    const int64_t t = w / (ntx * nty);
    const int64_t rem = w - t * ntx * nty;
    const int64_t tj = rem / ntx, ti = rem - tj * ntx;
    const int64_t oj0 = tj * kRedRows, oi0 = ti * kTileW;
    const int rows = (int)min((int64_t)kRedRows, a.out_h - oj0);
    const int64_t t1 = a.t_next ? a.t_next[t] : -1;
    Src<T> p;
    p.g0 = static_cast<const T*>(a.src) + t * a.src_st;
    p.g1 = t1 >= 0 ? static_cast<const T*>(a.src) + t1 * a.src_st : p.g0;
    p.sy = a.src_sy;
    const int64_t ic0 = oi0 * a.dx;
    const int kmax = (int)min((int64_t)band_w, iw - ic0);

    const bool two = ORDER == 1 && t1 >= 0;

    Fold<I> fold;
    for (int s0 = 0; s0 < ny; s0 += group) {
      const int g_n = min(group, ny - s0);
      // (A) sub-samples of rows s0 .. s0+g_n-1 into the band
      if (two) {
        fill_band<T, I, ORDER, RECOVER, true, KB>(a, p, ytab, xtab, buf, oj0, ic0, rows, s0,
                                                  g_n, kmax, row_stride);
      } else {
        fill_band<T, I, ORDER, RECOVER, false, KB>(a, p, ytab, xtab, buf, oj0, ic0, rows, s0,
                                                   g_n, kmax, row_stride);
      }
      __syncthreads();
      // (B) fold this thread's values row by row
      const int64_t oi = oi0 + tx;
      if (ty < rows && oi < a.out_w) {
        for (int g = 0; g < g_n; ++g) {
          const I* brow = buf + (ty * g_n + g) * row_stride;
          const int kb = tx * nx;
          fold.add_row(a.agg, nx, [&](int si) { return brow[lds_pos(kb + si)]; });
        }
      }
      __syncthreads();  // the next group overwrites the band
    }

    const int64_t oj = oj0 + ty, oi = oi0 + tx;
    if (ty < rows && oi < a.out_w) fold.store(a, t * a.dst_st + oj * a.dst_sy + oi);
  }
}

template <typename T, typename I, int ORDER, bool RECOVER>
__global__ void __launch_bounds__(kThreads)
affine_reduce_kernel(AffineArgs a, const AxisTab* __restrict__ ytab,
                     const AxisTab* __restrict__ xtab, int group) {
  reduce_body<T, I, ORDER, RECOVER>(a, ytab, xtab, group);
}


// K3i: coarsen reducers when every sub-sample of a pixel sits on a source
// pixel (scale 1 at the div-x grid with integral offsets — every aligned
// integer-factor coarsen, config 3 — or any order-0 grid at scale 1).  A
// sub-sample is then the source value itself, -0 -> +0 (scipy's weighted sum
// starts at 0.0); order 1 adds zero-weight taps (the column right of the run,
// the row below, the time neighbour) that only matter when non-finite (NaN).
//
// One thread per output pixel, lanes on consecutive output columns, a work
// item = 256 output columns x R output rows.  When the item's R*D sub-sample
// rows are one integral-contiguous run of source rows (everywhere but the
// image's last row, where scipy mirrors the tap), every source row the item
// needs is loaded up front — R*D (+1) DX-wide vector loads per lane, a wave
// reads 64*D contiguous elements per row — so one memory round trip serves R
// output rows.  The right tap column comes from the next lane.  A pixel whose
// columns are not integral-contiguous, or whose rect holds a non-finite value
// (order 1), is appended to a list that integral_slow_kernel evaluates
// through the exact per-sub-sample path — same result, slower.  A list
// longer than the workspace holds hands the whole launch to the generic K3.
// output rows per item: 16 (f32) / 8 (f64) sub-sample rows of D elements,
// 8 for f32 at D = 4.  Config 3 (round 4, items dealt to the XCDs band by
// band): R = 2 (9 source rows per item) 0.213-0.214 ms against R = 8 (33
// rows, 211 VGPRs, two waves per SIMD) 0.222 ms and R = 1 / 4 0.24 ms
// (profiles/r04_k3_ab.log); round 3's XCD-slice deal had preferred R = 8.
inline constexpr int64_t int_rows(int64_t d, int64_t esz) {
  return d >= 8 ? 1 : (d == 4 && esz == 4) ? 2 : (16 / d) / (esz / 4) < 1 ? 1 : (16 / d) / (esz / 4);
}
template <typename T, int D> struct IntItem {
  static constexpr int R = (int)int_rows(D, sizeof(T));
};

// DX consecutive elements; the compiler merges them into dwordx4 / dwordx2
// loads (global loads need only element alignment on gfx950).  No run-time
// alignment branch: a branch per row would serialise the item's loads.
template <typename T, int DX>
__device__ inline void load_run(const T* p, T (&v)[DX]) {
#pragma unroll
  for (int c = 0; c < DX; ++c) v[c] = p[c];
}

// W (K3w): the runs are contiguous but the weights fractional (scale 1 at the
// div-x grid, order 1, offsets off the integral layout — a target grid not
// aligned to the source).  The same loads; each sub-sample is scipy's sum of
// its 2 x 2 taps with the row / column weights of the tables (f64, scipy's
// corner order, cast to T), so a pixel's only exact-path case is a broken run
// (an image edge): non-finite taps are part of the formula.
template <typename T, int ORDER, int D, bool TWO, bool W = false>
// (K3w under launch bounds for 4 waves per SIMD: 0.273 vs 0.295 ms at the 3
// its 145 VGPRs allowed, profiles/r06d_*)
__global__ void __launch_bounds__(kThreads, W ? 4 : 1)
affine_reduce_integral_kernel(AffineArgs a, const int32_t* __restrict__ yrun,
                              const int32_t* __restrict__ xrun,
                              const int32_t* __restrict__ nonself, int32_t* __restrict__ nslow,
                              int64_t* __restrict__ slow_list, int64_t slow_cap) {
  // with time neighbours: the TWO=false instance serves launches where every
  // neighbour is the slice itself (its taps are the ones already checked)
  if (nonself && TWO != (*nonself != 0)) return;
  constexpr int R = IntItem<T, D>::R;
  constexpr int NE = R * D;                          // sub-sample rows of an item
  constexpr int NRT = NE + (ORDER == 1 ? 1 : 0);     // source rows loaded
  constexpr bool T1 = ORDER == 1 && TWO;
  const int lane = threadIdx.x & 63;
  const int64_t ntx = (a.out_w + kThreads - 1) / kThreads;
  const int64_t nty = (a.out_h + R - 1) / R;
  const int64_t nwork = ntx * nty * a.nt;
  // the XCDs take whole bands of items in turn (XCD x: bands x, x + 8, ...):
  // the chip's items in flight cover one contiguous run of source rows, and
  // the row two bands share is read by neighbouring XCDs at about the same
  // time.  Dealing each XCD one contiguous eighth of the image instead (eight
  // separate runs in flight) took 0.231 vs 0.222 ms at config 3, items dealt
  // one by one 0.261 ms (profiles/r04_k3_ab.log).
  // the slow list overflowed (seen by this wave): a grid off the integral
  // layout, which the finish hands to the generic K3 — stop appending
  bool full = false;
  for (XcdGroups sg = xcd_groups(nwork, ntx);; sg.i += sg.step) {
    const int64_t w = sg.item();
    if (w >= nwork) break;
    const int64_t t = w / (ntx * nty);
    const int64_t rem = w - t * ntx * nty;
    const int64_t tj = rem / ntx, ti = rem - tj * ntx;
    const int64_t oi = ti * kThreads + threadIdx.x;
    const bool active = oi < a.out_w;
    const int64_t t1 = T1 ? a.t_next[t] : -1;
    const T* g0 = static_cast<const T*>(a.src) + t * a.src_st;
    const T* g1 = T1 && t1 >= 0 ? static_cast<const T*>(a.src) + t1 * a.src_st : g0;

    // columns: the pixel's D sub-sample columns must be one contiguous run
    // c0 .. c0+D-1 (order 1: weight 0, right tap at +1) — the tables kernel's
    // run record (first column, -1 = not a run): 4 B per lane, one round trip
    const int32_t c0 = active ? xrun[oi] : -1;
    const bool col_fast = c0 >= 0;
    // rows: output rows q < nfast take the fast path — the leading rows whose
    // run records continue the item's first run (lane q checks output row q;
    // wave-uniform result).  The image's last output row (mirrored tap) and a
    // short last item no longer send the whole item to the exact path.
    const int64_t oj0 = tj * R;
    const int nrows = (int)min((int64_t)R, a.out_h - oj0);
    const int32_t el = yrun[oj0 + min(lane, nrows - 1)];
    const int32_t gf = __builtin_amdgcn_readfirstlane(el);   // lane 0's: scalar row math
    const uint64_t okm = __ballot(lane < nrows && el >= 0 && el == gf + lane * D);
    const int nfast = __builtin_ctzll(~okm);   // leading rows (R < 64)
    // (rows off the integral layout load nothing: nfast = 0)
    const bool rows_fast = nfast > 0;
    const bool fast = rows_fast && col_fast;
    // loads are unconditional (a branch per row would serialise them): lanes
    // off the fast path read column 0 of the same rows and ignore the values
    const int32_t cl = fast ? c0 : 0;
    const int32_t c0n = __shfl_down(c0, 1);
    const bool fast_n = __shfl_down((int)fast, 1) != 0;
    const bool nb_lane = lane < 63 && fast_n && c0n == c0 + D;
    const int32_t cnb = (fast && !nb_lane) ? c0 + D : cl;   // right tap column read here

    T v[NRT][D], nbv[NRT], v1[T1 ? NRT : 1][T1 ? D : 1], nbv1[T1 ? NRT : 1];
    if (rows_fast) {   // wave-uniform
#pragma unroll
      for (int r = 0; r < NRT; ++r) {
        // rows past the fast prefix are clamped into the image (values unused)
        const int32_t rr = min(gf + r, (int32_t)(a.src_h - 1));
        const T* row = g0 + (int64_t)rr * a.src_sy;
        load_run<T, D>(row + cl, v[r]);
        if constexpr (T1) {
          const T* row1 = g1 + (int64_t)rr * a.src_sy;
          load_run<T, D>(row1 + cl, v1[r]);
          nbv1[r] = row1[cnb];
        }
      }
      // the right-hand taps: from the next lane's run (shuffle below), loaded
      // only by lanes whose neighbour does not hold it (a wave's last lane,
      // a break in the runs) — one branch around all rows' loads
      if (ORDER == 1 && !nb_lane) {
#pragma unroll
        for (int r = 0; r < NRT; ++r) {
          const int32_t rr = min(gf + r, (int32_t)(a.src_h - 1));
          nbv[r] = g0[(int64_t)rr * a.src_sy + cnb];
        }
      }
      if (ORDER == 1) {
#pragma unroll
        for (int r = 0; r < NRT; ++r) {
          const T sh = __shfl_down(v[r][0], 1);
          nbv[r] = nb_lane ? sh : nbv[r];
          if constexpr (T1) {
            const T sh1 = __shfl_down(v1[r][0], 1);
            nbv1[r] = nb_lane ? sh1 : nbv1[r];
          }
        }
      }
    }
    // K3w: the lane's column weights (its D entries of the x table)
    double wx0[W ? D : 1], wx1[W ? D : 1];
    if constexpr (W) {
#pragma unroll
      for (int si = 0; si < D; ++si) {
        const AxisTab& e = a.xtab[(fast ? oi : 0) * D + si];
        wx0[si] = e.w0;
        wx1[si] = e.w1;
      }
    }
    bool overflow = false;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      if (q >= nrows) break;
      const int64_t oj = oj0 + q;
      const int64_t didx = t * a.dst_st + oj * a.dst_sy + oi;
      if (!active) continue;
      const bool lean = a.agg == AGG_MEAN || a.agg == AGG_SUM;
      const bool fq = fast && q < nfast;
      bool slow = !fq;
      if constexpr (W) {
        if (fq) {
          double wy0[D], wy1[D];   // the output row's D row entries (wave-uniform)
#pragma unroll
          for (int sj = 0; sj < D; ++sj) {
            const AxisTab& e = a.ytab[oj * D + sj];
            wy0[sj] = e.w0;
            wy1[sj] = e.w1;
          }
          // sub-sample (sj, si): Taps::eval's sum (affine_tables_kernel's
          // weights, corner order, the zero-weight time neighbour after)
          auto sub = [&](int sj, int si) -> T {
            const int r = q * D + sj;
            const T a00 = v[r][si], a01 = si + 1 < D ? v[r][si + 1] : nbv[r];
            const T a10 = v[r + 1][si], a11 = si + 1 < D ? v[r + 1][si + 1] : nbv[r + 1];
            double tt = 0.0;
            tt += ((double)a00 * wy0[sj]) * wx0[si];
            tt += ((double)a01 * wy0[sj]) * wx1[si];
            tt += ((double)a10 * wy1[sj]) * wx0[si];
            tt += ((double)a11 * wy1[sj]) * wx1[si];
            if constexpr (T1) {
              const T b00 = v1[r][si], b01 = si + 1 < D ? v1[r][si + 1] : nbv1[r];
              const T b10 = v1[r + 1][si], b11 = si + 1 < D ? v1[r + 1][si + 1] : nbv1[r + 1];
              tt += (((double)b00 * 0.0) * wy0[sj]) * wx0[si];
              tt += (((double)b01 * 0.0) * wy0[sj]) * wx1[si];
              tt += (((double)b10 * 0.0) * wy1[sj]) * wx0[si];
              tt += (((double)b11 * 0.0) * wy1[sj]) * wx1[si];
            }
            return ScipyOut<T>::cast(tt);
          };
          if (lean) {   // nanmean / nansum: NaN sub-samples skipped
            T total = (T)0;
            int cnt = 0;
#pragma unroll
            for (int sj = 0; sj < D; ++sj)
              total = total + pairwise_row<T>(D, [&](int si) {
                const T x = sub(sj, si);
                const bool nan = x != x;
                cnt += nan ? 0 : 1;
                return nan ? (T)0 : x;
              });
            const double res = a.agg == AGG_MEAN ? (double)(T)((double)total / (double)cnt)
                                                 : (double)total;
            store_any(a.dst, didx, a.dst_dtype, res, 0, false);
          } else {
            Fold<T> fold;
#pragma unroll
            for (int sj = 0; sj < D; ++sj)
              fold.add_row(a.agg, D, [&](int si) { return sub(sj, si); });
            fold.store(a, didx);
          }
          continue;
        }
      } else if (fq && lean) {
        // The values' sum equals numpy's whatever their zero signs (a signed
        // zero only flips the sign of a zero partial, and the total starts at
        // +0), so the -0 -> +0 map is not needed here.  Order 1: every value
        // and zero-weight tap is finite iff their sums are (an overflow to
        // inf only sends the pixel to the exact path).
        T total = (T)0;
        int cnt = D * D;
        if (ORDER == 1) {
#pragma unroll
          for (int sj = 0; sj < D; ++sj)
            total = total + pairwise_row<T>(D, [&](int si) { return v[q * D + sj][si]; });
          T extra = (T)0;   // zero-weight taps: right column, row below, t+1
#pragma unroll
          for (int r = q * D; r <= q * D + D; ++r) {
            extra = extra + nbv[r];
            if (T1) extra = extra + nbv1[T1 ? r : 0];
          }
#pragma unroll
          for (int c = 0; c < D; ++c) extra = extra + v[q * D + D][c];
          if (T1) {
#pragma unroll
            for (int r = q * D; r <= q * D + D; ++r)
#pragma unroll
              for (int c = 0; c < D; ++c) extra = extra + v1[T1 ? r : 0][c];
          }
          slow = !is_finite(total) || !is_finite(extra);
        } else {   // order 0: NaN values are skipped by the nan-reducers
          cnt = 0;
#pragma unroll
          for (int sj = 0; sj < D; ++sj)
            total = total + pairwise_row<T>(D, [&](int si) {
              const T x = v[q * D + sj][si];
              const bool nan = x != x;
              cnt += nan ? 0 : 1;
              return nan ? (T)0 : x;
            });
        }
        if (!slow) {
          const double res = a.agg == AGG_MEAN ? (double)(T)((double)total / (double)cnt)
                                               : (double)total;
          store_any(a.dst, didx, a.dst_dtype, res, 0, false);
          continue;
        }
      } else if (ORDER == 1 && fq) {   // zero-weight taps: right column, row below, t+1
#pragma unroll
        for (int r = q * D; r <= q * D + D; ++r) {
          slow = slow || !is_finite(nbv[r]);
          if (T1) slow = slow || !is_finite(nbv1[T1 ? r : 0]);
#pragma unroll
          for (int c = 0; c < D; ++c) {
            slow = slow || !is_finite(v[r][c]);
            if (T1) slow = slow || !is_finite(v1[T1 ? r : 0][c]);
          }
        }
      }
      // the exact path runs in integral_slow_kernel (keeps its registers out
      // of this streaming kernel); one atomic per wave and row reserves the
      // wave's slots (per-lane atomics on the one counter serialised at its
      // L2 channel: 3.9 ms of K3i for a 3.5x downscale, whose every pixel is
      // slow, profiles/r06e_*)
      const uint64_t sm = __ballot(slow && !full);
      if (sm) {   // wave-uniform
        const int first = __builtin_ctzll(sm);
        int32_t base = 0;
        if (lane == first) base = atomicAdd(nslow, __builtin_popcountll(sm));
        base = __builtin_amdgcn_readlane(base, first);
        if (slow) {
          const int32_t k = base + (int32_t)__builtin_amdgcn_mbcnt_hi(
                                       (uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0));
          if (k < slow_cap) slow_list[k] = (t * a.out_h + oj) * a.out_w + oi;
          else overflow = true;
        }
      }
      if (slow) continue;
      Fold<T> fold;
#pragma unroll
      for (int sj = 0; sj < D; ++sj)
        fold.add_row(a.agg, D, [&](int si) {
          const T x = v[q * D + sj][si];
          return x == (T)0 ? (T)0 : x;   // scipy's 0.0 + w*x: -0 -> +0
        });
      fold.store(a, didx);
    }
    // once the list has overflowed the finish reruns the whole launch through
    // the generic K3, so nothing K3i still does would be kept: stop (a grid
    // off the integral layout overflows within every wave's first item)
    full = full || __any(overflow);
    if (full) break;
  }
}

// K3i's slow pixels (exact path).  Lanes work on sub-samples, not pixels: a
// wave takes 64 / D^2 listed pixels, lane l evaluates sub-sample l % D^2 of
// its pixel through Taps (scipy's sum; all loads of a wave in flight
// together), and the pixel's first lane folds the D^2 values in numpy's order.
template <typename T, int ORDER, int D>
__device__ inline void slow_body(const AffineArgs& a, const AxisTab* __restrict__ ytab,
                                 const AxisTab* __restrict__ xtab,
                                 const int64_t* __restrict__ slow_list, int64_t n) {
  constexpr int S = D * D;     // sub-samples per pixel
  constexpr int G = 64 / S;    // pixels per wave
  const int lane = threadIdx.x & 63;
  const int grp = lane / S, sub = lane % S, sj = sub / D, si = sub % D;
  const int64_t nw = (int64_t)gridDim.x * (kThreads / 64);
  // wave-uniform trip count: the shuffles below always see all 64 lanes
  for (int64_t w = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); w * G < n;
       w += nw) {
    const int64_t k = w * G + grp;
    const bool valid = grp < G && k < n;
    T val = (T)0;
    int64_t didx = 0;
    if (valid) {
      const int64_t idx = slow_list[k];
      const int64_t oi = idx % a.out_w, rest = idx / a.out_w;
      const int64_t oj = rest % a.out_h, t = rest / a.out_h;
      const int64_t t1 = (ORDER == 1 && a.t_next) ? a.t_next[t] : -1;
      Src<T> p;
      p.g0 = static_cast<const T*>(a.src) + t * a.src_st;
      p.g1 = t1 >= 0 ? static_cast<const T*>(a.src) + t1 * a.src_st : p.g0;
      p.sy = a.src_sy;
      const AxisTab ey = ytab[oj * D + sj], ex = xtab[oi * D + si];
      Taps<T> tp;
      if (ORDER == 1 && t1 >= 0) {
        tp.template load<ORDER, true>(p, ey, ex);
        val = tp.template eval<T, ORDER, false, true>(ey, ex, a.cval);
      } else {
        tp.template load<ORDER, false>(p, ey, ex);
        val = tp.template eval<T, ORDER, false, false>(ey, ex, a.cval);
      }
      didx = t * a.dst_st + oj * a.dst_sy + oi;
    }
    T vals[S];
#pragma unroll
    for (int i = 0; i < S; ++i) vals[i] = __shfl(val, (grp < G ? grp : 0) * S + i, 64);
    if (valid && sub == 0) {
      Fold<T> fold;
#pragma unroll
      for (int r = 0; r < D; ++r) fold.add_row(a.agg, D, [&](int c) { return vals[r * D + c]; });
      fold.store(a, didx);
    }
  }
}

// The launch after K3i: its slow pixels when K3i worked and its list fit,
// else (a grid off the integral layout, or an overflowing list) the generic
// K3 over the whole launch — one launch either way.
template <typename T, int ORDER, int D>
__global__ void __launch_bounds__(kThreads)
integral_finish_kernel(AffineArgs a, const AxisTab* __restrict__ ytab,
                       const AxisTab* __restrict__ xtab, int group,
                       const int32_t* __restrict__ counters,
                       const int64_t* __restrict__ slow_list, int64_t slow_cap) {
  const int64_t n = counters[2];
  if (n < slow_cap) slow_body<T, ORDER, D>(a, ytab, xtab, slow_list, n);
  else reduce_body<T, T, ORDER, false>(a, ytab, xtab, group);
}

constexpr int kReduceLdsBudget = 32 * 1024;   // intermediate band

// LDS bytes of one intermediate row of a reduce tile
inline int64_t reduce_row_bytes(int64_t dx, int64_t isize) {
  const int64_t band_w = kTileW * dx;
  return (band_w + (band_w - 1) / 32) * isize;
}

// K3i candidates: square 2/4/8 coarsen factors of float rasters.  Whether the
// tables really are integral is known on the device only (affine_tables_kernel
// writes the run records), so K3i and its finish are launched; the finish runs
// the slow pixels K3i listed, or the generic K3 over the whole launch when the
// list overflowed (a grid off the integral layout: every wave of K3i returns
// at the first item in which it sees the list full, since the finish then
// overwrites everything K3i would store).
// xrs_testing_set(XRS_TESTING_AFFINE_GENERIC, 1) forces the generic K3 (tests).
template <typename T, typename I, bool RECOVER>
inline bool integral_candidate(const AffineArgs& a) {
  if (!std::is_floating_point<T>::value || !std::is_same<T, I>::value || RECOVER) return false;
  if (a.dx != a.dy || (a.dx != 2 && a.dx != 4 && a.dx != 8)) return false;
  if (sizeof(T) == 8 && a.dx == 8) return false;   // 9 rows of 8 doubles: too many registers
  return xrs_testing_value(XRS_TESTING_AFFINE_GENERIC) == 0;
}

// Slow pixels K3i lists (each takes the exact path): the image edges plus a
// little; a grid off the integral layout makes nearly every pixel slow and
// overflows the list, which hands the launch to the generic K3.
inline int64_t slow_capacity(int64_t ih, int64_t iw) { return 4 * (ih + iw) + 1024; }

template <typename T, typename I, int ORDER, bool RECOVER>
int launch(const AffineArgs& a, const AxisChunks& ay, const AxisChunks& ax, AxisTab* ytab,
           AxisTab* xtab, int32_t* nonint, bool run_weights, hipStream_t st) {
  const bool direct = a.agg == AGG_NONE || a.agg == AGG_FIRST || a.agg == AGG_LAST ||
                      a.agg == AGG_CENTER;
  // K3i / K3w need scale 1 at the div-x grid (div = ceil(scale) >= scale, so
  // it is an integer only at 1); any other grid goes straight to the generic
  // K3 — K3i would only overflow its slow list, and its appends to the one
  // counter serialised: 3.93 of 5.04 ms for a 3.5x downscale of 16384^2
  // (profiles/r06e_*, r06f_*)
  const bool k3i = !direct && integral_candidate<T, I, RECOVER>(a) && ay.scale == 1.0 &&
                   ax.scale == 1.0;
  // K3w: the caller's hint that the runs are contiguous but not integral
  // (scale 1, offsets off the integral layout); only the speed depends on it
  const bool k3w = k3i && ORDER == 1 && run_weights;
  // counters (set by the tables kernel, no memset): nonint[1] a time neighbour
  // other than the slice, nonint[2] K3i's slow-pixel count (list of slow_cap
  // entries after them); one slice: its only possible neighbour is itself ->
  // the TWO=false instance
  const bool t1_flag = k3i && ORDER == 1 && a.t_next != nullptr && a.nt > 1;
  int64_t* slow_list = reinterpret_cast<int64_t*>(nonint + 4);
  const int64_t slow_cap = slow_capacity(ay.n, ax.n);
  AffineArgs args = a;
  args.ytab = ytab;
  args.xtab = xtab;
  if (direct) {   // one launch: the kernel evaluates its two table entries inline
    const int64_t bands = (a.out_h + kTileH * kDirectRows - 1) / (kTileH * kDirectRows);
    const int64_t ntx = (a.out_w + kTileW - 1) / kTileW;
    constexpr int S = ORDER == 0 ? kDirectSlices0 : kDirectSlices1;
    if ((ORDER == 0 || a.t_next == nullptr) && a.nt >= S) {
      // slices share the geometry: grouped items, one item per block
      const int nb = grid_blocks(ntx * bands * ((a.nt + S - 1) / S), 1, 1 << 24);
      hipLaunchKernelGGL((affine_direct_group_kernel<T, I, ORDER, RECOVER, S>), dim3(nb),
                         dim3(kThreads), 0, st, args, ay, ax);
    } else {   // fewer slices than a group (config 1: one chunk, 7.2 us against
               // 7.7 us grouped with S = 1), or order 1 with the zero-weight
               // time neighbour: per slice
      const int nb = grid_blocks(ntx * bands * a.nt, 1, 256 * 64);
      hipLaunchKernelGGL((affine_direct_kernel<T, I, ORDER, RECOVER>), dim3(nb), dim3(kThreads),
                         0, st, args, ay, ax);
    }
    XRS_HIP_CHECK(hipGetLastError());
    return XRS_OK;
  }
  const int nbt = grid_blocks(ay.n + ax.n, kThreads, 1024);
  // K3i's run records (one int32 per output row / column) after the slow list
  int32_t* yrun = reinterpret_cast<int32_t*>(slow_list + slow_cap);
  int32_t* xrun = yrun + a.out_h;
  // run records by a wave ballot when every run sits inside one wave
  const bool wave_runs = k3i && a.dy > 0 && a.dx > 0 && 64 % a.dy == 0 && 64 % a.dx == 0 &&
                         ay.n % a.dy == 0 && ay.n % a.dx == 0 && ax.n % a.dx == 0;
  hipLaunchKernelGGL((affine_tables_kernel<ORDER>), dim3(nbt), dim3(kThreads), 0, st, ay, ax,
                     ytab, xtab, a.dy, a.dx, k3i ? nonint : nullptr, a.t_next, a.nt,
                     t1_flag, yrun, xrun, wave_runs, k3w);
  XRS_HIP_CHECK(hipGetLastError());
  if (k3i) {
    const int64_t ntiles = ((a.out_w + kThreads - 1) / kThreads) *
                           ((a.out_h + int_rows(a.dx, sizeof(T)) - 1) /
                            int_rows(a.dx, sizeof(T))) * a.nt;
    // one item per block (a persistent grid of 8 blocks per CU measured
    // 266 vs 238 us at config 3)
    const int nb = grid_blocks(ntiles, 1, 1 << 24);
    if constexpr (std::is_floating_point<T>::value && std::is_same<T, I>::value && !RECOVER) {
#define XRS_K3I(D, TWO, SELF)                                                             \
  do {                                                                                    \
    if (k3w)                                                                              \
      hipLaunchKernelGGL((affine_reduce_integral_kernel<T, ORDER, D, TWO, true>), dim3(nb), \
                         dim3(kThreads), 0, st, args, yrun, xrun, SELF, nonint + 2,      \
                         slow_list, slow_cap);                                           \
    else                                                                                  \
      hipLaunchKernelGGL((affine_reduce_integral_kernel<T, ORDER, D, TWO>), dim3(nb),     \
                         dim3(kThreads), 0, st, args, yrun, xrun, SELF, nonint + 2,      \
                         slow_list, slow_cap);                                           \
  } while (0)
      // with time neighbours both instances launch; nonint[1] picks one
      constexpr bool O1 = ORDER == 1;
      int32_t* self = t1_flag ? nonint + 1 : nullptr;
      if (a.dx == 2) { XRS_K3I(2, false, self); if (t1_flag) XRS_K3I(2, O1, self); }
      else if (a.dx == 4) { XRS_K3I(4, false, self); if (t1_flag) XRS_K3I(4, O1, self); }
      else if constexpr (sizeof(T) == 4) {
        XRS_K3I(8, false, self);
        if (t1_flag) XRS_K3I(8, O1, self);
      }
#undef XRS_K3I
    }
    XRS_HIP_CHECK(hipGetLastError());
  }
  const int64_t row_bytes = reduce_row_bytes(a.dx, sizeof(I));
  int64_t group = kReduceLdsBudget / (kRedRows * row_bytes);
  if (group < 1) group = 1;
  if (group > a.dy) group = a.dy;
  const int64_t band = group * kRedRows * row_bytes;
  if (band > 64 * 1024) {
    xrs_set_error("xrs_affine: coarsen factor too large for one LDS band");
    return XRS_ERR_ARG;
  }
  const int64_t nty = (a.out_h + kRedRows - 1) / kRedRows;
  const int64_t ntx = (a.out_w + kTileW - 1) / kTileW;
  const int64_t ntiles = ntx * nty * a.nt;
  const int nb = grid_blocks(ntiles, 1, 256 * 16);
  bool launched = false;
  if (k3i) {   // K3i's slow pixels, or the generic K3 when K3i did not work
    if constexpr (std::is_floating_point<T>::value && std::is_same<T, I>::value && !RECOVER) {
#define XRS_K3F(D)                                                                           \
  do {                                                                                       \
    hipLaunchKernelGGL((integral_finish_kernel<T, ORDER, D>), dim3(nb), dim3(kThreads),      \
                       (size_t)band, st, args, ytab, xtab, (int)group, nonint, slow_list,    \
                       slow_cap);                                                            \
    launched = true;                                                                         \
  } while (0)
      if (a.dx == 2) XRS_K3F(2);
      else if (a.dx == 4) XRS_K3F(4);
      else if constexpr (sizeof(T) == 4) { if (a.dx == 8) XRS_K3F(8); }
#undef XRS_K3F
    }
  }
  if (!launched)
    hipLaunchKernelGGL((affine_reduce_kernel<T, I, ORDER, RECOVER>), dim3(nb), dim3(kThreads),
                       (size_t)band, st, args, ytab, xtab, (int)group);
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
  // axis tables + the K3i flags (broken entries, time neighbour, slow count),
  // slow-pixel list
  // and K3i's run records (out_h + out_w <= inter_h + inter_w int32)
  return (inter_h + inter_w) * (int64_t)sizeof(xrs::AxisTab) + 16 +
         xrs::slow_capacity(inter_h, inter_w) * (int64_t)sizeof(int64_t) +
         (inter_h + inter_w) * (int64_t)sizeof(int32_t);
}

extern "C" int xrs_affine(const void* src, int src_dtype, int64_t nt, int64_t src_h,
                          int64_t src_w, int64_t src_st, int64_t src_sy, void* dst,
                          int dst_dtype, int64_t out_h, int64_t out_w, int64_t dst_st,
                          int64_t dst_sy, int64_t div_y, int64_t div_x, int agg, int order,
                          double scale_y, double scale_x, int64_t chunk_y,
                          const int64_t* rel_y, const int64_t* len_y, const double* off_y,
                          int64_t chunk_x, const int64_t* rel_x, const int64_t* len_x,
                          const double* off_x, const int64_t* t_next, double cval,
                          int recover_nan, int run_weights, void* workspace,
                          int64_t workspace_bytes, void* stream) {
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
  int32_t* nonint = reinterpret_cast<int32_t*>(xtab + iw);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool rw = run_weights != 0;
  return dispatch_dtype(src_dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    if constexpr (std::is_floating_point<T>::value) {
      if (recover_nan)
        return order ? launch<T, double, 1, true>(a, ay, ax, ytab, xtab, nonint, rw, st)
                     : launch<T, double, 0, true>(a, ay, ax, ytab, xtab, nonint, rw, st);
    }
    return order ? launch<T, T, 1, false>(a, ay, ax, ytab, xtab, nonint, rw, st)
                 : launch<T, T, 0, false>(a, ay, ax, ytab, xtab, nonint, rw, st);
  });
}
