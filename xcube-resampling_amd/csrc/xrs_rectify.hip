// xrs_rectify.hip — K4/K5/K6: irregular (2-D coordinates) -> regular grid for gfx950.
//
// K4 ij_bboxes   replaces gridmapping/bboxes.py:28-106 (compute_ij_bboxes, a
//                numba prange over boxes scanning every source pixel).  Here
//                every source pixel is visited once: each lane finds the boxes
//                that contain its (x, y) (for a tile grid only the matching
//                tile columns x rows), and the wave merges equal boxes with a
//                ballot-driven loop (wave min of the next candidate box, DPP/
//                shuffle min/max reductions, one lane issues the atomics) —
//                4 atomics per (wave, box) instead of per pixel.
// K5 rectify_ij  replaces rectify.py:373-576 (_compute_target_source_ij_block
//                -> _sequential -> _line): for every target tile, the source
//                quads inside its source bbox rasterise into the tile.  The
//                reference keeps the FIRST quad in raster order that hits a
//                target pixel; that is the minimum raster key of all hitting
//                quads, so K5a claims pixels with atomicMin (order-independent)
//                and K5b recomputes the winning quad's barycentric (u, v) with
//                the identical float64 expressions (_fdet/_fu/_fv, 737-768).
// K6 rectify_var replaces rectify.py:605-734 (_compute_var_image_block): per
//                target pixel, source sub-pixel position -> nearest /
//                triangular / bilinear in float64, stored in the variable dtype.
//                Formulated on global indices; the reference's per-tile source
//                sub-window (622-630) shifts indices by an integer, which leaves
//                every index, fraction and clamp unchanged.

#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "xrs_common.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;
constexpr int kStripW = 63;   // K5a strip: quads per row (64 point columns = one wave)
constexpr int kStripH = 16;   // K5a strip: quad rows

// ---- wave-level helpers (64 lanes) ------------------------------------------
__device__ inline int32_t wave_min(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ inline int32_t wave_max(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- K4 ----------------------------------------------------------------------
struct BBoxArgs {
  const double* x;        // source x image (h, w), row stride sy
  const double* y;
  int64_t h, w, sy;
  int64_t nboxes;
  // grid mode (ntx*nty == nboxes): box k = ty*ntx + tx has x range of column
  // tx and y range of row ty; otherwise every box is tested (ntx == 0)
  int64_t ntx, nty;
  const double* bx;       // grid: (ntx, 2) [x_min, x_max] (border included); else (nboxes, 4)
  const double* by;       // grid: (nty, 2) [y_min, y_max]
  int32_t* acc;           // (nboxes, 4): min i, min j, max i, max j
  uint32_t* fill;         // NULL or 16-byte aligned: fill_words words set to ~0
  int64_t fill_words;     // (the claim-key scratch of the K5 that follows)
};

// The claim-key scratch filled by K4's own grid: K4 reads the coordinates at
// well under the HBM rate, so the writes ride along instead of taking a
// memset pass of their own between K4 and the claim.  Non-temporal 16-byte
// stores; the block kernel stores a block's share of the scratch with each
// source block, the per-pixel kernel fills first.  (A fill on a side stream,
// or of a thread's whole share before / after its blocks, measured slower:
// DESIGN.md §3, round 4 (5).)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ inline void fill_scratch(const BBoxArgs& a) {
  if (!a.fill) return;
  const u32x4 v = {~0u, ~0u, ~0u, ~0u};
  const int64_t nt = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n4 = a.fill_words >> 2;
  u32x4* f4 = reinterpret_cast<u32x4*>(a.fill);
  for (int64_t k = t; k < n4; k += nt) __builtin_nontemporal_store(v, f4 + k);
  for (int64_t k = (n4 << 2) + t; k < a.fill_words; k += nt) a.fill[k] = ~0u;
}

// share [blk * per, (blk + 1) * per) of the scratch's 16-byte words, one
// wave (lane = 0..63); the word tail (fill_words % 4) goes with block 0
__device__ inline void fill_scratch_block(const BBoxArgs& a, int64_t blk, int64_t per,
                                          int lane) {
  const u32x4 v = {~0u, ~0u, ~0u, ~0u};
  const int64_t n4 = a.fill_words >> 2;
  const int64_t e = min((blk + 1) * per, n4);
  u32x4* f4 = reinterpret_cast<u32x4*>(a.fill);
  for (int64_t k = blk * per + lane; k < e; k += 64) __builtin_nontemporal_store(v, f4 + k);
  if (blk == 0 && lane < (a.fill_words & 3)) a.fill[(n4 << 2) + lane] = ~0u;
}

// Next candidate box > `after` that contains (x, y), or INT32_MAX.
__device__ inline int32_t next_box(const BBoxArgs& a, const double* bx, double x, double y,
                                   int32_t tx0, int32_t tx1, int32_t ty0, int32_t ty1,
                                   int32_t after) {
  if (a.ntx > 0) {  // grid: candidates = rectangle [ty0,ty1] x [tx0,tx1], row-major
    if (tx0 > tx1 || ty0 > ty1) return INT32_MAX;
    int32_t ty = ty0, tx = tx0;
    if (after >= 0) {
      ty = after / (int32_t)a.ntx;
      tx = after - ty * (int32_t)a.ntx + 1;
      if (tx > tx1) { tx = tx0; ++ty; }
      if (ty < ty0) { ty = ty0; tx = tx0; }
    }
    return ty <= ty1 ? ty * (int32_t)a.ntx + tx : INT32_MAX;
  }
  for (int32_t k = after + 1; k < (int32_t)a.nboxes; ++k) {
    const double* b = bx + 4 * k;
    if (b[0] <= x && x <= b[2] && b[1] <= y && y <= b[3]) return k;
  }
  return INT32_MAX;
}

// Tile rows / columns whose closed interval [b[2t], b[2t+1]] contains v, for
// interval arrays monotone in t (dir > 0: both ends non-decreasing, dir < 0:
// non-increasing): a contiguous run [t0, t1] (NaN -> empty), same inclusive
// compares as the scan.  Both ends are found by walking from an estimate
// (tiles are evenly spaced, so it is usually exact and a walk is 1-2 LDS
// reads) instead of two binary searches (2 x log2(n) dependent reads); the
// walk ends at the exact boundary whatever the estimate.
struct Axis1 {
  double lo0, scale;   // estimate of t: (v - lo0) * scale
};
__device__ inline Axis1 axis_estimate(const double* b, int32_t n) {
  const double span = b[2 * (n - 1)] - b[0];
  return Axis1{b[0], n > 1 && span != 0.0 ? (double)(n - 1) / span : 0.0};
}
__device__ inline void monotone_hits(const double* b, int32_t n, double v, int dir,
                                     const Axis1& est, int32_t& t0, int32_t& t1) {
  if (v != v) { t0 = 1; t1 = 0; return; }
  const double ef = fmin(fmax((v - est.lo0) * est.scale, 0.0), (double)(n - 1));
  const int32_t e = ef == ef ? (int32_t)ef : 0;
  // t0: first t with P(t) = (dir > 0 ? b_hi >= v : b_lo <= v), P false..true in t
  auto p0 = [&](int32_t t) { return dir > 0 ? b[2 * t + 1] >= v : b[2 * t] <= v; };
  int32_t t = e;
  if (p0(t)) { while (t > 0 && p0(t - 1)) --t; }
  else { while (t < n && !p0(t)) ++t; }
  t0 = t;
  // t1 + 1: first t with !Q(t), Q(t) = (dir > 0 ? b_lo <= v : b_hi >= v), Q true..false
  auto q1 = [&](int32_t u) { return dir > 0 ? b[2 * u] <= v : b[2 * u + 1] >= v; };
  t = e;
  if (q1(t)) { while (t < n && q1(t)) ++t; }
  else { while (t > 0 && !q1(t - 1)) --t; }
  t1 = t - 1;
}

// +1 / -1 if both interval ends are monotone non-decreasing / non-increasing
// in t, else 0 (then the candidates are found by a full scan)
__device__ inline int interval_dir(const double* b, int32_t n) {
  bool inc = true, dec = true;
  for (int32_t t = 1; t < n; ++t) {
    inc = inc && b[2 * t] >= b[2 * t - 2] && b[2 * t + 1] >= b[2 * t - 1];
    dec = dec && b[2 * t] <= b[2 * t - 2] && b[2 * t + 1] <= b[2 * t - 1];
  }
  return inc ? 1 : (dec ? -1 : 0);
}

// Each block owns one contiguous run of source pixels (spatially coherent:
// few boxes per block).  SHARED: the box geometry and the per-box accumulators
// live in LDS — the wave merges go to LDS atomics and each block flushes one
// set of global atomics per box it touched (thousands of waves hammering the
// same few hundred global words serialised at the L2 atomic units).
template <bool SHARED>
__global__ void __launch_bounds__(kThreads)
ij_bboxes_kernel(BBoxArgs a, int64_t chunk) {
  extern __shared__ __align__(16) unsigned char smem[];
  fill_scratch(a);
  const int64_t nbx = a.ntx > 0 ? 2 * a.ntx : 4 * a.nboxes;   // doubles of bx
  const int64_t nby = a.ntx > 0 ? 2 * a.nty : 0;
  double* sbx = reinterpret_cast<double*>(smem);
  double* sby = sbx + nbx;
  int32_t* sacc = reinterpret_cast<int32_t*>(sby + nby);
  const double* bx = a.bx;
  const double* by = a.by;
  int32_t* acc = a.acc;
  if (SHARED) {
    for (int64_t i = threadIdx.x; i < nbx; i += kThreads) sbx[i] = a.bx[i];
    for (int64_t i = threadIdx.x; i < nby; i += kThreads) sby[i] = a.by[i];
    for (int64_t i = threadIdx.x; i < 4 * a.nboxes; i += kThreads)
      sacc[i] = (i & 3) < 2 ? INT32_MAX : -1;
    __syncthreads();
    bx = sbx;
    by = sby;
    acc = sacc;
  }
  const int64_t n = a.h * a.w;
  const int64_t p0 = (int64_t)blockIdx.x * chunk, p1 = min(n, p0 + chunk);
  const int xdir = a.ntx > 0 ? interval_dir(bx, (int32_t)a.ntx) : 0;
  const int ydir = a.ntx > 0 ? interval_dir(by, (int32_t)a.nty) : 0;
  const Axis1 xest = a.ntx > 0 ? axis_estimate(bx, (int32_t)a.ntx) : Axis1{0.0, 0.0};
  const Axis1 yest = a.ntx > 0 ? axis_estimate(by, (int32_t)a.nty) : Axis1{0.0, 0.0};
  // the next batch's coordinates are requested before this batch's search
  // and merges (one memory round trip hidden per iteration)
  double xn = NAN, yn = NAN;
  // pixel index -> (row, column) in 32-bit arithmetic (h * w <= INT32_MAX,
  // checked by the launcher; a 64-bit division is a long VALU sequence)
  const uint32_t w32 = (uint32_t)a.w;
  if (p0 + threadIdx.x < p1) {
    const uint32_t idx = (uint32_t)(p0 + threadIdx.x);
    const uint32_t j = idx / w32;
    xn = a.x[(int64_t)j * a.sy + (idx - j * w32)];
    yn = a.y[(int64_t)j * a.sy + (idx - j * w32)];
  }
  // the lane's pixel as (row, column), stepped by kThreads pixels per
  // iteration without a division (i < w kept by subtracting whole rows)
  int32_t ci = 0, cj = 0;
  {
    const uint32_t idx = (uint32_t)min(p0 + (int64_t)threadIdx.x, n - 1);
    cj = (int32_t)(idx / w32);
    ci = (int32_t)(idx - (uint32_t)cj * w32);
  }
  auto step = [&](int32_t& i, int32_t& j) {
    i += kThreads;
    while (i >= (int32_t)w32) { i -= (int32_t)w32; ++j; }
  };
  // Wave accumulator (grid mode): the box every contributing lane of the
  // wave's recent iterations fell in, and its extremes so far — flushed to
  // the block's accumulators only when the wave meets another box (lanes
  // cross a tile every few hundred pixels) instead of four atomics per
  // iteration.  Wave-uniform values (scalar registers).
  int32_t wk = -1, wimin = INT32_MAX, wjmin = INT32_MAX, wimax = -1, wjmax = -1;
  auto wflush = [&]() {
    if (wk >= 0 && (threadIdx.x & 63) == 0) {
      atomicMin(&acc[4 * wk + 0], wimin);
      atomicMin(&acc[4 * wk + 1], wjmin);
      atomicMax(&acc[4 * wk + 2], wimax);
      atomicMax(&acc[4 * wk + 3], wjmax);
    }
    wk = -1;
  };
  // every lane of a wave iterates the same number of times (wave-uniform trip
  // count), so the wave-wide shuffles below always see all 64 lanes
  for (int64_t base = p0; base < p1; base += kThreads) {
    const int64_t idx = base + threadIdx.x;
    const bool valid = idx < p1;
    const double x = xn, y = yn;
    const int32_t i0 = valid ? ci : 0, j0 = valid ? cj : 0;
    step(ci, cj);
    if (idx + kThreads < p1) {
      const int64_t o = (int64_t)cj * a.sy + ci;
      xn = a.x[o];
      yn = a.y[o];
    }
    int32_t tx0 = 1, tx1 = 0, ty0 = 1, ty1 = 0;
    if (valid && a.ntx > 0) {  // x_min <= x <= x_max, y_min <= y <= y_max (bboxes.py:60-69)
      if (xdir != 0) {
        monotone_hits(bx, (int32_t)a.ntx, x, xdir, xest, tx0, tx1);
      } else {
        for (int32_t t = 0; t < (int32_t)a.ntx; ++t)
          if (bx[2 * t] <= x && x <= bx[2 * t + 1]) { if (tx0 > tx1) tx0 = t; tx1 = t; }
      }
      if (ydir != 0) {
        monotone_hits(by, (int32_t)a.nty, y, ydir, yest, ty0, ty1);
      } else {
        for (int32_t t = 0; t < (int32_t)a.nty; ++t)
          if (by[2 * t] <= y && y <= by[2 * t + 1]) { if (ty0 > ty1) ty0 = t; ty1 = t; }
      }
    }
    if (a.ntx > 0) {
      // one box per pixel for every lane that has one, the same box: the
      // wave accumulator takes the iteration (lanes are consecutive pixels:
      // when the first and the last contributing lane share a row, the
      // extremes are theirs)
      const bool any_box = valid && tx0 <= tx1 && ty0 <= ty1;
      const bool single = any_box && tx0 == tx1 && ty0 == ty1;
      const int32_t kl = single ? ty0 * (int32_t)a.ntx + tx0 : (any_box ? -2 : INT32_MAX);
      const uint64_t has = __ballot(kl != INT32_MAX);
      if (has == 0) continue;
      const int fl = __builtin_ctzll(has), ll = 63 - __builtin_clzll(has);
      const int32_t k0 = __builtin_amdgcn_readlane(kl, fl);
      if (k0 >= 0 && __all(kl == k0 || kl == INT32_MAX)) {
        int32_t imin, jmin, imax, jmax;
        const int32_t jf = __builtin_amdgcn_readlane(j0, fl);
        if (__builtin_amdgcn_readlane(j0, ll) == jf) {
          imin = __builtin_amdgcn_readlane(i0, fl);
          imax = __builtin_amdgcn_readlane(i0, ll);
          jmin = jmax = jf;
        } else {
          const bool mine = kl == k0;
          imin = wave_min(mine ? i0 : INT32_MAX);
          jmin = wave_min(mine ? j0 : INT32_MAX);
          imax = wave_max(mine ? i0 : -1);
          jmax = wave_max(mine ? j0 : -1);
        }
        if (k0 != wk) {
          wflush();
          wk = k0;
          wimin = imin; wjmin = jmin; wimax = imax; wjmax = jmax;
        } else {
          wimin = min(wimin, imin); wjmin = min(wjmin, jmin);
          wimax = max(wimax, imax); wjmax = max(wjmax, jmax);
        }
        continue;
      }
    }
    int32_t cur = valid ? next_box(a, bx, x, y, tx0, tx1, ty0, ty1, -1) : INT32_MAX;
    while (true) {
      // next box any lane of the wave contributes to; usually every lane's
      const int32_t c0 = __builtin_amdgcn_readfirstlane(cur);
      const bool uni = __all(cur == c0);
      const int32_t k = uni ? c0 : wave_min(cur);
      if (k == INT32_MAX) break;
      const bool mine = cur == k;
      int32_t imin, jmin, imax, jmax;
      // lanes hold consecutive pixels: when the first and the last lane
      // contributing to box k sit in one source row, every contributing lane
      // does, and the extremes are those two lanes' (scalar reads, no
      // cross-lane reductions)
      const uint64_t mm = __ballot(mine);
      const int fl = __builtin_ctzll(mm), ll = 63 - __builtin_clzll(mm);
      const int32_t jf = __builtin_amdgcn_readlane(j0, fl);
      if (__builtin_amdgcn_readlane(j0, ll) == jf) {
        imin = __builtin_amdgcn_readlane(i0, fl);
        imax = __builtin_amdgcn_readlane(i0, ll);
        jmin = jmax = jf;
      } else {
        imin = wave_min(mine ? i0 : INT32_MAX);
        jmin = wave_min(mine ? j0 : INT32_MAX);
        imax = wave_max(mine ? i0 : -1);
        jmax = wave_max(mine ? j0 : -1);
      }
      if ((threadIdx.x & 63) == 0) {
        atomicMin(&acc[4 * k + 0], imin);
        atomicMin(&acc[4 * k + 1], jmin);
        atomicMax(&acc[4 * k + 2], imax);
        atomicMax(&acc[4 * k + 3], jmax);
      }
      if (mine) cur = next_box(a, bx, x, y, tx0, tx1, ty0, ty1, k);
    }
  }
  wflush();
  if (SHARED) {
    __syncthreads();
    for (int64_t k = threadIdx.x; k < a.nboxes; k += kThreads) {
      if (sacc[4 * k + 2] < 0) continue;  // box not touched by this block
      atomicMin(&a.acc[4 * k + 0], sacc[4 * k + 0]);
      atomicMin(&a.acc[4 * k + 1], sacc[4 * k + 1]);
      atomicMax(&a.acc[4 * k + 2], sacc[4 * k + 2]);
      atomicMax(&a.acc[4 * k + 3], sacc[4 * k + 3]);
    }
  }
}

// K4 in grid mode, block-wise.  A wave takes a block of kBoxBlockRows source
// rows x 64 columns (lane l: column l, one pixel per row).  The wave's bbox of
// the coordinates (NaN skipped) selects the candidate tiles; for each one:
//  * every pixel of the block valid (no NaN coordinate) and the block's bbox
//    inside the tile's box: every pixel passes the reference's test
//    (x_min <= x <= x_max, y_min <= y <= y_max, bboxes.py:60-69), so the
//    block's whole index range is the tile's contribution;
//  * otherwise the reference's test per pixel, and the extremes from ballots:
//    the first / last lane with a pixel inside give i, the first / last row
//    with one give j (no cross-lane reductions).
// The extremes equal the per-pixel scan's.  Most blocks lie inside one tile;
// the per-pixel path is taken near tile edges (the boxes overlap by the
// border), so a pixel costs a few instructions instead of a tile search and a
// wave merge.  Boxes whose intervals are not monotone (never for a tile grid)
// make every tile a candidate: slow, same result.  16 rows measured best at
// config 4 (K4 124 -> 92 us against 4 rows; 2 / 8 rows slower or equal,
// profiles/r04_rectify_k4_rows_ab.log).
constexpr int kBoxBlockRows = 16;

// Wave min / max of a double (NaN ignored unless every lane's is NaN, as
// fmin / fmax), wave-uniform result.  DPP steps, no LDS round trip: each quad,
// then each half-row and row of 16 lanes (quad_perm, row_half_mirror,
// row_mirror), then rows 0+1 / 2+3 (row_bcast:15) and all four (row_bcast:31)
// into lane 63.  Lanes a step does not write keep their value (min(v, v)).
// (A butterfly of __shfl_xor — 12 dependent ds_bpermute round trips per
// value — made the four block extremes the longest chain of K4's block.)
template <int CTRL, int ROWS>
__device__ inline double dpp_keep_f64(double v) {
  const uint64_t b = __double_as_longlong(v);
  const int lo = (int)(uint32_t)b, hi = (int)(uint32_t)(b >> 32);
  const uint32_t l = (uint32_t)__builtin_amdgcn_update_dpp(lo, lo, CTRL, ROWS, 0xF, false);
  const uint32_t h = (uint32_t)__builtin_amdgcn_update_dpp(hi, hi, CTRL, ROWS, 0xF, false);
  return __longlong_as_double((int64_t)(((uint64_t)h << 32) | l));
}
template <bool MAX>
__device__ inline double wave_ext_f64(double v) {
  auto op = [](double x, double y) { return MAX ? fmax(x, y) : fmin(x, y); };
  v = op(v, dpp_keep_f64<0xB1, 0xF>(v));    // quad_perm [1, 0, 3, 2]
  v = op(v, dpp_keep_f64<0x4E, 0xF>(v));    // quad_perm [2, 3, 0, 1]
  v = op(v, dpp_keep_f64<0x141, 0xF>(v));   // row_half_mirror
  v = op(v, dpp_keep_f64<0x140, 0xF>(v));   // row_mirror
  v = op(v, dpp_keep_f64<0x142, 0xA>(v));   // row_bcast:15 -> rows 1, 3
  v = op(v, dpp_keep_f64<0x143, 0xC>(v));   // row_bcast:31 -> rows 2, 3
  const uint64_t b = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63);
  return __longlong_as_double((int64_t)(((uint64_t)hi << 32) | lo));
}
__device__ inline double wave_fmin_f64(double v) { return wave_ext_f64<false>(v); }
__device__ inline double wave_fmax_f64(double v) { return wave_ext_f64<true>(v); }

template <bool SHARED>
__global__ void __launch_bounds__(kThreads)
ij_bboxes_block_kernel(BBoxArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t nbx = 2 * a.ntx, nby = 2 * a.nty;
  double* sbx = reinterpret_cast<double*>(smem);
  double* sby = sbx + nbx;
  int32_t* sacc = reinterpret_cast<int32_t*>(sby + nby);
  const double* bx = a.bx;
  const double* by = a.by;
  int32_t* acc = a.acc;
  if (SHARED) {
    for (int64_t i = threadIdx.x; i < nbx; i += kThreads) sbx[i] = a.bx[i];
    for (int64_t i = threadIdx.x; i < nby; i += kThreads) sby[i] = a.by[i];
    for (int64_t i = threadIdx.x; i < 4 * a.nboxes; i += kThreads)
      sacc[i] = (i & 3) < 2 ? INT32_MAX : -1;
    __syncthreads();
    bx = sbx;
    by = sby;
    acc = sacc;
  }
  const int32_t ntx = (int32_t)a.ntx, nty = (int32_t)a.nty;
  const int xdir = interval_dir(bx, ntx), ydir = interval_dir(by, nty);
  const Axis1 xest = axis_estimate(bx, ntx), yest = axis_estimate(by, nty);
  const int lane = threadIdx.x & 63;
  const int64_t ncb = (a.w + 63) / 64, nrb = (a.h + kBoxBlockRows - 1) / kBoxBlockRows;
  const int64_t nblk = ncb * nrb;
  const int64_t nwaves = (int64_t)gridDim.x * (kThreads / 64);
  const int64_t fill_per = ((a.fill_words >> 2) + nblk - 1) / nblk;
  for (int64_t blk = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); blk < nblk;
       blk += nwaves) {   // wave-uniform
    const int64_t rb = blk / ncb, cb = blk - rb * ncb;
    const int32_t i0 = (int32_t)(cb * 64), j0 = (int32_t)(rb * kBoxBlockRows);
    const int32_t i = i0 + lane;
    const bool col_ok = i < a.w;
    const int nrows = (int)min((int64_t)kBoxBlockRows, a.h - j0);
    double x[kBoxBlockRows], y[kBoxBlockRows];
#pragma unroll
    for (int r = 0; r < kBoxBlockRows; ++r) {
      x[r] = y[r] = NAN;
      if (col_ok && r < nrows) {
        const int64_t o = (int64_t)(j0 + r) * a.sy + i;
        x[r] = a.x[o];
        y[r] = a.y[o];
      }
    }
    if (a.fill) fill_scratch_block(a, blk, fill_per, lane);
    double xmn = x[0], xmx = x[0], ymn = y[0], ymx = y[0];
    bool nan = col_ok && (x[0] != x[0] || y[0] != y[0]);
#pragma unroll
    for (int r = 1; r < kBoxBlockRows; ++r) {
      xmn = fmin(xmn, x[r]); xmx = fmax(xmx, x[r]);
      ymn = fmin(ymn, y[r]); ymx = fmax(ymx, y[r]);
      nan = nan || (col_ok && r < nrows && (x[r] != x[r] || y[r] != y[r]));
    }
    xmn = wave_fmin_f64(xmn); xmx = wave_fmax_f64(xmx);
    ymn = wave_fmin_f64(ymn); ymx = wave_fmax_f64(ymx);
    if (xmn != xmn || ymn != ymn) continue;   // no finite pixel (wave-uniform)
    const bool all_valid = __ballot(nan) == 0;
    // candidate tiles: intervals intersecting [xmn, xmx] x [ymn, ymx]
    int32_t tx0 = 0, tx1 = ntx - 1, ty0 = 0, ty1 = nty - 1, d0, d1;
    if (xdir > 0) { monotone_hits(bx, ntx, xmn, xdir, xest, tx0, d1); monotone_hits(bx, ntx, xmx, xdir, xest, d0, tx1); }
    if (xdir < 0) { monotone_hits(bx, ntx, xmx, xdir, xest, tx0, d1); monotone_hits(bx, ntx, xmn, xdir, xest, d0, tx1); }
    if (ydir > 0) { monotone_hits(by, nty, ymn, ydir, yest, ty0, d1); monotone_hits(by, nty, ymx, ydir, yest, d0, ty1); }
    if (ydir < 0) { monotone_hits(by, nty, ymx, ydir, yest, ty0, d1); monotone_hits(by, nty, ymn, ydir, yest, d0, ty1); }
    tx0 = __builtin_amdgcn_readfirstlane(tx0); tx1 = __builtin_amdgcn_readfirstlane(tx1);
    ty0 = __builtin_amdgcn_readfirstlane(ty0); ty1 = __builtin_amdgcn_readfirstlane(ty1);
    const int32_t ilast = (int32_t)min((int64_t)i0 + 63, a.w - 1);
    for (int32_t ty = ty0; ty <= ty1; ++ty) {
      const double ylo = by[2 * ty], yhi = by[2 * ty + 1];
      for (int32_t tx = tx0; tx <= tx1; ++tx) {
        const double xlo = bx[2 * tx], xhi = bx[2 * tx + 1];
        const int32_t k = ty * ntx + tx;
        int32_t imin, jmin, imax, jmax;
        if (all_valid && xlo <= xmn && xmx <= xhi && ylo <= ymn && ymx <= yhi) {
          imin = i0; imax = ilast; jmin = j0; jmax = j0 + nrows - 1;
        } else {
          bool any = false;
          int32_t rmask = 0;
#pragma unroll
          for (int r = 0; r < kBoxBlockRows; ++r) {
            const bool in = xlo <= x[r] && x[r] <= xhi && ylo <= y[r] && y[r] <= yhi;
            any = any || in;
            rmask |= __ballot(in) != 0 ? (1 << r) : 0;
          }
          const uint64_t lanes = __ballot(any);
          if (lanes == 0) continue;   // wave-uniform
          imin = i0 + __builtin_ctzll(lanes);
          imax = i0 + 63 - __builtin_clzll(lanes);
          jmin = j0 + __builtin_ctz(rmask);
          jmax = j0 + 31 - __builtin_clz(rmask);
        }
        if (lane == 0) {
          atomicMin(&acc[4 * k + 0], imin);
          atomicMin(&acc[4 * k + 1], jmin);
          atomicMax(&acc[4 * k + 2], imax);
          atomicMax(&acc[4 * k + 3], jmax);
        }
      }
    }
  }
  if (SHARED) {
    __syncthreads();
    for (int64_t k = threadIdx.x; k < a.nboxes; k += kThreads) {
      if (sacc[4 * k + 2] < 0) continue;  // box not touched by this block
      atomicMin(&a.acc[4 * k + 0], sacc[4 * k + 0]);
      atomicMin(&a.acc[4 * k + 1], sacc[4 * k + 1]);
      atomicMax(&a.acc[4 * k + 2], sacc[4 * k + 2]);
      atomicMax(&a.acc[4 * k + 3], sacc[4 * k + 3]);
    }
  }
}

// ---- rectify geometry (rectify.py:737-773) -----------------------------------
__device__ inline double fdet(double px0, double py0, double px1, double py1, double px2,
                              double py2) {
  return (px0 - px1) * (py0 - py2) - (px0 - px2) * (py0 - py1);
}
__device__ inline double fu(double px, double py, double px0, double py0, double px2,
                            double py2) {
  return (px0 - px) * (py0 - py2) - (py0 - py) * (px0 - px2);
}
__device__ inline double fv(double px, double py, double px0, double py0, double px1,
                            double py1) {
  return (py0 - py) * (px0 - px1) - (px0 - px) * (py0 - py1);
}
__device__ inline double fclamp(double x, double lo, double hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

struct TileInfo {      // one target tile (host-computed, rectify.py:391-418)
  int32_t r0, c0;      // first target row / column of the tile
  int32_t th, tw;      // tile height / width (edge tiles are short)
  int32_t si0, sj0;    // src_i_min, src_j_min (-1: no source)
  int32_t swin, shin;  // source window width / height (i_max+1-i_min clipped)
  double x_off, y_off; // dst_x_offset, dst_y_offset
};

struct RectArgs {
  const double* x;     // source coordinates (h, w) in the target CRS
  const double* y;
  int64_t h, w, sy;
  const TileInfo* tiles;
  int64_t ntiles;
  const int64_t* chunk_offs;   // (ntiles + 1): first quad strip of each tile
  int64_t dst_h, dst_w;
  double x_scale, y_scale;     // dst_x_res, dst_y_res (negated when j-axis down)
  double uv_delta;
  double inv_x, inv_y;         // 1 / x_scale, 1 / y_scale (claim fast paths)
  double margin;               // window floors: relative margin (inf: always exact)
  float margin_scale;          // form margin factor (tests: >1 widens the exact-test band)
  int narrow;                  // dst_h * dst_w < 2^30, dst_w < 2^24: claims use 32-bit byte
                               // offsets and 24-bit multiplies
  int key_shift;               // > 0: raster key = (qj << key_shift) | qi (lexicographic
                               // order = raster order; decoded by a shift and a mask);
                               // 0: qj * w + qi (decoded by a division)
  uint32_t key_mul;            // 1 << key_shift, or w
  int tri_bit;                 // h * w < 2^31: a claim key is (raster key << 1) | (the
                               // reference's triangle is B), so K5b evaluates one triangle
  uint32_t* keys;              // (dst_h, dst_w) claim keys, 0xFFFFFFFF = free
  double* ij;                  // (2, dst_h, dst_w) output
  int32_t* err_flags;          // XRS_EFLAG_STATE: an inconsistent record / key was skipped
};

// A tile record the claim and resolve passes can address without leaving the
// target, source or key rasters (records come from xrs_rectify_tiles or the
// host; anything else is skipped and reported, never dereferenced).
__device__ inline bool tile_ok(const RectArgs& a, const TileInfo& ti) {
  return ti.r0 >= 0 && ti.c0 >= 0 && ti.th >= 1 && ti.tw >= 1 &&
         (int64_t)ti.r0 + ti.th <= a.dst_h && (int64_t)ti.c0 + ti.tw <= a.dst_w &&
         (ti.si0 < 0 || (ti.sj0 >= 0 && ti.swin >= 0 && ti.shin >= 0 &&
                         (int64_t)ti.si0 + ti.swin <= a.w && (int64_t)ti.sj0 + ti.shin <= a.h));
}

struct Quad {          // corners p0 (qj, qi), p1 (qj, qi+1), p2 (qj+1, qi), p3 (qj+1, qi+1)
  double x0, y0, x1, y1, x2, y2, x3, y3;
};

__device__ inline Quad load_quad(const RectArgs& a, int64_t qj, int64_t qi) {
  const int64_t r0 = qj * a.sy, r1 = (qj + 1) * a.sy;
  return Quad{a.x[r0 + qi], a.y[r0 + qi], a.x[r0 + qi + 1], a.y[r0 + qi + 1],
              a.x[r1 + qi], a.y[r1 + qi], a.x[r1 + qi + 1], a.y[r1 + qi + 1]};
}

// Test triangle A then B of quad q for the target pixel centre (dx, dy)
// (rectify.py:556-573).  Returns 0 (no hit), 1 (triangle A: src = p0 +
// clamp(u, v)) or 2 (triangle B: src = p3 - clamp(u, v)); cu, cv receive the
// clamped barycentric coordinates.
__device__ inline int quad_hit(const RectArgs& a, const Quad& q, double dx, double dy,
                               double det_a, double det_b, double& cu, double& cv) {
  const double umin = -a.uv_delta, vmin = -a.uv_delta, uvmax = 1.0 + 2 * a.uv_delta;
  if (det_a != 0.0) {
    const double u = fu(dx, dy, q.x0, q.y0, q.x2, q.y2) / det_a;
    const double v = fv(dx, dy, q.x0, q.y0, q.x1, q.y1) / det_a;
    if (u >= umin && v >= vmin && u + v <= uvmax) {
      cu = fclamp(u, 0.0, 1.0);
      cv = fclamp(v, 0.0, 1.0);
      return 1;
    }
  }
  if (det_b != 0.0) {
    const double u = fu(dx, dy, q.x3, q.y3, q.x1, q.y1) / det_b;
    const double v = fv(dx, dy, q.x3, q.y3, q.x2, q.y2) / det_b;
    if (u >= umin && v >= vmin && u + v <= uvmax) {
      cu = fclamp(u, 0.0, 1.0);
      cv = fclamp(v, 0.0, 1.0);
      return 2;
    }
  }
  return 0;
}

// The clamped (u, v) of ONE triangle (A = (p0; p2, p1), B = (p3; p1, p2)) at
// pixel centre (dx, dy), with the reference's expressions and divisions
// (rectify.py:556-573, 737-768): origin O, fu's edge corner U, fv's corner V
// = (p0, p2, p1) or (p3, p1, p2); det = _fdet(O, V, U).  The claim picked the
// triangle (claim keys carry it), so the triangle hits here.
__device__ inline void tri_uv(const Quad& q, bool b, double dx, double dy, double& cu,
                              double& cv) {
  const double ox = b ? q.x3 : q.x0, oy = b ? q.y3 : q.y0;
  const double ux = b ? q.x1 : q.x2, uy = b ? q.y1 : q.y2;
  const double vx = b ? q.x2 : q.x1, vy = b ? q.y2 : q.y1;
  const double det = fdet(ox, oy, vx, vy, ux, uy);
  const double u = fu(dx, dy, ox, oy, ux, uy) / det;
  const double v = fv(dx, dy, ox, oy, vx, vy) / det;
  cu = fclamp(u, 0.0, 1.0);
  cv = fclamp(v, 0.0, 1.0);
}

__device__ inline void quad_dets(const Quad& q, double& det_a, double& det_b) {
  det_a = fdet(q.x0, q.y0, q.x1, q.y1, q.x2, q.y2);
  if (det_a != det_a) det_a = 0.0;
  det_b = fdet(q.x3, q.y3, q.x2, q.y2, q.x1, q.y1);
  if (det_b != det_b) det_b = 0.0;
}

// ---- division-free decisions with an exact fallback (K5a) ---------------------
// K5a only needs the integer pixel window of each corner and the hit / no-hit
// decision of each triangle.  Both are taken from a multiplication by the
// reciprocal (error <= a few ulps) whenever the value is clearly (relative
// margin 1e-9) away from the decision boundary — an integer for floor, the
// uv limits for a hit — and from the reference's exact divisions otherwise,
// so every decision equals the reference's (NaN / inf always take the exact
// path).  K5b recomputes the winner with the exact divisions.
constexpr double kMargin = 1e-9;

// ---- K5a: claim target pixels with the raster-order key of hitting quads -------
// Work item ("strip") = kStripH quad rows x kStripW quads of one tile's source
// window, walked by ONE wave: lane l owns point column l of the strip (64
// points = 63 quads), so each source point is loaded once per strip row (the
// next row's points are requested before this row's tests); the quad to its
// right takes the right-hand corners from the next lane (DPP wave shift) and,
// walking down, a row's bottom corners become the next row's top corners in
// registers.  Strips are dealt round-robin to the waves of the grid: for the
// per-lane walk a grid of 8x the resident blocks (one strip per wave at
// config 4, so the hardware dispatcher balances the CUs — a resident grid,
// 4-5 strips per wave, left a tail: claim 505 vs 466-472 us), for the
// compacted walk the resident grid (its LDS marks are cleared per block).  A dynamic work counter costs
// more than it balances: one global atomic per strip on one address
// serialises at its L2 channel (measured 0.45 vs 0.12 ms for the bare strip
// loop at config 4); staging a strip's points in LDS (rows then never wait on
// the claim atomics in flight) limits the grid to 2 waves per SIMD and was
// slower.
//
// Window.  The reference tests every pixel of the window spanned by the
// floors of the four corners' pixel coordinates (rectify.py:500-526); floor is
// monotone, so the window comes from the extreme corners: two floors per axis,
// taken by the reciprocal when clearly (relative margin) away from an integer,
// else from the reference's per-corner divisions.  The lane walks only the
// pixels whose centres can be hit (trim_pad: about a third of the window's
// area at config 4; the cut-off pixels are misses of both triangles).  Those
// lie inside the window whenever the pad is small, so the floors are taken
// only for windows the wave walks (or quads of many pixels).
//
// Tests.  Per triangle (A = p0 p1 p2, B = p3 p2 p1) the reference computes
// nu = _fu(...), nv = _fv(...) (rectify.py:737-768), u = nu / det, v = nv /
// det at every pixel centre of the window and hits when u >= umin, v >= umin,
// u + v <= uvmax.  In exact arithmetic u, v and u + v are affine in the
// window position (a, b): u = U0 + a Ui + b Uj.  The quad evaluates the three
// forms of both triangles in float32 (two FMAs each), shifted so that a hit is
// min3(u', v', s') >= 0, with a per-quad bound M on |form - the reference's
// float64 value| (float32 evaluation + conversion of the coefficients, plus
// the reference's own rounding of dx, ex, nu, u: TriForms2).  A pixel is
// decided by the forms when max over the triangles of min3 is >= 0 (some
// triangle surely hits) or < -2M (every triangle surely misses), else — a
// pixel centre within M of a triangle edge, rare — by the reference's exact
// float64 test (tri_exact), so every hit / miss equals the reference's.  Both
// triangles are walked in one loop on packed float32 FMAs (walk_pair).  A
// quad with a non-finite corner or a large M takes the exact test at every
// pixel of its untrimmed window.  Hits are claimed with a global atomicMin of
// the quad's key.
//
// Windows larger than kLaneWindow (a quad with a NaN corner spans its whole
// tile, rectify.py:500-526) are walked by the whole wave, 64 pixels per step,
// with the reference's exact test.  Strips are independent (no block
// synchronisation after the offsets are staged).
// Work list: chunk c belongs to the tile t with offs[t] <= c < offs[t+1] (the
// offsets come from xrs_rectify_tiles on the device, or from the host).
constexpr int kClaimThreads = 256;   // K5a block: 4 waves
constexpr int kClaimOffsLds = 1023;  // tiles whose offsets are copied to LDS (8 KB)
constexpr int kLaneWindow = 16;  // windows up to this many pixels: walked per lane
// the compacted walk: windows up to kCompactWindow pixels, the list of a
// wave-row's window pixels marked in LDS (kMarkCap positions, one byte each:
// owner lane + 1 at the owner's first position, 0 elsewhere)
constexpr int kCompactWindow = 48;
constexpr int kMarkCap = 64 * kCompactWindow;
// the product's choice, per launch: the compacted walk when the target has
// at least kCompactRatio pixels per source quad (dst_h dst_w / ((h - 1)
// (w - 1)): the quads' mean area in target pixels over the fraction of the
// target they cover).  Config 4: 2.32 (1.67 / 0.72), where the per-lane walk
// is 0.5-1.5 % faster; 2.81 (a 1.1x finer target) already favours
// compaction, 3.6 (1.25x) by 14 % (profiles/r06m_claim_walk_choice_ab.log).
constexpr double kCompactRatio = 2.6;
constexpr int kClaimGridMul = 8;   // the per-lane walk's grid: 8 x the resident blocks
constexpr double kEps64 = 0x1p-52;
constexpr double kEps32 = 0x1p-23;
constexpr double kMaxFormMargin = 1e-3;   // larger bound: exact test at every pixel

// the reference's test of one triangle at pixel centre (dx, dy)
// (rectify.py:556-573): A = (p0; p2, p1), B = (p3; p1, p2)
__device__ inline bool tri_exact(const Quad& q, bool tri_b, double dx, double dy, double umin,
                                 double uvmax) {
  double det, u, v;
  if (!tri_b) {
    det = fdet(q.x0, q.y0, q.x1, q.y1, q.x2, q.y2);
    if (det != det || det == 0.0) return false;
    u = fu(dx, dy, q.x0, q.y0, q.x2, q.y2) / det;
    v = fv(dx, dy, q.x0, q.y0, q.x1, q.y1) / det;
  } else {
    det = fdet(q.x3, q.y3, q.x2, q.y2, q.x1, q.y1);
    if (det != det || det == 0.0) return false;
    u = fu(dx, dy, q.x3, q.y3, q.x1, q.y1) / det;
    v = fv(dx, dy, q.x3, q.y3, q.x2, q.y2) / det;
  }
  return u >= umin && v >= umin && u + v <= uvmax;
}

// The reference's triangle for pixel centre (dx, dy): 1 = A hits, 2 = A
// misses and B hits, 0 = neither (rectify.py:556-573: A is tested first)
__device__ inline int tri_choice_exact(const Quad& q, double dx, double dy, double umin,
                                       double uvmax) {
  if (tri_exact(q, false, dx, dy, umin, uvmax)) return 1;
  return tri_exact(q, true, dx, dy, umin, uvmax) ? 2 : 0;
}

// The claim key of quad `key` for a pixel won by triangle `tri` (1 / 2).
__device__ inline uint32_t claim_key(const RectArgs& a, uint32_t key, int tri) {
  return a.tri_bit ? (key << 1) | (uint32_t)(tri - 1) : key;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// The three affine forms of both triangles over the quad's pixel window
// (float32; A in .x, B in .y: one packed v_pk_* instruction for the pair) and
// the decision threshold thr = -2M.  form(a, b) = c0 + a ci + b cj; (c0, ci,
// cj) of u - umin - M, v - umin - M, uvmax - M - (u + v).  Named members, not
// an array: an array of forms (read as overlapping float pairs by the packed
// walk) was kept in memory — the compiler put it in LDS, one 40-byte slot per
// lane, with bank conflicts on every read.
//
// Window position (0, 0) = the pixel centre at which the corner differences
// (ex, ey) are taken, in float64 exactly as the reference takes them.
// e1..e4: the edge factors of _fu(p, c, q) = ex e1 - ey e2 and _fv(p, c, r) =
// ey e3 - ex e4 (rectify.py:745-768); det = _fdet(...) != 0, r = 1 / det; the
// pixel centre moves by (sx, sy) per column / row (ex -= sx, ey -= sy).
// M bounds |form - the reference's float64 value| over the window:
//   float32: the inputs rounded to float (ex, ey, e, det), the reciprocal
//     (1 ulp), the products and sums of u0, v0 (terms pu = (|ex e1| + |ey e2|)
//     |r|, pv likewise), of the steps, and the two FMAs over the window
//     (T = |u0| + |v0| + g, g = wn (|ui| + |vi|) + hn (|uj| + |vj|)):
//     <= E eps32, E = 10 (pu + pv) + 8 g + 6 (T + 4), a factor >= 2 to spare
//     in every term
//   reference: dx = x_off + (i + 0.5) sx and ex = x0 - dx round by
//     <= eps64 (3 X + |x0|), X = |x_off| + (tw + 1) |sx|; the products of nu
//     by eps64 |ex e|; u = nu / det by eps64 |u|: <= 5 eps64 R + eps64 T,
//     R = ((X + |x0|) (|e1| + |e4|) + (Y + |y0|) (|e2| + |e3|)) |r|
// M = 2 (E eps32 + 10 eps64 R + 8 eps64 T), scaled up by 1.01 for its own
// float32 rounding, each magnitude taken by a simpler upper bound (a larger M
// sends more pixels to the exact test, never fewer): with S = |e1| + |e2| +
// |e3| + |e4|, Sr = S |r|: pu + pv <= (|ex| + |ey|) Sr = P, |u0| + |v0| <= P,
// g <= max(wn |sx|, hn |sy|) Sr = G, T <= P + G, E <= 16 P + 14 G + 24,
// R <= (2 max(X, Y) + |ex| + |ey|) Sr (a corner's |x0| <= |ex| + |dx0| and
// |dx0| <= X).  A triangle whose M is NaN / inf or above kMaxFormMargin
// (degenerate) sends every pixel of the window to the exact test.
struct TriForms2 {
  f32x2 u0, ui, uj, v0, vi, vj, w0, wi, wj;
  f32x2 thr;
};

// Status st.x / st.y per triangle: 1 = forms set up, 0 = no triangle (_fdet
// NaN or 0: never hits; forms -inf everywhere), -1 = no usable bound (the
// lane takes the reference's test over the untrimmed window).  Returned by
// value: the forms stay in registers.
__device__ inline TriForms2 tri_forms2(const double (&ex)[2], const double (&ey)[2],
                                       const double (&e1)[2], const double (&e2)[2],
                                       const double (&e3)[2], const double (&e4)[2],
                                       float sx, float sy, float XY2, float G0, float umin,
                                       float uvmax, float margin_scale, int2& st) {
  f32x2 fex, fey, f1, f2, f3, f4, fr, fS, fxy;
  bool tri[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const double det = e3[t] * e1[t] - e2[t] * e4[t];   // _fdet from the edge factors
    tri[t] = !(det != det || det == 0.0);
    fex[t] = (float)ex[t]; fey[t] = (float)ey[t];
    f1[t] = (float)e1[t]; f2[t] = (float)e2[t]; f3[t] = (float)e3[t]; f4[t] = (float)e4[t];
    fr[t] = __builtin_amdgcn_rcpf((float)det);
    fS[t] = (float)((fabs(e1[t]) + fabs(e2[t])) + (fabs(e3[t]) + fabs(e4[t])));
    fxy[t] = (float)(fabs(ex[t]) + fabs(ey[t]));
  }
  const f32x2 u0 = (fex * f1 - fey * f2) * fr, v0 = (fey * f3 - fex * f4) * fr;
  const f32x2 sxr = sx * fr, syr = sy * fr;
  const f32x2 ui = -(sxr * f1), uj = syr * f2, vi = sxr * f4, vj = -(syr * f3);
  const f32x2 Sr = fS * __builtin_elementwise_abs(fr);
  const f32x2 P = fxy * Sr, G = G0 * Sr;
  const f32x2 T = P + G;
  const f32x2 E = 16.0f * P + (14.0f * G + 24.0f);
  const f32x2 R = (XY2 + fxy) * Sr;
  const f32x2 M = ((float)kEps32 * E + (float)kEps64 * (10.0f * R + 8.0f * T)) *
                  (2.02f * margin_scale);
  TriForms2 F{(u0 - umin) - M, ui, uj, (v0 - umin) - M, vi, vj,
              (uvmax - (u0 + v0)) - M, -(ui + vi), -(uj + vj), -2.0f * M};
  int sts[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    sts[t] = !tri[t] ? 0 : (M[t] <= (float)kMaxFormMargin * margin_scale ? 1 : -1);
    if (!tri[t]) {   // never hits: forms -inf everywhere
      F.u0[t] = -INFINITY; F.ui[t] = F.uj[t] = 0.0f;
      F.v0[t] = F.vi[t] = F.vj[t] = 0.0f;
      F.w0[t] = F.wi[t] = F.wj[t] = 0.0f;
      F.thr[t] = 0.0f;
    }
  }
  st = int2{sts[0], sts[1]};
  return F;
}

// Walk the window's n pixels (row-major, nw per row) for both triangles at
// once: triangle A in the low and B in the high half of packed float32 FMAs
// (v_pk_fma_f32).  Returns a 2-bit code per pixel k at bits 2k, 2k + 1: 1 =
// A's (A surely hits, min3 >= 0), 2 = B's (B surely hits and A surely misses,
// min3 < -2M — the reference tests A first), 3 = undecided (some min3 >=
// -2M otherwise: the exact tests), 0 = miss.  One code word instead of three
// masks, and the column / row stepped in float (wn = nw - 1): fewer
// instructions per pixel.
__device__ inline uint32_t walk_pair(const TriForms2& F, int n, float wn) {
  uint32_t W = 0;
  float af = 0.0f, bf = 0.0f;
  for (int k = 0; k < n; ++k) {
    const f32x2 av = {af, af}, bv = {bf, bf};
    const f32x2 u = __builtin_elementwise_fma(bv, F.uj, __builtin_elementwise_fma(av, F.ui, F.u0));
    const f32x2 v = __builtin_elementwise_fma(bv, F.vj, __builtin_elementwise_fma(av, F.vi, F.v0));
    const f32x2 w = __builtin_elementwise_fma(bv, F.wj, __builtin_elementwise_fma(av, F.wi, F.w0));
    const float ha = fminf(u.x, fminf(v.x, w.x)), hb = fminf(u.y, fminf(v.y, w.y));
    const bool a_in = ha >= 0.0f, a_near = ha >= F.thr.x;
    const uint32_t c = a_in ? 1u
                     : (!a_near && hb >= 0.0f) ? 2u
                     : (a_near || hb >= F.thr.y) ? 3u : 0u;
    W |= c << (2 * k);
    const bool wrap = af == wn;
    af = wrap ? 0.0f : af + 1.0f;
    bf = wrap ? bf + 1.0f : bf;
  }
  return W;
}

// walk_pair's code of one window pixel (af, bf) (column, row from the window
// origin), for the compacted walk
__device__ inline int pixel_code(const TriForms2& F, float af, float bf) {
  const f32x2 av = {af, af}, bv = {bf, bf};
  const f32x2 u = __builtin_elementwise_fma(bv, F.uj, __builtin_elementwise_fma(av, F.ui, F.u0));
  const f32x2 v = __builtin_elementwise_fma(bv, F.vj, __builtin_elementwise_fma(av, F.vi, F.v0));
  const f32x2 w = __builtin_elementwise_fma(bv, F.wj, __builtin_elementwise_fma(av, F.wi, F.w0));
  const float ha = fminf(u.x, fminf(v.x, w.x)), hb = fminf(u.y, fminf(v.y, w.y));
  const bool a_in = ha >= 0.0f, a_near = ha >= F.thr.x;
  return a_in ? 1 : (!a_near && hb >= 0.0f) ? 2 : (a_near || hb >= F.thr.y) ? 3 : 0;
}

// Wave-wide inclusive scans (64 lanes) by DPP: row_shr 1, 2, 4, 8 within each
// row of 16 lanes (bound_ctrl: lanes shifted in from outside the row read 0),
// then row_bcast:15 (lane 15 of rows 0 / 2 into rows 1 / 3) and row_bcast:31
// (lane 31 into rows 2, 3).  Identity 0: v >= 0 for the max scan.
template <int CTRL, int ROWS, bool BC>
__device__ inline int32_t dpp0(int32_t v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, BC);
}
__device__ inline int32_t wave_scan_add(int32_t v) {
  v += dpp0<0x111, 0xF, true>(v);
  v += dpp0<0x112, 0xF, true>(v);
  v += dpp0<0x114, 0xF, true>(v);
  v += dpp0<0x118, 0xF, true>(v);
  v += dpp0<0x142, 0xA, false>(v);
  v += dpp0<0x143, 0xC, false>(v);
  return v;
}
__device__ inline int32_t wave_scan_max(int32_t v) {
  v = max(v, dpp0<0x111, 0xF, true>(v));
  v = max(v, dpp0<0x112, 0xF, true>(v));
  v = max(v, dpp0<0x114, 0xF, true>(v));
  v = max(v, dpp0<0x118, 0xF, true>(v));
  v = max(v, dpp0<0x142, 0xA, false>(v));
  v = max(v, dpp0<0x143, 0xC, false>(v));
  return v;
}

// lane (addr / 4)'s value (ds_bpermute: every source lane must be active)
__device__ inline float bperm_f32(int32_t addr, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}

// The trim pad of a quad's window (floors of the corners' extreme pixel
// units q, rectify.py:500-526): only pixels whose centre i + 0.5 lies within
// `pad` of [qx0, qx1] x [qy0, qy1] can be hit.  A point the reference counts
// as a hit has u, v >= -d, u + v <= 1 + 2d with d = |uv_delta| + its rounding
// (<= the form bound M <= kMaxFormMargin, checked by tri_forms2 for both
// triangles before a trimmed window is used); such points lie within
// 4 d (extent) of the triangle's bounding box, so pad = 8 d (W + H) plus an
// absolute 1e-6 (1 + max |q|) (the rounding of q itself) leaves a factor 2 to spare.
// Pixels cut off are misses of both triangles.
__device__ inline double trim_pad(double qx0, double qx1, double qy0, double qy1, double sq,
                                  double d) {   // sq >= max |q|
  return 8.0 * d * ((qx1 - qx0) + (qy1 - qy0)) + 1e-6 * (1.0 + sq);
}

__device__ inline double dpp_next_f64(double v) {   // lane i <- lane i + 1 (lane 63: 0)
  const uint64_t b = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, 0x130, 0xF, 0xF, true);
  const uint32_t hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), 0x130, 0xF, 0xF, true);
  return __longlong_as_double((int64_t)(((uint64_t)hi << 32) | lo));
}

__device__ inline float dpp_next_f32(float v) {      // lane i <- lane i + 1 (lane 63: 0)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xF, 0xF, true));
}

// trim_pad in float32 for the float32 window, widened by kPadEps32 (1 + sq):
// the conversion of each q to float32 (<= 2^-24 |q|), the two subtractions
// that place the window (<= 2^-24 (|q| + 1) each) and this expression's own
// roundings (<= 6 ulps of a value below 1) together stay below it
constexpr float kPadEps32 = 0x1p-20f;
__device__ inline float trim_pad32(float qx0, float qx1, float qy0, float qy1, float sq, float d) {
  return 8.0f * d * ((qx1 - qx0) + (qy1 - qy0)) + (1e-6f + kPadEps32) * (1.0f + sq);
}

struct PairQ {         // a point pair's extreme pixel units (float32); both finite
  float xmn, xmx, ymn, ymx;
  bool fin;
};

struct StripPoint {    // one source point of the strip
  double x, y;
};

__device__ inline StripPoint strip_next(const StripPoint& p) {
  return StripPoint{dpp_next_f64(p.x), dpp_next_f64(p.y)};
}

// floor of the extreme corner value q (min or max of the four corners' target
// pixel units) when it is clearly away from an integer: then it equals the
// min / max of the corners' exact np.floor((x - off) / scale) (the error of q
// is a few ulps, far below the margin); false -> exact per-corner path
__device__ inline bool floor_clear(double q, double margin, double& f) {
  f = floor(q);
  const double fr = q - f;
  const double m = margin * (1.0 + fabs(q));
  return fr > m && fr < 1.0 - m;
}

// the reference's int64 window bound of one axis from the four corners
// (rectify.py:500-507): exact divisions, NaN / huge -> INT64_MIN
__device__ inline void pix_range_exact(double c0, double c1, double c2, double c3, double off,
                                       double scale, int64_t& lo, int64_t& hi) {
  const int64_t p0 = f64_to_i64_x86(floor((c0 - off) / scale));
  const int64_t p1 = f64_to_i64_x86(floor((c1 - off) / scale));
  const int64_t p2 = f64_to_i64_x86(floor((c2 - off) / scale));
  const int64_t p3 = f64_to_i64_x86(floor((c3 - off) / scale));
  lo = min(min(p0, p1), min(p2, p3));
  hi = max(max(p0, p1), max(p2, p3));
}

__device__ inline Quad load_quad32(const RectArgs& a, int32_t qj, int32_t qi) {
  return load_quad(a, qj, qi);
}


// A quad the fast path cannot take (a non-finite corner, a pixel-unit extreme
// close to an integer, a degenerate quad, the test knob): the reference's
// window (rectify.py:500-526, exact divisions) and, for windows up to
// kLaneWindow, its exact test at every pixel; larger windows are handed back
// (imin, jmin, nw, big_cnt) for the wave-wide walk.
__device__ inline void claim_exact_lane(const RectArgs& a, const TileInfo& ti, int32_t qj,
                                              int32_t qi, uint32_t key, double umin,
                                              double uvmax, int32_t& imin, int32_t& jmin,
                                              int32_t& nw, int64_t& big_cnt) {
  const Quad Q = load_quad(a, qj, qi);
  int64_t i0, i1, j0, j1;
  pix_range_exact(Q.x0, Q.x1, Q.x2, Q.x3, ti.x_off, a.x_scale, i0, i1);
  pix_range_exact(Q.y0, Q.y1, Q.y2, Q.y3, ti.y_off, a.y_scale, j0, j1);
  if (i1 < 0 || j1 < 0 || i0 >= ti.tw || j0 >= ti.th) return;
  i0 = max(i0, (int64_t)0); j0 = max(j0, (int64_t)0);
  i1 = min(i1, (int64_t)ti.tw - 1); j1 = min(j1, (int64_t)ti.th - 1);
  double det_a, det_b;
  quad_dets(Q, det_a, det_b);
  if (det_a == 0.0 && det_b == 0.0) return;
  const int32_t w = (int32_t)(i1 - i0 + 1), h = (int32_t)(j1 - j0 + 1);
  const int64_t cnt = (int64_t)w * h;
  if (cnt > kLaneWindow) {
    imin = (int32_t)i0; jmin = (int32_t)j0; nw = w; big_cnt = cnt;
    return;
  }
  for (int32_t dj = (int32_t)j0; dj <= (int32_t)j1; ++dj) {
    const double dy = ti.y_off + ((double)dj + 0.5) * a.y_scale;
    for (int32_t di = (int32_t)i0; di <= (int32_t)i1; ++di) {
      const double dx = ti.x_off + ((double)di + 0.5) * a.x_scale;
      const int tri = tri_choice_exact(Q, dx, dy, umin, uvmax);
      if (tri) atomicMin(a.keys + (int64_t)(ti.r0 + dj) * a.dst_w + ti.c0 + di, claim_key(a, key, tri));
    }
  }
}

// LDS_OFFS: offsets staged in LDS (up to kClaimOffsLds tiles) or read from
// HBM; YPOS: the sign of y_scale (j axis up), which decides whether the
// corners' min or max y gives the first window row — a launch constant
// COMPACT: the wave-compacted walk (else per lane), chosen per launch
template <bool LDS_OFFS, bool YPOS, bool COMPACT>
__global__ void __launch_bounds__(kClaimThreads, 4)   // <= 128 VGPRs: 4 waves per SIMD
rectify_claim_kernel(RectArgs a) {
  __shared__ int64_t offs_s[kClaimOffsLds + 1];
  // the compacted walk, per wave (no block synchronisation): owner marks of
  // the list positions and the owners' forms (12 KB + 16 KB)
  constexpr int kW = COMPACT ? kClaimThreads / 64 : 1;
  __shared__ uint8_t mark_s[kW][COMPACT ? kMarkCap : 1];
  __shared__ f32x2 forms_s[kW][COMPACT ? 8 : 1][64];
  const int lane = threadIdx.x & 63;
  uint8_t* const mark = mark_s[COMPACT ? threadIdx.x >> 6 : 0];
  f32x2 (*const forms)[64] = forms_s[COMPACT ? threadIdx.x >> 6 : 0];
  if (COMPACT)
    for (int32_t k = lane; k < kMarkCap; k += 64) mark[k] = 0;   // cleared after each row
  // windows above kWin pixels leave the walks (the wave-wide exact walk)
  constexpr int kWin = COMPACT ? kCompactWindow : kLaneWindow;
  constexpr bool lds_offs = LDS_OFFS;
  if (lds_offs)
    for (int64_t t = threadIdx.x; t <= a.ntiles; t += kClaimThreads) offs_s[t] = a.chunk_offs[t];
  __syncthreads();
  // the offsets are read from the LDS copy or from global memory in two
  // instantiations: one pointer to either is a generic (flat) pointer, whose
  // loads wait on both the LDS and the vector-memory counters
  const int64_t nchunks = lds_offs ? offs_s[a.ntiles] : a.chunk_offs[a.ntiles];
  const double umin = -a.uv_delta, uvmax = 1.0 + 2 * a.uv_delta;
  const int64_t nwaves = (int64_t)gridDim.x * (kClaimThreads / 64);
  // the compacted walk takes each strip in two halves of kStripH / 2 quad rows
  // (work unit c2: strip c2 >> 1, half c2 & 1), the per-lane walk whole strips
  constexpr int kHalves = COMPACT ? 2 : 1;
  for (int64_t c2 = (int64_t)blockIdx.x * (kClaimThreads / 64) + (threadIdx.x >> 6);
       c2 < nchunks * kHalves; c2 += nwaves) {
    const int64_t c = c2 / kHalves;
    const int32_t half = (int32_t)(c2 - c * kHalves);
    int64_t lo = 0, hi = a.ntiles;   // last t with offs[t] <= c (c is wave-uniform)
    if (lds_offs) {
      while (hi - lo > 1) {
        const int64_t m = (lo + hi) >> 1;
        if (offs_s[m] <= c) lo = m; else hi = m;
      }
    } else {
      while (hi - lo > 1) {
        const int64_t m = (lo + hi) >> 1;
        if (a.chunk_offs[m] <= c) lo = m; else hi = m;
      }
    }
    lo = __builtin_amdgcn_readfirstlane((int32_t)lo);   // wave-uniform
    const int64_t off_lo = lds_offs ? offs_s[lo] : a.chunk_offs[lo];
    const TileInfo ti = a.tiles[lo];
    if (!tile_ok(a, ti) || ti.si0 < 0) {   // wave-uniform
      if (lane == 0) atomicOr(a.err_flags, XRS_EFLAG_STATE);
      continue;
    }
    const int32_t nq_i = ti.swin - 1, nq_j = ti.shin - 1;
    // form bound constants of the tile (tri_forms2): 2 max(X, Y) with X =
    // |x_off| + (tw + 1) |sx| bounding a pixel centre's |x| (Y likewise)
    const float sxf = (float)a.x_scale, syf = (float)a.y_scale;
    const float XY2 = 2.0f * fmaxf(fabsf((float)ti.x_off) + (float)(ti.tw + 1) * fabsf(sxf),
                                   fabsf((float)ti.y_off) + (float)(ti.th + 1) * fabsf(syf));
    const int32_t ncx = (nq_i + kStripW - 1) / kStripW;
    const int32_t cc = (int32_t)(c - off_lo);
    const int32_t cy = cc / ncx, cx = cc - cy * ncx;
    const int32_t pcol = cx * kStripW + lane;          // point column in the window
    const bool has_pt = pcol <= nq_i;
    const bool has_q = lane < kStripW && pcol < nq_i;  // quad (row, pcol) exists
    const int32_t qi = ti.si0 + pcol;
    const int32_t r0 = cy * kStripH + half * (kStripH / kHalves);
    const int32_t r_end = min(r0 + kStripH / kHalves, nq_j);
    if (r0 >= r_end) {   // wave-uniform: a strip past the window (inconsistent offsets),
                         // or the empty second half of a short strip
      if (half == 0 && lane == 0) atomicOr(a.err_flags, XRS_EFLAG_STATE);
      continue;
    }
    auto load_pt = [&](int32_t qj) {
      StripPoint p{NAN, NAN};
      if (has_pt) {
        const int64_t o = (int64_t)qj * a.sy + qi;
        p.x = a.x[o];
        p.y = a.y[o];
      }
      return p;
    };
    // target pixel units by the reciprocal (window floors)
    auto qx = [&](double x) { return (x - ti.x_off) * a.inv_x; };
    auto qy = [&](double y) { return (y - ti.y_off) * a.inv_y; };
    StripPoint t0 = load_pt(ti.sj0 + r0);
    // a row's point pairs (l, l + 1): the extremes of their tile-local pixel
    // units in float32 (each point converted once, its right-hand neighbour's
    // by DPP) and their finiteness, for the quads above and below the row
    auto pair_q = [&](const StripPoint& p) {
      const float ux = (float)qx(p.x), uy = (float)qy(p.y);
      const float vx = dpp_next_f32(ux), vy = dpp_next_f32(uy);
      const float sum = (ux + vx) + (uy + vy);   // NaN / inf if any is (or overflowed)
      return PairQ{fminf(ux, vx), fmaxf(ux, vx), fminf(uy, vy), fmaxf(uy, vy),
                   sum - sum == 0.0f};
    };
    PairQ et = pair_q(t0);
    StripPoint nxt = load_pt(ti.sj0 + r0 + 1);
    for (int32_t r = r0; r < r_end; ++r) {
      const int32_t qj = ti.sj0 + r;                    // global quad row (corner p0)
      // (the top row's right-hand corners are re-shifted, not kept: registers)
      const StripPoint t1 = strip_next(t0);
      const StripPoint b0 = nxt;
      // the next row's bottom points are requested before this row's tests
      if (r + 1 < r_end) nxt = load_pt(qj + 2);
      const StripPoint b1 = strip_next(b0);
      const PairQ eb = pair_q(b0);
      // corners p0 = t0, p1 = t1, p2 = b0, p3 = b1
      int32_t imin = 0, jmin = 0, nw = 0;
      int64_t big_cnt = 0;   // > 0: window above kLaneWindow, walked by the wave below
      bool slow = false;     // window not decided fast: claim_exact_lane
      uint32_t hit = 0, hit_b = 0, unsure = 0;   // bit 2k: window pixel k (row-major) hit
                                                  // (hit_b: by triangle B) / undecided
      int32_t nwalk = 0;     // compacted walk, > 0: the trimmed window's pixels, tested
                             // by the wave below with the forms F
      if (has_q) {
        // the corners' extreme pixel units (float32, tile-local: |q| is at most
        // a few tile widths for every quad the fast path takes)
        const float qx0 = fminf(et.xmn, eb.xmn), qx1 = fmaxf(et.xmx, eb.xmx);
        const float qy0 = fminf(et.ymn, eb.ymn), qy1 = fmaxf(et.ymx, eb.ymx);
        // sq >= every |q| (a sum, not a max: no NaN-quieting of the operands);
        // conditions combined with & (one branch, not one per term)
        const float sq = (fabsf(qx0) + fabsf(qx1)) + (fabsf(qy0) + fabsf(qy1));
        if (et.fin & eb.fin & (sq < 0x1p20f)) {
          // T: the pixel centres (i + 0.5) within `pad` of the corners'
          // extremes, clipped to the tile — every other pixel is a miss of
          // both triangles (trim_pad).  With pad + the reciprocal's error
          // < 0.5, T lies inside the reference's window R = [floor(qx0),
          // floor(qx1)] x [floor(qy0), floor(qy1)] (ceil(q - 0.5 - pad) >=
          // floor(q) and floor(q - 0.5 + pad) <= floor(q)), so R — its exact
          // floors — is needed only for the wave-wide walk of a large window
          // (R untrimmed) or a quad so large that pad >= 0.25.
          // In float32: every q carries the rounding of its conversion
          // (<= 2^-24 |q|) and the subtractions below round by <= 2^-24 (|q|
          // + 1); the pad is widened by kPadEps32 (1 + sq) >= all of them
          // together, so the float32 T holds every pixel of the float64 one.
          const float d = (float)(fabs(a.uv_delta) + kMaxFormMargin * a.margin_scale);
          const float pad = trim_pad32(qx0, qx1, qy0, qy1, sq, d);
          const float lo = 0.5f + pad, hi = 0.5f - pad;
          const float ci = ceilf(qx0 - lo), fi = floorf(qx1 - hi);
          const float cj = ceilf(qy0 - lo), fj = floorf(qy1 - hi);
          const float twm1 = (float)(ti.tw - 1), thm1 = (float)(ti.th - 1);
          const bool empty = !((ci <= fi) & (cj <= fj) & (fi >= 0.0f) & (fj >= 0.0f) &
                               (ci <= twm1) & (cj <= thm1));
          int32_t ti0 = 0, ti1 = -1, tj0 = 0, tj1 = -1;
          if (!empty) {   // clipped to the tile by selects (values in range here)
            ti0 = ci > 0.0f ? (int32_t)ci : 0;
            tj0 = cj > 0.0f ? (int32_t)cj : 0;
            ti1 = fi < twm1 ? (int32_t)fi : ti.tw - 1;
            tj1 = fj < thm1 ? (int32_t)fj : ti.th - 1;
          }
          int64_t cnt = (int64_t)(ti1 - ti0 + 1) * (tj1 - tj0 + 1);
          bool walk = !empty;
          // (the exact-decision test knob sets an infinite margin: R always)
          if (pad >= 0.25f || !(a.margin < 0.25) || (!empty && cnt > kWin)) {
            walk = false;
            // R from the float64 pixel units (rare: large windows / quads)
            const double dqx0 = qx(fmin(fmin(t0.x, t1.x), fmin(b0.x, b1.x)));
            const double dqx1 = qx(fmax(fmax(t0.x, t1.x), fmax(b0.x, b1.x)));
            const double ylo = fmin(fmin(t0.y, t1.y), fmin(b0.y, b1.y));
            const double yhi = fmax(fmax(t0.y, t1.y), fmax(b0.y, b1.y));
            const double dqy0 = qy(YPOS ? ylo : yhi);
            const double dqy1 = qy(YPOS ? yhi : ylo);
            double fx0, fx1, fy0, fy1;
            if (floor_clear(dqx0, a.margin, fx0) && floor_clear(dqx1, a.margin, fx1) &&
                floor_clear(dqy0, a.margin, fy0) && floor_clear(dqy1, a.margin, fy1)) {
              int32_t i0 = (int32_t)fx0, i1 = (int32_t)fx1, j0 = (int32_t)fy0, j1 = (int32_t)fy1;
              if (!empty && !(i1 < 0 || j1 < 0 || i0 >= ti.tw || j0 >= ti.th)) {
                i0 = max(i0, 0); j0 = max(j0, 0);
                i1 = min(i1, ti.tw - 1); j1 = min(j1, ti.th - 1);
                ti0 = max(ti0, i0); ti1 = min(ti1, i1);   // T inside R
                tj0 = max(tj0, j0); tj1 = min(tj1, j1);
                cnt = (int64_t)(ti1 - ti0 + 1) * (tj1 - tj0 + 1);
                if (ti0 > ti1 || tj0 > tj1) {
                  // no pixel centre near the quad: nothing to test
                } else if (cnt > kWin) {
                  imin = i0; jmin = j0; nw = i1 - i0 + 1;   // untrimmed: exact test everywhere
                  big_cnt = (int64_t)(i1 - i0 + 1) * (j1 - j0 + 1);   // (a quad without a
                                                                       // triangle is dropped there)
                } else {
                  walk = true;
                }
              }
            } else {
              slow = true;
            }
          }
          if (walk) {
            imin = ti0; jmin = tj0;
            nw = ti1 - ti0 + 1;
            const int32_t nh = tj1 - tj0 + 1;
            const int32_t n = (int32_t)cnt;
            const double dx0 = ti.x_off + ((double)imin + 0.5) * a.x_scale;   // pixel (imin, jmin)
            const double dy0 = ti.y_off + ((double)jmin + 0.5) * a.y_scale;
            const float wn = (float)(nw - 1), hn = (float)(nh - 1);
            // A = (p0, p1, p2): _fu(p, p0, p2), _fv(p, p0, p1), _fdet(p0, p1, p2)
            // B = (p3, p2, p1): _fu(p, p3, p1), _fv(p, p3, p2), _fdet(p3, p2, p1)
            const double ex[2] = {t0.x - dx0, b1.x - dx0}, ey[2] = {t0.y - dy0, b1.y - dy0};
            const double e1[2] = {t0.y - b0.y, b1.y - t1.y}, e2[2] = {t0.x - b0.x, b1.x - t1.x};
            const double e3[2] = {t0.x - t1.x, b1.x - b0.x}, e4[2] = {t0.y - t1.y, b1.y - b0.y};
            int2 st;
            const TriForms2 F = tri_forms2(ex, ey, e1, e2, e3, e4, sxf, syf, XY2,
                                           fmaxf(wn * fabsf(sxf), hn * fabsf(syf)), (float)umin,
                                           (float)uvmax, a.margin_scale, st);
            if (st.x < 0 || st.y < 0) {
              slow = true;   // a triangle without a usable bound: exact, untrimmed window
            } else if (st.x | st.y) {
              if constexpr (COMPACT) {
                nwalk = n;
                // the forms for the compacted walk below (wi, wj are recomputed
                // there); this wave's previous row has finished reading them
                forms[0][lane] = F.u0; forms[1][lane] = F.ui; forms[2][lane] = F.uj;
                forms[3][lane] = F.v0; forms[4][lane] = F.vi; forms[5][lane] = F.vj;
                forms[6][lane] = F.w0; forms[7][lane] = F.thr;
              } else {
                const uint32_t W = walk_pair(F, n, wn);
                hit = (W ^ (W >> 1)) & 0x55555555u;   // codes 1, 2 at bit 2k
                hit_b = W >> 1;                        // bit 2k: the code's high bit
                unsure = W & (W >> 1) & 0x55555555u;  // code 3
              }
            }
          }
        } else {
          slow = true;
        }
      }
      const uint32_t key = (uint32_t)qj * a.key_mul + (uint32_t)qi;   // raster order
      // claim keys of the two triangles (tri_bit: the low bit names B)
      const uint32_t key_a = claim_key(a, key, 1), key_b = claim_key(a, key, 2);
      if constexpr (COMPACT) {
        // ---- the compacted walk (rectify.py:547-573 for every trimmed window) ----
        // The lanes' window pixels form one list, pixel k of lane l at P_l + k
        // (P: exclusive prefix sum of nwalk); the wave tests them 64 at a time,
        // each lane one pixel of the list with its owner's forms (LDS) and
        // window (ds_bpermute), so a wave-row costs ceil(sum / 64) steps instead
        // of the longest window.  The owner of list position g is the last lane
        // whose window starts at or before g: each owner marks its start (LDS,
        // cleared again after the row) and a wave max-scan carries it over the
        // window.  The per-pixel decision is
        // the per-lane walk's (pixel_code: the same float32 forms at the same
        // (a, b)), so every claim is the per-lane walk's.
        const int32_t incl = wave_scan_add(nwalk);
        const int32_t total = __builtin_amdgcn_readlane(incl, 63);
        if (total > 0) {   // wave-uniform
          const int32_t P = incl - nwalk;
          if (nwalk > 0) mark[P] = (uint8_t)(lane + 1);   // owner's mark
          __builtin_amdgcn_wave_barrier();   // (one wave's LDS accesses complete in order)
          // nw (<= 48), n (<= 48) and P (< kMarkCap) of this lane, for its pixels' lanes
          const uint32_t pk = (uint32_t)nw | ((uint32_t)nwalk << 6) | ((uint32_t)P << 12);
          const float rnw_self = __builtin_amdgcn_rcpf((float)max(nw, 1));
          int32_t carry = 0;   // owner + 1 of the list position before this step
          for (int32_t base = 0; base < total; base += 64) {
            const int32_t g = base + lane;
            int32_t m = 0;
            if (g < total) m = mark[g];
            m = max(wave_scan_max(m), carry);
            carry = __builtin_amdgcn_readlane(m, 63);
            const int32_t o = (m - 1) & 63;   // owner lane (past the list: unused)
            const int32_t oa = o << 2;        // its bpermute address
            const uint32_t opk = (uint32_t)__builtin_amdgcn_ds_bpermute(oa, (int32_t)pk);
            const int32_t oimin = __builtin_amdgcn_ds_bpermute(oa, imin);
            const int32_t ojmin = __builtin_amdgcn_ds_bpermute(oa, jmin);
            const float ornw = bperm_f32(oa, rnw_self);
            const int32_t onw = (int32_t)(opk & 63u), on = (int32_t)((opk >> 6) & 63u);
            const int32_t k = g - (int32_t)(opk >> 12);
            if (g < total && m > 0 && k >= 0 && k < on) {
              // the owner's forms (wi, wj by tri_forms2's own expressions: the
              // same bits as the owner's)
              TriForms2 G;
              G.u0 = forms[0][o]; G.ui = forms[1][o]; G.uj = forms[2][o];
              G.v0 = forms[3][o]; G.vi = forms[4][o]; G.vj = forms[5][o];
              G.w0 = forms[6][o]; G.thr = forms[7][o];
              G.wi = -(G.ui + G.vi); G.wj = -(G.uj + G.vj);
              // window pixel k: row k / nw, column k % nw (exact in float for
              // k < 64: the quotient is >= 1/128 from an integer)
              const int32_t dj = (int32_t)(((float)k + 0.5f) * ornw);
              const int32_t di = k - dj * onw;
              int tri = pixel_code(G, (float)di, (float)dj);
              if (tri != 0) {
                const uint32_t okey = (uint32_t)qj * a.key_mul + (uint32_t)(qi - lane + o);
                const int32_t pj = ojmin + dj, pi = oimin + di;   // tile-local pixel
                if (tri == 3) {   // a pixel centre within the margin of an edge: exact
                  const Quad Q = load_quad(a, qj, qi - lane + o);
                  const double dy = ti.y_off + ((double)pj + 0.5) * a.y_scale;
                  const double dx = ti.x_off + ((double)pi + 0.5) * a.x_scale;
                  tri = tri_choice_exact(Q, dx, dy, umin, uvmax);
                }
                if (tri) {
                  const uint32_t ck = claim_key(a, okey, tri);
                  uint32_t* tile_keys = a.keys + (int64_t)ti.r0 * a.dst_w + ti.c0;
                  if (a.narrow)   // 32-bit byte offsets from the wave-uniform tile base
                    atomicMin(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(tile_keys) +
                                                          (((uint32_t)pj * (uint32_t)a.dst_w +
                                                            (uint32_t)pi) << 2)), ck);
                  else
                    atomicMin(tile_keys + (int64_t)pj * a.dst_w + pi, ck);
                }
              }
            }
          }
          if (nwalk > 0) mark[P] = 0;   // after this wave's reads of the row (in order)
        }
      }
      // claims: the window pixels hit (row k / nw, column k % nw: exact in float
      // for k < 16, the quotient is >= 1/32 from an integer)
      if (!COMPACT && (hit | unsure)) {
        const float rnw = 1.0f / (float)nw;
        uint32_t* tile_keys = a.keys + (int64_t)ti.r0 * a.dst_w + ti.c0;
        if (a.narrow) {
          // 32-bit offsets from the wave-uniform tile base (no 64-bit address
          // math per claim): pixel k of the window at lbase + k + dj (W - nw)
          const uint32_t w32 = (uint32_t)a.dst_w;
          const uint32_t lbase = (uint32_t)jmin * w32 + (uint32_t)imin;
          const uint32_t lstride = w32 - (uint32_t)nw;
          while (hit) {
            const int k2 = __builtin_ctz(hit), k = k2 >> 1;
            hit &= hit - 1;
            const uint32_t dj = (uint32_t)(((float)k + 0.5f) * rnw);
            const uint32_t off = lbase + (uint32_t)k + __umul24(dj, lstride);
            atomicMin(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(tile_keys) + (off << 2)),
                      (hit_b >> k2) & 1u ? key_b : key_a);
          }
        }
        while (hit) {
          const int k2 = __builtin_ctz(hit), k = k2 >> 1;
          hit &= hit - 1;
          const int32_t dj = (int32_t)(((float)k + 0.5f) * rnw);
          atomicMin(tile_keys + (int64_t)(jmin + dj) * a.dst_w + imin + k - dj * nw,
                    (hit_b >> k2) & 1u ? key_b : key_a);
        }
        if (unsure) {   // a pixel centre within the margin of an edge: the reference's test
          const Quad Q = load_quad(a, qj, qi);
          do {
            const int k = __builtin_ctz(unsure) >> 1;
            unsure &= unsure - 1;
            const int32_t dj = (int32_t)(((float)k + 0.5f) * rnw);
            const int32_t di = imin + k - dj * nw;
            const double dy = ti.y_off + ((double)(jmin + dj) + 0.5) * a.y_scale;
            const double dx = ti.x_off + ((double)di + 0.5) * a.x_scale;
            const int tri = tri_choice_exact(Q, dx, dy, umin, uvmax);
            if (tri)
              atomicMin(tile_keys + (int64_t)(jmin + dj) * a.dst_w + di, tri == 1 ? key_a : key_b);
          } while (unsure);
        }
      }
      if (slow) claim_exact_lane(a, ti, qj, qi, key, umin, uvmax, imin, jmin, nw, big_cnt);
      // large windows: one quad at a time, walked by the whole wave (exact test)
      uint64_t big = __ballot(big_cnt > 0);
      while (big) {
        const int o = __builtin_ctzll(big);
        big &= big - 1;
        const int32_t oqi = __builtin_amdgcn_readlane(qi, o);
        const Quad Q = load_quad32(a, qj, oqi);
        const int32_t wi0 = __builtin_amdgcn_readlane(imin, o);
        const int32_t wj0 = __builtin_amdgcn_readlane(jmin, o);
        const int32_t wnw = __builtin_amdgcn_readlane(nw, o);
        const uint32_t wkey_a = __builtin_amdgcn_readlane(key_a, o);
        const uint32_t wkey_b = __builtin_amdgcn_readlane(key_b, o);
        const int64_t wcnt =
            ((int64_t)__builtin_amdgcn_readlane((uint32_t)(big_cnt >> 32), o) << 32) |
            __builtin_amdgcn_readlane((uint32_t)big_cnt, o);
        // test k = lane + 64 s sits at (row k / wnw, column k % wnw), stepped exactly
        const int32_t step_r = 64 / wnw, step_c = 64 % wnw;
        int64_t dj = lane / wnw;
        int32_t di = lane % wnw;
        for (int64_t k = lane; k < wcnt; k += 64) {
          const double dy = ti.y_off + ((double)(wj0 + dj) + 0.5) * a.y_scale;
          const double dx = ti.x_off + ((double)(wi0 + di) + 0.5) * a.x_scale;
          const int tri = tri_choice_exact(Q, dx, dy, umin, uvmax);
          if (tri)
            atomicMin(a.keys + (int64_t)(ti.r0 + wj0 + dj) * a.dst_w + ti.c0 + wi0 + di,
                      tri == 1 ? wkey_a : wkey_b);
          dj += step_r;
          di += step_c;
          if (di >= wnw) { di -= wnw; ++dj; }
        }
      }
      t0 = b0;
      et = eb;
    }
  }
}

// ---- K6: per-variable sampling (rectify.py:663-734) ------------------------------
// One target pixel p of every dim-0 slice at source position (fi, fj); NaN
// positions -> fill.  Positions outside the source (never made by K5:
// src_i_min + src_i <= w - 1, rectify.py:574-576) are filled and reported
// (`bad`), never dereferenced.
template <typename T, int INTERP>
__device__ inline void sample_px(double fi, double fj, const T* __restrict__ src, int64_t n,
                                 int64_t src_h, int64_t src_w, int64_t src_sn, int64_t src_sy,
                                 T* __restrict__ dst, int64_t dst_sn, int64_t p, T tfill,
                                 bool& bad) {
  if (fi != fi || fj != fj) {
    for (int64_t s = 0; s < n; ++s) dst[s * dst_sn + p] = tfill;
    return;
  }
  if (!(fi >= 0.0 && fi < (double)src_w && fj >= 0.0 && fj < (double)src_h)) {
    bad = true;
    for (int64_t s = 0; s < n; ++s) dst[s * dst_sn + p] = tfill;
    return;
  }
  // int() truncation of values in [0, src_w) / [0, src_h), both < 2^31
  // (checked at launch): 32-bit conversions
  int64_t i0 = (int32_t)fi, j0 = (int32_t)fj;
  const double u = fi - (double)(int32_t)i0, v = fj - (double)(int32_t)j0;
  const int64_t imax = src_w - 1, jmax = src_h - 1;
  if (INTERP == XRS_INTERP_NEAREST) {
    if (u > 0.5) i0 = min(max(i0 + 1, (int64_t)0), imax);
    if (v > 0.5) j0 = min(max(j0 + 1, (int64_t)0), jmax);
    for (int64_t s = 0; s < n; ++s) dst[s * dst_sn + p] = src[s * src_sn + j0 * src_sy + i0];
    return;
  }
  const int64_t i1 = min(max(i0 + 1, (int64_t)0), imax), j1 = min(max(j0 + 1, (int64_t)0), jmax);
  for (int64_t s = 0; s < n; ++s) {
    const T* S = src + s * src_sn;
    double val;
    const double v01 = (double)S[j0 * src_sy + i1], v10 = (double)S[j1 * src_sy + i0];
    if (INTERP == XRS_INTERP_TRIANGULAR) {
      if (u + v < 1.0) {
        const double v00 = (double)S[j0 * src_sy + i0];
        val = v00 + u * (v01 - v00) + v * (v10 - v00);
      } else {
        const double v11 = (double)S[j1 * src_sy + i1];
        val = v11 + (1.0 - u) * (v10 - v11) + (1.0 - v) * (v01 - v11);
      }
    } else {
      const double v00 = (double)S[j0 * src_sy + i0], v11 = (double)S[j1 * src_sy + i1];
      const double u0 = v00 + u * (v01 - v00);
      const double u1 = v10 + u * (v11 - v10);
      val = u0 + v * (u1 - u0);
    }
    dst[s * dst_sn + p] = Conv<T>::from_f64(val);
  }
}

template <typename T, int INTERP>
__global__ void __launch_bounds__(kThreads)
rectify_var_kernel(const double* __restrict__ ij, int64_t ij_sn, int64_t dst_h, int64_t dst_w,
                   const T* __restrict__ src, int64_t n, int64_t src_h, int64_t src_w,
                   int64_t src_sn, int64_t src_sy, T* __restrict__ dst, int64_t dst_sn,
                   double fill, int32_t* err_flags) {
  const int64_t np = dst_h * dst_w;
  const T tfill = Conv<T>::from_f64(fill);
  bool bad = false;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < np;
       p += (int64_t)gridDim.x * kThreads)
    sample_px<T, INTERP>(ij[p], ij[ij_sn + p], src, n, src_h, src_w, src_sn, src_sy, dst,
                         dst_sn, p, tfill, bad);
  if (bad) atomicOr(err_flags, XRS_EFLAG_STATE);
}

// ---- K5b: resolve the winning quad of every target pixel ------------------------
// Work item = one tile x kResolveRows target rows (tile fields are block-
// uniform: no per-pixel tile search or 64-bit division); each thread takes one
// column of the item's rows and issues the key loads of all its rows, then the
// winning quads' corner loads of all its rows, before any arithmetic — three
// dependent memory round trips per kResolveRows pixels instead of per pixel.
// 2 rows per thread (items of 128 x 8 target pixels) since late round 6:
// resolve 272-275 vs 277-280 us with 3 (profiles/r06r_k4_grid_strips_ab.log)
constexpr int kResolveRows = 2;

// A variable sampled by the resolve pass itself (K6 fused into K5b: the
// first variable of a rectification needs no ij image round trip through HBM).
struct FusedVar {
  const void* src;
  int64_t n, src_h, src_w, src_sn, src_sy;
  void* dst;
  int64_t dst_sn;
  double fill;
  int interp;      // XRS_INTERP_*
  int write_ij;    // 0: the ij image is not needed by any other variable
};

// K6 of R target pixels (rows p0 + r * pstride) in one batch: positions
// classified, then the taps of every row requested before any is used, then
// the values — sample_px's arithmetic, with R rows' gathers in flight at once
// instead of one dependent chain per row.
template <typename T, int INTERP, int R>
__device__ inline void sample_rows(const double* fi, const double* fj, int nr,
                                   const FusedVar& fv, const T* __restrict__ src,
                                   T* __restrict__ dst, int64_t p0, int64_t pstride, T tfill,
                                   bool& bad) {
  // tap rows / columns as int32 (src_h, src_w < 2^31: checked at launch);
  // the 64-bit offsets are formed at the loads
  int32_t ti0[R], ti1[R], tj0[R], tj1[R];
  double u[R], v[R];
  bool ok[R];
  const int64_t imax = fv.src_w - 1, jmax = fv.src_h - 1;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    ok[r] = false;
    ti0[r] = ti1[r] = tj0[r] = tj1[r] = 0;
    u[r] = v[r] = 0.0;
    if (r >= nr || fi[r] != fi[r] || fj[r] != fj[r]) continue;
    if (!(fi[r] >= 0.0 && fi[r] < (double)fv.src_w && fj[r] >= 0.0 && fj[r] < (double)fv.src_h)) {
      bad = true;
      continue;
    }
    // int() truncation of values in [0, src_w) / [0, src_h), both < 2^31
    // (checked at launch): 32-bit conversions
    int32_t i0 = (int32_t)fi[r], j0 = (int32_t)fj[r];
    u[r] = fi[r] - (double)i0;
    v[r] = fj[r] - (double)j0;
    ok[r] = true;
    if (INTERP == XRS_INTERP_NEAREST) {
      if (u[r] > 0.5) i0 = (int32_t)min(max((int64_t)i0 + 1, (int64_t)0), imax);
      if (v[r] > 0.5) j0 = (int32_t)min(max((int64_t)j0 + 1, (int64_t)0), jmax);
    } else {
      ti1[r] = (int32_t)min(max((int64_t)i0 + 1, (int64_t)0), imax);
      tj1[r] = (int32_t)min(max((int64_t)j0 + 1, (int64_t)0), jmax);
    }
    ti0[r] = i0;
    tj0[r] = j0;
  }
  for (int64_t s = 0; s < fv.n; ++s) {
    const T* S = src + s * fv.src_sn;
    T t00[R], t01[R], t10[R], t11[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {   // rows without a sample read element 0
      const T* s0 = S + (int64_t)tj0[r] * fv.src_sy;
      t00[r] = s0[ti0[r]];
      if (INTERP != XRS_INTERP_NEAREST) {
        const T* s1 = S + (int64_t)tj1[r] * fv.src_sy;
        t01[r] = s0[ti1[r]];
        t10[r] = s1[ti0[r]];
        t11[r] = s1[ti1[r]];
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r >= nr) break;
      T out = tfill;
      if (ok[r]) {
        if (INTERP == XRS_INTERP_NEAREST) {
          out = t00[r];
        } else {
          const double v00 = (double)t00[r], v01 = (double)t01[r];
          const double v10 = (double)t10[r], v11 = (double)t11[r];
          double val;
          if (INTERP == XRS_INTERP_TRIANGULAR) {
            if (u[r] + v[r] < 1.0)
              val = v00 + u[r] * (v01 - v00) + v[r] * (v10 - v00);
            else
              val = v11 + (1.0 - u[r]) * (v10 - v11) + (1.0 - v[r]) * (v01 - v11);
          } else {
            const double u0 = v00 + u[r] * (v01 - v00);
            const double u1 = v10 + u[r] * (v11 - v10);
            val = u0 + v[r] * (u1 - u0);
          }
          out = Conv<T>::from_f64(val);
        }
      }
      dst[s * fv.dst_sn + p0 + r * pstride] = out;
    }
  }
}

// Seven waves per SIMD with the triangle in the key (TRI: 72 VGPRs, 2 values
// spilled outside the pixel loop), five otherwise.  Round 4 found 5 faster
// than 4 (1.131-1.135 vs 1.156-1.162 ms per config-4 pass,
// profiles/r04_rectify_lb5_ab.log); with 2 rows per thread (late round 6) the
// TRI kernels need 72-77 VGPRs: 7 waves 259-267 vs 275-280 us at 5, 6 waves no
// faster, 8 (7 VGPRs spilled) 333 us (profiles/r06s_*, r06t_*).
template <typename T, bool FUSE, int INTERP, bool TRI>   // TRI: a.tri_bit (compile time)
__global__ void __launch_bounds__(kThreads, TRI ? 7 : 5)
rectify_resolve_kernel(RectArgs a, FusedVar fv) {
  const int64_t n = a.dst_h * a.dst_w;
  const T tfill = FUSE ? Conv<T>::from_f64(fv.fill) : T{};
  // tile 0 has the full tile height (edge tiles are shorter)
  // 2-D items: 128 columns x 4 waves x kResolveRows rows (a compact target
  // patch, whose quads lie in a compact source patch: its corner rows are
  // shared by the block's own waves instead of by bands on other XCDs)
  constexpr int kSegW = 128, kBandH = 4 * kResolveRows;
  const int64_t segs = (a.tiles[0].tw + kSegW - 1) / kSegW;
  const int64_t bands = (a.tiles[0].th + kBandH - 1) / kBandH;
  const int64_t nitems = a.ntiles * bands * segs;
  const double inv_w = 1.0 / (double)a.w;
  bool bad = false;
  for (int64_t it = blockIdx.x; it < nitems; it += gridDim.x) {
    const int64_t t = it / (bands * segs);
    const int64_t rem = it - t * bands * segs;
    const int64_t band = rem / segs, seg = rem - band * segs;
    const int32_t rb = (int32_t)band * kBandH + (int32_t)(threadIdx.x >> 6) * kResolveRows;
    const TileInfo ti = a.tiles[t];
    if (!tile_ok(a, ti)) {   // block-uniform
      bad = true;
      continue;
    }
    if (rb >= ti.th || seg * kSegW >= ti.tw) continue;   // wave-uniform
    const int32_t nr = min(kResolveRows, ti.th - rb);
    // a thread's columns di, di + kThreads of the item in pairs: the second
    // column's keys are requested with the first's, so their round trip is
    // hidden behind the first column's quads and arithmetic
    auto column = [&](int32_t di, uint32_t (&key)[kResolveRows]) {
      const int64_t p0 = (int64_t)(ti.r0 + rb) * a.dst_w + ti.c0 + di;
      Quad Q[kResolveRows];
      int32_t qj[kResolveRows], qi[kResolveRows];   // < 2^31: h * w < 2^32 checked
      bool tri_b[kResolveRows];   // tri_bit: the claim found the reference's triangle B
#pragma unroll
      for (int r = 0; r < kResolveRows; ++r) {
        tri_b[r] = false;
        if (key[r] != 0xFFFFFFFFu) {
          if (TRI) {
            tri_b[r] = (key[r] & 1u) != 0;
            key[r] >>= 1;
          }
          int64_t j, i;
          if (a.key_shift > 0) {   // (qj << key_shift) | qi (uniform branch)
            j = key[r] >> a.key_shift;
            i = key[r] & (a.key_mul - 1u);
          } else {
            // key / w through the reciprocal, corrected to the exact quotient
            // (key < 2^32: a 32-bit conversion, not the long int64 sequence)
            j = (int64_t)(uint32_t)((double)key[r] * inv_w);
            i = (int64_t)key[r] - j * a.w;
            if (i < 0) { --j; i += a.w; } else if (i >= a.w) { ++j; i -= a.w; }
          }
          // a key that is no quad's (inconsistent inputs) is reported and
          // dropped; selects, not a branch: the corner loads of all rows stay
          // in flight together
          const bool ok = j >= 0 && j <= a.h - 2 && i >= 0 && i <= a.w - 2;
          bad |= !ok;
          key[r] = ok ? key[r] : 0xFFFFFFFFu;
          qj[r] = ok ? (int32_t)j : 0;
          qi[r] = ok ? (int32_t)i : 0;
          Q[r] = load_quad(a, qj[r], qi[r]);
        }
      }
      double fi[kResolveRows], fj[kResolveRows];   // the rows' source positions
#pragma unroll
      for (int r = 0; r < kResolveRows; ++r) {
        fi[r] = NAN;
        fj[r] = NAN;
        if (r >= nr) break;
        double oi = NAN, oj = NAN;
        if (key[r] != 0xFFFFFFFFu) {
          const int32_t dj = rb + r;
          const double dy = ti.y_off + ((double)dj + 0.5) * a.y_scale;
          const double dx = ti.x_off + ((double)di + 0.5) * a.x_scale;
          double cu, cv;
          int tri;
          if (TRI) {
            // the claim decided the reference's triangle: evaluate that one
            // only (rectify.py:556-573), its corners chosen by selects
            tri = tri_b[r] ? 2 : 1;
            tri_uv(Q[r], tri_b[r], dx, dy, cu, cv);
          } else {
            double det_a, det_b;
            quad_dets(Q[r], det_a, det_b);
            tri = quad_hit(a, Q[r], dx, dy, det_a, det_b, cu, cv);
          }
          if (tri) {
            // tile-local quad (|li|, |lj| < 2^31: int32 -> double converts in
            // one instruction, int64 -> double takes several)
            const int32_t li = qi[r] - ti.si0, lj = qj[r] - ti.sj0;
            double src_i, src_j;
            if (tri == 1) {
              src_i = (double)li + cu;                                 // src_i0 + clamp(u)
              src_j = (double)lj + cv;
            } else {
              src_i = (double)(li + 1) - cu;                           // src_i1 - clamp(u)
              src_j = (double)(lj + 1) - cv;
            }
            oi = (double)ti.si0 + src_i;                               // src_i_min + src_i
            oj = (double)ti.sj0 + src_j;
          }
        }
        const int64_t p = p0 + r * a.dst_w;
        if (!FUSE || fv.write_ij) {
          a.ij[p] = oi;
          a.ij[n + p] = oj;
        }
        fi[r] = oi;
        fj[r] = oj;
      }
      if constexpr (FUSE) {
        // the rows' samples: every row's taps in flight together
        const T* src = static_cast<const T*>(fv.src);
        T* dst = static_cast<T*>(fv.dst);
        sample_rows<T, INTERP, kResolveRows>(fi, fj, nr, fv, src, dst, p0, a.dst_w, tfill,
                                             bad);
      }
    };
    {
      const int32_t d0 = (int32_t)seg * kSegW + (int32_t)(threadIdx.x & 63);
      const int32_t d1 = d0 + 64;
      const bool has0 = d0 < ti.tw, has1 = d1 < ti.tw;
      const int64_t q0 = (int64_t)(ti.r0 + rb) * a.dst_w + ti.c0 + d0;
      uint32_t key0[kResolveRows], key1[kResolveRows];
#pragma unroll
      for (int r = 0; r < kResolveRows; ++r) {
        key0[r] = r < nr && has0 ? a.keys[q0 + r * a.dst_w] : 0xFFFFFFFFu;
        key1[r] = r < nr && has1 ? a.keys[q0 + 64 + r * a.dst_w] : 0xFFFFFFFFu;
      }
      if (has0) column(d0, key0);
      if (has1) column(d1, key1);
    }
  }
  if (bad) atomicOr(a.err_flags, XRS_EFLAG_STATE);
}


// ---- per-tile records + chunk offsets from the K4 accumulators ---------------
// Mirrors the host tiling (rectify.py:312-419 via base.py:565-629 and
// bboxes.py:90-106): ij bbox = [min i, min j, max i + 1, max j + 1] widened by
// ij_border and clipped, source window = [i_min, min(i_max + 1, w)), target
// offsets dst_x_min + c0 * res (python float arithmetic, no contraction).
// One block: records in parallel, then an exclusive scan of the per-tile
// strip counts (kStripH x kStripW quads).
__global__ void __launch_bounds__(kThreads)
rectify_tiles_kernel(const int32_t* __restrict__ acc, int64_t ntx, int64_t nty, int64_t tw,
                     int64_t th, int64_t dst_w, int64_t dst_h, int64_t src_w, int64_t src_h,
                     int64_t ij_border, double x_min, double y_min, double y_max,
                     double x_res, double y_res, int j_up, TileInfo* __restrict__ tiles,
                     int64_t* __restrict__ offs) {
  __shared__ int64_t part[kThreads];
  const int64_t n = ntx * nty;
  int64_t carry = 0;
  for (int64_t base = 0; base < n; base += kThreads) {
    const int64_t t = base + threadIdx.x;
    int64_t nch = 0;
    if (t < n) {
      const int64_t ty = t / ntx, tx = t - ty * ntx;
      TileInfo ti;
      ti.r0 = (int32_t)(ty * th);
      ti.c0 = (int32_t)(tx * tw);
      ti.th = (int32_t)min(th, dst_h - ty * th);
      ti.tw = (int32_t)min(tw, dst_w - tx * tw);
      int64_t i0 = -1, j0 = -1, i1 = -1, j1 = -1;
      if (acc[4 * t + 2] >= 0) {
        i0 = acc[4 * t + 0]; j0 = acc[4 * t + 1];
        i1 = (int64_t)acc[4 * t + 2] + 1; j1 = (int64_t)acc[4 * t + 3] + 1;
        if (ij_border != 0) {
          i0 = max(i0 - ij_border, (int64_t)0);
          j0 = max(j0 - ij_border, (int64_t)0);
          i1 = min(i1 + ij_border, src_w);
          j1 = min(j1 + ij_border, src_h);
        }
      }
      const bool none = i0 == -1;
      ti.si0 = (int32_t)(none ? -1 : i0);
      ti.sj0 = (int32_t)(none ? -1 : j0);
      ti.swin = (int32_t)(none ? 0 : min(i1 + 1, src_w) - i0);
      ti.shin = (int32_t)(none ? 0 : min(j1 + 1, src_h) - j0);
      ti.x_off = x_min + (double)ti.c0 * x_res;
      ti.y_off = j_up ? y_min + (double)ti.r0 * y_res : y_max - (double)ti.r0 * y_res;
      tiles[t] = ti;
      const int64_t nqi = none ? 0 : max((int64_t)ti.swin - 1, (int64_t)0);
      const int64_t nqj = none ? 0 : max((int64_t)ti.shin - 1, (int64_t)0);
      nch = ((nqi + kStripW - 1) / kStripW) * ((nqj + kStripH - 1) / kStripH);
    }
    // inclusive scan of nch over the block (Hillis-Steele in LDS)
    part[threadIdx.x] = nch;
    __syncthreads();
    for (int o = 1; o < kThreads; o <<= 1) {
      const int64_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    if (t < n) offs[t] = carry + part[threadIdx.x] - nch;
    carry += part[kThreads - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) offs[n] = carry;
}

}  // namespace
}  // namespace xrs

extern "C" int xrs_rectify_tiles(const int32_t* acc, int64_t ntiles_x, int64_t ntiles_y,
                                 int64_t tile_w, int64_t tile_h, int64_t dst_w, int64_t dst_h,
                                 int64_t src_w, int64_t src_h, int64_t ij_border,
                                 double dst_x_min, double dst_y_min, double dst_y_max,
                                 double dst_x_res, double dst_y_res, int j_axis_up, void* tiles,
                                 int64_t* chunk_offsets, void* stream) {
  using namespace xrs;
  if (!acc || !tiles || !chunk_offsets || ntiles_x < 1 || ntiles_y < 1 || tile_w < 1 ||
      tile_h < 1 || dst_w < 1 || dst_h < 1 || src_w < 1 || src_h < 1 || ij_border < 0 ||
      (ntiles_x - 1) * tile_w >= dst_w || (ntiles_y - 1) * tile_h >= dst_h) {
    xrs_set_error("xrs_rectify_tiles: invalid argument");
    return XRS_ERR_ARG;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(rectify_tiles_kernel, dim3(1), dim3(kThreads), 0, st, acc, ntiles_x,
                     ntiles_y, tile_w, tile_h, dst_w, dst_h, src_w, src_h, ij_border, dst_x_min,
                     dst_y_min, dst_y_max, dst_x_res, dst_y_res, j_axis_up,
                     static_cast<TileInfo*>(tiles), chunk_offsets);
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

extern "C" int xrs_ij_bboxes_fill(const double* x, const double* y, int64_t h, int64_t w,
                                  int64_t sy, int64_t nboxes, int64_t ntx, int64_t nty,
                                  const double* bx, const double* by, int32_t* acc,
                                  uint32_t* fill, int64_t fill_words, void* stream) {
  using namespace xrs;
  if (!x || !y || !bx || !acc || h < 1 || w < 1 || sy < w || nboxes < 0 ||
      (ntx > 0 && (ntx * nty != nboxes || !by)) || h * w > INT32_MAX || fill_words < 0 ||
      (fill_words > 0 && (!fill || (reinterpret_cast<uintptr_t>(fill) & 15) != 0))) {
    xrs_set_error("xrs_ij_bboxes: invalid argument");
    return XRS_ERR_ARG;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (nboxes == 0) {
    if (fill_words > 0)
      XRS_HIP_CHECK(hipMemsetAsync(fill, 0xFF, (size_t)fill_words * sizeof(uint32_t), st));
    return XRS_OK;
  }
  BBoxArgs a{x, y, h, w, sy, nboxes, ntx, nty, bx, by, acc, fill_words > 0 ? fill : nullptr,
             fill_words};
  const int nb = grid_blocks(h * w, kThreads, 256 * 8);
  const int64_t chunk = ((h * w + nb - 1) / nb + kThreads - 1) / kThreads * kThreads;
  const int64_t lds = (ntx > 0 ? 16 * (ntx + nty) : 32 * nboxes) + 16 * nboxes;
  if (ntx > 0) {   // a tile grid: block-wise (ij_bboxes_block_kernel)
    const int64_t nwave = ((w + 63) / 64) * ((h + kBoxBlockRows - 1) / kBoxBlockRows);
    // as many blocks as are resident at once: each wave walks its blocks in
    // turn (a grid of twice that — 2048 blocks — left a tail of waves with
    // one block more: K4 95-98 vs 101-102 us at config 4, r06q / r06r)
    const bool shared = lds <= 48 * 1024;
    const int nres = resident_blocks(shared ? reinterpret_cast<const void*>(ij_bboxes_block_kernel<true>)
                                            : reinterpret_cast<const void*>(ij_bboxes_block_kernel<false>),
                                     kThreads, shared ? (size_t)lds : 0);
    const int nbb = grid_blocks(nwave, kThreads / 64, nres);
    if (shared)
      hipLaunchKernelGGL(ij_bboxes_block_kernel<true>, dim3(nbb), dim3(kThreads), (size_t)lds, st,
                         a);
    else
      hipLaunchKernelGGL(ij_bboxes_block_kernel<false>, dim3(nbb), dim3(kThreads), 0, st, a);
    XRS_HIP_CHECK(hipGetLastError());
    return XRS_OK;
  }
  if (lds <= 48 * 1024)
    hipLaunchKernelGGL(ij_bboxes_kernel<true>, dim3(nb), dim3(kThreads), (size_t)lds, st, a,
                       chunk);
  else
    hipLaunchKernelGGL(ij_bboxes_kernel<false>, dim3(nb), dim3(kThreads), 0, st, a, chunk);
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

extern "C" int xrs_ij_bboxes(const double* x, const double* y, int64_t h, int64_t w,
                             int64_t sy, int64_t nboxes, int64_t ntx, int64_t nty,
                             const double* bx, const double* by, int32_t* acc, void* stream) {
  return xrs_ij_bboxes_fill(x, y, h, w, sy, nboxes, ntx, nty, bx, by, acc, nullptr, 0, stream);
}

namespace xrs {
namespace {
int rectify_ij_impl(const char* what, const double* x, const double* y, int64_t h, int64_t w,
                    int64_t sy, const void* tiles, int64_t ntiles, const int64_t* chunk_offsets,
                    int64_t max_chunks, int64_t dst_h, int64_t dst_w, double x_scale,
                    double y_scale, double uv_delta, uint32_t* keys, int keys_ready,
                    double* ij, int32_t* err_flags, const FusedVar* fv, int fv_dtype,
                    hipStream_t st) {
  if (!x || !y || !tiles || !keys || (!ij && !(fv && !fv->write_ij)) || !err_flags || h < 2 ||
      w < 2 || sy < w || ntiles < 1 || dst_h < 1 || dst_w < 1 || h * w >= (int64_t)UINT32_MAX ||
      !chunk_offsets || max_chunks < 0 || dst_h > INT32_MAX || dst_w > INT32_MAX) {
    xrs_set_error("%s: invalid argument", what);
    return XRS_ERR_ARG;
  }
  RectArgs a;
  a.x = x; a.y = y; a.h = h; a.w = w; a.sy = sy;
  a.tiles = static_cast<const TileInfo*>(tiles); a.ntiles = ntiles;
  a.chunk_offs = chunk_offsets;
  a.dst_h = dst_h; a.dst_w = dst_w; a.x_scale = x_scale; a.y_scale = y_scale;
  a.uv_delta = uv_delta; a.keys = keys; a.ij = ij; a.err_flags = err_flags;
  a.inv_x = 1.0 / x_scale; a.inv_y = 1.0 / y_scale;
  // tests: xrs_testing_set(XRS_TESTING_RECTIFY_EXACT, 1) takes the exact
  // divisions for every decision
  const bool exact = xrs_testing_value(XRS_TESTING_RECTIFY_EXACT) != 0;
  a.margin = exact ? INFINITY : kMargin;
  // tests: xrs_testing_set(XRS_TESTING_RECTIFY_MARGIN, k) widens the form
  // margin k-fold (more pixels take the exact test; same decisions)
  const int64_t widen = xrs_testing_value(XRS_TESTING_RECTIFY_MARGIN);
  a.margin_scale = widen > 1 ? (float)widen : 1.0f;
  a.narrow = (dst_h * dst_w < ((int64_t)1 << 30) && dst_w < ((int64_t)1 << 24)) ? 1 : 0;
  // tests: xrs_testing_set(XRS_TESTING_RECTIFY_PLAIN_KEYS, 1) takes the
  // plain-key path of very large swaths on any input
  a.tri_bit = h * w < ((int64_t)1 << 31) &&
              xrs_testing_value(XRS_TESTING_RECTIFY_PLAIN_KEYS) == 0 ? 1 : 0;
  // shifted raster keys when (h << b) fits the key (2^b >= w; the same order
  // as qj * w + qi); the plain-key test knob keeps the division decode too
  {
    int b = 1;
    while (((int64_t)1 << b) < w) ++b;
    const int64_t limit = a.tri_bit ? ((int64_t)1 << 31) : (int64_t)UINT32_MAX;
    a.key_shift = (h << b) <= limit && xrs_testing_value(XRS_TESTING_RECTIFY_PLAIN_KEYS) == 0
                      ? b : 0;
    a.key_mul = a.key_shift > 0 ? (uint32_t)1 << b : (uint32_t)w;
  }
  if (!keys_ready)   // else filled by K4 (xrs_ij_bboxes_fill) or the caller
    XRS_HIP_CHECK(hipMemsetAsync(keys, 0xFF, (size_t)(dst_h * dst_w) * sizeof(uint32_t), st));
  {
    // the walk (kCompactRatio); tests: xrs_testing_set(XRS_TESTING_RECTIFY_COMPACT,
    // 1 / 2) takes the compacted / the per-lane walk whatever the ratio
    const int64_t force = xrs_testing_value(XRS_TESTING_RECTIFY_COMPACT);
    const bool compact = force == 1 ||
        (force != 2 && (double)dst_h * (double)dst_w >= kCompactRatio * (double)(h - 1) * (double)(w - 1));
    // the grid: the compacted walk on as many blocks as are resident at once;
    // the per-lane walk on kClaimGridMul times that, so that the strips (dealt
    // round-robin to the waves) come one per wave and the dispatcher balances
    // the CUs instead of a resident wave's fixed share of 4-5 strips (config
    // 4: claim 466-472 vs 505 us, profiles/r06v_*, r06w_*; 2x slower than
    // resident, 4x 482 us; the compacted walk slower off the resident grid);
    // fewer blocks when the caller knows a smaller strip count
    constexpr int wpb = kClaimThreads / 64;
    static const int resident[2] = {   // one device model per process
        resident_blocks(reinterpret_cast<const void*>(rectify_claim_kernel<true, false, false>),
                        kClaimThreads),
        resident_blocks(reinterpret_cast<const void*>(rectify_claim_kernel<true, false, true>),
                        kClaimThreads)};
    const bool ypos = y_scale > 0, lds = ntiles <= kClaimOffsLds;
    auto launch = [&](auto mode) {
      constexpr bool C = decltype(mode)::value;
      const int64_t cap = (int64_t)resident[C] * (C ? 1 : kClaimGridMul);
      const int64_t want = max_chunks > 0 ? (max_chunks + wpb - 1) / wpb : cap;
      const int nb = (int)min(want, cap);
      if (lds && ypos)
        hipLaunchKernelGGL((rectify_claim_kernel<true, true, C>), dim3(nb), dim3(kClaimThreads), 0, st, a);
      else if (lds)
        hipLaunchKernelGGL((rectify_claim_kernel<true, false, C>), dim3(nb), dim3(kClaimThreads), 0, st, a);
      else if (ypos)
        hipLaunchKernelGGL((rectify_claim_kernel<false, true, C>), dim3(nb), dim3(kClaimThreads), 0, st, a);
      else
        hipLaunchKernelGGL((rectify_claim_kernel<false, false, C>), dim3(nb), dim3(kClaimThreads), 0, st, a);
    };
    if (compact)
      launch(std::true_type{});
    else
      launch(std::false_type{});
    XRS_HIP_CHECK(hipGetLastError());
  }
  // 16384 blocks (items of 128 x 8 pixels dealt grid-stride; config 4: ~2.7
  // items per block): resolve 259 vs 267 us with 8192, 4096 280, 32768 260,
  // 65536 271 (profiles/r06t_*, r06u_*)
  const int nb2 = grid_blocks(256 * 64, 1, 1 << 24);
  auto resolve = [&](auto tri) -> int {
    constexpr bool TRI = decltype(tri)::value;
    if (!fv) {
      hipLaunchKernelGGL((rectify_resolve_kernel<uint8_t, false, XRS_INTERP_NEAREST, TRI>),
                         dim3(nb2), dim3(kThreads), 0, st, a, FusedVar{});
      return XRS_OK;
    }
    return dispatch_dtype(fv_dtype, [&](auto tag) -> int {
      using T = decltype(tag);
      if (fv->interp == XRS_INTERP_NEAREST)
        hipLaunchKernelGGL((rectify_resolve_kernel<T, true, XRS_INTERP_NEAREST, TRI>), dim3(nb2),
                           dim3(kThreads), 0, st, a, *fv);
      else if (fv->interp == XRS_INTERP_TRIANGULAR)
        hipLaunchKernelGGL((rectify_resolve_kernel<T, true, XRS_INTERP_TRIANGULAR, TRI>),
                           dim3(nb2), dim3(kThreads), 0, st, a, *fv);
      else
        hipLaunchKernelGGL((rectify_resolve_kernel<T, true, XRS_INTERP_BILINEAR, TRI>),
                           dim3(nb2), dim3(kThreads), 0, st, a, *fv);
      return XRS_OK;
    });
  };
  {
    const int rc = a.tri_bit ? resolve(std::true_type{}) : resolve(std::false_type{});
    if (rc != XRS_OK) {
      xrs_set_error("%s: unsupported variable dtype %d", what, fv_dtype);
      return XRS_ERR_ARG;
    }
  }
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}
}  // namespace
}  // namespace xrs

extern "C" int xrs_rectify_ij(const double* x, const double* y, int64_t h, int64_t w,
                              int64_t sy, const void* tiles, int64_t ntiles, int64_t ntiles_x,
                              const int64_t* chunk_offsets, int64_t max_chunks,
                              int64_t dst_h, int64_t dst_w, double x_scale,
                              double y_scale, double uv_delta, uint32_t* keys,
                              int keys_ready, double* ij, int32_t* err_flags, void* stream) {
  (void)ntiles_x;
  return xrs::rectify_ij_impl("xrs_rectify_ij", x, y, h, w, sy, tiles, ntiles, chunk_offsets,
                              max_chunks, dst_h, dst_w, x_scale, y_scale, uv_delta, keys,
                              keys_ready, ij, err_flags, nullptr, 0,
                              static_cast<hipStream_t>(stream));
}

extern "C" int xrs_rectify_ij_var(const double* x, const double* y, int64_t h, int64_t w,
                                  int64_t sy, const void* tiles, int64_t ntiles,
                                  const int64_t* chunk_offsets, int64_t max_chunks,
                                  int64_t dst_h, int64_t dst_w, double x_scale, double y_scale,
                                  double uv_delta, uint32_t* keys, int keys_ready,
                                  double* ij, const void* src, int src_dtype, int64_t n,
                                  int64_t src_h,
                                  int64_t src_w, int64_t src_sn, int64_t src_sy, void* dst,
                                  int64_t dst_sn, int interp, double fill,
                                  int32_t* err_flags, void* stream) {
  using namespace xrs;
  if (interp != XRS_INTERP_NEAREST && interp != XRS_INTERP_BILINEAR &&
      interp != XRS_INTERP_TRIANGULAR) {
    xrs_set_error("interp_methods must be one of 0, 1, 'nearest', 'bilinear', 'triangular'");
    return XRS_ERR_NOTIMPL;
  }
  if (!src || !dst || n < 1 || src_h < 1 || src_w < 1 || src_sy < src_w ||
      dst_sn < dst_h * dst_w || src_h > INT32_MAX || src_w > INT32_MAX) {
    xrs_set_error("xrs_rectify_ij_var: invalid argument");
    return XRS_ERR_ARG;
  }
  const FusedVar fv{src, n, src_h, src_w, src_sn, src_sy, dst, dst_sn, fill, interp,
                    ij != nullptr ? 1 : 0};
  return rectify_ij_impl("xrs_rectify_ij_var", x, y, h, w, sy, tiles, ntiles, chunk_offsets,
                         max_chunks, dst_h, dst_w, x_scale, y_scale, uv_delta, keys,
                         keys_ready, ij, err_flags, &fv, src_dtype,
                         static_cast<hipStream_t>(stream));
}

extern "C" int xrs_rectify_var(const double* ij, int64_t ij_sn, int64_t dst_h, int64_t dst_w,
                               const void* src,
                               int src_dtype, int64_t n, int64_t src_h, int64_t src_w,
                               int64_t src_sn, int64_t src_sy, void* dst, int64_t dst_sn,
                               int interp, double fill, int32_t* err_flags, void* stream) {
  using namespace xrs;
  if (interp != XRS_INTERP_NEAREST && interp != XRS_INTERP_BILINEAR &&
      interp != XRS_INTERP_TRIANGULAR) {
    xrs_set_error("interp_methods must be one of 0, 1, 'nearest', 'bilinear', 'triangular'");
    return XRS_ERR_NOTIMPL;
  }
  if (!ij || !src || !dst || !err_flags || dst_h < 1 || dst_w < 1 || n < 1 || src_h < 1 || src_w < 1 ||
      src_sy < src_w || dst_sn < dst_h * dst_w || ij_sn < dst_h * dst_w || src_h > INT32_MAX ||
      src_w > INT32_MAX) {
    xrs_set_error("xrs_rectify_var: invalid argument");
    return XRS_ERR_ARG;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nb = grid_blocks(dst_h * dst_w, kThreads, 256 * 8);
  return dispatch_dtype(src_dtype, [&](auto tag) -> int {
    using T = decltype(tag);
    const T* s = static_cast<const T*>(src);
    T* d = static_cast<T*>(dst);
    if (interp == XRS_INTERP_NEAREST)
      hipLaunchKernelGGL((rectify_var_kernel<T, XRS_INTERP_NEAREST>), dim3(nb), dim3(kThreads),
                         0, st, ij, ij_sn, dst_h, dst_w, s, n, src_h, src_w, src_sn, src_sy, d, dst_sn, fill, err_flags);
    else if (interp == XRS_INTERP_TRIANGULAR)
      hipLaunchKernelGGL((rectify_var_kernel<T, XRS_INTERP_TRIANGULAR>), dim3(nb), dim3(kThreads),
                         0, st, ij, ij_sn, dst_h, dst_w, s, n, src_h, src_w, src_sn, src_sy, d, dst_sn, fill, err_flags);
    else
      hipLaunchKernelGGL((rectify_var_kernel<T, XRS_INTERP_BILINEAR>), dim3(nb), dim3(kThreads),
                         0, st, ij, ij_sn, dst_h, dst_w, s, n, src_h, src_w, src_sn, src_sy, d, dst_sn, fill, err_flags);
    XRS_HIP_CHECK(hipGetLastError());
    return XRS_OK;
  });
}
