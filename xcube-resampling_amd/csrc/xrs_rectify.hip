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

#include "xrs_common.hpp"

namespace xrs {
namespace {

constexpr int kThreads = 256;

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
};

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
// non-increasing): a contiguous run found by two binary searches instead of a
// scan over every tile (NaN -> empty).  Same inclusive compares as the scan.
__device__ inline void monotone_hits(const double* b, int32_t n, double v, int dir,
                                     int32_t& t0, int32_t& t1) {
  int32_t lo = 0, hi = n;   // t0: first t with (dir > 0 ? b_hi >= v : b_lo <= v)
  while (lo < hi) {
    const int32_t m = (lo + hi) >> 1;
    const bool ok = dir > 0 ? b[2 * m + 1] >= v : b[2 * m] <= v;
    if (ok) hi = m; else lo = m + 1;
  }
  t0 = lo;
  lo = 0; hi = n;           // t1 + 1: first t with !(dir > 0 ? b_lo <= v : b_hi >= v)
  while (lo < hi) {
    const int32_t m = (lo + hi) >> 1;
    const bool ok = dir > 0 ? b[2 * m] <= v : b[2 * m + 1] >= v;
    if (ok) lo = m + 1; else hi = m;
  }
  t1 = lo - 1;
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
  // every lane of a wave iterates the same number of times (wave-uniform trip
  // count), so the wave-wide shuffles below always see all 64 lanes
  for (int64_t base = p0; base < p1; base += kThreads) {
    const int64_t idx = base + threadIdx.x;
    const bool valid = idx < p1;
    double x = NAN, y = NAN;
    int32_t i0 = 0, j0 = 0;
    if (valid) {
      j0 = (int32_t)(idx / a.w);
      i0 = (int32_t)(idx - (int64_t)j0 * a.w);
      x = a.x[(int64_t)j0 * a.sy + i0];
      y = a.y[(int64_t)j0 * a.sy + i0];
    }
    int32_t tx0 = 1, tx1 = 0, ty0 = 1, ty1 = 0;
    if (valid && a.ntx > 0) {  // x_min <= x <= x_max, y_min <= y <= y_max (bboxes.py:60-69)
      if (xdir != 0) {
        monotone_hits(bx, (int32_t)a.ntx, x, xdir, tx0, tx1);
      } else {
        for (int32_t t = 0; t < (int32_t)a.ntx; ++t)
          if (bx[2 * t] <= x && x <= bx[2 * t + 1]) { if (tx0 > tx1) tx0 = t; tx1 = t; }
      }
      if (ydir != 0) {
        monotone_hits(by, (int32_t)a.nty, y, ydir, ty0, ty1);
      } else {
        for (int32_t t = 0; t < (int32_t)a.nty; ++t)
          if (by[2 * t] <= y && y <= by[2 * t + 1]) { if (ty0 > ty1) ty0 = t; ty1 = t; }
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
      const int32_t jf = __builtin_amdgcn_readfirstlane(j0);
      if (uni && __builtin_amdgcn_readlane(j0, 63) == jf) {
        // every lane, one source row: lanes hold consecutive pixels, so the
        // extremes are the first and the last lane's
        imin = __builtin_amdgcn_readfirstlane(i0);
        imax = __builtin_amdgcn_readlane(i0, 63);
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
  const int64_t* chunk_offs;   // (ntiles + 1): first 256-quad chunk of each tile
  int64_t dst_h, dst_w;
  double x_scale, y_scale;     // dst_x_res, dst_y_res (negated when j-axis down)
  double uv_delta;
  double inv_x, inv_y;         // 1 / x_scale, 1 / y_scale (claim fast paths)
  double margin;               // relative decision margin (inf: always exact)
  uint32_t* keys;              // (dst_h, dst_w) claim keys, 0xFFFFFFFF = free
  double* ij;                  // (2, dst_h, dst_w) output
};

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

__device__ inline void quad_dets(const Quad& q, double& det_a, double& det_b) {
  det_a = fdet(q.x0, q.y0, q.x1, q.y1, q.x2, q.y2);
  if (det_a != det_a) det_a = 0.0;
  det_b = fdet(q.x3, q.y3, q.x2, q.y2, q.x1, q.y1);
  if (det_b != det_b) det_b = 0.0;
}

// target pixel (column, row) of a source point relative to a tile, as
// np.floor(...).astype(np.int64) (rectify.py:500-501)
__device__ inline int64_t pix_i(const RectArgs& a, const TileInfo& ti, double x) {
  return f64_to_i64_x86(floor((x - ti.x_off) / a.x_scale));
}
__device__ inline int64_t pix_j(const RectArgs& a, const TileInfo& ti, double y) {
  return f64_to_i64_x86(floor((y - ti.y_off) / a.y_scale));
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

__device__ inline int64_t pix_fast(double x, double off, double scale, double inv,
                                   double margin) {
  const double d = x - off;
  const double q = d * inv;
  const double fq = floor(q);
  const double m = margin * (1.0 + fabs(q));
  if (q - fq > m && (fq + 1.0) - q > m) return f64_to_i64_x86(fq);
  return f64_to_i64_x86(floor(d / scale));
}

// triangle test of rectify.py:556-573 (u from fu over the (p0, p2) edge, v
// from fv over (p0, p1)), decided as above; r = 1 / det
__device__ inline bool tri_hit_fast(double dx, double dy, double ox, double oy, double ux,
                                    double uy, double vx, double vy, double det, double r,
                                    double umin, double uvmax, double margin) {
  if (det == 0.0) return false;
  const double nu = fu(dx, dy, ox, oy, ux, uy), nv = fv(dx, dy, ox, oy, vx, vy);
  const double u = nu * r, v = nv * r, s = u + v;
  // |u - nu/det| <= ~3 ulp(u): below 1e-9 for |u| < 1e5, and beyond that u is
  // farther than its error from every limit — an absolute margin suffices
  if (fabs(u - umin) > margin && fabs(v - umin) > margin && fabs(s - uvmax) > margin)
    return u >= umin && v >= umin && s <= uvmax;
  const double ue = nu / det, ve = nv / det;
  return ue >= umin && ve >= umin && ue + ve <= uvmax;
}

// ---- K5a: claim target pixels with the raster-order key of hitting quads -------
// Phase 1, one quad per lane: lanes take consecutive quads of a window row, so
// the right-hand corners (p1, p3) of a quad are the left-hand corners (p0, p2)
// of the next lane's quad and come from it by a shuffle (only the last quad of
// a row or of the wave loads them itself); the quad's clipped target-pixel
// window and determinants are parked in LDS.
// Phase 2, load-balanced: the wave's (quad, window pixel) tests are numbered by
// a wave prefix sum of the window sizes and dealt round-robin to the 64 lanes
// — every lane runs ceil(total / 64) tests instead of the wave running the
// largest window of any lane (quads culled by the tile or degenerate cost
// nothing), each test reading its quad from LDS.
// Work list: chunk c belongs to the tile t with offs[t] <= c < offs[t+1] (the
// offsets come from xrs_rectify_tiles on the device, or from the host); the
// offsets are staged in LDS and searched per chunk.
constexpr int kOffsLds = 2047;   // tiles whose offsets are copied to LDS (16 KB)
constexpr int kQd = 12;          // doubles per staged quad: 8 corners, det_a/b, 1/det_a/b

struct ClaimLds {
  double qd[kThreads / 64][kQd][64];
  int32_t qi[kThreads / 64][4][64];   // imin, jmin, nw, key
  int64_t qs[kThreads / 64][64];      // exclusive start of the quad's tests
};

__global__ void __launch_bounds__(kThreads)
rectify_claim_kernel(RectArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  ClaimLds& L = *reinterpret_cast<ClaimLds*>(smem);
  int64_t* offs_s = reinterpret_cast<int64_t*>(smem + sizeof(ClaimLds));
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool lds_offs = a.ntiles <= kOffsLds;
  if (lds_offs)
    for (int64_t t = threadIdx.x; t <= a.ntiles; t += kThreads) offs_s[t] = a.chunk_offs[t];
  __syncthreads();
  const int64_t* offs = lds_offs ? offs_s : a.chunk_offs;
  const int64_t nchunks = offs[a.ntiles];
  const double umin = -a.uv_delta, uvmax = 1.0 + 2 * a.uv_delta;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    int64_t lo = 0, hi = a.ntiles;   // last t with offs[t] <= c
    while (hi - lo > 1) {
      const int64_t m = (lo + hi) >> 1;
      if (offs[m] <= c) lo = m; else hi = m;
    }
    const TileInfo ti = a.tiles[lo];
    const int32_t nq_i = ti.swin - 1;
    const int64_t q = (c - offs[lo]) * kThreads + threadIdx.x;
    const bool valid = ti.si0 >= 0 && nq_i > 0 && q < (int64_t)nq_i * (int64_t)(ti.shin - 1);
    int32_t lj = 0, li = 0, qj = 0, qi = 0;
    Quad Q{NAN, NAN, NAN, NAN, NAN, NAN, NAN, NAN};
    int64_t pi0 = 0, pj0 = 0, pi2 = 0, pj2 = 0;
    if (valid) {
      lj = (int32_t)(q / nq_i);
      li = (int32_t)(q - (int64_t)lj * nq_i);  // quad within the tile window
      qj = ti.sj0 + lj;
      qi = ti.si0 + li;                        // global quad corner p0
      const int64_t r0 = (int64_t)qj * a.sy, r1 = (int64_t)(qj + 1) * a.sy;
      Q.x0 = a.x[r0 + qi]; Q.y0 = a.y[r0 + qi];
      Q.x2 = a.x[r1 + qi]; Q.y2 = a.y[r1 + qi];
      pi0 = pix_fast(Q.x0, ti.x_off, a.x_scale, a.inv_x, a.margin);
      pj0 = pix_fast(Q.y0, ti.y_off, a.y_scale, a.inv_y, a.margin);
      pi2 = pix_fast(Q.x2, ti.x_off, a.x_scale, a.inv_x, a.margin);
      pj2 = pix_fast(Q.y2, ti.y_off, a.y_scale, a.inv_y, a.margin);
    }
    // right-hand corners from the next lane (all lanes take part in shuffles)
    Q.x1 = __shfl_down(Q.x0, 1, 64); Q.y1 = __shfl_down(Q.y0, 1, 64);
    Q.x3 = __shfl_down(Q.x2, 1, 64); Q.y3 = __shfl_down(Q.y2, 1, 64);
    int64_t pi1 = __shfl_down(pi0, 1, 64), pj1 = __shfl_down(pj0, 1, 64);
    int64_t pi3 = __shfl_down(pi2, 1, 64), pj3 = __shfl_down(pj2, 1, 64);
    int64_t cnt = 0;   // window pixels: up to a whole (untiled) target
    int32_t imin32 = 0, jmin32 = 0, nw = 1;
    double det_a = 0.0, det_b = 0.0;
    if (valid) {
      if (lane == 63 || li + 1 >= nq_i) {      // neighbour lane is not quad (lj, li+1)
        const int64_t r0 = (int64_t)qj * a.sy, r1 = (int64_t)(qj + 1) * a.sy;
        Q.x1 = a.x[r0 + qi + 1]; Q.y1 = a.y[r0 + qi + 1];
        Q.x3 = a.x[r1 + qi + 1]; Q.y3 = a.y[r1 + qi + 1];
        pi1 = pix_fast(Q.x1, ti.x_off, a.x_scale, a.inv_x, a.margin);
        pj1 = pix_fast(Q.y1, ti.y_off, a.y_scale, a.inv_y, a.margin);
        pi3 = pix_fast(Q.x3, ti.x_off, a.x_scale, a.inv_x, a.margin);
        pj3 = pix_fast(Q.y3, ti.y_off, a.y_scale, a.inv_y, a.margin);
      }
      int64_t imin = min(min(pi0, pi1), min(pi2, pi3)), imax = max(max(pi0, pi1), max(pi2, pi3));
      int64_t jmin = min(min(pj0, pj1), min(pj2, pj3)), jmax = max(max(pj0, pj1), max(pj2, pj3));
      if (!(imax < 0 || jmax < 0 || imin >= ti.tw || jmin >= ti.th)) {
        imin = max(imin, (int64_t)0); jmin = max(jmin, (int64_t)0);
        imax = min(imax, (int64_t)ti.tw - 1); jmax = min(jmax, (int64_t)ti.th - 1);
        quad_dets(Q, det_a, det_b);
        if (!(det_a == 0.0 && det_b == 0.0)) {
          imin32 = (int32_t)imin;
          jmin32 = (int32_t)jmin;
          nw = (int32_t)(imax - imin + 1);
          cnt = (int64_t)nw * (jmax - jmin + 1);
        }
      }
    }
    // wave-exclusive prefix sum of the window sizes (int64: a quad with a NaN
    // corner spans its whole tile, rectify.py:500-526, and a tile may be a
    // whole untiled target)
    int64_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int64_t total = __shfl(incl, 63, 64);
    if (total == 0) continue;
    double* qd = &L.qd[wv][0][0];
    int32_t* qs = &L.qi[wv][0][0];
    int64_t* qst = &L.qs[wv][0];
    qd[0 * 64 + lane] = Q.x0; qd[1 * 64 + lane] = Q.y0;
    qd[2 * 64 + lane] = Q.x1; qd[3 * 64 + lane] = Q.y1;
    qd[4 * 64 + lane] = Q.x2; qd[5 * 64 + lane] = Q.y2;
    qd[6 * 64 + lane] = Q.x3; qd[7 * 64 + lane] = Q.y3;
    qd[8 * 64 + lane] = det_a; qd[9 * 64 + lane] = det_b;
    qd[10 * 64 + lane] = det_a != 0.0 ? 1.0 / det_a : 0.0;
    qd[11 * 64 + lane] = det_b != 0.0 ? 1.0 / det_b : 0.0;
    qs[0 * 64 + lane] = imin32; qs[1 * 64 + lane] = jmin32; qs[2 * 64 + lane] = nw;
    qs[3 * 64 + lane] = (int32_t)((int64_t)qj * a.w + qi);
    qst[lane] = incl - cnt;   // exclusive start
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int64_t k = lane; k < total; k += 64) {
      int32_t o = 0;                   // owner: last lane with start <= k
#pragma unroll
      for (int step = 32; step > 0; step >>= 1)
        if (qst[o + step] <= k) o += step;
      // (row, column) of test `local` in the owner's window of w_ columns: the
      // float quotient is within +-1 of local / w_ (window rows < 2^22, checked
      // by xrs_rectify_ij), the integer remainder corrects it exactly
      const int64_t local = k - qst[o];
      const int32_t w_ = qs[2 * 64 + o];
      int64_t q_ = (int64_t)((float)local / (float)w_);
      int64_t r_ = local - q_ * w_;
      if (r_ < 0) { --q_; r_ += w_; }
      else if (r_ >= w_) { ++q_; r_ -= w_; }
      const int32_t di = qs[0 * 64 + o] + (int32_t)r_;
      const int32_t dj = qs[1 * 64 + o] + (int32_t)q_;
      const double x0 = qd[0 * 64 + o], y0 = qd[1 * 64 + o], x1 = qd[2 * 64 + o],
                   y1 = qd[3 * 64 + o], x2 = qd[4 * 64 + o], y2 = qd[5 * 64 + o],
                   x3 = qd[6 * 64 + o], y3 = qd[7 * 64 + o];
      const double dy = ti.y_off + ((double)dj + 0.5) * a.y_scale;
      const double dx = ti.x_off + ((double)di + 0.5) * a.x_scale;
      const bool hit =
          tri_hit_fast(dx, dy, x0, y0, x2, y2, x1, y1, qd[8 * 64 + o], qd[10 * 64 + o], umin,
                       uvmax, a.margin) ||
          tri_hit_fast(dx, dy, x3, y3, x1, y1, x2, y2, qd[9 * 64 + o], qd[11 * 64 + o], umin,
                       uvmax, a.margin);
      if (hit)
        atomicMin(a.keys + (int64_t)(ti.r0 + dj) * a.dst_w + ti.c0 + di,
                  (uint32_t)qs[3 * 64 + o]);
    }
    __builtin_amdgcn_wave_barrier();   // the next chunk rewrites this wave's LDS slots
  }
}

// ---- K5b: resolve the winning quad of every target pixel ------------------------
__global__ void __launch_bounds__(kThreads)
rectify_resolve_kernel(RectArgs a, int64_t ntiles_x) {
  const int64_t n = a.dst_h * a.dst_w;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * kThreads) {
    const uint32_t key = a.keys[p];
    double oi = NAN, oj = NAN;
    if (key != 0xFFFFFFFFu) {
      const int64_t r = p / a.dst_w, c = p - r * a.dst_w;
      const TileInfo& ti0 = a.tiles[0];
      const int64_t t = (r / ti0.th) * ntiles_x + c / ti0.tw;  // tile 0 has the full tile size
      const TileInfo ti = a.tiles[t];
      const int64_t qj = key / a.w, qi = key - qj * a.w;
      const Quad Q = load_quad(a, qj, qi);
      double det_a, det_b;
      quad_dets(Q, det_a, det_b);
      const int64_t dj = r - ti.r0, di = c - ti.c0;
      const double dy = ti.y_off + ((double)dj + 0.5) * a.y_scale;
      const double dx = ti.x_off + ((double)di + 0.5) * a.x_scale;
      double cu, cv;
      const int tri = quad_hit(a, Q, dx, dy, det_a, det_b, cu, cv);
      if (tri) {
        const int64_t li = qi - ti.si0, lj = qj - ti.sj0;   // tile-local quad indices
        double src_i, src_j;
        if (tri == 1) {
          src_i = (double)li + cu;                           // src_i0 + clamp(u)
          src_j = (double)lj + cv;
        } else {
          src_i = (double)(li + 1) - cu;                     // src_i1 - clamp(u)
          src_j = (double)(lj + 1) - cv;
        }
        oi = (double)ti.si0 + src_i;                         // src_i_min + src_i
        oj = (double)ti.sj0 + src_j;
      }
    }
    a.ij[p] = oi;
    a.ij[n + p] = oj;
  }
}

// ---- K6: per-variable sampling (rectify.py:663-734) ------------------------------
template <typename T, int INTERP>
__global__ void __launch_bounds__(kThreads)
rectify_var_kernel(const double* __restrict__ ij, int64_t dst_h, int64_t dst_w,
                   const T* __restrict__ src, int64_t n, int64_t src_h, int64_t src_w,
                   int64_t src_sn, int64_t src_sy, T* __restrict__ dst, int64_t dst_sn,
                   double fill) {
  const int64_t np = dst_h * dst_w;
  const T tfill = Conv<T>::from_f64(fill);
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < np;
       p += (int64_t)gridDim.x * kThreads) {
    const double fi = ij[p], fj = ij[np + p];
    if (fi != fi || fj != fj) {
      for (int64_t s = 0; s < n; ++s) dst[s * dst_sn + p] = tfill;
      continue;
    }
    int64_t i0 = (int64_t)fi, j0 = (int64_t)fj;   // int() truncation (values >= 0)
    const double u = fi - (double)i0, v = fj - (double)j0;
    const int64_t imax = src_w - 1, jmax = src_h - 1;
    if (INTERP == XRS_INTERP_NEAREST) {
      if (u > 0.5) i0 = min(max(i0 + 1, (int64_t)0), imax);
      if (v > 0.5) j0 = min(max(j0 + 1, (int64_t)0), jmax);
      for (int64_t s = 0; s < n; ++s) dst[s * dst_sn + p] = src[s * src_sn + j0 * src_sy + i0];
      continue;
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
}

// ---- per-tile records + chunk offsets from the K4 accumulators ---------------
// Mirrors the host tiling (rectify.py:312-419 via base.py:565-629 and
// bboxes.py:90-106): ij bbox = [min i, min j, max i + 1, max j + 1] widened by
// ij_border and clipped, source window = [i_min, min(i_max + 1, w)), target
// offsets dst_x_min + c0 * res (python float arithmetic, no contraction).
// One block: records in parallel, then an exclusive scan of the per-tile
// 256-quad chunk counts.
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
      const int64_t nq = none ? 0 : max((int64_t)ti.swin - 1, (int64_t)0) *
                                        max((int64_t)ti.shin - 1, (int64_t)0);
      nch = (nq + kThreads - 1) / kThreads;
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

extern "C" int xrs_ij_bboxes(const double* x, const double* y, int64_t h, int64_t w,
                             int64_t sy, int64_t nboxes, int64_t ntx, int64_t nty,
                             const double* bx, const double* by, int32_t* acc, void* stream) {
  using namespace xrs;
  if (!x || !y || !bx || !acc || h < 1 || w < 1 || sy < w || nboxes < 0 ||
      (ntx > 0 && (ntx * nty != nboxes || !by)) || h * w > INT32_MAX) {
    xrs_set_error("xrs_ij_bboxes: invalid argument");
    return XRS_ERR_ARG;
  }
  if (nboxes == 0) return XRS_OK;
  BBoxArgs a{x, y, h, w, sy, nboxes, ntx, nty, bx, by, acc};
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nb = grid_blocks(h * w, kThreads, 256 * 8);
  const int64_t chunk = ((h * w + nb - 1) / nb + kThreads - 1) / kThreads * kThreads;
  const int64_t lds = (ntx > 0 ? 16 * (ntx + nty) : 32 * nboxes) + 16 * nboxes;
  if (lds <= 48 * 1024)
    hipLaunchKernelGGL(ij_bboxes_kernel<true>, dim3(nb), dim3(kThreads), (size_t)lds, st, a,
                       chunk);
  else
    hipLaunchKernelGGL(ij_bboxes_kernel<false>, dim3(nb), dim3(kThreads), 0, st, a, chunk);
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

extern "C" int xrs_rectify_ij(const double* x, const double* y, int64_t h, int64_t w,
                              int64_t sy, const void* tiles, int64_t ntiles, int64_t ntiles_x,
                              const int64_t* chunk_offsets, int64_t max_chunks,
                              int64_t dst_h, int64_t dst_w, double x_scale,
                              double y_scale, double uv_delta, uint32_t* keys, double* ij,
                              void* stream) {
  using namespace xrs;
  if (!x || !y || !tiles || !keys || !ij || h < 2 || w < 2 || sy < w || ntiles < 1 ||
      dst_h < 1 || dst_w < 1 || h * w >= (int64_t)UINT32_MAX || !chunk_offsets || max_chunks < 0 ||
      dst_h >= (1 << 22) || dst_w > INT32_MAX) {
    xrs_set_error("xrs_rectify_ij: invalid argument");
    return XRS_ERR_ARG;
  }
  RectArgs a;
  a.x = x; a.y = y; a.h = h; a.w = w; a.sy = sy;
  a.tiles = static_cast<const TileInfo*>(tiles); a.ntiles = ntiles;
  a.chunk_offs = chunk_offsets;
  a.dst_h = dst_h; a.dst_w = dst_w; a.x_scale = x_scale; a.y_scale = y_scale;
  a.uv_delta = uv_delta; a.keys = keys; a.ij = ij;
  a.inv_x = 1.0 / x_scale; a.inv_y = 1.0 / y_scale;
  // tests: xrs_testing_set(XRS_TESTING_RECTIFY_EXACT, 1) takes the exact
  // divisions for every decision
  a.margin = xrs_testing_value(XRS_TESTING_RECTIFY_EXACT) != 0 ? INFINITY : kMargin;
  hipStream_t st = static_cast<hipStream_t>(stream);
  XRS_HIP_CHECK(hipMemsetAsync(keys, 0xFF, (size_t)(dst_h * dst_w) * sizeof(uint32_t), st));
  {
    // one chunk per block when the caller knows the chunk count, else 16 blocks per CU
    const int nb = max_chunks > 0 ? grid_blocks(max_chunks, 1, 1 << 24)
                                  : grid_blocks(256 * 16, 1, 1 << 24);
    const size_t lds = sizeof(ClaimLds) +
                       (ntiles <= kOffsLds ? (size_t)(ntiles + 1) * sizeof(int64_t) : 0);
    hipLaunchKernelGGL(rectify_claim_kernel, dim3(nb), dim3(kThreads), lds, st, a);
    XRS_HIP_CHECK(hipGetLastError());
  }
  const int nb2 = grid_blocks(dst_h * dst_w, kThreads, 256 * 8);
  hipLaunchKernelGGL(rectify_resolve_kernel, dim3(nb2), dim3(kThreads), 0, st, a, ntiles_x);
  XRS_HIP_CHECK(hipGetLastError());
  return XRS_OK;
}

extern "C" int xrs_rectify_var(const double* ij, int64_t dst_h, int64_t dst_w, const void* src,
                               int src_dtype, int64_t n, int64_t src_h, int64_t src_w,
                               int64_t src_sn, int64_t src_sy, void* dst, int64_t dst_sn,
                               int interp, double fill, void* stream) {
  using namespace xrs;
  if (interp != XRS_INTERP_NEAREST && interp != XRS_INTERP_BILINEAR &&
      interp != XRS_INTERP_TRIANGULAR) {
    xrs_set_error("interp_methods must be one of 0, 1, 'nearest', 'bilinear', 'triangular'");
    return XRS_ERR_NOTIMPL;
  }
  if (!ij || !src || !dst || dst_h < 1 || dst_w < 1 || n < 1 || src_h < 1 || src_w < 1 ||
      src_sy < src_w || dst_sn < dst_h * dst_w) {
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
                         0, st, ij, dst_h, dst_w, s, n, src_h, src_w, src_sn, src_sy, d, dst_sn, fill);
    else if (interp == XRS_INTERP_TRIANGULAR)
      hipLaunchKernelGGL((rectify_var_kernel<T, XRS_INTERP_TRIANGULAR>), dim3(nb), dim3(kThreads),
                         0, st, ij, dst_h, dst_w, s, n, src_h, src_w, src_sn, src_sy, d, dst_sn, fill);
    else
      hipLaunchKernelGGL((rectify_var_kernel<T, XRS_INTERP_BILINEAR>), dim3(nb), dim3(kThreads),
                         0, st, ij, dst_h, dst_w, s, n, src_h, src_w, src_sn, src_sy, d, dst_sn, fill);
    XRS_HIP_CHECK(hipGetLastError());
    return XRS_OK;
  });
}
