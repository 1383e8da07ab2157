// xrs_common.hpp — shared device/host helpers for the libxrs HIP kernels (gfx950).
//
// Everything here restates numpy/x86 scalar semantics that the reference's CPU
// path relies on, so the kernels reproduce the reference bit for bit:
//   * float64 -> integer casts follow numpy-on-x86 (cvttsd2si to int32, then
//     keep the low bits; NaN / out-of-range -> INT32_MIN before narrowing),
//   * arithmetic differences of two source values are evaluated in the source
//     dtype (numpy `a - b` on two uint8 arrays wraps, on float32 rounds to f32),
//   * no FMA contraction: the library is compiled with -ffp-contract=off.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/xrs.h"

namespace xrs {

// ---- numpy float64 -> int casts (x86 semantics) -------------------------
// numpy lowers float64 -> {int8,int16,uint8,uint16,int32} through a 32-bit
// truncating conversion (cvttsd2si): NaN and values outside int32 produce the
// "integer indefinite" 0x80000000, which is then narrowed to the target width.
__device__ __host__ inline int32_t f64_to_i32_x86(double x) {
  if (!(x >= -2147483648.0 && x < 2147483648.0)) return INT32_MIN;  // also NaN
  return (int32_t)x;  // truncation toward zero
}
__device__ __host__ inline int64_t f64_to_i64_x86(double x) {
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)x;
}
// numpy float64 -> int16 (reproject.py:282-283,286-289,316-319 index casts)
__device__ __host__ inline int16_t f64_to_i16_np(double x) {
  return (int16_t)(uint16_t)(uint32_t)f64_to_i32_x86(x);
}

template <typename T> struct Conv;
template <> struct Conv<float> {
  __device__ static inline float from_f64(double v) { return (float)v; }
  __device__ static inline double to_f64(float v) { return (double)v; }
  __device__ static inline float diff(float a, float b) { return a - b; }
};
template <> struct Conv<double> {
  __device__ static inline double from_f64(double v) { return v; }
  __device__ static inline double to_f64(double v) { return v; }
  __device__ static inline double diff(double a, double b) { return a - b; }
};
#define XRS_SMALL_INT_CONV(T)                                                  \
  template <> struct Conv<T> {                                                 \
    __device__ static inline T from_f64(double v) {                            \
      return (T)(uint32_t)f64_to_i32_x86(v);                                   \
    }                                                                          \
    __device__ static inline double to_f64(T v) { return (double)v; }         \
    __device__ static inline T diff(T a, T b) { return (T)(a - b); }           \
  };
XRS_SMALL_INT_CONV(uint8_t)
XRS_SMALL_INT_CONV(int8_t)
XRS_SMALL_INT_CONV(uint16_t)
XRS_SMALL_INT_CONV(int16_t)
XRS_SMALL_INT_CONV(int32_t)
#undef XRS_SMALL_INT_CONV
template <> struct Conv<uint32_t> {
  __device__ static inline uint32_t from_f64(double v) {
    return (uint32_t)(uint64_t)f64_to_i64_x86(v);
  }
  __device__ static inline double to_f64(uint32_t v) { return (double)v; }
  __device__ static inline uint32_t diff(uint32_t a, uint32_t b) { return a - b; }
};
template <> struct Conv<int64_t> {
  __device__ static inline int64_t from_f64(double v) { return f64_to_i64_x86(v); }
  __device__ static inline double to_f64(int64_t v) { return (double)v; }
  __device__ static inline int64_t diff(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a - (uint64_t)b);
  }
};

// ---- XCD-contiguous work mapping -----------------------------------------
// Blocks are dealt round-robin over the 8 XCDs (blocks b and b+8 share an L2).
// Each XCD gets one contiguous slice of the row-major work list, walked by its
// blocks in order, so source rows fetched into that XCD's L2 are re-used by the
// next target rows it processes.  Placement affects speed only.
struct XcdSlice {
  int64_t begin, end, step, first;
};
__device__ inline XcdSlice xcd_slice(int64_t nwork) {
  const int64_t nxcd = 8;
  const int64_t b = blockIdx.x, nb = gridDim.x;  // launcher: nb % 8 == 0
  const int64_t xcd = b % nxcd, per = nb / nxcd, lane = b / nxcd;
  const int64_t chunk = (nwork + nxcd - 1) / nxcd;
  XcdSlice s;
  s.begin = xcd * chunk;
  s.end = s.begin + chunk < nwork ? s.begin + chunk : nwork;
  s.step = per;
  s.first = s.begin + lane;
  return s;
}

// Group-interleaved variant: the work list is cut into groups of `group`
// consecutive items and XCD x takes groups x, x + 8, x + 16, ...  For K1 a
// group is one band of target rows across the raster, so every XCD gets the
// same mix of cheap and expensive rows (a contiguous slice per XCD left the
// XCD holding the rows that read the most source rows 6 % behind the others);
// source-row reuse lives inside a work item, not across bands.
struct XcdGroups {
  int64_t xcd, group, nwork, i, step;
  __device__ inline int64_t item() const {
    const int64_t m = i / group;
    return (m * 8 + xcd) * group + (i - m * group);
  }
};
__device__ inline XcdGroups xcd_groups(int64_t nwork, int64_t group) {
  const int64_t b = blockIdx.x, nb = gridDim.x;  // launcher: nb % 8 == 0
  return XcdGroups{b % 8, group, nwork, b / 8, nb / 8};
}

// ---- numpy reduction helpers (K3 / coarsen) --------------------------------
template <typename T> __device__ inline bool is_nan(T v) { return false; }
template <> __device__ inline bool is_nan<float>(float v) { return v != v; }
template <> __device__ inline bool is_nan<double>(double v) { return v != v; }
template <typename T> __device__ inline bool is_finite(T v) { return true; }
template <> __device__ inline bool is_finite<float>(float v) { return v - v == 0.0f; }
template <> __device__ inline bool is_finite<double>(double v) { return v - v == 0.0; }

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

// numpy's full pairwise_sum (loops_utils.h.src): blocks of <= 128 as above,
// longer runs split at n2 = n/2 - (n/2)%8 and the halves summed recursively.
template <typename A, typename F>
__device__ A pairwise_sum(int off, int n, F&& val) {
  if (n <= 128) return pairwise_row<A>(n, [&](int i) { return val(off + i); });
  int n2 = n / 2;
  n2 -= n2 % 8;
  const A lo = pairwise_sum<A>(off, n2, val);
  return lo + pairwise_sum<A>(off + n2, n - n2, val);
}

// numpy add.reduce over the window axes (1, 3) of dask chunk.coarsen's
// (h/dy, dy, w/dx, dx) block, starting from the identity 0: each window row is
// one inner pairwise loop, rows accumulated in order — unless the block is a
// single window wide (chunk width == dx), where nditer coalesces the two axes
// into ONE pairwise loop over all dy*dx values (row-major).
template <typename A, typename F>
__device__ inline A window_sum(bool whole, int ny, int nx, F&& val2d) {
  if (whole) return (A)0.0 + pairwise_sum<A>(0, ny * nx, [&](int i) { return val2d(i / nx, i % nx); });
  A t = (A)0.0;
  for (int r = 0; r < ny; ++r)
    t = t + pairwise_sum<A>(0, nx, [&](int c) { return val2d(r, c); });
  return t;
}

__device__ inline void store_any(void* dst, int64_t idx, int dtype, double fv, int64_t iv,
                                 bool is_int) {
  switch (dtype) {
    // float results are written once and not read back by the kernel:
    // non-temporal stores (config 3's K3i 0.208 -> 0.203 ms,
    // profiles/r04_k3_ab.log)
    case XRS_DTYPE_F32: __builtin_nontemporal_store((float)fv, static_cast<float*>(dst) + idx); break;
    case XRS_DTYPE_F64: __builtin_nontemporal_store(fv, static_cast<double*>(dst) + idx); break;
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

template <typename F>
inline int dispatch_dtype(int dtype, F&& f) {
  switch (dtype) {
    case XRS_DTYPE_U8: return f((uint8_t)0);
    case XRS_DTYPE_I8: return f((int8_t)0);
    case XRS_DTYPE_U16: return f((uint16_t)0);
    case XRS_DTYPE_I16: return f((int16_t)0);
    case XRS_DTYPE_U32: return f((uint32_t)0);
    case XRS_DTYPE_I32: return f((int32_t)0);
    case XRS_DTYPE_I64: return f((int64_t)0);
    case XRS_DTYPE_F32: return f((float)0);
    case XRS_DTYPE_F64: return f((double)0);
    default: return XRS_ERR_ARG;
  }
}

inline int grid_blocks(int64_t nwork, int per_block, int cap) {
  int64_t nb = (nwork + per_block - 1) / per_block;
  if (nb > cap) nb = cap;
  nb = ((nb + 7) / 8) * 8;  // multiple of the XCD count
  if (nb < 8) nb = 8;
  return (int)nb;
}

// Blocks of `kernel` resident on the whole device at once (occupancy per CU x
// CU count), for grids that deal work round-robin and must not leave a tail
// of blocks that start only when others end.
inline int resident_blocks(const void* kernel, int threads, size_t dyn_lds = 0) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, dyn_lds) !=
          hipSuccess)
    return 256 * 4;
  return (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1);
}

// A kernel argument (an arguments struct at byte OFFSET of the kernel-argument
// segment: 0 for the first argument) read again, after `dep` is computed.
// The asm makes the segment address opaque at this point, so the scalar loads
// stay next to their uses: large argument structs kept live across a kernel's
// loop, together with the loop's own uniform values, outnumber the SGPRs, and
// the spilled ones are read back from VGPR lanes (v_readlane, one VALU
// instruction each) on every iteration.
template <typename A, size_t OFFSET = 0>
__device__ inline A kernel_arg_after(double dep) {
#if __HIP_DEVICE_COMPILE__   // (the host pass only parses device functions)
  typedef const __attribute__((address_space(4))) A* ArgPtr;
  uint64_t kp = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr()) + OFFSET;
  asm volatile("" : "+s"(kp) : "v"(dep));
  return *reinterpret_cast<ArgPtr>(kp);
#else
  return A{};
#endif
}

}  // namespace xrs

// Thread-local error message reported through xrs_last_error().
void xrs_set_error(const char* fmt, ...);
// Current value of a test-only path knob (xrs_testing_set, include/xrs.h).
int64_t xrs_testing_value(int knob);

#define XRS_HIP_CHECK(expr)                                                    \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      xrs_set_error("%s failed: %s", #expr, hipGetErrorString(_e));            \
      return XRS_ERR_HIP;                                                      \
    }                                                                          \
  } while (0)
