// xrs_bench.hip — measurement support for bench.py and the diagnostic
// scripts (libxrs_bench.so; never linked into the product libxrs.so).
//
//  * stream_copy: the same-run device-copy rate SURVEY §8(d) asks the headline
//    to be reported against (a streaming float4 copy of the source band:
//    every byte read once, every byte written once — K1's traffic shape).
//    Variants are kept so the fastest can be chosen on the box
//    (scripts/copy_variants.py); bench.py uses XRS_BENCH_COPY_BEST.
//  * clock_probe: the shader clock the chip holds at one moment
//    (MI355X_MICROARCH.md "DVFS give-back" item 6): d(s_memtime) /
//    d(s_memrealtime) x 100 MHz, stamped by one lane of every block around a
//    short VALU loop into a buffer of its own.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(64) clock_probe_kernel(uint64_t* out, int spin) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  float a = (float)threadIdx.x;
  for (int i = 0; i < spin; ++i) a = a * 1.0001f + 0.5f;
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = (r1 - r0) + (a == -1.0f ? 1 : 0);
  }
}

// grid-stride, one 16-byte element per thread and iteration
template <bool NT>
__global__ void __launch_bounds__(256) copy_stride_kernel(const f32x4* __restrict__ src,
                                                          f32x4* __restrict__ dst, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * 256) {
    if (NT) __builtin_nontemporal_store(src[i], &dst[i]);
    else dst[i] = src[i];
  }
}

// one block per 256 x U elements: all U loads in flight before the stores
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_unrolled_kernel(const f32x4* __restrict__ src,
                                                            f32x4* __restrict__ dst, int64_t n4) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  f32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n4) v[u] = src[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n4) {
      if (NT) __builtin_nontemporal_store(v[u], &dst[i]);
      else dst[i] = v[u];
    }
  }
}

// 4-byte lanes (traffic calibration): one block per 256 x U floats, lane l of
// each of the U rounds moves float (round * 256 + l) — every wave instruction
// reads / writes 256 contiguous bytes, the width of K1's dword taps.
template <int U>
__global__ void __launch_bounds__(256) copy_b32_kernel(const float* __restrict__ src,
                                                       float* __restrict__ dst, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  float v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n) v[u] = src[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n) dst[i] = v[u];
  }
}

// XCD-placement probe (diagnostic): block b copies chunk (b / 8) * 8 +
// (b % 8 + shift) % 8 of `chunk` bytes, i.e. rotates which of the 8 XCDs
// (blocks are dealt to them round-robin) moves which chunk of every group of
// 8: a time that depends on `shift` means the memory behind an address is
// nearer to some XCDs than to others at that granularity.
__global__ void __launch_bounds__(256) xcd_copy_kernel(const f32x4* __restrict__ src,
                                                       f32x4* __restrict__ dst, int64_t n4,
                                                       int64_t q, int shift) {
  const int64_t b = blockIdx.x;
  const int64_t c = (b >> 3) * 8 + (((b & 7) + shift) & 7);
  const int64_t base = c * q * 256 + threadIdx.x;
  for (int64_t u = 0; u < q; u += 4) {
    f32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = base + (u + k) * 256;
      if (u + k < q && i < n4) v[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = base + (u + k) * 256;
      if (u + k < q && i < n4) dst[i] = v[k];
    }
  }
}

extern "C" int xrs_bench_xcd_copy(const void* src, void* dst, int64_t bytes, int64_t chunk,
                                  int shift, void* stream) {
  if (bytes % chunk || chunk % 4096 || (bytes / chunk) % 8) return -1;
  const int64_t q = chunk / 4096;   // float4s per thread
  hipLaunchKernelGGL(xcd_copy_kernel, dim3((unsigned)(bytes / chunk)), dim3(256), 0,
                     (hipStream_t)stream, (const f32x4*)src, (f32x4*)dst, bytes / 16, q, shift);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Region copy in K1's work shape (diagnostic): a (rows x cols) f32 image cut
// into items of `band` rows x `segw` columns; one item per block, its float4s
// walked row-major by the 256 threads, RIF loads in flight before their stores.
// order 0: item = blockIdx (all XCDs on neighbouring items); order 1: K1's
// deal (XCD x takes whole bands x, x+8, ...).
template <int RIF, bool NT>
__global__ void __launch_bounds__(256) region_copy_kernel(const float* __restrict__ src,
                                                          float* __restrict__ dst, int64_t cols,
                                                          int64_t segw, int64_t band,
                                                          int64_t nsegs, int64_t nwork,
                                                          int order) {
  extern __shared__ float occupancy_pad[];   // dynamic LDS only limits blocks per CU
  if (threadIdx.x == 1024) occupancy_pad[0] = 0.0f;   // never true: keeps the allocation
  int64_t w = blockIdx.x;
  if (order == 1) {
    const int64_t xcd = blockIdx.x % 8, i = blockIdx.x / 8;
    const int64_t m = i / nsegs;
    w = (m * 8 + xcd) * nsegs + (i - m * nsegs);
  }
  if (w >= nwork) return;
  const int64_t b = w / nsegs, s = w - b * nsegs;
  const int64_t q_row = segw / 4, n = band * q_row;
  const f32x4* sp = (const f32x4*)(src + b * band * cols + s * segw);
  f32x4* dp = (f32x4*)(dst + b * band * cols + s * segw);
  const int64_t c4 = cols / 4;
  for (int64_t j0 = threadIdx.x; j0 < n; j0 += 256 * RIF) {
    f32x4 v[RIF];
#pragma unroll
    for (int u = 0; u < RIF; ++u) {
      const int64_t j = j0 + u * 256;
      if (j < n) v[u] = sp[(j / q_row) * c4 + j % q_row];
    }
#pragma unroll
    for (int u = 0; u < RIF; ++u) {
      const int64_t j = j0 + u * 256;
      if (j < n) {
        f32x4* p = &dp[(j / q_row) * c4 + j % q_row];
        if (NT) __builtin_nontemporal_store(v[u], p);
        else *p = v[u];
      }
    }
  }
}

extern "C" int xrs_bench_region_copy_lds(const void* src, void* dst, int64_t rows, int64_t cols,
                                         int64_t segw, int64_t band, int rif, int nt, int order,
                                         int lds_bytes, void* stream);

extern "C" int xrs_bench_region_copy(const void* src, void* dst, int64_t rows, int64_t cols,
                                     int64_t segw, int64_t band, int rif, int nt, int order,
                                     void* stream) {
  return xrs_bench_region_copy_lds(src, dst, rows, cols, segw, band, rif, nt, order, 0, stream);
}

extern "C" int xrs_bench_region_copy_lds(const void* src, void* dst, int64_t rows, int64_t cols,
                                         int64_t segw, int64_t band, int rif, int nt, int order,
                                         int lds_bytes, void* stream) {
  if (segw % 4 || cols % segw || rows % band || (band * segw / 4) % 64) return -1;
  const int64_t nsegs = cols / segw, nwork = (rows / band) * nsegs;
  const int64_t nb = ((nwork + 7) / 8) * 8;
  hipStream_t st = (hipStream_t)stream;
  const float* s = (const float*)src;
  float* d = (float*)dst;
#define XRS_RC(R, N)                                                                         \
  hipLaunchKernelGGL((region_copy_kernel<R, N>), dim3((unsigned)nb), dim3(256), lds_bytes, st, s, d, \
                     cols, segw, band, nsegs, nwork, order)
  if (rif == 1) { if (nt) XRS_RC(1, true); else XRS_RC(1, false); }
  else if (rif == 2) { if (nt) XRS_RC(2, true); else XRS_RC(2, false); }
  else if (rif == 4) { if (nt) XRS_RC(4, true); else XRS_RC(4, false); }
  else if (rif == 8) { if (nt) XRS_RC(8, true); else XRS_RC(8, false); }
  else return -1;
#undef XRS_RC
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Persistent region copy (diagnostic): items = one row x segw columns in
// raster order, a grid of `nblocks` walks them with stride nblocks (the chip's
// blocks advance over consecutive rows together); each thread moves Q float4
// per item, and the next item's loads are issued before this item's stores.
template <int Q, bool NT>
__global__ void __launch_bounds__(256) persistent_copy_kernel(const float* __restrict__ src,
                                                              float* __restrict__ dst,
                                                              int64_t cols, int64_t nseg,
                                                              int64_t nwork) {
  const int64_t segw = Q * 1024;
  auto addr = [&](int64_t w, int u) {
    const int64_t r = w / nseg, s = w - r * nseg;
    return r * cols + s * segw + (int64_t)(threadIdx.x + u * 256) * 4;
  };
  int64_t w = blockIdx.x;
  if (w >= nwork) return;
  f32x4 v[Q];
#pragma unroll
  for (int u = 0; u < Q; ++u) v[u] = *(const f32x4*)(src + addr(w, u));
  for (; w < nwork; w += gridDim.x) {
    const int64_t wn = w + gridDim.x;
    f32x4 nv[Q];
    if (wn < nwork) {
#pragma unroll
      for (int u = 0; u < Q; ++u) nv[u] = *(const f32x4*)(src + addr(wn, u));
    }
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      f32x4* p = (f32x4*)(dst + addr(w, u));
      if (NT) __builtin_nontemporal_store(v[u], p);
      else *p = v[u];
    }
#pragma unroll
    for (int u = 0; u < Q; ++u) v[u] = nv[u];
  }
}

extern "C" int xrs_bench_persistent_copy(const void* src, void* dst, int64_t rows, int64_t cols,
                                         int q, int nblocks, int nt, void* stream) {
  if (cols % (q * 1024)) return -1;
  const int64_t nseg = cols / (q * 1024), nwork = rows * nseg;
  hipStream_t st = (hipStream_t)stream;
  const float* s = (const float*)src;
  float* d = (float*)dst;
#define XRS_PC(Q, N)                                                                          \
  hipLaunchKernelGGL((persistent_copy_kernel<Q, N>), dim3(nblocks), dim3(256), 0, st, s, d, \
                     cols, nseg, nwork)
  if (q == 1) { if (nt) XRS_PC(1, true); else XRS_PC(1, false); }
  else if (q == 2) { if (nt) XRS_PC(2, true); else XRS_PC(2, false); }
  else if (q == 4) { if (nt) XRS_PC(4, true); else XRS_PC(4, false); }
  else return -1;
#undef XRS_PC
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int xrs_bench_clock_probe(void* out, int blocks, int spin, void* stream) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream,
                     (uint64_t*)out, spin);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// variant: 0 grid-stride nt (4096 blocks), 1 grid-stride plain, 2 unroll-1 plain,
// 3 unroll-4 plain, 4 unroll-4 nt, 5 unroll-8 plain, 6 unroll-8 nt,
// 7 4-byte lanes (8 floats per thread in flight)
extern "C" int xrs_bench_copy(const void* src, void* dst, int64_t bytes, int variant,
                              void* stream) {
  if (bytes % 16 != 0 || ((uintptr_t)src | (uintptr_t)dst) % 16 != 0) return -1;
  const int64_t n4 = bytes / 16;
  const f32x4* s = (const f32x4*)src;
  f32x4* d = (f32x4*)dst;
  hipStream_t st = (hipStream_t)stream;
  auto blocks = [&](int u) { return dim3((unsigned)((n4 + 256 * u - 1) / (256 * u))); };
  switch (variant) {
    case 0: hipLaunchKernelGGL((copy_stride_kernel<true>), dim3(4096), dim3(256), 0, st, s, d, n4); break;
    case 1: hipLaunchKernelGGL((copy_stride_kernel<false>), dim3(4096), dim3(256), 0, st, s, d, n4); break;
    case 2: hipLaunchKernelGGL((copy_unrolled_kernel<1, false>), blocks(1), dim3(256), 0, st, s, d, n4); break;
    case 3: hipLaunchKernelGGL((copy_unrolled_kernel<4, false>), blocks(4), dim3(256), 0, st, s, d, n4); break;
    case 4: hipLaunchKernelGGL((copy_unrolled_kernel<4, true>), blocks(4), dim3(256), 0, st, s, d, n4); break;
    case 5: hipLaunchKernelGGL((copy_unrolled_kernel<8, false>), blocks(8), dim3(256), 0, st, s, d, n4); break;
    case 6: hipLaunchKernelGGL((copy_unrolled_kernel<8, true>), blocks(8), dim3(256), 0, st, s, d, n4); break;
    case 7:
      hipLaunchKernelGGL((copy_b32_kernel<8>), dim3((unsigned)((bytes / 4 + 2047) / 2048)), dim3(256),
                         0, st, (const float*)src, (float*)dst, bytes / 4);
      break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
