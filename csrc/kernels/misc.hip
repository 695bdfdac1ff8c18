// Initial-condition, fill, halo pack/unpack and reduction kernels (gfx950).
//
//  * init_gaussian: device version of the host comprehension at
//    scripts/diffusion_2D_ap.jl:28 (exp of the squared distance to the domain
//    centre, using ImplicitGlobalGrid's x_g/y_g global coordinates).
//  * init_random: synthetic random temperature field (BASELINE.json north
//    star), counter-based and keyed by the global cell index so it is
//    decomposition-invariant.
//  * copy2d: the pack (K7) / unpack (K8) primitive of update_halo!: strided
//    plane <-> contiguous buffer copies, batched (one launch per halo
//    dimension for its packs, one for its unpacks); x-planes of a row-major
//    (ny,nx) field are nx-strided, y-planes are contiguous (sent unpacked).
//  * reduce: sum / max / min / max|.| / non-finite count for verification and
//    NaN guards.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "rma/hip_check.h"
#include "rma/kernels.h"
#include "rma/parallel_for.h"

namespace rma {
namespace {

__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ inline int64_t wrap_index(int64_t g, int64_t n, int periodic) {
  if (!periodic) return g;
  // first local cell of a periodic global grid is a ghost: shift by one.
  int64_t k = (g - 1) % n;
  return k < 0 ? k + n : k;
}

__host__ __device__ inline double global_coord(int64_t g, double d, double off, int64_t n,
                                               int periodic) {
  // ImplicitGlobalGrid x_g: (coords*(nx-ol) + ix-1)*dx + x0, periodic shift.
  double x = (double)g * d + off;
  if (periodic) {
    x = x - d;
    if (x > (double)(n - 1) * d) x = x - (double)n * d;
    if (x < 0) x = x + (double)n * d;
  }
  return x;
}

__host__ __device__ inline double uniform01(uint64_t seed, uint64_t idx) {
  const uint64_t z = mix64(seed + (idx + 1) * 0x9E3779B97F4A7C15ull);
  return (double)(z >> 11) * 0x1.0p-53;
}

__global__ void init_gaussian_kernel(double* __restrict__ T, int64_t nx, int64_t ny, TileGeom g,
                                     double lx, double ly) {
  const int64_t n = nx * ny;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t iy = i / nx, ix = i - iy * nx;
    const double x = global_coord(g.gx0 + ix, g.dx, g.xoff, g.nxg, g.periodx);
    const double y = global_coord(g.gy0 + iy, g.dy, g.yoff, g.nyg, g.periody);
    const double a = (x + g.dx / 2) - lx / 2;
    const double b = (y + g.dy / 2) - ly / 2;
    T[i] = exp(-(a * a) - (b * b));
  }
}

__global__ void init_random_kernel(double* __restrict__ A, int64_t nx, int64_t ny, TileGeom g,
                                   uint64_t seed, double lo, double hi) {
  const int64_t n = nx * ny;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t iy = i / nx, ix = i - iy * nx;
    const int64_t gx = wrap_index(g.gx0 + ix, g.nxg, g.periodx);
    const int64_t gy = wrap_index(g.gy0 + iy, g.nyg, g.periody);
    const double u = uniform01(seed, (uint64_t)(gy * g.nxg + gx));
    A[i] = lo + (hi - lo) * u;
  }
}

__global__ void fill_kernel(double* __restrict__ A, int64_t n, double v) {
  const int64_t n2 = n / 2;
  double2* A2 = reinterpret_cast<double2*>(A);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
       i += (int64_t)gridDim.x * blockDim.x) {
    A2[i] = make_double2(v, v);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) A[n - 1] = v;
}

__global__ void fill_scalar_kernel(double* __restrict__ A, int64_t n, double v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    A[i] = v;
}

struct alignas(16) E16 {
  uint64_t a, b;
};

// Batched strided 2D copy: blockIdx.y selects one of up to kCopy2dBatch copies
// (all packs, or all unpacks, of one halo dimension in one launch). No
// per-element index division: narrow rows (an x-plane row is K fp64) map
// each thread to a fixed (row, column) once and stride over rows; wide rows
// stride blocks over (row, 256-column chunk) with one scalar division per
// 256 elements.
struct Copy2dDev {
  void* dst;
  const void* src;
  int64_t dst_ld, src_ld, n_o, n_k;  // in elements of the launch's E
};
struct Copy2dBatchArgs {
  Copy2dDev c[kCopy2dBatch];
};

constexpr int kCopyBlock = 256;

template <typename E>
__global__ __launch_bounds__(kCopyBlock) void copy2d_batch_kernel(Copy2dBatchArgs b) {
  const Copy2dDev c = b.c[blockIdx.y];
  E* __restrict__ dst = static_cast<E*>(c.dst);
  const E* __restrict__ src = static_cast<const E*>(c.src);
  const unsigned t = threadIdx.x;
  if (c.n_k * 2 <= kCopyBlock) {
    const unsigned nk = (unsigned)c.n_k, R = kCopyBlock / nk;
    if (t >= R * nk) return;
    const unsigned r0 = t / nk, k = t - r0 * nk;
    for (int64_t o = (int64_t)blockIdx.x * R + r0; o < c.n_o; o += (int64_t)gridDim.x * R)
      dst[o * c.dst_ld + k] = src[o * c.src_ld + k];
  } else {
    const int64_t cpr = (c.n_k + kCopyBlock - 1) / kCopyBlock;
    for (int64_t w = blockIdx.x; w < c.n_o * cpr; w += gridDim.x) {
      const int64_t o = w / cpr, k = (w - o * cpr) * kCopyBlock + t;
      if (k < c.n_k) dst[o * c.dst_ld + k] = src[o * c.src_ld + k];
    }
  }
}

constexpr int kRedBlock = 256;
constexpr int kRedMaxBlocks = 1024;
constexpr int kStatsBlocks = 2048;  // field_stats: 3 partials per block

__device__ inline double red_init(int op) {
  switch (op) {
    case kMax: return -INFINITY;
    case kMin: return INFINITY;
    default: return 0.0;
  }
}

__device__ inline double red_map(int op, double v) {
  switch (op) {
    case kMaxAbs: return fabs(v);
    case kNonFinite: return isfinite(v) ? 0.0 : 1.0;
    default: return v;
  }
}

__device__ inline double red_comb(int op, double a, double b) {
  switch (op) {
    case kMax:
    case kMaxAbs: return fmax(a, b);
    case kMin: return fmin(a, b);
    default: return a + b;
  }
}

__device__ double block_reduce(double v, int op) {
  __shared__ double part[kRedBlock / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = red_comb(op, v, __shfl_down(v, off));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) part[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kRedBlock / 64; ++w) v = red_comb(op, v, part[w]);
  }
  return v;
}

__global__ __launch_bounds__(kRedBlock) void reduce_stage1(const double* __restrict__ A, int64_t n,
                                                           int op, double* __restrict__ partial) {
  double v = red_init(op);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    v = red_comb(op, v, red_map(op, A[i]));
  v = block_reduce(v, op);
  if (threadIdx.x == 0) partial[blockIdx.x] = v;
}

__global__ __launch_bounds__(kRedBlock) void reduce_stage2(const double* __restrict__ partial,
                                                           int nparts, int op,
                                                           double* __restrict__ out) {
  // map already applied in stage 1; only combine here (non-finite: sum of counts).
  const int cop = (op == kMaxAbs) ? kMax : (op == kNonFinite ? kSum : op);
  double v = red_init(cop);
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) v = red_comb(cop, v, partial[i]);
  v = block_reduce(v, cop);
  if (threadIdx.x == 0) *out = v;
}

typedef double dbl2 __attribute__((ext_vector_type(2)));

// One-pass field statistics (bench.py full-field check): non-finite count, min
// and max of the finite cells. 16-byte loads, 4 in flight per thread; the three
// per-block partials go to workspace[3*b .. 3*b+2]. Memory-bound: one read of
// the field (an 82 GB T tile in ~13 ms at 6.3 TB/s).
struct Stats3 {
  double bad, lo, hi;
};
__device__ inline void stats_add(Stats3& s, double v) {
  const bool fin = isfinite(v);
  s.bad += fin ? 0.0 : 1.0;
  s.lo = fin ? fmin(s.lo, v) : s.lo;
  s.hi = fin ? fmax(s.hi, v) : s.hi;
}
__device__ Stats3 block_stats(Stats3 s) {
  __shared__ double part[3][kRedBlock / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s.bad += __shfl_down(s.bad, off);
    s.lo = fmin(s.lo, __shfl_down(s.lo, off));
    s.hi = fmax(s.hi, __shfl_down(s.hi, off));
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    part[0][wave] = s.bad;
    part[1][wave] = s.lo;
    part[2][wave] = s.hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kRedBlock / 64; ++w) {
      s.bad += part[0][w];
      s.lo = fmin(s.lo, part[1][w]);
      s.hi = fmax(s.hi, part[2][w]);
    }
  }
  return s;
}
__global__ __launch_bounds__(kRedBlock) void field_stats_stage1(const double* __restrict__ A,
                                                                int64_t n,
                                                                double* __restrict__ partial) {
  Stats3 s{0.0, INFINITY, -INFINITY};
  const bool al = (reinterpret_cast<uintptr_t>(A) & 15) == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t tail = 0;
  if (al) {
    const dbl2* A2 = reinterpret_cast<const dbl2*>(A);
    const int64_t n2 = n / 2;
    for (; i + 3 * stride < n2; i += 4 * stride) {
      dbl2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(A2 + i + u * stride);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        stats_add(s, v[u].x);
        stats_add(s, v[u].y);
      }
    }
    for (; i < n2; i += stride) {
      const dbl2 v = A2[i];
      stats_add(s, v.x);
      stats_add(s, v.y);
    }
    tail = 2 * n2;  // odd n: the last cell, below
    i = tail + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  }
  for (; i < n; i += stride) stats_add(s, A[i]);
  s = block_stats(s);
  if (threadIdx.x == 0) {
    partial[3 * blockIdx.x] = s.bad;
    partial[3 * blockIdx.x + 1] = s.lo;
    partial[3 * blockIdx.x + 2] = s.hi;
  }
}
__global__ __launch_bounds__(kRedBlock) void field_stats_stage2(const double* __restrict__ partial,
                                                                int nparts,
                                                                double* __restrict__ out) {
  Stats3 s{0.0, INFINITY, -INFINITY};
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    s.bad += partial[3 * i];
    s.lo = fmin(s.lo, partial[3 * i + 1]);
    s.hi = fmax(s.hi, partial[3 * i + 2]);
  }
  s = block_stats(s);
  if (threadIdx.x == 0) {
    out[0] = s.bad;
    out[1] = s.lo;
    out[2] = s.hi;
  }
}

// Roofline probes: each thread keeps 4 independent 16-byte loads in flight per
// array (grid-strided so every wave-instruction is one contiguous 1 KiB).
template <bool NT>
__global__ __launch_bounds__(256) void stream_copy_kernel(dbl2* __restrict__ b,
                                                          const dbl2* __restrict__ a, int64_t n2) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    dbl2 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = a[i + k * stride];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (NT) __builtin_nontemporal_store(v[k], b + i + k * stride);
      else b[i + k * stride] = v[k];
    }
  }
  for (; i < n2; i += stride) b[i] = a[i];
}

// one 16-byte element per thread, full grid (the simplest streaming form)
template <bool NT>
__global__ __launch_bounds__(256) void stream_copy_flat(dbl2* __restrict__ b,
                                                        const dbl2* __restrict__ a, int64_t n2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n2) {
    if constexpr (NT) __builtin_nontemporal_store(a[i], b + i);
    else b[i] = a[i];
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void stream_triad_flat(dbl2* __restrict__ c,
                                                         const dbl2* __restrict__ a,
                                                         const dbl2* __restrict__ b, double s,
                                                         int64_t n2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n2) {
    const dbl2 r = a[i] + s * b[i];
    if constexpr (NT) __builtin_nontemporal_store(r, c + i);
    else c[i] = r;
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void stream_triad_kernel(dbl2* __restrict__ c,
                                                           const dbl2* __restrict__ a,
                                                           const dbl2* __restrict__ b, double s,
                                                           int64_t n2) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n2; i += 4 * stride) {
    dbl2 va[4], vb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      va[k] = a[i + k * stride];
      vb[k] = b[i + k * stride];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const dbl2 r = va[k] + s * vb[k];
      if constexpr (NT) __builtin_nontemporal_store(r, c + i + k * stride);
      else c[i + k * stride] = r;
    }
  }
  for (; i < n2; i += stride) c[i] = a[i] + s * b[i];
}

unsigned grid_stride_blocks(int64_t n, int block) {
  int64_t b = (n + block - 1) / block;
  if (b > 256 * 16) b = 256 * 16;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace

void init_gaussian_gpu(double* T, int64_t nx, int64_t ny, const TileGeom& g, double lx, double ly,
                       stream_t stream) {
  RMA_CHECK_ARG(nx > 0 && ny > 0, "empty tile");
  init_gaussian_kernel<<<grid_stride_blocks(nx * ny, 256), 256, 0, as_stream(stream)>>>(T, nx, ny, g,
                                                                                        lx, ly);
  RMA_HIP_LAUNCH_CHECK();
}

void init_random_gpu(double* A, int64_t nx, int64_t ny, const TileGeom& g, uint64_t seed,
                     double lo, double hi, stream_t stream) {
  RMA_CHECK_ARG(nx > 0 && ny > 0, "empty tile");
  init_random_kernel<<<grid_stride_blocks(nx * ny, 256), 256, 0, as_stream(stream)>>>(
      A, nx, ny, g, seed, lo, hi);
  RMA_HIP_LAUNCH_CHECK();
}

void fill_gpu(double* A, int64_t n, double value, stream_t stream) {
  if (n <= 0) return;
  if ((reinterpret_cast<uintptr_t>(A) & 15) == 0)
    fill_kernel<<<grid_stride_blocks(n / 2 + 1, 256), 256, 0, as_stream(stream)>>>(A, n, value);
  else
    fill_scalar_kernel<<<grid_stride_blocks(n, 256), 256, 0, as_stream(stream)>>>(A, n, value);
  RMA_HIP_LAUNCH_CHECK();
}

void copy2d_batch_gpu(const Copy2d* copies, int n, int elem_bytes, stream_t stream) {
  RMA_CHECK_ARG(n >= 0 && n <= kCopy2dBatch, "copy2d batch of " << n << " (max " << kCopy2dBatch << ")");
  RMA_CHECK_ARG(elem_bytes == 2 || elem_bytes == 4 || elem_bytes == 8 || elem_bytes == 16,
                "unsupported element size " << elem_bytes);
  Copy2dBatchArgs a{};
  int m = 0;
  // 8-byte planes whose rows are even and 16-B aligned move as 16-byte
  // elements (a width-K halo of fp64: K/2 dwordx4 per row instead of K)
  bool wide = elem_bytes == 8;
  for (int i = 0; i < n; ++i) {
    const Copy2d& c = copies[i];
    if (c.n_o <= 0 || c.n_k <= 0) continue;
    RMA_CHECK_ARG(c.dst_ld >= c.n_k && c.src_ld >= c.n_k, "leading dims smaller than row length");
    RMA_CHECK_ARG(c.dst && c.src, "null copy2d pointer");
    wide = wide && c.n_k % 2 == 0 && c.dst_ld % 2 == 0 && c.src_ld % 2 == 0 &&
           ((reinterpret_cast<uintptr_t>(c.dst) | reinterpret_cast<uintptr_t>(c.src)) & 15) == 0;
    a.c[m++] = {c.dst, c.src, c.dst_ld, c.src_ld, c.n_o, c.n_k};
  }
  if (m == 0) return;
  if (wide) {
    elem_bytes = 16;
    for (int i = 0; i < m; ++i) {
      a.c[i].dst_ld /= 2;
      a.c[i].src_ld /= 2;
      a.c[i].n_k /= 2;
    }
  }
  int64_t bx = 1;  // blocks along x: what the largest copy can use, capped (grid-stride)
  for (int i = 0; i < m; ++i) {
    const Copy2dDev& c = a.c[i];
    const int64_t need = c.n_k * 2 <= kCopyBlock
                             ? (c.n_o + kCopyBlock / c.n_k - 1) / (kCopyBlock / c.n_k)
                             : c.n_o * ((c.n_k + kCopyBlock - 1) / kCopyBlock);
    bx = std::max(bx, need);
  }
  const dim3 grid((unsigned)std::min<int64_t>(bx, 256 * 8), (unsigned)m);
  hipStream_t s = as_stream(stream);
  switch (elem_bytes) {
    case 2: copy2d_batch_kernel<uint16_t><<<grid, kCopyBlock, 0, s>>>(a); break;
    case 4: copy2d_batch_kernel<uint32_t><<<grid, kCopyBlock, 0, s>>>(a); break;
    case 8: copy2d_batch_kernel<uint64_t><<<grid, kCopyBlock, 0, s>>>(a); break;
    default: copy2d_batch_kernel<E16><<<grid, kCopyBlock, 0, s>>>(a); break;
  }
  RMA_HIP_LAUNCH_CHECK();
}

void copy2d_gpu(void* dst, int64_t dst_ld, const void* src, int64_t src_ld, int64_t n_o,
                int64_t n_k, int elem_bytes, stream_t stream) {
  const Copy2d c{dst, dst_ld, src, src_ld, n_o, n_k};
  copy2d_batch_gpu(&c, 1, elem_bytes, stream);
}

void stream_copy_gpu(double* b, const double* a, int64_t n, int nt, int blocks, stream_t stream) {
  RMA_CHECK_ARG(n % 2 == 0 && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0,
                "stream_copy needs even n and 16-byte aligned buffers");
  if (blocks <= 0) {  // flat: one element per thread
    const unsigned g = (unsigned)((n / 2 + 255) / 256);
    if (nt)
      stream_copy_flat<true><<<g, 256, 0, as_stream(stream)>>>((dbl2*)b, (const dbl2*)a, n / 2);
    else
      stream_copy_flat<false><<<g, 256, 0, as_stream(stream)>>>((dbl2*)b, (const dbl2*)a, n / 2);
  } else if (nt) {
    stream_copy_kernel<true><<<blocks, 256, 0, as_stream(stream)>>>((dbl2*)b, (const dbl2*)a, n / 2);
  } else {
    stream_copy_kernel<false><<<blocks, 256, 0, as_stream(stream)>>>((dbl2*)b, (const dbl2*)a, n / 2);
  }
  RMA_HIP_LAUNCH_CHECK();
}

void stream_triad_gpu(double* c, const double* a, const double* b, double s, int64_t n, int nt,
                      int blocks, stream_t stream) {
  RMA_CHECK_ARG(n % 2 == 0 && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                                reinterpret_cast<uintptr_t>(c)) & 15) == 0,
                "stream_triad needs even n and 16-byte aligned buffers");
  if (blocks <= 0) {
    const unsigned g = (unsigned)((n / 2 + 255) / 256);
    if (nt)
      stream_triad_flat<true><<<g, 256, 0, as_stream(stream)>>>((dbl2*)c, (const dbl2*)a,
                                                                 (const dbl2*)b, s, n / 2);
    else
      stream_triad_flat<false><<<g, 256, 0, as_stream(stream)>>>((dbl2*)c, (const dbl2*)a,
                                                                  (const dbl2*)b, s, n / 2);
  } else if (nt) {
    stream_triad_kernel<true><<<blocks, 256, 0, as_stream(stream)>>>((dbl2*)c, (const dbl2*)a,
                                                                      (const dbl2*)b, s, n / 2);
  } else {
    stream_triad_kernel<false><<<blocks, 256, 0, as_stream(stream)>>>((dbl2*)c, (const dbl2*)a,
                                                                       (const dbl2*)b, s, n / 2);
  }
  RMA_HIP_LAUNCH_CHECK();
}

int64_t reduce_workspace_doubles() { return kRedMaxBlocks; }
int64_t field_stats_workspace_doubles() { return 3 * kStatsBlocks; }

void reduce_gpu(const double* A, int64_t n, int op, double* out, double* workspace,
                stream_t stream) {
  RMA_CHECK_ARG(op >= kSum && op <= kNonFinite, "bad reduce op " << op);
  int64_t nb = (n + kRedBlock * 8 - 1) / (kRedBlock * 8);
  if (nb < 1) nb = 1;
  if (nb > kRedMaxBlocks) nb = kRedMaxBlocks;
  hipStream_t s = as_stream(stream);
  reduce_stage1<<<(unsigned)nb, kRedBlock, 0, s>>>(A, n, op, workspace);
  RMA_HIP_LAUNCH_CHECK();
  reduce_stage2<<<1, kRedBlock, 0, s>>>(workspace, (int)nb, op, out);
  RMA_HIP_LAUNCH_CHECK();
}

void field_stats_gpu(const double* A, int64_t n, double* out3, double* workspace,
                     stream_t stream) {
  RMA_CHECK_ARG(n >= 1, "field_stats of an empty field");
  // 8 blocks (32 waves) per CU keep enough 16-byte loads in flight for HBM
  int64_t nb = (n / 2 + kRedBlock * 4 - 1) / (kRedBlock * 4);
  nb = nb < 1 ? 1 : (nb > kStatsBlocks ? kStatsBlocks : nb);
  hipStream_t s = as_stream(stream);
  field_stats_stage1<<<(unsigned)nb, kRedBlock, 0, s>>>(A, n, workspace);
  RMA_HIP_LAUNCH_CHECK();
  field_stats_stage2<<<1, kRedBlock, 0, s>>>(workspace, (int)nb, out3);
  RMA_HIP_LAUNCH_CHECK();
}

// --------------------------- CPU twins (same formulas) ---------------------
void init_gaussian_cpu(double* T, int64_t nx, int64_t ny, const TileGeom& g, double lx,
                       double ly) {
  parallel_for(0, ny, 16, [&](int64_t iy) {
    const double y = global_coord(g.gy0 + iy, g.dy, g.yoff, g.nyg, g.periody);
    const double b = (y + g.dy / 2) - ly / 2;
    for (int64_t ix = 0; ix < nx; ++ix) {
      const double x = global_coord(g.gx0 + ix, g.dx, g.xoff, g.nxg, g.periodx);
      const double a = (x + g.dx / 2) - lx / 2;
      T[iy * nx + ix] = std::exp(-(a * a) - (b * b));
    }
  });
}

void init_random_cpu(double* A, int64_t nx, int64_t ny, const TileGeom& g, uint64_t seed,
                     double lo, double hi) {
  parallel_for(0, ny, 16, [&](int64_t iy) {
    const int64_t gy = wrap_index(g.gy0 + iy, g.nyg, g.periody);
    for (int64_t ix = 0; ix < nx; ++ix) {
      const int64_t gx = wrap_index(g.gx0 + ix, g.nxg, g.periodx);
      A[iy * nx + ix] = lo + (hi - lo) * uniform01(seed, (uint64_t)(gy * g.nxg + gx));
    }
  });
}

}  // namespace rma
