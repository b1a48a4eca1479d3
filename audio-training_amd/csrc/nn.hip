// Layer kernels around the convolutions of resnet/wr_resnet*.py:
//   BatchNormalization (Keras: axis=3, eps 1e-3, momentum 0.99, batch stats in
//   training, biased variance), ReLU, Add, Dropout, MaxPool2D, AveragePooling2D,
//   log-mean-exp pooling (wr_resnet_bird.py:83-87), GlobalAveragePooling2D,
//   Dense(+sigmoid), BCE / CCE losses (audiomodel.py:1206-1223) and Adam
//   (audiomodel.py:1226-1240, Keras defaults b1 .9, b2 .999, eps 1e-7).
// Activations are NHWC, bf16 or fp32 ("dtype" codes of acfe.h); per-channel
// parameters and statistics are fp32; cross-block reductions go through
// double-precision partial slabs reduced in a fixed order (deterministic).
#include "common.h"

using namespace acfe;

template <typename T> __device__ __forceinline__ float ld(const T* p, long long i);
template <> __device__ __forceinline__ float ld<uint16_t>(const uint16_t* p, long long i) { return bf2f(p[i]); }
template <> __device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <typename T> __device__ __forceinline__ void st(T* p, long long i, float v);
template <> __device__ __forceinline__ void st<uint16_t>(uint16_t* p, long long i, float v) { p[i] = f2bf(v); }
template <> __device__ __forceinline__ void st<float>(float* p, long long i, float v) { p[i] = v; }

#define DISPATCH1(dt, T, ...)                                   \
  do {                                                          \
    if ((dt) == ACFE_DTYPE_BF16) { typedef uint16_t T; __VA_ARGS__; } \
    else { typedef float T; __VA_ARGS__; }                      \
  } while (0)

static int grid_for(long long n, int per = 256, int cap = 8192) {
  long long g = (n + per - 1) / per;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

// Partial-slab row count used by every per-channel reduction below.
static int red_blocks(long long rows) {
  long long b = (rows + 255) / 256;
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}
ACFE_API int acfe_reduce_blocks(long long rows) { return red_blocks(rows); }

// ---------------------------------------------------------------- 8-wide access
// Channel-contiguous NHWC tensors are processed 8 elements per thread (16 B of
// bf16 / 32 B of fp32) when C % 8 == 0 and the buffers are 16-B aligned;
// scalar kernels remain as the fallback.
__device__ __forceinline__ void ld8(const uint16_t* p, float* f) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(w[j] << 16);
    f[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld8(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void st8(uint16_t* p, const float* f) {
  uint4 v;
  v.x = (uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16);
  v.y = (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16);
  v.z = (uint32_t)f2bf(f[4]) | ((uint32_t)f2bf(f[5]) << 16);
  v.w = (uint32_t)f2bf(f[6]) | ((uint32_t)f2bf(f[7]) << 16);
  *reinterpret_cast<uint4*>(p) = v;
}
__device__ __forceinline__ void st8(float* p, const float* f) {
  reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}

static bool al16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static bool vec_ok(long long n, int C, const void* a, const void* b = nullptr, const void* c = nullptr,
                   const void* d = nullptr) {
  return C % 8 == 0 && n % 8 == 0 && n / 8 < 0xFFFFFFFFll && al16(a) && al16(b) && al16(c) && al16(d);
}
static int vgrid(long long nvec) { return grid_for(nvec, 256, 16384); }



// Sum a [nrows][2][ld] double slab over rows for the 32 channels of this block
// (8 row groups x 32 channels, fixed order): s[j][cl] for j in {0, 1}.
// Fixed-order (deterministic) column sums of a partial-statistics slab
// part[nrows][2][ld] for the 32 channels of this block: 1024 threads = 32 row
// groups x 32 channels, each thread keeps four independent (sum, sum) pairs so
// eight loads are in flight, then a fixed-order tree over the row groups.
// (The finalizers were latency-bound at 40-60 us with 8 row groups.)
constexpr int SLAB_THREADS = 1024;
// A workgroup sums SLAB_CH channels of a [nrows][2][ld] double slab over its
// rows: 128 row groups x 8 channels, each thread with all of its (<= 8 for the
// usual 1024-row slabs) loads in flight, then a fixed-order sum of the 128
// group partials.  (32 channels x 32 row groups per workgroup left each thread
// 64 loads in eight dependent rounds and only C/32 workgroups on the GPU.)
constexpr int SLAB_CH = 8, SLAB_RG = SLAB_THREADS / SLAB_CH;
__device__ __forceinline__ void slab_sum(const double* __restrict__ part, int nrows, int ld, int C,
                                         double (*s)[SLAB_CH]) {
  __shared__ double tmp[SLAB_RG][2][SLAB_CH];
  const int cl = threadIdx.x % SLAB_CH, rg = threadIdx.x / SLAB_CH;
  const int c = blockIdx.x * SLAB_CH + cl;
  double a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = b[u] = 0.0;
  if (c < C) {
    int r = rg;
    for (; r + 7 * SLAB_RG < nrows; r += 8 * SLAB_RG) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] += part[((long long)(r + SLAB_RG * u) * 2 + 0) * ld + c];
        b[u] += part[((long long)(r + SLAB_RG * u) * 2 + 1) * ld + c];
      }
    }
    for (int u = 0; r < nrows; r += SLAB_RG, ++u) {
      a[u & 7] += part[((long long)r * 2 + 0) * ld + c];
      b[u & 7] += part[((long long)r * 2 + 1) * ld + c];
    }
  }
  double ta = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  double tb = ((b[0] + b[1]) + (b[2] + b[3])) + ((b[4] + b[5]) + (b[6] + b[7]));
  // fixed-order pairwise tree over the 128 row groups in LDS (7 barriers); a
  // 128-long serial sum of dependent LDS loads was the finalizers' 9-13 us
  tmp[rg][0][cl] = ta;
  tmp[rg][1][cl] = tb;
  __syncthreads();
#pragma unroll
  for (int h = SLAB_RG / 2; h >= 1; h >>= 1) {
    if (rg < h) {
      ta += tmp[rg + h][0][cl];
      tb += tmp[rg + h][1][cl];
      tmp[rg][0][cl] = ta;
      tmp[rg][1][cl] = tb;
    }
    __syncthreads();
  }
  if (threadIdx.x < 2 * SLAB_CH) {
    const int ch = threadIdx.x % SLAB_CH, w = threadIdx.x / SLAB_CH;
    s[w][ch] = tmp[0][w][ch];
  }
  __syncthreads();
}

// Per-thread 8-channel statistics -> block slab row part[blockIdx][2][C].
// Requires the grid stride (gridDim.x * 256 vectors) to be a multiple of C/8,
// so every vector a thread visits has the same channel group.
__device__ __forceinline__ void stats8_flush(const double* a, const double* b, int cv, int C, bool active,
                                             double* red, double* __restrict__ part, int nt = 256) {
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      atomicAdd(&red[cv * 8 + j], a[j]);
      atomicAdd(&red[C + cv * 8 + j], b[j]);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += nt) part[(long long)blockIdx.x * 2 * C + i] = red[i];
}

static bool stats8_ok(int C) { return C % 8 == 0 && C / 8 <= 256 && 256 % (C / 8) == 0 && C <= 2048; }

// ---------------------------------------------------------------- BN statistics
// part[blk][2][C] = {sum x, sum x^2} over the block's rows (double)
template <typename T>
__global__ void __launch_bounds__(256) k_bn_stats(const T* __restrict__ x, long long rows, int C,
                                                  double* __restrict__ part) {
  extern __shared__ double red[];  // [2][C]
  for (int i = threadIdx.x; i < 2 * C; i += 256) red[i] = 0.0;
  __syncthreads();
  const long long per = (rows + gridDim.x - 1) / gridDim.x;
  const long long r0 = (long long)blockIdx.x * per;
  long long r1 = r0 + per;
  if (r1 > rows) r1 = rows;
  const int tpr = C < 256 ? C : 256;
  const int rpp = 256 / tpr;
  const int c_base = threadIdx.x % tpr, rsub = threadIdx.x / tpr;
  if (rsub < rpp) {
    for (int c = c_base; c < C; c += tpr) {
      double s1 = 0.0, s2 = 0.0;
      float f1 = 0.f, f2 = 0.f;
      int cnt = 0;
      for (long long r = r0 + rsub; r < r1; r += rpp) {
        const float v = ld(x, r * C + c);
        f1 += v;
        f2 += v * v;
        if (++cnt == 256) { s1 += f1; s2 += f2; f1 = f2 = 0.f; cnt = 0; }
      }
      atomicAdd(&red[c], s1 + f1);
      atomicAdd(&red[C + c], s2 + f2);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) part[(long long)blockIdx.x * 2 * C + i] = red[i];
}

template <typename T>
__global__ void __launch_bounds__(256) k_bn_stats8(const T* __restrict__ x, long long rows, int C,
                                                   double* __restrict__ part) {
  extern __shared__ double red[];  // [2][C]
  for (int i = threadIdx.x; i < 2 * C; i += 256) red[i] = 0.0;
  __syncthreads();
  const long long per = (rows + gridDim.x - 1) / gridDim.x;
  const long long r0 = (long long)blockIdx.x * per;
  long long r1 = r0 + per;
  if (r1 > rows) r1 = rows;
  const int CV = C >> 3;
  const int tpr = CV < 256 ? CV : 256;
  const int rpp = 256 / tpr;
  const int cvb = threadIdx.x % tpr, rs = threadIdx.x / tpr;
  if (rs < rpp) {
    for (int cv = cvb; cv < CV; cv += tpr) {
      float a[8], b[8];
      double da[8], db[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = b[j] = 0.f, da[j] = db[j] = 0.0;
      int cnt = 0;
      for (long long r = r0 + rs; r < r1; r += rpp) {
        float f[8];
        ld8(x + r * C + cv * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[j] += f[j];
          b[j] += f[j] * f[j];
        }
        if (++cnt == 64) {
#pragma unroll
          for (int j = 0; j < 8; ++j) da[j] += a[j], db[j] += b[j], a[j] = b[j] = 0.f;
          cnt = 0;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&red[cv * 8 + j], da[j] + a[j]);
        atomicAdd(&red[C + cv * 8 + j], db[j] + b[j]);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) part[(long long)blockIdx.x * 2 * C + i] = red[i];
}

ACFE_API int acfe_bn_stats(const void* x, long long rows, int C, int dtype, double* part, void* stream) {
  if (!x || !part || rows <= 0 || C <= 0 || C > 2048) return ACFE_E_INVAL;
  const int nb = red_blocks(rows);
  if (vec_ok(rows * C, C, x)) {
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_bn_stats8<T>, dim3(nb), dim3(256), 2 * C * sizeof(double),
                                           strm(stream), (const T*)x, rows, C, part));
  } else {
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_bn_stats<T>, dim3(nb), dim3(256), 2 * C * sizeof(double),
                                           strm(stream), (const T*)x, rows, C, part));
  }
  return launch_rc("acfe_bn_stats");
}

// part: [nrows][2][ld] (ld >= C; conv epilogues use the padded K as ld)
// out (each fp32[C], any may be NULL except scale/shift):
//   scale = gamma * invstd, shift = beta - mean * scale, mean, invstd
// training: batch statistics + moving-average update (momentum); else moving stats.
__global__ void __launch_bounds__(SLAB_THREADS) k_bn_finalize(const double* __restrict__ part, int nrows, int ld, int C,
                                                     double count, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps, float momentum,
                                                     float* __restrict__ mmean, float* __restrict__ mvar,
                                                     int training, float* __restrict__ scale,
                                                     float* __restrict__ shift, float* __restrict__ mean_o,
                                                     float* __restrict__ invstd_o) {
  __shared__ double s[2][SLAB_CH];
  if (training) slab_sum(part, nrows, ld, C, s);
  const int c = blockIdx.x * SLAB_CH + threadIdx.x;
  if (threadIdx.x >= SLAB_CH || c >= C) return;
  double mean, var;
  if (training) {
    mean = s[0][threadIdx.x] / count;
    var = s[1][threadIdx.x] / count - mean * mean;
    if (var < 0) var = 0;
    if (mmean) mmean[c] = (float)(mmean[c] * (double)momentum + mean * (1.0 - momentum));
    if (mvar) mvar[c] = (float)(mvar[c] * (double)momentum + var * (1.0 - momentum));
  } else {
    mean = mmean[c];
    var = mvar[c];
  }
  const double inv = 1.0 / sqrt(var + (double)eps);
  const double g = gamma ? gamma[c] : 1.0, b = beta ? beta[c] : 0.0;
  const double sc = g * inv;
  scale[c] = (float)sc;
  shift[c] = (float)(b - mean * sc);
  if (mean_o) mean_o[c] = (float)mean;
  if (invstd_o) invstd_o[c] = (float)inv;
}

ACFE_API int acfe_bn_finalize(const double* part, int nrows, int ld, int C, double count, const float* gamma,
                              const float* beta, float eps, float momentum, float* moving_mean,
                              float* moving_var, int training, float* scale, float* shift, float* mean,
                              float* invstd, void* stream) {
  if (!scale || !shift || C <= 0 || (training && (!part || nrows <= 0 || count <= 0)) ||
      (!training && (!moving_mean || !moving_var)))
    return ACFE_E_INVAL;
  hipLaunchKernelGGL(k_bn_finalize, dim3(cdiv(C, SLAB_CH)), dim3(SLAB_THREADS), 0, strm(stream), part, nrows, ld, C, count,
                     gamma, beta, eps, momentum, moving_mean, moving_var, training, scale, shift, mean, invstd);
  return launch_rc("acfe_bn_finalize");
}

// y = x*scale[c] + shift[c] (+ReLU)
template <typename TI, typename TO>
__global__ void k_bn_apply(const TI* __restrict__ x, long long n, int C, const float* __restrict__ scale,
                           const float* __restrict__ shift, int relu, TO* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    float v = ld(x, i) * scale[c] + shift[c];
    if (relu) v = fmaxf(v, 0.f);
    st(y, i, v);
  }
}
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) k_bn_apply8(const TI* __restrict__ x, unsigned nvec, int C,
                                                   const float* __restrict__ scale, const float* __restrict__ shift,
                                                   int relu, TO* __restrict__ y) {
  extern __shared__ float sm[];
  const unsigned CV = C >> 3;
  const unsigned v0 = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  if (256 % CV == 0) {
    // a thread's 8 channels are fixed across the grid-stride loop: scale /
    // shift in registers, two iterations' loads issued together (same
    // arithmetic as below, so the BN-prologue kernels stay bit-identical)
    const int c0 = (int)(v0 % CV) * 8;
    float rs[8], rh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) rs[j] = scale[c0 + j], rh[j] = shift[c0 + j];
    unsigned v = v0;
    for (; v + stride < nvec; v += 2 * stride) {
      float f[8], h[8];
      ld8(x + (size_t)v * 8, f);
      ld8(x + (size_t)(v + stride) * 8, h);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f[j] = f[j] * rs[j] + rh[j];
        h[j] = h[j] * rs[j] + rh[j];
        if (relu) f[j] = fmaxf(f[j], 0.f), h[j] = fmaxf(h[j], 0.f);
      }
      st8(y + (size_t)v * 8, f);
      st8(y + (size_t)(v + stride) * 8, h);
    }
    if (v < nvec) {
      float f[8];
      ld8(x + (size_t)v * 8, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f[j] = f[j] * rs[j] + rh[j];
        if (relu) f[j] = fmaxf(f[j], 0.f);
      }
      st8(y + (size_t)v * 8, f);
    }
    return;
  }
  for (int i = threadIdx.x; i < C; i += 256) sm[i] = scale[i], sm[C + i] = shift[i];
  __syncthreads();
  for (unsigned v = v0; v < nvec; v += stride) {
    const int c0 = (int)(v % CV) * 8;
    float f[8];
    ld8(x + (size_t)v * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = f[j] * sm[c0 + j] + sm[C + c0 + j];
      if (relu) f[j] = fmaxf(f[j], 0.f);
    }
    st8(y + (size_t)v * 8, f);
  }
}

ACFE_API int acfe_bn_apply(const void* x, int x_dtype, long long rows, int C, const float* scale,
                           const float* shift, int relu, void* y, int y_dtype, void* stream) {
  if (!x || !y || !scale || !shift || rows < 0 || C <= 0) return ACFE_E_INVAL;
  const long long n = rows * C;
  if (n == 0) return ACFE_OK;
  if (vec_ok(n, C, x, y) && C <= 4096) {
    DISPATCH1(x_dtype, TI, DISPATCH1(y_dtype, TO,
        hipLaunchKernelGGL((k_bn_apply8<TI, TO>), dim3(vgrid(n / 8)), dim3(256), 2 * C * sizeof(float),
                           strm(stream), (const TI*)x, (unsigned)(n / 8), C, scale, shift, relu, (TO*)y)));
  } else {
    DISPATCH1(x_dtype, TI, DISPATCH1(y_dtype, TO,
        hipLaunchKernelGGL((k_bn_apply<TI, TO>), dim3(grid_for(n)), dim3(256), 0, strm(stream), (const TI*)x, n,
                           C, scale, shift, relu, (TO*)y)));
  }
  return launch_rc("acfe_bn_apply");
}

// Backward reduce: g = dy * (relu ? [x*scale+shift > 0] : 1); xhat = (x-mean)*invstd
// part[blk][2][C] = {sum g, sum g*xhat}
template <typename TG, typename TX>
__global__ void __launch_bounds__(256) k_bn_bwd_reduce(const TG* __restrict__ dy, const TX* __restrict__ x,
                                                       long long rows, int C, const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd, int relu,
                                                       double* __restrict__ part) {
  extern __shared__ double red[];
  for (int i = threadIdx.x; i < 2 * C; i += 256) red[i] = 0.0;
  __syncthreads();
  const long long per = (rows + gridDim.x - 1) / gridDim.x;
  const long long r0 = (long long)blockIdx.x * per;
  long long r1 = r0 + per;
  if (r1 > rows) r1 = rows;
  const int tpr = C < 256 ? C : 256;
  const int rpp = 256 / tpr;
  const int c_base = threadIdx.x % tpr, rsub = threadIdx.x / tpr;
  if (rsub < rpp) {
    for (int c = c_base; c < C; c += tpr) {
      const float sc = scale[c], sh = shift[c], mu = mean[c], is = invstd[c];
      double s1 = 0.0, s2 = 0.0;
      float f1 = 0.f, f2 = 0.f;
      int cnt = 0;
      for (long long r = r0 + rsub; r < r1; r += rpp) {
        const float xv = ld(x, r * C + c);
        float g = ld(dy, r * C + c);
        if (relu && !(xv * sc + sh > 0.f)) g = 0.f;
        f1 += g;
        f2 += g * ((xv - mu) * is);
        if (++cnt == 256) { s1 += f1; s2 += f2; f1 = f2 = 0.f; cnt = 0; }
      }
      atomicAdd(&red[c], s1 + f1);
      atomicAdd(&red[C + c], s2 + f2);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) part[(long long)blockIdx.x * 2 * C + i] = red[i];
}
template <typename TG, typename TX>
__global__ void __launch_bounds__(256) k_bn_bwd_reduce8(const TG* __restrict__ dy, const TX* __restrict__ x,
                                                        long long rows, int C, const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, int relu,
                                                        double* __restrict__ part) {
  extern __shared__ double red[];
  for (int i = threadIdx.x; i < 2 * C; i += 256) red[i] = 0.0;
  __syncthreads();
  const long long per = (rows + gridDim.x - 1) / gridDim.x;
  const long long r0 = (long long)blockIdx.x * per;
  long long r1 = r0 + per;
  if (r1 > rows) r1 = rows;
  const int CV = C >> 3;
  const int tpr = CV < 256 ? CV : 256;
  const int rpp = 256 / tpr;
  const int cvb = threadIdx.x % tpr, rs = threadIdx.x / tpr;
  if (rs < rpp) {
    for (int cv = cvb; cv < CV; cv += tpr) {
      float sc[8], sh[8], mu[8], is[8], a[8], b[8];
      double da[8], db[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = cv * 8 + j;
        sc[j] = scale[c], sh[j] = shift[c], mu[j] = mean[c], is[j] = invstd[c];
        a[j] = b[j] = 0.f, da[j] = db[j] = 0.0;
      }
      int cnt = 0;
      for (long long r = r0 + rs; r < r1; r += rpp) {
        float g[8], xv[8];
        ld8(dy + r * C + cv * 8, g);
        ld8(x + r * C + cv * 8, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gj = (relu && !(xv[j] * sc[j] + sh[j] > 0.f)) ? 0.f : g[j];
          a[j] += gj;
          b[j] += gj * ((xv[j] - mu[j]) * is[j]);
        }
        if (++cnt == 64) {
#pragma unroll
          for (int j = 0; j < 8; ++j) da[j] += a[j], db[j] += b[j], a[j] = b[j] = 0.f;
          cnt = 0;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&red[cv * 8 + j], da[j] + a[j]);
        atomicAdd(&red[C + cv * 8 + j], db[j] + b[j]);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) part[(long long)blockIdx.x * 2 * C + i] = red[i];
}

ACFE_API int acfe_bn_bwd_reduce(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows, int C,
                                const float* scale, const float* shift, const float* mean, const float* invstd,
                                int relu, double* part, void* stream) {
  if (!dy || !x || !scale || !shift || !mean || !invstd || !part || rows <= 0 || C <= 0 || C > 2048)
    return ACFE_E_INVAL;
  const int nb = red_blocks(rows);
  if (vec_ok(rows * C, C, dy, x)) {
    DISPATCH1(dy_dtype, TG, DISPATCH1(x_dtype, TX,
        hipLaunchKernelGGL((k_bn_bwd_reduce8<TG, TX>), dim3(nb), dim3(256), 2 * C * sizeof(double), strm(stream),
                           (const TG*)dy, (const TX*)x, rows, C, scale, shift, mean, invstd, relu, part)));
  } else {
    DISPATCH1(dy_dtype, TG, DISPATCH1(x_dtype, TX,
        hipLaunchKernelGGL((k_bn_bwd_reduce<TG, TX>), dim3(nb), dim3(256), 2 * C * sizeof(double), strm(stream),
                           (const TG*)dy, (const TX*)x, rows, C, scale, shift, mean, invstd, relu, part)));
  }
  return launch_rc("acfe_bn_bwd_reduce");
}

// coef[3][C] = {a, b, c} with dx = a*g + b*x + c; dgamma = sum g xhat, dbeta = sum g
__global__ void __launch_bounds__(SLAB_THREADS) k_bn_bwd_finalize(const double* __restrict__ part, int nrows, int C,
                                                         double count, const float* __restrict__ scale,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                         float* __restrict__ coef, int acc) {
  __shared__ double s[2][SLAB_CH];
  slab_sum(part, nrows, C, C, s);
  const int c = blockIdx.x * SLAB_CH + threadIdx.x;
  if (threadIdx.x >= SLAB_CH || c >= C) return;
  const double sg = s[0][threadIdx.x], sgx = s[1][threadIdx.x];
  if (dgamma) dgamma[c] = acc ? dgamma[c] + (float)sgx : (float)sgx;
  if (dbeta) dbeta[c] = acc ? dbeta[c] + (float)sg : (float)sg;
  const double sc = scale[c], is = invstd[c], mu = mean[c];
  const double mg = sg / count, mgx = sgx / count;
  coef[c] = (float)sc;
  coef[C + c] = (float)(-sc * mgx * is);
  coef[2 * C + c] = (float)(-sc * mg + sc * mgx * is * mu);
}

ACFE_API int acfe_bn_bwd_finalize_ex(const double* part, int nrows, int C, double count, const float* scale,
                                     const float* mean, const float* invstd, float* dgamma, float* dbeta,
                                     float* coef, int accumulate, void* stream) {
  if (!part || !scale || !mean || !invstd || !coef || nrows <= 0 || C <= 0) return ACFE_E_INVAL;
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3(cdiv(C, SLAB_CH)), dim3(SLAB_THREADS), 0, strm(stream), part, nrows, C, count, scale,
                     mean, invstd, dgamma, dbeta, coef, accumulate ? 1 : 0);
  return launch_rc("acfe_bn_bwd_finalize");
}

ACFE_API int acfe_bn_bwd_finalize(const double* part, int nrows, int C, double count, const float* scale,
                                  const float* mean, const float* invstd, float* dgamma, float* dbeta,
                                  float* coef, void* stream) {
  return acfe_bn_bwd_finalize_ex(part, nrows, C, count, scale, mean, invstd, dgamma, dbeta, coef, 0, stream);
}

// dx = a*g + b*x + c  (+ add[i] if add != NULL); g relu-masked as in the reduce
template <typename TG, typename TX, typename TO>
__global__ void k_bn_bwd_apply(const TG* __restrict__ dy, const TX* __restrict__ x, long long n, int C,
                               const float* __restrict__ scale, const float* __restrict__ shift, int relu,
                               const float* __restrict__ coef, const TO* __restrict__ add, Drop drop,
                               TO* __restrict__ dx) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const float xv = ld(x, i);
    float g = ld(dy, i);
    if ((relu & 1) && !(xv * scale[c] + shift[c] > 0.f)) g = 0.f;
    float v = __builtin_fmaf(coef[c], g, __builtin_fmaf(coef[C + c], xv, coef[2 * C + c]));
    if (add) v += ld(add, i);
    if ((relu & 2) && !(xv > 0.f)) v = 0.f;  // x = ReLU output upstream: its backward
    if (drop.on) v = drop_apply<TO>(drop, (uint64_t)i, rnd(v, TO()));
    st(dx, i, v);
  }
}
// Gradient of an AveragePooling2D(k, strides=k, "same") whose input is this
// BN's input x, added on the fly (the pooled gradient g [N][P][Q][C] spread
// over the window's in-bounds elements, as acfe_avgpool2d_bwd stores it).
// sub: instead, the input gradient of a 1x1 "valid" conv of stride k reading x
// (wr_resnet's transition shortcuts): g [N][P][Q][C] lands on the pixels
// (k p, k q) only -- the other pixels' shortcut gradient is zero.
struct PoolAdd {
  const void* g;
  int H, W, k, P, Q, pt, pl, sub;
};

// threads per workgroup of k_bn_bwd_apply8: with the channel-sum slab the grid
// is fixed at acfe_reduce_blocks(rows) workgroups (<= 1024), so the block size
// sets how many 16-B vectors are in flight per CU
// (256: the REG path and stats8_flush assume each thread keeps the same 8
// channels across its grid-stride loop, i.e. gridDim * 256 a multiple of
// C / 8, which stats8_ok guarantees for this block size only)
constexpr int BWD_APPLY_NT = 256;
template <typename TG, typename TX, typename TO, bool REG>
__global__ void __launch_bounds__(BWD_APPLY_NT) k_bn_bwd_apply8(const TG* __restrict__ dy, const TX* __restrict__ x,
                                                       unsigned nvec, int C, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int relu,
                                                       const float* __restrict__ coef, const TO* __restrict__ add,
                                                       Drop drop, TO* __restrict__ dx, double* __restrict__ sum_part,
                                                       PoolAdd pa) {
  // dynamic LDS: [2][C] doubles (channel sums, when sum_part) then scale, shift, a, b, c
  extern __shared__ double smd[];
  double* red = smd;
  float* sm = reinterpret_cast<float*>(smd + (sum_part ? 2 * C : 0));
  for (int i = threadIdx.x; i < C; i += BWD_APPLY_NT) {
    sm[i] = scale[i];
    sm[C + i] = shift[i];
    sm[2 * C + i] = coef[i];
    sm[3 * C + i] = coef[C + i];
    sm[4 * C + i] = coef[2 * C + i];
    if (sum_part) red[i] = red[C + i] = 0.0;
  }
  __syncthreads();
  const unsigned CV = C >> 3;
  const bool i32 = (uint64_t)nvec * 8 <= (1ull << 32);  // every element index < 2^32
  double sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.0;
  const unsigned v0 = blockIdx.x * BWD_APPLY_NT + threadIdx.x;
  // With the channel-sum slab (grid = acfe_reduce_blocks, 256 % (C / 8) == 0)
  // a thread's 8 channels are fixed across the grid-stride loop: its 5 x 8
  // coefficients are held in registers instead of read from LDS per element
  // (r05u, same box: 2.72 -> 2.62 ms at wr_resnet's stage-1 tensors with
  // dropout, 385 -> 341 us at T1's 64x128, 1.57 -> 1.35 ms at 64x257x128);
  // the many-workgroup grid without the slab keeps the LDS reads (measured
  // level or slower with registers; its own instantiation keeps 6 waves per
  // SIMD)
  {
    float kc[REG ? 5 : 1][8];
    if constexpr (REG) {
      const int cf = (int)(v0 % CV) * 8;
#pragma unroll
      for (int q = 0; q < 5; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) kc[q][j] = sm[q * C + cf + j];
    }
    auto kcf = [&](int q, int c, int j) __attribute__((always_inline)) {
      if constexpr (REG) return kc[q][j];
      else return sm[q * C + c];
    };
    for (unsigned v = v0; v < nvec; v += gridDim.x * BWD_APPLY_NT) {
      const int c0 = (int)(v % CV) * 8;
      float g[8], xv[8], o[8];
      ld8(dy + (size_t)v * 8, g);
      ld8(x + (size_t)v * 8, xv);
      if (add) ld8(add + (size_t)v * 8, o);
      if (pa.g && pa.sub) {
        const unsigned row = v / CV, t = row / (unsigned)pa.W;
        const int w = (int)(row - t * (unsigned)pa.W), h = (int)(t % (unsigned)pa.H), nn = (int)(t / (unsigned)pa.H);
        const int p = h / pa.k, q = w / pa.k;
        if (h == p * pa.k && w == q * pa.k && p < pa.P && q < pa.Q) {
          ld8(reinterpret_cast<const TO*>(pa.g) + (((size_t)nn * pa.P + p) * pa.Q + q) * C + c0, o);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = 0.f;  // (0 + r, as the materialised zero gradient adds)
        }
      } else if (pa.g) {
        const unsigned row = v / CV, t = row / (unsigned)pa.W;
        const int w = (int)(row - t * (unsigned)pa.W), h = (int)(t % (unsigned)pa.H), nn = (int)(t / (unsigned)pa.H);
        const int p = (h + pa.pt) / pa.k, q = (w + pa.pl) / pa.k;
        const int h0 = max(p * pa.k - pa.pt, 0), h1 = min(p * pa.k - pa.pt + pa.k, pa.H);
        const int w0 = max(q * pa.k - pa.pl, 0), w1 = min(q * pa.k - pa.pl + pa.k, pa.W);
        const float inv = 1.0f / (float)((h1 - h0) * (w1 - w0));
        ld8(reinterpret_cast<const TO*>(pa.g) + (((size_t)nn * pa.P + p) * pa.Q + q) * C + c0, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] *= inv;
      }
      const bool has_add = add || pa.g;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        const float gj = ((relu & 1) && !(xv[j] * kcf(0, c, j) + kcf(1, c, j) > 0.f)) ? 0.f : g[j];
        const float r = __builtin_fmaf(kcf(2, c, j), gj, __builtin_fmaf(kcf(3, c, j), xv[j], kcf(4, c, j)));
        o[j] = has_add ? o[j] + r : r;
        if ((relu & 2) && !(xv[j] > 0.f)) o[j] = 0.f;  // x = ReLU output upstream: its backward
      }
      if (drop.on) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rnd(o[j], TO());
        drop_apply8<TO>(drop, (uint64_t)v * 8, i32, o);
      }
      st8(dx + (size_t)v * 8, o);
      if (sum_part) {
        // (the slab's sum-of-squares row stays zero: only the bias gradient --
        // the first row, acfe_channel_sum_finalize -- reads this slab, and the
        // f64 square-sum was half of this pass's double-precision work)
#pragma unroll
        for (int j = 0; j < 8; ++j) sa[j] += rnd(o[j], TO());  // the stored value
      }
    }
  }
  if (sum_part) stats8_flush(sa, sb, (int)(v0 % CV), C, v0 < nvec, red, sum_part, BWD_APPLY_NT);
}

static int bn_bwd_apply_impl(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows, int C,
                             const float* scale, const float* shift, int relu, const float* coef, const void* add,
                             const Drop& d, void* dx, int dx_dtype, double* sum_part, void* stream,
                             PoolAdd pa = PoolAdd{nullptr, 0, 0, 0, 0, 0, 0, 0, 0}) {
  if (!dy || !x || !scale || !shift || !coef || !dx || rows < 0 || C <= 0) return ACFE_E_INVAL;
  const long long n = rows * C;
  if (n == 0) return ACFE_OK;
  if (pa.g && (!vec_ok(n, C, dy, x, pa.g, dx) || C > 2048 || add)) return ACFE_E_INVAL;
  if (vec_ok(n, C, dy, x, add, dx) && C <= 2048) {
    if (sum_part && !stats8_ok(C)) return ACFE_E_INVAL;
    const int grid = sum_part ? red_blocks(rows) : vgrid(n / 8);
    const size_t shm = 5 * C * sizeof(float) + (sum_part ? 2 * C * sizeof(double) : 0);
    DISPATCH1(dy_dtype, TG, DISPATCH1(x_dtype, TX, DISPATCH1(dx_dtype, TO,
        if (sum_part) hipLaunchKernelGGL((k_bn_bwd_apply8<TG, TX, TO, true>), dim3(grid), dim3(BWD_APPLY_NT), shm,
                                         strm(stream), (const TG*)dy, (const TX*)x, (unsigned)(n / 8), C, scale, shift,
                                         relu, coef, (const TO*)add, d, (TO*)dx, sum_part, pa);
        else hipLaunchKernelGGL((k_bn_bwd_apply8<TG, TX, TO, false>), dim3(grid), dim3(BWD_APPLY_NT), shm,
                                strm(stream), (const TG*)dy, (const TX*)x, (unsigned)(n / 8), C, scale, shift, relu,
                                coef, (const TO*)add, d, (TO*)dx, sum_part, pa))));
  } else {
    if (sum_part) return ACFE_E_INVAL;
    DISPATCH1(dy_dtype, TG, DISPATCH1(x_dtype, TX, DISPATCH1(dx_dtype, TO,
        hipLaunchKernelGGL((k_bn_bwd_apply<TG, TX, TO>), dim3(grid_for(n)), dim3(256), 0, strm(stream),
                           (const TG*)dy, (const TX*)x, n, C, scale, shift, relu, coef, (const TO*)add, d,
                           (TO*)dx))));
  }
  return launch_rc("acfe_bn_bwd_apply");
}

ACFE_API int acfe_bn_bwd_apply(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows, int C,
                               const float* scale, const float* shift, int relu, const float* coef,
                               const void* add, void* dx, int dx_dtype, void* stream) {
  return bn_bwd_apply_impl(dy, dy_dtype, x, x_dtype, rows, C, scale, shift, relu, coef, add, make_drop(0.f, 0),
                           dx, dx_dtype, nullptr, stream);
}

// As acfe_bn_bwd_apply, then the backward of a Dropout(rate, seed) that produced x.
ACFE_API int acfe_bn_bwd_apply_dropout(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows,
                                       int C, const float* scale, const float* shift, int relu, const float* coef,
                                       float drop_rate, unsigned long long seed, void* dx, int dx_dtype,
                                       void* stream) {
  if (drop_rate < 0.f || drop_rate >= 1.f) return ACFE_E_INVAL;
  return bn_bwd_apply_impl(dy, dy_dtype, x, x_dtype, rows, C, scale, shift, relu, coef, nullptr,
                           make_drop(drop_rate, seed), dx, dx_dtype, nullptr, stream);
}

// General form: optional residual add, optional Dropout backward, optional
// per-channel sums of the stored dx (slab as acfe_add_stats; the bias gradient
// of a convolution producing this BN's input).
ACFE_API int acfe_bn_bwd_apply_ex(const void* dy, int dy_dtype, const void* x, int x_dtype, long long rows, int C,
                                  const float* scale, const float* shift, int relu, const float* coef,
                                  const void* add, float drop_rate, unsigned long long seed, void* dx, int dx_dtype,
                                  double* sum_partial, void* stream) {
  if (drop_rate < 0.f || drop_rate >= 1.f || (add && drop_rate > 0.f)) return ACFE_E_INVAL;
  return bn_bwd_apply_impl(dy, dy_dtype, x, x_dtype, rows, C, scale, shift, relu, coef, add,
                           make_drop(drop_rate, seed), dx, dx_dtype, sum_partial, stream);
}

// acfe_bn_bwd_apply_ex with, instead of `add`, the backward of
// AveragePooling2D(k, strides=k, "same")(x): gpool [N][ceil(H/k)][ceil(W/k)][C].
ACFE_API int acfe_bn_bwd_apply_pool(const void* dy, int dy_dtype, const void* x, int x_dtype, int N, int H, int W,
                                    int C, const float* scale, const float* shift, int relu, const float* coef,
                                    const void* gpool, int k, void* dx, int dx_dtype, double* sum_partial,
                                    void* stream) {
  if (!gpool || N <= 0 || H <= 0 || W <= 0 || k <= 0) return ACFE_E_INVAL;
  PoolAdd pa;
  pa.g = gpool;
  pa.H = H;
  pa.W = W;
  pa.k = k;
  pa.P = (H + k - 1) / k;
  pa.Q = (W + k - 1) / k;
  pa.pt = ((pa.P - 1) * k + k - H) / 2;
  pa.pl = ((pa.Q - 1) * k + k - W) / 2;
  pa.sub = 0;
  return bn_bwd_apply_impl(dy, dy_dtype, x, x_dtype, (long long)N * H * W, C, scale, shift, relu, coef, nullptr,
                           make_drop(0.f, 0), dx, dx_dtype, sum_partial, stream, pa);
}

// acfe_bn_bwd_apply_ex with, instead of `add`, the input gradient of a 1x1
// "valid" Conv2D of stride k reading x: gsub [N][(H-1)/k+1][(W-1)/k+1][C] at
// the pixels (k p, k q), zero elsewhere (never materialised at H x W).
ACFE_API int acfe_bn_bwd_apply_sub(const void* dy, int dy_dtype, const void* x, int x_dtype, int N, int H, int W,
                                   int C, const float* scale, const float* shift, int relu, const float* coef,
                                   const void* gsub, int k, void* dx, int dx_dtype, double* sum_partial,
                                   void* stream) {
  if (!gsub || N <= 0 || H <= 0 || W <= 0 || k <= 0) return ACFE_E_INVAL;
  PoolAdd pa;
  pa.g = gsub;
  pa.H = H;
  pa.W = W;
  pa.k = k;
  pa.P = (H - 1) / k + 1;
  pa.Q = (W - 1) / k + 1;
  pa.pt = pa.pl = 0;
  pa.sub = 1;
  return bn_bwd_apply_impl(dy, dy_dtype, x, x_dtype, (long long)N * H * W, C, scale, shift, relu, coef, nullptr,
                           make_drop(0.f, 0), dx, dx_dtype, sum_partial, stream, pa);
}

// ---------------------------------------------------------------- elementwise
// z = a + b (+ReLU)
template <typename T>
__global__ void k_add(const T* __restrict__ a, const T* __restrict__ b, long long n, int relu, T* __restrict__ z) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float v = ld(a, i) + ld(b, i);
    if (relu) v = fmaxf(v, 0.f);
    st(z, i, v);
  }
}
template <typename T>
__global__ void k_add8(const T* __restrict__ a, const T* __restrict__ b, unsigned nvec, int relu,
                       T* __restrict__ z) {
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) {
    float x[8], y[8];
    ld8(a + (size_t)v * 8, x);
    ld8(b + (size_t)v * 8, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = relu ? fmaxf(x[j] + y[j], 0.f) : x[j] + y[j];
    st8(z + (size_t)v * 8, x);
  }
}
ACFE_API int acfe_add(const void* a, const void* b, long long n, int relu, void* z, int dtype, void* stream) {
  if (!a || !b || !z || n < 0) return ACFE_E_INVAL;
  if (n == 0) return ACFE_OK;
  if (vec_ok(n, 8, a, b, z))
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_add8<T>, dim3(vgrid(n / 8)), dim3(256), 0, strm(stream), (const T*)a,
                                           (const T*)b, (unsigned)(n / 8), relu, (T*)z));
  else
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_add<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream), (const T*)a,
                                           (const T*)b, n, relu, (T*)z));
  return launch_rc("acfe_add");
}

// dx = dy * [y > 0]
template <typename T>
__global__ void k_relu_bwd(const T* __restrict__ dy, const T* __restrict__ y, long long n, T* __restrict__ dx) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    st(dx, i, ld(y, i) > 0.f ? ld(dy, i) : 0.f);
}
template <typename T>
__global__ void k_relu_bwd8(const T* __restrict__ dy, const T* __restrict__ y, unsigned nvec, T* __restrict__ dx) {
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) {
    float g[8], yy[8];
    ld8(dy + (size_t)v * 8, g);
    ld8(y + (size_t)v * 8, yy);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
    st8(dx + (size_t)v * 8, g);
  }
}
ACFE_API int acfe_relu_bwd(const void* dy, const void* y, long long n, void* dx, int dtype, void* stream) {
  if (!dy || !y || !dx || n < 0) return ACFE_E_INVAL;
  if (n == 0) return ACFE_OK;
  if (vec_ok(n, 8, dy, y, dx))
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_relu_bwd8<T>, dim3(vgrid(n / 8)), dim3(256), 0, strm(stream),
                                           (const T*)dy, (const T*)y, (unsigned)(n / 8), (T*)dx));
  else
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_relu_bwd<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream),
                                           (const T*)dy, (const T*)y, n, (T*)dx));
  return launch_rc("acfe_relu_bwd");
}

// dx = dy * [y > 0] over [rows][C] plus per-channel sums of dx (bias gradient
// of the convolutions fed by an Add+ReLU; slab as acfe_add_stats).
template <typename T>
__global__ void __launch_bounds__(256) k_relu_bwd8s(const T* __restrict__ dy, const T* __restrict__ y, unsigned nvec,
                                                    int C, T* __restrict__ dx, double* __restrict__ part) {
  extern __shared__ double red[];
  for (int i = threadIdx.x; i < 2 * C; i += 256) red[i] = 0.0;
  __syncthreads();
  const int CV = C >> 3;
  double sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.0;
  const unsigned v0 = blockIdx.x * 256 + threadIdx.x;
  for (unsigned v = v0; v < nvec; v += gridDim.x * 256) {
    float g[8], yy[8];
    ld8(dy + (size_t)v * 8, g);
    ld8(y + (size_t)v * 8, yy);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] = yy[j] > 0.f ? g[j] : 0.f;
      sa[j] += g[j];
      sb[j] += (double)g[j] * g[j];
    }
    st8(dx + (size_t)v * 8, g);
  }
  stats8_flush(sa, sb, (int)(v0 % CV), C, v0 < nvec, red, part);
}
ACFE_API int acfe_relu_bwd_sum(const void* dy, const void* y, long long rows, int C, void* dx, int dtype,
                               double* partial, void* stream) {
  if (!dy || !y || !dx || !partial || rows <= 0 || !stats8_ok(C) || !vec_ok(rows * C, C, dy, y, dx))
    return ACFE_E_INVAL;
  DISPATCH1(dtype, T, hipLaunchKernelGGL(k_relu_bwd8s<T>, dim3(red_blocks(rows)), dim3(256), 2 * C * sizeof(double),
                                         strm(stream), (const T*)dy, (const T*)y, (unsigned)(rows * C / 8), C, (T*)dx,
                                         partial));
  return launch_rc("acfe_relu_bwd_sum");
}

// Dropout (tf.keras.layers.Dropout: keep with prob 1-rate, scale 1/(1-rate)).
// Mask: drop_keep (common.h), regenerated in the backward.
template <typename T>
__global__ void k_dropout(const T* __restrict__ x, long long n, float rate, unsigned long long seed,
                          T* __restrict__ y) {
  const Drop d = make_drop(rate, seed);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    st(y, i, drop_keep(d, (uint64_t)i) ? ld(x, i) * d.scl : 0.f);
}
template <typename T>
__global__ void k_dropout8(const T* __restrict__ x, unsigned nvec, float rate, unsigned long long seed,
                           T* __restrict__ y) {
  const Drop d = make_drop(rate, seed);
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) {
    float f[8];
    ld8(x + (size_t)v * 8, f);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const uint32_t h = drop_pair_hash(d, (uint64_t)v * 8 + j);
      f[j] = (h & 0xFFFFu) >= d.thr ? f[j] * d.scl : 0.f;
      f[j + 1] = (h >> 16) >= d.thr ? f[j + 1] * d.scl : 0.f;
    }
    st8(y + (size_t)v * 8, f);
  }
}
ACFE_API int acfe_dropout(const void* x, long long n, float rate, unsigned long long seed, void* y, int dtype,
                          void* stream) {
  if (!x || !y || n < 0 || rate < 0.f || rate >= 1.f) return ACFE_E_INVAL;
  if (n == 0) return ACFE_OK;
  if (vec_ok(n, 8, x, y))
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_dropout8<T>, dim3(vgrid(n / 8)), dim3(256), 0, strm(stream),
                                           (const T*)x, (unsigned)(n / 8), rate, seed, (T*)y));
  else
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_dropout<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream),
                                           (const T*)x, n, rate, seed, (T*)y));
  return launch_rc("acfe_dropout");
}

// ---------------------------------------------------------------- pooling (NHWC)
// MaxPool2D(pool=(kh,kw), strides=pool, padding="valid")
template <typename T>
__global__ void k_maxpool(const T* __restrict__ x, int N, int H, int W, int C, int kh, int kw, int P, int Q,
                          T* __restrict__ y) {
  const long long n_out = (long long)N * P * Q * C;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_out; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float m = -INFINITY;
    for (int a = 0; a < kh; ++a)
      for (int b = 0; b < kw; ++b)
        m = fmaxf(m, ld(x, (((long long)n * H + p * kh + a) * W + q * kw + b) * C + c));
    st(y, i, m);
  }
}
// gradient to the FIRST maximum of each window (row-major), 0 elsewhere
template <typename T>
__global__ void k_maxpool_bwd(const T* __restrict__ x, const T* __restrict__ dy, int N, int H, int W, int C, int kh,
                              int kw, int P, int Q, T* __restrict__ dx) {
  const long long n_in = (long long)N * H * W * C;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_in; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    const int p = h / kh, q = w / kw;
    float g = 0.f;
    if (p < P && q < Q) {
      float m = -INFINITY;
      int am = 0;
      for (int a = 0; a < kh; ++a)
        for (int b = 0; b < kw; ++b) {
          const float v = ld(x, (((long long)n * H + p * kh + a) * W + q * kw + b) * C + c);
          if (v > m) { m = v; am = a * kw + b; }
        }
      if (am == (h - p * kh) * kw + (w - q * kw)) g = ld(dy, (((long long)n * P + p) * Q + q) * C + c);
    }
    st(dx, i, g);
  }
}
// vectorised: one thread per (output window, 8 channels)
template <typename T, int KH, int KW>
__global__ void __launch_bounds__(256) k_maxpool8(const T* __restrict__ x, int N, int H, int W, int C, int P, int Q,
                                                  T* __restrict__ y) {
  const int CV = C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < total; v += gridDim.x * 256) {
    const int cv = (int)(v % CV);
    unsigned t = v / CV;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
#pragma unroll
    for (int a = 0; a < KH; ++a)
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        float f[8];
        ld8(x + (((size_t)n * H + p * KH + a) * W + q * KW + b) * C + cv * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
      }
    st8(y + (size_t)v * 8, m);
  }
}
template <typename T, int KH, int KW>
__global__ void __launch_bounds__(256) k_maxpool_bwd8(const T* __restrict__ x, const T* __restrict__ dy, int N,
                                                      int H, int W, int C, int P, int Q, T* __restrict__ dx) {
  const int CV = C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < total; v += gridDim.x * 256) {
    const int cv = (int)(v % CV);
    unsigned t = v / CV;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float f[KH * KW][8], m[8], g[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY, am[j] = 0;
#pragma unroll
    for (int a = 0; a < KH; ++a)
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        ld8(x + (((size_t)n * H + p * KH + a) * W + q * KW + b) * C + cv * 8, f[a * KW + b]);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[a * KW + b][j] > m[j]) m[j] = f[a * KW + b][j], am[j] = a * KW + b;
      }
    ld8(dy + (size_t)v * 8, g);
#pragma unroll
    for (int a = 0; a < KH; ++a)
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = am[j] == a * KW + b ? g[j] : 0.f;
        st8(dx + (((size_t)n * H + p * KH + a) * W + q * KW + b) * C + cv * 8, o);
      }
    // leftover columns / rows of a non-divisible input receive zero gradient
    const float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (q == Q - 1)
      for (int a = 0; a < KH; ++a)
        for (int w = Q * KW; w < W; ++w) st8(dx + (((size_t)n * H + p * KH + a) * W + w) * C + cv * 8, z);
    if (p == P - 1)
      for (int h = P * KH; h < H; ++h) {
        for (int w = q * KW; w < q * KW + KW; ++w) st8(dx + (((size_t)n * H + h) * W + w) * C + cv * 8, z);
        if (q == Q - 1)
          for (int w = Q * KW; w < W; ++w) st8(dx + (((size_t)n * H + h) * W + w) * C + cv * 8, z);
      }
  }
}
#define MAXPOOL_SHAPES(X) X(1, 2) X(2, 2) X(3, 3)

ACFE_API int acfe_maxpool2d(const void* x, int N, int H, int W, int C, int kh, int kw, void* y, int dtype,
                            void* stream) {
  if (!x || !y || N < 0 || kh <= 0 || kw <= 0 || H < kh || W < kw) return ACFE_E_INVAL;
  const int P = H / kh, Q = W / kw;
  const long long n = (long long)N * P * Q * C;
  if (n == 0) return ACFE_OK;
  if (vec_ok((long long)N * H * W * C, C, x, y) && (long long)N * P * Q * (C / 8) < 0xFFFFFFFFll) {
#define MP(A, B)                                                                                             \
  if (kh == A && kw == B) {                                                                                  \
    DISPATCH1(dtype, T, hipLaunchKernelGGL((k_maxpool8<T, A, B>), dim3(vgrid(n / 8)), dim3(256), 0,          \
                                           strm(stream), (const T*)x, N, H, W, C, P, Q, (T*)y));             \
    return launch_rc("acfe_maxpool2d");                                                                      \
  }
    MAXPOOL_SHAPES(MP)
#undef MP
  }
  DISPATCH1(dtype, T, hipLaunchKernelGGL(k_maxpool<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream), (const T*)x,
                                         N, H, W, C, kh, kw, P, Q, (T*)y));
  return launch_rc("acfe_maxpool2d");
}
ACFE_API int acfe_maxpool2d_bwd(const void* x, const void* dy, int N, int H, int W, int C, int kh, int kw,
                                void* dx, int dtype, void* stream) {
  if (!x || !dy || !dx || N < 0 || kh <= 0 || kw <= 0) return ACFE_E_INVAL;
  const int P = H / kh, Q = W / kw;
  const long long n = (long long)N * H * W * C;
  if (n == 0) return ACFE_OK;
  if (vec_ok(n, C, x, dy, dx) && (long long)N * P * Q * (C / 8) < 0xFFFFFFFFll && P > 0 && Q > 0) {
    const long long nw = (long long)N * P * Q * (C / 8);
#define MPB(A, B)                                                                                           \
  if (kh == A && kw == B) {                                                                                 \
    DISPATCH1(dtype, T, hipLaunchKernelGGL((k_maxpool_bwd8<T, A, B>), dim3(vgrid(nw)), dim3(256), 0,        \
                                           strm(stream), (const T*)x, (const T*)dy, N, H, W, C, P, Q, (T*)dx)); \
    return launch_rc("acfe_maxpool2d_bwd");                                                                 \
  }
    MAXPOOL_SHAPES(MPB)
#undef MPB
  }
  DISPATCH1(dtype, T, hipLaunchKernelGGL(k_maxpool_bwd<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream),
                                         (const T*)x, (const T*)dy, N, H, W, C, kh, kw, P, Q, (T*)dx));
  return launch_rc("acfe_maxpool2d_bwd");
}

// ---------------------------------------------------------------- fused pooling
// y = [dropout](maxpool(x)); optional argmax byte per output element (first
// maximum, as the backward of the reference), optional BN statistics of y.
template <typename T, int KH, int KW>
__global__ void __launch_bounds__(256) k_maxpool8x(const T* __restrict__ x, int N, int H, int W, int C, int P, int Q,
                                                   T* __restrict__ y, uint8_t* __restrict__ amax, Drop drop,
                                                   double* __restrict__ part, const float* __restrict__ bsc,
                                                   const float* __restrict__ bsh, int brelu) {
  extern __shared__ double red[];  // [2][C] when part
  if (part) {
    for (int i = threadIdx.x; i < 2 * C; i += 256) red[i] = 0.0;
    __syncthreads();
  }
  const int CV = C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  double sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.0;
  const unsigned v0 = blockIdx.x * 256 + threadIdx.x;
  for (unsigned v = v0; v < total; v += gridDim.x * 256) {
    const int cv = (int)(v % CV);
    unsigned t = v / CV;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float m[8], s8[8], h8[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY, am[j] = 0;
    if (bsc) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s8[j] = bsc[cv * 8 + j], h8[j] = bsh[cv * 8 + j];
    }
#pragma unroll
    for (int a = 0; a < KH; ++a)
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        float f[8];
        ld8(x + (((size_t)n * H + p * KH + a) * W + q * KW + b) * C + cv * 8, f);
        if (bsc) {
          // the BatchNormalization (+ReLU) output acfe_bn_apply would have stored
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float v = f[j] * s8[j] + h8[j];
            if (brelu) v = fmaxf(v, 0.f);
            f[j] = rnd(v, T());
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[j] > m[j]) m[j] = f[j], am[j] = a * KW + b;
      }
    if (drop.on) drop_apply8<T>(drop, (uint64_t)v * 8, (uint64_t)total * 8 <= (1ull << 32), m);
    st8(y + (size_t)v * 8, m);
    if (amax) {
      uint2 pk;
      pk.x = am[0] | (am[1] << 8) | (am[2] << 16) | (am[3] << 24);
      pk.y = am[4] | (am[5] << 8) | (am[6] << 16) | (am[7] << 24);
      *reinterpret_cast<uint2*>(amax + (size_t)v * 8) = pk;
    }
    if (part) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float r = rnd(m[j], T());
        sa[j] += r;
        sb[j] += (double)r * r;
      }
    }
  }
  if (part) stats8_flush(sa, sb, (int)(v0 % CV), C, v0 < total, red, part);
}

// dx from the saved argmax bytes: dy is first passed through the dropout of
// the forward (when drop.on), exactly as acfe_dropout would have stored it.
template <typename T, int KH, int KW>
__global__ void __launch_bounds__(256) k_maxpool_bwd8i(const uint8_t* __restrict__ amax, const T* __restrict__ dy,
                                                       int N, int H, int W, int C, int P, int Q, Drop drop,
                                                       T* __restrict__ dx) {
  const int CV = C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < total; v += gridDim.x * 256) {
    const int cv = (int)(v % CV);
    unsigned t = v / CV;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float g[8];
    ld8(dy + (size_t)v * 8, g);
    if (drop.on) drop_apply8<T>(drop, (uint64_t)v * 8, (uint64_t)total * 8 <= (1ull << 32), g);
    const uint2 pk = *reinterpret_cast<const uint2*>(amax + (size_t)v * 8);
    int am[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) am[j] = (pk.x >> (8 * j)) & 0xff, am[4 + j] = (pk.y >> (8 * j)) & 0xff;
#pragma unroll
    for (int a = 0; a < KH; ++a)
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = am[j] == a * KW + b ? g[j] : 0.f;
        st8(dx + (((size_t)n * H + p * KH + a) * W + q * KW + b) * C + cv * 8, o);
      }
    const float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (q == Q - 1)
      for (int a = 0; a < KH; ++a)
        for (int w = Q * KW; w < W; ++w) st8(dx + (((size_t)n * H + p * KH + a) * W + w) * C + cv * 8, z);
    if (p == P - 1)
      for (int h = P * KH; h < H; ++h) {
        for (int w = q * KW; w < q * KW + KW; ++w) st8(dx + (((size_t)n * H + h) * W + w) * C + cv * 8, z);
        if (q == Q - 1)
          for (int w = Q * KW; w < W; ++w) st8(dx + (((size_t)n * H + h) * W + w) * C + cv * 8, z);
      }
  }
}

// k_maxpool_bwd8i + the BatchNormalization backward reduce of the BN in front
// of the pool (the stem's BatchNormalization -> MaxPool2D((1, 2)),
// wr_resnet_bird.py:29-30): each expanded gradient value g is also masked by
// the BN's ReLU (x * scale + shift > 0 when relu) and summed as g and
// g * (x - mean) * invstd per channel, with x read at the same pixels --
// acfe_bn_bwd_reduce's slab [gridDim][2][C] without its second read of the
// expanded gradient.  Grid = red_blocks(N * H * W) (the slab rows the BN
// finalizer expects); positions outside the pooled windows (H, W not a
// multiple of the window) carry a zero gradient and add nothing.
template <typename T, int KH, int KW>
__global__ void __launch_bounds__(256) k_maxpool_bwd8i_bn(const uint8_t* __restrict__ amax, const T* __restrict__ dy,
                                                          int N, int H, int W, int C, int P, int Q,
                                                          T* __restrict__ dx, const T* __restrict__ x,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, int relu,
                                                          double* __restrict__ part) {
  extern __shared__ double red[];
  for (int i = threadIdx.x; i < 2 * C; i += 256) red[i] = 0.0;
  __syncthreads();
  // a workgroup walks pooled rows (n, p); its threads cover the row's Q * CV
  // 16-B vectors, JU of them per pass with all their loads issued first.
  // 256 % CV == 0 (stats8_ok): CV is a power of two and a thread's channel
  // vector cv is the same in every pass
  constexpr int JU = 2;
  const int CV = C >> 3, lcv = __builtin_ctz(CV), RV = Q * CV;
  const int cv = threadIdx.x & (CV - 1);
  float sc[8], sh[8], mu[8], is[8], a[8], b[8];
  double da[8], db[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[cv * 8 + j], sh[j] = shift[cv * 8 + j], mu[j] = mean[cv * 8 + j], is[j] = invstd[cv * 8 + j];
    a[j] = b[j] = 0.f, da[j] = db[j] = 0.0;
  }
  const float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int rows = N * P;
  int cnt = 0;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    const int n = r / P, p = r - n * P;
    const size_t pin = (size_t)r * RV;                       // first vector of the pooled row
    const size_t fin = ((size_t)n * H + p * KH) * W * CV;    // first vector of its full-resolution band
    for (int j0 = threadIdx.x; j0 < RV; j0 += 256 * JU) {
      float g[JU][8], xv[JU][KH * KW][8];
      uint2 pk[JU];
#pragma unroll
      for (int u = 0; u < JU; ++u) {
        const int j = j0 + 256 * u, jj = j < RV ? j : j0, q = jj >> lcv;
        ld8(dy + (pin + jj) * 8, g[u]);
        pk[u] = *reinterpret_cast<const uint2*>(amax + (pin + jj) * 8);
#pragma unroll
        for (int aa = 0; aa < KH; ++aa)
#pragma unroll
          for (int bb = 0; bb < KW; ++bb)
            ld8(x + (fin + ((size_t)aa * W + q * KW + bb) * CV + cv) * 8, xv[u][aa * KW + bb]);
      }
#pragma unroll
      for (int u = 0; u < JU; ++u) {
        const int j = j0 + 256 * u;
        if (j >= RV) break;
        const int q = j >> lcv;
        int am[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) am[k] = (pk[u].x >> (8 * k)) & 0xff, am[4 + k] = (pk[u].y >> (8 * k)) & 0xff;
#pragma unroll
        for (int aa = 0; aa < KH; ++aa)
#pragma unroll
          for (int bb = 0; bb < KW; ++bb) {
            const float* xw = xv[u][aa * KW + bb];
            float o[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              o[k] = am[k] == aa * KW + bb ? g[u][k] : 0.f;
              const float gk = (relu && !(xw[k] * sc[k] + sh[k] > 0.f)) ? 0.f : o[k];
              a[k] += gk;
              b[k] += gk * ((xw[k] - mu[k]) * is[k]);
            }
            st8(dx + (fin + ((size_t)aa * W + q * KW + bb) * CV + cv) * 8, o);
          }
        // positions outside the pooled windows: zero gradient (no sums)
        if (q == Q - 1)
          for (int aa = 0; aa < KH; ++aa)
            for (int w = Q * KW; w < W; ++w) st8(dx + (fin + ((size_t)aa * W + w) * CV + cv) * 8, z);
        if (p == P - 1)
          for (int h = P * KH; h < H; ++h) {
            const size_t hr = ((size_t)n * H + h) * W;
            for (int w = q * KW; w < q * KW + KW; ++w) st8(dx + ((hr + w) * CV + cv) * 8, z);
            if (q == Q - 1)
              for (int w = Q * KW; w < W; ++w) st8(dx + ((hr + w) * CV + cv) * 8, z);
          }
      }
    }
    if (++cnt == 16) {
#pragma unroll
      for (int j = 0; j < 8; ++j) da[j] += a[j], db[j] += b[j], a[j] = b[j] = 0.f;
      cnt = 0;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) da[j] += a[j], db[j] += b[j];
  stats8_flush(da, db, cv, C, true, red, part);
}


static int maxpool_fused_impl(const void* x, int N, int H, int W, int C, int kh, int kw, void* y, uint8_t* argmax,
                              float drop_rate, unsigned long long seed, double* stats_part, int dtype,
                              const float* bsc, const float* bsh, int brelu, void* stream) {
  if (!x || !y || N <= 0 || kh <= 0 || kw <= 0 || H < kh || W < kw || drop_rate < 0.f || drop_rate >= 1.f)
    return ACFE_E_INVAL;
  const int P = H / kh, Q = W / kw;
  const long long rows = (long long)N * P * Q;
  if (!vec_ok((long long)N * H * W * C, C, x, y) || ((uintptr_t)argmax & 7) || rows * (C / 8) >= 0xFFFFFFFFll ||
      (stats_part && !stats8_ok(C)) || (!bsc != !bsh))
    return ACFE_E_INVAL;
  const Drop d = make_drop(drop_rate, seed);
  const int grid = stats_part ? red_blocks(rows) : vgrid(rows * C / 8);
  const size_t shm = stats_part ? 2 * C * sizeof(double) : 0;
#define MPF(A, B)                                                                                           \
  if (kh == A && kw == B) {                                                                                 \
    DISPATCH1(dtype, T, hipLaunchKernelGGL((k_maxpool8x<T, A, B>), dim3(grid), dim3(256), shm, strm(stream),  \
                                           (const T*)x, N, H, W, C, P, Q, (T*)y, argmax, d, stats_part, bsc,  \
                                           bsh, brelu));                                                     \
    return launch_rc("acfe_maxpool2d_fused");                                                               \
  }
  MAXPOOL_SHAPES(MPF)
#undef MPF
  return ACFE_E_INVAL;
}

ACFE_API int acfe_maxpool2d_fused(const void* x, int N, int H, int W, int C, int kh, int kw, void* y,
                                  uint8_t* argmax, float drop_rate, unsigned long long seed, double* stats_part,
                                  int dtype, void* stream) {
  return maxpool_fused_impl(x, N, H, W, C, kh, kw, y, argmax, drop_rate, seed, stats_part, dtype, nullptr, nullptr, 0,
                            stream);
}

// MaxPool2D of BatchNormalization(x) (+ReLU): the normalised tensor is formed in
// registers at load time and never stored (scale / shift from acfe_bn_finalize).
ACFE_API int acfe_bn_maxpool2d_fused(const void* x, int N, int H, int W, int C, const float* scale,
                                     const float* shift, int relu, int kh, int kw, void* y, uint8_t* argmax,
                                     double* stats_part, int dtype, void* stream) {
  if (!scale || !shift) return ACFE_E_INVAL;
  return maxpool_fused_impl(x, N, H, W, C, kh, kw, y, argmax, 0.f, 0, stats_part, dtype, scale, shift, relu ? 1 : 0,
                            stream);
}

ACFE_API int acfe_maxpool2d_bwd_argmax(const uint8_t* argmax, const void* dy, int N, int H, int W, int C, int kh,
                                       int kw, float drop_rate, unsigned long long seed, void* dx, int dtype,
                                       void* stream) {
  if (!argmax || !dy || !dx || N <= 0 || kh <= 0 || kw <= 0 || H < kh || W < kw || drop_rate < 0.f ||
      drop_rate >= 1.f)
    return ACFE_E_INVAL;
  const int P = H / kh, Q = W / kw;
  const long long nw = (long long)N * P * Q * (C / 8);
  if (!vec_ok((long long)N * H * W * C, C, dy, dx) || ((uintptr_t)argmax & 7) || nw >= 0xFFFFFFFFll)
    return ACFE_E_INVAL;
  const Drop d = make_drop(drop_rate, seed);
#define MPBI(A, B)                                                                                          \
  if (kh == A && kw == B) {                                                                                 \
    DISPATCH1(dtype, T, hipLaunchKernelGGL((k_maxpool_bwd8i<T, A, B>), dim3(vgrid(nw)), dim3(256), 0,       \
                                           strm(stream), argmax, (const T*)dy, N, H, W, C, P, Q, d, (T*)dx)); \
    return launch_rc("acfe_maxpool2d_bwd_argmax");                                                          \
  }
  MAXPOOL_SHAPES(MPBI)
#undef MPBI
  return ACFE_E_INVAL;
}

// acfe_maxpool2d_bwd_argmax (no dropout) fused with acfe_bn_bwd_reduce of the
// BatchNormalization whose output was pooled: x = that BN's input [N][H][W][C],
// part = its reduce slab [acfe_reduce_blocks(N * H * W)][2][C].
ACFE_API int acfe_maxpool2d_bwd_argmax_bn(const uint8_t* argmax, const void* dy, int N, int H, int W, int C, int kh,
                                          int kw, void* dx, int dtype, const void* x, const float* scale,
                                          const float* shift, const float* mean, const float* invstd, int relu,
                                          double* part, void* stream) {
  if (!argmax || !dy || !dx || !x || !scale || !shift || !mean || !invstd || !part || N <= 0 || kh <= 0 ||
      kw <= 0 || H < kh || W < kw || !stats8_ok(C))
    return ACFE_E_INVAL;
  const int P = H / kh, Q = W / kw;
  if (!vec_ok((long long)N * H * W * C, C, dy, dx, x) || ((uintptr_t)argmax & 7) || (long long)N * P >= (1ll << 31))
    return ACFE_E_INVAL;
  const int grid = red_blocks((long long)N * H * W);
#define MPBB(A, B)                                                                                             \
  if (kh == A && kw == B) {                                                                                    \
    DISPATCH1(dtype, T, hipLaunchKernelGGL((k_maxpool_bwd8i_bn<T, A, B>), dim3(grid), dim3(256),               \
                                           2 * C * sizeof(double), strm(stream), argmax, (const T*)dy, N, H, W, C, \
                                           P, Q, (T*)dx, (const T*)x, scale, shift, mean, invstd, relu, part));   \
    return launch_rc("acfe_maxpool2d_bwd_argmax_bn");                                                          \
  }
  MAXPOOL_SHAPES(MPBB)
#undef MPBB
  return ACFE_E_INVAL;
}

// z = a + b (+ReLU) with the BN statistics of z (slab rows = acfe_reduce_blocks(rows)).
template <typename T>
__global__ void __launch_bounds__(256) k_add8s(const T* __restrict__ a, const T* __restrict__ b, unsigned nvec,
                                               int C, int relu, T* __restrict__ z, double* __restrict__ part) {
  extern __shared__ double red[];
  for (int i = threadIdx.x; i < 2 * C; i += 256) red[i] = 0.0;
  __syncthreads();
  const int CV = C >> 3;
  double sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sa[j] = sb[j] = 0.0;
  const unsigned v0 = blockIdx.x * 256 + threadIdx.x;
  for (unsigned v = v0; v < nvec; v += gridDim.x * 256) {
    float x[8], y[8];
    ld8(a + (size_t)v * 8, x);
    ld8(b + (size_t)v * 8, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x[j] = relu ? fmaxf(x[j] + y[j], 0.f) : x[j] + y[j];
      const float r = rnd(x[j], T());
      sa[j] += r;
      sb[j] += (double)r * r;
    }
    st8(z + (size_t)v * 8, x);
  }
  stats8_flush(sa, sb, (int)(v0 % CV), C, v0 < nvec, red, part);
}

ACFE_API int acfe_add_stats(const void* a, const void* b, long long rows, int C, int relu, void* z, int dtype,
                            double* part, void* stream) {
  if (!a || !b || !z || !part || rows <= 0 || !stats8_ok(C) || !vec_ok(rows * C, C, a, b, z)) return ACFE_E_INVAL;
  DISPATCH1(dtype, T, hipLaunchKernelGGL(k_add8s<T>, dim3(red_blocks(rows)), dim3(256), 2 * C * sizeof(double),
                                         strm(stream), (const T*)a, (const T*)b, (unsigned)(rows * C / 8), C, relu,
                                         (T*)z, part));
  return launch_rc("acfe_add_stats");
}

// AveragePooling2D(pool=k, strides=k, padding="same"): P = ceil(H/k); TF pads
// (total = (P-1)*k + k - H) with pad_top = total/2 and averages over the
// in-bounds elements only.
template <typename T>
__global__ void k_avgpool(const T* __restrict__ x, int N, int H, int W, int C, int k, int P, int Q, int pt, int pl,
                          T* __restrict__ y) {
  const long long n_out = (long long)N * P * Q * C;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_out; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float s = 0.f;
    int cnt = 0;
    for (int a = 0; a < k; ++a)
      for (int b = 0; b < k; ++b) {
        const int h = p * k - pt + a, w = q * k - pl + b;
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
          s += ld(x, (((long long)n * H + h) * W + w) * C + c);
          ++cnt;
        }
      }
    st(y, i, s / (float)cnt);
  }
}
template <typename T>
__global__ void k_avgpool_bwd(const T* __restrict__ dy, int N, int H, int W, int C, int k, int P, int Q, int pt,
                              int pl, T* __restrict__ dx) {
  const long long n_in = (long long)N * H * W * C;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_in; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    const int p = (h + pt) / k, q = (w + pl) / k;
    float g = 0.f;
    if (p < P && q < Q) {
      int cnt = 0;
      for (int a = 0; a < k; ++a)
        for (int b = 0; b < k; ++b) {
          const int hh = p * k - pt + a, ww = q * k - pl + b;
          cnt += ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) ? 1 : 0;
        }
      g = ld(dy, (((long long)n * P + p) * Q + q) * C + c) / (float)cnt;
    }
    st(dx, i, g);
  }
}
// 8-channel versions: one thread per (output window, 8 channels); the windows
// tile the padded input exactly (stride == pool), so the backward writes every
// input element once.
template <typename T>
__global__ void __launch_bounds__(256) k_avgpool8(const T* __restrict__ x, int N, int H, int W, int C, int k, int P,
                                                  int Q, int pt, int pl, T* __restrict__ y) {
  const int CV = C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < total; v += gridDim.x * 256) {
    const int cv = (int)(v % CV);
    unsigned t = v / CV;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int cnt = 0;
    for (int a = 0; a < k; ++a) {
      const int h = p * k - pt + a;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int b = 0; b < k; ++b) {
        const int w = q * k - pl + b;
        if ((unsigned)w >= (unsigned)W) continue;
        float f[8];
        ld8(x + (((size_t)n * H + h) * W + w) * C + cv * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
        ++cnt;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = s[j] / (float)cnt;
    st8(y + (size_t)v * 8, s);
  }
}
template <typename T>
__global__ void __launch_bounds__(256) k_avgpool_bwd8(const T* __restrict__ dy, int N, int H, int W, int C, int k,
                                                      int P, int Q, int pt, int pl, T* __restrict__ dx) {
  const int CV = C >> 3;
  const unsigned total = (unsigned)N * P * Q * CV;
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < total; v += gridDim.x * 256) {
    const int cv = (int)(v % CV);
    unsigned t = v / CV;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    const int h0 = max(p * k - pt, 0), h1 = min(p * k - pt + k, H);
    const int w0 = max(q * k - pl, 0), w1 = min(q * k - pl + k, W);
    const float inv = 1.0f / (float)((h1 - h0) * (w1 - w0));
    float g[8];
    ld8(dy + (size_t)v * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = g[j] * inv;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) st8(dx + (((size_t)n * H + h) * W + w) * C + cv * 8, g);
  }
}

ACFE_API int acfe_avgpool2d(const void* x, int N, int H, int W, int C, int k, void* y, int dtype, void* stream) {
  if (!x || !y || N < 0 || k <= 0) return ACFE_E_INVAL;
  const int P = (H + k - 1) / k, Q = (W + k - 1) / k;
  const int pt = ((P - 1) * k + k - H) / 2, pl = ((Q - 1) * k + k - W) / 2;
  const long long n = (long long)N * P * Q * C;
  if (n == 0) return ACFE_OK;
  if (vec_ok((long long)N * H * W * C, C, x, y) && n / 8 < 0xFFFFFFFFll) {
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_avgpool8<T>, dim3(vgrid(n / 8)), dim3(256), 0, strm(stream),
                                           (const T*)x, N, H, W, C, k, P, Q, pt, pl, (T*)y));
    return launch_rc("acfe_avgpool2d");
  }
  DISPATCH1(dtype, T, hipLaunchKernelGGL(k_avgpool<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream), (const T*)x,
                                         N, H, W, C, k, P, Q, pt, pl, (T*)y));
  return launch_rc("acfe_avgpool2d");
}
ACFE_API int acfe_avgpool2d_bwd(const void* dy, int N, int H, int W, int C, int k, void* dx, int dtype,
                                void* stream) {
  if (!dy || !dx || N < 0 || k <= 0) return ACFE_E_INVAL;
  const int P = (H + k - 1) / k, Q = (W + k - 1) / k;
  const int pt = ((P - 1) * k + k - H) / 2, pl = ((Q - 1) * k + k - W) / 2;
  const long long n = (long long)N * H * W * C;
  if (n == 0) return ACFE_OK;
  const long long nw = (long long)N * P * Q * (C / 8);
  if (vec_ok(n, C, dy, dx) && nw < 0xFFFFFFFFll) {
    DISPATCH1(dtype, T, hipLaunchKernelGGL(k_avgpool_bwd8<T>, dim3(vgrid(nw)), dim3(256), 0, strm(stream),
                                           (const T*)dy, N, H, W, C, k, P, Q, pt, pl, (T*)dx));
    return launch_rc("acfe_avgpool2d_bwd");
  }
  DISPATCH1(dtype, T, hipLaunchKernelGGL(k_avgpool_bwd<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream),
                                         (const T*)dy, N, H, W, C, k, P, Q, pt, pl, (T*)dx));
  return launch_rc("acfe_avgpool2d_bwd");
}

// ---------------------------------------------------------------- log-mean-exp / mean pooling
// x viewed as [outer][L][inner] -> y [outer][inner] fp32:
//   mode 0 (LME, wr_resnet_bird.py:83-87): (logsumexp(s*x) - log L) / s
//   mode 1 (mean, GlobalAveragePooling2D per axis): sum x / L
template <typename T>
__global__ void k_axis_pool(const T* __restrict__ x, long long outer, int L, int inner, float s, int mode,
                            float* __restrict__ y) {
  const long long n = outer * inner;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long o = i / inner;
    const int in = (int)(i % inner);
    const T* xp = x + o * (long long)L * inner + in;
    if (mode == 0) {
      // tfp.math.reduce_logmeanexp(s x) / s: s x rounded once (no fp
      // contraction: a fused fma(s, x, -m) left the max element's rounding
      // residual in the exponent, expf(+256) = inf at |s x| ~ 5e9), shifted by
      // its max -- by 0 when the max is not finite, as reduce_logsumexp does
#pragma clang fp contract(off)
      float m = -INFINITY;
      for (int l = 0; l < L; ++l) m = fmaxf(m, __fmul_rn(s, ld(xp, (long long)l * inner)));
      const float sh = isfinite(m) ? m : 0.f;
      float acc = 0.f;
      for (int l = 0; l < L; ++l) acc += expf(__fmul_rn(s, ld(xp, (long long)l * inner)) - sh);
      y[i] = (sh + logf(acc) - logf((float)L)) / s;
    } else {
      float acc = 0.f;
      for (int l = 0; l < L; ++l) acc += ld(xp, (long long)l * inner);
      y[i] = acc / (float)L;
    }
  }
}
// dx = dy * softmax(s*x) along L (LME) or dy / L (mean)
template <typename T>
__global__ void k_axis_pool_bwd(const T* __restrict__ x, const float* __restrict__ dy, long long outer, int L,
                                int inner, float s, int mode, T* __restrict__ dx) {
  const long long n = outer * inner;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long o = i / inner;
    const int in = (int)(i % inner);
    const long long base = o * (long long)L * inner + in;
    const float g = dy[i];
    if (mode == 0) {
      // (the forward's rounding of s x and its shift)
#pragma clang fp contract(off)
      float m = -INFINITY;
      for (int l = 0; l < L; ++l) m = fmaxf(m, __fmul_rn(s, ld(x, base + (long long)l * inner)));
      const float sh = isfinite(m) ? m : 0.f;
      float acc = 0.f;
      for (int l = 0; l < L; ++l) acc += expf(__fmul_rn(s, ld(x, base + (long long)l * inner)) - sh);
      const float inv = 1.f / acc;
      for (int l = 0; l < L; ++l) {
        const long long j = base + (long long)l * inner;
        st(dx, j, g * expf(__fmul_rn(s, ld(x, j)) - sh) * inv);
      }
    } else {
      for (int l = 0; l < L; ++l) st(dx, base + (long long)l * inner, g / (float)L);
    }
  }
}
ACFE_API int acfe_axis_pool(const void* x, int x_dtype, long long outer, int L, int inner, float sharpness,
                            int mode, float* y, void* stream) {
  if (!x || !y || outer < 0 || L <= 0 || inner <= 0 || (mode == 0 && sharpness == 0.f)) return ACFE_E_INVAL;
  const long long n = outer * inner;
  if (n == 0) return ACFE_OK;
  DISPATCH1(x_dtype, T, hipLaunchKernelGGL(k_axis_pool<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream),
                                           (const T*)x, outer, L, inner, sharpness, mode, y));
  return launch_rc("acfe_axis_pool");
}
ACFE_API int acfe_axis_pool_bwd(const void* x, int x_dtype, const float* dy, long long outer, int L, int inner,
                                float sharpness, int mode, void* dx, void* stream) {
  if (!x || !dy || !dx || outer < 0 || L <= 0 || inner <= 0) return ACFE_E_INVAL;
  const long long n = outer * inner;
  if (n == 0) return ACFE_OK;
  DISPATCH1(x_dtype, T, hipLaunchKernelGGL(k_axis_pool_bwd<T>, dim3(grid_for(n)), dim3(256), 0, strm(stream),
                                           (const T*)x, dy, outer, L, inner, sharpness, mode, (T*)dx));
  return launch_rc("acfe_axis_pool_bwd");
}

// ---------------------------------------------------------------- Dense (+sigmoid) and losses
// z[b][o] = sum_i x[b][i] * w[i][o] + bias[o]   (Keras kernel layout [in][out])
__global__ void k_dense(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
                        int B, int I, int O, float* __restrict__ z) {
  for (int t = blockIdx.x * 256 + threadIdx.x; t < B * O; t += gridDim.x * 256) {
    const int b = t / O, o = t % O;
    float acc = bias ? bias[o] : 0.f;
    for (int i = 0; i < I; ++i) acc += x[(long long)b * I + i] * w[(long long)i * O + o];
    z[t] = acc;
  }
}
ACFE_API int acfe_dense_fwd(const float* x, const float* w, const float* bias, int B, int I, int O, float* z,
                            void* stream) {
  if (!x || !w || !z || B < 0 || I <= 0 || O <= 0) return ACFE_E_INVAL;
  if (B == 0) return ACFE_OK;
  hipLaunchKernelGGL(k_dense, dim3(grid_for((long long)B * O)), dim3(256), 0, strm(stream), x, w, bias, B, I, O, z);
  return launch_rc("acfe_dense_fwd");
}
// dx = dz w^T ; dw = x^T dz ; db = sum_b dz   (dw/db overwritten)
__global__ void k_dense_bwd_x(const float* __restrict__ dz, const float* __restrict__ w, int B, int I, int O,
                              float* __restrict__ dx) {
  for (int t = blockIdx.x * 256 + threadIdx.x; t < B * I; t += gridDim.x * 256) {
    const int b = t / I, i = t % I;
    float acc = 0.f;
    for (int o = 0; o < O; ++o) acc += dz[(long long)b * O + o] * w[(long long)i * O + o];
    dx[t] = acc;
  }
}
// dw[i][o] = sum_b x[b][i] dz[b][o], db[o] = sum_b dz[b][o]: one wave per
// output, its lanes striding the batch (a thread-serial loop over B = 512 was
// bound by its dependent load latency: 132 us per T1 step), fixed-order
// butterfly sum in float64
__global__ void __launch_bounds__(256) k_dense_bwd_w(const float* __restrict__ x, const float* __restrict__ dz, int B,
                                                     int I, int O, float* __restrict__ dw, float* __restrict__ db) {
  const int lane = threadIdx.x & 63;
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < (I + 1) * O; t += gridDim.x * 4) {
    const int i = t / O, o = t % O;
    if (i == I && !db) continue;
    double acc = 0.0;
    for (int b = lane; b < B; b += 64) {
      const double g = dz[(long long)b * O + o];
      acc += i < I ? (double)x[(long long)b * I + i] * g : g;
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) acc += __shfl_xor(acc, m, 64);
    if (lane == 0) {
      if (i < I) dw[t] = (float)acc;
      else db[o] = (float)acc;
    }
  }
}
ACFE_API int acfe_dense_bwd(const float* x, const float* w, const float* dz, int B, int I, int O, float* dx,
                            float* dw, float* db, void* stream) {
  if (!x || !w || !dz || !dw || B < 0 || I <= 0 || O <= 0) return ACFE_E_INVAL;
  if (dx && B > 0)
    hipLaunchKernelGGL(k_dense_bwd_x, dim3(grid_for((long long)B * I)), dim3(256), 0, strm(stream), dz, w, B, I, O,
                       dx);
  const long long nw = (long long)(I + 1) * O;  // one wave per output
  hipLaunchKernelGGL(k_dense_bwd_w, dim3((unsigned)std::min<long long>((nw + 3) / 4, 8192)), dim3(256), 0,
                     strm(stream), x, dz, B, I, O, dw, db);
  return launch_rc("acfe_dense_bwd");
}

// Loss on Dense(sigmoid) outputs; z = logits [B][L], y = targets.
//  mode 0 BCE (tf.keras.losses.BinaryCrossentropy on a sigmoid output, computed
//         from the logits: max(z,0) - z*y + log1p(exp(-|z|)), mean over L then B)
//  mode 1 CCE (tf.keras.losses.CategoricalCrossentropy, from_logits=False:
//         q = p / sum p, clip to [1e-7, 1-1e-7], -sum y log q, mean over B)
// Writes loss[0] (mean over the batch) and dz = dL/dz.  One block per row.
__global__ void __launch_bounds__(256) k_loss(const float* __restrict__ z, const float* __restrict__ y, int B,
                                              int L, int mode, float inv_scale, float* __restrict__ row_loss,
                                              float* __restrict__ dz) {
  const int b = blockIdx.x;
  __shared__ float red[4];
  __shared__ float sh[2];
  const float* zr = z + (long long)b * L;
  const float* yr = y + (long long)b * L;
  float* dr = dz + (long long)b * L;
  if (mode == 0) {
    float acc = 0.f;
    for (int i = threadIdx.x; i < L; i += 256) {
      const float zz = zr[i], yy = yr[i];
      acc += fmaxf(zz, 0.f) - zz * yy + log1pf(expf(-fabsf(zz)));
      const float p = 1.f / (1.f + expf(-zz));
      dr[i] = (p - yy) / (float)L * inv_scale;
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) row_loss[b] = (red[0] + red[1] + red[2] + red[3]) / (float)L;
  } else {
    float sp = 0.f;
    for (int i = threadIdx.x; i < L; i += 256) sp += 1.f / (1.f + expf(-zr[i]));
    sp = wave_sum(sp);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sp;
    __syncthreads();
    const float S = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    const float lo = 1e-7f, hi = 1.f - 1e-7f;
    float acc = 0.f, gq = 0.f;
    for (int i = threadIdx.x; i < L; i += 256) {
      const float p = 1.f / (1.f + expf(-zr[i]));
      const float q = p / S;
      const float qc = fminf(fmaxf(q, lo), hi);
      acc += -yr[i] * logf(qc);
      const float g = (q >= lo && q <= hi) ? -yr[i] / qc : 0.f;  // dL/dq
      gq += g * q;
    }
    acc = wave_sum(acc);
    gq = wave_sum(gq);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) sh[0] = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = gq;
    __syncthreads();
    if (threadIdx.x == 0) sh[1] = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    const float sgq = sh[1];
    for (int i = threadIdx.x; i < L; i += 256) {
      const float p = 1.f / (1.f + expf(-zr[i]));
      const float q = p / S;
      const float qc = fminf(fmaxf(q, lo), hi);
      const float g = (q >= lo && q <= hi) ? -yr[i] / qc : 0.f;
      const float dp = (g - sgq) / S;  // dL/dp_j = (g_j - sum_i g_i q_i) / S
      dr[i] = dp * p * (1.f - p) * inv_scale;
    }
    if (threadIdx.x == 0) row_loss[b] = sh[0];
  }
}
__global__ void k_mean(const float* __restrict__ v, int n, float* __restrict__ out) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) acc += v[i];
  acc = wave_sumd(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (float)((red[0] + red[1] + red[2] + red[3]) / n);
}
// workspace: float[B]; grad_scale multiplies dz (e.g. 1/B for a batch mean)
ACFE_API int acfe_loss(const float* z, const float* y, int B, int L, int mode, float grad_scale, float* loss,
                       float* dz, float* workspace, void* stream) {
  if (!z || !y || !loss || !dz || !workspace || B <= 0 || L <= 0 || (mode != 0 && mode != 1))
    return ACFE_E_INVAL;
  hipLaunchKernelGGL(k_loss, dim3(B), dim3(256), 0, strm(stream), z, y, B, L, mode, grad_scale, workspace, dz);
  int rc = launch_rc("acfe_loss");
  if (rc) return rc;
  hipLaunchKernelGGL(k_mean, dim3(1), dim3(256), 0, strm(stream), workspace, B, loss);
  return launch_rc("acfe_loss(mean)");
}

__global__ void k_sigmoid(const float* __restrict__ z, long long n, float* __restrict__ p) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    p[i] = 1.f / (1.f + expf(-z[i]));
}
ACFE_API int acfe_sigmoid(const float* z, long long n, float* p, void* stream) {
  if (!z || !p || n < 0) return ACFE_E_INVAL;
  if (n == 0) return ACFE_OK;
  hipLaunchKernelGGL(k_sigmoid, dim3(grid_for(n)), dim3(256), 0, strm(stream), z, n, p);
  return launch_rc("acfe_sigmoid");
}

// ---------------------------------------------------------------- Adam (Keras 3)
// m += (g - m)(1-b1); v += (g^2 - v)(1-b2); p -= alpha * m / (sqrt(v) + eps),
// alpha = lr * sqrt(1 - b2^t) / (1 - b1^t) computed by the caller; g is scaled
// by grad_scale first (e.g. 1/world_size after a sum all-reduce).
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, long long n, float grad_scale, float b1, float b2, float eps,
                       float alpha) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float gi = g[i] * grad_scale;
    float mi = m[i], vi = v[i];
    mi += (gi - mi) * (1.f - b1);
    vi += (gi * gi - vi) * (1.f - b2);
    m[i] = mi;
    v[i] = vi;
    p[i] -= alpha * mi / (sqrtf(vi) + eps);
  }
}
ACFE_API int acfe_adam_step(float* params, const float* grads, float* m, float* v, long long n, float grad_scale,
                            float beta1, float beta2, float eps, float alpha, void* stream) {
  if (!params || !grads || !m || !v || n < 0) return ACFE_E_INVAL;
  if (n == 0) return ACFE_OK;
  hipLaunchKernelGGL(k_adam, dim3(grid_for(n, 256, 4096)), dim3(256), 0, strm(stream), params, grads, m, v, n,
                     grad_scale, beta1, beta2, eps, alpha);
  return launch_rc("acfe_adam_step");
}

// dst[i] = src[i] cast (bf16 <-> fp32), for packing model inputs / outputs
template <typename TI, typename TO>
__global__ void k_cast(const TI* __restrict__ x, long long n, TO* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    st(y, i, ld(x, i));
}
template <typename TI, typename TO>
__global__ void k_cast8(const TI* __restrict__ x, unsigned nvec, TO* __restrict__ y) {
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) {
    float f[8];
    ld8(x + (size_t)v * 8, f);
    st8(y + (size_t)v * 8, f);
  }
}
ACFE_API int acfe_cast(const void* x, int x_dtype, long long n, void* y, int y_dtype, void* stream) {
  if (!x || !y || n < 0) return ACFE_E_INVAL;
  if (n == 0) return ACFE_OK;
  if (vec_ok(n, 8, x, y)) {
    DISPATCH1(x_dtype, TI, DISPATCH1(y_dtype, TO,
        hipLaunchKernelGGL((k_cast8<TI, TO>), dim3(vgrid(n / 8)), dim3(256), 0, strm(stream), (const TI*)x,
                           (unsigned)(n / 8), (TO*)y)));
    return launch_rc("acfe_cast");
  }
  DISPATCH1(x_dtype, TI, DISPATCH1(y_dtype, TO,
      hipLaunchKernelGGL((k_cast<TI, TO>), dim3(grid_for(n)), dim3(256), 0, strm(stream), (const TI*)x, n,
                         (TO*)y)));
  return launch_rc("acfe_cast");
}

// out[c] = beta*out[c] + sum_rows x[r][c]  (bias gradients); part: bn_stats slab
__global__ void __launch_bounds__(SLAB_THREADS) k_chan_sum_fin(const double* __restrict__ part, int nrows, int C, float beta,
                                                      float* __restrict__ out) {
  __shared__ double s[2][SLAB_CH];
  slab_sum(part, nrows, C, C, s);
  const int c = blockIdx.x * SLAB_CH + threadIdx.x;
  if (threadIdx.x >= SLAB_CH || c >= C) return;
  out[c] = beta != 0.f ? out[c] * beta + (float)s[0][threadIdx.x] : (float)s[0][threadIdx.x];
}
// out[c] = beta*out[c] + sum of a slab's first row set (part [nrows][2][C]).
ACFE_API int acfe_channel_sum_finalize(const double* part, int nrows, int C, float beta, float* out, void* stream) {
  if (!part || !out || nrows <= 0 || C <= 0) return ACFE_E_INVAL;
  hipLaunchKernelGGL(k_chan_sum_fin, dim3(cdiv(C, SLAB_CH)), dim3(SLAB_THREADS), 0, strm(stream), part, nrows, C, beta, out);
  return launch_rc("acfe_channel_sum_finalize");
}
ACFE_API int acfe_channel_sum(const void* x, long long rows, int C, int dtype, double* part, float* out,
                              float beta, void* stream) {
  if (!out || C <= 0) return ACFE_E_INVAL;
  if (rows == 0) return hip_rc(hipMemsetAsync(out, 0, sizeof(float) * C, strm(stream)), "acfe_channel_sum");
  int rc = acfe_bn_stats(x, rows, C, dtype, part, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_chan_sum_fin, dim3(cdiv(C, SLAB_CH)), dim3(SLAB_THREADS), 0, strm(stream), part, red_blocks(rows), C, beta,
                     out);
  return launch_rc("acfe_channel_sum");
}
