// Feature front end: normalize, mix_up, STFT -> |X|^p -> banded mel, PCEN.
// Reference: tfdataset.py:1916-1934 (normalize), :930-955 (mix_up),
// :2007-2059 (raw_to_mel), predict_utils.py:163-239 (get_spect),
// custommel.py:18-61 (mel_f, mel_spec), tfpcen.py:8-110 (EMA, PCEN, minmax).
//
// Design (gfx950): one 256-thread workgroup per (clip, group of frames).
// The n_fft real FFT is computed as an n_fft/2-point complex FFT of
// z[n] = x[2n] + i x[2n+1] with radix-8/4/2 Stockham passes: each thread
// keeps its butterfly in VGPRs and exchanges through one LDS buffer
// (16 KB at n_fft=4096); the first pass reads HBM/L2 directly (framing,
// Hann window and optional per-clip normalisation fused into the load).
// Only the bins covered by the mel filterbank are post-processed into power,
// and the filterbank is applied as a banded sum (1839 taps at M=128 instead
// of the reference's dense 128x2049 batch_dot).
#include "common.h"

// ACFE_MEL_CUT stops each frame after pass N (timing only, wrong results):
// only in `make ablate` builds (libacfe_ablate.so)
#if !defined(ACFE_ABLATE) && defined(ACFE_MEL_CUT)
#error "ACFE_MEL_CUT belongs to `make ablate` builds only"
#endif
#include <cmath>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace acfe;

struct acfe_plan_s {
  int sr, n_fft, hop, n_mels, n_bins;
  int kmin, kmax;
  float2* d_tw;   // W_{n_fft/2}^k, k < n_fft/2
  float2* d_rtw;  // W_{n_fft}^k, k <= n_fft/2
  float* d_win;   // periodic Hann [n_fft]
  int* d_band;    // [n_mels][3]: start bin, length, offset into d_vals
  float* d_vals;
  int device;
};

// ------------------------------------------------------------ host: mel_f
// custommel.py:18-54 restated in C (float64 math, float32 storage; numpy's
// rfftfreq / linspace / in-place float32 *= float64 semantics reproduced).
ACFE_API int acfe_mel_filterbank(int sr, int n_mels, double fmin, double fmax, int n_fft,
                                 double break_freq, float* out) {
  if (sr <= 0 || n_mels <= 0 || n_fft <= 0 || !out || break_freq <= 0) return ACFE_E_INVAL;
  const int nb = 1 + n_fft / 2;
  const int nm2 = n_mels + 2;
  std::vector<double> ff(nb), mf(nm2);
  const double d = 1.0 / sr;
  const double val = 1.0 / (n_fft * d);  // numpy.fft.rfftfreq
  for (int k = 0; k < nb; ++k) ff[k] = k * val;
  const double lo = 2595.0 * std::log10(1.0 + fmin / break_freq);
  const double hi = 2595.0 * std::log10(1.0 + fmax / break_freq);
  const double step = (hi - lo) / (nm2 - 1);  // numpy.linspace
  for (int i = 0; i < nm2; ++i) {
    double m = (i == nm2 - 1) ? hi : i * step + lo;
    mf[i] = break_freq * (std::pow(10.0, m / 2595.0) - 1.0);
  }
  for (int i = 0; i < n_mels; ++i) {
    const double fd0 = mf[i + 1] - mf[i], fd1 = mf[i + 2] - mf[i + 1];
    const double enorm = 2.0 / (mf[i + 2] - mf[i]);
    for (int k = 0; k < nb; ++k) {
      const double lower = -(mf[i] - ff[k]) / fd0;
      const double upper = (mf[i + 2] - ff[k]) / fd1;
      double w = std::fmin(lower, upper);
      if (!(w > 0.0)) w = 0.0;
      const float w32 = (float)w;
      out[(size_t)i * nb + k] = (float)((double)w32 * enorm);
    }
  }
  return ACFE_OK;
}

ACFE_API int acfe_plan_create(int sr, int n_fft, int hop, int n_mels, double fmin, double fmax,
                              double break_freq, const float* w_host, acfe_plan_t* plan) {
  if (!plan || n_fft < 256 || n_fft > 4096 || (n_fft & (n_fft - 1)) || hop <= 0 || n_mels <= 0 ||
      n_mels > 1024)
    return ACFE_E_INVAL;
  const int nb = 1 + n_fft / 2, nc = n_fft / 2;
  std::vector<float> w;
  if (!w_host) {
    w.resize((size_t)n_mels * nb);
    int rc = acfe_mel_filterbank(sr, n_mels, fmin, fmax, n_fft, break_freq, w.data());
    if (rc) return rc;
    w_host = w.data();
  }
  std::vector<int> band(3 * n_mels);
  std::vector<float> vals;
  int kmin = nb, kmax = -1;
  for (int m = 0; m < n_mels; ++m) {
    int s = -1, e = -1;
    for (int k = 0; k < nb; ++k)
      if (w_host[(size_t)m * nb + k] != 0.f) {
        if (s < 0) s = k;
        e = k;
      }
    if (s < 0) {
      band[3 * m] = 0;
      band[3 * m + 1] = 0;
      band[3 * m + 2] = (int)vals.size();
      continue;
    }
    band[3 * m] = s;
    band[3 * m + 1] = e - s + 1;
    band[3 * m + 2] = (int)vals.size();
    for (int k = s; k <= e; ++k) vals.push_back(w_host[(size_t)m * nb + k]);
    while (vals.size() & 7) vals.push_back(0.f);  // k_mel_w4 reads whole 8-tap groups
    kmin = s < kmin ? s : kmin;
    kmax = e > kmax ? e : kmax;
  }
  if (kmax < 0) kmin = kmax = 0;
  if (vals.empty()) vals.push_back(0.f);
  std::vector<float2> tw(nc), rtw(nc + 1);
  std::vector<float> win(n_fft);
  for (int k = 0; k < nc; ++k) {
    const double a = -2.0 * M_PI * (double)k / nc;
    tw[k] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  for (int k = 0; k <= nc; ++k) {
    const double a = -2.0 * M_PI * (double)k / n_fft;
    rtw[k] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  for (int i = 0; i < n_fft; ++i) win[i] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * i / n_fft));

  acfe_plan_s* p = new acfe_plan_s();
  p->sr = sr; p->n_fft = n_fft; p->hop = hop; p->n_mels = n_mels; p->n_bins = nb;
  p->kmin = kmin; p->kmax = kmax;
  (void)hipGetDevice(&p->device);
  hipError_t e = hipSuccess;
  e = e ? e : hipMalloc(&p->d_tw, sizeof(float2) * nc);
  e = e ? e : hipMalloc(&p->d_rtw, sizeof(float2) * (nc + 1));
  e = e ? e : hipMalloc(&p->d_win, sizeof(float) * n_fft);
  e = e ? e : hipMalloc(&p->d_band, sizeof(int) * 3 * n_mels);
  e = e ? e : hipMalloc(&p->d_vals, sizeof(float) * vals.size());
  e = e ? e : hipMemcpy(p->d_tw, tw.data(), sizeof(float2) * nc, hipMemcpyHostToDevice);
  e = e ? e : hipMemcpy(p->d_rtw, rtw.data(), sizeof(float2) * (nc + 1), hipMemcpyHostToDevice);
  e = e ? e : hipMemcpy(p->d_win, win.data(), sizeof(float) * n_fft, hipMemcpyHostToDevice);
  e = e ? e : hipMemcpy(p->d_band, band.data(), sizeof(int) * 3 * n_mels, hipMemcpyHostToDevice);
  e = e ? e : hipMemcpy(p->d_vals, vals.data(), sizeof(float) * vals.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    acfe_plan_destroy(p);
    return hip_rc(e, "acfe_plan_create");
  }
  *plan = p;
  return ACFE_OK;
}

ACFE_API int acfe_plan_destroy(acfe_plan_t p) {
  if (!p) return ACFE_E_INVAL;
  (void)hipFree(p->d_tw); (void)hipFree(p->d_rtw); (void)hipFree(p->d_win); (void)hipFree(p->d_band); (void)hipFree(p->d_vals);
  delete p;
  return ACFE_OK;
}

ACFE_API int acfe_plan_num_frames(acfe_plan_t p, int n, int pad_mode) {
  if (!p || n <= 0) return ACFE_E_INVAL;
  if (pad_mode == ACFE_PAD_END) return (n + p->hop - 1) / p->hop;
  return 1 + n / p->hop;
}

// ------------------------------------------------------------ normalize
// One 1024-thread block per clip; 16-B loads (when the clip start is 16-B
// aligned) with four independent min/max pairs per thread keep enough loads in
// flight to stream the clip at HBM rate (the scalar 256-thread version ran at
// 1.2 TB/s).
__global__ void __launch_bounds__(1024) k_norm_stats(const float* __restrict__ x, int64_t cs, int n,
                                                     float* __restrict__ stats) {
  const float* xb = x + (int64_t)blockIdx.x * cs;
  float mn[4] = {INFINITY, INFINITY, INFINITY, INFINITY}, mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int head = 0;
  if ((reinterpret_cast<uintptr_t>(xb) & 15) == 0) {
    const int nv = n >> 2;
    const float4* xv = reinterpret_cast<const float4*>(xb);
    int i = threadIdx.x;
    for (; i + 3 * 1024 < nv; i += 4 * 1024) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = xv[i + u * 1024];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        mn[u] = fminf(fminf(mn[u], v[u].x), fminf(v[u].y, fminf(v[u].z, v[u].w)));
        mx[u] = fmaxf(fmaxf(mx[u], v[u].x), fmaxf(v[u].y, fmaxf(v[u].z, v[u].w)));
      }
    }
    for (; i < nv; i += 1024) {
      const float4 v = xv[i];
      mn[0] = fminf(fminf(mn[0], v.x), fminf(v.y, fminf(v.z, v.w)));
      mx[0] = fmaxf(fmaxf(mx[0], v.x), fmaxf(v.y, fmaxf(v.z, v.w)));
    }
    head = nv << 2;
  }
  for (int i = head + threadIdx.x; i < n; i += 1024) {
    const float v = xb[i];
    mn[1] = fminf(mn[1], v);
    mx[1] = fmaxf(mx[1], v);
  }
  float a = fminf(fminf(mn[0], mn[1]), fminf(mn[2], mn[3]));
  float c = fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3]));
  __shared__ float smn[16], smx[16];
  a = wave_min(a);
  c = wave_max(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smn[w] = a; smx[w] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = smn[0];
    c = smx[0];
    for (int k = 1; k < 16; ++k) a = fminf(a, smn[k]), c = fmaxf(c, smx[k]);
    stats[2 * blockIdx.x] = a;
    stats[2 * blockIdx.x + 1] = c - a;  // == max(x - min) (fl is monotone)
  }
}

// norm1 with the division as a multiply by rinv = RN(1 / rng) and one FMA
// correction (Markstein): q = RN(t rinv), e = t - rng q (exact by FMA),
// RN(q + e rinv) = RN(t / rng) -- the correctly rounded quotient without the
// ~10-instruction division sequence (k_mel_w4 divides every sample of every
// overlapping frame; exhaustive-style check of the identity: 20 000 random
// float32 pairs incl. all-ones-mantissa divisors, exact rational arithmetic)
__device__ __forceinline__ float norm1r(float v, float mn, float rng, float rinv) {
  const float t = __fsub_rn(v, mn);
  const float q0 = __fmul_rn(t, rinv);
  const float e = __builtin_fmaf(-q0, rng, t);
  float q = __builtin_fmaf(e, rinv, q0);
  q = __fadd_rn(q, 0.000001f);
  q = __fsub_rn(q, 0.5f);
  return __fmul_rn(q, 2.0f);
}
__device__ __forceinline__ float norm1(float v, float mn, float rng) {
  // tfdataset.py:1927-1931, float32, same order: -min, /max, +1e-6, -0.5, *2
  float t = __fsub_rn(v, mn);
  t = __fdiv_rn(t, rng);
  t = __fadd_rn(t, 0.000001f);
  t = __fsub_rn(t, 0.5f);
  return __fmul_rn(t, 2.0f);
}

ACFE_API int acfe_normalize_stats(const float* x, int64_t cs, int batch, int n, float* stats,
                                  void* stream) {
  if (batch == 0 && n > 0) return ACFE_OK;
  if (!x || !stats || batch < 0 || n <= 0) return ACFE_E_INVAL;
  if (batch == 0) return ACFE_OK;
  hipLaunchKernelGGL(k_norm_stats, dim3(batch), dim3(1024), 0, strm(stream), x, cs, n, stats);
  return launch_rc("acfe_normalize_stats");
}

// y may alias x (in place, cs == n): each element is read and written by one thread.
__global__ void k_norm_apply(const float* x, int64_t cs, int n, const float* __restrict__ stats, float* y) {
  const int b = blockIdx.y;
  const float mn = stats[2 * b], rng = stats[2 * b + 1];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    y[(int64_t)b * n + i] = norm1(x[(int64_t)b * cs + i], mn, rng);
}

ACFE_API int acfe_normalize_apply(const float* x, int64_t cs, int batch, int n, const float* stats,
                                  float* y, void* stream) {
  if (!x || !stats || !y || batch < 0 || n <= 0 || batch > 65535) return ACFE_E_INVAL;
  if (batch == 0) return ACFE_OK;
  hipLaunchKernelGGL(k_norm_apply, dim3(cdiv(n, 256 * 8), batch), dim3(256), 0, strm(stream), x, cs,
                     n, stats, y);
  return launch_rc("acfe_normalize_apply");
}

__global__ void k_mixup(const float* __restrict__ x1, const float* __restrict__ s1,
                        const float* __restrict__ x2, const float* __restrict__ s2,
                        const float* __restrict__ lam, int n, float* __restrict__ y) {
  // tfdataset.py:950 is two products and a sum, each rounded (TF ops, no
  // fusion): without this the a * l + (c * l1) pair contracts to an FMA
#pragma clang fp contract(off)
  const int b = blockIdx.y;
  const float l = lam[b];
  const float l1 = __fsub_rn(1.0f, l);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int64_t o = (int64_t)b * n + i;
    float a = x1[o], c = x2[o];
    if (s1) a = norm1(a, s1[2 * b], s1[2 * b + 1]);
    if (s2) c = norm1(c, s2[2 * b], s2[2 * b + 1]);
    // (plain operators: the contraction state of __fmul_rn / __fadd_rn is
    // their header's, where the pair still fuses)
    const float p1 = a * l, p2 = c * l1;
    y[o] = p1 + p2;  // tfdataset.py:950
  }
}

ACFE_API int acfe_mixup(const float* x1, const float* s1, const float* x2, const float* s2,
                        const float* lam, int batch, int n, float* y, void* stream) {
  if (!x1 || !x2 || !lam || !y || batch < 0 || n <= 0 || batch > 65535) return ACFE_E_INVAL;
  if (batch == 0) return ACFE_OK;
  hipLaunchKernelGGL(k_mixup, dim3(cdiv(n, 256 * 8), batch), dim3(256), 0, strm(stream), x1, s1, x2,
                     s2, lam, n, y);
  return launch_rc("acfe_mixup");
}

// Row copies of the loader's device-resident clip pool (tfdataset
// AudioDataset): dst[dst_idx[i]][0:n) = src[src_idx[i]][0:n) for i < count
// (a NULL index list is the identity): chunk -> free pool slots (scatter) and
// pool slots -> batch (gather); 16-B vectors when strides, n and both bases
// allow.
template <typename V>
__global__ void k_copy_rows(const V* __restrict__ src, int64_t ss, const int* __restrict__ si, V* __restrict__ dst,
                            int64_t ds, const int* __restrict__ di, int n) {
  const int b = blockIdx.y;
  const V* s = src + (int64_t)(si ? si[b] : b) * ss;
  V* d = dst + (int64_t)(di ? di[b] : b) * ds;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) d[i] = s[i];
}

ACFE_API int acfe_copy_rows(const float* src, int64_t src_stride, int64_t src_rows, const int* src_idx,
                            float* dst, int64_t dst_stride, int64_t dst_rows, const int* dst_idx, int count, int n,
                            void* stream) {
  if (!src || !dst || count < 0 || count > 65535 || n <= 0 || src_stride < n || dst_stride < n ||
      (!src_idx && count > src_rows) || (!dst_idx && count > dst_rows))
    return ACFE_E_INVAL;
  if (count == 0) return ACFE_OK;
  const bool v4 = src_stride % 4 == 0 && dst_stride % 4 == 0 && n % 4 == 0 && ((uintptr_t)src & 15) == 0 &&
                  ((uintptr_t)dst & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(k_copy_rows<float4>, dim3(cdiv(n / 4, 256 * 8), count), dim3(256), 0, strm(stream),
                       reinterpret_cast<const float4*>(src), src_stride / 4, src_idx, reinterpret_cast<float4*>(dst),
                       dst_stride / 4, dst_idx, n / 4);
  else
    hipLaunchKernelGGL(k_copy_rows<float>, dim3(cdiv(n, 256 * 8), count), dim3(256), 0, strm(stream), src,
                       src_stride, src_idx, dst, dst_stride, dst_idx, n);
  return launch_rc("acfe_copy_rows");
}

// ------------------------------------------------------------ FFT helpers
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // a * (-i)

template <int R>
__device__ __forceinline__ void dft(float2* v);

template <>
__device__ __forceinline__ void dft<2>(float2* v) {
  float2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
template <>
__device__ __forceinline__ void dft<4>(float2* v) {
  float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
  float2 t2 = cadd(v[1], v[3]), t3 = mul_mi(csub(v[1], v[3]));
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = cadd(t1, t3);
  v[3] = csub(t1, t3);
}
template <>
__device__ __forceinline__ void dft<8>(float2* v) {
  float2 e[4] = {v[0], v[2], v[4], v[6]};
  float2 o[4] = {v[1], v[3], v[5], v[7]};
  dft<4>(e);
  dft<4>(o);
  const float c = 0.70710678118654752440f;
  // W8^1 = c(1 - i), W8^2 = -i, W8^3 = -c(1 + i)
  float2 o1 = make_float2(c * (o[1].x + o[1].y), c * (o[1].y - o[1].x));
  float2 o2 = mul_mi(o[2]);
  float2 o3 = make_float2(c * (o[3].y - o[3].x), -c * (o[3].x + o[3].y));
  v[0] = cadd(e[0], o[0]); v[4] = csub(e[0], o[0]);
  v[1] = cadd(e[1], o1);   v[5] = csub(e[1], o1);
  v[2] = cadd(e[2], o2);   v[6] = csub(e[2], o2);
  v[3] = cadd(e[3], o3);   v[7] = csub(e[3], o3);
}

// LDS index with one float2 of padding per 8 (breaks the power-of-two strides
// of the Stockham writes: pass-1 stores go from 8-way conflicted to conflict-free).
__device__ __forceinline__ int padx(int i) { return i + (i >> 3); }

// One in-place Stockham pass (Govindaraju et al. formulation) over NC points
// held in LDS `buf`, radix R, span Ns.  256 threads.
template <int NC, int R>
__device__ __forceinline__ void stockham_pass(float2* buf, int Ns, const float2* __restrict__ tw) {
  constexpr int NB = NC / R;
  constexpr int PER = (NB + 255) / 256;
  float2 v[PER][R];
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int j = threadIdx.x + 256 * p;
    if (NB % 256 == 0 || j < NB) {
      const int jm = j & (Ns - 1);
      const int tstep = jm * (NC / (Ns * R));
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float2 a = buf[padx(j + r * NB)];
        if (r) a = cmul(a, tw[r * tstep]);
        v[p][r] = a;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int j = threadIdx.x + 256 * p;
    if (NB % 256 == 0 || j < NB) {
      dft<R>(v[p]);
      const int idxD = (j / Ns) * Ns * R + (j & (Ns - 1));
#pragma unroll
      for (int r = 0; r < R; ++r) buf[padx(idxD + r * Ns)] = v[p][r];
    }
  }
  __syncthreads();
}

// Fetch one (optionally normalised) sample of the framed signal.
__device__ __forceinline__ float fetch(const float* __restrict__ xb, int n, int idx, int pad_mode,
                                       bool do_norm, float mn, float rng) {
  if (pad_mode == ACFE_PAD_CENTER_REFLECT) {
    if (idx < 0) idx = -idx;
    if (idx >= n) idx = 2 * (n - 1) - idx;
  }
  if (idx < 0 || idx >= n) return 0.f;
  const float v = xb[idx];
  return do_norm ? norm1(v, mn, rng) : v;
}

// Whether fetch() reads a signal sample at idx (else it returns the zero pad).
__device__ __forceinline__ bool in_sig(int idx, int n, int pad_mode) {
  return pad_mode == ACFE_PAD_CENTER_REFLECT || (idx >= 0 && idx < n);
}

template <int NC>
__global__ void __launch_bounds__(256) k_mel(const float* __restrict__ raw, int64_t cs, int n,
                                             const float* __restrict__ stats, int pad_mode,
                                             int power, int n_frames, int fpb, int hop,
                                             const float2* __restrict__ tw,
                                             const float2* __restrict__ rtw,
                                             const float* __restrict__ win,
                                             const int* __restrict__ band,
                                             const float* __restrict__ vals, int n_mels, int kmin,
                                             int kmax, float* __restrict__ out, int layout) {
  constexpr int L = 2 * NC;
  constexpr int NB0 = NC / 8;  // first pass butterflies
  constexpr int PER0 = (NB0 + 255) / 256;
  __shared__ float2 buf[NC + NC / 8];
  __shared__ float pw[NC + 1];
  __shared__ float2 stw[NC];      // complex-FFT twiddles, staged once per block
  for (int i = threadIdx.x; i < NC; i += 256) stw[i] = tw[i];
  const int b = blockIdx.y;
  const float* xb = raw + (int64_t)b * cs;
  const bool do_norm = stats != nullptr;
  const float mn = do_norm ? stats[2 * b] : 0.f, rng = do_norm ? stats[2 * b + 1] : 1.f;
  const int nk = kmax - kmin + 1;
  const int f0 = blockIdx.x * fpb;
  for (int f = f0; f < f0 + fpb && f < n_frames; ++f) {
    const int start = (pad_mode == ACFE_PAD_END) ? f * hop : f * hop - L / 2;
    // ---- pass 1 (Ns = 1, radix 8) straight from memory: z[j + r*NB0]
    {
      float2 v[PER0][8];
#pragma unroll
      for (int p = 0; p < PER0; ++p) {
        const int j = threadIdx.x + 256 * p;
        if (NB0 % 256 == 0 || j < NB0) {
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int nn = j + r * NB0;
            const float a = fetch(xb, n, start + 2 * nn, pad_mode, do_norm, mn, rng) * win[2 * nn];
            const float c = fetch(xb, n, start + 2 * nn + 1, pad_mode, do_norm, mn, rng) * win[2 * nn + 1];
            v[p][r] = make_float2(a, c);
          }
          dft<8>(v[p]);
        }
      }
      __syncthreads();  // previous frame's readers of buf are done
#pragma unroll
      for (int p = 0; p < PER0; ++p) {
        const int j = threadIdx.x + 256 * p;
        if (NB0 % 256 == 0 || j < NB0) {
#pragma unroll
          for (int r = 0; r < 8; ++r) buf[padx(j * 8 + r)] = v[p][r];
        }
      }
      __syncthreads();
    }
    int Ns = 8;
    while (Ns * 8 <= NC) {
      stockham_pass<NC, 8>(buf, Ns, stw);
      Ns *= 8;
    }
    if (NC / Ns == 4) stockham_pass<NC, 4>(buf, Ns, stw);
    else if (NC / Ns == 2) stockham_pass<NC, 2>(buf, Ns, stw);
    // ---- real-FFT post-processing + power, only for bins in [kmin, kmax]
    for (int i = threadIdx.x; i < nk; i += 256) {
      const int k = kmin + i;
      const float2 zk = buf[padx(k & (NC - 1))];
      const float2 zm = buf[padx((NC - k) & (NC - 1))];
      // E = (zk + conj(zm))/2, O = (zk - conj(zm)) / (2i)
      const float2 E = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
      const float2 D = make_float2(zk.x - zm.x, zk.y + zm.y);
      const float2 O = make_float2(0.5f * D.y, -0.5f * D.x);
      const float2 X = cadd(E, cmul(rtw[k], O));
      const float p2 = X.x * X.x + X.y * X.y;
      pw[i] = power == 2 ? p2 : sqrtf(p2);
    }
    __syncthreads();
    // ---- banded mel
    for (int m = threadIdx.x; m < n_mels; m += 256) {
      const int s = band[3 * m], len = band[3 * m + 1], off = band[3 * m + 2];
      float acc = 0.f;
      for (int i = 0; i < len; ++i) acc += vals[off + i] * pw[s - kmin + i];
      const size_t o = layout == ACFE_LAYOUT_BTM ? ((size_t)b * n_frames + f) * n_mels + m
                                                 : ((size_t)b * n_mels + m) * n_frames + f;
      out[o] = acc;
    }
    // next frame's first __syncthreads protects buf/pw reuse
  }
}

// ---- k_mel_w4 (n_fft = 4096): two waves (128 threads) per frame, 4 frames
// per workgroup.  Frame + periodic Hann (computed, not loaded) + the 4096-point
// real FFT as a 2048-point complex FFT of the even / odd sample pairs (radix
// 16 / 16 / 8 Stockham passes through a 16 KB LDS frame buffer, base twiddles
// held in VGPRs and their powers recomputed per frame) + real-FFT
// post-processing and |X|^power of bins kmin..kmax + the banded mel sums (one
// band per lane, zero-padded 8-tap groups).  r04 over the r02-r03 kernel
// (k_mel_w2: padded LDS, pass-3 results stored and re-read by the
// post-processing, 148 VGPRs): one LDS round trip fewer, no bank conflicts,
// 128 VGPRs (4 waves per SIMD); T1 1.16 -> 0.91 ms per 512 clips (k_mel_w3).
//  * LDS holds the 2048 points unpadded under the XOR swizzle msw(i) = i ^
//    ((i >> 4) & 15): ds_write_b64 serves 16-lane groups on 32 banks (a
//    float2 index mod 16 per lane), ds_read_b64 32-lane groups on 64 banks
//    (mod 32), and under msw the pass-1 rows (stride 16), the pass-2 stores
//    (16-point runs) and the pass-2 / pass-3 reads (consecutive points) are all
//    conflict-free (the r04 first cut XORed bits 5..8 in: its pass-1 stores
//    were 2-way, 32 % of the LDS cycles in conflicts, SQ counters r04c).
//  * Pass 3 (radix 8, span 256) gives lane t the butterflies j0 = t and
//    j1 = 256 - t (j1 = 128 for t = 0), i.e. the complex bins j + 256 r that
//    the real-FFT post-processing pairs as k <-> 2048 - k: the |X|^power of
//    every bin is formed from the lane's own registers, with the post twiddle
//    W_4096^k = W_4096^j W_16^r from one per-lane base, and written straight
//    into the power vector (aliased onto the FFT buffer: 16 KB of LDS per
//    workgroup).
__device__ __forceinline__ int msw(int i) { return i ^ ((i >> 4) & 15); }

// W_16^r = exp(-2 pi i r / 16)
__device__ __forceinline__ float2 w16(int r) {
  constexpr float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f, h = 0.70710678118654752440f;
  switch (r & 15) {
    case 0: return make_float2(1.f, 0.f);
    case 1: return make_float2(c1, -s1);
    case 2: return make_float2(h, -h);
    case 3: return make_float2(s1, -c1);
    case 4: return make_float2(0.f, -1.f);
    case 5: return make_float2(-s1, -c1);
    case 6: return make_float2(-h, -h);
    case 7: return make_float2(-c1, -s1);
    case 8: return make_float2(-1.f, 0.f);
    case 9: return make_float2(-c1, s1);
    case 10: return make_float2(-h, h);
    case 11: return make_float2(-s1, c1);
    case 12: return make_float2(0.f, 1.f);
    case 13: return make_float2(s1, c1);
    case 14: return make_float2(h, h);
    default: return make_float2(c1, s1);
  }
}

// r05 (k_mel_w3 -> k_mel_w4): every complex value in a (re, im) register pair
// and its arithmetic in packed f32 (v_pk_add / v_pk_mul / v_pk_fma_f32: both
// halves per instruction, the f32 VALU's full rate -- k_mel_w3 issued one half
// per instruction and was VALU-issue bound: 4 890 VALU per wave of 4 frames on
// pre-normalised input, now 2 757; profiles/r05/sq_mel_r05z.md).  The products
// by -i (swap + negate) and by a conjugate fold into VOP3P op_sel / neg
// modifiers (inline asm: the compiler materialises the swap with moves);
// products by compile-time twiddles use w and (-w.y, w.x) so they stay one
// v_pk_mul + one v_pk_fma.  |X|^2 is kept as 4 |X|^2 and the band sums scaled
// by 1/4 (|X|: 1/2) -- a power of two, so the same bits.  The normalize-on-
// load arithmetic is the same IEEE sequence per lane (contraction off there);
// the FFT and the band sums (two partial sums per lane, even and odd taps)
// differ from the scalar kernel only in rounding.  The power is a template
// parameter (k_mel_w3 evaluated the |X| square root of every bin and selected).
typedef float v2f __attribute__((ext_vector_type(2)));
#ifndef ACFE_MEL_CUT
#define ACFE_MEL_CUT 0  // timing-only builds: stop each frame after pass 1 / 2 / 3 / the power spectrum
#endif

__device__ __forceinline__ v2f sp2(float x) { return v2f{x, x}; }
// a + (-i) b = (a.x + b.y, a.y - b.x)
__device__ __forceinline__ v2f pk_addmi(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a - (-i) b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ v2f pk_submi(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a + conj(b), a - conj(b)
__device__ __forceinline__ v2f pk_addc(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ v2f pk_subc(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a b: (a.x b.x, a.x b.y) then (.x - a.y b.y, .y + a.y b.x)
__device__ __forceinline__ v2f pk_cmul(v2f a, v2f b) {
  const v2f t = a.xx * b;
  v2f r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=v"(r)
      : "v"(a), "v"(b), "v"(t));
  return r;
}
// a w for a compile-time w, with wr = (-w.y, w.x)
__device__ __forceinline__ v2f pk_cmulk(v2f a, v2f w, v2f wr) { return __builtin_elementwise_fma(a.yy, wr, a.xx * w); }
__device__ __forceinline__ v2f w16v(int r) { const float2 w = w16(r); return v2f{w.x, w.y}; }
__device__ __forceinline__ v2f w16k(v2f a, int r) {
  const float2 w = w16(r);
  return pk_cmulk(a, v2f{w.x, w.y}, v2f{-w.y, w.x});
}
__device__ __forceinline__ v2f pk_conj(v2f a) { return a * v2f{1.f, -1.f}; }

// radix-4 DFT; MI2: v[2] enters multiplied by -i
template <bool MI2 = false>
__device__ __forceinline__ void pdft4(v2f* v) {
  const v2f t0 = MI2 ? pk_addmi(v[0], v[2]) : v[0] + v[2];
  const v2f t1 = MI2 ? pk_submi(v[0], v[2]) : v[0] - v[2];
  const v2f t2 = v[1] + v[3], d = v[1] - v[3];
  v[0] = t0 + t2;
  v[2] = t0 - t2;
  v[1] = pk_addmi(t1, d);
  v[3] = pk_submi(t1, d);
}
__device__ __forceinline__ void pdft8(v2f* v) {
  v2f e[4] = {v[0], v[2], v[4], v[6]};
  v2f o[4] = {v[1], v[3], v[5], v[7]};
  pdft4(e);
  pdft4(o);
  constexpr float c = 0.70710678118654752440f;
  // W8^1 = c(1 - i), W8^2 = -i, W8^3 = -c(1 + i)
  const v2f o1 = pk_cmulk(o[1], v2f{c, -c}, v2f{c, c});
  const v2f o3 = pk_cmulk(o[3], v2f{-c, -c}, v2f{c, -c});
  v[0] = e[0] + o[0]; v[4] = e[0] - o[0];
  v[1] = e[1] + o1;   v[5] = e[1] - o1;
  v[2] = pk_addmi(e[2], o[2]); v[6] = pk_submi(e[2], o[2]);
  v[3] = e[3] + o3;   v[7] = e[3] - o3;
}
__device__ __forceinline__ void pdft16(v2f* v) {
  v2f a[4][4];
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) a[n2][n1] = v[4 * n1 + n2];
    pdft4(a[n2]);
  }
  a[1][1] = w16k(a[1][1], 1);
  a[1][2] = w16k(a[1][2], 2);
  a[1][3] = w16k(a[1][3], 3);
  a[2][1] = w16k(a[2][1], 2);
  a[2][3] = w16k(a[2][3], 6);
  a[3][1] = w16k(a[3][1], 3);
  a[3][2] = w16k(a[3][2], 6);
  a[3][3] = w16k(a[3][3], 9);
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    v2f b[4] = {a[0][k1], a[1][k1], a[2][k1], a[3][k1]};
    if (k1 == 2)
      pdft4<true>(b);  // a[2][2] W16^4 = -i folded into the butterfly
    else
      pdft4(b);
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = b[k2];
  }
}
template <int R>
__device__ __forceinline__ void ptwiddle_pows(const v2f* bw, v2f* w) {
  w[0] = v2f{1.f, 0.f};
  w[1] = bw[0];
  w[2] = bw[1];
  w[3] = pk_cmul(w[1], w[2]);
  w[4] = bw[2];
#pragma unroll
  for (int r = 5; r < 8 && r < R; ++r) w[r] = pk_cmul(w[4], w[r - 4]);
  if constexpr (R == 16) {
    w[8] = bw[3];
#pragma unroll
    for (int r = 9; r < 16; ++r) w[r] = pk_cmul(w[8], w[r - 8]);
  }
}
// 4 |X_k|^2 from zk = Z[k], zm = Z[2048 - k], rt = W_4096^k (rbin_power with
// the halvings pulled out: 2 X = E2 + (-i) rt D)
__device__ __forceinline__ float rbin_power4_pk(v2f zk, v2f zm, v2f rt) {  // 4 |X_k|^2
  const v2f X = pk_addmi(pk_addc(zk, zm), pk_cmul(rt, pk_subc(zk, zm)));
  return X.x * X.x + X.y * X.y;
}
__device__ __forceinline__ v2f& lds2v(v2f* buf, unsigned a) {
  return *reinterpret_cast<v2f*>(reinterpret_cast<char*>(buf) + a);
}

template <int POW>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(4)))
k_mel_w4(const float* __restrict__ raw, int64_t cs, int n, const float* __restrict__ stats, int pad_mode, int,
         int n_frames, int fpw, int hop, const float2* __restrict__ tw, const float2* __restrict__ rtw,
         const int* __restrict__ band, const float* __restrict__ vals, int n_mels, int kmin, int kmax,
         float* __restrict__ out, int layout) {
  constexpr int NC = 2048, L = 2 * NC, NB0 = NC / 16;
  extern __shared__ float2 wbuf_[];
  v2f* wbuf = reinterpret_cast<v2f*>(wbuf_);
  float* pw = reinterpret_cast<float*>(wbuf_);
  const int nk = kmax - kmin + 1;
  const int tid = threadIdx.x;
  // XCD-aware work order: the hardware places workgroup L (x fastest) on XCD
  // L % 8, so consecutive frame groups of a clip -- whose 4096-sample frames
  // overlap by ~3.6 groups -- would land in eight different L2s and each
  // fetch the clip's samples again.  Give every XCD a contiguous range of
  // (clip, frame group) items instead (a bijection when the count is a
  // multiple of 8; otherwise the plain order; r03: 1.35 -> 0.30 GB of HBM
  // reads per launch).
  const int gx = gridDim.x, nwg = gx * gridDim.y, lin = blockIdx.x + gx * blockIdx.y;
  const int item = nwg % 8 == 0 ? (lin % 8) * (nwg / 8) + lin / 8 : lin;
  const int b = item / gx;
  const float* xb = raw + (int64_t)b * cs;
  const bool do_norm = stats != nullptr;
  const float mn = do_norm ? stats[2 * b] : 0.f, rng = do_norm ? stats[2 * b + 1] : 1.f;
  const float rinv = __fdiv_rn(1.0f, rng);
  const int f0 = (item - b * gx) * fpw;
  const int j0 = tid, j1 = tid ? 256 - tid : 128;
  v2f bw2[4], e0[3], rb0;
  {
    const int t = (tid & 15) * 8;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float2 w = tw[(t << q) & (NC - 1)];
      bw2[q] = v2f{w.x, w.y};
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float2 w = tw[(j0 << q) & (NC - 1)];
      e0[q] = v2f{w.x, w.y};
    }
    rb0 = v2f{rtw[j0].x, rtw[j0].y};
  }
  const unsigned ua = (unsigned)msw(16 * tid) * 8u, ub = (unsigned)msw(tid) * 8u;
  const unsigned uc = (unsigned)(256 * (tid >> 4) + (tid & 15)) * 8u;
  const unsigned ud0 = (unsigned)msw(j0) * 8u, ud1 = (unsigned)msw(j1) * 8u;
  constexpr int MAXG = 5;
  // the power spectrum is kept as 4 |X|^2 (|X|^2: 2 |X|); the band sums are
  // scaled back -- by a power of two, so bit for bit the sums of the scaled
  // terms
  constexpr float PSCALE = POW == 2 ? 0.25f : 0.5f;
  const int q0 = tid & 63;
  typedef float f2a __attribute__((ext_vector_type(2), aligned(4)));
  for (int f = f0; f < f0 + fpw && f < n_frames; ++f) {
    unsigned aa = ua, ab = ub, ac = uc, ad0 = ud0, ad1 = ud1;
    asm volatile("" : "+v"(aa), "+v"(ab), "+v"(ac), "+v"(ad0), "+v"(ad1));
    asm volatile("" : "+v"(rb0));
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(bw2[q]));
#pragma unroll
    for (int q = 0; q < 3; ++q) asm volatile("" : "+v"(e0[q]));
    const int start = (pad_mode == ACFE_PAD_END) ? f * hop : f * hop - L / 2;
    const bool inb = start >= 0 && start + L <= n;
    __syncthreads();  // the previous frame's readers of pw are done
    // ---- pass 1 (radix 16, span 1) straight from memory: rows 16 t + r
    {
      const int j = tid;
      v2f xv[16];
      if (inb) {
        const float* xs = xb + start + 2 * j;
#pragma unroll
        for (int r = 0; r < 16; ++r) xv[r] = *reinterpret_cast<const f2a*>(xs + 2 * r * NB0);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int nn = 2 * (j + r * NB0);
          xv[r] = v2f{fetch(xb, n, start + nn, pad_mode, false, 0.f, 1.f),
                      fetch(xb, n, start + nn + 1, pad_mode, false, 0.f, 1.f)};
        }
      }
      // periodic Hann w[n] = 0.5 - 0.5 cos(2 pi n / 4096) of the sample pair
      // n = 2 j + 256 r (+1): cos(theta + 2 pi r / 16) from the lane's cos /
      // sin theta (theta_e = 2 pi j / 2048 = arg conj(W^j), theta_o = theta_e +
      // 2 pi / 4096) -- no window loads, no window registers;
      // doubled (exactly: every rounding scales by 2) to absorb norm1r's final
      // "* 2": (q * 2) * w == q * (2 w) bit for bit
      const float ce = e0[0].x, se = -e0[0].y;
      constexpr float c1 = 0.99999882345170190993f, s1 = 0.00153398018628476550f;
      const float co = ce * c1 - se * s1, so = se * c1 + ce * s1;
      const v2f cc = v2f{ce, co}, ss = v2f{se, so};
      v2f v[16];
      auto hann2 = [&](int r) __attribute__((always_inline)) {
        const float2 u = w16(r);
        return __builtin_elementwise_fma(ss, sp2(-u.y), __builtin_elementwise_fma(cc, sp2(-u.x), sp2(1.f)));
      };
      if (do_norm) {
        // norm1r per lane: the same IEEE operations, packed
#pragma clang fp contract(off)
        const v2f vmn = sp2(mn), vrng = sp2(rng), vri = sp2(rinv);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const v2f t = xv[r] - vmn;
          const v2f q0v = t * vri;
          const v2f e = __builtin_elementwise_fma(-q0v, vrng, t);
          v2f q = __builtin_elementwise_fma(e, vri, q0v);
          q = q + sp2(0.000001f);
          q = q - sp2(0.5f);
          v[r] = q * hann2(r);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float2 u = w16(r);  // the window itself (no doubling)
          v[r] = xv[r] * __builtin_elementwise_fma(ss, sp2(-0.5f * u.y),
                                                   __builtin_elementwise_fma(cc, sp2(-0.5f * u.x), sp2(0.5f)));
        }
      }
      if (do_norm && !inb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int nn = 2 * (j + r * NB0);
          if (!in_sig(start + nn, n, pad_mode)) v[r].x = 0.f;
          if (!in_sig(start + nn + 1, n, pad_mode)) v[r].y = 0.f;
        }
      }
      pdft16(v);
#pragma unroll
      for (int r = 0; r < 16; ++r) lds2v(wbuf, aa ^ (8u * r)) = v[r];
    }
    __syncthreads();
#if ACFE_MEL_CUT == 1
    continue;
#endif
    // ---- pass 2 (radix 16, span 16)
    {
      v2f v[16], w[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = lds2v(wbuf, (ab ^ (64u * (r & 1))) + 1024u * r);
      ptwiddle_pows<16>(bw2, w);
#pragma unroll
      for (int r = 1; r < 16; ++r) v[r] = pk_cmul(v[r], w[r]);
      __syncthreads();
      pdft16(v);
#pragma unroll
      for (int r = 0; r < 16; ++r) lds2v(wbuf, (ac ^ (8u * r)) + 128u * r) = v[r];
    }
    __syncthreads();
#if ACFE_MEL_CUT == 2
    continue;
#endif
    // ---- pass 3 (radix 8, span 256): butterflies j0, j1 -> Z[j + 256 r] in registers
    v2f z[2][8];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const unsigned ad = p ? ad1 : ad0;
#pragma unroll
      for (int r = 0; r < 8; ++r) z[p][r] = lds2v(wbuf, ad + 2048u * r);
      v2f bw[4], w[8];
#pragma unroll
      for (int q = 0; q < 3; ++q) bw[q] = p == 0 ? e0[q] : (tid ? w16k(pk_conj(e0[q]), 2 << q) : w16v(1 << q));
      ptwiddle_pows<8>(bw, w);
#pragma unroll
      for (int r = 1; r < 8; ++r) z[p][r] = pk_cmul(z[p][r], w[r]);
      pdft8(z[p]);
    }
#if ACFE_MEL_CUT == 3
    pw[tid] = z[0][0].x + z[0][1].x + z[0][2].x + z[0][3].x + z[0][4].x + z[0][5].x + z[0][6].x + z[0][7].x + z[1][0].x + z[1][1].x + z[1][2].x + z[1][3].x + z[1][4].x + z[1][5].x + z[1][6].x + z[1][7].x + z[0][0].y + z[1][0].y;
    continue;
#endif
    __syncthreads();  // every lane's pass-3 reads precede the power writes (pw aliases the FFT buffer)
    const v2f rb1 = tid ? w16k(pk_conj(rb0), 1) : v2f{0.98078528040323044913f, -0.19509032201612826785f};
    {
      int tt = tid;
      asm volatile("" : "+v"(tt));
      int rhi0 = kmax >> 8, rhi1 = kmax >= 128 ? (kmax - 128) >> 8 : -1;
      int rlo0 = kmin > 127 ? (kmin - 127 + 255) >> 8 : 0, rlo1 = kmin > 255 ? (kmin - 255 + 255) >> 8 : 0;
      asm volatile("" : "+s"(rhi0), "+s"(rhi1), "+s"(rlo0), "+s"(rlo1));
      const bool l0 = tt == 0;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int kb = (p ? (l0 ? 128 : 256 - tt) : tt) - kmin;
        // bins in groups of four r (uniform skip of a group without a bin in
        // [kmin, kmax]: T1 r >= 4); inside a group no branches, so the four
        // dependent chains interleave (a dependent packed-f32 pair costs a
        // wait state); bins outside the range go to the buffer's last word,
        // which nothing reads (nk + 8 <= 2057 < 4095)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (4 * h + 3 < (p ? rlo1 : rlo0) || 4 * h > (p ? rhi1 : rhi0)) continue;
          // stage by stage over the four bins
          v2f ea[4], da[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = 4 * h + u;
            const v2f zm = l0 ? (p == 0 ? z[0][(8 - r) & 7] : z[1][7 - r]) : z[p ^ 1][7 - r];
            ea[u] = pk_addc(z[p][r], zm);
            da[u] = pk_subc(z[p][r], zm);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) da[u] = pk_cmul(w16k(p ? rb1 : rb0, 4 * h + u), da[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u) ea[u] = pk_addmi(ea[u], da[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = 4 * h + u;
            float pv = ea[u].x * ea[u].x + ea[u].y * ea[u].y;
            if constexpr (POW != 2) pv = sqrtf(pv);
            const int i = kb + 256 * r;
            pw[(unsigned)i < (unsigned)nk ? i : 2 * NC - 1] = pv;
          }
        }
      }
    }
    if (tid == 0 && kmax == NC) {  // Nyquist bin: Z[0] with itself, W_4096^2048 = -1
      float pv = rbin_power4_pk(z[0][0], z[0][0], v2f{-1.f, 0.f});
      if constexpr (POW != 2) pv = sqrtf(pv);
      pw[NC - kmin] = pv;
    }
#if ACFE_MEL_CUT == 4
    continue;
#endif
    if (tid < 8) pw[nk + tid] = 0.f;
    int tq = tid;
    asm volatile("" : "+v"(tq));
    const int m0 = tq < 64 ? q0 : n_mels - 1 - q0;
    const bool b0ok = q0 < (n_mels + 1) / 2 && !(tq >= 64 && m0 == q0);
    int bs0 = 0, bp0 = 0, bo0 = 0;
    if (b0ok) bs0 = band[3 * m0], bp0 = (band[3 * m0 + 1] + 7) & ~7, bo0 = band[3 * m0 + 2];
    float4 wg[MAXG][2];
    {
      const float4* v0 = reinterpret_cast<const float4*>(vals + bo0);
#pragma unroll
      for (int gi = 0; gi < MAXG; ++gi) {
        const bool ok = b0ok && 8 * gi < bp0;
        wg[gi][0] = ok ? v0[2 * gi] : make_float4(0.f, 0.f, 0.f, 0.f);
        wg[gi][1] = ok ? v0[2 * gi + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    __syncthreads();
    auto dot8 = [](v2f acc, const float4 a, const float4 c, const float* p) __attribute__((always_inline)) {
      acc = __builtin_elementwise_fma(v2f{a.x, a.y}, v2f{p[0], p[1]}, acc);
      acc = __builtin_elementwise_fma(v2f{a.z, a.w}, v2f{p[2], p[3]}, acc);
      acc = __builtin_elementwise_fma(v2f{c.x, c.y}, v2f{p[4], p[5]}, acc);
      return __builtin_elementwise_fma(v2f{c.z, c.w}, v2f{p[6], p[7]}, acc);
    };
    if (b0ok) {
      const float* p0 = pw + (bs0 - kmin);
      v2f acc = v2f{0.f, 0.f};
#pragma unroll
      for (int gi = 0; gi < MAXG; ++gi)
        if (8 * gi < bp0) acc = dot8(acc, wg[gi][0], wg[gi][1], p0 + 8 * gi);
      const float4* v0 = reinterpret_cast<const float4*>(vals + bo0);
      for (int i0 = 8 * MAXG; i0 < bp0; i0 += 8) acc = dot8(acc, v0[i0 / 4], v0[i0 / 4 + 1], p0 + i0);
      out[layout == ACFE_LAYOUT_BTM ? ((size_t)b * n_frames + f) * n_mels + m0
                                    : ((size_t)b * n_mels + m0) * n_frames + f] = (acc.x + acc.y) * PSCALE;
    }
    for (int q = q0 + 64; q < (n_mels + 1) / 2; q += 64) {
      const int m = tid < 64 ? q : n_mels - 1 - q;
      if (tid >= 64 && m == q) continue;
      const int s0 = band[3 * m], pl = (band[3 * m + 1] + 7) & ~7, off = band[3 * m + 2];
      const float4* v0 = reinterpret_cast<const float4*>(vals + off);
      const float* p0 = pw + (s0 - kmin);
      v2f acc = v2f{0.f, 0.f};
      for (int i0 = 0; i0 < pl; i0 += 8) acc = dot8(acc, v0[i0 / 4], v0[i0 / 4 + 1], p0 + i0);
      out[layout == ACFE_LAYOUT_BTM ? ((size_t)b * n_frames + f) * n_mels + m : ((size_t)b * n_mels + m) * n_frames + f] =
          (acc.x + acc.y) * PSCALE;
    }
  }
}

// ---- k_mel_w5 (n_fft = 4096): ONE wave per frame.
// The 2048-point complex FFT of k_mel_w4 with each lane running two of its
// 128 threads (virtual threads j = lane + 64 h, h = 0 / 1: the same radix
// 16 / 16 / 8 Stockham passes, the same swizzled 16 KB frame buffer, the same
// per-instruction address patterns, so the same conflict-free LDS accesses),
// every pass ordered by the wave's own in-order LDS queue instead of the six
// workgroup barriers per frame: a workgroup is one wave walking fpw frames,
// each wave's frame buffer its own.  Pass 1 issues both halves' 32 sample
// loads before the first DFT; pass 2 reads both halves before it writes (the
// in-place Stockham step); pass 3 holds the four butterflies j, 256 - j of both
// halves, then forms the power spectrum from registers as k_mel_w4.  Band m
// and its mirror n_mels - 1 - m per lane (balanced lengths).  Arithmetic per
// value identical to k_mel_w4 (same functions, same order): bit-identical.
#ifndef MEL_W5_WAVES
#define MEL_W5_WAVES 3
#endif
template <int POW>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MEL_W5_WAVES)))
k_mel_w5(const float* __restrict__ raw, int64_t cs, int n, const float* __restrict__ stats, int pad_mode,
         int n_frames, int fpw, int hop, const float2* __restrict__ tw, const float2* __restrict__ rtw,
         const int* __restrict__ band, const float* __restrict__ vals, int n_mels, int kmin, int kmax,
         float* __restrict__ out, int layout) {
  constexpr int NC = 2048, L = 2 * NC, NB0 = NC / 16;
  extern __shared__ float2 wbuf_[];
  v2f* wbuf = reinterpret_cast<v2f*>(wbuf_);
  float* pw = reinterpret_cast<float*>(wbuf_);
  const int nk = kmax - kmin + 1;
  const int t0 = threadIdx.x;
  const int gx = gridDim.x, nwg = gx * gridDim.y, lin = blockIdx.x + gx * blockIdx.y;
  const int item = nwg % 8 == 0 ? (lin % 8) * (nwg / 8) + lin / 8 : lin;  // XCD-contiguous (k_mel_w4)
  const int b = item / gx;
  const float* xb = raw + (int64_t)b * cs;
  const bool do_norm = stats != nullptr;
  const float mn = do_norm ? stats[2 * b] : 0.f, rng = do_norm ? stats[2 * b + 1] : 1.f;
  const float rinv = __fdiv_rn(1.0f, rng);
  const int f0 = (item - b * gx) * fpw;
  v2f bw2[4], e0[2][3], rb0[2];
  {
    const int tb = (t0 & 15) * 8;  // (lane + 64) & 15 == lane & 15: shared by both halves
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float2 w = tw[(tb << q) & (NC - 1)];
      bw2[q] = v2f{w.x, w.y};
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = t0 + 64 * h;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const float2 w = tw[(j << q) & (NC - 1)];
        e0[h][q] = v2f{w.x, w.y};
      }
      rb0[h] = v2f{rtw[j].x, rtw[j].y};
    }
  }
  constexpr float PSCALE = POW == 2 ? 0.25f : 0.5f;
  typedef float f2a __attribute__((ext_vector_type(2), aligned(4)));
  for (int f = f0; f < f0 + fpw && f < n_frames; ++f) {
    // the base twiddles opaque per frame: their powers, the Hann terms and the
    // addresses are recomputed each frame instead of hoisted (k_mel_w4)
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(bw2[q]));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      asm volatile("" : "+v"(rb0[h]));
#pragma unroll
      for (int q = 0; q < 3; ++q) asm volatile("" : "+v"(e0[h][q]));
    }
    const int start = (pad_mode == ACFE_PAD_END) ? f * hop : f * hop - L / 2;
    const bool inb = start >= 0 && start + L <= n;
    // ---- pass 1 (radix 16, span 1) straight from memory, both halves' loads first
    {
      v2f xv[2][16];
      if (inb) {
        const float* xs = xb + start + 2 * t;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 16; ++r) xv[h][r] = *reinterpret_cast<const f2a*>(xs + 128 * h + 2 * r * NB0);
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int nn = 2 * (t + 64 * h + r * NB0);
            xv[h][r] = v2f{fetch(xb, n, start + nn, pad_mode, false, 0.f, 1.f),
                           fetch(xb, n, start + nn + 1, pad_mode, false, 0.f, 1.f)};
          }
      }
      // the previous frame's band reads of pw precede this frame's stores
      // (in-order LDS queue of the wave; compiler ordering only)
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = t + 64 * h;
        const float ce = e0[h][0].x, se = -e0[h][0].y;
        constexpr float c1 = 0.99999882345170190993f, s1 = 0.00153398018628476550f;
        const float co = ce * c1 - se * s1, so = se * c1 + ce * s1;
        const v2f cc = v2f{ce, co}, ss = v2f{se, so};
        v2f v[16];
        auto hann2 = [&](int r) __attribute__((always_inline)) {
          const float2 u = w16(r);
          return __builtin_elementwise_fma(ss, sp2(-u.y), __builtin_elementwise_fma(cc, sp2(-u.x), sp2(1.f)));
        };
        if (do_norm) {
#pragma clang fp contract(off)
          const v2f vmn = sp2(mn), vrng = sp2(rng), vri = sp2(rinv);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const v2f tt = xv[h][r] - vmn;
            const v2f q0v = tt * vri;
            const v2f e = __builtin_elementwise_fma(-q0v, vrng, tt);
            v2f q = __builtin_elementwise_fma(e, vri, q0v);
            q = q + sp2(0.000001f);
            q = q - sp2(0.5f);
            v[r] = q * hann2(r);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float2 u = w16(r);
            v[r] = xv[h][r] * __builtin_elementwise_fma(ss, sp2(-0.5f * u.y),
                                                        __builtin_elementwise_fma(cc, sp2(-0.5f * u.x), sp2(0.5f)));
          }
        }
        if (do_norm && !inb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int nn = 2 * (j + r * NB0);
            if (!in_sig(start + nn, n, pad_mode)) v[r].x = 0.f;
            if (!in_sig(start + nn + 1, n, pad_mode)) v[r].y = 0.f;
          }
        }
        pdft16(v);
        const unsigned ua = (unsigned)msw(16 * j) * 8u;
#pragma unroll
        for (int r = 0; r < 16; ++r) lds2v(wbuf, ua ^ (8u * r)) = v[r];
        __builtin_amdgcn_sched_barrier(0);  // one half at a time (registers)
      }
    }
    __builtin_amdgcn_wave_barrier();
    // ---- pass 2 (radix 16, span 16): every read of the pass before its writes
    {
      v2f v[2][16], w[16];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const unsigned ub = (unsigned)msw(t + 64 * h) * 8u;
#pragma unroll
        for (int r = 0; r < 16; ++r) v[h][r] = lds2v(wbuf, (ub ^ (64u * (r & 1))) + 1024u * r);
      }
      ptwiddle_pows<16>(bw2, w);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int r = 1; r < 16; ++r) v[h][r] = pk_cmul(v[h][r], w[r]);
        pdft16(v[h]);
        const int j = t + 64 * h;
        const unsigned uc = (unsigned)(256 * (j >> 4) + (j & 15)) * 8u;
#pragma unroll
        for (int r = 0; r < 16; ++r) lds2v(wbuf, (uc ^ (8u * r)) + 128u * r) = v[h][r];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // ---- pass 3 (radix 8, span 256): butterflies j, 256 - j of both halves
    v2f z[2][2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = t + 64 * h;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const unsigned ad = (unsigned)msw(p ? (j ? 256 - j : 128) : j) * 8u;
#pragma unroll
        for (int r = 0; r < 8; ++r) z[h][p][r] = lds2v(wbuf, ad + 2048u * r);
      }
    }
    __builtin_amdgcn_wave_barrier();  // all pass-3 reads before the power writes (pw aliases the buffer)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = t + 64 * h;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        v2f bw[4], w[8];
#pragma unroll
        for (int q = 0; q < 3; ++q) bw[q] = p == 0 ? e0[h][q] : (j ? w16k(pk_conj(e0[h][q]), 2 << q) : w16v(1 << q));
        ptwiddle_pows<8>(bw, w);
#pragma unroll
        for (int r = 1; r < 8; ++r) z[h][p][r] = pk_cmul(z[h][p][r], w[r]);
        pdft8(z[h][p]);
      }
      const v2f rb1 = j ? w16k(pk_conj(rb0[h]), 1) : v2f{0.98078528040323044913f, -0.19509032201612826785f};
      int rhi0 = kmax >> 8, rhi1 = kmax >= 128 ? (kmax - 128) >> 8 : -1;
      int rlo0 = kmin > 127 ? (kmin - 127 + 255) >> 8 : 0, rlo1 = kmin > 255 ? (kmin - 255 + 255) >> 8 : 0;
      asm volatile("" : "+s"(rhi0), "+s"(rhi1), "+s"(rlo0), "+s"(rlo1));
      const bool l0 = j == 0;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int kb = (p ? (l0 ? 128 : 256 - j) : j) - kmin;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          if (4 * hh + 3 < (p ? rlo1 : rlo0) || 4 * hh > (p ? rhi1 : rhi0)) continue;
          v2f ea[4], da[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = 4 * hh + u;
            const v2f zm = l0 ? (p == 0 ? z[h][0][(8 - r) & 7] : z[h][1][7 - r]) : z[h][p ^ 1][7 - r];
            ea[u] = pk_addc(z[h][p][r], zm);
            da[u] = pk_subc(z[h][p][r], zm);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) da[u] = pk_cmul(w16k(p ? rb1 : rb0[h], 4 * hh + u), da[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u) ea[u] = pk_addmi(ea[u], da[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = 4 * hh + u;
            float pv = ea[u].x * ea[u].x + ea[u].y * ea[u].y;
            if constexpr (POW != 2) pv = sqrtf(pv);
            const int i = kb + 256 * r;
            pw[(unsigned)i < (unsigned)nk ? i : 2 * NC - 1] = pv;
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t == 0 && kmax == NC) {  // Nyquist bin: Z[0] with itself, W_4096^2048 = -1
      float pv = rbin_power4_pk(z[0][0][0], z[0][0][0], v2f{-1.f, 0.f});
      if constexpr (POW != 2) pv = sqrtf(pv);
      pw[NC - kmin] = pv;
    }
    if (t < 8) pw[nk + t] = 0.f;
    __builtin_amdgcn_wave_barrier();
    // ---- banded mel: bands q and n_mels - 1 - q per lane
    auto dot8 = [](v2f acc, const float4 a, const float4 c, const float* p) __attribute__((always_inline)) {
      acc = __builtin_elementwise_fma(v2f{a.x, a.y}, v2f{p[0], p[1]}, acc);
      acc = __builtin_elementwise_fma(v2f{a.z, a.w}, v2f{p[2], p[3]}, acc);
      acc = __builtin_elementwise_fma(v2f{c.x, c.y}, v2f{p[4], p[5]}, acc);
      return __builtin_elementwise_fma(v2f{c.z, c.w}, v2f{p[6], p[7]}, acc);
    };
    for (int q = t; q < (n_mels + 1) / 2; q += 64) {
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int m = side ? n_mels - 1 - q : q;
        if (side && m == q) continue;
        const int s0 = band[3 * m], pl = (band[3 * m + 1] + 7) & ~7, off = band[3 * m + 2];
        const float4* v0 = reinterpret_cast<const float4*>(vals + off);
        const float* p0 = pw + (s0 - kmin);
        v2f acc = v2f{0.f, 0.f};
        for (int i0 = 0; i0 < pl; i0 += 8) acc = dot8(acc, v0[i0 / 4], v0[i0 / 4 + 1], p0 + i0);
        out[layout == ACFE_LAYOUT_BTM ? ((size_t)b * n_frames + f) * n_mels + m
                                      : ((size_t)b * n_mels + m) * n_frames + f] = (acc.x + acc.y) * PSCALE;
      }
    }
  }
}

// n_fft = 4096 kernel choice: 0 = k_mel_w4 (two waves per frame), f > 0 =
// k_mel_w5 with f frames per wave; initial value from ACFE_MEL_W5
static std::atomic<int> g_mel_w5{[] {
  const char* e = getenv("ACFE_MEL_W5");
  return e ? atoi(e) : 0;
}()};
ACFE_API int acfe_mel_w5_frames(int fpw) {
  if (fpw < 0 || fpw > 64) return ACFE_E_INVAL;
  const int prev = g_mel_w5.load();
  g_mel_w5.store(fpw);
  return prev;
}

ACFE_API int acfe_mel_fwd(acfe_plan_t p, const float* raw, int64_t cs, int batch, int n,
                          const float* stats, int pad_mode, int power, float* out, int layout,
                          void* stream) {
  if (batch == 0 && p && n > 0) return ACFE_OK;
  if (!p || !raw || !out || batch < 0 || n <= 0 || batch > 65535 || (power != 1 && power != 2) ||
      pad_mode < 0 || pad_mode > 2 || (layout != 0 && layout != 1))
    return ACFE_E_INVAL;
  if (pad_mode == ACFE_PAD_CENTER_REFLECT && n <= p->n_fft / 2) return ACFE_E_INVAL;
  if (batch == 0) return ACFE_OK;
  const int T = acfe_plan_num_frames(p, n, pad_mode);
  if (p->n_fft == 4096) {
    const int w5 = g_mel_w5.load(std::memory_order_relaxed);
    if (w5 > 0) {  // one wave per frame, w5 frames per wave
      hipLaunchKernelGGL((power == 2 ? k_mel_w5<2> : k_mel_w5<1>), dim3(cdiv(T, w5), batch), dim3(64),
                         sizeof(float2) * 2048, strm(stream), raw, cs, n, stats, pad_mode, T, w5, p->hop, p->d_tw,
                         p->d_rtw, p->d_band, p->d_vals, p->n_mels, p->kmin, p->kmax, out, layout);
      return launch_rc("acfe_mel_fwd");
    }
    constexpr int fpw = 4;  // frames per workgroup (2: 1.51 ms, 8: equal, r01n/r02y; r03: 2 / 8 / 16 +3 / 0 / +2 %)
    hipLaunchKernelGGL((power == 2 ? k_mel_w4<2> : k_mel_w4<1>), dim3(cdiv(T, fpw), batch), dim3(128), sizeof(float2) * 2048, strm(stream), raw, cs, n,
                       stats, pad_mode, power, T, fpw, p->hop, p->d_tw, p->d_rtw, p->d_band, p->d_vals, p->n_mels,
                       p->kmin, p->kmax, out, layout);
    return launch_rc("acfe_mel_fwd");
  }
  const int fpb = 4;
  dim3 grid(cdiv(T, fpb), batch);
#define LAUNCH_MEL(NC)                                                                          \
  hipLaunchKernelGGL(k_mel<NC>, grid, dim3(256), 0, strm(stream), raw, cs, n, stats, pad_mode,     \
                     power, T, fpb, p->hop, p->d_tw, p->d_rtw, p->d_win, p->d_band, p->d_vals,  \
                     p->n_mels, p->kmin, p->kmax, out, layout)
  switch (p->n_fft) {
    case 4096: LAUNCH_MEL(2048); break;
    case 2048: LAUNCH_MEL(1024); break;
    case 1024: LAUNCH_MEL(512); break;
    case 512: LAUNCH_MEL(256); break;
    case 256: LAUNCH_MEL(128); break;
    default: return ACFE_E_INVAL;
  }
#undef LAUNCH_MEL
  return launch_rc("acfe_mel_fwd");
}

// ------------------------------------------------------------ stored spectrogram -> mel
// The load_raw=False path (tfdataset.py:1065-1102): a record holds the
// magnitude |STFT| [F = 1 + n_fft/2][T] written by audiodataset.load_data
// (:1302-1303); the model input is tensordot(MEL_WEIGHTS, S^power) [M][T]
// (power 1: the reference keeps the magnitude for PCEN, :1085-1089).  A
// 256-thread workgroup owns 64 frames of one clip: lanes = frames (S rows are
// frame-contiguous, so every tap is one coalesced 256-B load), the 4 waves
// take interleaved mel bands (m = wave + 4j) of the plan's banded filterbank;
// overlapping bands re-read a row from L1/L2, never from HBM.  [B][T][M]
// output goes through an LDS tile so its rows are written contiguously.
__global__ void __launch_bounds__(256) k_mel_spec(const float* __restrict__ spec, int64_t cs, int F, int T,
                                                  int power, const int* __restrict__ band,
                                                  const float* __restrict__ vals, int M, float* __restrict__ out,
                                                  int layout) {
  extern __shared__ float tile[];  // [64][M + 1] for layout btm
  const int b = blockIdx.y, t0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int t = t0 + lane;
  const bool ok = t < T;
  const float* S = spec + (int64_t)b * cs + (ok ? t : 0);
  for (int m = w; m < M; m += 4) {
    const int st = band[3 * m], len = band[3 * m + 1], off = band[3 * m + 2];
    float acc = 0.f;
    for (int k = 0; k < len; ++k) {
      float v = S[(int64_t)(st + k) * T];
      if (power == 2) v *= v;
      acc = fmaf(vals[off + k], v, acc);
    }
    if (layout == 1) {
      if (ok) out[((int64_t)b * M + m) * T + t] = acc;
    } else {
      tile[lane * (M + 1) + m] = acc;
    }
  }
  if (layout == 0) {
    __syncthreads();
    const int nt = min(64, T - t0);
    for (int i = threadIdx.x; i < nt * M; i += 256) {
      const int r = i / M, m = i - r * M;
      out[((int64_t)b * T + t0 + r) * M + m] = tile[r * (M + 1) + m];
    }
  }
}

ACFE_API int acfe_mel_from_spec(acfe_plan_t p, const float* spec, int64_t cs, int batch, int n_bins, int T,
                                int power, float* out, int layout, void* stream) {
  if (batch == 0 && p && T > 0) return ACFE_OK;
  if (!p || !spec || !out || batch < 0 || batch > 65535 || T <= 0 || n_bins != p->n_bins ||
      (power != 1 && power != 2) || (layout != 0 && layout != 1) || cs < (int64_t)n_bins * T)
    return ACFE_E_INVAL;
  const size_t shm = layout == 0 ? sizeof(float) * 64 * (p->n_mels + 1) : 0;
  if (shm > 65536) return ACFE_E_INVAL;
  hipLaunchKernelGGL(k_mel_spec, dim3(cdiv(T, 64), batch), dim3(256), shm, strm(stream), spec, cs, n_bins, T,
                     power, p->d_band, p->d_vals, p->n_mels, out, layout);
  return launch_rc("acfe_mel_from_spec");
}

// ------------------------------------------------------------ PCEN
// Thread per (b, m) row; the EMA recurrence runs sequentially over T (the
// reference's tf.scan), reading mel [B][T][M] coalesced across threads.
// Outputs go through an LDS tile so the [B][M][T] writes are row-contiguous.
constexpr int PCEN_TCH = 32;

// 64 (b, m) rows per 256-thread workgroup: one wave runs the sequential EMA of
// a 32-step chunk (a few dependent VALU ops per step, from LDS), then all four
// waves evaluate the compression terms (the pow / log bulk) of 8 steps each,
// so 4 waves per SIMD instead of one hide the transcendental latency.
constexpr int PCEN_RB = 64;
ACFE_API int acfe_pcen_partials(int batch, int n_mels) { return cdiv((int64_t)batch * n_mels, PCEN_RB); }

// a^b for a >= 0 from the hardware base-2 log / exp (v_log_f32, v_exp_f32,
// ~1 ulp each): OCML's correctly-rounded powf is ~280 VALU instructions and
// made the PCEN kernels compute-bound (33.6 M elements x 2 powf per batch of
// 512 clips).  a = 0 gives 0 for b > 0; a < 0 gives NaN, as powf does for a
// non-integer b.  The forward and the backward's recomputation use the same
// function, so y (and the min / max tie test on it) stay bit-identical.
__device__ __forceinline__ float pow_hw(float a, float b) {
  return __builtin_amdgcn_exp2f(__fmul_rn(b, __builtin_amdgcn_logf(a)));
}
__device__ __forceinline__ float ln_hw(float a) { return __fmul_rn(__builtin_amdgcn_logf(a), 0.693147180559945309f); }

struct PcenP {
  float g, b, r, w, inv_r, bpow;
};
__device__ __forceinline__ PcenP pcen_params(const float* __restrict__ prm) {
  PcenP p;
  p.g = fminf(prm[0], 1.0f);
  p.b = prm[1];
  p.r = fmaxf(prm[2], 1.0f);
  p.w = fminf(fmaxf(prm[3], 0.0f), 1.0f);
  p.inv_r = 1.0f / p.r;
  p.bpow = pow_hw(p.b, p.inv_r);  // so that x = 0 gives y = 0 exactly
  return p;
}

// tfpcen.py:37: w * x + (1.0 - w) * a, float32, no contraction (so forward and
// backward recompute identical values and the min/max tie test is exact).
__device__ __forceinline__ float ema_step(float w, float x, float a) {
  return __fadd_rn(__fmul_rn(w, x), __fmul_rn(__fsub_rn(1.0f, w), a));
}

__global__ void __launch_bounds__(256) k_pcen_fwd(const float* __restrict__ mel, int B, int T, int M,
                                                  const float* __restrict__ prm, float eps,
                                                  float* __restrict__ y, float* __restrict__ part) {
  __shared__ float xs[PCEN_TCH][PCEN_RB + 1];    // x chunk [t][row]
  __shared__ float as[PCEN_TCH][PCEN_RB + 1];    // EMA a_t
  __shared__ float tile[PCEN_RB][PCEN_TCH + 1];  // output chunk [row][t]
  const PcenP P = pcen_params(prm);
  const int64_t rows = (int64_t)B * M;
  const int64_t row0 = (int64_t)blockIdx.x * PCEN_RB;
  const int r = threadIdx.x & (PCEN_RB - 1), sub = threadIdx.x / PCEN_RB;
  const int64_t gr = row0 + r;
  const bool valid = gr < rows;
  const int bb = valid ? (int)(gr / M) : 0, m = valid ? (int)(gr % M) : 0;
  const float* xr = mel + (int64_t)bb * T * M + m;
  float a = (valid && sub == 0) ? xr[0] : 0.f;
  float lmin = INFINITY, lmax = -INFINITY;
  const int nrow = (int)((rows - row0) < PCEN_RB ? (rows - row0) : PCEN_RB);
  constexpr int PER = PCEN_TCH / 4;
  // the next chunk's x values are loaded into registers while this chunk is
  // scanned, transformed and stored (the chunk loop was load-latency bound)
  float px[PER];
  auto ldx = [&](int t0) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int tt = sub * PER + k;
      px[k] = (valid && t0 + tt < T) ? xr[(int64_t)(t0 + tt) * M] : 0.f;
    }
  };
  ldx(0);
  for (int t0 = 0; t0 < T; t0 += PCEN_TCH) {
    const int tn = (T - t0) < PCEN_TCH ? (T - t0) : PCEN_TCH;
    if (valid) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int tt = sub * PER + k;
        if (tt < tn) xs[tt][r] = px[k];
      }
    }
    __syncthreads();
    if (t0 + PCEN_TCH < T) ldx(t0 + PCEN_TCH);
    if (valid && sub == 0) {
      float xv[PCEN_TCH];
#pragma unroll
      for (int tt = 0; tt < PCEN_TCH; ++tt) xv[tt] = xs[tt][r];
#pragma unroll
      for (int tt = 0; tt < PCEN_TCH; ++tt)
        if (tt < tn) {
          a = ema_step(P.w, xv[tt], a);
          as[tt][r] = a;
        }
    }
    __syncthreads();
    if (valid) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int tt = sub * PER + k;
        if (tt < tn) {
          const float x = xs[tt][r], at = as[tt][r];
          const float v =
              __fsub_rn(pow_hw(__fadd_rn(__fdiv_rn(x, pow_hw(__fadd_rn(eps, at), P.g)), P.b), P.inv_r), P.bpow);
          tile[r][tt] = v;
          lmin = fminf(lmin, v);
          lmax = fmaxf(lmax, v);
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nrow * PCEN_TCH; i += 256) {
      const int r2 = i / PCEN_TCH, tt = i % PCEN_TCH;
      if (tt < tn) y[(row0 + r2) * T + t0 + tt] = tile[r2][tt];
    }
    // the next chunk writes xs, then (after a barrier) as, then tile: no barrier needed here
  }
  __shared__ float smn[4], smx[4];
  lmin = wave_min(lmin);
  lmax = wave_max(lmax);
  if ((threadIdx.x & 63) == 0) { smn[threadIdx.x >> 6] = lmin; smx[threadIdx.x >> 6] = lmax; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3]));
    part[2 * blockIdx.x + 1] = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
  }
}

ACFE_API int acfe_pcen_fwd(const float* mel, int batch, int t, int m, const float* params, float eps,
                           float* y, float* part, void* stream) {
  if (!mel || !params || !y || !part || batch <= 0 || t <= 0 || m <= 0) return ACFE_E_INVAL;
  hipLaunchKernelGGL(k_pcen_fwd, dim3(acfe_pcen_partials(batch, m)), dim3(256), 0, strm(stream), mel,
                     batch, t, m, params, eps, y, part);
  return launch_rc("acfe_pcen_fwd");
}

__device__ __forceinline__ void reduce_minmax_partials(const float* __restrict__ part, int np,
                                                       const float* __restrict__ scope, float& mn,
                                                       float& mx) {
  __shared__ float smn[4], smx[4];
  if (scope) {
    mn = scope[0];
    mx = scope[1];
    return;
  }
  float a = INFINITY, c = -INFINITY;
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    a = fminf(a, part[2 * i]);
    c = fmaxf(c, part[2 * i + 1]);
  }
  a = wave_min(a);
  c = wave_max(c);
  if ((threadIdx.x & 63) == 0) { smn[threadIdx.x >> 6] = a; smx[threadIdx.x >> 6] = c; }
  __syncthreads();
  mn = fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3]));
  mx = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
}

__global__ void __launch_bounds__(256) k_pcen_norm(const float* __restrict__ y, int64_t count,
                                                   const float* __restrict__ part, int np,
                                                   const float* __restrict__ scope, void* out,
                                                   int dtype, float* __restrict__ stats) {
  float mn, mx;
  reduce_minmax_partials(part, np, scope, mn, mx);
  const float d = mx - mn;
  float cmin = 0.f, cmax = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256) {
    const float v = y[i];
    cmin += (v == mn) ? 1.f : 0.f;
    cmax += (v == mx) ? 1.f : 0.f;
    const float o = 2.0f * ((v - mn) / d) - 1.0f;  // tfpcen.py:110
    if (dtype == ACFE_DTYPE_BF16) reinterpret_cast<uint16_t*>(out)[i] = f2bf(o);
    else reinterpret_cast<float*>(out)[i] = o;
  }
  cmin = wave_sum(cmin);
  cmax = wave_sum(cmax);
  if ((threadIdx.x & 63) == 0) {
    if (cmin != 0.f) atomicAdd(&stats[2], cmin);
    if (cmax != 0.f) atomicAdd(&stats[3], cmax);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    stats[0] = mn;
    stats[1] = mx;
  }
}

ACFE_API int acfe_pcen_normalize(const float* y, int64_t count, const float* part, int np,
                                 const float* scope, void* out, int dtype, float* stats,
                                 void* stream) {
  if (!y || !out || !stats || count <= 0 || (!part && !scope) || (dtype != 0 && dtype != 1))
    return ACFE_E_INVAL;
  int rc = hip_rc(hipMemsetAsync(stats, 0, 4 * sizeof(float), strm(stream)), "acfe_pcen_normalize");
  if (rc) return rc;
  int grid = cdiv(count, 256 * 8);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(k_pcen_norm, dim3(grid), dim3(256), 0, strm(stream), y, count, part, np, scope,
                     out, dtype, stats);
  return launch_rc("acfe_pcen_normalize");
}

// Backward.  One pass: per row, recompute the EMA a_t, its forward-mode
// derivative da_t/dw, y_t and the partials of y_t w.r.t. (g, b, r, w), and
// accumulate (d = dL/dout):
//   G_th  = sum d * dy/dth,  Smax_th = sum_{y == mx} dy/dth,
//   Smin_th = sum_{y == mn} dy/dth,  S0 = sum d,  Sy = sum d * y.
// The finaliser turns these into dL/dth through normalize_minmax (with the
// TF reduce_max/min tie rule: gradient shared equally among tied extrema).
constexpr int PCEN_NACC = 14;

__global__ void __launch_bounds__(256) k_pcen_bwd(const float* __restrict__ mel, int B, int T, int M,
                                                  const float* __restrict__ prm, float eps,
                                                  const float* __restrict__ st,
                                                  const void* __restrict__ dout, int ddt,
                                                  double* __restrict__ part) {
  __shared__ float xs[PCEN_TCH][PCEN_RB + 1];
  __shared__ float as[PCEN_TCH][PCEN_RB + 1];    // a_t
  __shared__ float das[PCEN_TCH][PCEN_RB + 1];   // d a_t / d w
  __shared__ float tile[PCEN_RB][PCEN_TCH + 1];  // dL/dout chunk [row][t]
  __shared__ double red[4][PCEN_NACC];
  const PcenP P = pcen_params(prm);
  const float mn = st[0], mx = st[1];
  const int64_t rows = (int64_t)B * M;
  const int64_t row0 = (int64_t)blockIdx.x * PCEN_RB;
  const int r = threadIdx.x & (PCEN_RB - 1), sub = threadIdx.x / PCEN_RB;
  const int64_t gr = row0 + r;
  const bool valid = gr < rows;
  const int bb = valid ? (int)(gr / M) : 0, m = valid ? (int)(gr % M) : 0;
  const float* xr = mel + (int64_t)bb * T * M + m;
  const int nrow = (int)((rows - row0) < PCEN_RB ? (rows - row0) : PCEN_RB);
  constexpr int PER = PCEN_TCH / 4;
  float acc[PCEN_NACC];
#pragma unroll
  for (int i = 0; i < PCEN_NACC; ++i) acc[i] = 0.f;
  float a = (valid && sub == 0) ? xr[0] : 0.f, da = 0.f;
  const float lnb = logf(P.b);
  // the next chunk's x values prefetched as in k_pcen_fwd (prefetching the
  // dL/dout chunk too measured slower: 180 -> 219 us, r04g11)
  float px[PER];
  auto ldx = [&](int t0) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int tt = sub * PER + k;
      px[k] = (valid && t0 + tt < T) ? xr[(int64_t)(t0 + tt) * M] : 0.f;
    }
  };
  ldx(0);
  for (int t0 = 0; t0 < T; t0 += PCEN_TCH) {
    const int tn = (T - t0) < PCEN_TCH ? (T - t0) : PCEN_TCH;
    for (int i = threadIdx.x; i < nrow * PCEN_TCH; i += 256) {
      const int r2 = i / PCEN_TCH, tt = i % PCEN_TCH;
      if (tt < tn) {
        const int64_t o = (row0 + r2) * T + t0 + tt;
        tile[r2][tt] = ddt == ACFE_DTYPE_BF16 ? bf2f(reinterpret_cast<const uint16_t*>(dout)[o])
                                              : reinterpret_cast<const float*>(dout)[o];
      }
    }
    if (valid) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int tt = sub * PER + k;
        if (tt < tn) xs[tt][r] = px[k];
      }
    }
    __syncthreads();
    if (t0 + PCEN_TCH < T) ldx(t0 + PCEN_TCH);
    if (valid && sub == 0) {
      float xv[PCEN_TCH];
#pragma unroll
      for (int tt = 0; tt < PCEN_TCH; ++tt) xv[tt] = xs[tt][r];
#pragma unroll
      for (int tt = 0; tt < PCEN_TCH; ++tt)
        if (tt < tn) {
          const float a_prev = a;
          a = ema_step(P.w, xv[tt], a);                // bit-identical to the forward
          da = (xv[tt] - a_prev) + (1.0f - P.w) * da;  // d a_t / d w
          as[tt][r] = a;
          das[tt][r] = da;
        }
    }
    __syncthreads();
    if (valid) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int tt = sub * PER + k;
        if (tt >= tn) continue;
        const float x = xs[tt][r], at = as[tt][r], dat = das[tt][r];
        const float s = __fadd_rn(eps, at);
        const float sg = pow_hw(s, P.g);
        const float q = __fdiv_rn(x, sg);
        const float u = __fadd_rn(q, P.b);
        const float ur = pow_hw(u, P.inv_r);
        const float y = __fsub_rn(ur, P.bpow);
        const float dydu = P.inv_r * ur * __builtin_amdgcn_rcpf(u);  // (gradient terms: v_rcp_f32, ~1 ulp)
        const float d_g = dydu * (-q * ln_hw(s));
        const float d_b = dydu - P.inv_r * P.bpow / P.b;
        const float d_r = -(P.inv_r * P.inv_r) * (ur * ln_hw(u) - P.bpow * lnb);
        const float d_w = dydu * (-P.g * q * __builtin_amdgcn_rcpf(s)) * dat;
        const float d = tile[r][tt];
        acc[0] += d * d_g; acc[1] += d * d_b; acc[2] += d * d_r; acc[3] += d * d_w;
        if (y == mx) { acc[4] += d_g; acc[5] += d_b; acc[6] += d_r; acc[7] += d_w; }
        if (y == mn) { acc[8] += d_g; acc[9] += d_b; acc[10] += d_r; acc[11] += d_w; }
        acc[12] += d;
        acc[13] += d * y;
      }
    }
    __syncthreads();  // tile / xs / as are rewritten by the next chunk
  }
#pragma unroll
  for (int i = 0; i < PCEN_NACC; ++i) {
    double v = wave_sumd((double)acc[i]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < PCEN_NACC)
    part[(int64_t)blockIdx.x * 16 + threadIdx.x] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

__global__ void __launch_bounds__(256) k_pcen_bwd_fin(const double* __restrict__ part, int np,
                                                      const float* __restrict__ prm,
                                                      const float* __restrict__ st,
                                                      float* __restrict__ dparams) {
  // 16 lanes per accumulator, each summing every 16th partial; fixed-order combine
  __shared__ double ps[PCEN_NACC][17];
  __shared__ double tot[PCEN_NACC];
  const int acc_i = threadIdx.x >> 4, l = threadIdx.x & 15;
  if (acc_i < PCEN_NACC) {
    double s = 0.0;
    for (int i = l; i < np; i += 16) s += part[(int64_t)i * 16 + acc_i];
    ps[acc_i][l] = s;
  }
  __syncthreads();
  if (threadIdx.x < PCEN_NACC) {
    double s = 0.0;
    for (int j = 0; j < 16; ++j) s += ps[threadIdx.x][j];
    tot[threadIdx.x] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double mn = st[0], mx = st[1], nmin = st[2], nmax = st[3];
    const double D = mx - mn;
    const double S0 = tot[12], Sy = tot[13];
    const double S1 = (2.0 / D) * (Sy - mn * S0);  // sum d * (out + 1)
    const double dmx = -S1 / D;
    const double dmn = (S1 - 2.0 * S0) / D;
    double g[4];
    for (int k = 0; k < 4; ++k)
      g[k] = (2.0 / D) * tot[k] + (nmax > 0 ? dmx / nmax * tot[4 + k] : 0.0) +
             (nmin > 0 ? dmn / nmin * tot[8 + k] : 0.0);
    // TF gradient masks: minimum(gain,1) -> gain <= 1; maximum(root,1) -> root >= 1;
    // clip_by_value(smooth,0,1) -> 0 <= smooth <= 1.
    dparams[0] = prm[0] <= 1.0f ? (float)g[0] : 0.f;
    dparams[1] = (float)g[1];
    dparams[2] = prm[2] >= 1.0f ? (float)g[2] : 0.f;
    dparams[3] = (prm[3] >= 0.0f && prm[3] <= 1.0f) ? (float)g[3] : 0.f;
  }
}

ACFE_API int acfe_pcen_bwd(const float* mel, int batch, int t, int m, const float* params, float eps,
                           const float* stats, const void* dout, int ddt, float* ws, float* dparams,
                           void* stream) {
  if (!mel || !params || !stats || !dout || !ws || !dparams || batch <= 0 || t <= 0 || m <= 0 ||
      (ddt != 0 && ddt != 1))
    return ACFE_E_INVAL;
  const int np = acfe_pcen_partials(batch, m);
  double* part = reinterpret_cast<double*>(ws);
  hipLaunchKernelGGL(k_pcen_bwd, dim3(np), dim3(256), 0, strm(stream), mel, batch, t, m, params, eps,
                     stats, dout, ddt, part);
  int rc = launch_rc("acfe_pcen_bwd");
  if (rc) return rc;
  hipLaunchKernelGGL(k_pcen_bwd_fin, dim3(1), dim3(256), 0, strm(stream), part, np, params, stats,
                     dparams);
  return launch_rc("acfe_pcen_bwd_fin");
}
