// Fused Conv2D(1x1, 16 -> K, bias) -> BatchNormalization (+ReLU) whose conv
// output is never stored.
//
// Reference: resnet/wr_resnet_bird.py:121-131 (basic_block, stride > 1):
//   BN -> ReLU -> Conv2D(height, 1x1) "res{stage}b0_branch2a0" -> BN -> ReLU.
// At stage 1 that conv maps the 16-channel block input x to 128 channels at
// 128x256 per clip: its output A = W x + b (4.3 GB per 512-clip batch in bf16)
// is the largest tensor of the model.  The unfused chain writes A, reads it
// for the BN, writes B = ReLU(BN(A)), and in the backward reads A twice more
// and writes / reads its gradient dA twice.  Here A is never stored, and every
// per-pixel pass is a stream over x (32 B / pixel) plus at most one K-channel
// tensor, because everything that sums over pixels is linear in small
// matrices of x:
//
//   forward statistics   S = sum x x^T (16x16), s = sum x  (MFMA Gram, reads x)
//                        sum A   = W s + M b,  sum A^2 = diag(W S W^T) + 2 b (W s) + M b^2
//   forward apply        B = ReLU(scale * (W x) + shift')      (the only forward store)
//   backward sums        g = dB * [scale * (W x) + shift' > 0];  G = g^T x (K x 16), sum g
//                        (MFMA over 32-pixel chunks, reads dB and x)
//   backward finalize    sum g*A = rowsum(W o G) + b sum g -> dgamma, dbeta and the
//                        BN input-gradient coefficients dA = ca g + cb A + cc;
//                        dW = ca o G + cb (W S + b s^T) + cc s^T,  db = ca sum g + cb sum A + M cc
//   backward dx          dx = (W^T diag(ca)) g + (W^T diag(cb) W) x + W^T (cb b + cc)
//                        ca = scale is known before the sums, so the first term
//                        P = (W^T diag(scale)) g (fp32, 64 B / pixel) is formed by
//                        the backward-sums pass, which already holds g; the dx pass
//                        then reads P and x (128 B / pixel) instead of dB and x
//                        (288 B / pixel)
//
// A is the fp32 MFMA result of the bf16 weights and inputs (the unfused conv
// rounds it to bf16 before the BN; the statistics and the ReLU mask here use
// the unrounded value, a difference below bf16 resolution).  BN semantics are
// Keras's (batch statistics, eps, momentum) through acfe_bn_finalize.
//
// Layouts: x [M][16] bf16 (NHWC, M = N*H*W pixels), w fp32 [K][16] (KRSC with
// R = S = 1), B / dB [M][K] bf16, dx [M][16] bf16.  K in {64, 128}.
//
// MFMA v_mfma_f32_16x16x32_bf16 in two orientations of the same registers:
//   mfma(wa, xb): lane (l16 = pixel, q = lane>>4) holds channels kb*16+q*4+r of one pixel
//   mfma(xb, wa): lane (l16 = channel kb*16+l16) holds pixels q*4+r of one channel
// (xb = 16 B of a pixel's input channels, wa = 16 B of an output channel's weights).
#include "common.h"

using namespace acfe;

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf4* lds_bf4p;

constexpr int CIN = 16;        // input channels of the fused conv
constexpr int UNR = 2;         // 16-pixel blocks per wave step (32 pixels: one MFMA k-chunk over pixels)
constexpr int NGRAM = 17 * 16; // S[16][16] then s[16]
constexpr int LDX = 48;        // x tile row stride (elements)

// zeros for the loads of pixels past M and of the padded input-channel slots
__device__ __attribute__((aligned(64))) uint4 c1_zero[4];

__device__ __forceinline__ f4 mfma16(const uint4& a, const uint4& b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b), c, 0, 0,
                                                 0);
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}
__device__ __forceinline__ float rbf(float v) { return bf2f(f2bf(v)); }  // bf16-rounded weight

// lane's 16 B of output channel (kb*16 + l16)'s weights: k-slots q*8..q*8+7 =
// input channels (q >= 2: zero padding up to the 32-deep MFMA)
template <int NKB>
__device__ __forceinline__ void load_wa(const float* __restrict__ w, int l16, int q, uint4 (&wa)[NKB]) {
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    uint4 v = {0u, 0u, 0u, 0u};
    if (q < 2) {
      const float* p = w + (kb * 16 + l16) * CIN + q * 8;
      v.x = pack2(p[0], p[1]);
      v.y = pack2(p[2], p[3]);
      v.z = pack2(p[4], p[5]);
      v.w = pack2(p[6], p[7]);
    }
    wa[kb] = v;
  }
}

// Optional BatchNormalization (+ReLU) prologue on x (the block's bn2a0 ->
// ReLU in front of the 1x1 conv, resnet/wr_resnet_bird.py:121-127): every
// pass reads the BN input and forms x' = (ReLU)(x * scale + shift) of its
// lane's 8 channels (acfe_bn_apply's arithmetic), so x' is never stored.
struct XPro {
  float sc[8], sh[8];
  bool on;
  bool relu;
};
__device__ __forceinline__ XPro make_xpro(const float* __restrict__ xsc, const float* __restrict__ xsh, int xrelu,
                                          int q) {
  XPro p;
  p.on = xsc != nullptr;
  p.relu = xrelu != 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    p.sc[j] = p.on && q < 2 ? xsc[q * 8 + j] : 0.f;
    p.sh[j] = p.on && q < 2 ? xsh[q * 8 + j] : 0.f;
  }
  return p;
}

__device__ __forceinline__ uint4 load_x(const uint16_t* __restrict__ X, long long px, long long M, int q,
                                        const XPro& pro) {
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(c1_zero);
  const bool in = px < M && q < 2;
  uint4 v = *reinterpret_cast<const uint4*>(in ? X + px * CIN + q * 8 : zp);
  if (pro.on) {
    unsigned d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float lo = __builtin_fmaf(__uint_as_float(d[i] << 16), pro.sc[2 * i], pro.sh[2 * i]);
      float hi = __builtin_fmaf(__uint_as_float(d[i] & 0xffff0000u), pro.sc[2 * i + 1], pro.sh[2 * i + 1]);
      if (pro.relu) {
        lo = fmaxf(lo, 0.f);
        hi = fmaxf(hi, 0.f);
      }
      d[i] = in ? pack2(lo, hi) : 0u;
    }
    v = uint4{d[0], d[1], d[2], d[3]};
  }
  return v;
}

__device__ __forceinline__ bf8 tr8(const uint16_t* t, int ld, int col, int lane) {
  // MFMA operand from a pixel-major LDS tile: row (channel) = col + (lane & 15),
  // k-slot (g = lane>>4, j) <-> pixel j<4: 4g+j, else 16+4g+(j-4)
  const int grp = lane >> 4, qq = (lane & 15) >> 2, p = lane & 3;
  const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf4p)(reinterpret_cast<const __bf16*>(t + (4 * grp + qq) * ld + col + 4 * p)));
  const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf4p)(reinterpret_cast<const __bf16*>(t + (16 + 4 * grp + qq) * ld + col + 4 * p)));
  return bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// constant x-tile columns 16..31 of a wave's 32-row tile: ones at 16, zeros after
__device__ __forceinline__ void x_tile_consts(uint16_t* tX, int l16, int q) {
  if (q >= 2) {
    const uint4 cst = q == 2 ? uint4{0x3F80u, 0u, 0u, 0u} : uint4{0u, 0u, 0u, 0u};
    *reinterpret_cast<uint4*>(tX + l16 * LDX + q * 8) = cst;
    *reinterpret_cast<uint4*>(tX + (16 + l16) * LDX + q * 8) = cst;
  }
}

// ---------------------------------------------------------------- forward statistics
// Per block: S = sum x x^T and s = sum x over its pixels -> slab[blk][NGRAM]
// (S[c][c'] at c*16 + c', s[c] at 256 + c).
__global__ void __launch_bounds__(256) k_c1bn_gram(const uint16_t* __restrict__ X, long long M,
                                                   float* __restrict__ slab, const float* __restrict__ xsc,
                                                   const float* __restrict__ xsh, int xrelu) {
  __shared__ __attribute__((aligned(16))) uint16_t tiles[4][32 * LDX];
  __shared__ float red[4][NGRAM];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4, wid = tid >> 6;
  uint16_t* tX = tiles[wid];
  x_tile_consts(tX, l16, q);
  const XPro pro = make_xpro(xsc, xsh, xrelu, q);
  f4 a0 = f4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
  const long long nblk = (M + 15) / 16;
  const long long wstride = (long long)gridDim.x * 4 * UNR;
  for (long long b0 = ((long long)blockIdx.x * 4 + wid) * UNR; b0 < nblk; b0 += wstride) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const uint4 xb = load_x(X, (b0 + u) * 16 + l16, M, q, pro);
      if (q < 2) *reinterpret_cast<uint4*>(tX + (u * 16 + l16) * LDX + q * 8) = xb;
    }
    const bf8 xt = tr8(tX, LDX, 0, lane), ones = tr8(tX, LDX, 16, lane);
    a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xt, xt, a0, 0, 0, 0);    // [c][c']
    a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xt, ones, a1, 0, 0, 0);  // [c][16] = s[c]
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wid][(q * 4 + r) * 16 + l16] = a0[r];
    if (l16 == 0) red[wid][256 + q * 4 + r] = a1[r];
  }
  __syncthreads();
  for (int i = tid; i < NGRAM; i += 256)
    slab[(long long)blockIdx.x * NGRAM + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// sum A, sum A^2 per output channel from the Gram totals -> part[0][2][K] (double)
__global__ void __launch_bounds__(128) k_c1bn_gram_fin(const float* __restrict__ gram, const float* __restrict__ w,
                                                       const float* __restrict__ bias, long long M, int K,
                                                       double* __restrict__ part) {
  __shared__ double S[16][16], s[16];
  for (int i = threadIdx.x; i < 256; i += 128) S[i >> 4][i & 15] = gram[i];
  if (threadIdx.x < 16) s[threadIdx.x] = gram[256 + threadIdx.x];
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += 128) {
    double wk[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) wk[c] = rbf(w[k * CIN + c]);
    double ws = 0.0, quad = 0.0;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      double t = 0.0;
#pragma unroll
      for (int c2 = 0; c2 < 16; ++c2) t += S[c][c2] * wk[c2];
      quad += wk[c] * t;
      ws += wk[c] * s[c];
    }
    const double b = bias ? bias[k] : 0.0, m = (double)M;
    part[k] = ws + m * b;
    part[K + k] = quad + 2.0 * b * ws + m * b * b;
  }
}

// ---------------------------------------------------------------- forward apply
// B = (ReLU)(scale * (W x) + shift'), shift' = shift + scale * b.  The wave's
// 16 x K output tile goes through a wave-private LDS tile so the global stores
// are 16-B row segments.  Per-channel parameters live in VGPRs.
template <int NKB>
__global__ void __launch_bounds__(256)
k_c1bn_apply(const uint16_t* __restrict__ X, const float* __restrict__ w, const float* __restrict__ bias, long long M,
             int relu, const float* __restrict__ scale, const float* __restrict__ shift, uint16_t* __restrict__ Y,
             const float* __restrict__ xsc, const float* __restrict__ xsh, int xrelu) {
  constexpr int K = NKB * 16, TROW = K * 2 + 16;
  constexpr int LPR = K / 8, RPI = 64 / LPR;  // lanes per 16-B pixel row, rows per store instruction
  __shared__ __attribute__((aligned(16))) unsigned char stile[4 * 16 * TROW];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4, wid = tid >> 6;
  uint4 wa[NKB];
  load_wa<NKB>(w, l16, q, wa);
  const XPro pro = make_xpro(xsc, xsh, xrelu, q);
  float psc[NKB * 4], psh[NKB * 4];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = kb * 16 + q * 4 + r;
      psc[kb * 4 + r] = scale[c];
      psh[kb * 4 + r] = shift[c] + scale[c] * (bias ? bias[c] : 0.f);
    }
  unsigned char* tile = stile + wid * 16 * TROW;
  const long long nblk = (M + 15) / 16;
  const long long wstride = (long long)gridDim.x * 4 * UNR;
  for (long long b0 = ((long long)blockIdx.x * 4 + wid) * UNR; b0 < nblk; b0 += wstride) {
    uint4 xb[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) xb[u] = load_x(X, (b0 + u) * 16 + l16, M, q, pro);
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        const f4 acc = mfma16(wa[kb], xb[u], f4{0.f, 0.f, 0.f, 0.f});
        float y[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          y[r] = fmaf(acc[r], psc[kb * 4 + r], psh[kb * 4 + r]);
          if (relu) y[r] = fmaxf(y[r], 0.f);
        }
        *reinterpret_cast<uint2*>(tile + l16 * TROW + (kb * 16 + q * 4) * 2) = uint2{pack2(y[0], y[1]),
                                                                                      pack2(y[2], y[3])};
      }
      const long long pxb = (b0 + u) * 16;
#pragma unroll
      for (int it = 0; it < 16 / RPI; ++it) {
        const int row = it * RPI + lane / LPR, seg = lane % LPR;
        const uint4 v = *reinterpret_cast<const uint4*>(tile + row * TROW + seg * 16);
        if (pxb + row < M) *reinterpret_cast<uint4*>(Y + (pxb + row) * K + seg * 8) = v;
      }
    }
  }
}

// ---------------------------------------------------------------- backward sums
// g = dB masked by the forward ReLU; per block G = g^T x (K x 16) and sum g
// -> slab[blk][K*17] (G[k][c] at k*16 + c, sum g[k] at K*16 + k).  The dB
// chunk (32 pixels x K) is staged in a wave-private LDS tile with 16-B loads
// and read transposed, so each lane holds 4 pixels x 1 channel per 16-pixel
// block: the layout of mfma(xb, wa) (the recomputed conv output) and of the
// MFMA A-operand over pixels.
template <int NKB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))  // <= 256 registers: 2 waves / SIMD
k_c1bn_bsum(const uint16_t* __restrict__ X, const float* __restrict__ w, const float* __restrict__ bias, long long M,
            int relu, const uint16_t* __restrict__ dY, const float* __restrict__ scale,
            const float* __restrict__ shift, float* __restrict__ slab, const float* __restrict__ xsc,
            const float* __restrict__ xsh, int xrelu, float* __restrict__ P) {
  constexpr int K = NKB * 16, LDB = K + 16, NOUT = K * 17, NKS = NKB / 2;
  constexpr int TB = 32 * LDB, TXE = 32 * LDX, WE = TB + TXE;  // elements per wave
  constexpr int GPL = 32 * K / 8 / 64;                          // 16-B dB granules per lane per chunk
  constexpr int SMB = 4 * WE * 2 > 4 * NOUT * 4 ? 4 * WE * 2 : 4 * NOUT * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMB];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4, wid = tid >> 6;
  uint16_t* tB = reinterpret_cast<uint16_t*>(smem) + wid * WE;
  uint16_t* tX = tB + TB;
  x_tile_consts(tX, l16, q);
  uint4 wa[NKB];
  load_wa<NKB>(w, l16, q, wa);
  const XPro pro = make_xpro(xsc, xsh, xrelu, q);
  float psc[NKB], psh[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    const int c = kb * 16 + l16;
    psc[kb] = scale[c];
    psh[kb] = shift[c] + scale[c] * (bias ? bias[c] : 0.f);
  }
  // (W o scale)^T as the A operand of P = (W^T diag(scale)) g: row = input
  // channel l16, k-slot q*8+j <-> output channel ks*32 + (j>>2)*16 + q*4 + (j&3)
  // (the k-slot order of 8-B dB row reads, as in k_c1bn_dx)
  uint4 wt[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = ks * 32 + (j >> 2) * 16 + q * 4 + (j & 3);
      v[j] = (float)((double)rbf(w[k * CIN + l16]) * (double)scale[k]);
    }
    wt[ks] = uint4{pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])};
  }
  f4 G[NKB], Gs[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) G[kb] = Gs[kb] = f4{0.f, 0.f, 0.f, 0.f};
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(c1_zero);
  const long long nblk = (M + 15) / 16;
  const long long wstride = (long long)gridDim.x * 4 * UNR;
  for (long long b0 = ((long long)blockIdx.x * 4 + wid) * UNR; b0 < nblk; b0 += wstride) {
    const long long px0 = b0 * 16;
    uint4 xb[UNR], db[GPL];
#pragma unroll
    for (int u = 0; u < UNR; ++u) xb[u] = load_x(X, px0 + u * 16 + l16, M, q, pro);
#pragma unroll
    for (int t = 0; t < GPL; ++t) {
      const int i = lane + 64 * t, row = i / (K / 8), cg = i - row * (K / 8);
      db[t] = *reinterpret_cast<const uint4*>(px0 + row < M ? dY + (px0 + row) * K + cg * 8 : zp);
    }
#pragma unroll
    for (int t = 0; t < GPL; ++t) {
      const int i = lane + 64 * t, row = i / (K / 8), cg = i - row * (K / 8);
      *reinterpret_cast<uint4*>(tB + row * LDB + cg * 8) = db[t];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (q < 2) *reinterpret_cast<uint4*>(tX + (u * 16 + l16) * LDX + q * 8) = xb[u];
    const bf8 xt = tr8(tX, LDX, 0, lane), ones = tr8(tX, LDX, 16, lane);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      const f4 a0 = mfma16(xb[0], wa[kb], f4{0.f, 0.f, 0.f, 0.f});  // pixels q*4+r of block 0, channel kb*16+l16
      const f4 a1 = mfma16(xb[1], wa[kb], f4{0.f, 0.f, 0.f, 0.f});
      bf8 g = tr8(tB, LDB, kb * 16, lane);
      if (relu) {
        const __bf16 z = (__bf16)0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (!(fmaf(a0[r], psc[kb], psh[kb]) > 0.f)) g[r] = z;
          if (!(fmaf(a1[r], psc[kb], psh[kb]) > 0.f)) g[4 + r] = z;
        }
        // masked g back into the tile for the P reads below (pixel rows 4q+r, 16+4q+r)
        __bf16* tb = reinterpret_cast<__bf16*>(tB) + kb * 16 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          tb[(4 * q + r) * LDB] = g[r];
          tb[(16 + 4 * q + r) * LDB] = g[4 + r];
        }
      }
      G[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(g, xt, G[kb], 0, 0, 0);
      Gs[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(g, ones, Gs[kb], 0, 0, 0);
    }
    // P = (W^T diag(scale)) g: lane = pixel l16 of block u, rows q*4+r = input channels
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const uint16_t* rowp = tB + (u * 16 + l16) * LDB + q * 4;
      f4 ax = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const uint2 g0 = *reinterpret_cast<const uint2*>(rowp + ks * 32);
        const uint2 g1 = *reinterpret_cast<const uint2*>(rowp + ks * 32 + 16);
        ax = mfma16(wt[ks], uint4{g0.x, g0.y, g1.x, g1.y}, ax);
      }
      const long long px = px0 + u * 16 + l16;
      if (px < M) *reinterpret_cast<f4*>(P + px * CIN + q * 4) = ax;
    }
  }
  __syncthreads();  // tiles dead; reuse smem for the cross-wave sum
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = kb * 16 + q * 4 + r;
      red[wid * NOUT + k * 16 + l16] = G[kb][r];
      if (l16 == 0) red[wid * NOUT + K * 16 + k] = Gs[kb][r];
    }
  __syncthreads();
  for (int i = tid; i < NOUT; i += 256)
    slab[(long long)blockIdx.x * NOUT + i] = (red[i] + red[NOUT + i]) + (red[2 * NOUT + i] + red[3 * NOUT + i]);
}

// ---------------------------------------------------------------- backward finalize (one block)
// From G, sum g (tot) and the forward Gram (gram): dgamma, dbeta, dw, db and the
// dx-pass constants dxp = {W o ca [K][16], M2 = W^T diag(cb) W [16][16], c0 [16]}.
// count = M in training, 1e300 in eval (statistics are constants).
__global__ void __launch_bounds__(128)
k_c1bn_bfin(const float* __restrict__ tot, const float* __restrict__ gram, const float* __restrict__ w,
            const float* __restrict__ bias, const float* __restrict__ scale, const float* __restrict__ mean,
            const float* __restrict__ invstd, long long M, double count, int K, float* __restrict__ dgamma,
            float* __restrict__ dbeta, float* __restrict__ dw, float* __restrict__ db, float* __restrict__ dxp) {
  __shared__ double S[16][16], s[16], cbs[128], cvs[128];
  __shared__ float wb[128][16];
  for (int i = threadIdx.x; i < 256; i += 128) S[i >> 4][i & 15] = gram[i];
  if (threadIdx.x < 16) s[threadIdx.x] = gram[256 + threadIdx.x];
  for (int i = threadIdx.x; i < K * 16; i += 128) wb[i >> 4][i & 15] = rbf(w[i]);
  __syncthreads();
  const double m = (double)M;
  for (int k = threadIdx.x; k < K; k += 128) {
    const double b = bias ? bias[k] : 0.0, sg = tot[K * 16 + k];
    double sga = b * sg, ws = 0.0;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      sga += (double)wb[k][c] * tot[k * 16 + c];
      ws += (double)wb[k][c] * s[c];
    }
    const double is = invstd[k], mu = mean[k], sc = scale[k];
    const double sgx = is * (sga - mu * sg);
    if (dgamma) dgamma[k] = (float)sgx;
    if (dbeta) dbeta[k] = (float)sg;
    const double mg = sg / count, mgx = sgx / count;
    const double ca = sc, cb = -sc * mgx * is, cc = -sc * mg + sc * mgx * is * mu;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      double wsc = b * s[c];
#pragma unroll
      for (int c2 = 0; c2 < 16; ++c2) wsc += (double)wb[k][c2] * S[c2][c];
      dw[k * 16 + c] = (float)(ca * tot[k * 16 + c] + cb * wsc + cc * s[c]);
      dxp[k * 16 + c] = (float)(wb[k][c] * ca);
    }
    if (db) db[k] = (float)(ca * sg + cb * (ws + m * b) + m * cc);
    cbs[k] = cb;
    cvs[k] = cb * b + cc;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += 128) {
    const int c = i >> 4, c2 = i & 15;
    double t = 0.0;
    for (int k = 0; k < K; ++k) t += (double)wb[k][c] * cbs[k] * wb[k][c2];
    dxp[K * 16 + i] = (float)t;
  }
  if (threadIdx.x < 16) {
    double t = 0.0;
    for (int k = 0; k < K; ++k) t += (double)wb[k][threadIdx.x] * cvs[k];
    dxp[K * 16 + 256 + threadIdx.x] = (float)t;
  }
}

// ---------------------------------------------------------------- backward dx
// dx = P + M2 x + c0 (P from k_c1bn_bsum).  Orientation mfma(m2, xb): lane =
// pixel l16, rows q*4 + r = input channels, the layout of P's 16-B row reads.
__global__ void __launch_bounds__(256)
k_c1bn_dx(const uint16_t* __restrict__ X, long long M, const float* __restrict__ P, const float* __restrict__ dxp,
          int K, uint16_t* __restrict__ dX, const float* __restrict__ xsc, const float* __restrict__ xsh, int xrelu) {
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4, wid = tid >> 6;
  const XPro pro = make_xpro(xsc, xsh, xrelu, q);
  uint4 m2 = {0u, 0u, 0u, 0u};
  if (q < 2) {
    const float* p = dxp + K * 16 + l16 * 16 + q * 8;  // M2[c = l16][c' = q*8 + j]
    m2 = uint4{pack2(p[0], p[1]), pack2(p[2], p[3]), pack2(p[4], p[5]), pack2(p[6], p[7])};
  }
  float c0[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) c0[r] = dxp[K * 16 + 256 + q * 4 + r];
  const long long nblk = (M + 15) / 16;
  const long long wstride = (long long)gridDim.x * 4 * UNR;
  for (long long b0 = ((long long)blockIdx.x * 4 + wid) * UNR; b0 < nblk; b0 += wstride) {
    uint4 xb[UNR];
    f4 pv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long px = (b0 + u) * 16 + l16;
      xb[u] = load_x(X, px, M, q, pro);
      pv[u] = px < M ? *reinterpret_cast<const f4*>(P + px * CIN + q * 4) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long px = (b0 + u) * 16 + l16;
      const f4 ax = mfma16(m2, xb[u], f4{0.f, 0.f, 0.f, 0.f});
      if (px < M)
        *reinterpret_cast<uint2*>(dX + px * CIN + q * 4) =
            uint2{pack2((pv[u][0] + ax[0]) + c0[0], (pv[u][1] + ax[1]) + c0[1]),
                  pack2((pv[u][2] + ax[2]) + c0[2], (pv[u][3] + ax[3]) + c0[3])};
    }
  }
}

// out[col] = sum_z slab[z][col], col < n (fixed order).
// 1024 threads = 64 row groups x 16 columns, four independent sums per thread.
__global__ void __launch_bounds__(1024)
k_c1bn_slab_sum(const float* __restrict__ slab, int nrows, int n, float* __restrict__ out) {
  __shared__ float tmp[64][16];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + cl;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < n) {
    int r = rg;
    for (; r + 192 < nrows; r += 256) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += slab[(long long)(r + 64 * u) * n + col];
    }
    for (int u = 0; r < nrows; r += 64, ++u) a[u & 3] += slab[(long long)r * n + col];
  }
  tmp[rg][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (rg == 0 && col < n) {
    float s = 0.f;
#pragma unroll 8
    for (int i = 0; i < 64; ++i) s += tmp[i][cl];
    out[col] = s;
  }
}

// grids are whole multiples of the resident workgroups (bsum: 228 registers -> 2 per CU; apply: 160 -> 3 per CU)
constexpr int GRAM_GRID = 1024, APPLY_GRID = 3072, BSUM_GRID = 512, DX_GRID = 2048;

int c1_grid(long long M, int cap) {
  const long long steps = ((M + 15) / 16 + 4 * UNR - 1) / (4 * UNR);
  const long long g = steps < cap ? steps : cap;
  return (int)(g < 1 ? 1 : g);
}

// float offset of P [M][16] in the backward workspace (16-B aligned)
long long p_offset(long long M, int K) {
  return ((long long)c1_grid(M, BSUM_GRID) * K * 17 + K * 17 + K * 16 + 256 + 16 + 3) & ~3ll;
}

bool shape_ok(long long M, int C, int K, const void* x) {
  return M > 0 && C == CIN && (K == 64 || K == 128) && x && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
}

}  // namespace

// ---------------------------------------------------------------- C ABI
ACFE_API int acfe_c1bn_supported(int C, int K) { return C == CIN && (K == 64 || K == 128); }

ACFE_API long long acfe_c1bn_workspace(long long M, int C, int K) {
  if (M <= 0 || C != CIN || K <= 0 || K > 128) return 0;
  const long long fwd = (long long)c1_grid(M, GRAM_GRID) * NGRAM;
  const long long bwd = p_offset(M, K) + M * CIN;  // slab, totals, dx constants, then P
  return fwd > bwd ? fwd : bwd;
}

static int c1bn_stats_impl(const void* x, long long M, int C, const float* w, int K, const float* bias,
                           double* part, float* gram, float* workspace, const float* xsc, const float* xsh, int xrelu,
                           void* stream) {
  if (!shape_ok(M, C, K, x) || !w || !part || !gram || !workspace) return ACFE_E_INVAL;
  const int grid = c1_grid(M, GRAM_GRID);
  hipLaunchKernelGGL(k_c1bn_gram, dim3(grid), dim3(256), 0, strm(stream), (const uint16_t*)x, M, workspace, xsc, xsh,
                     xrelu);
  hipLaunchKernelGGL(k_c1bn_slab_sum, dim3(cdiv(NGRAM, 16)), dim3(1024), 0, strm(stream), workspace, grid, NGRAM,
                     gram);
  hipLaunchKernelGGL(k_c1bn_gram_fin, dim3(1), dim3(128), 0, strm(stream), gram, w, bias, M, K, part);
  return launch_rc("acfe_c1bn_stats");
}

static int c1bn_apply_impl(const void* x, long long M, int C, const float* w, int K, const float* bias,
                           const float* scale, const float* shift, int relu, void* y, const float* xsc,
                           const float* xsh, int xrelu, void* stream) {
  if (!shape_ok(M, C, K, x) || !w || !scale || !shift || !y || (reinterpret_cast<uintptr_t>(y) & 15))
    return ACFE_E_INVAL;
  const int grid = c1_grid(M, APPLY_GRID);
  if (K == 128)
    hipLaunchKernelGGL((k_c1bn_apply<8>), dim3(grid), dim3(256), 0, strm(stream), (const uint16_t*)x, w, bias, M,
                       relu, scale, shift, (uint16_t*)y, xsc, xsh, xrelu);
  else
    hipLaunchKernelGGL((k_c1bn_apply<4>), dim3(grid), dim3(256), 0, strm(stream), (const uint16_t*)x, w, bias, M,
                       relu, scale, shift, (uint16_t*)y, xsc, xsh, xrelu);
  return launch_rc("acfe_c1bn_apply");
}

static int c1bn_bwd_impl(const void* dy, const void* x, long long M, int C, const float* w, int K,
                         const float* bias, const float* scale, const float* shift, const float* mean,
                         const float* invstd, int relu, double count, const float* gram, void* dx, float* dw,
                         float* db, float* dgamma, float* dbeta, float* workspace, const float* xsc,
                         const float* xsh, int xrelu, void* stream) {
  if (!shape_ok(M, C, K, x) || !dy || !w || !scale || !shift || !mean || !invstd || !gram || !dx || !dw ||
      !workspace || count <= 0 || (reinterpret_cast<uintptr_t>(dy) & 15) || (reinterpret_cast<uintptr_t>(dx) & 7))
    return ACFE_E_INVAL;
  const int gs = c1_grid(M, BSUM_GRID), n = K * 17;
  float* slab = workspace;
  float* tot = slab + (long long)gs * n;
  float* dxp = tot + n;
  float* P = workspace + p_offset(M, K);
  hipStream_t s = strm(stream);
  if (K == 128)
    hipLaunchKernelGGL((k_c1bn_bsum<8>), dim3(gs), dim3(256), 0, s, (const uint16_t*)x, w, bias, M, relu,
                       (const uint16_t*)dy, scale, shift, slab, xsc, xsh, xrelu, P);
  else
    hipLaunchKernelGGL((k_c1bn_bsum<4>), dim3(gs), dim3(256), 0, s, (const uint16_t*)x, w, bias, M, relu,
                       (const uint16_t*)dy, scale, shift, slab, xsc, xsh, xrelu, P);
  hipLaunchKernelGGL(k_c1bn_slab_sum, dim3(cdiv(n, 16)), dim3(1024), 0, s, slab, gs, n, tot);
  hipLaunchKernelGGL(k_c1bn_bfin, dim3(1), dim3(128), 0, s, tot, gram, w, bias, scale, mean, invstd, M, count, K,
                     dgamma, dbeta, dw, db, dxp);
  const int gd = c1_grid(M, DX_GRID);
  hipLaunchKernelGGL(k_c1bn_dx, dim3(gd), dim3(256), 0, s, (const uint16_t*)x, M, P, dxp, K, (uint16_t*)dx, xsc, xsh,
                     xrelu);
  return launch_rc("acfe_c1bn_bwd");
}

ACFE_API int acfe_c1bn_stats(const void* x, long long M, int C, const float* w, int K, const float* bias,
                             double* part, float* gram, float* workspace, void* stream) {
  return c1bn_stats_impl(x, M, C, w, K, bias, part, gram, workspace, nullptr, nullptr, 0, stream);
}

ACFE_API int acfe_c1bn_apply(const void* x, long long M, int C, const float* w, int K, const float* bias,
                             const float* scale, const float* shift, int relu, void* y, void* stream) {
  return c1bn_apply_impl(x, M, C, w, K, bias, scale, shift, relu, y, nullptr, nullptr, 0, stream);
}

ACFE_API int acfe_c1bn_bwd(const void* dy, const void* x, long long M, int C, const float* w, int K,
                           const float* bias, const float* scale, const float* shift, const float* mean,
                           const float* invstd, int relu, double count, const float* gram, void* dx, float* dw,
                           float* db, float* dgamma, float* dbeta, float* workspace, void* stream) {
  return c1bn_bwd_impl(dy, x, M, C, w, K, bias, scale, shift, mean, invstd, relu, count, gram, dx, dw, db, dgamma,
                       dbeta, workspace, nullptr, nullptr, 0, stream);
}

// The same three passes with the BatchNormalization (+ReLU) prologue on x
// (x_scale / x_shift: fp32 [16] from acfe_bn_finalize of the BN in front of
// the 1x1 conv): x is the BN INPUT, x' = (ReLU)(x * x_scale + x_shift) is
// formed in every pass and never stored; dx is the gradient for x'.
ACFE_API int acfe_c1bn_stats_bn(const void* x, long long M, int C, const float* w, int K, const float* bias,
                                double* part, float* gram, float* workspace, const float* x_scale,
                                const float* x_shift, int x_relu, void* stream) {
  if (!x_scale || !x_shift) return ACFE_E_INVAL;
  return c1bn_stats_impl(x, M, C, w, K, bias, part, gram, workspace, x_scale, x_shift, x_relu, stream);
}

ACFE_API int acfe_c1bn_apply_bn(const void* x, long long M, int C, const float* w, int K, const float* bias,
                                const float* scale, const float* shift, int relu, void* y, const float* x_scale,
                                const float* x_shift, int x_relu, void* stream) {
  if (!x_scale || !x_shift) return ACFE_E_INVAL;
  return c1bn_apply_impl(x, M, C, w, K, bias, scale, shift, relu, y, x_scale, x_shift, x_relu, stream);
}

ACFE_API int acfe_c1bn_bwd_bn(const void* dy, const void* x, long long M, int C, const float* w, int K,
                              const float* bias, const float* scale, const float* shift, const float* mean,
                              const float* invstd, int relu, double count, const float* gram, void* dx, float* dw,
                              float* db, float* dgamma, float* dbeta, float* workspace, const float* x_scale,
                              const float* x_shift, int x_relu, void* stream) {
  if (!x_scale || !x_shift) return ACFE_E_INVAL;
  return c1bn_bwd_impl(dy, x, M, C, w, K, bias, scale, shift, mean, invstd, relu, count, gram, dx, dw, db, dgamma,
                       dbeta, workspace, x_scale, x_shift, x_relu, stream);
}
