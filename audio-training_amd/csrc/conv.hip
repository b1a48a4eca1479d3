// Convolution engine for resnet/wr_resnet.py and resnet/wr_resnet_bird.py
// (Keras Conv2D, NHWC, "same"/"valid", bias, KRSC weights).
//
//  * k_conv_fwd   implicit-im2col GEMM on MFMA: M = N*P*Q output pixels,
//                 N = K output channels, reduction = R*S*C.  bf16 operands on
//                 v_mfma_f32_16x16x32_bf16, or exact fp32 on v_mfma_f32_16x16x4_f32.
//                 256 threads = 4 waves, BM=128 pixel rows x BN channels per tile,
//                 register-staged double-buffered LDS (rows padded by 16 B so the
//                 ds_read_b128 fragment reads are conflict-free), persistent loop
//                 over M tiles.  Epilogue: +bias, round to the storage type,
//                 per-channel sum / sum-of-squares of the ROUNDED outputs (the
//                 training-mode BatchNormalization statistics of the next layer)
//                 accumulated in double per block, tile staged in LDS and written
//                 as 16-byte rows.
//  * dgrad        stride 1: the same kernel on flipped/transposed weights
//                 (W'[c][r'][s'][k] = W[k][R-1-r'][S-1-s'][c], pad' = R-1-pad);
//                 stride > 1: zero-insert dY, then the same.
//  * k_conv_wgrad split-K GEMM dW[k][rsc] = sum_m dY[m][k] * im2col(X)[m][rsc]
//                 with both operands staged m-major and fed to the MFMA through
//                 ds_read_b64_tr_b16 (bf16) -- per-split fp32 slabs, then a
//                 deterministic reduction.
//  * stem         C = 1 direct kernels (the 3 identical input channels of
//                 tfdataset.py:2053 are folded into one by summing the stem
//                 weights over Cin; exact up to fp reassociation).
#include "conv_common.h"

// Timing-only ablations of the BN-fold weight gradient (they skip work and
// compute wrong results): only in `make ablate` builds (libacfe_ablate.so)
#if !defined(ACFE_ABLATE) && (defined(ACFE_FB_NOXFORM) || defined(ACFE_FB_NOSUM) || defined(ACFE_FB_NOSTORE) || \
                              defined(ACFE_FB_MID))
#error "ACFE_FB_* ablation switches belong to `make ablate` builds only"
#endif

using namespace acfe;



// 64 bytes of zeros in global memory: im2col taps that fall into the padding
// (or past the last pixel) load from here, so every load is unconditional
// (no branch around the load, no select after it).
__device__ __attribute__((aligned(64))) uint4 g_zero_page[4];


template <typename T> struct TT;
template <> struct TT<uint16_t> { static constexpr int GR = 8, BK = 64; };
template <> struct TT<float> { static constexpr int GR = 4, BK = 32; };

__device__ __forceinline__ void mma(f4& acc, const uint4& a, const uint4& b, uint16_t) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b), acc,
                                                0, 0, 0);
}
__device__ __forceinline__ void mma(f4& acc, const uint4& a, const uint4& b, float) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
}
__device__ __forceinline__ uint16_t cvt_out(float v, uint16_t) { return f2bf(v); }
__device__ __forceinline__ float cvt_out(float v, float) { return v; }
__device__ __forceinline__ float to_f(uint16_t v) { return bf2f(v); }
__device__ __forceinline__ float to_f(float v) { return v; }

template <typename T, int BM, int BN>
constexpr int conv_smem() {
  constexpr int LR = TT<T>::BK + TT<T>::GR;
  constexpr int a = 2 * (BM + BN) * LR * (int)sizeof(T);
  constexpr int b = BM * (BN + TT<T>::GR) * (int)sizeof(T);
  constexpr int c = 2 * 2 * BN * 8;
  return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

// ------------------------------------------------------------------ forward
template <typename T, int BM, int BN, int WM, int WN, bool FAST_A>
__global__ void __launch_bounds__(256)
k_conv_fwd(ConvGeom g, const T* __restrict__ X, const T* __restrict__ Wp, const float* __restrict__ bias,
           T* __restrict__ Y, double* __restrict__ stats, int tiles_m) {
  constexpr int GR = TT<T>::GR, BK = TT<T>::BK, LR = BK + GR, LC = BN + GR;
  constexpr int RA = BM / 32, RB = BN / 32;
  constexpr int TWM = BM / WM, TWN = BN / WN, FM = TWM / 16, FN = TWN / 16;
  constexpr int KF = 4 * GR;
  static_assert(WM * WN == 4 && BN >= 32 && FM >= 1 && FN >= 1, "tile");
  __shared__ __attribute__((aligned(16))) unsigned char smem[conv_smem<T, BM, BN>()];
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + 2 * BM * LR;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int gc = tid & 7, rr = tid >> 3;
  const int n0 = blockIdx.y * BN;
  const int nkt = g.Kdp / BK;
  const long long PQ = (long long)g.P * g.Q;
  __shared__ double sstat[2][BN];  // per-block BN statistics (sum, sum of squares)
  if (stats)
    for (int i = tid; i < 2 * BN; i += 256) (&sstat[0][0])[i] = 0.0;
  const T* zp = reinterpret_cast<const T*>(g_zero_page);

  const TileWalk walk(tiles_m);
  for (int tm = walk.tm; tm < walk.end; tm += walk.step) {
    const long long m0 = (long long)tm * BM;
    const T* rowp[RA];
    int h0[RA], w0[RA];
    bool mv[RA];
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const long long m = m0 + rr + 32 * i;
      mv[i] = m < g.M;
      const long long mm = mv[i] ? m : 0;
      const int n = (int)(mm / PQ);
      const int rem = (int)(mm - (long long)n * PQ);
      const int p = rem / g.Q, q = rem - (rem / g.Q) * g.Q;
      h0[i] = p * g.st - g.pt;
      w0[i] = q * g.st - g.pl;
      rowp[i] = X + (((long long)n * g.H + h0[i]) * g.W + w0[i]) * g.C;
    }
    int kk0 = gc * GR, c0, r, s;
    {
      const int rs = kk0 / g.C;
      c0 = kk0 - rs * g.C;
      r = rs / g.S;
      s = rs - r * g.S;
    }
    uint4 ra[RA], rb[RB];
    auto gload = [&](int kt) __attribute__((always_inline)) {
      if constexpr (FAST_A) {
        const bool kv = kk0 < g.Kd;
        const int off = (r * g.W + s) * g.C + c0;
#pragma unroll
        for (int i = 0; i < RA; ++i) {
          const int h = h0[i] + r, w = w0[i] + s;
          const bool ok = kv && mv[i] && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
          ra[i] = *reinterpret_cast<const uint4*>(ok ? rowp[i] + off : zp);
        }
      } else {
#pragma unroll
        for (int i = 0; i < RA; ++i) {
          T e[GR];
#pragma unroll
          for (int j = 0; j < GR; ++j) {
            const int kk = kk0 + j;
            bool ok = mv[i] && kk < g.Kd;
            const int rs = kk / g.C, c = kk - rs * g.C, rq = rs / g.S, sq = rs - rq * g.S;
            const int h = h0[i] + rq, w = w0[i] + sq;
            ok = ok && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
            const T* src = ok ? rowp[i] + (rq * g.W + sq) * g.C + c : X;
            const T v = *src;
            e[j] = ok ? v : (T)0;
          }
          ra[i] = *reinterpret_cast<const uint4*>(e);
        }
      }
#pragma unroll
      for (int i = 0; i < RB; ++i)
        rb[i] = *reinterpret_cast<const uint4*>(Wp + (long long)(n0 + rr + 32 * i) * g.Kdp + kt * BK + gc * GR);
    };
    auto advance = [&]() __attribute__((always_inline)) {
      kk0 += BK;
      if constexpr (FAST_A) {
        c0 += BK;
        while (c0 >= g.C) {
          c0 -= g.C;
          if (++s == g.S) { s = 0; ++r; }
        }
      }
    };
    auto sstore = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < RA; ++i)
        *reinterpret_cast<uint4*>(As + (buf * BM + rr + 32 * i) * LR + gc * GR) = ra[i];
#pragma unroll
      for (int i = 0; i < RB; ++i)
        *reinterpret_cast<uint4*>(Bs + (buf * BN + rr + 32 * i) * LR + gc * GR) = rb[i];
    };
    f4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

    gload(0);
    advance();
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const bool more = kt + 1 < nkt;
      if (more) {
        gload(kt + 1);
        advance();
      }
      const int buf = kt & 1;
#pragma unroll
      for (int kk = 0; kk < BK / KF; ++kk) {
        uint4 af[FM], bfr[FN];
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
          af[fm] = *reinterpret_cast<const uint4*>(
              As + (buf * BM + wm * TWM + fm * 16 + (lane & 15)) * LR + kk * KF + (lane >> 4) * GR);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          bfr[fn] = *reinterpret_cast<const uint4*>(
              Bs + (buf * BN + wn * TWN + fn * 16 + (lane & 15)) * LR + kk * KF + (lane >> 4) * GR);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) mma(acc[fm][fn], af[fm], bfr[fn], T());
      }
      if (more) sstore(buf ^ 1);
      __syncthreads();
    }
    // ---- epilogue
    T* Cs = As;
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int col = wn * TWN + fn * 16 + (lane & 15);
      const int gcn = n0 + col;
      const float bv = (bias && gcn < g.K) ? bias[gcn] : 0.f;
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = wm * TWM + fm * 16 + (lane >> 4) * 4 + j;
          T tv = cvt_out(acc[fm][fn][j] + bv, T());
          if (g.drop.on)
            tv = cvt_out(drop_apply<T>(g.drop, (uint64_t)(m0 + row) * g.K + gcn, to_f(tv)), T());
          Cs[row * LC + col] = tv;
          if (m0 + row < g.M) {
            const float f = to_f(tv);
            t1 += f;
            t2 += f * f;
          }
        }
      if (stats) {
        t1 += __shfl_xor(t1, 16, 64);
        t1 += __shfl_xor(t1, 32, 64);
        t2 += __shfl_xor(t2, 16, 64);
        t2 += __shfl_xor(t2, 32, 64);
        if (lane < 16) {
          atomicAdd(&sstat[0][col], (double)t1);
          atomicAdd(&sstat[1][col], (double)t2);
        }
      }
    }
    __syncthreads();
    constexpr int GPR = BN / GR;
    if (n0 + BN <= g.K && (g.ldy % GR) == 0) {
      for (int idx = tid; idx < BM * GPR; idx += 256) {
        const int row = idx / GPR, cg = idx - (idx / GPR) * GPR;
        const long long m = m0 + row;
        if (m < g.M)
          *reinterpret_cast<uint4*>(Y + m * g.ldy + n0 + cg * GR) =
              *reinterpret_cast<const uint4*>(Cs + row * LC + cg * GR);
      }
    } else {
      for (int idx = tid; idx < BM * BN; idx += 256) {
        const int row = idx / BN, col = idx - (idx / BN) * BN;
        const long long m = m0 + row;
        if (m < g.M && n0 + col < g.K) Y[m * g.ldy + n0 + col] = Cs[row * LC + col];
      }
    }
    __syncthreads();
  }
  if (stats) {
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      stats[((long long)blockIdx.x * 2 + 0) * g.Kp + n0 + c] = sstat[0][c];
      stats[((long long)blockIdx.x * 2 + 1) * g.Kp + n0 + c] = sstat[1][c];
    }
  }
}


// ------------------------------------------------------------------ forward, LDS-DMA staged
// C % GR == 0 path.  Each K-tile (BK elements = 128 B per row) of the im2col A
// tile and of the packed weight tile is copied HBM/L2 -> LDS by
// global_load_lds_dwordx4 (no staging VGPRs, no ds_write).  One wave
// instruction fills 8 rows x 128 B lane-linearly; lane l holds row l>>3, LDS
// slot l&7, and fetches global granule (l&7) ^ (row&7): the XOR swizzle lives on
// the source address, so the 16-lane ds_read_b128 fragment reads (granule g of
// row r at slot g ^ (r&7)) are bank-conflict free.  Two LDS buffers, prefetch
// of tile t+1 issued before the MFMAs of tile t, one vmcnt(0)+barrier per tile.

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_base, 16, 0, 0);
}

// The same 16-B LDS-DMA issued from inline asm.  hipcc does not track it, so
// it never inserts the conservative vmcnt(0) before ds_reads of the OTHER
// stage buffer (which it does for the intrinsic: it cannot tell the stages
// apart), and the prefetch stays in flight under the MFMAs.  The caller owns
// the vmcnt bookkeeping.  M0 = LDS base of the wave's 1 KiB destination.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16_async(const void* src, unsigned char* lds_base) {
  const unsigned m0v = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)lds_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0v)
               : "memory", "m0");
}
#pragma clang diagnostic pop

template <typename T, int BM, int BN>
constexpr int conv_g_smem() {
  constexpr int a = 2 * (BM + BN) * 128;
  constexpr int b = BM * (BN + TT<T>::GR) * (int)sizeof(T);
  return a > b ? a : b;
}

template <typename T, int BM, int BN, int WM, int WN, bool RES = false>
__global__ void __launch_bounds__(256, 2)
k_conv_fwd_g(ConvGeom g, const T* __restrict__ X, const T* __restrict__ Wp, const float* __restrict__ bias,
             T* __restrict__ Y, double* __restrict__ stats, int tiles_m) {
  constexpr int GR = TT<T>::GR, BK = TT<T>::BK, LC = BN + GR;
  static_assert(BK * (int)sizeof(T) == 128, "128-byte K rows");
  constexpr int AJ = BM / 32, BJ = BN / 32;
  constexpr int TWM = BM / WM, TWN = BN / WN, FM = TWM / 16, FN = TWN / 16;
  constexpr int KF = 4 * GR;
  static_assert(WM * WN == 4 && BN >= 32 && FM >= 1 && FN >= 1, "tile");
  // ONE __shared__ array: [2 stages][BM + BN rows][128 B], then the epilogue's
  // statistics accumulators (the C staging tile reuses the stages).
  constexpr int STG = (BM + BN) * 128;
  constexpr int CST = BM * (BN + GR) * (int)sizeof(T);
  constexpr int SOFF = (2 * STG > CST ? 2 * STG : CST);
  __shared__ __attribute__((aligned(16))) unsigned char smem[SOFF + 2 * BN * (int)sizeof(double)];
  double (*sstat)[BN] = reinterpret_cast<double (*)[BN]>(smem + SOFF);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int lrow = lane >> 3;                       // row within an 8-row wave piece
  const int gsw = (lane & 7) ^ (lrow & 7);          // granule column this lane fetches
  const int n0 = blockIdx.y * BN;
  const int nkt = g.Kdp / BK;
  const long long PQ = (long long)g.P * g.Q;
  const T* zp = reinterpret_cast<const T*>(g_zero_page);
  if (stats)
    for (int i = tid; i < 2 * BN; i += 256) (&sstat[0][0])[i] = 0.0;
  const T* wrow[BJ];
#pragma unroll
  for (int j = 0; j < BJ; ++j) wrow[j] = Wp + (long long)(n0 + (wid * BJ + j) * 8 + lrow) * g.Kdp + gsw * GR;

  // fp32 (configs I / S): K-tiles chunk-major (32-channel chunk outermost,
  // then the taps) instead of tap-major.  The tiles resident on one XCD cover
  // ~32 output rows; tap-major, each reads all C channels of its three input
  // rows over the tile, a live set of ~4.5 MB per XCD at 128 fp32 channels --
  // more than the 4 MB L2, so rows came from HBM again (S: 1.86x algorithmic,
  // profiles/pmc_dominant_stream_fp32_r04.json).  Chunk-major, the live set is
  // one chunk of those rows (a quarter)
  const bool cmaj = sizeof(T) == 4 && g.cmaj && g.R * g.S > 1 && g.C % BK == 0;
  const TileWalk walk(tiles_m);
  for (int tm = walk.tm; tm < walk.end; tm += walk.step) {
    const long long m0 = (long long)tm * BM;
    const T* rowp[AJ];
    int h0[AJ], w0[AJ];
    bool mv[AJ];
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const long long m = m0 + (wid * AJ + j) * 8 + lrow;
      mv[j] = m < g.M;
      const long long mm = mv[j] ? m : 0;
      const int n = (int)(mm / PQ);
      const int rem = (int)(mm - (long long)n * PQ);
      const int p = rem / g.Q, q = rem - (rem / g.Q) * g.Q;
      h0[j] = p * g.st - g.pt;
      w0[j] = q * g.st - g.pl;
      rowp[j] = X + (((long long)n * g.H + h0[j]) * g.W + w0[j]) * g.C;
    }
    int kk0 = gsw * GR, c0, r, s;
    {
      const int rs = kk0 / g.C;
      c0 = kk0 - rs * g.C;
      r = rs / g.S;
      s = rs - r * g.S;
    }
#define CONV_G_ISSUE(KT, BUF)                                                                     \
    {                                                                                             \
      const bool kv = kk0 < g.Kd;                                                                 \
      const int off = (r * g.W + s) * g.C + c0;                                                   \
      _Pragma("unroll") for (int j = 0; j < AJ; ++j) {                                            \
        const int h = h0[j] + r, w = w0[j] + s;                                                   \
        const bool ok = kv && mv[j] && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W; \
        glds16_async(ok ? (const void*)(rowp[j] + off) : (const void*)zp,                        \
                     (BUF) + ((wid * AJ + j) * 8) * 128);                                         \
      }                                                                                           \
      const int wcol = cmaj ? (r * g.S + s) * g.C + c0 - gsw * GR : (KT) * BK;                    \
      _Pragma("unroll") for (int j = 0; j < BJ; ++j)                                              \
        glds16_async(wrow[j] + wcol, (BUF) + (BM + (wid * BJ + j) * 8) * 128);                    \
      kk0 += BK;                                                                                  \
      if (cmaj) {                                                                                 \
        if (++s == g.S) {                                                                         \
          s = 0;                                                                                  \
          if (++r == g.R) { r = 0; c0 += BK; }                                                    \
        }                                                                                         \
      } else {                                                                                    \
        c0 += BK;                                                                                 \
        while (c0 >= g.C) {                                                                       \
          c0 -= g.C;                                                                              \
          if (++s == g.S) { s = 0; ++r; }                                                         \
        }                                                                                         \
      }                                                                                           \
    }
    f4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#define CONV_G_COMPUTE(BUF)                                                                       \
    {                                                                                             \
      const unsigned char* Ab = (BUF);                                                            \
      const unsigned char* Bb = (BUF) + BM * 128;                                                 \
      _Pragma("unroll") for (int kk = 0; kk < BK / KF; ++kk) {                                    \
        const int gi = kk * 4 + (lane >> 4);                                                      \
        uint4 af[FM], bfr[FN];                                                                    \
        _Pragma("unroll") for (int fm = 0; fm < FM; ++fm) {                                       \
          const int row = wm * TWM + fm * 16 + (lane & 15);                                       \
          af[fm] = *reinterpret_cast<const uint4*>(Ab + row * 128 + ((gi ^ (row & 7)) << 4));     \
        }                                                                                         \
        _Pragma("unroll") for (int fn = 0; fn < FN; ++fn) {                                       \
          const int row = wn * TWN + fn * 16 + (lane & 15);                                       \
          bfr[fn] = *reinterpret_cast<const uint4*>(Bb + row * 128 + ((gi ^ (row & 7)) << 4));    \
        }                                                                                         \
        _Pragma("unroll") for (int fm = 0; fm < FM; ++fm)                                         \
          _Pragma("unroll") for (int fn = 0; fn < FN; ++fn) mma(acc[fm][fn], af[fm], bfr[fn], T()); \
      }                                                                                           \
    }
    CONV_G_ISSUE(0, smem)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      unsigned char* cur = smem + (kt & 1) * STG;
      // prefetch the next stage (inline-asm DMA: stays in flight under the MFMAs)
      if (kt + 1 < nkt) CONV_G_ISSUE(kt + 1, smem + ((kt + 1) & 1) * STG)
      CONV_G_COMPUTE(cur)
      // next stage landed (vmcnt) and this stage's fragment reads retired
      // (lgkmcnt) before anyone passes the barrier and restages `cur`
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __syncthreads();
    }
#undef CONV_G_COMPUTE
#undef CONV_G_ISSUE
    // ---- epilogue: +bias, round, BN statistics of the rounded values, LDS-staged 16-B row stores
    // (g.res: the residual Add (+ReLU) of ops.conv_add is applied in the row
    // stores and the statistics are those of z = (ReLU)(y + res))
    constexpr bool res = RES && sizeof(T) == 2;
    constexpr int GPR = BN / GR, NR = BM * GPR / 256;
    u32x4 rvs[NR];
    T* Cs = reinterpret_cast<T*>(smem);
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int col = wn * TWN + fn * 16 + (lane & 15);
      const int gcn = n0 + col;
      const float bv = (bias && gcn < g.K) ? bias[gcn] : 0.f;
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = wm * TWM + fm * 16 + (lane >> 4) * 4 + j;
          T tv = cvt_out(acc[fm][fn][j] + bv, T());
          if (g.drop.on)
            tv = cvt_out(drop_apply<T>(g.drop, (uint64_t)(m0 + row) * g.K + gcn, to_f(tv)), T());
          Cs[row * LC + col] = tv;
          if (m0 + row < g.M) {
            const float f = to_f(tv);
            t1 += f;
            t2 += f * f;
          }
        }
      if (stats && !res) {
        t1 += __shfl_xor(t1, 16, 64);
        t1 += __shfl_xor(t1, 32, 64);
        t2 += __shfl_xor(t2, 16, 64);
        t2 += __shfl_xor(t2, 32, 64);
        if (lane < 16) {
          atomicAdd(&sstat[0][col], (double)t1);
          atomicAdd(&sstat[1][col], (double)t2);
        }
      }
    }
    if constexpr (res) {
      // the residual rows of this thread's stores are requested before the
      // barrier, all at once (rows past M read the zero page)
#pragma unroll
      for (int u = 0; u < NR; ++u) {
        const long long m = m0 + (tid + 256 * u) / GPR;
        rvs[u] = *reinterpret_cast<const u32x4*>(m < g.M ? reinterpret_cast<const uint16_t*>(g.res) + m * g.ldy +
                                                               n0 + (tid % GPR) * GR
                                                         : reinterpret_cast<const uint16_t*>(g_zero_page));
      }
    }
    __syncthreads();
    if constexpr (res && 256 % GPR == 0) {
      {
        // z = bf16((ReLU)(y + r)) for 8 channels per thread; the thread's
        // channel group cg is fixed (256 % GPR == 0), so its statistics stay in
        // registers over its rows and are combined across the lanes holding the
        // same cg, then one LDS f64 atomic per value (the caller guarantees
        // n0 + BN <= K and 16-B rows)
        float z1[GR], z2[GR];
#pragma unroll
        for (int j = 0; j < GR; ++j) z1[j] = z2[j] = 0.f;
        const int cg = tid % GPR;
#pragma unroll
        for (int u = 0; u < NR; ++u) {
          const int row = (tid + 256 * u) / GPR;
          const long long m = m0 + row;
          if (m < g.M) {
            const u32x4 yv = *reinterpret_cast<const u32x4*>(Cs + row * LC + cg * GR);
            const u32x4 rv = rvs[u];
            u32x4 zv;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float a = __uint_as_float(yv[q] << 16) + __uint_as_float(rv[q] << 16);
              float c = __uint_as_float(yv[q] & 0xffff0000u) + __uint_as_float(rv[q] & 0xffff0000u);
              if (g.res_relu) a = fmaxf(a, 0.f), c = fmaxf(c, 0.f);
              const unsigned ba = f2bf(a), bc = f2bf(c);
              zv[q] = ba | (bc << 16);
              const float fa = __uint_as_float(ba << 16), fc = __uint_as_float(bc << 16);
              z1[2 * q] += fa, z2[2 * q] += fa * fa;
              z1[2 * q + 1] += fc, z2[2 * q + 1] += fc * fc;
            }
            *reinterpret_cast<u32x4*>(Y + m * g.ldy + n0 + cg * GR) = zv;
          }
        }
        if (stats) {
#pragma unroll
          for (int off = GPR; off < 64; off <<= 1)
#pragma unroll
            for (int j = 0; j < GR; ++j) z1[j] += __shfl_xor(z1[j], off, 64), z2[j] += __shfl_xor(z2[j], off, 64);
          if (lane < GPR) {
#pragma unroll
            for (int j = 0; j < GR; ++j) {
              atomicAdd(&sstat[0][cg * GR + j], (double)z1[j]);
              atomicAdd(&sstat[1][cg * GR + j], (double)z2[j]);
            }
          }
        }
        __syncthreads();
        continue;
      }
    }
    if (n0 + BN <= g.K && (g.ldy % GR) == 0) {
      for (int idx = tid; idx < BM * GPR; idx += 256) {
        const int row = idx / GPR, cg = idx - (idx / GPR) * GPR;
        const long long m = m0 + row;
        if (m < g.M)
          *reinterpret_cast<uint4*>(Y + m * g.ldy + n0 + cg * GR) =
              *reinterpret_cast<const uint4*>(Cs + row * LC + cg * GR);
      }
    } else {
      for (int idx = tid; idx < BM * BN; idx += 256) {
        const int row = idx / BN, col = idx - (idx / BN) * BN;
        const long long m = m0 + row;
        if (m < g.M && n0 + col < g.K) Y[m * g.ldy + n0 + col] = Cs[row * LC + col];
      }
    }
    __syncthreads();
  }
  if (stats) {
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      stats[((long long)blockIdx.x * 2 + 0) * g.Kp + n0 + c] = sstat[0][c];
      stats[((long long)blockIdx.x * 2 + 1) * g.Kp + n0 + c] = sstat[1][c];
    }
  }
}

// ------------------------------------------------------------------ forward, 3-stage LDS-DMA pipeline
// bf16, C % 64 == 0, K % BN == 0 (every 3x3 / 1x1 / (4,10) layer of both
// networks with >= 64 input channels, and their stride-1 dgrads).
//  * 512 threads = 8 waves as 4 (M) x 2 (N), each 64 pixels x BN/2 channels on
//    v_mfma_f32_16x16x32_bf16; tile 256 pixel rows x BN channels, BK = 64.
//  * Because C % 64 == 0 a K-tile never straddles a filter tap: the tap (r, s)
//    and channel base are wave-uniform scalars, and each lane keeps one bit per
//    filter row / column saying whether its pixel's tap is inside the image, so
//    the im2col address of an LDS-DMA piece is one 64-bit add and one select.
//  * Three LDS stages, one raw barrier per K-tile, two K-tiles in flight across
//    it (counted vmcnt); the stream of K-tiles runs on across M tiles, so the
//    next tile's first two K-tiles are in flight while this tile's epilogue runs.
//  * The MFMA operands are swapped (weights x pixels) so each lane ends with 4
//    consecutive channels of a pixel: the epilogue stores 8-byte rows straight
//    from registers (no LDS staging) and reduces the BatchNormalization sums
//    with a butterfly (reduce-scatter over 16 lanes, 30 shuffles) before one
//    LDS double atomic per value.  Out-of-range pixel rows store to a sink so
//    every wave always issues the same number of stores (vmcnt bookkeeping).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 16-B LDS-DMA with a wave-uniform LDS byte address already in an SGPR.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16_m0(const void* src, unsigned m0v) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0v)
               : "memory", "m0");
}
#pragma clang diagnostic pop


// ACFE_CONV_DBG=8 diagnostic: per-wave cycle totals of the conv main-loop
// segments (top / wait / barrier / issue / compute / epilogue), read back by
// acfe_debug_conv_stamps().  Written only when g.dbg == 8.
__device__ unsigned long long g_conv_stamps[4096 * 8];
ACFE_API int acfe_debug_conv_stamps(unsigned long long* host, int n) {
  if (n > 4096 * 8) n = 4096 * 8;
  return hip_rc(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_conv_stamps), sizeof(unsigned long long) * n), "stamps");
}
struct Stamps {
  unsigned long long acc[6] = {0, 0, 0, 0, 0, 0}, last = 0;
  bool on;
  __device__ explicit Stamps(bool o) : on(o) { if (on) last = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void mark(int i) {
    if (on) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc[i] += t - last;
      last = t;
    }
  }
  __device__ void flush(int wid) {
    if (on && (threadIdx.x & 63) == 0) {
      const int slot = (blockIdx.x * gridDim.y + blockIdx.y) * 8 + wid;
      if (slot < 4096)
        for (int i = 0; i < 6; ++i) g_conv_stamps[slot * 8 + i] = acc[i];
    }
  }
};

__device__ uint2 g_store_sink[64];  // never read: target of masked-off epilogue stores
__device__ u32x4 g_store_sink16[64];  // the same for 16-B stores
__device__ __attribute__((aligned(16))) uint16_t g_store_sink_rows[64 * 64];  // the same, one 128-B row per lane


// RES (acfe_conv2d_fwd_add where the row-halo kernels do not apply, e.g.
// wr_resnet's 256-channel stage 3): z = (ReLU)(conv + g.res) in the epilogue,
// as ops.add stores it, statistics of z; the tile's residual quads are loaded
// two K-tiles before its epilogue
template <int BN, bool S2D = false, bool RES = false>
__global__ void __launch_bounds__(512, 1)
k_conv_fwd_p(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
             const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats, int tiles_m,
             int srows) {
  using T = uint16_t;
  constexpr int BM = 256, BK = 64, NST = 3;
  constexpr int AJ = BM / 64, BJ = BN / 64;  // 8-row LDS-DMA pieces per wave per stage
  constexpr int LPS = AJ + BJ;               // vmcnt entries of one stage, per wave
  constexpr int TWM = 64, TWN = BN / 2, FM = TWM / 16, FN = TWN / 16, KF = 32;
  constexpr int NSTORE = FM * FN;            // epilogue stores per lane per tile
  constexpr int NV = 8 * FN;                 // BN-statistics values per lane (2 x FN x 4)
  constexpr int STG = (BM + BN) * 128;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NST * STG + 2 * BN * 8];
  double* sstat = reinterpret_cast<double*>(smem + NST * STG);  // [2][BN]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int lrow = lane >> 3, gsw = (lane & 7) ^ (lrow & 7);
  const int n0 = blockIdx.y * BN;
  const int nkt = g.Kdp / BK;
  const int PQ = g.P * g.Q, M = (int)g.M;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;
  for (int i = tid; i < 2 * BN; i += 512) sstat[i] = 0.0;
  // bias of this lane's output channels, read before any LDS-DMA is in flight
  float bv[FN][4];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      bv[fn][jj] = bias ? bias[n0 + wn * TWN + fn * 16 + (lane >> 4) * 4 + jj] : 0.f;
  // ---- issue side: runs up to two K-tiles ahead of the compute, across M tiles.
  // A and B pieces are buffer_load ... lds with a wave-uniform descriptor whose
  // base carries the tap / channel offset of the K-tile (SALU only) and a
  // per-row voffset fixed for the tile; an invalid tap selects an
  // out-of-range voffset, which the hardware loads as zeros.
  const TileWalk walk(tiles_m);
  int itm = walk.tm, ikt = 0, ir = 0, is = 0, ic = 0, ibuf = 0, issued = 0;
  const long long padshift = ((long long)g.pt * g.W + g.pl) * g.C * 2;
  long long abase = 0;  // byte address of the tile's first image, shifted back by the padding
  unsigned voffA[AJ], tmlo[AJ], tmhi[AJ];
  unsigned voffB[BJ];
#pragma unroll
  for (int j = 0; j < BJ; ++j) voffB[j] = ((unsigned)(n0 + (wid * BJ + j) * 8 + lrow) * g.Kdp + gsw * 8) * 2u;
  const long long bbase = (long long)(uintptr_t)Wp;
  auto setup = [&](int tm) __attribute__((always_inline)) {
    const int nfirst = (tm * BM) / PQ;
    abase = (long long)(uintptr_t)X + (long long)nfirst * g.H * g.W * g.C * 2 - padshift;
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int m = tm * BM + (wid * AJ + j) * 8 + lrow;
      const bool valid = m < M;
      const int mm = valid ? m : 0;
      const int n = mm / PQ, rem = mm - n * PQ;
      const int p = rem / g.Q, q = rem - p * g.Q;
      const int h0 = p * g.st - g.pt, w0 = q * g.st - g.pl;
      voffA[j] = (unsigned)(((((n - nfirst) * g.H + h0 + g.pt) * g.W + w0 + g.pl) * g.C + gsw * 8) * 2);
      // filter rows / columns whose tap lies inside the image
      const int rlo = h0 < 0 ? -h0 : 0, rhi = g.H - h0 < g.R ? g.H - h0 : g.R;
      const int slo = w0 < 0 ? -w0 : 0, shi = g.W - w0 < g.S ? g.W - w0 : g.S;
      const unsigned hm = (valid && rhi > rlo) ? (((1u << rhi) - 1u) & ~((1u << rlo) - 1u)) : 0u;
      const unsigned long long wmk = shi > slo ? (((1ull << shi) - 1ull) & ~((1ull << slo) - 1ull)) : 0ull;
      unsigned long long t = 0;
      for (int r = 0; r < g.R; ++r)
        if ((hm >> r) & 1u) t |= wmk << (r * g.S);
      tmlo[j] = (unsigned)t;
      tmhi[j] = (unsigned)(t >> 32);
    }
  };
  auto issue = [&]() __attribute__((always_inline)) {
    const unsigned base = lds0 + ibuf * STG + wid * (AJ * 1024);
    const int tap = ir * g.S + is;
    const long long a = abase + ((long long)(ir * g.W + is) * g.C + ic) * 2;
    const i4 da = {(int)(unsigned)a, (int)(unsigned)(a >> 32), (int)0x80000000u, 0x00020000};
    const bool lo = tap < 32;
    const unsigned tw = lo ? tap : tap - 32;
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const unsigned mk = lo ? tmlo[j] : tmhi[j];
      const unsigned vo = ((mk >> tw) & 1u) ? voffA[j] : 0x80000000u;
      bldsx4(vo, da, base + j * 1024);
    }
    const long long bb = bbase + (long long)ikt * BK * 2;
    const i4 db = {(int)(unsigned)bb, (int)(unsigned)(bb >> 32), (int)0x80000000u, 0x00020000};
    const unsigned bbase_l = lds0 + ibuf * STG + BM * 128 + wid * (BJ * 1024);
#pragma unroll
    for (int j = 0; j < BJ; ++j) bldsx4(voffB[j], db, bbase_l + j * 1024);
    ++issued;
    ibuf = ibuf == NST - 1 ? 0 : ibuf + 1;
    ic += BK;
    if (ic == g.C) {
      ic = 0;
      if (++is == g.S) { is = 0; ++ir; }
    }
    if (++ikt == nkt) {
      ikt = ir = is = ic = 0;
      itm += walk.step;
      if (itm < walk.end) setup(itm);
    }
  };

  if (itm < walk.end) {
    setup(itm);
    issue();
    if (itm < walk.end) issue();
  }
  int ctm = walk.tm, ckt = 0, cbuf = 0, done = 0;
  bool pend = false;  // the previous iteration ended a tile: its stores are in the vmcnt queue
  // (letting them stay in flight one step longer, behind the next stage's
  // loads, measured slower: r05s, T1 -0.3 %, wr_resnet -0.7 %)
  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  Stamps stp(g.dbg == 8);
  uint2 rres[RES ? FM : 1][RES ? FN : 1];
  // RES: the residual quads are issued right after the stage issue of K-step
  // rk = nkt - 3, so they have two K-steps to land (at the last K-step's
  // start, r05: the epilogue waited on them, the conv + add 256 -> 256 ran
  // 1.50 ms vs 1.24 ms without the add); the two step-top waits in between
  // leave them in flight (they are younger than the stage being waited for)
  // (reductions of fewer than 3 K-steps: issued before the last K-step's
  // stage, as r05 did)
  constexpr int NRES = FM * FN;
  const bool rearly = nkt >= 3;
  const int rk = rearly ? nkt - 3 : nkt - 1;
  bool rfly = false, rissued = false;
  while (ctm < walk.end) {
    stp.mark(0);
    // stage `done` landed: leave the younger stage (if issued) and stores in flight
    const bool two = issued - done >= 2;
    if (pend) {
      if (two) wait_vmcnt<LPS + NSTORE>();
      else wait_vmcnt<NSTORE>();
    } else if (RES && rfly) {
      if (two) wait_vmcnt<LPS + NRES>();
      else wait_vmcnt<NRES>();
    } else {
      if (two) wait_vmcnt<LPS>();
      else wait_vmcnt<0>();
    }
    stp.mark(1);
    lds_barrier();
    stp.mark(2);
    pend = false;
    auto rload = [&]() __attribute__((always_inline)) {
      const int pb = ctm * BM + wm * TWM + (lane & 15);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int pix = pb + fm * 16, c = n0 + wn * TWN + fn * 16 + (lane >> 4) * 4;
          rres[fm][fn] = *reinterpret_cast<const uint2*>(
              pix < M ? g.res + (long long)pix * g.ldy + c : reinterpret_cast<const uint16_t*>(g_zero_page));
        }
    };
    if constexpr (RES) {
      if (!rearly && ckt == rk) {
        rload();
        rissued = itm < walk.end;
      }
    }
    if (itm < walk.end) issue();
    if constexpr (RES) {
      if (rearly && ckt == rk) {
        rload();
        rfly = true;
      }
    }
    stp.mark(3);
    {
      const unsigned char* Ab = smem + cbuf * STG;
      const unsigned char* Bb = Ab + BM * 128;
#pragma unroll
      for (int kk = 0; kk < BK / KF; ++kk) {
        const int gi = kk * 4 + (lane >> 4);
        uint4 af[FM], bfr[FN];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int row = wn * TWN + fn * 16 + (lane & 15);
          bfr[fn] = *reinterpret_cast<const uint4*>(Bb + row * 128 + ((gi ^ (row & 7)) << 4));
        }
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int row = wm * TWM + fm * 16 + (lane & 15);
          af[fm] = *reinterpret_cast<const uint4*>(Ab + row * 128 + ((gi ^ (row & 7)) << 4));
        }
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) mma(acc[fm][fn], bfr[fn], af[fm], T());
      }
    }
    stp.mark(4);
    cbuf = cbuf == NST - 1 ? 0 : cbuf + 1;
    ++done;
    if (++ckt < nkt) continue;
    // ---- epilogue of tile ctm (acc[fm][fn][jj] = channel (lane>>4)*4+jj of pixel lane&15)
    ckt = 0;
    if constexpr (RES) {
      if (rearly) {  // the residual quads: older than every stage still in flight
        const int younger = issued - done;
        if (younger >= 2) wait_vmcnt<2 * LPS>();
        else if (younger == 1) wait_vmcnt<LPS>();
        else wait_vmcnt<0>();
        rfly = false;
      } else {  // older than the last K-step's stage (if issued)
        if (rissued) wait_vmcnt<LPS>();
        else wait_vmcnt<0>();
      }
    }
    float sv[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) sv[i] = 0.f;
    const int pbase = ctm * BM + wm * TWM + (lane & 15);
    const int c0 = n0 + wn * TWN + (lane >> 4) * 4;  // the lane's first channel (fn = 0)
    // S2D: per fragment column fn, the lane's channel quad c -> block position
    // (a, b) and channel cc (s2d_C a power of two, a = ab * amul >> 5 for the
    // st^2 < 32 positions), as an element offset from the block origin
    int s2a[S2D ? FN : 1], s2b[S2D ? FN : 1], s2o[S2D ? FN : 1];
    if constexpr (S2D) {
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int c = c0 + fn * 16;
        const int ab = g.s2d_fill ? 0 : c >> g.s2d_lc, cc = c & (g.s2d_C - 1);
        const int a = (ab * g.s2d_amul) >> 5, b = ab - a * g.s2d;
        s2a[fn] = a;
        s2b[fn] = c < g.K ? b : -(1 << 20);  // (past K: never stored)
        s2o[fn] = (a * g.s2d_W + b) * g.s2d_C + cc;
      }
    }
    // The tile's values as bf16 words (two channels each, pk_bf2 = f2bf's
    // rounding), Dropout by acfe_dropout's pair hashes -- one per channel pair,
    // from a Weyl term advanced by constants when every index is < 2^32 (the
    // per-element 64-bit hash cost 4 quarter-rate multiplies per value, r06l)
    // -- then the residual add, the statistics of the stored values and one
    // 8-byte store per fragment through a per-row pointer (fn: immediate offset).
    auto epi = [&](auto drop_c) __attribute__((always_inline)) {
      constexpr bool DROP = decltype(drop_c)::value;
      const bool w32 = DROP && g.idx32;
      const uint32_t hwl = (((uint32_t)pbase * (uint32_t)g.K + (uint32_t)c0) >> 1) * 0x9E3779B1u +
                           (uint32_t)g.drop.seed;
      const uint32_t hwm = (uint32_t)(8 * g.K) * 0x9E3779B1u;  // + 16 pixels (pair index + 8 K)
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int pix = pbase + fm * 16;
        const bool inb = pix < M;
        // super-pixel store (g.s2d): this pixel's dX block origin (sn, sh, sw),
        // the divisions by P Q and Q through a float reciprocal (pix < 2^24) and
        // one correction step
        int sh = 0, sw = 0;
        long long sbase = 0;
        if constexpr (S2D) {
          const int pp = inb ? pix : 0;
          int sn = (int)((float)pp * g.s2d_rpq);
          sn -= sn * PQ > pp ? 1 : 0;
          sn += (sn + 1) * PQ <= pp ? 1 : 0;
          const int rem = pp - sn * PQ;
          int u = (int)((float)rem * g.s2d_rq);
          u -= u * g.Q > rem ? 1 : 0;
          u += (u + 1) * g.Q <= rem ? 1 : 0;
          sh = u * g.s2d - g.s2d_pt;
          sw = (rem - u * g.Q) * g.s2d - g.s2d_pl;
          sbase = (((long long)sn * g.s2d_H + sh) * g.s2d_W + sw) * g.s2d_C;
        }
        uint16_t* rowp = inb ? Y + (long long)pix * g.ldy + c0 : g_store_sink_rows + lane * 64;
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          unsigned wv[2];
#pragma unroll
          for (int p = 0; p < 2; ++p)
            wv[p] = pk_bf2(acc[fm][fn][2 * p] + bv[fn][2 * p], acc[fm][fn][2 * p + 1] + bv[fn][2 * p + 1]);
          if constexpr (DROP) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
              const uint32_t hsh =
                  w32 ? hash_u32_lo_w(g.drop.seed, hwl + (uint32_t)fm * hwm + (uint32_t)(8 * fn + p) * 0x9E3779B1u)
                      : hash_u32(g.drop.seed, ((uint64_t)pix * g.K + c0 + fn * 16 + 2 * p) >> 1);
              const bool klo = (hsh & 0xFFFFu) >= g.drop.thr, khi = (hsh >> 16) >= g.drop.thr;
              const float lo = klo ? bf2f(f2bf(__uint_as_float(wv[p] << 16) * g.drop.scl)) : 0.f;
              const float hi = khi ? bf2f(f2bf(__uint_as_float(wv[p] & 0xffff0000u) * g.drop.scl)) : 0.f;
              wv[p] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
            }
          }
          if constexpr (RES) {
            const unsigned rw[2] = {rres[fm][fn].x, rres[fm][fn].y};
#pragma unroll
            for (int p = 0; p < 2; ++p) {
              float lo = __uint_as_float(wv[p] << 16) + __uint_as_float(rw[p] << 16);
              float hi = __uint_as_float(wv[p] & 0xffff0000u) + __uint_as_float(rw[p] & 0xffff0000u);
              if (g.res_relu) lo = fmaxf(lo, 0.f), hi = fmaxf(hi, 0.f);
              wv[p] = pk_bf2(lo, hi);
            }
          }
          if constexpr (!S2D) {  // (the dgrad has no statistics)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const unsigned w = wv[jj >> 1];
              const float f = inb ? __uint_as_float((jj & 1) ? (w & 0xffff0000u) : (w << 16)) : 0.f;
              sv[fn * 4 + jj] += f;
              sv[FN * 4 + fn * 4 + jj] += f * f;
            }
          }
          uint2 v;
          v.x = wv[0];
          v.y = wv[1];
          uint2* dst = reinterpret_cast<uint2*>(rowp + fn * 16);
          if constexpr (S2D) {
            dst = (inb && (unsigned)(sh + s2a[fn]) < (unsigned)g.s2d_H && (unsigned)(sw + s2b[fn]) < (unsigned)g.s2d_W)
                      ? reinterpret_cast<uint2*>(Y + sbase + s2o[fn])
                      : &g_store_sink[lane];
          }
          *dst = v;
          acc[fm][fn] = f4{0.f, 0.f, 0.f, 0.f};
        }
      }
    };
    if (g.drop.on) epi(std::true_type{});
    else epi(std::false_type{});
    pend = true;
    if (stats) {
      // butterfly reduce-scatter over the 16 lanes of equal lane>>4, partners
      // by DPP (no LDS traffic): row_ror:8 pairs bit 3, row_half_mirror pairs
      // bit 2 (keeping bit 3), quad_perm xor-2 / xor-1 pair bits 1 / 0
      butterfly_step<NV, 8, 0x128>(sv, lane);
      butterfly_step<NV / 2, 4, 0x141>(sv, lane);
      butterfly_step<NV / 4, 2, 0x4E>(sv, lane);
      butterfly_step<NV / 8, 1, 0xB1>(sv, lane);
      const int l4 = lane & 15;
      const int b0 = ((l4 >> 3) & 1) * (NV / 2) + ((l4 >> 2) & 1) * (NV / 4) + ((l4 >> 1) & 1) * (NV / 8) +
                     (l4 & 1) * (NV / 16);
#pragma unroll
      for (int k = 0; k < NV / 16; ++k) {
        const int idx = b0 + k, st = idx / (FN * 4), rm = idx - st * (FN * 4);
        const int col = wn * TWN + (rm >> 2) * 16 + (lane >> 4) * 4 + (rm & 3);
        atomicAdd(&sstat[st * BN + col], (double)sv[k]);
      }
    }
    ctm += walk.step;
    stp.mark(5);
  }
  stp.flush(wid);
  wait_vmcnt<0>();
  lds_barrier();
  if (stats) {
    for (int c = tid; c < BN; c += 512) {
      stats[((long long)blockIdx.x * 2 + 0) * g.Kp + n0 + c] = sstat[c];
      stats[((long long)blockIdx.x * 2 + 1) * g.Kp + n0 + c] = sstat[BN + c];
    }
    // the persistent grid is smaller than acfe_conv2d_stats_rows(): zero the rest
    for (int rr = blockIdx.x + gridDim.x; rr < srows; rr += gridDim.x)
      for (int c = tid; c < 2 * BN; c += 512) stats[((long long)rr * 2 + (c / BN)) * g.Kp + n0 + (c % BN)] = 0.0;
  }
}

// ------------------------------------------------------------------ 3x3 stride-1 conv, row-halo steps
// Forward (and stride-1 dgrad) of the 3x3 layers with C % 64 == 0,
// K in {64, 128} (a partial last 64-pixel column tile is masked: wr_resnet's
// 513- / 257-wide stages).  Built like k_wgrad3x3_halo, whose measured
// lesson is that each pipeline step carries a fixed ~1 us of non-MFMA time,
// so the matrix work per step has to be large: a workgroup owns 3 output rows
// x 64 pixels x K channels, and one step = one 64-channel chunk x one filter
// row r (three taps): the 3 input rows (h0 + i + r - pt) x 66 pixels and the
// weights W[k][r][0..2][chunk] are staged in LDS once (register-staged double
// buffer, one barrier per step) and feed 72 MFMAs per wave (vs 32 per K-tile
// in k_conv_fwd_p).  Input rows are 144-B padded (16 consecutive pixels of a
// fragment read hit distinct banks at any tap shift); weight rows are 128 B
// with the k & 7 XOR swizzle.  Operands swapped (weights x pixels) so the
// epilogue is k_conv_fwd_p's: 8-byte channel quads straight from registers,
// bias gathered by ds_bpermute, fused Dropout, DPP-butterfly BatchNormalization
// sums.  XRES (K = 128: 4 rows, K = 64: 6 rows) stages the TR + 2 halo rows of
// a chunk once for its three filter-row steps (see the XROWS comment below).
// PM (epilogue mode): 0 plain; 4 = plain + Dropout (its own instantiation:
// the dropout epilogue's registers would spill the K = 128 dgrad); 3 = z = (ReLU)(conv + residual g.res) as
// ops.add stores it, BN sums of z; 1 = the output feeds MaxPool2D(2, 2) -> Dropout:
// the epilogue pools row pairs x column pairs (waves own 16-column strips of
// all TR rows), stores only the pooled values, their first-maximum argmax byte
// (amax) and their BN statistics; 2 = dgrad whose dY is the 2x2 max-pool
// backward of X = the pooled gradient with argmax bytes amax (expanded while
// staging, the full-resolution dY is never stored).
template <int KB, int TR, int PM, bool XRES = false, bool PRO = false>
__global__ void __launch_bounds__(512, 1)
k_conv3x3_rows(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
               const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats, int tiles_h,
               int tiles_w, int ntiles, int srows, uint8_t* __restrict__ amax) {
  static_assert(PM != 1 || TR % 2 == 0, "2x2 pooling needs row pairs");
  using T = uint16_t;
  // PM 1 with the MFMA operands in pixels x weights order: each A row block
  // of four rows is one 2x2 window, so a lane's four accumulators are a whole
  // window of one channel and the pooling needs no cross-lane traffic
  constexpr bool SWP = PM == 1;
  // CPERM (weights x pixels epilogues with the weight DMA): fragment fn, A row
  // m = output channel KB/2 wk + 4 FN (m >> 2) + 4 fn + (m & 3), so lane group
  // q = lane >> 4 holds 4 FN consecutive channels of its pixel across the FN
  // fragments and the epilogue stores them with FN / 2 16-B stores (not FN
  // 8-B ones); weight LDS rows keep 128 B with the granule swizzle
  // swzp(k) = ((k >> LQ) & 3) << 1 | ((k >> 1) & 1), which keeps the fragment
  // reads conflict-free under the permuted rows
  constexpr bool CPERM = !SWP && TR > 3;
  constexpr int LQ = KB == 128 ? 4 : 3;  // log2(4 FN), FN = KB / 32
  constexpr int FN = KB / 32, FM = TR;                           // per wave: KB/2 channels x TR*16 pixels
  // 6-row tiles: weights by LDS-DMA into a double buffer (no staging VGPRs,
  // which spilled at K = 128), input rows register-staged.  LDS buffers of the
  // input image: two (the next step's rows are stored right after this step's
  // MFMAs, one barrier per step) where they fit -- K = 64 and the 3-row tiles --,
  // else one (stored between two barriers, the MFMA pipe idle meanwhile).
  constexpr bool WDMA = TR > 3;
  // XRES: the TR + 2 halo rows of a 64-channel chunk are staged once and serve
  // its three filter-row steps (single buffer, restaged between two barriers
  // once per chunk instead of once per step: a third of the LDS stores and of
  // the input reads); the steps in between only wait for their weight pieces
  constexpr int XROWS = XRES ? TR + 2 : TR;
  constexpr int NBUF = XRES ? 1 : (TR <= 3 || KB == 64) ? 2 : 1;
  static_assert(!XRES || WDMA, "XRES needs the weight DMA");
  // PRO: the BatchNormalization (+ReLU) prologue on the staged input (C <= 256)
  static_assert(!PRO || (XRES && PM != 2), "prologue: chunk-resident forward");
  // pixels per row, halo row bytes: 160-B rows make the fragment reads
  // conflict-free under ds_read_b128's lane grouping at every tap shift (144-B
  // rows had 2-way conflicts: a third of the LDS cycles, rocprofv3 r02c); the
  // double-buffered K = 64 image only fits with 144-B rows
  // 160-B pixel pitch wherever the LDS allows it (conflict-free fragment reads);
  // 144 B only for the 6-row K = 64 double buffer (37 % of its LDS cycles are
  // bank conflicts, SQ counters r02z; the conflict-free 5-row variant,
  // ACFE_ROWS64_TR=5, measured the same: those kernels are not LDS-bound)
  constexpr int SEGW = 64, HWX = SEGW + 2;
  constexpr int WB_ = 3 * KB * 128;
  constexpr int SMEM160 = (WDMA ? NBUF * XROWS * HWX * 160 + 2 * WB_ : NBUF * (XROWS * HWX * 160 + WB_)) +
                          (KB == 64 ? 0 : 2 * KB * 8);
  constexpr int XRB = SMEM160 <= 163840 ? 160 : 144;
  constexpr int NV = 8 * FN;
  constexpr int XBYTES = XROWS * HWX * XRB, WBYTES = 3 * KB * 128, BUFB = XBYTES + WBYTES;
  constexpr int XG = XROWS * HWX * 8, WG = 3 * KB * 8;          // 16-B granules per step
  constexpr int XPT = (XG + 511) / 512, WPT = WG / 512;
  static_assert(WG % 512 == 0, "weight granules per thread");
  // WDMA layout [X0 (X1)][W0][W1]; else [X0 W0][X1 W1]
  constexpr int WBASE = WDMA ? NBUF * XBYTES : XBYTES;
  constexpr int SMEM0 = WDMA ? NBUF * XBYTES + 2 * WBYTES : NBUF * BUFB;
  // BN sums: K = 64 (LDS full with the double buffer) keeps per-lane double
  // partials in registers, reduced over the waves once at the end; K = 128 (at
  // the register limit) accumulates them with LDS double atomics per tile
  constexpr bool REGSTAT = KB == 64;
  constexpr int SMEMS = SMEM0 + (REGSTAT ? 0 : 2 * KB * 8);
  // PM 5: the BN backward coefficient table [scale | shift | mean | invstd][KB]
  static_assert(PM != 5 || (KB == 64 && CPERM && !PRO), "PM 5: the K = 64 dgrad");
  constexpr int SMEMB = SMEMS + (PRO ? 2 * 256 * 4 : 0);
  constexpr int SMEM = SMEMB + (PM == 5 ? 4 * KB * 4 : 0);
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  double* sstat = reinterpret_cast<double*>(smem + SMEM0);
  float* pss = reinterpret_cast<float*>(smem + SMEMS);  // PRO: scale[256], shift[256]
  float* bnt = reinterpret_cast<float*>(smem + SMEMB);  // PM 5
  auto xbuf = [&](int b) __attribute__((always_inline)) { return smem + (WDMA ? b * XBYTES : b * BUFB); };
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wid >> 2, wp = wid & 3;
  const int nch = g.C / 64, nsteps_t = nch * 3;
  const int tpi = tiles_h * tiles_w;
  const T* zp = reinterpret_cast<const T*>(g_zero_page);
  constexpr int NV16 = 8 * FN / 16;
  double dstat[REGSTAT ? NV16 : 1];
#pragma unroll
  for (int k = 0; k < (REGSTAT ? NV16 : 1); ++k) dstat[k] = 0.0;
  if constexpr (!REGSTAT)
    for (int i = tid; i < 2 * KB; i += 512) sstat[i] = 0.0;
  if constexpr (PRO)
    for (int i = tid; i < g.C; i += 512) pss[i] = g.pro_sc[i], pss[256 + i] = g.pro_sh[i];
  if constexpr (PM == 5)  // (read only by the epilogues, after the main loop's first barrier)
    for (int i = tid; i < KB; i += 512)
      bnt[i] = g.bn_sc[i], bnt[KB + i] = g.bn_sh[i], bnt[2 * KB + i] = g.bn_mu[i], bnt[3 * KB + i] = g.bn_is[i];
  // bias: lane l holds channel wk * KB/2 + (l mod KB/2), one VGPR across the
  // main loop (the K = 128 variants sit at the 256-VGPR limit; no LDS left for
  // a copy); each epilogue gathers its quads with ds_bpermute, once per
  // fragment column (a global f4 load per fragment waited on its full L2
  // latency twelve times per tile)
  const float blane = (bias && PM != 2) ? bias[wk * (KB / 2) + (lane & (KB / 2 - 1))] : 0.f;
  const TileWalk walk(ntiles);
  const int ntl = walk.tm < walk.end ? (walk.end - walk.tm + walk.step - 1) / walk.step : 0;
  const int L = ntl * nsteps_t;

  // ---- global -> register staging of step t (tile, chunk, filter row)
  u32x4 rx[XPT], rw[WDMA ? 1 : WPT];
  // PM 2: argmax bytes and window taps of the staged granules, applied at the
  // LDS store (after the MFMAs) so the loads stay in flight during the step
  uint2 ra[PM == 2 ? XPT : 1];
  unsigned rpos = 0;
  // WDMA: piece j of this wave = 8 weight rows (s*KB + k) of 128 B, granule
  // slot (lane & 7) holds global granule slot ^ (row & 7) (source-side swizzle)
  constexpr int WPW = WG / 64 / 8;  // pieces per wave per step
  // Weight pieces.  non-SWP: LDS rows [s][k] of 128 B (one tap's 64-channel
  // chunk), granule slot = granule ^ (k & 7); piece j = rows R0 + l8,
  // R0 = (wid WPW + j) 8, l8 = lane >> 3, slot = lane & 7.
  // SWP: rows [kk][s][phys(k)] of 64 B (channel half kk of the chunk), slot =
  // granule ^ f(k); with the lane's fragment rows k = base + FN l16 + fn,
  // phys(k) & 3 = fn ^ (l16 & 3) (FN 4; FN 2: k bit 2 into bit 0) and
  // f = (l16 >> 2) & 2 place every ds_read_b128 lane group on 16 distinct
  // 16-B bank slots, and kk / s are immediate offsets of the read; piece j =
  // rows R0 + l, R0 = (wid WPW + j) 16, l = lane >> 2, slot = lane & 3.
  // The lane-dependent part of a piece's source offset is one VGPR (vwl); the
  // rest (its first row, tap, channel half and swizzle) is wave-uniform.
  constexpr int LGB = FN == 4 ? 3 : 1;  // SWP: phys(k) = k ^ ((k >> 2) & LGB)
  // piece j: wave-uniform source byte offset (its first row, tap, channel
  // half) and the lane's SWP swizzle term
  auto piece_so = [&](int j) __attribute__((always_inline)) {
    if constexpr (SWP) {
      const int R0 = (wid * WPW + j) * 16, kh = R0 / (3 * KB), rr = R0 - kh * 3 * KB;
      const int s_ = rr / KB, kb = rr - s_ * KB;
      return (unsigned)((kb * g.Kdp + s_ * g.C + kh * 32) * 2);
    } else {
      const int R0 = (wid * WPW + j) * 8, s_ = R0 / KB, kb = R0 - s_ * KB;
      return (unsigned)((kb * g.Kdp + s_ * g.C) * 2);
    }
  };
  auto piece_vx = [&](int j) __attribute__((always_inline)) {
    if constexpr (SWP) {
      const int R0 = (wid * WPW + j) * 16, kb = R0 % KB;
      const unsigned fu = (unsigned)((((kb % (KB / 2)) / FN) >> 2) & 2);  // f of the piece's rows
      return (((unsigned)lane & 3u) ^ fu) << 4;
    } else {
      return 0u;
    }
  };
  // VOFF: each piece's full source offset held in a VGPR (no per-step
  // scalar offset arithmetic); the 6-row K = 128 tiles, at the VGPR limit,
  // keep one VGPR and form the rest in soffset
  constexpr bool VOFF = !(KB == 128 && TR == 6) || CPERM;
  // MFMA groups (of 6) that carry the next step's weight pieces (r02ak same-box
  // A/B: 6 -> fwd_pool 4.61 ms, 3 -> 4.73, 2 -> 4.61); K = 64: the iglp_opt(0)
  // interleave is better without the pieces between the groups (r02ap)
  constexpr int WGRP = 6;
  constexpr bool WILV = WDMA && KB == 128;
  unsigned vwo[VOFF ? WPW : 1];
  unsigned vwl = 0;
  if constexpr (WDMA) {
    if constexpr (SWP) {
      const int l = lane >> 2;
      vwl = (unsigned)((l ^ ((l >> 2) & LGB)) * g.Kdp * 2);
    } else {
      const int l8 = lane >> 3;
      vwl = (unsigned)(l8 * g.Kdp * 2 + (((lane & 7) ^ l8) << 4));
    }
    if constexpr (VOFF) {
#pragma unroll
      for (int j = 0; j < WPW; ++j) {
        if constexpr (CPERM) {
          const int R0 = (wid * WPW + j) * 8, s_ = R0 / KB, k = R0 - s_ * KB + (lane >> 3);
          const int sw = (((k >> LQ) & 3) << 1) | ((k >> 1) & 1);
          vwo[j] = (unsigned)((k * g.Kdp + s_ * g.C + (((lane & 7) ^ sw) << 3)) * 2);
        } else {
          vwo[j] = vwl + piece_so(j) + piece_vx(j);
        }
      }
    }
  }
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;
  // weight pieces of step st into buffer wb: descriptor + LDS base, then the
  // pieces (all at once, or one by one between the MFMA groups: WILV)
  i4 wdw = {0, 0, 0, 0};
  unsigned wlb = 0;
  auto wprep = [&](int st, int wb) __attribute__((always_inline)) {
    const int cc = st / 3, r = st - cc * 3;
    const long long base = (long long)(uintptr_t)Wp + ((long long)r * 3 * g.C + cc * 64) * 2;
    wdw = i4{(int)(unsigned)base, (int)(unsigned)(base >> 32), (int)0x80000000u, 0x00020000};
    wlb = lds0 + WBASE + wb * WBYTES + wid * WPW * 1024;
  };
  auto wpiece = [&](int j) __attribute__((always_inline)) {
    // (wave-uniform; readfirstlane keeps them in SGPRs when the piece is
    // issued from inside the MFMA groups)
    const i4 dw = {__builtin_amdgcn_readfirstlane(wdw[0]), __builtin_amdgcn_readfirstlane(wdw[1]),
                   __builtin_amdgcn_readfirstlane(wdw[2]), __builtin_amdgcn_readfirstlane(wdw[3])};
    const unsigned lb = (unsigned)__builtin_amdgcn_readfirstlane((int)(wlb + j * 1024));
    if constexpr (VOFF) bldsx4(vwo[j], dw, lb);
    else bldsx4s(vwl + piece_vx(j), dw, piece_so(j), lb);
  };
  auto wdma = [&](int st, int wb) __attribute__((always_inline)) {
    wprep(st, wb);
#pragma unroll
    for (int j = 0; j < (WDMA ? WPW : 0); ++j) wpiece(j);
  };
  // Input staging without per-step address arithmetic: granule i of this
  // thread is halo row xrow[i], halo pixel xpix[i], 16-B channel slot gr of the
  // 64-channel chunk -- fixed for the whole kernel.  When the staged tile
  // changes, each granule's byte offset inside its image (filter row 0, chunk
  // 0) and a 3-bit mask of the filter rows r for which it lies inside the image
  // are computed once; a step then adds the wave-uniform (r, chunk) delta and
  // selects an out-of-range offset for masked granules, whose buffer loads
  // return zeros (no branches, no 64-bit math).
  const int gr = tid & 7;
  // PM 2 (K = 128 sits at the register limit with the argmax bytes in flight)
  // keeps no per-granule state: its offsets are recomputed per step from the
  // wave-uniform tile origin (sh0, sw0)
  int xoffs[PM == 2 ? 1 : XPT];
  int sh0 = 0, sw0 = 0;       // PM 2: input row / column of halo pixel (0, 0) at filter row 0 (wave-uniform)
  // mask bits per granule: filter rows 0..2 inside the image (XRES: row 0
  // only; PRO: + the granule is one of the tile's own pixels, stored to pro_out)
  constexpr int MB = XRES ? (PRO ? 2 : 1) : 4;
  static_assert(MB * XPT <= 32, "granule mask bits");
  unsigned xm = 0;
  int stl = -1;  // walk index of the tile the offsets belong to
  long long pimg = 0;  // PRO: byte offset of the staged tile's image
  __amdgpu_buffer_rsrc_t xrs, ars;
  const int CB = g.C * 2;  // bytes per pixel
  auto stage_tile = [&](int tl) __attribute__((always_inline)) {
    const int tm = walk.tm + tl * walk.step;
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
    const int h0 = hb * TR - g.pt, w0 = wb * SEGW - g.pl;
    sh0 = h0;
    sw0 = w0;
    if constexpr (PM == 2) {
      // X = pooled gradient [N][H/2][W/2][C], amax its argmax bytes
      const long long img = (long long)n * (g.H >> 1) * (g.W >> 1) * g.C;
      const int nb = (g.H >> 1) * (g.W >> 1) * g.C;
      xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + img), (short)0, nb * 2, 0x00020000);
      ars = __builtin_amdgcn_make_buffer_rsrc((void*)(amax + img), (short)0, nb, 0x00020000);
    } else {
      const long long img = (long long)n * g.H * g.W * g.C;
      xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + img), (short)0, g.H * g.W * CB, 0x00020000);
      pimg = img * 2;
    }
    xm = 0;
#pragma unroll
    for (int i = 0; i < (PM == 2 ? 0 : XPT); ++i) {
      const int idx = tid + 512 * i;
      const int xrow = idx / (HWX * 8), xpix = (idx - xrow * (HWX * 8)) >> 3;
      const int hin = h0 + xrow, win = w0 + xpix;
      const bool ok = idx < XG && (unsigned)win < (unsigned)g.W;
      unsigned m = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) m |= ((unsigned)(hin + r) < (unsigned)g.H ? 1u : 0u) << r;
      m = ok ? m : 0u;
      xoffs[i] = (hin * g.W + win) * CB + gr * 16;
      unsigned mm = XRES ? m & 1u : m;
      if constexpr (PRO) {
        const bool own = xrow >= 1 && xrow <= TR && xpix >= 1 && xpix <= SEGW;
        mm |= (own && (m & 1u)) ? 2u : 0u;
      }
      xm |= mm << (MB * i);
    }
  };
  auto gload = [&](int tl, int st) __attribute__((always_inline)) {
    const int cc = st / 3, r = XRES ? 0 : st - cc * 3;
    if (tl != stl) {
      stage_tile(tl);
      stl = tl;
    }
    if constexpr (PM == 2) {
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int idx = tid + 512 * i;
        const int xrow = idx / (HWX * 8), xpix = (idx - xrow * (HWX * 8)) >> 3;
        const int hin = sh0 + xrow + r, win = sw0 + xpix;
        const bool ok = idx < XG && (unsigned)hin < (unsigned)g.H && (unsigned)win < (unsigned)g.W;
        const int e = ((hin >> 1) * (g.W >> 1) + (win >> 1)) * g.C + gr * 8 + cc * 64;
        rx[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, ok ? e * 2 : 0x80000000, 0, 0);
        const auto a8 = __builtin_amdgcn_raw_buffer_load_b64(ars, ok ? e : 0x80000000, 0, 0);
        ra[i] = uint2{a8[0], a8[1]};
        if (i == 0) rpos = 0;
        rpos |= (((unsigned)(hin & 1) << 1) | ((unsigned)win & 1u)) << (2 * i);
      }
    } else {
      const int delta = r * g.W * CB + cc * 128;
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const bool ok = (xm >> (MB * i + r)) & 1u;
        rx[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, ok ? xoffs[i] + delta : 0x80000000, 0, 0);
      }
    }
    if constexpr (!WDMA) {
#pragma unroll
      for (int i = 0; i < WPT; ++i) {
        const int idx = tid + 512 * i;
        const int s = idx / (KB * 8), r2 = idx - s * (KB * 8), k = r2 >> 3, gw = r2 & 7;
        rw[i] = *reinterpret_cast<const u32x4*>(Wp + (long long)k * g.Kdp + (r * 3 + s) * g.C + cc * 64 + gw * 8);
      }
    }
  };
  // LDS image slot of granule i: halo pixel (tid >> 3) + 64 i, channel slot gr
  const int xsto = (tid >> 3) * XRB + gr * 16;
  auto sstore = [&](int buf) __attribute__((always_inline)) {
    unsigned char* Xl = xbuf(buf);
    unsigned char* Wl = Xl + XBYTES;  // (register-staged weights: non-WDMA layout)
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 512 * i;
      if constexpr (PM == 2) {
        if (idx < XG)
          *reinterpret_cast<u32x4*>(Xl + xsto + i * 64 * XRB) = rx[i] & unpool_mask(ra[i], (rpos >> (2 * i)) & 3u);
      } else {
        if (idx < XG) *reinterpret_cast<u32x4*>(Xl + xsto + i * 64 * XRB) = rx[i];
      }
    }
    if constexpr (!WDMA) {
#pragma unroll
      for (int i = 0; i < WPT; ++i) {
        const int idx = tid + 512 * i;
        const int row = idx >> 3, gw = idx & 7;  // row = s * KB + k
        *reinterpret_cast<u32x4*>(Wl + row * 128 + ((gw ^ (row & 7)) << 4)) = rw[i];
      }
    }
  };
  // PRO: rx (chunk cc of the staged tile) -> (ReLU)(x * scale + shift) in
  // bf16 (FMA, max, round to nearest even: acfe_bn_apply's values), zero for
  // granules outside the image (the conv's padding is applied after the BN);
  // the tile's own pixels also go to pro_out
  auto xform = [&](int cc) __attribute__((always_inline)) {
    if constexpr (PRO) {
      typedef float f2v __attribute__((ext_vector_type(2)));
      typedef __bf16 b2v __attribute__((ext_vector_type(2)));
      const f4* ps = reinterpret_cast<const f4*>(pss + cc * 64 + gr * 8);
      const f4 sc0 = ps[0], sc1 = ps[1], sh0 = ps[64], sh1 = ps[65];
      const float scv[8] = {sc0[0], sc0[1], sc0[2], sc0[3], sc1[0], sc1[1], sc1[2], sc1[3]};
      const float shv[8] = {sh0[0], sh0[1], sh0[2], sh0[3], sh1[0], sh1[1], sh1[2], sh1[3]};
      const bool relu = g.pro_relu != 0;
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        u32x4 v = rx[i];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          float lo = __builtin_fmaf(__uint_as_float(v[d] << 16), scv[2 * d], shv[2 * d]);
          float hi = __builtin_fmaf(__uint_as_float(v[d] & 0xffff0000u), scv[2 * d + 1], shv[2 * d + 1]);
          if (relu) {
            lo = fmaxf(lo, 0.f);
            hi = fmaxf(hi, 0.f);
          }
          const b2v pk = __builtin_convertvector((f2v){lo, hi}, b2v);
          v[d] = __builtin_bit_cast(unsigned, pk);
        }
        const bool in = (xm >> (MB * i)) & 1u;
        rx[i] = in ? v : u32x4{0u, 0u, 0u, 0u};
        if (g.pro_out && ((xm >> (MB * i + 1)) & 1u))
          *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(g.pro_out) + pimg + xoffs[i] + cc * 128) = v;
      }
    }
  };

  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // this wave's three 16-pixel fragments: tile pixel wp*48 + fm*16 + l16 = (row, col)
  int xoff[FM];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    // PM 1: wave wp owns columns wp*16.. of every row (fragment fm = row fm) so
    // each lane holds both rows of its 2x2 windows
    const int p = PM == 1 ? fm * SEGW + wp * 16 : wp * (TR * 16) + fm * 16;
    xoff[fm] = ((p / SEGW) * HWX + (p % SEGW) + l16) * XRB + (lane >> 4) * 16;
    if constexpr (SWP) {
      // A row m = 4q + j: window q of fragment fm (row pair fm / 2, pooled
      // column wp*8 + (fm & 1)*4 + (q ^ (q >> 1)): windows q and q ^ 3 share a
      // ds_read_b128 lane group and sit two pooled columns apart, which makes
      // the 16 lanes of every group hit 16 distinct 16-B bank slots at the
      // 160-B pitch), pixel j = (dy, dx) of the window
      const int q = l16 >> 2, j = l16 & 3;
      const int a = wp * 8 + (fm & 1) * 4 + (q ^ (q >> 1));
      xoff[fm] = (((fm >> 1) * 2 + (j >> 1)) * HWX + 2 * a + (j & 1)) * XRB + (lane >> 4) * 16;
    }
  }
  // weight fragment fn, column l16 = output channel woff[fn]; SWP: FN
  // consecutive channels per lane (a lane's pooled window covers channels
  // wk * KB/2 + FN * l16 + [0, FN)), woffp = that row's LDS row, wsw its
  // granule swizzle
  // wrb[fn]: byte offset of this lane's weight fragment fn in the weight
  // buffer (non-SWP: of kk = 0 in tap 0; kk = 1 flips bit 6 -- granule
  // kk * 4 + hi, hi < 4, XOR the swizzle; SWP: in [kk = 0][s = 0])
  int wrb[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    if constexpr (SWP) {
      const int k = wk * (KB / 2) + FN * l16 + fn;
      wrb[fn] = (k ^ ((k >> 2) & LGB)) * 64 + (((lane >> 4) ^ ((l16 >> 2) & 2)) << 4);
    } else if constexpr (CPERM) {
      const int k = wk * (KB / 2) + (l16 >> 2) * 4 * FN + fn * 4 + (l16 & 3);
      const int sw = (((k >> LQ) & 3) << 1) | ((k >> 1) & 1);
      wrb[fn] = k * 128 + (((lane >> 4) ^ sw) << 4);
    } else {
      const int k = wk * (KB / 2) + fn * 16 + l16;
      wrb[fn] = k * 128 + (((lane >> 4) ^ (k & 7)) << 4);
    }
  }

  // PM 3 with K = 64: the tile's residual quads are loaded at the start of its
  // last step (in flight during that step's MFMAs) instead of in the epilogue
  constexpr bool RPRE = PM == 3 && KB == 64 && FM <= 6;  // (8 rows: its registers spill)
  uint2 rres[RPRE ? FM : 1][RPRE ? FN : 1];
  auto rload = [&](int tm) __attribute__((always_inline)) {
    if constexpr (RPRE) {
      const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int p = wp * (TR * 16) + fm * 16;
        const int h = hb * TR + p / SEGW, w = wb * SEGW + (p % SEGW) + l16;
        const bool inb = h < g.P && w < g.Q;
        const long long pix = ((long long)n * g.P + h) * g.Q + w;
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int c = wk * (KB / 2) + (CPERM ? (lane >> 4) * 4 * FN + fn * 4 : fn * 16 + (lane >> 4) * 4);
          rres[fm][fn] = *reinterpret_cast<const uint2*>(inb ? g.res + pix * g.ldy + c : zp);
        }
      }
    }
  };
  // PM 5: the BN input x at the tile's pixels (the lane's 4 FN = 8 channels of
  // each fragment row: one 16-B load), requested at the start of the epilogue
  // (prefetched during the tile's last step, its 32 VGPRs spilled 163)
  u32x4 xbn[PM == 5 ? FM : 1];
  // (buffer loads of the tile's image, out-of-image pixels at an
  // out-of-range offset: no branches; one image < 2^31 bytes, launcher)
  auto xbn_load = [&](int tm) __attribute__((always_inline)) {
    if constexpr (PM == 5) {
      const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
      const int cq = wk * (KB / 2) + (lane >> 4) * 4 * FN;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(g.res + (long long)n * g.P * g.Q * g.ldy), (short)0, g.P * g.Q * g.ldy * 2, 0x00020000);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int p = wp * (TR * 16) + fm * 16;
        const int h = hb * TR + p / SEGW, w = wb * SEGW + (p % SEGW) + l16;
        const bool inb = (h < g.P) & (w < g.Q);
        const unsigned o = ((unsigned)(h * g.Q + w) * (unsigned)g.ldy + cq) * 2u;
        xbn[fm] = __builtin_amdgcn_raw_buffer_load_b128(rr, inb ? o : 0x80000000u, 0, 0);
      }
    }
  };
  auto epilogue = [&](int tm) __attribute__((always_inline)) {
    xbn_load(tm);
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
    float sv[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) sv[i] = 0.f;
    // bias quad of fragment column fn (PM 2, the dgrad, has none)
    auto bias4 = [&](int fn) __attribute__((always_inline)) {
      f4 r = {0.f, 0.f, 0.f, 0.f};
      if constexpr (PM != 2) {
        const int src = CPERM ? (lane >> 4) * 4 * FN + fn * 4 : fn * 16 + (lane >> 4) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          r[j] = __int_as_float(__builtin_amdgcn_ds_bpermute((src + j) * 4, __float_as_int(blane)));
      }
      return r;
    };
    if constexpr (SWP) {
      // lane = (window q = lane >> 4 of each fragment, channels cf + [0, FN));
      // accumulator j of fragment fm = pixel (dy, dx) = (j >> 1, j & 1) of
      // that window, so the window order (0,0),(0,1),(1,0),(1,1) with the
      // first maximum winning (acfe_maxpool2d_fused's argmax bytes) is the
      // register order.  Lanes 2t, 2t + 1 hold channels 2 FN t + [0, 2 FN) of
      // the same windows: one DPP swap per fragment pair gives the even lane
      // fragment fm2's and the odd lane fragment fm2 + 1's 2 FN channels, so a
      // tile's stores are FM / 2 x (2 FN x 2 B pooled + 2 FN argmax bytes) per
      // lane (the per-CU store issue rate, not bytes, bounds this epilogue)
      const int P2 = g.P >> 1, Q2 = g.Q >> 1, q = lane >> 4;
      const int cf = wk * (KB / 2) + FN * l16;
      const long long img = (long long)n * P2 * Q2;  // pooled pixels before this image
      unsigned char* const yb = reinterpret_cast<unsigned char*>(Y + img * g.ldy);
      unsigned char* const ab = amax + img * g.K;
      const bool odd = (lane & 1) != 0;
      constexpr int NY = FN / 2;  // dwords of a lane's FN bf16 values
      float sb[FN], sq[FN], bch[FN];
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        sb[fn] = sq[fn] = 0.f;
        bch[fn] = __int_as_float(__builtin_amdgcn_ds_bpermute((FN * l16 + fn) * 4, __float_as_int(blane)));
      }
#pragma unroll
      for (int fm2 = 0; fm2 < FM; fm2 += 2) {
        __builtin_amdgcn_sched_barrier(0);
        // fragments fm2, fm2 + 1: pooled row hp2, pooled columns wq, wq + 4
        const int hp2 = ((hb * TR) >> 1) + (fm2 >> 1);
        unsigned yv[2][NY], av[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int fm = fm2 + hf;
          const int wq = ((wb * SEGW) >> 1) + wp * 8 + hf * 4 + (q ^ (q >> 1));
          const bool inb = hp2 < P2 && wq < Q2;
          const unsigned pp = ((unsigned)n * P2 + hp2) * Q2 + wq;  // < 2^32 (acfe_conv2d_pool_supported)
          // Dropout keep bits of the lane's FN channels (bit fn), one pair
          // hash per channel pair, taken before the accumulators are read
          unsigned keep = (1u << FN) - 1u;
          if (g.drop.on) {
            keep = 0u;
#pragma unroll
            for (int pr = 0; pr < NY; ++pr) {
              const uint32_t h = drop_pair_hash32(g.drop, pp * (unsigned)g.K + cf + 2 * pr);
              keep |= ((h & 0xFFFFu) >= g.drop.thr ? 1u : 0u) << (2 * pr);
              keep |= ((h >> 16) >= g.drop.thr ? 1u : 0u) << (2 * pr + 1);
            }
          }
          float mv[FN];
          av[hf] = 0u;
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) {
            float a[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = bf2f(f2bf(acc[fm][fn][j] + bch[fn]));
            float m = a[0];
            unsigned am = 0;
            if (a[1] > m) m = a[1], am = 1;
            if (a[2] > m) m = a[2], am = 2;
            if (a[3] > m) m = a[3], am = 3;
            if (g.drop.on) m = ((keep >> fn) & 1u) ? bf2f(f2bf(m * g.drop.scl)) : 0.f;
            mv[fn] = m;
            av[hf] |= am << (8 * fn);
            acc[fm][fn] = f4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) {
            const float f = inb ? mv[fn] : 0.f;
            sb[fn] += f;
            sq[fn] += f * f;
          }
          // rounded values are bf16-exact: packing is a bit move
#pragma unroll
          for (int pr = 0; pr < NY; ++pr)
            yv[hf][pr] = (__float_as_uint(mv[2 * pr]) >> 16) | (__float_as_uint(mv[2 * pr + 1]) & 0xffff0000u);
        }
        // (no scheduling across fragment pairs: hoisting the next pair's
        // hashes and addresses over these stores spilled at K = 128)
        __builtin_amdgcn_sched_barrier(0);
        // even lane: fragment fm2 (own | partner's), odd lane: fm2 + 1 (partner's | own)
        unsigned ys[NY], yo[NY], as, ao;
#pragma unroll
        for (int pr = 0; pr < NY; ++pr) {
          const unsigned send = odd ? yv[0][pr] : yv[1][pr];
          ys[pr] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)send, 0xB1, 0xF, 0xF, false);
          yo[pr] = odd ? yv[1][pr] : yv[0][pr];
        }
        {
          const unsigned send = odd ? av[0] : av[1];
          as = (unsigned)__builtin_amdgcn_update_dpp(0, (int)send, 0xB1, 0xF, 0xF, false);
          ao = odd ? av[1] : av[0];
        }
        // stores at the image base + a 32-bit offset (out-of-image windows
        // masked off)
        const int hs = odd ? 1 : 0;
        const int wq = ((wb * SEGW) >> 1) + wp * 8 + hs * 4 + (q ^ (q >> 1));
        const bool inb = hp2 < P2 && wq < Q2;
        const int c0 = wk * (KB / 2) + FN * (l16 & ~1);  // first of the pair's 2 FN channels
        const unsigned pix = (unsigned)(hp2 * Q2 + wq);
        const unsigned yo_ = (pix * (unsigned)g.ldy + c0) * 2u, ao_ = pix * (unsigned)g.K + c0;
        if constexpr (FN == 4) {
          const u32x4 yw = odd ? u32x4{ys[0], ys[1], yo[0], yo[1]} : u32x4{yo[0], yo[1], ys[0], ys[1]};
          const u32x2 aw = odd ? u32x2{as, ao} : u32x2{ao, as};
          if (inb) {
            *reinterpret_cast<u32x4*>(yb + yo_) = yw;
            *reinterpret_cast<u32x2*>(ab + ao_) = aw;
          }
        } else {
          const u32x2 yw = odd ? u32x2{ys[0], yo[0]} : u32x2{yo[0], ys[0]};
          const unsigned aw = odd ? ((as & 0xFFFFu) | (ao << 16)) : ((ao & 0xFFFFu) | (as << 16));
          if (inb) {
            *reinterpret_cast<u32x2*>(yb + yo_) = yw;
            *reinterpret_cast<unsigned*>(ab + ao_) = aw;
          }
        }
      }
      if (stats) {
        // sums over the four windows (lane groups), then lane group q keeps
        // values q * NV16 + k of [sb[0..FN), sq[0..FN)]
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          sb[fn] += __shfl_xor(sb[fn], 16, 64);
          sq[fn] += __shfl_xor(sq[fn], 16, 64);
          sb[fn] += __shfl_xor(sb[fn], 32, 64);
          sq[fn] += __shfl_xor(sq[fn], 32, 64);
        }
#pragma unroll
        for (int k = 0; k < NV16; ++k) {
          float v = 0.f;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int idx = qq * NV16 + k, fn = idx % FN;
            const float vv = idx < FN ? sb[fn] : sq[fn];
            v = q == qq ? vv : v;
          }
          const int idx = q * NV16 + k, st = idx / FN, col = cf + idx % FN;
          if constexpr (REGSTAT) dstat[k] += (double)v;
          else atomicAdd(&sstat[st * KB + col], (double)v);
        }
      }
    }
    if constexpr (PM == 1 && !SWP) {
      // 2x2 windows: rows (2i, 2i+1) in this lane's fragments, columns (l16,
      // l16 ^ 1) in the neighbouring lane.  The lane pair splits each channel
      // quad: the even lane pools channels 0-1, the odd lane 2-3, each getting
      // the partner's column by one DPP swap per row -- half the max / argmax /
      // dropout work of both lanes pooling all four.  Window order (0,0),(0,1),
      // (1,0),(1,1), first maximum wins (acfe_maxpool2d_fused's argmax bytes).
      const int P2 = g.P >> 1, Q2 = g.Q >> 1;
      const int wq = (wb * SEGW + wp * 16 + l16) >> 1;
      const bool odd = (l16 & 1) != 0;
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const f4 rb = bias4(fn);
        const int c = wk * (KB / 2) + fn * 16 + (lane >> 4) * 4 + (odd ? 2 : 0);
#pragma unroll
        for (int i = 0; i < TR / 2; ++i) {
          const int hp2 = ((hb * TR) >> 1) + i;
          const bool inb = hp2 < P2 && wq < Q2;
          const unsigned pp = ((unsigned)n * P2 + hp2) * Q2 + wq;  // < 2^32 (acfe_conv2d_pool_supported)
          float hv[2];
          unsigned amb = 0;
          uint32_t dh = 0;
#pragma unroll
          for (int jp = 0; jp < 2; ++jp) {
            // conv outputs rounded to the storage type (conv -> maxpool), own and partner channel
            const float e0 = bf2f(f2bf(acc[2 * i][fn][jp] + rb[jp]));
            const float e1 = bf2f(f2bf(acc[2 * i + 1][fn][jp] + rb[jp]));
            const float u0 = bf2f(f2bf(acc[2 * i][fn][jp + 2] + rb[jp + 2]));
            const float u1 = bf2f(f2bf(acc[2 * i + 1][fn][jp + 2] + rb[jp + 2]));
            const float o0 = odd ? u0 : e0, o1 = odd ? u1 : e1;   // this lane's channel
            const float s0 = odd ? e0 : u0, s1 = odd ? e1 : u1;   // the partner's channel
            const float r0 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s0), 0xB1, 0xF, 0xF, false));
            const float r1 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s1), 0xB1, 0xF, 0xF, false));
            const float a0 = odd ? r0 : o0, a1 = odd ? o0 : r0;   // row 0: left, right column
            const float a2 = odd ? r1 : o1, a3 = odd ? o1 : r1;   // row 1
            float m = a0;
            unsigned am = 0;
            if (a1 > m) m = a1, am = 1;
            if (a2 > m) m = a2, am = 2;
            if (a3 > m) m = a3, am = 3;
            if (g.drop.on) {
              if (jp == 0) dh = drop_pair_hash32(g.drop, pp * (unsigned)g.K + c);  // channels c, c + 1
              m = ((jp ? dh >> 16 : dh & 0xFFFFu) >= g.drop.thr) ? bf2f(f2bf(m * g.drop.scl)) : 0.f;
            }
            hv[jp] = m;
            const float f = inb ? m : 0.f;
            sv[fn * 4 + jp] += f;
            sv[FN * 4 + fn * 4 + jp] += f * f;
            amb |= am << (8 * jp);
          }
          if (inb) {
            *reinterpret_cast<unsigned*>(Y + (size_t)pp * g.ldy + c) =
                (unsigned)f2bf(hv[0]) | ((unsigned)f2bf(hv[1]) << 16);
            *reinterpret_cast<uint16_t*>(amax + (size_t)pp * g.K + c) = (uint16_t)amb;
          }
          acc[2 * i][fn] = acc[2 * i + 1][fn] = f4{0.f, 0.f, 0.f, 0.f};
        }
      }
      // odd lanes hold channels 2-3 of each quad in slots 0-1: move them to the
      // slots of the butterfly's channel order
#pragma unroll
      for (int k = 0; k < 2 * FN; ++k) {
        const int b = (k / FN) * FN * 4 + (k % FN) * 4;
        const float x0 = sv[b], x1 = sv[b + 1];
        sv[b] = odd ? 0.f : x0;
        sv[b + 1] = odd ? 0.f : x1;
        sv[b + 2] = odd ? x0 : 0.f;
        sv[b + 3] = odd ? x1 : 0.f;
      }
    }
    // PM 0 / 3: per (fragment row, channel quad) -- bias, rounding to the
    // storage type, Dropout with one hash per channel pair, the residual Add
    // (+ReLU), BN sums; rounded values are bf16-exact, so packing is a bit move.
    // Templated on (dropout on, 32-bit index) so the per-element work has no
    // uniform branches and the dgrad / eval paths carry no dropout code.
    auto epi03 = [&](auto dropc, auto idxc) __attribute__((always_inline)) {
      constexpr bool DRP = decltype(dropc)::value, I32 = decltype(idxc)::value;
      uint2 vout[CPERM ? FM : 1][CPERM ? FN : 1];  // CPERM: packed values, stored per fragment row below
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const f4 rb = bias4(fn);
        const int c = wk * (KB / 2) + (CPERM ? (lane >> 4) * 4 * FN + fn * 4 : fn * 16 + (lane >> 4) * 4);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int p = wp * (TR * 16) + fm * 16;
          const int h = hb * TR + p / SEGW, w = wb * SEGW + (p % SEGW) + l16;
          const bool inb = h < g.P && w < g.Q;
          const long long pix = ((long long)n * g.P + h) * g.Q + w;
          float r[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) r[jj] = bf2f(f2bf(acc[fm][fn][jj] + rb[jj]));
          if constexpr (DRP) {
            uint32_t h2[2];
            if constexpr (I32) hash_u32_lo_run<2>(g.drop.seed, ((unsigned)pix * (unsigned)g.K + c) >> 1, h2);
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
              uint32_t hh;
              if constexpr (I32) hh = h2[pr];
              else hh = drop_pair_hash(g.drop, (uint64_t)pix * g.K + c + 2 * pr);
              r[2 * pr] = (hh & 0xFFFFu) >= g.drop.thr ? bf2f(f2bf(r[2 * pr] * g.drop.scl)) : 0.f;
              r[2 * pr + 1] = (hh >> 16) >= g.drop.thr ? bf2f(f2bf(r[2 * pr + 1] * g.drop.scl)) : 0.f;
            }
          }
          if constexpr (PM == 3) {
            uint2 rv;
            if constexpr (RPRE) rv = rres[fm][fn];
            else rv = *reinterpret_cast<const uint2*>(inb ? g.res + pix * g.ldy + c : zp);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const unsigned rw = jj < 2 ? rv.x : rv.y;
              float z = r[jj] + __uint_as_float((jj & 1) ? (rw & 0xffff0000u) : (rw << 16));
              if (g.res_relu) z = fmaxf(z, 0.f);
              r[jj] = bf2f(f2bf(z));
            }
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const float f = inb ? r[jj] : 0.f;
            sv[fn * 4 + jj] += f;
            sv[FN * 4 + fn * 4 + jj] += f * f;
          }
          uint2 v;
          v.x = (__float_as_uint(r[0]) >> 16) | (__float_as_uint(r[1]) & 0xffff0000u);
          v.y = (__float_as_uint(r[2]) >> 16) | (__float_as_uint(r[3]) & 0xffff0000u);
          if constexpr (CPERM) {
            vout[fm][fn] = v;
          } else {
            uint2* dst = inb ? reinterpret_cast<uint2*>(Y + pix * g.ldy + c) : &g_store_sink[lane];
            *dst = v;
          }
          acc[fm][fn] = f4{0.f, 0.f, 0.f, 0.f};
        }
      }
      if constexpr (CPERM) {
        // 4 FN consecutive channels of one pixel per lane: FN / 2 16-B stores
        const int cq = wk * (KB / 2) + (lane >> 4) * 4 * FN;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int p = wp * (TR * 16) + fm * 16;
          const int h = hb * TR + p / SEGW, w = wb * SEGW + (p % SEGW) + l16;
          const bool inb = h < g.P && w < g.Q;
          const long long pix = ((long long)n * g.P + h) * g.Q + w;
          u32x4* dst = inb ? reinterpret_cast<u32x4*>(Y + pix * g.ldy + cq) : &g_store_sink16[lane];
#pragma unroll
          for (int hq = 0; hq < FN / 2; ++hq)
            dst[inb ? hq : 0] = u32x4{vout[fm][2 * hq].x, vout[fm][2 * hq].y, vout[fm][2 * hq + 1].x,
                                      vout[fm][2 * hq + 1].y};
        }
      }
    };
    // PM 5 (the dgrad, no bias): the dX rows rounded to bf16 (what the dgrad
    // stores), packed and stored first -- the tile's x quads, loaded at the
    // start of the epilogue, in flight meanwhile -- then acfe_bn_bwd_reduce's
    // terms of the stored values: gm = dX masked by the BN's ReLU, summed as
    // gm and gm * (x - mean) * invstd (its arithmetic).  Branch-free: masks
    // combined bitwise, out-of-image rows stored to the sink.  (Forming the
    // sums row by row beside the stores, with the coefficient quads re-read per
    // row behind an opaque offset, spilled 150 VGPRs; the same order with the
    // rows' packed values all live and per-element xhat, 7-11.)
    auto epi5 = [&]() __attribute__((always_inline)) {
      const int cq = wk * (KB / 2) + (lane >> 4) * 4 * FN;
      const bool norelu = g.bn_relu == 0;
      // rows rounded, packed and stored first (the x loads in flight), then the sums
      unsigned pk[FM][2 * FN];
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int p = wp * (TR * 16) + fm * 16;
        const int h = hb * TR + p / SEGW, w = wb * SEGW + (p % SEGW) + l16;
        const bool inb = (h < g.P) & (w < g.Q);
        const long long pix = ((long long)n * g.P + h) * g.Q + w;
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          float r[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) r[jj] = bf2f(f2bf(acc[fm][fn][jj]));
          pk[fm][2 * fn] = (__float_as_uint(r[0]) >> 16) | (__float_as_uint(r[1]) & 0xffff0000u);
          pk[fm][2 * fn + 1] = (__float_as_uint(r[2]) >> 16) | (__float_as_uint(r[3]) & 0xffff0000u);
          acc[fm][fn] = f4{0.f, 0.f, 0.f, 0.f};
        }
        u32x4* dst = inb ? reinterpret_cast<u32x4*>(Y + pix * g.ldy + cq) : &g_store_sink16[lane];
#pragma unroll
        for (int hq = 0; hq < FN / 2; ++hq)
          dst[inb ? hq : 0] = u32x4{pk[fm][4 * hq], pk[fm][4 * hq + 1], pk[fm][4 * hq + 2], pk[fm][4 * hq + 3]};
      }
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const f4 csc = *reinterpret_cast<const f4*>(bnt + cq + fn * 4);
        const f4 csh = *reinterpret_cast<const f4*>(bnt + KB + cq + fn * 4);
        const f4 cmu = *reinterpret_cast<const f4*>(bnt + 2 * KB + cq + fn * 4);
        const f4 cis = *reinterpret_cast<const f4*>(bnt + 3 * KB + cq + fn * 4);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int p = wp * (TR * 16) + fm * 16;
          const int h = hb * TR + p / SEGW, w = wb * SEGW + (p % SEGW) + l16;
          const bool inb = (h < g.P) & (w < g.Q);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const unsigned xw = xbn[fm][2 * fn + (jj >> 1)], gw = pk[fm][2 * fn + (jj >> 1)];
            const float xf = __uint_as_float((jj & 1) ? (xw & 0xffff0000u) : (xw << 16));
            const float gf = __uint_as_float((jj & 1) ? (gw & 0xffff0000u) : (gw << 16));
            const bool on = inb & (norelu | (xf * csc[jj] + csh[jj] > 0.f));
            const float gm = on ? gf : 0.f;
            sv[fn * 4 + jj] += gm;
            sv[FN * 4 + fn * 4 + jj] += gm * ((xf - cmu[jj]) * cis[jj]);
          }
        }
      }
    };
    // only PM 4 carries a Dropout, launched with 32-bit element indices (launch_fwd_t)
    if constexpr (PM == 5) epi5();
    else if constexpr (PM != 1) epi03(std::bool_constant<PM == 4>{}, std::true_type{});
    if (stats && !SWP) {
      butterfly_step<NV, 8, 0x128>(sv, lane);
      butterfly_step<NV / 2, 4, 0x141>(sv, lane);
      butterfly_step<NV / 4, 2, 0x4E>(sv, lane);
      butterfly_step<NV / 8, 1, 0xB1>(sv, lane);
      const int b0 = ((l16 >> 3) & 1) * (NV / 2) + ((l16 >> 2) & 1) * (NV / 4) + ((l16 >> 1) & 1) * (NV / 8) +
                     (l16 & 1) * (NV / 16);
#pragma unroll
      for (int k = 0; k < NV16; ++k) {
        if constexpr (REGSTAT) {
          dstat[k] += (double)sv[k];
        } else {
          const int idx = b0 + k, st = idx / (FN * 4), rm = idx - st * (FN * 4);
          const int col = wk * (KB / 2) + (CPERM ? (lane >> 4) * 4 * FN + rm : (rm >> 2) * 16 + (lane >> 4) * 4 + (rm & 3));
          atomicAdd(&sstat[st * KB + col], (double)sv[k]);
        }
      }
    }
  };

  if constexpr (PRO) __syncthreads();  // pss
  if (L > 0) {
    gload(0, 0);
    if constexpr (WDMA) wdma(0, 0);
    xform(0);
    sstore(0);
  }
  if constexpr (WDMA) wait_vmcnt<0>();
  __syncthreads();
  int buf = 0, cst = 0, ctm = walk.tm;
  // ACFE_CONV_DBG=8 in a -DACFE_ROWS_STAMPS build (make stamps): per-wave
  // cycles of issue / MFMA / epilogue / first barrier / restage + second
  // barrier (tools/rows_stamps.py); compiled out of the production library
#ifdef ACFE_ROWS_STAMPS
  Stamps stp(g.dbg == 8);
#else
  Stamps stp(false);
#endif
  int ctl = 0;  // walk-local index of the current tile (step t = ctl * nsteps_t + cst)
  for (int t = 0; t < L; ++t) {
    const bool more = t + 1 < L;
    // (tile, step) of steps t + 1 and t + 2, without divisions
    const bool w1 = cst + 1 == nsteps_t, w2 = cst + 2 >= nsteps_t;
    const int st1 = w1 ? 0 : cst + 1, tl1 = ctl + (w1 ? 1 : 0);
    const int st2 = w2 ? cst + 2 - nsteps_t : cst + 2, tl2 = ctl + (w2 ? 1 : 0);
    // XRES: filter row of this step and whether the next one starts a chunk
    // (XRES: the next chunk's rows are requested one step early, at rs == 1,
    // and land by that step's closing wait; PRO transforms them during rs == 2)
    const int rs = XRES ? cst - 3 * (cst / 3) : 0;
    const bool xnext = more && (!XRES || rs == 2);
    const bool xload = XRES && rs == 1 && t + 2 < L;  // this step requests the next chunk's rows
    if constexpr (XRES) {
      if (xload) gload(tl2, st2);
    } else {
      if (more) gload(tl1, st1);
    }
    if (more) {
      if constexpr (WDMA) {
        if constexpr (WILV) wprep(st1, (t + 1) & 1);
        else wdma(st1, (t + 1) & 1);
      }
    }
    if constexpr (PRO) {
      if (xnext) xform(st1 / 3);
    }
    if constexpr (RPRE) {
      if (cst + 1 == nsteps_t) rload(ctm);
    }
    stp.mark(0);
    const unsigned char* Xl = xbuf(buf) + rs * (HWX * XRB);
    const unsigned char* Wl = WDMA ? smem + WBASE + (t & 1) * WBYTES : xbuf(buf) + XBYTES;
    // K = 64: let the scheduler interleave the fragment reads with the MFMAs
    // (fwd_add 128->64 1.084 -> 1.013 ms, dropout 64->64 0.649 -> 0.625 ms;
    // at K = 128 the same hint spills: fwd_pool 4.96 -> 5.35 ms, r02o)
    if constexpr (KB == 64) __builtin_amdgcn_iglp_opt(0);
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        // WILV: the next step's weight pieces are issued between the MFMA
        // groups (piece j before group j * WGRP / WPW of the six), so their
        // issue waits overlap this step's MFMAs instead of preceding them
        if constexpr (WILV) {
#pragma unroll
          for (int j = 0; j < WPW; ++j)
            if ((j * WGRP) / WPW == s * 2 + kk && more) wpiece(j);
        }
        uint4 wf[FN], xf[FM];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          wf[fn] = *reinterpret_cast<const uint4*>(SWP ? Wl + (kk * 3 + s) * KB * 64 + wrb[fn]
                                                       : Wl + s * KB * 128 + (wrb[fn] ^ (kk << 6)));
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
          xf[fm] = *reinterpret_cast<const uint4*>(Xl + xoff[fm] + s * XRB + kk * 64);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) {
            if constexpr (SWP) mma(acc[fm][fn], xf[fm], wf[fn], T());
            else mma(acc[fm][fn], wf[fn], xf[fm], T());
          }
      }
    stp.mark(1);
    if (NBUF == 2 && more) sstore(buf ^ 1);
    // PM 5: the tile's epilogue runs after the next chunk's rows are stored
    // (below): its BN-input loads and sums need the registers the staged rows
    // hold until then (before them: 9 VGPRs spilled, reloaded every step)
    bool epi_late = false;
    if (++cst == nsteps_t) {
      cst = 0;
      ++ctl;
      if constexpr (PM == 5) {
        epi_late = true;
      } else {
        epilogue(ctm);
        ctm += walk.step;
      }
    }
    stp.mark(2);
    if constexpr (WDMA && NBUF == 2) wait_vmcnt<0>();  // next step's weight pieces landed
    if constexpr (XRES) {
      if (!xnext) wait_vmcnt<0>();
    }
    __syncthreads();
    stp.mark(3);
    if (NBUF == 2) {
      buf ^= 1;
    } else if (xnext) {
      sstore(0);  // single buffer: every wave has finished reading it
      if constexpr (WDMA) wait_vmcnt<0>();  // next step's weight pieces landed
      __syncthreads();
    }
    if constexpr (PM == 5) {
      if (epi_late) {
        epilogue(ctm);
        ctm += walk.step;
      }
    }
    stp.mark(4);
  }
  stp.flush(wid);
  if (stats && !REGSTAT) {
    for (int c = tid; c < KB; c += 512) {
      stats[((long long)blockIdx.x * 2 + 0) * g.Kp + c] = sstat[c];
      stats[((long long)blockIdx.x * 2 + 1) * g.Kp + c] = sstat[KB + c];
    }
  }
  if (stats && REGSTAT) {
    // the 4 waves of one channel half (wid = wk * 4 + wp) hold partials of the
    // same (channel, sum / sum-of-squares) slots in the same lanes: fixed-order
    // sum through LDS (free after the main loop), wave wp = 0 writes the row
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);
#pragma unroll
    for (int k = 0; k < NV16; ++k) red[(wid * 64 + lane) * NV16 + k] = dstat[k];
    __syncthreads();
    if (wp == 0) {
      const int b0 = ((l16 >> 3) & 1) * (NV / 2) + ((l16 >> 2) & 1) * (NV / 4) + ((l16 >> 1) & 1) * (NV / 8) +
                     (l16 & 1) * (NV / 16);
#pragma unroll
      for (int k = 0; k < NV16; ++k) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v += red[((wk * 4 + q) * 64 + lane) * NV16 + k];
        int st, col;
        if constexpr (SWP) {
          const int idx = (lane >> 4) * NV16 + k;
          st = idx / FN;
          col = wk * (KB / 2) + FN * l16 + idx % FN;
        } else {
          const int idx = b0 + k, rm = idx - (idx / (FN * 4)) * (FN * 4);
          st = idx / (FN * 4);
          col = wk * (KB / 2) + (CPERM ? (lane >> 4) * 4 * FN + rm : (rm >> 2) * 16 + (lane >> 4) * 4 + (rm & 3));
        }
        stats[((long long)blockIdx.x * 2 + st) * g.Kp + col] = v;
      }
    }
  }
  if (stats) {
    for (int rr = blockIdx.x + gridDim.x; rr < srows; rr += gridDim.x)
      for (int c = tid; c < 2 * KB; c += 512) stats[((long long)rr * 2 + (c / KB)) * g.Kp + (c % KB)] = 0.0;
  }
}


// ------------------------------------------------------------------ 3x3 stride 1, narrow output (K in {16, 32})
// wr_resnet_bird's stage-2/3 branch21 convolutions whose output channel count
// is the feature height (resnet/wr_resnet_bird.py:139: 128 -> 32 at 32 x 64,
// 256 -> 16 at 16 x 32) and the dgrads of the branch2b convolutions (32 / 16
// output channels).  With K <= 32 an im2col GEMM tile does 4-8 MFMAs per
// K-tile and wave (k_conv_fwd_g: 125-310 TFLOP/s).  Here the whole packed
// weight matrix (9 taps x C x K <= 72 KB) stays in LDS for the workgroup's
// lifetime, and one pipeline step stages a 64-channel chunk of the input halo
// (TR + 2 rows x SEGW + 2 pixels, TR x SEGW = NW x 32 output pixels) ONCE for
// all nine taps: NW waves x 32 pixels x K, 36 x K / 16 MFMAs per wave per step.
// Fragment reads as k_conv3x3_rows (160-B pixel pitch, XOR-swizzled 128-B
// weight rows), register-staged double buffer, one barrier per step; epilogue:
// bias, bf16 rounding, the pair-hash Dropout (PM 4's), BN sums through
// 16-lane shuffles and LDS f64 atomics.  Persistent, XCD-aware tile walk.
template <int KB, int SEGW, bool DROP, int NW>
__global__ void __launch_bounds__(NW * 64, 1)
k_conv3x3_narrow(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
                 const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats, int tiles_h,
                 int tiles_w, int ntiles, int srows) {
  // NW = 4: 128-pixel tiles, double-buffered input image (one wave per SIMD);
  // NW = 8: 256-pixel tiles, one image buffer stored between two barriers
  // (two waves per SIMD hide each other's latency)
  constexpr int NT = NW * 64, NXB = NW == 8 ? 1 : 2;
  constexpr int TR = NW * 32 / SEGW, HWX = SEGW + 2, XR = TR + 2, XRB = 160;
  constexpr int FM = 2, FN = KB / 16;
  constexpr int XBYTES = XR * HWX * XRB, WBYTES = 576 * 128;
  constexpr int XG = XR * HWX * 8, XPT = (XG + NT - 1) / NT;
  constexpr int SMEM = NXB * XBYTES + WBYTES + 2 * KB * 8;
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  unsigned char* Wl = smem + NXB * XBYTES;
  double* sstat = reinterpret_cast<double*>(smem + NXB * XBYTES + WBYTES);
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nch = g.C / 64, tpi = tiles_h * tiles_w;
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(g_zero_page);
  for (int i = tid; i < 2 * KB; i += NT) sstat[i] = 0.0;
  // resident weights: row (t * nch + cc) * KB + k = W[k][tap t][chunk cc], granule gw at slot gw ^ (k & 7)
  {
    const int wrows = 9 * nch * KB;
    for (int gi = tid; gi < wrows * 8; gi += NT) {
      const int row = gi >> 3, gw = gi & 7;
      const int k = row % KB, tc = row / KB, cc = tc % nch, t = tc / nch;
      const u32x4 v = *reinterpret_cast<const u32x4*>(Wp + (long long)k * g.Kdp + t * g.C + cc * 64 + gw * 8);
      *reinterpret_cast<u32x4*>(Wl + row * 128 + ((gw ^ (k & 7)) << 4)) = v;
    }
  }
  const TileWalk walk(ntiles);
  const int ntl = walk.tm < walk.end ? (walk.end - walk.tm + walk.step - 1) / walk.step : 0;
  const int L = ntl * nch;
  // two register sets: step t + 2 is requested while step t computes, so a
  // load has two steps of MFMA work to land (one wave per SIMD hides nothing)
  u32x4 ra[XPT], rb[XPT];
  auto gload = [&](u32x4 (&rx)[XPT], int t) __attribute__((always_inline)) {
    const int tl = t / nch, cc = t - tl * nch;
    const int tm = walk.tm + tl * walk.step;
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
    const int h0 = hb * TR - g.pt, w0 = wb * SEGW - g.pl;
    const uint16_t* img = X + (long long)n * g.H * g.W * g.C + cc * 64;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + NT * i;
      const int xrow = idx / (HWX * 8), xpix = (idx - xrow * (HWX * 8)) >> 3, gr = idx & 7;
      const int hin = h0 + xrow, win = w0 + xpix;
      const bool ok = idx < XG && (unsigned)hin < (unsigned)g.H && (unsigned)win < (unsigned)g.W;
      rx[i] = *reinterpret_cast<const u32x4*>(ok ? img + ((long long)hin * g.W + win) * g.C + gr * 8 : zp);
    }
  };
  auto sstore = [&](const u32x4 (&rx)[XPT], int buf) __attribute__((always_inline)) {
    unsigned char* Xl = smem + buf * XBYTES;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + NT * i;
      if (idx < XG) *reinterpret_cast<u32x4*>(Xl + (idx >> 3) * XRB + (idx & 7) * 16) = rx[i];
    }
  };
  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // this wave's two 16-pixel fragments: tile pixel wid * 32 + fm * 16 + l16 = (row, col)
  // this lane's bias quads, loaded once
  f4 bq[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn)
    bq[fn] = bias ? *reinterpret_cast<const f4*>(bias + fn * 16 + (lane >> 4) * 4) : f4{0.f, 0.f, 0.f, 0.f};
  int xoff[FM];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int p = wid * 32 + fm * 16;
    xoff[fm] = ((p / SEGW) * HWX + (p % SEGW) + l16) * XRB + (lane >> 4) * 16;
  }
  auto epilogue = [&](int tm) __attribute__((always_inline)) {
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
    float s1[FN][4], s2[FN][4];
#pragma unroll
    for (int fn = 0; fn < FN; ++fn)
#pragma unroll
      for (int j = 0; j < 4; ++j) s1[fn][j] = s2[fn][j] = 0.f;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int p = wid * 32 + fm * 16 + l16;
      const int h = hb * TR + p / SEGW, w = wb * SEGW + p % SEGW;
      const bool inb = h < g.P && w < g.Q;
      const unsigned pix = ((unsigned)n * g.P + h) * g.Q + w;  // < 2^32: launch checks M * K < 2^32
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int c = fn * 16 + (lane >> 4) * 4;
        float r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = bf2f(f2bf(acc[fm][fn][j] + bq[fn][j]));
        if constexpr (DROP) {
          uint32_t h2[2];
          hash_u32_lo_run<2>(g.drop.seed, (pix * (unsigned)g.K + c) >> 1, h2);
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            const uint32_t hh = h2[pr];
            r[2 * pr] = (hh & 0xFFFFu) >= g.drop.thr ? bf2f(f2bf(r[2 * pr] * g.drop.scl)) : 0.f;
            r[2 * pr + 1] = (hh >> 16) >= g.drop.thr ? bf2f(f2bf(r[2 * pr + 1] * g.drop.scl)) : 0.f;
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float f = inb ? r[j] : 0.f;
          s1[fn][j] += f;
          s2[fn][j] += f * f;
        }
        uint2 v;
        v.x = (__float_as_uint(r[0]) >> 16) | (__float_as_uint(r[1]) & 0xffff0000u);
        v.y = (__float_as_uint(r[2]) >> 16) | (__float_as_uint(r[3]) & 0xffff0000u);
        uint2* dst = inb ? reinterpret_cast<uint2*>(Y + (size_t)pix * g.ldy + c) : &g_store_sink[lane];
        *dst = v;
        acc[fm][fn] = f4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (stats) {
      // sum over the 16 pixels (lanes l16) of each channel, then one LDS atomic per value
#pragma unroll
      for (int fn = 0; fn < FN; ++fn)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) {
            s1[fn][j] += __shfl_xor(s1[fn][j], off, 64);
            s2[fn][j] += __shfl_xor(s2[fn][j], off, 64);
          }
          if (l16 == 0) {
            const int c = fn * 16 + (lane >> 4) * 4 + j;
            atomicAdd(&sstat[c], (double)s1[fn][j]);
            atomicAdd(&sstat[KB + c], (double)s2[fn][j]);
          }
        }
    }
  };

  if (L > 0) {
    gload(ra, 0);
    sstore(ra, 0);
  }
  if (L > 1) gload(rb, 1);
  __syncthreads();
  int cst = 0, ctm = walk.tm;
  // at entry of step t: LDS buffer t & 1 holds step t, rnext holds (in flight) step t + 1
  auto step = [&](int t, const u32x4 (&rnext)[XPT], u32x4 (&rfree)[XPT]) __attribute__((always_inline)) {
    if (t + 2 < L) gload(rfree, t + 2);
    const int cc = t % nch;
    const unsigned char* Xl = smem + (NXB == 2 ? (t & 1) * XBYTES : 0);
    __builtin_amdgcn_iglp_opt(0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int r = tap / 3, s = tap - 3 * (tap / 3);
        uint4 wf[FN], xf[FM];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int k = fn * 16 + l16;
          const int row = (tap * nch + cc) * KB + k;
          wf[fn] = *reinterpret_cast<const uint4*>(Wl + row * 128 + (((kk * 4 + (lane >> 4)) ^ (k & 7)) << 4));
        }
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
          xf[fm] = *reinterpret_cast<const uint4*>(Xl + xoff[fm] + (r * HWX + s) * XRB + kk * 64);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) mma(acc[fm][fn], wf[fn], xf[fm], uint16_t());
      }
    if constexpr (NXB == 2) {
      if (t + 1 < L) sstore(rnext, (t + 1) & 1);
    }
    if (++cst == nch) {
      cst = 0;
      epilogue(ctm);
      ctm += walk.step;
    }
    __syncthreads();
    if constexpr (NXB == 1) {
      if (t + 1 < L) {  // every wave is done with the image: restage it
        sstore(rnext, 0);
        __syncthreads();
      }
    }
  };
  for (int t = 0; t < L; t += 2) {
    step(t, rb, ra);
    if (t + 1 < L) step(t + 1, ra, rb);
  }
  if (stats) {
    __syncthreads();
    for (int c = tid; c < g.Kp; c += NT) {
      stats[((long long)blockIdx.x * 2 + 0) * g.Kp + c] = c < KB ? sstat[c] : 0.0;
      stats[((long long)blockIdx.x * 2 + 1) * g.Kp + c] = c < KB ? sstat[KB + c] : 0.0;
    }
    for (int rr = blockIdx.x + gridDim.x; rr < srows; rr += gridDim.x)
      for (int c = tid; c < 2 * g.Kp; c += NT) stats[((long long)rr * 2 + (c / g.Kp)) * g.Kp + (c % g.Kp)] = 0.0;
  }
}

// ------------------------------------------------------------------ 3x3 stride 1, few input channels, wide output
// k_conv3x3_cw<CW, KB>: CW = 32 -> KB = 128 (wr_resnet_bird's stage-2 branch2b
// forward + residual and branch21 dgrad, 32 x 64; resnet/wr_resnet_bird.py:
// 150-152) and CW = 16 -> KB = 256 (stage 3 at 16 x 32).  With C = 16 / 32 the
// im2col GEMM (k_conv_fwd_g) runs 3-5 K-tiles per 128-pixel tile, its
// prologue / epilogue dominating (T1: 245 / 178 us per 32 -> 128 call, ~0.3
// PFLOP/s).  Here, as in k_conv3x3_narrow: the packed weights (9 x CW x KB
// bf16, 72 / 80 KB) stay in LDS for the workgroup's lifetime as NQ 32-deep
// k-steps (CW = 32: one tap each; CW = 16: taps 2 qs, 2 qs + 1, the last
// step's second half the packing's zeros), a tile (256 pixels: TR rows x SEGW)
// stages its (TR + 2) x (SEGW + 2) input halo once for all nine taps (80- /
// 48-B pixel pitch: 16 consecutive pixels of a fragment read start on
// distinct 4-bank groups), 8 waves x 32 pixels x KB channels, 9 / 5 k-steps of
// v_mfma_f32_16x16x32_bf16 per tile.  Weight rows are permuted (fragment fn,
// A row m = output channel 4 FN (m >> 2) + 4 fn + (m & 3)) so a lane holds
// 4 FN consecutive channels of its pixel (16-B stores; granule slot
// g ^ ((k >> LQ) & 3) keeps a fragment's 16 rows on distinct banks).
// Epilogue per 32-channel half: bias (LDS table), bf16 rounding, the pair-hash
// Dropout or (ADD, acfe_conv2d_fwd_add) the residual g.res (+ReLU) as ops.add
// stores it, BN sums by a DPP butterfly into per-lane f64 partials (one
// fixed-order cross-wave sum at the end).  The next tile's halo is in flight
// in registers during the MFMAs (CW = 32: the residual words too).
template <int CW, int KB, int SEGW, bool DROP, bool ADD = false>
__global__ void __launch_bounds__(512, 1)
k_conv3x3_cw(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
             const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats, int tiles_h,
             int tiles_w, int ntiles, int srows) {
  static_assert((CW == 32 && KB == 128) || (CW == 16 && KB == 256), "shapes");
  static_assert(!(DROP && ADD), "modes");
  // FM pixel fragments per wave (KB = 256: one, the 128 accumulators of two spilled)
  constexpr int FM = KB == 256 ? 1 : 2, TP = 128 * FM;  // tile pixels (8 waves x 16 FM)
  constexpr int NT = 512, TR = TP / SEGW, HWX = SEGW + 2, XR = TR + 2, XRB = CW == 32 ? 80 : 48;
  constexpr int NQ = (9 * CW + 31) / 32, FN = KB / 16, CPL = 4 * FN, LQ = CPL == 32 ? 5 : 6;
  constexpr int NH = FN / 8, NV = 64;  // 32-channel epilogue halves; BN-sum values per half
  constexpr int GPP = CW / 8, XG = XR * HWX * GPP, XPT = (XG + NT - 1) / NT;
  constexpr int XBYTES = XR * HWX * XRB, WBYTES = NQ * KB * 64;
  constexpr int SMEM = XBYTES + WBYTES + KB * 4;
  static_assert(SMEM <= 163840 && 8 * 64 * NH * 4 * 8 <= SMEM, "LDS");
  constexpr bool RPF = ADD && NH == 1;  // residual words prefetched before the MFMAs
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  unsigned char* Wl = smem + XBYTES;
  float* btab = reinterpret_cast<float*>(smem + XBYTES + WBYTES);
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tpi = tiles_h * tiles_w;
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(g_zero_page);
  // resident weights: row qs * KB + k = k-dim [32 qs, 32 qs + 32) of output
  // channel k (64 B), granule gw at slot gw ^ ((k >> LQ) & 3)
  for (int gi = tid; gi < NQ * KB * 4; gi += NT) {
    const int row = gi >> 2, gw = gi & 3, k = row % KB, qs = row / KB;
    const u32x4 v = *reinterpret_cast<const u32x4*>(Wp + (long long)k * g.Kdp + qs * 32 + gw * 8);
    *reinterpret_cast<u32x4*>(Wl + row * 64 + ((gw ^ ((k >> LQ) & 3)) << 4)) = v;
  }
  for (int i = tid; i < KB; i += NT) btab[i] = bias ? bias[i] : 0.f;
  const TileWalk walk(ntiles);
  const int ntl = walk.tm < walk.end ? (walk.end - walk.tm + walk.step - 1) / walk.step : 0;
  u32x4 rx[XPT];
  auto gload = [&](int tl) __attribute__((always_inline)) {
    const int tm = walk.tm + tl * walk.step;
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
    const int h0 = hb * TR - g.pt, w0 = wb * SEGW - g.pl;
    const uint16_t* img = X + (long long)n * g.H * g.W * CW;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + NT * i;
      const int px = idx / GPP, xrow = px / HWX, xpix = px - xrow * HWX;
      const int hin = h0 + xrow, win = w0 + xpix;
      const bool ok = idx < XG && (unsigned)hin < (unsigned)g.H && (unsigned)win < (unsigned)g.W;
      rx[i] = *reinterpret_cast<const u32x4*>(ok ? img + ((long long)hin * g.W + win) * CW + (idx % GPP) * 8 : zp);
    }
  };
  auto sstore = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + NT * i;
      if (idx < XG) *reinterpret_cast<u32x4*>(smem + (idx / GPP) * XRB + (idx % GPP) * 16) = rx[i];
    }
  };
  // fragment read offsets: weights of fragment fn (row k = CPL (l16 >> 2) +
  // 4 fn + (l16 & 3), granule q); input pixels of fragment fm; per k-step the
  // lane's tap (k-dim 32 qs + 8 q) and channel offset in the halo
  // (k >> LQ) = l16 >> 2 for every fn: fragment fn is the lane's base + 256 fn B)
  int xoff[FM], xq[NQ];
  const int kw0 = CPL * (l16 >> 2) + (l16 & 3);
  const int woff0 = kw0 * 64 + ((q ^ ((l16 >> 2) & 3)) << 4);
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int p = wid * 16 * FM + fm * 16 + l16;
    xoff[fm] = ((p / SEGW) * HWX + (p % SEGW)) * XRB;
  }
#pragma unroll
  for (int qs = 0; qs < NQ; ++qs) {
    const int kd = 32 * qs + 8 * q, t = kd / CW < 9 ? kd / CW : 8, c0 = kd % CW;  // (t 9: zero weights)
    xq[qs] = ((t / 3) * HWX + (t % 3)) * XRB + c0 * 2;
  }
  double dstat[NH][NV / 16];
#pragma unroll
  for (int hh = 0; hh < NH; ++hh)
#pragma unroll
    for (int k = 0; k < NV / 16; ++k) dstat[hh][k] = 0.0;
  const int cq = CPL * q;  // this lane's output channels cq + [0, CPL)
  f4 acc[FM][FN];
  if (ntl > 0) {
    gload(0);
    sstore();
  }
  __syncthreads();
  u32x4 rres[FM][4];
  auto res_load = [&](int tm, int fm, int hh) __attribute__((always_inline)) {
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
    const int p = wid * 16 * FM + fm * 16 + l16;
    const int h = hb * TR + p / SEGW, w = wb * SEGW + p % SEGW;
    const bool inb = (h < g.P) & (w < g.Q);
    const u32x4* rs =
        inb ? reinterpret_cast<const u32x4*>(g.res + ((size_t)((unsigned)n * g.P + h) * g.Q + w) * g.ldy + cq + 32 * hh)
            : reinterpret_cast<const u32x4*>(zp);
#pragma unroll
    for (int hq = 0; hq < 4; ++hq) rres[fm][hq] = rs[inb ? hq : 0];
  };
  for (int tl = 0; tl < ntl; ++tl) {
    const int tm = walk.tm + tl * walk.step;
    if (tl + 1 < ntl) gload(tl + 1);
    if constexpr (RPF) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) res_load(tm, fm, 0);
    }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = f4{0.f, 0.f, 0.f, 0.f};
    __builtin_amdgcn_iglp_opt(0);
#pragma unroll
    for (int qs = 0; qs < NQ; ++qs) {
      uint4 xf[FM];
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) xf[fm] = *reinterpret_cast<const uint4*>(smem + xoff[fm] + xq[qs]);
#pragma unroll
      for (int f0 = 0; f0 < FN; f0 += 8) {  // weight fragments 8 at a time (KB = 256: registers)
        uint4 wf[8];
#pragma unroll
        for (int fn = 0; fn < 8; ++fn) wf[fn] = *reinterpret_cast<const uint4*>(Wl + woff0 + qs * KB * 64 + (f0 + fn) * 256);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < 8; ++fn) mma(acc[fm][f0 + fn], wf[fn], xf[fm], uint16_t());
      }
    }
    // epilogue: lane = pixel l16 of fragment fm, channels cq + 4 fn + j, by 32-channel halves
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      if constexpr (ADD && !RPF) {
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) res_load(tm, fm, hh);
      }
      float sv[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) sv[i] = 0.f;
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int p = wid * 16 * FM + fm * 16 + l16;
        const int h = hb * TR + p / SEGW, w = wb * SEGW + p % SEGW;
        const bool inb = (h < g.P) & (w < g.Q);
        const unsigned pix = ((unsigned)n * g.P + h) * g.Q + w;  // < 2^32: launcher checks M * K < 2^32
        unsigned pk[16];
#pragma unroll
        for (int f8 = 0; f8 < 8; ++f8) {
          const int fn = 8 * hh + f8, c = cq + 4 * fn;
          const f4 b4 = *reinterpret_cast<const f4*>(btab + c);
          float rr[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) rr[j] = bf2f(f2bf(acc[fm][fn][j] + b4[j]));
          if constexpr (ADD) {
            // z = (ReLU)(conv + residual), rounded to bf16 (ops.add's values)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const unsigned rw = rres[fm][f8 >> 1][2 * (f8 & 1) + (j >> 1)];
              float z = rr[j] + __uint_as_float((j & 1) ? (rw & 0xffff0000u) : (rw << 16));
              if (g.res_relu) z = fmaxf(z, 0.f);
              rr[j] = bf2f(f2bf(z));
            }
          }
          if constexpr (DROP) {
            uint32_t h2[2];
            hash_u32_lo_run<2>(g.drop.seed, (pix * (unsigned)KB + c) >> 1, h2);
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
              const uint32_t hs = h2[pr];
              rr[2 * pr] = (hs & 0xFFFFu) >= g.drop.thr ? bf2f(f2bf(rr[2 * pr] * g.drop.scl)) : 0.f;
              rr[2 * pr + 1] = (hs >> 16) >= g.drop.thr ? bf2f(f2bf(rr[2 * pr + 1] * g.drop.scl)) : 0.f;
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float f = inb ? rr[j] : 0.f;
            sv[f8 * 4 + j] += f;
            sv[32 + f8 * 4 + j] += f * f;
          }
          pk[2 * f8] = (__float_as_uint(rr[0]) >> 16) | (__float_as_uint(rr[1]) & 0xffff0000u);
          pk[2 * f8 + 1] = (__float_as_uint(rr[2]) >> 16) | (__float_as_uint(rr[3]) & 0xffff0000u);
        }
        u32x4* dst = inb ? reinterpret_cast<u32x4*>(Y + (size_t)pix * g.ldy + cq + 32 * hh) : &g_store_sink16[lane];
#pragma unroll
        for (int hq = 0; hq < 4; ++hq)
          dst[inb ? hq : 0] = u32x4{pk[4 * hq], pk[4 * hq + 1], pk[4 * hq + 2], pk[4 * hq + 3]};
      }
      if (stats) {
        // reduce-scatter over the 16 pixel lanes: lane l16 keeps values b0 + k of sv
        butterfly_step<NV, 8, 0x128>(sv, lane);
        butterfly_step<NV / 2, 4, 0x141>(sv, lane);
        butterfly_step<NV / 4, 2, 0x4E>(sv, lane);
        butterfly_step<NV / 8, 1, 0xB1>(sv, lane);
#pragma unroll
        for (int k = 0; k < NV / 16; ++k) dstat[hh][k] += (double)sv[k];
      }
    }
    __syncthreads();  // every wave is done with the halo
    if (tl + 1 < ntl) {
      sstore();
      __syncthreads();
    }
  }
  if (stats) {
    // fixed-order sum of the 8 waves' partials (same slots in the same lanes)
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);
#pragma unroll
    for (int hh = 0; hh < NH; ++hh)
#pragma unroll
      for (int k = 0; k < NV / 16; ++k) red[((wid * 64 + lane) * NH + hh) * (NV / 16) + k] = dstat[hh][k];
    __syncthreads();
    if (wid == 0) {
      const int b0 = ((l16 >> 3) & 1) * (NV / 2) + ((l16 >> 2) & 1) * (NV / 4) + ((l16 >> 1) & 1) * (NV / 8) +
                     (l16 & 1) * (NV / 16);
#pragma unroll
      for (int hh = 0; hh < NH; ++hh)
#pragma unroll
        for (int k = 0; k < NV / 16; ++k) {
          double v = 0.0;
#pragma unroll
          for (int w = 0; w < 8; ++w) v += red[((w * 64 + lane) * NH + hh) * (NV / 16) + k];
          const int idx = b0 + k, st = idx / 32, rm = idx - st * 32;
          stats[((long long)blockIdx.x * 2 + st) * g.Kp + cq + 32 * hh + rm] = v;
        }
    }
    for (int rr = blockIdx.x + gridDim.x; rr < srows; rr += gridDim.x)
      for (int c = tid; c < 2 * KB; c += NT) stats[((long long)rr * 2 + (c / KB)) * g.Kp + (c % KB)] = 0.0;
  }
}

// ------------------------------------------------------------------ 3x3 stride 1, 16 input channels
// wr_resnet's stage-1 block-0 conv2a (resnet/wr_resnet.py:22: 3x3 16 -> 64 at
// 128 x 513, 1.2 GFLOP per clip).  With C = 16 the generic im2col GEMM
// gathers 32-byte pixel granules per tap and ran at ~130 TFLOP/s (r03e
// profile: 4.76 ms per 512 clips).  Here the MFMA k dimension is tap-major:
// k-step q covers taps 2q and 2q + 1 (16 channels each; the fifth step's
// second half is the zero padding of the packed weights), so the nine taps are
// five k-steps of v_mfma_f32_16x16x32_bf16 (90 % useful).  The packed weight
// matrix (64 x 160 bf16) sits in VGPRs as A fragments for the workgroup's
// lifetime; each 8-row x 64-pixel tile stages its 10 x 66-pixel, 16-channel
// input halo in LDS once (48-B pixel pitch) and every lane reads its im2col B
// fragment (8 channels of one tap) straight from it; the next tile's halo is
// prefetched into registers during the MFMAs.  Epilogue of k_conv3x3_narrow:
// bias, bf16 rounding, the pair-hash Dropout, BN sums.  Persistent, XCD-aware.
template <bool DROP>
__global__ void __launch_bounds__(512, 1)
k_conv3x3_c16(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
              const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats, int tiles_h,
              int tiles_w, int ntiles, int srows) {
  constexpr int KB = 64, TR = 8, SEGW = 64, HWX = SEGW + 2, XR = TR + 2, XRB = 48;
  constexpr int FM = 4, FN = 4, NQ = 5;  // per wave: one tile row = 4 x 16 pixels x 64 channels
  constexpr int XG = XR * HWX * 2;       // 16-B granules of the halo (two per pixel)
  constexpr int XPT = (XG + 511) / 512;
  __shared__ __attribute__((aligned(16))) unsigned char xs[XR * HWX * XRB];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // the wave's tile row
  const int tpi = tiles_h * tiles_w;
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(g_zero_page);
  // BN sums: per-lane f64 partials of the DPP butterfly's slots, one
  // fixed-order cross-wave sum at the end (per-tile LDS f64 atomics of 16-lane
  // shuffle sums before, r04)
  constexpr int NV = 2 * FN * 4;
  double dstat[NV / 16] = {0.0, 0.0};
  // A fragments: lane (l16, lg) of channel fragment fn holds W[fn * 16 + l16][q * 32 + lg * 8 .. + 7]
  uint4 wa[NQ][FN];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn)
      wa[q][fn] = *reinterpret_cast<const uint4*>(Wp + (long long)(fn * 16 + l16) * g.Kdp + q * 32 + lg * 8);
  f4 bq[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn)
    bq[fn] = bias ? *reinterpret_cast<const f4*>(bias + fn * 16 + lg * 4) : f4{0.f, 0.f, 0.f, 0.f};
  // B fragment offsets (tile-invariant): k-step q -> tap min(2q + lg / 2, 8), channel half lg & 1
  int boff[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int t = min(2 * q + (lg >> 1), 8), r = t / 3, sx = t - 3 * r;
    boff[q] = ((wid + r) * HWX + l16 + sx) * XRB + (lg & 1) * 16;
  }
  const TileWalk walk(ntiles);
  u32x4 rx[XPT];
  auto gload = [&](int tm) __attribute__((always_inline)) {
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
    const int h0 = hb * TR - g.pt, w0 = wb * SEGW - g.pl;
    const uint16_t* img = X + (long long)n * g.H * g.W * 16;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 512 * i, px = idx >> 1;
      const int xrow = px / HWX, xpix = px - xrow * HWX;
      const int hin = h0 + xrow, win = w0 + xpix;
      const bool ok = idx < XG && (unsigned)hin < (unsigned)g.H && (unsigned)win < (unsigned)g.W;
      rx[i] = *reinterpret_cast<const u32x4*>(ok ? img + ((long long)hin * g.W + win) * 16 + (idx & 1) * 8 : zp);
    }
  };
  int tm = walk.tm;
  if (tm < walk.end) gload(tm);
  for (; tm < walk.end; tm += walk.step) {
    __syncthreads();  // every wave is done reading the previous tile's halo
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 512 * i;
      if (idx < XG) *reinterpret_cast<u32x4*>(xs + (idx >> 1) * XRB + (idx & 1) * 16) = rx[i];
    }
    __syncthreads();
    if (tm + walk.step < walk.end) gload(tm + walk.step);
    f4 acc[FM][FN];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      uint4 xb[FM];
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) xb[fm] = *reinterpret_cast<const uint4*>(xs + boff[q] + fm * 16 * XRB);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) mma(acc[fm][fn], wa[q][fn], xb[fm], uint16_t());
    }
    // epilogue (k_conv3x3_narrow's): pixel (row wid, column fm * 16 + l16), channels fn * 16 + lg * 4 + j
    const int n = tm / tpi, rem = tm - n * tpi, hb = rem / tiles_w, wb = rem - hb * tiles_w;
    const int h = hb * TR + wid;
    float sv[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) sv[i] = 0.f;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int w = wb * SEGW + fm * 16 + l16;
      const bool inb = h < g.P && w < g.Q;
      const unsigned pix = ((unsigned)n * g.P + h) * g.Q + w;  // < 2^32: launch checks M * K < 2^32
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int c = fn * 16 + lg * 4;
        float r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = bf2f(f2bf(acc[fm][fn][j] + bq[fn][j]));
        if constexpr (DROP) {
          uint32_t h2[2];
          hash_u32_lo_run<2>(g.drop.seed, (pix * (unsigned)g.K + c) >> 1, h2);
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            const uint32_t hh = h2[pr];
            r[2 * pr] = (hh & 0xFFFFu) >= g.drop.thr ? bf2f(f2bf(r[2 * pr] * g.drop.scl)) : 0.f;
            r[2 * pr + 1] = (hh >> 16) >= g.drop.thr ? bf2f(f2bf(r[2 * pr + 1] * g.drop.scl)) : 0.f;
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float f = inb ? r[j] : 0.f;
          sv[fn * 4 + j] += f;
          sv[FN * 4 + fn * 4 + j] += f * f;
        }
        uint2 v;
        v.x = (__float_as_uint(r[0]) >> 16) | (__float_as_uint(r[1]) & 0xffff0000u);
        v.y = (__float_as_uint(r[2]) >> 16) | (__float_as_uint(r[3]) & 0xffff0000u);
        uint2* dst = inb ? reinterpret_cast<uint2*>(Y + (size_t)pix * g.ldy + c) : &g_store_sink[lane];
        *dst = v;
      }
    }
    if (stats) {
      // reduce-scatter over the 16 pixel lanes: lane l16 keeps values b0 + k of sv
      butterfly_step<NV, 8, 0x128>(sv, lane);
      butterfly_step<NV / 2, 4, 0x141>(sv, lane);
      butterfly_step<NV / 4, 2, 0x4E>(sv, lane);
      butterfly_step<NV / 8, 1, 0xB1>(sv, lane);
#pragma unroll
      for (int k = 0; k < NV / 16; ++k) dstat[k] += (double)sv[k];
    }
  }
  if (stats) {
    // fixed-order sum of the 8 waves' partials (same slots in the same lanes;
    // the halo image is free after the loop)
    __syncthreads();
    double* red = reinterpret_cast<double*>(xs);
#pragma unroll
    for (int k = 0; k < NV / 16; ++k) red[(wid * 64 + lane) * (NV / 16) + k] = dstat[k];
    __syncthreads();
    if (wid == 0) {
      const int b0 = ((l16 >> 3) & 1) * (NV / 2) + ((l16 >> 2) & 1) * (NV / 4) + ((l16 >> 1) & 1) * (NV / 8) +
                     (l16 & 1) * (NV / 16);
#pragma unroll
      for (int k = 0; k < NV / 16; ++k) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < 8; ++w) v += red[(w * 64 + lane) * (NV / 16) + k];
        const int idx = b0 + k, st = idx / (FN * 4), rm = idx - st * (FN * 4);
        stats[((long long)blockIdx.x * 2 + st) * g.Kp + (rm >> 2) * 16 + lg * 4 + (rm & 3)] = v;
      }
    }
    for (int c = KB + tid; c < g.Kp; c += 512)  // (padded channels)
      stats[((long long)blockIdx.x * 2 + 0) * g.Kp + c] = stats[((long long)blockIdx.x * 2 + 1) * g.Kp + c] = 0.0;
    for (int rr = blockIdx.x + gridDim.x; rr < srows; rr += gridDim.x)
      for (int c = tid; c < 2 * g.Kp; c += 512) stats[((long long)rr * 2 + (c / g.Kp)) * g.Kp + (c % g.Kp)] = 0.0;
  }
}

// ------------------------------------------------------------------ 1x1 conv, register-resident weights
// 1x1 stride-1 convolutions with few input or few output channels (C or K <= 32:
// the 16->128 stage-1 entry conv, the 16->64 shortcut, and their dgrads
// 128->16 / 64->16).  These are HBM-streaming problems (a few FLOP per byte),
// so the whole packed weight matrix lives in VGPRs as MFMA A-fragments and each
// wave streams 16-pixel blocks: one 16-B load per lane per 32-channel step,
// v_mfma_f32_16x16x32_bf16 (weights x pixels), then k_conv_fwd_p's epilogue
// (8-byte channel quads, bias, Dropout, BatchNormalization sums kept in
// registers across the whole grid-stride loop and reduced once per wave by the
// DPP butterfly).  C padded to 32 reads zeros from the packed weights and from
// a lane-constant select on the pixel side.
template <int NCS, int NKB>
__global__ void __launch_bounds__(256)
k_conv1x1_reg(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
              const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats) {
  using T = uint16_t;
  constexpr int KB = NKB * 16, NV = 8 * NKB, UNR = 2;
  // wide outputs (K >= 64) go through a wave-private LDS tile so that every
  // global store is 16 B per lane over whole pixel rows (4 rows per wave store)
  constexpr bool WIDE = NKB >= 4;
  constexpr int TROW = KB * 2 + 16;  // padded tile row (bytes): conflict-free 8-B quad writes
  __shared__ double sstat[2 * KB];
  __shared__ float sbias[KB];
  __shared__ __attribute__((aligned(16))) unsigned char stile[WIDE ? 4 * 16 * TROW : 16];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4;
  const int wid = tid >> 6;
  for (int i = tid; i < 2 * KB; i += 256) sstat[i] = 0.0;
  for (int i = tid; i < KB; i += 256) sbias[i] = (bias && i < g.K) ? bias[i] : 0.f;
  uint4 wa[NKB][NCS];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs)
      wa[kb][cs] = *reinterpret_cast<const uint4*>(Wp + (long long)(kb * 16 + l16) * g.Kdp + cs * 32 + q * 8);
  __syncthreads();
  bool cok[NCS];
#pragma unroll
  for (int cs = 0; cs < NCS; ++cs) cok[cs] = cs * 32 + q * 8 < g.C;
  constexpr int NSV = WIDE ? 4 : NV;  // WIDE: lane owns channels 2*lane, 2*lane+1 (sum, sum of squares)
  float sv[NSV];
#pragma unroll
  for (int i = 0; i < NSV; ++i) sv[i] = 0.f;
  const T* zp = reinterpret_cast<const T*>(g_zero_page);
  const long long nblk = (g.M + 15) / 16;
  const long long wstride = (long long)gridDim.x * 4 * UNR;
  for (long long b0 = ((long long)blockIdx.x * 4 + wid) * UNR; b0 < nblk; b0 += wstride) {
    uint4 xb[UNR][NCS];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long px = (b0 + u) * 16 + l16;
      const bool pv = px < g.M;
#pragma unroll
      for (int cs = 0; cs < NCS; ++cs)
        xb[u][cs] = *reinterpret_cast<const uint4*>((pv && cok[cs]) ? X + px * g.C + cs * 32 + q * 8 : zp);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long px = (b0 + u) * 16 + l16;
      const bool inb = px < g.M;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cs = 0; cs < NCS; ++cs) mma(acc, wa[kb][cs], xb[u][cs], T());
        const int c = kb * 16 + q * 4;
        uint16_t hv[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          hv[jj] = f2bf(acc[jj] + sbias[c + jj]);
          if (g.drop.on) hv[jj] = f2bf(drop_apply<T>(g.drop, (uint64_t)px * g.K + c + jj, bf2f(hv[jj])));
          if constexpr (!WIDE) {
            const float f = (inb && c + jj < g.K) ? bf2f(hv[jj]) : 0.f;
            sv[kb * 4 + jj] += f;
            sv[NKB * 4 + kb * 4 + jj] += f * f;
          }
        }
        uint2 v;
        v.x = (unsigned)hv[0] | ((unsigned)hv[1] << 16);
        v.y = (unsigned)hv[2] | ((unsigned)hv[3] << 16);
        if constexpr (WIDE) {
          *reinterpret_cast<uint2*>(stile + wid * 16 * TROW + l16 * TROW + c * 2) = v;
        } else if (inb && c < g.K) {
          *reinterpret_cast<uint2*>(Y + px * g.ldy + c) = v;
        }
      }
      if constexpr (WIDE) {
        // the wave's 16 pixel rows (K channels each) back out as 16-B row segments
        constexpr int LPR = KB / 8;          // lanes per pixel row
        constexpr int RPI = 64 / LPR;        // rows per store instruction
        const long long pxb = (b0 + u) * 16;
        if (stats && 2 * lane < KB) {
#pragma unroll 4
          for (int row = 0; row < 16; ++row) {
            const unsigned pr = *reinterpret_cast<const unsigned*>(stile + wid * 16 * TROW + row * TROW + lane * 4);
            const float f0 = pxb + row < g.M ? __uint_as_float(pr << 16) : 0.f;
            const float f1 = pxb + row < g.M ? __uint_as_float(pr & 0xffff0000u) : 0.f;
            sv[0] += f0;
            sv[1] += f0 * f0;
            sv[2] += f1;
            sv[3] += f1 * f1;
          }
        }
#pragma unroll
        for (int it = 0; it < 16 / RPI; ++it) {
          const int row = it * RPI + lane / LPR, seg = lane % LPR;
          const uint4 v = *reinterpret_cast<const uint4*>(stile + wid * 16 * TROW + row * TROW + seg * 16);
          if (pxb + row < g.M) *reinterpret_cast<uint4*>(Y + (pxb + row) * g.ldy + seg * 8) = v;
        }
      }
    }
  }
  if (stats && WIDE) {
    if (2 * lane < KB) {
      atomicAdd(&sstat[2 * lane], (double)sv[0]);
      atomicAdd(&sstat[KB + 2 * lane], (double)sv[1]);
      atomicAdd(&sstat[2 * lane + 1], (double)sv[2]);
      atomicAdd(&sstat[KB + 2 * lane + 1], (double)sv[3]);
    }
    __syncthreads();
    for (int c = tid; c < g.Kp; c += 256) {
      stats[((long long)blockIdx.x * 2 + 0) * g.Kp + c] = c < KB ? sstat[c] : 0.0;
      stats[((long long)blockIdx.x * 2 + 1) * g.Kp + c] = c < KB ? sstat[KB + c] : 0.0;
    }
  } else if (stats) {
    butterfly_step<NV, 8, 0x128>(sv, lane);
    butterfly_step<NV / 2, 4, 0x141>(sv, lane);
    butterfly_step<NV / 4, 2, 0x4E>(sv, lane);
    butterfly_step<NV / 8, 1, 0xB1>(sv, lane);
    const int b0i = ((l16 >> 3) & 1) * (NV / 2) + ((l16 >> 2) & 1) * (NV / 4) + ((l16 >> 1) & 1) * (NV / 8) +
                    (l16 & 1) * (NV / 16);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV / 16; ++k) {
      const int idx = b0i + k, st = idx / (NKB * 4), rm = idx - st * (NKB * 4);
      const int col = (rm >> 2) * 16 + q * 4 + (rm & 3);
      atomicAdd(&sstat[st * KB + col], (double)sv[k]);
    }
    __syncthreads();
    for (int c = tid; c < g.Kp; c += 256) {
      stats[((long long)blockIdx.x * 2 + 0) * g.Kp + c] = c < KB ? sstat[c] : 0.0;
      stats[((long long)blockIdx.x * 2 + 1) * g.Kp + c] = c < KB ? sstat[KB + c] : 0.0;
    }
  }
}

// ------------------------------------------------------------------ weight packing
// forward:  out[k][(r*S+s)*C + c] = w[k][r][s][c]      (KRSC, zero-padded to [Kp][Kdp])
// flipped:  out[c][(r*S+s)*K + k] = w[k][R-1-r][S-1-s][c]   (dgrad operand)
template <typename T>
__global__ void k_pack_w(const float* __restrict__ w, int K, int R, int S, int C, int flip, int rows_p,
                         int cols_p, T* __restrict__ out) {
  const long long total = (long long)rows_p * cols_p;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int row = (int)(i / cols_p), col = (int)(i - (i / cols_p) * cols_p);
    float v = 0.f;
    if (!flip) {
      if (row < K && col < R * S * C) v = w[(long long)row * R * S * C + col];
    } else {
      if (row < C && col < R * S * K) {
        const int k = col % K, rs = col / K, r = rs / S, s = rs % S;
        v = w[(((long long)k * R + (R - 1 - r)) * S + (S - 1 - s)) * C + row];
      }
    }
    out[i] = cvt_out(v, T());
  }
}

// All conv weights of a training step in one launch (acfe_conv2d_pack_weights_batch):
// the descriptor table lists each (weight, orientation) with its packed
// geometry and its first element in the concatenated index space; a thread
// finds its descriptor by binary search over the table's start offsets (in LDS).
struct PackDesc {
  const float* w;
  void* out;
  long long begin;
  int K, R, S, C, flip, rows_p, cols_p, pad;
};
static_assert(sizeof(PackDesc) == 56, "PackDesc layout (acfe/ops.py WeightPacker)");

template <typename T>
__global__ void __launch_bounds__(256) k_pack_w_batch(const PackDesc* __restrict__ d, int n, long long total) {
  __shared__ long long beg[257];
  for (int i = threadIdx.x; i <= n; i += 256) beg[i] = i < n ? d[i].begin : total;
  __syncthreads();
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (beg[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const PackDesc& p = d[lo];
    const long long e = i - beg[lo];
    const int row = (int)(e / p.cols_p), col = (int)(e - (e / p.cols_p) * p.cols_p);
    float v = 0.f;
    if (!p.flip) {
      if (row < p.K && col < p.R * p.S * p.C) v = p.w[(long long)row * p.R * p.S * p.C + col];
    } else {
      if (row < p.C && col < p.R * p.S * p.K) {
        const int k = col % p.K, rs = col / p.K, r = rs / p.S, s = rs % p.S;
        v = p.w[(((long long)k * p.R + (p.R - 1 - r)) * p.S + (p.S - 1 - s)) * p.C + row];
      }
    }
    reinterpret_cast<T*>(p.out)[e] = cvt_out(v, T());
  }
}


// ------------------------------------------------------------------ wgrad
// Block: 256 threads; output tile BMW (k rows) x 128 (rsc cols); reduction over
// a contiguous chunk of pixels m in steps of BR (64 for bf16 = two MFMA
// k-chunks per barrier, 32 for fp32).  LDS images are m-major:
// Ds[BR][BMW + 16], Xs[BR][128 + 16]; register staging (straight-line code:
// no closures, so the staging arrays stay in VGPRs), zero-page loads for
// padding taps and tails.
template <typename T, int BMW, bool FAST_D, bool FAST_X>
__global__ void __launch_bounds__(256)
k_conv_wgrad(ConvGeom g, const T* __restrict__ X, const T* __restrict__ dY, float* __restrict__ ws,
             long long chunk, int tiles_x, int tiles_y) {
  constexpr int GR = TT<T>::GR, BNW = 128, BR = sizeof(T) == 2 ? 64 : 32;
  constexpr int LDD = BMW + 16, LDX = BNW + 16;
  constexpr int WM = BMW >= 64 ? 2 : 1, WN = 4 / WM;
  constexpr int TWM = BMW / WM, TWN = BNW / WN, FM = TWM / 16, FN = TWN / 16;
  constexpr int DG = BR * BMW / GR, XG = BR * BNW / GR;  // granules per stage
  constexpr int DPT = (DG + 255) / 256, XPT = XG / 256;
  static_assert(XG % 256 == 0, "x tile");
  __shared__ __attribute__((aligned(16))) T Ds[2][BR * LDD];
  __shared__ __attribute__((aligned(16))) T Xs[2][BR * LDX];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  // 1-D grid of tiles_x * tiles_y * splits (splits % 8 == 0): the workgroups
  // of one pixel chunk (same dY rows, overlapping X rows) all land on one XCD
  // (linear id % 8) and share its L2; split = 8 * (i / T) + xcd.
  const int T_ = tiles_x * tiles_y, xcd = blockIdx.x & 7, bi = blockIdx.x >> 3;
  const int tile = bi % T_, split = (bi / T_) * 8 + xcd;
  const int k0 = (tile / tiles_x) * BMW, c0blk = (tile % tiles_x) * BNW;
  const long long mbeg = (long long)split * chunk;
  long long mend = mbeg + chunk;
  if (mend > g.M) mend = g.M;
  const int nsteps = mbeg < mend ? (int)((mend - mbeg + BR - 1) / BR) : 0;
  const long long PQ = (long long)g.P * g.Q;
  const T* zp = reinterpret_cast<const T*>(g_zero_page);

  constexpr int XGPR = BNW / GR, DGPR = BMW / GR;
  int xrow[XPT], xr[XPT], xs[XPT], xc[XPT], xn[XPT], xp[XPT], xq[XPT];
  bool xkv[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int idx = tid + 256 * i;
    xrow[i] = idx / XGPR;
    const int cg = idx - xrow[i] * XGPR;
    const int kk = c0blk + cg * GR;
    xkv[i] = kk < g.Kd;
    const int kkc = xkv[i] ? kk : 0;
    const int rs = kkc / g.C;
    xc[i] = kkc - rs * g.C;
    xr[i] = rs / g.S;
    xs[i] = rs - xr[i] * g.S;
    const long long m = mbeg + xrow[i];
    const int n = (int)(m / PQ);
    const int rem = (int)(m - (long long)n * PQ);
    xn[i] = n;
    xp[i] = rem / g.Q;
    xq[i] = rem - xp[i] * g.Q;
  }
  u32x4 rd[DPT], rx[XPT];
  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  if (nsteps > 0) {
#define STEPV 0
#define BUFV 0

  {
    const long long mb = mbeg + (long long)(STEPV) * BR;
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / DGPR, cg = idx - (idx / DGPR) * DGPR;
      const long long m = mb + row;
      const bool ok = idx < DG && m < mend;
      if constexpr (FAST_D) {
        const bool okk = ok && (k0 + cg * GR) < g.K;
        rd[i] = *reinterpret_cast<const u32x4*>(okk ? dY + m * g.ldy + k0 + cg * GR : zp);
      } else {
        T e[GR];
#pragma unroll
        for (int j = 0; j < GR; ++j) {
          const int k = k0 + cg * GR + j;
          const bool okk = ok && k < g.K;
          e[j] = *(okk ? dY + m * g.ldy + k : zp);
        }
        rd[i] = *reinterpret_cast<const u32x4*>(e);
      }
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const long long m = mb + xrow[i];
      const int h = xp[i] * g.st - g.pt + xr[i], w = xq[i] * g.st - g.pl + xs[i];
      const bool ok = xkv[i] && m < mend && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      if constexpr (FAST_X) {
        rx[i] = *reinterpret_cast<const u32x4*>(ok ? X + (((long long)xn[i] * g.H + h) * g.W + w) * g.C + xc[i] : zp);
      } else {
        T e[GR];
        const int cg = (tid + 256 * i) - xrow[i] * XGPR;
#pragma unroll
        for (int j = 0; j < GR; ++j) {
          const int kk = c0blk + cg * GR + j;
          bool okj = kk < g.Kd && m < mend;
          const int rs = kk / g.C, c = kk - rs * g.C, rq = rs / g.S, sq = rs - rq * g.S;
          const int hh = xp[i] * g.st - g.pt + rq, ww = xq[i] * g.st - g.pl + sq;
          okj = okj && (unsigned)hh < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
          e[j] = *(okj ? X + (((long long)xn[i] * g.H + hh) * g.W + ww) * g.C + c : zp);
        }
        rx[i] = *reinterpret_cast<const u32x4*>(e);
      }
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      xq[i] += BR;
      while (xq[i] >= g.Q) {
        xq[i] -= g.Q;
        if (++xp[i] == g.P) { xp[i] = 0; ++xn[i]; }
      }
    }
  }

  {
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int idx = tid + 256 * i;
      if (idx < DG) {
        const int row = idx / DGPR, cg = idx - (idx / DGPR) * DGPR;
        *reinterpret_cast<u32x4*>(&Ds[BUFV][row * LDD + cg * GR]) = rd[i];
      }
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 256 * i;
      const int cg = idx - xrow[i] * XGPR;
      *reinterpret_cast<u32x4*>(&Xs[BUFV][xrow[i] * LDX + cg * GR]) = rx[i];
    }
  }

#undef STEPV
#undef BUFV
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const bool more = step + 1 < nsteps;
    if (more) {
#define STEPV (step + 1)

  {
    const long long mb = mbeg + (long long)(STEPV) * BR;
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / DGPR, cg = idx - (idx / DGPR) * DGPR;
      const long long m = mb + row;
      const bool ok = idx < DG && m < mend;
      if constexpr (FAST_D) {
        const bool okk = ok && (k0 + cg * GR) < g.K;
        rd[i] = *reinterpret_cast<const u32x4*>(okk ? dY + m * g.ldy + k0 + cg * GR : zp);
      } else {
        T e[GR];
#pragma unroll
        for (int j = 0; j < GR; ++j) {
          const int k = k0 + cg * GR + j;
          const bool okk = ok && k < g.K;
          e[j] = *(okk ? dY + m * g.ldy + k : zp);
        }
        rd[i] = *reinterpret_cast<const u32x4*>(e);
      }
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const long long m = mb + xrow[i];
      const int h = xp[i] * g.st - g.pt + xr[i], w = xq[i] * g.st - g.pl + xs[i];
      const bool ok = xkv[i] && m < mend && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      if constexpr (FAST_X) {
        rx[i] = *reinterpret_cast<const u32x4*>(ok ? X + (((long long)xn[i] * g.H + h) * g.W + w) * g.C + xc[i] : zp);
      } else {
        T e[GR];
        const int cg = (tid + 256 * i) - xrow[i] * XGPR;
#pragma unroll
        for (int j = 0; j < GR; ++j) {
          const int kk = c0blk + cg * GR + j;
          bool okj = kk < g.Kd && m < mend;
          const int rs = kk / g.C, c = kk - rs * g.C, rq = rs / g.S, sq = rs - rq * g.S;
          const int hh = xp[i] * g.st - g.pt + rq, ww = xq[i] * g.st - g.pl + sq;
          okj = okj && (unsigned)hh < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
          e[j] = *(okj ? X + (((long long)xn[i] * g.H + hh) * g.W + ww) * g.C + c : zp);
        }
        rx[i] = *reinterpret_cast<const u32x4*>(e);
      }
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      xq[i] += BR;
      while (xq[i] >= g.Q) {
        xq[i] -= g.Q;
        if (++xp[i] == g.P) { xp[i] = 0; ++xn[i]; }
      }
    }
  }

#undef STEPV
    }
    const int buf = step & 1;
#pragma unroll
    for (int kc = 0; kc < BR / 32; ++kc) {
      if constexpr (sizeof(T) == 2) {
        // MFMA k-slot (g = lane>>4, j) <-> m: j<4: 4g+j, j>=4: 16+4g+(j-4)  (within this 32-row chunk)
        const int grp = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
        const int rb = kc * 32;
        typedef __attribute__((address_space(3))) bf4* lp;
        bf8 af[FM], bfr[FN];
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int col = wm * TWM + fm * 16 + 4 * p;
          const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lp)(reinterpret_cast<const __bf16*>(&Ds[buf][(rb + 4 * grp + q) * LDD + col])));
          const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lp)(reinterpret_cast<const __bf16*>(&Ds[buf][(rb + 16 + 4 * grp + q) * LDD + col])));
          af[fm] = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int col = wn * TWN + fn * 16 + 4 * p;
          const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lp)(reinterpret_cast<const __bf16*>(&Xs[buf][(rb + 4 * grp + q) * LDX + col])));
          const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lp)(reinterpret_cast<const __bf16*>(&Xs[buf][(rb + 16 + 4 * grp + q) * LDX + col])));
          bfr[fn] = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[fm], bfr[fn], acc[fm][fn], 0, 0, 0);
      } else {
#pragma unroll
        for (int k4 = 0; k4 < 8; ++k4) {
          const int mrow = kc * 32 + k4 * 4 + (lane >> 4);
          float a[FM], b[FN];
#pragma unroll
          for (int fm = 0; fm < FM; ++fm)
            a[fm] = reinterpret_cast<const float*>(Ds[buf])[mrow * LDD + wm * TWM + fm * 16 + (lane & 15)];
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            b[fn] = reinterpret_cast<const float*>(Xs[buf])[mrow * LDX + wn * TWN + fn * 16 + (lane & 15)];
#pragma unroll
          for (int fm = 0; fm < FM; ++fm)
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
              acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[fm], b[fn], acc[fm][fn], 0, 0, 0);
        }
      }
    }
    if (more) {
#define BUFV (buf ^ 1)

  {
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int idx = tid + 256 * i;
      if (idx < DG) {
        const int row = idx / DGPR, cg = idx - (idx / DGPR) * DGPR;
        *reinterpret_cast<u32x4*>(&Ds[BUFV][row * LDD + cg * GR]) = rd[i];
      }
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 256 * i;
      const int cg = idx - xrow[i] * XGPR;
      *reinterpret_cast<u32x4*>(&Xs[BUFV][xrow[i] * LDX + cg * GR]) = rx[i];
    }
  }

#undef BUFV
    }
    __syncthreads();
  }
  // partial slab: ws[z][k][kk] (k < K, kk < Kd)
  float* out = ws + (long long)split * g.K * g.Kd;
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + wm * TWM + fm * 16 + (lane >> 4) * 4 + j;
        const int kk = c0blk + wn * TWN + fn * 16 + (lane & 15);
        if (k < g.K && kk < g.Kd) out[(long long)k * g.Kd + kk] = acc[fm][fn][j];
      }
}

// sum of split slabs -> dW (optionally accumulated, optionally replicated over
// `rep` input channels for the folded stem)
// ------------------------------------------------------------------ wgrad, 3x3 stride 1, halo-staged
// dW[k][r][s][c] for the 3x3 stride-1 layers with C % 64 == 0, K in {64, 128}
// (wr_resnet_bird stages 1-2: ~70 % of the step's wgrad time; a partial last
// 64-pixel segment of a row reads zeros past Q).
// A workgroup owns one 64-channel chunk and ALL nine taps (output tile
// K x 576) and reduces over a contiguous range of 64-pixel output-row segments
// (split-K over pixels, slabs combined by k_wgrad_reduce).  Per segment it
// stages dY[64 px][K] and the input halo X[3 rows][66 px][64 ch] in LDS ONCE;
// the nine taps are shifted views of the halo (the im2col kernel re-reads every
// input pixel nine times).  Per 64-pixel step each wave runs 72 MFMAs (vs 32),
// so the per-step synchronisation is amortised over 4.5x the matrix work.
// LDS images are pixel-major with rows padded to 160 / 288 B so the
// ds_read_b64_tr_b16 fragment reads (8 pixel rows x 32 B per half-wave) hit 64
// distinct banks; register-staged double buffer, one barrier per step.
// UNP: dY is the 2x2 max-pool backward of the pooled gradient dY (argmax bytes
// amax), expanded while staging.
// NR: output rows per pipeline step (a "segment" = NR rows x 64 pixels, P % NR
// == 0): NR = 2 doubles the MFMAs per barrier for K = 64 (36 -> 72 per wave),
// the halo then being NR + 2 input rows.
// BWD (acfe_conv2d_wgrad_bnbwd): dY is not stored; the kernel stages the
// output gradient of the BatchNormalization (+ReLU) -> Dropout that follows the
// conv and that BN's input x, forms dY = Dropout'(a g [x sc + sh > 0] + b x + c)
// exactly as acfe_bn_bwd_apply_ex rounds and drops it, writes it (g.fb_out: the
// dgrad reads it next) and sums it per channel (the conv bias gradient) -- the
// BN backward apply pass over the tensor is gone.  Each dY element is staged
// by one workgroup of chunk 0 (the others only read it).
// SEGW: segment width -- 64 (NR rows x 64 pixels), or 16 (4 NR rows x 16
// pixels) for the Q % 64 pixels left of each row, launched separately over
// qs segment columns from column wofs, with the same grid, adding (wadd) its
// partial slabs and BWD channel-sum rows into the first launch's (wr_resnet's
// 513- / 257-wide stages otherwise run a whole 64-pixel segment per row group
// for the last pixel).
template <int KB, bool UNP, int CW = 64, int NR = 1, bool BWD = false, bool KEEP = false, int SEGW = 64>
__global__ void __launch_bounds__(512, 1)
k_wgrad3x3_halo(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ dY,
                float* __restrict__ ws, int nchunk, int nseg, int segs_per_split, const uint8_t* __restrict__ amax,
                int qs = 0, int wofs = 0, int wadd = 0) {
  static_assert(!(BWD && UNP), "BN backward fold: plain dY");
  // KEEP: the dropout keep bits of the forward (g.keep_in, one byte per 8-channel
  // granule) instead of the regenerated pair hashes (9 quarter-rate multiplies
  // per granule)
  static_assert(!KEEP || BWD, "keep bits: the BN-fold wgrad");
#ifndef ACFE_FB_MID
#define ACFE_FB_MID 0
#endif
  constexpr int FBMID = ACFE_FB_MID < 2 * NR ? ACFE_FB_MID : 0;
  static_assert(SEGW == 64 || SEGW == 16, "segment width");
  // ROWS output rows per segment (SEGW 16: four times NR, the same 64 NR pixels)
  constexpr int ROWS = SEGW == 64 ? NR : 4 * NR, HW = SEGW + 2, HR = ROWS + 2;
  // CW-channel chunks (C = 16 / 32 layers: the stage-2/3 branch2b): the 8 waves
  // are WC = CW / 16 channel blocks x WK = 8 / WC slices of K; a wave's nine
  // blocks are the nine taps of its channel block (CW = 64: 2 K halves x 4
  // groups of 9 (tap, block) pairs)
  // CW = 128 (K = 16: wr_resnet_bird's stage-3 branch21, 256 -> 16): the 8
  // waves are the 8 channel blocks of the chunk, each all 16 K rows x 9 taps.
  // K < 16 * 8 / WC (wr_resnet's stage-1 conv2a, 16 -> 64): WP pixel groups
  // of waves take alternate 32-pixel halves and write separate split slabs
  // (the combine adds them like any other split).
  static_assert(CW == 64 || (CW == 32 && !UNP) || (CW == 16 && !UNP) || (CW == 128 && KB == 16 && !UNP), "chunk");
  constexpr int WC = CW == 64 ? 4 : CW / 16;
  constexpr int WK = 8 / WC < KB / 16 ? 8 / WC : KB / 16, WP = 8 / (WC * WK);
  static_assert(WC * WK * WP == 8 && (2 * NR) % WP == 0, "wave split");
  static_assert(SEGW == 64 || !UNP, "16-pixel segments: plain dY");
  constexpr int LDD = KB + 16, LDX = CW + 16;
  constexpr int DS = ROWS * SEGW * LDD, XS = HR * HW * LDX;
  constexpr int FM = KB / (16 * WK), FN = 9;
  static_assert(FM >= 1, "K slice");
  constexpr int XGR = CW / 8;
  constexpr int DGR = KB / 8, DG = ROWS * SEGW * DGR, XG = HR * HW * XGR;
  constexpr int DPT = (DG + 511) / 512, XPT = (XG + 511) / 512;
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (DS + XS)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wp = wid / (WC * WK), wkc = wid - wp * (WC * WK);
  const int wk = wkc / WC, wc = wkc - (wkc / WC) * WC;
  const int xcd = blockIdx.x & 7, bi = blockIdx.x >> 3;
  const int cc = bi % nchunk, split = (bi / nchunk) * 8 + xcd;
  const int sbeg = split * segs_per_split;
  const int send = sbeg + segs_per_split < nseg ? sbeg + segs_per_split : nseg;
  // segment columns (the last one may be partial)
  const int QS = qs > 0 ? qs : (g.Q + SEGW - 1) / SEGW;
  const T16* zp = reinterpret_cast<const T16*>(g_zero_page);
  // BWD: [scale | shift | a | b | c][KB] and the channel sums of this workgroup
  __shared__ float ftab[BWD ? 5 * KB : 1];
  __shared__ double fsum[BWD ? KB : 1];
  if constexpr (BWD) {
    for (int i = tid; i < 5 * KB; i += 512)
      ftab[i] = i < KB ? g.fb_sc[i] : (i < 2 * KB ? g.fb_sh[i - KB] : g.fb_coef[i - 2 * KB]);
    for (int i = tid; i < KB; i += 512) fsum[i] = 0.0;
    __syncthreads();  // (read by the first sstore)
  }
  // BWD: this thread's 8 channels are fixed (cg = tid % DGR: 512 is a multiple
  // of DGR), so their 5 x 8 coefficients stay in registers across the walk
  // instead of 10 LDS reads per staged granule
  f4 fcv[BWD ? 10 : 1];
  if constexpr (BWD) {
    const f4* tb = reinterpret_cast<const f4*>(ftab + (tid % (KB / 8)) * 8);
#pragma unroll
    for (int q5 = 0; q5 < 5; ++q5) fcv[2 * q5] = tb[q5 * (KB / 4)], fcv[2 * q5 + 1] = tb[q5 * (KB / 4) + 1];
  }

  u32x4 rd[DPT], rx[XPT];
  uint2 rda[UNP ? DPT : 1];  // UNP: argmax bytes + window taps, applied at the LDS store
  unsigned dpos = 0;
  // BWD: the BN input x at the staged dY granules, the staged segment's first
  // element index and column, and the lane's channel sums (its 8 channels
  // cg * 8 + j are fixed: 512 is a multiple of DGR)
  u32x4 rdx[BWD ? DPT : 1], rdr[BWD ? DPT : 1];  // BN input x, residual gradient
  unsigned rkb[KEEP ? DPT : 1];                  // KEEP: the granules' keep-bit bytes
  long long fbase = 0;
  int fw0 = 0;
  float fs[BWD ? 8 : 1];
#pragma unroll
  for (int j = 0; j < (BWD ? 8 : 1); ++j) fs[j] = 0.f;
  // part bit 0: the dY granules, bit 1: the input halo granules
  // lane constants of the staging granules (segment independent): dY
  // granule i = pixel (ro, pw) of the segment, channels cg * 8; halo granule i
  // = halo row hr, pixel hp, channels cg * 8.  A step's offsets are a scalar
  // segment base plus these -- no per-step lane multiplies (v_mul_lo_u32 is
  // quarter rate); granules past the tile get a row / pixel that fails the
  // bounds test.
  int dlo[DPT], dro[DPT], dpw[DPT];
#pragma unroll
  for (int i = 0; i < DPT; ++i) {
    const int idx = tid + 512 * i;
    const int px = idx / DGR, cg = idx - px * DGR, ro = px / SEGW, pw = px - ro * SEGW;
    dro[i] = ro;
    dpw[i] = idx < DG ? pw : (1 << 24);
    dlo[i] = UNP ? (pw >> 1) * g.K + cg * 8 : (ro * g.Q + pw) * g.K + cg * 8;
  }
  int xlo[XPT], xhr[XPT], xhp[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int idx = tid + 512 * i;
    const int hr = idx / (HW * XGR), r2 = idx - hr * (HW * XGR), hp = r2 / XGR, cg = r2 - hp * XGR;
    xhr[i] = idx < XG ? hr : (1 << 24);
    xhp[i] = hp;
    xlo[i] = (hr * g.W + hp) * g.C + cc * CW + cg * 8;
  }
  auto gload = [&](int sg, int part = 3) __attribute__((always_inline)) {
    // segments walk down a 64-pixel column (row fastest): consecutive steps
    // share NR + 1 of their NR + 2 halo rows (and, UNP, their pooled dY row),
    // so the overlap is re-read from L2 one step later instead of a whole
    // image row later (r03v: 9.8 GB of HBM reads per launch vs 5.9 GB algorithmic)
    // row groups per image (SEGW 16: the last may be partial, its rows past
    // P loading zeros -- the plain kernels only; launcher)
    const int PR = SEGW == 64 ? g.P / ROWS : (g.P + ROWS - 1) / ROWS;
    const int n = sg / (PR * QS), rem = sg - n * (PR * QS);
    const int h = (rem % PR) * ROWS, w0 = wofs + (rem / PR) * SEGW;
    // buffer loads on the segment's image (offsets < 2^31: halo_ok); an
    // element outside the image or the tile takes the out-of-range offset,
    // which loads zeros -- no 64-bit address arithmetic, no branches
    constexpr unsigned OOR = 0x80000000u;
    const long long imgy = UNP ? (long long)n * (g.P >> 1) * (g.Q >> 1) * g.K : (long long)n * g.P * g.Q * g.K;
    const int nby = UNP ? (g.P >> 1) * (g.Q >> 1) * g.K : g.P * g.Q * g.K;
    const __amdgpu_buffer_rsrc_t yrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(dY + imgy), (short)0, nby * 2, 0x00020000);
    // UNP: (h + ro) >> 1 == h >> 1 (NR <= 2, h a multiple of NR) and
    // (w0 + pw) >> 1 == w0 / 2 + pw >> 1 (w0 a multiple of 64)
    const int dbase = UNP ? ((h >> 1) * (g.Q >> 1) + (w0 >> 1)) * g.K : (h * g.Q + w0) * g.K;
#pragma unroll
    for (int i = 0; i < ((part & 1) ? DPT : 0); ++i) {
      const bool okd = (w0 + dpw[i] < g.Q) && (SEGW == 64 || h + dro[i] < g.P);
      const unsigned e = (unsigned)(dbase + dlo[i]);
      if constexpr (UNP) {
        const __amdgpu_buffer_rsrc_t ars =
            __builtin_amdgcn_make_buffer_rsrc((void*)(amax + imgy), (short)0, nby, 0x00020000);
        rd[i] = __builtin_amdgcn_raw_buffer_load_b128(yrs, okd ? e * 2u : OOR, 0, 0);
        const auto a8 = __builtin_amdgcn_raw_buffer_load_b64(ars, okd ? e : OOR, 0, 0);
        rda[i] = uint2{a8[0], a8[1]};
        if (i == 0) dpos = 0;
        dpos |= (unsigned)((((h + dro[i]) & 1) << 1) | (dpw[i] & 1)) << (2 * i);
      } else {
        rd[i] = __builtin_amdgcn_raw_buffer_load_b128(yrs, okd ? e * 2u : OOR, 0, 0);
        if constexpr (BWD) {
          const long long e0 = (((long long)n * g.P + h) * g.Q + w0) * g.K;
          const __amdgpu_buffer_rsrc_t brs =
              __builtin_amdgcn_make_buffer_rsrc((void*)(g.fb_x + imgy), (short)0, nby * 2, 0x00020000);
          rdx[i] = __builtin_amdgcn_raw_buffer_load_b128(brs, okd ? e * 2u : OOR, 0, 0);
          if (g.fb_add) {
            const __amdgpu_buffer_rsrc_t rrs =
                __builtin_amdgcn_make_buffer_rsrc((void*)(g.fb_add + imgy), (short)0, nby * 2, 0x00020000);
            rdr[i] = __builtin_amdgcn_raw_buffer_load_b128(rrs, okd ? e * 2u : OOR, 0, 0);
          }
          if constexpr (KEEP) {  // byte e / 8 of the image's [P Q][K / 8] keep bits (e: a granule start)
            const __amdgpu_buffer_rsrc_t krs =
                __builtin_amdgcn_make_buffer_rsrc((void*)(g.keep_in + imgy / 8), (short)0, nby / 8, 0x00020000);
            rkb[i] = __builtin_amdgcn_raw_buffer_load_b8(krs, okd ? e >> 3 : OOR, 0, 0);
          }
          if (i == 0) fbase = e0, fw0 = w0;
        }
      }
    }
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(X + (long long)n * g.H * g.W * g.C), (short)0, g.H * g.W * g.C * 2, 0x00020000);
    const int hx = h - g.pt, wx = w0 - g.pl, xbase = (hx * g.W + wx) * g.C;
#pragma unroll
    for (int i = 0; i < ((part & 2) ? XPT : 0); ++i) {
      const bool ok = (unsigned)(hx + xhr[i]) < (unsigned)g.H && (unsigned)(wx + xhp[i]) < (unsigned)g.W;
      rx[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, ok ? (unsigned)(xbase + xlo[i]) * 2u : OOR, 0, 0);
    }
  };
  auto sstore = [&](int buf) __attribute__((always_inline)) {
    uint16_t* Ds = smem + buf * (DS + XS);
    uint16_t* Xh = Ds + DS;
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int idx = tid + 512 * i;
      const int px = idx / DGR, cg = idx - px * DGR;
      if constexpr (UNP) {
        if (idx < DG)
          *reinterpret_cast<u32x4*>(Ds + px * LDD + cg * 8) = rd[i] & unpool_mask(rda[i], (dpos >> (2 * i)) & 3u);
      } else if constexpr (BWD) {
        // acfe_bn_bwd_apply_ex's arithmetic per element (k_bn_bwd_apply8):
        // g masked by the BN's ReLU, a g + b x + c, rounded to bf16, then the
        // Dropout backward of the rounded value (keep: round(v * scale))
        // (the granule's lane constants: dpw fails the column test past the
        // tile, dlo = (ro Q + pw) K + cg 8)
        const bool ok = fw0 + dpw[i] < g.Q;
        const long long e = fbase + dlo[i];
        u32x4 v;
        // one pair hash per dword (channels 2d, 2d + 1; e is even), the four
        // from one Weyl multiply when the indices fit 32 bits
        uint32_t hl[4] = {0u, 0u, 0u, 0u};
        if (!KEEP && g.drop.on) {
          if (g.idx32) {
            hash_u32_lo_run<4>(g.drop.seed, (uint32_t)((uint64_t)e >> 1), hl);
          } else {
#pragma unroll
            for (int d = 0; d < 4; ++d) hl[d] = hash_u32(g.drop.seed, ((uint64_t)e >> 1) + d);
          }
        }
        // straight-line, one channel pair per packed-f32 op (r06: the
        // per-element select of the dropout arm compiled to 16 exec-mask
        // branches per step): the pair's words and masks are selected
        // bitwise, the roundings are v_cvt_pk_bf16_f32 of the pair -- the
        // same values element by element
        const unsigned okm = ok ? ~0u : 0u;
        const bool relu1 = (g.fb_relu & 1) != 0, relu2 = (g.fb_relu & 2) != 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const f4 sc = fcv[d >> 1], sh = fcv[2 + (d >> 1)], ca = fcv[4 + (d >> 1)], cb = fcv[6 + (d >> 1)],
                   c0 = fcv[8 + (d >> 1)];
          const int jj = (d & 1) * 2;
          const unsigned xw = rdx[i][d], gw = rd[i][d];
          const f2v xv = {__uint_as_float(xw << 16), __uint_as_float(xw & 0xffff0000u)};
          const f2v gv = {__uint_as_float(gw << 16), __uint_as_float(gw & 0xffff0000u)};
          const f2v t = __builtin_elementwise_fma(xv, (f2v){sc[jj], sc[jj + 1]}, (f2v){sh[jj], sh[jj + 1]});
          const f2v gj = {(relu1 && !(t.x > 0.f)) ? 0.f : gv.x, (relu1 && !(t.y > 0.f)) ? 0.f : gv.y};
#ifdef ACFE_FB_NOXFORM
          f2v o = gv;
#else
          f2v o = __builtin_elementwise_fma(
              (f2v){ca[jj], ca[jj + 1]}, gj,
              __builtin_elementwise_fma((f2v){cb[jj], cb[jj + 1]}, xv, (f2v){c0[jj], c0[jj + 1]}));
#endif
          if (g.fb_add) {
            const unsigned rw = rdr[i][d];
            o += (f2v){__uint_as_float(rw << 16), __uint_as_float(rw & 0xffff0000u)};
          }
          // x = a ReLU output upstream: its backward
          o.x = (relu2 && !(xv.x > 0.f)) ? 0.f : o.x;
          o.y = (relu2 && !(xv.y > 0.f)) ? 0.f : o.y;
          unsigned w = pk_bf2(o.x, o.y);
          unsigned km = okm;
          if (KEEP || g.drop.on) {
            // the rounded pair times the keep scale, rounded again; the keep
            // bits (bit 2d / 2d + 1 of the granule's byte, or the pair hash's
            // halves against the threshold) as a 16-bit-per-element mask
            const f2v r = (f2v){__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)} * g.drop.scl;
            w = pk_bf2(r.x, r.y);
            unsigned klo, khi;
            if constexpr (KEEP) {
              klo = (unsigned)((int)(rkb[i] << (31 - 2 * d)) >> 31);
              khi = (unsigned)((int)(rkb[i] << (30 - 2 * d)) >> 31);
            } else {
              klo = (hl[d] & 0xFFFFu) >= g.drop.thr ? ~0u : 0u;
              khi = (hl[d] >> 16) >= g.drop.thr ? ~0u : 0u;
            }
            km &= (klo & 0x0000ffffu) | (khi & 0xffff0000u);
          }
          w &= km;
#ifndef ACFE_FB_NOSUM
          fs[2 * d] += __uint_as_float(w << 16);
          fs[2 * d + 1] += __uint_as_float(w & 0xffff0000u);
#endif
          v[d] = w;
        }
        if (idx < DG) *reinterpret_cast<u32x4*>(Ds + px * LDD + cg * 8) = v;
#ifndef ACFE_FB_NOSTORE
        if (ok && g.fb_out && cc == 0) *reinterpret_cast<u32x4*>(g.fb_out + e) = v;
#endif
      } else {
        if (idx < DG) *reinterpret_cast<u32x4*>(Ds + px * LDD + cg * 8) = rd[i];
      }
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 512 * i;
      const int row = idx / XGR, cg = idx - row * XGR;  // row = hr * HW + hp
      if (idx < XG) *reinterpret_cast<u32x4*>(Xh + row * LDX + cg * 8) = rx[i];
    }
  };

  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // this wave's nine 16-column blocks: block b = wc * 9 + fn -> tap b / 4, channels (b % 4) * 16
  int boff[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int b = wc * 9 + fn, t = CW == 64 ? b >> 2 : fn, cb = CW == 64 ? b & 3 : wc;
    boff[fn] = ((t / 3) * HW + (t % 3)) * LDX + cb * 16;
  }
  const int grp = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  typedef __attribute__((address_space(3))) bf4* lp;

  // BWD: the lanes' channel sums over the 64 / DGR lanes of a wave that hold
  // the same channels, added into the workgroup's LDS doubles (every 16
  // segments: f32 partials of at most 16 * DPT values)
  auto fflush = [&]() __attribute__((always_inline)) {
    if constexpr (BWD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = fs[j];
#pragma unroll
        for (int m = DGR; m < 64; m <<= 1) v += __shfl_xor(v, m, 64);
        if (lane < DGR) atomicAdd(&fsum[lane * 8 + j], (double)v);
        fs[j] = 0.f;
      }
    }
  };
  if (sbeg < send) {
    gload(sbeg);
    sstore(0);
  }
  __syncthreads();
  int buf = 0;
  // WGI: the next segment's input-halo loads are issued after the first
  // 32-pixel half's MFMAs (their issue stalls then overlap MFMA work)
  // (K = 64: no measurable difference, r02as: 0.518-0.522 vs 0.521-0.530 ms)
  constexpr bool WGI = KB >= 128;
  static_assert(!WGI || WP == 1, "split halves");
  for (int sg = sbeg; sg < send; ++sg) {
    const bool more = sg + 1 < send;
    if (more) gload(sg + 1, WGI ? 1 : 3);
    const uint16_t* Ds = smem + buf * (DS + XS);
    const uint16_t* Xh = Ds + DS;
#pragma unroll
    for (int kq = WP > 1 ? wp : 0; kq < 2 * NR; kq += WP) {
      const int kc = kq & 1, ro = kq >> 1;  // 32-pixel half, output row of the group
      if constexpr (WGI) {
        if (kq == NR) {
          __builtin_amdgcn_sched_barrier(0);
          if (more) gload(sg + 1, 2);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // BWD: the next segment's dY transform (and LDS store into the other
      // buffer) between the MFMA halves, so its VALU runs beside the partner
      // wave's MFMAs instead of after every wave's MFMAs (FBMID)
      if constexpr (BWD && FBMID) {
        if (kq == FBMID) {
          if (more) sstore(buf ^ 1);
        }
      }
      const int rb = kq * 32;  // dY pixel row of this half (SEGW 64: row ro, pixels kc 32 ..)
      // its first pixel's halo offset (tap offsets in boff) and that of its
      // second 16 pixels (SEGW 64: the same row, 16 on; 16: the next row)
      const int xr = SEGW == 64 ? ro * HW + kc * 32 : 2 * kq * HW;
      constexpr int XH = SEGW == 64 ? 16 : HW;
      bf8 af[FM];
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int col = wk * (KB / WK) + fm * 16 + 4 * pp;
        const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lp)(reinterpret_cast<const __bf16*>(Ds + (rb + 4 * grp + q) * LDD + col)));
        const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lp)(reinterpret_cast<const __bf16*>(Ds + (rb + 16 + 4 * grp + q) * LDD + col)));
        af[fm] = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const uint16_t* xb = Xh + boff[fn] + 4 * pp;
        const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lp)(reinterpret_cast<const __bf16*>(xb + (xr + 4 * grp + q) * LDX)));
        const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lp)(reinterpret_cast<const __bf16*>(xb + (xr + XH + 4 * grp + q) * LDX)));
        const bf8 bv = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[fm], bv, acc[fm][fn], 0, 0, 0);
      }
    }
    if constexpr (!BWD || !FBMID) {
      if (more) sstore(buf ^ 1);
    }
    if constexpr (BWD) {
      if (((sg - sbeg) & 15) == 15) fflush();
    }
    __syncthreads();
    buf ^= 1;
  }
  if constexpr (BWD) {
    // this workgroup's slab row of the channel sums (zeros for chunks > 0,
    // whose staged values chunk 0 also summed)
    fflush();
    __syncthreads();
    for (int c = tid; c < KB; c += 512) {
      double* fr = g.fb_sums + (long long)blockIdx.x * 2 * KB;
      const double v = cc == 0 ? fsum[c] : 0.0;
      fr[c] = wadd ? fr[c] + v : v;
      if (!wadd) fr[KB + c] = 0.0;
    }
  }
  // slab write: D[k][c] -> ws[split][k][tap * C + cc * 64 + c]
  const long long kd = 9ll * g.C;
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int b = wc * 9 + fn, t = CW == 64 ? b >> 2 : fn, cb = CW == 64 ? b & 3 : wc;
      const int col = t * g.C + cc * CW + cb * 16 + (lane & 15);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int k = wk * (KB / WK) + fm * 16 + (lane >> 4) * 4 + jj;
        float* o = ws + ((long long)(split * WP + wp) * g.K + k) * kd + col;
        *o = wadd ? *o + acc[fm][fn][jj] : acc[fm][fn][jj];
      }
    }
}

// ------------------------------------------------------------------ wgrad, R x S stride 1, one filter row per workgroup
// dW[k][r][s][c] of the wide-kernel layer of wr_resnet_bird's head (Conv2D
// (4, 10) 256 -> 128 at 16 x 32, resnet/wr_resnet_bird.py:47-52), whose
// im2col wgrad re-reads every input pixel 40 times (k_conv_wgrad: 500
// TFLOP/s).  A workgroup owns one filter row r, one 64-channel chunk and ALL
// S taps of that row (output tile K x S*64) and reduces over a contiguous
// range of SEGW-pixel output-row segments, NSEG per pipeline step: per step
// it stages dY[NSEG x SEGW px][K] and the matching input rows (row h + r - pt)
// as NSEG halo strips of SEGW + S - 1 pixels x 64 channels ONCE; the S taps
// are shifted views of a strip.  8 waves = 2 halves of K x 4 groups of S
// (tap, 16-channel) blocks; per step each wave runs NSEG * (SEGW / 32) *
// (K / 32) * S MFMAs (160 for the head).  LDS images and fragment reads as in
// k_wgrad3x3_halo (pixel-major, 288-B / 160-B padded rows read by
// ds_read_b64_tr_b16), register-staged double buffer, one barrier per step;
// split-K slabs combined by k_wgrad_reduce_g.
template <int KB, int S, int SEGW, int NSEG>
__global__ void __launch_bounds__(512, 1)
k_wgrad_row_halo(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ dY,
                 float* __restrict__ ws, int ngroups, int nchunk, int nseg, int segs_per_split) {
  constexpr int HWX = SEGW + S - 1;
  constexpr int LDD = KB + 16, LDX = 64 + 16;
  constexpr int DS = NSEG * SEGW * LDD, XS = NSEG * HWX * LDX;
  constexpr int FM = KB / 32, FN = S;  // 4 wave groups x S blocks = S taps x 4 channel blocks
  constexpr int DGR = KB / 8, DG = NSEG * SEGW * DGR, XG = NSEG * HWX * 8;
  constexpr int DPT = (DG + 511) / 512, XPT = (XG + 511) / 512;
  static_assert(SEGW % 32 == 0, "segment = whole 32-pixel MFMA k-chunks");
  static_assert(2 * (DS + XS) * 2 <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (DS + XS)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wid >> 2, wc = wid & 3;
  const int xcd = blockIdx.x & 7, bi = blockIdx.x >> 3;
  const int grp = bi % ngroups, split = (bi / ngroups) * 8 + xcd;
  const int r = grp / nchunk, cc = grp - r * nchunk;
  const int sbeg = split * segs_per_split;
  const int send = sbeg + segs_per_split < nseg ? sbeg + segs_per_split : nseg;
  const int QS = (g.Q + SEGW - 1) / SEGW;
  const T16* zp = reinterpret_cast<const T16*>(g_zero_page);

  u32x4 rd[DPT], rx[XPT];
  auto gload = [&](int s0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int idx = tid + 512 * i;
      const int px = idx / DGR, cg = idx - px * DGR;
      const int sg = px / SEGW, pxs = px - sg * SEGW;
      const int seg = s0 + sg;
      const int n = seg / (g.P * QS), rem = seg - n * (g.P * QS);
      const int h = rem / QS, w = (rem - h * QS) * SEGW + pxs;
      const bool ok = idx < DG && seg < send && w < g.Q;
      rd[i] = *reinterpret_cast<const u32x4*>(ok ? dY + (((long long)n * g.P + h) * g.Q + w) * g.K + cg * 8 : zp);
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 512 * i;
      const int row = idx >> 3, cg = idx & 7;
      const int sg = row / HWX, hp = row - sg * HWX;
      const int seg = s0 + sg;
      const int n = seg / (g.P * QS), rem = seg - n * (g.P * QS);
      const int h = rem / QS, w0 = (rem - h * QS) * SEGW;
      const int hin = h + r - g.pt, win = w0 - g.pl + hp;
      const bool ok = idx < XG && seg < send && (unsigned)hin < (unsigned)g.H && (unsigned)win < (unsigned)g.W;
      rx[i] = *reinterpret_cast<const u32x4*>(
          ok ? X + (((long long)n * g.H + hin) * g.W + win) * g.C + cc * 64 + cg * 8 : zp);
    }
  };
  auto sstore = [&](int buf) __attribute__((always_inline)) {
    uint16_t* Ds = smem + buf * (DS + XS);
    uint16_t* Xh = Ds + DS;
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int idx = tid + 512 * i;
      const int px = idx / DGR, cg = idx - px * DGR;
      if (idx < DG) *reinterpret_cast<u32x4*>(Ds + px * LDD + cg * 8) = rd[i];
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + 512 * i;
      if (idx < XG) *reinterpret_cast<u32x4*>(Xh + (idx >> 3) * LDX + (idx & 7) * 8) = rx[i];
    }
  };

  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // this wave's S blocks: block b = wc * S + fn -> tap b / 4, channels (b % 4) * 16
  const int grp4 = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  typedef __attribute__((address_space(3))) bf4* lp;

  if (sbeg < send) {
    gload(sbeg);
    sstore(0);
  }
  __syncthreads();
  int buf = 0;
  for (int s0 = sbeg; s0 < send; s0 += NSEG) {
    const bool more = s0 + NSEG < send;
    if (more) gload(s0 + NSEG);
    const uint16_t* Ds = smem + buf * (DS + XS);
    const uint16_t* Xh = Ds + DS;
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg)
#pragma unroll
      for (int kc = 0; kc < SEGW / 32; ++kc) {
        const int rb = sg * SEGW + kc * 32;  // dY pixel row of this 32-pixel chunk
        const int xb0 = sg * HWX + kc * 32;  // halo pixel of tap 0
        bf8 af[FM];
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int col = wk * (KB / 2) + fm * 16 + 4 * pp;
          const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lp)(reinterpret_cast<const __bf16*>(Ds + (rb + 4 * grp4 + q) * LDD + col)));
          const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lp)(reinterpret_cast<const __bf16*>(Ds + (rb + 16 + 4 * grp4 + q) * LDD + col)));
          af[fm] = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int b = wc * FN + fn, t = b >> 2;
          const uint16_t* xb = Xh + (xb0 + t) * LDX + (b & 3) * 16 + 4 * pp;
          const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lp)(reinterpret_cast<const __bf16*>(xb + (4 * grp4 + q) * LDX)));
          const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lp)(reinterpret_cast<const __bf16*>(xb + (16 + 4 * grp4 + q) * LDX)));
          const bf8 bv = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int fm = 0; fm < FM; ++fm)
            acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[fm], bv, acc[fm][fn], 0, 0, 0);
        }
      }
    if (more) sstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // slab write: D[k][c] -> ws[split][k][(r * S + tap) * C + cc * 64 + c]
  const long long kd = (long long)g.R * S * g.C;
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int b = wc * FN + fn, t = b >> 2;
      const int col = (r * S + t) * g.C + cc * 64 + (b & 3) * 16 + (lane & 15);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int k = wk * (KB / 2) + fm * 16 + (lane >> 4) * 4 + jj;
        ws[((long long)split * g.K + k) * kd + col] = acc[fm][fn][jj];
      }
    }
}

// Deterministic split-K combine: dw = beta*dw + sum_z ws[z].  Each thread owns
// four consecutive outputs (16-B loads) and keeps eight slab loads in flight
// (independent partial sums, fixed combine order), so the pass runs at HBM
// rate instead of one dependent load per split.
// Split-K combine with the splits spread over the workgroup: 16 columns of
// float4 x 16 split groups per 256 threads (each thread sums every 16th slab of
// its column, eight loads in flight), then a fixed-order LDS sum of the 16
// group partials -- deterministic, and enough workgroups for the narrow 3x3
// layers whose column-only version ran 36-144 workgroups of long serial sums.
__global__ void __launch_bounds__(256) k_wgrad_reduce_g(const float* __restrict__ ws, int nsplit, long long nv,
                                                        long long n, float beta, float* __restrict__ dw) {
  __shared__ f4 part[16][17];
  const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const long long v = (long long)blockIdx.x * 16 + col;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  if (v < nv) {
    const float* src = ws + v * 4;
    int z = grp;
    for (; z + 7 * 16 < nsplit; z += 8 * 16) {
      f4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = *reinterpret_cast<const f4*>(src + (long long)(z + 16 * u) * n);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += t[u];
    }
    for (; z < nsplit; z += 16) acc += *reinterpret_cast<const f4*>(src + (long long)z * n);
  }
  part[grp][col] = acc;
  __syncthreads();
  if (grp == 0 && v < nv) {
    f4 t = part[0][col];
#pragma unroll
    for (int g = 1; g < 16; ++g) t += part[g][col];
    f4* d = reinterpret_cast<f4*>(dw + v * 4);
    *d = beta != 0.f ? *d * beta + t : t;
  }
}

__global__ void __launch_bounds__(256) k_wgrad_reduce(const float* __restrict__ ws, int nsplit, long long n,
                                                      float beta, float* __restrict__ dw) {
  // vector path only when every slab (z * n floats) stays 16-B aligned
  const long long nv = ((n & 3) == 0 && ((uintptr_t)ws & 15) == 0 && ((uintptr_t)dw & 15) == 0) ? n >> 2 : 0;
  for (long long v = (long long)blockIdx.x * 256 + threadIdx.x; v < nv; v += (long long)gridDim.x * 256) {
    f4 s[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] = f4{0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 8 <= nsplit; z += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += *reinterpret_cast<const f4*>(ws + (long long)(z + u) * n + v * 4);
    }
    for (; z < nsplit; ++z) s[0] += *reinterpret_cast<const f4*>(ws + (long long)z * n + v * 4);
    const f4 t = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    f4* d = reinterpret_cast<f4*>(dw + v * 4);
    *d = beta != 0.f ? *d * beta + t : t;
  }
  // scalar tail (n % 4)
  for (long long i = (nv << 2) + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float t = 0.f;
    for (int z = 0; z < nsplit; ++z) t += ws[(long long)z * n + i];
    dw[i] = beta != 0.f ? dw[i] * beta + t : t;
  }
}

// ------------------------------------------------------------------ host side
ACFE_API int acfe_conv2d_bn_prologue_supported(int N, int H, int W, int C, int K, int dtype);
static bool pro_args_ok(const float* sc, const float* sh, const void* xo);
static ConvGeom make_geom(int N, int H, int W, int C, int K, int R, int S, int st, int pt, int pl, int P,
                          int Q, int BK, int BN) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.P = P; g.Q = Q;
  g.R = R; g.S = S; g.st = st; g.pt = pt; g.pl = pl;
  g.Kd = R * S * C;
  g.Kdp = (g.Kd + BK - 1) / BK * BK;
  g.Kp = (K + BN - 1) / BN * BN;
  g.ldy = K;
  g.M = (long long)N * P * Q;
  g.drop = make_drop(0.f, 0);
  g.res = nullptr;
  g.res_relu = 0;
  g.pro_sc = g.pro_sh = nullptr;
  g.pro_relu = 0;
  g.pro_out = nullptr;
  g.bn_sc = g.bn_sh = g.bn_mu = g.bn_is = nullptr;
  g.bn_relu = 0;
  g.fb_x = nullptr;
  g.fb_add = nullptr;
  g.fb_sc = g.fb_sh = g.fb_coef = nullptr;
  g.fb_relu = 0;
  g.fb_out = nullptr;
  g.fb_sums = nullptr;
  g.keep_out = nullptr;
  g.keep_in = nullptr;
  g.s2d = g.s2d_C = g.s2d_H = g.s2d_W = g.s2d_pt = g.s2d_pl = g.s2d_fill = g.s2d_lc = g.s2d_amul = 0;
  g.s2d_rpq = g.s2d_rq = 0.f;
  static const int cmaj = !getenv("ACFE_CONVG_CMAJ") || atoi(getenv("ACFE_CONVG_CMAJ")) != 0;
  g.cmaj = cmaj;
  g.idx32 = g.M * K < (1ll << 32) ? 1 : 0;
  static const int dbg = getenv("ACFE_CONV_DBG") ? atoi(getenv("ACFE_CONV_DBG")) : 0;
  g.dbg = dbg;
  return g;
}

static int pick_bn(int K) { return K <= 32 ? 32 : (K <= 64 ? 64 : 128); }



// k_conv3x3_narrow with 8 waves per workgroup (4 waves measured slower, r02v)
template <int KB, int SW>
static void launch_narrow(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y,
                          double* stats, int tiles_h, int tiles_w, long long nt, int grid_m, int gp, hipStream_t s) {
  const uint16_t *xx = (const uint16_t*)x, *ww = (const uint16_t*)wp;
  uint16_t* yy = (uint16_t*)y;
  if (g.drop.on)
    hipLaunchKernelGGL((k_conv3x3_narrow<KB, SW, true, 8>), dim3(gp), dim3(512), 0, s, g, xx, ww, bias, yy, stats,
                       tiles_h, tiles_w, (int)nt, grid_m);
  else
    hipLaunchKernelGGL((k_conv3x3_narrow<KB, SW, false, 8>), dim3(gp), dim3(512), 0, s, g, xx, ww, bias, yy, stats,
                       tiles_h, tiles_w, (int)nt, grid_m);
}

template <typename T, int BN, int WM, int WN>
static int launch_fwd_t(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y,
                        double* stats, int grid_m, hipStream_t s) {
  const int tiles_m = (int)((g.M + 127) / 128);
  dim3 grid(grid_m, g.Kp / BN);
  if constexpr (sizeof(T) == 2 && BN >= 64) {
    if (g.R == 3 && g.S == 3 && g.st == 1 && g.C % 64 == 0 && g.K == BN && (!g.drop.on || g.idx32) &&
        ((uintptr_t)y & 15) == 0) {  // (16-B epilogue stores)
      // chunk-resident halo rows: 4-row tiles at K = 128, 8 at K = 64 (r02z-ba:
      // the 6-row per-step staging, 3-row and 5-row tiles all measured slower)
      constexpr int tr = BN == 128 ? 4 : 8;
      const int tiles_h = (g.P + tr - 1) / tr, tiles_w = (g.Q + 63) / 64;  // partial last column tile
      const long long nt = (long long)g.N * tiles_h * tiles_w;
      if (nt < (1ll << 31)) {
        int gp = 256;
        if (gp > nt) gp = (int)nt;
        if (gp >= 64) gp &= ~7;
        // each workgroup writes statistics slab row blockIdx.x: never more
        // workgroups than the caller's slab rows (narrow images have more
        // tiles than 128-pixel slab rows)
        if (stats && gp > grid_m) gp = grid_m;
        if constexpr (BN == 128) {
          // one wave per SIMD (pool1w.hip), the previous tile's epilogue beside this tile's MFMAs
          const int rc = launch_plain1w(g, x, wp, bias, y, stats, grid_m, s, "acfe_conv2d_fwd", 0);
          if (rc != ACFE_E_INVAL) return rc;
        }
        if constexpr (BN == 64) {
          // the epilogue beside the next tile's MFMAs (rows64.hip)
          const int rc = launch_r64(g, x, wp, bias, y, stats, grid_m, s, "acfe_conv2d_fwd", g.drop.on ? 4 : 0);
          if (rc != ACFE_E_INVAL) return rc;
        }
#define ROWS(TR_, PM_, ...)                                                                                   \
  hipLaunchKernelGGL((k_conv3x3_rows<BN, TR_, PM_, ##__VA_ARGS__>), dim3(gp), dim3(512), 0, s, g, (const uint16_t*)x, \
                     (const uint16_t*)wp, bias, (uint16_t*)y, stats, tiles_h, tiles_w, (int)nt, grid_m, nullptr)
        if (g.drop.on) ROWS(tr, 4, true); else ROWS(tr, 0, true);
#undef ROWS
        return launch_rc("acfe_conv2d_fwd");
      }
    }
    // k_conv_fwd_p preconditions: whole K-tiles per tap, whole N tiles, a
    // 64-bit tap mask, 32-bit pixel index and < 2 GiB of input per M tile
    const long long img = (long long)g.H * g.W * g.C * 2;
    const long long span = ((256 + (long long)g.P * g.Q - 1) / ((long long)g.P * g.Q) + 1) * img;
    if (g.C % 64 == 0 && g.K % BN == 0 && g.R * g.S <= 64 && g.R < 32 && g.M < (1ll << 31) &&
        span < (1ll << 31)) {
      // persistent: one 512-thread workgroup per CU (256 CUs), a multiple of 8
      const int ny = g.Kp / BN, tiles = (int)((g.M + 255) / 256);
      int gp = 256 / ny;
      if (gp > tiles) gp = tiles;
      if (gp >= 64) gp &= ~7;
      hipLaunchKernelGGL((k_conv_fwd_p<BN>), dim3(gp, ny), dim3(512), 0, s, g, (const uint16_t*)x,
                         (const uint16_t*)wp, bias, (uint16_t*)y, stats, tiles, grid_m);
      return launch_rc("acfe_conv2d_fwd");
    }
  }
  if (g.C % TT<T>::GR == 0)
    hipLaunchKernelGGL((k_conv_fwd_g<T, 128, BN, WM, WN>), grid, dim3(256), 0, s, g, (const T*)x,
                       (const T*)wp, bias, (T*)y, stats, tiles_m);
  else
    hipLaunchKernelGGL((k_conv_fwd<T, 128, BN, WM, WN, false>), grid, dim3(256), 0, s, g, (const T*)x,
                       (const T*)wp, bias, (T*)y, stats, tiles_m);
  return launch_rc("acfe_conv2d_fwd");
}

template <int NCS, int NKB>
static int launch_1x1(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
                      int grid_m, hipStream_t s) {
  hipLaunchKernelGGL((k_conv1x1_reg<NCS, NKB>), dim3(grid_m), dim3(256), 0, s, g, (const uint16_t*)x,
                     (const uint16_t*)wp, bias, (uint16_t*)y, stats);
  return launch_rc("acfe_conv2d_fwd(1x1)");
}

template <typename T>
static int launch_fwd(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y,
                      double* stats, int grid_m, hipStream_t s) {
  // (k_conv1x1_reg maps output pixel m to input pixel m: P x Q must be H x W --
  // the strided dgrad's phase convs can have one more output row / column)
  if (sizeof(T) == 2 && g.R == 1 && g.S == 1 && g.st == 1 && g.pt == 0 && g.pl == 0 && g.P == g.H &&
      g.Q == g.W && g.C % 8 == 0 && g.K % 4 == 0 && g.ldy == g.K &&
      ((g.C <= 32 && g.K <= 128) || (g.K <= 32 && g.C <= 128))) {
    const int ncs = (g.C + 31) / 32, nkb = (g.K + 15) / 16;
    if (nkb >= 4 && g.K != nkb * 16) goto general;  // WIDE tile stores whole 16-channel blocks
    // dispatch on (reduction steps, 16-channel output blocks)
#define L1(A, B) if (ncs == A && nkb == B) return launch_1x1<A, B>(g, x, wp, bias, y, stats, grid_m, s)
    L1(1, 1); L1(1, 2); L1(1, 4); L1(1, 8);
    L1(2, 1); L1(2, 2); L1(4, 1); L1(4, 2);
#undef L1
  }
general:
  if constexpr (sizeof(T) == 2) {
    if (g.R == 3 && g.S == 3 && g.st == 1 && g.pt == 1 && g.pl == 1 && g.P == g.H && g.Q == g.W && g.C == 16 &&
        g.K == 64 && g.Kp == 64 && g.Kdp >= 160 && g.ldy == g.K && g.M * g.K < (1ll << 32) &&
        ((uintptr_t)x & 15) == 0 && ((uintptr_t)wp & 15) == 0 && ((uintptr_t)y & 7) == 0) {
      const int tiles_h = (g.P + 7) / 8, tiles_w = (g.Q + 63) / 64;
      const long long nt = (long long)g.N * tiles_h * tiles_w;
      if (nt < (1ll << 31)) {
        int gp = 256;
        if (gp > nt) gp = (int)nt;
        if (gp >= 64) gp &= ~7;
        if (stats && gp > grid_m) gp = grid_m;  // one statistics slab row per workgroup
        if (g.drop.on)
          hipLaunchKernelGGL(k_conv3x3_c16<true>, dim3(gp), dim3(512), 0, s, g, (const uint16_t*)x,
                             (const uint16_t*)wp, bias, (uint16_t*)y, stats, tiles_h, tiles_w, (int)nt, grid_m);
        else
          hipLaunchKernelGGL(k_conv3x3_c16<false>, dim3(gp), dim3(512), 0, s, g, (const uint16_t*)x,
                             (const uint16_t*)wp, bias, (uint16_t*)y, stats, tiles_h, tiles_w, (int)nt, grid_m);
        return launch_rc("acfe_conv2d_fwd(c16)");
      }
    }
    if (g.R == 3 && g.S == 3 && g.st == 1 && g.pt == 1 && g.pl == 1 && g.P == g.H && g.Q == g.W &&
        ((g.C == 32 && g.K == 128) || (g.C == 16 && g.K == 256 && g.Kdp >= 160)) && g.Kp == g.K && g.ldy == g.K &&
        g.M * g.K < (1ll << 32) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)wp & 15) == 0 && ((uintptr_t)y & 15) == 0) {
      // 32 -> 128 / 16 -> 256 (k_conv3x3_cw): 256- / 128-pixel tiles, 64 (32 for narrow images) wide
      const int segw = g.Q <= 32 ? 32 : 64, tr = (g.K == 256 ? 128 : 256) / segw;
      const int tiles_h = (g.P + tr - 1) / tr, tiles_w = (g.Q + segw - 1) / segw;
      const long long nt = (long long)g.N * tiles_h * tiles_w;
      if (nt < (1ll << 31)) {
        int gp = 256;
        if (gp > nt) gp = (int)nt;
        if (gp >= 64) gp &= ~7;
        if (stats && gp > grid_m) gp = grid_m;  // one statistics slab row per workgroup
#define CWL(CW_, KB_, SW_, D_)                                                                              \
  hipLaunchKernelGGL((k_conv3x3_cw<CW_, KB_, SW_, D_>), dim3(gp), dim3(512), 0, s, g, (const uint16_t*)x,    \
                     (const uint16_t*)wp, bias, (uint16_t*)y, stats, tiles_h, tiles_w, (int)nt, grid_m)
#define CWD(CW_, KB_)                                                                                       \
  if (segw == 64) {                                                                                         \
    if (g.drop.on) CWL(CW_, KB_, 64, true); else CWL(CW_, KB_, 64, false);                                  \
  } else {                                                                                                  \
    if (g.drop.on) CWL(CW_, KB_, 32, true); else CWL(CW_, KB_, 32, false);                                  \
  }
        if (g.C == 32) { CWD(32, 128) } else { CWD(16, 256) }
#undef CWD
#undef CWL
        return launch_rc("acfe_conv2d_fwd(cw)");
      }
    }
    if (g.R == 3 && g.S == 3 && g.st == 1 && g.pt == 1 && g.pl == 1 && g.P == g.H && g.Q == g.W &&
        g.C % 64 == 0 && (g.K == 32 || g.K == 16) && g.C * g.K <= 4096 && g.ldy == g.K &&
        g.M * g.K < (1ll << 32)) {
      constexpr int nw = 8;
      // tiles of nw * 32 pixels: segw columns x tr rows
      const int segw = g.Q <= 32 ? 32 : 64, tr = nw * 32 / segw;
      const int tiles_h = (g.P + tr - 1) / tr, tiles_w = (g.Q + segw - 1) / segw;
      const long long nt = (long long)g.N * tiles_h * tiles_w;
      if (nt < (1ll << 31)) {
        int gp = 256;
        if (gp > nt) gp = (int)nt;
        if (gp >= 64) gp &= ~7;
        if (stats && gp > grid_m) gp = grid_m;  // one statistics slab row per workgroup
        if (g.K == 32) {
          if (segw == 64) launch_narrow<32, 64>(g, x, wp, bias, y, stats, tiles_h, tiles_w, nt, grid_m, gp, s);
          else launch_narrow<32, 32>(g, x, wp, bias, y, stats, tiles_h, tiles_w, nt, grid_m, gp, s);
        } else {
          if (segw == 64) launch_narrow<16, 64>(g, x, wp, bias, y, stats, tiles_h, tiles_w, nt, grid_m, gp, s);
          else launch_narrow<16, 32>(g, x, wp, bias, y, stats, tiles_h, tiles_w, nt, grid_m, gp, s);
        }
        return launch_rc("acfe_conv2d_fwd(narrow)");
      }
    }
  }
  const int bn = pick_bn(g.K);
  if (bn == 32) return launch_fwd_t<T, 32, 4, 1>(g, x, wp, bias, y, stats, grid_m, s);
  if (bn == 64) return launch_fwd_t<T, 64, 2, 2>(g, x, wp, bias, y, stats, grid_m, s);
  return launch_fwd_t<T, 128, 2, 2>(g, x, wp, bias, y, stats, grid_m, s);
}

static int grid_m_for(long long M, int ny) {
  const long long tiles = (M + 127) / 128;
  long long gm = 2048 / ny;
  if (gm < 1) gm = 1;
  gm = tiles < gm ? tiles : gm;
  if (gm >= 64) gm &= ~7ll;  // a multiple of 8: XCD-chunked tile walk (TileWalk)
  return (int)gm;
}

// Packed-weight geometry so callers can size buffers: rows_p x cols_p.
ACFE_API int acfe_conv2d_packed_shape(int K, int R, int S, int C, int dtype, int flip, int* rows_p,
                                      int* cols_p) {
  if (K <= 0 || R <= 0 || S <= 0 || C <= 0 || !rows_p || !cols_p || (dtype != 0 && dtype != 1))
    return ACFE_E_INVAL;
  const int BK = dtype == ACFE_DTYPE_BF16 ? 64 : 32;
  const int outc = flip ? C : K, red = R * S * (flip ? K : C);
  const int bn = pick_bn(outc);
  *rows_p = (outc + bn - 1) / bn * bn;
  *cols_p = (red + BK - 1) / BK * BK;
  return ACFE_OK;
}

ACFE_API int acfe_conv2d_pack_weights(const float* w, int K, int R, int S, int C, int dtype, int flip,
                                      void* out, void* stream) {
  int rp, cp;
  int rc = acfe_conv2d_packed_shape(K, R, S, C, dtype, flip, &rp, &cp);
  if (rc) return rc;
  if (!w || !out) return ACFE_E_INVAL;
  const long long total = (long long)rp * cp;
  int grid = cdiv(total, 256);
  if (grid > 4096) grid = 4096;
  if (dtype == ACFE_DTYPE_BF16)
    hipLaunchKernelGGL(k_pack_w<uint16_t>, dim3(grid), dim3(256), 0, strm(stream), w, K, R, S, C, flip, rp, cp,
                       (uint16_t*)out);
  else
    hipLaunchKernelGGL(k_pack_w<float>, dim3(grid), dim3(256), 0, strm(stream), w, K, R, S, C, flip, rp, cp,
                       (float*)out);
  return launch_rc("acfe_conv2d_pack_weights");
}

ACFE_API int acfe_conv2d_pack_weights_batch(const void* descs, int n, long long total, int dtype, void* stream) {
  if (!descs || n <= 0 || n > 256 || total <= 0 || (dtype != 0 && dtype != 1)) return ACFE_E_INVAL;
  long long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  if (dtype == ACFE_DTYPE_BF16)
    hipLaunchKernelGGL(k_pack_w_batch<uint16_t>, dim3((unsigned)g), dim3(256), 0, strm(stream),
                       (const PackDesc*)descs, n, total);
  else
    hipLaunchKernelGGL(k_pack_w_batch<float>, dim3((unsigned)g), dim3(256), 0, strm(stream), (const PackDesc*)descs,
                       n, total);
  return launch_rc("acfe_conv2d_pack_weights_batch");
}

ACFE_API int acfe_conv2d_stats_rows(long long M, int K) {
  return grid_m_for(M, (K + pick_bn(K) - 1) / pick_bn(K));
}

static int conv2d_fwd_impl(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int R, int S,
                           int stride, int pad_top, int pad_left, int P, int Q, const float* bias, void* y,
                           int dtype, double* stats_partial, const Drop& drop, void* stream) {
  if (!x || !wpacked || !y || N < 0 || H <= 0 || W <= 0 || C <= 0 || K <= 0 || R <= 0 || S <= 0 ||
      stride <= 0 || P <= 0 || Q <= 0 || (dtype != 0 && dtype != 1))
    return ACFE_E_INVAL;
  if (N == 0) return ACFE_OK;
  const int BK = dtype == ACFE_DTYPE_BF16 ? 64 : 32;
  const int bn = pick_bn(K);
  ConvGeom g = make_geom(N, H, W, C, K, R, S, stride, pad_top, pad_left, P, Q, BK, bn);
  g.drop = drop;
  const int gm = grid_m_for(g.M, g.Kp / bn);
  if (dtype == ACFE_DTYPE_BF16) return launch_fwd<uint16_t>(g, x, wpacked, bias, y, stats_partial, gm, strm(stream));
  return launch_fwd<float>(g, x, wpacked, bias, y, stats_partial, gm, strm(stream));
}

ACFE_API int acfe_conv2d_fwd(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int R,
                             int S, int stride, int pad_top, int pad_left, int P, int Q,
                             const float* bias, void* y, int dtype, double* stats_partial,
                             void* stream) {
  return conv2d_fwd_impl(x, N, H, W, C, wpacked, K, R, S, stride, pad_top, pad_left, P, Q, bias, y, dtype,
                         stats_partial, make_drop(0.f, 0), stream);
}

// y = Dropout(rate, seed)(conv(x)): the epilogue applies acfe_dropout's mask to
// the rounded outputs; the statistics are those of the dropped-out values.
ACFE_API int acfe_conv2d_fwd_dropout(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int R,
                                     int S, int stride, int pad_top, int pad_left, int P, int Q,
                                     const float* bias, void* y, int dtype, double* stats_partial,
                                     float drop_rate, unsigned long long seed, void* stream) {
  if (drop_rate < 0.f || drop_rate >= 1.f) return ACFE_E_INVAL;
  return conv2d_fwd_impl(x, N, H, W, C, wpacked, K, R, S, stride, pad_top, pad_left, P, Q, bias, y, dtype,
                         stats_partial, make_drop(drop_rate, seed), stream);
}

// dX = conv^T(dY, W).  wflip = acfe_conv2d_pack_weights(..., flip=1).
//
// stride 1: a stride-1 conv of dY with the flipped weights.
// stride > 1: sub-pixel (phase) decomposition instead of zero insertion.  The
// rows of dX with h = a (mod st) receive contributions only from the filter
// rows r = (a + pad_top) (mod st); for each of the st x st phases (a, b) the
// phase image dX[:, a::st, b::st, :] is a stride-1 conv of dY itself with the
// (Ra x Sb)-tap sub-kernel of those rows / columns -- every MFMA multiplies a
// real dY value (zero insertion spent 4x / 9x the MACs on inserted zeros at
// stride 2 / 3 and wrote an st^2-times larger upsampled copy of dY) -- written
// to a phase buffer and scattered into dX; phases without taps are zero.
//   For phase row a: r0 = (a + pt) % st, Ra = ceil((R - r0) / st) taps r0 + st j,
//   da = (a + pt - r0) / st; output row i of the phase reads dY row
//   i + da - j, i.e. the sub-kernel flipped (t = Ra-1-j) is a stride-1 conv
//   with offset c = da - (Ra - 1): pad_top = max(0, -c), and max(0, c) extra
//   leading output rows that the scatter skips.
namespace {
struct PhaseAxis {
  int n;    // phase rows (or columns) of dX: ceil((H - a) / st)
  int r0;   // first filter row of the phase
  int taps; // filter rows of the phase (0: no contribution)
  int pad;  // top pad of the phase conv
  int off;  // leading output rows skipped by the scatter
};
PhaseAxis phase_axis(int H, int R, int st, int pt, int a) {
  PhaseAxis x{};
  x.n = H > a ? (H - a + st - 1) / st : 0;
  x.r0 = (a + pt) % st;
  x.taps = x.r0 < R ? (R - x.r0 + st - 1) / st : 0;
  const int da = (a + pt - x.r0) / st;
  const int c = da - (x.taps - 1);
  x.pad = c < 0 ? -c : 0;
  x.off = c > 0 ? c : 0;
  return x;
}
size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }
}  // namespace

// phase sub-kernel, packed for the forward conv of dY (K inputs -> C outputs):
// out[c][(t*Sb + u)*K + k] = wflip[c][((R-1-r)*S + (S-1-s))*K + k] with
// r = r0 + st*(Ra-1-t), s = s0 + st*(Sb-1-u); rows padded to rows_p, columns
// zero-padded to cols_p
template <typename T>
__global__ void k_pack_phase(const T* __restrict__ wflip, int ld_flip, int K, int R, int S, int st, int r0, int ra,
                             int s0, int sb, int rows_p, int cols_p, T* __restrict__ out) {
  const long long total = (long long)rows_p * cols_p;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int row = (int)(i / cols_p), col = (int)(i - (long long)row * cols_p);
    T v = (T)0;
    if (col < ra * sb * K) {
      const int k = col % K, tu = col / K, t = tu / sb, u = tu % sb;
      const int r = r0 + st * (ra - 1 - t), sx = s0 + st * (sb - 1 - u);
      v = wflip[(long long)row * ld_flip + ((R - 1 - r) * S + (S - 1 - sx)) * K + k];
    }
    out[i] = v;
  }
}

// Super-pixel (space-to-depth) form of the strided bf16 dgrad.  With
// h + pt = st u + a (a in [0, st)), dX row h receives dY row u - m through
// filter row r = a + st m only (m = 0 .. Mr - 1, Mr = ceil(R / st)); so the
// st x st blocks of dX -- block (u, v), channel o = (a st + b) C + c -- are ONE
// stride-1 conv of dY (K channels) with an Mr x Ms window (pad Mr - 1 / Ms - 1)
// and st^2 C output channels, run by k_conv_fwd_p with its super-pixel store
// (ConvGeom::s2d), no phase buffer and no scatter pass.  The window's packed
// weights hold w[k][a + st m][b + st n][c], zero where that tap lies past the
// filter (wr_resnet: 9 of 16 at 3x3 / stride 2, all 9 at stride 3, 1 of 4 / 9
// for the 1x1 shortcuts, whose zero rows write the tap-less pixels' zeros).
namespace {
struct S2dPlan {
  int mr, ms, kout, bn, rows_p, cols_p;
  bool ok, fill;
};
S2dPlan s2d_plan(int N, int P, int Q, int K, int C, int R, int S, int st, int pt, int pl, int H, int W,
                 int dtype) {
  static const bool on = !getenv("ACFE_DGRAD_S2D") || atoi(getenv("ACFE_DGRAD_S2D")) != 0;
  S2dPlan p{};
  p.mr = (R + st - 1) / st;
  p.ms = (S + st - 1) / st;
  // a 1x1 "valid" shortcut feeds only block position (0, 0): C outputs into
  // a zeroed dX (ConvGeom::s2d_fill)
  p.fill = R == 1 && S == 1 && pt == 0 && pl == 0;
  p.kout = p.fill ? C : st * st * C;
  p.bn = p.kout % 128 == 0 ? 128 : 64;
  p.rows_p = (p.kout + p.bn - 1) / p.bn * p.bn;
  p.cols_p = p.mr * p.ms * K;
  const long long U = (H + pt + st - 1) / st, V = (W + pl + st - 1) / st;
  const long long img = (long long)P * Q * K * 2;
  const long long span = ((256 + (long long)P * Q - 1) / ((long long)P * Q) + 1) * img;
  // st <= 4: the epilogue's block row a = (ab * ceil(32 / st)) >> 5 is exact
  // for ab < st * st only at strides 2, 3 and 4 (stride 5: ab = 23 gives 5)
  p.ok = on && dtype == ACFE_DTYPE_BF16 && st > 1 && st <= 4 && (C & (C - 1)) == 0 && K % 64 == 0 &&
         p.kout % p.bn == 0 && p.mr * p.ms <= 64 && (long long)N * ((H + pt + st - 1) / st) * ((W + pl + st - 1) / st) < (1 << 24) &&
         pt >= 0 && pl >= 0 && pt < st && pl < st && (long long)N * U * V < (1ll << 31) && span < (1ll << 31);
  return p;
}
}  // namespace

// out[o][(tr * ms + tc) * K + k] = w[k][a + st (mr-1-tr)][b + st (ms-1-tc)][c] for
// o = (a st + b) C + c (0 past the filter or past kout), read from the dgrad
// packing wflip[c][((R-1-r) * S + (S-1-s)) * K + k]
__global__ void k_pack_s2d(const uint16_t* __restrict__ wflip, int ld_flip, int K, int C, int R, int S, int st,
                           int mr, int ms, int kout, int rows_p, int cols_p, uint16_t* __restrict__ out) {
  const long long total = (long long)rows_p * cols_p;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int o = (int)(i / cols_p), col = (int)(i - (long long)o * cols_p);
    uint16_t v = 0;
    if (o < kout) {
      const int ab = o / C, c = o - ab * C, a = ab / st, b = ab - a * st;
      const int k = col % K, tap = col / K, tr = tap / ms, tc = tap - tr * ms;
      const int r = a + st * (mr - 1 - tr), sx = b + st * (ms - 1 - tc);
      if (r < R && sx < S) v = wflip[(long long)c * ld_flip + ((R - 1 - r) * S + (S - 1 - sx)) * K + k];
    }
    out[i] = v;
  }
}

// dX[n][a + st i][b + st j][:] = ph[n][off_r + i][off_c + j][:] (ph == NULL: zeros)
template <typename T>
__global__ void k_phase_scatter(const T* __restrict__ ph, int N, int PH, int PW, int C, int off_r, int off_c, int a,
                                int b, int st, int Ha, int Wa, int H, int W, T* __restrict__ dx) {
  constexpr int V = 16 / sizeof(T);  // elements per 16-B vector
  const int cv = C / V;
  const long long total = (long long)N * Ha * Wa * cv;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int c = (int)(e % cv);
    long long t = e / cv;
    const int j = (int)(t % Wa);
    t /= Wa;
    const int i = (int)(t % Ha);
    const int n = (int)(t / Ha);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (ph) v = *reinterpret_cast<const uint4*>(ph + (((long long)n * PH + off_r + i) * PW + off_c + j) * C + c * V);
    *reinterpret_cast<uint4*>(dx + (((long long)n * H + a + st * i) * W + b + st * j) * C + c * V) = v;
  }
}

ACFE_API long long acfe_conv2d_dgrad_workspace(int N, int P, int Q, int K, int C, int R, int S, int stride,
                                               int pad_top, int pad_left, int H, int W, int dtype) {
  if (N < 0 || P <= 0 || Q <= 0 || K <= 0 || C <= 0 || R <= 0 || S <= 0 || stride <= 0 || H <= 0 || W <= 0 ||
      (dtype != 0 && dtype != 1))
    return ACFE_E_INVAL;
  if (stride == 1) return 0;
  const S2dPlan sp = s2d_plan(N, P, Q, K, C, R, S, stride, pad_top, pad_left, H, W, dtype);
  if (sp.ok) return (long long)align256((size_t)sp.rows_p * sp.cols_p * 2);
  const size_t es = dtype == ACFE_DTYPE_BF16 ? 2 : 4;
  const int BK = dtype == ACFE_DTYPE_BF16 ? 64 : 32;
  const int rows_p = (C + pick_bn(C) - 1) / pick_bn(C) * pick_bn(C);
  size_t wbytes = 0, tmax = 0;
  for (int a = 0; a < stride; ++a)
    for (int b = 0; b < stride; ++b) {
      const PhaseAxis ra = phase_axis(H, R, stride, pad_top, a), cb = phase_axis(W, S, stride, pad_left, b);
      if (!ra.n || !cb.n || !ra.taps || !cb.taps) continue;
      const int cols_p = (ra.taps * cb.taps * K + BK - 1) / BK * BK;
      wbytes += align256((size_t)rows_p * cols_p * es);
      const size_t tb = (size_t)N * (ra.n + ra.off) * (cb.n + cb.off) * C * es;
      if (tb > tmax) tmax = tb;
    }
  return (long long)(wbytes + align256(tmax));
}

ACFE_API int acfe_conv2d_dgrad(const void* dy, int N, int P, int Q, int K, const void* wflip, int C, int R,
                               int S, int stride, int pad_top, int pad_left, int H, int W, void* dx,
                               int dtype, void* workspace, void* stream) {
  if (!dy || !wflip || !dx || N < 0 || P <= 0 || Q <= 0 || K <= 0 || C <= 0 || stride <= 0 ||
      (dtype != 0 && dtype != 1))
    return ACFE_E_INVAL;
  if (N == 0) return ACFE_OK;
  if (stride == 1)  // stride-1 conv of dY with flipped weights: input channels K, output C
    return acfe_conv2d_fwd(dy, N, P, Q, K, wflip, C, R, S, 1, R - 1 - pad_top, S - 1 - pad_left, H, W,
                           nullptr, dx, dtype, nullptr, stream);
  const size_t es = dtype == ACFE_DTYPE_BF16 ? 2 : 4;
  if (!workspace || (C * es) % 16 != 0 || ((uintptr_t)dx & 15)) return ACFE_E_INVAL;
  const int BK = dtype == ACFE_DTYPE_BF16 ? 64 : 32;
  const int rows_p = (C + pick_bn(C) - 1) / pick_bn(C) * pick_bn(C);
  int ld_flip, rp_full;
  {
    int rc = acfe_conv2d_packed_shape(K, R, S, C, dtype, 1, &rp_full, &ld_flip);
    if (rc) return rc;
  }
  const S2dPlan sp = s2d_plan(N, P, Q, K, C, R, S, stride, pad_top, pad_left, H, W, dtype);
  if (sp.ok) {
    hipStream_t s = strm(stream);
    uint16_t* wp = static_cast<uint16_t*>(workspace);
    const long long tot = (long long)sp.rows_p * sp.cols_p;
    const int grid = (int)std::min<long long>(cdiv(tot, 256), 2048);
    hipLaunchKernelGGL(k_pack_s2d, dim3(grid), dim3(256), 0, s, (const uint16_t*)wflip, ld_flip, K, C, R, S, stride,
                       sp.mr, sp.ms, sp.kout, sp.rows_p, sp.cols_p, wp);
    int rc = launch_rc("acfe_conv2d_dgrad(pack_s2d)");
    if (rc) return rc;
    const int pt = sp.mr - 1, pl = sp.ms - 1;
    const int U = (H + pad_top + stride - 1) / stride, V = (W + pad_left + stride - 1) / stride;
    ConvGeom g = make_geom(N, P, Q, K, sp.kout, sp.mr, sp.ms, 1, pt, pl, U, V, 64, sp.bn);
    g.s2d = stride;
    g.s2d_fill = sp.fill;
    g.s2d_lc = __builtin_ctz((unsigned)C);
    g.s2d_amul = (32 + stride - 1) / stride;
    g.s2d_rpq = 1.0f / (float)((long long)U * V);
    g.s2d_rq = 1.0f / (float)V;
    g.s2d_C = C;
    g.s2d_H = H;
    g.s2d_W = W;
    g.s2d_pt = pad_top;
    g.s2d_pl = pad_left;
    if (sp.fill) {
      // the tap-less pixels' zeros: one memset of dX ahead of the conv (as
      // extra epilogue stores they held the vmcnt waits of every K-tile)
      rc = hip_rc(hipMemsetAsync(dx, 0, (size_t)N * H * W * C * 2, s), "acfe_conv2d_dgrad(zero)");
      if (rc) return rc;
    }
    const int ny = g.Kp / sp.bn, tiles = (int)((g.M + 255) / 256);
    int gp = 256 / ny;
    if (gp < 8) gp = 8;
    if (gp > tiles) gp = tiles;
    if (gp >= 64) gp &= ~7;
    if (sp.bn == 128)
      hipLaunchKernelGGL((k_conv_fwd_p<128, true>), dim3(gp, ny), dim3(512), 0, s, g, (const uint16_t*)dy,
                         (const uint16_t*)wp, nullptr, (uint16_t*)dx, nullptr, tiles, 0);
    else
      hipLaunchKernelGGL((k_conv_fwd_p<64, true>), dim3(gp, ny), dim3(512), 0, s, g, (const uint16_t*)dy,
                         (const uint16_t*)wp, nullptr, (uint16_t*)dx, nullptr, tiles, 0);
    return launch_rc("acfe_conv2d_dgrad(s2d)");
  }
  // weights of every phase first (one region each), then the phase image buffer
  size_t wbytes = 0;
  for (int a = 0; a < stride; ++a)
    for (int b = 0; b < stride; ++b) {
      const PhaseAxis ra = phase_axis(H, R, stride, pad_top, a), cb = phase_axis(W, S, stride, pad_left, b);
      if (!ra.n || !cb.n || !ra.taps || !cb.taps) continue;
      wbytes += align256((size_t)rows_p * ((ra.taps * cb.taps * K + BK - 1) / BK * BK) * es);
    }
  unsigned char* wsb = static_cast<unsigned char*>(workspace);
  void* tmp = wsb + wbytes;
  hipStream_t s = strm(stream);
  size_t wo = 0;
  for (int a = 0; a < stride; ++a)
    for (int b = 0; b < stride; ++b) {
      const PhaseAxis ra = phase_axis(H, R, stride, pad_top, a), cb = phase_axis(W, S, stride, pad_left, b);
      if (!ra.n || !cb.n) continue;
      const bool taps = ra.taps && cb.taps;
      const int PH = ra.n + ra.off, PW = cb.n + cb.off;
      if (taps) {
        const int cols_p = (ra.taps * cb.taps * K + BK - 1) / BK * BK;
        void* wph = wsb + wo;
        wo += align256((size_t)rows_p * cols_p * es);
        const long long tot = (long long)rows_p * cols_p;
        int grid = cdiv(tot, 256);
        if (grid > 2048) grid = 2048;
        if (dtype == ACFE_DTYPE_BF16)
          hipLaunchKernelGGL(k_pack_phase<uint16_t>, dim3(grid), dim3(256), 0, s, (const uint16_t*)wflip, ld_flip,
                             K, R, S, stride, ra.r0, ra.taps, cb.r0, cb.taps, rows_p, cols_p, (uint16_t*)wph);
        else
          hipLaunchKernelGGL(k_pack_phase<float>, dim3(grid), dim3(256), 0, s, (const float*)wflip, ld_flip, K, R,
                             S, stride, ra.r0, ra.taps, cb.r0, cb.taps, rows_p, cols_p, (float*)wph);
        int rc = launch_rc("acfe_conv2d_dgrad(pack_phase)");
        if (rc) return rc;
        rc = acfe_conv2d_fwd(dy, N, P, Q, K, wph, C, ra.taps, cb.taps, 1, ra.pad, cb.pad, PH, PW, nullptr, tmp,
                             dtype, nullptr, stream);
        if (rc) return rc;
      }
      const long long tot = (long long)N * ra.n * cb.n * (C * (long long)es / 16);
      int grid = cdiv(tot, 256);
      if (grid > 8192) grid = 8192;
      if (dtype == ACFE_DTYPE_BF16)
        hipLaunchKernelGGL(k_phase_scatter<uint16_t>, dim3(grid), dim3(256), 0, s,
                           taps ? (const uint16_t*)tmp : nullptr, N, PH, PW, C, ra.off, cb.off, a, b, stride, ra.n,
                           cb.n, H, W, (uint16_t*)dx);
      else
        hipLaunchKernelGGL(k_phase_scatter<float>, dim3(grid), dim3(256), 0, s, taps ? (const float*)tmp : nullptr,
                           N, PH, PW, C, ra.off, cb.off, a, b, stride, ra.n, cb.n, H, W, (float*)dx);
      const int rc = launch_rc("acfe_conv2d_dgrad(phase_scatter)");
      if (rc) return rc;
    }
  return ACFE_OK;
}

// Split-K plan of the wgrad: `splits` pixel chunks of `chunk` rows, splits a
// multiple of 8 so the XCD mapping of k_conv_wgrad is a bijection.
static void wgrad_combine(const float* ws, int nsplit, long long n, float beta, float* dw, int grid,
                          hipStream_t st) {
  const bool vec = (n & 3) == 0 && ((uintptr_t)ws & 15) == 0 && ((uintptr_t)dw & 15) == 0;
  if (vec && nsplit >= 16) {
    const long long nv = n >> 2;
    hipLaunchKernelGGL(k_wgrad_reduce_g, dim3((unsigned)((nv + 15) / 16)), dim3(256), 0, st, ws, nsplit, nv, n, beta,
                       dw);
  } else {
    hipLaunchKernelGGL(k_wgrad_reduce, dim3(grid), dim3(256), 0, st, ws, nsplit, n, beta, dw);
  }
}

static void wgrad_plan(long long M, int kd, int K, long long* splits_o, long long* chunk_o) {
  const int bmw = K <= 32 ? 32 : (K <= 64 ? 64 : 128);
  const long long tiles = (long long)((kd + 127) / 128) * ((K + bmw - 1) / bmw);
  // target workgroup count of the split-K grid: 4096 measured 1.1 ms/step
  // faster than 1024 once the combine ran split-parallel (k_wgrad_reduce_g),
  // the halo kernels gaining most from the finer pixel ranges (r01r)
  constexpr long long target = 4096;
  long long splits = (target + tiles - 1) / tiles;
  long long chunk = (M + splits - 1) / splits;
  chunk = (chunk + 63) / 64 * 64;
  if (chunk < 512) chunk = 512;
  splits = (M + chunk - 1) / chunk;
  if (splits < 1) splits = 1;
  splits = (splits + 7) / 8 * 8;
  *splits_o = splits;
  *chunk_o = chunk;
}

ACFE_API long long acfe_conv2d_wgrad_workspace(int N, int H, int W, int C, int K, int R, int S, int P, int Q) {
  long long splits, chunk;
  wgrad_plan((long long)N * P * Q, R * S * C, K, &splits, &chunk);
  return splits * K * (long long)(R * S * C);  // floats
}

template <typename T, int BMW>
static int launch_wgrad_t(const ConvGeom& g, const void* x, const void* dy, float* ws, long long chunk,
                          int splits, hipStream_t s) {
  const int tx = (g.Kd + 127) / 128, ty = (g.K + BMW - 1) / BMW;
  dim3 grid(tx * ty * splits);  // 1-D: k_conv_wgrad maps it XCD-aware
  const bool fd = g.K % TT<T>::GR == 0, fx = g.C % TT<T>::GR == 0;
#define WG(FD, FX)                                                                                       \
  hipLaunchKernelGGL((k_conv_wgrad<T, BMW, FD, FX>), grid, dim3(256), 0, s, g, (const T*)x, (const T*)dy, \
                     ws, chunk, tx, ty)
  if (fd && fx) WG(true, true);
  else if (fd) WG(true, false);
  else if (fx) WG(false, true);
  else WG(false, false);
#undef WG
  return launch_rc("acfe_conv2d_wgrad");
}

// k_wgrad3x3_halo launch (3x3 stride 1; C % 64 == 0 with K in {32, 64, 128,
// 256}, or C in {16, 32} with K in {128, 256}; a partial last 64-pixel column
// segment is masked): split count within the planned workspace (`splits`),
// returned in *used.
struct HaloPlan {
  int cw, nr, wp, nchunk, nseg, sp, per;
  bool c16k64, k16c64;
  // the Q % 64 remainder columns as 16-pixel segments (4 nr rows each) by a
  // second launch over the same grid (plain K = 64 / 128 and the K = 64 BN
  // fold): qs whole 64-pixel segment columns, then qse 16-pixel ones from wofs
  bool edge;
  int qs, qse, wofs, nsege, pere;
};
static HaloPlan halo_plan(const ConvGeom& g, bool amax, long long splits) {
  HaloPlan hp;
  // 16 / 32-channel layers: one chunk of C; K = 256 (wr_resnet's stage-3
  // 256 -> 256): 32-channel chunks, so the K x 9 x CW accumulators stay 36
  // tiles per wave
  // tiles per wave; K = 16 (wr_resnet_bird's stage-3 256 -> 16): 128-channel
  // chunks, one 16-channel block per wave
  // (ACFE_WG16_CW=64: the 64-channel-chunk form below for C % 128 == 0 too;
  // r04g7: 120.5 vs 103.9 us for the 256 -> 16 layer at 512 clips)
  static const int cw16 = getenv("ACFE_WG16_CW") ? atoi(getenv("ACFE_WG16_CW")) : 128;
  const int cw = g.C % 64 == 0 ? (g.K == 256 ? 32 : (g.K == 16 && cw16 == 128 && g.C % 128 == 0 ? 128 : 64)) : g.C;
  // two output rows per step for the K = 64 (plain or pooled dY) and K = 32
  // layers (r02au-aw: 72 instead of 36 MFMAs per wave per barrier); the K =
  // 128 pooled-gradient variant spills at two rows (138 VGPRs) and keeps one
  // C = 16 -> K = 64 (wr_resnet's stage-1 conv2a): two pixel groups of 4
  // waves, each its own split slab (the caller guarantees splits >= 16)
  const bool c16k64 = cw == 16 && g.K == 64;
  // K = 16 on 64-channel chunks (C = 64 * odd): the 4 wave groups' 9 (tap,
  // block) pairs x two pixel groups (one 32-pixel half each), 72 KB of LDS ->
  // 2 workgroups per CU
  const bool k16c64 = cw == 64 && g.K == 16;
  const int nr = ((cw == 64 || c16k64) && g.P % 2 == 0 && (g.K == 64 || (g.K == 32 && !amax))) ? 2 : 1;
  const int wp = (c16k64 || k16c64) ? 2 : 1;
  const int rem = g.Q >= 64 ? g.Q % 64 : 0;
  // (the BN fold writes its dY rows: whole 4 nr row groups only, and the
  // plain K = 64 kernel splits exactly as the fold does, so that their dW
  // stay bit-identical; K = 128 / 256 mask the rows of a partial last group)
  // (C = 16 -> K = 64, two pixel groups of waves: the same rule as K = 64)
  const bool edge = rem && !amax &&
                    ((((cw == 64 && wp == 1) || c16k64) && g.K == 64 && nr == 2 && g.P % 8 == 0) ||
                     (!g.fb_sc && wp == 1 &&
                      ((cw == 64 && g.K == 128 && nr == 1) || (cw == 32 && g.K == 256 && nr == 1))));
  const int qs = edge ? g.Q / 64 : (g.Q + 63) / 64;
  const int nchunk = g.C / cw, nseg = (int)((long long)g.N * (g.P / nr) * qs);
  // c16k64: 75 KB of LDS and 114 VGPRs -> two workgroups per CU
  int sp = (c16k64 || k16c64 ? 512 : 256) / nchunk;
  if (sp > splits / wp) sp = (int)(splits / wp);
  sp &= ~7;
  if (sp < 8) sp = 8;
  if (sp > splits) sp = (int)splits;  // splits is a multiple of 8 (wgrad_plan)
  hp.cw = cw;
  hp.nr = nr;
  hp.wp = wp;
  hp.nchunk = nchunk;
  hp.nseg = nseg;
  hp.sp = sp;
  hp.per = (nseg + sp - 1) / sp;
  hp.c16k64 = c16k64;
  hp.k16c64 = k16c64;
  hp.edge = edge;
  hp.qs = qs;
  hp.qse = edge ? (rem + 15) / 16 : 0;
  hp.wofs = g.Q - rem;
  hp.nsege = edge ? (int)((long long)g.N * ((g.P + 4 * nr - 1) / (4 * nr)) * hp.qse) : 0;
  hp.pere = edge ? (hp.nsege + sp - 1) / sp : 0;
  return hp;
}

static int wgrad_halo_launch(const ConvGeom& g, const void* x, const void* dy, const uint8_t* amax, float* ws,
                             long long splits, hipStream_t s, int* used) {
  const HaloPlan hp = halo_plan(g, amax != nullptr, splits);
  const int cw = hp.cw, nr = hp.nr, wp = hp.wp, nchunk = hp.nchunk, nseg = hp.nseg, sp = hp.sp, per = hp.per;
  const bool c16k64 = hp.c16k64, k16c64 = hp.k16c64;
  const dim3 gr(nchunk * sp);
  const int qs = hp.qs, qse = hp.qse, wofs = hp.wofs, nsege = hp.nsege, pere = hp.pere;
  if (g.fb_sc) {  // acfe_conv2d_wgrad_bnbwd: the BN backward formed while staging dY
#define WB(KB_, CW_, NR_, KP_)                                                                                  \
  hipLaunchKernelGGL((k_wgrad3x3_halo<KB_, false, CW_, NR_, true, KP_>), gr, dim3(512), 0, s, g,                 \
                     (const uint16_t*)x, (const uint16_t*)dy, ws, nchunk, nseg, per, nullptr, qs, 0, 0)
#define WBE(KB_, CW_, NR_, KP_)                                                                                 \
  hipLaunchKernelGGL((k_wgrad3x3_halo<KB_, false, CW_, NR_, true, KP_, 16>), gr, dim3(512), 0, s, g,             \
                     (const uint16_t*)x, (const uint16_t*)dy, ws, nchunk, nsege, pere, nullptr, qse, wofs, 1)
    if (amax || (wp != 1 && !c16k64)) return ACFE_E_INVAL;
    // keep bits: the stage-1 K = 64 fold only (the forward that writes them: k_conv3x3_r64 PM 4)
    if (g.keep_in && !(cw == 64 && g.K == 64 && nr == 2 && !c16k64 && g.drop.on)) return ACFE_E_INVAL;
    if (c16k64 && nr == 2) {
      WB(64, 16, 2, false);
      if (hp.edge) WBE(64, 16, 2, false);
    } else if (cw == 64 && g.K == 64 && nr == 2 && g.keep_in) {
      WB(64, 64, 2, true);
      if (hp.edge) WBE(64, 64, 2, true);
    } else if (cw == 64 && g.K == 64 && nr == 2) {
      WB(64, 64, 2, false);
      if (hp.edge) WBE(64, 64, 2, false);
    } else if (cw == 64 && g.K == 32 && nr == 2) WB(32, 64, 2, false);
    else return ACFE_E_INVAL;
#undef WBE
#undef WB
    *used = sp * wp;
    return launch_rc("acfe_conv2d_wgrad_bnbwd");
  }
#define WH(KB_, U_)                                                                                              \
  hipLaunchKernelGGL((k_wgrad3x3_halo<KB_, U_>), gr, dim3(512), 0, s, g, (const uint16_t*)x, (const uint16_t*)dy, \
                     ws, nchunk, nseg, per, amax, qs, 0, 0)
#define WHC(KB_, CW_)                                                                                              \
  hipLaunchKernelGGL((k_wgrad3x3_halo<KB_, false, CW_>), gr, dim3(512), 0, s, g, (const uint16_t*)x,               \
                     (const uint16_t*)dy, ws, nchunk, nseg, per, nullptr)
  if (cw == 128) {  // wr_resnet_bird stage 3 (256 -> 16)
    WHC(16, 128);
  } else if (k16c64) {
    WHC(16, 64);
  } else if (c16k64) {
    if (nr == 2) {
      hipLaunchKernelGGL((k_wgrad3x3_halo<64, false, 16, 2>), gr, dim3(512), 0, s, g, (const uint16_t*)x,
                         (const uint16_t*)dy, ws, nchunk, nseg, per, nullptr, qs, 0, 0);
      if (hp.edge)
        hipLaunchKernelGGL((k_wgrad3x3_halo<64, false, 16, 2, false, false, 16>), gr, dim3(512), 0, s, g,
                           (const uint16_t*)x, (const uint16_t*)dy, ws, nchunk, nsege, pere, nullptr, qse, wofs, 1);
    } else WHC(64, 16);
  } else if (cw == 32) {  // the stage-2/3 branch2b (32 -> 128 / 256); wr_resnet's stage 3 (256 -> 256)
    if (g.K == 128) WHC(128, 32);
    else {
      hipLaunchKernelGGL((k_wgrad3x3_halo<256, false, 32>), gr, dim3(512), 0, s, g, (const uint16_t*)x,
                         (const uint16_t*)dy, ws, nchunk, nseg, per, nullptr, qs, 0, 0);
      if (hp.edge)
        hipLaunchKernelGGL((k_wgrad3x3_halo<256, false, 32, 1, false, false, 16>), gr, dim3(512), 0, s, g,
                           (const uint16_t*)x, (const uint16_t*)dy, ws, nchunk, nsege, pere, nullptr, qse, wofs, 1);
    }
  } else if (cw == 16) {  // stage 3 (16 -> 256)
    WHC(256, 16);
  } else if (g.K == 128) {
    if (amax) WH(128, true);
    else {
      WH(128, false);
      if (hp.edge)
        hipLaunchKernelGGL((k_wgrad3x3_halo<128, false, 64, 1, false, false, 16>), gr, dim3(512), 0, s, g,
                           (const uint16_t*)x, (const uint16_t*)dy, ws, nchunk, nsege, pere, nullptr, qse, wofs, 1);
    }
  } else if (g.K == 64) {
    if (amax && nr == 2)
      hipLaunchKernelGGL((k_wgrad3x3_halo<64, true, 64, 2>), gr, dim3(512), 0, s, g, (const uint16_t*)x,
                         (const uint16_t*)dy, ws, nchunk, nseg, per, amax, qs, 0, 0);
    else if (amax) WH(64, true);
    else if (nr == 2) {
      hipLaunchKernelGGL((k_wgrad3x3_halo<64, false, 64, 2>), gr, dim3(512), 0, s, g, (const uint16_t*)x,
                         (const uint16_t*)dy, ws, nchunk, nseg, per, nullptr, qs, 0, 0);
      if (hp.edge)
        hipLaunchKernelGGL((k_wgrad3x3_halo<64, false, 64, 2, false, false, 16>), gr, dim3(512), 0, s, g,
                           (const uint16_t*)x, (const uint16_t*)dy, ws, nchunk, nsege, pere, nullptr, qse, wofs, 1);
    } else WH(64, false);
  } else if (nr == 2) {  // the stage-2 branch21 (128 -> 32): 36 MFMAs per wave per two-row step
    hipLaunchKernelGGL((k_wgrad3x3_halo<32, false, 64, 2>), gr, dim3(512), 0, s, g, (const uint16_t*)x,
                       (const uint16_t*)dy, ws, nchunk, nseg, per, nullptr);
  } else {
    WH(32, false);  // (18 MFMAs per wave per segment)
  }
#undef WHC
#undef WH
  *used = sp * wp;
  return launch_rc(amax ? "acfe_conv2d_wgrad_unpool" : "acfe_conv2d_wgrad(halo)");
}

// k_wgrad_row_halo launch (the (4, 10) head conv: bf16, stride 1, K = 128,
// C % 64 == 0): split count within the planned workspace, returned in *used.
static int wgrad_row_halo_launch(const ConvGeom& g, const void* x, const void* dy, float* ws, long long splits,
                                 hipStream_t s, int* used) {
  constexpr int SEGW = 32, NSEG = 3;
  const int nchunk = g.C / 64, ngroups = g.R * nchunk;
  const int nseg = (int)((long long)g.N * g.P * ((g.Q + SEGW - 1) / SEGW));
  // one 126-KB workgroup per CU: about one grid-wave of workgroups
  int sp = (256 / ngroups) & ~7;
  if (sp < 8) sp = 8;
  if (sp > splits) sp = (int)splits;  // splits is a multiple of 8 (wgrad_plan)
  int per = (nseg + sp - 1) / sp;
  per = (per + NSEG - 1) / NSEG * NSEG;  // whole steps per split
  hipLaunchKernelGGL((k_wgrad_row_halo<128, 10, SEGW, NSEG>), dim3(ngroups * sp), dim3(512), 0, s, g,
                     (const uint16_t*)x, (const uint16_t*)dy, ws, ngroups, nchunk, nseg, per);
  *used = sp;
  return launch_rc("acfe_conv2d_wgrad(row halo)");
}

static bool halo_ok(int N, int C, int K, int R, int S, int stride, int P, int Q, long long splits) {
  // (k_wgrad3x3_halo's buffer loads address one image of x / dY in 32 bits)
  if ((long long)P * Q * (C > K ? C : K) * 2 >= (1ll << 31)) return false;
  return R == 3 && S == 3 && stride == 1 &&
         ((C % 64 == 0 && (K == 64 || K == 128 || K == 32 || K == 256)) || (C % 64 == 0 && K == 16 && splits >= 16) ||
          ((C == 32 && (K == 128 || K == 256)) || (C == 16 && (K == 256 || (K == 64 && splits >= 16))))) &&
         (long long)N * P * ((Q + 63) / 64) < (1ll << 31);
}

// dW[k][r][s][c] (fp32, KRSC) = sum over pixels.  beta: dW = beta*dW + grad.
ACFE_API int acfe_conv2d_wgrad(const void* x, int N, int H, int W, int C, const void* dy, int K, int R, int S,
                               int stride, int pad_top, int pad_left, int P, int Q, float* dw, float beta,
                               int dtype, float* workspace, void* stream) {
  if (!x || !dy || !dw || !workspace || N < 0 || C <= 0 || K <= 0 || (dtype != 0 && dtype != 1))
    return ACFE_E_INVAL;
  const long long M = (long long)N * P * Q;
  const int kd = R * S * C;
  if (N == 0) return hip_rc(hipMemsetAsync(dw, 0, sizeof(float) * K * kd, strm(stream)), "wgrad");
  const int bmw = K <= 32 ? 32 : (K <= 64 ? 64 : 128);
  long long splits, chunk;
  wgrad_plan(M, kd, K, &splits, &chunk);
  ConvGeom g = make_geom(N, H, W, C, K, R, S, stride, pad_top, pad_left, P, Q, 64, 128);
  g.ldy = K;
  int rc;
  if (dtype == ACFE_DTYPE_BF16 && halo_ok(N, C, K, R, S, stride, P, Q, splits)) {
    // halo-staged kernel; its split count stays within the planned workspace
    int used = 0;
    rc = wgrad_halo_launch(g, x, dy, nullptr, workspace, splits, strm(stream), &used);
    if (rc) return rc;
    splits = used;
  } else if (dtype == ACFE_DTYPE_BF16 && S == 10 && stride == 1 && C % 64 == 0 && K == 128 &&
             (long long)N * P * ((Q + 31) / 32) < (1ll << 31)) {
    int used = 0;
    rc = wgrad_row_halo_launch(g, x, dy, workspace, splits, strm(stream), &used);
    if (rc) return rc;
    splits = used;
  } else if (dtype == ACFE_DTYPE_BF16) {
    if (bmw == 32) rc = launch_wgrad_t<uint16_t, 32>(g, x, dy, workspace, chunk, (int)splits, strm(stream));
    else if (bmw == 64) rc = launch_wgrad_t<uint16_t, 64>(g, x, dy, workspace, chunk, (int)splits, strm(stream));
    else rc = launch_wgrad_t<uint16_t, 128>(g, x, dy, workspace, chunk, (int)splits, strm(stream));
    if (rc) return rc;
  } else {
    if (bmw == 32) rc = launch_wgrad_t<float, 32>(g, x, dy, workspace, chunk, (int)splits, strm(stream));
    else if (bmw == 64) rc = launch_wgrad_t<float, 64>(g, x, dy, workspace, chunk, (int)splits, strm(stream));
    else rc = launch_wgrad_t<float, 128>(g, x, dy, workspace, chunk, (int)splits, strm(stream));
    if (rc) return rc;
  }
  const long long n = (long long)K * kd;
  int grid = cdiv((n + 3) / 4, 256);
  if (grid > 2048) grid = 2048;
  wgrad_combine(workspace, (int)splits, n, beta, dw, grid, strm(stream));
  return launch_rc("acfe_conv2d_wgrad(reduce)");
}

// ------------------------------------------------------------------ wgrad + BN backward apply
// The weight gradient of a 3x3 stride-1 "same" bf16 conv whose output u feeds
// [Dropout ->] BatchNormalization (+ReLU) (resnet/wr_resnet.py:58-71: conv2a ->
// Dropout -> bn2b -> ReLU; resnet/wr_resnet_bird.py:139-154: conv21 -> Dropout
// -> bn2b -> ReLU), given that BN's OUTPUT gradient gy, its input u_bn (the
// dropped-out conv output) and its backward coefficients: the conv output
// gradient dy = acfe_bn_bwd_apply_ex(gy, u_bn, scale, shift, relu, coef, NULL,
// rate, seed) -- or, with `add`, acfe_bn_bwd_apply_ex(gy, u_bn, ..., relu
// (bit 1: u_bn is a ReLU output), coef, add, 0, 0): a BN whose input is this
// conv's (ReLU'd) residual output z and whose gradient carries the identity
// shortcut's (resnet/wr_resnet.py:82-89, bn2a of the next block) -- is formed
// while the wgrad stages it, written to `dy` (the dgrad
// reads it) and summed per channel into `sums` ([rows][2][K], rows =
// acfe_conv2d_wgrad_bnbwd_rows; the conv bias gradient via
// acfe_channel_sum_finalize) -- the separate apply pass over the tensor is not
// run.  Same dW as acfe_conv2d_wgrad on that dy.
ACFE_API int acfe_conv2d_wgrad_bnbwd_rows(int N, int H, int W, int C, int K) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || K <= 0) return 0;
  long long splits, chunk;
  wgrad_plan((long long)N * H * W, 9 * C, K, &splits, &chunk);
  if (!halo_ok(N, C, K, 3, 3, 1, H, W, splits)) return 0;
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, 1, 1, H, W, 64, 128);
  const HaloPlan hp = halo_plan(g, false, splits);
  // (K = 128, one row per step: 19 VGPRs spilled -- not covered)
  const bool ok = (hp.c16k64 && hp.nr == 2) || (hp.cw == 64 && ((K == 64 || K == 32) && hp.nr == 2));
  return ok ? hp.nchunk * hp.sp : 0;
}

static int wgrad_bnbwd_impl(const void* x, int N, int H, int W, int C, const void* gy, const void* u_bn, int K,
                            const float* scale, const float* shift, int relu, const float* coef, const void* add,
                            float drop_rate, unsigned long long seed, const uint8_t* keep, void* dy, float* dw,
                            float beta, float* workspace, double* sums, void* stream);

ACFE_API int acfe_conv2d_wgrad_bnbwd(const void* x, int N, int H, int W, int C, const void* gy, const void* u_bn,
                                     int K, const float* scale, const float* shift, int relu, const float* coef,
                                     const void* add, float drop_rate, unsigned long long seed, void* dy, float* dw,
                                     float beta, float* workspace, double* sums, void* stream) {
  return wgrad_bnbwd_impl(x, N, H, W, C, gy, u_bn, K, scale, shift, relu, coef, add, drop_rate, seed, nullptr, dy,
                          dw, beta, workspace, sums, stream);
}

// the same with the dropout mask read from the forward's keep bits
// (acfe_conv2d_fwd_*_keep) instead of regenerated: identical results
ACFE_API int acfe_conv2d_wgrad_bnbwd_keep(const void* x, int N, int H, int W, int C, const void* gy,
                                          const void* u_bn, int K, const float* scale, const float* shift, int relu,
                                          const float* coef, float drop_rate, unsigned long long seed,
                                          const uint8_t* keep, void* dy, float* dw, float beta, float* workspace,
                                          double* sums, void* stream) {
  if (!keep || drop_rate <= 0.f) return ACFE_E_INVAL;
  return wgrad_bnbwd_impl(x, N, H, W, C, gy, u_bn, K, scale, shift, relu, coef, nullptr, drop_rate, seed, keep, dy,
                          dw, beta, workspace, sums, stream);
}

static int wgrad_bnbwd_impl(const void* x, int N, int H, int W, int C, const void* gy, const void* u_bn, int K,
                            const float* scale, const float* shift, int relu, const float* coef, const void* add,
                            float drop_rate, unsigned long long seed, const uint8_t* keep, void* dy, float* dw,
                            float beta, float* workspace, double* sums, void* stream) {
  if (!x || !gy || !u_bn || !scale || !shift || !coef || !dy || !dw || !workspace || !sums || drop_rate < 0.f ||
      drop_rate >= 1.f || (add && drop_rate > 0.f))
    return ACFE_E_INVAL;
  if (((uintptr_t)gy | (uintptr_t)u_bn | (uintptr_t)dy | (uintptr_t)add) & 15) return ACFE_E_INVAL;
  const int rows = acfe_conv2d_wgrad_bnbwd_rows(N, H, W, C, K);
  if (!rows) return ACFE_E_INVAL;
  long long splits, chunk;
  wgrad_plan((long long)N * H * W, 9 * C, K, &splits, &chunk);
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, 1, 1, H, W, 64, 128);
  g.ldy = K;
  g.drop = make_drop(drop_rate, seed);
  g.fb_x = (const uint16_t*)u_bn;
  g.fb_sc = scale;
  g.fb_sh = shift;
  g.fb_coef = coef;
  g.fb_add = (const uint16_t*)add;
  g.fb_relu = relu & 3;
  g.fb_out = (uint16_t*)dy;
  g.fb_sums = sums;
  g.keep_in = keep;
  int used = 0;
  int rc = wgrad_halo_launch(g, x, gy, nullptr, workspace, splits, strm(stream), &used);
  if (rc) return rc;
  const long long n = (long long)K * 9 * C;
  int grid = cdiv((n + 3) / 4, 256);
  if (grid > 2048) grid = 2048;
  wgrad_combine(workspace, used, n, beta, dw, grid, strm(stream));
  return launch_rc("acfe_conv2d_wgrad_bnbwd(reduce)");
}

// ------------------------------------------------------------------ conv + 2x2 max-pool
// Conv2D 3x3 "same" stride 1 followed by MaxPool2D(2, 2) -> Dropout
// (resnet/wr_resnet_bird.py:139-148: res{s}b0_branch21 -> pooling -> dropout):
// k_conv3x3_rows<K, 6, 1> pools in its epilogue, so the full-resolution conv
// output is never written; the backward reads the pooled gradient + argmax
// bytes and expands them in its input staging (dgrad: k_conv3x3_rows<C, 6, 2>,
// wgrad: k_wgrad3x3_halo<K, true>).
// Rows-kernel tiles: K = 128 4-row tiles with chunk-resident halo rows (r02z:
// fwd_pool 4.97 -> 4.89 ms, dgrad_unpool 5.19 -> 4.75 ms against the 6-row
// per-step staging); K = 64 8 chunk-resident rows, the BN-prologue kernels too,
// so prologue and plain paths tile alike (r02ay/ba: fwd_add 128->64 0.89 vs
// 0.92 ms at 6 rows, dropout 0.53 vs 0.56; the per-step staging 1.04 / 0.61).
template <int KB, int PM, int TR, bool XR = false, bool PR = false>
static int launch_rows_tr(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y,
                          double* stats, int srows, uint8_t* amax, hipStream_t s, const char* what) {
  if ((uintptr_t)y & 15) return ACFE_E_INVAL;  // 16-B epilogue stores
  const int tiles_h = (g.P + TR - 1) / TR, tiles_w = (g.Q + 63) / 64;
  const long long nt = (long long)g.N * tiles_h * tiles_w;
  int gp = 256;
  if (gp > nt) gp = (int)nt;
  if (gp >= 64) gp &= ~7;
  if (stats && gp > srows) gp = srows;  // one statistics slab row per workgroup
  hipLaunchKernelGGL((k_conv3x3_rows<KB, TR, PM, XR, PR>), dim3(gp), dim3(512), 0, s, g, (const uint16_t*)x,
                     (const uint16_t*)wp, bias, (uint16_t*)y, stats, tiles_h, tiles_w, (int)nt, srows, amax);
  return launch_rc(what);
}

template <int KB, int PM>
static int launch_rows(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
                       int srows, uint8_t* amax, hipStream_t s, const char* what) {
  if constexpr (KB == 128) {
    if constexpr (PM == 1) {
      // one wave per SIMD, the previous tile's epilogue beside this tile's MFMAs
      const int rc = launch_pool1w(g, x, wp, bias, y, stats, srows, amax, s, what);
      if (rc != ACFE_E_INVAL) return rc;
    }
    if constexpr (PM == 2) {
      const int rc = launch_unpool1w(g, x, wp, y, amax, s, what);
      if (rc != ACFE_E_INVAL) return rc;
    }
    if constexpr (PM == 3) {
      const int rc = launch_plain1w(g, x, wp, bias, y, stats, srows, s, what, 3);
      if (rc != ACFE_E_INVAL) return rc;
    }
    return launch_rows_tr<KB, PM, 4, true>(g, x, wp, bias, y, stats, srows, amax, s, what);
  } else {
    static_assert(KB == 64, "rows kernels: K in {64, 128}");
    if constexpr (PM == 0 || PM == 3 || PM == 4) {
      // the epilogue beside the next tile's MFMAs (rows64.hip)
      const int rc = launch_r64(g, x, wp, bias, y, stats, srows, s, what, PM);
      if (rc != ACFE_E_INVAL) return rc;
    }
    if constexpr (PM != 2) {
      // BatchNormalization prologue (acfe_conv2d_bn_prologue_supported)
      if (g.pro_sc) return launch_rows_tr<KB, PM, 8, true, true>(g, x, wp, bias, y, stats, srows, amax, s, what);
    }
    return launch_rows_tr<KB, PM, 8, true>(g, x, wp, bias, y, stats, srows, amax, s, what);
  }
}

// ------------------------------------------------------------------ dgrad + BN backward reduce
// The stride-1 3x3 dgrad whose dX is the output gradient of a
// BatchNormalization (+ReLU) -- wr_resnet's bn2a / bn2b -> conv2a / conv2b
// (resnet/wr_resnet.py:56-80) -- with that BN's acfe_bn_bwd_reduce sums formed
// in the dgrad's epilogue (k_conv3x3_rows PM 5): the reduce pass and its
// re-read of dX are gone, the epilogue reads the BN input x instead.
// 64 dX channels (k_conv3x3_rows PM 5), any K % 64 == 0 dY channels.  The
// same sums in the one-wave K = C = 128 dgrad's units (r04p) cost more issue
// time than the separate reduce pass (+0.85 ms vs 0.75 ms per wr_resnet stage-2
// call): that kernel is issue-bound, the reduce runs at the copy rate.
// ACFE_DGRADBN128=0: the K = C = 128 dgrads keep the separate reduce pass (A/B)
static bool rows_pm5_128_enabled() {
  static const int v = getenv("ACFE_DGRADBN128") ? atoi(getenv("ACFE_DGRADBN128")) : 1;
  return v != 0;
}

ACFE_API int acfe_conv2d_dgrad_bn_rows(int N, int H, int W, int C, int K, int R, int S, int stride, int dtype) {
  // C = 64: the K = 64 row-halo kernels (rows64.hip PM 5); C = K = 128: the
  // one-wave kernel (pool1w.hip PM 5, wr_resnet's stage 2)
  if (dtype != ACFE_DTYPE_BF16 || N <= 0 || H <= 0 || W <= 0 || stride != 1 || R != 3 || S != 3 || K <= 0 ||
      !((C == 64 && K % 64 == 0) || (C == 128 && K == 128 && rows_pm5_128_enabled())) ||
      (long long)N * ((H + 3) / 4) * ((W + 63) / 64) >= (1ll << 31) || (long long)H * W * C * 2 >= (1ll << 31))
    return 0;
  return grid_m_for((long long)N * H * W, 1);
}

ACFE_API int acfe_conv2d_dgrad_bn(const void* dy, int N, int P, int Q, int K, const void* wflip, int C, int R,
                                  int S, int stride, int pad_top, int pad_left, int H, int W, void* dx, int dtype,
                                  const void* x_bn, const float* scale, const float* shift, const float* mean,
                                  const float* invstd, int relu, double* part, int part_rows, void* stream) {
  const int rows = acfe_conv2d_dgrad_bn_rows(N, H, W, C, K, R, S, stride, dtype);
  if (!rows || part_rows != rows || !dy || !wflip || !dx || !x_bn || !scale || !shift || !mean || !invstd ||
      !part || P != H || Q != W || pad_top < 0 || pad_top > 2 || pad_left < 0 || pad_left > 2 ||
      ((uintptr_t)dx & 15) || ((uintptr_t)x_bn & 15))
    return ACFE_E_INVAL;
  // the dgrad as a forward conv of dY with the flipped weights (acfe_conv2d_dgrad)
  ConvGeom g = make_geom(N, P, Q, K, C, R, S, 1, R - 1 - pad_top, S - 1 - pad_left, H, W, 64, C == 128 ? 128 : 64);
  g.res = (const uint16_t*)x_bn;
  g.bn_sc = scale;
  g.bn_sh = shift;
  g.bn_mu = mean;
  g.bn_is = invstd;
  g.bn_relu = relu ? 1 : 0;
  if (C == 128) return launch_dgradbn1w(g, dy, wflip, dx, part, rows, strm(stream), "acfe_conv2d_dgrad_bn");
  const int rc = launch_r64(g, dy, wflip, nullptr, dx, part, rows, strm(stream), "acfe_conv2d_dgrad_bn", 5);
  if (rc != ACFE_E_INVAL) return rc;
  return launch_rows_tr<64, 5, 8, true>(g, dy, wflip, nullptr, dx, part, rows, nullptr, strm(stream),
                                        "acfe_conv2d_dgrad_bn");
}

ACFE_API int acfe_conv2d_pool_supported(int N, int H, int W, int C, int K, int R, int S, int dtype) {
  return dtype == ACFE_DTYPE_BF16 && N > 0 && R == 3 && S == 3 && C > 0 && C % 64 == 0 &&
         (K == 64 || K == 128) && W >= 2 && W % 2 == 0 && H >= 2 && H % 2 == 0 &&
         (long long)N * ((H + 5) / 6) * ((W + 63) / 64) < (1ll << 31) &&
         (long long)N * H * ((W + 63) / 64) < (1ll << 31) &&
         (long long)N * (H / 2) * (W / 2) * (C > K ? C : K) < (1ll << 32);  // 32-bit pooled element index
}

ACFE_API int acfe_conv2d_fwd_pool(const void* x, int N, int H, int W, int C, const void* wpacked, int K,
                                  int pad_top, int pad_left, const float* bias, void* y, uint8_t* argmax,
                                  float drop_rate, unsigned long long seed, double* stats_partial, int dtype,
                                  void* stream) {
  if (!x || !wpacked || !y || !argmax || drop_rate < 0.f || drop_rate >= 1.f ||
      !acfe_conv2d_pool_supported(N, H, W, C, K, 3, 3, dtype) || ((uintptr_t)y & 7) || ((uintptr_t)argmax & 3))
    return ACFE_E_INVAL;
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, K);
  g.drop = make_drop(drop_rate, seed);
  const int srows = grid_m_for(g.M, 1);  // == acfe_conv2d_stats_rows(N*H*W, K)
  if (K == 128)
    return launch_rows<128, 1>(g, x, wpacked, bias, y, stats_partial, srows, argmax, strm(stream),
                               "acfe_conv2d_fwd_pool");
  return launch_rows<64, 1>(g, x, wpacked, bias, y, stats_partial, srows, argmax, strm(stream),
                            "acfe_conv2d_fwd_pool");
}

// acfe_conv2d_fwd_pool with the BatchNormalization (+ReLU) prologue of
// acfe_conv2d_fwd_bn (bn2a -> ReLU -> branch21 -> MaxPool2D of the stride-2
// blocks, resnet/wr_resnet_bird.py:121-145).
ACFE_API int acfe_conv2d_fwd_pool_bn(const void* x, int N, int H, int W, int C, const void* wpacked, int K,
                                     int pad_top, int pad_left, const float* bias, void* y, uint8_t* argmax,
                                     float drop_rate, unsigned long long seed, double* stats_partial,
                                     const float* bn_scale, const float* bn_shift, int bn_relu, void* x_bn_out,
                                     int dtype, void* stream) {
  if (!x || !wpacked || !y || !argmax || drop_rate < 0.f || drop_rate >= 1.f ||
      !acfe_conv2d_pool_supported(N, H, W, C, K, 3, 3, dtype) ||
      !acfe_conv2d_bn_prologue_supported(N, H, W, C, K, dtype) || !pro_args_ok(bn_scale, bn_shift, x_bn_out) ||
      ((uintptr_t)x & 15) || ((uintptr_t)y & 7) || ((uintptr_t)argmax & 3))
    return ACFE_E_INVAL;
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, K);
  g.drop = make_drop(drop_rate, seed);
  g.pro_sc = bn_scale;
  g.pro_sh = bn_shift;
  g.pro_relu = bn_relu ? 1 : 0;
  g.pro_out = (uint16_t*)x_bn_out;
  const int srows = grid_m_for(g.M, 1);
  return launch_rows<64, 1>(g, x, wpacked, bias, y, stats_partial, srows, argmax, strm(stream),
                            "acfe_conv2d_fwd_pool_bn");
}

ACFE_API int acfe_conv2d_dgrad_unpool(const void* dyp, const uint8_t* argmax, int N, int P, int Q, int K,
                                      const void* wflip, int C, int pad_top, int pad_left, void* dx, int dtype,
                                      void* stream) {
  if (!dyp || !argmax || !wflip || !dx || !acfe_conv2d_pool_supported(N, P, Q, K, C, 3, 3, dtype) ||
      ((uintptr_t)dyp & 15) || ((uintptr_t)argmax & 7))
    return ACFE_E_INVAL;
  // stride-1 conv of the (virtual) unpooled dY with the flipped weights: K -> C channels
  ConvGeom g = make_geom(N, P, Q, K, C, 3, 3, 1, 2 - pad_top, 2 - pad_left, P, Q, 64, C);
  if (C == 128)
    return launch_rows<128, 2>(g, dyp, wflip, nullptr, dx, nullptr, 0, const_cast<uint8_t*>(argmax),
                               strm(stream), "acfe_conv2d_dgrad_unpool");
  return launch_rows<64, 2>(g, dyp, wflip, nullptr, dx, nullptr, 0, const_cast<uint8_t*>(argmax), strm(stream),
                            "acfe_conv2d_dgrad_unpool");
}

ACFE_API int acfe_conv2d_wgrad_unpool(const void* x, int N, int H, int W, int C, const void* dyp,
                                      const uint8_t* argmax, int K, int pad_top, int pad_left, float* dw,
                                      float beta, int dtype, float* workspace, void* stream) {
  if (!x || !dyp || !argmax || !dw || !workspace || !acfe_conv2d_pool_supported(N, H, W, C, K, 3, 3, dtype) ||
      ((uintptr_t)dyp & 15) || ((uintptr_t)argmax & 7))
    return ACFE_E_INVAL;
  long long splits, chunk;
  wgrad_plan((long long)N * H * W, 9 * C, K, &splits, &chunk);
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, 128);
  g.ldy = K;
  int used = 0;
  int rc = wgrad_halo_launch(g, x, dyp, argmax, workspace, splits, strm(stream), &used);
  if (rc) return rc;
  const long long n = (long long)K * 9 * C;
  int grid = cdiv((n + 3) / 4, 256);
  if (grid > 2048) grid = 2048;
  wgrad_combine(workspace, used, n, beta, dw, grid, strm(stream));
  return launch_rc("acfe_conv2d_wgrad_unpool(reduce)");
}

// Conv2D 3x3 "same" stride 1 whose output is summed with the block shortcut
// (resnet/wr_resnet_bird.py:173-178: res{s}{b}_branch2b + Add (+ReLU)):
// y = (ReLU)(conv(x) + res) stored by the conv epilogue with its BN statistics
// (slab rows = acfe_conv2d_stats_rows(N*H*W, K), nullable); the conv output
// itself is never stored.  Shapes: acfe_conv2d_rows_supported.
ACFE_API int acfe_conv2d_rows_supported(int N, int H, int W, int C, int K, int R, int S, int dtype) {
  return dtype == ACFE_DTYPE_BF16 && N > 0 && R == 3 && S == 3 && C > 0 && C % 64 == 0 &&
         (K == 64 || K == 128) && W > 0 && H > 0 && (long long)N * ((H + 5) / 6) * ((W + 63) / 64) < (1ll << 31);
}

// Shapes the generic (C % 8 == 0) kernel takes with the Add in its row stores:
// wr_resnet_bird's stage-2/3 conv2b (32 -> 128, 16 / 32 -> 256 channels).
static bool fwd_add_generic_ok(int N, int H, int W, int C, int K, int dtype) {
  return dtype == ACFE_DTYPE_BF16 && N > 0 && H > 0 && W > 0 && C % 8 == 0 && K % 128 == 0 &&
         pick_bn(K) == 128 && (long long)N * H * W < (1ll << 31);
}

ACFE_API int acfe_conv2d_fwd_add_supported(int N, int H, int W, int C, int K, int dtype) {
  return acfe_conv2d_rows_supported(N, H, W, C, K, 3, 3, dtype) || fwd_add_generic_ok(N, H, W, C, K, dtype);
}

ACFE_API int acfe_conv2d_fwd_add(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                                 int pad_left, const float* bias, const void* res, int relu, void* y,
                                 double* stats_partial, int dtype, void* stream) {
  if (!x || !wpacked || !y || !res || !acfe_conv2d_fwd_add_supported(N, H, W, C, K, dtype) ||
      ((uintptr_t)y & 7) || ((uintptr_t)res & 7))
    return ACFE_E_INVAL;
  if (!acfe_conv2d_rows_supported(N, H, W, C, K, 3, 3, dtype)) {
    // generic kernel: 16-B residual / output rows
    if (((uintptr_t)y & 15) || ((uintptr_t)res & 15)) return ACFE_E_INVAL;
    ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, 128);
    g.res = (const uint16_t*)res;
    g.res_relu = relu ? 1 : 0;
    const int ny = g.Kp / 128, gm = grid_m_for(g.M, ny);
    const int tiles_m = (int)((g.M + 127) / 128);
    if (((C == 32 && K == 128) || (C == 16 && K == 256 && g.Kdp >= 160)) && pad_top == 1 && pad_left == 1 &&
        g.M * K < (1ll << 32) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)wpacked & 15) == 0) {
      // k_conv3x3_cw with the residual epilogue (wr_resnet_bird's stage-2 / 3 branch2b)
      const int segw = W <= 32 ? 32 : 64, tr = (K == 256 ? 128 : 256) / segw;
      const int tiles_h = (H + tr - 1) / tr, tiles_w = (W + segw - 1) / segw;
      const long long nt = (long long)N * tiles_h * tiles_w;
      if (nt < (1ll << 31)) {
        int gp = 256;
        if (gp > nt) gp = (int)nt;
        if (gp >= 64) gp &= ~7;
        const int srows = acfe_conv2d_stats_rows(g.M, K);  // (the caller's slab rows)
        if (stats_partial && gp > srows) gp = srows;
#define CWA(CW_, KB_, SW_)                                                                                  \
  hipLaunchKernelGGL((k_conv3x3_cw<CW_, KB_, SW_, false, true>), dim3(gp), dim3(512), 0, strm(stream), g,    \
                     (const uint16_t*)x, (const uint16_t*)wpacked, bias, (uint16_t*)y, stats_partial, tiles_h, \
                     tiles_w, (int)nt, srows)
        if (C == 32) {
          if (segw == 64) CWA(32, 128, 64); else CWA(32, 128, 32);
        } else {
          if (segw == 64) CWA(16, 256, 64); else CWA(16, 256, 32);
        }
#undef CWA
        return launch_rc("acfe_conv2d_fwd_add(cw)");
      }
    }
    const long long img = (long long)H * W * C * 2;
    const long long span = ((256 + (long long)H * W - 1) / ((long long)H * W) + 1) * img;
    if (C % 64 == 0 && span < (1ll << 31)) {
      // the persistent GEMM with the residual epilogue (wr_resnet's stage 3)
      const int tiles = (int)((g.M + 255) / 256);
      int gp = 256 / ny;
      if (gp > tiles) gp = tiles;
      if (gp >= 64) gp &= ~7;
      hipLaunchKernelGGL((k_conv_fwd_p<128, false, true>), dim3(gp, ny), dim3(512), 0, strm(stream), g,
                         (const uint16_t*)x, (const uint16_t*)wpacked, bias, (uint16_t*)y, stats_partial, tiles,
                         acfe_conv2d_stats_rows(g.M, K));
      return launch_rc("acfe_conv2d_fwd_add(persistent)");
    }
    hipLaunchKernelGGL((k_conv_fwd_g<uint16_t, 128, 128, 2, 2, true>), dim3(gm, ny), dim3(256), 0, strm(stream), g,
                       (const uint16_t*)x, (const uint16_t*)wpacked, bias, (uint16_t*)y, stats_partial, tiles_m);
    return launch_rc("acfe_conv2d_fwd_add(generic)");
  }
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, K);
  g.res = (const uint16_t*)res;
  g.res_relu = relu ? 1 : 0;
  const int srows = grid_m_for(g.M, 1);
  if (K == 128)
    return launch_rows<128, 3>(g, x, wpacked, bias, y, stats_partial, srows, nullptr, strm(stream),
                               "acfe_conv2d_fwd_add");
  return launch_rows<64, 3>(g, x, wpacked, bias, y, stats_partial, srows, nullptr, strm(stream),
                            "acfe_conv2d_fwd_add");
}

// ------------------------------------------------------------------ BatchNormalization (+ReLU) prologue
// The pre-activation BN -> ReLU -> Conv2D 3x3 of wr_resnet_bird's blocks
// (resnet/wr_resnet_bird.py:136-145 bn2a -> conv21, :152-161 bn2b -> conv2b)
// as one pass: the conv reads the BN input x and stages x' = (ReLU)(x * scale
// + shift) (acfe_bn_apply's values), so no separate apply pass reads x and
// writes x'; x' is still written (x_bn_out, nullable) for the weight gradient,
// from the staging registers of the tile's own pixels.  Shapes: K = 64, C % 64
// == 0, C <= 256, 3x3 stride-1 "same" bf16 (the stage-1 layers).
// K = 64: k_conv3x3_rows PRO; K = C = 128: k_conv3x3_1w PRO (one image < 2^31 bytes)
ACFE_API int acfe_conv2d_bn_prologue_supported(int N, int H, int W, int C, int K, int dtype) {
  return acfe_conv2d_rows_supported(N, H, W, C, K, 3, 3, dtype) &&
         ((K == 64 && C <= 256) || (K == 128 && C == 128 && (long long)H * W * 128 * 2 < (1ll << 31))) &&
         (long long)N * H * W * K < (1ll << 32);
}

static bool pro_args_ok(const float* sc, const float* sh, const void* xo) {
  return sc && sh && ((uintptr_t)sc & 15) == 0 && ((uintptr_t)sh & 15) == 0 && ((uintptr_t)xo & 15) == 0;
}

ACFE_API int acfe_conv2d_fwd_bn(const void* x, int N, int H, int W, int C, const void* wpacked, int K, int pad_top,
                                int pad_left, const float* bias, void* y, double* stats_partial, float drop_rate,
                                unsigned long long seed, const float* bn_scale, const float* bn_shift, int bn_relu,
                                void* x_bn_out, int dtype, void* stream) {
  if (!x || !wpacked || !y || !acfe_conv2d_bn_prologue_supported(N, H, W, C, K, dtype) ||
      !pro_args_ok(bn_scale, bn_shift, x_bn_out) || ((uintptr_t)x & 15) || drop_rate < 0.f || drop_rate >= 1.f)
    return ACFE_E_INVAL;
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, K);
  g.drop = make_drop(drop_rate, seed);
  g.pro_sc = bn_scale;
  g.pro_sh = bn_shift;
  g.pro_relu = bn_relu ? 1 : 0;
  g.pro_out = (uint16_t*)x_bn_out;
  const int srows = grid_m_for(g.M, 1);
  if (K == 128) return launch_plain1w(g, x, wpacked, bias, y, stats_partial, srows, strm(stream), "acfe_conv2d_fwd_bn", 0);
  if (g.drop.on)
    return launch_rows<64, 4>(g, x, wpacked, bias, y, stats_partial, srows, nullptr, strm(stream),
                              "acfe_conv2d_fwd_bn");
  return launch_rows<64, 0>(g, x, wpacked, bias, y, stats_partial, srows, nullptr, strm(stream),
                            "acfe_conv2d_fwd_bn");
}

// ---- dropout keep bits (the K = 64 stage-1 Conv2D -> Dropout -> BN nodes,
// resnet/wr_resnet.py:58-71, resnet/wr_resnet_bird.py:136-161): the forward
// writes one bit per element, [N][H][W][K / 8] bytes, the BN-fold weight
// gradient reads them instead of regenerating the pair hashes
ACFE_API int acfe_conv2d_dropout_keep_supported(int N, int H, int W, int C, int K, int dtype) {
  const int nch = C / 64;
  return acfe::r64_enabled() && dtype == ACFE_DTYPE_BF16 && N > 0 && H > 0 && W > 0 && K == 64 && C % 64 == 0 &&
         (nch == 1 || nch == 2 || nch == 4) && (long long)H * W * C * 2 < (1ll << 31) &&
         (long long)H * W * K * 2 < (1ll << 31) && (long long)N * H * W * K < (1ll << 32) &&
         (long long)N * ((H + 7) / 8) * ((W + 63) / 64) < (1ll << 31);
}

static int keep_launch(ConvGeom& g, const void* x, const void* wpacked, const float* bias, void* y,
                       double* stats, uint8_t* keep, hipStream_t s, const char* what) {
  if (!keep || !g.drop.on || !acfe_conv2d_dropout_keep_supported(g.N, g.H, g.W, g.C, g.K, ACFE_DTYPE_BF16))
    return ACFE_E_INVAL;
  g.keep_out = keep;
  return launch_r64(g, x, wpacked, bias, y, stats, grid_m_for(g.M, 1), s, what, 4);
}

ACFE_API int acfe_conv2d_fwd_dropout_keep(const void* x, int N, int H, int W, int C, const void* wpacked, int K,
                                          int pad_top, int pad_left, const float* bias, void* y, double* stats_partial,
                                          float drop_rate, unsigned long long seed, uint8_t* keep, void* stream) {
  if (!x || !wpacked || !y || drop_rate <= 0.f || drop_rate >= 1.f || pad_top != 1 || pad_left != 1 ||
      ((uintptr_t)x & 15) || ((uintptr_t)y & 15))
    return ACFE_E_INVAL;
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, K);
  g.drop = make_drop(drop_rate, seed);
  return keep_launch(g, x, wpacked, bias, y, stats_partial, keep, strm(stream), "acfe_conv2d_fwd_dropout_keep");
}

ACFE_API int acfe_conv2d_fwd_bn_keep(const void* x, int N, int H, int W, int C, const void* wpacked, int K,
                                     int pad_top, int pad_left, const float* bias, void* y, double* stats_partial,
                                     float drop_rate, unsigned long long seed, const float* bn_scale,
                                     const float* bn_shift, int bn_relu, void* x_bn_out, uint8_t* keep, int dtype,
                                     void* stream) {
  if (!x || !wpacked || !y || dtype != ACFE_DTYPE_BF16 || !acfe_conv2d_bn_prologue_supported(N, H, W, C, K, dtype) ||
      !pro_args_ok(bn_scale, bn_shift, x_bn_out) || ((uintptr_t)x & 15) || drop_rate <= 0.f || drop_rate >= 1.f ||
      pad_top != 1 || pad_left != 1)
    return ACFE_E_INVAL;
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, K);
  g.drop = make_drop(drop_rate, seed);
  g.pro_sc = bn_scale;
  g.pro_sh = bn_shift;
  g.pro_relu = bn_relu ? 1 : 0;
  g.pro_out = (uint16_t*)x_bn_out;
  return keep_launch(g, x, wpacked, bias, y, stats_partial, keep, strm(stream), "acfe_conv2d_fwd_bn_keep");
}

ACFE_API int acfe_conv2d_fwd_add_bn(const void* x, int N, int H, int W, int C, const void* wpacked, int K,
                                    int pad_top, int pad_left, const float* bias, const void* res, int relu, void* y,
                                    double* stats_partial, const float* bn_scale, const float* bn_shift, int bn_relu,
                                    void* x_bn_out, int dtype, void* stream) {
  if (!x || !wpacked || !y || !res || !acfe_conv2d_bn_prologue_supported(N, H, W, C, K, dtype) ||
      !pro_args_ok(bn_scale, bn_shift, x_bn_out) || ((uintptr_t)x & 15) || ((uintptr_t)y & 7) ||
      ((uintptr_t)res & 7))
    return ACFE_E_INVAL;
  ConvGeom g = make_geom(N, H, W, C, K, 3, 3, 1, pad_top, pad_left, H, W, 64, K);
  g.res = (const uint16_t*)res;
  g.res_relu = relu ? 1 : 0;
  g.pro_sc = bn_scale;
  g.pro_sh = bn_shift;
  g.pro_relu = bn_relu ? 1 : 0;
  g.pro_out = (uint16_t*)x_bn_out;
  const int srows = grid_m_for(g.M, 1);
  if (K == 128)
    return launch_plain1w(g, x, wpacked, bias, y, stats_partial, srows, strm(stream), "acfe_conv2d_fwd_add_bn", 3);
  return launch_rows<64, 3>(g, x, wpacked, bias, y, stats_partial, srows, nullptr, strm(stream),
                            "acfe_conv2d_fwd_add_bn");
}

// ------------------------------------------------------------------ stem (C = 1)
// y[n,h,w,k] = sum_{r,s} x[n, h - pt + r, w - pl + s] * weff[k][r][s] + b[k]
// (stride 1, P = H, Q = W).  Tile: 16 rows x 64 cols; thread = one column x
// 4 rows (lane = column, so LDS reads of consecutive lanes are consecutive
// words or 32 B pixels: conflict-free).  The 16 x R x S weights are read
// with wave-uniform indices (scalar loads), all R x S x 16 taps unrolled.
constexpr int STEM_TH = 16, STEM_TW = 64, STEM_K = 16, STEM_MAXR = 7, STEM_CAP = 2048;

// 16 channels of one pixel (32 B bf16 / 64 B fp32) from LDS -> fp32
__device__ __forceinline__ void unpack16(const uint16_t* p, float* f) {
  const u32x4 a = *reinterpret_cast<const u32x4*>(p), b = *reinterpret_cast<const u32x4*>(p + 8);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(a[i] << 16);
    f[2 * i + 1] = __uint_as_float(a[i] & 0xffff0000u);
    f[8 + 2 * i] = __uint_as_float(b[i] << 16);
    f[8 + 2 * i + 1] = __uint_as_float(b[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void unpack16(const float* p, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f4 v = *reinterpret_cast<const f4*>(p + 4 * i);
    f[4 * i] = v[0]; f[4 * i + 1] = v[1]; f[4 * i + 2] = v[2]; f[4 * i + 3] = v[3];
  }
}
__device__ __forceinline__ void store16(uint16_t* d, const float* f) {
  u32x4 a, b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = (unsigned)f2bf(f[2 * i]) | ((unsigned)f2bf(f[2 * i + 1]) << 16);
    b[i] = (unsigned)f2bf(f[8 + 2 * i]) | ((unsigned)f2bf(f[8 + 2 * i + 1]) << 16);
  }
  *reinterpret_cast<u32x4*>(d) = a;
  *reinterpret_cast<u32x4*>(d + 8) = b;
}
__device__ __forceinline__ void store16(float* d, const float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f4 v = {f[4 * i], f[4 * i + 1], f[4 * i + 2], f[4 * i + 3]};
    *reinterpret_cast<f4*>(d + 4 * i) = v;
  }
}

// x halo tile (single channel) -> fp32 LDS, zero outside the image.
template <typename TI, int XH, int XW>
__device__ __forceinline__ void stem_load_x(const TI* __restrict__ x, int n, int H, int W, int gh0, int gw0,
                                            float* xs) {
  for (int i = threadIdx.x; i < XH * XW; i += 256) {
    const int yy = i / XW, xx = i - (i / XW) * XW;
    const int h = gh0 + yy, w = gw0 + xx;
    float v = 0.f;
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) v = to_f(x[((long long)n * H + h) * W + w]);
    xs[i] = v;
  }
}

// Folded weights are laid out weff[r][s][k] (RSK): the 16 weights of one tap
// are one 64 B scalar load, used as SGPR operands of v_fmac.
template <typename TI, typename TO, int R, int S>
__global__ void __launch_bounds__(256)
k_stem_fwd(const TI* __restrict__ x, int N, int H, int W, int pt, int pl,
           const float* __restrict__ weff, const float* __restrict__ bias, TO* __restrict__ y,
           double* __restrict__ stats, int tiles_h, int tiles_w) {
  constexpr int XH = STEM_TH + R - 1, XW = STEM_TW + S - 1, RH = 4 + R - 1;
  __shared__ float xs[XH * XW];
  __shared__ double red[4][2][STEM_K];
  const int tid = threadIdx.x, ox = tid & 63, q = tid >> 6;
  const long long ntiles = (long long)N * tiles_h * tiles_w;
  double s1[STEM_K], s2[STEM_K];
#pragma unroll
  for (int k = 0; k < STEM_K; ++k) s1[k] = 0.0, s2[k] = 0.0;
  for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tw = (int)(t % tiles_w);
    const int th = (int)((t / tiles_w) % tiles_h);
    const int n = (int)(t / ((long long)tiles_w * tiles_h));
    const int h0 = th * STEM_TH, w0 = tw * STEM_TW;
    __syncthreads();
    stem_load_x<TI, XH, XW>(x, n, H, W, h0 - pt, w0 - pl, xs);
    __syncthreads();
    float acc[4][STEM_K];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < STEM_K; ++k) acc[j][k] = bias ? bias[k] : 0.f;
    // column s of the thread's halo: RH values; output row j uses halo row j + r
#pragma unroll 1
    for (int s = 0; s < S; ++s) {
      float xc[RH];
#pragma unroll
      for (int i = 0; i < RH; ++i) xc[i] = xs[(4 * q + i) * XW + ox + s];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float* wt = weff + (r * S + s) * STEM_K;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int k = 0; k < STEM_K; ++k) acc[j][k] += xc[j + r] * wt[k];
      }
    }
    const int w = w0 + ox;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = h0 + 4 * q + j;
      if (h < H && w < W) {
        float o[STEM_K];
#pragma unroll
        for (int k = 0; k < STEM_K; ++k) o[k] = to_f(cvt_out(acc[j][k], TO()));  // stats of stored values
        store16(y + (((long long)n * H + h) * W + w) * STEM_K, o);
        if (stats) {
#pragma unroll
          for (int k = 0; k < STEM_K; ++k) s1[k] += o[k], s2[k] += (double)o[k] * o[k];
        }
      }
    }
  }
  if (stats) {
    const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
    for (int k = 0; k < STEM_K; ++k) {
      const double a = wave_sumd(s1[k]), b = wave_sumd(s2[k]);
      if (lane == 0) red[wid][0][k] = a, red[wid][1][k] = b;
    }
    __syncthreads();
    if (tid < 2 * STEM_K) {
      const int which = tid / STEM_K, k = tid % STEM_K;
      stats[((long long)blockIdx.x * 2 + which) * STEM_K + k] =
          red[0][which][k] + red[1][which][k] + red[2][which][k] + red[3][which][k];
    }
  }
}

// dx[n,h,w] = sum_{k,r,s} dy[n, h + pt - r, w + pl - s, k] * weff[r][s][k]
// dy halo tile kept pixel-major in LDS (16 channels = 32 B per pixel, copied
// with 16 B loads/stores); one tile per block.  Per halo column the thread
// holds its RH x 16 dy values in registers and applies all R taps of that
// column to its 4 output rows.
template <typename TG, typename TO, int R, int S>
__global__ void __launch_bounds__(256)
k_stem_dgrad(const TG* __restrict__ dy, int N, int H, int W, int pt, int pl,
             const float* __restrict__ weff, TO* __restrict__ dx, int tiles_h, int tiles_w) {
  constexpr int XH = STEM_TH + R - 1, XW = STEM_TW + S - 1, RH = 4 + R - 1;
  constexpr int CPP = STEM_K * (int)sizeof(TG) / 16;  // 16 B chunks per pixel
  __shared__ __attribute__((aligned(16))) TG gs[XH * XW * STEM_K];
  const int tid = threadIdx.x, ox = tid & 63, q = tid >> 6;
  const long long t = blockIdx.x;
  const int tw = (int)(t % tiles_w);
  const int th = (int)((t / tiles_w) % tiles_h);
  const int n = (int)(t / ((long long)tiles_w * tiles_h));
  const int h0 = th * STEM_TH, w0 = tw * STEM_TW;
  const int gh0 = h0 - (R - 1 - pt), gw0 = w0 - (S - 1 - pl);
  for (int i = tid; i < XH * XW * CPP; i += 256) {
    const int pos = i / CPP, c = i - (i / CPP) * CPP;
    const int yy = pos / XW, xx = pos - (pos / XW) * XW;
    const int h = gh0 + yy, w = gw0 + xx;
    u32x4 v = {0u, 0u, 0u, 0u};
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
      v = *reinterpret_cast<const u32x4*>(dy + (((long long)n * H + h) * W + w) * STEM_K + c * (16 / (int)sizeof(TG)));
    *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(gs) + (long long)i * 16) = v;
  }
  __syncthreads();
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // halo row 4q + i, col ox + cc holds dy for output row j with r = j + R-1-i, s = S-1-cc
#pragma unroll 1
  for (int cc = 0; cc < S; ++cc) {
    float g[RH][STEM_K];
#pragma unroll
    for (int i = 0; i < RH; ++i) unpack16(gs + ((4 * q + i) * XW + ox + cc) * STEM_K, g[i]);
    const int s = S - 1 - cc;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float* wt = weff + (r * S + s) * STEM_K;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < STEM_K; ++k) acc[j] += g[j + R - 1 - r][k] * wt[k];
    }
  }
  const int w = w0 + ox;
  if (w < W) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = h0 + 4 * q + j;
      if (h < H) dx[((long long)n * H + h) * W + w] = cvt_out(acc[j], TO());
    }
  }
}

// dweff[k][r][s] partials per block: thread -> (column ox = lane, channels
// 4*kq .. 4*kq+3 with kq = wave), R*S*4 fp32 accumulators over the block's
// tiles, reduced across the wave in double at the end.  The x window of the
// thread (R rows x S cols) slides down the tile in registers.
template <typename TI, typename TG, int R, int S>
__global__ void __launch_bounds__(256)
k_stem_wgrad(const TI* __restrict__ x, const TG* __restrict__ dy, int N, int H, int W, int pt,
             int pl, double* __restrict__ part, int tiles_h, int tiles_w) {
  constexpr int XH = STEM_TH + R - 1, XW = STEM_TW + S - 1;
  __shared__ float xs[XH * XW];
  const int tid = threadIdx.x, ox = tid & 63, kq = tid >> 6;
  float acc[4][R * S];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int i = 0; i < R * S; ++i) acc[kk][i] = 0.f;
  const long long ntiles = (long long)N * tiles_h * tiles_w;
  for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tw = (int)(t % tiles_w);
    const int th = (int)((t / tiles_w) % tiles_h);
    const int n = (int)(t / ((long long)tiles_w * tiles_h));
    const int h0 = th * STEM_TH, w0 = tw * STEM_TW;
    __syncthreads();
    stem_load_x<TI, XH, XW>(x, n, H, W, h0 - pt, w0 - pl, xs);
    __syncthreads();
    const int w = w0 + ox;
    float win[R][S];
#pragma unroll
    for (int r = 0; r < R - 1; ++r)
#pragma unroll
      for (int s = 0; s < S; ++s) win[r + 1][s] = xs[r * XW + ox + s];
#pragma unroll 1
    for (int oy = 0; oy < STEM_TH; ++oy) {
#pragma unroll
      for (int r = 0; r < R - 1; ++r)
#pragma unroll
        for (int s = 0; s < S; ++s) win[r][s] = win[r + 1][s];
#pragma unroll
      for (int s = 0; s < S; ++s) win[R - 1][s] = xs[(oy + R - 1) * XW + ox + s];
      const int h = h0 + oy;
      float g[4] = {0.f, 0.f, 0.f, 0.f};
      if (h < H && w < W) {
        const TG* gp = dy + (((long long)n * H + h) * W + w) * STEM_K + 4 * kq;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) g[kk] = to_f(gp[kk]);
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) acc[kk][r * S + s] += g[kk] * win[r][s];
    }
  }
  const int lane = tid & 63;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int i = 0; i < R * S; ++i) {
      const double v = wave_sumd((double)acc[kk][i]);
      if (lane == 0) part[(long long)blockIdx.x * STEM_K * R * S + (4 * kq + kk) * R * S + i] = v;
    }
}

// dweff partials [blocks][k][r][s] -> dw[k][r][s][rep] (+beta*dw); one block per tap.
__global__ void k_stem_wgrad_reduce(const double* __restrict__ part, int np, int n, int rep, float beta,
                                    float* __restrict__ dw) {
  __shared__ double red[4];
  const int i = blockIdx.x;
  double s = 0.0;
  for (int j = threadIdx.x; j < np; j += 256) s += part[(long long)j * n + i];
  s = wave_sumd(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x < rep) {
    const double tot = red[0] + red[1] + red[2] + red[3];
    float* d = dw + (long long)i * rep + threadIdx.x;
    *d = beta != 0.f ? *d * beta + (float)tot : (float)tot;
  }
}

// weff[r][s][k] = sum_c w[k][r][s][c]  (folds the identical input channels)
__global__ void k_stem_fold(const float* __restrict__ w, int K, int RS, int rep, float* __restrict__ weff) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < K * RS; i += gridDim.x * 256) {
    const int k = i % K, rs = i / K;
    float s = 0.f;
    for (int c = 0; c < rep; ++c) s += w[((long long)k * RS + rs) * rep + c];
    weff[i] = s;
  }
}

// ---- MFMA stem (bf16 activations; R*S <= 32 taps) -------------------------
// Same tiles (16 rows x 64 columns, grid-stride) and slab contracts as the
// VALU kernels above; the 5x5 taps become the 32-deep reduction of
// v_mfma_f32_16x16x32_bf16 (zero-padded from 25), so the VALU work per pixel
// is an LDS gather instead of 400 FMAs:
//   fwd:   D[k][px] = sum_t weff[t][k] * x[px + off_t]      (A = weights, B = im2col gather)
//   dgrad: D[.][px] = sum_{t,k} dy[px - off_t][k] weff[t][k] (B = 16-B dy reads, 2 taps x 16
//          channels per k-step; the A rows are replicated, one row is the result)
//   wgrad: D[k][t]  = sum_px dy[px][k] * x[px + off_t]      (A = dy chunk read transposed,
//          B = im2col gather; k-dimension = 32 pixels of one row)
// Weights are bf16 (the VALU kernels keep fp32 weights: the fp32 path).
typedef __attribute__((address_space(3))) bf4* stem_lp;

__device__ __forceinline__ unsigned stem_pack2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}

template <int R, int S>
__global__ void __launch_bounds__(256)
k_stem_fwd_mfma(const uint16_t* __restrict__ x, int N, int H, int W, int pt, int pl, const float* __restrict__ weff,
                const float* __restrict__ bias, uint16_t* __restrict__ y, double* __restrict__ stats, int tiles_h,
                int tiles_w) {
  constexpr int XH = STEM_TH + R - 1, XW = STEM_TW + S - 1, NT = R * S;
  static_assert(NT <= 32, "taps");
  __shared__ uint16_t xs[XH * XW];
  __shared__ double red[2][STEM_K];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4, wid = tid >> 6;
  for (int i = tid; i < 2 * STEM_K; i += 256) (&red[0][0])[i] = 0.0;
  uint4 wa;
  int toff[8];
  {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = q * 8 + j;
      v[j] = t < NT ? weff[t * STEM_K + l16] : 0.f;
      toff[j] = t < NT ? (t / S) * XW + (t % S) : 0;
    }
    wa = uint4{stem_pack2(v[0], v[1]), stem_pack2(v[2], v[3]), stem_pack2(v[4], v[5]), stem_pack2(v[6], v[7])};
  }
  float bk[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bk[r] = bias ? bias[q * 4 + r] : 0.f;
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  const long long ntiles = (long long)N * tiles_h * tiles_w;
  for (long long tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
    const int tw = (int)(tt % tiles_w), th = (int)((tt / tiles_w) % tiles_h);
    const int n = (int)(tt / ((long long)tiles_w * tiles_h));
    const int h0 = th * STEM_TH, w0 = tw * STEM_TW;
    __syncthreads();
    for (int i = tid; i < XH * XW; i += 256) {
      const int yy = i / XW, xx = i - yy * XW;
      const int h = h0 - pt + yy, w = w0 - pl + xx;
      xs[i] = ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) ? x[((long long)n * H + h) * W + w] : 0;
    }
    __syncthreads();
#pragma unroll 2
    for (int blk = 0; blk < 16; ++blk) {
      const int ry = wid * 4 + (blk >> 2), cx = (blk & 3) * 16 + l16;
      const uint16_t* src = xs + ry * XW + cx;
      unsigned tv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) tv[j] = (q * 8 + j < NT) ? src[toff[j]] : 0u;
      const uint4 b = uint4{tv[0] | (tv[1] << 16), tv[2] | (tv[3] << 16), tv[4] | (tv[5] << 16), tv[6] | (tv[7] << 16)};
      const f4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, wa), __builtin_bit_cast(bf8, b),
                                                             f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const int h = h0 + ry, w = w0 + cx;
      if (h < H && w < W) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = bf2f(f2bf(acc[r] + bk[r]));
        *reinterpret_cast<uint2*>(y + (((long long)n * H + h) * W + w) * STEM_K + q * 4) =
            uint2{stem_pack2(o[0], o[1]), stem_pack2(o[2], o[3])};
        if (stats) {
#pragma unroll
          for (int r = 0; r < 4; ++r) s1[r] += o[r], s2[r] += (double)o[r] * o[r];
        }
      }
    }
  }
  if (stats) {
    // lanes with the same q hold the same 4 channels: reduce over l16
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        s1[r] += __shfl_xor(s1[r], o, 64);
        s2[r] += __shfl_xor(s2[r], o, 64);
      }
    }
    __syncthreads();
    if (l16 == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        atomicAdd(&red[0][q * 4 + r], s1[r]);
        atomicAdd(&red[1][q * 4 + r], s2[r]);
      }
    }
    __syncthreads();
    if (tid < 2 * STEM_K) stats[(long long)blockIdx.x * 2 * STEM_K + tid] = (&red[0][0])[tid];
  }
}

template <int R, int S>
__global__ void __launch_bounds__(256)
k_stem_dgrad_mfma(const uint16_t* __restrict__ dy, int N, int H, int W, int pt, int pl,
                  const float* __restrict__ weff, uint16_t* __restrict__ dx, int tiles_h, int tiles_w) {
  constexpr int XH = STEM_TH + R - 1, XW = STEM_TW + S - 1, NT = R * S, NKT = (NT + 1) / 2;
  __shared__ __attribute__((aligned(16))) uint16_t gs[XH * XW * STEM_K];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4, wid = tid >> 6;
  // k-step kt: k-slot q*8 + j <-> (tap 2kt + (q >> 1), channel (q & 1)*8 + j); A rows replicated
  uint4 wa[NKT];
  int goff[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const int t = 2 * kt + (q >> 1), r = t / S, s = t % S;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t < NT ? weff[t * STEM_K + (q & 1) * 8 + j] : 0.f;
    wa[kt] = uint4{stem_pack2(v[0], v[1]), stem_pack2(v[2], v[3]), stem_pack2(v[4], v[5]), stem_pack2(v[6], v[7])};
    goff[kt] = t < NT ? ((R - 1 - r) * XW + (S - 1 - s)) * STEM_K + (q & 1) * 8 : -1;
  }
  const uint4 z4 = {0u, 0u, 0u, 0u};
  const long long ntiles = (long long)N * tiles_h * tiles_w;
  for (long long tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
    const int tw = (int)(tt % tiles_w), th = (int)((tt / tiles_w) % tiles_h);
    const int n = (int)(tt / ((long long)tiles_w * tiles_h));
    const int h0 = th * STEM_TH, w0 = tw * STEM_TW;
    const int gh0 = h0 - (R - 1 - pt), gw0 = w0 - (S - 1 - pl);
    __syncthreads();
    for (int i = tid; i < XH * XW * 2; i += 256) {
      const int pos = i >> 1, c = i & 1;
      const int yy = pos / XW, xx = pos - yy * XW;
      const int h = gh0 + yy, w = gw0 + xx;
      u32x4 v = {0u, 0u, 0u, 0u};
      if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
        v = *reinterpret_cast<const u32x4*>(dy + (((long long)n * H + h) * W + w) * STEM_K + c * 8);
      *reinterpret_cast<u32x4*>(gs + (long long)i * 8) = v;
    }
    __syncthreads();
#pragma unroll 2
    for (int blk = 0; blk < 16; ++blk) {
      const int ry = wid * 4 + (blk >> 2), cx = (blk & 3) * 16 + l16;
      const uint16_t* base = gs + (ry * XW + cx) * STEM_K;
      f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const uint4 b = goff[kt] >= 0 ? *reinterpret_cast<const uint4*>(base + goff[kt]) : z4;
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, wa[kt]), __builtin_bit_cast(bf8, b), acc,
                                                      0, 0, 0);
      }
      const int h = h0 + ry, w = w0 + cx;
      if (q == 0 && h < H && w < W) dx[((long long)n * H + h) * W + w] = f2bf(acc[0]);
    }
  }
}

template <int R, int S>
__global__ void __launch_bounds__(256)
k_stem_wgrad_mfma(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy, int N, int H, int W, int pt,
                  int pl, double* __restrict__ part, int tiles_h, int tiles_w) {
  constexpr int XH = STEM_TH + R - 1, XW = STEM_TW + S - 1, NT = R * S, LDG = 24;
  __shared__ uint16_t xs[XH * XW];
  __shared__ __attribute__((aligned(16))) uint16_t gch[4][32 * LDG];  // per wave: 32 px x 16 ch of dy
  __shared__ float red[4][STEM_K][32];
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4, wid = tid >> 6;
  const int grp = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  // B k-slot (q, j) <-> chunk pixel j<4: 4q+j, else 16+4q+(j-4) (the transposed-read order)
  int tof0, tof1;
  {
    const int t0 = l16, t1 = 16 + l16;
    tof0 = t0 < NT ? (t0 / S) * XW + (t0 % S) : -1;
    tof1 = t1 < NT ? (t1 / S) * XW + (t1 % S) : -1;
  }
  f4 d0 = f4{0.f, 0.f, 0.f, 0.f}, d1 = d0;
  uint16_t* gw = gch[wid];
  const long long ntiles = (long long)N * tiles_h * tiles_w;
  for (long long tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
    const int tw = (int)(tt % tiles_w), th = (int)((tt / tiles_w) % tiles_h);
    const int n = (int)(tt / ((long long)tiles_w * tiles_h));
    const int h0 = th * STEM_TH, w0 = tw * STEM_TW;
    __syncthreads();
    for (int i = tid; i < XH * XW; i += 256) {
      const int yy = i / XW, xx = i - yy * XW;
      const int h = h0 - pt + yy, w = w0 - pl + xx;
      xs[i] = ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) ? x[((long long)n * H + h) * W + w] : 0;
    }
    __syncthreads();
    for (int c = 0; c < 8; ++c) {  // the wave's 4 rows x 64 columns in 32-pixel chunks
      const int ry = wid * 4 + (c >> 1), cx0 = (c & 1) * 32;
      const int h = h0 + ry;
      {
        const int px = lane >> 1, half = lane & 1, w = w0 + cx0 + px;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (h < H && w < W)
          v = *reinterpret_cast<const u32x4*>(dy + (((long long)n * H + h) * W + w) * STEM_K + half * 8);
        *reinterpret_cast<u32x4*>(gw + px * LDG + half * 8) = v;
      }
      const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (stem_lp)(reinterpret_cast<const __bf16*>(gw + (4 * grp + qq) * LDG + 4 * pp)));
      const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (stem_lp)(reinterpret_cast<const __bf16*>(gw + (16 + 4 * grp + qq) * LDG + 4 * pp)));
      const bf8 a = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const uint16_t* src = xs + ry * XW + cx0;
      unsigned b0[8], b1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int px = j < 4 ? 4 * q + j : 16 + 4 * q + (j - 4);
        b0[j] = tof0 >= 0 ? src[px + tof0] : 0u;
        b1[j] = tof1 >= 0 ? src[px + tof1] : 0u;
      }
      const uint4 B0 = uint4{b0[0] | (b0[1] << 16), b0[2] | (b0[3] << 16), b0[4] | (b0[5] << 16), b0[6] | (b0[7] << 16)};
      const uint4 B1 = uint4{b1[0] | (b1[1] << 16), b1[2] | (b1[3] << 16), b1[4] | (b1[5] << 16), b1[6] | (b1[7] << 16)};
      d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf8, B0), d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf8, B1), d1, 0, 0, 0);
    }
  }
  // D lane: row k = q*4 + r, column t = l16 (+16)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wid][q * 4 + r][l16] = d0[r];
    red[wid][q * 4 + r][16 + l16] = d1[r];
  }
  __syncthreads();
  for (int i = tid; i < STEM_K * NT; i += 256) {
    const int k = i / NT, t = i - k * NT;
    part[(long long)blockIdx.x * STEM_K * NT + i] =
        ((double)red[0][k][t] + (double)red[1][k][t]) + ((double)red[2][k][t] + (double)red[3][k][t]);
  }
}


// ------------------------------------------------------------------ stem backward with the BN backward apply
// wr_resnet_bird's stem conv1_1 (5 x 5, 16 filters, bias) -> BatchNormalization
// -> MaxPool2D((1, 2)) (resnet/wr_resnet_bird.py:22-30).  The BN backward's
// elementwise pass dX_bn = a*g*[x*scale+shift > 0] + b*x + c (k_bn_bwd_apply8:
// reads g and x, writes dX_bn, 3 x 1.07 GB per T1 step) is formed while the
// stem dgrad stages its dY halo; the weight gradient and the conv-bias sums
// read the same LDS image, so dX_bn is never stored and the separate wgrad's
// re-read of it is gone.  dX bit-identical to the apply8 -> k_stem_dgrad_mfma
// chain (the same bf16 dX_bn and MFMA operands); dW the k_stem_wgrad_mfma
// arithmetic over stem_bwd_grid's workgroups (its fp32 partials summed in
// another grouping than acfe_stem_wgrad's); bias sums [block][2][16] of the
// bf16 dX_bn values over each tile's own pixels.
template <int R, int S>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
k_stem_bwd_bn(const uint16_t* __restrict__ g, const uint16_t* __restrict__ xb, const uint16_t* __restrict__ xin,
              int N, int H, int W, int pt, int pl, const float* __restrict__ weff, const float* __restrict__ scale,
              const float* __restrict__ shift, const float* __restrict__ coef, int relu, uint16_t* __restrict__ dxin,
              double* __restrict__ wpart, double* __restrict__ bpart, int tiles_h, int tiles_w) {
  constexpr int XH = STEM_TH + R - 1, XW = STEM_TW + S - 1, NT = R * S, NKT = (NT + 1) / 2;
  constexpr int GSZ = XH * XW * STEM_K;
  static_assert(GSZ * 2 >= 4 * STEM_K * 32 * 4, "the wgrad reduction aliases the dY image");
  __shared__ __attribute__((aligned(16))) uint16_t gs[GSZ];
  __shared__ uint16_t xs[XH * XW];
  __shared__ double bred[4][STEM_K];
  __shared__ __attribute__((aligned(16))) float bnc[5][STEM_K];  // scale, shift, coef a, b, c
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4, wid = tid >> 6;
  if (tid < 5 * STEM_K) {
    const int a = tid / STEM_K, k = tid - a * STEM_K;
    bnc[a][k] = a == 0 ? scale[k] : (a == 1 ? shift[k] : coef[(a - 2) * STEM_K + k]);
  }
  // dgrad A operand (k_stem_dgrad_mfma): flipped folded weights, k-slot q*8 + j <-> (tap 2kt + (q >> 1), ch (q & 1)*8 + j)
  uint4 wa[NKT];
  int goff[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const int t = 2 * kt + (q >> 1), r = t / S, s = t % S;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t < NT ? weff[t * STEM_K + (q & 1) * 8 + j] : 0.f;
    wa[kt] = uint4{stem_pack2(v[0], v[1]), stem_pack2(v[2], v[3]), stem_pack2(v[4], v[5]), stem_pack2(v[6], v[7])};
    goff[kt] = t < NT ? ((R - 1 - r) * XW + (S - 1 - s)) * STEM_K + (q & 1) * 8 : -1;
  }
  // wgrad B operand (k_stem_wgrad_mfma): tap of column l16 / 16 + l16
  const int grp = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  int tof0, tof1;
  {
    const int t0 = l16, t1 = 16 + l16;
    tof0 = t0 < NT ? (t0 / S) * XW + (t0 % S) : -1;
    tof1 = t1 < NT ? (t1 / S) * XW + (t1 % S) : -1;
  }
  // this thread's 8 staging channels: its index parity
  const int c8 = (tid & 1) * 8;
  double s1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = 0.0;
  f4 d0 = f4{0.f, 0.f, 0.f, 0.f}, d1 = d0;
  const uint4 z4 = {0u, 0u, 0u, 0u};
  const long long ntiles = (long long)N * tiles_h * tiles_w;
  for (long long tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
    const int tw = (int)(tt % tiles_w), th = (int)((tt / tiles_w) % tiles_h);
    const int n = (int)(tt / ((long long)tiles_w * tiles_h));
    const int h0 = th * STEM_TH, w0 = tw * STEM_TW;
    const int gh0 = h0 - (R - 1 - pt), gw0 = w0 - (S - 1 - pl);
    __syncthreads();
    for (int i = tid; i < XH * XW * 2; i += 256) {
      const int pos = i >> 1;
      const int yy = pos / XW, xx = pos - yy * XW;
      const int h = gh0 + yy, w = gw0 + xx;
      u32x4 v = {0u, 0u, 0u, 0u};
      if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
        const long long e = (((long long)n * H + h) * W + w) * STEM_K + c8;
        const u32x4 gv = *reinterpret_cast<const u32x4*>(g + e);
        const u32x4 xv = *reinterpret_cast<const u32x4*>(xb + e);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned gw = gv[j >> 1], xw = xv[j >> 1];
          const float gf = __uint_as_float((j & 1) ? (gw & 0xffff0000u) : (gw << 16));
          const float xf = __uint_as_float((j & 1) ? (xw & 0xffff0000u) : (xw << 16));
          const float gj = (relu && !(xf * bnc[0][c8 + j] + bnc[1][c8 + j] > 0.f)) ? 0.f : gf;
          o[j] = __builtin_fmaf(bnc[2][c8 + j], gj, __builtin_fmaf(bnc[3][c8 + j], xf, bnc[4][c8 + j]));  // as k_bn_bwd_apply8
        }
        v = u32x4{stem_pack2(o[0], o[1]), stem_pack2(o[2], o[3]), stem_pack2(o[4], o[5]), stem_pack2(o[6], o[7])};
        if ((unsigned)(yy - (R - 1 - pt)) < (unsigned)STEM_TH && (unsigned)(xx - (S - 1 - pl)) < (unsigned)STEM_TW) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const unsigned vw = v[j >> 1];
            s1[j] += (double)__uint_as_float((j & 1) ? (vw & 0xffff0000u) : (vw << 16));
          }
        }
      }
      *reinterpret_cast<u32x4*>(gs + (long long)i * 8) = v;
    }
    for (int i = tid; i < XH * XW; i += 256) {
      const int yy = i / XW, xx = i - yy * XW;
      const int h = h0 - pt + yy, w = w0 - pl + xx;
      xs[i] = ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) ? xin[((long long)n * H + h) * W + w] : 0;
    }
    __syncthreads();
    // dX of the stem input (k_stem_dgrad_mfma)
#pragma unroll 2
    for (int blk = 0; blk < 16; ++blk) {
      const int ry = wid * 4 + (blk >> 2), cx = (blk & 3) * 16 + l16;
      const uint16_t* base = gs + (ry * XW + cx) * STEM_K;
      f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const uint4 b = goff[kt] >= 0 ? *reinterpret_cast<const uint4*>(base + goff[kt]) : z4;
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, wa[kt]), __builtin_bit_cast(bf8, b), acc,
                                                      0, 0, 0);
      }
      const int h = h0 + ry, w = w0 + cx;
      if (q == 0 && h < H && w < W) dxin[((long long)n * H + h) * W + w] = f2bf(acc[0]);
    }
    // dW (k_stem_wgrad_mfma): dY^T chunks read from the tile's own pixels of the image
    for (int c = 0; c < 8; ++c) {
      const int ry = wid * 4 + (c >> 1), cx0 = (c & 1) * 32;
      const uint16_t* gw = gs + ((ry + R - 1 - pt) * XW + cx0 + S - 1 - pl) * STEM_K;
      const bf4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (stem_lp)(reinterpret_cast<const __bf16*>(gw + (4 * grp + qq) * STEM_K + 4 * pp)));
      const bf4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (stem_lp)(reinterpret_cast<const __bf16*>(gw + (16 + 4 * grp + qq) * STEM_K + 4 * pp)));
      const bf8 a = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const uint16_t* src = xs + ry * XW + cx0;
      unsigned b0[8], b1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int px = j < 4 ? 4 * q + j : 16 + 4 * q + (j - 4);
        b0[j] = tof0 >= 0 ? src[px + tof0] : 0u;
        b1[j] = tof1 >= 0 ? src[px + tof1] : 0u;
      }
      const uint4 B0 = uint4{b0[0] | (b0[1] << 16), b0[2] | (b0[3] << 16), b0[4] | (b0[5] << 16), b0[6] | (b0[7] << 16)};
      const uint4 B1 = uint4{b1[0] | (b1[1] << 16), b1[2] | (b1[3] << 16), b1[4] | (b1[5] << 16), b1[6] | (b1[7] << 16)};
      d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf8, B0), d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf8, B1), d1, 0, 0, 0);
    }
  }
  // bias sums: lanes of one parity hold the same 8 channels
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int o = 2; o < 64; o <<= 1) s1[j] += __shfl_xor(s1[j], o, 64);
  }
  __syncthreads();  // last tile's image reads done: the wgrad reduction reuses it
  float(*red)[STEM_K][32] = reinterpret_cast<float(*)[STEM_K][32]>(gs);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wid][q * 4 + r][l16] = d0[r];
    red[wid][q * 4 + r][16 + l16] = d1[r];
  }
  if (lane < 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) bred[wid][lane * 8 + j] = s1[j];
  }
  __syncthreads();
  for (int i = tid; i < STEM_K * NT; i += 256) {
    const int k = i / NT, t = i - k * NT;
    wpart[(long long)blockIdx.x * STEM_K * NT + i] =
        ((double)red[0][k][t] + (double)red[1][k][t]) + ((double)red[2][k][t] + (double)red[3][k][t]);
  }
  // row 1 of the [2][16] slab (sums of squares in the statistics layout) is not used by the channel sums
  if (tid < 2 * STEM_K)
    bpart[(long long)blockIdx.x * 2 * STEM_K + tid] =
        tid < STEM_K ? (bred[0][tid] + bred[1][tid]) + (bred[2][tid] + bred[3][tid]) : 0.0;
}

ACFE_API int acfe_stem_blocks(int N, int H, int W) {
  const long long t = (long long)N * ((H + STEM_TH - 1) / STEM_TH) * ((W + STEM_TW - 1) / STEM_TW);
  return (int)(t < STEM_CAP ? t : STEM_CAP);
}

// weff[r][s][k] = sum_c w[k][r][s][c]  (folds the identical input channels)
ACFE_API int acfe_stem_fold_weights(const float* w, int K, int R, int S, int C, float* weff, void* stream) {
  if (!w || !weff || K != STEM_K || R > STEM_MAXR || S > STEM_MAXR || C <= 0) return ACFE_E_INVAL;
  hipLaunchKernelGGL(k_stem_fold, dim3(cdiv(K * R * S, 256)), dim3(256), 0, strm(stream), w, K, R * S, C, weff);
  return launch_rc("acfe_stem_fold_weights");
}

ACFE_API int acfe_stem_fwd(const void* x, int x_dtype, int N, int H, int W, int R, int S, int pad_top,
                           int pad_left, const float* weff, const float* bias, void* y, int y_dtype,
                           double* stats_partial, void* stream) {
  if (!x || !weff || !y || N < 0 || H <= 0 || W <= 0 || R != S || (R != 5 && R != 3)) return ACFE_E_INVAL;
  if (N == 0) return ACFE_OK;
  const int th = (H + STEM_TH - 1) / STEM_TH, tw = (W + STEM_TW - 1) / STEM_TW;
  const int grid = acfe_stem_blocks(N, H, W);
#define SF1(TI, TO, RR)                                                                                      \
  hipLaunchKernelGGL((k_stem_fwd<TI, TO, RR, RR>), dim3(grid), dim3(256), 0, strm(stream), (const TI*)x, N, H, W, \
                     pad_top, pad_left, weff, bias, (TO*)y, stats_partial, th, tw)
#define SF(TI, TO) if (R == 5) SF1(TI, TO, 5); else SF1(TI, TO, 3)
  if (x_dtype == ACFE_DTYPE_BF16 && y_dtype == ACFE_DTYPE_BF16) {
    // one resident round (7 workgroups per CU at 62 VGPRs) instead of 2048 in
    // 1.14 rounds; the statistics slab rows past the grid are zeroed
    const int g1 = grid < 7 * 256 ? grid : 7 * 256;
    if (stats_partial && g1 < grid) {
      const hipError_t e = hipMemsetAsync(stats_partial + (size_t)g1 * 2 * STEM_K, 0,
                                          sizeof(double) * 2 * STEM_K * (grid - g1), strm(stream));
      if (e != hipSuccess) return hip_rc(e, "acfe_stem_fwd");
    }
    if (R == 5)
      hipLaunchKernelGGL((k_stem_fwd_mfma<5, 5>), dim3(g1), dim3(256), 0, strm(stream), (const uint16_t*)x, N, H, W,
                         pad_top, pad_left, weff, bias, (uint16_t*)y, stats_partial, th, tw);
    else
      hipLaunchKernelGGL((k_stem_fwd_mfma<3, 3>), dim3(g1), dim3(256), 0, strm(stream), (const uint16_t*)x, N, H, W,
                         pad_top, pad_left, weff, bias, (uint16_t*)y, stats_partial, th, tw);
  } else if (x_dtype == ACFE_DTYPE_BF16 && y_dtype == ACFE_DTYPE_BF16) SF(uint16_t, uint16_t);
  else if (x_dtype == ACFE_DTYPE_BF16) SF(uint16_t, float);
  else if (y_dtype == ACFE_DTYPE_BF16) SF(float, uint16_t);
  else SF(float, float);
#undef SF
  return launch_rc("acfe_stem_fwd");
}

ACFE_API int acfe_stem_dgrad(const void* dy, int dy_dtype, int N, int H, int W, int R, int S, int pad_top,
                             int pad_left, const float* weff, void* dx, int dx_dtype, void* stream) {
  if (!dy || !weff || !dx || N < 0 || R != S || (R != 5 && R != 3)) return ACFE_E_INVAL;
  if (N == 0) return ACFE_OK;
  const int th = (H + STEM_TH - 1) / STEM_TH, tw = (W + STEM_TW - 1) / STEM_TW;
  const long long grid = (long long)N * th * tw;  // one tile per block
#define SD1(TG, TO, RR)                                                                                      \
  hipLaunchKernelGGL((k_stem_dgrad<TG, TO, RR, RR>), dim3(grid), dim3(256), 0, strm(stream), (const TG*)dy, N, H, \
                     W, pad_top, pad_left, weff, (TO*)dx, th, tw)
#define SD(TG, TO) if (R == 5) SD1(TG, TO, 5); else SD1(TG, TO, 3)
  if (dy_dtype == ACFE_DTYPE_BF16 && dx_dtype == ACFE_DTYPE_BF16) {
    const int g2 = acfe_stem_blocks(N, H, W);
    if (R == 5)
      hipLaunchKernelGGL((k_stem_dgrad_mfma<5, 5>), dim3(g2), dim3(256), 0, strm(stream), (const uint16_t*)dy, N, H,
                         W, pad_top, pad_left, weff, (uint16_t*)dx, th, tw);
    else
      hipLaunchKernelGGL((k_stem_dgrad_mfma<3, 3>), dim3(g2), dim3(256), 0, strm(stream), (const uint16_t*)dy, N, H,
                         W, pad_top, pad_left, weff, (uint16_t*)dx, th, tw);
  } else if (dy_dtype == ACFE_DTYPE_BF16 && dx_dtype == ACFE_DTYPE_BF16) SD(uint16_t, uint16_t);
  else if (dy_dtype == ACFE_DTYPE_BF16) SD(uint16_t, float);
  else if (dx_dtype == ACFE_DTYPE_BF16) SD(float, uint16_t);
  else SD(float, float);
#undef SD
  return launch_rc("acfe_stem_dgrad");
}

// Workgroups of k_stem_bwd_bn: one resident round (3 per CU: 168 VGPRs, 46 KB
// of LDS) each walking its share of the tiles, instead of acfe_stem_blocks'
// 2048 in 2.7 rounds.  <= acfe_stem_blocks, which sizes the workspaces.
static int stem_bwd_grid(int N, int H, int W) {
  static const int cap = getenv("ACFE_STEM_BWD_GRID") ? atoi(getenv("ACFE_STEM_BWD_GRID")) : 768;
  const int nb = acfe_stem_blocks(N, H, W);
  return cap > 0 && cap < nb ? cap : nb;
}

// workspace: double[acfe_stem_blocks(N,H,W) * 16 * R * S]
ACFE_API int acfe_stem_wgrad(const void* x, int x_dtype, const void* dy, int dy_dtype, int N, int H, int W,
                             int R, int S, int pad_top, int pad_left, int rep, float* dw, float beta,
                             double* workspace, void* stream) {
  if (!x || !dy || !dw || !workspace || N <= 0 || R != S || (R != 5 && R != 3) || rep <= 0) return ACFE_E_INVAL;
  const int th = (H + STEM_TH - 1) / STEM_TH, tw = (W + STEM_TW - 1) / STEM_TW;
  const int grid = acfe_stem_blocks(N, H, W);
#define SW1(TI, TG, RR)                                                                                      \
  hipLaunchKernelGGL((k_stem_wgrad<TI, TG, RR, RR>), dim3(grid), dim3(256), 0, strm(stream), (const TI*)x,        \
                     (const TG*)dy, N, H, W, pad_top, pad_left, workspace, th, tw)
#define SW(TI, TG) if (R == 5) SW1(TI, TG, 5); else SW1(TI, TG, 3)
  if (x_dtype == ACFE_DTYPE_BF16 && dy_dtype == ACFE_DTYPE_BF16) {
    if (R == 5)
      hipLaunchKernelGGL((k_stem_wgrad_mfma<5, 5>), dim3(grid), dim3(256), 0, strm(stream), (const uint16_t*)x,
                         (const uint16_t*)dy, N, H, W, pad_top, pad_left, workspace, th, tw);
    else
      hipLaunchKernelGGL((k_stem_wgrad_mfma<3, 3>), dim3(grid), dim3(256), 0, strm(stream), (const uint16_t*)x,
                         (const uint16_t*)dy, N, H, W, pad_top, pad_left, workspace, th, tw);
  } else if (x_dtype == ACFE_DTYPE_BF16 && dy_dtype == ACFE_DTYPE_BF16) SW(uint16_t, uint16_t);
  else if (x_dtype == ACFE_DTYPE_BF16) SW(uint16_t, float);
  else if (dy_dtype == ACFE_DTYPE_BF16) SW(float, uint16_t);
  else SW(float, float);
#undef SW
  int rc = launch_rc("acfe_stem_wgrad");
  if (rc) return rc;
  const int n = STEM_K * R * S;
  if (rep > 256) return ACFE_E_INVAL;
  hipLaunchKernelGGL(k_stem_wgrad_reduce, dim3(n), dim3(256), 0, strm(stream), workspace, grid, n, rep, beta, dw);
  return launch_rc("acfe_stem_wgrad(reduce)");
}

// The stem backward with the BN backward apply folded in (k_stem_bwd_bn): g =
// the BN output gradient (bf16 [N][H][W][16], e.g. acfe_maxpool2d_bwd_argmax_bn's
// dX), xb = the BN input (= the stem output), coef = acfe_bn_bwd_finalize_ex's
// [3][16] coefficients.  dxin: the stem input gradient (bf16 [N][H][W]); dw: [16][R][S][rep] fp32 (beta as acfe_stem_wgrad); bias_part:
// double[acfe_stem_blocks(N,H,W)][2][16] channel sums of dX_bn (for
// acfe_channel_sum_finalize); workspace: double[acfe_stem_blocks(N,H,W) * 16 * R * S].
ACFE_API int acfe_stem_bwd_bn(const void* g, const void* xb, const void* xin, int N, int H, int W, int R, int S,
                              int pad_top, int pad_left, const float* weff, const float* scale, const float* shift,
                              const float* coef, int relu, void* dxin, int rep, float* dw, float beta,
                              double* bias_part, double* workspace, void* stream) {
  if (!g || !xb || !xin || !weff || !scale || !shift || !coef || !dw || !bias_part || !workspace || N <= 0 ||
      H <= 0 || W <= 0 || R != S || (R != 5 && R != 3) || rep <= 0 || rep > 256 || ((uintptr_t)g & 15) ||
      ((uintptr_t)xb & 15))
    return ACFE_E_INVAL;
  const int th = (H + STEM_TH - 1) / STEM_TH, tw = (W + STEM_TW - 1) / STEM_TW;
  const int nb = acfe_stem_blocks(N, H, W), grid = stem_bwd_grid(N, H, W);
  if (grid < nb) {  // bias slab rows past the grid: zero
    const hipError_t e =
        hipMemsetAsync(bias_part + (size_t)grid * 2 * STEM_K, 0, sizeof(double) * 2 * STEM_K * (nb - grid), strm(stream));
    if (e != hipSuccess) return hip_rc(e, "acfe_stem_bwd_bn");
  }
  uint16_t* dxo = (uint16_t*)dxin;
  if (!dxo) return ACFE_E_INVAL;
#define SB(RR)                                                                                                \
  hipLaunchKernelGGL((k_stem_bwd_bn<RR, RR>), dim3(grid), dim3(256), 0, strm(stream), (const uint16_t*)g,        \
                     (const uint16_t*)xb, (const uint16_t*)xin, N, H, W, pad_top, pad_left, weff, scale, shift, coef, \
                     relu, dxo, workspace, bias_part, th, tw)
  if (R == 5) SB(5); else SB(3);
#undef SB
  int rc = launch_rc("acfe_stem_bwd_bn");
  if (rc) return rc;
  const int n = STEM_K * R * S;
  hipLaunchKernelGGL(k_stem_wgrad_reduce, dim3(n), dim3(256), 0, strm(stream), workspace, grid, n, rep, beta, dw);
  return launch_rc("acfe_stem_bwd_bn(reduce)");
}
