// Definitions shared by the convolution translation units (conv.hip,
// pool1w.hip): vector types, the launch geometry, the XCD-aware tile walk and
// the LDS-DMA / wait helpers.
#pragma once
#include "common.h"

#include <type_traits>

namespace acfe {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
// Native 16-byte vector for register staging (HIP's uint4 struct-with-union
// defeats SROA: arrays of it were demoted to scratch).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t T16;
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 b2v __attribute__((ext_vector_type(2)));
// two floats -> one word of two bf16 (lo in bits 0-15), f2bf's RNE rounding
// in one v_cvt_pk_bf16_f32
__device__ __forceinline__ unsigned pk_bf2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f2v){lo, hi}, b2v));
}

struct ConvGeom {
  int N, H, W, C;    // input
  int K, P, Q;       // output
  int R, S, st, pt, pl;
  int Kd, Kdp, Kp;   // R*S*C, padded to BK, K padded to BN
  int ldy;           // output row stride (elements)
  long long M;       // N*P*Q
  Drop drop;         // optional Dropout of the output (flat index m*K + k), fused in the epilogue
  int dbg;           // diagnostics (ACFE_CONV_DBG=8: loop-segment cycle stamps), 0 in production
  const uint16_t* res;  // k_conv3x3_rows PM 3: residual added in the epilogue (same layout as Y)
  int res_relu;         // PM 3: ReLU after the residual add
  int idx32;            // M * K < 2^32: output element (dropout) indices fit 32 bits
  // k_conv3x3_rows PRO: BatchNormalization (+ReLU) of the input applied while
  // staging it, x' = (ReLU)(x * pro_sc[c] + pro_sh[c]) (acfe_bn_apply's
  // arithmetic); x' is also stored to pro_out (nullable) for the backward
  const float* pro_sc;
  const float* pro_sh;
  int pro_relu;
  uint16_t* pro_out;
  // k_conv3x3_rows PM 5 (acfe_conv2d_dgrad_bn): the BatchNormalization whose
  // output is this dgrad's dX -- its input x (g.res, Y's layout), affine
  // scale / shift (ReLU mask x * bn_sc + bn_sh > 0 when bn_relu) and batch
  // mean / invstd -- so the epilogue forms acfe_bn_bwd_reduce's sums
  const float* bn_sc;
  const float* bn_sh;
  const float* bn_mu;
  const float* bn_is;
  int bn_relu;
  // k_wgrad3x3_halo BWD (acfe_conv2d_wgrad_bnbwd): the wgrad's dY is the
  // backward of a BatchNormalization (+ReLU) -> Dropout (g.drop) whose output
  // gradient is the kernel's dY argument and whose input is fb_x (dY's layout),
  // formed while staging as acfe_bn_bwd_apply_ex forms it: fb_sc / fb_sh [K]
  // (ReLU mask), fb_coef [3][K] = a, b, c (dY = a g + b x + c); the values are
  // also stored to fb_out (for the dgrad) and summed per channel into fb_sums
  // (slab [gridDim][2][K], the conv bias gradient)
  const uint16_t* fb_x;
  const uint16_t* fb_add;  // nullable: the residual gradient added to a g + b x + c (ResidualLink)
  const float* fb_sc;
  const float* fb_sh;
  const float* fb_coef;
  int fb_relu;  // bit 0: the BN's ReLU mask on g; bit 1: x is a ReLU output, dY zeroed where x <= 0
  uint16_t* fb_out;
  double* fb_sums;
  // k_conv_fwd_p super-pixel store (the strided dgrad, acfe_conv2d_dgrad): s2d
  // = the stride st of the forward conv (0: plain NHWC store).  Output pixel
  // (n, u, v) x channel o = (a st + b) s2d_C + c is dX[n][st u + a - s2d_pt]
  // [st v + b - s2d_pl][c] of an s2d_H x s2d_W image, stored when inside it;
  // s2d_fill: the output channels are position (0, 0)'s only (o = c; the
  // caller zeroes the block's other st^2 - 1 pixels)
  int s2d, s2d_C, s2d_H, s2d_W, s2d_pt, s2d_pl, s2d_fill;
  int s2d_lc, s2d_amul;     // log2(s2d_C); block position a = (ab * s2d_amul) >> 5
  float s2d_rpq, s2d_rq;    // 1 / (P Q), 1 / Q of the block grid
  int cmaj;  // k_conv_fwd_g fp32: K-tiles chunk-major (ACFE_CONVG_CMAJ=0: tap-major, A/B)
  // Dropout keep bits [M][K / 8] (bit j of byte (m, c / 8) = element (m, 8 (c / 8) + j)
  // kept): written by the K = 64 dropout forward (k_conv3x3_r64 PM 4,
  // acfe_conv2d_fwd_*_keep), read by the BN-fold weight gradient
  // (acfe_conv2d_wgrad_bnbwd_keep) instead of regenerating the pair hashes
  uint8_t* keep_out;
  const uint8_t* keep_in;
};

// XCD-aware walk over the M tiles of a persistent grid.  Workgroups are
// dispatched round-robin over the 8 XCDs (linear id % 8), each with its own
// L2; neighbouring M tiles share im2col input rows (a 3x3 conv reads every
// input row from 3 output rows), so each XCD takes one contiguous eighth of the
// tiles and its G/8 resident workgroups sweep that range side by side.
// Falls back to the plain stride when the grid is not a multiple of 8.
struct TileWalk {
  int tm, end, step;
  __device__ TileWalk(int tiles_m) {
    const int G = gridDim.x;
    if (G >= 8 && (G & 7) == 0) {
      const int xcd = blockIdx.x & 7, chunk = (tiles_m + 7) >> 3;
      tm = xcd * chunk + (blockIdx.x >> 3);
      end = min((xcd + 1) * chunk, tiles_m);
      step = G >> 3;
    } else {
      tm = blockIdx.x;
      end = tiles_m;
      step = G;
    }
  }
};

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16-B buffer_load ... lds: LDS byte address (wave-uniform) in M0, descriptor
// in SGPRs, per-lane voffset; an out-of-range voffset lands zeros in LDS.
typedef int i4 __attribute__((ext_vector_type(4)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void bldsx4(unsigned voff, i4 desc, unsigned m0v) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(desc),
               "s"(m0v)
               : "memory", "m0");
}
// the same with a wave-uniform byte offset in soffset
__device__ __forceinline__ void bldsx4s(unsigned voff, i4 desc, unsigned soff, unsigned m0v) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(desc),
               "s"(soff), "s"(m0v)
               : "memory", "m0");
}
#pragma clang diagnostic pop

// 2x2 max-pool backward on the fly: 8 bf16 of the pooled gradient and their 8
// argmax bytes -> the values that land on tap `pos` ((row & 1) * 2 + (col & 1)) of
// the window, zeros elsewhere (acfe_maxpool2d_bwd_argmax's scatter, gathered).
// Byte-parallel: the argmax bytes are window taps 0..3, so byte ^ pos is zero
// exactly where it matches and (t | t >> 1) & 1 per byte is its "differs" bit;
// 255 * (equal bit) is the byte mask, and v_perm doubles each byte into the
// channel's 16-bit mask (7 VALU per 4 channels instead of 10-12 compares and
// selects).
__device__ __forceinline__ u32x4 unpool_mask(uint2 a, unsigned pos) {
  const unsigned rep = __builtin_amdgcn_perm(0u, pos, 0u);  // pos in every byte (no v_mul_lo_u32)
  u32x4 m;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const unsigned t = (h ? a.y : a.x) ^ rep;
    const unsigned eq = ~(t | (t >> 1)) & 0x01010101u;
    unsigned e8 = eq << 8;
    asm volatile("" : "+v"(e8));  // (kept a shift and a subtract, not a quarter-rate multiply by 255)
    const unsigned e = e8 - eq;   // 0xff per matching byte
    m[2 * h] = __builtin_amdgcn_perm(0u, e, 0x01010000u);
    m[2 * h + 1] = __builtin_amdgcn_perm(0u, e, 0x03030202u);
  }
  return m;
}

// One step of a 16-lane butterfly reduce-scatter: lanes whose `BIT` is set keep
// the upper half of v[0..CNT), the others the lower half, each adding the
// partner's copy of the half it keeps (partner = DPP pattern CTRL).
template <int CNT, int BIT, int CTRL, int NV>
__device__ __forceinline__ void butterfly_step(float (&v)[NV], int lane) {
  const bool up = (lane & BIT) != 0;
#pragma unroll
  for (int k = 0; k < CNT / 2; ++k) {
    const float send = up ? v[k] : v[k + CNT / 2];
    const float keep = up ? v[k + CNT / 2] : v[k];
    const float got = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), CTRL, 0xF, 0xF, false));
    v[k] = keep + got;
  }
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// acfe_conv2d_fwd_pool at K = C = 128 on the one-wave-per-SIMD kernel
// (pool1w.hip); returns ACFE_E_INVAL when the shape is not its case
int launch_pool1w(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
                  int srows, uint8_t* amax, hipStream_t s, const char* what);
// 3x3 stride-1 forward / dgrad at K = C = 128 (plain, + dropout, + BN sums) on the same kernel (PM 0)
// (pm 0: plain / dropout / BN sums; pm 3: + the residual g.res (+ReLU) of acfe_conv2d_fwd_add)
int launch_plain1w(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
                   int srows, hipStream_t s, const char* what, int pm);
// the K = 64 row-halo convolutions with the epilogue between the next tile's
// MFMA groups (rows64.hip): pm 0 plain / BN sums, 4 + dropout, 3 + residual,
// 5 the dgrad with the BN backward reduce; ACFE_E_INVAL when not its case
int launch_r64(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
               int srows, hipStream_t s, const char* what, int pm);
bool r64_enabled();
// acfe_conv2d_dgrad_bn at K = C = 128 on the same kernel (PM 5: dX + the BN backward reduce sums)
int launch_dgradbn1w(const ConvGeom& g, const void* dy, const void* wflip, void* dx, double* part, int srows,
                     hipStream_t s, const char* what);
// acfe_conv2d_dgrad_unpool at K = C = 128 on the same kernel (PM 2)
int launch_unpool1w(const ConvGeom& g, const void* dyp, const void* wflip, void* dx, uint8_t* amax, hipStream_t s,
                    const char* what);

}  // namespace acfe
