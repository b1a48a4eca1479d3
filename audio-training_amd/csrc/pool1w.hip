// k_conv3x3_1w: the 3x3 stride-1 convolutions at K = C = 128 -- the two
// dominant ones of the T1 step (the pooled forward of acfe_conv2d_fwd_pool,
// the unpooling dgrad of acfe_conv2d_dgrad_unpool) and the plain / dropout /
// residual-add forwards and stride-1 dgrads (wr_resnet's 128-channel stages)
// -- with one wave per SIMD (built with -fno-slp-vectorize: packed f32 VALU
// beside MFMAs costs more issue time than the two scalar ops).
#include "conv_common.h"

using namespace acfe;

// ------------------------------------------------------------------ 3x3 conv, one wave per SIMD
// k_conv3x3_1w<PM, NCH, DROP, ST>, K = 128 output channels, C = 64 NCH input
// channels (NCH even).  PM 1: acfe_conv2d_fwd_pool (stage-1 block-0 branch21
// 128 -> 128 @ 128 x 256 -> MaxPool2D(2) -> Dropout -> BN,
// resnet/wr_resnet_bird.py:136-147); PM 2: its dgrad from the pooled gradient
// and the argmax bytes (the 2x2 max-pool backward expanded while staging);
// PM 0: acfe_conv2d_fwd / fwd_dropout / stride-1 dgrad (bias, optional pair-
// hash Dropout, optional BN sums ST); PM 3: acfe_conv2d_fwd_add (+ the
// residual, +ReLU, BN sums of the sum; resnet/wr_resnet.py:46-90).
//
// Same tile, LDS images and weight pieces as k_conv3x3_rows<128, 4, PM, true>
// (4 rows x 64 px x 128 channels, chunk-resident halo rows: a step is one
// 64-channel chunk x one filter row), but four waves, one per SIMD, each
// owning a quarter of the tile's pixels and ALL 128 channels: 8 weight
// fragments per 4 pixel fragments (0.375 instead of 0.5 ds_read_b128 per
// MFMA) and 128 accumulators per lane in the accumulator file.
//  * The epilogue of tile i - 1 runs beside the MFMAs of tile i: each
//    accumulator's last MFMA of a tile is followed by its packing (biased,
//    rounded to bf16: the value a separate conv would have stored) into 64
//    packed registers, the tile's first MFMA of it takes C = 0, and the
//    epilogue of the packed values (PM 1: max / first-maximum argmax / dropout
//    / BN sums / stores; PM 2: 16-B channel-run stores) runs in units between
//    the MFMA groups of steps 0..3.  The 8-wave kernel stopped its MFMAs for
//    the whole epilogue (16 % of every step).
//  * Every step is one straight block (no branches: the last tile's loads are
//    clamped, out-of-image and phantom stores are buffer stores at an
//    out-of-range offset), its MFMA groups fenced by sched_barrier with the
//    next group's fragments read during the current one, the next step's
//    weight pieces (LDS-DMA) in groups 0..2 and the next chunk's halo loads
//    after them, so the step's closing vmcnt wait leaves the halo loads and
//    epilogue stores in flight.
//  * MFMA operand order: PM 1 pixels x weights (a lane's four accumulators
//    are one 2x2 window of one channel), PM 0 / 2 / 3 weights x pixels (a
//    lane holds 16 consecutive channels of a pixel per channel half: 16-B
//    stores; the BN sums are reduced over the 16 pixel lanes by a DPP
//    butterfly once per half and tile).
#ifdef ACFE_P1W_STAMPS
// diagnostic build (make stamps): per-wave s_memtime totals of the step
// segments, read back by acfe_debug_pool1w_stamps (tools/pool1w_stamps.py)
__device__ unsigned long long g_p1w_stamps[4096 * 8];
#endif
// SEGW: tile width -- 64 (4 rows x 64 pixels), or 16 (16 rows x 16 pixels,
// PM 0 / 3) for the Q % 64 pixels left of each row, launched separately from
// column wofs (wr_resnet's 257-wide stage 2 ran a whole 64-pixel tile per 4
// rows for its last pixel); srow0: the first statistics slab row it writes.
template <int PM, int NCH, bool DROP, bool ST = true, bool PRO = false, int SEGW = 64>
__global__ void __launch_bounds__(256, 1)
k_conv3x3_1w(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
             const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats, int tiles_h,
             int tiles_w, int ntiles, int srows, uint8_t* __restrict__ amax, int wofs = 0, int srow0 = 0) {
  static_assert(NCH % 2 == 0, "even step count per tile: weight buffer parity is static");
  // PM 5: the stride-1 dgrad whose dX is a BatchNormalization's output
  // gradient, with acfe_bn_bwd_reduce's sums of the stored dX in the epilogue
  // (g.res = the BN input, g.bn_*; wr_resnet's stage-2 conv dgrads, rows64.hip
  // PM 5's K = 128 counterpart)
  static_assert(PM == 0 || PM == 1 || ((PM == 2 || PM == 3 || PM == 5) && !DROP), "modes");
  // PRO: the BatchNormalization (+ReLU) of the input applied while staging it
  // (acfe_conv2d_fwd_bn / fwd_add_bn at K = C = 128: wr_resnet's stage-2
  // bn2a / bn2b -> conv2a / conv2b), x' = (ReLU)(x * pro_sc + pro_sh) rounded to
  // bf16 (acfe_bn_apply's values); the tile's own pixels of x' also go to
  // pro_out for the weight gradient
  static_assert(!PRO || PM == 0 || PM == 3, "prologue: plain / residual forward");
  static_assert(SEGW == 64 || (SEGW == 16 && (PM == 0 || PM == 3 || PM == 5)), "16-pixel tiles: the dense modes");
  constexpr bool CPERM = PM != 1;     // weights x pixels operand order (PM 0 / 2 / 3)
  constexpr bool DENSE = PM == 0 || PM == 3 || PM == 5;  // full-resolution output with bias (PM 3: + residual)
  constexpr bool RLD = PM == 3 || PM == 5;                // per-unit words of g.res (residual / BN input)
  constexpr int KB = 128, TR = 256 / SEGW, FM = 4, FN = 4, NH = 2, NF = NH * FN, HWX = SEGW + 2, XRB = 160;
  constexpr int NT = 256, NS = 3 * NCH;                          // threads, steps per tile
  constexpr int XROWS = TR + 2, XBYTES = XROWS * HWX * XRB;      // 63 360 B
  constexpr int WBYTES = 3 * KB * 128, WBASE = XBYTES;           // 2 x 49 152 B
  constexpr int XG = XROWS * HWX * 8, XPT = (XG + NT - 1) / NT;  // 16-B input granules
  constexpr int WPW = 3 * KB * 8 / 64 / (NT / 64);               // 12 weight pieces per wave per step
  constexpr int WPG = 4;                                         // pieces per MFMA group (groups 0..2)
  constexpr bool BTAB = PM == 0 || PM == 3;                          // (PM 5: the dgrad has no bias)
  constexpr int SMEMP = XBYTES + 2 * WBYTES + (BTAB ? KB * 4 : 0);   // (PM 0 / 3: bias table)
  constexpr int SMEMB = SMEMP + (PRO ? 2 * 64 * NCH * 4 : 0);         // (PRO: scale / shift of the C channels)
  constexpr int SMEM = SMEMB + (PM == 5 ? 4 * KB * 4 : 0);            // (PM 5: [scale | shift | mean | invstd][KB])
  static_assert(SMEM <= 163840, "LDS");
  static_assert(XPT * NT - XG <= 2 * XROWS * HWX, "spare granules fit the pixel pads");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 b2v __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4;
  const int wp = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tpi = tiles_h * tiles_w;
  const TileWalk walk(ntiles);
  const int ntl = walk.tm < walk.end ? (walk.end - walk.tm + walk.step - 1) / walk.step : 0;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;
#ifdef ACFE_P1W_STAMPS
  unsigned long long stv[6] = {0, 0, 0, 0, 0, 0}, stl = __builtin_amdgcn_s_memtime();
  auto stamp = [&](int i) __attribute__((always_inline)) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    stv[i] += t - stl;
    stl = t;
  };
#else
  auto stamp = [](int) __attribute__((always_inline)) {};
#endif
  auto tile_of = [&](int tm, int& n, int& hb, int& wb) __attribute__((always_inline)) {
    n = tm / tpi;
    const int rem = tm - n * tpi;
    hb = rem / tiles_w;
    wb = rem - hb * tiles_w;
  };

  // bias of the lane's channels h * 64 + 4 l16 + [0, 4) (PM 1); PM 0: a 128-entry
  // LDS table (a lane's accumulators there are 4 channels each)
  f4 bch[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h)
    bch[h] = (PM == 1 && bias) ? *reinterpret_cast<const f4*>(bias + h * 64 + 4 * l16) : f4{0.f, 0.f, 0.f, 0.f};
  float* btab = reinterpret_cast<float*>(smem + XBYTES + 2 * WBYTES);
  float* pss = reinterpret_cast<float*>(smem + SMEMP);  // PRO: scale[C], shift[C]
  float* bnt = reinterpret_cast<float*>(smem + SMEMB);  // PM 5: the BN's scale, shift, mean, invstd
  if constexpr (PM == 5)
    for (int i = tid; i < KB; i += NT)
      bnt[i] = g.bn_sc[i], bnt[KB + i] = g.bn_sh[i], bnt[2 * KB + i] = g.bn_mu[i], bnt[3 * KB + i] = g.bn_is[i];
  if constexpr (PRO)
    for (int i = tid; i < 64 * NCH; i += NT) pss[i] = g.pro_sc[i], pss[64 * NCH + i] = g.pro_sh[i];
  if constexpr (BTAB)
    if (tid < KB) btab[tid] = bias ? bias[tid] : 0.f;

  // ---- weight pieces (LDS-DMA, 1 KB each, 48 per step).  The lane part of a
  // piece's source offset is one of two VGPRs per wave, the rest a uniform
  // soffset formed per piece; LDS destination in M0.
  //  PM 1 (k_conv3x3_rows' SWP layout): LDS rows [kk][s][phys(k)] of 64 B,
  //   phys(k) = k ^ ((k >> 2) & 3), granule slot ^ ((l16 >> 2) & 2) on the
  //   reading side; piece (kk, s, b) = 16 rows of row block 2 wp + b, whose
  //   swizzle term (kb >> 1) & 1 = wp & 1.
  //  PM 2 (CPERM layout): LDS rows [s][k] of 128 B, slot sigma holds granule
  //   sigma ^ sw(k), sw(k) = ((k >> 4) & 3) << 1 | ((k >> 1) & 1); piece (s, b)
  //   = 8 rows 32 wp + 8 b .., whose (k >> 4) & 3 = (2 wp + (b >> 1)) & 3.
  unsigned vw[2];
  int sob;
  if constexpr (!CPERM) {
    const int l4 = lane >> 2;
    vw[0] = vw[1] = (unsigned)((l4 ^ ((l4 >> 2) & 3)) * g.Kdp * 2) +
                    ((((unsigned)lane & 3u) ^ ((wp & 1) ? 2u : 0u)) << 4);
    sob = __builtin_amdgcn_readfirstlane(2 * wp * 16 * g.Kdp * 2);  // row block 2 wp
  } else {
    const int l8 = lane >> 3;
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const unsigned sw = ((unsigned)((2 * wp + bb) & 3) << 1) | ((unsigned)(lane >> 4) & 1u);
      vw[bb] = (unsigned)(l8 * g.Kdp * 2) + ((((unsigned)lane & 7u) ^ sw) << 4);
    }
    sob = __builtin_amdgcn_readfirstlane(32 * wp * g.Kdp * 2);  // row 32 wp
  }
  unsigned wlo = 0, whi = 0, wlb = 0;
  auto wprep = [&](int st, int wb) __attribute__((always_inline)) {
    const int cc = st / 3, r = st - cc * 3;
    const unsigned long long base = (unsigned long long)(uintptr_t)Wp + ((unsigned)(r * 3 * g.C + cc * 64) * 2u);
    wlo = (unsigned)base;
    whi = (unsigned)(base >> 32);
    wlb = lds0 + WBASE + wb * WBYTES;
  };
  auto wpiece = [&](int j) __attribute__((always_inline)) {
    const i4 dw = {__builtin_amdgcn_readfirstlane((int)wlo), __builtin_amdgcn_readfirstlane((int)whi),
                   (int)0x80000000u, 0x00020000};
    int sb_ = sob;
    asm volatile("" : "+s"(sb_));  // formed here, not hoisted into a dozen live registers
    unsigned so, lb, vo;
    if constexpr (!CPERM) {  // j = 2 (kk * 3 + s) + b
      const int ks = j >> 1, b = j & 1, kk = ks / 3, s_ = ks - kk * 3;
      so = (unsigned)(sb_ + s_ * g.C * 2 + kk * 64 + b * 16 * g.Kdp * 2);
      lb = wlb + (ks * 128 + 2 * wp * 16 + b * 16) * 64;
      vo = vw[0];
    } else {  // j = 4 s + b: rows 32 wp + 8 b .. of tap s
      const int s_ = j >> 2, b = j & 3;
      so = (unsigned)(sb_ + s_ * g.C * 2 + b * 8 * g.Kdp * 2);
      lb = wlb + (s_ * 128 + 32 * wp + 8 * b) * 128;
      vo = vw[b >> 1];
    }
    bldsx4s(vo, dw, so, (unsigned)__builtin_amdgcn_readfirstlane((int)lb));
  };

  // ---- input halo rows of a 64-channel chunk, register-staged: granule i of
  // this thread = halo pixel (tid >> 3) + 32 i (row xrow_i, pixel xpix_i: tile
  // independent), channel slot gr = tid & 7
  const int gr = tid & 7, CB = g.C * 2;
  u32x4 rx[XPT];
  uint2 ra[PM == 2 ? XPT : 1];  // PM 2: the granules' argmax bytes
  __amdgpu_buffer_rsrc_t xrs, ars;
  // PM 1: rel[i] = byte offset of granule i from the tile's halo origin
  // (computed once); per tile the origin's offset (may be negative) and a
  // mask of the granules whose column lies inside the image (rows outside the
  // image fall outside the image's buffer range, which loads zeros).
  // PM 2: per tile, gel[i] = element offset of granule i's pooled-gradient
  // granule in the image, a validity mask and the 2-bit window tap of each
  // granule (unpool mask applied at the LDS store).
  int rel[XPT];
  int tbase = 0;
  unsigned cmask = 0, pos0 = 0, pos1 = 0;
  // PRO: granules inside the image (zero after the transform otherwise: the
  // conv pads x', not x) and the tile's own pixels (stored to pro_out)
  unsigned vmask = 0, omask = 0;
  __amdgpu_buffer_rsrc_t prs;
  if constexpr (PM != 2) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = tid + NT * i;
      const int xrow = idx / (HWX * 8), xpix = (idx - xrow * (HWX * 8)) >> 3;
      rel[i] = (xrow * g.W + xpix) * CB + gr * 16;
    }
  }
  auto stage_tile = [&](int tl) __attribute__((always_inline)) {
    const int tm = walk.tm + tl * walk.step;
    int n, hb, wb;
    tile_of(tm, n, hb, wb);
    const int sh0 = hb * TR - g.pt, sw0 = wofs + wb * SEGW - g.pl;
    int t0 = tid;
    asm volatile("" : "+v"(t0));  // (per tile, not hoisted)
    cmask = 0;
    if constexpr (PM != 2) {
      tbase = (sh0 * g.W + sw0) * CB;
      xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (long long)n * g.H * g.W * g.C), (short)0,
                                              g.H * g.W * CB, 0x00020000);
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const unsigned idx = (unsigned)t0 + NT * i;
        const unsigned xpix = (idx % (HWX * 8)) >> 3;
        const bool ok = idx < (unsigned)XG && (unsigned)(sw0 + (int)xpix) < (unsigned)g.W;
        cmask |= (ok ? 1u : 0u) << i;
      }
      if constexpr (PRO) {
        prs = __builtin_amdgcn_make_buffer_rsrc((void*)(g.pro_out + (long long)n * g.H * g.W * g.C), (short)0,
                                                g.H * g.W * CB, 0x00020000);
        vmask = omask = 0;
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
          const unsigned idx = (unsigned)t0 + NT * i;
          const int xrow = (int)(idx / (HWX * 8)), xpix = (int)((idx % (HWX * 8)) >> 3);
          const bool ok = ((cmask >> i) & 1u) && (unsigned)(sh0 + xrow) < (unsigned)g.H;
          const bool own = ok && xrow >= 1 && xrow <= TR && xpix >= 1 && xpix <= SEGW;
          vmask |= (ok ? 1u : 0u) << i;
          omask |= (own ? 1u : 0u) << i;
        }
      }
    } else {
      // X = pooled gradient [N][H/2][W/2][C], amax its argmax bytes
      const long long img = (long long)n * (g.H >> 1) * (g.W >> 1) * g.C;
      const int nb = (g.H >> 1) * (g.W >> 1) * g.C;
      xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + img), (short)0, nb * 2, 0x00020000);
      ars = __builtin_amdgcn_make_buffer_rsrc((void*)(amax + img), (short)0, nb, 0x00020000);
      pos0 = pos1 = 0;
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int idx = t0 + NT * i;
        const int xrow = idx / (HWX * 8), xpix = (idx - xrow * (HWX * 8)) >> 3;
        const int hin = sh0 + xrow, win = sw0 + xpix;
        const bool ok = idx < XG && (unsigned)hin < (unsigned)g.H && (unsigned)win < (unsigned)g.W;
        rel[i] = ((hin >> 1) * (g.W >> 1) + (win >> 1)) * g.C + gr * 8;
        cmask |= (ok ? 1u : 0u) << i;
        const unsigned p = ((unsigned)(hin & 1) << 1) | ((unsigned)win & 1u);
        if (i < 8) pos0 |= p << (4 * i);
        else pos1 |= p << (4 * (i - 8));
      }
    }
  };
  auto gload = [&](int cc, int i0, int i1) __attribute__((always_inline)) {
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const bool ok = (cmask >> i) & 1u;
      if constexpr (PM != 2) {
        rx[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, ok ? (unsigned)(tbase + cc * 128 + rel[i]) : 0x80000000u,
                                                      0, 0);
      } else {
        const unsigned e = (unsigned)(rel[i] + cc * 64);
        rx[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, ok ? e * 2u : 0x80000000u, 0, 0);
        const auto a8 = __builtin_amdgcn_raw_buffer_load_b64(ars, ok ? e : 0x80000000u, 0, 0);
        ra[i] = uint2{a8[0], a8[1]};
      }
    }
  };
  // LDS slot of granule i; the last round's threads past the image write
  // their (zero) granule into the never-read 32-B pads of pixels 0..79, so
  // the restage is one branch-free block
  auto sslot = [&](int i) __attribute__((always_inline)) {
    const int idx = tid + NT * i, e = idx - XG;
    return idx < XG ? (idx >> 3) * XRB + gr * 16 : (e >> 1) * XRB + 128 + (e & 1) * 16;
  };
  auto sstore = [&](int scc) __attribute__((always_inline)) {
    f4 sc0, sc1, sh0_, sh1_;
    bool relu = false;
    if constexpr (PRO) {  // this thread's 8 channels scc * 64 + gr * 8 ..
      const f4* ps = reinterpret_cast<const f4*>(pss + scc * 64 + gr * 8);
      sc0 = ps[0], sc1 = ps[1], sh0_ = ps[16 * NCH], sh1_ = ps[16 * NCH + 1];
      relu = g.pro_relu != 0;
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      u32x4 v = rx[i];
      if constexpr (PM == 2) v &= unpool_mask(ra[i], ((i < 8 ? pos0 >> (4 * i) : pos1 >> (4 * (i - 8)))) & 3u);
      if constexpr (PRO) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const float s0 = d < 2 ? sc0[2 * d] : sc1[2 * d - 4], s1 = d < 2 ? sc0[2 * d + 1] : sc1[2 * d - 3];
          const float h0 = d < 2 ? sh0_[2 * d] : sh1_[2 * d - 4], h1 = d < 2 ? sh0_[2 * d + 1] : sh1_[2 * d - 3];
          float lo = __builtin_fmaf(__uint_as_float(v[d] << 16), s0, h0);
          float hi = __builtin_fmaf(__uint_as_float(v[d] & 0xffff0000u), s1, h1);
          if (relu) lo = fmaxf(lo, 0.f), hi = fmaxf(hi, 0.f);
          const b2v pk = __builtin_convertvector((f2v){lo, hi}, b2v);
          v[d] = __builtin_bit_cast(unsigned, pk);
        }
        v = ((vmask >> i) & 1u) ? v : u32x4{0u, 0u, 0u, 0u};
        __builtin_amdgcn_raw_buffer_store_b128(v, prs,
                                               ((omask >> i) & 1u) ? (unsigned)(tbase + scc * 128 + rel[i]) : 0x80000000u,
                                               0, 0);
      }
      *reinterpret_cast<u32x4*>(smem + sslot(i)) = v;
    }
  };

  // ---- fragment offsets
  int xoff[FM];
  int wrb[2][NH][FN];  // [kk] (PM 1: both equal)
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    if constexpr (!CPERM) {
      // A rows 4 q' + j = window q' of fragment fm (row pair fm / 2, pooled
      // column wp * 8 + (fm & 1) * 4 + (q' ^ (q' >> 1))), pixel j
      const int qq = l16 >> 2, j = l16 & 3;
      const int a = wp * 8 + (fm & 1) * 4 + (qq ^ (qq >> 1));
      xoff[fm] = (((fm >> 1) * 2 + (j >> 1)) * HWX + 2 * a + (j & 1)) * XRB + q * 16;
    } else {
      // B columns = tile pixels wp * 64 + fm * 16 + l16 (SEGW 64: tile row wp)
      const int p0 = wp * 64 + fm * 16;
      xoff[fm] = ((p0 / SEGW) * HWX + p0 % SEGW + l16) * XRB + q * 16;
    }
  }
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      if constexpr (!CPERM) {
        const int k = h * 64 + FN * l16 + fn;
        wrb[0][h][fn] = wrb[1][h][fn] = (k ^ ((k >> 2) & 3)) * 64 + ((q ^ ((l16 >> 2) & 2)) << 4);
      } else {
        // A row m = l16 = channel h * 64 + 16 (m >> 2) + 4 fn + (m & 3)
        const int k = h * 64 + 16 * (l16 >> 2) + 4 * fn + (l16 & 3);
        const int sw = (((k >> 4) & 3) << 1) | ((k >> 1) & 1);
        wrb[0][h][fn] = k * 128 + ((q ^ sw) << 4);
        wrb[1][h][fn] = k * 128 + (((q + 4) ^ sw) << 4);
      }
    }
  // weight fragment of group (s, kk) relative to the buffer base
  auto wfrag_off = [&](int s, int kk, int h, int fn) __attribute__((always_inline)) {
    return !CPERM ? (kk * 3 + s) * KB * 64 + wrb[0][h][fn] : s * KB * 128 + wrb[kk][h][fn];
  };

  f4 acc[FM][NF];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // the previous tile's conv outputs, biased and rounded to bf16, packed:
  // PM 1 pixels j = 0, 1 | 2, 3 of window q of fragment fm, channel n;
  // PM 2 channels 4 fn + 0, 1 | 2, 3 of its 16-channel run, pixel l16 of fm
  u32x2 prev[FM][NF];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) prev[i][j] = u32x2{0u, 0u};
  auto pack1 = [&](int fm, int n) __attribute__((always_inline)) {
    f4 b4;
    if constexpr (BTAB) {  // channels h * 64 + 16 q + 4 fn + j
      b4 = *reinterpret_cast<const f4*>(btab + (n / FN) * 64 + 16 * q + 4 * (n % FN));
    } else if constexpr (PM == 5) {
      b4 = f4{0.f, 0.f, 0.f, 0.f};
    } else {
      const float b = bch[n / FN][n % FN];
      b4 = f4{b, b, b, b};
    }
    const b2v lo = __builtin_convertvector((f2v){acc[fm][n][0] + b4[0], acc[fm][n][1] + b4[1]}, b2v);
    const b2v hi = __builtin_convertvector((f2v){acc[fm][n][2] + b4[2], acc[fm][n][3] + b4[3]}, b2v);
    prev[fm][n] = u32x2{__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi)};
  };

  // ---- PM 1 epilogue: part (h, fm2) = channel half h, fragment pair fm2
  // (pooled row fm2 / 2 of the tile), in units: unit (hf, pr) pools channels
  // 2 pr, 2 pr + 1 of fragment fm2 + hf (their dropout pair hash, max /
  // first-maximum argmax, BN sums) into eyv / eav; the store unit exchanges
  // fragment halves between lane pairs and writes 16 B pooled + 8 B argmax
  // per lane.  Pooled output and argmax bytes < 2^31 bytes (launcher).
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)Y, (short)0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)amax, (short)0, 0x7FFFFFFF, 0x00020000);
  const int P2 = g.P >> 1, Q2 = g.Q >> 1;
  const bool odd = (lane & 1) != 0;
  float sb[FN], sq[FN];  // BN sums of the half in progress
  double dstat[NH][2];
#pragma unroll
  for (int k = 0; k < FN; ++k) sb[k] = sq[k] = 0.f;
#pragma unroll
  for (int h = 0; h < NH; ++h) dstat[h][0] = dstat[h][1] = 0.0;
  unsigned eyv[2][2], eav[2];
  auto epi_unit = [&](int h, int fm2, int hf, int pr, int tm, bool live) __attribute__((always_inline)) {
    int n, hb, wb;
    tile_of(tm, n, hb, wb);
    const int cf = h * 64 + FN * l16;
    const int hp2 = hb * (TR / 2) + (fm2 >> 1);
    const int fm = fm2 + hf;
    const int wq = wb * (SEGW / 2) + wp * 8 + hf * 4 + (q ^ (q >> 1));
    const bool inb = live && hp2 < P2 && wq < Q2;
    unsigned keep = 3u;
    if constexpr (DROP) {
      const unsigned pp = ((unsigned)n * P2 + hp2) * Q2 + wq;
      const uint32_t hh = drop_pair_hash32(g.drop, pp * (unsigned)KB + cf + 2 * pr);
      keep = ((hh & 0xFFFFu) >= g.drop.thr ? 1u : 0u) | ((hh >> 16) >= g.drop.thr ? 2u : 0u);
    }
    float mv[2];
    unsigned avb = 0u;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int fn = 2 * pr + e;
      const u32x2 pv = prev[fm][h * FN + fn];
      const float a[4] = {__uint_as_float(pv[0] << 16), __uint_as_float(pv[0] & 0xffff0000u),
                          __uint_as_float(pv[1] << 16), __uint_as_float(pv[1] & 0xffff0000u)};
      float m = a[0];
      unsigned am = 0;
      if (a[1] > m) m = a[1], am = 1;
      if (a[2] > m) m = a[2], am = 2;
      if (a[3] > m) m = a[3], am = 3;
      if constexpr (DROP) m = ((keep >> e) & 1u) ? bf2f(f2bf(m * g.drop.scl)) : 0.f;
      mv[e] = m;
      avb |= am << (8 * fn);
      const float f = inb ? m : 0.f;
      sb[fn] += f;
      sq[fn] += f * f;
    }
    eav[hf] = pr == 0 ? avb : (eav[hf] | avb);
    eyv[hf][pr] = (__float_as_uint(mv[0]) >> 16) | (__float_as_uint(mv[1]) & 0xffff0000u);
  };
  auto epi_store = [&](int h, int fm2, int tm, bool live) __attribute__((always_inline)) {
    int n, hb, wb;
    tile_of(tm, n, hb, wb);
    const int hp2 = hb * (TR / 2) + (fm2 >> 1);
    // even lane: fragment fm2 (own | partner's channels), odd lane: fm2 + 1
    unsigned ys[2], yo[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      ys[pr] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(odd ? eyv[0][pr] : eyv[1][pr]), 0xB1, 0xF, 0xF, false);
      yo[pr] = odd ? eyv[1][pr] : eyv[0][pr];
    }
    const unsigned as = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(odd ? eav[0] : eav[1]), 0xB1, 0xF, 0xF, false);
    const unsigned ao = odd ? eav[1] : eav[0];
    const int wq = wb * (SEGW / 2) + wp * 8 + (odd ? 4 : 0) + (q ^ (q >> 1));
    const bool inb = live && hp2 < P2 && wq < Q2;
    const unsigned c0 = h * 64 + FN * (l16 & ~1);
    const unsigned pix = ((unsigned)n * P2 + hp2) * Q2 + wq;
    __builtin_amdgcn_raw_buffer_store_b128(odd ? u32x4{ys[0], ys[1], yo[0], yo[1]} : u32x4{yo[0], yo[1], ys[0], ys[1]},
                                           yr, inb ? (pix * (unsigned)g.ldy + c0) * 2u : 0x80000000u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(odd ? u32x2{as, ao} : u32x2{ao, as}, ar,
                                          inb ? pix * (unsigned)KB + c0 : 0x80000000u, 0, 0);
  };
  // statistics of half h of a finished tile: sums over the four window groups,
  // lane group q keeps values 2 q + k of [sb[0..4), sq[0..4)]
  auto epi_stats = [&](int h) __attribute__((always_inline)) {
    // (lane-group butterflies by v_permlane16_swap / v_permlane32_swap: with
    // both operands x, the two results hold x of the partner rows, so their
    // sum is the sum over lanes l, l ^ 16 (then l ^ 32))
    auto bfly = [](float& v, auto swp) __attribute__((always_inline)) {
      const auto r = swp(__float_as_uint(v));
      v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    };
    auto s16 = [](unsigned x) { return __builtin_amdgcn_permlane16_swap(x, x, false, false); };
    auto s32 = [](unsigned x) { return __builtin_amdgcn_permlane32_swap(x, x, false, false); };
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      bfly(sb[fn], s16);
      bfly(sq[fn], s16);
      bfly(sb[fn], s32);
      bfly(sq[fn], s32);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float v = 0.f;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int idx = qq * 2 + k, fn = idx % FN;
        v = q == qq ? (idx < FN ? sb[fn] : sq[fn]) : v;
      }
      dstat[h][k] += (double)v;
    }
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) sb[fn] = sq[fn] = 0.f;
  };
  // ---- PM 2 epilogue: unit (fm, h) stores the 16 consecutive channels
  // h * 64 + 16 q .. of pixel (tile row wp, column fm * 16 + l16) as two 16-B
  // stores into the image's dX (per-image buffer, < 2^31 bytes: launcher)
  auto dx_unit = [&](int fm, int h, int tm, bool live) __attribute__((always_inline)) {
    int n, hb, wb;
    tile_of(tm, n, hb, wb);
    // tile pixels wp * 64 + fm * 16 + l16: SEGW 64 row wp, 16 row 4 wp + fm
    const int hh = hb * TR + (SEGW == 64 ? wp : 4 * wp + fm), ww = wofs + wb * SEGW + (SEGW == 64 ? fm * 16 : 0) + l16;
    const bool inb = live && hh < g.P && ww < g.Q;
    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Y + (long long)n * g.P * g.Q * g.ldy), (short)0, g.P * g.Q * g.ldy * 2, 0x00020000);
    const unsigned o = ((unsigned)(hh * g.Q + ww) * (unsigned)g.ldy + h * 64 + 16 * q) * 2u;
    const u32x2 p0 = prev[fm][h * FN + 0], p1 = prev[fm][h * FN + 1], p2 = prev[fm][h * FN + 2],
                p3 = prev[fm][h * FN + 3];
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{p0[0], p0[1], p1[0], p1[1]}, dr, inb ? o : 0x80000000u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{p2[0], p2[1], p3[0], p3[1]}, dr, inb ? o + 16u : 0x80000000u, 0, 0);
  };
  // ---- PM 0 epilogue: unit (fm, h) = the 16 consecutive channels
  // c0 = h * 64 + 16 q .. of pixel (tile row wp, column fm * 16 + l16):
  // dropout (one pair hash per channel pair, acfe_dropout's mask), the BN sums
  // of the stored values (ds[16] / dq[16] of the half in progress, reduced over
  // the 16 pixel lanes by a DPP butterfly after its last unit), two 16-B stores
  // into the image's output (per-image buffer, < 2^31 bytes: launcher)
  float ds[16], dq[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) ds[i] = dq[i] = 0.f;
  // PM 3: the residual words of the step's two units, loaded in its group 0
  u32x4 rres[2][2];
  auto res_load = [&](int u, int fm, int h, int tm, bool live) __attribute__((always_inline)) {
    int n, hb, wb;
    tile_of(tm, n, hb, wb);
    // tile pixels wp * 64 + fm * 16 + l16: SEGW 64 row wp, 16 row 4 wp + fm
    const int hh = hb * TR + (SEGW == 64 ? wp : 4 * wp + fm), ww = wofs + wb * SEGW + (SEGW == 64 ? fm * 16 : 0) + l16;
    const bool inb = live && hh < g.P && ww < g.Q;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(g.res + (long long)n * g.P * g.Q * g.ldy), (short)0, g.P * g.Q * g.ldy * 2, 0x00020000);
    const unsigned o = ((unsigned)(hh * g.Q + ww) * (unsigned)g.ldy + h * 64 + 16 * q) * 2u;
    rres[u][0] = __builtin_amdgcn_raw_buffer_load_b128(rr, inb ? o : 0x80000000u, 0, 0);
    rres[u][1] = __builtin_amdgcn_raw_buffer_load_b128(rr, inb ? o + 16u : 0x80000000u, 0, 0);
  };
  auto dense_unit = [&](int fm, int h, int tm, bool live, int u = 0) __attribute__((always_inline)) {
    int n, hb, wb;
    tile_of(tm, n, hb, wb);
    // tile pixels wp * 64 + fm * 16 + l16: SEGW 64 row wp, 16 row 4 wp + fm
    const int hh = hb * TR + (SEGW == 64 ? wp : 4 * wp + fm), ww = wofs + wb * SEGW + (SEGW == 64 ? fm * 16 : 0) + l16;
    const bool inb = live && hh < g.P && ww < g.Q;
    const int c0 = h * 64 + 16 * q;
    unsigned w8[8];
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) w8[2 * fn] = prev[fm][h * FN + fn][0], w8[2 * fn + 1] = prev[fm][h * FN + fn][1];
    if constexpr (PM == 3) {
      // z = (ReLU)(conv + residual), rounded to bf16 (ops.add's values)
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) {
        const unsigned rw = rres[u][pr >> 2][pr & 3];
        float lo = __uint_as_float(w8[pr] << 16) + __uint_as_float(rw << 16);
        float hi = __uint_as_float(w8[pr] & 0xffff0000u) + __uint_as_float(rw & 0xffff0000u);
        if (g.res_relu) lo = fmaxf(lo, 0.f), hi = fmaxf(hi, 0.f);
        const b2v pk = __builtin_convertvector((f2v){lo, hi}, b2v);
        w8[pr] = __builtin_bit_cast(unsigned, pk);
      }
    }
    if constexpr (PM == 5) {
      // acfe_bn_bwd_reduce's terms of the stored dX: gm = dX masked by the BN's
      // ReLU (x * scale + shift > 0), summed as gm and gm * (x - mean) * invstd
      // (the table's pair reads from a per-unit opaque base: not hoisted into
      // 64 live registers)
      const bool norelu = g.bn_relu == 0;
      unsigned bo = (unsigned)(c0 * 4);
      asm volatile("" : "+v"(bo));
      const unsigned char* tb = reinterpret_cast<const unsigned char*>(bnt) + bo;
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) {
        const unsigned xw = rres[u][pr >> 2][pr & 3];
        const f2v csc = *reinterpret_cast<const f2v*>(tb + 8 * pr), csh = *reinterpret_cast<const f2v*>(tb + KB * 4 + 8 * pr),
                  cmu = *reinterpret_cast<const f2v*>(tb + 2 * KB * 4 + 8 * pr),
                  cis = *reinterpret_cast<const f2v*>(tb + 3 * KB * 4 + 8 * pr);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int j = 2 * pr + e;
          const float xf = __uint_as_float(e ? (xw & 0xffff0000u) : (xw << 16));
          const float gf = __uint_as_float(e ? (w8[pr] & 0xffff0000u) : (w8[pr] << 16));
          const bool on = inb && (norelu || xf * csc[e] + csh[e] > 0.f);
          const float gm = on ? gf : 0.f;
          ds[j] += gm;
          dq[j] += gm * ((xf - cmu[e]) * cis[e]);
        }
      }
    } else if constexpr (DROP || ST) {
      const unsigned pix = ((unsigned)n * g.P + hh) * g.Q + ww;  // (M * K < 2^32: launcher)
      // the Weyl term of the first pair; the other pairs add a constant (one
      // quarter-rate multiply instead of eight)
      const uint32_t hw0 = DROP ? ((pix * (unsigned)KB + c0) >> 1) * 0x9E3779B1u + (uint32_t)g.drop.seed : 0u;
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) {
        float lo = __uint_as_float(w8[pr] << 16), hi = __uint_as_float(w8[pr] & 0xffff0000u);
        if constexpr (DROP) {
          const uint32_t hsh = hash_u32_lo_w(g.drop.seed, hw0 + (uint32_t)pr * 0x9E3779B1u);
          lo = (hsh & 0xFFFFu) >= g.drop.thr ? bf2f(f2bf(lo * g.drop.scl)) : 0.f;
          hi = (hsh >> 16) >= g.drop.thr ? bf2f(f2bf(hi * g.drop.scl)) : 0.f;
          w8[pr] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
        }
        if constexpr (ST) {
          const float fl = inb ? lo : 0.f, fh = inb ? hi : 0.f;
          ds[2 * pr] += fl;
          dq[2 * pr] += fl * fl;
          ds[2 * pr + 1] += fh;
          dq[2 * pr + 1] += fh * fh;
        }
      }
    }
    const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Y + (long long)n * g.P * g.Q * g.ldy), (short)0, g.P * g.Q * g.ldy * 2, 0x00020000);
    const unsigned o = ((unsigned)(hh * g.Q + ww) * (unsigned)g.ldy + c0) * 2u;
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{w8[0], w8[1], w8[2], w8[3]}, orr, inb ? o : 0x80000000u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{w8[4], w8[5], w8[6], w8[7]}, orr, inb ? o + 16u : 0x80000000u, 0, 0);
  };
  // half h's sums: reduce-scatter over the 16 pixel lanes of each lane group
  // (lane l16 keeps values b0 + k, k < 2, of [ds[0..16), dq[0..16)])
  auto dense_stats = [&](int h) __attribute__((always_inline)) {
    if constexpr (ST) {
      float sv[32];
#pragma unroll
      for (int i = 0; i < 16; ++i) sv[i] = ds[i], sv[16 + i] = dq[i], ds[i] = dq[i] = 0.f;
      butterfly_step<32, 8, 0x128>(sv, lane);
      butterfly_step<16, 4, 0x141>(sv, lane);
      butterfly_step<8, 2, 0x4E>(sv, lane);
      butterfly_step<4, 1, 0xB1>(sv, lane);
      dstat[h][0] += (double)sv[0];
      dstat[h][1] += (double)sv[1];
    }
  };
  // epilogue work in step cst (0..3), MFMA group grp.  EPI_LATE: its vector-
  // memory stores issued AFTER the step's last weight piece (group 2), which
  // the step's closing wait may leave in flight: PM 1 the store unit of group
  // 4, PM 0 / 2 / 3 the unit of group 3 (the group-1 unit's stores precede the
  // group-2 pieces and must not be counted, or the wait would let the last
  // pieces land after the barrier)
  constexpr int EPI_LATE = 2;  // per step 0..3
  auto epi_slot = [&](auto cstc, auto grpc, int ptm, bool live) __attribute__((always_inline)) {
    constexpr int cst = decltype(cstc)::value, grp = decltype(grpc)::value;
    if constexpr (PM == 1) {
      // part p = cst (h = p >> 1, fm2 = 2 (p & 1)) over groups 0..4 of steps
      // 0..3, the statistics of half h in group 5 of steps 1 / 3
      if constexpr (grp < 4) epi_unit(cst >> 1, (cst & 1) * 2, grp >> 1, grp & 1, ptm, live);
      if constexpr (grp == 4) epi_store(cst >> 1, (cst & 1) * 2, ptm, live);
      if constexpr (grp == 5 && (cst & 1)) epi_stats(cst >> 1);
    } else if constexpr (PM == 2) {
      // units (fm = cst, h = 0 / 1) in groups 1 / 3
      if constexpr (grp == 1 || grp == 3) dx_unit(cst, grp >> 1, ptm, live);
    } else {
      // units (fm, h) with h = cst >> 1, fm = 2 (cst & 1) + (grp == 3) in
      // groups 1 / 3 (PM 3: their residual loads in group 0); half h's
      // statistics in group 5 of steps 1 / 3
      if constexpr (RLD && grp == 0) {
        res_load(0, 2 * (cst & 1), cst >> 1, ptm, live);
        res_load(1, 2 * (cst & 1) + 1, cst >> 1, ptm, live);
      }
      if constexpr (grp == 1 || grp == 3)
        dense_unit(2 * (cst & 1) + (grp == 3 ? 1 : 0), cst >> 1, ptm, live, grp == 3 ? 1 : 0);
      if constexpr (grp == 5 && (cst & 1)) dense_stats(cst >> 1);
    }
  };

  // ---- one tile: NS steps (chunk cc = cst / 3, filter row rs = cst % 3),
  // with the previous tile's epilogue (tile ptm; `live` false before the
  // first tile: every store dropped, no statistics)
  auto run_tile = [&](int tl, int ptm, bool live) __attribute__((always_inline)) {
    static_for<0, NS>([&](auto I) __attribute__((always_inline)) {
      constexpr int cst = decltype(I)::value, cc = cst / 3, rs = cst % 3;
      // next step's weights (weights depend on the step only, not the tile)
      wprep((cst + 1) % NS, (cst + 1) & 1);
      // vector-memory ops issued after this step's last weight piece, left in
      // flight by its closing wait: the next chunk's halo loads (rs == 1,
      // needed one step later) and the epilogue's stores
      constexpr int NLATE = (rs == 1 ? XPT * (PM == 2 ? 2 : 1) : 0) + (cst <= 3 ? EPI_LATE : 0);
      const unsigned char* Xl = smem + rs * (HWX * XRB);
      // (this buffer's base as an opaque per-step value: the fragment row
      // addresses are formed once per step, the group offsets are immediates
      // -- hoisted, the 2 x 6 x 8 address registers spilled)
      unsigned wofs = WBASE + (cst & 1) * WBYTES;
      asm volatile("" : "+v"(wofs));
      const unsigned char* Wl = smem + wofs;
      // MFMA group grp = (tap s, channel half kk); its fragments are read
      // during the previous group
      uint4 wfa[NH][FN], xfa[FM], wfb[NH][FN], xfb[FM];
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) wfa[h][fn] = *reinterpret_cast<const uint4*>(Wl + wfrag_off(0, 0, h, fn));
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) xfa[fm] = *reinterpret_cast<const uint4*>(Xl + xoff[fm]);
      static_for<0, 6>([&](auto G) __attribute__((always_inline)) {
        constexpr int grp = decltype(G)::value;
        auto body = [&](uint4 (&wf)[NH][FN], uint4 (&xf)[FM], uint4 (&wn)[NH][FN], uint4 (&xn)[FM])
                        __attribute__((always_inline)) {
          constexpr int gs = (grp + 1) >> 1, gk = (grp + 1) & 1;  // next group's tap / channel half
          if constexpr (grp + 1 < 6) {
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
              xn[fm] = *reinterpret_cast<const uint4*>(Xl + xoff[fm] + gs * XRB + gk * 64);
          }
          // next step's weight pieces (groups 0..2), then the next chunk's
          // halo rows spread over groups 2..5 (the next tile's first chunk
          // after the last one; clamped to this tile at the end of the walk)
#pragma unroll
          for (int j = 0; j < WPW; ++j)
            if (j / WPG == grp) wpiece(j);
          constexpr int G0 = (WPW - 1) / WPG, NGL = 6 - G0, per = (XPT + NGL - 1) / NGL;
          if constexpr (rs == 1 && grp >= G0) {
            if constexpr (cc + 1 == NCH && grp == G0) stage_tile(tl + 1 < ntl ? tl + 1 : tl);
            gload(cc + 1 == NCH ? 0 : cc + 1, (grp - G0) * per, (grp - G0 + 1) * per < XPT ? (grp - G0 + 1) * per : XPT);
          }
          // weight fragment n feeds its four MFMAs, then its register takes the
          // next group's fragment n
#pragma unroll
          for (int n = 0; n < NF; ++n) {
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) {
              // a tile's first MFMA of an accumulator takes C = 0; its last one
              // is followed by the packing of the finished value
              const f4 cin = (cst == 0 && grp == 0) ? f4{0.f, 0.f, 0.f, 0.f} : acc[fm][n];
              const bf8 xa = __builtin_bit_cast(bf8, xf[fm]), wa = __builtin_bit_cast(bf8, wf[n / FN][n % FN]);
              if constexpr (!CPERM) acc[fm][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, wa, cin, 0, 0, 0);
              else acc[fm][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, xa, cin, 0, 0, 0);
              if constexpr (cst == NS - 1 && grp == 5) pack1(fm, n);
            }
            if constexpr (grp + 1 < 6)
              wn[n / FN][n % FN] = *reinterpret_cast<const uint4*>(Wl + wfrag_off(gs, gk, n / FN, n % FN));
          }
          if constexpr (cst <= 3) epi_slot(std::integral_constant<int, cst>{}, std::integral_constant<int, grp>{}, ptm,
                                           live);
        };
        if constexpr ((grp & 1) == 0) body(wfa, xfa, wfb, xfb);
        else body(wfb, xfb, wfa, xfa);
        __builtin_amdgcn_sched_barrier(0);
      });
      stamp(0);
      if constexpr (rs == 2) {
        __syncthreads();  // every wave has finished reading the chunk's rows
        stamp(3);
        sstore(cc + 1 == NCH ? 0 : cc + 1);
        stamp(4);
        wait_vmcnt<NLATE>();  // next step's weight pieces landed
        __syncthreads();
        stamp(5);
      } else {
        wait_vmcnt<NLATE>();
        stamp(1);
        __syncthreads();
        stamp(2);
      }
    });
  };

  if (ntl > 0) {
    stage_tile(0);
    gload(0, 0, XPT);
    wprep(0, 0);
#pragma unroll
    for (int j = 0; j < WPW; ++j) wpiece(j);
    if constexpr (PRO) __syncthreads();  // pss
    sstore(0);
  }
  wait_vmcnt<0>();
  __syncthreads();
  for (int tl = 0; tl < ntl; ++tl) {
    const int tm = walk.tm + tl * walk.step;
    run_tile(tl, tl > 0 ? tm - walk.step : tm, tl > 0);
  }
  // the last tile's epilogue (packed by its last step)
  if (ntl > 0) {
    const int tm = walk.tm + (ntl - 1) * walk.step;
    if constexpr (PM == 1) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int u = 0; u < 4; ++u) epi_unit(p >> 1, (p & 1) * 2, u >> 1, u & 1, tm, true);
        epi_store(p >> 1, (p & 1) * 2, tm, true);
        if (p & 1) epi_stats(p >> 1);
      }
    } else if constexpr (PM == 2) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int h = 0; h < NH; ++h) dx_unit(fm, h, tm, true);
    } else {
#pragma unroll
      for (int h = 0; h < NH; ++h) {
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          if constexpr (RLD) res_load(0, fm, h, tm, true);
          dense_unit(fm, h, tm, true, 0);
        }
        dense_stats(h);
      }
    }
  }
#ifdef ACFE_P1W_STAMPS
  if (PM == 1 && lane == 0 && blockIdx.x * 4 + wp < 4096)
    for (int i = 0; i < 6; ++i) g_p1w_stamps[(blockIdx.x * 4 + wp) * 8 + i] = stv[i];
#endif
  wait_vmcnt<0>();
  __syncthreads();
  if ((PM == 1 || (DENSE && ST)) && stats) {
    // fixed-order sum of the four waves' partials (same slots in the same lanes)
    double* red = reinterpret_cast<double*>(smem);
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int k = 0; k < 2; ++k) red[((wp * 64 + lane) * NH + h) * 2 + k] = dstat[h][k];
    __syncthreads();
    if (wp < NH) {
      const int h = wp;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += red[((w * 64 + lane) * NH + h) * 2 + k];
        if constexpr (PM == 1) {
          const int idx = q * 2 + k;
          stats[((long long)blockIdx.x * 2 + idx / FN) * g.Kp + h * 64 + FN * l16 + idx % FN] = v;
        } else {
          const int idx = ((l16 >> 3) & 1) * 16 + ((l16 >> 2) & 1) * 8 + ((l16 >> 1) & 1) * 4 + (l16 & 1) * 2 + k;
          stats[((long long)(srow0 + blockIdx.x) * 2 + idx / 16) * g.Kp + h * 64 + 16 * q + idx % 16] = v;
        }
      }
    }
    // (the first launch zeroes every row past its own; the remainder-column
    // launch writes its rows afterwards)
    if (srow0 == 0)
      for (int rr = blockIdx.x + gridDim.x; rr < srows; rr += gridDim.x)
      for (int c = tid; c < 2 * KB; c += NT) stats[((long long)rr * 2 + (c / KB)) * g.Kp + (c % KB)] = 0.0;
  }
}

namespace acfe {

static void grid_1w(const ConvGeom& g, double* stats, int srows, int* tiles_h, int* tiles_w, long long* nt, int* gp) {
  *tiles_h = (g.P + 3) / 4;
  *tiles_w = (g.Q + 63) / 64;
  *nt = (long long)g.N * *tiles_h * *tiles_w;
  int n = 256;
  if (n > *nt) n = (int)*nt;
  if (n >= 64) n &= ~7;
  if (stats && n > srows) n = srows;  // one statistics slab row per workgroup
  *gp = n;
}

int launch_pool1w(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
                  int srows, uint8_t* amax, hipStream_t s, const char* what) {
  if (g.K != 128 || g.C != 128 || (long long)g.N * (g.P / 2) * (g.Q / 2) * g.ldy * 2 >= (1ll << 31))
    return ACFE_E_INVAL;
  if ((uintptr_t)y & 15) return ACFE_E_INVAL;
  int th, tw, gp;
  long long nt;
  grid_1w(g, stats, srows, &th, &tw, &nt, &gp);
  if (g.drop.on)
    hipLaunchKernelGGL((k_conv3x3_1w<1, 2, true>), dim3(gp), dim3(256), 0, s, g, (const uint16_t*)x,
                       (const uint16_t*)wp, bias, (uint16_t*)y, stats, th, tw, (int)nt, srows, amax);
  else
    hipLaunchKernelGGL((k_conv3x3_1w<1, 2, false>), dim3(gp), dim3(256), 0, s, g, (const uint16_t*)x,
                       (const uint16_t*)wp, bias, (uint16_t*)y, stats, th, tw, (int)nt, srows, amax);
  return launch_rc(what);
}

int launch_plain1w(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
                   int srows, hipStream_t s, const char* what, int pm) {
  // 3x3 stride 1, K = C = 128, one image's output < 2^31 bytes, 32-bit
  // dropout element indices, 16-B channel runs
  if (g.K != 128 || g.C != 128 || g.R != 3 || g.S != 3 || g.st != 1 || g.ldy != 128 ||
      (long long)g.P * g.Q * g.ldy * 2 >= (1ll << 31) || (g.drop.on && !g.idx32) || ((uintptr_t)y & 15))
    return ACFE_E_INVAL;
  if (g.pro_sc && (!g.pro_sh || !g.pro_out || ((uintptr_t)g.pro_out & 15) || ((uintptr_t)x & 15)))
    return ACFE_E_INVAL;
  if (pm == 3 && (!g.res || g.drop.on)) return ACFE_E_INVAL;
  // the image's whole 64-pixel columns in 4 x 64 tiles, the Q % 64 pixels left
  // of each row (when Q >= 64) in 16 x 16 tiles by a second launch writing the
  // statistics slab rows after the first one's (per-pixel values unchanged:
  // an accumulator's MFMA sequence does not depend on the tiling)
  const int rem = g.Q >= 64 ? g.Q % 64 : 0;
  const int th = (g.P + 3) / 4, tw = rem ? g.Q / 64 : (g.Q + 63) / 64;
  const long long nt = (long long)g.N * th * tw;
  const int the = (g.P + 15) / 16, twe = (rem + 15) / 16;
  const long long nte = rem ? (long long)g.N * the * twe : 0;
  if (nt >= (1ll << 31) || nte >= (1ll << 31)) return ACFE_E_INVAL;
  auto grid_for = [&](long long n, int rows_left) {
    int gp = 256;
    if (gp > n) gp = (int)n;
    if (gp >= 64) gp &= ~7;
    if (stats && gp > rows_left) gp = rows_left;  // one statistics slab row per workgroup
    return gp;
  };
  // (small slabs: leave the second launch up to half of the rows)
  const int gp = grid_for(nt, nte && stats ? srows - (int)(srows / 2 < nte ? srows / 2 : nte) : srows);
  const int gpe = nte ? grid_for(nte, srows - gp) : 0;
  if (nte && gpe <= 0) return ACFE_E_INVAL;
#define P1W_L(PM_, D, S_, PRO_)                                                                                  \
  do {                                                                                                          \
    hipLaunchKernelGGL((k_conv3x3_1w<PM_, 2, D, S_, PRO_, 64>), dim3(gp), dim3(256), 0, s, g, (const uint16_t*)x, \
                       (const uint16_t*)wp, bias, (uint16_t*)y, stats, th, tw, (int)nt, srows, nullptr, 0, 0);   \
    if (nte)                                                                                                    \
      hipLaunchKernelGGL((k_conv3x3_1w<PM_, 2, D, S_, PRO_, 16>), dim3(gpe), dim3(256), 0, s, g,                \
                         (const uint16_t*)x, (const uint16_t*)wp, bias, (uint16_t*)y, stats, the, twe, (int)nte,  \
                         srows, nullptr, g.Q - rem, gp);                                                         \
  } while (0)
  if (g.pro_sc) {  // BN prologue (acfe_conv2d_fwd_bn / fwd_add_bn)
    if (pm == 3) {
      if (stats) P1W_L(3, false, true, true);
      else P1W_L(3, false, false, true);
    } else if (g.drop.on) {
      P1W_L(0, true, true, true);
    } else if (stats) {
      P1W_L(0, false, true, true);
    } else {
      P1W_L(0, false, false, true);
    }
  } else if (pm == 3) {
    if (stats) P1W_L(3, false, true, false);
    else P1W_L(3, false, false, false);
  } else if (g.drop.on) {
    P1W_L(0, true, true, false);
  } else if (stats) {
    P1W_L(0, false, true, false);
  } else {
    P1W_L(0, false, false, false);
  }
#undef P1W_L
  return launch_rc(what);
}

int launch_dgradbn1w(const ConvGeom& g, const void* dy, const void* wflip, void* dx, double* part, int srows,
                     hipStream_t s, const char* what) {
  // acfe_conv2d_dgrad_bn at K = C = 128 (PM 5), tiled as launch_plain1w
  if (g.K != 128 || g.C != 128 || g.R != 3 || g.S != 3 || g.st != 1 || g.ldy != 128 || !part || !g.res ||
      !g.bn_sc || !g.bn_sh || !g.bn_mu || !g.bn_is || (long long)g.P * g.Q * g.ldy * 2 >= (1ll << 31) ||
      ((uintptr_t)dx & 15) || ((uintptr_t)g.res & 15))
    return ACFE_E_INVAL;
  const int rem = g.Q >= 64 ? g.Q % 64 : 0;
  const int th = (g.P + 3) / 4, tw = rem ? g.Q / 64 : (g.Q + 63) / 64;
  const long long nt = (long long)g.N * th * tw;
  const int the = (g.P + 15) / 16, twe = (rem + 15) / 16;
  const long long nte = rem ? (long long)g.N * the * twe : 0;
  if (nt >= (1ll << 31) || nte >= (1ll << 31)) return ACFE_E_INVAL;
  auto grid_for = [&](long long n, int rows_left) {
    int gp = 256;
    if (gp > n) gp = (int)n;
    if (gp >= 64) gp &= ~7;
    if (gp > rows_left) gp = rows_left;
    return gp;
  };
  const int gp = grid_for(nt, nte ? srows - (int)(srows / 2 < nte ? srows / 2 : nte) : srows);
  const int gpe = nte ? grid_for(nte, srows - gp) : 0;
  if (gp <= 0 || (nte && gpe <= 0)) return ACFE_E_INVAL;
  hipLaunchKernelGGL((k_conv3x3_1w<5, 2, false, true, false, 64>), dim3(gp), dim3(256), 0, s, g, (const uint16_t*)dy,
                     (const uint16_t*)wflip, nullptr, (uint16_t*)dx, part, th, tw, (int)nt, srows, nullptr, 0, 0);
  if (nte)
    hipLaunchKernelGGL((k_conv3x3_1w<5, 2, false, true, false, 16>), dim3(gpe), dim3(256), 0, s, g,
                       (const uint16_t*)dy, (const uint16_t*)wflip, nullptr, (uint16_t*)dx, part, the, twe, (int)nte,
                       srows, nullptr, g.Q - rem, gp);
  return launch_rc(what);
}

int launch_unpool1w(const ConvGeom& g, const void* dyp, const void* wflip, void* dx, uint8_t* amax, hipStream_t s,
                    const char* what) {
  // dX of one image < 2^31 bytes (per-image buffer stores), 16-B channel runs
  if (g.K != 128 || g.C != 128 || (long long)g.P * g.Q * g.ldy * 2 >= (1ll << 31) || ((uintptr_t)dx & 15))
    return ACFE_E_INVAL;
  int th, tw, gp;
  long long nt;
  grid_1w(g, nullptr, 0, &th, &tw, &nt, &gp);
  hipLaunchKernelGGL((k_conv3x3_1w<2, 2, false>), dim3(gp), dim3(256), 0, s, g, (const uint16_t*)dyp,
                     (const uint16_t*)wflip, nullptr, (uint16_t*)dx, nullptr, th, tw, (int)nt, 0, amax);
  return launch_rc(what);
}

}  // namespace acfe

#ifdef ACFE_P1W_STAMPS
ACFE_API int acfe_debug_pool1w_stamps(unsigned long long* host, int n) {
  if (n > 4096 * 8) n = 4096 * 8;
  return hip_rc(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_p1w_stamps), sizeof(unsigned long long) * n), "stamps");
}
#endif
