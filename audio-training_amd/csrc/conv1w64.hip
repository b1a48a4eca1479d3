// k_conv3x3_1w64: the 3x3 stride-1 convolutions with K = 64 output channels
// (wr_resnet's stage-1 64-channel layers at 128 x 513 and wr_resnet_bird's
// stage-1 blocks 1 / 2 at 64 x 128, resnet/wr_resnet.py:56-80,
// resnet/wr_resnet_bird.py:136-161) with one wave per SIMD: the plain /
// dropout forward (+ BN sums), the residual-add forward (+ReLU, + BN sums) and
// the stride-1 dgrad, each optionally with the BatchNormalization (+ReLU)
// prologue of acfe_conv2d_fwd_bn / acfe_conv2d_fwd_add_bn (the conv reads the
// BN input x and stages x' = (ReLU)(x * scale + shift), storing x' of its own
// pixels for the weight gradient).  Built with -fno-slp-vectorize (packed f32
// VALU beside MFMAs costs more issue time than the two scalar ops).
//
// The structure is pool1w.hip's at K = 64:
//  * tile TR rows x 64 px x 64 channels; four waves, one per SIMD, wave w owns
//    the TR 16-pixel fragments w TR .. w TR + TR - 1 of the tile (fragment f =
//    tile row f / 4, columns 16 (f % 4) ..) and all 64 channels: 4 weight
//    fragments per TR pixel fragments per MFMA group, 4 TR accumulators;
//  * chunk-resident halo rows: the TR + 2 rows x 66 px of a 64-channel chunk
//    are staged once (160-B pixel pitch) for its three filter-row steps; the
//    three taps' weights of a step arrive by LDS-DMA into a double buffer
//    (rows [s][k] of 128 B, granule swizzle of pool1w's CPERM layout);
//  * the previous tile's epilogue (bias, bf16 rounding, dropout pair hash /
//    residual add + ReLU, BN sums, two 16-B stores per pixel fragment) runs in
//    units between the MFMA groups of this tile's first steps;
//  * MFMA operands weights x pixels: a lane holds 16 consecutive channels of
//    its pixel (permuted weight rows), so stores are 16-B channel runs and the
//    BN sums are reduced over the 16 pixel lanes once per tile.
// Tiles whose step count is odd (C = 64: three steps) alternate the weight
// buffer parity from tile to tile, so the buffer is chosen at run time.
#include "conv_common.h"

using namespace acfe;

template <int TR, int PM, int NCH, bool PRO, bool DROP, bool ST>
__global__ void __launch_bounds__(256, 1)
k_conv3x3_1w64(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
               const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats, int tiles_h,
               int tiles_w, int ntiles, int srows) {
  static_assert(PM == 0 || (PM == 3 && !DROP), "modes: 0 plain / dropout, 3 residual add");
  constexpr int KB = 64, FM = TR, FN = 4, SEGW = 64, HWX = SEGW + 2, XRB = 160;
  constexpr int NT = 256, NS = 3 * NCH;                          // threads, steps per tile
  constexpr int XROWS = TR + 2, XBYTES = XROWS * HWX * XRB;
  constexpr int WBYTES = 3 * KB * 128, WBASE = XBYTES;           // 2 x 24 576 B
  constexpr int XG = XROWS * HWX * 8, XPT = (XG + NT - 1) / NT;  // 16-B input granules
  constexpr int WPW = 3 * KB * 8 / 64 / (NT / 64);               // 6 weight pieces per wave per step
  constexpr int WPG = 2;                                         // pieces per MFMA group (groups 0..2)
  constexpr int CM = 64 * NCH;
  constexpr int BTAB = XBYTES + 2 * WBYTES, PSS = BTAB + KB * 4;
  constexpr int SMEM = PSS + (PRO ? 2 * CM * 4 : 0);
  static_assert(SMEM <= 163840, "LDS");
  static_assert(XPT * NT - XG <= 2 * XROWS * HWX, "spare granules fit the pixel pads");
  static_assert(XPT <= 32, "granule masks");
  static_assert(TR % 2 == 0, "two epilogue units per step");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 b2v __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4;
  const int wp = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tpi = tiles_h * tiles_w;
  const TileWalk walk(ntiles);
  const int ntl = walk.tm < walk.end ? (walk.end - walk.tm + walk.step - 1) / walk.step : 0;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_void*)smem;
  auto tile_of = [&](int tm, int& n, int& hb, int& wb) __attribute__((always_inline)) {
    n = tm / tpi;
    const int rem = tm - n * tpi;
    hb = rem / tiles_w;
    wb = rem - hb * tiles_w;
  };

  float* btab = reinterpret_cast<float*>(smem + BTAB);
  if (tid < KB) btab[tid] = bias ? bias[tid] : 0.f;
  float* pss = reinterpret_cast<float*>(smem + PSS);  // PRO: scale[CM], shift[CM]
  if constexpr (PRO) {
    for (int c = tid; c < g.C; c += NT) {
      pss[c] = g.pro_sc[c];
      pss[CM + c] = g.pro_sh[c];
    }
  }

  // ---- weight pieces (LDS-DMA, 1 KB each, 24 per step): rows [s][k] of 128 B
  // (the chunk's 64 input channels of output channel k at tap s), slot sigma
  // of a row holds granule sigma ^ sw(k), sw(k) = ((k >> 4) & 3) << 1 |
  // ((k >> 1) & 1); piece (s, b) of wave wp = rows 16 wp + 8 b .. + 8 of tap s,
  // whose (k >> 4) & 3 = wp: one lane offset per wave
  unsigned vw;
  {
    const int l8 = lane >> 3;
    const unsigned sw = ((unsigned)(wp & 3) << 1) | ((unsigned)(lane >> 4) & 1u);
    vw = (unsigned)(l8 * g.Kdp * 2) + ((((unsigned)lane & 7u) ^ sw) << 4);
  }
  const int sob = __builtin_amdgcn_readfirstlane(16 * wp * g.Kdp * 2);
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
    asm volatile("" : "+s"(sb_));
    const int s_ = j >> 1, b = j & 1;
    const unsigned so = (unsigned)(sb_ + s_ * g.C * 2 + b * 8 * g.Kdp * 2);
    const unsigned lb = wlb + (s_ * KB + 16 * wp + 8 * b) * 128;
    bldsx4s(vw, dw, so, (unsigned)__builtin_amdgcn_readfirstlane((int)lb));
  };

  // ---- input halo rows of a 64-channel chunk, register-staged: granule i of
  // this thread = halo pixel (tid >> 3) + 32 i, channel slot gr = tid & 7
  const int gr = tid & 7, CB = g.C * 2;
  u32x4 rx[XPT];
  __amdgpu_buffer_rsrc_t xrs, prs;
  int rel[XPT];
  int tbase = 0;
  // cmask: granule's column inside the image (rows outside the image fall
  // outside the image's buffer range, which loads zeros); PRO: imask = row and
  // column inside (zero after the BN), omask = one of the tile's own pixels
  unsigned cmask = 0, imask = 0, omask = 0;
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int idx = tid + NT * i;
    const int xrow = idx / (HWX * 8), xpix = (idx - xrow * (HWX * 8)) >> 3;
    rel[i] = (xrow * g.W + xpix) * CB + gr * 16;
  }
  auto stage_tile = [&](int tl) __attribute__((always_inline)) {
    const int tm = walk.tm + tl * walk.step;
    int n, hb, wb;
    tile_of(tm, n, hb, wb);
    const int sh0 = hb * TR - g.pt, sw0 = wb * SEGW - g.pl;
    int t0 = tid;
    asm volatile("" : "+v"(t0));  // (per tile, not hoisted)
    cmask = imask = omask = 0;
    tbase = (sh0 * g.W + sw0) * CB;
    const long long img = (long long)n * g.H * g.W * g.C;
    xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + img), (short)0, g.H * g.W * CB, 0x00020000);
    if constexpr (PRO)
      prs = __builtin_amdgcn_make_buffer_rsrc((void*)(g.pro_out + img), (short)0, g.pro_out ? g.H * g.W * CB : 0,
                                              0x00020000);
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const unsigned idx = (unsigned)t0 + NT * i;
      const unsigned xrow = idx / (HWX * 8), xpix = (idx % (HWX * 8)) >> 3;
      const bool col = idx < (unsigned)XG && (unsigned)(sw0 + (int)xpix) < (unsigned)g.W;
      cmask |= (col ? 1u : 0u) << i;
      if constexpr (PRO) {
        const bool in = col && (unsigned)(sh0 + (int)xrow) < (unsigned)g.H;
        imask |= (in ? 1u : 0u) << i;
        const bool own = xrow >= 1 && xrow <= (unsigned)TR && xpix >= 1 && xpix <= (unsigned)SEGW;
        omask |= (in && own ? 1u : 0u) << i;
      }
    }
  };
  auto gload = [&](int cc, int i0, int i1) __attribute__((always_inline)) {
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const bool ok = (cmask >> i) & 1u;
      rx[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, ok ? (unsigned)(tbase + cc * 128 + rel[i]) : 0x80000000u, 0,
                                                    0);
    }
  };
  // PRO: rx (chunk cc) -> (ReLU)(x * scale + shift) in bf16 (FMA, max, round
  // to nearest even: acfe_bn_apply's values), zero outside the image; the
  // tile's own pixels also go to pro_out (out-of-range offset otherwise)
  auto xform = [&](int cc) __attribute__((always_inline)) {
    if constexpr (PRO) {
      const f4* ps = reinterpret_cast<const f4*>(pss + cc * 64 + gr * 8);
      const f4 sc0 = ps[0], sc1 = ps[1], sh0 = ps[CM / 4], sh1 = ps[CM / 4 + 1];
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
        rx[i] = ((imask >> i) & 1u) ? v : u32x4{0u, 0u, 0u, 0u};
        __builtin_amdgcn_raw_buffer_store_b128(
            v, prs, ((omask >> i) & 1u) ? (unsigned)(tbase + cc * 128 + rel[i]) : 0x80000000u, 0, 0);
      }
    }
  };
  // LDS slot of granule i; the last round's threads past the image write
  // their (zero) granule into the never-read 32-B pixel pads
  auto sslot = [&](int i) __attribute__((always_inline)) {
    const int idx = tid + NT * i, e = idx - XG;
    return idx < XG ? (idx >> 3) * XRB + gr * 16 : (e >> 1) * XRB + 128 + (e & 1) * 16;
  };
  auto sstore = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) *reinterpret_cast<u32x4*>(smem + sslot(i)) = rx[i];
  };

  // ---- fragment offsets: pixel fragment fm of this wave = tile fragment
  // f = wp TR + fm: B columns = pixels (tile row f / 4, column 16 (f % 4) + l16);
  // weight fragment fn: A row m = l16 = channel 16 (m >> 2) + 4 fn + (m & 3)
  int xoff[FM];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int f = wp * TR + fm;
    xoff[fm] = ((f >> 2) * HWX + (f & 3) * 16 + l16) * XRB + q * 16;
  }
  int wrb[2][FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int k = 16 * (l16 >> 2) + 4 * fn + (l16 & 3);
    const int sw = (((k >> 4) & 3) << 1) | ((k >> 1) & 1);
    wrb[0][fn] = k * 128 + ((q ^ sw) << 4);
    wrb[1][fn] = k * 128 + (((q + 4) ^ sw) << 4);
  }

  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // the previous tile's conv outputs, biased and rounded to bf16, packed:
  // channels 16 q + 4 fn + 0, 1 | 2, 3 of pixel l16 of fragment fm
  u32x2 prev[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) prev[i][j] = u32x2{0u, 0u};
  auto pack1 = [&](int fm, int n) __attribute__((always_inline)) {
    const f4 b4 = *reinterpret_cast<const f4*>(btab + 16 * q + 4 * n);
    const b2v lo = __builtin_convertvector((f2v){acc[fm][n][0] + b4[0], acc[fm][n][1] + b4[1]}, b2v);
    const b2v hi = __builtin_convertvector((f2v){acc[fm][n][2] + b4[2], acc[fm][n][3] + b4[3]}, b2v);
    prev[fm][n] = u32x2{__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi)};
  };

  // ---- epilogue units: unit fm = the 16 consecutive channels 16 q .. of the
  // pixel of fragment fm: dropout (one pair hash per channel pair, acfe_dropout's
  // mask) / residual add (+ReLU), the BN sums of the stored values (ds / dq,
  // reduced over the 16 pixel lanes once per tile), two 16-B stores into the
  // image's output (per-image buffer, < 2^31 bytes: launcher)
  float ds[16], dq[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) ds[i] = dq[i] = 0.f;
  double dstat[2] = {0.0, 0.0};
  u32x4 rres[2][2];  // PM 3: the residual words of the step's two units, loaded in its group 0
  auto pix_of = [&](int fm, int tm, int& n, int& hh, int& ww) __attribute__((always_inline)) {
    int hb, wb;
    tile_of(tm, n, hb, wb);
    const int f = wp * TR + fm;
    hh = hb * TR + (f >> 2);
    ww = wb * SEGW + (f & 3) * 16 + l16;
  };
  auto res_load = [&](int u, int fm, int tm, bool live) __attribute__((always_inline)) {
    int n, hh, ww;
    pix_of(fm, tm, n, hh, ww);
    const bool inb = live && hh < g.P && ww < g.Q;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(g.res + (long long)n * g.P * g.Q * g.ldy), (short)0, g.P * g.Q * g.ldy * 2, 0x00020000);
    const unsigned o = ((unsigned)(hh * g.Q + ww) * (unsigned)g.ldy + 16 * q) * 2u;
    rres[u][0] = __builtin_amdgcn_raw_buffer_load_b128(rr, inb ? o : 0x80000000u, 0, 0);
    rres[u][1] = __builtin_amdgcn_raw_buffer_load_b128(rr, inb ? o + 16u : 0x80000000u, 0, 0);
  };
  auto dense_unit = [&](int fm, int tm, bool live, int u) __attribute__((always_inline)) {
    int n, hh, ww;
    pix_of(fm, tm, n, hh, ww);
    const bool inb = live && hh < g.P && ww < g.Q;
    const int c0 = 16 * q;
    unsigned w8[8];
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) w8[2 * fn] = prev[fm][fn][0], w8[2 * fn + 1] = prev[fm][fn][1];
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
    if constexpr (DROP || ST) {
      const unsigned pix = ((unsigned)n * g.P + hh) * g.Q + ww;  // (M * K < 2^32: launcher)
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) {
        float lo = __uint_as_float(w8[pr] << 16), hi = __uint_as_float(w8[pr] & 0xffff0000u);
        if constexpr (DROP) {
          const uint32_t hsh = drop_pair_hash32(g.drop, pix * (unsigned)KB + c0 + 2 * pr);
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
  // the tile's sums: reduce-scatter over the 16 pixel lanes of each lane group
  // (lane l16 keeps values 2 j + k of [ds[0..16), dq[0..16)], j the lane's slot)
  auto dense_stats = [&]() __attribute__((always_inline)) {
    if constexpr (ST) {
      float sv[32];
#pragma unroll
      for (int i = 0; i < 16; ++i) sv[i] = ds[i], sv[16 + i] = dq[i], ds[i] = dq[i] = 0.f;
      butterfly_step<32, 8, 0x128>(sv, lane);
      butterfly_step<16, 4, 0x141>(sv, lane);
      butterfly_step<8, 2, 0x4E>(sv, lane);
      butterfly_step<4, 1, 0xB1>(sv, lane);
      dstat[0] += (double)sv[0];
      dstat[1] += (double)sv[1];
    }
  };
  // epilogue work in step cst, MFMA group grp: units fm = 2 cst, 2 cst + 1 in
  // groups 1 / 3 (PM 3: their residual loads in group 0), the tile's sums in
  // group 5 of the last unit step.  EPI_LATE: the stores issued after the
  // step's last weight piece (group 2), left in flight by its closing wait
  constexpr int EPI_STEPS = TR / 2, EPI_LATE = 2;
  auto epi_slot = [&](auto cstc, auto grpc, int ptm, bool live) __attribute__((always_inline)) {
    constexpr int cst = decltype(cstc)::value, grp = decltype(grpc)::value;
    if constexpr (cst < EPI_STEPS) {
      if constexpr (PM == 3 && grp == 0) {
        res_load(0, 2 * cst, ptm, live);
        res_load(1, 2 * cst + 1, ptm, live);
      }
      if constexpr (grp == 1 || grp == 3) dense_unit(2 * cst + (grp == 3 ? 1 : 0), ptm, live, grp == 3 ? 1 : 0);
      if constexpr (grp == 5 && cst == EPI_STEPS - 1) dense_stats();
    }
  };
  static_assert(EPI_STEPS <= NS, "epilogue fits the tile's steps");

  // ---- one tile: NS steps (chunk cc = cst / 3, filter row rs = cst % 3),
  // with the previous tile's epilogue (tile ptm; `live` false before the
  // first tile: every store dropped, no statistics)
  auto run_tile = [&](int tl, int ptm, bool live) __attribute__((always_inline)) {
    const int tpar = (tl * NS) & 1;  // weight buffer of the tile's step 0
    static_for<0, NS>([&](auto I) __attribute__((always_inline)) {
      constexpr int cst = decltype(I)::value, cc = cst / 3, rs = cst % 3;
      const int par = (tpar + cst) & 1;
      wprep((cst + 1) % NS, par ^ 1);
      constexpr int NLATE = (rs == 1 ? XPT : 0) + (cst < EPI_STEPS ? EPI_LATE : 0);
      const unsigned char* Xl = smem + rs * (HWX * XRB);
      unsigned wofs = WBASE + par * WBYTES;
      asm volatile("" : "+v"(wofs));
      const unsigned char* Wl = smem + wofs;
      uint4 wfa[FN], xfa[FM], wfb[FN], xfb[FM];
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) wfa[fn] = *reinterpret_cast<const uint4*>(Wl + wrb[0][fn]);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) xfa[fm] = *reinterpret_cast<const uint4*>(Xl + xoff[fm]);
      static_for<0, 6>([&](auto G) __attribute__((always_inline)) {
        constexpr int grp = decltype(G)::value;
        auto body = [&](uint4 (&wf)[FN], uint4 (&xf)[FM], uint4 (&wn)[FN], uint4 (&xn)[FM])
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
            constexpr int i0 = (grp - G0) * per, i1 = (grp - G0 + 1) * per < XPT ? (grp - G0 + 1) * per : XPT;
            if constexpr (i0 < i1) gload(cc + 1 == NCH ? 0 : cc + 1, i0, i1);
          }
          // weight fragment n feeds its FM MFMAs, then its register takes the
          // next group's fragment n
#pragma unroll
          for (int n = 0; n < FN; ++n) {
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) {
              // a tile's first MFMA of an accumulator takes C = 0; its last one
              // is followed by the packing of the finished value
              const f4 cin = (cst == 0 && grp == 0) ? f4{0.f, 0.f, 0.f, 0.f} : acc[fm][n];
              const bf8 xa = __builtin_bit_cast(bf8, xf[fm]), wa = __builtin_bit_cast(bf8, wf[n]);
              acc[fm][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, xa, cin, 0, 0, 0);
              if constexpr (cst == NS - 1 && grp == 5) pack1(fm, n);
            }
            if constexpr (grp + 1 < 6) wn[n] = *reinterpret_cast<const uint4*>(Wl + gs * KB * 128 + wrb[gk][n]);
          }
          epi_slot(std::integral_constant<int, cst>{}, std::integral_constant<int, grp>{}, ptm, live);
        };
        if constexpr ((grp & 1) == 0) body(wfa, xfa, wfb, xfb);
        else body(wfb, xfb, wfa, xfa);
        __builtin_amdgcn_sched_barrier(0);
      });
      if constexpr (rs == 2) {
        __syncthreads();  // every wave has finished reading the chunk's rows
        xform(cc + 1 == NCH ? 0 : cc + 1);
        sstore();
        wait_vmcnt<PRO ? XPT : 0>();  // next step's weight pieces landed (pro_out stores may stay in flight)
        __syncthreads();
      } else {
        wait_vmcnt<NLATE>();
        __syncthreads();
      }
    });
  };

  if constexpr (PRO) __syncthreads();  // pss
  if (ntl > 0) {
    stage_tile(0);
    gload(0, 0, XPT);
    wprep(0, 0);
#pragma unroll
    for (int j = 0; j < WPW; ++j) wpiece(j);
    xform(0);
    sstore();
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
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      if constexpr (PM == 3) res_load(0, fm, tm, true);
      dense_unit(fm, tm, true, 0);
    }
    dense_stats();
  }
  wait_vmcnt<0>();
  __syncthreads();
  if (ST && stats) {
    // fixed-order sum of the four waves' partials (same slots in the same lanes)
    double* red = reinterpret_cast<double*>(smem);
#pragma unroll
    for (int k = 0; k < 2; ++k) red[(wp * 64 + lane) * 2 + k] = dstat[k];
    __syncthreads();
    if (wp == 0) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += red[(w * 64 + lane) * 2 + k];
        const int idx = ((l16 >> 3) & 1) * 16 + ((l16 >> 2) & 1) * 8 + ((l16 >> 1) & 1) * 4 + (l16 & 1) * 2 + k;
        stats[((long long)blockIdx.x * 2 + idx / 16) * g.Kp + 16 * q + idx % 16] = v;
      }
    }
    for (int rr = blockIdx.x + gridDim.x; rr < srows; rr += gridDim.x)
      for (int c = tid; c < 2 * KB; c += NT) stats[((long long)rr * 2 + (c / KB)) * g.Kp + (c % KB)] = 0.0;
  }
}

namespace acfe {

// tile rows of the K = 64 one-wave kernel
constexpr int kTR64 = 6;

int launch_conv1w64(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
                    int srows, hipStream_t s, const char* what, int pm) {
  // 3x3 stride 1, K = 64, C = 64 or 128, one image's output < 2^31 bytes,
  // 32-bit dropout element indices, 16-B channel runs
  if (g.K != 64 || (g.C != 64 && g.C != 128) || g.R != 3 || g.S != 3 || g.st != 1 || g.ldy != 64 ||
      (long long)g.P * g.Q * g.ldy * 2 >= (1ll << 31) || (long long)g.H * g.W * g.C * 2 >= (1ll << 31) ||
      (g.drop.on && !g.idx32) || ((uintptr_t)y & 15) || ((uintptr_t)x & 15) ||
      (g.pro_sc && (g.P != g.H || g.Q != g.W)))
    return ACFE_E_INVAL;
  const int th = (g.P + kTR64 - 1) / kTR64, tw = (g.Q + 63) / 64;
  const long long nt = (long long)g.N * th * tw;
  if (nt >= (1ll << 31)) return ACFE_E_INVAL;
  int gp = 256;
  if (gp > nt) gp = (int)nt;
  if (gp >= 64) gp &= ~7;
  if (stats && gp > srows) gp = srows;  // one statistics slab row per workgroup
  const bool pro = g.pro_sc != nullptr;
#define C1W(PM_, NCH_, PRO_, D, S_)                                                                           \
  hipLaunchKernelGGL((k_conv3x3_1w64<kTR64, PM_, NCH_, PRO_, D, S_>), dim3(gp), dim3(256), 0, s, g,          \
                     (const uint16_t*)x, (const uint16_t*)wp, bias, (uint16_t*)y, stats, th, tw, (int)nt, srows)
#define C1W_NCH(PM_, PRO_, D, S_) \
  do {                            \
    if (g.C == 64)                \
      C1W(PM_, 1, PRO_, D, S_);   \
    else                          \
      C1W(PM_, 2, PRO_, D, S_);   \
  } while (0)
#define C1W_PRO(PM_, D, S_)          \
  do {                               \
    if (pro)                         \
      C1W_NCH(PM_, true, D, S_);     \
    else                             \
      C1W_NCH(PM_, false, D, S_);    \
  } while (0)
  if (pm == 3) {
    if (!g.res || g.drop.on) return ACFE_E_INVAL;
    if (stats) C1W_PRO(3, false, true);
    else C1W_PRO(3, false, false);
  } else if (g.drop.on) {
    C1W_PRO(0, true, true);
  } else if (stats) {
    C1W_PRO(0, false, true);
  } else {
    C1W_PRO(0, false, false);
  }
#undef C1W_PRO
#undef C1W_NCH
#undef C1W
  return launch_rc(what);
}

}  // namespace acfe
