// k_conv3x3_r64: the K = 64 3x3 stride-1 convolutions (wr_resnet's stage-1
// conv2a / conv2b and their dgrads, resnet/wr_resnet.py:46-90; wr_resnet_bird's
// 64-filter conv2b, resnet/wr_resnet_bird.py:152-178) with the epilogue of
// tile i - 1 run between the MFMA groups of tile i.
//
// Tile, LDS images and weight pieces are k_conv3x3_rows<64, 8, PM, XRES>'s:
// 8 rows x 64 pixels x 64 output channels per workgroup of 8 waves (wave =
// channel half wk x row pair wp: 32 channels x 128 pixels, FM = 8 pixel
// fragments x FN = 2 channel fragments), one pipeline step = one 64-channel
// chunk x one filter row (6 MFMA groups of 16), the chunk's 10 halo rows
// staged once (register-staged, optionally through the BatchNormalization
// prologue), the step's weight rows by LDS-DMA into a double buffer.
//
// What changes: k_conv3x3_rows runs its epilogue --
// bias, rounding, dropout pair hashes, the residual Add, the BN sums, the
// stores -- after the tile's last step, with every wave of the workgroup in
// it at once and the MFMA pipes idle (r04 loop stamps: 34-43 % of the cycles
// in the epilogue, 20-35 % in MFMAs; SQ r05: MFMA busy 29.5 %, 7.9 VALU per
// MFMA).  Here, as in the one-wave K = 128 kernel (pool1w.hip):
//  * each accumulator's last MFMA of a tile is followed by its packing (the
//    biased, bf16-rounded value a separate conv stores) into 32 registers,
//    and the tile's first MFMA of it takes C = 0;
//  * the epilogue of the packed tile runs in eight units (one pixel fragment:
//    8 channels of one pixel per lane, one 16-B store) placed after MFMA
//    groups 1 / 3 / 5 of the next tile's first three steps, the residual or
//    BN-input words of a unit loaded one group earlier, the BN sums reduced
//    by a DPP butterfly in the last slot;
//  * the prologue transform of the next chunk's halo rows runs between the
//    MFMA groups of the step before they are stored (k_conv3x3_rows: before
//    the MFMAs);
//  * every step is static code (NCH = C / 64 chunks per tile, a template
//    parameter), so unit and group placement are compile-time.
// Modes: PM 0 plain (+ BN sums ST), 4 + pair-hash Dropout, 3 (ReLU)(conv +
// residual g.res) as ops.add stores it, 5 the dgrad whose dX is a BN's output
// gradient with acfe_bn_bwd_reduce's sums of the stored dX (g.res = the BN
// input, g.bn_*).  PRO: the BN (+ReLU) prologue of the input (x' also stored
// to g.pro_out for the weight gradient).  Results are bit-identical to
// k_conv3x3_rows (same MFMA order per accumulator, same epilogue arithmetic).
#include "conv_common.h"

#include <atomic>
#include <cstdlib>

using namespace acfe;

#ifdef ACFE_R64_STAMPS
// diagnostic build (make stamps): per-wave s_memtime totals of the step
// segments (groups of rs = 0 / 1 / 2, the closing wait + barrier of each, the
// restage + pack), read back by acfe_debug_r64_stamps (tools/r64_stamps.py)
__device__ unsigned long long g_r64_stamps[4096 * 8];
#endif

// SEGW: tile width -- 64 (8 rows x 64 pixels) for the image's whole 64-pixel
// columns, 16 (32 rows x 16 pixels) for the Q % 64 pixels left of a row
// (wofs: the first column of tile column 0), so that wr_resnet's 513-wide
// stage 1 does not run a whole 64-pixel tile per 8 rows for its last pixel;
// srow0: the first statistics slab row of this launch.
template <int PM, int NCH, bool PRO, bool ST, int SEGW = 64>
__global__ void __launch_bounds__(512, 1)
k_conv3x3_r64(ConvGeom g, const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wp,
              const float* __restrict__ bias, uint16_t* __restrict__ Y, double* __restrict__ stats, int tiles_h,
              int tiles_w, int ntiles, int srows, int wofs, int srow0) {
  static_assert(PM == 0 || PM == 3 || PM == 4 || PM == 5, "modes");
  static_assert(SEGW == 64 || SEGW == 16, "tile width");
  static_assert(!PRO || PM != 5, "prologue: forwards");
  constexpr bool DROP = PM == 4;
  constexpr bool SUMS = ST || PM == 5;
  constexpr int KB = 64, TR = 512 / SEGW, FM = 8, FN = 2, HWX = SEGW + 2, XRB = 160, NT = 512;
  constexpr int NS = 3 * NCH;                                   // steps per tile
  constexpr int XROWS = TR + 2, XBYTES = XROWS * HWX * XRB;     // 105 600 B (SEGW 16: 97 920 B)
  constexpr int WBYTES = 3 * KB * 128, WBASE = XBYTES;          // 2 x 24 576 B
  constexpr int XG = XROWS * HWX * 8, XPT = (XG + NT - 1) / NT;  // 16-B halo granules: 11 per thread
  constexpr int WPW = 3 * KB * 8 / 64 / 8;                       // 3 weight pieces per wave per step
  constexpr int SMEM0 = XBYTES + 2 * WBYTES;
  constexpr int SMEMP = SMEM0 + (PRO ? 2 * 64 * NCH * 4 : 0);   // PRO: scale / shift of the C channels
  constexpr int SMEM = SMEMP + (PM == 5 ? 4 * KB * 4 : 0);       // PM 5: [scale | shift | mean | invstd][64]
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  float* pss = reinterpret_cast<float*>(smem + SMEM0);
  float* bnt = reinterpret_cast<float*>(smem + SMEMP);
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, q = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wid >> 2, wp = wid & 3;
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
  if constexpr (PRO)
    for (int i = tid; i < 64 * NCH; i += NT) pss[i] = g.pro_sc[i], pss[64 * NCH + i] = g.pro_sh[i];
  if constexpr (PM == 5)
    for (int i = tid; i < KB; i += NT)
      bnt[i] = g.bn_sc[i], bnt[KB + i] = g.bn_sh[i], bnt[2 * KB + i] = g.bn_mu[i], bnt[3 * KB + i] = g.bn_is[i];
  // the lane's 8 output channels c0 + [0, 8), c0 = 32 wk + 8 q (accumulator
  // (fm, fn) element j = channel c0 + 4 fn + j of pixel fm * 16 + l16)
  const int c0 = wk * 32 + 8 * q;
  float bl[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bl[j] = (PM != 5 && bias) ? bias[c0 + j] : 0.f;

  // ---- weight pieces (LDS-DMA, 1 KB = 8 rows of 128 B, 3 per wave per step):
  // LDS rows [s][k] of one tap's 64-channel chunk, 16-B slot sigma holds
  // granule sigma ^ sw(k), sw(k) = ((k >> 3) & 3) << 1 | ((k >> 1) & 1)
  unsigned vwo[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int R0 = (wid * WPW + j) * 8, s_ = R0 / KB, k = R0 - s_ * KB + (lane >> 3);
    const int sw = (((k >> 3) & 3) << 1) | ((k >> 1) & 1);
    vwo[j] = (unsigned)((k * g.Kdp + s_ * g.C + (((lane & 7) ^ sw) << 3)) * 2);
  }
  unsigned wlo = 0, whi = 0, wlb = 0;
  auto wprep = [&](int st, int wb) __attribute__((always_inline)) {
    const int cc = st / 3, r = st - cc * 3;
    const unsigned long long base = (unsigned long long)(uintptr_t)Wp + ((unsigned)(r * 3 * g.C + cc * 64) * 2u);
    wlo = (unsigned)base;
    whi = (unsigned)(base >> 32);
    wlb = lds0 + WBASE + wb * WBYTES + wid * WPW * 1024;
  };
  auto wpiece = [&](int j) __attribute__((always_inline)) {
    const i4 dw = {__builtin_amdgcn_readfirstlane((int)wlo), __builtin_amdgcn_readfirstlane((int)whi),
                   (int)0x80000000u, 0x00020000};
    bldsx4(vwo[j], dw, (unsigned)__builtin_amdgcn_readfirstlane((int)(wlb + j * 1024)));
  };

  // ---- halo rows of a 64-channel chunk, register-staged: granule i of this
  // thread = halo pixel (tid >> 3) + 64 i (row xrow_i, pixel xpix_i, tile
  // independent), channel slot gr = tid & 7
  const int gr = tid & 7, CB = g.C * 2;
  u32x4 rx[XPT];
  int rel[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int idx = tid + NT * i;
    const int xrow = idx / (HWX * 8), xpix = (idx - xrow * (HWX * 8)) >> 3;
    rel[i] = (xrow * g.W + xpix) * CB + gr * 16;
  }
  int tbase = 0;
  unsigned cmask = 0, vmask = 0, omask = 0;
  __amdgpu_buffer_rsrc_t xrs, prs;
  // per tile: the halo origin's byte offset (rows outside the image fall
  // outside its buffer: zeros), the granules whose column lies inside the
  // image (PRO: and whose row does; the tile's own pixels -> pro_out)
  auto stage_tile = [&](int tl) __attribute__((always_inline)) {
    const int tm = walk.tm + tl * walk.step;
    int n, hb, wb;
    tile_of(tm, n, hb, wb);
    const int sh0 = hb * TR - g.pt, sw0 = wofs + wb * SEGW - g.pl;
    int t0 = tid;
    asm volatile("" : "+v"(t0));  // (per tile, not hoisted)
    tbase = (sh0 * g.W + sw0) * CB;
    xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (long long)n * g.H * g.W * g.C), (short)0, g.H * g.W * CB,
                                            0x00020000);
    cmask = vmask = omask = 0;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const unsigned idx = (unsigned)t0 + NT * i;
      const int xrow = (int)(idx / (HWX * 8)), xpix = (int)((idx % (HWX * 8)) >> 3);
      // (bitwise: no branches)
      const bool ok = (idx < (unsigned)XG) & ((unsigned)(sw0 + xpix) < (unsigned)g.W);
      cmask |= (ok ? 1u : 0u) << i;
      if constexpr (PRO) {
        const bool in = ok & ((unsigned)(sh0 + xrow) < (unsigned)g.H);
        const bool own = in & (xrow >= 1) & (xrow <= TR) & (xpix >= 1) & (xpix <= SEGW);
        vmask |= (in ? 1u : 0u) << i;
        omask |= (own ? 1u : 0u) << i;
      }
    }
    if constexpr (PRO)
      prs = __builtin_amdgcn_make_buffer_rsrc((void*)(g.pro_out + (long long)n * g.H * g.W * g.C), (short)0,
                                              g.H * g.W * CB, 0x00020000);
  };
  auto gload = [&](int cc, int i0, int i1) __attribute__((always_inline)) {
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const bool ok = (cmask >> i) & 1u;
      rx[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, ok ? (unsigned)(tbase + cc * 128 + rel[i]) : 0x80000000u,
                                                    0, 0);
    }
  };
  // PRO: granules i0 .. i1 of chunk cc -> (ReLU)(x * scale + shift) in bf16
  // (FMA, max, round to nearest even: acfe_bn_apply's values), zero outside the
  // image (the conv pads x', not x); the tile's own pixels also to pro_out
  auto xform = [&](int cc, int i0, int i1) __attribute__((always_inline)) {
    if constexpr (PRO) {
      const f4* ps = reinterpret_cast<const f4*>(pss + cc * 64 + gr * 8);
      const f4 sc0 = ps[0], sc1 = ps[1], sh0 = ps[16 * NCH], sh1 = ps[16 * NCH + 1];
      const bool relu = g.pro_relu != 0;
#pragma unroll
      for (int i = i0; i < i1; ++i) {
        u32x4 v = rx[i];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const float s0 = d < 2 ? sc0[2 * d] : sc1[2 * d - 4], s1 = d < 2 ? sc0[2 * d + 1] : sc1[2 * d - 3];
          const float h0 = d < 2 ? sh0[2 * d] : sh1[2 * d - 4], h1 = d < 2 ? sh0[2 * d + 1] : sh1[2 * d - 3];
          float lo = __builtin_fmaf(__uint_as_float(v[d] << 16), s0, h0);
          float hi = __builtin_fmaf(__uint_as_float(v[d] & 0xffff0000u), s1, h1);
          if (relu) lo = fmaxf(lo, 0.f), hi = fmaxf(hi, 0.f);
          const b2v pk = __builtin_convertvector((f2v){lo, hi}, b2v);
          v[d] = __builtin_bit_cast(unsigned, pk);
        }
        v = ((vmask >> i) & 1u) ? v : u32x4{0u, 0u, 0u, 0u};
        rx[i] = v;
        __builtin_amdgcn_raw_buffer_store_b128(
            v, prs, ((omask >> i) & 1u) ? (unsigned)(tbase + cc * 128 + rel[i]) : 0x80000000u, 0, 0);
      }
    }
  };
  const int xsto = (tid >> 3) * XRB + gr * 16;
  auto sstore = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < XPT; ++i)
      if (tid + NT * i < XG) *reinterpret_cast<u32x4*>(smem + xsto + i * 64 * XRB) = rx[i];
  };

  // ---- fragment offsets: pixel fragment fm = tile pixels wp * 128 + fm * 16
  // + l16 (tile rows 2 wp, 2 wp + 1); weight fragment fn, A row m = l16 =
  // channel 32 wk + 8 (m >> 2) + 4 fn + (m & 3)
  int xoff[FM], wrb[FN];
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int p = wp * 128 + fm * 16;
    xoff[fm] = ((p / SEGW) * HWX + (p % SEGW) + l16) * XRB + q * 16;
  }
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int k = wk * 32 + (l16 >> 2) * 8 + fn * 4 + (l16 & 3);
    const int sw = (((k >> 3) & 3) << 1) | ((k >> 1) & 1);
    wrb[fn] = k * 128 + ((q ^ sw) << 4);
  }

  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // the previous tile's outputs (biased, rounded to bf16), packed: pk[fm][2 fn
  // + h] = channels c0 + 4 fn + 2 h, + 1 of pixel fragment fm
  unsigned pk[FM][2 * FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 2 * FN; ++j) pk[i][j] = 0u;
  auto pack1 = [&](int fm, int fn) __attribute__((always_inline)) {
    f4 v = acc[fm][fn];
    if constexpr (PM != 5) v += f4{bl[4 * fn], bl[4 * fn + 1], bl[4 * fn + 2], bl[4 * fn + 3]};
    pk[fm][2 * fn] = __builtin_bit_cast(unsigned, __builtin_convertvector((f2v){v[0], v[1]}, b2v));
    pk[fm][2 * fn + 1] = __builtin_bit_cast(unsigned, __builtin_convertvector((f2v){v[2], v[3]}, b2v));
  };

  // ---- epilogue units.  Unit u = pixel fragment u of the finished tile ptm:
  // one pixel per lane, its 8 channels c0 .. c0 + 7 (one 16-B store); `live`
  // false before the first tile (stores dropped, nothing summed).  Per-image
  // buffers (< 2^31 bytes: launcher) with an out-of-range offset for pixels
  // outside the image.
  float sv[16];  // [sum | sum of squares][8 channels] of the tile in progress
#pragma unroll
  for (int i = 0; i < 16; ++i) sv[i] = 0.f;
  double dstat = 0.0;
  // PM 3: residual words, PM 5: BN input words of units u .. u + 2 (ring of
  // three, slot u % 3: unit u's words are requested three units ahead)
  u32x4 eld[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) eld[i] = u32x4{0u, 0u, 0u, 0u};
  // unit u's pixel: tile row 2 wp + u / 4 (wave-uniform: scalar), column
  // (u % 4) * 16 + l16; the lane parts of its byte offset and of its dropout
  // Weyl term are formed once (no per-unit multiplies; mod 2^32 like the
  // direct form).  Bitwise, not short-circuit: no branches inside an MFMA group.
  const unsigned lane_o = ((unsigned)l16 * (unsigned)g.ldy + (unsigned)c0) * 2u;
  const unsigned lane_h = ((unsigned)l16 * (unsigned)(KB / 2) + (unsigned)(c0 >> 1)) * 0x9E3779B1u;
  const unsigned lane_k = (unsigned)l16 * (KB / 8) + (unsigned)(c0 >> 3);  // keep-bit byte of the lane
  auto unit_px = [&](int u, int tm, bool live, int& n, unsigned& o, bool& inb, unsigned* spx = nullptr)
                     __attribute__((always_inline)) {
    int hb, wb;
    tile_of(tm, n, hb, wb);
    // the unit's 16 pixels: tile pixels wp * 128 + u * 16 + l16
    // (SEGW 64: row 2 wp + u / 4, column (u % 4) 16; SEGW 16: row 8 wp + u)
    const int hh = hb * TR + (SEGW == 64 ? 2 * wp + (u >> 2) : 8 * wp + u), wc = wofs + wb * SEGW + (SEGW == 64 ? (u & 3) * 16 : 0);
    inb = live & (hh < g.P) & (wc + l16 < g.Q);
    o = (unsigned)(hh * g.Q + wc) * (unsigned)g.ldy * 2u + lane_o;
    if (spx) *spx = (unsigned)(hh * g.Q + wc);  // the unit's first pixel in its image (scalar)
  };
  auto unit_load = [&](int u, int tm, bool live) __attribute__((always_inline)) {
    if constexpr (PM == 3 || PM == 5) {
      int n;
      unsigned o;
      bool inb;
      unit_px(u, tm, live, n, o, inb);
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(g.res + (long long)n * g.P * g.Q * g.ldy), (short)0, g.P * g.Q * g.ldy * 2, 0x00020000);
      eld[u % 3] = __builtin_amdgcn_raw_buffer_load_b128(rr, inb ? o : 0x80000000u, 0, 0);
    }
  };
  auto unit = [&](int u, int tm, bool live) __attribute__((always_inline)) {
    int n;
    unsigned o, spx;
    bool inb;
    unit_px(u, tm, live, n, o, inb, &spx);
    unsigned w8[4] = {pk[u][0], pk[u][1], pk[u][2], pk[u][3]};
    if constexpr (PM == 3) {
      // z = (ReLU)(conv + residual), rounded to bf16 (ops.add's values)
      const u32x4 rv = eld[u % 3];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float lo = __uint_as_float(w8[d] << 16) + __uint_as_float(rv[d] << 16);
        float hi = __uint_as_float(w8[d] & 0xffff0000u) + __uint_as_float(rv[d] & 0xffff0000u);
        if (g.res_relu) lo = fmaxf(lo, 0.f), hi = fmaxf(hi, 0.f);
        w8[d] = __builtin_bit_cast(unsigned, __builtin_convertvector((f2v){lo, hi}, b2v));
      }
    }
    if constexpr (DROP) {
      // acfe_dropout's mask: one pair hash per channel pair, the Weyl term of
      // the first pair advanced by a constant (M * K < 2^32: launcher)
      // ((n P + hh) Q + wc): the unit's first pixel (spx) plus the image's
      const unsigned spix = (unsigned)n * (unsigned)(g.P * g.Q) + spx;
      // ((pix K + c0) >> 1) W + seed with pix = spix + l16 (K = 64, c0 even)
      const uint32_t hw0 = spix * (unsigned)(KB / 2) * 0x9E3779B1u + lane_h + (uint32_t)g.drop.seed;
      // per dword (channel pair): both values times the keep scale, rounded
      // by one v_cvt_pk_bf16_f32, then ANDed with the pair's 16-bit keep
      // masks; the keep bits gathered from the masks (bit 2 d <- bit 0,
      // bit 2 d + 1 <- bit 16) -- the same words as rounding each kept value
      // separately and zeroing the dropped ones (r06: 16 -> ~10 VALU per pair)
      unsigned kacc = 0;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t hsh = hash_u32_lo_w(g.drop.seed, hw0 + (uint32_t)d * 0x9E3779B1u);
        const unsigned m = ((hsh & 0xFFFFu) >= g.drop.thr ? 0x0000ffffu : 0u) |
                           ((hsh >> 16) >= g.drop.thr ? 0xffff0000u : 0u);
        const float lo = __uint_as_float(w8[d] << 16) * g.drop.scl;
        const float hi = __uint_as_float(w8[d] & 0xffff0000u) * g.drop.scl;
        w8[d] = pk_bf2(lo, hi) & m;
        kacc |= (m & 0x00010001u) << (2 * d);
      }
      const unsigned kbits = (kacc | (kacc >> 15)) & 0xffu;
      // the keep bits of channels c0 .. c0 + 7: one byte at (pixel, c0 / 8) of
      // [M][K / 8] (g.keep_out; a null buffer drops the store)
      const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(g.keep_out + (long long)n * g.P * g.Q * (KB / 8)), (short)0,
          g.keep_out ? g.P * g.Q * (KB / 8) : 0, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b8((unsigned char)kbits, kr, inb ? spx * (KB / 8) + lane_k : 0x80000000u, 0, 0);
    }
    const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Y + (long long)n * g.P * g.Q * g.ldy), (short)0, g.P * g.Q * g.ldy * 2, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{w8[0], w8[1], w8[2], w8[3]}, orr, inb ? o : 0x80000000u, 0, 0);
    // pixels outside the image: their (dropped) values count as zeros in the sums
#pragma unroll
    for (int d = 0; d < 4; ++d) w8[d] = inb ? w8[d] : 0u;
    if constexpr (PM == 5) {
      // acfe_bn_bwd_reduce's terms of the stored dX: gm = dX masked by the BN's
      // ReLU, summed as gm and gm * (x - mean) * invstd
      const u32x4 xv = eld[u % 3];
      const bool norelu = g.bn_relu == 0;
      unsigned bo = (unsigned)(c0 * 4);
      asm volatile("" : "+v"(bo));  // (read per unit, not hoisted into 32 live registers)
      const f4* bt = reinterpret_cast<const f4*>(reinterpret_cast<const unsigned char*>(bnt) + bo);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const f4 csc = bt[hf], csh = bt[16 + hf], cmu = bt[32 + hf], cis = bt[48 + hf];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int e = 4 * hf + jj;
          const unsigned xw = xv[e >> 1], gw = w8[e >> 1];
          const float xf = __uint_as_float((e & 1) ? (xw & 0xffff0000u) : (xw << 16));
          const float gf = __uint_as_float((e & 1) ? (gw & 0xffff0000u) : (gw << 16));
          const bool on = inb & (norelu | (xf * csc[jj] + csh[jj] > 0.f));
          const float gm = on ? gf : 0.f;
          sv[e] += gm;
          sv[8 + e] += gm * ((xf - cmu[jj]) * cis[jj]);
        }
      }
    } else if constexpr (ST) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const unsigned wv = w8[e >> 1];
        const float f = __uint_as_float((e & 1) ? (wv & 0xffff0000u) : (wv << 16));
        sv[e] += f;
        sv[8 + e] += f * f;
      }
    }
    // the ring slot just read takes unit u + 3's words
    if (u + 3 < FM) unit_load(u + 3, tm, live);
  };
  // the finished tile's sums: reduce-scatter over the 16 pixel lanes of each
  // lane group (lane l16 keeps value l16 of sv), accumulated in double
  auto unit_stats = [&]() __attribute__((always_inline)) {
    if constexpr (SUMS) {
      butterfly_step<16, 8, 0x128>(sv, lane);
      butterfly_step<8, 4, 0x141>(sv, lane);
      butterfly_step<4, 2, 0x4E>(sv, lane);
      butterfly_step<2, 1, 0xB1>(sv, lane);
      dstat += (double)sv[0];
#pragma unroll
      for (int i = 0; i < 16; ++i) sv[i] = 0.f;
    }
  };
  // units of the previous tile: u = grp in step 0, u = 6 + grp in groups 0 / 1
  // of step 1, the sums in its group 2 -- all done before step 1's halo loads
  // (groups 3..5), so the packed outputs and the staged rows are never live
  // together
  auto epi_slot = [&](auto cstc, auto grpc, int ptm, bool live) __attribute__((always_inline)) {
    constexpr int cst = decltype(cstc)::value, grp = decltype(grpc)::value;
    if constexpr (cst == 0) unit(grp, ptm, live);
    if constexpr (cst == 1 && grp < 2) unit(6 + grp, ptm, live);
    if constexpr (cst == 1 && grp == 2) unit_stats();
  };
  // VMEM operations a step issues after its last weight piece (group 2's) and
  // leaves in flight at its closing wait: step 0 the stores of units 3..5 (and
  // their keep-bit bytes) and the loads of units 6, 7; rs == 1 the next chunk's halo loads (groups
  // 3..5); the last step the loads of the next epilogue's units 0..2
  constexpr bool ELD = PM == 3 || PM == 5;
  auto late_ops = [](int cst) constexpr {
    int n = (cst % 3 == 1) ? XPT : 0;
    if (cst == 0) n += 3 * (DROP ? 2 : 1) + (ELD ? 2 : 0);  // (DROP: + the keep-bit byte stores)
    if (cst == NS - 1 && ELD) n += 3;
    return n;
  };

#ifdef ACFE_R64_STAMPS
  unsigned long long stv[8] = {0, 0, 0, 0, 0, 0, 0, 0}, stl = __builtin_amdgcn_s_memtime();
  auto stamp = [&](int i) __attribute__((always_inline)) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    stv[i] += t - stl;
    stl = t;
  };
#else
  auto stamp = [](int) __attribute__((always_inline)) {};
#endif
#ifdef ACFE_R64_PRIO
  if (wk) __builtin_amdgcn_s_setprio(1);  // static priority for the second-dispatched half (A/B)
#endif
  int wpar = 0;  // weight buffer of the current step (NS may be odd)
  // ---- one tile: NS steps (chunk cc = cst / 3, filter row rs = cst % 3) with
  // the previous tile's epilogue in steps 0 / 1
  auto run_tile = [&](int tl, int tm, int ptm, bool live) __attribute__((always_inline)) {
    static_for<0, NS>([&](auto I) __attribute__((always_inline)) {
      constexpr int cst = decltype(I)::value, cc = cst / 3, rs = cst % 3;
      constexpr int cn = cc + 1 == NCH ? 0 : cc + 1;  // chunk staged during this chunk
      wprep((cst + 1) % NS, wpar ^ 1);
      constexpr int NLATE = late_ops(cst);
      const unsigned char* Xl = smem + rs * (HWX * XRB);
      unsigned wofs = WBASE + wpar * WBYTES;
      asm volatile("" : "+v"(wofs));
      const unsigned char* Wl = smem + wofs;
      static_for<0, 6>([&](auto G) __attribute__((always_inline)) {
        constexpr int grp = decltype(G)::value, s = grp >> 1, kk = grp & 1;
        // next step's weight pieces (groups 0..2)
        if constexpr (grp < WPW) wpiece(grp);
        // rs == 1: the next chunk's halo rows over groups 3..5 (the next
        // tile's first chunk after the last one; clamped at the end of the walk)
        if constexpr (rs == 1 && grp >= 3) {
          constexpr int per = (XPT + 2) / 3, i0 = (grp - 3) * per, i1 = i0 + per < XPT ? i0 + per : XPT;
          if constexpr (cc + 1 == NCH && grp == 3) stage_tile(tl + 1 < ntl ? tl + 1 : tl);
          gload(cn, i0, i1);
        }
        // rs == 2: their prologue transform between the MFMA groups
        if constexpr (PRO && rs == 2) {
          constexpr int per = (XPT + 5) / 6, i0 = grp * per, i1 = i0 + per < XPT ? i0 + per : XPT;
          if constexpr (i0 < XPT) xform(cn, i0, i1);
        }
        uint4 wf[FN], xf[FM];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          wf[fn] = *reinterpret_cast<const uint4*>(Wl + s * KB * 128 + (wrb[fn] ^ (kk << 6)));
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) xf[fm] = *reinterpret_cast<const uint4*>(Xl + xoff[fm] + s * XRB + kk * 64);
        auto mfmas = [&]() __attribute__((always_inline)) {
#pragma unroll
          for (int fm = 0; fm < FM; ++fm)
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
              // a tile's first MFMA of an accumulator takes C = 0
              const f4 cin = (cst == 0 && grp == 0) ? f4{0.f, 0.f, 0.f, 0.f} : acc[fm][fn];
              acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, wf[fn]),
                                                                    __builtin_bit_cast(bf8, xf[fm]), cin, 0, 0, 0);
            }
        };
#ifdef ACFE_R64_STAGGER
        // the two waves of a SIMD (wid, wid + 4: channel halves wk 0 / 1) in
        // complementary order: wk 0 MFMAs then the epilogue unit, wk 1 the
        // unit (its fragment reads in flight) then the MFMAs
        constexpr bool HAS_UNIT = cst == 0 || (cst == 1 && grp < 3);
        if (HAS_UNIT && wk) {
          epi_slot(std::integral_constant<int, cst>{}, std::integral_constant<int, grp>{}, ptm, live);
          __builtin_amdgcn_sched_barrier(0);
          mfmas();
        } else {
          mfmas();
          if constexpr (HAS_UNIT) {
            __builtin_amdgcn_sched_barrier(0);
            epi_slot(std::integral_constant<int, cst>{}, std::integral_constant<int, grp>{}, ptm, live);
          }
        }
#elif defined(ACFE_R64_VFIRST)
        // the unit's VALU first (the group's fragment reads in flight), then the MFMAs
        epi_slot(std::integral_constant<int, cst>{}, std::integral_constant<int, grp>{}, ptm, live);
        mfmas();
#else
        mfmas();
        epi_slot(std::integral_constant<int, cst>{}, std::integral_constant<int, grp>{}, ptm, live);
#endif
        __builtin_amdgcn_sched_barrier(0);
      });
      wpar ^= 1;
      stamp(rs);
      if constexpr (rs == 2) {
        __syncthreads();  // every wave has finished reading the chunk's rows
        stamp(5);
        sstore();
        if constexpr (cst == NS - 1) {
          // the finished tile packed (after the restage: its rows and the
          // packed outputs are never live together), its first units' loads
#pragma unroll
          for (int fm = 0; fm < FM; ++fm)
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) pack1(fm, fn);
#pragma unroll
          for (int u = 0; u < 3; ++u) unit_load(u, tm, true);
        }
        stamp(6);
        wait_vmcnt<NLATE>();  // next step's weight pieces landed
        __syncthreads();
        stamp(7);
      } else {
        wait_vmcnt<NLATE>();
        __syncthreads();
        stamp(3 + rs);
      }
    });
  };

  if constexpr (PRO || PM == 5) __syncthreads();  // pss / bnt
  if (ntl > 0) {
    stage_tile(0);
    gload(0, 0, XPT);
    wprep(0, 0);
#pragma unroll
    for (int j = 0; j < WPW; ++j) wpiece(j);
    xform(0, 0, XPT);
    sstore();
  }
  wait_vmcnt<0>();
  __syncthreads();
  for (int tl = 0; tl < ntl; ++tl) {
    const int tm = walk.tm + tl * walk.step;
    run_tile(tl, tm, tl > 0 ? tm - walk.step : tm, tl > 0);
  }
  // the last tile's epilogue (packed, its first loads issued, by its last step)
  if (ntl > 0) {
    const int tm = walk.tm + (ntl - 1) * walk.step;
#pragma unroll
    for (int u = 0; u < FM; ++u) unit(u, tm, true);
    unit_stats();
  }
#ifdef ACFE_R64_STAMPS
  if (lane == 0 && blockIdx.x * 8 + wid < 4096)
    for (int i = 0; i < 8; ++i) g_r64_stamps[(blockIdx.x * 8 + wid) * 8 + i] = stv[i];
#endif
  wait_vmcnt<0>();
  __syncthreads();
  if (SUMS && stats) {
    // the 4 waves of one channel half (wid = wk * 4 + wp) hold partials of the
    // same (channel, sum / sum-of-squares) slots in the same lanes: fixed-order
    // sum through LDS (free after the main loop), wave wp = 0 writes the row
    double* red = reinterpret_cast<double*>(smem);
    red[wid * 64 + lane] = dstat;
    __syncthreads();
    if (wp == 0) {
      double v = 0.0;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[(wk * 4 + w) * 64 + lane];
      // lane l16 keeps value l16 of [sums | squares][8 channels c0 + ..]
      stats[((long long)(srow0 + blockIdx.x) * 2 + (l16 >> 3)) * g.Kp + c0 + (l16 & 7)] = v;
    }
    // (the first launch zeroes every row past its own; a remainder-column
    // launch writes its rows afterwards)
    if (srow0 == 0)
      for (int rr = blockIdx.x + gridDim.x; rr < srows; rr += gridDim.x)
      for (int c = tid; c < 2 * KB; c += NT) stats[((long long)rr * 2 + (c / KB)) * g.Kp + (c % KB)] = 0.0;
  }
}

namespace acfe {

// ACFE_R64=0 / acfe_conv_r64_enable(0): the K = 64 row-halo convolutions on
// k_conv3x3_rows (A/B, parity tests)
static std::atomic<int> g_r64{-1};
static bool r64_on() {
  int v = g_r64.load(std::memory_order_relaxed);
  if (v < 0) {
    v = (!getenv("ACFE_R64") || atoi(getenv("ACFE_R64")) != 0) ? 1 : 0;
    g_r64.store(v, std::memory_order_relaxed);
  }
  return v != 0;
}

bool r64_enabled() { return r64_on(); }

int launch_r64(const ConvGeom& g, const void* x, const void* wp, const float* bias, void* y, double* stats,
               int srows, hipStream_t s, const char* what, int pm) {
  // 3x3 stride 1 "same"-shaped halo (pads 0..2), K = 64, C in {64, 128, 256},
  // one image's input / output < 2^31 bytes, 32-bit dropout element indices,
  // 16-B channel runs
  const int nch = g.C / 64;
  if (!r64_on() || g.K != 64 || g.Kp != 64 || g.C % 64 != 0 || (nch != 1 && nch != 2 && nch != 4) || g.R != 3 ||
      g.S != 3 || g.st != 1 || g.pt < 0 || g.pt > 2 || g.pl < 0 || g.pl > 2 || g.ldy % 8 != 0 ||
      (long long)g.P * g.Q * g.ldy * 2 >= (1ll << 31) || (long long)g.H * g.W * g.C * 2 >= (1ll << 31) ||
      (g.drop.on && (pm != 4 || !g.idx32)) || ((uintptr_t)y & 15) || ((uintptr_t)x & 15))
    return ACFE_E_INVAL;
  const bool pro = g.pro_sc != nullptr;
  if (pro && (pm == 5 || !g.pro_sh || g.pt != 1 || g.pl != 1 || ((uintptr_t)g.pro_out & 15) || !g.pro_out))
    return ACFE_E_INVAL;
  if ((pm == 3 || pm == 5) && (!g.res || ((uintptr_t)g.res & 15))) return ACFE_E_INVAL;
  if (g.keep_out && (pm != 4 || !g.drop.on)) return ACFE_E_INVAL;
  if (pm == 5 && (!stats || !g.bn_sc || !g.bn_sh || !g.bn_mu || !g.bn_is)) return ACFE_E_INVAL;
  if (pm != 0 && pm != 3 && pm != 4 && pm != 5) return ACFE_E_INVAL;
  if (pm == 4 && !stats) return ACFE_E_INVAL;
  const bool st = stats != nullptr;
  // the image's whole 64-pixel columns in 8 x 64 tiles, the Q % 64 pixels
  // left of each row (when Q >= 64) in 32 x 16 tiles by a second launch that
  // writes the statistics slab rows after the first one's (the per-pixel
  // values are the same either way: each accumulator's MFMA sequence does not
  // depend on the tiling)
  const int rem = g.Q >= 64 ? g.Q % 64 : 0;
  const int tiles_h = (g.P + 7) / 8, tiles_w = rem ? g.Q / 64 : (g.Q + 63) / 64;
  const long long nt = (long long)g.N * tiles_h * tiles_w;
  const int tiles_he = (g.P + 31) / 32, tiles_we = (rem + 15) / 16;
  const long long nte = rem ? (long long)g.N * tiles_he * tiles_we : 0;
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
#define R64L(SW_, PM_, NCH_, PRO_, ST_, G_, TH_, TW_, NT_, WO_, SR_)                                              \
  hipLaunchKernelGGL((k_conv3x3_r64<PM_, NCH_, PRO_, ST_, SW_>), dim3(G_), dim3(512), 0, s, g, (const uint16_t*)x, \
                     (const uint16_t*)wp, bias, (uint16_t*)y, stats, TH_, TW_, (int)(NT_), srows, WO_, SR_)
#define R64N(PM_, PRO_, ST_)                                                                                   \
  do {                                                                                                         \
    if (nch == 1) R64L(64, PM_, 1, PRO_, ST_, gp, tiles_h, tiles_w, nt, 0, 0);                                 \
    else if (nch == 2) R64L(64, PM_, 2, PRO_, ST_, gp, tiles_h, tiles_w, nt, 0, 0);                            \
    else R64L(64, PM_, 4, PRO_, ST_, gp, tiles_h, tiles_w, nt, 0, 0);                                          \
    if (nte) {                                                                                                 \
      if (nch == 1) R64L(16, PM_, 1, PRO_, ST_, gpe, tiles_he, tiles_we, nte, g.Q - rem, gp);                  \
      else if (nch == 2) R64L(16, PM_, 2, PRO_, ST_, gpe, tiles_he, tiles_we, nte, g.Q - rem, gp);             \
      else R64L(16, PM_, 4, PRO_, ST_, gpe, tiles_he, tiles_we, nte, g.Q - rem, gp);                           \
    }                                                                                                          \
  } while (0)
  switch (pm) {
    case 0:
      if (pro) { if (st) R64N(0, true, true); else R64N(0, true, false); }
      else { if (st) R64N(0, false, true); else R64N(0, false, false); }
      break;
    case 4:
      if (pro) R64N(4, true, true); else R64N(4, false, true);
      break;
    case 3:
      if (pro) { if (st) R64N(3, true, true); else R64N(3, true, false); }
      else { if (st) R64N(3, false, true); else R64N(3, false, false); }
      break;
    case 5:
      R64N(5, false, true);
      break;
  }
#undef R64N
#undef R64L
  return launch_rc(what);
}

}  // namespace acfe

ACFE_API int acfe_conv_r64_enable(int on) {
  const int prev = acfe::r64_on() ? 1 : 0;
  acfe::g_r64.store(on ? 1 : 0, std::memory_order_relaxed);
  return prev;
}

#ifdef ACFE_R64_STAMPS
ACFE_API int acfe_debug_r64_stamps(unsigned long long* host, int n) {
  if (n > 4096 * 8) n = 4096 * 8;
  return hip_rc(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_r64_stamps), sizeof(unsigned long long) * n), "stamps");
}
#endif
