// Shared helpers for the acfe HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include "../../include/acfe.h"

#define ACFE_API extern "C" __attribute__((visibility("default")))

namespace acfe {

void set_error(hipError_t e, const char* where);

inline int hip_rc(hipError_t e, const char* where) {
  if (e == hipSuccess) return ACFE_OK;
  set_error(e, where);
  return -(int)e;
}

// Check a kernel launch (hipGetLastError) and convert to an ABI code.
inline int launch_rc(const char* where) { return hip_rc(hipGetLastError(), where); }

inline hipStream_t strm(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// ---- bf16 helpers: bit-level, round-to-nearest-even (NaN kept NaN) ----------
__device__ __forceinline__ float bf2f(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  // plain cast lowers to v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN preserving)
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sumd(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Counter-based RNG (splitmix-style hash) for dropout masks: deterministic in
// (seed, index), so the backward regenerates the forward's mask.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  // counter-based 32-bit hash (murmur3 finalizer of a Weyl step): three 32-bit
  // multiplies, cheap enough for the conv epilogue's fused dropout
  uint32_t h = (uint32_t)idx * 0x9E3779B1u + (uint32_t)seed;
  h ^= (uint32_t)(idx >> 32) * 0x85EBCA77u ^ (uint32_t)(seed >> 32);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Rounding to the storage type (the value a separate kernel would have stored).
__device__ __forceinline__ float rnd(float v, uint16_t) { return bf2f(f2bf(v)); }
__device__ __forceinline__ float rnd(float v, float) { return v; }

// Dropout keep test + scale of acfe_dropout (flat element index idx).
struct Drop {
  uint32_t thr;
  float scl;
  unsigned long long seed;
  bool on;
};
// Dropout mask: element idx is kept iff its 16-bit slice of the hash of its
// PAIR, hash(seed, idx >> 1) (low half for even idx, high half for odd), is
// >= rate * 2^16 -- one hash per two elements, so the conv epilogues (whose
// lanes own consecutive channel pairs) pay half the hashing; every kernel that
// applies or regenerates a mask goes through drop_keep*, so they all agree.
__host__ __device__ inline Drop make_drop(float rate, unsigned long long seed) {
  Drop d;
  d.on = rate > 0.f;
  const float t = rate * 65536.0f;  // exact (power-of-two scale)
  d.thr = t >= 65536.0f ? 65536u : (uint32_t)t;
  d.scl = 1.0f / (1.0f - rate);
  d.seed = seed;
  return d;
}
__device__ __forceinline__ bool drop_keep(const Drop& d, uint64_t idx) {
  const uint32_t h = hash_u32(d.seed, idx >> 1);
  return ((idx & 1) ? (h >> 16) : (h & 0xFFFFu)) >= d.thr;
}
template <typename T>
__device__ __forceinline__ float drop_apply(const Drop& d, uint64_t idx, float v) {
  return drop_keep(d, idx) ? rnd(v * d.scl, T()) : 0.f;
}
// The same mask for an index known to be < 2^32 (hash_u32 with idx >> 32 == 0),
// without the 64-bit index arithmetic.
__device__ __forceinline__ uint32_t hash_u32_lo(uint64_t seed, uint32_t idx) {
  uint32_t h = idx * 0x9E3779B1u + (uint32_t)seed;
  h ^= (uint32_t)(seed >> 32);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
// pair hash of an even element index e < 2^32 (elements e and e + 1):
// keep(e) = (h & 0xFFFF) >= thr, keep(e + 1) = (h >> 16) >= thr
__device__ __forceinline__ uint32_t drop_pair_hash32(const Drop& d, uint32_t e) {
  return hash_u32_lo(d.seed, e >> 1);
}
__device__ __forceinline__ uint32_t drop_pair_hash(const Drop& d, uint64_t e) { return hash_u32(d.seed, e >> 1); }
// hash_u32_lo(seed, q) from its Weyl term w = q * 0x9E3779B1 + (uint32)seed
__device__ __forceinline__ uint32_t hash_u32_lo_w(uint64_t seed, uint32_t w) {
  uint32_t x = w ^ (uint32_t)(seed >> 32);
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
// hash_u32_lo of the NP consecutive indices q0 .. q0 + NP - 1: the first
// (Weyl) multiply advances by a constant, so only the first index pays it
// (v_mul_lo_u32 is a quarter-rate instruction; identical values)
template <int NP>
__device__ __forceinline__ void hash_u32_lo_run(uint64_t seed, uint32_t q0, uint32_t (&h)[NP]) {
  const uint32_t b = q0 * 0x9E3779B1u + (uint32_t)seed;
#pragma unroll
  for (int p = 0; p < NP; ++p) h[p] = hash_u32_lo_w(seed, b + (uint32_t)p * 0x9E3779B1u);
}

// Dropout of 8 consecutive elements from the even flat index e0: the 4 pair
// hashes of drop_keep's mask (one hash per element pair instead of per
// element, the 32-bit form when every index is < 2^32 -- i32, uniform -- with
// one Weyl multiply for the four): the hashes' 32-bit multiplies made the
// dropout passes VALU-bound
template <typename T>
__device__ __forceinline__ void drop_apply8(const Drop& d, uint64_t e0, bool i32, float (&v)[8]) {
  uint32_t hl[4];
  if (i32) hash_u32_lo_run<4>(d.seed, (uint32_t)(e0 >> 1), hl);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint64_t e = e0 + 2 * p;
    const uint32_t h = i32 ? hl[p] : hash_u32(d.seed, e >> 1);
    v[2 * p] = (h & 0xFFFFu) >= d.thr ? rnd(v[2 * p] * d.scl, T()) : 0.f;
    v[2 * p + 1] = (h >> 16) >= d.thr ? rnd(v[2 * p + 1] * d.scl, T()) : 0.f;
  }
}
template <typename T>
__device__ __forceinline__ float drop_apply32(const Drop& d, uint32_t idx, float v) {
  const uint32_t h = hash_u32_lo(d.seed, idx >> 1);
  return ((idx & 1) ? (h >> 16) : (h & 0xFFFFu)) >= d.thr ? rnd(v * d.scl, T()) : 0.f;
}

}  // namespace acfe
