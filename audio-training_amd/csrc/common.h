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
inline Drop make_drop(float rate, unsigned long long seed) {
  Drop d;
  d.on = rate > 0.f;
  const float t = rate * 4294967296.0f;  // exact (power-of-two scale); saturate like v_cvt_u32_f32
  d.thr = t >= 4294967296.0f ? 0xFFFFFFFFu : (uint32_t)t;
  d.scl = 1.0f / (1.0f - rate);
  d.seed = seed;
  return d;
}
template <typename T>
__device__ __forceinline__ float drop_apply(const Drop& d, uint64_t idx, float v) {
  return hash_u32(d.seed, idx) >= d.thr ? rnd(v * d.scl, T()) : 0.f;
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
template <typename T>
__device__ __forceinline__ float drop_apply32(const Drop& d, uint32_t idx, float v) {
  return hash_u32_lo(d.seed, idx) >= d.thr ? rnd(v * d.scl, T()) : 0.f;
}

}  // namespace acfe
