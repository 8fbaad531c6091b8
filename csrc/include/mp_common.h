// Shared device helpers for the mipipe gfx950 (CDNA4) kernels.
//
// Conventions:
//  * bf16 tensors are moved as raw 16-bit words (uint16_t) in 16-byte vectors
//    (8 x bf16 per lane): hipcc does not vectorise scalar bf16 loads on its own.
//  * f32 <-> bf16: bf16 -> f32 is an exact shift; f32 -> bf16 uses the compiler's
//    cast (lowers to v_cvt_pk_bf16_f32 on gfx950, round-to-nearest-even, NaN-safe).
//  * Wave = 64 lanes.  Reductions use DPP/shuffle over 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define MP_WAVE 64

namespace mp {

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) uint16_t u16x8;
typedef __attribute__((ext_vector_type(4))) uint16_t u16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// 8-element vector I/O for kernels templated on the storage type (bf16 or f32): the
// reference-precision (f32) path runs the same normalisation / loss / embedding kernels as
// the bf16 one.  Raw = the packed registers (16 B of bf16, 32 B of f32).
template <typename T>
struct IO8;
template <>
struct IO8<bf16_t> {
  typedef u16x8 Raw;
  static __device__ __forceinline__ Raw load(const bf16_t* p) { return *reinterpret_cast<const u16x8*>(p); }
  static __device__ __forceinline__ void store(bf16_t* p, const Raw& r) { *reinterpret_cast<u16x8*>(p) = r; }
  static __device__ __forceinline__ float get(const Raw& r, int e) { return __uint_as_float(((uint32_t)r[e]) << 16); }
  static __device__ __forceinline__ void set(Raw& r, int e, float v) {
    __bf16 b = (__bf16)v;
    r[e] = __builtin_bit_cast(uint16_t, b);
  }
  static __device__ __forceinline__ float round(float v) { return get_round(v); }
  static __device__ __forceinline__ float get_round(float v) {
    __bf16 b = (__bf16)v;
    return __uint_as_float(((uint32_t)__builtin_bit_cast(uint16_t, b)) << 16);
  }
  static __device__ __forceinline__ float load1(const bf16_t* p) { return __uint_as_float(((uint32_t)*p) << 16); }
  static __device__ __forceinline__ void store1(bf16_t* p, float v) {
    __bf16 b = (__bf16)v;
    *p = __builtin_bit_cast(uint16_t, b);
  }
};
struct f32x8_raw {
  float4 a, b;
  __device__ __forceinline__ float operator[](int e) const {
    return e < 4 ? (e == 0 ? a.x : e == 1 ? a.y : e == 2 ? a.z : a.w) : (e == 4 ? b.x : e == 5 ? b.y : e == 6 ? b.z : b.w);
  }
};
template <>
struct IO8<float> {
  typedef f32x8_raw Raw;
  static __device__ __forceinline__ Raw load(const float* p) {
    Raw r;
    r.a = reinterpret_cast<const float4*>(p)[0];
    r.b = reinterpret_cast<const float4*>(p)[1];
    return r;
  }
  static __device__ __forceinline__ void store(float* p, const Raw& r) {
    reinterpret_cast<float4*>(p)[0] = r.a;
    reinterpret_cast<float4*>(p)[1] = r.b;
  }
  static __device__ __forceinline__ float get(const Raw& r, int e) { return r[e]; }
  static __device__ __forceinline__ void set(Raw& r, int e, float v) {
    float* f = e < 4 ? &r.a.x : &r.b.x;
    f[e & 3] = v;
  }
  static __device__ __forceinline__ float round(float v) { return v; }
  static __device__ __forceinline__ float load1(const float* p) { return *p; }
  static __device__ __forceinline__ void store1(float* p, float v) { *p = v; }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64).  `red` is >= NT/64 floats of LDS.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (NT == 64) return v;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (NT == 64) return v;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  return t;
}

// Counter-based RNG, deterministic in (seed, index) so dropout masks are regenerated in
// the backward pass instead of stored.  32-bit arithmetic only: two keys from the seed and
// the index's high word (the attention kernels put (b, h) there and compute the keys once,
// `drop_key`), the low word through the "lowbias32" integer finaliser (two v_mul_lo_u32 +
// three xorshifts) with the second key xored in mid-way, so streams whose inputs overlap
// after the additive offset still differ.  The round-1 64-bit splitmix chain (emulated
// 64-bit multiplies per element) made the dropout attention kernels run 1.8-2.7x their
// dropout-free form and pushed them into register spills.
// Per-stream keys (scalar work: seed and the index's high word are wave-uniform).
struct DropKey {
  uint32_t k0, k1;
};
__device__ __forceinline__ DropKey drop_key(uint64_t seed, uint32_t hi) {
  DropKey k;
  k.k0 = ((uint32_t)seed ^ 0x9E3779B9u) + hi * 0x85EBCA6Bu;
  k.k1 = ((uint32_t)(seed >> 32) ^ hi) * 0xC2B2AE35u + 0x27D4EB2Fu;
  return k;
}
__device__ __forceinline__ uint32_t hash_lo(DropKey k, uint32_t lo) {
  uint32_t x = lo + k.k0;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= k.k1;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  return hash_lo(drop_key(seed, (uint32_t)(idx >> 32)), (uint32_t)idx);
}
// keep threshold / scale of a drop probability, hoisted out of element loops
__device__ __forceinline__ uint32_t drop_thr(float p) { return (uint32_t)(p * 4294967296.0f); }
__device__ __forceinline__ float drop_scale_lo(DropKey k, uint32_t lo, uint32_t thr, float inv) {
  return hash_lo(k, lo) >= thr ? inv : 0.0f;
}

// Graph-safe dropout: every kernel that drops mixes a per-process training-step counter
// into its seed on entry.  The counter lives in device memory (one copy per translation
// unit, written by a 1-thread kernel before each step, outside any captured graph), so a
// HIP graph captured once draws a fresh mask every replay while the forward and the
// backward of one step still agree.
static __device__ uint64_t mp_drop_step;
__device__ __forceinline__ uint64_t step_seed(uint64_t seed) {
  return seed ^ (mp_drop_step * 0xA24BAED4963EE407ull + 0x2545F4914F6CDD1Dull);
}
#define MP_DROP_STEP_SETTER(NAME)                                                     \
  __global__ void NAME##_kernel(uint64_t v) { mp_drop_step = v; }                    \
  extern "C" int NAME(uint64_t v, hipStream_t st) {                                  \
    NAME##_kernel<<<1, 1, 0, st>>>(v);                                               \
    return (int)hipGetLastError();                                                   \
  }

// keep with probability (1-p): returns scale (1/(1-p)) or 0
__device__ __forceinline__ float dropout_scale(uint64_t seed, uint64_t idx, float p) {
  const uint32_t thr = (uint32_t)(p * 4294967296.0f);
  return hash_u32(seed, idx) >= thr ? 1.0f / (1.0f - p) : 0.0f;
}

// tanh-GELU through one v_exp_f32 + one v_rcp_f32 (0.5(1+tanh u) = sigmoid(2u));
// libm tanhf is a long branchy sequence and dominated the GEMM epilogues.
__device__ __forceinline__ float sigmoid_fast(float z) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * z));
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return x * sigmoid_fast(2.0f * u);
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u = k0 * (x + k1 * x2 * x);
  const float sg = sigmoid_fast(2.0f * u);  // = 0.5(1 + tanh u)
  // d/dx [x sg(2u)] = sg + x * 2 sg (1 - sg) * u'
  return sg + 2.0f * x * sg * (1.0f - sg) * k0 * (1.0f + 3.0f * k1 * x2);
}

// GELU and its derivative from one sigmoid: the forward GEMM epilogue saves the derivative
// (bf16) for the backward, whose dX epilogue is then a plain multiply (no exp / rcp there)
__device__ __forceinline__ void gelu_tanh_and_grad(float x, float& g, float& d) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u = k0 * (x + k1 * x2 * x);
  const float sg = sigmoid_fast(2.0f * u);
  g = x * sg;
  d = sg + 2.0f * x * sg * (1.0f - sg) * k0 * (1.0f + 3.0f * k1 * x2);
}

// max of three as ONE v_max3_f32.  fmaxf makes the compiler canonicalise each input first
// (an extra v_max_f32 x, x, x per value under IEEE mode: 32 per attention tile, ~2 per logit
// in the fused CE); the values here are never signalling NaNs (MI355X_MICROARCH.md)
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

}  // namespace mp
