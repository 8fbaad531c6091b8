// Fused softmax cross-entropy, forward + backward in one kernel.
//
// One 256-thread block per token row of the [T, Vp] bf16 logits:
//   pass 1: online max / sum-exp over the row (16-byte loads), block-reduced;
//   pass 2: dlogits = (softmax - onehot(target)) * grad_scale written IN PLACE over
//           the logits (the row is L2-resident from pass 1), so the [T, V] logits are
//           never re-read by a separate backward kernel and no second buffer exists.
// Columns >= V (vocab padded to a multiple of 64 for the GEMMs, e.g. GPT-2's 50257
// -> 50304) are excluded from the softmax and get zero gradient.  Targets equal to
// ignore_index produce zero loss and zero gradient.
#include <cstdlib>

#include "mp_common.h"

using namespace mp;

template <bool WRITE_GRAD, typename LT = bf16_t>
__global__ void __launch_bounds__(256) xent_kernel(LT* __restrict__ logits, const int64_t* __restrict__ target,
                                                   float* __restrict__ loss, int T, int V, int Vp, float grad_scale,
                                                   int64_t ignore_index) {
  using IO = IO8<LT>;
  __shared__ float red[8];
  const int row = blockIdx.x;
  LT* x = logits + (size_t)row * Vp;
  const int64_t tgt = target[row];
  const int nvec = V >> 3;  // full 8-wide chunks inside the real vocab
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < nvec; c += 256) {
    const typename IO::Raw v = IO::load(x + c * 8);
    float f[8];
    float lm = m;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      f[e] = IO::get(v, e);
      lm = fmaxf(lm, f[e]);
    }
    s *= __expf(m - lm);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += __expf(f[e] - lm);
    m = lm;
  }
  for (int j = nvec * 8 + threadIdx.x; j < V; j += 256) {
    float f = IO::load1(x + j);
    float lm = fmaxf(m, f);
    s = s * __expf(m - lm) + __expf(f - lm);
    m = lm;
  }
  const float gm = block_max<256>(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  __syncthreads();
  const float gs = block_sum<256>(s, red);
  const float lse = gm + __logf(gs);
  const bool valid = tgt != ignore_index && tgt >= 0 && tgt < V;
  if (threadIdx.x == 0) loss[row] = valid ? lse - IO::load1(x + tgt) : 0.f;
  if (!WRITE_GRAD) return;
  __syncthreads();  // everyone has read x[tgt] before it is overwritten
  const float sc = valid ? grad_scale : 0.f;
  const int nvec_p = Vp >> 3;
  for (int c = threadIdx.x; c < nvec_p; c += 256) {
    const typename IO::Raw v = IO::load(x + c * 8);
    typename IO::Raw o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = c * 8 + e;
      float g = 0.f;
      if (j < V) g = (__expf(IO::get(v, e) - lse) - (j == tgt ? 1.f : 0.f)) * sc;
      IO::set(o, e, g);
    }
    IO::store(x + c * 8, o);
  }
}

// Register-resident variant: 512 threads hold the whole row (CPT 16-byte chunks each), so
// the logits are read from HBM exactly once and the gradient written once; exp2 with
// log2(e) folded into one fma.
// opaque to the optimizer: keeps the row as packed bf16 words between passes instead of
// 8x as many live unpacked floats (which capped the kernel at 1 row in flight per CU)
template <int CPT>
__device__ __forceinline__ void keep_packed(u16x8 (&v)[CPT]) {
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    uint4 w = __builtin_bit_cast(uint4, v[i]);
    asm volatile("" : "+v"(w.x), "+v"(w.y), "+v"(w.z), "+v"(w.w));
    v[i] = __builtin_bit_cast(u16x8, w);
  }
}

// MINB: blocks per CU to fit (waves per SIMD = MINB x NTH / 256)
template <int CPT, bool WRITE_GRAD, int NTH = 512, int MINB = 1>
__global__ void __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(MINB * NTH / 256, 8))) xent_reg_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ target,
                                                       float* __restrict__ loss, int T, int V, int Vp,
                                                       float grad_scale, int64_t ignore_index) {
  __shared__ float red[16];
  constexpr float L2E = 1.4426950408889634f;
  const int row = blockIdx.x;
  bf16_t* x = logits + (size_t)row * Vp;
  const int64_t tgt = target[row];
  const int nchunk = Vp >> 3;
  const int nfull = V >> 3;  // chunks entirely inside the real vocabulary: no per-element checks
  u16x8 v[CPT];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + NTH * i;
    if (c < nchunk) v[i] = *reinterpret_cast<const u16x8*>(x + c * 8);
  }
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + NTH * i;
    if (c < nfull) {
#pragma unroll
      for (int e = 0; e < 8; ++e) m = fmaxf(m, bf2f(v[i][e]));
    } else if (c < nchunk) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c * 8 + e < V) m = fmaxf(m, bf2f(v[i][e]));
    }
  }
  keep_packed<CPT>(v);
  const float gm = block_max<NTH>(m, red);
  const float mc = gm * L2E;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + NTH * i;
    if (c < nfull) {
#pragma unroll
      for (int e = 0; e < 8; ++e) s += __builtin_amdgcn_exp2f(__builtin_fmaf(bf2f(v[i][e]), L2E, -mc));
    } else if (c < nchunk) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c * 8 + e < V) s += __builtin_amdgcn_exp2f(__builtin_fmaf(bf2f(v[i][e]), L2E, -mc));
    }
  }
  keep_packed<CPT>(v);
  __syncthreads();
  const float gs = block_sum<NTH>(s, red);
  const float lse = gm + __logf(gs);
  const bool valid = tgt != ignore_index && tgt >= 0 && tgt < V;
  if (threadIdx.x == 0) loss[row] = valid ? lse - bf2f(x[tgt]) : 0.f;
  if (!WRITE_GRAD) return;
  __syncthreads();  // x[tgt] read before it is overwritten
  const float sc = valid ? grad_scale : 0.f;
  const float lc = lse * L2E;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + NTH * i;
    if (c < nfull) {
      u16x8 o;
      const int te = tgt - 8 * c;   // target's slot in this chunk (usually out of range)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o[e] = f2bf((__builtin_amdgcn_exp2f(__builtin_fmaf(bf2f(v[i][e]), L2E, -lc)) - (e == te ? 1.f : 0.f)) * sc);
      *reinterpret_cast<u16x8*>(x + c * 8) = o;
    } else if (c < nchunk) {
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = c * 8 + e;
        float g = 0.f;
        if (j < V) g = (__builtin_amdgcn_exp2f(__builtin_fmaf(bf2f(v[i][e]), L2E, -lc)) - (j == tgt ? 1.f : 0.f)) * sc;
        o[e] = f2bf(g);
      }
      *reinterpret_cast<u16x8*>(x + c * 8) = o;
    }
  }
}

extern "C" int mp_xent_fwd_bwd(void* logits, const int64_t* target, float* loss, int T, int V, int Vp,
                               float grad_scale, int64_t ignore_index, int write_grad, int f32, hipStream_t st) {
  if (Vp % 8 != 0 || V > Vp) return -1;
  if (f32) {   // f32 logits (reference-precision path): the streaming two-pass kernel
    if (write_grad)
      xent_kernel<true, float><<<T, 256, 0, st>>>((float*)logits, target, loss, T, V, Vp, grad_scale, ignore_index);
    else
      xent_kernel<false, float><<<T, 256, 0, st>>>((float*)logits, target, loss, T, V, Vp, grad_scale, ignore_index);
    return (int)hipGetLastError();
  }
  const int nchunk = Vp / 8;
  // MIPIPE_XENT=occ3 | t1024: occupancy variants of the register-resident kernel (A/B)
  static const int variant = [] {
    const char* e = getenv("MIPIPE_XENT");
    if (e && e[0] == 'o') return 1;
    if (e && e[0] == 't') return 2;
    return 0;
  }();
  if (variant == 1 && nchunk <= 512 * 13) {   // 3 blocks of 512 threads per CU
    if (write_grad)
      xent_reg_kernel<13, true, 512, 3><<<T, 512, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale,
                                                           ignore_index);
    else
      xent_reg_kernel<13, false, 512, 3><<<T, 512, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale,
                                                            ignore_index);
    return (int)hipGetLastError();
  }
  if (variant == 2 && nchunk <= 1024 * 7) {   // 1024 threads, 7 chunks each
    if (write_grad)
      xent_reg_kernel<7, true, 1024, 2><<<T, 1024, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale,
                                                         ignore_index);
    else
      xent_reg_kernel<7, false, 1024, 2><<<T, 1024, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale,
                                                          ignore_index);
    return (int)hipGetLastError();
  }
#define MP_XR(CPT)                                                                                               \
  if (nchunk <= 512 * CPT) {                                                                                     \
    if (write_grad)                                                                                              \
      xent_reg_kernel<CPT, true><<<T, 512, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale,          \
                                                    ignore_index);                                              \
    else                                                                                                         \
      xent_reg_kernel<CPT, false><<<T, 512, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale,         \
                                                     ignore_index);                                             \
    return (int)hipGetLastError();                                                                               \
  }
  MP_XR(4) MP_XR(13) MP_XR(16)
#undef MP_XR
  if (nchunk <= 1024 * 16) {  // large vocabularies (Llama-3: 128256): 1024 threads, 16 chunks each
    if (write_grad)
      xent_reg_kernel<16, true, 1024><<<T, 1024, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale,
                                                         ignore_index);
    else
      xent_reg_kernel<16, false, 1024><<<T, 1024, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale,
                                                          ignore_index);
    return (int)hipGetLastError();
  }
  if (write_grad)
    xent_kernel<true><<<T, 256, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale, ignore_index);
  else
    xent_kernel<false><<<T, 256, 0, st>>>((bf16_t*)logits, target, loss, T, V, Vp, grad_scale, ignore_index);
  return (int)hipGetLastError();
}
