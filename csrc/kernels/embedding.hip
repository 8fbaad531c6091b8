// Token (+ learned position) embedding gather and its backward scatter-add
// (SURVEY §2.5 K1), bf16 or f32 storage.  Forward: one wave per token row, 8-element vectors.  Backward:
// f32 atomics straight into the flat f32 gradient buffer, one 256-byte contiguous
// wave-instruction per row segment (the shape that runs at the chip-wide atomic
// rate on gfx950); a [T, D] gradient at D=768 is ~25 MB of adds -> ~20 us.
#include "mp_common.h"

using namespace mp;

template <typename T>
__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ idx, const T* __restrict__ wte,
                                                        const T* __restrict__ wpe, T* __restrict__ out, int T_, int S,
                                                        int D, int pos_offset) {
  using IO = IO8<T>;
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T_) return;
  const int64_t tok = idx[t];
  const int pos = t % S + pos_offset;
  const T* src = wte + (size_t)tok * D;
  const T* psrc = wpe ? wpe + (size_t)pos * D : nullptr;
  T* dst = out + (size_t)t * D;
  for (int c = lane; c < D / 8; c += 64) {
    typename IO::Raw v = IO::load(src + c * 8);
    if (psrc) {
      const typename IO::Raw p = IO::load(psrc + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) IO::set(v, e, IO::get(v, e) + IO::get(p, e));
    }
    IO::store(dst + c * 8, v);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) embed_bwd_kernel(const int64_t* __restrict__ idx, const T* __restrict__ dout,
                                                        float* __restrict__ dwte, float* __restrict__ dwpe, int T_,
                                                        int S, int D, int pos_offset) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T_) return;
  const int64_t tok = idx[t];
  const int pos = t % S + pos_offset;
  const T* g = dout + (size_t)t * D;
  // lane-consecutive columns: each atomic wave-instruction covers 256 contiguous bytes
  for (int c = lane; c < D; c += 64) {
    const float f = IO8<T>::load1(g + c);
    atomicAdd(dwte + (size_t)tok * D + c, f);
    if (dwpe) atomicAdd(dwpe + (size_t)pos * D + c, f);
  }
}

// f32 != 0: wte / wpe / out (resp. dout) in f32 (the reference-precision path), else bf16
extern "C" int mp_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int T, int S, int D,
                            int pos_offset, int f32, hipStream_t st) {
  if (D % 8) return -1;
  if (f32)
    embed_fwd_kernel<float><<<(T + 3) / 4, 256, 0, st>>>(idx, (const float*)wte, (const float*)wpe, (float*)out, T, S,
                                                         D, pos_offset);
  else
    embed_fwd_kernel<bf16_t><<<(T + 3) / 4, 256, 0, st>>>(idx, (const bf16_t*)wte, (const bf16_t*)wpe, (bf16_t*)out, T,
                                                          S, D, pos_offset);
  return (int)hipGetLastError();
}

extern "C" int mp_embed_bwd(const int64_t* idx, const void* dout, float* dwte, float* dwpe, int T, int S, int D,
                            int pos_offset, int f32, hipStream_t st) {
  if (D % 4) return -1;
  if (f32)
    embed_bwd_kernel<float><<<(T + 3) / 4, 256, 0, st>>>(idx, (const float*)dout, dwte, dwpe, T, S, D, pos_offset);
  else
    embed_bwd_kernel<bf16_t><<<(T + 3) / 4, 256, 0, st>>>(idx, (const bf16_t*)dout, dwte, dwpe, T, S, D, pos_offset);
  return (int)hipGetLastError();
}
