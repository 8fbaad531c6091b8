// Token (+ learned position) embedding gather and its backward scatter-add
// (SURVEY §2.5 K1).  Forward: one wave per token row, 16-byte vectors.  Backward:
// f32 atomics straight into the flat f32 gradient buffer, one 256-byte contiguous
// wave-instruction per row segment (the shape that runs at the chip-wide atomic
// rate on gfx950); a [T, D] gradient at D=768 is ~25 MB of adds -> ~20 us.
#include "mp_common.h"

using namespace mp;

__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ idx, const bf16_t* __restrict__ wte,
                                                        const bf16_t* __restrict__ wpe, bf16_t* __restrict__ out, int T,
                                                        int S, int D, int pos_offset) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int64_t tok = idx[t];
  const int pos = t % S + pos_offset;
  const bf16_t* src = wte + (size_t)tok * D;
  const bf16_t* psrc = wpe ? wpe + (size_t)pos * D : nullptr;
  bf16_t* dst = out + (size_t)t * D;
  for (int c = lane; c < D / 8; c += 64) {
    u16x8 v = *reinterpret_cast<const u16x8*>(src + c * 8);
    if (psrc) {
      u16x8 p = *reinterpret_cast<const u16x8*>(psrc + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(p[e]));
    }
    *reinterpret_cast<u16x8*>(dst + c * 8) = v;
  }
}

__global__ void __launch_bounds__(256) embed_bwd_kernel(const int64_t* __restrict__ idx, const bf16_t* __restrict__ dout,
                                                        float* __restrict__ dwte, float* __restrict__ dwpe, int T, int S,
                                                        int D, int pos_offset) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int64_t tok = idx[t];
  const int pos = t % S + pos_offset;
  const bf16_t* g = dout + (size_t)t * D;
  // lane-consecutive columns: each atomic wave-instruction covers 256 contiguous bytes
  for (int c = lane; c < D; c += 64) {
    const float f = bf2f(g[c]);
    atomicAdd(dwte + (size_t)tok * D + c, f);
    if (dwpe) atomicAdd(dwpe + (size_t)pos * D + c, f);
  }
}

extern "C" int mp_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int T, int S, int D,
                            int pos_offset, hipStream_t st) {
  if (D % 8) return -1;
  embed_fwd_kernel<<<(T + 3) / 4, 256, 0, st>>>(idx, (const bf16_t*)wte, (const bf16_t*)wpe, (bf16_t*)out, T, S, D,
                                                pos_offset);
  return (int)hipGetLastError();
}

extern "C" int mp_embed_bwd(const int64_t* idx, const void* dout, float* dwte, float* dwpe, int T, int S, int D,
                            int pos_offset, hipStream_t st) {
  if (D % 4) return -1;
  embed_bwd_kernel<<<(T + 3) / 4, 256, 0, st>>>(idx, (const bf16_t*)dout, dwte, dwpe, T, S, D, pos_offset);
  return (int)hipGetLastError();
}
