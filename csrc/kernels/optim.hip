// Fused AdamW over the flat parameter arena + global grad-norm.
//
// Every stage keeps its parameters in one flat f32 master buffer (+ a bf16 working
// copy used by the kernels) and its gradients in one flat f32 buffer, so the whole
// optimizer step is two launches: a sum-of-squares reduction for clipping, and one
// streaming AdamW pass that also refreshes the bf16 weights and zeroes the grads
// (no separate zero_grad / cast kernels).  The clip factor is computed on device and
// read by the AdamW kernel from device memory: no host sync.  Weight decay applies
// to elements [0, n_decay) (the arena orders decayed tensors first).
#include "mp_common.h"

using namespace mp;

__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 v = reinterpret_cast<const float4*>(g)[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += g[i] * g[i];
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) atomicAdd(out, acc);
}

// microbatch lanes (parallel/runtime.py): g0 += g1 + g2 + g3 and the lane buffers zeroed
// for the next step, in one pass (a torch add + fill per lane read g0 once per lane and
// took ~10 % of the reference model's 4-lane step)
__global__ void __launch_bounds__(256) lane_merge_kernel(float* __restrict__ g0, float* __restrict__ g1,
                                                         float* __restrict__ g2, float* __restrict__ g3, int64_t n) {
  const int64_t n4 = n / 4;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 a = reinterpret_cast<float4*>(g0)[i];
    float4 b = reinterpret_cast<float4*>(g1)[i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    reinterpret_cast<float4*>(g1)[i] = z;
    if (g2 != nullptr) {
      b = reinterpret_cast<float4*>(g2)[i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      reinterpret_cast<float4*>(g2)[i] = z;
    }
    if (g3 != nullptr) {
      b = reinterpret_cast<float4*>(g3)[i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      reinterpret_cast<float4*>(g3)[i] = z;
    }
    reinterpret_cast<float4*>(g0)[i] = a;
  }
  for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float a = g0[i] + g1[i];
    g1[i] = 0.f;
    if (g2 != nullptr) { a += g2[i]; g2[i] = 0.f; }
    if (g3 != nullptr) { a += g3[i]; g3[i] = 0.f; }
    g0[i] = a;
  }
}

// lane merge + the clipping norm's sum of squares in ONE pass (the optimizer then reads
// the merged g0 once more): g0 = g0 + g1 (+ g2 + g3), lanes zeroed, *sumsq += |g0|^2.  The
// separate sumsq pass re-read the merged buffer (98 us of the reference model's step,
// profiles/r2_end_ref_L8H8_kernel_stats.csv).
__global__ void __launch_bounds__(256) lane_merge_sumsq_kernel(float* __restrict__ g0, float* __restrict__ g1,
                                                               float* __restrict__ g2, float* __restrict__ g3,
                                                               int64_t n, float* __restrict__ sumsq) {
  __shared__ float red[4];
  const int64_t n4 = n / 4;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  float acc = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 a = reinterpret_cast<float4*>(g0)[i];
    float4 b = reinterpret_cast<float4*>(g1)[i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    reinterpret_cast<float4*>(g1)[i] = z;
    if (g2 != nullptr) {
      b = reinterpret_cast<float4*>(g2)[i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      reinterpret_cast<float4*>(g2)[i] = z;
    }
    if (g3 != nullptr) {
      b = reinterpret_cast<float4*>(g3)[i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      reinterpret_cast<float4*>(g3)[i] = z;
    }
    reinterpret_cast<float4*>(g0)[i] = a;
    acc += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
  }
  for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float a = g0[i] + g1[i];
    g1[i] = 0.f;
    if (g2 != nullptr) { a += g2[i]; g2[i] = 0.f; }
    if (g3 != nullptr) { a += g3[i]; g3[i] = 0.f; }
    g0[i] = a;
    acc += a * a;
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) atomicAdd(sumsq, acc);
}

extern "C" int mp_lane_merge(float* g0, float* g1, float* g2, float* g3, int64_t n, float* sumsq, hipStream_t st) {
  if (n <= 0) return 0;
  const int blocks = (int)std::min<int64_t>((n / 4 + 255) / 256 + 1, 8192);
  if (sumsq != nullptr) lane_merge_sumsq_kernel<<<blocks, 256, 0, st>>>(g0, g1, g2, g3, n, sumsq);
  else lane_merge_kernel<<<blocks, 256, 0, st>>>(g0, g1, g2, g3, n);
  return (int)hipGetLastError();
}

// clip: coef = min(1, max_norm / (sqrt(sumsq) + 1e-6)) (if max_norm > 0)
__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, bf16_t* __restrict__ w16, int64_t n,
                                                    int64_t n_decay, float lr, float b1, float b2, float eps, float wd,
                                                    float bc1, float bc2, const float* __restrict__ sumsq,
                                                    float max_norm, float grad_scale, int zero_grad) {
  float coef = grad_scale;
  if (max_norm > 0.f && sumsq != nullptr) {
    const float nrm = sqrtf(*sumsq) * grad_scale;
    coef *= fminf(1.f, max_norm / (nrm + 1e-6f));
  }
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pa = &pp.x; float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
    u16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t idx = i * 4 + e;
      const float gr = ga[e] * coef;
      ma[e] = b1 * ma[e] + (1.f - b1) * gr;
      va[e] = b2 * va[e] + (1.f - b2) * gr * gr;
      const float upd = (ma[e] / bc1) / (sqrtf(va[e] / bc2) + eps);
      const float decay = idx < n_decay ? wd : 0.f;
      pa[e] = pa[e] - lr * (upd + decay * pa[e]);
      o[e] = f2bf(pa[e]);
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (zero_grad) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (w16) reinterpret_cast<u16x4*>(w16)[i] = o;
  }
  for (int64_t idx = n4 * 4 + blockIdx.x * 256 + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * 256) {
    const float gr = g[idx] * coef;
    m[idx] = b1 * m[idx] + (1.f - b1) * gr;
    v[idx] = b2 * v[idx] + (1.f - b2) * gr * gr;
    const float upd = (m[idx] / bc1) / (sqrtf(v[idx] / bc2) + eps);
    const float decay = idx < n_decay ? wd : 0.f;
    p[idx] = p[idx] - lr * (upd + decay * p[idx]);
    if (zero_grad) g[idx] = 0.f;
    if (w16) w16[idx] = f2bf(p[idx]);
  }
}

__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst,
                                                            int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = f2bf(src[i]);
}

static int grid_for(int64_t n) {
  int64_t b = (n / 4 + 255) / 256;
  return (int)(b < 2048 ? (b < 1 ? 1 : b) : 2048);
}

// out[0] = scale * sum(x[0 .. n)) in one workgroup, fixed order (deterministic): the
// microbatch's mean token loss (the row losses of the fused cross-entropy)
__global__ void __launch_bounds__(256) scaled_sum_kernel(const float* __restrict__ x, int64_t n, float scale,
                                                         float* __restrict__ out) {
  __shared__ float part[4];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) acc += x[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = scale * ((part[0] + part[1]) + (part[2] + part[3]));
}

extern "C" int mp_scaled_sum(const float* x, int64_t n, float scale, float* out, hipStream_t st) {
  scaled_sum_kernel<<<1, 256, 0, st>>>(x, n, scale, out);
  return (int)hipGetLastError();
}

extern "C" int mp_sumsq(const float* g, int64_t n, float* out, hipStream_t st) {
  sumsq_kernel<<<grid_for(n), 256, 0, st>>>(g, n, out);
  return (int)hipGetLastError();
}

extern "C" int mp_adamw(float* p, float* g, float* m, float* v, void* w16, int64_t n, int64_t n_decay, float lr,
                        float b1, float b2, float eps, float wd, int step, const float* sumsq, float max_norm,
                        float grad_scale, int zero_grad, hipStream_t st) {
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  adamw_kernel<<<grid_for(n), 256, 0, st>>>(p, g, m, v, (bf16_t*)w16, n, n_decay, lr, b1, b2, eps, wd, bc1, bc2,
                                            sumsq, max_norm, grad_scale, zero_grad);
  return (int)hipGetLastError();
}

extern "C" int mp_cast_f32_bf16(const float* src, void* dst, int64_t n, hipStream_t st) {
  cast_f32_bf16_kernel<<<grid_for(n * 4), 256, 0, st>>>(src, (bf16_t*)dst, n);
  return (int)hipGetLastError();
}
