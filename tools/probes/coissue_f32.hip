// Does the f32 MFMA pipe run concurrently with f32 VALU (v_pk_fma_f32) issued by the other
// wave of the same SIMD?  Register-only chains, equal FLOPs per wave in every mode:
//   mode 0: all 8 waves MFMA (v_mfma_f32_32x32x2_f32, 4 independent accumulators)
//   mode 1: all 8 waves VALU (64 independent float2 FMA chains -> v_pk_fma_f32)
//   mode 2: waves 0-3 MFMA, waves 4-7 VALU (one of each per SIMD)
// If the pipes overlap, mode 2 takes ~half of mode 0 / mode 1.
// hipcc --offload-arch=gfx950 -O3 -o coissue coissue_f32.hip && ./coissue
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) float f32x2;

__global__ void __launch_bounds__(512) coissue(float* out, int iters, int mode) {
  const int wave = threadIdx.x >> 6;
  const bool mf = mode == 0 || (mode == 2 && wave < 4);
  float r = 0.f;
  if (mf) {
    f32x16 acc[4];
    for (int j = 0; j < 4; ++j) acc[j] = f32x16{};
    const float a = 1e-3f * (threadIdx.x & 63), b = 0.999f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
    }
    for (int j = 0; j < 4; ++j)
      for (int e = 0; e < 16; ++e) r += acc[j][e];
  } else {
    f32x2 x[64];
    for (int j = 0; j < 64; ++j) x[j] = f32x2{1e-3f * j, 2e-3f * j};
    const f32x2 m = {0.999f, 0.998f}, c = {1e-4f, 2e-4f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 64; ++j) x[j] = __builtin_elementwise_fma(x[j], m, c);
    }
    for (int j = 0; j < 64; ++j) r += x[j][0] + x[j][1];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  const int blocks = 256 * 4, iters = 2000;
  float* out;
  hipMalloc(&out, (size_t)blocks * 512 * sizeof(float));
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  // FLOPs per wave per iteration: 4 MFMA x 32*32*2*2 = 16384 = 64 pk_fma x 64 lanes x 4
  const double flop = (double)blocks * 8 * iters * 16384.0;
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 3; ++mode) {
      coissue<<<blocks, 512>>>(out, 10, mode);
      hipEventRecord(s);
      coissue<<<blocks, 512>>>(out, iters, mode);
      hipEventRecord(e);
      hipEventSynchronize(e);
      float ms = 0.f;
      hipEventElapsedTime(&ms, s, e);
      printf("rep %d mode %d (%s): %.3f ms  %.1f TF\n", rep, mode, mode == 0 ? "mfma" : mode == 1 ? "valu" : "mfma||valu",
             ms, flop / (ms * 1e-3) / 1e12);
    }
  }
  hipFree(out);
  return 0;
}
