// f32 GEMM on the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 products, f32
// accumulate, 64 FLOP/clk/SIMD -- gfx950 has no xf32/TF32 fast path; cdna guide §3
// "FP32-input MFMA").  The matmul of the reference-precision path: the reference trains
// its model in f32 (helper:36-46, no autocast), and NativeModel(dtype=float32) runs every
// linear of it here, forward (bias / bias+ReLU+dropout / residual epilogues), dX (dReLU x
// dropout-mask epilogue) and dW (f32 accumulate into the gradient arena).
//
//   C[M][N] (f32, row stride ldc) = epi(alpha * A B (+ C if accumulate))
//   A(m, k) = A[m * lda + k] (A_KC: K-contiguous) or A[k * lda + m] (M-contiguous)
//   B(k, n) = B[n * ldb + k] (B_KC: K-contiguous) or B[k * ldb + n] (N-contiguous)
//
// Design (f32 MFMA is 16x slower than bf16 per clock, so the operand traffic per MFMA is
// tiny and the kernel is issue-bound on the matrix pipe):
//  * no LDS staging: each lane loads its own fragments straight from L2 into registers.
//    The k index an MFMA lane supplies is free to permute as long as A and B agree, so
//    for 4 consecutive 32x32x2 MFMAs lane half hl supplies k = 8g + 4 hl + j (j = 0..3):
//    a K-contiguous operand is ONE float4 load per lane per 4 MFMAs, an outer-contiguous
//    one four dword loads, each coalesced over 32 lanes;
//  * a 4-deep register ring of those fragments keeps ~1000 cycles of loads in flight;
//  * one wave = one 32x32 output block; a 4-wave workgroup covers 4/KS blocks side by side
//    and splits K over KS waves, reducing the partial sums through LDS -- deterministic
//    split-K without slabs or atomics.  KS is chosen so the grid fills every SIMD
//    (the reference's 1024-token GEMMs have 768-2304 blocks for 1024 SIMDs).
#include "mp_common.h"

using namespace mp;

namespace gf32 {

enum Epi { E_NONE = 0, E_BIAS = 1, E_BIAS_RELU = 2, E_RES = 3, E_BIAS_RES = 4, E_DRELU = 5 };

constexpr int NTH = 256, RING = 4;

template <bool KC>
__device__ __forceinline__ float4 frag(const float* __restrict__ P, int64_t ld, int outer, int k, int n_outer, int K) {
  // 4 consecutive k (k, k+1, k+2, k+3) of row / column `outer`
  if (outer >= n_outer || k >= K) return float4{0.f, 0.f, 0.f, 0.f};
  if constexpr (KC) {
    return *reinterpret_cast<const float4*>(P + (int64_t)outer * ld + k);
  } else {
    const float* p = P + (int64_t)k * ld + outer;
    return float4{p[0], p[ld], p[2 * ld], p[3 * ld]};
  }
}

template <int KS, bool A_KC, bool B_KC, int EPI>
__global__ void __launch_bounds__(NTH) gemm_f32_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                          float* __restrict__ C, const float* __restrict__ bias,
                                                          const float* __restrict__ R, float* __restrict__ X, int M,
                                                          int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                          int64_t ldr, int64_t ldx, float alpha, int accumulate,
                                                          float p_drop, uint64_t seed) {
  constexpr int NBW = 4 / KS;                  // 32x32 blocks per workgroup (along n)
  __shared__ float red[KS > 1 ? (KS - 1) * 16 * 64 : 1];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hl = lane >> 5;
  const int wave = tid >> 6;
  const int blk = wave % NBW, kp = wave / NBW;
  const int gn = (N + 32 * NBW - 1) / (32 * NBW);
  const int m0 = (blockIdx.x / gn) * 32, n0 = (blockIdx.x % gn) * 32 * NBW + 32 * blk;
  // this wave's share of the 8-deep k groups
  const int ng = (K + 7) / 8;
  const int g0 = kp * ng / KS, g1 = (kp + 1) * ng / KS;
  const int arow = m0 + l32, bcol = n0 + l32;

  f32x16 acc = f32x16{};
  float4 ra[RING], rb[RING];
#pragma unroll
  for (int u = 0; u < RING; ++u) {
    const int k = (g0 + u) * 8 + 4 * hl;
    if (g0 + u < g1) {
      ra[u] = frag<A_KC>(A, lda, arow, k, M, K);
      rb[u] = frag<B_KC>(B, ldb, bcol, k, N, K);
    }
  }
  for (int g = g0; g < g1; g += RING) {
#pragma unroll
    for (int u = 0; u < RING; ++u) {
      if (g + u < g1) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u].x, rb[u].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u].y, rb[u].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u].z, rb[u].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u].w, rb[u].w, acc, 0, 0, 0);
        const int gn_ = g + u + RING;
        if (gn_ < g1) {
          const int k = gn_ * 8 + 4 * hl;
          ra[u] = frag<A_KC>(A, lda, arow, k, M, K);
          rb[u] = frag<B_KC>(B, ldb, bcol, k, N, K);
        }
      }
    }
  }
  if constexpr (KS > 1) {
    // partial sums of waves kp > 0 -> LDS; the kp == 0 wave of each block adds them
    if (kp > 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(((kp - 1) * NBW + blk) * 16 + r) * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (kp > 0) return;
#pragma unroll
    for (int q = 1; q < KS; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += red[(((q - 1) * NBW + blk) * 16 + r) * 64 + lane];
  }
  // acc element r -> row m0 + (r & 3) + 8 (r >> 2) + 4 hl, column n0 + l32
  const int col = n0 + l32;
  if (col >= N) return;
  float bv = 0.f;
  if constexpr (EPI == E_BIAS || EPI == E_BIAS_RELU || EPI == E_BIAS_RES) bv = bias[col];
  const float thr_p = p_drop;
  uint32_t thr = 0;
  float inv = 1.f;
  if ((EPI == E_BIAS_RELU || EPI == E_DRELU) && thr_p > 0.f) {
    seed = step_seed(seed);
    thr = drop_thr(thr_p);
    inv = 1.f / (1.f - thr_p);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * hl;
    if (row >= M) continue;
    float* cp = C + (int64_t)row * ldc + col;
    float v = alpha * acc[r];
    if (accumulate) v += *cp;
    if constexpr (EPI == E_BIAS || EPI == E_BIAS_RELU || EPI == E_BIAS_RES) v += bv;
    if constexpr (EPI == E_BIAS_RELU) {
      X[(int64_t)row * ldx + col] = v;            // pre-activation, for the backward
      v = fmaxf(v, 0.f);
      if (thr_p > 0.f) v *= hash_u32(seed, (uint64_t)row * N + col) >= thr ? inv : 0.f;
    }
    if constexpr (EPI == E_DRELU) {
      const float pre = R[(int64_t)row * ldr + col];
      v = pre > 0.f ? v : 0.f;
      if (thr_p > 0.f) v *= hash_u32(seed, (uint64_t)row * N + col) >= thr ? inv : 0.f;
    }
    if constexpr (EPI == E_RES || EPI == E_BIAS_RES) v += R[(int64_t)row * ldr + col];
    *cp = v;
  }
}

template <bool A_KC, bool B_KC, int EPI>
static int launch(int ks, const float* A, const float* B, float* C, const float* bias, const float* R, float* X, int M,
                  int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha,
                  int accumulate, float p_drop, uint64_t seed, hipStream_t st) {
  const int nbw = 4 / ks;
  const int grid = ((M + 31) / 32) * ((N + 32 * nbw - 1) / (32 * nbw));
#define MP_L(KS_)                                                                                             \
  gemm_f32_kernel<KS_, A_KC, B_KC, EPI><<<grid, NTH, 0, st>>>(A, B, C, bias, R, X, M, N, K, lda, ldb, ldc, ldr, \
                                                              ldx, alpha, accumulate, p_drop, seed)
  if (ks == 4) MP_L(4);
  else if (ks == 2) MP_L(2);
  else MP_L(1);
#undef MP_L
  return (int)hipGetLastError();
}

// K split per workgroup: enough waves for ~3 per SIMD (256 CUs x 4 SIMDs), while every
// wave keeps at least 16 k-groups of work
static int pick_ks(int M, int N, int K) {
  const int64_t blocks = (int64_t)((M + 31) / 32) * ((N + 31) / 32);
  const int ng = (K + 7) / 8;
  int ks = 1;
  while (ks < 4 && blocks * ks < 3072 && ng / (ks * 2) >= 16) ks *= 2;
  return ks;
}

}  // namespace gf32

// epi: 0 none, 1 bias, 2 bias+ReLU (+dropout p_drop; pre-activation -> X), 3 residual,
// 4 bias+residual, 5 dReLU (pre-activation in R) x dropout mask.  Dropout element index =
// row * N + col (identical in the forward and the backward).  Returns -1 if the operand
// layouts do not fit (A/B inner stride != 1 / float4 alignment of a K-contiguous operand).
extern "C" int mp_gemm_f32_ex(const float* A, const float* B, float* C, const float* bias, const float* R, float* X,
                              int M, int N, int K, int64_t lda, int a_kc, int64_t ldb, int b_kc, int64_t ldc,
                              int64_t ldr, int64_t ldx, int epi, float alpha, int accumulate, float p_drop,
                              uint64_t seed, int force_ks, hipStream_t st) {
  using namespace gf32;
  if (M <= 0 || N <= 0) return 0;
  if (K % 4) return -1;
  if (a_kc && (lda % 4 || (reinterpret_cast<uintptr_t>(A) & 15))) return -1;
  if (b_kc && (ldb % 4 || (reinterpret_cast<uintptr_t>(B) & 15))) return -1;
  const int ks = force_ks > 0 ? force_ks : pick_ks(M, N, K);
#define MP_E(E)                                                                                                   \
  case E:                                                                                                         \
    if (a_kc && b_kc) return launch<true, true, E>(ks, A, B, C, bias, R, X, M, N, K, lda, ldb, ldc, ldr, ldx,     \
                                                   alpha, accumulate, p_drop, seed, st);                          \
    if (a_kc) return launch<true, false, E>(ks, A, B, C, bias, R, X, M, N, K, lda, ldb, ldc, ldr, ldx, alpha,     \
                                            accumulate, p_drop, seed, st);                                        \
    if (b_kc) return launch<false, true, E>(ks, A, B, C, bias, R, X, M, N, K, lda, ldb, ldc, ldr, ldx, alpha,     \
                                            accumulate, p_drop, seed, st);                                        \
    return launch<false, false, E>(ks, A, B, C, bias, R, X, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, accumulate,  \
                                   p_drop, seed, st);
  switch (epi) {
    MP_E(E_NONE) MP_E(E_BIAS) MP_E(E_BIAS_RELU) MP_E(E_RES) MP_E(E_BIAS_RES) MP_E(E_DRELU)
    default: return -2;
  }
#undef MP_E
}

// the round-2 interface (ops.linear_f32 / f32_linears): B_NC = N-contiguous B
extern "C" int mp_gemm_f32(const float* A, const float* B, float* C, const float* bias, int M, int N, int K,
                           int64_t lda, int a_kc, int64_t ldb, int b_nc, int64_t ldc, float alpha, int accumulate,
                           hipStream_t st) {
  return mp_gemm_f32_ex(A, B, C, bias, nullptr, nullptr, M, N, K, lda, a_kc, ldb, b_nc ? 0 : 1, ldc, 0, 0,
                        bias != nullptr ? gf32::E_BIAS : gf32::E_NONE, alpha, accumulate, 0.f, 0, 0, st);
}

MP_DROP_STEP_SETTER(mp_set_drop_step_gemm_f32)
