// f32 GEMM on the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 products, f32
// accumulate, 64 FLOP/clk/SIMD -- gfx950 has no xf32/TF32 fast path; cdna guide §3
// "FP32-input MFMA").  SURVEY §7.1 gemm_f32.hip: the reference's own workload runs in
// f32 (helper:36-46, no autocast), and this is the matmul of the reference-precision
// path (ops.linear_f32 / ops.f32_linears(): every nn.Linear / MultiheadAttention
// projection of an f32 module, forward and both backward GEMMs).
//
//   C[M][N] (f32, row stride ldc) = alpha * A B (+ bias[N]) (+ C if accumulate)
//   A(m, k) = A[m * lda + k] (A_KC: K-contiguous) or A[k * lda + m] (M-contiguous)
//   B(k, n) = B[k * ldb + n] (B_NC: N-contiguous) or B[n * ldb + k] (K-contiguous)
//
// 128x128 (or, for grids of few tiles, 64x64) tiles, BK = 32, 256 threads (2 x 2 waves).  Both
// operands are staged k-major in LDS ([k][m], [k][n], padded rows), so a 32x32x2 fragment
// read (lane l: row/col base + l % 32, k = kk + l / 32) is one conflict-free ds_read_b32
// per operand.  Global -> register prefetch of K-tile t+1 overlaps the MFMAs of tile t;
// two LDS buffers, one barrier per K-tile.  Grids of few tiles split K (f32 atomics into C).
#include "mp_common.h"

using namespace mp;

namespace gf32 {

constexpr int BK = 32, NTH = 256, PAD = 4;

// T = 128: 2 x 2 waves of 64x64 (2 x 2 MFMA blocks each); T = 64: 2 x 2 waves of 32x32 (one
// block each) -- 4x the workgroups for the short-token shapes without split-K atomics
template <int T, bool A_KC, bool B_NC>
__global__ void __launch_bounds__(NTH, 2) gemm_f32_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                          float* __restrict__ C, const float* __restrict__ bias,
                                                          int M, int N, int K, int64_t lda, int64_t ldb,
                                                          int64_t ldc, float alpha, int accumulate) {
  constexpr int BM = T, BN = T, LDA_S = BM + PAD, LDB_S = BN + PAD;
  constexpr int WT = T / 2, NB = WT / 32;      // wave tile, 32x32 blocks per wave side
  constexpr int U = BM * BK / 4 / NTH;          // float4 per thread per operand tile
  constexpr int CPR = BK / 4;                   // float4 per k-row of a K-contiguous operand row
  constexpr int RPR = BM / 4;                   // float4 per k-row of an outer-contiguous operand
  __shared__ __attribute__((aligned(16))) float As[2][BK][LDA_S];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][LDB_S];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hl = lane >> 5;
  const int wave = tid >> 6, wm = (wave >> 1) * WT, wn = (wave & 1) * WT;
  const int gn = (N + BN - 1) / BN;
  const int m0 = (blockIdx.x / gn) * BM, n0 = (blockIdx.x % gn) * BN;
  // split-K (blockIdx.y of gridDim.y): K-tiles [kt0, kt0 + nk); partial sums are added to C
  // with f32 atomics (C zeroed by the host unless accumulating), the bias by split 0
  const int ktiles = (K + BK - 1) / BK;
  const int nsplit = gridDim.y;
  const int kt0 = (int)blockIdx.y * ktiles / nsplit;
  const int nk = ((int)blockIdx.y + 1) * ktiles / nsplit - kt0;

  float4 ra[U], rb[U];
  auto load = [&](int kt) {
    const int k0 = (kt0 + kt) * BK;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = tid + NTH * u;
      // A
      if constexpr (A_KC) {         // rows m, CPR float4 along k
        const int r = idx / CPR, k = k0 + (idx % CPR) * 4;
        const int m = m0 + r;
        ra[u] = (m < M && k < K) ? *reinterpret_cast<const float4*>(A + (int64_t)m * lda + k) : float4{0, 0, 0, 0};
      } else {                      // k-rows, RPR float4 along m
        const int kr = idx / RPR, m = m0 + (idx % RPR) * 4;
        const int k = k0 + kr;
        ra[u] = (m < M && k < K) ? *reinterpret_cast<const float4*>(A + (int64_t)k * lda + m) : float4{0, 0, 0, 0};
      }
      // B
      if constexpr (B_NC) {         // k-rows, RPR float4 along n
        const int kr = idx / RPR, n = n0 + (idx % RPR) * 4;
        const int k = k0 + kr;
        rb[u] = (n < N && k < K) ? *reinterpret_cast<const float4*>(B + (int64_t)k * ldb + n) : float4{0, 0, 0, 0};
      } else {                      // rows n, CPR float4 along k
        const int r = idx / CPR, k = k0 + (idx % CPR) * 4;
        const int n = n0 + r;
        rb[u] = (n < N && k < K) ? *reinterpret_cast<const float4*>(B + (int64_t)n * ldb + k) : float4{0, 0, 0, 0};
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = tid + NTH * u;
      if constexpr (A_KC) {
        const int r = idx / CPR, kq = (idx % CPR) * 4;
        As[buf][kq + 0][r] = ra[u].x;
        As[buf][kq + 1][r] = ra[u].y;
        As[buf][kq + 2][r] = ra[u].z;
        As[buf][kq + 3][r] = ra[u].w;
      } else {
        *reinterpret_cast<float4*>(&As[buf][idx / RPR][(idx % RPR) * 4]) = ra[u];
      }
      if constexpr (B_NC) {
        *reinterpret_cast<float4*>(&Bs[buf][idx / RPR][(idx % RPR) * 4]) = rb[u];
      } else {
        const int r = idx / CPR, kq = (idx % CPR) * 4;
        Bs[buf][kq + 0][r] = rb[u].x;
        Bs[buf][kq + 1][r] = rb[u].y;
        Bs[buf][kq + 2][r] = rb[u].z;
        Bs[buf][kq + 3][r] = rb[u].w;
      }
    }
  };

  f32x16 acc[NB][NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x16{};

  load(0);
  store(0);
  __syncthreads();
#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    if (t + 1 < nk) load(t + 1);           // in flight during this tile's MFMAs
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[NB], b[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) a[i] = As[buf][kk + hl][wm + 32 * i + l32];
#pragma unroll
      for (int j = 0; j < NB; ++j) b[j] = Bs[buf][kk + hl][wn + 32 * j + l32];
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nk) store(buf ^ 1);        // the other buffer: last read one barrier ago
    __syncthreads();
  }
  // acc[i][j] element r -> row wm + 32 i + (r & 3) + 8 (r >> 2) + 4 hl, column wn + 32 j + l32
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = n0 + wn + 32 * j + l32;
      if (col >= N) continue;
      const float bv = (bias != nullptr && blockIdx.y == 0) ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (row < M) {
          float* cp = C + (int64_t)row * ldc + col;
          const float v = alpha * acc[i][j][r] + bv;
          if (nsplit > 1) atomicAdd(cp, v);
          else *cp = accumulate ? *cp + v : v;
        }
      }
    }
}

}  // namespace gf32

// returns -1 if the operand layouts do not fit (inner stride != 1 / float4 alignment)
extern "C" int mp_gemm_f32(const float* A, const float* B, float* C, const float* bias, int M, int N, int K,
                           int64_t lda, int a_kc, int64_t ldb, int b_nc, int64_t ldc, float alpha, int accumulate,
                           hipStream_t st) {
  using namespace gf32;
  if (M <= 0 || N <= 0) return 0;
  if (K % 4 || M % 4 || N % 4 || lda % 4 || ldb % 4) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -1;
  // 128x128 tiles when they fill the chip four times over; else 64x64 tiles; split-K (f32
  // atomics) while the grid is under 1.5 workgroups per CU and each split keeps >= 4 K-tiles
  const int g128 = ((M + 127) / 128) * ((N + 127) / 128);
  const bool big = g128 >= 1024;
  const int T = big ? 128 : 64;
  const int grid = ((M + T - 1) / T) * ((N + T - 1) / T);
  const int ktiles = (K + BK - 1) / BK;
  int split = 1;
  while (split < 8 && grid * split < 384 && ktiles / (split * 2) >= 4) split *= 2;
  if (split > 1 && !accumulate) {
    const hipError_t e = hipMemset2DAsync(C, (size_t)ldc * sizeof(float), 0, (size_t)N * sizeof(float), M, st);
    if (e != hipSuccess) return (int)e;
  }
#define MP_F32(TT, AK, BNC)                                                                                   \
  gemm_f32_kernel<TT, AK, BNC><<<dim3(grid, split), NTH, 0, st>>>(A, B, C, bias, M, N, K, lda, ldb, ldc, alpha, \
                                                                  accumulate)
  if (big) {
    if (a_kc && b_nc) MP_F32(128, true, true);
    else if (a_kc) MP_F32(128, true, false);
    else if (b_nc) MP_F32(128, false, true);
    else MP_F32(128, false, false);
  } else {
    if (a_kc && b_nc) MP_F32(64, true, true);
    else if (a_kc) MP_F32(64, true, false);
    else if (b_nc) MP_F32(64, false, true);
    else MP_F32(64, false, false);
  }
#undef MP_F32
  return (int)hipGetLastError();
}
