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
// Design.  f32 MFMA runs at 1/16 of the bf16 rate, so a 64x64 workgroup tile makes the
// kernel matrix-pipe-bound provided operands come from LDS (a one-wave-per-block design
// that loads its fragments straight from L2 -- the round-3 first cut -- tops out at half
// of peak on the vector-memory path: every wave re-fetches its 32 rows per MFMA group):
//  * 64x64 tiles, 8 waves: waves 0-3 own the even 32-deep K-tiles, waves 4-7 the odd ones
//    (a 32x32 block each, 2x2 over the tile), so two K-tiles are in flight per workgroup
//    and a SIMD holds 2 waves of it; the two halves are summed through LDS at the end;
//  * operands staged in LDS as K-contiguous rows [row][32 + 4]: one ds_read_b128 gives a
//    lane 4 consecutive k, which feed 4 MFMAs -- the k index a lane supplies is permuted
//    (lane half hl supplies k = 8g + 4 hl + j for MFMA j of group g; A and B agree), so the
//    LDS reads are conflict-free b128 and there is no per-k shuffling;
//  * a K-contiguous global operand is copied with float4 loads / ds_write_b128; an
//    outer-contiguous one (dX's weight, both dW operands) is loaded as 4x4 blocks (4
//    float4 along the outer dim) and transposed in registers on the way into LDS;
//  * the next pair of K-tiles is loaded into registers during the current pair's MFMAs
//    (two LDS buffers, one barrier per pair);
//  * few tiles (the reference's 1024-token GEMMs: 192-576 tiles for 256 CUs): split K over
//    workgroups into f32 slabs, summed by one reduce + epilogue pass -- deterministic.
#include "mp_common.h"

using namespace mp;

namespace gf32 {

enum Epi { E_NONE = 0, E_BIAS = 1, E_BIAS_RELU = 2, E_RES = 3, E_BIAS_RES = 4, E_DRELU = 5 };

constexpr int NTH = 512, BT = 64, BK = 32, KS = BK + 4;   // tile, K-tile, LDS row stride
constexpr int OPS = 2 * BT * KS;                          // one operand, both K halves (floats)

struct Args {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  const float* R;
  float* X;
  float* ws;        // split-K slabs [split][M][N] (null: no split)
  int M, N, K;
  int64_t lda, ldb, ldc, ldr, ldx;
  float alpha;
  int accumulate;
  float p_drop;
  uint64_t seed;
};

// epilogue of one element (row, col) with accumulator value a
template <int EPI>
__device__ __forceinline__ void epi_store(const Args& p, int row, int col, float a, uint32_t thr, float inv,
                                          uint64_t seed) {
  float* cp = p.C + (int64_t)row * p.ldc + col;
  float v = p.alpha * a;
  if (p.accumulate) v += *cp;
  if constexpr (EPI == E_BIAS || EPI == E_BIAS_RELU || EPI == E_BIAS_RES) v += p.bias[col];
  if constexpr (EPI == E_BIAS_RELU) {
    p.X[(int64_t)row * p.ldx + col] = v;            // pre-activation, for the backward
    v = fmaxf(v, 0.f);
    if (thr) v *= hash_u32(seed, (uint64_t)row * p.N + col) >= thr ? inv : 0.f;
  }
  if constexpr (EPI == E_DRELU) {
    const float pre = p.R[(int64_t)row * p.ldr + col];
    v = pre > 0.f ? v : 0.f;
    if (thr) v *= hash_u32(seed, (uint64_t)row * p.N + col) >= thr ? inv : 0.f;
  }
  if constexpr (EPI == E_RES || EPI == E_BIAS_RES) v += p.R[(int64_t)row * p.ldr + col];
  *cp = v;
}

// staging of one operand (rows `outer` 0..63 of the tile, k 0..63 of the K-tile pair) via
// registers: K-contiguous -> 2 float4 per thread; outer-contiguous -> a 4x4 block (4
// float4) for each thread of the operand's half of the workgroup (`half` 0: threads 0-255)
template <bool KC>
struct Stage {
  float4 r[KC ? 2 : 4];
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int o0, int n_outer, int k0, int K,
                                       int half) {
    const int t = threadIdx.x;
    if constexpr (KC) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int f = t + NTH * u;                  // 1024 float4: [kh 2][row 64][c 8]
        const int kh = f >> 9, row = (f >> 3) & 63, c = f & 7;
        const int o = o0 + row, k = k0 + 32 * kh + 4 * c;
        r[u] = (o < n_outer && k < K) ? *reinterpret_cast<const float4*>(P + (int64_t)o * ld + k)
                                      : float4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      const int tt = t - 256 * half;
      if (tt < 0 || tt >= 256) return;
      const int kh = tt >> 7, q = tt & 127, kq = q >> 4, oq = q & 15;   // [kh 2][kq 8][oq 16]
      const int o = o0 + 4 * oq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + 32 * kh + 4 * kq + i;
        r[i] = (o < n_outer && k < K) ? *reinterpret_cast<const float4*>(P + (int64_t)k * ld + o)
                                      : float4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  // -> LDS image [kh][row][KS] (k-contiguous rows)
  __device__ __forceinline__ void store(float* __restrict__ s, int half) const {
    const int t = threadIdx.x;
    if constexpr (KC) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int f = t + NTH * u;
        const int kh = f >> 9, row = (f >> 3) & 63, c = f & 7;
        *reinterpret_cast<float4*>(s + (kh * BT + row) * KS + 4 * c) = r[u];
      }
    } else {
      const int tt = t - 256 * half;
      if (tt < 0 || tt >= 256) return;
      const int kh = tt >> 7, q = tt & 127, kq = q >> 4, oq = q & 15;
      // row 4 oq + j gets k 4 kq .. 4 kq + 3: column j of the 4x4 block
      float* d = s + (kh * BT + 4 * oq) * KS + 4 * kq;
      *reinterpret_cast<float4*>(d) = float4{r[0].x, r[1].x, r[2].x, r[3].x};
      *reinterpret_cast<float4*>(d + KS) = float4{r[0].y, r[1].y, r[2].y, r[3].y};
      *reinterpret_cast<float4*>(d + 2 * KS) = float4{r[0].z, r[1].z, r[2].z, r[3].z};
      *reinterpret_cast<float4*>(d + 3 * KS) = float4{r[0].w, r[1].w, r[2].w, r[3].w};
    }
  }
};

template <bool A_KC, bool B_KC, int EPI>
__global__ void __launch_bounds__(NTH, 2) gemm_f32_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * OPS];   // [buf][A|B][kh][row][KS]
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hl = lane >> 5;
  const int wave = tid >> 6, kh = wave >> 2, wm = ((wave >> 1) & 1) * 32, wn = (wave & 1) * 32;
  const int gn = (p.N + BT - 1) / BT;
  const int tile = blockIdx.x;
  const int m0 = (tile / gn) * BT, n0 = (tile % gn) * BT;
  // split-K over workgroups: K-tile pairs [kp0, kp1) of this split
  const int npairs = (p.K + 2 * BK - 1) / (2 * BK);
  const int nsplit = gridDim.y;
  const int kp0 = (int)blockIdx.y * npairs / nsplit, kp1 = ((int)blockIdx.y + 1) * npairs / nsplit;

  Stage<A_KC> sa;
  Stage<B_KC> sb;
  f32x16 acc = f32x16{};
  if (kp0 < kp1) {
    sa.load(p.A, p.lda, m0, p.M, kp0 * 2 * BK, p.K, 0);
    sb.load(p.B, p.ldb, n0, p.N, kp0 * 2 * BK, p.K, 1);
    sa.store(smem, 0);
    sb.store(smem + OPS, 1);
  }
  __syncthreads();
  for (int kp = kp0; kp < kp1; ++kp) {
    const int buf = (kp - kp0) & 1;
    const float* As = smem + buf * 2 * OPS + kh * BT * KS;
    const float* Bs = smem + buf * 2 * OPS + OPS + kh * BT * KS;
    const bool more = kp + 1 < kp1;
    if (more) {   // the next pair in flight during this pair's MFMAs
      sa.load(p.A, p.lda, m0, p.M, (kp + 1) * 2 * BK, p.K, 0);
      sb.load(p.B, p.ldb, n0, p.N, (kp + 1) * 2 * BK, p.K, 1);
    }
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const float4 a = *reinterpret_cast<const float4*>(As + (wm + l32) * KS + 8 * g + 4 * hl);
      const float4 b = *reinterpret_cast<const float4*>(Bs + (wn + l32) * KS + 8 * g + 4 * hl);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
    }
    if (more) {
      float* nb = smem + (buf ^ 1) * 2 * OPS;     // last read before the previous barrier
      sa.store(nb, 0);
      sb.store(nb + OPS, 1);
    }
    __syncthreads();
  }
  // the odd-K-tile waves hand their sums to the even ones through LDS
  float* red = smem;
  if (kh == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((wave & 3) * 16 + r) * 64 + lane] = acc[r];
  }
  __syncthreads();
  if (kh == 1) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] += red[(wave * 16 + r) * 64 + lane];
  // acc element r -> row m0 + wm + (r & 3) + 8 (r >> 2) + 4 hl, column n0 + wn + l32
  const int col = n0 + wn + l32;
  if (col >= p.N) return;
  if (p.ws != nullptr) {   // split-K: this split's partial sums -> its slab
    float* slab = p.ws + (int64_t)blockIdx.y * p.M * p.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * hl;
      if (row < p.M) slab[(int64_t)row * p.N + col] = acc[r];
    }
    return;
  }
  uint32_t thr = 0;
  float inv = 1.f;
  uint64_t seed = p.seed;
  if ((EPI == E_BIAS_RELU || EPI == E_DRELU) && p.p_drop > 0.f) {
    seed = step_seed(seed);
    thr = drop_thr(p.p_drop);
    inv = 1.f / (1.f - p.p_drop);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * hl;
    if (row < p.M) epi_store<EPI>(p, row, col, acc[r], thr, inv, seed);
  }
}

// sum of the split-K slabs + the epilogue, 4 columns per thread
template <int EPI>
__global__ void __launch_bounds__(256) reduce_kernel(Args p, int nsplit) {
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)p.M * p.N;
  if (i4 * 4 >= total) return;
  uint32_t thr = 0;
  float inv = 1.f;
  uint64_t seed = p.seed;
  if ((EPI == E_BIAS_RELU || EPI == E_DRELU) && p.p_drop > 0.f) {
    seed = step_seed(seed);
    thr = drop_thr(p.p_drop);
    inv = 1.f / (1.f - p.p_drop);
  }
  float4 s = reinterpret_cast<const float4*>(p.ws)[i4];
  for (int q = 1; q < nsplit; ++q) {
    const float4 t = reinterpret_cast<const float4*>(p.ws + (int64_t)q * total)[i4];
    s.x += t.x;
    s.y += t.y;
    s.z += t.z;
    s.w += t.w;
  }
  const int row = (int)((i4 * 4) / p.N), col = (int)((i4 * 4) % p.N);
  epi_store<EPI>(p, row, col, s.x, thr, inv, seed);
  epi_store<EPI>(p, row, col + 1, s.y, thr, inv, seed);
  epi_store<EPI>(p, row, col + 2, s.z, thr, inv, seed);
  epi_store<EPI>(p, row, col + 3, s.w, thr, inv, seed);
}

template <bool A_KC, bool B_KC, int EPI>
static int launch(Args p, int split, hipStream_t st) {
  const int tiles = ((p.M + BT - 1) / BT) * ((p.N + BT - 1) / BT);
  gemm_f32_kernel<A_KC, B_KC, EPI><<<dim3(tiles, split), NTH, 0, st>>>(p);
  if (split > 1) {
    const int64_t n4 = (int64_t)p.M * p.N / 4;
    reduce_kernel<EPI><<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(p, split);
  }
  return (int)hipGetLastError();
}

// split-K factor: fill the 512 workgroup slots (256 CUs x 2) in as few, as full rounds as
// possible, each split keeping at least 4 K-tile pairs (256 k)
static int pick_split(int M, int N, int K) {
  const int tiles = ((M + BT - 1) / BT) * ((N + BT - 1) / BT);
  const int npairs = (K + 2 * BK - 1) / (2 * BK);
  int best = 1;
  double best_eff = 0.0;
  for (int s = 1; s <= 8; ++s) {
    if (s > 1 && npairs / s < 4) break;
    const int wg = tiles * s;
    const int rounds = (wg + 511) / 512;
    // useful fraction of the slots, with a small price per split for the slab pass
    const double eff = (double)wg / (rounds * 512.0) / (1.0 + 0.04 * (s - 1));
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = s;
    }
  }
  return best;
}

}  // namespace gf32

// floats of split-K workspace a problem needs (0: no split)
extern "C" int64_t mp_gemm_f32_ws_elems(int M, int N, int K, int force_split) {
  const int s = force_split > 0 ? force_split : gf32::pick_split(M, N, K);
  return (s > 1 && M % 4 == 0 && N % 4 == 0) ? (int64_t)s * M * N : 0;
}

// epi: 0 none, 1 bias, 2 bias+ReLU (+dropout p_drop; pre-activation -> X), 3 residual,
// 4 bias+residual, 5 dReLU (pre-activation in R) x dropout mask.  Dropout element index =
// row * N + col (identical in the forward and the backward).  ws: the split-K workspace
// (mp_gemm_f32_ws_elems floats; null: no split).  Returns -1 if the operand layouts do not
// fit the float4 loads (M, N, K, lda, ldb multiples of 4; 16-byte aligned A, B).
extern "C" int mp_gemm_f32_ex(const float* A, const float* B, float* C, const float* bias, const float* R, float* X,
                              int M, int N, int K, int64_t lda, int a_kc, int64_t ldb, int b_kc, int64_t ldc,
                              int64_t ldr, int64_t ldx, int epi, float alpha, int accumulate, float p_drop,
                              uint64_t seed, int force_split, float* ws, hipStream_t st) {
  using namespace gf32;
  if (M <= 0 || N <= 0) return 0;
  if (K % 4 || M % 4 || N % 4 || lda % 4 || ldb % 4) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -1;
  int split = force_split > 0 ? force_split : pick_split(M, N, K);
  if (ws == nullptr) split = 1;
  Args p{A, B, C, bias, R, X, split > 1 ? ws : nullptr, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, accumulate,
         p_drop, seed};
#define MP_E(E)                                                                                      \
  case E:                                                                                            \
    if (a_kc && b_kc) return launch<true, true, E>(p, split, st);                                    \
    if (a_kc) return launch<true, false, E>(p, split, st);                                           \
    if (b_kc) return launch<false, true, E>(p, split, st);                                           \
    return launch<false, false, E>(p, split, st);
  switch (epi) {
    MP_E(E_NONE) MP_E(E_BIAS) MP_E(E_BIAS_RELU) MP_E(E_RES) MP_E(E_BIAS_RES) MP_E(E_DRELU)
    default: return -2;
  }
#undef MP_E
}

// the round-2 interface (ops.linear_f32 / f32_linears): B_NC = N-contiguous B; no split-K
extern "C" int mp_gemm_f32(const float* A, const float* B, float* C, const float* bias, int M, int N, int K,
                           int64_t lda, int a_kc, int64_t ldb, int b_nc, int64_t ldc, float alpha, int accumulate,
                           hipStream_t st) {
  return mp_gemm_f32_ex(A, B, C, bias, nullptr, nullptr, M, N, K, lda, a_kc, ldb, b_nc ? 0 : 1, ldc, 0, 0,
                        bias != nullptr ? gf32::E_BIAS : gf32::E_NONE, alpha, accumulate, 0.f, 0, 1, nullptr, st);
}

MP_DROP_STEP_SETTER(mp_set_drop_step_gemm_f32)
