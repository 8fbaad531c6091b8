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
//  * the k index an MFMA lane supplies is permuted (lane half hl supplies k = 8g + 4 hl + j
//    for MFMA j of group g; A and B agree): a K-contiguous operand is staged in LDS as
//    rows [row][32 + 4] and one conflict-free ds_read_b128 feeds 4 MFMAs; an outer-
//    contiguous one (dX's weight, both dW operands) keeps its global layout in LDS,
//    [k][64 + 8], read as 4 conflict-free ds_read_b32 -- both are filled by plain float4
//    copies (ds_write_b128), no register transposes;
//  * two register sets and two LDS buffers: pair kp + 2 loads while pair kp + 1 waits in
//    registers and pair kp is in the MFMAs (one barrier per pair; a low-occupancy grid --
//    one workgroup per CU -- still hides the HBM latency);
//  * two accumulator chains per wave (even / odd 8-deep k groups), summed at the end;
//  * few tiles (the reference's 1024-token GEMMs: 192-576 tiles for 256 CUs): split K over
//    workgroups into f32 slabs, summed by one reduce + epilogue pass -- deterministic.
#include <cstdlib>

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

// staging of one operand (rows `outer` 0..63 of the tile, k 0..63 of the K-tile pair):
// 2 float4 per thread, copied as they are -- a K-contiguous operand into the row image
// [kh][outer 64][KS] (fragment = one ds_read_b128 of 4 consecutive k), an outer-contiguous
// one into the column image [kh][k 32][CS] (fragment = 4 ds_read_b32 of one column; CS =
// 72: the two lane halves' rows k and k + 4 land 32 banks apart).  Both images are 2304
// floats per K-tile.  Loads are unconditional from clamped addresses (no branch around a
// load: hipcc would wait for it right there); k past K is zeroed when the registers are
// written to LDS, rows past the edge only feed outputs that are never stored.
constexpr int CS = BT + 8;
static_assert(BK * CS == BT * KS, "row and column images must have the same size");

template <bool KC>
struct Stage {
  float4 r[2];
  uint32_t ok;
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int o0, int n_outer, int k0, int K) {
    const int t = threadIdx.x;
    ok = 0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = t + NTH * u;
      if constexpr (KC) {        // 1024 float4: [kh 2][row 64][c 8]
        const int kh = f >> 9, row = (f >> 3) & 63, c = f & 7;
        const int o = min(o0 + row, n_outer - 1), k = k0 + 32 * kh + 4 * c;
        ok |= (k < K ? 1u : 0u) << u;
        r[u] = *reinterpret_cast<const float4*>(P + (int64_t)o * ld + min(k, K - 4));
      } else {                   // 1024 float4: [kh 2][k 32][c 16]
        const int kh = f >> 9, kk = (f >> 4) & 31, c = f & 15;
        const int o = min(o0 + 4 * c, n_outer - 4), k = k0 + 32 * kh + kk;
        ok |= (k < K ? 1u : 0u) << u;
        r[u] = *reinterpret_cast<const float4*>(P + (int64_t)min(k, K - 1) * ld + o);
      }
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ s) const {
    const int t = threadIdx.x;
    const float4 z = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = t + NTH * u;
      const float4 v = (ok >> u) & 1u ? r[u] : z;
      if constexpr (KC) {
        const int kh = f >> 9, row = (f >> 3) & 63, c = f & 7;
        *reinterpret_cast<float4*>(s + (kh * BT + row) * KS + 4 * c) = v;
      } else {
        const int kh = f >> 9, kk = (f >> 4) & 31, c = f & 15;
        *reinterpret_cast<float4*>(s + (kh * BK + kk) * CS + 4 * c) = v;
      }
    }
  }
  // the lane's 4 operand values (k = 8g + 4hl + j, j = 0..3) of outer index w0 + l32
  static __device__ __forceinline__ float4 frag(const float* __restrict__ s, int w0, int g, int l32, int hl) {
    if constexpr (KC) {
      return *reinterpret_cast<const float4*>(s + (w0 + l32) * KS + 8 * g + 4 * hl);
    } else {
      const float* c = s + (8 * g + 4 * hl) * CS + w0 + l32;
      return float4{c[0], c[CS], c[2 * CS], c[3 * CS]};
    }
  }
};

// one K-tile pair: (issue the loads of pair kp + 2 into the register set that held pair
// kp) -> MFMAs on LDS buffer `buf` -> (registers of pair kp + 1 -> the other buffer) -> barrier
template <bool A_KC, bool B_KC>
__device__ __forceinline__ void pair_step(const Args& p, float* smem, int buf, int kp, int kp1, int m0, int n0,
                                          int kh, int wm, int wn, int l32, int hl, f32x16& acc0, f32x16& acc1,
                                          Stage<A_KC>& ld_a, Stage<B_KC>& ld_b, const Stage<A_KC>& st_a,
                                          const Stage<B_KC>& st_b) {
  // unconditional (past the end: clamped addresses, never stored) -- a load inside a branch
  // leaves hipcc unsure how many are in flight, and it then waits for all of them
  ld_a.load(p.A, p.lda, m0, p.M, (kp + 2) * 2 * BK, p.K);
  ld_b.load(p.B, p.ldb, n0, p.N, (kp + 2) * 2 * BK, p.K);
  const float* As = smem + buf * 2 * OPS + kh * BT * KS;
  const float* Bs = smem + buf * 2 * OPS + OPS + kh * BT * KS;
#pragma unroll
  for (int g = 0; g < BK / 8; ++g) {
    const float4 a = Stage<A_KC>::frag(As, wm, g, l32, hl);
    const float4 b = Stage<B_KC>::frag(Bs, wn, g, l32, hl);
    f32x16& acc = (g & 1) ? acc1 : acc0;     // two independent chains
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
  }
  if (kp + 1 < kp1) {
    float* nb = smem + (buf ^ 1) * 2 * OPS;     // last read before the previous barrier
    st_a.store(nb);
    st_b.store(nb + OPS);
  }
  __syncthreads();
}

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

  // two register sets: pair kp + 2 is loading while pair kp + 1 waits in registers and
  // pair kp is in the MFMAs
  Stage<A_KC> sa0, sa1;
  Stage<B_KC> sb0, sb1;
  f32x16 acc0 = f32x16{}, acc1 = f32x16{};
  if (kp0 < kp1) {
    sa0.load(p.A, p.lda, m0, p.M, kp0 * 2 * BK, p.K);
    sb0.load(p.B, p.ldb, n0, p.N, kp0 * 2 * BK, p.K);
    sa1.load(p.A, p.lda, m0, p.M, (kp0 + 1) * 2 * BK, p.K);
    sb1.load(p.B, p.ldb, n0, p.N, (kp0 + 1) * 2 * BK, p.K);
    sa0.store(smem);
    sb0.store(smem + OPS);
  }
  __syncthreads();
  int kp = kp0;
  for (; kp + 1 < kp1; kp += 2) {
    pair_step<A_KC, B_KC>(p, smem, 0, kp, kp1, m0, n0, kh, wm, wn, l32, hl, acc0, acc1, sa0, sb0, sa1, sb1);
    pair_step<A_KC, B_KC>(p, smem, 1, kp + 1, kp1, m0, n0, kh, wm, wn, l32, hl, acc0, acc1, sa1, sb1, sa0, sb0);
  }
  if (kp < kp1)   // odd count: the last pair
    pair_step<A_KC, B_KC>(p, smem, 0, kp, kp1, m0, n0, kh, wm, wn, l32, hl, acc0, acc1, sa0, sb0, sa1, sb1);
  f32x16 acc = acc0 + acc1;
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

// ---------------------------------------------------------------------------------------
// Stream-K over the 64x64 engine.  The reference's 1024-token GEMMs are 192-576 tiles: at
// split 1 a 192-tile grid leaves 64 of 256 CUs idle, and split-K cannot spread 192 tiles
// evenly either (split 2 = 384 workgroups: half the CUs run two, the makespan is the same).
// Here the grid is G workgroups (one or two per CU) and the tiles x K-pairs work units are
// cut into G equal chunks of c <= 2 npairs consecutive units (k-fastest): a workgroup
// computes the pieces of the (at most SK_SEG) tiles its chunk touches, each into its own
// dense 64x64 partial ws[g][seg] (the same pipeline, kh halves and LDS combine as the tiled
// kernel); one pass sums the partials of every tile in workgroup order (deterministic) and
// applies the epilogue.
// ---------------------------------------------------------------------------------------
constexpr int SK_SEG = 3;

template <bool A_KC, bool B_KC>
__global__ void __launch_bounds__(NTH, 2) gemm_f32_sk_kernel(Args p, int npairs, int chunk) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * OPS];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hl = lane >> 5;
  const int wave = tid >> 6, kh = wave >> 2, wm = ((wave >> 1) & 1) * 32, wn = (wave & 1) * 32;
  const int gn = (p.N + BT - 1) / BT;
  const int tiles = ((p.M + BT - 1) / BT) * gn;
  const int g = blockIdx.x;
  const int units = tiles * npairs;
  int u = g * chunk;
  const int u_end = min(units, u + chunk);
#pragma unroll 1
  for (int seg = 0; seg < SK_SEG && u < u_end; ++seg) {
    const int tile = u / npairs;
    const int kp0 = u - tile * npairs, kp1 = min(npairs, u_end - tile * npairs);
    const int m0 = (tile / gn) * BT, n0 = (tile % gn) * BT;
    Stage<A_KC> sa0, sa1;
    Stage<B_KC> sb0, sb1;
    f32x16 acc0 = f32x16{}, acc1 = f32x16{};
    sa0.load(p.A, p.lda, m0, p.M, kp0 * 2 * BK, p.K);
    sb0.load(p.B, p.ldb, n0, p.N, kp0 * 2 * BK, p.K);
    sa1.load(p.A, p.lda, m0, p.M, (kp0 + 1) * 2 * BK, p.K);
    sb1.load(p.B, p.ldb, n0, p.N, (kp0 + 1) * 2 * BK, p.K);
    sa0.store(smem);
    sb0.store(smem + OPS);
    __syncthreads();
    int kp = kp0;
    for (; kp + 1 < kp1; kp += 2) {
      pair_step<A_KC, B_KC>(p, smem, 0, kp, kp1, m0, n0, kh, wm, wn, l32, hl, acc0, acc1, sa0, sb0, sa1, sb1);
      pair_step<A_KC, B_KC>(p, smem, 1, kp + 1, kp1, m0, n0, kh, wm, wn, l32, hl, acc0, acc1, sa1, sb1, sa0, sb0);
    }
    if (kp < kp1)
      pair_step<A_KC, B_KC>(p, smem, 0, kp, kp1, m0, n0, kh, wm, wn, l32, hl, acc0, acc1, sa0, sb0, sa1, sb1);
    f32x16 acc = acc0 + acc1;
    float* red = smem;
    if (kh == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((wave & 3) * 16 + r) * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (kh == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += red[(wave * 16 + r) * 64 + lane];
      // dense partial tile: local row wm + (r & 3) + 8 (r >> 2) + 4 hl, local col wn + l32
      float* part = p.ws + ((int64_t)g * SK_SEG + seg) * (BT * BT);
#pragma unroll
      for (int r = 0; r < 16; ++r) part[(wm + (r & 3) + 8 * (r >> 2) + 4 * hl) * BT + wn + l32] = acc[r];
    }
    __syncthreads();   // red / the staging buffers are reused by the next segment
    u = (tile + 1) * npairs;
  }
}

// C = epi(sum of the partial tiles that cover each output, in workgroup order), 4 columns
// per thread
template <int EPI>
__global__ void __launch_bounds__(256) reduce_sk_kernel(Args p, int npairs, int chunk) {
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
  const int row = (int)((i4 * 4) / p.N), col = (int)((i4 * 4) % p.N);
  const int gn = (p.N + BT - 1) / BT;
  const int tile = (row / BT) * gn + col / BT;
  const int off = (row % BT) * BT + col % BT;
  const int u0 = tile * npairs, u1 = u0 + npairs;      // this tile's units
  float4 s = float4{0.f, 0.f, 0.f, 0.f};
  for (int g = u0 / chunk; g * chunk < u1; ++g) {
    const int seg = tile - (g * chunk) / npairs;          // this tile's index among g's tiles
    const float4 t = *reinterpret_cast<const float4*>(p.ws + ((int64_t)g * SK_SEG + seg) * (BT * BT) + off);
    s.x += t.x;
    s.y += t.y;
    s.z += t.z;
    s.w += t.w;
  }
  epi_store<EPI>(p, row, col, s.x, thr, inv, seed);
  epi_store<EPI>(p, row, col + 1, s.y, thr, inv, seed);
  epi_store<EPI>(p, row, col + 2, s.z, thr, inv, seed);
  epi_store<EPI>(p, row, col + 3, s.w, thr, inv, seed);
}

template <bool A_KC, bool B_KC, int EPI>
static int launch_sk(Args p, int grid, int npairs, int chunk, hipStream_t st) {
  gemm_f32_sk_kernel<A_KC, B_KC><<<grid, NTH, 0, st>>>(p, npairs, chunk);
  const int64_t n4 = (int64_t)p.M * p.N / 4;
  reduce_sk_kernel<EPI><<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(p, npairs, chunk);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// 128x128 engine (the guide's "128x128x32 block, 2x2 tiles of 32x32 per wave" shape, cdna
// guide §3 'FP32-input MFMA': 122 TF untuned at 4096^3).  Per byte staged it does twice the
// MFMA work of the 64x64 engine (32 vs 16 FLOP/B of operand), and each wave keeps FOUR
// independent 32x32 accumulators (64 AGPRs) -- the f32 MFMA's 64-cycle dependent latency
// equals its issue interval, so 4 chains keep the pipe full from one wave per SIMD:
//  * 256 threads = 4 waves, wave (wr, wc) owns rows 64 wr.., cols 64 wc.. of the tile;
//  * K-tile 32, two LDS buffers (row image [128][36] or column image [32][136] per
//    operand, 18 KiB each); the next K-tile's 4 float4 per thread per operand are loaded
//    into registers while the current one feeds 64 MFMAs per wave, then stored to the
//    other buffer -- one barrier per K-tile;
//  * fragments, k permutation, split-K slabs and epilogue as the 64x64 engine.
constexpr int NTH2 = 256, BT2 = 128, CS2 = BT2 + 8;
constexpr int OPS2 = BT2 * KS;      // 4608 floats >= BK * CS2 = 4352
static_assert(BK * CS2 <= OPS2, "column image must fit the operand slot");

template <bool KC>
struct Stage2 {
  float4 r[4];
  uint32_t ok;
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int o0, int n_outer, int k0, int K) {
    const int t = threadIdx.x;
    ok = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int f = t + NTH2 * u;
      if constexpr (KC) {        // 1024 float4: [row 128][c 8]
        const int row = f >> 3, c = f & 7;
        const int o = min(o0 + row, n_outer - 1), k = k0 + 4 * c;
        ok |= (k < K ? 1u : 0u) << u;
        r[u] = *reinterpret_cast<const float4*>(P + (int64_t)o * ld + min(k, K - 4));
      } else {                   // 1024 float4: [k 32][c 32]
        const int kk = f >> 5, c = f & 31;
        const int o = min(o0 + 4 * c, n_outer - 4), k = k0 + kk;
        ok |= (k < K ? 1u : 0u) << u;
        r[u] = *reinterpret_cast<const float4*>(P + (int64_t)min(k, K - 1) * ld + o);
      }
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ s) const {
    const int t = threadIdx.x;
    const float4 z = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int f = t + NTH2 * u;
      const float4 v = (ok >> u) & 1u ? r[u] : z;
      if constexpr (KC) {
        const int row = f >> 3, c = f & 7;
        *reinterpret_cast<float4*>(s + row * KS + 4 * c) = v;
      } else {
        const int kk = f >> 5, c = f & 31;
        *reinterpret_cast<float4*>(s + kk * CS2 + 4 * c) = v;
      }
    }
  }
  // the lane's 4 operand values (k = 8g + 4hl + j) of outer index w0 + l32
  static __device__ __forceinline__ float4 frag(const float* __restrict__ s, int w0, int g, int l32, int hl) {
    if constexpr (KC) {
      return *reinterpret_cast<const float4*>(s + (w0 + l32) * KS + 8 * g + 4 * hl);
    } else {
      const float* c = s + (8 * g + 4 * hl) * CS2 + w0 + l32;
      return float4{c[0], c[CS2], c[2 * CS2], c[3 * CS2]};
    }
  }
};

template <bool A_KC, bool B_KC, int EPI>
__global__ void __launch_bounds__(NTH2, 2) gemm_f32_big_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * OPS2];   // [buf][A|B][image]
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hl = lane >> 5;
  const int wave = tid >> 6, wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int gn = (p.N + BT2 - 1) / BT2;
  const int tile = blockIdx.x;
  const int m0 = (tile / gn) * BT2, n0 = (tile % gn) * BT2;
  const int nkt = (p.K + BK - 1) / BK;
  const int nsplit = gridDim.y;
  const int kt0 = (int)blockIdx.y * nkt / nsplit, kt1 = ((int)blockIdx.y + 1) * nkt / nsplit;

  Stage2<A_KC> sa;
  Stage2<B_KC> sb;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = f32x16{};
  if (kt0 < kt1) {
    sa.load(p.A, p.lda, m0, p.M, kt0 * BK, p.K);
    sb.load(p.B, p.ldb, n0, p.N, kt0 * BK, p.K);
    sa.store(smem);
    sb.store(smem + OPS2);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {     // next K-tile in flight while this one is in the MFMAs
      sa.load(p.A, p.lda, m0, p.M, (kt + 1) * BK, p.K);
      sb.load(p.B, p.ldb, n0, p.N, (kt + 1) * BK, p.K);
    }
    const float* As = smem + buf * 2 * OPS2;
    const float* Bs = As + OPS2;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      float4 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = Stage2<A_KC>::frag(As, wm + 32 * i, g, l32, hl);
        b[i] = Stage2<B_KC>::frag(Bs, wn + 32 * i, g, l32, hl);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
    }
    if (more) {
      float* nb = smem + (buf ^ 1) * 2 * OPS2;   // last read before the previous barrier
      sa.store(nb);
      sb.store(nb + OPS2);
    }
    __syncthreads();
  }
  uint32_t thr = 0;
  float inv = 1.f;
  uint64_t seed = p.seed;
  if ((EPI == E_BIAS_RELU || EPI == E_DRELU) && p.p_drop > 0.f && p.ws == nullptr) {
    seed = step_seed(seed);
    thr = drop_thr(p.p_drop);
    inv = 1.f / (1.f - p.p_drop);
  }
  float* slab = p.ws != nullptr ? p.ws + (int64_t)blockIdx.y * p.M * p.N : nullptr;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    // acc[i][j] element r -> row m0 + wm + 32 i + (r & 3) + 8 (r >> 2) + 4 hl, col n0 + wn + 32 j + l32
    const int col = n0 + wn + 32 * j + l32;
    if (col >= p.N) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (row >= p.M) continue;
        if (slab != nullptr) slab[(int64_t)row * p.N + col] = acc[i][j][r];
        else epi_store<EPI>(p, row, col, acc[i][j][r], thr, inv, seed);
      }
  }
}

template <bool A_KC, bool B_KC, int EPI>
static int launch_big(Args p, int split, hipStream_t st) {
  const int tiles = ((p.M + BT2 - 1) / BT2) * ((p.N + BT2 - 1) / BT2);
  gemm_f32_big_kernel<A_KC, B_KC, EPI><<<dim3(tiles, split), NTH2, 0, st>>>(p);
  if (split > 1) {
    const int64_t n4 = (int64_t)p.M * p.N / 4;
    reduce_kernel<EPI><<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(p, split);
  }
  return (int)hipGetLastError();
}

// split-K factor: minimise the busiest CU's work, in K-tile-pair units: the workgroups it
// runs (tiles x s over 256 CUs) x (its pairs + ~3 pairs of prologue / epilogue latency),
// plus ~1 for the slab pass.  Fitted to the measured s = 1..8 sweep of the reference's
// GEMMs (profiles/r3_f32_gemm_sweep.json): e.g. dX of the LM head (192 tiles, 157 pairs)
// -> 4, the forward out_proj (192 tiles, 12 pairs) -> 1.
// CUs one GEMM can count on.  With L microbatch lanes replaying concurrently, each lane's
// GEMM shares the chip with the others, so the split is planned for 256 / L CUs: fewer
// slabs and reduce passes, whose only purpose was to fill CUs the other lanes now fill.
// mp_gemm_f32_set_lanes (the runtime's set_lanes) sets it; MIPIPE_F32_CUS overrides it.
static int g_lanes = 1;
static int plan_cus() {
  static const int env = [] {
    const char* e = getenv("MIPIPE_F32_CUS");
    return e ? atoi(e) : 0;
  }();
  if (env > 0) return env;
  const int c = 256 / (g_lanes > 0 ? g_lanes : 1);
  return c < 32 ? 32 : c;
}

static int pick_split(int M, int N, int K) {
  const int tiles = ((M + BT - 1) / BT) * ((N + BT - 1) / BT);
  const int npairs = (K + 2 * BK - 1) / (2 * BK);
  const int cus = plan_cus();
  int best = 1;
  double best_cost = 1e30;
  for (int s = 1; s <= 8; ++s) {
    if (s > 1 && npairs < 2 * s) break;
    const double rounds = (double)((tiles * s + cus - 1) / cus);
    const double cost = rounds * ((double)npairs / s + 3.0) + (s > 1 ? 1.0 : 0.0);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = s;
    }
  }
  return best;
}

// the 128x128 engine's split and cost in the same units as pick_split's (one 64x64 K-tile
// pair = 2 K-tiles of 64x64x32; a 128x128 K-tile is 2 such pairs' MFMA work): rounds of
// 256 CUs x (pairs + fixed latency), with the measured MFMA efficiencies folded in
static int pick_split_big(int M, int N, int K, double* cost_out) {
  const int tiles = ((M + BT2 - 1) / BT2) * ((N + BT2 - 1) / BT2);
  const int nkt = (K + BK - 1) / BK;
  int best = 1;
  double best_cost = 1e30;
  for (int s = 1; s <= 8; ++s) {
    if (s > 1 && nkt < 2 * s) break;
    const double rounds = (double)((tiles * s + 255) / 256);
    const double cost = rounds * (2.0 * nkt / s + 4.0) + (s > 1 ? 1.0 : 0.0);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = s;
    }
  }
  if (cost_out) *cost_out = best_cost;
  return best;
}

// engine + split: MIPIPE_F32_TILE = 64 | 128 | auto.  auto takes the 128x128 engine only
// when its grid fills whole rounds of 2 workgroups per CU (>= 85 % of the last round) --
// measured on the reference's 1024-token shapes (profiles/r4_f32_gemm_sweep_64_vs_128.txt):
// the dW of the LM head (474 tiles) 152 vs 164 us, while every few-tile layer GEMM needs a
// split the 64x64 engine does better (dX of qkv: 48 tiles, 56 us at split 8 vs 47 us)
struct Plan {
  bool big;
  int split;
  int sk_grid, sk_chunk;   // stream-K (64x64 engine): workgroups, units each; 0 = off
};

// stream-K instead of split-K when its busiest CU finishes earlier, in pick_split's units:
// (workgroups per CU) x (chunk + ~3 pairs of pipeline fill per tile piece) + 1 for the
// reduce pass, against rounds x (pairs / s + 3) (+ 1) of the best split.  Opt-in:
// MIPIPE_F32_SK=auto plans it, =1 (or force_split = -2, the tests) forces it wherever the
// chunk fits.  Off by default: +11 % on an isolated few-tile long-K GEMM (fwd linear2, 37.0
// vs 41.5 us) but -1.4 % on the reference's fp32 step (182.6K vs 185.2K tok/s, 2 A/B
// pairs, profiles/r4_f32_stream_k.txt) -- the microbatch lanes already fill the idle CUs
// and the partial-tile pass is extra traffic.
static void plan_sk(int M, int N, int K, Plan& pl, bool force) {
  static const int mode = [] {   // 0 off (default), 1 forced, -1 planned ("auto")
    const char* e = getenv("MIPIPE_F32_SK");
    if (e && e[0] == 'a') return -1;
    return e ? atoi(e) : 0;
  }();
  pl.sk_grid = pl.sk_chunk = 0;
  if ((mode == 0 && !force) || pl.big) return;
  const int tiles = ((M + BT - 1) / BT) * ((N + BT - 1) / BT);
  const int npairs = (K + 2 * BK - 1) / (2 * BK);
  const int units = tiles * npairs;
  const int s = pl.split;
  const double split_cost = (double)((tiles * s + 255) / 256) * ((double)npairs / s + 3.0) + (s > 1 ? 1.0 : 0.0);
  double best = (mode == 1 || force) ? 1e30 : 0.97 * split_cost;
  for (int per_cu = 1; per_cu <= 2; ++per_cu) {
    const int G0 = 256 * per_cu;
    const int c = (units + G0 - 1) / G0;
    if (c < 4 || c > 2 * npairs) continue;
    const double pieces = 1.0 + (double)(c - 1) / npairs;      // tiles a chunk touches, on average
    const double cost = per_cu * (c + 3.0 * pieces) + 1.0;
    if (cost < best) {
      best = cost;
      pl.sk_grid = (units + c - 1) / c;
      pl.sk_chunk = c;
    }
  }
}
static Plan plan(int M, int N, int K, int force_split) {
  static const int mode = [] {
    const char* e = getenv("MIPIPE_F32_TILE");
    if (e && e[0] == '6') return 64;
    if (e && e[0] == '1') return 128;
    return 0;
  }();
  bool big = mode == 128;
  if (mode == 0) {
    const int tiles = ((M + BT2 - 1) / BT2) * ((N + BT2 - 1) / BT2);
    const int rounds = (tiles + 511) / 512;
    big = tiles >= 448 && (double)tiles >= 0.85 * 512.0 * rounds;
  }
  if (force_split == -2) big = false;   // forced stream-K (64x64 engine)
  int split = big ? pick_split_big(M, N, K, nullptr) : pick_split(M, N, K);
  if (big && mode == 0) split = 1;      // a full grid needs no split
  if (force_split > 0) split = force_split;
  Plan pl{big, split, 0, 0};
  if (force_split <= 0) plan_sk(M, N, K, pl, force_split == -2);
  return pl;
}

}  // namespace gf32

// floats of split-K workspace a problem needs (0: no split)
extern "C" int64_t mp_gemm_f32_ws_elems(int M, int N, int K, int force_split) {
  const gf32::Plan pl = gf32::plan(M, N, K, force_split);
  if (M % 4 || N % 4) return 0;
  if (pl.sk_grid > 0) return (int64_t)pl.sk_grid * gf32::SK_SEG * gf32::BT * gf32::BT;
  return pl.split > 1 ? (int64_t)pl.split * M * N : 0;
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
  const Plan pl = plan(M, N, K, force_split);
  int split = pl.split;
  if (ws == nullptr) split = 1;
  const bool sk = pl.sk_grid > 0 && ws != nullptr;
  Args p{A, B, C, bias, R, X, (split > 1 || sk) ? ws : nullptr, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, accumulate,
         p_drop, seed};
  const int npairs = (K + 2 * BK - 1) / (2 * BK);
#define MP_E(E)                                                                                      \
  case E:                                                                                            \
    if (sk) {                                                                                        \
      if (a_kc && b_kc) return launch_sk<true, true, E>(p, pl.sk_grid, npairs, pl.sk_chunk, st);     \
      if (a_kc) return launch_sk<true, false, E>(p, pl.sk_grid, npairs, pl.sk_chunk, st);            \
      if (b_kc) return launch_sk<false, true, E>(p, pl.sk_grid, npairs, pl.sk_chunk, st);            \
      return launch_sk<false, false, E>(p, pl.sk_grid, npairs, pl.sk_chunk, st);                     \
    }                                                                                                \
    if (pl.big) {                                                                                    \
      if (a_kc && b_kc) return launch_big<true, true, E>(p, split, st);                              \
      if (a_kc) return launch_big<true, false, E>(p, split, st);                                     \
      if (b_kc) return launch_big<false, true, E>(p, split, st);                                     \
      return launch_big<false, false, E>(p, split, st);                                              \
    }                                                                                                \
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

// concurrent microbatch lanes the split-K planner assumes (see plan_cus); returns the CUs
// it now plans for
extern "C" int mp_gemm_f32_set_lanes(int lanes) {
  gf32::g_lanes = lanes > 0 ? lanes : 1;
  return gf32::plan_cus();
}
