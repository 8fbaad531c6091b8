// f32 flash attention, forward and backward, on the f32-input MFMA (v_mfma_f32_32x32x2_f32:
// exact f32 products, f32 accumulate).  The attention core of the reference-precision path:
// the reference's nn.TransformerDecoderLayer runs math SDPA in f32 (SURVEY §2.5 K4:
// non-causal self- and cross-attention, d_h = 64 / 96 / 192, dropout 0.1 on the
// probabilities, helper:52).  Same interface, dropout hash and log2-unit LSE as the bf16
// kernels (attention.hip), so ops.attn_fwd / attn_bwd dispatch on the dtype.
//
// Fragment algebra (one wave = 32 rows; lane = (l32, hl = lane >> 5)):
//  * 32x32x2 MFMA operands: lane supplies A[m = l32][k slot hl], B[k slot hl][n = l32];
//    C/D element r of lane -> (row m = (r&3) + 8(r>>2) + 4 hl, column n = l32).
//  * the k index is permuted freely (A and B agree): for 4 consecutive MFMAs j = 0..3 of a
//    group g, k slot hl means k = 8g + 4 hl + j -- so a k-contiguous row gives a lane its 4
//    values with ONE 16-byte load, and the C element r = 4g + j of an accumulator is
//    exactly the k = 8g + 4hl + j that the next MFMA's B operand needs from this lane.
//  * forward / dQ: S^T = K Q^T (A = K rows, B = the lane's own Q row) puts the query on
//    the LANE, the keys on the registers: the softmax row statistics are per lane, and P^T
//    (registers) is directly the B operand of O^T = V^T P^T.  Output O^T: query on the lane.
//  * dK / dV: S = Q K^T (A = Q rows, B = the lane's own K row) puts the KEY on the lane;
//    dV^T = dO^T P and dK^T = Q^T dS take P / dS straight from registers.
//
// Work decomposition.  f32 MFMA runs at 1/16 of the bf16 rate, so at the reference's
// shape (B 8, S 128, 4-12 heads: 32-96 (b, h) pairs) one wave per 32 rows looping over
// all 128 columns leaves most of the 1024 SIMDs idle and each wave 4 blocks deep.  Here a
// workgroup owns ONE 32-row block and its 8 waves split the work two ways: the loop
// dimension (keys for the forward and dQ, queries for dK/dV) round-robin over 4 wave
// pairs, and d_h in halves within a pair -- each wave computes S (and dP) over its half of
// d_h, the pair adds the halves through LDS, and each then produces its half of the
// output columns.  The loop partials are combined through LDS at the end (forward: with
// the per-way softmax statistics; backward: a plain sum -- deterministic).  Grid = 32-row
// blocks x (b, h), 2 waves per SIMD; at S = 128 every wave pair does one block, and
// d_h = 192 needs no separate dK / dV passes.  Operand fragments are loaded straight from global
// (L2-resident rows; 16-byte row chunks for A/B rows, 128-byte coalesced column slices for
// the transposed A operands) -- no LDS staging, so LDS holds only the combine buffers.
// H == Hkv only (the reference has no GQA).
#include "mp_common.h"

using namespace mp;

namespace af32 {

// 8 waves: wave w = (pw = w & 3: which loop blocks, hf = w >> 2: which half of d_h)
constexpr int NTH = 512, RB = 32, NW = 4, CS = RB + 1;   // combine buffer row stride (floats)
constexpr float L2E = 1.4426950408889634f;

template <int D>
struct Sz {
  static constexpr int NB = D / 32, NG = D / 8;
  static constexpr int NGH = NG / 2;            // 8-deep k groups of one d_h half
  static constexpr int NBH = (NB + 1) / 2;      // 32-wide output column blocks per half
  static_assert(NG % 2 == 0, "d_h must be a multiple of 16");
};

__device__ __forceinline__ f32x16 mfma4(float4 a, float4 b, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ int crow(int r, int hl) { return (r & 3) + 8 * (r >> 2) + 4 * hl; }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// A operand of a transposed product (X^T . Y, X token-major [rows][D]): lane (l32 = column
// `col`, hl) supplies X[r0 + 4hl + j][col], j = 0..3; rows clamped to `rows - 1` (their B
// operand is zero)
__device__ __forceinline__ float4 ld_t(const float* __restrict__ x, int64_t stride, int r0, int rows, int col) {
  const int hl = (threadIdx.x >> 5) & 1;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = x[(int64_t)min(r0 + 4 * hl + j, rows - 1) * stride + col];
  return float4{v[0], v[1], v[2], v[3]};
}

// the two d_h halves of a block's S (and dP) are computed by waves w and w ^ 4: each adds
// the other's partial through LDS (xb: [2 parity][8 waves][NA][16][64] floats)
template <int NA>
__device__ __forceinline__ void exchange(float* __restrict__ xb, int it, f32x16 (&v)[NA]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* mine = xb + ((it & 1) * 8 + w) * NA * 16 * 64;
  const float* other = xb + ((it & 1) * 8 + (w ^ 4)) * NA * 16 * 64;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) mine[(a * 16 + r) * 64 + lane] = v[a][r];
  __syncthreads();   // (the other parity's buffer is rewritten only after the next barrier)
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[a][r] += other[(a * 16 + r) * 64 + lane];
}

// acc[i] = output columns 32 (hf NBH + i) + crow(r) of this wave's rows (lane l32) ->
// the combine slice buf[pw][D][CS]
template <int D>
__device__ __forceinline__ void put_partial(float* __restrict__ buf, const f32x16 (&acc)[Sz<D>::NBH]) {
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5, w = threadIdx.x >> 6;
  float* o = buf + (w & 3) * D * CS;
#pragma unroll
  for (int i = 0; i < Sz<D>::NBH; ++i) {
    const int nb = (w >> 2) * Sz<D>::NBH + i;
    if (nb < Sz<D>::NB) {
#pragma unroll
      for (int r = 0; r < 16; ++r) o[(32 * nb + crow(r, hl)) * CS + l32] = acc[i][r];
    }
  }
}

// sum of the 4 loop-block partials (optionally weighted per row by wt[pw][row]) * scale ->
// token-major rows r0 .. r0 + 31 of `out` (coalesced along d)
template <int D, bool WEIGHTED>
__device__ __forceinline__ void combine_store(const float* __restrict__ buf, const float* __restrict__ wt,
                                              float* __restrict__ out, int64_t stride, int r0, int rows,
                                              float scale) {
  for (int i = threadIdx.x; i < RB * D; i += NTH) {
    const int row = i / D, d = i % D;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float x = buf[(w * D + d) * CS + row];
      acc += WEIGHTED ? x * wt[w * RB + row] : x;
    }
    if (r0 + row < rows) out[(int64_t)(r0 + row) * stride + d] = acc * scale;
  }
}

template <int D, int NA>
struct Lds {
  static constexpr int X = 2 * 8 * NA * 16 * 64;   // exchange buffers
  static constexpr int C = NW * D * CS;            // combine buffers
  static constexpr int N = X > C ? X : C;
};

// ----------------------------------------------------------------------------------- forward
// One workgroup = 32 queries; loop blocks = 32-key blocks (wave pw takes pw, pw + 4, ...).
template <int D, bool DROP>
__global__ void __launch_bounds__(NTH, 1) fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                     const float* __restrict__ v, float* __restrict__ o,
                                                     float* __restrict__ lse, int B, int Sq, int Sk, int H,
                                                     int64_t qs, int64_t ks, int64_t vs, int64_t os, float scale,
                                                     float p_drop, uint64_t seed) {
  using Z = Sz<D>;
  __shared__ __attribute__((aligned(16))) float smem[Lds<D, 1>::N + 3 * NW * RB];
  float* Ms = smem + Lds<D, 1>::N;   // per loop-way row max / row sum / combine weight
  float* Ls = Ms + NW * RB;
  float* Ws = Ls + NW * RB;
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5, w = threadIdx.x >> 6;
  const int pw = w & 3, hf = w >> 2;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int q0 = blockIdx.x * RB;
  const int qi = q0 + l32;
  const float c = scale * L2E;
  const int dof = hf * (D / 2) + 4 * hl;   // this wave's d_h half, lane-half offset
  // the lane's query row (this half), pre-scaled into log2 units
  float4 qf[Z::NGH];
  {
    const float* qp = q + (int64_t)(b * Sq + min(qi, Sq - 1)) * qs + h * D + dof;
#pragma unroll
    for (int g = 0; g < Z::NGH; ++g) {
      const float4 t = ld4(qp + 8 * g);
      qf[g] = float4{t.x * c, t.y * c, t.z * c, t.w * c};
    }
  }
  DropKey dk{0u, 0u};
  uint32_t thr = 0;
  float inv = 1.f;
  if constexpr (DROP) {
    dk = drop_key(step_seed(seed), (uint32_t)bh);
    thr = drop_thr(p_drop);
    inv = 1.f / (1.f - p_drop);
  }
  f32x16 acc[Z::NBH];
#pragma unroll
  for (int i = 0; i < Z::NBH; ++i) acc[i] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;
  const float* kb = k + (int64_t)b * Sk * ks + h * D;
  const float* vb = v + (int64_t)b * Sk * vs + h * D;
  const int iters = (Sk + NW * RB - 1) / (NW * RB);
  for (int it = 0; it < iters; ++it) {   // same trip count in every wave (barriers inside)
    const int k0 = RB * (NW * it + pw);
    // S^T block (half of d_h): keys on registers (row crow), queries on lanes
    const float* kr = kb + (int64_t)min(k0 + l32, Sk - 1) * ks + dof;
    f32x16 s[1] = {f32x16{}};
#pragma unroll
    for (int g = 0; g < Z::NGH; ++g) s[0] = mfma4(ld4(kr + 8 * g), qf[g], s[0]);
    exchange<1>(smem, it, s);
    float mb = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (k0 + crow(r, hl) >= Sk) s[0][r] = -INFINITY;
      mb = fmaxf(mb, s[0][r]);
    }
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    const float m_new = fmaxf(m_run, mb);
    const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = m_new == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[0][r] - m_new);
      ls += p;
      float pd = p;
      if constexpr (DROP)
        pd = hash_lo(dk, (uint32_t)qi * (uint32_t)Sk + (uint32_t)(k0 + crow(r, hl))) >= thr ? p * inv : 0.f;
      s[0][r] = pd;
    }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
    if (k0 < Sk) {   // O^T (this half's column blocks) += V^T P^T
#pragma unroll
      for (int i = 0; i < Z::NBH; ++i) {
        const int nb = hf * Z::NBH + i;
        if (nb < Z::NB) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][r] *= alpha;
#pragma unroll
          for (int g = 0; g < 4; ++g)
            acc[i] = mfma4(ld_t(vb, vs, k0 + 8 * g, Sk, 32 * nb + l32),
                           float4{s[0][4 * g], s[0][4 * g + 1], s[0][4 * g + 2], s[0][4 * g + 3]}, acc[i]);
        }
      }
    }
  }
  // combine the 4 loop ways' (m, l, O^T): weight = 2^(m_w - m) / l
  __syncthreads();   // exchange buffers -> combine buffers
  put_partial<D>(smem, acc);
  if (hl == 0 && hf == 0) {
    Ms[pw * RB + l32] = m_run;
    Ls[pw * RB + l32] = l_run;
  }
  __syncthreads();
  if (threadIdx.x < RB) {
    const int row = threadIdx.x;
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < NW; ++i) m = fmaxf(m, Ms[i * RB + row]);
    float l = 0.f, e[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      e[i] = Ms[i * RB + row] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(Ms[i * RB + row] - m);
      l += Ls[i * RB + row] * e[i];
    }
    const float il = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) Ws[i * RB + row] = e[i] * il;
    if (q0 + row < Sq) lse[(int64_t)bh * Sq + q0 + row] = m + __log2f(l);
  }
  __syncthreads();
  combine_store<D, true>(smem, Ws, o + (int64_t)b * Sq * os + h * D, os, q0, Sq, 1.f);
}

// delta[bh][i] = sum_d dO[i][d] O[i][d]  (one wave per query row)
__global__ void __launch_bounds__(256) delta_kernel(const float* __restrict__ o, const float* __restrict__ dout,
                                                    float* __restrict__ delta, int B, int Sq, int H, int D,
                                                    int64_t os, int64_t dos) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);   // (b, i, h) flattened as (b*Sq + i)*H + h
  if (row >= B * Sq * H) return;
  const int h = row % H, bi = row / H;
  const float* op = o + (int64_t)bi * os + h * D;
  const float* dp = dout + (int64_t)bi * dos + h * D;
  float acc = 0.f;
  for (int d = lane; d < D; d += 64) acc += op[d] * dp[d];
  acc = wave_sum(acc);
  const int b = bi / Sq, i = bi % Sq;
  if (lane == 0) delta[(int64_t)(b * H + h) * Sq + i] = acc;
}

// ----------------------------------------------------------------------------- dK, dV
// One workgroup = 32 keys; loop blocks = 32-query blocks.
template <int D, bool DROP>
__global__ void __launch_bounds__(NTH, 1) dkv_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                     const float* __restrict__ v, const float* __restrict__ dout,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     float* __restrict__ dk_out, float* __restrict__ dv_out, int B,
                                                     int Sq, int Sk, int H, int64_t qs, int64_t ks, int64_t vs,
                                                     int64_t dos, int64_t dks, int64_t dvs, float scale, float p_drop,
                                                     uint64_t seed) {
  using Z = Sz<D>;
  __shared__ __attribute__((aligned(16))) float smem[Lds<D, 2>::N];
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5, w = threadIdx.x >> 6;
  const int pw = w & 3, hf = w >> 2;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int kbase = blockIdx.x * RB;
  const int kj = kbase + l32;
  const float c = scale * L2E;
  const int dof = hf * (D / 2) + 4 * hl;
  // the lane's key / value rows (this half of d_h), re-read from L1/L2 per loop block:
  // kept in registers beside the two accumulator sets they spill at d_h >= 96
  const float* kp = k + (int64_t)(b * Sk + min(kj, Sk - 1)) * ks + h * D + dof;
  const float* vp = v + (int64_t)(b * Sk + min(kj, Sk - 1)) * vs + h * D + dof;
  DropKey dkey{0u, 0u};
  uint32_t thr = 0;
  float inv = 1.f;
  if constexpr (DROP) {
    dkey = drop_key(step_seed(seed), (uint32_t)bh);
    thr = drop_thr(p_drop);
    inv = 1.f / (1.f - p_drop);
  }
  f32x16 adk[Z::NBH], adv[Z::NBH];
#pragma unroll
  for (int i = 0; i < Z::NBH; ++i) adk[i] = adv[i] = f32x16{};
  const float* qb = q + (int64_t)b * Sq * qs + h * D;
  const float* db = dout + (int64_t)b * Sq * dos + h * D;
  const float* lb = lse + (int64_t)bh * Sq;
  const float* deb = delta + (int64_t)bh * Sq;
  const int iters = (Sq + NW * RB - 1) / (NW * RB);
  for (int it = 0; it < iters; ++it) {
    const int q0 = RB * (NW * it + pw);
    // S and dP (half of d_h) with queries on registers (row crow), keys on lanes
    const int qr = min(q0 + l32, Sq - 1);
    const float* qp = qb + (int64_t)qr * qs + dof;
    const float* dp_ = db + (int64_t)qr * dos + dof;
    int zero = 0;
    asm volatile("" : "+v"(zero));   // keeps the K / V row loads inside the loop
    f32x16 sd[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int g = 0; g < Z::NGH; ++g) {
      sd[0] = mfma4(ld4(qp + 8 * g), ld4(kp + zero + 8 * g), sd[0]);
      sd[1] = mfma4(ld4(dp_ + 8 * g), ld4(vp + zero + 8 * g), sd[1]);
    }
    exchange<2>(smem, it, sd);
    if (q0 >= Sq) continue;   // (after the barrier: every wave reaches every exchange)
    float pz[16], ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = q0 + crow(r, hl);
      const bool ok = kj < Sk && qi < Sq;
      const int qc = min(qi, Sq - 1);
      const float p = ok ? __builtin_amdgcn_exp2f(sd[0][r] * c - lb[qc]) : 0.f;
      float z = 1.f;
      if constexpr (DROP) z = hash_lo(dkey, (uint32_t)qi * (uint32_t)Sk + (uint32_t)kj) >= thr ? inv : 0.f;
      pz[r] = p * z;
      ds[r] = p * (sd[1][r] * z - deb[qc]);
    }
    // dV^T += dO^T (P z),  dK^T += Q^T dS  (this half's column blocks)
#pragma unroll
    for (int i = 0; i < Z::NBH; ++i) {
      const int nb = hf * Z::NBH + i;
      if (nb < Z::NB) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          adv[i] = mfma4(ld_t(db, dos, q0 + 8 * g, Sq, 32 * nb + l32),
                         float4{pz[4 * g], pz[4 * g + 1], pz[4 * g + 2], pz[4 * g + 3]}, adv[i]);
          adk[i] = mfma4(ld_t(qb, qs, q0 + 8 * g, Sq, 32 * nb + l32),
                         float4{ds[4 * g], ds[4 * g + 1], ds[4 * g + 2], ds[4 * g + 3]}, adk[i]);
        }
      }
    }
  }
  __syncthreads();
  put_partial<D>(smem, adv);
  __syncthreads();
  combine_store<D, false>(smem, nullptr, dv_out + (int64_t)b * Sk * dvs + h * D, dvs, kbase, Sk, 1.f);
  __syncthreads();
  put_partial<D>(smem, adk);
  __syncthreads();
  combine_store<D, false>(smem, nullptr, dk_out + (int64_t)b * Sk * dks + h * D, dks, kbase, Sk, scale);
}

// --------------------------------------------------------------------------------- dQ
// One workgroup = 32 queries; loop blocks = 32-key blocks.
template <int D, bool DROP>
__global__ void __launch_bounds__(NTH, 1) dq_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                    const float* __restrict__ v, const float* __restrict__ dout,
                                                    const float* __restrict__ lse, const float* __restrict__ delta,
                                                    float* __restrict__ dq_out, int B, int Sq, int Sk, int H,
                                                    int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dqs,
                                                    float scale, float p_drop, uint64_t seed) {
  using Z = Sz<D>;
  __shared__ __attribute__((aligned(16))) float smem[Lds<D, 2>::N];
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5, w = threadIdx.x >> 6;
  const int pw = w & 3, hf = w >> 2;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int q0 = blockIdx.x * RB;
  const int qi = q0 + l32;
  const float c = scale * L2E;
  const int dof = hf * (D / 2) + 4 * hl;
  float4 qf[Z::NGH], df[Z::NGH];
  {
    const int qr = min(qi, Sq - 1);
    const float* qp = q + (int64_t)(b * Sq + qr) * qs + h * D + dof;
    const float* dp = dout + (int64_t)(b * Sq + qr) * dos + h * D + dof;
#pragma unroll
    for (int g = 0; g < Z::NGH; ++g) {
      qf[g] = ld4(qp + 8 * g);
      df[g] = ld4(dp + 8 * g);
    }
  }
  const float lq = qi < Sq ? lse[(int64_t)bh * Sq + qi] : INFINITY;
  const float dl = qi < Sq ? delta[(int64_t)bh * Sq + qi] : 0.f;
  DropKey dkey{0u, 0u};
  uint32_t thr = 0;
  float inv = 1.f;
  if constexpr (DROP) {
    dkey = drop_key(step_seed(seed), (uint32_t)bh);
    thr = drop_thr(p_drop);
    inv = 1.f / (1.f - p_drop);
  }
  f32x16 acc[Z::NBH];
#pragma unroll
  for (int i = 0; i < Z::NBH; ++i) acc[i] = f32x16{};
  const float* kb = k + (int64_t)b * Sk * ks + h * D;
  const float* vb = v + (int64_t)b * Sk * vs + h * D;
  const int iters = (Sk + NW * RB - 1) / (NW * RB);
  for (int it = 0; it < iters; ++it) {
    const int k0 = RB * (NW * it + pw);
    // S^T and dP^T (half of d_h): keys on registers, queries on lanes
    const int kr = min(k0 + l32, Sk - 1);
    const float* kp = kb + (int64_t)kr * ks + dof;
    const float* vp = vb + (int64_t)kr * vs + dof;
    f32x16 sd[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int g = 0; g < Z::NGH; ++g) {
      sd[0] = mfma4(ld4(kp + 8 * g), qf[g], sd[0]);
      sd[1] = mfma4(ld4(vp + 8 * g), df[g], sd[1]);
    }
    exchange<2>(smem, it, sd);
    if (k0 >= Sk) continue;
    float ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kj = k0 + crow(r, hl);
      const float p = (kj < Sk && qi < Sq) ? __builtin_amdgcn_exp2f(sd[0][r] * c - lq) : 0.f;
      float z = 1.f;
      if constexpr (DROP) z = hash_lo(dkey, (uint32_t)qi * (uint32_t)Sk + (uint32_t)kj) >= thr ? inv : 0.f;
      ds[r] = p * (sd[1][r] * z - dl);
    }
    // dQ^T (this half's column blocks) += K^T dS^T
#pragma unroll
    for (int i = 0; i < Z::NBH; ++i) {
      const int nb = hf * Z::NBH + i;
      if (nb < Z::NB) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          acc[i] = mfma4(ld_t(kb, ks, k0 + 8 * g, Sk, 32 * nb + l32),
                         float4{ds[4 * g], ds[4 * g + 1], ds[4 * g + 2], ds[4 * g + 3]}, acc[i]);
      }
    }
  }
  __syncthreads();
  put_partial<D>(smem, acc);
  __syncthreads();
  combine_store<D, false>(smem, nullptr, dq_out + (int64_t)b * Sq * dqs + h * D, dqs, q0, Sq, scale);
}

template <int D>
static int fwd(const float* q, const float* k, const float* v, float* o, float* lse, int B, int Sq, int Sk, int H,
               int64_t qs, int64_t ks, int64_t vs, int64_t os, float scale, float p, uint64_t seed, hipStream_t st) {
  dim3 grid((Sq + RB - 1) / RB, B * H);
  if (p > 0.f) fwd_kernel<D, true><<<grid, NTH, 0, st>>>(q, k, v, o, lse, B, Sq, Sk, H, qs, ks, vs, os, scale, p, seed);
  else fwd_kernel<D, false><<<grid, NTH, 0, st>>>(q, k, v, o, lse, B, Sq, Sk, H, qs, ks, vs, os, scale, p, seed);
  return (int)hipGetLastError();
}

template <int D>
static int bwd(const float* q, const float* k, const float* v, const float* o, const float* dout, const float* lse,
               float* delta, float* dq, float* dk, float* dv, int B, int Sq, int Sk, int H, int64_t qs, int64_t ks,
               int64_t vs, int64_t os, int64_t dqs, int64_t dks, int64_t dvs, float scale, float p, uint64_t seed,
               hipStream_t st) {
  // dO shares O's layout (the caller's contiguous [T, H*D] gradient); delta from O and dO
  const int64_t dos = os;
  delta_kernel<<<(B * Sq * H + 3) / 4, 256, 0, st>>>(o, dout, delta, B, Sq, H, D, os, dos);
  dim3 gk((Sk + RB - 1) / RB, B * H), gq((Sq + RB - 1) / RB, B * H);
  if (p > 0.f) {
    dkv_kernel<D, true><<<gk, NTH, 0, st>>>(q, k, v, dout, lse, delta, dk, dv, B, Sq, Sk, H, qs, ks, vs, dos, dks, dvs,
                                            scale, p, seed);
    dq_kernel<D, true><<<gq, NTH, 0, st>>>(q, k, v, dout, lse, delta, dq, B, Sq, Sk, H, qs, ks, vs, dos, dqs, scale, p,
                                           seed);
  } else {
    dkv_kernel<D, false><<<gk, NTH, 0, st>>>(q, k, v, dout, lse, delta, dk, dv, B, Sq, Sk, H, qs, ks, vs, dos, dks,
                                             dvs, scale, p, seed);
    dq_kernel<D, false><<<gq, NTH, 0, st>>>(q, k, v, dout, lse, delta, dq, B, Sq, Sk, H, qs, ks, vs, dos, dqs, scale,
                                            p, seed);
  }
  return (int)hipGetLastError();
}

}  // namespace af32

// q/k/v/o: token-major f32 views (row stride qs/ks/vs/os, head h at columns h*D), rows of
// 16-byte aligned heads; lse f32 [B*H*Sq] (log2 units).  Non-causal, H == Hkv.  Returns -1
// for an unsupported shape / layout.
extern "C" int mp_attn_f32_fwd(const float* q, const float* k, const float* v, float* o, float* lse, int B, int Sq,
                               int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os,
                               int causal, float scale, float p_drop, uint64_t seed, hipStream_t st) {
  if (causal || H != Hkv || (qs | ks | vs | os) % 4 || Sq <= 0 || Sk <= 0) return -1;
  switch (D) {
    case 64: return af32::fwd<64>(q, k, v, o, lse, B, Sq, Sk, H, qs, ks, vs, os, scale, p_drop, seed, st);
    case 96: return af32::fwd<96>(q, k, v, o, lse, B, Sq, Sk, H, qs, ks, vs, os, scale, p_drop, seed, st);
    case 128: return af32::fwd<128>(q, k, v, o, lse, B, Sq, Sk, H, qs, ks, vs, os, scale, p_drop, seed, st);
    case 192: return af32::fwd<192>(q, k, v, o, lse, B, Sq, Sk, H, qs, ks, vs, os, scale, p_drop, seed, st);
    default: return -1;
  }
}

// dq/dk/dv: token-major f32 outputs (written, not accumulated); delta: f32 [B*H*Sq] scratch;
// dout has o's layout (stride os)
extern "C" int mp_attn_f32_bwd(const float* q, const float* k, const float* v, const float* o, const float* dout,
                               const float* lse, float* delta, float* dq, float* dk, float* dv, int B, int Sq, int Sk,
                               int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dqs,
                               int64_t dks, int64_t dvs, int causal, float scale, float p_drop, uint64_t seed,
                               hipStream_t st) {
  if (causal || H != Hkv || (qs | ks | vs | os | dqs | dks | dvs) % 4 || Sq <= 0 || Sk <= 0) return -1;
#define MP_BW(DD)                                                                                                  \
  case DD:                                                                                                         \
    return af32::bwd<DD>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, H, qs, ks, vs, os, dqs, dks, dvs, scale, \
                         p_drop, seed, st);
  switch (D) {
    MP_BW(64) MP_BW(96) MP_BW(128) MP_BW(192)
    default: return -1;
  }
#undef MP_BW
}

MP_DROP_STEP_SETTER(mp_set_drop_step_attn_f32)
