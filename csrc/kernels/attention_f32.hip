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
//    group g, k slot hl means k = 8g + 4 hl + j -- so a k-contiguous LDS row gives a lane its
//    4 values with ONE ds_read_b128, and the C element r = 4g + j of an accumulator is
//    exactly the k = 8g + 4hl + j that the next MFMA's B operand needs from this lane.
//  * forward / dQ: S^T = K Q^T (A = K rows from LDS, B = the lane's own Q row from
//    registers) puts the query on the LANE, the keys on the registers: the softmax row
//    statistics are per lane, and P^T (registers) is directly the B operand of
//    O^T = V^T P^T (A = V^T rows from LDS).  Output O^T: query on the lane again.
//  * dK / dV: S = Q K^T (A = Q rows from LDS, B = the lane's own K row) puts the KEY on the
//    lane; dV^T = dO^T P and dK^T = Q^T dS take P / dS straight from registers.
// K/V (resp. Q/dO) blocks of 32 rows are staged through LDS in [row][D+4] and [D][32+4]
// layouts (conflict-free ds_read_b128 for both), the next block prefetched into registers
// during the current block's MFMAs.  H == Hkv only (the reference has no GQA).
#include "mp_common.h"

using namespace mp;

namespace af32 {

constexpr int NTH = 256, RB = 32, TS = RB + 4;
constexpr float L2E = 1.4426950408889634f;

template <int D>
struct Blk {
  static constexpr int RS = D + 4;            // row-layout stride (floats)
  static constexpr int NL = D / 32;           // float4 per thread for a 32 x D block
};

// one 32-row x D block of a token-major tensor (rows [r0, r0 + 32) of sequence b, head
// column offset hc) -> registers, zero-filled past `rows`
template <int D>
__device__ __forceinline__ void gload(float4 (&v)[Blk<D>::NL], const float* __restrict__ base, int64_t stride,
                                      int r0, int rows) {
#pragma unroll
  for (int u = 0; u < Blk<D>::NL; ++u) {
    const int idx = threadIdx.x + NTH * u;
    const int row = idx % RB, c = idx / RB;
    v[u] = (r0 + row < rows) ? *reinterpret_cast<const float4*>(base + (int64_t)(r0 + row) * stride + 4 * c)
                             : float4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int D>
__device__ __forceinline__ void st_rows(float* __restrict__ s, const float4 (&v)[Blk<D>::NL]) {
#pragma unroll
  for (int u = 0; u < Blk<D>::NL; ++u) {
    const int idx = threadIdx.x + NTH * u;
    const int row = idx % RB, c = idx / RB;
    *reinterpret_cast<float4*>(s + row * Blk<D>::RS + 4 * c) = v[u];
  }
}

template <int D>
__device__ __forceinline__ void st_trans(float* __restrict__ s, const float4 (&v)[Blk<D>::NL]) {
#pragma unroll
  for (int u = 0; u < Blk<D>::NL; ++u) {
    const int idx = threadIdx.x + NTH * u;
    const int row = idx % RB, c = idx / RB;
    s[(4 * c + 0) * TS + row] = v[u].x;
    s[(4 * c + 1) * TS + row] = v[u].y;
    s[(4 * c + 2) * TS + row] = v[u].z;
    s[(4 * c + 3) * TS + row] = v[u].w;
  }
}

__device__ __forceinline__ f32x16 mfma4(float4 a, float4 b, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ int crow(int r, int hl) { return (r & 3) + 8 * (r >> 2) + 4 * hl; }

// wave-tile [32 rows (lane l32)][D] accumulators acc[nb] (element r -> column 32 nb + crow)
// -> token-major global rows, through the wave's LDS scratch (coalesced 16-B stores)
template <int D>
__device__ __forceinline__ void store_lane_rows(const f32x16 (&acc)[D / 32], float scale_per_lane, float* scratch,
                                                float* __restrict__ out, int64_t stride, int r0, int rows) {
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5;
#pragma unroll
  for (int nb = 0; nb < D / 32; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) scratch[l32 * Blk<D>::RS + 32 * nb + crow(r, hl)] = acc[nb][r] * scale_per_lane;
  __syncthreads();   // (each wave reads back only its own region; every wave calls this)
  for (int i = lane; i < RB * D / 4; i += 64) {
    const int row = i / (D / 4), c = i % (D / 4);
    if (r0 + row < rows)
      *reinterpret_cast<float4*>(out + (int64_t)(r0 + row) * stride + 4 * c) =
          *reinterpret_cast<const float4*>(scratch + row * Blk<D>::RS + 4 * c);
  }
}

// ----------------------------------------------------------------------------------- forward
template <int D, bool DROP>
__global__ void __launch_bounds__(NTH, 1) fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                     const float* __restrict__ v, float* __restrict__ o,
                                                     float* __restrict__ lse, int B, int Sq, int Sk, int H,
                                                     int64_t qs, int64_t ks, int64_t vs, int64_t os, float scale,
                                                     float p_drop, uint64_t seed) {
  constexpr int RS = Blk<D>::RS, NL = Blk<D>::NL, NB = D / 32, NG = D / 8;
  constexpr int LDS_KV = RB * RS + D * TS;
  constexpr int LDS_O = 4 * RB * RS;
  __shared__ __attribute__((aligned(16))) float smem[LDS_KV > LDS_O ? LDS_KV : LDS_O];
  float* Ks = smem;
  float* Vt = smem + RB * RS;
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int q0 = blockIdx.x * 128 + 32 * wave;
  const int qi = q0 + l32;
  const float c = scale * L2E;
  // the lane's query row, pre-scaled into log2 units: qf[g] = Q[qi][8g + 4hl .. +3]
  float4 qf[NG];
  {
    const float* qp = q + (int64_t)(b * Sq + qi) * qs + h * D + 4 * hl;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      float4 t = qi < Sq ? *reinterpret_cast<const float4*>(qp + 8 * g) : float4{0.f, 0.f, 0.f, 0.f};
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
  f32x16 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;
  const float* kb = k + (int64_t)b * Sk * ks + h * D;
  const float* vb = v + (int64_t)b * Sk * vs + h * D;
  float4 pk[NL], pv[NL];
  gload<D>(pk, kb, ks, 0, Sk);
  gload<D>(pv, vb, vs, 0, Sk);
  for (int k0 = 0; k0 < Sk; k0 += RB) {
    __syncthreads();
    st_rows<D>(Ks, pk);
    st_trans<D>(Vt, pv);
    __syncthreads();
    if (k0 + RB < Sk) {
      gload<D>(pk, kb, ks, k0 + RB, Sk);
      gload<D>(pv, vb, vs, k0 + RB, Sk);
    }
    // S^T block: keys on registers (row crow), queries on lanes
    f32x16 s = f32x16{};
#pragma unroll
    for (int g = 0; g < NG; ++g) s = mfma4(*reinterpret_cast<const float4*>(Ks + l32 * RS + 8 * g + 4 * hl), qf[g], s);
    float mb = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (k0 + crow(r, hl) >= Sk) s[r] = -INFINITY;
      mb = fmaxf(mb, s[r]);
    }
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    const float m_new = fmaxf(m_run, mb);
    const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = m_new == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[r] - m_new);
      ls += p;
      float pd = p;
      if constexpr (DROP)
        pd = hash_lo(dk, (uint32_t)qi * (uint32_t)Sk + (uint32_t)(k0 + crow(r, hl))) >= thr ? p * inv : 0.f;
      s[r] = pd;
    }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
    // O^T += V^T P^T
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[nb][r] *= alpha;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        acc[nb] = mfma4(*reinterpret_cast<const float4*>(Vt + (32 * nb + l32) * TS + 8 * g + 4 * hl),
                        float4{s[4 * g], s[4 * g + 1], s[4 * g + 2], s[4 * g + 3]}, acc[nb]);
    }
  }
  __syncthreads();   // LDS is reused for the output transpose
  const float il = l_run > 0.f ? 1.f / l_run : 0.f;
  if (hl == 0 && qi < Sq) lse[(int64_t)bh * Sq + qi] = m_run + __log2f(l_run);
  store_lane_rows<D>(acc, il, smem + wave * RB * RS, o + (int64_t)b * Sq * os + h * D, os, q0, Sq);
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
// PART: 0 = dK and dV, 1 = dV only, 2 = dK only (d_h = 192: the two accumulator sets plus
// both operand rows do not fit 512 registers, so each runs in its own pass)
template <int D, bool DROP, int PART>
__global__ void __launch_bounds__(NTH, 1) dkv_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                     const float* __restrict__ v, const float* __restrict__ dout,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     float* __restrict__ dk_out, float* __restrict__ dv_out, int B,
                                                     int Sq, int Sk, int H, int64_t qs, int64_t ks, int64_t vs,
                                                     int64_t dos, int64_t dks, int64_t dvs, float scale, float p_drop,
                                                     uint64_t seed) {
  constexpr int RS = Blk<D>::RS, NL = Blk<D>::NL, NB = D / 32, NG = D / 8;
  constexpr int LDS_Q = 2 * RB * RS + 2 * D * TS + 2 * RB;
  constexpr int LDS_O = 4 * RB * RS;
  __shared__ __attribute__((aligned(16))) float smem[LDS_Q > LDS_O ? LDS_Q : LDS_O];
  float* Qs = smem;
  float* dOs = Qs + RB * RS;
  float* Qt = dOs + RB * RS;
  float* dOt = Qt + D * TS;
  float* Ls = dOt + D * TS;     // lse (log2 units) of the block's queries
  float* Ds = Ls + RB;          // delta
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int kbase = blockIdx.x * 128 + 32 * wave;
  const int kj = kbase + l32;
  const float c = scale * L2E;
  // the lane's key / value rows: kf[g] = K[kj][8g + 4hl ..], vf likewise
  constexpr bool WANT_DV = PART != 2, WANT_DK = PART != 1;
  float4 kf[NG], vf[WANT_DK ? NG : 1];
  {
    const float* kp = k + (int64_t)(b * Sk + kj) * ks + h * D + 4 * hl;
    const float* vp = v + (int64_t)(b * Sk + kj) * vs + h * D + 4 * hl;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      kf[g] = kj < Sk ? *reinterpret_cast<const float4*>(kp + 8 * g) : float4{0.f, 0.f, 0.f, 0.f};
      if constexpr (WANT_DK)
        vf[g] = kj < Sk ? *reinterpret_cast<const float4*>(vp + 8 * g) : float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  DropKey dkey{0u, 0u};
  uint32_t thr = 0;
  float inv = 1.f;
  if constexpr (DROP) {
    dkey = drop_key(step_seed(seed), (uint32_t)bh);
    thr = drop_thr(p_drop);
    inv = 1.f / (1.f - p_drop);
  }
  f32x16 adk[WANT_DK ? NB : 1], adv[WANT_DV ? NB : 1];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if constexpr (WANT_DK) adk[nb] = f32x16{};
    if constexpr (WANT_DV) adv[nb] = f32x16{};
  }
  const float* qb = q + (int64_t)b * Sq * qs + h * D;
  const float* db = dout + (int64_t)b * Sq * dos + h * D;
  float4 pq[NL], pd[NL];
  gload<D>(pq, qb, qs, 0, Sq);
  gload<D>(pd, db, dos, 0, Sq);
  for (int q0 = 0; q0 < Sq; q0 += RB) {
    __syncthreads();
    st_rows<D>(Qs, pq);
    if constexpr (WANT_DK) st_trans<D>(Qt, pq);
    if constexpr (WANT_DK) st_rows<D>(dOs, pd);
    if constexpr (WANT_DV) st_trans<D>(dOt, pd);
    if (threadIdx.x < RB) {
      const int qi = q0 + threadIdx.x;
      Ls[threadIdx.x] = qi < Sq ? lse[(int64_t)bh * Sq + qi] : INFINITY;
      Ds[threadIdx.x] = qi < Sq ? delta[(int64_t)bh * Sq + qi] : 0.f;
    }
    __syncthreads();
    if (q0 + RB < Sq) {
      gload<D>(pq, qb, qs, q0 + RB, Sq);
      gload<D>(pd, db, dos, q0 + RB, Sq);
    }
    // S and dP with queries on registers (row crow), this wave's keys on lanes
    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      s = mfma4(*reinterpret_cast<const float4*>(Qs + l32 * RS + 8 * g + 4 * hl), kf[g], s);
      if constexpr (WANT_DK) dp = mfma4(*reinterpret_cast<const float4*>(dOs + l32 * RS + 8 * g + 4 * hl), vf[g], dp);
    }
    float pz[16], ds[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 l4 = *reinterpret_cast<const float4*>(Ls + 8 * g + 4 * hl);
      const float4 d4 = *reinterpret_cast<const float4*>(Ds + 8 * g + 4 * hl);
      const float la[4] = {l4.x, l4.y, l4.z, l4.w}, da[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * g + j;
        const int qi = q0 + crow(r, hl);
        float p = (kj < Sk && qi < Sq) ? __builtin_amdgcn_exp2f(s[r] * c - la[j]) : 0.f;
        float z = 1.f;
        if constexpr (DROP) z = hash_lo(dkey, (uint32_t)qi * (uint32_t)Sk + (uint32_t)kj) >= thr ? inv : 0.f;
        pz[r] = p * z;
        ds[r] = p * (dp[r] * z - da[j]);
      }
    }
    // dV^T += dO^T (P z),  dK^T += Q^T dS
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if constexpr (WANT_DV)
          adv[nb] = mfma4(*reinterpret_cast<const float4*>(dOt + (32 * nb + l32) * TS + 8 * g + 4 * hl),
                          float4{pz[4 * g], pz[4 * g + 1], pz[4 * g + 2], pz[4 * g + 3]}, adv[nb]);
        if constexpr (WANT_DK)
          adk[nb] = mfma4(*reinterpret_cast<const float4*>(Qt + (32 * nb + l32) * TS + 8 * g + 4 * hl),
                          float4{ds[4 * g], ds[4 * g + 1], ds[4 * g + 2], ds[4 * g + 3]}, adk[nb]);
      }
  }
  __syncthreads();
  float* scr = smem + wave * RB * RS;
  if constexpr (WANT_DV) store_lane_rows<D>(adv, 1.f, scr, dv_out + (int64_t)b * Sk * dvs + h * D, dvs, kbase, Sk);
  if constexpr (WANT_DV && WANT_DK) __syncthreads();
  if constexpr (WANT_DK) store_lane_rows<D>(adk, scale, scr, dk_out + (int64_t)b * Sk * dks + h * D, dks, kbase, Sk);
}

// --------------------------------------------------------------------------------- dQ
template <int D, bool DROP>
__global__ void __launch_bounds__(NTH, 1) dq_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                    const float* __restrict__ v, const float* __restrict__ dout,
                                                    const float* __restrict__ lse, const float* __restrict__ delta,
                                                    float* __restrict__ dq_out, int B, int Sq, int Sk, int H,
                                                    int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dqs,
                                                    float scale, float p_drop, uint64_t seed) {
  constexpr int RS = Blk<D>::RS, NL = Blk<D>::NL, NB = D / 32, NG = D / 8;
  constexpr int LDS_K = 2 * RB * RS + D * TS;
  constexpr int LDS_O = 4 * RB * RS;
  __shared__ __attribute__((aligned(16))) float smem[LDS_K > LDS_O ? LDS_K : LDS_O];
  float* Ks = smem;
  float* Vs = Ks + RB * RS;
  float* Kt = Vs + RB * RS;
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int q0 = blockIdx.x * 128 + 32 * wave;
  const int qi = q0 + l32;
  const float c = scale * L2E;
  float4 qf[NG], df[NG];
  {
    const float* qp = q + (int64_t)(b * Sq + qi) * qs + h * D + 4 * hl;
    const float* dp = dout + (int64_t)(b * Sq + qi) * dos + h * D + 4 * hl;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      qf[g] = qi < Sq ? *reinterpret_cast<const float4*>(qp + 8 * g) : float4{0.f, 0.f, 0.f, 0.f};
      df[g] = qi < Sq ? *reinterpret_cast<const float4*>(dp + 8 * g) : float4{0.f, 0.f, 0.f, 0.f};
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
  f32x16 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x16{};
  const float* kb = k + (int64_t)b * Sk * ks + h * D;
  const float* vb = v + (int64_t)b * Sk * vs + h * D;
  float4 pk[NL], pv[NL];
  gload<D>(pk, kb, ks, 0, Sk);
  gload<D>(pv, vb, vs, 0, Sk);
  for (int k0 = 0; k0 < Sk; k0 += RB) {
    __syncthreads();
    st_rows<D>(Ks, pk);
    st_trans<D>(Kt, pk);
    st_rows<D>(Vs, pv);
    __syncthreads();
    if (k0 + RB < Sk) {
      gload<D>(pk, kb, ks, k0 + RB, Sk);
      gload<D>(pv, vb, vs, k0 + RB, Sk);
    }
    // S^T and dP^T: keys on registers, queries on lanes
    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      s = mfma4(*reinterpret_cast<const float4*>(Ks + l32 * RS + 8 * g + 4 * hl), qf[g], s);
      dp = mfma4(*reinterpret_cast<const float4*>(Vs + l32 * RS + 8 * g + 4 * hl), df[g], dp);
    }
    float ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kj = k0 + crow(r, hl);
      const float p = (kj < Sk && qi < Sq) ? __builtin_amdgcn_exp2f(s[r] * c - lq) : 0.f;
      float z = 1.f;
      if constexpr (DROP) z = hash_lo(dkey, (uint32_t)qi * (uint32_t)Sk + (uint32_t)kj) >= thr ? inv : 0.f;
      ds[r] = p * (dp[r] * z - dl);
    }
    // dQ^T += K^T dS^T
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        acc[nb] = mfma4(*reinterpret_cast<const float4*>(Kt + (32 * nb + l32) * TS + 8 * g + 4 * hl),
                        float4{ds[4 * g], ds[4 * g + 1], ds[4 * g + 2], ds[4 * g + 3]}, acc[nb]);
  }
  __syncthreads();
  store_lane_rows<D>(acc, scale, smem + wave * RB * RS, dq_out + (int64_t)b * Sq * dqs + h * D, dqs, q0, Sq);
}

template <int D>
static int fwd(const float* q, const float* k, const float* v, float* o, float* lse, int B, int Sq, int Sk, int H,
               int64_t qs, int64_t ks, int64_t vs, int64_t os, float scale, float p, uint64_t seed, hipStream_t st) {
  dim3 grid((Sq + 127) / 128, B * H);
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
  dim3 gk((Sk + 127) / 128, B * H), gq((Sq + 127) / 128, B * H);
#define MP_DKV(DR, PART)                                                                                        \
  dkv_kernel<D, DR, PART><<<gk, NTH, 0, st>>>(q, k, v, dout, lse, delta, dk, dv, B, Sq, Sk, H, qs, ks, vs, dos, dks, \
                                              dvs, scale, p, seed)
  if (p > 0.f) {
    if constexpr (D > 128) {
      MP_DKV(true, 1);
      MP_DKV(true, 2);
    } else {
      MP_DKV(true, 0);
    }
    dq_kernel<D, true><<<gq, NTH, 0, st>>>(q, k, v, dout, lse, delta, dq, B, Sq, Sk, H, qs, ks, vs, dos, dqs, scale, p,
                                           seed);
  } else {
    if constexpr (D > 128) {
      MP_DKV(false, 1);
      MP_DKV(false, 2);
    } else {
      MP_DKV(false, 0);
    }
    dq_kernel<D, false><<<gq, NTH, 0, st>>>(q, k, v, dout, lse, delta, dq, B, Sq, Sk, H, qs, ks, vs, dos, dqs, scale,
                                            p, seed);
  }
#undef MP_DKV
  return (int)hipGetLastError();
}

}  // namespace af32

// q/k/v/o: token-major f32 views (row stride qs/ks/vs/os, head h at columns h*D), rows of
// 16-byte aligned heads; lse f32 [B*H*Sq] (log2 units).  Non-causal, H == Hkv.  Returns -1
// for an unsupported shape / layout.
extern "C" int mp_attn_f32_fwd(const float* q, const float* k, const float* v, float* o, float* lse, int B, int Sq,
                               int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os,
                               int causal, float scale, float p_drop, uint64_t seed, hipStream_t st) {
  if (causal || H != Hkv || (qs | ks | vs | os) % 4) return -1;
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
  if (causal || H != Hkv || (qs | ks | vs | os | dqs | dks | dvs) % 4) return -1;
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
