// Flash attention forward / backward for gfx950 (bf16 in, f32 accumulate, MFMA 32x32x16).
// SURVEY §2.5 K4 (self + cross attention, causal / non-causal, head dims 64..256,
// GQA, in-kernel counter-based dropout regenerated in the backward).
//
// Layout: q/k/v/o are token-major rows ([B*S, row_stride] bf16), head h at column h*D,
// i.e. exactly what the fused QKV projection writes and the output projection reads:
// no transposes or head-major copies anywhere.  LSE is kept per (b, h, query) in log2
// units (lse2 = m + log2(l)) for the backward.
//
// Forward (one workgroup = 4 waves = 128 queries of one (b, h); 64-key tiles):
//   * "swapped" QK^T: each wave computes S^T = K . Q^T so the QUERY is on the MFMA lane and
//     the 32 keys of a 32x32 tile are in its registers: the row max / row sum are
//     in-lane (+1 cross-half shuffle), and the online-softmax rescale of O is a per-lane
//     scalar because O is also kept transposed (O^T = V^T . P^T).
//   * P^T never leaves registers: the S^T accumulator is already the B operand of
//     V^T . P^T (k order permuted, see cdna guide §3); V^T fragments come from
//     ds_read_b64_tr_b16 hardware-transposed LDS reads.
//   * K and V tiles are register-staged into a double-buffered LDS ring (loads for tile
//     j+1 issued before computing tile j, written after), XOR-swizzled in 16-byte chunks
//     so both the b128 row reads (K) and the transposed reads (V) are bank-conflict free.
//   * causal: heavy query blocks launch first; per-wave skip of fully masked tiles.
// Backward = two deterministic kernels (no f32 atomics):
//   dkdv: one workgroup = 128 keys of one (b, kv-head), loops over all query heads of the
//         group (GQA) and all query tiles; key on the MFMA lane so P and dS are directly
//         the B operands of dV^T += dO^T P and dK^T += Q^T dS.
//   dq:   one workgroup = 128 queries (forward structure), recomputes P^T and dP^T and
//         accumulates dQ^T += K^T dS^T.
#include "mp_common.h"

#include <cstdlib>
#include <type_traits>

using namespace mp;

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

#define LOG2E 1.4426950408889634f

// ------------------------------------------------------------------------------------------
// LDS image: [rows][DP] bf16, 16-byte chunks XOR-swizzled per row.
// ------------------------------------------------------------------------------------------
template <int DP>
__device__ __forceinline__ int chunk_swz(int row) {
  if constexpr (DP == 64) return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
  else return ((row & 3) << 2) | ((row >> 2) & 3);
}

template <int DP>
__device__ __forceinline__ int lds_off(int row, int chunk) {  // byte offset of a 16-byte chunk
  return row * (DP * 2) + 16 * (chunk ^ chunk_swz<DP>(row));
}

// 16-byte row read (A operand: rows on lanes 0..31, 8 consecutive columns)
template <int DP>
__device__ __forceinline__ bf16x8 lds_row8(const char* base, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(base + lds_off<DP>(row, chunk));
}

// Transposed read: returns for this lane the 4 rows r0..r0+3 of column (c0 + (lane&15)).
// Lane 4q+p of each 16-lane group addresses row r0+q, columns c0+4p..c0+4p+3.
template <int DP>
__device__ __forceinline__ s16x4 lds_tr4(const char* base, int r0, int c0) {
  const int i = threadIdx.x & 15;
  const int q = i >> 2, p = i & 3;
  const int row = r0 + q;
  const int col = c0 + 4 * p;
  const char* a = base + lds_off<DP>(row, col >> 3) + ((col & 7) << 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a));
}

__device__ __forceinline__ bf16x8 cat44(s16x4 lo, s16x4 hi) {
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& acc, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)acc[8 * s + j];
  return r;
}

// load 8 bf16 of a global row (zero outside [0, D) or invalid row)
__device__ __forceinline__ u16x8 gload8(const bf16_t* rowp, int col, int D, bool valid) {
  u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!valid || col >= D) return z;
  return *reinterpret_cast<const u16x8*>(rowp + col);
}

// Stage a [64][DP] tile of rows (row0 .. row0+63 of a token-major tensor) into registers.
template <int DP>
struct Stage64 {
  static constexpr int PER = DP / 32;  // 16-byte chunks per thread
  u16x8 v[PER];
  __device__ __forceinline__ void load(const bf16_t* base, int64_t stride, int row0, int nrows, int D) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx / (DP / 8), c = idx % (DP / 8);
      const int gr = row0 + r;
      v[i] = gload8(base + (int64_t)gr * stride, c * 8, D, gr < nrows);
    }
  }
  __device__ __forceinline__ void store(char* lds) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx / (DP / 8), c = idx % (DP / 8);
      *reinterpret_cast<u16x8*>(lds + lds_off<DP>(r, c)) = v[i];
    }
  }
};

// dropout element index of score (bh, q, k): bh in the high word, q * Sk + k in the low
// word (the kernels use drop_key(seed, bh) + the low word directly; this is the reference)
__device__ __forceinline__ uint64_t drop_idx(int bh, int q, int k, int Sk) {
  return ((uint64_t)bh * 0x100000000ull) + (uint64_t)q * (uint64_t)Sk + (uint64_t)k;
}

// ==========================================================================================
// forward
// ==========================================================================================
template <int DP, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, DP <= 128 ? 2 : 1) attn_fwd_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, bf16_t* __restrict__ O,
    float* __restrict__ LSE, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs,
    int64_t os, float scale, float p_drop, uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;  // bytes per [64][DP] tile
#define kbuf(i) (smem + (i) * TILE)
#define vbuf(i) (smem + (2 + (i)) * TILE)

  const int nmb = (Sq + 127) / 128;
  // causal: longest-first over the WHOLE grid (workgroups are dispatched in linear id
  // order): every (b, h)'s last query block, then the second to last, ...  Heavy-first
  // within each (b, h) row only interleaved heavy and light blocks and left a tail of
  // late heavy blocks -- causal took as long as full attention at S = 1024
  const int lin = (int)blockIdx.x + (int)gridDim.x * (int)blockIdx.y;
  const int nbh = (int)gridDim.y;
  const int mb = CAUSAL ? (nmb - 1 - lin / nbh) : (int)blockIdx.x;
  const int bh = CAUSAL ? lin % nbh : (int)blockIdx.y;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, hl = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // wave-uniform: scalar branches
  const int m0 = mb * 128;
  const int qrow = m0 + 32 * w + l32;  // this lane's query
  const bool qvalid = qrow < Sq;
  const bf16_t* Qb = Q + (int64_t)b * Sq * qs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * Sk * ks + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * Sk * vs + (int64_t)hk * D;

  // Q as the B operand of S^T = K Q^T: lane holds Q[qrow][16s + 8hl + j]
  bf16x8 qf[DP / 16];
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    u16x8 t = gload8(Qb + (int64_t)qrow * qs, 16 * s + 8 * hl, D, qvalid);
    qf[s] = __builtin_bit_cast(bf16x8, t);
  }
  const float c = scale * LOG2E;
  // dropout stream of this (b, h): keys once, 32-bit index q * Sk + key (drop_idx's low word)
  const DropKey dkey = drop_key(seed, (uint32_t)bh);
  const uint32_t dthr = drop_thr(p_drop), qoff = (uint32_t)qrow * (uint32_t)Sk;
  const float dinv = 1.0f / (1.0f - p_drop);
  f32x16 o[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) o[d] = {};
  float m_run = -INFINITY, l_run = 0.f;

  // causal alignment: query i may attend keys <= i + (Sk - Sq)
  const int shift = Sk - Sq;
  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + 128 + shift);
  const int ntiles = (n_end + 63) / 64;

  Stage64<DP> kst, vst;
  kst.load(Kb, ks, 0, Sk, D);
  vst.load(Vb, vs, 0, Sk, D);
  kst.store(kbuf(0));
  vst.store(vbuf(0));
  const int wave_last_q = m0 + 32 * w + 31 + shift;

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const int n0 = t * 64;
    if (t + 1 < ntiles) {
      kst.load(Kb, ks, n0 + 64, Sk, D);
      vst.load(Vb, vs, n0 + 64, Sk, D);
    }
    __syncthreads();
    const bool skip = CAUSAL && n0 > wave_last_q;
    if (!skip) {
      const char* kb = kbuf(cur);
      const char* vb = vbuf(cur);
      // ---- S^T = K Q^T (two 32-key sub tiles)
      f32x16 s0 = {}, s1 = {};
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        bf16x8 a0 = lds_row8<DP>(kb, l32, 2 * s + hl);
        bf16x8 a1 = lds_row8<DP>(kb, 32 + l32, 2 * s + hl);
        s0 = mfma32(a0, qf[s], s0);
        s1 = mfma32(a1, qf[s], s1);
      }
      // ---- mask (only tiles that cross the causal diagonal or the key end), tile max on
      // raw scores; p = 2^(s*c - m) is one v_fma + one v_exp (scale folded, log2 units)
      const bool edge = (n0 + 64 > Sk) || (CAUSAL && n0 + 63 > m0 + 32 * w + shift);
      if (edge) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kr = (r & 3) + 8 * (r >> 2) + 4 * hl;
          const int ka = n0 + kr, kb2 = n0 + 32 + kr;
          if (ka >= Sk || (CAUSAL && ka > qrow + shift)) s0[r] = -INFINITY;
          if (kb2 >= Sk || (CAUSAL && kb2 > qrow + shift)) s1[r] = -INFINITY;
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = max3_raw(mx, s0[r], s1[r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx * c);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
      // dropout: the 32 keep bits of this lane's scores first (only the bit mask stays live
      // across the hashes: computed beside the probabilities the DP = 128 build spilled)
      uint32_t keep = 0xffffffffu;
      if (DROP) {
        keep = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t kr = (uint32_t)(n0 + (r & 3) + 8 * (r >> 2) + 4 * hl);
          keep |= (hash_lo(dkey, qoff + kr) >= dthr ? 1u : 0u) << r;
          keep |= (hash_lo(dkey, qoff + kr + 32u) >= dthr ? 1u : 0u) << (16 + r);
        }
      }
      float rs = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(s0[r], c, -m_use));
        float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(s1[r], c, -m_use));
        rs += p0 + p1;
        if (DROP) {
          p0 = (keep >> r) & 1u ? p0 * dinv : 0.f;
          p1 = (keep >> (16 + r)) & 1u ? p1 * dinv : 0.f;
        }
        s0[r] = p0;
        s1[r] = p1;
      }
      rs += __shfl_xor(rs, 32, 64);
      l_run = l_run * alpha + rs;
      m_run = m_new;
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) o[d] *= alpha;
      // ---- O^T += V^T P^T
      const bf16x8 p00 = pack8(s0, 0), p01 = pack8(s0, 1), p10 = pack8(s1, 0), p11 = pack8(s1, 1);
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
        const int c0 = 32 * d + 16 * ((lane >> 4) & 1);
        bf16x8 a;
        a = cat44(lds_tr4<DP>(vb, 0 + 4 * hl, c0), lds_tr4<DP>(vb, 8 + 4 * hl, c0));
        o[d] = mfma32(a, p00, o[d]);
        a = cat44(lds_tr4<DP>(vb, 16 + 4 * hl, c0), lds_tr4<DP>(vb, 24 + 4 * hl, c0));
        o[d] = mfma32(a, p01, o[d]);
        a = cat44(lds_tr4<DP>(vb, 32 + 4 * hl, c0), lds_tr4<DP>(vb, 40 + 4 * hl, c0));
        o[d] = mfma32(a, p10, o[d]);
        a = cat44(lds_tr4<DP>(vb, 48 + 4 * hl, c0), lds_tr4<DP>(vb, 56 + 4 * hl, c0));
        o[d] = mfma32(a, p11, o[d]);
      }
    }
    if (t + 1 < ntiles) {
      kst.store(kbuf(cur ^ 1));
      vst.store(vbuf(cur ^ 1));
    }
  }
  // ---- epilogue: O = O^T / l ; LSE
  if (qvalid) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    bf16_t* orow = O + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = f2bf(o[d][4 * g + e] * inv);
          *reinterpret_cast<u16x4*>(orow + col) = pk;
        }
      }
    }
    if (hl == 0) LSE[(int64_t)bh * Sq + qrow] = l_run > 0.f ? m_run + log2f(l_run) : INFINITY;
  }
}

// ==========================================================================================
// forward, short sequences: workgroup = 64 queries, keys split over two wave pairs
// ==========================================================================================
// At the reference's shape (B 8, S 128, non-causal, 4-12 heads) the 128-query workgroups
// above are 32-96 for 256 CUs and every wave walks both 64-key tiles back to back.  Here
// a workgroup owns 64 queries: waves (qs = w & 1: which 32 queries, kh = w >> 1: which key
// tiles -- kh, kh + 2, ...).  Each wave pair streams its own K/V tiles into the same
// swizzled image by LDS-DMA (no staging registers), keeps its own online-softmax state,
// and the kh = 1 waves hand (O^T, m, l) to their kh = 0 partners through LDS at the end:
// twice the workgroups, half the serial tile chain per wave.  Non-causal only.
template <int DP>
struct GTileP {   // a [64][DP] tile by the 2 waves of one pair, LDS-DMA (the GTile scheme below)
  static constexpr int CPR = DP / 8;           // 16-byte chunks per row
  static constexpr int PR = 1024 / (DP * 2);   // rows per 1 KiB piece
  static constexpr int PPW = (64 / PR) / 2;    // pieces per wave
  int lr, phys;
  __device__ __forceinline__ void init() {
    const int lane = threadIdx.x & 63;
    lr = lane / CPR;
    phys = lane % CPR;
  }
  __device__ __forceinline__ void issue(const bf16_t* base, int64_t stride, int row0, int nrows, int D, char* img,
                                        int wv) const {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wv + 2 * i;
      const int row = p * PR + lr;
      const int chunk = (phys & ~15) | ((phys & 15) ^ chunk_swz<DP>(row));
      int col = chunk * 8;
      col = col < D ? col : 0;
      int gr = row0 + row;
      gr = gr < nrows ? gr : nrows - 1;   // rows past the end: masked keys / zero probabilities
      __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)gr * stride + col),
                                       (__attribute__((address_space(3))) void*)(img + p * 1024), 16, 0, 0);
    }
  }
};

template <int DP, bool DROP>
__global__ void __launch_bounds__(256, 2) attn_fwd_ks2_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, bf16_t* __restrict__ O,
    float* __restrict__ LSE, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs,
    int64_t os, float scale, float p_drop, uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
  const int bh = (int)blockIdx.y;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, l32 = lane & 31;
  const int qsub = w & 1, kh = w >> 1;
  const int ntiles = (Sk + 63) / 64;
  const int niter = (ntiles + 1) / 2;   // the same trip count in both pairs (barriers inside)
  // this pair's K / V tiles: double-buffered when it walks more than one tile (S = 128:
  // one tile per pair, 64 KB of LDS in all, as much as the 128-query kernel)
  const int nbuf = niter > 1 ? 2 : 1;
  char* gbase = smem + kh * 2 * nbuf * TILE;
#define kbuf2(i) (gbase + (i) * TILE)
#define vbuf2(i) (gbase + (nbuf + (i)) * TILE)
  const int m0 = (int)blockIdx.x * 64;
  const int qrow = m0 + 32 * qsub + l32;
  const bool qvalid = qrow < Sq;
  const bf16_t* Qb = Q + (int64_t)b * Sq * qs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * Sk * ks + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * Sk * vs + (int64_t)hk * D;
  bf16x8 qf[DP / 16];
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    u16x8 t = gload8(Qb + (int64_t)qrow * qs, 16 * s + 8 * hl, D, qvalid);
    qf[s] = __builtin_bit_cast(bf16x8, t);
  }
  const float c = scale * LOG2E;
  const DropKey dkey = drop_key(seed, (uint32_t)bh);
  const uint32_t dthr = drop_thr(p_drop), qoff = (uint32_t)qrow * (uint32_t)Sk;
  const float dinv = 1.0f / (1.0f - p_drop);
  f32x16 o[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) o[d] = {};
  float m_run = -INFINITY, l_run = 0.f;
  GTileP<DP> gp;
  gp.init();
  const int wv = __builtin_amdgcn_readfirstlane(qsub);
  gp.issue(Kb, ks, 64 * kh, Sk, D, kbuf2(0), wv);
  gp.issue(Vb, vs, 64 * kh, Sk, D, vbuf2(0), wv);
  for (int it = 0; it < niter; ++it) {
    const int cur = it & 1;
    const int n0 = 64 * (2 * it + kh);
    __syncthreads();   // (waits for this wave's LDS-DMA first: tile `it` is in LDS for the pair)
    if (it + 1 < niter) {   // the next tile into the buffer the pair finished before this barrier
      gp.issue(Kb, ks, n0 + 128, Sk, D, kbuf2(cur ^ 1), wv);
      gp.issue(Vb, vs, n0 + 128, Sk, D, vbuf2(cur ^ 1), wv);
    }
    if (n0 < Sk) {
      const char* kb = kbuf2(cur);
      const char* vb = vbuf2(cur);
      f32x16 s0 = {}, s1 = {};
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        bf16x8 a0 = lds_row8<DP>(kb, l32, 2 * s + hl);
        bf16x8 a1 = lds_row8<DP>(kb, 32 + l32, 2 * s + hl);
        s0 = mfma32(a0, qf[s], s0);
        s1 = mfma32(a1, qf[s], s1);
      }
      if (n0 + 64 > Sk) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kr = (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (n0 + kr >= Sk) s0[r] = -INFINITY;
          if (n0 + 32 + kr >= Sk) s1[r] = -INFINITY;
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = max3_raw(mx, s0[r], s1[r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx * c);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
      uint32_t keep = 0xffffffffu;
      if (DROP) {
        keep = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t kr = (uint32_t)(n0 + (r & 3) + 8 * (r >> 2) + 4 * hl);
          keep |= (hash_lo(dkey, qoff + kr) >= dthr ? 1u : 0u) << r;
          keep |= (hash_lo(dkey, qoff + kr + 32u) >= dthr ? 1u : 0u) << (16 + r);
        }
      }
      float rs = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(s0[r], c, -m_use));
        float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(s1[r], c, -m_use));
        rs += p0 + p1;
        if (DROP) {
          p0 = (keep >> r) & 1u ? p0 * dinv : 0.f;
          p1 = (keep >> (16 + r)) & 1u ? p1 * dinv : 0.f;
        }
        s0[r] = p0;
        s1[r] = p1;
      }
      rs += __shfl_xor(rs, 32, 64);
      l_run = l_run * alpha + rs;
      m_run = m_new;
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) o[d] *= alpha;
      const bf16x8 p00 = pack8(s0, 0), p01 = pack8(s0, 1), p10 = pack8(s1, 0), p11 = pack8(s1, 1);
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
        const int c0 = 32 * d + 16 * ((lane >> 4) & 1);
        bf16x8 a;
        a = cat44(lds_tr4<DP>(vb, 0 + 4 * hl, c0), lds_tr4<DP>(vb, 8 + 4 * hl, c0));
        o[d] = mfma32(a, p00, o[d]);
        a = cat44(lds_tr4<DP>(vb, 16 + 4 * hl, c0), lds_tr4<DP>(vb, 24 + 4 * hl, c0));
        o[d] = mfma32(a, p01, o[d]);
        a = cat44(lds_tr4<DP>(vb, 32 + 4 * hl, c0), lds_tr4<DP>(vb, 40 + 4 * hl, c0));
        o[d] = mfma32(a, p10, o[d]);
        a = cat44(lds_tr4<DP>(vb, 48 + 4 * hl, c0), lds_tr4<DP>(vb, 56 + 4 * hl, c0));
        o[d] = mfma32(a, p11, o[d]);
      }
    }
  }
#undef kbuf2
#undef vbuf2
  // the kh = 1 pair hands (O^T, m, l) to the kh = 0 pair
  __syncthreads();
  float* xo = reinterpret_cast<float*>(smem) + qsub * (DP / 32 * 16 * 64 + 128);
  if (kh == 1) {
#pragma unroll
    for (int d = 0; d < DP / 32; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) xo[(d * 16 + r) * 64 + lane] = o[d][r];
    xo[DP / 32 * 16 * 64 + lane] = m_run;
    xo[DP / 32 * 16 * 64 + 64 + lane] = l_run;
  }
  __syncthreads();
  if (kh == 1) return;
  const float m1 = xo[DP / 32 * 16 * 64 + lane], l1 = xo[DP / 32 * 16 * 64 + 64 + lane];
  const float mm = fmaxf(m_run, m1);
  const float mu = mm == -INFINITY ? 0.f : mm;
  const float a0 = __builtin_amdgcn_exp2f(m_run - mu), a1 = __builtin_amdgcn_exp2f(m1 - mu);
  const float l = l_run * a0 + l1 * a1;
#pragma unroll
  for (int d = 0; d < DP / 32; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = o[d][r] * a0 + xo[(d * 16 + r) * 64 + lane] * a1;
  if (qvalid) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* orow = O + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = f2bf(o[d][4 * g + e] * inv);
          *reinterpret_cast<u16x4*>(orow + col) = pk;
        }
      }
    }
    if (hl == 0) LSE[(int64_t)bh * Sq + qrow] = l > 0.f ? mm + log2f(l) : INFINITY;
  }
}

// ==========================================================================================
// glds staging of [64][DP] row tiles straight into the swizzled LDS image
// ==========================================================================================
// A 1 KiB LDS-DMA piece is PR = 1024 / (2 DP) image rows; lane l lands at byte 16 l of the
// piece, so the XOR swizzle is applied on the SOURCE column (cdna guide §5.4 rule 21).
// Columns past D (head dim padded to DP) read column 0 of the same row instead: finite
// data that only meets zero K/V columns or feeds unwritten output columns.
template <int DP>
struct GTile {
  static constexpr int CPR = DP / 8;           // 16-byte chunks per row
  static constexpr int PR = 1024 / (DP * 2);   // rows per piece
  static constexpr int PPW = (64 / PR) / 4;    // pieces per wave (4 waves)
  int lr, phys;
  __device__ __forceinline__ void init() {
    const int lane = threadIdx.x & 63;
    lr = lane / CPR;
    phys = lane % CPR;
  }
  // rows row0 .. row0+63 of a token-major tensor (row stride `stride`, column offset
  // already in `base`) -> LDS image `img`
  __device__ __forceinline__ void issue(const bf16_t* base, int64_t stride, int row0, int nrows, int D, char* img,
                                        int wave) const {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wave + 4 * i;
      const int row = p * PR + lr;
      const int chunk = (phys & ~15) | ((phys & 15) ^ chunk_swz<DP>(row));
      int col = chunk * 8;
      col = col < D ? col : 0;
      int gr = row0 + row;
      gr = gr < nrows ? gr : nrows - 1;
      __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)gr * stride + col),
                                       (__attribute__((address_space(3))) void*)(img + p * 1024), 16, 0, 0);
    }
  }
};

// Column sums over a workgroup's 128 token rows of a [rows][D] f32 register tile (lane =
// row 32 w + l32, register 4g + e of acc[d] = column 32d + 8g + 4hl + e), times `mul`,
// atomically added to out[0 .. D): the bias gradient of the QKV projection, fused into the
// attention backward instead of a second pass over dQKV.  Sums over the 32 lanes of each
// half by xor-shuffles, over the 4 waves through LDS (`red`, >= 4 * DP floats; the caller
// has synchronised so it is free), then one atomic per column per workgroup.
template <int DP>
__device__ __forceinline__ void wg_colsum_atomic(const f32x16 (&acc)[DP / 32], float mul, bool valid, float* red,
                                                 float* __restrict__ out, int D) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int d = 0; d < DP / 32; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float x = valid ? acc[d][r] * mul : 0.f;
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) x += __shfl_xor(x, o, 64);
      if (l32 == 0) red[w * DP + 32 * d + 8 * (r >> 2) + 4 * hl + (r & 3)] = x;
    }
  __syncthreads();
  for (int c = threadIdx.x; c < DP; c += 256)
    if (c < D) atomicAdd(out + c, red[c] + red[DP + c] + red[2 * DP + c] + red[3 * DP + c]);
}

template <int N>
__device__ __forceinline__ void attn_wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | (((N >> 4) & 3) << 14));
}

// ==========================================================================================
// forward v2: paired query blocks, LDS-DMA K/V ring, lazy rescale (the default at d_h 64)
// ==========================================================================================
// Same tile structure as attn_fwd_kernel (4 waves x 32 queries, 64-key tiles, swapped
// S^T = K Q^T with P^T kept in registers), with the per-tile VALU cut and the grid reshaped
// (the forward issued ~18 VALU per MFMA at 0.26 MFMA busy, profiles/r5_attention_pmc.md):
//   * K/V tiles stream through a 3-deep LDS ring by buffer-load-to-LDS DMA (GTile's piece
//     layout; 32-bit per-lane offsets fixed at entry + a scalar per-tile offset; rows past
//     the key end read as zero): two tiles in flight, counted vmcnt, one raw barrier per tile.  v1 staged one
//     tile ahead through registers, so every tile waited out a full load latency (v1 -> v2
//     with register staging kept: 2-4 %; the dQ kernel, on the ring, ran 1.5x v1's MFMA
//     work per tile in less time).
//   * causal / key-end mask: one compare against a per-lane limit and one select per score
//     (the key's in-tile position is a compile-time constant per accumulator register).
//   * cross-half max / sum by v_permlane32_swap instead of an LDS bpermute.
//   * lazy rescale: the subtracted row maximum moves only when a lane's tile maximum exceeds
//     it by more than 2^8 (wave-uniform branch); otherwise O and l are not rescaled (P stays
//     <= 2^8, exact in f32 sums and bf16 products).
//   * causal: one workgroup runs query block nmb-1-p and then block p of the same (b, h), so
//     every workgroup does the same number of tiles (no heavy-first tail); the pairs of one
//     (b, h) sit on one XCD (workgroup id mod 8) next to each other, so their K/V tiles are
//     read while the others still hold them in that XCD's L2.
__device__ __forceinline__ float xhalf_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return max3_raw(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// GTile's 1 KiB-piece layout issued as buffer_load ... lds: the per-lane byte offset of each
// piece is fixed at kernel entry (32-bit), the tile's row offset is a scalar, and rows past
// the buffer's range (keys >= Sk) land as zeros -- no 64-bit address math per tile
template <int DP>
struct BTile {
  static constexpr int CPR = DP / 8, PR = 1024 / (DP * 2), PPW = (64 / PR) / 4;
  int voff[PPW];
  __device__ __forceinline__ void init(int64_t stride, int D, int wave) {
    const int lane = threadIdx.x & 63, lr = lane / CPR, phys = lane % CPR;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int row = (wave + 4 * i) * PR + lr;
      const int chunk = (phys & ~15) | ((phys & 15) ^ chunk_swz<DP>(row));
      const int col = chunk * 8 < D ? chunk * 8 : 0;
      voff[i] = (int)(((int64_t)row * stride + col) * 2);
    }
  }
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, int soff, char* img, int wave) const {
    // (the builtin exists for the gfx950 pass only; the host pass would drop the kernel's stubs)
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < PPW; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + (wave + 4 * i) * 1024),
                                               16, voff[i], soff, 0, 0);
#endif
  }
};

// max over the 32 scores of a lane (two 32x32 accumulators): 16 dependent v_max3_f32 in two
// asm blocks (fmaxf would canonicalise every MFMA output first; one asm statement per max3
// made the compiler pad each with an s_nop)
__device__ __forceinline__ float tile_max32(const f32x16& a, const f32x16& b) {
  float m;
  asm("v_max3_f32 %0, %1, %2, %3\n\t"
      "v_max3_f32 %0, %0, %4, %5\n\t"
      "v_max3_f32 %0, %0, %6, %7\n\t"
      "v_max3_f32 %0, %0, %8, %9\n\t"
      "v_max3_f32 %0, %0, %10, %11\n\t"
      "v_max3_f32 %0, %0, %12, %13\n\t"
      "v_max3_f32 %0, %0, %14, %15\n\t"
      "v_max3_f32 %0, %0, %16, %17"
      : "=&v"(m)
      : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]),
        "v"(a[5]), "v"(b[5]), "v"(a[6]), "v"(b[6]), "v"(a[7]), "v"(b[7]), "v"(-INFINITY));
  float m2;
  asm("v_max3_f32 %0, %1, %2, %3\n\t"
      "v_max3_f32 %0, %0, %4, %5\n\t"
      "v_max3_f32 %0, %0, %6, %7\n\t"
      "v_max3_f32 %0, %0, %8, %9\n\t"
      "v_max3_f32 %0, %0, %10, %11\n\t"
      "v_max3_f32 %0, %0, %12, %13\n\t"
      "v_max3_f32 %0, %0, %14, %15\n\t"
      "v_max3_f32 %0, %0, %16, %17"
      : "=&v"(m2)
      : "v"(m), "v"(a[8]), "v"(b[8]), "v"(a[9]), "v"(b[9]), "v"(a[10]), "v"(b[10]), "v"(a[11]), "v"(b[11]),
        "v"(a[12]), "v"(b[12]), "v"(a[13]), "v"(b[13]), "v"(a[14]), "v"(b[14]), "v"(a[15]), "v"(b[15]));
  return m2;
}

// in-tile key offset of accumulator register r (lane half hl adds 4)
__device__ __forceinline__ constexpr int key_of(int r) { return (r & 3) + 8 * (r >> 2); }

#ifndef MP_FWD_NBUF
#define MP_FWD_NBUF 2
#endif
template <int DP, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, DROP ? 2 : (MP_FWD_NBUF == 2 ? 4 : 3)) attn_fwd2_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, bf16_t* __restrict__ O,
    float* __restrict__ LSE, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs,
    int64_t os, float scale, float p_drop, uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
  constexpr float TAU = 8.f;   // lazy-rescale threshold (log2 units)
  const int nmb = (Sq + 127) / 128;
  const int npair = CAUSAL ? (nmb + 1) / 2 : nmb;   // workgroups per (b, h)
  const int nbh = B * H;
  // workgroup -> (bh, p): the npair workgroups of one bh are consecutive on one XCD
  const int lin = (int)blockIdx.x;
  int bh, p;
  if ((nbh & 7) == 0) {
    const int xcd = lin & 7, j = lin >> 3;
    bh = (j / npair) * 8 + xcd;
    p = j % npair;
  } else {
    bh = lin / npair;
    p = lin % npair;
  }
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, hl = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const bf16_t* Qb = Q + (int64_t)b * Sq * qs + (int64_t)h * D;
  // range: through the last valid row's head slice (the launcher keeps it below 2^31)
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(K + (int64_t)b * Sk * ks + (int64_t)hk * D), 0, (int)(((int64_t)(Sk - 1) * ks + D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(V + (int64_t)b * Sk * vs + (int64_t)hk * D), 0, (int)(((int64_t)(Sk - 1) * vs + D) * 2), 0x00020000);
  // K / V ring: NBUF buffers of (K tile, V tile), LOOK tiles in flight
  // ring depth (build-time A/B, MP_FWD_NBUF): 2 = 32 KB of LDS, 4 workgroups per CU (B 64:
  // 190 vs 200 us at 3 = 48 KB, 3 per CU; profiles/r6_attention_v2.md)
  constexpr int NBUF = MP_FWD_NBUF, LOOK = NBUF - 1, BUFB = 2 * TILE;
  static_assert(NBUF == 2 || NBUF == 3, "the tile loop below is unrolled by NBUF");
  constexpr int PER_TILE = 2 * BTile<DP>::PPW;   // DMA instructions per tile per wave
  BTile<DP> kt, vt;
  kt.init(ks, D, w);
  vt.init(vs, D, w);
  const int kstep = (int)(64 * ks * 2), vstep = (int)(64 * vs * 2);
  // per-lane LDS byte offsets of the fragment reads inside a tile (swizzle included; the rows
  // a lane reads 32 / 16 apart share the swizzle, so the rest are immediate offsets):
  //   K rows l32 (+32: +4096) at chunk 2s + hl;  V^T transposed reads of rows 8j + 4hl + q
  //   at column 32d + 16 (lane>>4 & 1) + 4p: j = jp + 2m is voff[d][jp] + 2048 m
  int koff[DP / 16], vtoff[DP / 32][2];
  {
    const int i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) koff[s] = lds_off<DP>(l32, 2 * s + hl);
#pragma unroll
    for (int d = 0; d < DP / 32; ++d)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int row = 8 * jp + 4 * hl + q, col = 32 * d + 16 * ((lane >> 4) & 1) + 4 * pp;
        vtoff[d][jp] = lds_off<DP>(row, col >> 3) + ((col & 7) << 1);
      }
  }
  auto issue = [&](int t) {
    char* buf = smem + (t % NBUF) * BUFB;
    kt.issue(krs, t * kstep, buf, w);
    vt.issue(vrs, t * vstep, buf + TILE, w);
  };
  const float c = scale * LOG2E;
  const DropKey dkey = drop_key(seed, (uint32_t)bh);
  const uint32_t dthr = drop_thr(p_drop);
  const float dinv = 1.0f / (1.0f - p_drop);
  const int shift = Sk - Sq;
  const u16x8 ones_u = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};   // bf16 1.0
  const bf16x8 ones = __builtin_bit_cast(bf16x8, ones_u);
  const int npass = CAUSAL && (nmb - 1 - p) != p ? 2 : 1;

  for (int pass = 0; pass < npass; ++pass) {
    const int mb = CAUSAL ? (pass == 0 ? nmb - 1 - p : p) : p;
    const int m0 = mb * 128;
    const int qrow = m0 + 32 * w + l32;
    const bool qvalid = qrow < Sq;
    bf16x8 qf[DP / 16];
#pragma unroll
    for (int s = 0; s < DP / 16; ++s)
      qf[s] = __builtin_bit_cast(bf16x8, gload8(Qb + (int64_t)qrow * qs, 16 * s + 8 * hl, D, qvalid));
    const uint32_t qoff = (uint32_t)qrow * (uint32_t)Sk;
    f32x16 o[DP / 32];
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) o[d] = {};
    float m_run = -INFINITY;   // running maximum (log2 units) ...
    float m_sub = 0.f;         // ... and the finite value the probabilities subtract
    f32x16 lsum = {};          // running row sum (every register: this lane's query) ...
    float l_drop = 0.f;        // ... or, with dropout, the pre-mask sum on the VALU
    int n_end = Sk;
    if (CAUSAL) n_end = min(Sk, m0 + 128 + shift);
    const int ntiles = n_end > 0 ? (n_end + 63) / 64 : 0;
    const int wave_last_q = m0 + 32 * w + 31 + shift;
    // per-lane mask limit: a key of in-tile offset k (+4 hl) is kept iff k <= lim - n0
    const int lim0 = (CAUSAL ? min(qrow + shift, Sk - 1) : Sk - 1) - 4 * hl;

    if (pass > 0) {   // every wave has read the previous pass's last tiles
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < LOOK; ++i)
      if (i < ntiles) issue(i);
    // one tile on ring buffer BUF (a compile-time constant: every LDS address of the tile is
    // an immediate offset, and the refill target (BUF + LOOK) % NBUF too)
    auto tile = [&](auto bufc, int t) {
      constexpr int BUF = decltype(bufc)::value;
      const int n0 = t * 64;
      // tile t landed (the younger one may stay in flight), then publish it to all waves
      if (LOOK >= 2 && t + 1 < ntiles) attn_wait_vmcnt<PER_TILE>();
      else attn_wait_vmcnt<0>();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // every wave is done with tile t-1: its buffer takes tile t+LOOK
      if (t + LOOK < ntiles) {
        char* buf = smem + ((BUF + LOOK) % NBUF) * BUFB;
        kt.issue(krs, (t + LOOK) * kstep, buf, w);
        vt.issue(vrs, (t + LOOK) * vstep, buf + TILE, w);
      }
      const bool skip = CAUSAL && n0 > wave_last_q;
      if (!skip) {
        const char* kb = smem + BUF * BUFB;
        const char* vb = kb + TILE;
        f32x16 s0 = {}, s1 = {};
#pragma unroll
        for (int s = 0; s < DP / 16; ++s) {
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(kb + koff[s]);
          const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(kb + koff[s] + 32 * DP * 2);
          s0 = mfma32(a0, qf[s], s0);
          s1 = mfma32(a1, qf[s], s1);
        }
        const bool edge = (n0 + 64 > Sk) || (CAUSAL && n0 + 63 > m0 + 32 * w + shift);
        if (edge) {
          const int lim = lim0 - n0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            s0[r] = key_of(r) > lim ? -INFINITY : s0[r];
            s1[r] = key_of(r) + 32 > lim ? -INFINITY : s1[r];
          }
        }
        float mx = tile_max32(s0, s1);
        mx = xhalf_max(mx);
        const float mxc = mx * c;
        // lazy rescale: wave-uniform, taken on the first tile and when a maximum jumps
        if (__builtin_amdgcn_ballot_w64(mxc > m_run + TAU)) {
          const float m_new = fmaxf(m_run, mxc);
          const float s_new = m_new == -INFINITY ? 0.f : m_new;
          const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_sub - s_new);
#pragma unroll
          for (int d = 0; d < DP / 32; ++d) o[d] *= alpha;
          lsum *= alpha;
          l_drop *= alpha;
          m_run = m_new;
          m_sub = s_new;
        }
        uint32_t keep = 0xffffffffu;
        if (DROP) {
          keep = 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t kr = (uint32_t)(n0 + key_of(r) + 4 * hl);
            keep |= (hash_lo(dkey, qoff + kr) >= dthr ? 1u : 0u) << r;
            keep |= (hash_lo(dkey, qoff + kr + 32u) >= dthr ? 1u : 0u) << (16 + r);
          }
        }
        float rs0 = 0.f, rs1 = 0.f;   // dropout: the normaliser sums P BEFORE the mask
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(s0[r], c, -m_sub));
          float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(s1[r], c, -m_sub));
          if (DROP) {
            rs0 += p0;
            rs1 += p1;
            p0 = (keep >> r) & 1u ? p0 * dinv : 0.f;
            p1 = (keep >> (16 + r)) & 1u ? p1 * dinv : 0.f;
          }
          s0[r] = p0;
          s1[r] = p1;
        }
        const bf16x8 p00 = pack8(s0, 0), p01 = pack8(s0, 1), p10 = pack8(s1, 0), p11 = pack8(s1, 1);
        if constexpr (DROP) {
          l_drop += xhalf_sum(rs0 + rs1);
        } else {
          // row sums on the matrix cores: ones^T . P^T puts sum_k P[q][k] (of the bf16 P that
          // the PV product uses) in every register of lane q -- 4 MFMAs in place of 32 adds
          // and a cross-half exchange on the VALU, which is the busier pipe here
          lsum = mfma32(ones, p00, lsum);
          lsum = mfma32(ones, p01, lsum);
          lsum = mfma32(ones, p10, lsum);
          lsum = mfma32(ones, p11, lsum);
        }
#pragma unroll
        for (int d = 0; d < DP / 32; ++d) {
          auto tr = [&](int jp, int m) {
            return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(vb + vtoff[d][jp] + 16 * DP * 2 * m));
          };
          o[d] = mfma32(cat44(tr(0, 0), tr(1, 0)), p00, o[d]);
          o[d] = mfma32(cat44(tr(0, 1), tr(1, 1)), p01, o[d]);
          o[d] = mfma32(cat44(tr(0, 2), tr(1, 2)), p10, o[d]);
          o[d] = mfma32(cat44(tr(0, 3), tr(1, 3)), p11, o[d]);
        }
      }
    };
    for (int t0 = 0; t0 < ntiles; t0 += NBUF) {
      tile(std::integral_constant<int, 0>{}, t0);
      if (t0 + 1 < ntiles) tile(std::integral_constant<int, 1>{}, t0 + 1);
      if constexpr (NBUF == 3)
        if (t0 + 2 < ntiles) tile(std::integral_constant<int, 2 % NBUF>{}, t0 + 2);
    }
    const float l_run = DROP ? l_drop : lsum[0];
    if (qvalid) {
      const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
      bf16_t* orow = O + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = 32 * d + 8 * g + 4 * hl;
          if (col < D) {
            u16x4 pk;
#pragma unroll
            for (int e = 0; e < 4; ++e) pk[e] = f2bf(o[d][4 * g + e] * inv);
            *reinterpret_cast<u16x4*>(orow + col) = pk;
          }
        }
      }
      if (hl == 0) LSE[(int64_t)bh * Sq + qrow] = l_run > 0.f ? m_sub + log2f(l_run) : INFINITY;
    }
  }
}


// ==========================================================================================
// backward dK / dV: workgroup = 128 keys (4 waves x 32) of one (b, kv head)
// ==========================================================================================
// Q / dO tiles and the per-row LSE / delta stream through an NBUF-deep LDS ring by
// LDS-DMA (2 tiles in flight for DP <= 128): no staging registers, one raw barrier per
// tile, counted vmcnt.  Same math as before: key on the MFMA lane, P and dS are the B
// operands of dV^T += dO^T P and dK^T += Q^T dS.
template <int DP, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, DP <= 64 ? 2 : 1) attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs,
    int64_t ks, int64_t vs, int64_t os, int64_t dks, int64_t dvs, float scale, float p_drop, uint64_t seed,
    float* __restrict__ CSK, float* __restrict__ CSV) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
  constexpr int BUFB = 2 * TILE + 512;               // Q, dO, lse[64], delta[64]
  // ring depth: MIPIPE-tunable at build time (MP_DKDV_NBUF); 4 buffers keep 3 tiles in flight
#ifndef MP_DKDV_NBUF
#define MP_DKDV_NBUF 4
#endif
  constexpr int NBUF = DP <= 128 ? MP_DKDV_NBUF : 2;
  constexpr int LOOK = NBUF - 1;                     // tiles issued ahead
  using GT = GTile<DP>;

  // causal: key block 0 sees every query -> longest-first over the whole grid (all (b, h)'s
  // first key block, then the second, ...), as in the forward
  const int lin = (int)blockIdx.x + (int)gridDim.x * (int)blockIdx.y;
  const int kb = CAUSAL ? lin / (int)gridDim.y : (int)blockIdx.x;
  const int bhk = CAUSAL ? lin % (int)gridDim.y : (int)blockIdx.y;
  const int b = bhk / Hkv, hk = bhk % Hkv;
  const int grp = H / Hkv;
  const int lane = threadIdx.x & 63, hl = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int k0 = kb * 128;
  const int key = k0 + 32 * w + l32;  // this lane's key (MFMA column)
  const bool kvalid = key < Sk;
  const int shift = Sk - Sq;

  // K and V of this wave's 32 keys as B operands: lane holds K[key][16s + 8hl + j]
  bf16x8 kf[DP / 16], vf[DP / 16];
  const bf16_t* Krow = K + ((int64_t)b * Sk + key) * ks + (int64_t)hk * D;
  const bf16_t* Vrow = V + ((int64_t)b * Sk + key) * vs + (int64_t)hk * D;
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    kf[s] = __builtin_bit_cast(bf16x8, gload8(Krow, 16 * s + 8 * hl, D, kvalid));
    vf[s] = __builtin_bit_cast(bf16x8, gload8(Vrow, 16 * s + 8 * hl, D, kvalid));
  }
  f32x16 dk[DP / 32], dv[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) {
    dk[d] = {};
    dv[d] = {};
  }
  const float c = scale * LOG2E;
  const uint32_t dthr = drop_thr(p_drop);
  const float dinv = 1.0f / (1.0f - p_drop);
  // first query that can see key k0: q >= k0 - shift
  const int q_begin = CAUSAL ? max(0, ((k0 - shift) / 64) * 64) : 0;
  const int ntq = (Sq - q_begin + 63) / 64;
  const int total = ntq * grp;

  GT gt;
  gt.init();
  auto issue = [&](int it) {
    const int hq = hk * grp + it / ntq;
    const int q0 = q_begin + (it % ntq) * 64;
    char* buf = smem + (it % NBUF) * BUFB;
    gt.issue(Q + (int64_t)b * Sq * qs + (int64_t)hq * D, qs, q0, Sq, D, buf, w);
    gt.issue(dO + (int64_t)b * Sq * os + (int64_t)hq * D, os, q0, Sq, D, buf + TILE, w);
    if (w == 0) {  // per-row stats, 4 bytes per lane (rows past Sq are masked in the math)
      const int q = min(q0 + lane, Sq - 1);
      const int64_t idx = ((int64_t)b * H + hq) * Sq + q;
      __builtin_amdgcn_global_load_lds((const void*)(LSE + idx),
                                       (__attribute__((address_space(3))) void*)(buf + 2 * TILE), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(DELTA + idx),
                                       (__attribute__((address_space(3))) void*)(buf + 2 * TILE + 256), 4, 0, 0);
    }
  };
  constexpr int PER_TILE = 2 * GT::PPW;  // DMA instructions per tile per wave (+2 on wave 0)
#pragma unroll
  for (int i = 0; i < LOOK; ++i)
    if (i < total) issue(i);

  for (int it = 0; it < total; ++it) {
    const int hq = hk * grp + it / ntq;
    const int q0 = q_begin + (it % ntq) * 64;
    const int bhq = b * H + hq;
    const DropKey dkey = drop_key(seed, (uint32_t)bhq);
    // tile `it` landed (up to LOOK-1 younger tiles may stay in flight), then publish to all
    // waves; wave 0 issues 2 extra DMAs per tile (the row stats)
    if (LOOK >= 3 && it + 2 < total) {
      if (w == 0) attn_wait_vmcnt<2 * (PER_TILE + 2)>(); else attn_wait_vmcnt<2 * PER_TILE>();
    } else if (LOOK >= 2 && it + 1 < total) {
      if (w == 0) attn_wait_vmcnt<PER_TILE + 2>(); else attn_wait_vmcnt<PER_TILE>();
    } else {
      attn_wait_vmcnt<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // the buffer of tile it-1 is free now: refill it with tile it+LOOK
    if (it + LOOK < total) issue(it + LOOK);
    const char* qb = smem + (it % NBUF) * BUFB;
    const char* gb = qb + TILE;
    const float* ls = reinterpret_cast<const float*>(qb + 2 * TILE);
    const float* dl = ls + 64;
    const bool skip = CAUSAL && (k0 + 32 * w > q0 + 63 + shift);  // all of this wave's keys masked
    if (!skip) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // S[q][key] = Q K^T, dP[q][key] = dO V^T   (query rows u*32.. in registers, key on lane)
        f32x16 sacc = {}, pacc = {};
#pragma unroll
        for (int s = 0; s < DP / 16; ++s) {
          bf16x8 aq = lds_row8<DP>(qb, 32 * u + l32, 2 * s + hl);
          bf16x8 ag = lds_row8<DP>(gb, 32 * u + l32, 2 * s + hl);
          sacc = mfma32(aq, kf[s], sacc);
          pacc = mfma32(ag, vf[s], pacc);
        }
        f32x16 pm, ds;
        // per-row stats: rows 32u + 8g + 4hl + 0..3 are contiguous -> one 16-byte LDS read
        float4 lsv[4], dlv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          lsv[g] = *reinterpret_cast<const float4*>(ls + 32 * u + 8 * g + 4 * hl);
          dlv[g] = *reinterpret_cast<const float4*>(dl + 32 * u + 8 * g + 4 * hl);
        }
        // masks only where needed: the causal diagonal and query rows past Sq (their
        // stats were clamped); keys past Sk only feed their own unwritten outputs
        const bool edge = (q0 + 64 > Sq) || (CAUSAL && (k0 + 32 * w + 31 > q0 + 32 * u + shift));
        // the element math twice, masked and unmasked, behind one wave-uniform branch: as a
        // per-element select the mask's index compares and cndmasks were issued on every
        // tile (~half of the loop's VALU, profiles/r2_attention_pmc_counters.json)
        // dropout keep bits first (only the mask stays live across the hashes)
        uint32_t keep = 0xffffu;
        if (DROP) {
          keep = 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t q = (uint32_t)(q0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hl);
            keep |= (hash_lo(dkey, q * (uint32_t)Sk + (uint32_t)key) >= dthr ? 1u : 0u) << r;
          }
        }
        auto elems = [&](auto masked) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int qr = 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hl;
            const int q = q0 + qr;
            const float lv = (&lsv[r >> 2].x)[r & 3], dv_ = (&dlv[r >> 2].x)[r & 3];
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[r], c, -lv));
            if constexpr (decltype(masked)::value) {
              if (q >= Sq || (CAUSAL && key > q + shift)) p = 0.f;
            }
            float dpv = pacc[r];
            float pd = p;
            if (DROP) {
              const float msk = (keep >> r) & 1u ? dinv : 0.f;
              pd = p * msk;
              dpv = dpv * msk;
            }
            pm[r] = pd;                      // dropped P for dV
            ds[r] = p * (dpv - dv_);         // dS
          }
        };
        if (edge) elems(std::true_type{});
        else elems(std::false_type{});
        // dV^T += dO^T P ;  dK^T += Q^T dS     (A via transposed LDS reads of the row images)
        const bf16x8 pb0 = pack8(pm, 0), pb1 = pack8(pm, 1);
        const bf16x8 db0 = pack8(ds, 0), db1 = pack8(ds, 1);
#pragma unroll
        for (int d = 0; d < DP / 32; ++d) {
          const int c0 = 32 * d + 16 * ((lane >> 4) & 1);
          const int rb = 32 * u + 4 * hl;
          bf16x8 ag0 = cat44(lds_tr4<DP>(gb, rb + 0, c0), lds_tr4<DP>(gb, rb + 8, c0));
          bf16x8 ag1 = cat44(lds_tr4<DP>(gb, rb + 16, c0), lds_tr4<DP>(gb, rb + 24, c0));
          dv[d] = mfma32(ag0, pb0, dv[d]);
          dv[d] = mfma32(ag1, pb1, dv[d]);
          bf16x8 aq0 = cat44(lds_tr4<DP>(qb, rb + 0, c0), lds_tr4<DP>(qb, rb + 8, c0));
          bf16x8 aq1 = cat44(lds_tr4<DP>(qb, rb + 16, c0), lds_tr4<DP>(qb, rb + 24, c0));
          dk[d] = mfma32(aq0, db0, dk[d]);
          dk[d] = mfma32(aq1, db1, dk[d]);
        }
      }
    }
  }
  // ---- fused bias-gradient column sums of dK (scaled) and dV
  if (CSK != nullptr) {
    __syncthreads();   // the Q / dO ring is free
    float* red = reinterpret_cast<float*>(smem);
    wg_colsum_atomic<DP>(dk, scale, kvalid, red, CSK + (int64_t)hk * D, D);
    __syncthreads();
    wg_colsum_atomic<DP>(dv, 1.f, kvalid, red, CSV + (int64_t)hk * D, D);
  }
  // ---- epilogue: lane = key, registers = d
  if (kvalid) {
    bf16_t* dkrow = dK + ((int64_t)b * Sk + key) * dks + (int64_t)hk * D;
    bf16_t* dvrow = dV + ((int64_t)b * Sk + key) * dvs + (int64_t)hk * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 a, bb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] = f2bf(dk[d][4 * g + e] * scale);
            bb[e] = f2bf(dv[d][4 * g + e]);
          }
          *reinterpret_cast<u16x4*>(dkrow + col) = a;
          *reinterpret_cast<u16x4*>(dvrow + col) = bb;
        }
      }
    }
  }
}

// backward dK / dV v2 (d_h 64, the default): attn_bwd_dkdv_kernel's math on the forward v2
// tile machinery (buffer-load-to-LDS Q / dO ring, lane offsets fixed at entry, the tile loop
// unrolled over the 4-deep ring so every LDS address is an immediate)
template <int DP, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, 2) attn_bwd_dkdv2_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs,
    int64_t ks, int64_t vs, int64_t os, int64_t dks, int64_t dvs, float scale, float p_drop, uint64_t seed,
    float* __restrict__ CSK, float* __restrict__ CSV) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
  constexpr int BUFB = 2 * TILE + 512;               // Q, dO, lse[64], delta[64]
  // ring depth: MIPIPE-tunable at build time (MP_DKDV_NBUF); 4 buffers keep 3 tiles in flight
#ifndef MP_DKDV_NBUF
#define MP_DKDV_NBUF 4
#endif
  constexpr int NBUF = 4;
  constexpr int LOOK = NBUF - 1;                     // tiles issued ahead

  // causal: key block 0 sees every query -> longest-first over the whole grid (all (b, h)'s
  // first key block, then the second, ...), as in the forward
  const int lin = (int)blockIdx.x + (int)gridDim.x * (int)blockIdx.y;
  const int kb = CAUSAL ? lin / (int)gridDim.y : (int)blockIdx.x;
  const int bhk = CAUSAL ? lin % (int)gridDim.y : (int)blockIdx.y;
  const int b = bhk / Hkv, hk = bhk % Hkv;
  const int grp = H / Hkv;
  const int lane = threadIdx.x & 63, hl = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int k0 = kb * 128;
  const int key = k0 + 32 * w + l32;  // this lane's key (MFMA column)
  const bool kvalid = key < Sk;
  const int shift = Sk - Sq;

  // K and V of this wave's 32 keys as B operands: lane holds K[key][16s + 8hl + j]
  bf16x8 kf[DP / 16], vf[DP / 16];
  const bf16_t* Krow = K + ((int64_t)b * Sk + key) * ks + (int64_t)hk * D;
  const bf16_t* Vrow = V + ((int64_t)b * Sk + key) * vs + (int64_t)hk * D;
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    kf[s] = __builtin_bit_cast(bf16x8, gload8(Krow, 16 * s + 8 * hl, D, kvalid));
    vf[s] = __builtin_bit_cast(bf16x8, gload8(Vrow, 16 * s + 8 * hl, D, kvalid));
  }
  f32x16 dk[DP / 32], dv[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) {
    dk[d] = {};
    dv[d] = {};
  }
  const float c = scale * LOG2E;
  const uint32_t dthr = drop_thr(p_drop);
  const float dinv = 1.0f / (1.0f - p_drop);
  // first query that can see key k0: q >= k0 - shift
  const int q_begin = CAUSAL ? max(0, ((k0 - shift) / 64) * 64) : 0;
  const int ntq = (Sq - q_begin + 63) / 64;
  const int total = ntq * grp;

  // Q / dO tiles by buffer-load-to-LDS DMA (the forward v2 scheme): per-lane offsets fixed
  // here, the tile's row offset a scalar, one buffer resource per query head (rows past Sq
  // land as zeros); the loop below is unrolled over the ring, so LDS addresses are immediates
  BTile<DP> qt, gt2;
  qt.init(qs, D, w);
  gt2.init(os, D, w);
  auto issue_to = [&](int it, char* buf) {
    const int hq = hk * grp + it / ntq;
    const int q0 = q_begin + (it % ntq) * 64;
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Q + (int64_t)b * Sq * qs + (int64_t)hq * D), 0, (int)(((int64_t)(Sq - 1) * qs + D) * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(dO + (int64_t)b * Sq * os + (int64_t)hq * D), 0, (int)(((int64_t)(Sq - 1) * os + D) * 2), 0x00020000);
    qt.issue(qrs, (int)((int64_t)q0 * qs * 2), buf, w);
    gt2.issue(grs, (int)((int64_t)q0 * os * 2), buf + TILE, w);
    if (w == 0) {  // per-row stats, 4 bytes per lane (rows past Sq are masked in the math)
      const int q = min(q0 + lane, Sq - 1);
      const int64_t idx = ((int64_t)b * H + hq) * Sq + q;
      __builtin_amdgcn_global_load_lds((const void*)(LSE + idx),
                                       (__attribute__((address_space(3))) void*)(buf + 2 * TILE), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(DELTA + idx),
                                       (__attribute__((address_space(3))) void*)(buf + 2 * TILE + 256), 4, 0, 0);
    }
  };
  constexpr int PER_TILE = 2 * BTile<DP>::PPW;  // DMA instructions per tile per wave (+2 on wave 0)
#pragma unroll
  for (int i = 0; i < LOOK; ++i)
    if (i < total) issue_to(i, smem + i * BUFB);
  // per-lane fragment offsets (see attn_fwd2_kernel): row reads of rows 32u + l32 at chunk
  // 2s + hl; transposed reads of rows 32u + 8j + 4hl + q at column 32d + 16 (lane>>4 & 1) + 4p
  int roff[DP / 16], troff[DP / 32][2];
  {
    const int i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) roff[s] = lds_off<DP>(l32, 2 * s + hl);
#pragma unroll
    for (int d = 0; d < DP / 32; ++d)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int row = 8 * jp + 4 * hl + q, col = 32 * d + 16 * ((lane >> 4) & 1) + 4 * pp;
        troff[d][jp] = lds_off<DP>(row, col >> 3) + ((col & 7) << 1);
      }
  }
  auto tile = [&](auto bufc, int it) {
    constexpr int BUF = decltype(bufc)::value;
    const int hq = hk * grp + it / ntq;
    const int q0 = q_begin + (it % ntq) * 64;
    const int bhq = b * H + hq;
    const DropKey dkey = drop_key(seed, (uint32_t)bhq);
    // tile `it` landed (up to LOOK-1 younger tiles may stay in flight), then publish to all
    // waves; wave 0 issues 2 extra DMAs per tile (the row stats)
    if (LOOK >= 3 && it + 2 < total) {
      if (w == 0) attn_wait_vmcnt<2 * (PER_TILE + 2)>(); else attn_wait_vmcnt<2 * PER_TILE>();
    } else if (LOOK >= 2 && it + 1 < total) {
      if (w == 0) attn_wait_vmcnt<PER_TILE + 2>(); else attn_wait_vmcnt<PER_TILE>();
    } else {
      attn_wait_vmcnt<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // the buffer of tile it-1 is free now: refill it with tile it+LOOK
    if (it + LOOK < total) issue_to(it + LOOK, smem + ((BUF + LOOK) % NBUF) * BUFB);
    const char* qb = smem + BUF * BUFB;
    const char* gb = qb + TILE;
    const float* ls = reinterpret_cast<const float*>(qb + 2 * TILE);
    const float* dl = ls + 64;
    const bool skip = CAUSAL && (k0 + 32 * w > q0 + 63 + shift);  // all of this wave's keys masked
    if (!skip) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // S[q][key] = Q K^T, dP[q][key] = dO V^T   (query rows u*32.. in registers, key on lane)
        f32x16 sacc = {}, pacc = {};
#pragma unroll
        for (int s = 0; s < DP / 16; ++s) {
          const bf16x8 aq = *reinterpret_cast<const bf16x8*>(qb + roff[s] + u * 32 * DP * 2);
          const bf16x8 ag = *reinterpret_cast<const bf16x8*>(gb + roff[s] + u * 32 * DP * 2);
          sacc = mfma32(aq, kf[s], sacc);
          pacc = mfma32(ag, vf[s], pacc);
        }
        f32x16 pm, ds;
        // per-row stats: rows 32u + 8g + 4hl + 0..3 are contiguous -> one 16-byte LDS read
        float4 lsv[4], dlv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          lsv[g] = *reinterpret_cast<const float4*>(ls + 32 * u + 8 * g + 4 * hl);
          dlv[g] = *reinterpret_cast<const float4*>(dl + 32 * u + 8 * g + 4 * hl);
        }
        // masks only where needed: the causal diagonal and query rows past Sq (their
        // stats were clamped); keys past Sk only feed their own unwritten outputs
        const bool edge = (q0 + 64 > Sq) || (CAUSAL && (k0 + 32 * w + 31 > q0 + 32 * u + shift));
        // the element math twice, masked and unmasked, behind one wave-uniform branch: as a
        // per-element select the mask's index compares and cndmasks were issued on every
        // tile (~half of the loop's VALU, profiles/r2_attention_pmc_counters.json)
        // dropout keep bits first (only the mask stays live across the hashes)
        uint32_t keep = 0xffffu;
        if (DROP) {
          keep = 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t q = (uint32_t)(q0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hl);
            keep |= (hash_lo(dkey, q * (uint32_t)Sk + (uint32_t)key) >= dthr ? 1u : 0u) << r;
          }
        }
        auto elems = [&](auto masked) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int qr = 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hl;
            const int q = q0 + qr;
            const float lv = (&lsv[r >> 2].x)[r & 3], dv_ = (&dlv[r >> 2].x)[r & 3];
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[r], c, -lv));
            if constexpr (decltype(masked)::value) {
              if (q >= Sq || (CAUSAL && key > q + shift)) p = 0.f;
            }
            float dpv = pacc[r];
            float pd = p;
            if (DROP) {
              const float msk = (keep >> r) & 1u ? dinv : 0.f;
              pd = p * msk;
              dpv = dpv * msk;
            }
            pm[r] = pd;                      // dropped P for dV
            ds[r] = p * (dpv - dv_);         // dS
          }
        };
        if (edge) elems(std::true_type{});
        else elems(std::false_type{});
        // dV^T += dO^T P ;  dK^T += Q^T dS     (A via transposed LDS reads of the row images)
        const bf16x8 pb0 = pack8(pm, 0), pb1 = pack8(pm, 1);
        const bf16x8 db0 = pack8(ds, 0), db1 = pack8(ds, 1);
#pragma unroll
        for (int d = 0; d < DP / 32; ++d) {
          auto tr = [&](const char* img, int jp, int m) {
            return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(img + troff[d][jp] + u * 32 * DP * 2 + 16 * DP * 2 * m));
          };
          dv[d] = mfma32(cat44(tr(gb, 0, 0), tr(gb, 1, 0)), pb0, dv[d]);
          dv[d] = mfma32(cat44(tr(gb, 0, 1), tr(gb, 1, 1)), pb1, dv[d]);
          dk[d] = mfma32(cat44(tr(qb, 0, 0), tr(qb, 1, 0)), db0, dk[d]);
          dk[d] = mfma32(cat44(tr(qb, 0, 1), tr(qb, 1, 1)), db1, dk[d]);
        }
      }
    }
  };
  for (int t0 = 0; t0 < total; t0 += NBUF) {
    tile(std::integral_constant<int, 0>{}, t0);
    if (t0 + 1 < total) tile(std::integral_constant<int, 1>{}, t0 + 1);
    if (t0 + 2 < total) tile(std::integral_constant<int, 2>{}, t0 + 2);
    if (t0 + 3 < total) tile(std::integral_constant<int, 3>{}, t0 + 3);
  }
  // ---- fused bias-gradient column sums of dK (scaled) and dV
  if (CSK != nullptr) {
    __syncthreads();   // the Q / dO ring is free
    float* red = reinterpret_cast<float*>(smem);
    wg_colsum_atomic<DP>(dk, scale, kvalid, red, CSK + (int64_t)hk * D, D);
    __syncthreads();
    wg_colsum_atomic<DP>(dv, 1.f, kvalid, red, CSV + (int64_t)hk * D, D);
  }
  // ---- epilogue: lane = key, registers = d
  if (kvalid) {
    bf16_t* dkrow = dK + ((int64_t)b * Sk + key) * dks + (int64_t)hk * D;
    bf16_t* dvrow = dV + ((int64_t)b * Sk + key) * dvs + (int64_t)hk * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 a, bb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] = f2bf(dk[d][4 * g + e] * scale);
            bb[e] = f2bf(dv[d][4 * g + e]);
          }
          *reinterpret_cast<u16x4*>(dkrow + col) = a;
          *reinterpret_cast<u16x4*>(dvrow + col) = bb;
        }
      }
    }
  }
}

// dK / dV v3 (the default; MIPIPE_ATTN_BWD_DKDV=2 selects v2): v2 with paired causal key blocks
// on one XCD
template <int DP, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, 2) attn_bwd_dkdv3_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs,
    int64_t ks, int64_t vs, int64_t os, int64_t dks, int64_t dvs, float scale, float p_drop, uint64_t seed,
    float* __restrict__ CSK, float* __restrict__ CSV) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
  constexpr int BUFB = 2 * TILE + 512;               // Q, dO, lse[64], delta[64]
  // ring depth: MIPIPE-tunable at build time (MP_DKDV_NBUF); 4 buffers keep 3 tiles in flight
#ifndef MP_DKDV_NBUF
#define MP_DKDV_NBUF 4
#endif
  constexpr int NBUF = 4;
  constexpr int LOOK = NBUF - 1;                     // tiles issued ahead

  // causal: one workgroup runs key block p (it sees the most queries) and then block
  // nkb-1-p of the same (b, kv head), so every workgroup does about the same work; the pairs
  // of one (b, kv head) are consecutive on one XCD (workgroup id mod 8), so their Q / dO tiles
  // are read while the others still hold them in that XCD's L2 (the forward v2 mapping)
  const int nkb = (Sk + 127) / 128;
  const int npair = CAUSAL ? (nkb + 1) / 2 : nkb;
  const int nbhk = B * Hkv;
  const int lin = (int)blockIdx.x;
  int bhk, p;
  if ((nbhk & 7) == 0) {
    const int xcd = lin & 7, j = lin >> 3;
    bhk = (j / npair) * 8 + xcd;
    p = j % npair;
  } else {
    bhk = lin / npair;
    p = lin % npair;
  }
  const int b = bhk / Hkv, hk = bhk % Hkv;
  const int grp = H / Hkv;
  const int lane = threadIdx.x & 63, hl = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int shift = Sk - Sq;
  const float c = scale * LOG2E;
  const uint32_t dthr = drop_thr(p_drop);
  const float dinv = 1.0f / (1.0f - p_drop);
  BTile<DP> qt, gt2;
  qt.init(qs, D, w);
  gt2.init(os, D, w);
  // per-lane fragment offsets (see attn_fwd2_kernel): row reads of rows 32u + l32 at chunk
  // 2s + hl; transposed reads of rows 32u + 8j + 4hl + q at column 32d + 16 (lane>>4 & 1) + 4p
  int roff[DP / 16], troff[DP / 32][2];
  {
    const int i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) roff[s] = lds_off<DP>(l32, 2 * s + hl);
#pragma unroll
    for (int d = 0; d < DP / 32; ++d)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int row = 8 * jp + 4 * hl + q, col = 32 * d + 16 * ((lane >> 4) & 1) + 4 * pp;
        troff[d][jp] = lds_off<DP>(row, col >> 3) + ((col & 7) << 1);
      }
  }
  const int npass = CAUSAL && (nkb - 1 - p) != p ? 2 : 1;
  for (int pass = 0; pass < npass; ++pass) {
  const int kb = CAUSAL ? (pass == 0 ? p : nkb - 1 - p) : p;
  const int k0 = kb * 128;
  const int key = k0 + 32 * w + l32;  // this lane's key (MFMA column)
  const bool kvalid = key < Sk;
  if (pass > 0) {   // the ring and the column-sum scratch of the previous pass are free
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // K and V of this wave's 32 keys as B operands: lane holds K[key][16s + 8hl + j]
  bf16x8 kf[DP / 16], vf[DP / 16];
  const bf16_t* Krow = K + ((int64_t)b * Sk + key) * ks + (int64_t)hk * D;
  const bf16_t* Vrow = V + ((int64_t)b * Sk + key) * vs + (int64_t)hk * D;
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    kf[s] = __builtin_bit_cast(bf16x8, gload8(Krow, 16 * s + 8 * hl, D, kvalid));
    vf[s] = __builtin_bit_cast(bf16x8, gload8(Vrow, 16 * s + 8 * hl, D, kvalid));
  }
  f32x16 dk[DP / 32], dv[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) {
    dk[d] = {};
    dv[d] = {};
  }
  // first query that can see key k0: q >= k0 - shift
  const int q_begin = CAUSAL ? max(0, ((k0 - shift) / 64) * 64) : 0;
  const int ntq = (Sq - q_begin + 63) / 64;
  const int total = ntq * grp;

  // Q / dO tiles by buffer-load-to-LDS DMA (the forward v2 scheme): per-lane offsets fixed
  // here, the tile's row offset a scalar, one buffer resource per query head (rows past Sq
  // land as zeros); the loop below is unrolled over the ring, so LDS addresses are immediates
  auto issue_to = [&](int it, char* buf) {
    const int hq = hk * grp + it / ntq;
    const int q0 = q_begin + (it % ntq) * 64;
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Q + (int64_t)b * Sq * qs + (int64_t)hq * D), 0, (int)(((int64_t)(Sq - 1) * qs + D) * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(dO + (int64_t)b * Sq * os + (int64_t)hq * D), 0, (int)(((int64_t)(Sq - 1) * os + D) * 2), 0x00020000);
    qt.issue(qrs, (int)((int64_t)q0 * qs * 2), buf, w);
    gt2.issue(grs, (int)((int64_t)q0 * os * 2), buf + TILE, w);
    if (w == 0) {  // per-row stats, 4 bytes per lane (rows past Sq are masked in the math)
      const int q = min(q0 + lane, Sq - 1);
      const int64_t idx = ((int64_t)b * H + hq) * Sq + q;
      __builtin_amdgcn_global_load_lds((const void*)(LSE + idx),
                                       (__attribute__((address_space(3))) void*)(buf + 2 * TILE), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(DELTA + idx),
                                       (__attribute__((address_space(3))) void*)(buf + 2 * TILE + 256), 4, 0, 0);
    }
  };
  constexpr int PER_TILE = 2 * BTile<DP>::PPW;  // DMA instructions per tile per wave (+2 on wave 0)
#pragma unroll
  for (int i = 0; i < LOOK; ++i)
    if (i < total) issue_to(i, smem + i * BUFB);
  auto tile = [&](auto bufc, int it) {
    constexpr int BUF = decltype(bufc)::value;
    const int hq = hk * grp + it / ntq;
    const int q0 = q_begin + (it % ntq) * 64;
    const int bhq = b * H + hq;
    const DropKey dkey = drop_key(seed, (uint32_t)bhq);
    // tile `it` landed (up to LOOK-1 younger tiles may stay in flight), then publish to all
    // waves; wave 0 issues 2 extra DMAs per tile (the row stats)
    if (LOOK >= 3 && it + 2 < total) {
      if (w == 0) attn_wait_vmcnt<2 * (PER_TILE + 2)>(); else attn_wait_vmcnt<2 * PER_TILE>();
    } else if (LOOK >= 2 && it + 1 < total) {
      if (w == 0) attn_wait_vmcnt<PER_TILE + 2>(); else attn_wait_vmcnt<PER_TILE>();
    } else {
      attn_wait_vmcnt<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // the buffer of tile it-1 is free now: refill it with tile it+LOOK
    if (it + LOOK < total) issue_to(it + LOOK, smem + ((BUF + LOOK) % NBUF) * BUFB);
    const char* qb = smem + BUF * BUFB;
    const char* gb = qb + TILE;
    const float* ls = reinterpret_cast<const float*>(qb + 2 * TILE);
    const float* dl = ls + 64;
    const bool skip = CAUSAL && (k0 + 32 * w > q0 + 63 + shift);  // all of this wave's keys masked
    if (!skip) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // S[q][key] = Q K^T, dP[q][key] = dO V^T   (query rows u*32.. in registers, key on lane)
        f32x16 sacc = {}, pacc = {};
#pragma unroll
        for (int s = 0; s < DP / 16; ++s) {
          const bf16x8 aq = *reinterpret_cast<const bf16x8*>(qb + roff[s] + u * 32 * DP * 2);
          const bf16x8 ag = *reinterpret_cast<const bf16x8*>(gb + roff[s] + u * 32 * DP * 2);
          sacc = mfma32(aq, kf[s], sacc);
          pacc = mfma32(ag, vf[s], pacc);
        }
        f32x16 pm, ds;
        // per-row stats: rows 32u + 8g + 4hl + 0..3 are contiguous -> one 16-byte LDS read
        float4 lsv[4], dlv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          lsv[g] = *reinterpret_cast<const float4*>(ls + 32 * u + 8 * g + 4 * hl);
          dlv[g] = *reinterpret_cast<const float4*>(dl + 32 * u + 8 * g + 4 * hl);
        }
        // masks only where needed: the causal diagonal and query rows past Sq (their
        // stats were clamped); keys past Sk only feed their own unwritten outputs
        const bool edge = (q0 + 64 > Sq) || (CAUSAL && (k0 + 32 * w + 31 > q0 + 32 * u + shift));
        // the element math twice, masked and unmasked, behind one wave-uniform branch: as a
        // per-element select the mask's index compares and cndmasks were issued on every
        // tile (~half of the loop's VALU, profiles/r2_attention_pmc_counters.json)
        // dropout keep bits first (only the mask stays live across the hashes)
        uint32_t keep = 0xffffu;
        if (DROP) {
          keep = 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t q = (uint32_t)(q0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hl);
            keep |= (hash_lo(dkey, q * (uint32_t)Sk + (uint32_t)key) >= dthr ? 1u : 0u) << r;
          }
        }
        auto elems = [&](auto masked) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int qr = 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hl;
            const int q = q0 + qr;
            const float lv = (&lsv[r >> 2].x)[r & 3], dv_ = (&dlv[r >> 2].x)[r & 3];
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[r], c, -lv));
            if constexpr (decltype(masked)::value) {
              if (q >= Sq || (CAUSAL && key > q + shift)) p = 0.f;
            }
            float dpv = pacc[r];
            float pd = p;
            if (DROP) {
              const float msk = (keep >> r) & 1u ? dinv : 0.f;
              pd = p * msk;
              dpv = dpv * msk;
            }
            pm[r] = pd;                      // dropped P for dV
            ds[r] = p * (dpv - dv_);         // dS
          }
        };
        if (edge) elems(std::true_type{});
        else elems(std::false_type{});
        // dV^T += dO^T P ;  dK^T += Q^T dS     (A via transposed LDS reads of the row images)
        const bf16x8 pb0 = pack8(pm, 0), pb1 = pack8(pm, 1);
        const bf16x8 db0 = pack8(ds, 0), db1 = pack8(ds, 1);
#pragma unroll
        for (int d = 0; d < DP / 32; ++d) {
          auto tr = [&](const char* img, int jp, int m) {
            return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(img + troff[d][jp] + u * 32 * DP * 2 + 16 * DP * 2 * m));
          };
          dv[d] = mfma32(cat44(tr(gb, 0, 0), tr(gb, 1, 0)), pb0, dv[d]);
          dv[d] = mfma32(cat44(tr(gb, 0, 1), tr(gb, 1, 1)), pb1, dv[d]);
          dk[d] = mfma32(cat44(tr(qb, 0, 0), tr(qb, 1, 0)), db0, dk[d]);
          dk[d] = mfma32(cat44(tr(qb, 0, 1), tr(qb, 1, 1)), db1, dk[d]);
        }
      }
    }
  };
  for (int t0 = 0; t0 < total; t0 += NBUF) {
    tile(std::integral_constant<int, 0>{}, t0);
    if (t0 + 1 < total) tile(std::integral_constant<int, 1>{}, t0 + 1);
    if (t0 + 2 < total) tile(std::integral_constant<int, 2>{}, t0 + 2);
    if (t0 + 3 < total) tile(std::integral_constant<int, 3>{}, t0 + 3);
  }
  // ---- fused bias-gradient column sums of dK (scaled) and dV
  if (CSK != nullptr) {
    __syncthreads();   // the Q / dO ring is free
    float* red = reinterpret_cast<float*>(smem);
    wg_colsum_atomic<DP>(dk, scale, kvalid, red, CSK + (int64_t)hk * D, D);
    __syncthreads();
    wg_colsum_atomic<DP>(dv, 1.f, kvalid, red, CSV + (int64_t)hk * D, D);
  }
  // ---- epilogue: lane = key, registers = d
  if (kvalid) {
    bf16_t* dkrow = dK + ((int64_t)b * Sk + key) * dks + (int64_t)hk * D;
    bf16_t* dvrow = dV + ((int64_t)b * Sk + key) * dvs + (int64_t)hk * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 a, bb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] = f2bf(dk[d][4 * g + e] * scale);
            bb[e] = f2bf(dv[d][4 * g + e]);
          }
          *reinterpret_cast<u16x4*>(dkrow + col) = a;
          *reinterpret_cast<u16x4*>(dvrow + col) = bb;
        }
      }
    }
  }
  }
}

// ==========================================================================================
// backward dQ: workgroup = 128 queries of one (b, h) (forward structure)
// ==========================================================================================
template <int DP, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, DP <= 64 ? 2 : 1) attn_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    float* __restrict__ DELTA,
    bf16_t* __restrict__ dQ, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs,
    int64_t os, int64_t dqs, float scale, float p_drop, uint64_t seed, float* __restrict__ CSQ) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
#define kbuf(i) (smem + (i) * TILE)
#define vbuf(i) (smem + (2 + (i)) * TILE)
  const int nmb = (Sq + 127) / 128;
  // causal: longest-first over the whole grid (see attn_fwd_kernel)
  const int lin = (int)blockIdx.x + (int)gridDim.x * (int)blockIdx.y;
  const int nbh = (int)gridDim.y;
  const int mb = CAUSAL ? (nmb - 1 - lin / nbh) : (int)blockIdx.x;
  const int bh = CAUSAL ? lin % nbh : (int)blockIdx.y;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, l32 = lane & 31;
  const int m0 = mb * 128;
  const int qrow = m0 + 32 * w + l32;
  const bool qvalid = qrow < Sq;
  const int shift = Sk - Sq;
  const bf16_t* Kb = K + (int64_t)b * Sk * ks + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * Sk * vs + (int64_t)hk * D;
  bf16x8 qf[DP / 16], gf[DP / 16];
  const bf16_t* Qrow = Q + ((int64_t)b * Sq + qrow) * qs + (int64_t)h * D;
  const bf16_t* Grow = dO + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    qf[s] = __builtin_bit_cast(bf16x8, gload8(Qrow, 16 * s + 8 * hl, D, qvalid));
    gf[s] = __builtin_bit_cast(bf16x8, gload8(Grow, 16 * s + 8 * hl, D, qvalid));
  }
  const int64_t sidx = (int64_t)bh * Sq + qrow;
  const float lse = qvalid ? LSE[sidx] : INFINITY;
  // delta = rowsum(dO * O), fused here (each lane holds half of the row's d range)
  float dlt = 0.f;
  {
    const bf16_t* Orow = O + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) {
      const u16x8 ov = gload8(Orow, 16 * s + 8 * hl, D, qvalid);
      const bf16x8 g = gf[s];
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += bf2f(ov[j]) * (float)g[j];
    }
    dlt += __shfl_xor(dlt, 32, 64);
    if (qvalid && hl == 0) DELTA[sidx] = dlt;
  }
  const float c = scale * LOG2E;
  const DropKey dkey = drop_key(seed, (uint32_t)bh);
  const uint32_t dthr = drop_thr(p_drop), qoff = (uint32_t)qrow * (uint32_t)Sk;
  const float dinv = 1.0f / (1.0f - p_drop);
  f32x16 dq[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) dq[d] = {};
  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + 128 + shift);
  const int ntiles = (n_end + 63) / 64;
  // K / V tiles stream through an NBUF-deep LDS ring by LDS-DMA (the dK/dV kernel's
  // scheme): LOOK tiles in flight, counted vmcnt, one raw barrier per tile
  constexpr int NBUF = DP <= 128 ? 4 : 2;
  constexpr int LOOK = NBUF - 1;
  constexpr int BUFB = 2 * TILE;
  using GT = GTile<DP>;
  constexpr int PER_TILE = 2 * GT::PPW;
  GT gt;
  gt.init();
  const int wv = __builtin_amdgcn_readfirstlane(w);
  auto issue = [&](int t) {
    char* buf = smem + (t % NBUF) * BUFB;
    gt.issue(Kb, ks, t * 64, Sk, D, buf, wv);
    gt.issue(Vb, vs, t * 64, Sk, D, buf + TILE, wv);
  };
#pragma unroll
  for (int i = 0; i < LOOK; ++i)
    if (i < ntiles) issue(i);
  const int wave_last_q = m0 + 32 * w + 31 + shift;
  for (int t = 0; t < ntiles; ++t) {
    const int n0 = t * 64;
    if (LOOK >= 3 && t + 2 < ntiles) attn_wait_vmcnt<2 * PER_TILE>();
    else if (LOOK >= 2 && t + 1 < ntiles) attn_wait_vmcnt<PER_TILE>();
    else attn_wait_vmcnt<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // every wave is done with tile t-1: its buffer takes tile t+LOOK
    if (t + LOOK < ntiles) issue(t + LOOK);
    if (!(CAUSAL && n0 > wave_last_q)) {
      const char* kb = smem + (t % NBUF) * BUFB;
      const char* vb = kb + TILE;
      f32x16 s0 = {}, s1 = {}, p0 = {}, p1 = {};
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        bf16x8 ak0 = lds_row8<DP>(kb, l32, 2 * s + hl);
        bf16x8 ak1 = lds_row8<DP>(kb, 32 + l32, 2 * s + hl);
        bf16x8 av0 = lds_row8<DP>(vb, l32, 2 * s + hl);
        bf16x8 av1 = lds_row8<DP>(vb, 32 + l32, 2 * s + hl);
        s0 = mfma32(ak0, qf[s], s0);
        s1 = mfma32(ak1, qf[s], s1);
        p0 = mfma32(av0, gf[s], p0);  // dP^T = V dO^T
        p1 = mfma32(av1, gf[s], p1);
      }
      // causal / key-end mask only on edge tiles; invalid query rows have lse = +inf
      const bool edge = (n0 + 64 > Sk) || (CAUSAL && n0 + 63 > m0 + 32 * w + shift);
      // masked / unmasked element math behind one wave-uniform branch (see the dK/dV kernel)
      // dropout keep bits first (only the mask stays live across the hashes)
      uint32_t keep = 0xffffffffu;
      if (DROP) {
        keep = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t kr = (uint32_t)(n0 + (r & 3) + 8 * (r >> 2) + 4 * hl);
          keep |= (hash_lo(dkey, qoff + kr) >= dthr ? 1u : 0u) << r;
          keep |= (hash_lo(dkey, qoff + kr + 32u) >= dthr ? 1u : 0u) << (16 + r);
        }
      }
      auto elems = [&](auto masked) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kr = (r & 3) + 8 * (r >> 2) + 4 * hl;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int kk = n0 + 32 * half + kr;
            float sv = half ? s1[r] : s0[r];
            float dpv = half ? p1[r] : p0[r];
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -lse));
            if constexpr (decltype(masked)::value) {
              if (kk >= Sk || (CAUSAL && kk > qrow + shift)) p = 0.f;
            }
            if (DROP) dpv = (keep >> (16 * half + r)) & 1u ? dpv * dinv : 0.f;
            const float dsv = p * (dpv - dlt);
            if (half) s1[r] = dsv; else s0[r] = dsv;
          }
        }
      };
      if (edge) elems(std::true_type{});
      else elems(std::false_type{});
      const bf16x8 d00 = pack8(s0, 0), d01 = pack8(s0, 1), d10 = pack8(s1, 0), d11 = pack8(s1, 1);
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
        const int c0 = 32 * d + 16 * ((lane >> 4) & 1);
        bf16x8 a;
        a = cat44(lds_tr4<DP>(kb, 0 + 4 * hl, c0), lds_tr4<DP>(kb, 8 + 4 * hl, c0));
        dq[d] = mfma32(a, d00, dq[d]);
        a = cat44(lds_tr4<DP>(kb, 16 + 4 * hl, c0), lds_tr4<DP>(kb, 24 + 4 * hl, c0));
        dq[d] = mfma32(a, d01, dq[d]);
        a = cat44(lds_tr4<DP>(kb, 32 + 4 * hl, c0), lds_tr4<DP>(kb, 40 + 4 * hl, c0));
        dq[d] = mfma32(a, d10, dq[d]);
        a = cat44(lds_tr4<DP>(kb, 48 + 4 * hl, c0), lds_tr4<DP>(kb, 56 + 4 * hl, c0));
        dq[d] = mfma32(a, d11, dq[d]);
      }
    }
  }
  if (CSQ != nullptr) {
    __syncthreads();   // K / V tiles no longer read
    wg_colsum_atomic<DP>(dq, scale, qvalid, reinterpret_cast<float*>(smem), CSQ + (int64_t)h * D, D);
  }
  if (qvalid) {
    bf16_t* drow = dQ + ((int64_t)b * Sq + qrow) * dqs + (int64_t)h * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = f2bf(dq[d][4 * g + e] * scale);
          *reinterpret_cast<u16x4*>(drow + col) = pk;
        }
      }
    }
  }
}

// backward dQ v2 (d_h 64, the default): attn_bwd_dq_kernel's math on the forward v2 tile
// machinery -- buffer-load-to-LDS K/V ring with entry-time lane offsets, the tile loop
// unrolled over the 4-deep ring (immediate LDS offsets), one-compare masks
template <int DP, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, 2) attn_bwd_dq2_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    float* __restrict__ DELTA,
    bf16_t* __restrict__ dQ, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs,
    int64_t os, int64_t dqs, float scale, float p_drop, uint64_t seed, float* __restrict__ CSQ) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
#define kbuf(i) (smem + (i) * TILE)
#define vbuf(i) (smem + (2 + (i)) * TILE)
  const int nmb = (Sq + 127) / 128;
  // causal: longest-first over the whole grid (see attn_fwd_kernel)
  const int lin = (int)blockIdx.x + (int)gridDim.x * (int)blockIdx.y;
  const int nbh = (int)gridDim.y;
  const int mb = CAUSAL ? (nmb - 1 - lin / nbh) : (int)blockIdx.x;
  const int bh = CAUSAL ? lin % nbh : (int)blockIdx.y;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, l32 = lane & 31;
  const int m0 = mb * 128;
  const int qrow = m0 + 32 * w + l32;
  const bool qvalid = qrow < Sq;
  const int shift = Sk - Sq;
  const bf16_t* Kb = K + (int64_t)b * Sk * ks + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * Sk * vs + (int64_t)hk * D;
  bf16x8 qf[DP / 16], gf[DP / 16];
  const bf16_t* Qrow = Q + ((int64_t)b * Sq + qrow) * qs + (int64_t)h * D;
  const bf16_t* Grow = dO + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    qf[s] = __builtin_bit_cast(bf16x8, gload8(Qrow, 16 * s + 8 * hl, D, qvalid));
    gf[s] = __builtin_bit_cast(bf16x8, gload8(Grow, 16 * s + 8 * hl, D, qvalid));
  }
  const int64_t sidx = (int64_t)bh * Sq + qrow;
  const float lse = qvalid ? LSE[sidx] : INFINITY;
  // delta = rowsum(dO * O), fused here (each lane holds half of the row's d range)
  float dlt = 0.f;
  {
    const bf16_t* Orow = O + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) {
      const u16x8 ov = gload8(Orow, 16 * s + 8 * hl, D, qvalid);
      const bf16x8 g = gf[s];
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += bf2f(ov[j]) * (float)g[j];
    }
    dlt += __shfl_xor(dlt, 32, 64);
    if (qvalid && hl == 0) DELTA[sidx] = dlt;
  }
  const float c = scale * LOG2E;
  const DropKey dkey = drop_key(seed, (uint32_t)bh);
  const uint32_t dthr = drop_thr(p_drop), qoff = (uint32_t)qrow * (uint32_t)Sk;
  const float dinv = 1.0f / (1.0f - p_drop);
  f32x16 dq[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) dq[d] = {};
  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + 128 + shift);
  const int ntiles = (n_end + 63) / 64;
  // K / V tiles stream through an NBUF-deep LDS ring by LDS-DMA (the dK/dV kernel's
  // scheme): LOOK tiles in flight, counted vmcnt, one raw barrier per tile
  // K / V ring (the forward v2 scheme): NBUF buffers, LOOK tiles in flight, buffer-load-to-LDS
  // DMA with per-lane offsets fixed here and a scalar tile offset; the tile loop is unrolled
  // over the ring so every LDS address is an immediate
  constexpr int NBUF = 4, LOOK = NBUF - 1, BUFB = 2 * TILE;
  constexpr int PER_TILE = 2 * BTile<DP>::PPW;
  const int wv = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t krs =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kb, 0, (int)(((int64_t)(Sk - 1) * ks + D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vb, 0, (int)(((int64_t)(Sk - 1) * vs + D) * 2), 0x00020000);
  BTile<DP> kt, vt;
  kt.init(ks, D, wv);
  vt.init(vs, D, wv);
  const int kstep = (int)(64 * ks * 2), vstep = (int)(64 * vs * 2);
  auto issue_to = [&](int t, char* buf) {
    kt.issue(krs, t * kstep, buf, wv);
    vt.issue(vrs, t * vstep, buf + TILE, wv);
  };
  int koff[DP / 16], ktoff[DP / 32][2];   // (see attn_fwd2_kernel)
  {
    const int i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) koff[s] = lds_off<DP>(l32, 2 * s + hl);
#pragma unroll
    for (int d = 0; d < DP / 32; ++d)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int row = 8 * jp + 4 * hl + q, col = 32 * d + 16 * ((lane >> 4) & 1) + 4 * pp;
        ktoff[d][jp] = lds_off<DP>(row, col >> 3) + ((col & 7) << 1);
      }
  }
  // per-lane mask limit (see attn_fwd2_kernel): key k (+4 hl) of a tile at n0 is kept iff k <= lim0 - n0
  const int lim0 = (CAUSAL ? min(qrow + shift, Sk - 1) : Sk - 1) - 4 * hl;
#pragma unroll
  for (int i = 0; i < LOOK; ++i)
    if (i < ntiles) issue_to(i, smem + i * BUFB);
  const int wave_last_q = m0 + 32 * w + 31 + shift;
  auto tile = [&](auto bufc, int t) {
    constexpr int BUF = decltype(bufc)::value;
    const int n0 = t * 64;
    if (t + 2 < ntiles) attn_wait_vmcnt<2 * PER_TILE>();
    else if (t + 1 < ntiles) attn_wait_vmcnt<PER_TILE>();
    else attn_wait_vmcnt<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // every wave is done with tile t-1: its buffer takes tile t+LOOK
    if (t + LOOK < ntiles) issue_to(t + LOOK, smem + ((BUF + LOOK) % NBUF) * BUFB);
    if (!(CAUSAL && n0 > wave_last_q)) {
      const char* kb = smem + BUF * BUFB;
      const char* vb = kb + TILE;
      f32x16 s0 = {}, s1 = {}, p0 = {}, p1 = {};
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        const bf16x8 ak0 = *reinterpret_cast<const bf16x8*>(kb + koff[s]);
        const bf16x8 ak1 = *reinterpret_cast<const bf16x8*>(kb + koff[s] + 32 * DP * 2);
        const bf16x8 av0 = *reinterpret_cast<const bf16x8*>(vb + koff[s]);
        const bf16x8 av1 = *reinterpret_cast<const bf16x8*>(vb + koff[s] + 32 * DP * 2);
        s0 = mfma32(ak0, qf[s], s0);
        s1 = mfma32(ak1, qf[s], s1);
        p0 = mfma32(av0, gf[s], p0);  // dP^T = V dO^T
        p1 = mfma32(av1, gf[s], p1);
      }
      // causal / key-end mask only on edge tiles; invalid query rows have lse = +inf
      const bool edge = (n0 + 64 > Sk) || (CAUSAL && n0 + 63 > m0 + 32 * w + shift);
      // masked / unmasked element math behind one wave-uniform branch (see the dK/dV kernel)
      // dropout keep bits first (only the mask stays live across the hashes)
      uint32_t keep = 0xffffffffu;
      if (DROP) {
        keep = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t kr = (uint32_t)(n0 + (r & 3) + 8 * (r >> 2) + 4 * hl);
          keep |= (hash_lo(dkey, qoff + kr) >= dthr ? 1u : 0u) << r;
          keep |= (hash_lo(dkey, qoff + kr + 32u) >= dthr ? 1u : 0u) << (16 + r);
        }
      }
      auto elems = [&](auto masked) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kr = (r & 3) + 8 * (r >> 2) + 4 * hl;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int kk = n0 + 32 * half + kr;
            float sv = half ? s1[r] : s0[r];
            float dpv = half ? p1[r] : p0[r];
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -lse));
            if constexpr (decltype(masked)::value) {
              if (key_of(r) + 32 * half > lim0 - n0) p = 0.f;
            }
            if (DROP) dpv = (keep >> (16 * half + r)) & 1u ? dpv * dinv : 0.f;
            const float dsv = p * (dpv - dlt);
            if (half) s1[r] = dsv; else s0[r] = dsv;
          }
        }
      };
      if (edge) elems(std::true_type{});
      else elems(std::false_type{});
      const bf16x8 d00 = pack8(s0, 0), d01 = pack8(s0, 1), d10 = pack8(s1, 0), d11 = pack8(s1, 1);
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
        auto tr = [&](int jp, int m) {
          return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(kb + ktoff[d][jp] + 16 * DP * 2 * m));
        };
        dq[d] = mfma32(cat44(tr(0, 0), tr(1, 0)), d00, dq[d]);
        dq[d] = mfma32(cat44(tr(0, 1), tr(1, 1)), d01, dq[d]);
        dq[d] = mfma32(cat44(tr(0, 2), tr(1, 2)), d10, dq[d]);
        dq[d] = mfma32(cat44(tr(0, 3), tr(1, 3)), d11, dq[d]);
      }
    }
  };
  for (int t0 = 0; t0 < ntiles; t0 += NBUF) {
    tile(std::integral_constant<int, 0>{}, t0);
    if (t0 + 1 < ntiles) tile(std::integral_constant<int, 1>{}, t0 + 1);
    if (t0 + 2 < ntiles) tile(std::integral_constant<int, 2>{}, t0 + 2);
    if (t0 + 3 < ntiles) tile(std::integral_constant<int, 3>{}, t0 + 3);
  }
  if (CSQ != nullptr) {
    __syncthreads();   // K / V tiles no longer read
    wg_colsum_atomic<DP>(dq, scale, qvalid, reinterpret_cast<float*>(smem), CSQ + (int64_t)h * D, D);
  }
  if (qvalid) {
    bf16_t* drow = dQ + ((int64_t)b * Sq + qrow) * dqs + (int64_t)h * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = f2bf(dq[d][4 * g + e] * scale);
          *reinterpret_cast<u16x4*>(drow + col) = pk;
        }
      }
    }
  }
}

// dQ v3 (the default; MIPIPE_ATTN_BWD_DQ=2 selects v2): v2 with paired causal query blocks on
// one XCD
template <int DP, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, 2) attn_bwd_dq3_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    float* __restrict__ DELTA,
    bf16_t* __restrict__ dQ, int B, int Sq, int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs,
    int64_t os, int64_t dqs, float scale, float p_drop, uint64_t seed, float* __restrict__ CSQ) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
  const int nmb = (Sq + 127) / 128;
  // causal: one workgroup runs query block nmb-1-p and then block p of the same (b, h), the
  // pairs of one (b, h) consecutive on one XCD (the forward v2 mapping)
  const int npair = CAUSAL ? (nmb + 1) / 2 : nmb;
  const int nbh = B * H;
  const int lin = (int)blockIdx.x;
  int bh, p;
  if ((nbh & 7) == 0) {
    const int xcd = lin & 7, j = lin >> 3;
    bh = (j / npair) * 8 + xcd;
    p = j % npair;
  } else {
    bh = lin / npair;
    p = lin % npair;
  }
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, l32 = lane & 31;
  const int npass = CAUSAL && (nmb - 1 - p) != p ? 2 : 1;
  for (int pass = 0; pass < npass; ++pass) {
  const int mb = CAUSAL ? (pass == 0 ? nmb - 1 - p : p) : p;
  if (pass > 0) {   // the ring and the column-sum scratch of the previous pass are free
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  const int m0 = mb * 128;
  const int qrow = m0 + 32 * w + l32;
  const bool qvalid = qrow < Sq;
  const int shift = Sk - Sq;
  const bf16_t* Kb = K + (int64_t)b * Sk * ks + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * Sk * vs + (int64_t)hk * D;
  bf16x8 qf[DP / 16], gf[DP / 16];
  const bf16_t* Qrow = Q + ((int64_t)b * Sq + qrow) * qs + (int64_t)h * D;
  const bf16_t* Grow = dO + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    qf[s] = __builtin_bit_cast(bf16x8, gload8(Qrow, 16 * s + 8 * hl, D, qvalid));
    gf[s] = __builtin_bit_cast(bf16x8, gload8(Grow, 16 * s + 8 * hl, D, qvalid));
  }
  const int64_t sidx = (int64_t)bh * Sq + qrow;
  const float lse = qvalid ? LSE[sidx] : INFINITY;
  // delta = rowsum(dO * O), fused here (each lane holds half of the row's d range)
  float dlt = 0.f;
  {
    const bf16_t* Orow = O + ((int64_t)b * Sq + qrow) * os + (int64_t)h * D;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) {
      const u16x8 ov = gload8(Orow, 16 * s + 8 * hl, D, qvalid);
      const bf16x8 g = gf[s];
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += bf2f(ov[j]) * (float)g[j];
    }
    dlt += __shfl_xor(dlt, 32, 64);
    if (qvalid && hl == 0) DELTA[sidx] = dlt;
  }
  const float c = scale * LOG2E;
  const DropKey dkey = drop_key(seed, (uint32_t)bh);
  const uint32_t dthr = drop_thr(p_drop), qoff = (uint32_t)qrow * (uint32_t)Sk;
  const float dinv = 1.0f / (1.0f - p_drop);
  f32x16 dq[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) dq[d] = {};
  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + 128 + shift);
  const int ntiles = (n_end + 63) / 64;
  // K / V tiles stream through an NBUF-deep LDS ring by LDS-DMA (the dK/dV kernel's
  // scheme): LOOK tiles in flight, counted vmcnt, one raw barrier per tile
  // K / V ring (the forward v2 scheme): NBUF buffers, LOOK tiles in flight, buffer-load-to-LDS
  // DMA with per-lane offsets fixed here and a scalar tile offset; the tile loop is unrolled
  // over the ring so every LDS address is an immediate
  constexpr int NBUF = 4, LOOK = NBUF - 1, BUFB = 2 * TILE;
  constexpr int PER_TILE = 2 * BTile<DP>::PPW;
  const int wv = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t krs =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kb, 0, (int)(((int64_t)(Sk - 1) * ks + D) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vb, 0, (int)(((int64_t)(Sk - 1) * vs + D) * 2), 0x00020000);
  BTile<DP> kt, vt;
  kt.init(ks, D, wv);
  vt.init(vs, D, wv);
  const int kstep = (int)(64 * ks * 2), vstep = (int)(64 * vs * 2);
  auto issue_to = [&](int t, char* buf) {
    kt.issue(krs, t * kstep, buf, wv);
    vt.issue(vrs, t * vstep, buf + TILE, wv);
  };
  int koff[DP / 16], ktoff[DP / 32][2];   // (see attn_fwd2_kernel)
  {
    const int i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) koff[s] = lds_off<DP>(l32, 2 * s + hl);
#pragma unroll
    for (int d = 0; d < DP / 32; ++d)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int row = 8 * jp + 4 * hl + q, col = 32 * d + 16 * ((lane >> 4) & 1) + 4 * pp;
        ktoff[d][jp] = lds_off<DP>(row, col >> 3) + ((col & 7) << 1);
      }
  }
  // per-lane mask limit (see attn_fwd2_kernel): key k (+4 hl) of a tile at n0 is kept iff k <= lim0 - n0
  const int lim0 = (CAUSAL ? min(qrow + shift, Sk - 1) : Sk - 1) - 4 * hl;
#pragma unroll
  for (int i = 0; i < LOOK; ++i)
    if (i < ntiles) issue_to(i, smem + i * BUFB);
  const int wave_last_q = m0 + 32 * w + 31 + shift;
  auto tile = [&](auto bufc, int t) {
    constexpr int BUF = decltype(bufc)::value;
    const int n0 = t * 64;
    if (t + 2 < ntiles) attn_wait_vmcnt<2 * PER_TILE>();
    else if (t + 1 < ntiles) attn_wait_vmcnt<PER_TILE>();
    else attn_wait_vmcnt<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // every wave is done with tile t-1: its buffer takes tile t+LOOK
    if (t + LOOK < ntiles) issue_to(t + LOOK, smem + ((BUF + LOOK) % NBUF) * BUFB);
    if (!(CAUSAL && n0 > wave_last_q)) {
      const char* kb = smem + BUF * BUFB;
      const char* vb = kb + TILE;
      f32x16 s0 = {}, s1 = {}, p0 = {}, p1 = {};
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        const bf16x8 ak0 = *reinterpret_cast<const bf16x8*>(kb + koff[s]);
        const bf16x8 ak1 = *reinterpret_cast<const bf16x8*>(kb + koff[s] + 32 * DP * 2);
        const bf16x8 av0 = *reinterpret_cast<const bf16x8*>(vb + koff[s]);
        const bf16x8 av1 = *reinterpret_cast<const bf16x8*>(vb + koff[s] + 32 * DP * 2);
        s0 = mfma32(ak0, qf[s], s0);
        s1 = mfma32(ak1, qf[s], s1);
        p0 = mfma32(av0, gf[s], p0);  // dP^T = V dO^T
        p1 = mfma32(av1, gf[s], p1);
      }
      // causal / key-end mask only on edge tiles; invalid query rows have lse = +inf
      const bool edge = (n0 + 64 > Sk) || (CAUSAL && n0 + 63 > m0 + 32 * w + shift);
      // masked / unmasked element math behind one wave-uniform branch (see the dK/dV kernel)
      // dropout keep bits first (only the mask stays live across the hashes)
      uint32_t keep = 0xffffffffu;
      if (DROP) {
        keep = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t kr = (uint32_t)(n0 + (r & 3) + 8 * (r >> 2) + 4 * hl);
          keep |= (hash_lo(dkey, qoff + kr) >= dthr ? 1u : 0u) << r;
          keep |= (hash_lo(dkey, qoff + kr + 32u) >= dthr ? 1u : 0u) << (16 + r);
        }
      }
      auto elems = [&](auto masked) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kr = (r & 3) + 8 * (r >> 2) + 4 * hl;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int kk = n0 + 32 * half + kr;
            float sv = half ? s1[r] : s0[r];
            float dpv = half ? p1[r] : p0[r];
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -lse));
            if constexpr (decltype(masked)::value) {
              if (key_of(r) + 32 * half > lim0 - n0) p = 0.f;
            }
            if (DROP) dpv = (keep >> (16 * half + r)) & 1u ? dpv * dinv : 0.f;
            const float dsv = p * (dpv - dlt);
            if (half) s1[r] = dsv; else s0[r] = dsv;
          }
        }
      };
      if (edge) elems(std::true_type{});
      else elems(std::false_type{});
      const bf16x8 d00 = pack8(s0, 0), d01 = pack8(s0, 1), d10 = pack8(s1, 0), d11 = pack8(s1, 1);
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
        auto tr = [&](int jp, int m) {
          return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(kb + ktoff[d][jp] + 16 * DP * 2 * m));
        };
        dq[d] = mfma32(cat44(tr(0, 0), tr(1, 0)), d00, dq[d]);
        dq[d] = mfma32(cat44(tr(0, 1), tr(1, 1)), d01, dq[d]);
        dq[d] = mfma32(cat44(tr(0, 2), tr(1, 2)), d10, dq[d]);
        dq[d] = mfma32(cat44(tr(0, 3), tr(1, 3)), d11, dq[d]);
      }
    }
  };
  for (int t0 = 0; t0 < ntiles; t0 += NBUF) {
    tile(std::integral_constant<int, 0>{}, t0);
    if (t0 + 1 < ntiles) tile(std::integral_constant<int, 1>{}, t0 + 1);
    if (t0 + 2 < ntiles) tile(std::integral_constant<int, 2>{}, t0 + 2);
    if (t0 + 3 < ntiles) tile(std::integral_constant<int, 3>{}, t0 + 3);
  }
  if (CSQ != nullptr) {
    __syncthreads();   // K / V tiles no longer read
    wg_colsum_atomic<DP>(dq, scale, qvalid, reinterpret_cast<float*>(smem), CSQ + (int64_t)h * D, D);
  }
  if (qvalid) {
    bf16_t* drow = dQ + ((int64_t)b * Sq + qrow) * dqs + (int64_t)h * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = f2bf(dq[d][4 * g + e] * scale);
          *reinterpret_cast<u16x4*>(drow + col) = pk;
        }
      }
    }
  }
  }
}

#undef kbuf
#undef vbuf

// ==========================================================================================
// backward, short non-causal sequences (Sq, Sk <= 128): dQ and dK/dV workgroups in ONE grid
// ==========================================================================================
// At the reference's shape (B 8, S 128, H 8, d_h 96) the two kernels above are 64
// workgroups each for 256 CUs, run back to back (dK/dV reads the delta the dQ kernel
// writes), and every wave walks both 64-row tiles serially.  Here one launch holds both
// roles, each on 64-row blocks with the other dimension split over two wave pairs:
//   blockIdx.x <  nq: dQ of 64 queries.  Wave (qsub = w & 1: which 32 queries, half =
//                     w >> 1: which 64-key tile) -- the half = 1 pair's partial dQ is added
//                     to the half = 0 pair's through LDS.
//   blockIdx.x >= nq: dK / dV of 64 keys.  Wave (ksub = w & 1: which 32 keys, half: which
//                     64-query tile); partial dK / dV added the same way.
// Both roles compute delta = rowsum(dO * O) themselves (the dK/dV pairs stream the O tile
// beside Q / dO and reduce it in LDS), so the roles are independent: 4x the workgroups of
// one kernel above in one launch, and no serial tile chain.  One tile per pair: every
// buffer is loaded once (LDS-DMA, the GTileP scheme), no ring.  The math per tile is the
// two kernels' (same dropout indices, same masks).  Non-causal, H == Hkv, d_h <= 128 (at
// d_h 256 -- the O slot of the dK/dV pairs refilled with Q after delta, 129 KB of LDS --
// the two roles' registers spill 69 VGPRs, so the launcher keeps the two-kernel path).
template <int DP, bool DROP>
__global__ void __launch_bounds__(256, 1) attn_bwd_short_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    bf16_t* __restrict__ dQ, bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int Sq, int Sk, int H, int D,
    int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dqs, int64_t dks, int64_t dvs, float scale, float p_drop,
    uint64_t seed, float* __restrict__ CSQ, float* __restrict__ CSK, float* __restrict__ CSV) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE = 64 * DP * 2;
  constexpr bool SEQ_O = DP > 128;     // O and Q share one slot (delta first)
  const int bh = (int)blockIdx.y;
  const int b = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, l32 = lane & 31;
  const int sub = w & 1, half = w >> 1;
  const int nq = (Sq + 63) / 64;
  const float c = scale * LOG2E;
  const DropKey dkey = drop_key(seed, (uint32_t)bh);
  const uint32_t dthr = drop_thr(p_drop);
  const float dinv = 1.0f / (1.0f - p_drop);
  GTileP<DP> gp;
  gp.init();
  const int wv = __builtin_amdgcn_readfirstlane(sub);
  const bf16_t* Qb = Q + (int64_t)b * Sq * qs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * Sk * ks + (int64_t)h * D;
  const bf16_t* Vb = V + (int64_t)b * Sk * vs + (int64_t)h * D;
  const bf16_t* Ob = O + (int64_t)b * Sq * os + (int64_t)h * D;
  const bf16_t* Gb = dO + (int64_t)b * Sq * os + (int64_t)h * D;

  if ((int)blockIdx.x < nq) {
    // =================================== dQ role ===================================
    const int m0 = (int)blockIdx.x * 64;
    const int qrow = m0 + 32 * sub + l32;
    const bool qvalid = qrow < Sq;
    const int n0 = 64 * half;                 // this pair's key tile
    char* kb = smem + half * 2 * TILE;
    char* vb = kb + TILE;
    if (n0 < Sk) {
      gp.issue(Kb, ks, n0, Sk, D, kb, wv);
      gp.issue(Vb, vs, n0, Sk, D, vb, wv);
    }
    bf16x8 qf[DP / 16], gf[DP / 16];
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) {
      qf[s] = __builtin_bit_cast(bf16x8, gload8(Qb + (int64_t)qrow * qs, 16 * s + 8 * hl, D, qvalid));
      gf[s] = __builtin_bit_cast(bf16x8, gload8(Gb + (int64_t)qrow * os, 16 * s + 8 * hl, D, qvalid));
    }
    const float lse = qvalid ? LSE[(int64_t)bh * Sq + qrow] : INFINITY;
    float dlt = 0.f;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) {
      const u16x8 ov = gload8(Ob + (int64_t)qrow * os, 16 * s + 8 * hl, D, qvalid);
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += bf2f(ov[j]) * (float)gf[s][j];
    }
    dlt += __shfl_xor(dlt, 32, 64);
    const uint32_t qoff = (uint32_t)qrow * (uint32_t)Sk;
    f32x16 dq[DP / 32];
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) dq[d] = {};
    __syncthreads();   // (waits for this wave's LDS-DMA first: the pair's K / V tile is in LDS)
    if (n0 < Sk) {
      f32x16 s0 = {}, s1 = {}, p0 = {}, p1 = {};
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        bf16x8 ak0 = lds_row8<DP>(kb, l32, 2 * s + hl);
        bf16x8 ak1 = lds_row8<DP>(kb, 32 + l32, 2 * s + hl);
        bf16x8 av0 = lds_row8<DP>(vb, l32, 2 * s + hl);
        bf16x8 av1 = lds_row8<DP>(vb, 32 + l32, 2 * s + hl);
        s0 = mfma32(ak0, qf[s], s0);
        s1 = mfma32(ak1, qf[s], s1);
        p0 = mfma32(av0, gf[s], p0);
        p1 = mfma32(av1, gf[s], p1);
      }
      uint32_t keep = 0xffffffffu;
      if (DROP) {
        keep = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t kr = (uint32_t)(n0 + (r & 3) + 8 * (r >> 2) + 4 * hl);
          keep |= (hash_lo(dkey, qoff + kr) >= dthr ? 1u : 0u) << r;
          keep |= (hash_lo(dkey, qoff + kr + 32u) >= dthr ? 1u : 0u) << (16 + r);
        }
      }
      auto elems = [&](auto masked) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kr = (r & 3) + 8 * (r >> 2) + 4 * hl;
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            float sv = hf ? s1[r] : s0[r];
            float dpv = hf ? p1[r] : p0[r];
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -lse));
            if constexpr (decltype(masked)::value) {
              if (n0 + 32 * hf + kr >= Sk) p = 0.f;
            }
            if (DROP) dpv = (keep >> (16 * hf + r)) & 1u ? dpv * dinv : 0.f;
            const float dsv = p * (dpv - dlt);
            if (hf) s1[r] = dsv; else s0[r] = dsv;
          }
        }
      };
      if (n0 + 64 > Sk) elems(std::true_type{});
      else elems(std::false_type{});
      const bf16x8 d00 = pack8(s0, 0), d01 = pack8(s0, 1), d10 = pack8(s1, 0), d11 = pack8(s1, 1);
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
        const int c0 = 32 * d + 16 * ((lane >> 4) & 1);
        bf16x8 a;
        a = cat44(lds_tr4<DP>(kb, 0 + 4 * hl, c0), lds_tr4<DP>(kb, 8 + 4 * hl, c0));
        dq[d] = mfma32(a, d00, dq[d]);
        a = cat44(lds_tr4<DP>(kb, 16 + 4 * hl, c0), lds_tr4<DP>(kb, 24 + 4 * hl, c0));
        dq[d] = mfma32(a, d01, dq[d]);
        a = cat44(lds_tr4<DP>(kb, 32 + 4 * hl, c0), lds_tr4<DP>(kb, 40 + 4 * hl, c0));
        dq[d] = mfma32(a, d10, dq[d]);
        a = cat44(lds_tr4<DP>(kb, 48 + 4 * hl, c0), lds_tr4<DP>(kb, 56 + 4 * hl, c0));
        dq[d] = mfma32(a, d11, dq[d]);
      }
    }
    // the half = 1 pair hands its partial dQ^T to the half = 0 pair
    __syncthreads();
    float* xo = reinterpret_cast<float*>(smem) + sub * (DP / 32 * 16 * 64);
    if (half == 1) {
#pragma unroll
      for (int d = 0; d < DP / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) xo[(d * 16 + r) * 64 + lane] = dq[d][r];
    }
    __syncthreads();
    if (half == 0) {
#pragma unroll
      for (int d = 0; d < DP / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[d][r] += xo[(d * 16 + r) * 64 + lane];
    }
    if (CSQ != nullptr) {
      __syncthreads();   // the hand-off area is free
      wg_colsum_atomic<DP>(dq, scale, qvalid && half == 0, reinterpret_cast<float*>(smem), CSQ + (int64_t)h * D, D);
    }
    if (qvalid && half == 0) {
      bf16_t* drow = dQ + ((int64_t)b * Sq + qrow) * dqs + (int64_t)h * D;
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = 32 * d + 8 * g + 4 * hl;
          if (col < D) {
            u16x4 pk;
#pragma unroll
            for (int e = 0; e < 4; ++e) pk[e] = f2bf(dq[d][4 * g + e] * scale);
            *reinterpret_cast<u16x4*>(drow + col) = pk;
          }
        }
      }
    }
    return;
  }

  // ================================= dK / dV role =================================
  constexpr int BUFB = (SEQ_O ? 2 : 3) * TILE + 512;   // Q, dO, (O), lse[64], delta[64]
  const int k0 = ((int)blockIdx.x - nq) * 64;
  const int key = k0 + 32 * sub + l32;
  const bool kvalid = key < Sk;
  const int q0 = 64 * half;                  // this pair's query tile
  char* qb = smem + half * BUFB;
  char* gb = qb + TILE;
  char* ob = SEQ_O ? qb : qb + 2 * TILE;     // O (d_h 256: in Q's slot until delta is done)
  float* ls = reinterpret_cast<float*>(qb + (SEQ_O ? 2 : 3) * TILE);
  float* dl = ls + 64;
  const bool qtile = q0 < Sq;
  if (qtile) {
    if (!SEQ_O) gp.issue(Qb, qs, q0, Sq, D, qb, wv);
    gp.issue(Gb, os, q0, Sq, D, gb, wv);
    gp.issue(Ob, os, q0, Sq, D, ob, wv);
    if (wv == 0) {   // per-row LSE, 4 bytes per lane (rows past Sq are masked in the math)
      const int q = min(q0 + lane, Sq - 1);
      __builtin_amdgcn_global_load_lds((const void*)(LSE + (int64_t)bh * Sq + q),
                                       (__attribute__((address_space(3))) void*)ls, 4, 0, 0);
    }
  }
  bf16x8 kf[DP / 16], vf[DP / 16];
  {
    const bf16_t* Krow = Kb + (int64_t)key * ks;
    const bf16_t* Vrow = Vb + (int64_t)key * vs;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) {
      kf[s] = __builtin_bit_cast(bf16x8, gload8(Krow, 16 * s + 8 * hl, D, kvalid));
      vf[s] = __builtin_bit_cast(bf16x8, gload8(Vrow, 16 * s + 8 * hl, D, kvalid));
    }
  }
  f32x16 dk[DP / 32], dv[DP / 32];
#pragma unroll
  for (int d = 0; d < DP / 32; ++d) {
    dk[d] = {};
    dv[d] = {};
  }
  __syncthreads();   // the pair's dO / O (/ Q) tiles and LSE are in LDS
  // delta of the tile's 64 rows: the pair's 128 lanes, two per row (16-byte chunks c, c + 2, ...)
  if (qtile) {
    const int t = 64 * sub + lane, row = t >> 1, part = t & 1;
    float acc = 0.f;
#pragma unroll
    for (int ch = part; ch < DP / 8; ch += 2) {
      if (8 * ch < D) {
        const bf16x8 gv = lds_row8<DP>(gb, row, ch), ov = lds_row8<DP>(ob, row, ch);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += (float)gv[j] * (float)ov[j];
      }
    }
    acc += __shfl_xor(acc, 1, 64);
    if (part == 0) dl[row] = acc;
  }
  __syncthreads();
  if constexpr (SEQ_O) {   // O is consumed: Q into its slot
    if (qtile) gp.issue(Qb, qs, q0, Sq, D, qb, wv);
    __syncthreads();
  }
  if (qtile) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      f32x16 sacc = {}, pacc = {};
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        bf16x8 aq = lds_row8<DP>(qb, 32 * u + l32, 2 * s + hl);
        bf16x8 ag = lds_row8<DP>(gb, 32 * u + l32, 2 * s + hl);
        sacc = mfma32(aq, kf[s], sacc);
        pacc = mfma32(ag, vf[s], pacc);
      }
      f32x16 pm, ds;
      float4 lsv[4], dlv[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        lsv[g] = *reinterpret_cast<const float4*>(ls + 32 * u + 8 * g + 4 * hl);
        dlv[g] = *reinterpret_cast<const float4*>(dl + 32 * u + 8 * g + 4 * hl);
      }
      uint32_t keep = 0xffffu;
      if (DROP) {
        keep = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t q = (uint32_t)(q0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hl);
          keep |= (hash_lo(dkey, q * (uint32_t)Sk + (uint32_t)key) >= dthr ? 1u : 0u) << r;
        }
      }
      auto elems = [&](auto masked) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = q0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hl;
          const float lv = (&lsv[r >> 2].x)[r & 3], dv_ = (&dlv[r >> 2].x)[r & 3];
          float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[r], c, -lv));
          if constexpr (decltype(masked)::value) {
            if (q >= Sq) p = 0.f;
          }
          float dpv = pacc[r];
          float pd = p;
          if (DROP) {
            const float msk = (keep >> r) & 1u ? dinv : 0.f;
            pd = p * msk;
            dpv = dpv * msk;
          }
          pm[r] = pd;
          ds[r] = p * (dpv - dv_);
        }
      };
      if (q0 + 64 > Sq) elems(std::true_type{});
      else elems(std::false_type{});
      const bf16x8 pb0 = pack8(pm, 0), pb1 = pack8(pm, 1);
      const bf16x8 db0 = pack8(ds, 0), db1 = pack8(ds, 1);
#pragma unroll
      for (int d = 0; d < DP / 32; ++d) {
        const int c0 = 32 * d + 16 * ((lane >> 4) & 1);
        const int rb = 32 * u + 4 * hl;
        bf16x8 ag0 = cat44(lds_tr4<DP>(gb, rb + 0, c0), lds_tr4<DP>(gb, rb + 8, c0));
        bf16x8 ag1 = cat44(lds_tr4<DP>(gb, rb + 16, c0), lds_tr4<DP>(gb, rb + 24, c0));
        dv[d] = mfma32(ag0, pb0, dv[d]);
        dv[d] = mfma32(ag1, pb1, dv[d]);
        bf16x8 aq0 = cat44(lds_tr4<DP>(qb, rb + 0, c0), lds_tr4<DP>(qb, rb + 8, c0));
        bf16x8 aq1 = cat44(lds_tr4<DP>(qb, rb + 16, c0), lds_tr4<DP>(qb, rb + 24, c0));
        dk[d] = mfma32(aq0, db0, dk[d]);
        dk[d] = mfma32(aq1, db1, dk[d]);
      }
    }
  }
  // the half = 1 pair hands its partial dK^T / dV^T to the half = 0 pair
  __syncthreads();
  float* xk = reinterpret_cast<float*>(smem) + sub * (2 * DP / 32 * 16 * 64);
  float* xv = xk + DP / 32 * 16 * 64;
  if (half == 1) {
#pragma unroll
    for (int d = 0; d < DP / 32; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        xk[(d * 16 + r) * 64 + lane] = dk[d][r];
        xv[(d * 16 + r) * 64 + lane] = dv[d][r];
      }
  }
  __syncthreads();
  if (half == 0) {
#pragma unroll
    for (int d = 0; d < DP / 32; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dk[d][r] += xk[(d * 16 + r) * 64 + lane];
        dv[d][r] += xv[(d * 16 + r) * 64 + lane];
      }
  }
  if (CSK != nullptr) {
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();
    wg_colsum_atomic<DP>(dk, scale, kvalid && half == 0, red, CSK + (int64_t)h * D, D);
    __syncthreads();
    wg_colsum_atomic<DP>(dv, 1.f, kvalid && half == 0, red, CSV + (int64_t)h * D, D);
  }
  if (kvalid && half == 0) {
    bf16_t* dkrow = dK + ((int64_t)b * Sk + key) * dks + (int64_t)h * D;
    bf16_t* dvrow = dV + ((int64_t)b * Sk + key) * dvs + (int64_t)h * D;
#pragma unroll
    for (int d = 0; d < DP / 32; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = 32 * d + 8 * g + 4 * hl;
        if (col < D) {
          u16x4 a, bb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] = f2bf(dk[d][4 * g + e] * scale);
            bb[e] = f2bf(dv[d][4 * g + e]);
          }
          *reinterpret_cast<u16x4*>(dkrow + col) = a;
          *reinterpret_cast<u16x4*>(dvrow + col) = bb;
        }
      }
    }
  }
}

// LDS of attn_bwd_short_kernel: max over the roles' tiles and hand-off areas
template <int DP>
constexpr size_t short_bwd_lds() {
  constexpr size_t tile = 64 * DP * 2;
  constexpr size_t dq_tiles = 4 * tile;
  constexpr size_t dkdv_tiles = 2 * ((DP > 128 ? 2 : 3) * tile + 512);
  constexpr size_t xq = 2 * (DP / 32) * 16 * 64 * 4;
  constexpr size_t xkv = 2 * xq;
  constexpr size_t red = 4 * DP * 4;
  size_t m = dq_tiles;
  m = dkdv_tiles > m ? dkdv_tiles : m;
  m = xq > m ? xq : m;
  m = xkv > m ? xkv : m;
  m = red > m ? red : m;
  return m;
}

// ==========================================================================================
// launchers
// ==========================================================================================
template <int DP, bool CAUSAL, bool DROP>
static int launch_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq, int Sk, int H,
                      int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, float scale, float p,
                      uint64_t seed, hipStream_t st) {
  // short non-causal problems (fewer 128-query blocks than CUs): the key-split kernel
  if constexpr (!CAUSAL && DP <= 128) {
    static const bool ks2_off = [] { const char* e = getenv("MIPIPE_ATTN_KS2"); return e && e[0] == '0'; }();
    if (!ks2_off && (int64_t)((Sq + 127) / 128) * B * H < 256) {
      const int niter = ((Sk + 63) / 64 + 1) / 2;
      const size_t lds2 = (niter > 1 ? 8 : 4) * 64 * DP * 2;
      auto kern2 = attn_fwd_ks2_kernel<DP, DROP>;
      if (lds2 > 64 * 1024)
        hipFuncSetAttribute((const void*)kern2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
      dim3 grid2((Sq + 63) / 64, B * H);
      kern2<<<grid2, 256, lds2, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse, B, Sq,
                                      Sk, H, Hkv, D, qs, ks, vs, os, scale, p, seed);
      return (int)hipGetLastError();
    }
  }
  const size_t lds = 4 * 64 * DP * 2;
  // v2 (default at d_h 64); MIPIPE_ATTN_FWD=1 selects v1 (A/B)
  static const bool v1 = [] { const char* e = getenv("MIPIPE_ATTN_FWD"); return e && e[0] == '1'; }();
  if constexpr (DP == 64) {
  if (!v1 && (int64_t)(Sk + 128) * ks * 2 < (1ll << 31) && (int64_t)(Sk + 128) * vs * 2 < (1ll << 31)) {
    // (d_h 128 / 256 spill at 3 waves per SIMD)
    const int nmb = (Sq + 127) / 128;
    const int npair = CAUSAL ? (nmb + 1) / 2 : nmb;
    hipLaunchKernelGGL((attn_fwd2_kernel<DP, CAUSAL, DROP>), dim3(npair * B * H), dim3(256), MP_FWD_NBUF * 2 * 64 * 64 * 2, st,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse, B, Sq, Sk, H, Hkv, D, qs,
                       ks, vs, os, scale, p, seed);
    return (int)hipGetLastError();
  }
  }
  auto kern = attn_fwd_kernel<DP, CAUSAL, DROP>;
  if (lds > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((Sq + 127) / 128, B * H);
  kern<<<grid, 256, lds, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse, B, Sq, Sk, H,
                               Hkv, D, qs, ks, vs, os, scale, p, seed);
  return (int)hipGetLastError();
}

template <int DP, bool CAUSAL, bool DROP>
static int launch_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                      float* delta, void* dq, void* dk, void* dv, int B, int Sq, int Sk, int H, int Hkv, int D,
                      int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dqs, int64_t dks, int64_t dvs,
                      float scale, float p, uint64_t seed, float* csq, float* csk, float* csv, hipStream_t st) {
  // short non-causal problems: dQ and dK/dV in one launch (MIPIPE_ATTN_BWD_SHORT=0: the
  // two-kernel path, for A/B)
  if constexpr (!CAUSAL && DP <= 128) {   // (d_h 256: the role-merged register file spills)
    static const bool short_off = [] { const char* e = getenv("MIPIPE_ATTN_BWD_SHORT"); return e && e[0] == '0'; }();
    if (!short_off && Sq <= 128 && Sk <= 128 && H == Hkv) {
      constexpr size_t lds = short_bwd_lds<DP>();
      auto kern = attn_bwd_short_kernel<DP, DROP>;
      if (lds > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      dim3 grid((Sq + 63) / 64 + (Sk + 63) / 64, B * H);
      kern<<<grid, 256, lds, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)o,
                                   (const bf16_t*)dout, lse, (bf16_t*)dq, (bf16_t*)dk, (bf16_t*)dv, B, Sq, Sk, H, D, qs,
                                   ks, vs, os, dqs, dks, dvs, scale, p, seed, csq, csk, csv);
      return (int)hipGetLastError();
    }
  }
  static const bool dq1 = [] { const char* e = getenv("MIPIPE_ATTN_BWD_DQ"); return e && e[0] == '1'; }();
  // v3 (paired query blocks on one XCD) by default: +0.35 % on the step over v2 (2 same-box
  // runs each); MIPIPE_ATTN_BWD_DQ=2 / 1 select v2 / v1
  static const bool dq3 = [] { const char* e = getenv("MIPIPE_ATTN_BWD_DQ"); return !(e && e[0] == '2'); }();
  bool dq_done = false;
  if constexpr (DP == 64) {
    if (!dq1 && (int64_t)(Sk + 128) * ks * 2 < (1ll << 31) && (int64_t)(Sk + 128) * vs * 2 < (1ll << 31)) {
      if (dq3) {
        const int nmb = (Sq + 127) / 128;
        hipLaunchKernelGGL((attn_bwd_dq3_kernel<DP, CAUSAL, DROP>), dim3((CAUSAL ? (nmb + 1) / 2 : nmb) * B * H),
                           dim3(256), 4 * 2 * 64 * DP * 2, st, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                           (const bf16_t*)o, (const bf16_t*)dout, lse, delta, (bf16_t*)dq, B, Sq, Sk, H, Hkv, D, qs,
                           ks, vs, os, dqs, scale, p, seed, csq);
      } else {
        hipLaunchKernelGGL((attn_bwd_dq2_kernel<DP, CAUSAL, DROP>), dim3((Sq + 127) / 128, B * H), dim3(256),
                           4 * 2 * 64 * DP * 2, st, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                           (const bf16_t*)o, (const bf16_t*)dout, lse, delta, (bf16_t*)dq, B, Sq, Sk, H, Hkv, D, qs,
                           ks, vs, os, dqs, scale, p, seed, csq);
      }
      dq_done = true;
    }
  }
  if (!dq_done) {
    const size_t lds = (DP <= 128 ? 4 : 2) * 2 * 64 * DP * 2;
    auto kern = attn_bwd_dq_kernel<DP, CAUSAL, DROP>;
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dim3 grid((Sq + 127) / 128, B * H);
    kern<<<grid, 256, lds, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)o,
                                 (const bf16_t*)dout, lse, delta, (bf16_t*)dq, B, Sq, Sk, H, Hkv, D, qs, ks, vs, os,
                                 dqs, scale, p, seed, csq);
  }
  static const bool dkdv1 = [] { const char* e = getenv("MIPIPE_ATTN_BWD_DKDV"); return e && e[0] == '1'; }();
  // v3 (paired key blocks on one XCD) by default: +0.4 % on the step over v2 (2 same-box runs
  // each, profiles/r6_attention_v2.md); MIPIPE_ATTN_BWD_DKDV=2 / 1 select v2 / v1
  static const bool dkdv3 = [] { const char* e = getenv("MIPIPE_ATTN_BWD_DKDV"); return !(e && e[0] == '2'); }();
  bool dkdv_done = false;
  if constexpr (DP == 64) {
    if (!dkdv1 && (int64_t)(Sq + 128) * qs * 2 < (1ll << 31) && (int64_t)(Sq + 128) * os * 2 < (1ll << 31)) {
      if (dkdv3) {
        const int nkb = (Sk + 127) / 128;
        hipLaunchKernelGGL((attn_bwd_dkdv3_kernel<DP, CAUSAL, DROP>), dim3((CAUSAL ? (nkb + 1) / 2 : nkb) * B * Hkv),
                           dim3(256), 4 * (2 * 64 * DP * 2 + 512), st, (const bf16_t*)q, (const bf16_t*)k,
                           (const bf16_t*)v, (const bf16_t*)dout, lse, delta, (bf16_t*)dk, (bf16_t*)dv, B, Sq, Sk, H,
                           Hkv, D, qs, ks, vs, os, dks, dvs, scale, p, seed, csk, csv);
        return (int)hipGetLastError();
      }
      hipLaunchKernelGGL((attn_bwd_dkdv2_kernel<DP, CAUSAL, DROP>), dim3((Sk + 127) / 128, B * Hkv), dim3(256),
                         4 * (2 * 64 * DP * 2 + 512), st, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                         (const bf16_t*)dout, lse, delta, (bf16_t*)dk, (bf16_t*)dv, B, Sq, Sk, H, Hkv, D, qs, ks, vs, os,
                         dks, dvs, scale, p, seed, csk, csv);
      dkdv_done = true;
    }
  }
  if (!dkdv_done) {
    const size_t lds = (DP <= 128 ? MP_DKDV_NBUF : 2) * (2 * 64 * DP * 2 + 512);
    auto kern = attn_bwd_dkdv_kernel<DP, CAUSAL, DROP>;
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dim3 grid((Sk + 127) / 128, B * Hkv);
    kern<<<grid, 256, lds, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse,
                                 delta, (bf16_t*)dk, (bf16_t*)dv, B, Sq, Sk, H, Hkv, D, qs, ks, vs, os, dks, dvs,
                                 scale, p, seed, csk, csv);
  }
  return (int)hipGetLastError();
}

static int pick_dp(int D) { return D <= 64 ? 64 : (D <= 128 ? 128 : (D <= 256 ? 256 : -1)); }

extern "C" int mp_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq, int Sk,
                           int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, int causal,
                           float scale, float p_drop, uint64_t seed, hipStream_t st) {
  const int DP = pick_dp(D);
  if (DP < 0 || D % 8 || H % Hkv) return -1;
  const bool drop = p_drop > 0.f;
#define MP_F(DPV)                                                                                                     \
  if (DP == DPV) {                                                                                                    \
    if (causal) return drop ? launch_fwd<DPV, true, true>(q, k, v, o, lse, B, Sq, Sk, H, Hkv, D, qs, ks, vs, os, scale, \
                                                          p_drop, seed, st)                                           \
                            : launch_fwd<DPV, true, false>(q, k, v, o, lse, B, Sq, Sk, H, Hkv, D, qs, ks, vs, os,     \
                                                           scale, p_drop, seed, st);                                  \
    return drop ? launch_fwd<DPV, false, true>(q, k, v, o, lse, B, Sq, Sk, H, Hkv, D, qs, ks, vs, os, scale, p_drop,  \
                                               seed, st)                                                              \
                : launch_fwd<DPV, false, false>(q, k, v, o, lse, B, Sq, Sk, H, Hkv, D, qs, ks, vs, os, scale, p_drop, \
                                                seed, st);                                                            \
  }
  MP_F(64) MP_F(128) MP_F(256)
#undef MP_F
  return -1;
}

extern "C" int mp_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                           const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int Sq,
                           int Sk, int H, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dqs,
                           int64_t dks, int64_t dvs, int causal, float scale, float p_drop, uint64_t seed,
                           float* csq, float* csk, float* csv, hipStream_t st) {
  const int DP = pick_dp(D);
  if ((csq == nullptr) != (csk == nullptr) || (csk == nullptr) != (csv == nullptr)) return -1;
  if (DP < 0 || D % 8 || H % Hkv) return -1;
  const bool drop = p_drop > 0.f;
#define MP_B(DPV, C, DR)                                                                                             \
  if (DP == DPV && (bool)causal == C && drop == DR)                                                                  \
    return launch_bwd<DPV, C, DR>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, H, Hkv, D, qs, ks, vs, os, dqs, \
                                  dks, dvs, scale, p_drop, seed, csq, csk, csv, st);
  MP_B(64, true, false) MP_B(64, false, false) MP_B(64, true, true) MP_B(64, false, true)
  MP_B(128, true, false) MP_B(128, false, false) MP_B(128, true, true) MP_B(128, false, true)
  MP_B(256, true, false) MP_B(256, false, false) MP_B(256, true, true) MP_B(256, false, true)
#undef MP_B
  return -1;
}

MP_DROP_STEP_SETTER(mp_set_drop_step_attn)
