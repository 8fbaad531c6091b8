// v2 bf16 MFMA GEMM: 8 waves, large tiles, direct-to-LDS staging (global_load_lds_dwordx4).
//
//   C[M,N] (+)= alpha * op(A) op(B) (+ fused epilogue); same contract as gemm.hip
//   (TA/TB layouts, epilogues, f32 split-K accumulate), different engine:
//
// * Tiles BMxBN (256x256, 256x192, 256x128, 128x128) chosen per problem by the host so
//   the tile count fills whole "waves" of 256 CUs (GPT-2: N = 768 / 2304 / 3072 divide
//   by 192/256 -> zero quantisation loss at T = 16384 tokens).
// * Staging: every 1 KiB piece of a tile is one wave-instruction of global_load_lds
//   (no VGPR round trip, no ds_write).  The LDS destination is lane-linear, so the
//   bank-conflict swizzle of the image is applied on the *source* address (cdna guide
//   §5.4 rule 21): lane l fetches the logical chunk that belongs at its physical slot.
// * Pipeline: 2 LDS stages; tile t+1 is in flight while tile t is consumed; counted
//   `s_waitcnt vmcnt(P)` (P = pieces per wave per tile) + raw s_barrier, never
//   __syncthreads() (which would drain the in-flight DMA).
// * MFMA 32x32x16 bf16, per wave (BM/WM)x(BN/WN); fragments by ds_read_b128 (K-contiguous
//   images) or two ds_read_b64_tr_b16 (outer-contiguous images).
// * Epilogue staged through LDS one wave-row group at a time -> coalesced 16-byte bias /
//   residual / activation / store, or lane-consecutive f32 atomics for split-K.
#include "mp_common.h"

using namespace mp;

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

// tile rows per raster group of the ping-pong engine: GPT-2 bench (3 interleaved runs
// each, one box) 841K tok/s at 8, 851K at 4, 856K at 2, 863-864K vs 870K at 1 vs 2 on a
// second box, 829K at 16 -- the isolated GEMM is flat (+-1 %); inside the step (dW GEMMs on
// the side stream sharing L2) short groups win
#ifndef MP_G3_GROUP
#define MP_G3_GROUP 2
#endif
#ifndef MP_G2_GROUP
#define MP_G2_GROUP 8
#endif

// gemm4: accumulator row blocks (of 8) whose store is deferred into the next tile
#ifndef MP_G4_SR
#define MP_G4_SR 2
#endif

#ifndef MP_GROUP_MAX
#define MP_GROUP_MAX 8
#endif

namespace g2 {

enum Epi { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_RELU = 3, EPI_BIAS_RES = 4, EPI_RES = 5,
           EPI_DGELU = 6, EPI_DRELU = 7 };

constexpr int BK = 64;
constexpr int NT = 512;

__device__ __forceinline__ int swz8(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int swz16(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
// K-contiguous image swizzle for the 16x16x32 fragment read (lane = 16 q + i reads row
// r0 + i, chunk c + q): chunk ^ g(row bits 1-3) with g mapping row pairs {0,1,6,7} ->
// {6,7,4,5} and {2..5} -> {0..3} makes all four ds_read_b128 lane groups hit 16
// distinct 16-byte bank slots (MI355X_MICROARCH.md LDS table); swz8 would be 2-way here
__device__ __forceinline__ int swzq(int row) { return (((row >> 1) & 7) + 6) & 7; }
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// K-contiguous image [rows][64 k]: 128-byte rows, 8 chunks
__device__ __forceinline__ int offK(int row, int chunk) { return row * 128 + 16 * (chunk ^ swz8(row)); }
// outer-contiguous image [64 k][COLS]: 2*COLS-byte rows; swizzle the low 4 chunk bits
// (COLS = 64, the small engine's TT tiles: 8 chunks per row, chunk pairs XORed by row bits
// 1 and 3 -- the 8 rows a 32-lane ds_read_b64_tr_b16 group touches land in 8 distinct
// 8-bank groups, conflict-free)
__device__ __forceinline__ int swz8o(int row) { return 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1)); }
template <int COLS>
__device__ __forceinline__ int offO(int row, int chunk) {
  if constexpr (COLS == 64) return row * 128 + 16 * (chunk ^ swz8o(row));
  return row * (COLS * 2) + 16 * ((chunk & ~15) | ((chunk & 15) ^ swz16(row)));
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <bool OUTER, int COLS>
__device__ __forceinline__ bf16x8 frag(const char* img, int rc, int s, int hl) {
  if constexpr (!OUTER) {
    return *reinterpret_cast<const bf16x8*>(img + offK(rc, 2 * s + hl));
  } else {
    const int i = threadIdx.x & 15, q = i >> 2, p = i & 3;
    const int col = (rc & ~15) + 4 * p;
    const int r0 = 16 * s + 8 * hl;
    const char* a0 = img + offO<COLS>(r0 + q, col >> 3) + ((col & 7) << 1);
    const char* a1 = img + offO<COLS>(r0 + 4 + q, col >> 3) + ((col & 7) << 1);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

// 16x16x32 fragment: lane l holds rows/cols base + (l & 15), k = 32 s + 8 (l >> 4) + 0..7
// (K-contiguous images use the swzq swizzle; outer-contiguous ones two tr reads, 8 k-rows
// per 16-lane group, conflict-free under offO's swz16)
template <bool OUTER, int COLS>
__device__ __forceinline__ bf16x8 frag16(const char* img, int base, int s) {
  const int lane = threadIdx.x & 63;
  if constexpr (!OUTER) {
    const int row = base + (lane & 15), chunk = 4 * s + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + 16 * (chunk ^ swzq(row)));
  } else {
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const int col = base + 4 * p;
    const int r0 = 32 * s + 8 * (lane >> 4);
    const char* a0 = img + offO<COLS>(r0 + q, col >> 3) + ((col & 7) << 1);
    const char* a1 = img + offO<COLS>(r0 + 4 + q, col >> 3) + ((col & 7) << 1);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

// global source (bf16 element pointer) of the 16 bytes that land at byte `pos` of an image
template <bool OUTER, int ROWS, bool M16 = false>
__device__ __forceinline__ const bf16_t* src_of(const bf16_t* base, int64_t ld, int pos, int outer0, int outer_lim,
                                                int k0) {
  if constexpr (!OUTER) {  // [ROWS][64k]
    const int row = pos >> 7, phys = (pos >> 4) & 7;
    const int chunk = phys ^ (M16 ? swzq(row) : swz8(row));
    int o = outer0 + row;
    o = o < outer_lim ? o : outer_lim - 1;  // clamp: rows past the edge only feed masked outputs
    return base + (int64_t)o * ld + k0 + chunk * 8;
  } else {  // [64k][ROWS cols]
    constexpr int PITCH = ROWS * 2;
    const int row = pos / PITCH, phys = (pos % PITCH) >> 4;
    const int chunk = ROWS == 64 ? (phys ^ swz8o(row)) : ((phys & ~15) | ((phys & 15) ^ swz16(row)));
    int o = outer0 + chunk * 8;
    o = o < outer_lim ? o : outer_lim - 8;
    return base + (int64_t)(k0 + row) * ld + o;
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  // s_waitcnt simm16 for gfx9: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | (((N >> 4) & 3) << 14));
}

// ---- epilogue: one wave-row group at a time through LDS -> coalesced 16-byte bias /
// residual / activation / store, or lane-consecutive f32 atomics for split-K
// the fused epilogue of 8 consecutive outputs (row gr, columns gc..gc+7) -> bf16 C
template <int EPI>
__device__ __forceinline__ void epi_store8(float (&v)[8], int gr, int gc, bf16_t* __restrict__ C, int64_t ldc,
                                           const bf16_t* __restrict__ bias, const bf16_t* __restrict__ R,
                                           int64_t ldr, bf16_t* __restrict__ AUX, int64_t ldx, float p_drop,
                                           uint64_t seed) {
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_RES) {
    u16x8 bv = *reinterpret_cast<const u16x8*>(bias + gc);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += bf2f(bv[e]);
  }
  if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU) {
    // AUX: what the backward's dX epilogue needs -- the pre-activation for ReLU (its sign),
    // GELU's derivative for GELU (computed here beside the activation from one sigmoid, so
    // the backward multiplies instead of re-evaluating it: dGELU dX 505 -> ~440 us at 64K x
    // 3072, profiles/r5_gemm_epilogue_cost.md)
    u16x8 sv;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = bf2f(f2bf(v[e]));   // the activation of the bf16-rounded pre-activation
      if constexpr (EPI == EPI_BIAS_GELU) {
        float d;
        gelu_tanh_and_grad(x, v[e], d);
        sv[e] = f2bf(d);
      } else {
        sv[e] = f2bf(x);
        v[e] = fmaxf(x, 0.f);
      }
      // dropout after the activation (the reference FFN's drop(relu(.))), mask index =
      // element index of the contiguous output, as act_fwd / act_bwd regenerate it
      if (p_drop > 0.f) v[e] *= dropout_scale(seed, (uint64_t)gr * ldc + gc + e, p_drop);
    }
    *reinterpret_cast<u16x8*>(AUX + (int64_t)gr * ldx + gc) = sv;
  }
  if constexpr (EPI == EPI_BIAS_RES || EPI == EPI_RES) {
    u16x8 rv = *reinterpret_cast<const u16x8*>(R + (int64_t)gr * ldr + gc);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += bf2f(rv[e]);
  }
  if constexpr (EPI == EPI_DGELU || EPI == EPI_DRELU) {
    u16x8 xv = *reinterpret_cast<const u16x8*>(AUX + (int64_t)gr * ldx + gc);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = bf2f(xv[e]);   // GELU: the saved derivative; ReLU: the pre-activation
      v[e] *= EPI == EPI_DGELU ? x : (x > 0.f ? 1.f : 0.f);
      if (p_drop > 0.f) v[e] *= dropout_scale(seed, (uint64_t)gr * ldc + gc + e, p_drop);
    }
  }
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e]);
#ifndef MP_GEMM_PLAIN_STORE
  // non-temporal: the bf16 C tiles stream out without displacing the A/B panels other
  // workgroups still read from L2 (GPT-2 bench +0.9 %, 3 interleaved pairs on one box;
  // MP_GEMM_PLAIN_STORE builds the plain store for A/B)
  __builtin_nontemporal_store(o, reinterpret_cast<u16x8*>(C + (int64_t)gr * ldc + gc));
#else
  *reinterpret_cast<u16x8*>(C + (int64_t)gr * ldc + gc) = o;
#endif
}

// accumulator layout of the 32x32x16 engines: acc[i][j] element r -> wave-local
// row 32 i + (r & 3) + 8 (r >> 2) + 4 hl, column wn + 32 j + l32
template <int WTM, int WTN>
struct Stage32 {
  f32x16 (&acc)[WTM][WTN];
  int wn, hl, l32;
  __device__ __forceinline__ void operator()(float* ct, int CP) const {
#pragma unroll
    for (int i = 0; i < WTM; ++i)
#pragma unroll
      for (int j = 0; j < WTN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
          const int col = wn + 32 * j + l32;
          ct[row * CP + col] = acc[i][j][r];
        }
  }
};

// accumulator layout of the 16x16x32 engines: acc[i][j] element r -> wave-local
// row 16 i + 4 (lane >> 4) + r, column wn + 16 j + (lane & 15)
template <int TM, int TN>
struct Stage16 {
  f32x4 (&acc)[TM][TN];
  int wn, lane;
  __device__ __forceinline__ void operator()(float* ct, int CP) const {
    const int rq = 4 * (lane >> 4), c = wn + (lane & 15);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ct[(16 * i + rq + r) * CP + c + 16 * j] = acc[i][j][r];
  }
};

template <int BM, int BN, int WM, int WN, int EPI, bool ACC, int NTH = NT, bool PARTS = false, class StageF>
__device__ __forceinline__ void epilogue(const StageF& stage, char* smem, int m0, int n0, int wr,
                                         void* __restrict__ Cv,
                                         const bf16_t* __restrict__ bias, const bf16_t* __restrict__ R,
                                         bf16_t* __restrict__ AUX, float* __restrict__ WS, int M, int N, int64_t ldc,
                                         int64_t ldr, int64_t ldx, float alpha, int nsplit, float p_drop,
                                         uint64_t seed, const float* __restrict__ parts = nullptr,
                                         int64_t pstep = 0, int nparts = 0, int split_idx = -1) {
  // parts (gemm7's tile owner): nparts row-major [BM][BN] f32 partial tiles at parts + p *
  // pstep, added to the accumulator before the epilogue (published with sc1 stores; the
  // caller's agent-scope acquire precedes)
  constexpr int RG = BM / WM;      // rows per group
  constexpr int CP = BN + 4;       // f32 pitch
  // 8-column chunks per tile row; the store loop runs on the first NTE threads, a multiple
  // of CH (all NTH threads for power-of-two widths; 504 of 512 for BN = 192)
  constexpr int CH = BN / 8, NTE = (NTH / CH) * CH;
  float* ct = reinterpret_cast<float*>(smem);
  // bf16 outputs with WS != nullptr: also accumulate the column sums of the final values
  // into WS[N] (f32; the bias gradient of the next layer).  Every thread keeps the same 8
  // columns over all its rows (its chunk idx % CH is fixed because the loop strides by NTE),
  // so the sums stay in registers until one LDS reduction and BN atomics per tile.
  constexpr bool CS_OK = !ACC;
  const bool cs = CS_OK && WS != nullptr;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int pass = 0; pass < WM; ++pass) {
    if (wr == pass) stage(ct, CP);
    __syncthreads();
    if constexpr (!ACC && PARTS) {
      if (nparts > 0) {
        // the partial row blocks added into the staged rows: every thread's loads of one
        // partial in flight at once (a load inside the store loop would wait per element)
        constexpr int Q4 = RG * BN / 4, N4 = (Q4 + NTH - 1) / NTH;
        for (int pp = 0; pp < nparts; ++pp) {
          const float* src = parts + pp * pstep + (int64_t)(pass * RG) * BN;
          float4 pv[N4];
#pragma unroll
          for (int u = 0; u < N4; ++u) {
            const int idx = min((int)threadIdx.x + u * NTH, Q4 - 1);
            pv[u] = *reinterpret_cast<const float4*>(src + (idx / (BN / 4)) * BN + (idx % (BN / 4)) * 4);
          }
#pragma unroll
          for (int u = 0; u < N4; ++u) {
            const int idx = threadIdx.x + u * NTH;
            if (idx >= Q4) break;
            float4* d = reinterpret_cast<float4*>(ct + (idx / (BN / 4)) * CP + (idx % (BN / 4)) * 4);
            float4 t = *d;
            t.x += pv[u].x; t.y += pv[u].y; t.z += pv[u].z; t.w += pv[u].w;
            *d = t;
          }
        }
        __syncthreads();
      }
    }
    const int rbase = m0 + pass * RG;
    if constexpr (ACC) {
      if (nsplit > 1 && WS != nullptr) {
        // split-K partial slab [split][M][N] with plain 16-byte stores; a reduce kernel
        // adds the slabs into C (f32 atomics run at ~1.3 TB/s chip-wide and bounded the
        // dW GEMMs; MI355X_MICROARCH.md "Global float atomics")
        float* slab = WS + (int64_t)(split_idx >= 0 ? split_idx : (int)blockIdx.y) * M * N;
        for (int idx = threadIdx.x; idx < RG * BN / 4; idx += NTH) {
          const int row = idx / (BN / 4), c4 = (idx % (BN / 4)) * 4;
          const int gr = rbase + row, gc = n0 + c4;
          if (gr < M && gc < N) {
            float4 v = *reinterpret_cast<const float4*>(ct + row * CP + c4);
            v.x *= alpha; v.y *= alpha; v.z *= alpha; v.w *= alpha;
            *reinterpret_cast<float4*>(slab + (int64_t)gr * N + gc) = v;
          }
        }
        __syncthreads();
        continue;
      }
      if (nsplit > 1) {
        float* C = reinterpret_cast<float*>(Cv);
        for (int idx = threadIdx.x; idx < RG * BN; idx += NTH) {
          const int row = idx / BN, col = idx % BN;
          const int gr = rbase + row, gc = n0 + col;
          if (gr < M && gc < N) atomicAdd(C + (int64_t)gr * ldc + gc, alpha * ct[row * CP + col]);
        }
        __syncthreads();
        continue;
      }
    }
    for (int idx = threadIdx.x < NTE ? (int)threadIdx.x : RG * CH; idx < RG * CH; idx += NTE) {
      const int row = idx / CH, c8 = (idx % CH) * 8;
      const int gr = rbase + row, gc = n0 + c8;
      if (gr >= M || gc >= N) continue;
      float v[8];
      const float4 lo = *reinterpret_cast<const float4*>(ct + row * CP + c8);
      const float4 hi = *reinterpret_cast<const float4*>(ct + row * CP + c8 + 4);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= alpha;
      if constexpr (ACC) {
        float* cp = reinterpret_cast<float*>(Cv) + (int64_t)gr * ldc + gc;
        float4 c0 = *reinterpret_cast<float4*>(cp), c1 = *reinterpret_cast<float4*>(cp + 4);
        c0.x += v[0]; c0.y += v[1]; c0.z += v[2]; c0.w += v[3];
        c1.x += v[4]; c1.y += v[5]; c1.z += v[6]; c1.w += v[7];
        *reinterpret_cast<float4*>(cp) = c0;
        *reinterpret_cast<float4*>(cp + 4) = c1;
      } else {
        epi_store8<EPI>(v, gr, gc, reinterpret_cast<bf16_t*>(Cv), ldc, bias, R, ldr, AUX, ldx, p_drop, seed);
        if (cs) {
#pragma unroll
          for (int e = 0; e < 8; ++e) csum[e] += v[e];
        }
      }
    }
    __syncthreads();
  }
  if constexpr (CS_OK) {
    if (cs) {
      float* red = ct;   // [NTH][8]
#pragma unroll
      for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = csum[e];
      __syncthreads();
      constexpr int GRP = NTE / CH;   // threads per column chunk
      for (int c = threadIdx.x; c < BN; c += NTH) {
        float t = 0.f;
#pragma unroll 4
        for (int g = 0; g < GRP; ++g) t += red[(g * CH + c / 8) * 8 + (c & 7)];
        if (n0 + c < N) atomicAdd(WS + n0 + c, t);
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB, int EPI, bool ACC, bool M16>
__global__ void __launch_bounds__(NT, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) gemm2_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                      void* __restrict__ Cv, const bf16_t* __restrict__ bias,
                                                      const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX,
                                                      float* __restrict__ WS, int M, int N, int K, int64_t lda,
                                                      int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx,
                                                      float alpha, float p_drop, uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  static_assert(WM * WN == 8, "8 waves");
  constexpr int WTM = BM / WM / 32, WTN = BN / WN / 32;
  static_assert(WTM * 32 * WM == BM && WTN * 32 * WN == BN, "tile/wave mismatch");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PIECES = STAGE / 1024, PW = PIECES / 8;
  static_assert(PW * 8 == PIECES, "pieces must split over 8 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  const int nwg = gm * gn;
  const int wg = xcd_remap((int)blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int group = wg / (GROUP * gn);
  const int first_m = group * GROUP;
  const int gsz = min(gm - first_m, GROUP);
  const int tm = first_m + (wg % (GROUP * gn)) % gsz;
  const int tn = (wg % (GROUP * gn)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63, hl = lane >> 5, l32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int wm = wr * (BM / WM), wn = wc * (BN / WN);

  // split-K: split y owns k-tiles [y*KT/S, (y+1)*KT/S) (uneven splits allowed, so the
  // split count can be chosen for CU fill rather than divisibility)
  const int nsplit = gridDim.y;
  const int ktiles = K / BK;
  const int kt0 = (int)blockIdx.y * ktiles / nsplit;
  const int nk = ((int)blockIdx.y + 1) * ktiles / nsplit - kt0;
  const int kbase = kt0 * BK;

  // per-lane source pointers of every piece this wave stages, at k = kbase; a later
  // k-tile only adds a wave-uniform offset (k0 elements for K-contiguous images,
  // k0 rows for outer-contiguous ones)
  const bf16_t* psrc[PW];
  bool pisA[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int p = wave + 8 * i;            // wave-uniform piece index
    const int pos = p * 1024 + lane * 16;  // this lane's byte in the stage
    pisA[i] = p * 1024 < A_BYTES;
    if (pisA[i]) psrc[i] = src_of<TA, BM, M16>(A, lda, pos, m0, M, kbase);
    else psrc[i] = src_of<TB, BN, M16>(B, ldb, pos - A_BYTES, n0, N, kbase);
  }
  auto issue = [&](int stage, int kt) {
    char* sb = smem + stage * STAGE;
    const int64_t dA = TA ? (int64_t)kt * BK * lda : (int64_t)kt * BK;
    const int64_t dB = TB ? (int64_t)kt * BK * ldb : (int64_t)kt * BK;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int p = wave + 8 * i;
      const bf16_t* src = psrc[i] + (pisA[i] ? dA : dB);
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(sb + p * 1024),
                                       16, 0, 0);
    }
  };

  if constexpr (!M16) {
  f32x16 acc[WTM][WTN];
#pragma unroll
  for (int i = 0; i < WTM; ++i)
#pragma unroll
    for (int j = 0; j < WTN; ++j) acc[i][j] = {};

  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    wait_vmcnt<PW>();
  } else {
    wait_vmcnt<0>();
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int t = 0; t < nk; ++t) {
    const char* sa = smem + (t & 1) * STAGE;
    const char* sbB = sa + A_BYTES;
    // fragments double-buffered in registers: k-substep s+1 is read from LDS while the
    // MFMAs of substep s issue (the loop is fully unrolled, so [s & 1] is static)
    bf16x8 af[2][WTM], bfr[2][WTN];
#pragma unroll
    for (int i = 0; i < WTM; ++i) af[0][i] = frag<TA, BM>(sa, wm + 32 * i + l32, 0, hl);
#pragma unroll
    for (int j = 0; j < WTN; ++j) bfr[0][j] = frag<TB, BN>(sbB, wn + 32 * j + l32, 0, hl);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int c = s & 1;
      if (s + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < WTM; ++i) af[c ^ 1][i] = frag<TA, BM>(sa, wm + 32 * i + l32, s + 1, hl);
#pragma unroll
        for (int j = 0; j < WTN; ++j) bfr[c ^ 1][j] = frag<TB, BN>(sbB, wn + 32 * j + l32, s + 1, hl);
      }
      // pin the order: substep s+1's LDS reads are in flight under substep s's MFMAs
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j) acc[i][j] = mfma32(af[c][i], bfr[c][j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // everyone finished reading this stage before it is refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nk) {
      issue(t & 1, t + 2);
      wait_vmcnt<PW>();  // tile t+1 landed, tile t+2 still in flight
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  epilogue<BM, BN, WM, WN, EPI, ACC>(Stage32<WTM, WTN>{acc, wn, hl, l32}, smem, m0, n0, wr, Cv, bias, R, AUX, WS, M,
                                     N, ldc, ldr, ldx, alpha, nsplit, p_drop, seed);  } else {
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{};

  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    wait_vmcnt<PW>();
  } else {
    wait_vmcnt<0>();
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int t = 0; t < nk; ++t) {
    const char* sa = smem + (t & 1) * STAGE;
    const char* sbB = sa + A_BYTES;
    // two 32-deep k-substeps; substep 1's fragments are read under substep 0's MFMAs
    // (transposed layouts: one fragment set, the compiler overlaps what registers allow --
    // double-buffering the 256x256 TT tile spilled)
    if constexpr (TA || TB) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af1[TM], bf1[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af1[i] = frag16<TA, BM>(sa, wm + 16 * i, s);
#pragma unroll
        for (int j = 0; j < TN; ++j) bf1[j] = frag16<TB, BN>(sbB, wn + 16 * j, s);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af1[i], bf1[j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    } else {
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[0][i] = frag16<TA, BM>(sa, wm + 16 * i, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[0][j] = frag16<TB, BN>(sbB, wn + 16 * j, 0);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) af[1][i] = frag16<TA, BM>(sa, wm + 16 * i, 1);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[1][j] = frag16<TB, BN>(sbB, wn + 16 * j, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[s][i], bfr[s][j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nk) {
      issue(t & 1, t + 2);
      wait_vmcnt<PW>();
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  epilogue<BM, BN, WM, WN, EPI, ACC>(Stage16<TM, TN>{acc, wn, lane}, smem, m0, n0, wr, Cv, bias, R, AUX, WS, M, N, ldc,
                                     ldr, ldx, alpha, nsplit, p_drop, seed);
  }

}


// ---------------------------------------------------------------------------------------
// gemm3: 256x256 NT (both operands K-contiguous) with a ping-pong phase schedule.
//
// The K-tile (BK = 64) is cut into four 16 KiB half-tiles, each one LDS image of 128 rows:
//   A0 = rows {0..63, 128..191}   A1 = rows {64..127, 192..255}     (wave-row halves)
//   B0 = cols {0..31, 64..95, ..} B1 = cols {32..63, 96..127, ..}  (wave-col halves)
// A wave (wr, wc) owns a 128x64 output tile = four 64x32 quadrants, one per phase:
//   phase 1: A0 x B0 (reads A0 + B0)  phase 2: A0 x B1 (reads B1)
//   phase 3: A1 x B0 (reads A1)       phase 4: A1 x B1 (no reads)
// Phase p of K-tile t also streams half-tile p of K-tile t+1 into the other LDS buffer
// (2 glds per thread) -- DMA is spread evenly over the loop instead of bursting once
// per K-tile -- and a counted vmcnt(4) retires the half-tile the NEXT phase reads.
// Wave rows run one barrier apart (waves 4-7 take an extra s_barrier up front), so on
// every SIMD one wave issues MFMAs while its partner issues ds_reads / DMA: the
// cdna guide's 8-phase template (§5 "256^2 8-phase template"), with 32x32x16 MFMAs.
// ---------------------------------------------------------------------------------------
template <int EPI, bool ACC, bool M16, bool TT = false>
__global__ void __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm3_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, void* __restrict__ Cv,
             const bf16_t* __restrict__ bias, const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX,
             float* __restrict__ WS, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr,
             int64_t ldx, float alpha, float p_drop, uint64_t seed, int tile_lim) {
  if (p_drop > 0.f) seed = step_seed(seed);
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4;
  constexpr int HALF = 128 * 128;          // one half-tile image: 128 rows x 128 B
  constexpr int BUF = 4 * HALF;            // A0 A1 B0 B1
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  const int nwg = tile_lim > 0 ? tile_lim : gm * gn;
  // split-K grids: workgroups are dealt to the 8 XCDs round-robin in LINEAR id order
  // (x + gridDim.x * y), so remap that id, then cut it into (split, tile): an XCD's L2 holds
  // the panels of ONE split's neighbouring tiles.  Remapping blockIdx.x alone assumed XCD =
  // x % 8, which is wrong for y > 0 whenever gridDim.x % 8 != 0 and scattered the tiles that
  // share a panel over all XCDs (the dW GEMMs read ~4x their unique bytes from HBM)
  int wg, split;
  if (gridDim.y > 1 && tile_lim == 0) {   // (tile_lim = -1: the x-only remap, the default)
    const int v = xcd_remap((int)blockIdx.x + (int)gridDim.x * (int)blockIdx.y, nwg * (int)gridDim.y);
    split = v / nwg;
    wg = v % nwg;
  } else {
    wg = xcd_remap((int)blockIdx.x, nwg);
    split = (int)blockIdx.y;
  }
  constexpr int GROUP = MP_G3_GROUP;   // tile rows per raster group (L2 reuse of the A panels)
  const int group = wg / (GROUP * gn);
  const int first_m = group * GROUP;
  const int gsz = min(gm - first_m, GROUP);
  // tile_lim > 0 (gemm7's leading rounds): the first tile_lim tiles in row-major order
  const int tm = tile_lim > 0 ? wg / gn : first_m + (wg % (GROUP * gn)) % gsz;
  const int tn = tile_lim > 0 ? wg % gn : (wg % (GROUP * gn)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63, hl = lane >> 5, l32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int wm = wr * (BM / WM), wn = wc * (BN / WN);

  const int nsplit = gridDim.y;
  const int ktiles = K / BK;
  const int kt0 = split * ktiles / nsplit;
  const int nk = (split + 1) * ktiles / nsplit - kt0;

  // staging: this wave's two 1 KiB pieces (j = 0, 1) of every half-tile.  Piece rows
  // i = 64 j + 8 wave + (lane >> 3); swz8 reads row bits 1-3, i.e. i & 15 = 8 (wave & 1) + lr.
  static_assert(!TT || M16, "the TT build exists with 16x16x32 MFMAs only");
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ (M16 ? swzq(8 * (wave & 1) + lr) : swz8(8 * (wave & 1) + lr));
  const bf16_t* pa[2];
  const bf16_t* pb[2];
  // TT (both operands stored k-major: A^T [K][M], B [K][N], the dW GEMMs): a half-tile is a
  // [64 k][128 col] image with 256-byte rows; piece p = wave + 8 j holds k-rows 4p..4p+3,
  // lane l lands at k-row 4p + (l >> 4), physical chunk l & 15 = logical chunk ^ swz16(k-row)
  // (swz16 of that row = ((l >> 4) << 2) | (wave & 3)).  Image column c of A0 is tile row
  // c < 64 ? c : c + 64 (A1: + 64); of B0 tile column 64 (c / 32) + c % 32 (B1: + 32).
  const bf16_t* ta1[2];
  const bf16_t* tb1[2];
  if constexpr (TT) {
    const int kr = lane >> 4;
    const int ic = 8 * ((lane & 15) ^ ((kr << 2) | (wave & 3)));
    const int am = ic < 64 ? ic : ic + 64, bn = 64 * (ic >> 5) + (ic & 31);
    auto cm = [&](int m) { return m < M ? m : M - 8; };
    auto cn = [&](int n) { return n < N ? n : N - 8; };
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t krow = (int64_t)kt0 * BK + 4 * wave + 32 * j + kr;
      pa[j] = A + krow * lda + cm(m0 + am);
      ta1[j] = A + krow * lda + cm(m0 + am + 64);
      pb[j] = B + krow * ldb + cn(n0 + bn);
      tb1[j] = B + krow * ldb + cn(n0 + bn + 32);
    }
  }
#pragma unroll
  for (int j = 0; j < 2 && !TT; ++j) {
    int ra = m0 + 128 * j + 8 * wave + lr;          // A0 row; A1 = +64
    ra = ra < M ? ra : M - 1;
    int rb = n0 + 64 * ((wave >> 2) + 2 * j) + 8 * (wave & 3) + lr;   // B0 row (= output col); B1 = +32
    rb = rb < N ? rb : N - 1;
    pa[j] = A + (int64_t)ra * lda + (int64_t)kt0 * BK + lc * 8;
    pb[j] = B + (int64_t)rb * ldb + (int64_t)kt0 * BK + lc * 8;
  }
  // rows past the M/N edge of the A1/B1 halves: clamp by pointer (the +64/+32 offsets)
  const bool a1_ok0 = m0 + 64 + 8 * wave + lr < M, a1_ok1 = m0 + 192 + 8 * wave + lr < M;
  const bool b1_ok0 = n0 + 64 * (wave >> 2) + 32 + 8 * (wave & 3) + lr < N;
  const bool b1_ok1 = n0 + 64 * ((wave >> 2) + 2) + 32 + 8 * (wave & 3) + lr < N;
  const int64_t a1_off0 = a1_ok0 ? 64 * lda : 0, a1_off1 = a1_ok1 ? 64 * lda : 0;
  const int64_t b1_off0 = b1_ok0 ? 32 * ldb : 0, b1_off1 = b1_ok1 ? 32 * ldb : 0;

  // half-tile h (0 = A0, 1 = B0, 2 = B1, 3 = A1: consumption order) of K-tile kt -> buffer kt & 1
  auto issue = [&](int h, int kt) {
    char* img = smem + (kt & 1) * BUF + (h == 0 ? 0 : h == 3 ? HALF : h == 1 ? 2 * HALF : 3 * HALF);
    if constexpr (TT) {
      const int64_t da = (int64_t)kt * BK * lda, db = (int64_t)kt * BK * ldb;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16_t* src = h == 0 ? pa[j] + da : h == 3 ? ta1[j] + da : h == 1 ? pb[j] + db : tb1[j] + db;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(img + (wave + 8 * j) * 1024), 16,
                                         0, 0);
      }
      return;
    }
    const int64_t dk = (int64_t)kt * BK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16_t* src;
      if (h == 0) src = pa[j] + dk;
      else if (h == 3) src = pa[j] + dk + (j ? a1_off1 : a1_off0);
      else if (h == 1) src = pb[j] + dk;
      else src = pb[j] + dk + (j ? b1_off1 : b1_off0);
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(img + (wave + 8 * j) * 1024), 16, 0,
                                       0);
    }
  };

  if constexpr (!M16) {
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x16{};

  // Half-tile DMA runs ~1.5 K-tiles ahead, one half-tile (2 glds per thread) per phase so
  // the DMA issue cost is spread evenly; a slot is re-filled >= 2 phases after its last
  // ds_read (WAR across the staggered wave rows, cdna guide §5 "8-phase template"):
  //   tile t  phase 1: B1(t+1)   phase 2: A1(t+1)   phase 3: A0(t+2)   phase 4: B0(t+2)
  // Each phase's counted vmcnt(8) retires exactly the half-tile the next phase reads; the
  // last two K-tiles drain with vmcnt(0).
  issue(0, 0);
  issue(1, 0);
  issue(2, 0);
  issue(3, 0);
  if (nk > 1) {
    issue(0, 1);
    issue(1, 1);
    wait_vmcnt<8>();
  } else {
    wait_vmcnt<4>();
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier
  asm volatile("" ::: "memory");

  bf16x8 af[2][4], b0[4], b1[4];
  const int rA = wr * 64 + l32;   // image row of this wave's quadrant row-block 0
  const int rB = wc * 32 + l32;

#define G3_MFMA(I0, BF, CI)                                                           \
  __builtin_amdgcn_sched_barrier(0);                                                  \
  __builtin_amdgcn_s_setprio(1);                                                      \
  _Pragma("unroll") for (int s_ = 0; s_ < 4; ++s_) {                                  \
    acc[I0][CI] = mfma32(af[0][s_], BF[s_], acc[I0][CI]);                             \
    acc[I0 + 1][CI] = mfma32(af[1][s_], BF[s_], acc[I0 + 1][CI]);                     \
  }                                                                                   \
  __builtin_amdgcn_s_setprio(0);                                                      \
  __builtin_amdgcn_sched_barrier(0);
#define G3_BAR()                          \
  asm volatile("" ::: "memory");          \
  __builtin_amdgcn_s_barrier();           \
  asm volatile("" ::: "memory");

  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    const bool steady = t + 2 < nk;
    // ---- phase 1: A0 x B0
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_) {
      af[0][s_] = frag<false, BM>(buf, rA, s_, hl);
      af[1][s_] = frag<false, BM>(buf, rA + 32, s_, hl);
      b0[s_] = frag<false, BN>(buf + 2 * HALF, rB, s_, hl);
    }
    if (t + 1 < nk) issue(2, t + 1);
    if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();   // B1(t) landed
    G3_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G3_MFMA(0, b0, 0);
    G3_BAR();
    // ---- phase 2: A0 x B1
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_) b1[s_] = frag<false, BN>(buf + 3 * HALF, rB, s_, hl);
    if (t + 1 < nk) issue(3, t + 1);
    if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();   // A1(t) landed
    G3_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G3_MFMA(0, b1, 1);
    G3_BAR();
    // ---- phase 3: A1 x B0; refill A0 of this buffer for K-tile t+2
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_) {
      af[0][s_] = frag<false, BM>(buf + HALF, rA, s_, hl);
      af[1][s_] = frag<false, BM>(buf + HALF, rA + 32, s_, hl);
    }
    if (steady) issue(0, t + 2);
    G3_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G3_MFMA(2, b0, 0);
    G3_BAR();
    // ---- phase 4: A1 x B1; refill B0; A0/B0 of K-tile t+1 retired for the next phase 1
    if (steady) {
      issue(1, t + 2);
      wait_vmcnt<8>();
    } else {
      wait_vmcnt<0>();
    }
    G3_BAR();
    G3_MFMA(2, b1, 1);
    G3_BAR();
  }
#undef G3_MFMA
#undef G3_BAR
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the staggered wave rows
  __syncthreads();
  epilogue<BM, BN, WM, WN, EPI, ACC>(Stage32<4, 2>{acc, wn, hl, l32}, smem, m0, n0, wr, Cv, bias, R, AUX, WS, M,
                                     N, ldc, ldr, ldx, alpha, nsplit, p_drop, seed, nullptr, 0, 0, split);
  } else {
  // 16x16x32 MFMAs: same phases, DMA and barriers; a phase quadrant (64 rows x 32 cols)
  // is 4 x 2 blocks of 16x16, K = 64 in two 32-deep steps (16 MFMAs of 16 cycles)
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  // Half-tile DMA runs ~1.5 K-tiles ahead, one half-tile (2 glds per thread) per phase so
  // the DMA issue cost is spread evenly; a slot is re-filled >= 2 phases after its last
  // ds_read (WAR across the staggered wave rows, cdna guide §5 "8-phase template"):
  //   tile t  phase 1: B1(t+1)   phase 2: A1(t+1)   phase 3: A0(t+2)   phase 4: B0(t+2)
  // Each phase's counted vmcnt(8) retires exactly the half-tile the next phase reads; the
  // last two K-tiles drain with vmcnt(0).
  issue(0, 0);
  issue(1, 0);
  issue(2, 0);
  issue(3, 0);
  if (nk > 1) {
    issue(0, 1);
    issue(1, 1);
    wait_vmcnt<8>();
  } else {
    wait_vmcnt<4>();
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier
  asm volatile("" ::: "memory");

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  const int q = lane >> 4;
  const int rA = wr * 64 + (lane & 15);
  const int rB = wc * 32 + (lane & 15);
  auto fq = [&](const char* img, int row, int st) -> bf16x8 {
    if constexpr (TT) return frag16<true, 128>(img, row - (lane & 15), st);   // row = base + (lane & 15)
    else return *reinterpret_cast<const bf16x8*>(img + row * 128 + 16 * ((4 * st + q) ^ swzq(row)));
  };

#define G4_MFMA(R0, BF, C0)                                                              \
  __builtin_amdgcn_sched_barrier(0);                                                     \
  __builtin_amdgcn_s_setprio(1);                                                         \
  _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                       \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                       \
  _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                       \
    acc[R0 + i_][C0 + j_] = mfma16(af[i_][s_], BF[j_][s_], acc[R0 + i_][C0 + j_]);       \
  __builtin_amdgcn_s_setprio(0);                                                         \
  __builtin_amdgcn_sched_barrier(0);
#define G3_BAR()                          \
  asm volatile("" ::: "memory");          \
  __builtin_amdgcn_s_barrier();           \
  asm volatile("" ::: "memory");

  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    const bool steady = t + 2 < nk;
    // ---- phase 1: A0 x B0
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_) {
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][s_] = fq(buf, rA + 16 * i, s_);
#pragma unroll
      for (int j = 0; j < 2; ++j) b0[j][s_] = fq(buf + 2 * HALF, rB + 16 * j, s_);
    }
    if (t + 1 < nk) issue(2, t + 1);
    if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();   // B1(t) landed
    G3_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G4_MFMA(0, b0, 0);
    G3_BAR();
    // ---- phase 2: A0 x B1
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
      for (int j = 0; j < 2; ++j) b1[j][s_] = fq(buf + 3 * HALF, rB + 16 * j, s_);
    if (t + 1 < nk) issue(3, t + 1);
    if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();   // A1(t) landed
    G3_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G4_MFMA(0, b1, 2);
    G3_BAR();
    // ---- phase 3: A1 x B0; refill A0 of this buffer for K-tile t+2
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][s_] = fq(buf + HALF, rA + 16 * i, s_);
    if (steady) issue(0, t + 2);
    G3_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G4_MFMA(4, b0, 0);
    G3_BAR();
    // ---- phase 4: A1 x B1; refill B0
    if (steady) {
      issue(1, t + 2);
      wait_vmcnt<8>();
    } else {
      wait_vmcnt<0>();
    }
    G3_BAR();
    G4_MFMA(4, b1, 2);
    G3_BAR();
  }
#undef G4_MFMA
#undef G3_BAR
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the staggered wave rows
  __syncthreads();
  epilogue<BM, BN, WM, WN, EPI, ACC>(Stage16<8, 4>{acc, wn, lane}, smem, m0, n0, wr, Cv, bias, R, AUX, WS, M, N, ldc,
                                     ldr, ldx, alpha, nsplit, p_drop, seed, nullptr, 0, 0, split);
  }
}

template <int EPI, bool ACC, bool M16, bool TT = false>
static int launch3(const void* A, const void* B, void* C, const void* bias, const void* R, void* X, float* ws, int M,
                   int N, int K,
                   int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha, int split,
                   float p_drop, uint64_t seed, hipStream_t st, int tile_lim = 0) {
  constexpr int LDS_MAIN = 2 * 4 * 128 * 128;
  constexpr int EPI_BYTES = 128 * (256 + 4) * 4;
  constexpr int LDS = LDS_MAIN > EPI_BYTES ? LDS_MAIN : EPI_BYTES;
  auto kern = gemm3_kernel<EPI, ACC, M16, TT>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int nwg = tile_lim > 0 ? tile_lim : ((M + 255) / 256) * ((N + 255) / 256);
  // opt-in (MIPIPE_G3_SPLIT_REMAP=1): +3-10 % on GPT-2 small's dW GEMMs standalone, neutral
  // in that step, but -0.8 % on the GPT-2 large step (2 same-box pairs,
  // profiles/r5_gemm3_splitk_xcd_remap.md)
  static const bool split_remap = [] {
    const char* e = getenv("MIPIPE_G3_SPLIT_REMAP");
    return e && e[0] == '1';
  }();
  if (tile_lim == 0 && !split_remap) tile_lim = -1;
  kern<<<dim3(nwg, split), NT, LDS, st>>>((const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias,
                                          (const bf16_t*)R, (bf16_t*)X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed,
                                          tile_lim);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// gemm6: gemm3's ping-pong phase schedule (16x16x32 MFMAs, NT) on 256x192 tiles.
//
// Why: at the 32K-token microbatch of a PP > 1 rank the N = 768 GEMMs (fwd wo / fc2, dX of
// qkv / wo / fc1) are 128 x 3 = 384 tiles of 256x256 = 1.5 rounds of 256 CUs: the second
// round runs on half the chip (profiles/r3_gemm_tail_probe.txt: 0.83-0.92x hipBLASLt there,
// 1.0x+ at M = 65536 where the grid is 3 whole rounds).  256x192 tiles make N = 768 four
// tile columns (512 tiles = 2 whole rounds) and N = 2304 twelve (6 rounds instead of 4.5).
// gemm2's 256x192 build (cfg 1) has the tile but not the schedule (2 stages, 4x slower
// feed: 0.95x of gemm3 in the same probe).
//
// Layout: 8 waves as 4 (rows) x 2 (cols), 64 x 96 outputs each.  A K-tile (BK = 64) is four
// LDS images, streamed one per phase exactly as in gemm3:
//   A0 = rows {0..31, 64..95, 128..159, 192..223} (the first 32 rows of each wave row)
//   A1 = the other 128 rows                                      (16 KiB each)
//   B0 = cols {0..47, 96..143}   B1 = cols {48..95, 144..191}    (96 rows, 12 KiB each)
// phase 1: A0 x B0, 2: A0 x B1, 3: A1 x B0, 4: A1 x B1 -- 2 x 3 blocks of 16x16, K = 64
// in two 32-deep steps = 12 MFMAs per phase.  An A image is 16 one-KiB pieces (2 per
// wave); a B image 12 (waves 0-3 issue 2, waves 4-7 one), so each wave's counted vmcnt
// is 4 + 2 b (b = its B pieces per image): the wait retires exactly the image the next
// phase reads, per issuing wave, and the barrier after it publishes it to all waves.
// Waves 4-7 (one per SIMD, the partner of wave w - 4) run one barrier behind waves 0-3.
// ---------------------------------------------------------------------------------------
template <int EPI, bool ACC>
__global__ void __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm6_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, void* __restrict__ Cv,
             const bf16_t* __restrict__ bias, const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX,
             float* __restrict__ WS, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr,
             int64_t ldx, float alpha, float p_drop, uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  constexpr int BM = 256, BN = 192, WM = 4, WN = 2;
  constexpr int HA = 32, HB = 48;                 // a wave's rows / cols in one A / B image
  constexpr int IMG_A = 128 * 128, IMG_B = 96 * 128;
  constexpr int O_A1 = IMG_A, O_B0 = 2 * IMG_A, O_B1 = 2 * IMG_A + IMG_B;
  constexpr int BUF = 2 * IMG_A + 2 * IMG_B;      // 56 KiB per K-tile, two buffers
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  const int nwg = gm * gn;
  const int wg = xcd_remap((int)blockIdx.x, nwg);
  constexpr int GROUP = MP_G3_GROUP;
  const int group = wg / (GROUP * gn);
  const int first_m = group * GROUP;
  const int gsz = min(gm - first_m, GROUP);
  const int tm = first_m + (wg % (GROUP * gn)) % gsz;
  const int tn = (wg % (GROUP * gn)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int grp = wave >> 2;                      // ping-pong group (waves w, w + 4 share a SIMD)
  const int wn = wc * (BN / WN);

  const int nk = K / BK;

  // staging: piece p = wave + 8 j holds image rows 8 p .. 8 p + 7 (lane row lr = lane >> 3,
  // 16-byte chunk lane & 7); image row r & 15 = 8 (wave & 1) + lr for every piece
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ swzq(8 * (wave & 1) + lr);
  const bool two_b = wave < 4;                    // B images: 12 pieces, waves 0-3 take the last 4
  const bf16_t* pa0[2];
  const bf16_t* pa1[2];
  const bf16_t* pb0[2];
  const bf16_t* pb1[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 8 * (wave + 8 * j) + lr;        // image row
    int a0 = m0 + (r / HA) * (BM / WM) + r % HA, a1 = a0 + HA;
    a0 = a0 < M ? a0 : M - 1;                     // rows past the edge only feed masked outputs
    a1 = a1 < M ? a1 : M - 1;
    pa0[j] = A + (int64_t)a0 * lda + lc * 8;
    pa1[j] = A + (int64_t)a1 * lda + lc * 8;
    const int rb = r < 96 ? r : r - 64;           // waves 4-7, j = 1: no piece (never issued)
    int b0 = n0 + (rb / HB) * (BN / WN) + rb % HB, b1 = b0 + HB;
    b0 = b0 < N ? b0 : N - 1;
    b1 = b1 < N ? b1 : N - 1;
    pb0[j] = B + (int64_t)b0 * ldb + lc * 8;
    pb1[j] = B + (int64_t)b1 * ldb + lc * 8;
  }

  // image h (0 = A0, 1 = B0, 2 = B1, 3 = A1: consumption order) of K-tile kt -> buffer kt & 1
  auto issue = [&](int h, int kt) {
    char* img = smem + (kt & 1) * BUF + (h == 0 ? 0 : h == 3 ? O_A1 : h == 1 ? O_B0 : O_B1);
    const int64_t dk = (int64_t)kt * BK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j == 1 && (h == 1 || h == 2) && !two_b) continue;
      const bf16_t* src = (h == 0 ? pa0[j] : h == 3 ? pa1[j] : h == 1 ? pb0[j] : pb1[j]) + dk;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(img + (wave + 8 * j) * 1024), 16, 0,
                                       0);
    }
  };
  // counted waits (derivation in the header): 4 + 2 b outstanding pieces, 2 + b for nk = 1
  auto wait_steady = [&]() {
    if (two_b) wait_vmcnt<8>(); else wait_vmcnt<6>();
  };

  f32x4 acc[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{};

  issue(0, 0);
  issue(1, 0);
  issue(2, 0);
  issue(3, 0);
  if (nk > 1) {
    issue(0, 1);
    issue(1, 1);
    wait_steady();
  } else {
    if (two_b) wait_vmcnt<4>(); else wait_vmcnt<3>();
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger the two wave groups by one barrier
  asm volatile("" ::: "memory");

  bf16x8 af[2][2], b0[3][2], b1[3][2];
  const int q = lane >> 4;
  const int rA = wr * HA + (lane & 15);
  const int rB = wc * HB + (lane & 15);
  auto fq = [&](const char* img, int row, int st) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + 16 * ((4 * st + q) ^ swzq(row)));
  };

#define G6_MFMA(R0, BF, C0)                                                              \
  __builtin_amdgcn_sched_barrier(0);                                                     \
  __builtin_amdgcn_s_setprio(1);                                                         \
  _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                       \
  _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_)                                       \
  _Pragma("unroll") for (int j_ = 0; j_ < 3; ++j_)                                       \
    acc[R0 + i_][C0 + j_] = mfma16(af[i_][s_], BF[j_][s_], acc[R0 + i_][C0 + j_]);       \
  __builtin_amdgcn_s_setprio(0);                                                         \
  __builtin_amdgcn_sched_barrier(0);
#define G6_BAR()                          \
  asm volatile("" ::: "memory");          \
  __builtin_amdgcn_s_barrier();           \
  asm volatile("" ::: "memory");

  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    const bool steady = t + 2 < nk;
    // ---- phase 1: A0 x B0
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_) {
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i][s_] = fq(buf, rA + 16 * i, s_);
#pragma unroll
      for (int j = 0; j < 3; ++j) b0[j][s_] = fq(buf + O_B0, rB + 16 * j, s_);
    }
    if (t + 1 < nk) issue(2, t + 1);
    if (steady) wait_steady(); else wait_vmcnt<0>();   // B1(t) landed
    G6_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G6_MFMA(0, b0, 0);
    G6_BAR();
    // ---- phase 2: A0 x B1
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
      for (int j = 0; j < 3; ++j) b1[j][s_] = fq(buf + O_B1, rB + 16 * j, s_);
    if (t + 1 < nk) issue(3, t + 1);
    if (steady) wait_steady(); else wait_vmcnt<0>();   // A1(t) landed
    G6_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G6_MFMA(0, b1, 3);
    G6_BAR();
    // ---- phase 3: A1 x B0; refill A0 of this buffer for K-tile t+2
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i][s_] = fq(buf + O_A1, rA + 16 * i, s_);
    if (steady) issue(0, t + 2);
    G6_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G6_MFMA(2, b0, 0);
    G6_BAR();
    // ---- phase 4: A1 x B1; refill B0; A0/B0 of K-tile t+1 retired for the next phase 1
    if (steady) {
      issue(1, t + 2);
      wait_steady();
    } else {
      wait_vmcnt<0>();
    }
    G6_BAR();
    G6_MFMA(2, b1, 3);
    G6_BAR();
  }
#undef G6_MFMA
#undef G6_BAR
  if (grp == 0) __builtin_amdgcn_s_barrier();  // re-align the staggered groups
  __syncthreads();
  epilogue<BM, BN, WM, WN, EPI, ACC>(Stage16<4, 6>{acc, wn, lane}, smem, m0, n0, wr, Cv, bias, R, AUX, WS, M, N, ldc,
                                     ldr, ldx, alpha, 1, p_drop, seed);
}

template <int EPI, bool ACC>
static int launch6(const void* A, const void* B, void* C, const void* bias, const void* R, void* X, float* ws, int M,
                   int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha,
                   float p_drop, uint64_t seed, hipStream_t st) {
  constexpr int LDS_MAIN = 2 * (2 * 128 * 128 + 2 * 96 * 128);
  constexpr int EPI_BYTES = 64 * (192 + 4) * 4;
  constexpr int LDS = LDS_MAIN > EPI_BYTES ? LDS_MAIN : EPI_BYTES;
  auto kern = gemm6_kernel<EPI, ACC>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int nwg = ((M + 255) / 256) * ((N + 191) / 192);
  kern<<<dim3(nwg, 1), NT, LDS, st>>>((const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias, (const bf16_t*)R,
                                      (bf16_t*)X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// gemm8: 256x192 NT, FOUR waves -- one wave per SIMD, a 128 x 96 accumulator tile per wave
// (8 x 6 blocks of 16x16x32, 192 accumulator registers) -- register-staged with a whole
// K-tile of prefetch in flight.  The main-loop shape of the library kernel torch picks for
// GPT-2's K = 768 GEMMs on gfx950 (hipBLASLt MT192x256x64 MI16x16x1 MIWT6_8 PGR2, its
// .s read in profiles/r6_hipblaslt_mainloop.md), where gemm3's two ping-pong waves per SIMD
// run at 0.6-0.89x the library (profiles/r6_gemm_step_shapes.md).
//
// Per K-tile (BK = 64) a wave issues 96 MFMAs (2 k-steps x 8 x 6) and, in the MFMA gaps:
//   * the 14 ds_read_b128 fragments of the NEXT k-step (register double buffer), the
//     k-step-0 ones of the next K-tile right after the barrier, under the last 18 MFMAs;
//   * the 14 staging pairs: ds_write_b128 of K-tile t+1 (loaded during tile t-1) into the
//     other LDS buffer, then buffer_load_dwordx4 of K-tile t+2 into the freed registers
//     (the compiler's counted vmcnt(13) per write retires exactly its own load).
// One barrier per K-tile; two LDS buffers 64 KiB apart.  Nothing here is a DMA-to-LDS
// (global_load_lds): a register-staged ring keeps one K-tile more in flight than two LDS
// buffers of glds can (the gemm5 probe: 0.7-0.8x gemm3 with a one-tile glds ring).
// The epilogue is gemm2's LDS-staged one (2 passes of 128 rows).
// ---------------------------------------------------------------------------------------
typedef unsigned int u32x4g8 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void g8_wait_lgkm0() {
  // s_waitcnt lgkmcnt(0), vmcnt / expcnt left at their maxima (no wait)
  __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
}

template <int EPI, bool ACC, int PGR>
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm8_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, void* __restrict__ Cv,
             const bf16_t* __restrict__ bias, const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX,
             float* __restrict__ WS, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr,
             int64_t ldx, float alpha, float p_drop, uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  constexpr int BM = 256, BN = 192, NTH8 = 256;
  constexpr int AIMG = BM * 128;     // A image [256 rows][64 k], 128-byte rows (swzq)
  constexpr int BUFSTRIDE = 0x10000; // B image at +AIMG; buffer 1 at +64 KiB
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  const int nwg = gm * gn;
  const int wg = xcd_remap((int)blockIdx.x, nwg);
  constexpr int GROUP = MP_G3_GROUP;
  const int group = wg / (GROUP * gn);
  const int first_m = group * GROUP;
  const int gsz = min(gm - first_m, GROUP);
  const int tm = first_m + (wg % (GROUP * gn)) % gsz;
  const int tn = (wg % (GROUP * gn)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = K / BK;

  // staging: thread t moves 16-byte chunk (t & 7) of tile rows (t >> 3) + 32 u; the LDS
  // slot is that row's chunk ^ swz8(row) (row bits 1-3 = those of t >> 3: one base).  One
  // buffer resource per operand at the tile's first row: row u of a thread is a scalar
  // offset (32 u rows), and rows past the M / N edge fall outside num_records, so the
  // hardware returns zeros for them (masked outputs only) -- no per-row clamp registers
  const int srow = tid >> 3, sch = tid & 7;
  const int mrows = min(BM, M - m0), nrows = min(BN, N - n0);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A + (int64_t)m0 * lda), 0, (int)(((int64_t)(mrows - 1) * lda + K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(B + (int64_t)n0 * ldb), 0, (int)(((int64_t)(nrows - 1) * ldb + K) * 2), 0x00020000);
  const int voa = (int)(((int64_t)srow * lda + sch * 8) * 2);
  const int vob = (int)(((int64_t)srow * ldb + sch * 8) * 2);
  const int rsa = (int)(32 * lda * 2), rsb = (int)(32 * ldb * 2);   // bytes per 32 rows
  const int dst = srow * 128 + 16 * (sch ^ swz8(srow));   // + 4096 u (A), + AIMG + 4096 u (B)

  // fragment reads (32x32x16: lane reads row base + (lane & 31), k-chunk 2 s + hl of the
  // 16-deep k-step s): chunk ^ swz8(row) with row bits 1-3 = lane bits 1-3, so per k-step one
  // base per operand and + 4096 per 32-row block
  const int hl = lane >> 5, l32 = lane & 31;
  const int c0 = hl ^ swz8(l32);
  int fa_off[4], fb_off[4];
#pragma unroll
  for (int s_ = 0; s_ < 4; ++s_) {
    fa_off[s_] = (wr * 128 + l32) * 128 + 16 * ((2 * s_) ^ c0);
    fb_off[s_] = AIMG + (wc * 96 + l32) * 128 + 16 * ((2 * s_) ^ c0);
  }

  // PGR K-tiles in flight: K-tile t+1 waits in register set (t+1) % NSET while the loads of
  // K-tile t+PGR go out into the set just written (PGR 2: one set, hipBLASLt's PGR2)
  constexpr int NSET = PGR - 1;
  u32x4g8 st[NSET][14];
  bf16x8 fx[7], fy[7];     // fragments of even / odd k-steps: A blocks 0-3, B blocks 0-2
  f32x16 acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x16{};

  auto gload = [&](auto SET, int u, int kt) {
    constexpr int S = decltype(SET)::value;
    if (u < 8) st[S][u] = __builtin_amdgcn_raw_buffer_load_b128(ra, voa, kt * 128 + u * rsa, 0);
    else st[S][u] = __builtin_amdgcn_raw_buffer_load_b128(rb, vob, kt * 128 + (u - 8) * rsb, 0);
  };
  auto swrite = [&](auto SET, int boff, int u) {
    constexpr int S = decltype(SET)::value;
    const int off = u < 8 ? dst + 4096 * u : AIMG + dst + 4096 * (u - 8);
    *reinterpret_cast<u32x4g8*>(smem + boff + off) = st[S][u];
  };
  auto fread = [&](bf16x8 (&f)[7], int boff, int s_) {
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = *reinterpret_cast<const bf16x8*>(smem + boff + fa_off[s_] + 4096 * i);
#pragma unroll
    for (int j = 0; j < 3; ++j) f[4 + j] = *reinterpret_cast<const bf16x8*>(smem + boff + fb_off[s_] + 4096 * j);
  };
  auto mma = [&](const bf16x8 (&f)[7]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[i][j] = mfma32(f[i], f[4 + j], acc[i][j]);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, NSET - 1>;   // set of odd K-tiles

  // prologue: K-tiles 0 .. PGR-1 in flight, K-tile 0 into LDS buffer 0, k-step-0 fragments
#pragma unroll
  for (int u = 0; u < 14; ++u) gload(I0{}, u, 0);
  if constexpr (NSET > 1) {
#pragma unroll
    for (int u = 0; u < 14; ++u) gload(I1{}, u, min(1, nk - 1));
  }
#pragma unroll
  for (int u = 0; u < 14; ++u) swrite(I0{}, 0, u);
#pragma unroll
  for (int u = 0; u < 14; ++u) gload(I0{}, u, min(NSET, nk - 1));
  g8_wait_lgkm0();
  __builtin_amdgcn_s_barrier();
  fread(fx, 0, 0);

  // K-tile t from the buffer at `cur` (0 / 64 KiB, toggled per K-tile); K-tile t+1 staged
  // into the other one during k-steps 0-2 (5 + 5 + 4 write / load pairs), one barrier, and
  // the next K-tile's k-step-0 fragments read under k-step 3
  int cur = 0;
  auto ktile = [&](int t, auto SET) {
    const int nxt = cur ^ BUFSTRIDE;
    const int kl = min(t + PGR, nk - 1);   // the tail re-loads the last K-tile: never read
    // k-steps 0-2: each issues the next k-step's 7 fragment reads under its first 7 MFMAs,
    // then (ds_write, buffer_load) staging pairs under the rest (5 + 5 + 4 pairs); a
    // sched_barrier closes every k-step, so no MFMA moves next to the reads it waits on
    auto kstep = [&](auto& fcur, auto& fnext, int s_next, int u0, auto U1) {
      constexpr int u1 = decltype(U1)::value, rest = u1 == 14 ? 2 : 0;
      fread(fnext, cur, s_next);
      mma(fcur);
#pragma unroll
      for (int u = u0; u < u1; ++u) {
        swrite(SET, nxt, u);
        gload(SET, u, kl);
      }
#pragma unroll
      for (int g = 0; g < 7; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int g = 0; g < u1 - u0; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      if constexpr (rest > 0) __builtin_amdgcn_sched_group_barrier(0x008, rest, 0);
      __builtin_amdgcn_sched_barrier(0);
    };
    kstep(fx, fy, 1, 0, std::integral_constant<int, 5>{});
    kstep(fy, fx, 2, 5, std::integral_constant<int, 10>{});
    kstep(fx, fy, 3, 10, std::integral_constant<int, 14>{});
    // every wave's staging writes of K-tile t+1 and fragment reads of K-tile t are done
    g8_wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    // k-step 3 covers the next K-tile's k-step-0 fragment reads
    fread(fx, nxt, 0);
    mma(fy);
#pragma unroll
    for (int g = 0; g < 7; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 5, 1);
    __builtin_amdgcn_sched_barrier(0);
    cur = nxt;
  };
  int t = 0;
  if constexpr (NSET == 1) {
#pragma unroll 1
    for (; t < nk; ++t) ktile(t, I0{});
  } else {
#pragma unroll 1
    for (; t + 1 < nk; t += 2) {
      ktile(t, I1{});       // K-tile t+1 (odd) waits in set 1
      ktile(t + 1, I0{});
    }
    if (t < nk) ktile(t, I1{});
  }
  __syncthreads();
  epilogue<BM, BN, 2, 2, EPI, ACC, NTH8>(Stage32<4, 3>{acc, wc * 96, hl, l32}, smem, m0, n0, wr, Cv, bias, R, AUX,
                                         WS, M, N, ldc, ldr, ldx, alpha, 1, p_drop, seed);
}

template <int EPI, bool ACC, int PGR = 2>
static int launch8(const void* A, const void* B, void* C, const void* bias, const void* R, void* X, float* ws, int M,
                   int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha,
                   float p_drop, uint64_t seed, hipStream_t st) {
  constexpr int LDS_MAIN = 0x10000 + 256 * 128 + 192 * 128;   // buffer 1 ends at 120 KiB
  constexpr int EPI_BYTES = 128 * (192 + 4) * 4;
  constexpr int LDS = LDS_MAIN > EPI_BYTES ? LDS_MAIN : EPI_BYTES;
  auto kern = gemm8_kernel<EPI, ACC, PGR>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int nwg = ((M + 255) / 256) * ((N + 191) / 192);
  kern<<<dim3(nwg, 1), 256, LDS, st>>>((const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias, (const bf16_t*)R,
                                       (bf16_t*)X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// gemm7: the PARTIAL round of a 256x256 NT GEMM split over all CUs -- a pipeline rank's
// 8K-32K-token microbatches are 96-384 tiles of 256x256 for N = 768, i.e. 0.4-1.5 rounds of
// 256 CUs (profiles/r5_gemm7_*).  The host runs the whole rounds as a plain gemm3 launch on
// the leading rows and this kernel on the remaining tail rows (mp_gemm2, cfg 14).
//
// The tail's tiles are split into 8 XCD groups (consecutive tile ids; block b runs on XCD
// b % 8) and each of a group's c tiles into S K-chunks: the group's workgroup l (b = x + 8 l,
// in dispatch order) computes chunk j = l / c of tile l % c.  Workgroups of one chunk index
// walk the same K range of neighbouring tiles at the same time, so A panels are shared in
// the XCD's L2 (a stream-K walk that staggers K offsets across the tiles of one row band
// measured 2.4x slower: the A panel is re-read from HBM per tile).  Chunks 0..S-2 publish
// f32 partials; the last chunk's workgroup owns the tile: it absorbs the others (they were
// dispatched before it, hold a CU or are done -- no deadlock even when other kernels occupy
// CUs) and runs the fused epilogue.
//
// Hand-off (cdna guide §6 Guideline 16, R1): the partial is staged through LDS like the
// epilogue and stored row-major with sc1 (write-through) 16-byte buffer stores, every wave
// drains vmcnt, workgroup barrier, one agent-scope 8-byte flag store of a 64-bit tag; the
// owner's thread 0 polls the flags (bounded: a lost hand-off sets an error word instead of
// hanging), clears them, takes one agent-scope acquire, barrier, and the epilogue adds the
// partials (plain loads) to the LDS-staged accumulator before the fused epilogue.  So every flag is back to 0 when a launch ends and no
// memset node is needed before the next (one measured 5.3 us per call): a fresh workspace
// from the caching allocator can only hold the tag by a 2^-64 accident.
// ---------------------------------------------------------------------------------------
#ifndef MP_G7_SC1
#define MP_G7_SC1 0   // 1: partials by sc1 write-through buffer stores (no release fence)
#endif
constexpr int SK_SLOT = 256 * 256;          // floats per partial tile
constexpr int SK_FLAGS = 2 * 256 + 16;      // 256 64-bit flags + the error word (floats of workspace)
constexpr int SK_ERR = 2 * 256;             // error word (as a 32-bit index)
constexpr int SK_MAX_G = 256;
constexpr unsigned long long SK_TAG = 0x7FF7A5A55A5AC3C3ull;   // a NaN payload: never f32 data

__device__ __forceinline__ void g7_mainloop(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, int M, int N,
                                            int64_t lda, int64_t ldb, int m0, int n0, int kt0, int nk, char* smem,
                                            f32x4 (&acc)[8][4]) {
  constexpr int HALF = 128 * 128;
  constexpr int BUF = 4 * HALF;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / 4, wc = wave % 4;
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ swzq(8 * (wave & 1) + lr);
  const bf16_t* pa[2];
  const bf16_t* pb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int ra = m0 + 128 * j + 8 * wave + lr;
    ra = ra < M ? ra : M - 1;
    int rb = n0 + 64 * ((wave >> 2) + 2 * j) + 8 * (wave & 3) + lr;
    rb = rb < N ? rb : N - 1;
    pa[j] = A + (int64_t)ra * lda + (int64_t)kt0 * BK + lc * 8;
    pb[j] = B + (int64_t)rb * ldb + (int64_t)kt0 * BK + lc * 8;
  }
  const bool a1_ok0 = m0 + 64 + 8 * wave + lr < M, a1_ok1 = m0 + 192 + 8 * wave + lr < M;
  const bool b1_ok0 = n0 + 64 * (wave >> 2) + 32 + 8 * (wave & 3) + lr < N;
  const bool b1_ok1 = n0 + 64 * ((wave >> 2) + 2) + 32 + 8 * (wave & 3) + lr < N;
  const int64_t a1_off0 = a1_ok0 ? 64 * lda : 0, a1_off1 = a1_ok1 ? 64 * lda : 0;
  const int64_t b1_off0 = b1_ok0 ? 32 * ldb : 0, b1_off1 = b1_ok1 ? 32 * ldb : 0;
  auto issue = [&](int h, int kt) {
    char* img = smem + (kt & 1) * BUF + (h == 0 ? 0 : h == 3 ? HALF : h == 1 ? 2 * HALF : 3 * HALF);
    const int64_t dk = (int64_t)kt * BK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16_t* src;
      if (h == 0) src = pa[j] + dk;
      else if (h == 3) src = pa[j] + dk + (j ? a1_off1 : a1_off0);
      else if (h == 1) src = pb[j] + dk;
      else src = pb[j] + dk + (j ? b1_off1 : b1_off0);
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(img + (wave + 8 * j) * 1024), 16, 0,
                                       0);
    }
  };
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};
  issue(0, 0);
  issue(1, 0);
  issue(2, 0);
  issue(3, 0);
  if (nk > 1) {
    issue(0, 1);
    issue(1, 1);
    wait_vmcnt<8>();
  } else {
    wait_vmcnt<4>();
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier
  asm volatile("" ::: "memory");

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  const int q = lane >> 4;
  const int rA = wr * 64 + (lane & 15);
  const int rB = wc * 32 + (lane & 15);
  auto fq = [&](const char* img, int row, int st) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + 16 * ((4 * st + q) ^ swzq(row)));
  };
#define G7_MFMA(R0, BF, C0)                                                              \
  __builtin_amdgcn_sched_barrier(0);                                                     \
  __builtin_amdgcn_s_setprio(1);                                                         \
  _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                       \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                       \
  _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                       \
    acc[R0 + i_][C0 + j_] = mfma16(af[i_][s_], BF[j_][s_], acc[R0 + i_][C0 + j_]);       \
  __builtin_amdgcn_s_setprio(0);                                                         \
  __builtin_amdgcn_sched_barrier(0);
#define G7_BAR()                          \
  asm volatile("" ::: "memory");          \
  __builtin_amdgcn_s_barrier();           \
  asm volatile("" ::: "memory");
  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    const bool steady = t + 2 < nk;
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_) {
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][s_] = fq(buf, rA + 16 * i, s_);
#pragma unroll
      for (int j = 0; j < 2; ++j) b0[j][s_] = fq(buf + 2 * HALF, rB + 16 * j, s_);
    }
    if (t + 1 < nk) issue(2, t + 1);
    if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();
    G7_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G7_MFMA(0, b0, 0);
    G7_BAR();
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
      for (int j = 0; j < 2; ++j) b1[j][s_] = fq(buf + 3 * HALF, rB + 16 * j, s_);
    if (t + 1 < nk) issue(3, t + 1);
    if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();
    G7_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G7_MFMA(0, b1, 2);
    G7_BAR();
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][s_] = fq(buf + HALF, rA + 16 * i, s_);
    if (steady) issue(0, t + 2);
    G7_BAR();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G7_MFMA(4, b0, 0);
    G7_BAR();
    if (steady) {
      issue(1, t + 2);
      wait_vmcnt<8>();
    } else {
      wait_vmcnt<0>();
    }
    G7_BAR();
    G7_MFMA(4, b1, 2);
    G7_BAR();
  }
#undef G7_MFMA
#undef G7_BAR
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the staggered wave rows
  __syncthreads();
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// a contributor's partial tile -> its slot, row-major [256][256] f32: staged through LDS one
// wave-row group at a time exactly like the epilogue (so the accumulators die as they are
// staged), then sc1 (write-through) 16-byte buffer stores; every wave drains them, a
// barrier, one agent-scope flag store
template <class StageF>
__device__ __forceinline__ void g7_publish(const StageF& stage, char* smem, int wr, float* slot,
                                           unsigned long long* flag) {
  constexpr int RG = 128, CP = 256 + 4;
  float* ct = reinterpret_cast<float*>(smem);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(slot, 0, SK_SLOT * 4, 0x00020000);
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    if (wr == pass) stage(ct, CP);
    __syncthreads();
    for (int idx = threadIdx.x; idx < RG * 64; idx += NT) {
      const int row = idx >> 6, c4 = (idx & 63) * 4;
      const float4 v = *reinterpret_cast<const float4*>(ct + row * CP + c4);
#if MP_G7_SC1
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, ((pass * RG + row) * 256 + c4) * 4, 0,
                                             16 /* sc1 */);
#else
      *reinterpret_cast<float4*>(slot + (pass * RG + row) * 256 + c4) = v;   // into this XCD's L2
#endif
    }
    __syncthreads();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its stores
  __syncthreads();
  if (threadIdx.x == 0) {
#if !MP_G7_SC1
    // plain stores: one agent-scope release writes the XCD L2's dirty lines back (the
    // cdna guide's split-K recipe: fence, then an explicit wait, then the signal)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __hip_atomic_store(flag, SK_TAG, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the owner waits for its contributors' flags (thread 0, bounded poll), clears them for the
// next launch, and makes their partials visible to this CU: one agent-scope acquire (drops
// this CU's L1) before a barrier; the epilogue then reads them with plain loads
__device__ __forceinline__ void g7_await(unsigned long long* flags, int first, int step, int n, unsigned* err) {
  if (threadIdx.x == 0) {
    for (int p = 0; p < n; ++p) {
      unsigned long long* f = flags + first + p * step;
      unsigned spins = 0;
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != SK_TAG) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 24)) {     // ~0.5 s: a lost hand-off ends the kernel, flagged
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __hip_atomic_store(f, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <int EPI>
__global__ void __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm7_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, bf16_t* __restrict__ C,
             const bf16_t* __restrict__ bias, const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX,
             float* __restrict__ colsum, float* __restrict__ ws, int M, int N, int K, int64_t lda, int64_t ldb,
             int64_t ldc, int64_t ldr, int64_t ldx, float alpha, float p_drop, uint64_t seed, int S, int tile0) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  // the tail tiles [tile0, T) of the whole output in row-major tile order (full-matrix
  // indices: the fused dropout's mask index is the element of the whole output)
  const int gn = (N + 255) / 256, T = ((M + 255) / 256) * gn - tile0;
  const int kt = K / BK;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / 4, wn = (wave % 4) * 64;
  unsigned long long* flags = reinterpret_cast<unsigned long long*>(ws);
  float* part = ws + SK_FLAGS;
  // XCD group x owns tiles [t0, t1) (c of them); workgroup l of the group takes chunk
  // l / c of tile l % c, so one chunk index walks the same K range of neighbouring tiles
  const int x = b & 7, l = b >> 3;
  const int t0 = (int)((int64_t)x * T / 8), t1 = (int)((int64_t)(x + 1) * T / 8);
  const int c = t1 - t0;
  if (c <= 0 || l >= c * S) return;
  const int ti = l % c, j = l / c;
  const int k0 = (int)((int64_t)j * kt / S), k1 = (int)((int64_t)(j + 1) * kt / S);
  const int tile = tile0 + t0 + ti;
  const int m0 = (tile / gn) * 256, n0 = (tile % gn) * 256;
  f32x4 acc[8][4];
  g7_mainloop(A, B, M, N, lda, ldb, m0, n0, k0, k1 - k0, smem, acc);
  if (j < S - 1) {   // contributor: partial + flag
    g7_publish(Stage16<8, 4>{acc, wn, lane}, smem, wr, part + (int64_t)b * SK_SLOT, flags + b);
    return;
  }
  // owner (the last chunk): the lower chunks of this tile were dispatched before it
  g7_await(flags, x + 8 * ti, 8 * c, S - 1, reinterpret_cast<unsigned*>(ws) + SK_ERR);
  epilogue<256, 256, 2, 4, EPI, false, NT, true>(Stage16<8, 4>{acc, wn, lane}, smem, m0, n0, wr, C, bias, R, AUX,
                                       colsum, M, N, ldc, ldr, ldx, alpha, 1, p_drop, seed,
                                       part + (int64_t)(x + 8 * ti) * SK_SLOT,
                                       (int64_t)8 * c * SK_SLOT, S - 1);
}

// plan of the split-tail engine: 0 if it should not be used for this grid, else 1 with the
// tiles of the leading data-parallel rounds (dp, row-major, run by gemm3), the tail tiles and
// the chunks per tail tile (S)
struct Plan7 {
  int dp, tail, S;
};
static int plan7(int M, int N, int K, Plan7* out) {
  const int G = SK_MAX_G, q = G / 8;
  const int T = ((M + 255) / 256) * ((N + 255) / 256);
  const int kt = K / BK;
  if (T < 64 || T % G == 0 || kt < 4) return 0;
  const int dp = (T / G) * G, tail = T - dp;
  const int cmax = (tail + 7) / 8;                  // tail tiles of the fullest XCD group
  // modelled k-iteration units: a tile costs kt + 3 (prologue fill, C write); a chunked
  // tail tile ceil(kt / S) + 3, plus 2 per partial its owner reads (256 KiB at the
  // cross-XCD rate) and 1 for the contributors' publish; + 2 for a second launch
  const float plain = (float)((T + G - 1) / G) * (kt + 3);
  const float lead = (float)(dp / G) * (kt + 3) + (dp > 0 ? 2.f : 0.f);
  float best = 3.0e38f;
  int bestS = 0;
  for (int S = 2; S * cmax <= q && S <= 8; ++S) {
    const float t = lead + (float)((kt + S - 1) / S) + 3.f + 2.f * (S - 1) + 1.f;
    if (t < best) {
      best = t;
      bestS = S;
    }
  }
  static const int forceS = [] { const char* e = getenv("MIPIPE_GEMM7_S"); return e ? atoi(e) : 0; }();
  if (forceS >= 1 && forceS * cmax <= q) bestS = forceS, best = 0.f;   // A/B probes
  if (bestS == 0 || best > 0.95f * plain) return 0;
  out->dp = dp;
  out->tail = tail;
  out->S = bestS;
  return 1;
}

template <int EPI>
static int launch7(const void* A, const void* B, void* C, const void* bias, const void* R, void* X, float* colsum,
                   float* ws, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx,
                   float alpha, float p_drop, uint64_t seed, hipStream_t st) {
  Plan7 pl{};
  if (!plan7(M, N, K, &pl) || ws == nullptr) return -1;
  constexpr int LDS_MAIN = 2 * 4 * 128 * 128;
  constexpr int EPI_BYTES = 128 * (256 + 4) * 4;
  constexpr int LDS = LDS_MAIN > EPI_BYTES ? LDS_MAIN : EPI_BYTES;
  if (pl.dp > 0) {   // the whole rounds: the ping-pong engine on the first dp tiles (row-major)
    const int rc = launch3<EPI, false, true>(A, B, C, bias, R, X, colsum, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, 1,
                                             p_drop, seed, st, pl.dp);
    if (rc != 0) return rc;
  }
  auto kern = gemm7_kernel<EPI>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  // the tail tiles [dp, T)
  const int cmax = (pl.tail + 7) / 8;
  kern<<<dim3(8 * cmax * pl.S), NT, LDS, st>>>((const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, (const bf16_t*)bias,
                                               (const bf16_t*)R, (bf16_t*)X, colsum, ws, M, N, K, lda, ldb, ldc, ldr,
                                               ldx, alpha, p_drop, seed, pl.S, pl.dp);
  return (int)hipGetLastError();
}

// gemm4 / gemm5: probe engines with recorded null results (profiles/r2_probes.md), built only
// into the A/B variant (tools/build_ext.py --variant probes -D MP_PROBE_ENGINES), not _C.so.
#ifdef MP_PROBE_ENGINES
// ---------------------------------------------------------------------------------------
// gemm4: persistent 256x256 NT GEMM (gemm3's 16x16x32 phase schedule) whose C write is
// deferred into the NEXT tile's main loop.
//
// At K = 768 about a third of a gemm3 launch is the C write of each tile wave: all 256
// CUs store their 128 KiB at the same moment while the matrix cores idle
// (profiles/r2_probes.md "fixed vs per-K-tile cost"; hipBLASLt pays the same).  Here one
// workgroup per CU walks tiles vb = blockIdx.x + k * gridDim.x (same XCD for every k); a
// finished tile is packed to bf16 in registers (64 VGPRs, epilogue applied) and its 32
// 8-byte stores per lane go out one per phase during the first 8 K-tiles of the next
// tile, so HBM drains C while the MFMAs run.  The last tile is written after the loop.
//
// Operand roles are swapped by the host: the kernel computes D = A B^T with A = the
// weight [N][K] and B = the activations [M][K], and writes D transposed into the
// row-major C[M][N].  A lane's 16x16x32 accumulator holds 4 consecutive D rows = 4
// consecutive C columns: one 8-byte store, one 8-byte bias load.
//
// vmcnt: stores retire through the same in-order counter as the half-tile DMA, so every
// counted wait of gemm3 grows by the stores issued after its target half-tile (derivation
// at the waits; the drain phases keep vmcnt(0)).
// ---------------------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {   // wave-uniform n: scalar branch to the immediate form
    case 8: wait_vmcnt<8>(); break;
    case 9: wait_vmcnt<9>(); break;
    case 10: wait_vmcnt<10>(); break;
    case 11: wait_vmcnt<11>(); break;
    case 12: wait_vmcnt<12>(); break;
    default: wait_vmcnt<0>(); break;
  }
}

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

template <int EPI>
__global__ void __launch_bounds__(NT, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm4_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, bf16_t* __restrict__ C,
             const bf16_t* __restrict__ bias, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
             float alpha) {
  static_assert(EPI == EPI_NONE || EPI == EPI_BIAS, "gemm4 epilogues: none, bias");
  constexpr int BM = 256, BN = 256, WN = 4;
  constexpr int HALF = 128 * 128;
  constexpr int BUF = 4 * HALF;
  constexpr int SK = MP_G4_SR;   // K-tiles that carry the previous tile's deferred rows (one store per phase)
  constexpr int SR = MP_G4_SR;   // accumulator row blocks deferred (the other 8 - SR are stored at the tile end)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  const int nwg = gm * gn;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ swzq(8 * (wave & 1) + lr);
  const int q = lane >> 4;
  const int nk = K / BK;
  const int rA = wr * 64 + (lane & 15);
  const int rB = wc * 32 + (lane & 15);

  // previous tile: stash[i][j] = D rows pm0 + 128 wr + 16 (i + shifts) + 4 q .. +3 at
  // column pn0 + 64 wc + 16 j + (lane & 15); rows leave through stash[0] (shift())
  u32x2 stash[SR][4];
  int pm0 = 0, pn0 = 0;
  bool has_prev = false;
  auto put = [&](int j, int srow) {
    const int r = pm0 + wr * 128 + 16 * srow + 4 * q;
    const int c = pn0 + 64 * wc + 16 * j + (lane & 15);
    if (r < M && c < N) __builtin_nontemporal_store(stash[0][j], reinterpret_cast<u32x2*>(C + (int64_t)c * ldc + r));
  };
  auto shift = [&]() {
#pragma unroll
    for (int i = 0; i < SR - 1; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) stash[i][j] = stash[i + 1][j];
  };

#define G4_MFMA(R0, BF, C0)                                                              \
  __builtin_amdgcn_sched_barrier(0);                                                     \
  __builtin_amdgcn_s_setprio(1);                                                         \
  _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                       \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                       \
  _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                       \
    acc[R0 + i_][C0 + j_] = mfma16(af[i_][s_], BF[j_][s_], acc[R0 + i_][C0 + j_]);       \
  __builtin_amdgcn_s_setprio(0);                                                         \
  __builtin_amdgcn_sched_barrier(0);
#define G4_BAR()                          \
  asm volatile("" ::: "memory");          \
  __builtin_amdgcn_s_barrier();           \
  asm volatile("" ::: "memory");

#pragma unroll 1
  for (int vb = blockIdx.x; vb < nwg; vb += gridDim.x) {
    const int wg = xcd_remap(vb, nwg);
    constexpr int GROUP = MP_G3_GROUP;
    const int group = wg / (GROUP * gn);
    const int first_m = group * GROUP;
    const int gsz = min(gm - first_m, GROUP);
    const int tm = first_m + (wg % (GROUP * gn)) % gsz;
    const int tn = (wg % (GROUP * gn)) / gsz;
    const int m0 = tm * BM, n0 = tn * BN;

    const bf16_t* pa[2];
    const bf16_t* pb[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int ra = m0 + 128 * j + 8 * wave + lr;
      ra = ra < M ? ra : M - 1;
      int rb = n0 + 64 * ((wave >> 2) + 2 * j) + 8 * (wave & 3) + lr;
      rb = rb < N ? rb : N - 1;
      pa[j] = A + (int64_t)ra * lda + lc * 8;
      pb[j] = B + (int64_t)rb * ldb + lc * 8;
    }
    const bool a1_ok0 = m0 + 64 + 8 * wave + lr < M, a1_ok1 = m0 + 192 + 8 * wave + lr < M;
    const bool b1_ok0 = n0 + 64 * (wave >> 2) + 32 + 8 * (wave & 3) + lr < N;
    const bool b1_ok1 = n0 + 64 * ((wave >> 2) + 2) + 32 + 8 * (wave & 3) + lr < N;
    const int64_t a1_off0 = a1_ok0 ? 64 * lda : 0, a1_off1 = a1_ok1 ? 64 * lda : 0;
    const int64_t b1_off0 = b1_ok0 ? 32 * ldb : 0, b1_off1 = b1_ok1 ? 32 * ldb : 0;

    auto issue = [&](int h, int kt) {
      char* img = smem + (kt & 1) * BUF + (h == 0 ? 0 : h == 3 ? HALF : h == 1 ? 2 * HALF : 3 * HALF);
      const int64_t dk = (int64_t)kt * BK;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16_t* src;
        if (h == 0) src = pa[j] + dk;
        else if (h == 3) src = pa[j] + dk + (j ? a1_off1 : a1_off0);
        else if (h == 1) src = pb[j] + dk;
        else src = pb[j] + dk + (j ? b1_off1 : b1_off0);
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(img + (wave + 8 * j) * 1024), 16,
                                         0, 0);
      }
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

    issue(0, 0);
    issue(1, 0);
    issue(2, 0);
    issue(3, 0);
    if (nk > 1) {
      issue(0, 1);
      issue(1, 1);
      wait_vmcnt<8>();
    } else {
      wait_vmcnt<4>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier
    asm volatile("" ::: "memory");

    bf16x8 af[4][2], b0[2][2], b1[2][2];
    auto fq = [&](const char* img, int row, int st) -> bf16x8 {
      return *reinterpret_cast<const bf16x8*>(img + row * 128 + 16 * ((4 * st + q) ^ swzq(row)));
    };

#pragma unroll 1
    for (int t = 0; t < nk; ++t) {
      const char* buf = smem + (t & 1) * BUF;
      const bool steady = t + 2 < nk;
      // sc: this K-tile's four phases each store one stash entry right after their wait;
      // sp: the previous K-tile's did
      const int sc = (has_prev && t < SK) ? 1 : 0;
      const int sp = (has_prev && t >= 1 && t - 1 < SK) ? 1 : 0;
      // ---- phase 1: A0 x B0.  Target B1(t), issued in phase 1 of t-1 (t = 0: prologue);
      // younger: 4 half-tiles (8 ops) + the 4 stores of K-tile t-1
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) {
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i][s_] = fq(buf, rA + 16 * i, s_);
#pragma unroll
        for (int j = 0; j < 2; ++j) b0[j][s_] = fq(buf + 2 * HALF, rB + 16 * j, s_);
      }
      if (t + 1 < nk) issue(2, t + 1);
      wait_vm_rt(steady ? 8 + 4 * sp : 0);
      G4_BAR();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (sc) put(0, t);
      G4_MFMA(0, b0, 0);
      G4_BAR();
      // ---- phase 2: A0 x B1.  Target A1(t) (phase 2 of t-1); younger: 8 DMA ops, the
      // stores of phases 2-4 of t-1 and of phase 1 of t
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
        for (int j = 0; j < 2; ++j) b1[j][s_] = fq(buf + 3 * HALF, rB + 16 * j, s_);
      if (t + 1 < nk) issue(3, t + 1);
      wait_vm_rt(steady ? 8 + 3 * sp + sc : 0);
      G4_BAR();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (sc) put(1, t);
      G4_MFMA(0, b1, 2);
      G4_BAR();
      // ---- phase 3: A1 x B0; refill A0 of this buffer for K-tile t+2
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i][s_] = fq(buf + HALF, rA + 16 * i, s_);
      if (steady) issue(0, t + 2);
      G4_BAR();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (sc) put(2, t);
      G4_MFMA(4, b0, 0);
      G4_BAR();
      // ---- phase 4: A1 x B1; refill B0.  Target B0(t+1) (phase 4 of t-1; t = 0: the last
      // prologue issue); younger: 8 DMA ops, the store of phase 4 of t-1, phases 1-3 of t
      if (steady) {
        issue(1, t + 2);
        wait_vm_rt(8 + sp + 3 * sc);
      } else {
        wait_vmcnt<0>();
      }
      G4_BAR();
      if (sc) put(3, t);
      G4_MFMA(4, b1, 2);
      G4_BAR();
      if (sc) shift();
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the staggered wave rows
    __syncthreads();
    // short K (< SK K-tiles): the rest of the previous tile
    if (has_prev) {
#pragma unroll 1
      for (int s = nk; s < SK; ++s) {
        put(0, s);
        put(1, s);
        put(2, s);
        put(3, s);
        shift();
      }
    }
    // this tile: alpha (+ bias) -> bf16; row blocks SR.. stored now, 0..SR-1 deferred
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = m0 + wr * 128 + 16 * i + 4 * q;
      u32x2 bz = {0u, 0u};
      if constexpr (EPI == EPI_BIAS) bz = *reinterpret_cast<const u32x2*>(bias + (r < M ? r : 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * alpha;
        if constexpr (EPI == EPI_BIAS) {
          v[0] += __uint_as_float(bz[0] << 16);
          v[1] += __uint_as_float(bz[0] & 0xffff0000u);
          v[2] += __uint_as_float(bz[1] << 16);
          v[3] += __uint_as_float(bz[1] & 0xffff0000u);
        }
        const u32x2 o = u32x2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
        if (i < SR) {
          stash[i < SR ? i : 0][j] = o;
        } else {
          const int c = n0 + 64 * wc + 16 * j + (lane & 15);
          if (r < M && c < N) __builtin_nontemporal_store(o, reinterpret_cast<u32x2*>(C + (int64_t)c * ldc + r));
        }
      }
    }
    pm0 = m0;
    pn0 = n0;
    has_prev = true;
  }
#undef G4_MFMA
#undef G4_BAR
  if (has_prev) {
#pragma unroll 1
    for (int s = 0; s < SK; ++s) {
      put(0, s);
      put(1, s);
      put(2, s);
      put(3, s);
      shift();
    }
  }
}

// C[M][N] (bf16, row stride ldc) = alpha * X[M][K] W[N][K]^T (+ bias[N]) on gemm4
// (kernel space: D = W X^T, Mk = N, Nk = M); one workgroup per CU once the tiles
// outnumber the CUs
template <int EPI>
static int launch4(const void* X, const void* W, void* C, const void* bias, int M, int N, int K, int64_t ldx,
                   int64_t ldw, int64_t ldc, float alpha, int grid_override, hipStream_t st) {
  constexpr int LDS = 2 * 4 * 128 * 128;
  auto kern = gemm4_kernel<EPI>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int nwg = ((N + 255) / 256) * ((M + 255) / 256);
  int grid = nwg < 256 ? nwg : 256;
  if (grid_override > 0) grid = grid_override < nwg ? grid_override : nwg;   // tests: several tiles per workgroup
  kern<<<grid, NT, LDS, st>>>((const bf16_t*)W, (const bf16_t*)X, (bf16_t*)C, (const bf16_t*)bias, N, M, K, ldw,
                              ldx, ldc, alpha);
  return (int)hipGetLastError();
}


// ---------------------------------------------------------------------------------------
// gemm5 (probe, opt-in: 0.7-0.8x gemm3, profiles/r2_probes.md): 256x256 NT with 4 waves, ONE wave per SIMD (512 registers: a 128x128
// accumulator per wave in 256 AGPRs), instead of gemm3's 8 waves in ping-pong pairs.
// Per K-tile (BK = 64) a wave reads 32 KiB of fragments (gemm3: 24 KiB x 8 waves) and
// issues 128 MFMAs; fragments are register double-buffered by 32-deep k-step, so the
// ds_reads of the next k-step (and the next K-tile's DMA) interleave with the current
// k-step's MFMAs (sched_group_barrier).  2 LDS buffers, one barrier per K-tile.
// ---------------------------------------------------------------------------------------
template <int EPI>
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm5_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, void* __restrict__ Cv,
             const bf16_t* __restrict__ bias, const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX,
             float* __restrict__ WS, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr,
             int64_t ldx, float alpha, float p_drop, uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  constexpr int BM = 256, BN = 256, NTH5 = 256;
  constexpr int IMG = 256 * 128;          // one operand image: 256 rows x 64 k (128 B rows)
  constexpr int BUF = 2 * IMG;            // A | B
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  const int nwg = gm * gn;
  const int wg = xcd_remap((int)blockIdx.x, nwg);
  constexpr int GROUP = MP_G3_GROUP;
  const int group = wg / (GROUP * gn);
  const int first_m = group * GROUP;
  const int gsz = min(gm - first_m, GROUP);
  const int tm = first_m + (wg % (GROUP * gn)) % gsz;
  const int tn = (wg % (GROUP * gn)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63, q = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = K / BK;

  // DMA: 64 pieces of 1 KiB per K-tile (A rows 0..255 = pieces 0..31, B = 32..63); wave w
  // issues pieces w, w + 4, ..., each lane 16 bytes: image row 8 p' + (lane >> 3), physical
  // chunk lane & 7 <- logical chunk (lane & 7) ^ swzq(row)
  const int lr = lane >> 3;
  const bf16_t* src[16];
  int dst[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int piece = wave + 4 * u;                  // 0..63
    const bool isb = piece >= 32;
    const int prow = (piece & 31) * 8 + lr;          // image row
    const int lc = (lane & 7) ^ swzq(prow);
    int gr = (isb ? n0 : m0) + prow;
    const int lim = isb ? N : M;
    gr = gr < lim ? gr : lim - 1;
    src[u] = (isb ? B : A) + (int64_t)gr * (isb ? ldb : lda) + lc * 8;
    dst[u] = (isb ? IMG : 0) + (piece & 31) * 1024;
  }
  auto issue = [&](int kt) {
    char* base = smem + (kt & 1) * BUF;
#pragma unroll
    for (int u = 0; u < 16; ++u)
      __builtin_amdgcn_global_load_lds((const void*)(src[u] + (int64_t)kt * BK),
                                       (__attribute__((address_space(3))) void*)(base + dst[u]), 16, 0, 0);
  };
  auto fq = [&](const char* img, int row, int st) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + 16 * ((4 * st + q) ^ swzq(row)));
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};

  const int rA = wr * 128 + (lane & 15), rB = wc * 128 + (lane & 15);
  bf16x8 a0[8], b0[8], a1[8], b1[8];

  issue(0);
  if (nk > 1) issue(1);
  if (nk > 1) wait_vmcnt<16>(); else wait_vmcnt<0>();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a0[i] = fq(smem, rA + 16 * i, 0);
    b0[i] = fq(smem + IMG, rB + 16 * i, 0);
  }

#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    // (A) k-step 0 MFMAs; the k-step 1 fragments of this K-tile load meanwhile
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a1[i] = fq(buf, rA + 16 * i, 1);
      b1[i] = fq(buf + IMG, rB + 16 * i, 1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(a0[i], b0[j], acc[i][j]);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
    }
    // (B) every wave done reading this buffer, the next K-tile landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_vmcnt<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // (C, D) DMA of K-tile t+2 into this buffer; k-step 1 MFMAs while the next K-tile's
    // k-step 0 fragments load
    if (t + 2 < nk) issue(t + 2);
    const char* nbuf = smem + ((t + 1) & 1) * BUF;
    if (t + 1 < nk) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        a0[i] = fq(nbuf, rA + 16 * i, 0);
        b0[i] = fq(nbuf + IMG, rB + 16 * i, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  epilogue<BM, BN, 2, 2, EPI, false, NTH5>(Stage16<8, 8>{acc, wc * 128, lane}, smem, m0, n0, wr, Cv, bias, R, AUX,
                                           WS, M, N, ldc, ldr, ldx, alpha, 1, p_drop, seed);
}

template <int EPI>
static int launch5(const void* A, const void* B, void* C, const void* bias, const void* R, void* X, float* ws, int M,
                   int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha,
                   float p_drop, uint64_t seed, hipStream_t st) {
  constexpr int LDS_MAIN = 2 * 2 * 256 * 128;
  constexpr int EPI_BYTES = 128 * (256 + 4) * 4;
  constexpr int LDS = LDS_MAIN > EPI_BYTES ? LDS_MAIN : EPI_BYTES;
  auto kern = gemm5_kernel<EPI>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int nwg = ((M + 255) / 256) * ((N + 255) / 256);
  kern<<<nwg, 256, LDS, st>>>((const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias, (const bf16_t*)R,
                              (bf16_t*)X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed);
  return (int)hipGetLastError();
}


#endif  // MP_PROBE_ENGINES
// ---------------------------------------------------------------------------------------
// gemms: small-tile NT engine for short-token problems (the reference model's 1024-token
// microbatches: M = 1024, N = 768..2304).  A 256x256 grid there has 12-36 tiles for 256
// CUs, and split-K to fill the chip costs an f32 slab round trip plus a reduce/epilogue
// kernel per GEMM (~40 % of those GEMMs' time, profiles/r2_ref_L8H8_kernel_stats.csv).
// Here: 256-thread workgroups (2x2 waves), BM x BN in {64x64, 64x32, 32x32}, 16x16x32
// MFMAs, the same 2-stage global_load_lds pipeline / swizzled K-contiguous images as
// gemm2, several workgroups per CU (32 KiB LDS at 64x64), and the fused epilogue applied
// directly -- one launch per GEMM, no split-K.
// ---------------------------------------------------------------------------------------
// one BM x BN output tile (workgroup-linear index wg of the problem's tile grid, split
// ``split`` of ``nsplit``) of the small engine; shared by gemms_kernel and the grouped
// weight-gradient kernel below
template <int BM, int BN, int EPI, bool ACC, bool TA, bool TB>
__device__ __forceinline__ void gemms_tile(char* smem, const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                           void* __restrict__ Cv, const bf16_t* __restrict__ bias,
                                           const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX,
                                           float* __restrict__ WS, int M, int N, int K, int64_t lda, int64_t ldb,
                                           int64_t ldc, int64_t ldr, int64_t ldx, float alpha, float p_drop,
                                           uint64_t seed, int wg, int nsplit, int split) {
  constexpr int NTH = 256, WM = 2, WN = 2;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(TM >= 1 && TN >= 1 && TM * 16 * WM == BM && TN * 16 * WN == BN, "tile/wave mismatch");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PIECES = STAGE / 1024, PW = PIECES / 4;
  static_assert(PW * 4 == PIECES, "pieces must split over 4 waves");

  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  constexpr int GROUP = 8;
  const int group = wg / (GROUP * gn);
  const int first_m = group * GROUP;
  const int gsz = min(gm - first_m, GROUP);
  const int tm = first_m + (wg % (GROUP * gn)) % gsz;
  const int tn = (wg % (GROUP * gn)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int wm = wr * (BM / WM), wn = wc * (BN / WN);

  const int ktiles = K / BK;
  const int kt0 = split * ktiles / nsplit;
  const int nk = (split + 1) * ktiles / nsplit - kt0;
  const int kbase = kt0 * BK;

  const bf16_t* psrc[PW];
  bool pisA[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int p = wave + 4 * i;
    const int pos = p * 1024 + lane * 16;
    pisA[i] = p * 1024 < A_BYTES;
    if (pisA[i]) psrc[i] = src_of<TA, BM, true>(A, lda, pos, m0, M, kbase);
    else psrc[i] = src_of<TB, BN, true>(B, ldb, pos - A_BYTES, n0, N, kbase);
  }
  auto issue = [&](int stage, int kt) {
    char* sb = smem + stage * STAGE;
    const int64_t dA = TA ? (int64_t)kt * BK * lda : (int64_t)kt * BK;
    const int64_t dB = TB ? (int64_t)kt * BK * ldb : (int64_t)kt * BK;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int p = wave + 4 * i;
      __builtin_amdgcn_global_load_lds((const void*)(psrc[i] + (pisA[i] ? dA : dB)),
                                       (__attribute__((address_space(3))) void*)(sb + p * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{};

  if (nk > 0) {
    issue(0, 0);
    if (nk > 1) {
      issue(1, 1);
      wait_vmcnt<PW>();
    } else {
      wait_vmcnt<0>();
    }
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int t = 0; t < nk; ++t) {
    const char* sa = smem + (t & 1) * STAGE;
    const char* sbB = sa + A_BYTES;
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_) {
#pragma unroll
      for (int i = 0; i < TM; ++i) af[s_][i] = frag16<TA, BM>(sa, wm + 16 * i, s_);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[s_][j] = frag16<TB, BN>(sbB, wn + 16 * j, s_);
    }
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[s_][i], bfr[s_][j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nk) {
      issue(t & 1, t + 2);
      wait_vmcnt<PW>();
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  epilogue<BM, BN, WM, WN, EPI, ACC, NTH>(Stage16<TM, TN>{acc, wn, lane}, smem, m0, n0, wr, Cv, bias, R, AUX, WS, M,
                                          N, ldc, ldr, ldx, alpha, nsplit, p_drop, seed);
}

template <int BM, int BN, int EPI, bool ACC, bool TA = false, bool TB = false>
__global__ void __launch_bounds__(256) gemms_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                    void* __restrict__ Cv, const bf16_t* __restrict__ bias,
                                                    const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX,
                                                    float* __restrict__ WS, int M, int N, int K, int64_t lda,
                                                    int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha, float p_drop, uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  gemms_tile<BM, BN, EPI, ACC, TA, TB>(smem, A, B, Cv, bias, R, AUX, WS, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop,
                                       seed, xcd_remap((int)blockIdx.x, nwg), (int)gridDim.y, (int)blockIdx.y);
}

// ---------------------------------------------------------------------------------------
// Grouped weight-gradient GEMMs: up to MP_GROUP_MAX independent TT problems
// C_g[M_g, N_g] += alpha * A_g^T B_g (A_g [K_g][M_g], B_g [K_g][N_g] k-major, f32 C) in ONE
// launch of 64x64 tiles.  A layer's dW GEMMs at 1024-token microbatches are 144-432 tiles
// each: one launch per GEMM leaves most of the 256 CUs idle and pays the short k-loop's
// latency per GEMM (97-230 TF, tools/wbatch_probe.py); grouped, ~1900 tiles of a layer
// share the chip, several workgroups per CU hide each other's load latency.  Workgroup
// b -> problem g with tile_start[g] <= b' < tile_start[g + 1] (b' = XCD-remapped b;
// wave-uniform scan of <= 8 entries), then the problem-local tile of gemms_tile.
// ---------------------------------------------------------------------------------------
struct GroupTT {
  const bf16_t* A[MP_GROUP_MAX];
  const bf16_t* B[MP_GROUP_MAX];
  float* C[MP_GROUP_MAX];
  int64_t lda[MP_GROUP_MAX], ldb[MP_GROUP_MAX], ldc[MP_GROUP_MAX];
  int M[MP_GROUP_MAX], N[MP_GROUP_MAX], K[MP_GROUP_MAX];
  int tile_start[MP_GROUP_MAX + 1];
  int n;
  float alpha;
};

__global__ void __launch_bounds__(256) gemms_tt_grouped_kernel(const GroupTT g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int total = g.tile_start[g.n];
  const int b = xcd_remap((int)blockIdx.x, total);
  int p = 0;
#pragma unroll
  for (int i = 1; i < MP_GROUP_MAX; ++i)
    if (i < g.n && b >= g.tile_start[i]) p = i;
  gemms_tile<64, 64, EPI_NONE, true, true, true>(smem, g.A[p], g.B[p], g.C[p], nullptr, nullptr, nullptr, nullptr,
                                                 g.M[p], g.N[p], g.K[p], g.lda[p], g.ldb[p], g.ldc[p], 0, 0, g.alpha,
                                                 0.f, 0, b - g.tile_start[p], 1, 0);
}

template <int BM, int BN, int EPI, bool ACC, bool TA = false, bool TB = false>
static int launchs(const void* A, const void* B, void* C, const void* bias, const void* R, void* X, float* ws, int M,
                   int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha, int split,
                   float p_drop, uint64_t seed, hipStream_t st) {
  constexpr int STAGE = (BM + BN) * BK * 2;
  constexpr int EPI_BYTES = (BM / 2) * (BN + 4) * 4;
  constexpr int RED_BYTES = 256 * 8 * 4;   // the column-sum reduction reuses the staging area
  constexpr int LDS0 = 2 * STAGE > EPI_BYTES ? 2 * STAGE : EPI_BYTES;
  constexpr int LDS = LDS0 > RED_BYTES ? LDS0 : RED_BYTES;
  auto kern = gemms_kernel<BM, BN, EPI, ACC, TA, TB>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  kern<<<dim3(nwg, split), 256, LDS, st>>>((const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias,
                                           (const bf16_t*)R, (bf16_t*)X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB, int EPI, bool ACC>
static int launch(const void* A, const void* B, void* C, const void* bias, const void* R, void* X, float* ws, int M,
                  int N, int K,
                  int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha, int split,
                  float p_drop, uint64_t seed, hipStream_t st) {
  constexpr int STAGE = (BM + BN) * BK * 2;
  constexpr int EPI_BYTES = (BM / WM) * (BN + 4) * 4;
  constexpr int LDS = 2 * STAGE > EPI_BYTES ? 2 * STAGE : EPI_BYTES;
  static const bool m16 = [] { const char* e = getenv("MIPIPE_GEMM_M16"); return !(e && e[0] == '0'); }();
  // 16x16x32 only for K-contiguous operands: with the transposed (tr-read) images of the
  // TT dW GEMMs it measured 1.8x slower (dw_qkv 374 vs 688 TF), so those keep 32x32x16
  static const bool m16t = [] { const char* e = getenv("MIPIPE_GEMM_M16T"); return e && e[0] == '1'; }();
  auto kern = (m16 && (m16t || (!TA && !TB))) ? gemm2_kernel<BM, BN, WM, WN, TA, TB, EPI, ACC, true>
                                  : gemm2_kernel<BM, BN, WM, WN, TA, TB, EPI, ACC, false>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  kern<<<dim3(nwg, split), NT, LDS, st>>>((const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias,
                                          (const bf16_t*)R, (bf16_t*)X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed);
  return (int)hipGetLastError();
}

// tile configurations: 0: 256x256 (2x4 waves), 1: 256x192 (4x2), 2: 256x128 (4x2), 3: 128x128 (2x4)
struct Cfg {
  int bm, bn;
  float eff;  // relative efficiency of the tile shape (bigger tiles reuse more)
};
static const Cfg CFGS[4] = {{256, 256, 1.00f}, {256, 192, 0.96f}, {256, 128, 0.90f}, {128, 128, 0.72f}};

static int choose(int M, int N, int K, bool acc, bool outer, int* split_out) {
  // minimise modelled time = (#rounds of CU slots) x (per-item k-loop + epilogue) / tile efficiency;
  // padded tiles are charged like real ones, so quantisation and padding waste both count
  int best = 3, best_split = 1;
  float best_t = 3.0e38f;
  const int kt = K / BK;
  for (int c = 0; c < 4; ++c) {
    const int cus = 256;
    const int slots = c == 3 ? 2 * cus : cus;  // 128x128 tiles fit two workgroups per CU
    if (outer && CFGS[c].bn == 192) continue;  // outer-contig images need power-of-two widths
    const int tiles = ((M + CFGS[c].bm - 1) / CFGS[c].bm) * ((N + CFGS[c].bn - 1) / CFGS[c].bn);
    const float area = (float)(CFGS[c].bm * CFGS[c].bn) / (256.f * 256.f) * (c == 3 ? 2.f : 1.f);
    // bf16 outputs split too (f32 slabs + one reduce pass that applies the epilogue):
    // small-M problems (1024-token microbatches) otherwise fill 24-48 of 256 CUs
    // MIPIPE_DW_MAXSPLIT: cap on the f32-accumulate split-K factor (default 32)
    static const int acc_cap = [] {
      const char* e = getenv("MIPIPE_DW_MAXSPLIT");
      const int v = e ? atoi(e) : 32;
      return v > 0 ? v : 32;
    }();
    const int acc_max = kt / 4 < acc_cap ? kt / 4 : acc_cap;
    const int max_split = acc ? acc_max : (kt / 3 < 8 ? kt / 3 : 8);
    for (int s = 1; s <= (max_split > 1 ? max_split : 1); ++s) {
      const int work = tiles * s;
      const int rounds = (work + slots - 1) / slots;
      const int kper = (kt + s - 1) / s;
      // f32 slab store (+ the reduce pass for bf16 outputs) vs a direct store, in k-tile units
      const float epi = s > 1 ? (acc ? 6.f : 8.f) : 2.f;
      const float t = rounds * (kper + epi + 2.f) * area / CFGS[c].eff;  // +2: prologue fill
      if (t < best_t * 0.999f) {
        best_t = t;
        best = c;
        best_split = s;
      }
    }
  }
  *split_out = best_split;
  return best;
}

}  // namespace g2

using namespace g2;

template <bool TA, bool TB, int EPI, bool ACC>
static int dispatch(int cfg, const void* A, const void* B, void* C, const void* bias, const void* R, void* X, float* ws,
                    int M,
                    int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha,
                    int split, float p_drop, uint64_t seed, hipStream_t st) {
  if constexpr (TA && TB && ACC && EPI == EPI_NONE) {
    if (cfg == 13) return launchs<64, 64, EPI, ACC, true, true>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    if (cfg == 6) return launch3<EPI, ACC, true, true>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
  }
  if constexpr (!TA && !TB) {
    if (cfg == 10) return launchs<64, 64, EPI, ACC>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    if (cfg == 11) return launchs<64, 32, EPI, ACC>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    if (cfg == 12) return launchs<32, 32, EPI, ACC>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    if (cfg == 4) return launch3<EPI, ACC, false>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    if (cfg == 5) return launch3<EPI, ACC, true>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    if (cfg == 9) return launch6<EPI, ACC>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed, st);
    if (cfg == 15) return launch8<EPI, ACC, 2>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed, st);
    if (cfg == 16) return launch8<EPI, ACC, 3>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed, st);
#ifdef MP_PROBE_ENGINES
    if constexpr (!ACC) {
      if (cfg == 8) return launch5<EPI>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, p_drop, seed, st);
    }
#endif
  }
  switch (cfg) {
    case 0: return launch<256, 256, 2, 4, TA, TB, EPI, ACC>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    case 1: return launch<256, 192, 4, 2, TA, TB, EPI, ACC>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    case 2: return launch<256, 128, 4, 2, TA, TB, EPI, ACC>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
    default: return launch<128, 128, 2, 4, TA, TB, EPI, ACC>(A, B, C, bias, R, X, ws, M, N, K, lda, ldb, ldc, ldr, ldx, alpha, split, p_drop, seed, st);
  }
}

// C[M,N] (f32, row stride ldc) += sum over the split-K slabs ws[s][M][N]
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ C, int M,
                                                            int N, int64_t ldc, int split) {
  const int64_t n4 = (int64_t)M * N / 4;
  const int64_t slab = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 4;
    const int m = (int)(e / N), n = (int)(e % N);
    float4 acc = *reinterpret_cast<const float4*>(ws + e);
    for (int s = 1; s < split; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(ws + s * slab + e);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    float4* cp = reinterpret_cast<float4*>(C + (int64_t)m * ldc + n);
    float4 c = *cp;
    c.x += acc.x; c.y += acc.y; c.z += acc.z; c.w += acc.w;
    *cp = c;
  }
}

// bf16 C[M,N] = epilogue(alpha-scaled sum of the split-K slabs ws[s][M][N])
template <int EPI>
__global__ void __launch_bounds__(256) splitk_epi_kernel(const float* __restrict__ ws, bf16_t* __restrict__ C, int M,
                                                         int N, int64_t ldc, int split, const bf16_t* __restrict__ bias,
                                                         const bf16_t* __restrict__ R, int64_t ldr,
                                                         bf16_t* __restrict__ AUX, int64_t ldx, float p_drop,
                                                         uint64_t seed) {
  if (p_drop > 0.f) seed = step_seed(seed);
  const int64_t n8 = (int64_t)M * N / 8;
  const int64_t slab = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 8;
    const int m = (int)(e / N), n = (int)(e % N);
    float4 a = *reinterpret_cast<const float4*>(ws + e), b = *reinterpret_cast<const float4*>(ws + e + 4);
    for (int s = 1; s < split; ++s) {
      const float4 c = *reinterpret_cast<const float4*>(ws + s * slab + e);
      const float4 d = *reinterpret_cast<const float4*>(ws + s * slab + e + 4);
      a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
      b.x += d.x; b.y += d.y; b.z += d.z; b.w += d.w;
    }
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    epi_store8<EPI>(v, m, n, C, ldc, bias, R, ldr, AUX, ldx, p_drop, seed);
  }
}

template <int EPI>
static int launch_splitk_epi(const float* ws, void* C, int M, int N, int64_t ldc, int split, const void* bias,
                             const void* R, int64_t ldr, void* X, int64_t ldx, float p_drop, uint64_t seed,
                             hipStream_t st) {
  const int64_t n8 = (int64_t)M * N / 8;
  const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 4096);
  splitk_epi_kernel<EPI><<<blocks, 256, 0, st>>>(ws, (bf16_t*)C, M, N, ldc, split, (const bf16_t*)bias,
                                                 (const bf16_t*)R, ldr, (bf16_t*)X, ldx, p_drop, seed);
  return (int)hipGetLastError();
}

// tile config + split-K factor the engine will use for this problem (callers size the
// split-K workspace from it: split * M * N f32)
// 1 when the probe engines (gemm4 cfg 7 / 100+G, gemm5 cfg 8) are compiled in
extern "C" int mp_gemm2_has_probe_engines() {
#ifdef MP_PROBE_ENGINES
  return 1;
#else
  return 0;
#endif
}

// f32 workspace elements the planned engine needs (split-K slabs, or the stream-K flags +
// partial-tile slots)
extern "C" int64_t mp_gemm2_ws_floats(int cfg, int split, int M, int N, int K) {
  if (cfg == 14) {
    // partial slots are indexed by block id; contributors are blocks x + 8 l with
    // l < c (S - 1) for the fullest XCD group's c tail tiles
    Plan7 pl{};
    if (!plan7(M, N, K, &pl)) return (int64_t)SK_FLAGS + (int64_t)SK_MAX_G * SK_SLOT;
    const int cmax = (pl.tail + 7) / 8;
    const int64_t slots = (int64_t)8 * cmax * (pl.S - 1);
    return (int64_t)SK_FLAGS + slots * SK_SLOT;
  }
  return split > 1 ? (int64_t)split * M * N : 0;
}

extern "C" int mp_gemm2_plan(int M, int N, int K, int transA, int transB, int c_f32_accum, int force_cfg,
                             int* split_out) {
  int split = 1;
  // 7: the persistent deferred-store engine (gemm4); 100 + G: gemm4 on a grid of G
  // workgroups (tests drive several tiles per workgroup through small problems)
#ifdef MP_PROBE_ENGINES
  if (force_cfg == 7 || force_cfg >= 100) {
    *split_out = 1;
    return 7;
  }
#else
  if (force_cfg == 7 || force_cfg == 8 || force_cfg >= 100) return -1;   // probe engines not built
#endif
  // 8: the 4-wave / one-wave-per-SIMD 256x256 NT engine (gemm5 probe; MIPIPE_GEMM5=1 uses
  // it wherever gemm3's M16 build would run without split-K)
#ifdef MP_PROBE_ENGINES
  static const bool use5 = [] { const char* e = getenv("MIPIPE_GEMM5"); return e && e[0] == '1'; }();
  if (force_cfg == 8) {
    *split_out = 1;
    return 8;
  }
#else
  constexpr bool use5 = false;
#endif
  int cfg = choose(M, N, K, c_f32_accum != 0, transA || transB, &split);
  if (force_cfg >= 0 && force_cfg < 7) cfg = force_cfg;
  if (force_cfg >= 10) cfg = 0;   // placeholder; the small-engine branches below set it
  // the ping-pong 256x256 engine for both-K-contiguous operands (MIPIPE_GEMM3=0 disables;
  // MIPIPE_GEMM_M16=1 selects its 16x16x32-MFMA build)
  static const bool use3 = [] { const char* e = getenv("MIPIPE_GEMM3"); return !(e && e[0] == '0'); }();
  static const bool m16 = [] { const char* e = getenv("MIPIPE_GEMM_M16"); return !(e && e[0] == '0'); }();
  if (cfg == 0 && !transA && !transB && use3 && force_cfg < 0) cfg = m16 ? 5 : 4;
  // 16x16x32 MFMAs hold a higher clock under load (MI355X_MICROARCH.md DVFS item 7): the
  // M16 ping-pong engine beat the 256x192 / 256x128 gemm2 tiles on every measured NT
  // shape, including grids of fewer tiles than CUs (N = 768: 27.5 vs 30.8 us)
  if (!transA && !transB && use3 && m16 && force_cfg < 0 && split == 1 && cfg != 5) {
    const int t256 = ((M + 255) / 256) * ((N + 255) / 256);
    if (t256 >= 96) cfg = 5;
  }
  // the 256x192 ping-pong engine (gemm6) where its grid fills whole rounds of 256 CUs
  // better than 256x256 does on a multi-round grid: modelled time = rounds x tile area /
  // tile efficiency, 0.84 measured (profiles/r4_gemm6_tail_probe.txt: N = 768 at 32K
  // tokens 2 rounds x 0.89 vs 2 rounds with the second half empty, +3-7 %; 12 MFMAs per
  // phase against gemm3's 16 under the same barriers cost 16 % per tile, so 4.5-round
  // grids and one-round grids stay on gemm3).  Opt-in (MIPIPE_GEMM6=1; force_cfg 9 selects
  // it): inside the step it lost -- 946K vs 973K tok/s with 2 lanes, 929K vs 933K with one,
  // at the PP > 1 per-rank work (r4_gemm6_tail_probe.txt) -- the lanes already fill the
  // half-empty round that it fixes, and it pays its lower per-tile rate everywhere
  static const bool use6 = [] { const char* e = getenv("MIPIPE_GEMM6"); return e && e[0] == '1'; }();
  if (!transA && !transB && use6 && force_cfg < 0 && split == 1 && cfg == 5) {
    const int gm = (M + 255) / 256;
    const int t256 = gm * ((N + 255) / 256);
    const float r256 = (float)((t256 + 255) / 256);
    const float r192 = (float)((gm * ((N + 191) / 192) + 255) / 256) * (0.75f / 0.84f);
    if (t256 > 256 && r192 < 0.97f * r256) cfg = 9;
  }
  if (force_cfg == 9) {
    cfg = (transA || transB) ? 0 : 9;
    split = 1;
  }
  // the TT (dW) build of the ping-pong engine: 256x256 tiles, split-K f32 accumulate
  // (MIPIPE_GEMM3T=0 keeps the 2-stage gemm2 TT engine)
  static const bool use3t = [] { const char* e = getenv("MIPIPE_GEMM3T"); return !(e && e[0] == '0'); }();
  if (cfg == 0 && transA && transB && c_f32_accum && use3t && force_cfg < 0 && M % 8 == 0 && N % 8 == 0) cfg = 6;
  if (cfg == 6 && !(transA && transB && c_f32_accum)) cfg = 0;
  if (cfg >= 4 && cfg != 6 && (transA || transB)) cfg = 0;
  if ((transA || transB) && cfg == 1) cfg = 2;
  // bf16-output split-K runs the f32-accumulate instantiation (NT or TT) into slabs
  if (!c_f32_accum && transA != transB) split = 1;
  if (!c_f32_accum && split > 1 && (cfg == 4 || cfg == 5)) cfg = transA ? 0 : cfg;
  // short-token NT problems (few 256-row tiles): the small-tile engine, one launch, no
  // split-K (MIPIPE_GEMM_SMALL=0 disables; MIPIPE_GEMMS_MINWG = workgroups to aim for)
  static const bool use_small = [] { const char* e = getenv("MIPIPE_GEMM_SMALL"); return !(e && e[0] == '0'); }();
  static const int minwg = [] {
    const char* e = getenv("MIPIPE_GEMMS_MINWG");
    const int v = e ? atoi(e) : 256;
    return v > 0 ? v : 256;
  }();
  if (!transA && !transB && use_small && (force_cfg < 0 || force_cfg >= 10)) {
    const int t256 = ((M + 255) / 256) * ((N + 255) / 256);
    if (force_cfg >= 10 && force_cfg <= 12) {
      cfg = force_cfg;
      split = 1;
    } else if (t256 < 64 && !c_f32_accum && K <= 4096) {   // long K: the big split-K plan wins
      const int w64 = ((M + 63) / 64) * ((N + 63) / 64);
      const int w6432 = ((M + 63) / 64) * ((N + 31) / 32);
      cfg = w64 >= minwg ? 10 : (w6432 >= minwg ? 11 : 12);
      split = 1;
    }
  }
  // short-token dW GEMMs (both operands k-major, f32 accumulate): the small engine's TT
  // build, 64x64 tiles, no split-K (the slabs + reduce pass cost as much as the GEMM here)
  if (transA && transB && c_f32_accum && use_small && (force_cfg < 0 || force_cfg == 13) && M % 8 == 0 &&
      N % 8 == 0) {
    const int t256 = ((M + 255) / 256) * ((N + 255) / 256);
    if (force_cfg == 13 || (t256 < 64 && K <= 4096)) {
      cfg = 13;
      split = 1;
    }
  }
  if (use5 && cfg == 5 && split == 1 && !c_f32_accum && force_cfg < 0) cfg = 8;
  // 15: the four-wave register-staged 256x192 NT engine (gemm8); MIPIPE_GEMM8=1 uses it
  // wherever gemm3's M16 build would run without split-K
  // wherever gemm3's M16 build would run without split-K; MIPIPE_GEMM8=auto where its
  // 256x192 grid fills whole rounds of 256 CUs better than 256x256 does: modelled time =
  // rounds x tile area / tile efficiency, 0.9 measured per 256x192 tile against gemm3's
  // 256x256 (profiles/r6_gemm8_engine.md: standalone, the 16K-token N = 768 / 2304 grids run
  // 1.11-1.15x gemm3 and the 64K-token grids 0.88-0.95x).  Off by default: inside the step
  // (2 lanes, 16K-token microbatches) auto measured 910K vs 942K tok/s -- the second lane
  // already fills gemm3's partial rounds, and gemm8 pays its lower per-tile rate
  static const int use8 = [] {
    const char* e = getenv("MIPIPE_GEMM8");
    return (e && e[0] == '1') ? 1 : ((e && e[0] == 'a') ? 2 : 0);
  }();
  bool pick8 = use8 == 1;
  if (use8 == 2 && !transA && !transB && !c_f32_accum && cfg == 5 && split == 1 && force_cfg < 0) {
    const float r256 = (float)((((M + 255) / 256) * ((N + 255) / 256) + 255) / 256);
    const float r192 = (float)((((M + 255) / 256) * ((N + 191) / 192) + 255) / 256) * (0.75f / 0.9f);
    pick8 = r192 < 0.97f * r256;
  }
  if (!transA && !transB && (force_cfg == 15 || force_cfg == 16 || (pick8 && cfg == 5 && split == 1 && force_cfg < 0))) {
    *split_out = 1;
    return force_cfg == 16 ? 16 : 15;
  }
  // the stream-K engine (gemm7) where the 256x256 grid is not whole rounds of 256 CUs
  // (force_cfg 14 selects it wherever plan7 accepts the grid)
  // Opt-in (MIPIPE_GEMM_SK=1): measured null -- on the all-tail M = 8192 grids the split
  // tail (S = 2) takes 37 vs 23.5 us at K = 768 and 60 vs 55 us at K = 3072; the hand-off of
  // a 256x256 f32 partial (LDS staging + 256 KiB out and back in, sc1 or plain + release
  // alike) costs about what the halved K loop saves (profiles/r5_gemm7_split_tail_null.txt)
  // Probe-only: a timed-out partial hand-off cannot be reported to the host, so
  // cfg 14 is reachable only in the A/B probe build (tools/build_ext.py --variant probes
  // -D MP_PROBE_ENGINES), where test_gemm7_stream_k checks it
#ifdef MP_PROBE_ENGINES
  static const bool use_sk = [] { const char* e = getenv("MIPIPE_GEMM_SK"); return e && e[0] == '1'; }();
#else
  constexpr bool use_sk = false;
  if (force_cfg == 14) return -1;
#endif
  // replaces the ping-pong engine's partial rounds and the bf16-output split-K slabs (f32
  // slab round trip through HBM + a reduce pass) of the gemm2 tiles alike
  if (!transA && !transB && !c_f32_accum && (force_cfg == 14 || (use_sk && force_cfg < 0 && cfg != 10 &&
                                                                 cfg != 11 && cfg != 12 && cfg != 8))) {
    Plan7 pl{};
    if (plan7(M, N, K, &pl) > 0) {
      cfg = 14;
      split = 1;
    }
  }
  *split_out = split;
  return cfg;
}

// returns -2 if the (layout, epilogue) combination is not instantiated here (caller falls back to v1).
// With split-K (f32 accumulate) and a workspace of split*M*N floats the partial products go
// to slabs + one reduce pass; without a workspace they are added with f32 atomics.
extern "C" int mp_gemm2(const void* A, const void* B, void* C, const void* bias, const void* residual, void* aux,
                        int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ld_res, int64_t ld_aux,
                        int transA, int transB, int epilogue, int c_f32_accum, float alpha, int force_cfg, float* ws,
                        float* colsum, float p_drop, uint64_t seed, hipStream_t st) {
  if (K % BK != 0 || N % 8 != 0 || M % 8 != 0) return -1;
  int split = 1;
  const int cfg = mp_gemm2_plan(M, N, K, transA, transB, c_f32_accum, force_cfg, &split);
  if (cfg == 14) {
    if (ws == nullptr) return -1;
    switch (epilogue) {
#define MP_G7(E_) case E_: return launch7<E_>(A, B, C, bias, residual, aux, colsum, ws, M, N, K, lda, ldb, ldc, ld_res, ld_aux, alpha, p_drop, seed, st);
      MP_G7(EPI_NONE) MP_G7(EPI_BIAS) MP_G7(EPI_BIAS_GELU) MP_G7(EPI_BIAS_RELU) MP_G7(EPI_BIAS_RES) MP_G7(EPI_RES)
      MP_G7(EPI_DGELU) MP_G7(EPI_DRELU)
#undef MP_G7
      default: return -2;
    }
  }
  if (colsum != nullptr) {
    // fused output column sums: bf16 outputs, one pass (no split-K); -3 tells the caller
    // to sum separately
    if (c_f32_accum || split > 1) return -3;
    ws = colsum;
  }
  // plain / bias NT GEMMs of more 256x256 tiles than CUs: the persistent engine that
  // writes part of each tile's C during the next tile's main loop.  Opt-in
  // (MIPIPE_GEMM4=1): correct, but 1.2-2x slower than gemm3 -- the 64-VGPR stash does not
  // fit beside gemm3's 222 VGPRs at 2 waves/SIMD, and the spill reloads in the MFMA loop
  // drain the DMA pipeline (profiles/r2_probes.md "gemm4")
  if (cfg < 0) return -1;
#ifdef MP_PROBE_ENGINES
  static const bool use4 = [] { const char* e = getenv("MIPIPE_GEMM4"); return e && e[0] == '1'; }();
  const bool g4_ok = split == 1 && colsum == nullptr && !c_f32_accum && !transA && !transB &&
                     (epilogue == EPI_NONE || epilogue == EPI_BIAS) && ldc % 4 == 0;
  const int t256_all = ((M + 255) / 256) * ((N + 255) / 256);
  if (g4_ok && (cfg == 7 || (use4 && cfg == 5 && force_cfg < 0 && t256_all > 256))) {
    const int grid = force_cfg >= 100 ? force_cfg - 100 : 0;
    if (epilogue == EPI_NONE) return launch4<EPI_NONE>(A, B, C, nullptr, M, N, K, lda, ldb, ldc, alpha, grid, st);
    return launch4<EPI_BIAS>(A, B, C, bias, M, N, K, lda, ldb, ldc, alpha, grid, st);
  }
#endif
  if (cfg == 7) return -2;
  float* wsp = (split > 1 || colsum != nullptr) ? ws : nullptr;
  int rc = -2;
  if (!c_f32_accum && split > 1) {
    // bf16 output, split-K: partial products into f32 slabs (alpha applied there), then
    // one pass sums them and applies the fused epilogue
    if (ws == nullptr) return -1;
    if (transA && transB) rc = dispatch<true, true, EPI_NONE, true>(cfg, A, B, nullptr, nullptr, nullptr, nullptr, ws, M, N, K,
                                                              lda, ldb, N, 0, 0, alpha, split, p_drop, seed, st);
    else rc = dispatch<false, false, EPI_NONE, true>(cfg, A, B, nullptr, nullptr, nullptr, nullptr, ws, M, N, K, lda, ldb,
                                                     N, 0, 0, alpha, split, p_drop, seed, st);
    if (rc != 0) return rc;
    switch (epilogue) {
      case EPI_NONE: return launch_splitk_epi<EPI_NONE>(ws, C, M, N, ldc, split, bias, residual, ld_res, aux, ld_aux, p_drop, seed, st);
      case EPI_BIAS: return launch_splitk_epi<EPI_BIAS>(ws, C, M, N, ldc, split, bias, residual, ld_res, aux, ld_aux, p_drop, seed, st);
      case EPI_BIAS_GELU: return launch_splitk_epi<EPI_BIAS_GELU>(ws, C, M, N, ldc, split, bias, residual, ld_res, aux, ld_aux, p_drop, seed, st);
      case EPI_BIAS_RELU: return launch_splitk_epi<EPI_BIAS_RELU>(ws, C, M, N, ldc, split, bias, residual, ld_res, aux, ld_aux, p_drop, seed, st);
      case EPI_BIAS_RES: return launch_splitk_epi<EPI_BIAS_RES>(ws, C, M, N, ldc, split, bias, residual, ld_res, aux, ld_aux, p_drop, seed, st);
      case EPI_RES: return launch_splitk_epi<EPI_RES>(ws, C, M, N, ldc, split, bias, residual, ld_res, aux, ld_aux, p_drop, seed, st);
      case EPI_DGELU: return launch_splitk_epi<EPI_DGELU>(ws, C, M, N, ldc, split, bias, residual, ld_res, aux, ld_aux, p_drop, seed, st);
      case EPI_DRELU: return launch_splitk_epi<EPI_DRELU>(ws, C, M, N, ldc, split, bias, residual, ld_res, aux, ld_aux, p_drop, seed, st);
      default: return -2;
    }
  }
#define MP_G(TA_, TB_, E_, ACC_)                                                                                  \
  if (rc == -2 && (bool)transA == TA_ && (bool)transB == TB_ && epilogue == E_ && (bool)c_f32_accum == ACC_)     \
    rc = dispatch<TA_, TB_, E_, ACC_>(cfg, A, B, C, bias, residual, aux, wsp, M, N, K, lda, ldb, ldc, ld_res,       \
                                      ld_aux, alpha, split, p_drop, seed, st);
  MP_G(false, false, EPI_NONE, false)
  MP_G(false, false, EPI_BIAS, false)
  MP_G(false, false, EPI_BIAS_GELU, false)
  MP_G(false, false, EPI_BIAS_RELU, false)
  MP_G(false, false, EPI_BIAS_RES, false)
  MP_G(false, false, EPI_RES, false)
  MP_G(false, false, EPI_DGELU, false)
  MP_G(false, false, EPI_DRELU, false)
  MP_G(true, true, EPI_NONE, true)
  MP_G(false, false, EPI_NONE, true)
#undef MP_G
  if (rc == 0 && wsp != nullptr && split > 1) {
    const int64_t n4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 4096);
    splitk_reduce_kernel<<<blocks, 256, 0, st>>>(wsp, reinterpret_cast<float*>(C), M, N, ldc, split);
    rc = (int)hipGetLastError();
  }
  return rc;
}

MP_DROP_STEP_SETTER(mp_set_drop_step_gemm)

// C_g += alpha * A_g^T B_g for n <= MP_GROUP_MAX problems (A_g [K_g][M_g], B_g [K_g][N_g]
// bf16 k-major, C_g f32 [M_g][N_g] row stride ldc_g) in one launch; -1 if a shape does not
// fit the 64x64 TT tile contract (M, N multiples of 8, K of 64)
extern "C" int mp_gemm_tt_grouped(int n, const void* const* A, const void* const* B, float* const* C, const int* M,
                                  const int* N, const int* K, const int64_t* lda, const int64_t* ldb,
                                  const int64_t* ldc, float alpha, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > MP_GROUP_MAX) return -1;
  GroupTT g{};
  g.n = n;
  g.alpha = alpha;
  int t = 0;
  for (int i = 0; i < n; ++i) {
    if (M[i] % 8 || N[i] % 8 || K[i] % BK || M[i] <= 0 || N[i] <= 0) return -1;
    g.A[i] = (const bf16_t*)A[i];
    g.B[i] = (const bf16_t*)B[i];
    g.C[i] = C[i];
    g.M[i] = M[i];
    g.N[i] = N[i];
    g.K[i] = K[i];
    g.lda[i] = lda[i];
    g.ldb[i] = ldb[i];
    g.ldc[i] = ldc[i];
    g.tile_start[i] = t;
    t += ((M[i] + 63) / 64) * ((N[i] + 63) / 64);
  }
  for (int i = n; i <= MP_GROUP_MAX; ++i) g.tile_start[i] = t;
  constexpr int STAGE = (64 + 64) * BK * 2;
  constexpr int EPI_BYTES = 32 * (64 + 4) * 4;
  constexpr int LDS = 2 * STAGE > EPI_BYTES ? 2 * STAGE : EPI_BYTES;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemms_tt_grouped_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  gemms_tt_grouped_kernel<<<t, 256, LDS, st>>>(g);
  return (int)hipGetLastError();
}
