// bf16 MFMA GEMM with fused epilogues for the transformer's linear layers (SURVEY §2.5
// K2/K3/K5/K8/K9 and their backward).
//
//   C[M,N] = alpha * op(A) op(B) (+ epilogue)            op(A): [M,K],  op(B)^T: [N,K]
//   A stored [M][K] (TA=0, K contiguous) or [K][M] (TA=1, M contiguous)
//   B stored [N][K] (TB=0, K contiguous: nn.Linear weight) or [K][N] (TB=1, N contiguous)
//
// Every use in a transformer layer maps onto this without transposes:
//   forward   Y  = X W^T (+b, +GELU/ReLU with pre-activation saved, +residual)  TA=0 TB=0
//   dX        dX = dY W             (+GELU'/ReLU' of the saved pre-activation)   TA=0 TB=1
//   dW        dW += dY^T X          (f32 accumulate into the flat grad arena)    TA=1 TB=1
//
// Tiles are staged from global in their natural layout (coalesced 16-byte loads) into an
// XOR-swizzled LDS image; the MFMA fragments are read with ds_read_b128 when the
// reduction dim is contiguous and with ds_read_b64_tr_b16 (hardware transpose) when it is
// not.  128x128x64 tile, 4 waves (2x2, 64x64 per wave = 2x2 MFMA 32x32x16), LDS double
// buffer with register staging (global loads for k-tile t+1 in flight during the MFMAs of
// tile t, one barrier per k-tile), XCD-aware + grouped block order, and an LDS-staged
// epilogue so the bias / activation / residual / accumulate pass is fully coalesced.
#include "mp_common.h"

using namespace mp;

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

enum Epi {
  EPI_NONE = 0,
  EPI_BIAS = 1,
  EPI_BIAS_GELU = 2,
  EPI_BIAS_RELU = 3,
  EPI_BIAS_RES = 4,
  EPI_RES = 5,
  EPI_DGELU = 6,
  EPI_DRELU = 7,
};

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand tile
constexpr int CPITCH = BN + 4;           // f32 epilogue tile pitch (floats)

// LDS images:
//  K-contiguous tile: [128 rows][64 k] -> 128-byte rows (8 chunks)
//  outer-contiguous tile: [64 k][128 cols] -> 256-byte rows (16 chunks)
__device__ __forceinline__ int swz8(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int swz16(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int off_k(int row, int chunk) { return row * 128 + 16 * (chunk ^ swz8(row)); }
__device__ __forceinline__ int off_o(int row, int chunk) { return row * 256 + 16 * (chunk ^ swz16(row)); }

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// fragment (8 consecutive k of row/col `rc` within the tile, k-step s of 16) from an image
template <bool OUTER>
__device__ __forceinline__ bf16x8 frag(const char* img, int rc, int s, int hl) {
  if constexpr (!OUTER) {
    return *reinterpret_cast<const bf16x8*>(img + off_k(rc, 2 * s + hl));
  } else {
    // transposed read: 16-lane group g covers cols c0..c0+15, lane gets column c0 + (lane & 15)
    const int i = threadIdx.x & 15, q = i >> 2, p = i & 3;
    const int c0 = (rc & ~15);  // rc = tile col of this lane; its 16-aligned group base
    const int col = c0 + 4 * p;
    const int r0 = 16 * s + 8 * hl;
    const char* a0 = img + off_o(r0 + q, col >> 3) + ((col & 7) << 1);
    const char* a1 = img + off_o(r0 + 4 + q, col >> 3) + ((col & 7) << 1);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

// global -> register staging of one operand tile (4 x 16 bytes per thread)
template <bool OUTER>
struct Stager {
  u16x8 v[4];
  // base points at element (outer0, k0) ; ld = leading dim (elements) ; outer_lim = #valid rows/cols
  __device__ __forceinline__ void load(const bf16_t* base, int64_t ld, int outer0, int outer_lim, int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + 256 * i;
      u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (!OUTER) {  // [128 outer][64 k]: 8 chunks per row
        const int r = idx >> 3, c = idx & 7;
        const int o = outer0 + r;
        v[i] = o < outer_lim ? *reinterpret_cast<const u16x8*>(base + (int64_t)o * ld + k0 + c * 8) : z;
      } else {  // [64 k][128 outer]: 16 chunks per row
        const int r = idx >> 4, c = idx & 15;
        const int o = outer0 + c * 8;
        v[i] = o < outer_lim ? *reinterpret_cast<const u16x8*>(base + (int64_t)(k0 + r) * ld + o) : z;
      }
    }
  }
  __device__ __forceinline__ void store(char* img) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + 256 * i;
      if constexpr (!OUTER) {
        *reinterpret_cast<u16x8*>(img + off_k(idx >> 3, idx & 7)) = v[i];
      } else {
        *reinterpret_cast<u16x8*>(img + off_o(idx >> 4, idx & 15)) = v[i];
      }
    }
  }
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <bool TA, bool TB, int EPI, bool ACC>
__global__ void __launch_bounds__(256, 2) gemm_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                      void* __restrict__ Cv, const bf16_t* __restrict__ bias,
                                                      const bf16_t* __restrict__ R, bf16_t* __restrict__ AUX, int M,
                                                      int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                      int64_t ldr, int64_t ldx, float alpha) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define abuf(i) (smem + (i) * TILE_BYTES)
#define bbuf(i) (smem + (2 + (i)) * TILE_BYTES)

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

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hl = lane >> 5, l32 = lane & 31;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;

  Stager<TA> sa;
  Stager<TB> sb;
  // A base: TA=0 -> A[m][k] ; TA=1 -> A[k][m]
  auto loadA = [&](int k0) { sa.load(A, lda, m0, M, k0); };
  auto loadB = [&](int k0) { sb.load(B, ldb, n0, N, k0); };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = {};

  // split-K: blockIdx.y selects a contiguous K range (f32 accumulate path only)
  const int nsplit = gridDim.y;
  const int nk = K / BK / nsplit;
  const int kbase = (int)blockIdx.y * nk * BK;
  loadA(kbase);
  loadB(kbase);
  sa.store(abuf(0));
  sb.store(bbuf(0));
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      loadA(kbase + (kt + 1) * BK);
      loadB(kbase + (kt + 1) * BK);
    }
    const char* ai = abuf(cur);
    const char* bi = bbuf(cur);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = frag<TA>(ai, wm + 32 * i + l32, s, hl);
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = frag<TB>(bi, wn + 32 * j + l32, s, hl);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(af[i], bf[j], acc[i][j]);
    }
    if (kt + 1 < nk) {
      sa.store(abuf(cur ^ 1));
      sb.store(bbuf(cur ^ 1));
    }
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS (f32) -> coalesced rows of 8 columns per thread
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const int col = wn + 32 * j + l32;
        ct[row * CPITCH + col] = acc[i][j][r];
      }
  __syncthreads();
  if constexpr (ACC) {
    if (nsplit > 1) {
      // lane-consecutive columns: each f32 atomic wave-instruction covers 256 contiguous bytes
      float* C = reinterpret_cast<float*>(Cv);
      for (int idx = threadIdx.x; idx < BM * BN; idx += 256) {
        const int row = idx >> 7, col = idx & 127;
        const int gr = m0 + row, gc = n0 + col;
        if (gr < M && gc < N) atomicAdd(C + (int64_t)gr * ldc + gc, alpha * ct[row * CPITCH + col]);
      }
      return;
    }
  }
#pragma unroll
  for (int it = 0; it < (BM * BN / 8) / 256; ++it) {
    const int idx = threadIdx.x + 256 * it;
    const int row = idx >> 4, c8 = (idx & 15) * 8;
    const int gr = m0 + row, gc = n0 + c8;
    if (gr >= M || gc >= N) continue;
    float v[8];
    const float4 lo = *reinterpret_cast<const float4*>(ct + row * CPITCH + c8);
    const float4 hi = *reinterpret_cast<const float4*>(ct + row * CPITCH + c8 + 4);
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
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_RES) {
        u16x8 bv = *reinterpret_cast<const u16x8*>(bias + gc);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bf2f(bv[e]);
      }
      if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU) {
        u16x8 sv;   // ReLU: the pre-activation; GELU: its derivative (gemm2.hip epi_store8)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = bf2f(f2bf(v[e]));
          if constexpr (EPI == EPI_BIAS_GELU) {
            float d;
            gelu_tanh_and_grad(x, v[e], d);
            sv[e] = f2bf(d);
          } else {
            sv[e] = f2bf(x);
            v[e] = fmaxf(x, 0.f);
          }
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
          const float x = bf2f(xv[e]);
          v[e] *= EPI == EPI_DGELU ? x : (x > 0.f ? 1.f : 0.f);
        }
      }
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e]);
      *reinterpret_cast<u16x8*>(reinterpret_cast<bf16_t*>(Cv) + (int64_t)gr * ldc + gc) = o;
    }
  }
}

#undef abuf
#undef bbuf

template <bool TA, bool TB, int EPI, bool ACC>
static int launch(const void* A, const void* B, void* C, const void* bias, const void* R, void* X, int M, int N, int K,
                  int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int64_t ldx, float alpha, hipStream_t st) {
  const size_t lds = (size_t)BM * CPITCH * 4 > 4 * TILE_BYTES ? (size_t)BM * CPITCH * 4 : 4 * TILE_BYTES;
  auto kern = gemm_kernel<TA, TB, EPI, ACC>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int split = 1;
  if (ACC) {
    // enough workgroups to fill 256 CUs twice, each K slice >= 512 deep and a divisor of K/BK
    const int ktiles = K / BK;
    int want = (512 + nwg - 1) / nwg;
    for (int s = want > 16 ? 16 : want; s > 1; --s)
      if (ktiles % s == 0 && ktiles / s >= 8) { split = s; break; }
  }
  kern<<<dim3(nwg, split), 256, lds, st>>>((const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias, (const bf16_t*)R,
                              (bf16_t*)X, M, N, K, lda, ldb, ldc, ldr, ldx, alpha);
  return (int)hipGetLastError();
}

extern "C" int mp_gemm(const void* A, const void* B, void* C, const void* bias, const void* residual, void* aux, int M,
                       int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ld_res, int64_t ld_aux,
                       int transA, int transB, int epilogue, int c_f32_accum, float alpha, hipStream_t st) {
  if (K % BK != 0 || N % 8 != 0) return -1;
  if (transA && M % 8 != 0) return -1;
#define MP_G(TA_, TB_, E_, ACC_)                                                                               \
  if ((bool)transA == TA_ && (bool)transB == TB_ && epilogue == E_ && (bool)c_f32_accum == ACC_)              \
    return launch<TA_, TB_, E_, ACC_>(A, B, C, bias, residual, aux, M, N, K, lda, ldb, ldc, ld_res, ld_aux, alpha, \
                                      st);
  // forward projections (TA=0, TB=0)
  MP_G(false, false, EPI_NONE, false)
  MP_G(false, false, EPI_BIAS, false)
  MP_G(false, false, EPI_BIAS_GELU, false)
  MP_G(false, false, EPI_BIAS_RELU, false)
  MP_G(false, false, EPI_BIAS_RES, false)
  MP_G(false, false, EPI_RES, false)
  // input grads (TA=0, TB=1)
  MP_G(false, true, EPI_NONE, false)
  MP_G(false, true, EPI_DGELU, false)
  MP_G(false, true, EPI_DRELU, false)
  MP_G(false, true, EPI_RES, false)
  // weight grads (TA=1, TB=1), f32 accumulate
  MP_G(true, true, EPI_NONE, true)
  // misc
  MP_G(false, false, EPI_NONE, true)
  MP_G(true, false, EPI_NONE, true)
#undef MP_G
  return -2;
}
