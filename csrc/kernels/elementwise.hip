// Memory-bound elementwise kernels of the transformer block, all with 16-byte
// bf16 vectors and, where a bias gradient is needed, a fused column reduction
// (per-block partials in registers -> LDS across waves -> one f32 atomic per column).
//
//   act_fwd         g = dropout(act(a))                 (FFN activation when not fused in a GEMM)
//   act_bwd         da = dg * dropout_mask * act'(a);  dbias += colsum(da)
//   colsum          dbias += colsum(x)                  (bias grads of the projections)
//   swiglu_fwd/bwd  y = silu(gate) * up  over a [T, 2F] gate|up buffer (Llama-3 FFN)
//   rope            rotate-half RoPE on the q/k heads of the packed qkv buffer, in place
//                   (forward: +theta, backward: -theta), f32 cos/sin table from the host
#include "mp_common.h"

#include <stdlib.h>

using namespace mp;

enum Act { ACT_NONE = 0, ACT_GELU_TANH = 1, ACT_RELU = 2 };

__device__ __forceinline__ float act_f(float x, int act) {
  if (act == ACT_GELU_TANH) return gelu_tanh(x);
  if (act == ACT_RELU) return fmaxf(x, 0.f);
  return x;
}
__device__ __forceinline__ float act_g(float x, int act) {
  if (act == ACT_GELU_TANH) return gelu_tanh_grad(x);
  if (act == ACT_RELU) return x > 0.f ? 1.f : 0.f;
  return 1.f;
}

__global__ void __launch_bounds__(256) act_fwd_kernel(const bf16_t* __restrict__ a, bf16_t* __restrict__ g, int64_t n,
                                                      int act, float p, uint64_t seed) {
  if (p > 0.f) seed = step_seed(seed);
  const int64_t n8 = n / 8;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    u16x8 v = reinterpret_cast<const u16x8*>(a)[i];
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float y = act_f(bf2f(v[e]), act);
      if (p > 0.f) y *= dropout_scale(seed, i * 8 + e, p);
      o[e] = f2bf(y);
    }
    reinterpret_cast<u16x8*>(g)[i] = o;
  }
}

// MODE 0: colsum(x) -> dbias ; MODE 1: da = dg*act'(a)*mask (written), dbias += colsum(da)
template <int MODE, typename T = bf16_t>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ x, const bf16_t* __restrict__ a,
                                                     bf16_t* __restrict__ da, float* __restrict__ dbias, int rows,
                                                     int cols, int rows_per_block, int act, float p, uint64_t seed,
                                                     float* __restrict__ part) {
  if (p > 0.f) seed = step_seed(seed);
  __shared__ float red[4][64 * 8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int chunk = blockIdx.y * 64 + lane;
  const bool active = chunk * 8 < cols;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  if (active) {
    for (int r = r0 + wv; r < r1; r += 4) {
      const size_t off = (size_t)r * cols + chunk * 8;
      if constexpr (MODE == 0) {
        const typename IO8<T>::Raw xv = IO8<T>::load(x + off);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += IO8<T>::get(xv, e);
      } else {
        u16x8 xv = *reinterpret_cast<const u16x8*>(x + off);
        u16x8 av = *reinterpret_cast<const u16x8*>(a + off);
        u16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float d = bf2f(xv[e]) * act_g(bf2f(av[e]), act);
          if (p > 0.f) d *= dropout_scale(seed, off + e, p);
          o[e] = f2bf(d);
          acc[e] += bf2f(o[e]);
        }
        *reinterpret_cast<u16x8*>(da + off) = o;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[wv][lane * 8 + e] = acc[e];
  __syncthreads();
  if (dbias == nullptr) return;
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int col = blockIdx.y * 512 + i;
    if (col >= cols) continue;
    const float v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    // with a partial buffer: plain stores, summed by colpart_reduce_kernel (every block
    // adding into the same few KB with atomics serialised at the memory side)
    if (part != nullptr) part[(int64_t)blockIdx.x * cols + col] = v;
    else atomicAdd(dbias + col, v);
  }
}

// out_s[col] += sum over blocks b of part[b][s][col]  (s < nslot; null outputs skipped).
// grid (ceil(D / 256), nslot, block groups); one f32 atomic per column per block group.
__global__ void __launch_bounds__(256) colpart_reduce_kernel(const float* __restrict__ part, int nblk, int nslot,
                                                             int D, float* __restrict__ o0, float* __restrict__ o1,
                                                             float* __restrict__ o2, float* __restrict__ o3,
                                                             int per_group) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  const int sl = blockIdx.y;
  float* out = sl == 0 ? o0 : sl == 1 ? o1 : sl == 2 ? o2 : o3;
  if (out == nullptr || col >= D) return;
  const int b0 = blockIdx.z * per_group, b1 = min(nblk, b0 + per_group);
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
  int b = b0;
  for (; b + 3 < b1; b += 4) {
    acc0 += part[((int64_t)b * nslot + sl) * D + col];
    acc1 += part[((int64_t)(b + 1) * nslot + sl) * D + col];
    acc2 += part[((int64_t)(b + 2) * nslot + sl) * D + col];
    acc3 += part[((int64_t)(b + 3) * nslot + sl) * D + col];
  }
  for (; b < b1; ++b) acc0 += part[((int64_t)b * nslot + sl) * D + col];
  atomicAdd(out + col, (acc0 + acc1) + (acc2 + acc3));
}

extern "C" int mp_colpart_reduce(const float* part, int nblk, int nslot, int D, float* o0, float* o1, float* o2,
                                 float* o3, hipStream_t st) {
  const int per = 32;
  dim3 grid((D + 255) / 256, nslot, (nblk + per - 1) / per);
  colpart_reduce_kernel<<<grid, 256, 0, st>>>(part, nblk, nslot, D, o0, o1, o2, o3, per);
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ y, int T,
                                                         int F) {
  const int64_t n8 = (int64_t)T * F / 8;
  const int f8 = F / 8;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t t = i / f8, c = i % f8;
    u16x8 g = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + c * 8);
    u16x8 u = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + F + c * 8);
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(silu(bf2f(g[e])) * bf2f(u[e]));
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
}

__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dy,
                                                         bf16_t* __restrict__ dgu, int T, int F) {
  const int64_t n8 = (int64_t)T * F / 8;
  const int f8 = F / 8;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t t = i / f8, c = i % f8;
    u16x8 g = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + c * 8);
    u16x8 u = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + F + c * 8);
    u16x8 d = reinterpret_cast<const u16x8*>(dy)[i];
    u16x8 og, ou;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gf = bf2f(g[e]), uf = bf2f(u[e]), df = bf2f(d[e]);
      const float sg = 1.f / (1.f + __expf(-gf));
      const float sl = gf * sg;
      ou[e] = f2bf(df * sl);
      og[e] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
    }
    *reinterpret_cast<u16x8*>(dgu + t * 2 * F + c * 8) = og;
    *reinterpret_cast<u16x8*>(dgu + t * 2 * F + F + c * 8) = ou;
  }
}

// qkv: [T, (H + 2*Hkv) * Dh] with heads laid out q(H) | k(Hkv) | v(Hkv).  Rotates q and k
// in place; cos/sin: [S, Dh/2] f32.  sign = +1 forward, -1 backward (inverse rotation).
__global__ void __launch_bounds__(256) rope_kernel(bf16_t* __restrict__ qkv, const float* __restrict__ cs,
                                                   const float* __restrict__ sn, int T, int S, int H, int Hkv, int Dh,
                                                   int pos_offset, float sign) {
  const int half = Dh / 2;
  const int nh = H + Hkv;  // rotated heads per token
  const int64_t total = (int64_t)T * nh * (half / 4);
  const int stride = (H + 2 * Hkv) * Dh;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int q4 = (int)(i % (half / 4));
    const int64_t th = i / (half / 4);
    const int h = (int)(th % nh);
    const int64_t t = th / nh;
    const int pos = (int)(t % S) + pos_offset;
    bf16_t* base = qkv + t * stride + (int64_t)h * Dh;
    u16x4 x1 = *reinterpret_cast<u16x4*>(base + q4 * 4);
    u16x4 x2 = *reinterpret_cast<u16x4*>(base + half + q4 * 4);
    u16x4 o1, o2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = q4 * 4 + e;
      const float c = cs[(int64_t)pos * half + j], s = sign * sn[(int64_t)pos * half + j];
      const float a = bf2f(x1[e]), b = bf2f(x2[e]);
      o1[e] = f2bf(a * c - b * s);
      o2[e] = f2bf(b * c + a * s);
    }
    *reinterpret_cast<u16x4*>(base + q4 * 4) = o1;
    *reinterpret_cast<u16x4*>(base + half + q4 * 4) = o2;
  }
}

// out[C][R] = in[R][C] (bf16), 64x64 tiles through LDS (+1 pad); in/out row strides given.
__global__ void __launch_bounds__(256) transpose_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                        int R, int C, int64_t ldi, int64_t ldo) {
  __shared__ bf16_t tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? in[(int64_t)r * ldi + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) out[(int64_t)c * ldo + r] = tile[tx][i];
  }
}

// All W^T copies of a parameter arena in ONE launch (refreshed after every optimizer step).
// desc[i] = {src offset, dst offset, R, C} (elements, into the w16 / wt16 arenas); block b
// transposes 64x64 tile (b - tile0[i]) of matrix i, found by binary search over the tile
// prefix.  16-byte global loads and stores (C and R are multiples of 8), LDS tile in between.
__global__ void __launch_bounds__(256) transpose_batched_kernel(const bf16_t* __restrict__ src,
                                                                bf16_t* __restrict__ dst,
                                                                const int64_t* __restrict__ desc,
                                                                const int* __restrict__ tile0, int n) {
  __shared__ bf16_t tile[64][72];   // 144-byte rows: 16-byte aligned, rows spread over banks
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {  // last i with tile0[i] <= b
    const int mid = (lo + hi + 1) >> 1;
    if (tile0[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const int64_t so = desc[4 * lo], dof = desc[4 * lo + 1];
  const int R = (int)desc[4 * lo + 2], C = (int)desc[4 * lo + 3];
  const int t = b - tile0[lo], tcols = (C + 63) / 64;
  const int r0 = (t / tcols) * 64, c0 = (t % tcols) * 64;
  const int tid = threadIdx.x;
  // load: 64 rows x 8 chunks of 8 columns = 512 chunks, 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k, rr = idx >> 3, cc = (idx & 7) * 8;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + rr < R && c0 + cc < C) v = *reinterpret_cast<const u16x8*>(src + so + (int64_t)(r0 + rr) * C + c0 + cc);
    *reinterpret_cast<u16x8*>(&tile[rr][cc]) = v;
  }
  __syncthreads();
  // store: output row = input column (64 of them), 8 chunks of 8 input rows each
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k, oc = idx >> 3, orr = (idx & 7) * 8;   // output row oc, cols orr..orr+7
    if (c0 + oc < C && r0 + orr < R) {
      u16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = tile[orr + e][oc];
      *reinterpret_cast<u16x8*>(dst + dof + (int64_t)(c0 + oc) * R + r0 + orr) = v;
    }
  }
}

extern "C" int mp_transpose_batched(const void* src, void* dst, const int64_t* desc, const int* tile0, int n,
                                    int total_tiles, hipStream_t st) {
  if (n <= 0 || total_tiles <= 0) return 0;
  transpose_batched_kernel<<<total_tiles, 256, 0, st>>>((const bf16_t*)src, (bf16_t*)dst, desc, tile0, n);
  return (int)hipGetLastError();
}

static int grid_n8(int64_t n) {
  int64_t b = (n / 8 + 255) / 256;
  return (int)(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

extern "C" int mp_act_fwd(const void* a, void* g, int64_t n, int act, float p, uint64_t seed, hipStream_t st) {
  if (n % 8) return -1;
  act_fwd_kernel<<<grid_n8(n), 256, 0, st>>>((const bf16_t*)a, (bf16_t*)g, n, act, p, seed);
  return (int)hipGetLastError();
}

static void colsum_grid(int rows, int cols, dim3& grid, int& rpb) {
  // every block ends with one f32 atomic per column: at least MIPIPE_COLSUM_RPB (32) rows
  // per block, so short (1024-row) problems do not turn into atomic contention
  static const int min_rpb = [] {
    const char* e = getenv("MIPIPE_COLSUM_RPB");
    const int v = e ? atoi(e) : 32;
    return v > 0 ? v : 32;
  }();
  const int ny = (cols / 8 + 63) / 64;
  int nx = 1024 / ny;
  if (nx < 1) nx = 1;
  if (nx > (rows + 3) / 4) nx = (rows + 3) / 4;
  if (nx > (rows + min_rpb - 1) / min_rpb) nx = (rows + min_rpb - 1) / min_rpb;
  if (nx < 1) nx = 1;
  rpb = (rows + nx - 1) / nx;
  grid = dim3((rows + rpb - 1) / rpb, ny);
}

// f32 elements of the partial-sum buffer a colsum of [rows, cols] can use (0: atomics only)
// partials only pay off with many blocks: a 32-block column sum (1024 rows) measured
// 9.2 us with partials + reduce vs 4.0 us with atomics; 512 blocks: 9.7 vs 15.3 us
static constexpr int kColpartMinBlocks = 256;

// MIPIPE_COLPART=0: per-column f32 atomics from every block instead of per-block partials
// plus colpart_reduce_kernel (A/B knob)
extern "C" int mp_colpart_enabled() {
  static const int on = [] {
    const char* e = getenv("MIPIPE_COLPART");
    return e ? atoi(e) : 1;
  }();
  return on;
}

extern "C" int64_t mp_colsum_part_elems(int rows, int cols) {
  if (!mp_colpart_enabled()) return 0;
  dim3 grid;
  int rpb;
  colsum_grid(rows, cols, grid, rpb);
  return grid.x >= kColpartMinBlocks ? (int64_t)grid.x * cols : 0;
}

extern "C" int mp_act_bwd(const void* dg, const void* a, void* da, float* dbias, int rows, int cols, int act, float p,
                          uint64_t seed, float* part, hipStream_t st) {
  if (cols % 8) return -1;
  dim3 grid;
  int rpb;
  colsum_grid(rows, cols, grid, rpb);
  if (grid.x < kColpartMinBlocks || dbias == nullptr) part = nullptr;
  colsum_kernel<1><<<grid, 256, 0, st>>>((const bf16_t*)dg, (const bf16_t*)a, (bf16_t*)da, dbias, rows, cols, rpb, act,
                                         p, seed, part);
  if (part != nullptr) return mp_colpart_reduce(part, grid.x, 1, cols, dbias, nullptr, nullptr, nullptr, st);
  return (int)hipGetLastError();
}

extern "C" int mp_colsum(const void* x, float* dbias, int rows, int cols, float* part, int f32, hipStream_t st) {
  if (cols % 8) return -1;
  dim3 grid;
  int rpb;
  colsum_grid(rows, cols, grid, rpb);
  if (grid.x < kColpartMinBlocks) part = nullptr;
  if (f32)
    colsum_kernel<0, float><<<grid, 256, 0, st>>>((const float*)x, nullptr, nullptr, dbias, rows, cols, rpb, 0, 0.f, 0,
                                                  part);
  else
    colsum_kernel<0><<<grid, 256, 0, st>>>((const bf16_t*)x, nullptr, nullptr, dbias, rows, cols, rpb, 0, 0.f, 0, part);
  if (part != nullptr) return mp_colpart_reduce(part, grid.x, 1, cols, dbias, nullptr, nullptr, nullptr, st);
  return (int)hipGetLastError();
}

extern "C" int mp_swiglu_fwd(const void* gu, void* y, int T, int F, hipStream_t st) {
  if (F % 8) return -1;
  swiglu_fwd_kernel<<<grid_n8((int64_t)T * F), 256, 0, st>>>((const bf16_t*)gu, (bf16_t*)y, T, F);
  return (int)hipGetLastError();
}

extern "C" int mp_swiglu_bwd(const void* gu, const void* dy, void* dgu, int T, int F, hipStream_t st) {
  if (F % 8) return -1;
  swiglu_bwd_kernel<<<grid_n8((int64_t)T * F), 256, 0, st>>>((const bf16_t*)gu, (const bf16_t*)dy, (bf16_t*)dgu, T, F);
  return (int)hipGetLastError();
}

extern "C" int mp_rope(void* qkv, const float* cs, const float* sn, int T, int S, int H, int Hkv, int Dh,
                       int pos_offset, int inverse, hipStream_t st) {
  if (Dh % 8) return -1;
  const int64_t total = (int64_t)T * (H + Hkv) * (Dh / 8);
  int64_t b = (total + 255) / 256;
  rope_kernel<<<(int)(b < 4096 ? b : 4096), 256, 0, st>>>((bf16_t*)qkv, cs, sn, T, S, H, Hkv, Dh, pos_offset,
                                                          inverse ? -1.f : 1.f);
  return (int)hipGetLastError();
}

extern "C" int mp_transpose(const void* in, void* out, int R, int C, int64_t ldi, int64_t ldo, hipStream_t st) {
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  transpose_kernel<<<grid, 256, 0, st>>>((const bf16_t*)in, (bf16_t*)out, R, C, ldi, ldo);
  return (int)hipGetLastError();
}

MP_DROP_STEP_SETTER(mp_set_drop_step_elem)
