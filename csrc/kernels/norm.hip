// Fused residual-add (+dropout) + LayerNorm / RMSNorm, forward and backward.
//
// Storage type T = bf16 (16-byte vectors) or f32 (the reference-precision path, 32-byte
// vectors); statistics and accumulation always f32.
// Forward (one wave per row, 8-element vectors, row kept in registers):
//     s = a + dropout(b)        (optional; written out as the new residual stream)
//     y = norm(s) * w (+ bias)  (LayerNorm or RMSNorm)
//     mean / rstd saved in f32 for the backward
// Backward:
//     dxhat = dy * w
//     ds = rstd * (dxhat - mean(dxhat) - xhat * mean(dxhat * xhat))   (LN; RMS drops the mean term)
//     ds += dres                 (gradient arriving through the residual path, fused)
//     db_branch = ds * mask      (optional: grad into the dropout branch)
//     dw += sum_rows(dy * xhat), dbias += sum_rows(dy): per-block partials in
//     registers, reduced across the block's waves in LDS, one f32 atomic per column.
// SURVEY §2.5 K7 (post-LN: 3 per layer + final) and the pre-norm GPT-2 / Llama blocks.
#include "mp_common.h"

#include <stdlib.h>

using namespace mp;

template <typename T, int MAXJ, bool RMS, bool HAS_B, bool HAS_BIAS>
__global__ void __launch_bounds__(256) norm_fwd_kernel(
    const T* __restrict__ a, const T* __restrict__ b, const T* __restrict__ w,
    const T* __restrict__ bias, T* __restrict__ s_out, T* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int rows, int D, float eps, float p_drop, uint64_t seed) {
  using IO = IO8<T>;
  using Raw = typename IO::Raw;
  if (p_drop > 0.f) seed = step_seed(seed);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nchunk = D >> 3;
  float v[MAXJ][8];
  const size_t base = (size_t)row * D;
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    if (c < nchunk) {
      Raw av = IO::load(a + base + c * 8);
      Raw bv;
      if (HAS_B) bv = IO::load(b + base + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = IO::get(av, e);
        if (HAS_B) {
          float bb = IO::get(bv, e);
          if (p_drop > 0.f) bb *= dropout_scale(seed, base + c * 8 + e, p_drop);
          x = IO::round(x + bb);  // residual stream is stored in T: normalise what is stored
        }
        v[j][e] = x;
        sum += x;
      }
      if (HAS_B) {
        Raw sv;
#pragma unroll
        for (int e = 0; e < 8; ++e) IO::set(sv, e, v[j][e]);
        IO::store(s_out + base + c * 8, sv);
      }
    }
  }
  float mean = 0.f;
  if (!RMS) mean = wave_sum(sum) / D;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    if (c < nchunk) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float d = v[j][e] - mean;
        sq += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / D + eps);
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    if (c < nchunk) {
      Raw wv = IO::load(w + c * 8);
      Raw bv;
      if (HAS_BIAS) bv = IO::load(bias + c * 8);
      Raw out;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float o = (v[j][e] - mean) * rstd * IO::get(wv, e);
        if (HAS_BIAS) o += IO::get(bv, e);
        IO::set(out, e, o);
      }
      IO::store(y + base + c * 8, out);
    }
  }
}

// Backward.  grid.x blocks, each handling a contiguous slab of rows (4 waves, wave-strided).
// COLS: also accumulate column sums of dres and of ds -- or, with a dropped branch, of the
// branch gradient (the bias grads of the projections that feed / consume this residual
// point: GPT-2's FFN-out and attn-out biases, the reference block's out_proj / linear2)
template <typename T, int MAXJ, bool RMS, bool HAS_DRES, bool HAS_BIAS, bool BRANCH_GRAD, bool COLS>
__global__ void __launch_bounds__(256) norm_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ s, const T* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, const T* __restrict__ dres,
    T* __restrict__ ds_out, T* __restrict__ dbranch, float* __restrict__ dw, float* __restrict__ dbias,
    float* __restrict__ cs_res, float* __restrict__ cs_ds, int rows, int D, int rows_per_block, float p_drop,
    uint64_t seed, float* __restrict__ part) {
  using IO = IO8<T>;
  using Raw = typename IO::Raw;
  if (p_drop > 0.f) seed = step_seed(seed);
  __shared__ float red[4][2][MAXJ * 64 * 8 > 1024 ? 1024 : MAXJ * 64 * 8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nchunk = D >> 3;
  float acc_w[MAXJ][8], acc_b[MAXJ][8];
  float acc_r[COLS ? MAXJ : 1][8], acc_s[COLS ? MAXJ : 1][8];
  float wreg[MAXJ][8];
  if constexpr (COLS) {
#pragma unroll
    for (int j = 0; j < MAXJ; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc_r[j][e] = acc_s[j][e] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      acc_w[j][e] = 0.f;
      acc_b[j][e] = 0.f;
      wreg[j][e] = 0.f;
    }
    if (c < nchunk) {
      Raw wvv = IO::load(w + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) wreg[j][e] = IO::get(wvv, e);
    }
  }
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  // software pipeline over this wave's rows: row i+1's dy / s / dres loads are in flight
  // while row i is reduced and written (one row at a time exposed the load latency)
  Raw pdv[MAXJ], psv[MAXJ], prv[HAS_DRES ? MAXJ : 1];
  auto fetch = [&](int row) {
    const size_t b = (size_t)row * D;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nchunk) {
        pdv[j] = IO::load(dy + b + c * 8);
        psv[j] = IO::load(s + b + c * 8);
        if constexpr (HAS_DRES) prv[j] = IO::load(dres + b + c * 8);
      }
    }
  };
  if (r0 + wv < r1) fetch(r0 + wv);
  for (int row = r0 + wv; row < r1; row += 4) {
    const size_t base = (size_t)row * D;
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    Raw cdv[MAXJ], csv[MAXJ], crv[HAS_DRES ? MAXJ : 1];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      cdv[j] = pdv[j];
      csv[j] = psv[j];
      if constexpr (HAS_DRES) crv[j] = prv[j];
    }
    if (row + 4 < r1) fetch(row + 4);
    float xh[MAXJ][8], g[MAXJ][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nchunk) {
        Raw dv = cdv[j];
        Raw sv = csv[j];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float d = IO::get(dv, e);
          float x = (IO::get(sv, e) - mean) * rstd;
          xh[j][e] = x;
          float gg = d * wreg[j][e];
          g[j][e] = gg;
          s1 += gg;
          s2 += gg * x;
          acc_w[j][e] += d * x;
          if (HAS_BIAS) acc_b[j][e] += d;
        }
      }
    }
    s1 = RMS ? 0.f : wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nchunk) {
        Raw rv;
        if constexpr (HAS_DRES) rv = crv[j];
        Raw out, bout;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = rstd * (g[j][e] - s1 - xh[j][e] * s2);
          if (HAS_DRES) v += IO::get(rv, e);
          IO::set(out, e, v);
          if (BRANCH_GRAD) IO::set(bout, e, v * dropout_scale(seed, base + c * 8 + e, p_drop));
          if constexpr (COLS) {
            if constexpr (HAS_DRES) acc_r[j][e] += IO::get(rv, e);
            // with a dropped branch: the branch gradient's column sums (its projection's bias grad)
            acc_s[j][e] += BRANCH_GRAD ? IO::get(bout, e) : IO::get(out, e);
          }
        }
        IO::store(ds_out + base + c * 8, out);
        if (BRANCH_GRAD) IO::store(dbranch + base + c * 8, bout);
      }
    }
  }
  // reduce per-column partials over the 4 waves, then one atomic per column
  constexpr int CAP = MAXJ * 64 * 8 > 1024 ? 1024 : MAXJ * 64 * 8;
#pragma unroll
  for (int q = 0; q < (COLS ? 2 : 1); ++q) {
    float (*x0)[8] = q == 0 ? acc_w : acc_r;
    float (*x1)[8] = q == 0 ? acc_b : acc_s;
    float* o0 = q == 0 ? dw : cs_res;
    float* o1 = q == 0 ? (HAS_BIAS ? dbias : nullptr) : cs_ds;
#pragma unroll
    for (int j0 = 0; j0 < MAXJ; j0 += CAP / 512) {
      __syncthreads();
#pragma unroll
      for (int jj = 0; jj < CAP / 512; ++jj) {
        const int j = j0 + jj;
        if (j < MAXJ) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            red[wv][0][(jj * 64 + lane) * 8 + e] = x0[j][e];
            red[wv][1][(jj * 64 + lane) * 8 + e] = x1[j][e];
          }
        }
      }
      __syncthreads();
      for (int i = threadIdx.x; i < CAP; i += 256) {
        const int jj = i / 512, rem = i % 512, ln = rem / 8, e = rem % 8;
        const int j = j0 + jj;
        const int c = ln + 64 * j;
        if (j < MAXJ && c < nchunk) {
          const float v0 = red[0][0][i] + red[1][0][i] + red[2][0][i] + red[3][0][i];
          const float v1 = red[0][1][i] + red[1][1][i] + red[2][1][i] + red[3][1][i];
          if (part != nullptr) {
            // per-block partials [block][slot][D] (slots dw, dbias, cs_res, cs_ds), summed by
            // colpart_reduce_kernel: every block atomically adding into the same few KB
            // serialises at the memory side (the COLS build ran 3x the plain one)
            float* pb = part + (int64_t)blockIdx.x * 4 * D;
            if (o0 != nullptr) pb[(2 * q) * D + c * 8 + e] = v0;
            if (o1 != nullptr) pb[(2 * q + 1) * D + c * 8 + e] = v1;
          } else {
            if (o0 != nullptr) atomicAdd(o0 + c * 8 + e, v0);
            if (o1 != nullptr) atomicAdd(o1 + c * 8 + e, v1);
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ launchers
template <typename T, bool RMS, bool HAS_B, bool HAS_BIAS>
static void launch_fwd(int maxj, const void* a, const void* b, const void* w, const void* bias, void* s_out, void* y,
                       float* mean, float* rstd, int rows, int D, float eps, float p, uint64_t seed, hipStream_t st) {
  dim3 grid((rows + 3) / 4), block(256);
#define MP_FWD(J)                                                                                                  \
  case J:                                                                                                          \
    norm_fwd_kernel<T, J, RMS, HAS_B, HAS_BIAS><<<grid, block, 0, st>>>(                                          \
        (const T*)a, (const T*)b, (const T*)w, (const T*)bias, (T*)s_out, (T*)y, mean, rstd, rows, D, eps, p, seed); \
    break;
  switch (maxj) { MP_FWD(1) MP_FWD(2) MP_FWD(4) MP_FWD(8) MP_FWD(10) MP_FWD(16) }
#undef MP_FWD
}

static int pick_j(int D) {
  int n = (D / 8 + 63) / 64;
  if (n <= 1) return 1;
  if (n <= 2) return 2;
  if (n <= 4) return 4;
  if (n <= 8) return 8;
  if (n <= 10) return 10;
  return 16;
}

template <typename T>
static int norm_fwd_t(int rms, const void* a, const void* b, const void* w, const void* bias, void* s_out, void* y,
                      float* mean, float* rstd, int rows, int D, float eps, float p, uint64_t seed, hipStream_t st) {
  if (D % 8 != 0 || D > 16 * 512) return -1;
  const int J = pick_j(D);
  const bool hb = b != nullptr, hbias = bias != nullptr;
  if (rms) {
    if (hb) hbias ? launch_fwd<T, true, true, true>(J, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st)
            : launch_fwd<T, true, true, false>(J, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st);
    else hbias ? launch_fwd<T, true, false, true>(J, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st)
               : launch_fwd<T, true, false, false>(J, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st);
  } else {
    if (hb) hbias ? launch_fwd<T, false, true, true>(J, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st)
            : launch_fwd<T, false, true, false>(J, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st);
    else hbias ? launch_fwd<T, false, false, true>(J, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st)
               : launch_fwd<T, false, false, false>(J, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st);
  }
  return (int)hipGetLastError();
}

// f32 != 0: every tensor but mean / rstd in f32 (the reference-precision path), else bf16
extern "C" int mp_norm_fwd(int f32, int rms, const void* a, const void* b, const void* w, const void* bias,
                           void* s_out, void* y, float* mean, float* rstd, int rows, int D, float eps, float p,
                           uint64_t seed, hipStream_t st) {
  if (f32) return norm_fwd_t<float>(rms, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st);
  return norm_fwd_t<bf16_t>(rms, a, b, w, bias, s_out, y, mean, rstd, rows, D, eps, p, seed, st);
}

extern "C" int mp_colpart_reduce(const float* part, int nblk, int nslot, int D, float* o0, float* o1, float* o2,
                                 float* o3, hipStream_t st);

static int norm_bwd_blocks(int rows) {
  // rows per workgroup: every workgroup ends with one f32 sum per column and output
  // (dw, dbias, column sums), so short problems want few, long workgroups (1024 rows: 512
  // workgroups of 2 rows measured 20-22 us)
  static const int min_rpb = [] {
    const char* e = getenv("MIPIPE_NORM_BWD_RPB");
    const int v = e ? atoi(e) : 8;
    return v > 0 ? v : 8;
  }();
  // workgroup cap (MIPIPE_NORM_BWD_BLOCKS, A/B): 512 = 2 per CU, one row in flight per wave
  static const int max_blk = [] {
    const char* e = getenv("MIPIPE_NORM_BWD_BLOCKS");
    const int v = e ? atoi(e) : 512;
    return v > 0 ? v : 512;
  }();
  int nblk = rows < max_blk ? (rows + 3) / 4 : max_blk;
  if ((rows + nblk - 1) / nblk < min_rpb) nblk = (rows + min_rpb - 1) / min_rpb;
  return nblk < 1 ? 1 : nblk;
}

// f32 elements of the partial-sum buffer the backward of [rows, D] uses (0: atomics only)
extern "C" int mp_colpart_enabled();

extern "C" int64_t mp_norm_bwd_part_elems(int rows, int D) {
  if (!mp_colpart_enabled()) return 0;
  const int nblk = norm_bwd_blocks(rows);
  const int rpb = (rows + nblk - 1) / nblk;
  const int g = (rows + rpb - 1) / rpb;
  return g >= 256 ? (int64_t)g * 4 * D : 0;  // as kColpartMinBlocks (elementwise.hip)
}

template <typename T, bool RMS, bool HAS_DRES, bool HAS_BIAS, bool BG, bool COLS>
static void launch_bwd(int maxj, const void* dy, const void* s, const void* w, const float* mean, const float* rstd,
                       const void* dres, void* ds, void* dbr, float* dw, float* db, float* csr, float* css, int rows,
                       int D, float p, uint64_t seed, float* part, hipStream_t st) {
  const int nblk = norm_bwd_blocks(rows);
  const int rpb = (rows + nblk - 1) / nblk;
  dim3 grid((rows + rpb - 1) / rpb), block(256);
  if (grid.x < 256) part = nullptr;
#define MP_BWD(J)                                                                                                   \
  case J:                                                                                                           \
    norm_bwd_kernel<T, J, RMS, HAS_DRES, HAS_BIAS, BG, COLS><<<grid, block, 0, st>>>(                               \
        (const T*)dy, (const T*)s, (const T*)w, mean, rstd, (const T*)dres, (T*)ds, (T*)dbr, dw, db, csr, css, rows, \
        D, rpb, p, seed, part);                                                                                     \
    break;
  switch (maxj) { MP_BWD(1) MP_BWD(2) MP_BWD(4) MP_BWD(8) MP_BWD(10) MP_BWD(16) }
#undef MP_BWD
  if (part != nullptr) mp_colpart_reduce(part, grid.x, 4, D, dw, db, csr, css, st);
}

template <typename T>
static int norm_bwd_t(int rms, const void* dy, const void* s, const void* w, const float* mean,
                           const float* rstd, const void* dres, void* ds, void* dbranch, float* dw, float* dbias,
                           float* cs_res, float* cs_ds, int rows, int D, float p, uint64_t seed, float* part,
                           hipStream_t st) {
  if (D % 8 != 0 || D > 16 * 512) return -1;
  const int J = pick_j(D);
  const bool hd = dres != nullptr, hb = dbias != nullptr, bg = dbranch != nullptr;
  if (cs_res != nullptr || cs_ds != nullptr) {
    // column sums of dres and of ds / the branch gradient (bias grads of the adjacent
    // projections), LayerNorm rows of up to 2048
    if (rms || J > 4 || (cs_res != nullptr && !hd)) return -3;
#define MP_C(HD, HB, BG_)                                                                                        \
    if (hd == HD && hb == HB && bg == BG_) {                                                                       \
      launch_bwd<T, false, HD, HB, BG_, true>(J, dy, s, w, mean, rstd, dres, ds, dbranch, dw, dbias, cs_res, cs_ds,   \
                                           rows, D, p, seed, part, st);                                            \
      return (int)hipGetLastError();                                                                               \
    }
    MP_C(1, 1, 0) MP_C(1, 0, 0) MP_C(0, 1, 1) MP_C(0, 0, 1) MP_C(1, 1, 1) MP_C(1, 0, 1) MP_C(0, 1, 0) MP_C(0, 0, 0)
#undef MP_C
    return -2;
  }
#define MP_B(R, HD, HB, BG_)                                                                                   \
  if (rms == R && hd == HD && hb == HB && bg == BG_) {                                                          \
    launch_bwd<T, R, HD, HB, BG_, false>(J, dy, s, w, mean, rstd, dres, ds, dbranch, dw, dbias, nullptr, nullptr, \
                                      rows, D, p, seed, part, st);                                             \
    return (int)hipGetLastError();                                                                            \
  }
  MP_B(0, 0, 0, 0) MP_B(0, 0, 0, 1) MP_B(0, 0, 1, 0) MP_B(0, 0, 1, 1)
  MP_B(0, 1, 0, 0) MP_B(0, 1, 0, 1) MP_B(0, 1, 1, 0) MP_B(0, 1, 1, 1)
  MP_B(1, 0, 0, 0) MP_B(1, 0, 0, 1) MP_B(1, 1, 0, 0) MP_B(1, 1, 0, 1)
#undef MP_B
  return -2;
}

extern "C" int mp_norm_bwd(int f32, int rms, const void* dy, const void* s, const void* w, const float* mean,
                           const float* rstd, const void* dres, void* ds, void* dbranch, float* dw, float* dbias,
                           float* cs_res, float* cs_ds, int rows, int D, float p, uint64_t seed, float* part,
                           hipStream_t st) {
  if (f32)
    return norm_bwd_t<float>(rms, dy, s, w, mean, rstd, dres, ds, dbranch, dw, dbias, cs_res, cs_ds, rows, D, p, seed,
                             part, st);
  return norm_bwd_t<bf16_t>(rms, dy, s, w, mean, rstd, dres, ds, dbranch, dw, dbias, cs_res, cs_ds, rows, D, p, seed,
                            part, st);
}

MP_DROP_STEP_SETTER(mp_set_drop_step_norm)
