// Python bindings of the mipipe HIP kernels (torch tensors in, launches on the current
// HIP stream).  Kernels live in csrc/kernels/*.hip behind plain C launchers so only
// this file pays for the torch headers.  No hipify: written against HIP directly.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

extern "C" {
int mp_norm_fwd(int f32, int rms, const void* a, const void* b, const void* w, const void* bias, void* s_out, void* y,
                float* mean, float* rstd, int rows, int D, float eps, float p, uint64_t seed, hipStream_t st);
int mp_norm_bwd(int f32, int rms, const void* dy, const void* s, const void* w, const float* mean, const float* rstd,
                const void* dres, void* ds, void* dbranch, float* dw, float* dbias, float* cs_res, float* cs_ds,
                int rows, int D, float p, uint64_t seed, float* part, hipStream_t st);
int64_t mp_norm_bwd_part_elems(int rows, int D);
int64_t mp_colsum_part_elems(int rows, int cols);
int mp_xent_fwd_bwd(void* logits, const int64_t* target, float* loss, int T, int V, int Vp, float grad_scale,
                    int64_t ignore_index, int write_grad, int f32, hipStream_t st);
int mp_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int T, int S, int D, int pos_offset,
                 int f32, hipStream_t st);
int mp_embed_bwd(const int64_t* idx, const void* dout, float* dwte, float* dwpe, int T, int S, int D, int pos_offset,
                 int f32, hipStream_t st);
int mp_sumsq(const float* g, int64_t n, float* out, hipStream_t st);
int mp_scaled_sum(const float* x, int64_t n, float scale, float* out, hipStream_t st);
int mp_gemm_f32(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int64_t lda,
                int a_kc, int64_t ldb, int b_nc, int64_t ldc, float alpha, int accumulate, hipStream_t st);
int mp_gemm_f32_ex(const float* A, const float* B, float* C, const float* bias, const float* R, float* X, int M, int N,
                   int K, int64_t lda, int a_kc, int64_t ldb, int b_kc, int64_t ldc, int64_t ldr, int64_t ldx, int epi,
                   float alpha, int accumulate, float p_drop, uint64_t seed, int force_split, float* ws,
                   hipStream_t st);
int64_t mp_gemm_f32_ws_elems(int M, int N, int K, int force_split);
int mp_lane_merge(float* g0, float* g1, float* g2, float* g3, int64_t n, float* sumsq, hipStream_t st);
int mp_adamw(float* p, float* g, float* m, float* v, void* w16, int64_t n, int64_t n_decay, float lr, float b1,
             float b2, float eps, float wd, int step, const float* sumsq, float max_norm, float grad_scale,
             int zero_grad, hipStream_t st);
int mp_cast_f32_bf16(const float* src, void* dst, int64_t n, hipStream_t st);
int mp_act_fwd(const void* a, void* g, int64_t n, int act, float p, uint64_t seed, hipStream_t st);
int mp_act_bwd(const void* dg, const void* a, void* da, float* dbias, int rows, int cols, int act, float p,
               uint64_t seed, float* part, hipStream_t st);
int mp_colsum(const void* x, float* dbias, int rows, int cols, float* part, int f32, hipStream_t st);
int mp_swiglu_fwd(const void* gu, void* y, int T, int F, hipStream_t st);
int mp_swiglu_bwd(const void* gu, const void* dy, void* dgu, int T, int F, hipStream_t st);
int mp_rope(void* qkv, const float* cs, const float* sn, int T, int S, int H, int Hkv, int Dh, int pos_offset,
            int inverse, hipStream_t st);
int mp_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq, int Sk, int H,
                int Hkv, int D, int64_t q_stride, int64_t k_stride, int64_t v_stride, int64_t o_stride, int causal,
                float scale, float p_drop, uint64_t seed, hipStream_t st);
int mp_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                float* delta, void* dq, void* dk, void* dv, int B, int Sq, int Sk, int H, int Hkv, int D,
                int64_t q_stride, int64_t k_stride, int64_t v_stride, int64_t o_stride, int64_t dq_stride,
                int64_t dk_stride, int64_t dv_stride, int causal, float scale, float p_drop, uint64_t seed,
                float* csq, float* csk, float* csv, hipStream_t st);
int mp_attn_f32_fwd(const float* q, const float* k, const float* v, float* o, float* lse, int B, int Sq, int Sk, int H,
                    int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, int causal, float scale,
                    float p_drop, uint64_t seed, hipStream_t st);
int mp_attn_f32_bwd(const float* q, const float* k, const float* v, const float* o, const float* dout,
                    const float* lse, float* delta, float* dq, float* dk, float* dv, int B, int Sq, int Sk, int H,
                    int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dqs, int64_t dks,
                    int64_t dvs, int causal, float scale, float p_drop, uint64_t seed, hipStream_t st);
int mp_set_drop_step_attn_f32(uint64_t v, hipStream_t st);
int mp_set_drop_step_gemm_f32(uint64_t v, hipStream_t st);
int mp_gemm_f32_set_lanes(int lanes);
int mp_transpose(const void* in, void* out, int R, int C, int64_t ldi, int64_t ldo, hipStream_t st);
int mp_transpose_batched(const void* src, void* dst, const int64_t* desc, const int* tile0, int n, int total_tiles,
                         hipStream_t st);
int mp_set_drop_step_attn(uint64_t v, hipStream_t st);
int mp_set_drop_step_elem(uint64_t v, hipStream_t st);
int mp_set_drop_step_norm(uint64_t v, hipStream_t st);
int mp_set_drop_step_gemm(uint64_t v, hipStream_t st);
int mp_gemm2(const void* A, const void* B, void* C, const void* bias, const void* residual, void* aux, int M, int N,
             int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ld_res, int64_t ld_aux, int transA, int transB,
             int epilogue, int c_f32_accum, float alpha, int force_cfg, float* ws, float* colsum, float p_drop,
             uint64_t seed, hipStream_t st);
int mp_gemm2_plan(int M, int N, int K, int transA, int transB, int c_f32_accum, int force_cfg, int* split_out);
int64_t mp_gemm2_ws_floats(int cfg, int split, int M, int N, int K);
int mp_gemm2_has_probe_engines();
int mp_gemm_tt_grouped(int n, const void* const* A, const void* const* B, float* const* C, const int* M, const int* N,
                       const int* K, const int64_t* lda, const int64_t* ldb, const int64_t* ldc, float alpha,
                       hipStream_t st);
int mp_probe_spin(unsigned* flag, unsigned expect, int64_t timeout_us, unsigned* result, hipStream_t waiter);
int mp_probe_set(unsigned* flag, unsigned value, hipStream_t setter);
int mp_probe_clock_khz();
int mp_gemm(const void* A, const void* B, void* C, const void* bias, const void* residual, void* aux, int M, int N,
            int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ld_res, int64_t ld_aux, int transA, int transB,
            int epilogue, int c_f32_accum, float alpha, hipStream_t st);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* what) { TORCH_CHECK(rc == 0, "mipipe kernel ", what, " failed with code ", rc); }

const void* ptr_or_null(const c10::optional<torch::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// storage dtype of the normalisation / loss / embedding kernels: bf16, or f32 (the
// reference-precision path); returns 1 for f32
int storage(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32, name,
              " must be bf16 or f32, got ", t.scalar_type());
  return t.scalar_type() == torch::kFloat32 ? 1 : 0;
}
void* mptr_or_null(const c10::optional<torch::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

void req(const torch::Tensor& t, torch::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be on the GPU");
  TORCH_CHECK(t.scalar_type() == dt, name, " has wrong dtype ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void norm_fwd(bool rms, torch::Tensor a, c10::optional<torch::Tensor> b, torch::Tensor w,
              c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> s_out, torch::Tensor y,
              c10::optional<torch::Tensor> mean, torch::Tensor rstd, double eps, double p, int64_t seed) {
  const int f32 = storage(a, "a");
  const auto dt = a.scalar_type();
  req(a, dt, "a");
  req(y, dt, "y");
  req(w, dt, "w");
  if (b.has_value()) req(*b, dt, "b");
  if (bias.has_value()) req(*bias, dt, "bias");
  if (s_out.has_value()) req(*s_out, dt, "s_out");
  req(rstd, torch::kFloat32, "rstd");
  const int D = a.size(-1);
  const int rows = a.numel() / D;
  TORCH_CHECK(!b.has_value() || (s_out.has_value() && b->numel() == a.numel()), "b needs s_out");
  TORCH_CHECK(rms || mean.has_value(), "LayerNorm needs mean");
  TORCH_CHECK(rstd.numel() >= rows && w.numel() == D, "bad norm shapes");
  check(mp_norm_fwd(f32, rms, a.data_ptr(), ptr_or_null(b), w.data_ptr(), ptr_or_null(bias), mptr_or_null(s_out),
                    y.data_ptr(), mean.has_value() ? mean->data_ptr<float>() : nullptr, rstd.data_ptr<float>(), rows,
                    D, (float)eps, (float)p, (uint64_t)seed, cur_stream()),
        "norm_fwd");
}

// returns 0, or -3 when the requested fused column sums are not available for this shape
// (the caller then sums separately); other failures raise
int64_t norm_bwd(bool rms, torch::Tensor dy, torch::Tensor s, torch::Tensor w, c10::optional<torch::Tensor> mean,
              torch::Tensor rstd, c10::optional<torch::Tensor> dres, torch::Tensor ds,
              c10::optional<torch::Tensor> dbranch, torch::Tensor dw, c10::optional<torch::Tensor> dbias, double p,
              int64_t seed, c10::optional<torch::Tensor> cs_res, c10::optional<torch::Tensor> cs_ds) {
  const int f32 = storage(dy, "dy");
  const auto dt = dy.scalar_type();
  req(dy, dt, "dy");
  req(s, dt, "s");
  req(ds, dt, "ds");
  req(w, dt, "w");
  if (dres.has_value()) req(*dres, dt, "dres");
  if (dbranch.has_value()) req(*dbranch, dt, "dbranch");
  req(dw, torch::kFloat32, "dw");
  const int D = dy.size(-1);
  const int rows = dy.numel() / D;
  TORCH_CHECK(s.numel() == dy.numel() && ds.numel() == dy.numel() && dw.numel() == D, "bad norm_bwd shapes");
  // per-block partial column sums (two-stage reduction instead of contended atomics)
  const int64_t pe = mp_norm_bwd_part_elems(rows, D);
  torch::Tensor part;
  if (pe > 0) part = torch::empty({pe}, dy.options().dtype(torch::kFloat32));
  const int rc = mp_norm_bwd(f32, rms, dy.data_ptr(), s.data_ptr(), w.data_ptr(),
                             mean.has_value() ? mean->data_ptr<float>() : nullptr, rstd.data_ptr<float>(),
                             ptr_or_null(dres), ds.data_ptr(), mptr_or_null(dbranch), dw.data_ptr<float>(),
                             dbias.has_value() ? dbias->data_ptr<float>() : nullptr,
                             cs_res.has_value() ? cs_res->data_ptr<float>() : nullptr,
                             cs_ds.has_value() ? cs_ds->data_ptr<float>() : nullptr, rows, D, (float)p,
                             (uint64_t)seed, part.defined() ? part.data_ptr<float>() : nullptr, cur_stream());
  if (rc == -3) return -3;
  check(rc, "norm_bwd");
  return 0;
}

void xent(torch::Tensor logits, torch::Tensor target, torch::Tensor loss, int64_t V, double grad_scale,
          int64_t ignore_index, bool write_grad) {
  const int f32 = storage(logits, "logits");
  req(logits, logits.scalar_type(), "logits");
  req(target, torch::kInt64, "target");
  req(loss, torch::kFloat32, "loss");
  const int Vp = logits.size(-1);
  const int T = logits.numel() / Vp;
  TORCH_CHECK(target.numel() == T && loss.numel() == T, "bad xent shapes");
  check(mp_xent_fwd_bwd(logits.data_ptr(), target.data_ptr<int64_t>(), loss.data_ptr<float>(), T, V, Vp,
                        (float)grad_scale, ignore_index, write_grad, f32, cur_stream()),
        "xent");
}

void embed_fwd(torch::Tensor idx, torch::Tensor wte, c10::optional<torch::Tensor> wpe, torch::Tensor out, int64_t S,
               int64_t pos_offset) {
  req(idx, torch::kInt64, "idx");
  const int f32 = storage(out, "out");
  req(out, out.scalar_type(), "out");
  req(wte, out.scalar_type(), "wte");
  if (wpe.has_value()) req(*wpe, out.scalar_type(), "wpe");
  const int D = wte.size(1);
  const int T = idx.numel();
  TORCH_CHECK(out.numel() == (int64_t)T * D, "bad embed shapes");
  check(mp_embed_fwd(idx.data_ptr<int64_t>(), wte.data_ptr(), ptr_or_null(wpe), out.data_ptr(), T, S, D, pos_offset,
                     f32, cur_stream()),
        "embed_fwd");
}

void embed_bwd(torch::Tensor idx, torch::Tensor dout, torch::Tensor dwte, c10::optional<torch::Tensor> dwpe,
               int64_t S, int64_t pos_offset) {
  req(idx, torch::kInt64, "idx");
  req(dwte, torch::kFloat32, "dwte");
  const int f32 = storage(dout, "dout");
  req(dout, dout.scalar_type(), "dout");
  const int D = dwte.size(-1);
  const int T = idx.numel();
  TORCH_CHECK(dout.numel() == (int64_t)T * D, "bad embed_bwd shapes");
  check(mp_embed_bwd(idx.data_ptr<int64_t>(), dout.data_ptr(), dwte.data_ptr<float>(),
                     dwpe.has_value() ? dwpe->data_ptr<float>() : nullptr, T, S, D, pos_offset, f32, cur_stream()),
        "embed_bwd");
}

// g0 += sum(lanes); lanes zeroed (1..3 extra f32 lane buffers of g0's size); with
// `sumsq` (f32 [1]) also *sumsq += |merged g0|^2 in the same pass
void lane_merge(torch::Tensor g0, std::vector<torch::Tensor> lanes, c10::optional<torch::Tensor> sumsq) {
  TORCH_CHECK(lanes.size() >= 1 && lanes.size() <= 3, "lane_merge: 1..3 lane buffers");
  req(g0, torch::kFloat32, "g0");
  float* p[3] = {nullptr, nullptr, nullptr};
  for (size_t i = 0; i < lanes.size(); ++i) {
    req(lanes[i], torch::kFloat32, "lane");
    TORCH_CHECK(lanes[i].numel() == g0.numel(), "lane_merge: size mismatch");
    p[i] = lanes[i].data_ptr<float>();
  }
  if (sumsq.has_value()) req(*sumsq, torch::kFloat32, "sumsq");
  check(mp_lane_merge(g0.data_ptr<float>(), p[0], p[1], p[2], g0.numel(),
                      sumsq.has_value() ? sumsq->data_ptr<float>() : nullptr, cur_stream()),
        "lane_merge");
}

void sumsq(torch::Tensor g, torch::Tensor out) {
  req(g, torch::kFloat32, "g");
  check(mp_sumsq(g.data_ptr<float>(), g.numel(), out.data_ptr<float>(), cur_stream()), "sumsq");
}

// contiguous tensor <- 0 with hipMemsetAsync on the current stream (graph-capturable)
void zero_(torch::Tensor t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "zero_: contiguous GPU tensor");
  TORCH_CHECK(hipMemsetAsync(t.data_ptr(), 0, t.numel() * t.element_size(), cur_stream()) == hipSuccess, "zero_");
}

// out (f32 scalar) = scale * sum(x): one workgroup, deterministic
void scaled_sum(torch::Tensor x, double scale, torch::Tensor out) {
  req(x, torch::kFloat32, "x");
  req(out, torch::kFloat32, "out");
  check(mp_scaled_sum(x.data_ptr<float>(), x.numel(), (float)scale, out.data_ptr<float>(), cur_stream()),
        "scaled_sum");
}

void adamw(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> w16,
           int64_t n_decay, double lr, double b1, double b2, double eps, double wd, int64_t step,
           c10::optional<torch::Tensor> sumsq_buf, double max_norm, double grad_scale, bool zero_grad) {
  req(p, torch::kFloat32, "p");
  req(g, torch::kFloat32, "g");
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel(), "bad adamw shapes");
  check(mp_adamw(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), mptr_or_null(w16),
                 p.numel(), n_decay, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step,
                 sumsq_buf.has_value() ? sumsq_buf->data_ptr<float>() : nullptr, (float)max_norm, (float)grad_scale,
                 zero_grad, cur_stream()),
        "adamw");
}

void cast_f32_bf16(torch::Tensor src, torch::Tensor dst) {
  req(src, torch::kFloat32, "src");
  check(mp_cast_f32_bf16(src.data_ptr<float>(), dst.data_ptr(), src.numel(), cur_stream()), "cast");
}

void act_fwd(torch::Tensor a, torch::Tensor g, int64_t act, double p, int64_t seed) {
  req(a, torch::kBFloat16, "a");
  check(mp_act_fwd(a.data_ptr(), g.data_ptr(), a.numel(), act, (float)p, (uint64_t)seed, cur_stream()), "act_fwd");
}

void act_bwd(torch::Tensor dg, torch::Tensor a, torch::Tensor da, c10::optional<torch::Tensor> dbias, int64_t act,
             double p, int64_t seed) {
  req(dg, torch::kBFloat16, "dg");
  const int cols = dg.size(-1);
  const int rows = dg.numel() / cols;
  const int64_t pe = dbias.has_value() ? mp_colsum_part_elems(rows, cols) : 0;
  torch::Tensor part;
  if (pe > 0) part = torch::empty({pe}, dg.options().dtype(torch::kFloat32));
  check(mp_act_bwd(dg.data_ptr(), a.data_ptr(), da.data_ptr(), dbias.has_value() ? dbias->data_ptr<float>() : nullptr,
                   rows, cols, act, (float)p, (uint64_t)seed, part.defined() ? part.data_ptr<float>() : nullptr,
                   cur_stream()),
        "act_bwd");
}

void colsum(torch::Tensor x, torch::Tensor dbias) {
  const int f32 = storage(x, "x");
  req(x, x.scalar_type(), "x");
  req(dbias, torch::kFloat32, "dbias");
  const int cols = x.size(-1);
  const int rows = x.numel() / cols;
  const int64_t pe = mp_colsum_part_elems(rows, cols);
  torch::Tensor part;
  if (pe > 0) part = torch::empty({pe}, x.options().dtype(torch::kFloat32));
  check(mp_colsum(x.data_ptr(), dbias.data_ptr<float>(), rows, cols, part.defined() ? part.data_ptr<float>() : nullptr,
                  f32, cur_stream()),
        "colsum");
}

void swiglu_fwd(torch::Tensor gu, torch::Tensor y) {
  const int F = y.size(-1);
  check(mp_swiglu_fwd(gu.data_ptr(), y.data_ptr(), y.numel() / F, F, cur_stream()), "swiglu_fwd");
}

void swiglu_bwd(torch::Tensor gu, torch::Tensor dy, torch::Tensor dgu) {
  const int F = dy.size(-1);
  check(mp_swiglu_bwd(gu.data_ptr(), dy.data_ptr(), dgu.data_ptr(), dy.numel() / F, F, cur_stream()), "swiglu_bwd");
}

void rope(torch::Tensor qkv, torch::Tensor cs, torch::Tensor sn, int64_t S, int64_t H, int64_t Hkv, int64_t Dh,
          int64_t pos_offset, bool inverse) {
  const int T = qkv.numel() / ((H + 2 * Hkv) * Dh);
  check(mp_rope(qkv.data_ptr(), cs.data_ptr<float>(), sn.data_ptr<float>(), T, S, H, Hkv, Dh, pos_offset, inverse,
                cur_stream()),
        "rope");
}

// q/k/v/o are [B*S, stride] row views (token-major), heads at h*D inside a row.
void attn_fwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, torch::Tensor o, torch::Tensor lse, int64_t B,
              int64_t Sq, int64_t Sk, int64_t H, int64_t Hkv, int64_t D, bool causal, double scale, double p,
              int64_t seed) {
  req(lse, torch::kFloat32, "lse");
  TORCH_CHECK(lse.numel() >= B * H * Sq, "lse too small");
  TORCH_CHECK(q.stride(1) == 1 && k.stride(1) == 1 && v.stride(1) == 1 && o.stride(1) == 1, "attn: token-major rows");
  if (q.scalar_type() == torch::kFloat32) {
    // f32 flash attention (attention_f32.hip): the reference-precision path
    TORCH_CHECK(k.scalar_type() == torch::kFloat32 && v.scalar_type() == torch::kFloat32 &&
                    o.scalar_type() == torch::kFloat32, "attn f32: q/k/v/o all f32");
    check(mp_attn_f32_fwd(q.data_ptr<float>(), k.data_ptr<float>(), v.data_ptr<float>(), o.data_ptr<float>(),
                          lse.data_ptr<float>(), B, Sq, Sk, H, Hkv, D, q.stride(0), k.stride(0), v.stride(0),
                          o.stride(0), causal, (float)scale, (float)p, (uint64_t)seed, cur_stream()),
          "attn_f32_fwd");
    return;
  }
  TORCH_CHECK(q.scalar_type() == torch::kBFloat16 && o.scalar_type() == torch::kBFloat16, "attn: bf16 or f32");
  check(mp_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), B, Sq, Sk, H, Hkv,
                    D, q.stride(0), k.stride(0), v.stride(0), o.stride(0), causal, (float)scale, (float)p,
                    (uint64_t)seed, cur_stream()),
        "attn_fwd");
}

void attn_bwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, torch::Tensor o, torch::Tensor dout,
              torch::Tensor lse, torch::Tensor delta, torch::Tensor dq, torch::Tensor dk, torch::Tensor dv,
              int64_t B, int64_t Sq, int64_t Sk, int64_t H, int64_t Hkv, int64_t D, bool causal,
              double scale, double p, int64_t seed, c10::optional<torch::Tensor> dbias) {
  TORCH_CHECK(o.stride(0) == dout.stride(0), "o and dout must share a row stride");
  if (q.scalar_type() == torch::kFloat32) {
    TORCH_CHECK(!dbias.has_value(), "attn_bwd f32: no fused bias sums");
    for (const torch::Tensor* t : {&k, &v, &o, &dout, &dq, &dk, &dv})
      TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->stride(1) == 1, "attn_bwd f32: f32 token-major rows");
    check(mp_attn_f32_bwd(q.data_ptr<float>(), k.data_ptr<float>(), v.data_ptr<float>(), o.data_ptr<float>(),
                          dout.data_ptr<float>(), lse.data_ptr<float>(), delta.data_ptr<float>(), dq.data_ptr<float>(),
                          dk.data_ptr<float>(), dv.data_ptr<float>(), B, Sq, Sk, H, Hkv, D, q.stride(0), k.stride(0),
                          v.stride(0), o.stride(0), dq.stride(0), dk.stride(0), dv.stride(0), causal, (float)scale,
                          (float)p, (uint64_t)seed, cur_stream()),
          "attn_f32_bwd");
    return;
  }
  // dbias: f32 [(H + 2 Hkv) D] QKV bias gradient, accumulated by the kernels (q | k | v)
  float* cs = nullptr;
  if (dbias.has_value()) {
    TORCH_CHECK(dbias->scalar_type() == torch::kFloat32 && dbias->is_contiguous() &&
                    dbias->numel() == (H + 2 * Hkv) * D,
                "attn_bwd: dbias must be a contiguous f32 [(H + 2 Hkv) D] tensor");
    cs = dbias->data_ptr<float>();
  }
  check(mp_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                    delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), B,
                    Sq, Sk, H, Hkv, D, q.stride(0), k.stride(0), v.stride(0), o.stride(0), dq.stride(0), dk.stride(0),
                    dv.stride(0), causal, (float)scale, (float)p, (uint64_t)seed, cs,
                    cs ? cs + H * D : nullptr, cs ? cs + (H + Hkv) * D : nullptr, cur_stream()),
        "attn_bwd");
}

// C[M,N] (+)= alpha * op(A) @ op(B) with fused epilogue.
//   A: [M,K] row-major (transA=0) or [K,M] (transA=1); B: [N,K] (transB=0, "NT") or [K,N] (transB=1)
void gemm(torch::Tensor A, torch::Tensor B, torch::Tensor C, c10::optional<torch::Tensor> bias,
          c10::optional<torch::Tensor> residual, c10::optional<torch::Tensor> aux, bool transA, bool transB,
          int64_t epilogue, bool accum, double alpha) {
  const int M = C.size(0), N = C.size(1);
  const int K = transA ? A.size(0) : A.size(1);
  TORCH_CHECK((transA ? A.size(1) : A.size(0)) == M, "gemm: A/M mismatch");
  TORCH_CHECK((transB ? B.size(0) : B.size(1)) == K && (transB ? B.size(1) : B.size(0)) == N, "gemm: B mismatch");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1, "gemm: inner dims must be contiguous");
  TORCH_CHECK(!accum || C.scalar_type() == torch::kFloat32, "gemm: accumulate needs f32 C");
  check(mp_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), ptr_or_null(bias), ptr_or_null(residual), mptr_or_null(aux),
                M, N, K, A.stride(0), B.stride(0), C.stride(0), residual.has_value() ? residual->stride(0) : 0,
                aux.has_value() ? aux->stride(0) : 0, transA, transB, epilogue, accum, (float)alpha, cur_stream()),
        "gemm");
}

// v2 engine (8 waves, glds staging).  Returns false if the combination is not provided
// by v2 (the caller then uses gemm()).
// returns 1 if done, 0 if the combination is not provided by v2 (caller uses gemm()),
// 2 if done WITHOUT the requested fused column sums (caller sums separately)
int64_t gemm2(torch::Tensor A, torch::Tensor B, torch::Tensor C, c10::optional<torch::Tensor> bias,
              c10::optional<torch::Tensor> residual, c10::optional<torch::Tensor> aux, bool transA, bool transB,
              int64_t epilogue, bool accum, double alpha, int64_t force_cfg, c10::optional<torch::Tensor> colsum,
              double p_drop, int64_t seed) {
  const int M = C.size(0), N = C.size(1);
  const int K = transA ? A.size(0) : A.size(1);
  TORCH_CHECK((transA ? A.size(1) : A.size(0)) == M, "gemm2: A/M mismatch");
  TORCH_CHECK((transB ? B.size(0) : B.size(1)) == K && (transB ? B.size(1) : B.size(0)) == N, "gemm2: B mismatch");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1, "gemm2: inner dims must be contiguous");
  TORCH_CHECK(!accum || C.scalar_type() == torch::kFloat32, "gemm2: accumulate needs f32 C");
  TORCH_CHECK(!colsum.has_value() || (colsum->scalar_type() == torch::kFloat32 && colsum->is_contiguous() &&
                                      colsum->numel() >= N),
              "gemm2: colsum must be a contiguous f32 [N] tensor");
  // split-K slabs (plain stores + one reduce pass instead of f32 atomics)
  // split-K slabs (plain stores + one reduce pass instead of f32 atomics), or the stream-K
  // engine's flags + partial tiles: from the caching allocator on the current stream (graph
  // captures take it from their private pool), so concurrent streams never share one
  int split = 1;
  const int cfg = mp_gemm2_plan(M, N, K, transA, transB, accum, (int)force_cfg, &split);
  torch::Tensor ws;
  const int64_t ws_n = mp_gemm2_ws_floats(cfg, split, M, N, K);
  if (ws_n > 0) ws = torch::empty({ws_n}, C.options().dtype(torch::kFloat32));
  const int rc = mp_gemm2(A.data_ptr(), B.data_ptr(), C.data_ptr(), ptr_or_null(bias), ptr_or_null(residual),
                          mptr_or_null(aux), M, N, K, A.stride(0), B.stride(0), C.stride(0),
                          residual.has_value() ? residual->stride(0) : 0, aux.has_value() ? aux->stride(0) : 0,
                          transA, transB, epilogue, accum, (float)alpha, (int)force_cfg,
                          ws.defined() ? ws.data_ptr<float>() : nullptr,
                          colsum.has_value() ? colsum->data_ptr<float>() : nullptr, (float)p_drop, (uint64_t)seed,
                          cur_stream());
  if (rc == -3) {
    const int rc2 = mp_gemm2(A.data_ptr(), B.data_ptr(), C.data_ptr(), ptr_or_null(bias), ptr_or_null(residual),
                             mptr_or_null(aux), M, N, K, A.stride(0), B.stride(0), C.stride(0),
                             residual.has_value() ? residual->stride(0) : 0, aux.has_value() ? aux->stride(0) : 0,
                             transA, transB, epilogue, accum, (float)alpha, (int)force_cfg,
                             ws.defined() ? ws.data_ptr<float>() : nullptr, nullptr, (float)p_drop, (uint64_t)seed,
                             cur_stream());
    if (rc2 == -2 || rc2 == -1) return 0;
    check(rc2, "gemm2");
    return 2;
  }
  if (rc == -2 || rc == -1) return 0;
  check(rc, "gemm2");
  return 1;
}

// grouped weight-gradient GEMMs: C[i] (f32 [N_i, K_i]) += alpha * dy[i]^T x[i]
// (dy [T_i, N_i], x [T_i, K_i] bf16, unit inner stride) in one launch of 64x64 tiles
void gemm_tt_grouped(std::vector<torch::Tensor> dy, std::vector<torch::Tensor> x, std::vector<torch::Tensor> C,
                     double alpha) {
  const int n = (int)dy.size();
  TORCH_CHECK(n == (int)x.size() && n == (int)C.size() && n >= 1 && n <= 8, "gemm_tt_grouped: 1..8 problems");
  const void* A[8];
  const void* B[8];
  float* Cp[8];
  int M[8], N[8], K[8];
  int64_t lda[8], ldb[8], ldc[8];
  for (int i = 0; i < n; ++i) {
    TORCH_CHECK(dy[i].is_cuda() && dy[i].scalar_type() == torch::kBFloat16 && x[i].scalar_type() == torch::kBFloat16 &&
                    C[i].scalar_type() == torch::kFloat32,
                "gemm_tt_grouped: bf16 dy/x, f32 C");
    TORCH_CHECK(dy[i].dim() == 2 && x[i].dim() == 2 && C[i].dim() == 2 && dy[i].stride(1) == 1 &&
                    x[i].stride(1) == 1 && C[i].stride(1) == 1,
                "gemm_tt_grouped: 2-D, unit inner stride");
    TORCH_CHECK(dy[i].size(0) == x[i].size(0) && C[i].size(0) == dy[i].size(1) && C[i].size(1) == x[i].size(1),
                "gemm_tt_grouped: shape mismatch");
    A[i] = dy[i].data_ptr();
    B[i] = x[i].data_ptr();
    Cp[i] = C[i].data_ptr<float>();
    M[i] = (int)dy[i].size(1);
    N[i] = (int)x[i].size(1);
    K[i] = (int)dy[i].size(0);
    lda[i] = dy[i].stride(0);
    ldb[i] = x[i].stride(0);
    ldc[i] = C[i].stride(0);
  }
  check(mp_gemm_tt_grouped(n, A, B, Cp, M, N, K, lda, ldb, ldc, (float)alpha, cur_stream()), "gemm_tt_grouped");
}

void transpose(torch::Tensor in, torch::Tensor out) {
  TORCH_CHECK(in.dim() == 2 && out.dim() == 2 && in.stride(1) == 1 && out.stride(1) == 1, "transpose: 2-D rows");
  TORCH_CHECK(out.size(0) == in.size(1) && out.size(1) == in.size(0), "transpose: shape");
  check(mp_transpose(in.data_ptr(), out.data_ptr(), in.size(0), in.size(1), in.stride(0), out.stride(0),
                     cur_stream()),
        "transpose");
}

// every W^T copy of an arena in one launch: desc int64 [n, 4] = (src off, dst off, R, C),
// tile0 int32 [n] = first 64x64 tile of each matrix
void transpose_batched(torch::Tensor src, torch::Tensor dst, torch::Tensor desc, torch::Tensor tile0,
                       int64_t total_tiles) {
  TORCH_CHECK(desc.scalar_type() == torch::kInt64 && tile0.scalar_type() == torch::kInt32 && desc.is_cuda() &&
                  tile0.is_cuda() && desc.size(0) == tile0.size(0),
              "transpose_batched: bad descriptors");
  check(mp_transpose_batched(src.data_ptr(), dst.data_ptr(), desc.data_ptr<int64_t>(), tile0.data_ptr<int>(),
                             (int)desc.size(0), (int)total_tiles, cur_stream()),
        "transpose_batched");
}

// A private HIP stream (not from torch's round-robin pool, whose streams other users --
// graph capture, process groups -- may also be handed).  Never destroyed: it lives as
// long as the process, like the streams it is used beside.  priority: 0 = default,
// -1 = the device's highest.
int64_t create_stream(int64_t device, int64_t priority) {
  int cur = 0;
  TORCH_CHECK(hipGetDevice(&cur) == hipSuccess, "hipGetDevice");
  TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "hipSetDevice");
  int lo = 0, hi = 0;
  TORCH_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess, "priority range");
  hipStream_t s = nullptr;
  const hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority < 0 ? hi : lo);
  hipSetDevice(cur);
  TORCH_CHECK(e == hipSuccess, "hipStreamCreateWithPriority: ", hipGetErrorString(e));
  return reinterpret_cast<int64_t>(s);
}

// training-step counter the dropout kernels mix into their seeds (mp_common.h
// step_seed): stream-ordered, issued before a step's first replay, never captured
void set_dropout_step(int64_t step) {
  const uint64_t v = (uint64_t)step;
  check(mp_set_drop_step_attn(v, cur_stream()), "set_drop_step");
  check(mp_set_drop_step_attn_f32(v, cur_stream()), "set_drop_step");
  check(mp_set_drop_step_gemm_f32(v, cur_stream()), "set_drop_step");
  check(mp_set_drop_step_elem(v, cur_stream()), "set_drop_step");
  check(mp_set_drop_step_norm(v, cur_stream()), "set_drop_step");
  check(mp_set_drop_step_gemm(v, cur_stream()), "set_drop_step");
}

// hardware-queue probe (csrc/kernels/probe.hip, parallel/queues.py): enqueue the bounded
// spinner on stream `waiter` / the flag store on stream `setter` (raw HIP stream handles;
// 0 = the current stream).  flag: int32 [1], result: int32 [2] device tensors.
void probe_spin(torch::Tensor flag, int64_t expect, int64_t timeout_us, torch::Tensor result, int64_t waiter) {
  req(flag, torch::kInt32, "flag");
  req(result, torch::kInt32, "result");
  TORCH_CHECK(result.numel() >= 2 && timeout_us > 0 && timeout_us <= 2000000, "probe_spin: result[2], timeout <= 2 s");
  hipStream_t s = waiter ? reinterpret_cast<hipStream_t>(waiter) : cur_stream();
  check(mp_probe_spin(reinterpret_cast<unsigned*>(flag.data_ptr()), (unsigned)expect, timeout_us,
                      reinterpret_cast<unsigned*>(result.data_ptr()), s),
        "probe_spin");
}

void probe_set(torch::Tensor flag, int64_t value, int64_t setter) {
  req(flag, torch::kInt32, "flag");
  hipStream_t s = setter ? reinterpret_cast<hipStream_t>(setter) : cur_stream();
  check(mp_probe_set(reinterpret_cast<unsigned*>(flag.data_ptr()), (unsigned)value, s), "probe_set");
}

}  // namespace

namespace mipipe_comm {
void register_rccl(pybind11::module& m);
}
namespace mipipe_runtime {
void register_runner(pybind11::module& m);
}

// f32 MFMA GEMM: C (+)= alpha * A @ B (+ bias); A [M,K], B [K,N] 2-D views with either inner
// stride 1; returns 1 if done, 0 if the layout is not supported (caller falls back)
int64_t gemm_f32(torch::Tensor A, torch::Tensor B, torch::Tensor C, c10::optional<torch::Tensor> bias, double alpha,
                 bool accumulate) {
  TORCH_CHECK(A.scalar_type() == torch::kFloat32 && B.scalar_type() == torch::kFloat32 &&
                  C.scalar_type() == torch::kFloat32, "gemm_f32: f32 tensors");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm_f32: 2-D");
  const int M = A.size(0), K = A.size(1), N = B.size(1);
  TORCH_CHECK(B.size(0) == K && C.size(0) == M && C.size(1) == N, "gemm_f32: shape mismatch");
  if (C.stride(1) != 1) return 0;
  int a_kc, b_nc;
  int64_t lda, ldb;
  if (A.stride(1) == 1) { a_kc = 1; lda = A.stride(0); }
  else if (A.stride(0) == 1) { a_kc = 0; lda = A.stride(1); }
  else return 0;
  if (B.stride(1) == 1) { b_nc = 1; ldb = B.stride(0); }
  else if (B.stride(0) == 1) { b_nc = 0; ldb = B.stride(1); }
  else return 0;
  if (bias.has_value()) TORCH_CHECK(bias->is_contiguous() && bias->numel() == N, "gemm_f32: bias [N]");
  const int rc = mp_gemm_f32(A.data_ptr<float>(), B.data_ptr<float>(), C.data_ptr<float>(),
                             bias.has_value() ? bias->data_ptr<float>() : nullptr, M, N, K, lda, a_kc, ldb, b_nc,
                             C.stride(0), (float)alpha, accumulate ? 1 : 0, cur_stream());
  if (rc == -1) return 0;
  check(rc, "gemm_f32");
  return 1;
}

// f32 GEMM with fused epilogues (gemm_f32.hip mp_gemm_f32_ex): C = epi(alpha * A @ B (+ C)).
// A [M,K], B [K,N] 2-D views with either inner stride 1 (a transposed view of an [N,K]
// weight is the K-contiguous B); C row-major.  epi: 0 none, 1 bias, 2 bias+ReLU(+dropout,
// pre-activation -> X), 3 residual R, 4 bias+residual, 5 dReLU(R = pre-activation) x mask.
// Returns 1 if done, 0 if the layout is not supported.
int64_t gemm_f32_ex(torch::Tensor A, torch::Tensor B, torch::Tensor C, c10::optional<torch::Tensor> bias,
                    c10::optional<torch::Tensor> R, c10::optional<torch::Tensor> X, int64_t epi, double alpha,
                    bool accumulate, double p_drop, int64_t seed, int64_t force_ks) {
  TORCH_CHECK(A.scalar_type() == torch::kFloat32 && B.scalar_type() == torch::kFloat32 &&
                  C.scalar_type() == torch::kFloat32, "gemm_f32_ex: f32 tensors");
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "gemm_f32_ex: GPU tensors");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm_f32_ex: 2-D");
  const int M = A.size(0), K = A.size(1), N = B.size(1);
  TORCH_CHECK(B.size(0) == K && C.size(0) == M && C.size(1) == N, "gemm_f32_ex: shape mismatch");
  if (C.stride(1) != 1) return 0;
  int a_kc, b_kc;
  int64_t lda, ldb;
  if (A.stride(1) == 1) { a_kc = 1; lda = A.stride(0); }
  else if (A.stride(0) == 1) { a_kc = 0; lda = A.stride(1); }
  else return 0;
  if (B.stride(0) == 1) { b_kc = 1; ldb = B.stride(1); }
  else if (B.stride(1) == 1) { b_kc = 0; ldb = B.stride(0); }
  else return 0;
  const bool need_bias = epi == 1 || epi == 2 || epi == 4, need_r = epi >= 3, need_x = epi == 2;
  TORCH_CHECK(!need_bias || (bias.has_value() && bias->is_contiguous() && bias->numel() == N), "gemm_f32_ex: bias [N]");
  int64_t ldr = 0, ldx = 0;
  if (need_r) {
    TORCH_CHECK(R.has_value() && R->scalar_type() == torch::kFloat32 && R->dim() == 2 && R->stride(1) == 1 &&
                    R->size(0) == M && R->size(1) == N, "gemm_f32_ex: R [M,N] f32 rows");
    ldr = R->stride(0);
  }
  if (need_x) {
    TORCH_CHECK(X.has_value() && X->scalar_type() == torch::kFloat32 && X->dim() == 2 && X->stride(1) == 1 &&
                    X->size(0) == M && X->size(1) == N, "gemm_f32_ex: X [M,N] f32 rows");
    ldx = X->stride(0);
  }
  // split-K slabs from the caching allocator (inside a graph capture: the graph's pool)
  const int64_t ws_n = mp_gemm_f32_ws_elems(M, N, K, (int)force_ks);
  torch::Tensor ws;
  if (ws_n > 0) ws = torch::empty({ws_n}, A.options());
  const int rc = mp_gemm_f32_ex(A.data_ptr<float>(), B.data_ptr<float>(), C.data_ptr<float>(),
                                need_bias ? bias->data_ptr<float>() : nullptr, need_r ? R->data_ptr<float>() : nullptr,
                                need_x ? X->data_ptr<float>() : nullptr, M, N, K, lda, a_kc, ldb, b_kc, C.stride(0), ldr,
                                ldx, (int)epi, (float)alpha, accumulate ? 1 : 0, (float)p_drop, (uint64_t)seed,
                                (int)force_ks, ws_n > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
  if (rc == -1) return 0;
  check(rc, "gemm_f32_ex");
  return 1;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  mipipe_comm::register_rccl(m);
  mipipe_runtime::register_runner(m);
  m.doc() = "mipipe gfx950 HIP kernels";
  m.def("norm_fwd", &norm_fwd);
  m.def("norm_bwd", &norm_bwd);
  m.def("xent", &xent);
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd);
  m.def("sumsq", &sumsq);
  m.def("scaled_sum", &scaled_sum);
  m.def("zero_", &zero_);
  m.def("gemm_f32", &gemm_f32);
  m.def("gemm_f32_set_lanes", &mp_gemm_f32_set_lanes);
  m.def("gemm_f32_ex", &gemm_f32_ex, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("bias"),
        pybind11::arg("R"), pybind11::arg("X"), pybind11::arg("epi") = 0, pybind11::arg("alpha") = 1.0,
        pybind11::arg("accumulate") = false, pybind11::arg("p_drop") = 0.0, pybind11::arg("seed") = 0,
        pybind11::arg("force_ks") = 0);
  m.def("adamw", &adamw);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("act_fwd", &act_fwd);
  m.def("act_bwd", &act_bwd);
  m.def("colsum", &colsum);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("rope", &rope);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("gemm", &gemm);
  m.def("lane_merge", &lane_merge, pybind11::arg("g0"), pybind11::arg("lanes"), pybind11::arg("sumsq") = pybind11::none());
  m.def("gemm_tt_grouped", &gemm_tt_grouped, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("C"),
        pybind11::arg("alpha") = 1.0);
  m.def("gemm2", &gemm2, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("bias"),
        pybind11::arg("residual"), pybind11::arg("aux"), pybind11::arg("transA"), pybind11::arg("transB"),
        pybind11::arg("epilogue"), pybind11::arg("accum"), pybind11::arg("alpha"), pybind11::arg("force_cfg"),
        pybind11::arg("colsum"), pybind11::arg("p_drop") = 0.0, pybind11::arg("seed") = 0);
  m.def("transpose", &transpose);
  m.def("set_dropout_step", &set_dropout_step);
  m.def("create_stream", &create_stream, pybind11::arg("device"), pybind11::arg("priority") = 0);
  m.def("transpose_batched", &transpose_batched);
  m.def("probe_spin", &probe_spin, pybind11::arg("flag"), pybind11::arg("expect"), pybind11::arg("timeout_us"),
        pybind11::arg("result"), pybind11::arg("waiter") = 0);
  m.def("probe_set", &probe_set, pybind11::arg("flag"), pybind11::arg("value"), pybind11::arg("setter") = 0);
  m.def("probe_clock_khz", []() { return mp_probe_clock_khz(); });
  m.def("gemm2_plan", [](int64_t M, int64_t N, int64_t K, bool transA, bool transB, bool accum, int64_t force_cfg) {
    int split = 1;
    const int cfg = mp_gemm2_plan((int)M, (int)N, (int)K, transA, transB, accum, (int)force_cfg, &split);
    return std::make_tuple(cfg, split);
  }, "engine config + split-K factor the v2 GEMM picks (14: stream-K gemm7)");
  m.def("gemm2_has_probe_engines", []() { return mp_gemm2_has_probe_engines() != 0; });
}
