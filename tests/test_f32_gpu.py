"""The reference-precision (f32) GPU path on our kernels vs PyTorch f32/f64 references.

The reference trains its model in f32 (helper:36-46, no autocast; SURVEY §2.5 "dtype: fp32
everywhere").  ``NativeModel(dtype=torch.float32)`` on a GPU runs every op of the reference
block on hand-written kernels: the f32 MFMA GEMM with fused epilogues (gemm_f32.hip), f32
flash attention (attention_f32.hip), and the storage-type-templated norm / cross-entropy /
embedding / column-sum kernels.  Each is compared here with the same op in PyTorch, and
the whole block with the real ``nn.TransformerDecoderLayer`` reference (1e-4)."""
import math

import pytest
import torch

import mipipe  # noqa: F401
from mipipe import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def setup_module(module):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert ops.ext_available(), "HIP extension must be built for GPU tests"


def close(a, b, atol=1e-4, rtol=1e-4):
    torch.testing.assert_close(a.double().cpu(), b.double().cpu(), atol=atol, rtol=rtol)


# ----------------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(1024, 2304, 768), (1000, 776, 520), (64, 10000, 768), (2048, 768, 1024),
                                   (40, 72, 36)])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_f32_layouts(M, N, K, layout):
    """C = A @ B for every operand layout (K- or outer-contiguous A and B), tails included."""
    torch.manual_seed(0)
    a64, b64 = torch.randn(M, K, dtype=torch.float64), torch.randn(K, N, dtype=torch.float64)
    A = a64.float().to(DEV) if layout[0] == "n" else a64.t().contiguous().float().to(DEV).t()
    B = b64.t().contiguous().float().to(DEV).t() if layout[1] == "t" else b64.float().to(DEV)
    C = torch.empty(M, N, device=DEV)
    ops.kernels._gemm_f32(A, B, C)
    ref = a64.float().double() @ b64.float().double()
    close(C, ref, atol=2e-4 * math.sqrt(K), rtol=1e-5)


@pytest.mark.parametrize("epi", ["bias", "bias_relu", "res", "bias_res", "drelu", "accum"])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm_f32_epilogues(epi, p):
    torch.manual_seed(1)
    M, N, K = 1024, 2048, 768
    x, w = torch.randn(M, K), torch.randn(N, K) / math.sqrt(K)
    b, r = torch.randn(N), torch.randn(M, N)
    xg, wg, bg, rg = (t.to(DEV) for t in (x, w, b, r))
    y = torch.empty(M, N, device=DEV)
    lin = (x.double() @ w.double().t())
    K_ = ops.kernels
    if epi == "bias":
        K_._gemm_f32(xg, wg.t(), y, bias=bg, epi=K_.F32_BIAS)
        close(y, lin + b.double())
    elif epi == "bias_relu":
        aux = torch.empty_like(y)
        K_._gemm_f32(xg, wg.t(), y, bias=bg, X=aux, epi=K_.F32_BIAS_RELU, p_drop=p, seed=7)
        pre = lin + b.double()
        close(aux, pre)
        keep = (y.double().cpu() != 0) | (pre <= 0)
        if p > 0:
            pos = pre > 0
            rate = ((y.cpu() != 0) & pos).sum().item() / pos.sum().item()
            assert abs(rate - (1 - p)) < 0.01, rate
        close(y, torch.relu(pre) * keep / (1 - p))
        # the backward regenerates the same mask: dReLU x mask on dy = 1
        dx = torch.empty_like(y)
        K_._gemm_f32(torch.ones(M, 8, device=DEV), torch.ones(8, N, device=DEV) / 8, dx, R=aux, epi=K_.F32_DRELU,
                     p_drop=p, seed=7)
        close(dx, (pre > 0).double() * keep / (1 - p))
    elif epi == "res":
        K_._gemm_f32(xg, wg.t(), y, R=rg, epi=K_.F32_RES)
        close(y, lin + r.double())
    elif epi == "bias_res":
        K_._gemm_f32(xg, wg.t(), y, bias=bg, R=rg, epi=K_.F32_BIAS_RES)
        close(y, lin + b.double() + r.double())
    elif epi == "drelu":
        pre = torch.randn(M, N)
        K_._gemm_f32(xg, wg.t(), y, R=pre.to(DEV), epi=K_.F32_DRELU)
        close(y, lin * (pre > 0).double())
    else:   # f32 accumulate into C with alpha (the dW GEMM)
        y.copy_(rg)
        K_._gemm_f32(xg, wg.t(), y, alpha=0.5, accumulate=True)
        close(y, 0.5 * lin + r.double())


@pytest.mark.parametrize("M,N,K", [(1024, 768, 2048), (1000, 776, 3000), (1024, 768, 768), (200, 136, 4096),
                                   (1024, 2304, 768)])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("epi", ["none", "bias_relu", "accum"])
def test_gemm_f32_stream_k(M, N, K, layout, epi):
    """The stream-K schedule of the 64x64 engine (force_ks = -2): workgroup chunks that end
    inside a tile and span up to three tiles, tails in M / N / K, every layout class and the
    epilogues applied by the partial-tile reduce pass (ReLU + dropout with the forward mask
    the backward regenerates, f32 accumulate with alpha)."""
    torch.manual_seed(3)
    a64, b64 = torch.randn(M, K, dtype=torch.float64), torch.randn(K, N, dtype=torch.float64) / math.sqrt(K)
    A = a64.float().to(DEV) if layout[0] == "n" else a64.t().contiguous().float().to(DEV).t()
    B = b64.t().contiguous().float().to(DEV).t() if layout[1] == "t" else b64.float().to(DEV)
    ref = a64.float().double() @ b64.float().double()
    e = ops.kernels._ext()
    C = torch.full((M, N), float("nan"), device=DEV)
    if epi == "none":
        assert e.gemm_f32_ex(A, B, C, None, None, None, 0, 1.0, False, 0.0, 0, -2)
        close(C, ref, atol=2e-4 * math.sqrt(K / 64), rtol=1e-5)
    elif epi == "bias_relu":
        bias = torch.randn(N, device=DEV)
        X = torch.empty(M, N, device=DEV)
        assert e.gemm_f32_ex(A, B, C, bias, None, X, 2, 1.0, False, 0.1, 11, -2)
        pre = ref + bias.double().cpu()
        close(X, pre, atol=2e-4 * math.sqrt(K / 64), rtol=1e-5)
        C2 = torch.empty(M, N, device=DEV)     # the tiled engine: same dropout mask
        assert e.gemm_f32_ex(A, B, C2, bias, None, torch.empty_like(X), 2, 1.0, False, 0.1, 11, 1)
        assert torch.equal((C != 0), (C2 != 0))
        close(C, C2, atol=2e-4 * math.sqrt(K / 64), rtol=1e-5)
    else:
        base = torch.randn(M, N, device=DEV)
        C.copy_(base)
        assert e.gemm_f32_ex(A, B, C, None, None, None, 0, 0.5, True, 0.0, 0, -2)
        close(C, 0.5 * ref + base.double().cpu(), atol=2e-4 * math.sqrt(K / 64), rtol=1e-5)


@pytest.mark.parametrize("lanes", [1, 2, 4])
def test_gemm_f32_lane_aware_split(lanes):
    """The split-K planner counts 256 / lanes CUs (PipelineRuntime.set_lanes): the splits it
    picks for the reference's 1024-token shapes change, the results do not (plain store and
    f32 accumulate; the dX of the LM head has K = vocab = 10000)."""
    e = ops.kernels._ext()
    try:
        assert e.gemm_f32_set_lanes(lanes) == 256 // lanes
        torch.manual_seed(4)
        for M, N, K in ((1024, 768, 10000), (1024, 768, 3072), (768, 3072, 1024), (1024, 2304, 768)):
            a64, b64 = torch.randn(M, K, dtype=torch.float64), torch.randn(K, N, dtype=torch.float64) / math.sqrt(K)
            A, B = a64.float().to(DEV), b64.float().to(DEV)
            ref = a64.float().double() @ b64.float().double()
            C = torch.full((M, N), float("nan"), device=DEV)
            ops.kernels._gemm_f32(A, B, C)
            close(C, ref, atol=2e-4 * math.sqrt(K / 64), rtol=1e-5)
            base = torch.randn(M, N, device=DEV)
            C.copy_(base)
            ops.kernels._gemm_f32(A, B, C, alpha=0.5, accumulate=True)
            close(C, 0.5 * ref + base.double().cpu(), atol=2e-4 * math.sqrt(K / 64), rtol=1e-5)
    finally:
        e.gemm_f32_set_lanes(1)


def test_linear_dw_f32_matches_torch():
    torch.manual_seed(2)
    T, N, K = 1024, 2304, 768
    dy, x = torch.randn(T, N), torch.randn(T, K)
    dw = torch.zeros(N, K, device=DEV)
    ops.linear_dw(dy.to(DEV), x.to(DEV), dw)
    close(dw, dy.double().t() @ x.double(), atol=2e-3, rtol=1e-5)


# ------------------------------------------------------------------------------ attention
def _attn_ref(q, k, v, B, Sq, Sk, H, D, scale):
    Q = q.double().view(B, Sq, H, D).transpose(1, 2)
    Kk = k.double().view(B, Sk, H, D).transpose(1, 2)
    V = v.double().view(B, Sk, H, D).transpose(1, 2)
    s = (Q @ Kk.transpose(-1, -2)) * scale
    p = torch.softmax(s, -1)
    o = (p @ V).transpose(1, 2).reshape(B * Sq, H * D)
    return o, torch.logsumexp(s, -1) / math.log(2.0)


@pytest.mark.parametrize("D", [64, 96, 128, 192])
@pytest.mark.parametrize("S", [128, 100])
@pytest.mark.parametrize("packed", [True, False])
def test_attention_f32_fwd_bwd(D, S, packed):
    """Self-attention layout (q, k, v column slices of one packed [T, 3HD] buffer) and the
    cross-attention layout (q alone, k / v slices of a [T, 2HD] buffer), vs f64 math."""
    torch.manual_seed(3)
    B, H = 2, 3
    T = B * S
    scale = 1.0 / math.sqrt(D)
    if packed:
        qkv = torch.randn(T, 3 * H * D, device=DEV)
        q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv[:, :H * D], dqkv[:, H * D:2 * H * D], dqkv[:, 2 * H * D:]
    else:
        q = torch.randn(T, H * D, device=DEV)
        kv = torch.randn(T, 2 * H * D, device=DEV)
        k, v = kv[:, :H * D], kv[:, H * D:]
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        dk, dv = dkv[:, :H * D], dkv[:, H * D:]
    o = torch.empty(T, H * D, device=DEV)
    lse = torch.empty(B * H * S, device=DEV)
    ops.attn_fwd(q, k, v, o, lse, B, S, S, H, H, D, False)
    qd, kd, vd = (t.detach().cpu().double().requires_grad_() for t in (q, k, v))
    o_ref, lse_ref = _attn_ref(qd, kd, vd, B, S, S, H, D, scale)
    close(o, o_ref, atol=1e-5, rtol=1e-4)
    close(lse, lse_ref.reshape(-1), atol=1e-5, rtol=1e-5)
    do = torch.randn(T, H * D, device=DEV)
    ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, S, H, H, D, False)
    o_ref.backward(do.cpu().double())
    close(dq, qd.grad, atol=2e-5, rtol=1e-4)
    close(dk, kd.grad, atol=2e-5, rtol=1e-4)
    close(dv, vd.grad, atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("p", [0.1, 0.3])
def test_attention_f32_dropout_mask_exact(p):
    """The f32 kernels regenerate the forward's dropout mask in the backward, at the keep
    rate -- and it is the SAME mask the bf16 kernels draw (one hash, both precisions)."""
    B, S, H, D = 4, 64, 4, 64
    T = B * S
    ops.set_dropout_step(3)
    masks = {}
    for dt in (torch.float32, torch.bfloat16):
        q = torch.zeros(T, H * D, dtype=dt, device=DEV)
        k = torch.zeros_like(q)
        v = torch.eye(S, D, dtype=dt, device=DEV).repeat(B, H)
        o = torch.empty_like(q)
        lse = torch.empty(B * H * S, device=DEV)
        ops.attn_fwd(q, k, v, o, lse, B, S, S, H, H, D, False, p_drop=p, seed=1234)
        do = v.clone()
        dq, dk, dv = torch.zeros_like(q), torch.zeros_like(q), torch.zeros_like(q)
        ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, S, H, H, D, False, p_drop=p, seed=1234)
        torch.cuda.synchronize()
        m_f = (o.float().view(B, S, H, D) > 0)
        m_b = (dv.float().view(B, S, H, D) > 0).transpose(1, 3)
        assert torch.equal(m_f, m_b), f"{dt}: forward and backward dropout masks differ"
        masks[dt] = m_f
        if dt == torch.float32:
            kept = o.view(B, S, H, D)[m_f]
            torch.testing.assert_close(kept, torch.full_like(kept, 1.0 / (S * (1 - p))), rtol=1e-5, atol=0)
            rate = m_f.float().mean().item()
            assert abs(rate - (1 - p)) < 5 * math.sqrt(p * (1 - p) / m_f.numel())
    assert torch.equal(masks[torch.float32], masks[torch.bfloat16])


# -------------------------------------------------------------------- memory-bound kernels
@pytest.mark.parametrize("D", [768, 64, 2048])
def test_norm_f32(D):
    torch.manual_seed(4)
    T = 300
    x, w, b, br, dy, dres = (torch.randn(T, D), torch.randn(D), torch.randn(D), torch.randn(T, D),
                             torch.randn(T, D), torch.randn(T, D))
    outs = []
    for dev in ("cpu", DEV):
        mv = lambda t: t.to(dev)
        y, s, mean, rstd = ops.norm_fwd(mv(x), mv(w), mv(b), mv(br))
        dw, db, cs = torch.zeros(D, device=dev), torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        ds, _ = ops.norm_bwd(mv(dy), s, mv(w), mean, rstd, dres=mv(dres), dw=dw, dbias=db, colsum_dres=cs)
        outs.append((y, s, mean, rstd, ds, dw, db, cs))
    for a, g in zip(*outs):
        close(g, a, atol=1e-4, rtol=1e-4)


def test_xent_embed_colsum_f32():
    torch.manual_seed(5)
    T, V, Vp, D, S = 256, 10000, 10000, 768, 128
    logits = torch.randn(T, Vp) * 3
    tgt = torch.randint(0, V, (T,))
    lc, lg = logits.clone(), logits.to(DEV)
    loss_c = ops.xent_fwd_bwd(lc, tgt, V, 0.5)
    loss_g = ops.xent_fwd_bwd(lg, tgt.to(DEV), V, 0.5)
    close(loss_g, loss_c, atol=1e-5, rtol=1e-5)
    close(lg, lc, atol=1e-7, rtol=1e-5)
    wte = torch.randn(V, D)
    idx = torch.randint(0, V, (T,))
    close(ops.embed_fwd(idx.to(DEV), wte.to(DEV), None, S), wte[idx], atol=0, rtol=0)
    dout = torch.randn(T, D)
    g = torch.zeros(V, D, device=DEV)
    ops.embed_bwd(idx.to(DEV), dout.to(DEV), g, None, S)
    ref = torch.zeros(V, D, dtype=torch.float64).index_add_(0, idx, dout.double())
    close(g, ref, atol=1e-5, rtol=1e-5)
    cs = torch.zeros(D, device=DEV)
    ops.colsum(dout.to(DEV), cs)
    close(cs, dout.double().sum(0), atol=1e-4, rtol=1e-5)


# --------------------------------------------------------------- the reference block, f32
@pytest.mark.parametrize("dim,H", [(256, 4), (192, 2), (384, 2)])
def test_reference_block_f32_gpu_matches_torch_transformer(dim, H):
    """NativeModel(reference cfg, f32) on the GPU kernels vs the reference's own module
    (nn.TransformerDecoderLayer stack, CPU f32, dropout 0): loss and every gradient to
    1e-4 -- d_h = 64 / 96 / 192, the reference's head sizes."""
    from mipipe.models.config import NativeConfig
    from mipipe.models.native import MBContext, NativeModel
    from mipipe.models.ref_transformer import ModelArgs, Transformer, tokenwise_loss_fn
    from mipipe.utils.checkpoint import load_reference_state_dict
    torch.manual_seed(0)
    a = ModelArgs(dim=dim, n_layers=2, n_heads=H, vocab_size=1000, dim_feedforward=512, dropout=0.0)
    ref = Transformer(a).float()
    B, S = 2, 64
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, a.vocab_size, (B, S), generator=g)
    y = torch.randint(0, a.vocab_size, (B, S), generator=g)
    loss_ref = tokenwise_loss_fn(a.vocab_size)(ref(x), y)
    loss_ref.backward()
    cfg = NativeConfig.reference(n_layers=2, n_heads=H, dim=dim, vocab_size=1000, dropout=0.0, dim_feedforward=512)
    nat = NativeModel(cfg, 0, 1, torch.device(DEV), dtype=torch.float32)
    assert nat.arena.master.dtype == torch.float32 and nat.arena.w16 is nat.arena.master
    load_reference_state_dict([nat.arena], cfg, ref.state_dict())
    ctx = MBContext(0, 5)
    loss = nat.forward(x.to(DEV), ctx, B, S, target=y.to(DEV), loss_scale=1.0)
    nat.backward(None, ctx, B, S)
    torch.cuda.synchronize()
    assert float(loss) == pytest.approx(float(loss_ref), rel=1e-4)
    for n, p in ref.named_parameters():
        mine = nat.arena.g(n)
        if mine.shape != p.grad.shape:
            mine = mine[: p.grad.shape[0]]
        scale = p.grad.abs().max().item() + 1e-12
        torch.testing.assert_close(mine.cpu() / scale, p.grad / scale, atol=1e-4, rtol=0, msg=lambda m: f"{n}: {m}")


def test_trainer_f32_gpu_graphs_learns():
    """PipelineTrainer(dtype=f32) on one GPU with HIP graphs + the native tape: the
    reference block (dropout 0.1) trains on a repeated batch."""
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig
    cfg = NativeConfig.reference(n_layers=2, n_heads=8, dim=768, vocab_size=10000)
    tr = PipelineTrainer(cfg, pp=1, n_microbatches=4, mbs=8, seq_len=128, device=torch.device(DEV),
                         dtype=torch.float32, graphs=True, lr=1e-3)
    gen = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randint(0, cfg.vocab_size, (32, 128), device=DEV, generator=gen)
    y = torch.randint(0, cfg.vocab_size, (32, 128), device=DEV, generator=gen)
    tr.capture_graphs(x, y)
    losses = [float(tr.train_step(x, y)) for _ in range(6)]
    assert all(math.isfinite(l) for l in losses)
    assert losses[-1] < losses[0]
    assert tr.runtime.native_runner is not None, tr.runtime.native_reason


def test_compat_reference_api_runs_native_tape_fp32():
    """The reference-compatible API (helper:98-235 signatures) on one GPU: build_reference_stage
    in f32 with HIP graphs, Schedule1F1B, the last rank's step(target=y, losses=...) returning
    merged logits -- and still replayed from the native tape."""
    import multiprocessing as _mp
    from mipipe.bench.compat import worker_process
    q = _mp.get_context("spawn").Queue()
    from mipipe.bench.compat import _free_port
    worker_process(0, 1, 4, 8, "1F1B", 32, 128, 3, q, port=_free_port())
    m = q.get(timeout=10)
    assert "error" not in m, m
    assert m["precision"] == "fp32" and m["native_runner"], m
    assert m["throughput"] > 0 and m["lanes"] >= 1


def test_mean_and_zero_kernels():
    """ops.mean (one-workgroup deterministic sum, the microbatch loss) and ops.zero_
    (hipMemsetAsync) -- the step's last ATen reductions / fills."""
    x = torch.randn(1000, device=DEV)
    m1, m2 = ops.mean(x), ops.mean(x)
    assert m1.shape == () and m1.item() == m2.item()
    close(m1, x.double().mean(), atol=1e-6, rtol=1e-6)
    y = torch.randn(37, 5, device=DEV)
    ops.zero_(y)
    assert int((y != 0).sum()) == 0
