"""CPU reference ops (the numerics oracle for the HIP kernels) vs torch.nn.functional /
autograd, including the explicit backward formulas."""
import math

import pytest
import torch
import torch.nn.functional as F

import mipipe  # noqa: F401
from mipipe import ops


def f32(*s):
    return torch.randn(*s)


@pytest.mark.parametrize("kind", ["layernorm", "rmsnorm"])
def test_norm_matches_autograd(kind):
    torch.manual_seed(0)
    T, D = 16, 64
    x, br, w, b = f32(T, D), f32(T, D), f32(D), f32(D)
    dy, dres = f32(T, D), f32(T, D)
    xa, bra, wa, ba = [t.clone().requires_grad_() for t in (x, br, w, b)]
    s = xa + bra
    if kind == "layernorm":
        y = F.layer_norm(s, (D,), wa, ba, 1e-5)
    else:
        y = s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + 1e-5) * wa
    (y * dy).sum().backward()
    yo, so, mean, rstd = ops.norm_fwd(x, w, b if kind == "layernorm" else None, br, kind=kind)
    torch.testing.assert_close(yo, y.detach(), atol=1e-5, rtol=1e-5)
    dw, db = torch.zeros(D), torch.zeros(D)
    ds, _ = ops.norm_bwd(dy, so, w, mean, rstd, kind=kind, dres=None, dw=dw,
                         dbias=db if kind == "layernorm" else None)
    torch.testing.assert_close(ds, xa.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(dw, wa.grad, atol=1e-4, rtol=1e-4)
    if kind == "layernorm":
        torch.testing.assert_close(db, ba.grad, atol=1e-4, rtol=1e-4)
    ds2, _ = ops.norm_bwd(dy, so, w, mean, rstd, kind=kind, dres=dres, dw=torch.zeros(D))
    torch.testing.assert_close(ds2, xa.grad + dres, atol=1e-4, rtol=1e-4)


def test_xent_matches_torch():
    torch.manual_seed(0)
    T, V, Vp = 12, 50, 64
    lg = f32(T, Vp)
    tg = torch.randint(0, V, (T,))
    la = lg[:, :V].clone().requires_grad_()
    ref = F.cross_entropy(la, tg)
    ref.backward()
    g = lg.clone()
    loss = ops.xent_fwd_bwd(g, tg, V, 1.0 / T)
    torch.testing.assert_close(loss.mean(), ref.detach(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(g[:, :V], la.grad, atol=1e-6, rtol=1e-5)
    assert torch.all(g[:, V:] == 0)


@pytest.mark.parametrize("causal,Hkv", [(True, 4), (False, 4), (True, 2)])
def test_attention_matches_sdpa(causal, Hkv):
    torch.manual_seed(0)
    B, S, H, D = 2, 16, 4, 8
    T = B * S
    qkv = f32(T, (H + 2 * Hkv) * D)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:]
    o = torch.empty(T, H * D)
    lse = torch.empty(B * H * S)
    ops.attn_fwd(q, k, v, o, lse, B, S, S, H, Hkv, D, causal)
    Q = q.reshape(B, S, H, D).transpose(1, 2).clone().requires_grad_()
    K = k.reshape(B, S, Hkv, D).transpose(1, 2).clone().requires_grad_()
    V = v.reshape(B, S, Hkv, D).transpose(1, 2).clone().requires_grad_()
    rep = H // Hkv
    ref = F.scaled_dot_product_attention(Q, K.repeat_interleave(rep, 1), V.repeat_interleave(rep, 1),
                                         is_causal=causal)
    torch.testing.assert_close(o, ref.transpose(1, 2).reshape(T, H * D).detach(), atol=1e-5, rtol=1e-5)
    do = f32(T, H * D)
    ref.backward(do.reshape(B, S, H, D).transpose(1, 2))
    dq, dk, dv = torch.empty(T, H * D), torch.empty(T, Hkv * D), torch.empty(T, Hkv * D)
    ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, S, H, Hkv, D, causal)
    torch.testing.assert_close(dq, Q.grad.transpose(1, 2).reshape(T, -1), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(dk, K.grad.transpose(1, 2).reshape(T, -1), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(dv, V.grad.transpose(1, 2).reshape(T, -1), atol=1e-4, rtol=1e-4)


def test_linear_family_matches_autograd():
    torch.manual_seed(0)
    T, K, N = 10, 16, 24
    x, w, b, r = f32(T, K), f32(N, K), f32(N), f32(T, N)
    xa, wa, ba = [t.clone().requires_grad_() for t in (x, w, b)]
    pre = xa @ wa.t() + ba
    y = F.gelu(pre, approximate="tanh")
    dy = f32(T, N)
    (y * dy).sum().backward()
    yo, aux = ops.linear(x, w, b, act="gelu_tanh")
    torch.testing.assert_close(yo, y.detach(), atol=1e-5, rtol=1e-5)
    # GELU: aux is the derivative at the pre-activation (act_bwd takes the pre-activation)
    p0 = pre.detach()
    torch.testing.assert_close(aux, torch.autograd.functional.jvp(lambda t: F.gelu(t, approximate="tanh"), p0,
                                                                  torch.ones_like(p0))[1], atol=1e-5, rtol=1e-5)
    da = ops.act_bwd(dy, p0, "gelu_tanh", dbias=(db := torch.zeros(N)))
    torch.testing.assert_close(db, ba.grad, atol=1e-4, rtol=1e-4)
    dw = ops.linear_dw(da, x, torch.zeros(N, K))
    torch.testing.assert_close(dw, wa.grad, atol=1e-4, rtol=1e-4)
    dx = ops.linear_dx(da, w)
    torch.testing.assert_close(dx, xa.grad, atol=1e-4, rtol=1e-4)
    # fused dgelu in the dX GEMM of the *next* layer == act_bwd after plain dX
    w2 = f32(5, N)
    dz = f32(T, 5)
    fused = ops.linear_dx(dz, w2, act_input=aux, act="gelu_tanh")
    unf = ops.act_bwd(ops.linear_dx(dz, w2), p0, "gelu_tanh")
    torch.testing.assert_close(fused, unf, atol=1e-5, rtol=1e-5)
    # linear's GELU aux is the derivative -- act_bwd takes it only as saved="grad"
    via_aux = ops.act_bwd(ops.linear_dx(dz, w2), aux, "gelu_tanh", saved="grad")
    torch.testing.assert_close(via_aux, unf, atol=1e-5, rtol=1e-5)
    wrong = ops.act_bwd(ops.linear_dx(dz, w2), aux, "gelu_tanh")   # the pre-activation form
    assert not torch.allclose(wrong, unf, atol=1e-3)
    with pytest.raises(ValueError):
        ops.act_bwd(dz, dz, "gelu_tanh", saved="derivative")
    yr, _ = ops.linear(x, w, b, residual=r)
    torch.testing.assert_close(yr, x @ w.t() + b + r, atol=1e-5, rtol=1e-5)


def test_swiglu_rope_embedding_adamw():
    torch.manual_seed(0)
    T, Fd = 6, 8
    gu = f32(T, 2 * Fd).requires_grad_()
    y = F.silu(gu[:, :Fd]) * gu[:, Fd:]
    dy = f32(T, Fd)
    (y * dy).sum().backward()
    torch.testing.assert_close(ops.swiglu_fwd(gu.detach()), y.detach())
    torch.testing.assert_close(ops.swiglu_bwd(gu.detach(), dy), gu.grad, atol=1e-5, rtol=1e-5)
    S, H, Hkv, Dh = 5, 2, 1, 8
    qkv = f32(S, (H + 2 * Hkv) * Dh)
    cs, sn = ops.rope_tables(S, Dh, 10000.0, "cpu")
    r = ops.rope_(qkv.clone(), cs, sn, S, H, Hkv, Dh)
    back = ops.rope_(r.clone(), cs, sn, S, H, Hkv, Dh, inverse=True)
    torch.testing.assert_close(back, qkv, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(r[:, (H + Hkv) * Dh:], qkv[:, (H + Hkv) * Dh:])  # v untouched
    # embedding
    wte, wpe = f32(20, 8), f32(4, 8)
    idx = torch.randint(0, 20, (8,))
    e = ops.embed_fwd(idx, wte, wpe, 4)
    torch.testing.assert_close(e, wte[idx] + wpe[torch.arange(8) % 4])
    # adamw vs torch.optim.AdamW
    p = torch.nn.Parameter(f32(50))
    p.grad = f32(50)
    opt = torch.optim.AdamW([p], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    pf, gf = p.detach().clone(), p.grad.clone()
    opt.step()
    m, v = torch.zeros(50), torch.zeros(50)
    ops.adamw_(pf, gf, m, v, None, 50, 1e-2, 0.9, 0.95, 1e-8, 0.1, 1)
    torch.testing.assert_close(pf, p.detach(), atol=1e-6, rtol=1e-6)


def test_use_f32_kernels_swaps_module_classes_only():
    """ops.use_f32_kernels() routes the reference layer's linears and attention projections
    to the f32 GEMM by swapping submodule classes (no global F.linear patch):
    parameters, state_dict keys and CPU outputs are unchanged, torch.nn.functional is never
    touched, and switching off restores the stock classes."""
    from mipipe.ops import kernels as K
    orig_linear = F.linear
    torch.manual_seed(0)
    layer = torch.nn.TransformerDecoderLayer(32, 4, dim_feedforward=64, dropout=0.0, batch_first=True)
    keys = list(layer.state_dict())
    x = torch.randn(2, 5, 32)
    ref = layer(x, x)
    n = K.use_f32_kernels(layer, True)
    assert n == 6   # self_attn + out_proj, multihead_attn + out_proj, linear1, linear2
    assert type(layer.self_attn) is K.F32MultiheadAttention and type(layer.linear1) is K.F32Linear
    assert list(layer.state_dict()) == keys
    torch.testing.assert_close(layer(x, x), ref)          # CPU: the stock path
    # the f32 attention path itself (projections + SDPA; on GPUs the projections are the
    # f32 GEMM) with ATen linears on CPU, vs the stock module: self, k-v-shared, separate
    mha = layer.multihead_attn
    q, kv, v2 = torch.randn(2, 5, 32), torch.randn(2, 7, 32), torch.randn(2, 7, 32)
    for args in ((q, q, q), (q, kv, kv), (q, kv, v2)):
        want = torch.nn.MultiheadAttention.forward(mha, *args, need_weights=False)[0]
        torch.testing.assert_close(K._mha_projected(mha, *args, False, F.linear), want, atol=1e-5, rtol=1e-5)
    assert K.use_f32_kernels(layer, False) == 6
    assert type(layer.self_attn) is torch.nn.MultiheadAttention
    assert type(layer.self_attn.out_proj) is torch.nn.modules.linear.NonDynamicallyQuantizableLinear
    torch.testing.assert_close(layer(x, x), ref)
    assert F.linear is orig_linear


def test_gemm_planner_split_tail_is_opt_in(monkeypatch):
    """gemm2.hip mp_gemm2_plan (host code, runs without a GPU): the split-tail engine (cfg
    14, opt-in) accepts NT grids that are not whole rounds of 256 CUs -- a pipeline rank's
    8K-32K-token microbatches -- and never whole rounds (64K tokens, N = 768: 768 tiles = 3
    rounds), dW (TT, f32 accumulate) or short-token grids."""
    from mipipe.ops import kernels as K
    e = K.load_ext()
    if e is None or not hasattr(e, "gemm2_plan"):
        pytest.skip("extension not built")
    # default: off (a measured null, gemm2.hip); force_cfg 14 plans it where it applies
    assert e.gemm2_plan(8192, 768, 768, False, False, False, -1)[0] != 14
    if not e.gemm2_has_probe_engines():
        # the default _C.so does not carry the probe engines (tools/build_ext.py --variant
        # probes -D MP_PROBE_ENGINES): the planner refuses to plan one it cannot launch
        assert e.gemm2_plan(8192, 768, 768, False, False, False, 14)[0] == -1
        return
    assert e.gemm2_plan(8192, 768, 768, False, False, False, 14)[0] == 14
    plan = lambda M, N, Kd, ta=False, tb=False, acc=False: e.gemm2_plan(M, N, Kd, ta, tb, acc, 14)[0]  # noqa: E731
    for M, N, Kd in ((8192, 768, 768), (8192, 768, 3072), (32768, 768, 3072), (32768, 768, 2304)):
        assert plan(M, N, Kd) == 14, (M, N, Kd)
    # whole rounds, or a tail too wide to split into chunks (16K x 768: 192 tiles)
    for M, N, Kd in ((65536, 768, 768), (65536, 768, 3072), (65536, 3072, 768), (16384, 768, 3072)):
        assert plan(M, N, Kd) != 14, (M, N, Kd)
    assert plan(2048, 768, 768) != 14                       # 24 tiles: below the split threshold
    assert plan(768, 3072, 32768, True, True, True) != 14    # dW


def test_comm_progress_report_formats_incomplete_groups():
    """The watchdog's comm block: engines without progress() are skipped, incomplete groups
    are listed oldest first with a cap."""
    from mipipe.parallel.comm import comm_progress_report

    class Eng:
        rank, nranks = 2, 4

        def progress(self):
            return [{"seq": 40 + i, "channel": i % 2, "kind": "p2p", "sends": [3], "recvs": [1],
                     "bytes": 3_145_728, "age_s": 61.0 - i} for i in range(8)]

        def issued(self):
            return 48

        def async_error(self):
            return ""

    rep = comm_progress_report({"p2p": Eng(), "dp": None, "x": object()}, limit=3)
    lines = rep.splitlines()
    assert lines[0] == "[comm] p2p engine (rank 2/4): 48 groups issued, 8 incomplete"
    assert lines[1] == "[comm]   #40 channel 0 p2p send->[3] recv<-[1] 3.15 MB, issued 61.0s ago"
    assert lines[-1] == "[comm]   ... 5 more" and len(lines) == 5
    assert comm_progress_report({}) == "[comm] no native RCCL engine on this rank"
