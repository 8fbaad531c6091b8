"""The native reference block against the REAL reference module, and reference-layout
checkpoint interop.

* Parity: ``ref_transformer.Transformer`` is the reference's model verbatim
  (nn.Embedding -> nn.TransformerDecoderLayer(dim, heads, batch_first=True) called as
  ``layer(h, h)`` -> nn.LayerNorm -> nn.Linear, helper:31-55) and its loss is the
  reference's token-wise CE (helper:197-201).  Its weights are loaded into
  ``NativeModel(NativeConfig.reference(...))`` (f32, CPU, dropout 0): loss and every
  parameter gradient must match to 1e-5 -- this pins the post-LN / self+cross-attention
  (memory = layer input) semantics the reference numbers depend on.
* Interop: a reference per-stage ``state_dict`` from ``manual_model_split`` (global FQNs,
  unpadded 10000-row vocab, helper:38-44, :83-91) loads into the native stage and exports
  back bit-identically, at any split.
"""
import pytest
import torch

import mipipe  # noqa: F401
from mipipe.models.config import NativeConfig
from mipipe.models.native import MBContext, NativeModel, balanced_layer_ranges
from mipipe.models.ref_transformer import ModelArgs, Transformer, manual_model_split, tokenwise_loss_fn
from mipipe.utils.checkpoint import load_reference_state_dict, reference_state_dict


def _args(L=2, H=4, dim=64, V=100, F=128):
    return ModelArgs(dim=dim, n_layers=L, n_heads=H, vocab_size=V, dim_feedforward=F, dropout=0.0)


def _cfg(a):
    return NativeConfig.reference(n_layers=a.n_layers, n_heads=a.n_heads, dim=a.dim, vocab_size=a.vocab_size,
                                  dropout=0.0, dim_feedforward=a.dim_feedforward)


@pytest.mark.parametrize("L,H", [(2, 4), (3, 8), (2, 2)])
def test_native_reference_block_matches_torch_transformer(L, H):
    torch.manual_seed(0)
    a = _args(L=L, H=H)
    ref = Transformer(a).float()
    B, S = 2, 16
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, a.vocab_size, (B, S), generator=g)
    y = torch.randint(0, a.vocab_size, (B, S), generator=g)
    loss_ref = tokenwise_loss_fn(a.vocab_size)(ref(x), y)
    loss_ref.backward()

    cfg = _cfg(a)
    nat = NativeModel(cfg, 0, 1, torch.device("cpu"), dtype=torch.float32)
    load_reference_state_dict([nat.arena], cfg, ref.state_dict())
    ctx = MBContext(0, 5)
    loss = nat.forward(x, ctx, B, S, target=y, loss_scale=1.0)
    nat.backward(None, ctx, B, S)
    assert float(loss) == pytest.approx(float(loss_ref), rel=1e-5, abs=1e-6)
    grads = {n: p.grad for n, p in ref.named_parameters()}
    assert set(grads) == set(nat.arena.order)
    for n, gr in grads.items():
        mine = nat.arena.g(n)
        if mine.shape != gr.shape:   # padded vocabulary rows
            assert not mine[gr.shape[0]:].any(), n
            mine = mine[: gr.shape[0]]
        torch.testing.assert_close(mine.float(), gr, atol=1e-5, rtol=1e-4, msg=lambda m: f"{n}: {m}")


@pytest.mark.parametrize("num_stages", [1, 2, 4])
def test_reference_stage_state_dict_roundtrip(num_stages):
    """manual_model_split stage dicts <-> native stages (reference split rule)."""
    torch.manual_seed(0)
    a = _args(L=4, V=10000)
    cfg = _cfg(a)
    full = Transformer(a)
    ranges = balanced_layer_ranges(cfg, num_stages, reference_rule=True)
    for s in range(num_stages):
        part = Transformer(a)
        part.load_state_dict(full.state_dict())
        sd = manual_model_split(part, s, num_stages, "cpu").submod.state_dict()
        nat = NativeModel(cfg, s, num_stages, torch.device("cpu"), layer_range=ranges[s], dtype=torch.float32)
        load_reference_state_dict([nat.arena], cfg, sd)
        out = reference_state_dict([nat.arena], cfg)
        assert set(out) == set(sd), (set(out) ^ set(sd))
        for k in sd:
            assert out[k].shape == sd[k].shape, k
            assert torch.equal(out[k], sd[k].float()), k
        if s == 0:
            assert out["tok_embeddings.weight"].shape == (10000, 64)
        if s == num_stages - 1:
            assert out["output.weight"].shape == (10000, 64) and out["output.bias"].shape == (10000,)


def test_trainer_reference_export_import_with_distributed_head():
    """PipelineTrainer at PP=1 (head on the last stage) and the compat export helpers."""
    from mipipe.engine import PipelineTrainer
    from mipipe.utils.checkpoint import export_reference_stage, import_reference_stage
    torch.manual_seed(0)
    a = _args(L=2)
    full = Transformer(a)
    tr = PipelineTrainer(_cfg(a), pp=1, n_microbatches=2, mbs=1, seq_len=16, device=torch.device("cpu"),
                         dtype=torch.float32)
    loaded = import_reference_stage(tr, full.state_dict())
    assert set(loaded) == set(full.state_dict())
    out = export_reference_stage(tr)
    for k, v in full.state_dict().items():
        assert torch.equal(out[k], v), k


@pytest.mark.gpu
@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_graphed_autograd_stage_matches_eager(dropout):
    """PipelineStage(graphs=True): the reference's own f32 nn.Module replayed as one HIP
    graph per direction and microbatch slot gives the eager stage's loss and gradients
    (dropout 0: to f32 tolerance over 3 steps of 4 microbatches; dropout 0.1: finite,
    different masks per replay)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mipipe.parallel.api import Schedule1F1B
    dev = torch.device("cuda", 0)
    torch.backends.cuda.matmul.allow_tf32 = False
    a = ModelArgs(dim=128, n_layers=2, n_heads=4, vocab_size=256, dim_feedforward=256, dropout=dropout)
    torch.manual_seed(0)
    base = Transformer(a)
    g = torch.Generator().manual_seed(1)
    xs = [torch.randint(0, 256, (16, 32), generator=g).to(dev) for _ in range(3)]
    ys = [torch.randint(0, 256, (16, 32), generator=g).to(dev) for _ in range(3)]
    res = {}
    for graphs in (False, True, "eager2"):
        model = Transformer(a)
        model.load_state_dict(base.state_dict())
        stage = manual_model_split(model, 0, 1, dev)
        stage.graphs = graphs is True
        sched = Schedule1F1B(stage, n_microbatches=4, loss_fn=tokenwise_loss_fn(256))
        losses = []
        for x, y in zip(xs, ys):
            ls = []
            sched.step(x, target=y, losses=ls)
            losses.append(torch.stack([l.detach() for l in ls]).cpu())
        grads = {n: p.grad.detach().cpu().clone() for n, p in stage.submod.named_parameters()}
        res[graphs] = (torch.stack(losses), grads)
        assert (len(stage._graph_fns) == 4) == (graphs is True)
    (l0, g0), (l1, g1), (_, g2) = res[False], res[True], res["eager2"]
    assert torch.isfinite(l1).all()
    if dropout == 0.0:
        torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-5)
        bad = []
        for n in g0:
            # tolerance: a few times the eager-vs-eager spread (atomic-order effects) + f32 noise
            spread = (g2[n] - g0[n]).abs().max().item()
            dev_g = (g1[n] - g0[n]).abs().max().item()
            scale = g0[n].abs().max().item()
            print(n, f"eager-eager {spread:.3g} graph-eager {dev_g:.3g} |g| {scale:.3g}")
            if dev_g > 4 * spread + 1e-5 * max(1e-2, scale):
                bad.append((n, dev_g, spread, scale))
        assert not bad, bad
    else:
        assert not torch.equal(l1[0], l1[1])


@pytest.mark.gpu
def test_f32_kernel_stage_matches_aten():
    """PipelineStage.f32_kernels: the reference's own f32 module with every linear and
    attention projection on the f32 MFMA GEMM (graphs on) vs ATen f32 (TF32 off)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mipipe.parallel.api import Schedule1F1B
    dev = torch.device("cuda", 0)
    torch.backends.cuda.matmul.allow_tf32 = False
    a = ModelArgs(dim=256, n_layers=2, n_heads=4, vocab_size=512, dim_feedforward=512, dropout=0.0)
    torch.manual_seed(0)
    base = Transformer(a)
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 512, (16, 64), generator=g).to(dev)
    y = torch.randint(0, 512, (16, 64), generator=g).to(dev)
    res = {}
    for f32k in (False, True):
        model = Transformer(a)
        model.load_state_dict(base.state_dict())
        stage = manual_model_split(model, 0, 1, dev)
        stage.graphs = True
        stage.f32_kernels = f32k
        sched = Schedule1F1B(stage, n_microbatches=4, loss_fn=tokenwise_loss_fn(512))
        ls = []
        sched.step(x, target=y, losses=ls)
        res[f32k] = (torch.stack([l.detach() for l in ls]).cpu(),
                     {n: p.grad.detach().cpu().clone() for n, p in stage.submod.named_parameters()})
    (l0, g0), (l1, g1) = res[False], res[True]
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-5)
    for n in g0:
        scale = g0[n].abs().max().item()
        assert (g1[n] - g0[n]).abs().max().item() <= 1e-4 * max(scale, 1e-3), n
