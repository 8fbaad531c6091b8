"""Explicit-backward native models vs the autograd functional reference (CPU, f32).

Covers GPT-2 (pre-LN, GELU, learned pos, tied), Llama-3 (RMSNorm, RoPE, SwiGLU, GQA) and
the reference post-LN self+cross-attention block, plus: pipeline split into stages,
full activation recompute and the zero-bubble I/W backward split give identical grads."""
import pytest
import torch

import mipipe  # noqa: F401
from mipipe.models import torch_ref
from mipipe.models.config import NativeConfig
from mipipe.models.native import MBContext, NativeModel, balanced_layer_ranges

CFGS = {
    "gpt2": NativeConfig.gpt2("tiny", vocab_size=100, d_model=64, n_layers=2, n_heads=4, d_ff=256, max_seq_len=32),
    "llama": NativeConfig.llama3("tiny", vocab_size=100, d_model=64, n_layers=2, n_heads=4, n_kv_heads=2, d_ff=128,
                                 max_seq_len=32),
    "reference": NativeConfig.reference(n_layers=2, n_heads=4, dim=64, vocab_size=100, dropout=0.0,
                                        dim_feedforward=128),
}
B, S = 2, 16


def _data(cfg):
    g = torch.Generator().manual_seed(3)
    return (torch.randint(0, cfg.vocab_size, (B, S), generator=g),
            torch.randint(0, cfg.vocab_size, (B, S), generator=g))


def _ref_grads(cfg, model):
    P = {n: model.arena.master_view(n).clone().requires_grad_() for n in model.arena.order}
    x, y = _data(cfg)
    loss = torch_ref.forward_loss(cfg, P, x, y)
    loss.backward()
    return loss.item(), {n: p.grad for n, p in P.items()}


def _run_native(models, cfg, recompute=False, split=False):
    x, y = _data(cfg)
    ctxs = [MBContext(0, 11) for _ in models]
    h = x
    loss = None
    for i, m in enumerate(models):
        m.recompute = recompute
        out = m.forward(h, ctxs[i], B, S, target=y if m.last else None)
        if m.last:
            loss = out
        else:
            h = out
    dy = None
    for i in reversed(range(len(models))):
        dy = models[i].backward(dy, ctxs[i], B, S, weight_grads=not split)
        if split:
            models[i].backward_weight(0)
    return loss.item()


@pytest.mark.parametrize("name", list(CFGS))
def test_native_matches_autograd(name):
    cfg = CFGS[name]
    model = NativeModel(cfg, 0, 1, "cpu", seed=5, dtype=torch.float32)
    ref_loss, ref_g = _ref_grads(cfg, model)
    loss = _run_native([model], cfg)
    assert loss == pytest.approx(ref_loss, rel=1e-5)
    for n, g in ref_g.items():
        got = model.arena.g(n)
        if n.startswith("tok_embeddings") or n.startswith("output"):
            got, g = got[: cfg.vocab_size], g[: cfg.vocab_size]
        torch.testing.assert_close(got, g, atol=2e-5, rtol=1e-4, msg=lambda m: f"{name}:{n}: {m}")


@pytest.mark.parametrize("name", list(CFGS))
@pytest.mark.parametrize("mode", ["split_stages", "recompute", "iw_split"])
def test_native_variants_same_grads(name, mode):
    cfg = CFGS[name]
    full = NativeModel(cfg, 0, 1, "cpu", seed=5, dtype=torch.float32)
    base_loss = _run_native([full], cfg)
    if mode == "split_stages":
        ranges = [(0, 1), (1, 2)]
        models = [NativeModel(cfg, s, 2, "cpu", layer_range=ranges[s], seed=5, dtype=torch.float32) for s in range(2)]
        if cfg.tie_embeddings:  # emulate the first/last-stage embedding grad all-reduce
            models[1].arena.load_state_dict({"tok_embeddings.weight": models[0].arena.master_view("tok_embeddings.weight")},
                                            strict=False)
        loss = _run_native(models, cfg)
        got = {}
        for m in models:
            for n in m.arena.order:
                got[n] = got.get(n, 0) + m.arena.g(n)
    else:
        m = NativeModel(cfg, 0, 1, "cpu", seed=5, dtype=torch.float32)
        loss = _run_native([m], cfg, recompute=mode == "recompute", split=mode == "iw_split")
        got = {n: m.arena.g(n) for n in m.arena.order}
    assert loss == pytest.approx(base_loss, rel=1e-6)
    for n in full.arena.order:
        torch.testing.assert_close(got[n], full.arena.g(n), atol=1e-6, rtol=1e-5, msg=lambda msg: f"{n}: {msg}")


def test_balanced_split_covers_layers():
    for name in ("gpt2-small", "gpt2-medium", "llama-8b"):
        cfg = NativeConfig.by_name(name)
        for P in (1, 2, 4, 8):
            r = balanced_layer_ranges(cfg, P)
            assert r[0][0] == 0 and r[-1][1] == cfg.n_layers
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
    ref = NativeConfig.reference(n_layers=12)
    assert balanced_layer_ranges(ref, 8, reference_rule=True)[-1] == (7, 12)  # helper:70-75
