"""Functional PyTorch (autograd) reference of the native model family.

Takes the same global-FQN parameter dict as :class:`~mipipe.models.native.ParamArena`
and computes the mean token cross-entropy with plain torch ops.  Used as the numerics
oracle for the explicit-backward native models (tests/test_native_model.py)."""
from __future__ import annotations

import math
from typing import Dict

import torch
import torch.nn.functional as F

from .config import NativeConfig


def _norm(cfg, x, w, b):
    if cfg.norm == "layernorm":
        return F.layer_norm(x, (x.shape[-1],), w, b, cfg.norm_eps)
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + cfg.norm_eps) * w


def _rope(x, S, theta):  # x [B, h, S, Dh], rotate-half
    Dh = x.shape[-1]
    inv = 1.0 / (theta ** (torch.arange(0, Dh, 2, dtype=torch.float64) / Dh))
    ang = torch.arange(S, dtype=torch.float64)[:, None] * inv[None, :]
    c, s = torch.cos(ang).to(x.dtype), torch.sin(ang).to(x.dtype)
    a, b = x[..., : Dh // 2], x[..., Dh // 2:]
    return torch.cat([a * c - b * s, b * c + a * s], -1)


def _attn(cfg, q, k, v, B, S, causal):
    H, KV, Dh = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
    q = q.reshape(B, S, H, Dh).transpose(1, 2)
    k = k.reshape(B, S, KV, Dh).transpose(1, 2)
    v = v.reshape(B, S, KV, Dh).transpose(1, 2)
    if cfg.pos == "rope":
        q, k = _rope(q, S, cfg.rope_theta), _rope(k, S, cfg.rope_theta)
    rep = H // KV
    k, v = k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
    o = F.scaled_dot_product_attention(q, k, v, is_causal=causal)
    return o.transpose(1, 2).reshape(B * S, H * Dh)


def forward_loss(cfg: NativeConfig, P: Dict[str, torch.Tensor], tokens: torch.Tensor, targets: torch.Tensor,
                 layers=None) -> torch.Tensor:
    B, S = tokens.shape
    d = cfg.d_model
    x = P["tok_embeddings.weight"][tokens.reshape(-1)]
    if cfg.pos == "learned":
        x = x + P["pos_embeddings.weight"][torch.arange(B * S) % S]
    layers = range(cfg.n_layers) if layers is None else layers
    for i in layers:
        p = lambda n: P.get(f"layers.{i}.{n}")
        if cfg.cross_attn:
            h = x
            W, b = p("self_attn.in_proj_weight"), p("self_attn.in_proj_bias")
            qkv = h @ W.t() + b
            sa = _attn(cfg, qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], B, S, False)
            sa = sa @ p("self_attn.out_proj.weight").t() + p("self_attn.out_proj.bias")
            x1 = F.layer_norm(h + sa, (d,), p("norm1.weight"), p("norm1.bias"), cfg.norm_eps)
            W, b = p("multihead_attn.in_proj_weight"), p("multihead_attn.in_proj_bias")
            q = x1 @ W[:d].t() + b[:d]
            kv = h @ W[d:].t() + b[d:]
            ca = _attn(cfg, q, kv[:, :d], kv[:, d:], B, S, False)
            ca = ca @ p("multihead_attn.out_proj.weight").t() + p("multihead_attn.out_proj.bias")
            x2 = F.layer_norm(x1 + ca, (d,), p("norm2.weight"), p("norm2.bias"), cfg.norm_eps)
            f = torch.relu(x2 @ p("linear1.weight").t() + p("linear1.bias")) @ p("linear2.weight").t() + p("linear2.bias")
            x = F.layer_norm(x2 + f, (d,), p("norm3.weight"), p("norm3.bias"), cfg.norm_eps)
            continue
        h = _norm(cfg, x, p("attn_norm.weight"), p("attn_norm.bias"))
        qkv = h @ p("attn.wqkv.weight").t()
        if cfg.bias:
            qkv = qkv + p("attn.wqkv.bias")
        H, KV, Dh = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
        o = _attn(cfg, qkv[:, :H * Dh], qkv[:, H * Dh:(H + KV) * Dh], qkv[:, (H + KV) * Dh:], B, S, cfg.causal)
        o = o @ p("attn.wo.weight").t()
        if cfg.bias:
            o = o + p("attn.wo.bias")
        x = x + o
        h = _norm(cfg, x, p("ffn_norm.weight"), p("ffn_norm.bias"))
        if cfg.activation == "swiglu":
            gu = h @ p("ffn.w13.weight").t()
            f = F.silu(gu[:, :cfg.d_ff]) * gu[:, cfg.d_ff:]
            f = f @ p("ffn.w2.weight").t()
        else:
            a = h @ p("ffn.w1.weight").t()
            if cfg.bias:
                a = a + p("ffn.w1.bias")
            a = F.gelu(a, approximate="tanh") if cfg.activation == "gelu_tanh" else torch.relu(a)
            f = a @ p("ffn.w2.weight").t()
            if cfg.bias:
                f = f + p("ffn.w2.bias")
        x = x + f
    if cfg.final_norm:
        x = _norm(cfg, x, P["norm.weight"], P.get("norm.bias"))
    W = P["tok_embeddings.weight"] if cfg.tie_embeddings else P["output.weight"]
    logits = x @ W[: cfg.vocab_size].t()
    if "output.bias" in P:
        logits = logits + P["output.bias"][: cfg.vocab_size]
    return F.cross_entropy(logits, targets.reshape(-1))
