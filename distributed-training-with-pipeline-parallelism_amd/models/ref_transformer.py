"""The reference's toy Transformer and manual splitter (reference-compatible API).

Behavior (reference helper:23-94):

* ``ModelArgs(dim=768, n_layers=8, n_heads=8, vocab_size=10000)``.
* ``Transformer``: ``tok_embeddings`` -> ``layers`` (a ``ModuleDict`` keyed
  ``"0".."L-1"`` of ``nn.TransformerDecoderLayer(dim, heads, batch_first=True)``:
  post-LN, FFN 2048, ReLU, dropout 0.1) -> ``norm`` -> ``output``.  Each layer is
  called as ``layer(h, h)`` (cross-attention memory = its own input, no masks),
  and missing pieces (``None``) are skipped so a split stage runs only its part.
* ``manual_model_split``: ``L // num_stages`` layers per stage, remainder on the
  last stage; stage 0 keeps the embedding, the last stage keeps norm + output;
  deleted layers keep their global keys, so stage ``state_dict`` s use global FQNs.

This module is the autograd (``nn.Module``) form used by the compat API and as
the numerics oracle.  The same architecture runs on HIP kernels through
``mipipe.models.native`` (``NativeConfig.reference(...)``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.nn as nn

from ..parallel.stage import PipelineStage


@dataclass
class ModelArgs:
    dim: int = 768  # divisible by 4, 8 and 12 heads (helper:25)
    n_layers: int = 8
    n_heads: int = 8
    vocab_size: int = 10000
    dim_feedforward: int = 2048
    dropout: float = 0.1


class Transformer(nn.Module):
    def __init__(self, model_args: ModelArgs):
        super().__init__()
        self.model_args = model_args
        self.tok_embeddings = nn.Embedding(model_args.vocab_size, model_args.dim)
        self.layers = nn.ModuleDict()
        for layer_id in range(model_args.n_layers):
            self.layers[str(layer_id)] = nn.TransformerDecoderLayer(
                model_args.dim, model_args.n_heads, dim_feedforward=model_args.dim_feedforward,
                dropout=model_args.dropout, batch_first=True)
        self.norm = nn.LayerNorm(model_args.dim)
        self.output = nn.Linear(model_args.dim, model_args.vocab_size)

    def forward(self, tokens: torch.Tensor):
        h = self.tok_embeddings(tokens) if self.tok_embeddings is not None else tokens
        for layer in self.layers.values():
            h = layer(h, h)
        h = self.norm(h) if self.norm is not None else h
        return self.output(h).clone() if self.output is not None else h


def stage_layer_range(n_layers: int, stage_index: int, num_stages: int):
    """[start, end) of the layers a stage owns (reference helper:70-75)."""
    per = n_layers // num_stages
    start = stage_index * per
    end = start + per if stage_index < num_stages - 1 else n_layers
    return start, end


def split_module_(model: Transformer, stage_index: int, num_stages: int) -> Transformer:
    """In-place split of a full model down to one stage's part (helper:78-91)."""
    n_layers = len(model.layers)
    start, end = stage_layer_range(n_layers, stage_index, num_stages)
    for i in range(n_layers):
        if i < start or i >= end:
            del model.layers[str(i)]
    if stage_index != 0:
        model.tok_embeddings = None
    if stage_index != num_stages - 1:
        model.norm = None
        model.output = None
    return model


def manual_model_split(model: nn.Module, stage_index: int, num_stages: int, device,
                       group=None) -> PipelineStage:
    """Reference API (helper:60-94): split, then wrap as a :class:`PipelineStage`."""
    split_module_(model, stage_index, num_stages)
    model.to(device)
    return PipelineStage(model, stage_index, num_stages, device, group=group)


def tokenwise_loss_fn(vocab_size: int):
    """CrossEntropy(mean) over flattened tokens (helper:197-201)."""
    ce = nn.CrossEntropyLoss()

    def loss_fn(outputs, targets):
        return ce(outputs.reshape(-1, vocab_size), targets.reshape(-1))

    return loss_fn
