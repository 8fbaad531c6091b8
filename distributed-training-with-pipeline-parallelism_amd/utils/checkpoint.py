"""Checkpoint / resume for pipeline-parallel training.

The reference has no save/load code; its implied layout is a per-stage ``state_dict``
keyed by *global* FQNs (``layers.5.self_attn.in_proj_weight`` stays
``layers.5...`` on whatever stage owns layer 5 -- helper:38-44, :83-84).  This
module makes that layout explicit:

    <dir>/manifest.json                 model config, PP/DP/v, layer split, step, files
    <dir>/stage-pp{r}.safetensors       f32 master weights of pipeline rank r (global FQNs)
    <dir>/optim-pp{r}.safetensors       AdamW moments (``<fqn>.exp_avg`` / ``.exp_avg_sq``)
    <dir>/head.safetensors              distributed-head weights + moments (written once)

Only DP replica 0 writes (replicas are bit-identical after the all-reduced update).
Every tensor is addressed by FQN, so :func:`load_checkpoint` works for ANY pipeline
degree / virtual-stage count / head mode: each rank opens the shards lazily
(``safetensors.safe_open``) and copies exactly the tensors its arenas own -- resume
re-splits.  Loading never unpickles (safetensors + JSON only).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

FORMAT = "mipipe-ckpt-v1"


def _arenas(trainer):
    """(arena, optimizer-slot index, owner tag) for every arena on this rank."""
    out = []
    for i, st in enumerate(trainer.stages):
        out.append((st.arena, i, f"stage{st.stage_index}"))
    if getattr(trainer, "head", None) is not None:
        out.append((trainer.head.arena, len(trainer.stages), "head"))
    return out


def _flat_view(flat: torch.Tensor, arena, name: str) -> torch.Tensor:
    o = arena.offsets[name]
    shape = arena.specs[name].shape
    return flat[o: o + int(math.prod(shape))].view(shape)


def _full(arena, t: torch.Tensor) -> torch.Tensor:
    """An optimizer moment of ``arena`` over the whole arena (gathered when ZeRO-sharded)."""
    return t if arena.shard is None else arena.shard[2](t)


def _barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def save_checkpoint(trainer, path: str, step: Optional[int] = None, extra: Optional[dict] = None) -> None:
    """Collective: every rank calls it; DP replica 0 of each pipeline rank writes."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    mesh = trainer.mesh
    opt = trainer.optimizer
    files: Dict[str, List[str]] = {}
    params, moments = {}, {}
    head_params, head_moments = {}, {}
    for arena, slot, tag in _arenas(trainer):
        # an arena ZeRO-sharded over DP is gathered by all of its replicas (a collective);
        # everything else only by DP replica 0, which writes
        if mesh.dp_rank != 0 and not (arena.shard is not None and arena.shard_scope == "dp"):
            continue
        is_head = tag == "head"
        fm, fv = _full(arena, opt.m[slot]), _full(arena, opt.v[slot])
        with arena.unsharded():
            if mesh.dp_rank != 0:
                continue
            for name in arena.order:
                p = arena.master_view(name).detach().float().cpu().contiguous()
                m = _flat_view(fm, arena, name).detach().float().cpu().contiguous()
                v = _flat_view(fv, arena, name).detach().float().cpu().contiguous()
                (head_params if is_head else params)[name] = p
                (head_moments if is_head else moments)[name + ".exp_avg"] = m
                (head_moments if is_head else moments)[name + ".exp_avg_sq"] = v
    if mesh.dp_rank == 0:
        r = mesh.pp_rank
        if params:
            save_file(params, os.path.join(path, f"stage-pp{r}.safetensors"), metadata={"format": FORMAT})
            save_file(moments, os.path.join(path, f"optim-pp{r}.safetensors"), metadata={"format": FORMAT})
        if head_params and r == 0:
            save_file(head_params, os.path.join(path, "head.safetensors"), metadata={"format": FORMAT})
            save_file(head_moments, os.path.join(path, "optim-head.safetensors"), metadata={"format": FORMAT})
    _barrier()
    is_root = (not dist.is_initialized()) or dist.get_rank() == 0
    if is_root:
        shards = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
        manifest = {
            "format": FORMAT,
            "step": opt.step_count if step is None else step,
            "optimizer_step": opt.step_count,
            "data_step": trainer.stages[0].step_id if trainer.stages else 0,
            "pp": mesh.pp, "dp": mesh.dp, "v": trainer.v, "schedule": trainer.schedule,
            "layer_ranges": [list(r) for r in trainer.layer_ranges],
            "split_head": trainer.head is not None,
            "model": asdict(trainer.cfg),
            "shards": shards,
            "extra": extra or {},
        }
        with open(os.path.join(path, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1)
    _barrier()


def read_manifest(path: str) -> dict:
    with open(os.path.join(path, "manifest.json")) as f:
        man = json.load(f)
    if man.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    return man


def _index(path: str, man: dict) -> Dict[str, str]:
    """FQN -> shard file (params and moments)."""
    from safetensors import safe_open

    idx = {}
    for fn in man["shards"]:
        with safe_open(os.path.join(path, fn), framework="pt") as f:
            for k in f.keys():
                idx.setdefault(k, fn)
    return idx


def load_checkpoint(trainer, path: str, load_optimizer: bool = True, strict: bool = True) -> dict:
    """Load a checkpoint written at any PP degree into ``trainer`` (any PP degree).
    Returns the manifest."""
    from safetensors import safe_open

    man = read_manifest(path)
    idx = _index(path, man)
    opt = trainer.optimizer
    handles = {}

    def get(key):
        fn = idx.get(key)
        if fn is None:
            return None
        if fn not in handles:
            handles[fn] = safe_open(os.path.join(path, fn), framework="pt")
        return handles[fn].get_tensor(key)

    missing = []
    for arena, slot, _ in _arenas(trainer):
        sharded = arena.shard is not None
        # moments of a ZeRO-sharded arena: loaded full, this rank's range kept
        fm = torch.zeros(arena.numel, device=arena.device) if sharded else opt.m[slot]
        fv = torch.zeros(arena.numel, device=arena.device) if sharded else opt.v[slot]
        lo_hi = arena.shard[:2] if sharded else None
        with arena.unsharded():
            for name in arena.order:
                t = get(name)
                if t is None:
                    missing.append(name)
                    continue
                arena.master_view(name).copy_(t.reshape(arena.specs[name].shape).to(arena.device, torch.float32))
                if load_optimizer:
                    m, v = get(name + ".exp_avg"), get(name + ".exp_avg_sq")
                    if m is not None and v is not None:
                        _flat_view(fm, arena, name).copy_(m.reshape(arena.specs[name].shape))
                        _flat_view(fv, arena, name).copy_(v.reshape(arena.specs[name].shape))
                    elif strict:
                        missing.append(name + ".exp_avg")
            arena.sync_w16()
        if sharded and load_optimizer:
            opt.m[slot].copy_(fm[lo_hi[0]:lo_hi[1]])
            opt.v[slot].copy_(fv[lo_hi[0]:lo_hi[1]])
    if strict and missing:
        raise KeyError(f"checkpoint {path} lacks {len(missing)} tensors, e.g. {missing[:4]}")
    if load_optimizer:
        opt.step_count = int(man["optimizer_step"])
    for st in trainer.stages:
        st.step_id = int(man.get("data_step", 0))
    handles.clear()
    _barrier()
    return man


# ----------------------------------------------------------------------------------------
# reference layout interop (helper:36-46, :78-91): global FQNs, unpadded vocabulary
# ----------------------------------------------------------------------------------------
VOCAB_ROWS = ("tok_embeddings.weight", "output.weight", "output.bias")


def reference_state_dict(arenas, cfg) -> Dict[str, torch.Tensor]:
    """f32 CPU ``state_dict`` of native arenas in the reference's layout: the FQNs of
    ``nn.TransformerDecoderLayer`` / ``Transformer`` (the native reference block uses them
    verbatim) and the vocabulary rows cut back from the kernel-friendly padding
    (``vocab_padded``) to ``vocab_size`` -- what ``manual_model_split(...).submod.state_dict()``
    holds for the same stage."""
    out: Dict[str, torch.Tensor] = {}
    for arena in arenas:
        with arena.unsharded():
            for name in arena.order:
                t = arena.master_view(name).detach().float().cpu()
                if name in VOCAB_ROWS:
                    t = t[: cfg.vocab_size]
                out[name] = t.clone().contiguous()
    return out


def load_reference_state_dict(arenas, cfg, state_dict: Dict[str, torch.Tensor], strict: bool = True) -> List[str]:
    """Copy a reference-layout ``state_dict`` (e.g. a split stage's, or a full
    ``Transformer``'s) into native arenas; padded vocabulary rows are zeroed.  Keys the
    arenas do not own are ignored (a full model's dict loads into any stage); with
    ``strict`` every arena tensor must be present.  Returns the keys that were loaded."""
    loaded, missing = [], []
    for arena in arenas:
        with arena.unsharded():
            for name in arena.order:
                src = state_dict.get(name)
                if src is None:
                    missing.append(name)
                    continue
                dst = arena.master_view(name)
                src = src.detach().to(dst.device, torch.float32)
                if name in VOCAB_ROWS and src.shape[0] != dst.shape[0]:
                    dst.zero_()
                    dst[: src.shape[0]].copy_(src)
                else:
                    dst.copy_(src.reshape(dst.shape))
                loaded.append(name)
            arena.sync_w16()
    if strict and missing:
        raise KeyError(f"reference state_dict lacks {len(missing)} tensors, e.g. {missing[:4]}")
    return loaded


def export_reference_stage(trainer) -> Dict[str, torch.Tensor]:
    """This rank's part of the model as the reference's per-stage ``state_dict`` (global
    FQNs, unpadded).  A distributed head (replicated on every rank) is exported by the
    rank holding the last stage, where the reference keeps ``output``."""
    arenas = [st.arena for st in trainer.stages]
    if getattr(trainer, "head", None) is not None and any(st.is_last for st in trainer.stages):
        arenas.append(trainer.head.arena)
    return reference_state_dict(arenas, trainer.cfg)


def import_reference_stage(trainer, state_dict: Dict[str, torch.Tensor], strict: bool = True) -> List[str]:
    """Load reference-layout weights (one stage's dict, several merged, or a full model's)
    into every arena of this rank (including a replicated distributed head)."""
    arenas = [st.arena for st in trainer.stages]
    if getattr(trainer, "head", None) is not None:
        arenas.append(trainer.head.arena)
    return load_reference_state_dict(arenas, trainer.cfg, state_dict, strict=strict)
