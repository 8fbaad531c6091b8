"""Native transformer stages: explicit per-layer forward/backward on the HIP kernels.

Why explicit instead of autograd:
* every tensor a backward needs is stashed in a per-microbatch slot that the pipeline
  schedule bounds (GPipe: m slots, 1F1B: <= P - s), and nothing else is kept alive;
* the fused epilogues (bias+GELU with saved pre-activation, residual adds, GELU' in the
  dX GEMM, f32 dW accumulation into the flat grad arena) cross what would be separate
  autograd nodes;
* the backward splits into an input-grad part (I) and a weight-grad part (W) for
  zero-bubble schedules, and supports full activation recompute (Llama-3 8B config).

Parameters of a stage live in one :class:`ParamArena` (flat f32 master + flat bf16 working
copy + flat f32 grad).  Names are global FQNs (``layers.7.attn.wqkv.weight``;
the reference architecture uses the reference's own nn.TransformerDecoderLayer names),
so checkpoints are per-stage shards that re-split to any PP degree.
"""
from __future__ import annotations

import contextlib
import hashlib
import os
import math
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from .. import ops
from .config import NativeConfig

# ======================================================================================
# parameter arena
# ======================================================================================


@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    init: str          # normal | zeros | ones | normal_scaled
    decay: bool
    std: float = 0.02
    transpose: bool = False  # keep a bf16 W^T copy (dX GEMMs run both-K-contiguous)


def _name_seed(seed: int, name: str) -> int:
    h = hashlib.blake2b(f"{seed}:{name}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & 0x7FFFFFFFFFFFFFFF


class ParamArena:
    """Flat storage for one stage's parameters: f32 master, bf16 copy, f32 grads.

    Decayed tensors come first so weight decay is a prefix ``[0, n_decay)`` of the
    flat buffer (one AdamW launch for the whole stage)."""

    def __init__(self, specs: Sequence[ParamSpec], device, dtype=torch.bfloat16, seed: int = 0,
                 init: bool = True, numel_multiple: int = 8):
        specs = sorted(specs, key=lambda s: (not s.decay,))
        self.specs = {s.name: s for s in specs}
        self.order = [s.name for s in specs]
        self.offsets: Dict[str, int] = {}
        off = 0
        for s in specs:
            n = int(math.prod(s.shape))
            # keep every tensor 16-byte aligned in the bf16 copy (8 elements)
            off = (off + 7) // 8 * 8
            self.offsets[s.name] = off
            off += n
        mult = max(8, int(numel_multiple))
        self.numel = (off + mult - 1) // mult * mult
        # ZeRO-1 (shard_master): this rank keeps only master[lo:hi] (and the optimizer
        # moments of that range); ``unsharded()`` gathers the full master when needed
        self.shard: Optional[Tuple[int, int, Callable]] = None
        self.shard_scope: Optional[str] = None   # "pp" (ZeRO-1 head) | "dp" (ZeRO-1 over DP replicas)
        self.n_decay = 0
        for s in specs:
            if s.decay:
                self.n_decay = self.offsets[s.name] + int(math.prod(s.shape))
        self.device = torch.device(device)
        self.dtype = dtype
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        # per-lane gradient buffers (microbatch lanes, parallel/runtime.py): lane 0 is
        # ``grad`` itself; the others are summed into it at the end of the step
        self.grad_lanes: List[torch.Tensor] = [self.grad]
        self.merged_sumsq: Optional[torch.Tensor] = None   # set by merge_lanes (GPU, lanes > 1)
        # the kernels' working copy of the weights: bf16, or -- f32 arenas (the reference-
        # precision path) -- the f32 master itself (AdamW then writes no second copy)
        self.w_is_master = dtype == torch.float32
        self.w16 = self.master if self.w_is_master else torch.zeros(self.numel, dtype=dtype, device=self.device)
        # transposed bf16 copies of the matrices used as B in dX = dY W (GPU bf16 only: the f32
        # GEMM reads either operand layout)
        self.t_offsets: Dict[str, int] = {}
        toff = 0
        if self.device.type == "cuda" and dtype == torch.bfloat16:
            for s in specs:
                if s.transpose and len(s.shape) == 2:
                    self.t_offsets[s.name] = toff
                    toff += (int(math.prod(s.shape)) + 7) // 8 * 8
        self.wt16 = torch.zeros(max(toff, 1), dtype=dtype, device=self.device)
        if init:
            self.init_params(seed)

    def init_params(self, seed: int = 0) -> None:
        for name in self.order:
            s = self.specs[name]
            v = self.master_view(name)
            if s.init == "zeros":
                v.zero_()
            elif s.init == "ones":
                v.fill_(1.0)
            else:
                gdev = "cuda" if self.device.type == "cuda" else "cpu"
                g = torch.Generator(device=gdev).manual_seed(_name_seed(seed, name))
                v.copy_(torch.randn(s.shape, generator=g, device=gdev, dtype=torch.float32) * s.std)
        self.sync_w16()

    def sync_w16(self) -> None:
        if self.shard is not None:
            raise RuntimeError("sync_w16 on a sharded arena: use `with arena.unsharded(): arena.sync_w16()`")
        if self.w_is_master:
            self.w16 = self.master       # (re-bound: load paths may have swapped the master tensor)
            return
        ops.cast_f32_bf16(self.master, self.w16)
        self.refresh_transposes()

    def refresh_transposes(self) -> None:
        """W^T copies from the bf16 weights: one batched launch on GPU (a 16-byte-vector
        tile transpose over a static descriptor table), per-matrix on CPU."""
        if not self.t_offsets:
            return
        if self.w16.is_cuda and all(self.specs[n].shape[0] % 8 == 0 and self.specs[n].shape[1] % 8 == 0
                                    and self.offsets[n] % 8 == 0 and o % 8 == 0
                                    for n, o in self.t_offsets.items()):
            if getattr(self, "_tdesc", None) is None:
                rows, t0, tiles = [], [], 0
                for name, o in self.t_offsets.items():
                    r, c = self.specs[name].shape
                    rows.append([self.offsets[name], o, r, c])
                    t0.append(tiles)
                    tiles += ((r + 63) // 64) * ((c + 63) // 64)
                self._tdesc = torch.tensor(rows, dtype=torch.int64, device=self.w16.device)
                self._ttile0 = torch.tensor(t0, dtype=torch.int32, device=self.w16.device)
                self._ttiles = tiles
            ops.load_ext().transpose_batched(self.w16, self.wt16, self._tdesc, self._ttile0, self._ttiles)
            return
        for name in self.t_offsets:
            ops.transpose(self.w(name), self.wt(name))

    def wt(self, name: str) -> Optional[torch.Tensor]:
        """W^T ([in, out]) view of a 2-D weight, or None if no copy is kept."""
        o = self.t_offsets.get(name)
        if o is None:
            return None
        r, c = self.specs[name].shape
        return self.wt16[o: o + r * c].view(c, r)

    def _view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        s = self.specs[name]
        o = self.offsets[name]
        return buf[o: o + int(math.prod(s.shape))].view(s.shape)

    def w(self, name: str) -> torch.Tensor:
        return self._view(self.w16, name)

    def g(self, name: str) -> torch.Tensor:
        return self._view(self.grad, name)

    def master_view(self, name: str) -> torch.Tensor:
        return self._view(self.master, name)

    def has(self, name: str) -> bool:
        return name in self.specs

    def state_dict(self) -> Dict[str, torch.Tensor]:
        with self.unsharded():
            return {n: self.master_view(n).detach().clone() for n in self.order}

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        missing = [n for n in self.order if n not in sd]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:5]}...")
        with self.unsharded():
            for n in self.order:
                if n in sd:
                    self.master_view(n).copy_(sd[n].to(self.device, torch.float32).reshape(self.specs[n].shape))
            self.sync_w16()

    def zero_grad(self) -> None:
        for g in self.grad_lanes:
            ops.zero_(g)

    # ------------------------------------------------------------------ ZeRO-1
    def shard_master(self, lo: int, hi: int, gather: Callable[[torch.Tensor], torch.Tensor],
                     scope: str = "pp") -> None:
        """Keep only ``master[lo:hi]`` on this rank (``gather(shard) -> full`` rebuilds the
        whole f32 master: a collective over ``scope``, the group the arena is sharded over).
        bf16 weights and f32 gradients stay full-size (every rank computes with the whole
        matrix and accumulates its whole gradient)."""
        if self.shard is not None:
            raise RuntimeError("arena already sharded")
        if not self.w_is_master:
            self.master = self.master[lo:hi].clone()
        # f32 arenas: the master is the working copy, so it stays full-size; the optimizer
        # updates master[lo:hi] (opt_views) and the step's all-gather of w16 (= master)
        # refreshes the rest -- only the Adam moments are sharded
        self.shard = (int(lo), int(hi), gather)
        self.shard_scope = scope

    @contextlib.contextmanager
    def unsharded(self):
        """Full f32 master inside the block (checkpoint save / load, state_dict); writes to
        it are kept (this rank's range) when the block ends.  Collective when sharded."""
        if self.shard is None:
            yield self
            return
        lo, hi, gather = self.shard
        if self.w_is_master:      # full and current on every rank already
            self.shard = None
            try:
                yield self
            finally:
                self.shard = (lo, hi, gather)
            return
        shard = self.master
        self.master = gather(shard)
        self.shard = None
        try:
            yield self
        finally:
            shard.copy_(self.master[lo:hi])
            self.master = shard
            self.shard = (lo, hi, gather)

    def opt_views(self):
        """(master, grad, w16, n_decay) that the optimizer updates: the whole arena, or
        this rank's range of a sharded one (n_decay relative to it)."""
        if self.shard is None:
            return self.master, self.grad, (None if self.w_is_master else self.w16), self.n_decay
        lo, hi, _ = self.shard
        nd = max(0, min(self.n_decay, hi) - lo)
        if self.w_is_master:
            return self.master[lo:hi], self.grad[lo:hi], None, nd
        return self.master, self.grad[lo:hi], self.w16[lo:hi], nd

    def set_lanes(self, n: int) -> None:
        """Keep ``n`` gradient buffers: two microbatches of different lanes run their
        backwards concurrently, and the dW GEMMs' f32 read-modify-write accumulation (and
        the norm-weight reductions) must not race on one buffer."""
        while len(self.grad_lanes) < n:
            self.grad_lanes.append(torch.zeros_like(self.grad_lanes[0]))
        del self.grad_lanes[max(n, 1):]

    @contextlib.contextmanager
    def lane(self, idx: int):
        """Route every gradient view taken inside (``g(name)``, ``grad``) to lane ``idx``."""
        if idx == 0 or len(self.grad_lanes) <= 1:
            yield
            return
        prev = self.grad
        self.grad = self.grad_lanes[idx]
        try:
            yield
        finally:
            self.grad = prev

    def merge_lanes(self) -> None:
        """grad += every other lane's gradient; those are zeroed for the next step (one
        fused pass on GPU: optim.hip lane_merge_sumsq_kernel, which also leaves the merged
        gradient's sum of squares in ``merged_sumsq`` for the optimizer's clipping norm --
        engine.FlatAdamW then skips its own pass over this arena)."""
        g0 = self.grad_lanes[0]
        rest = self.grad_lanes[1:]
        if g0.is_cuda:
            if len(rest) <= 3 and _FUSED_MERGE_NORM:
                if self.merged_sumsq is None:
                    self.merged_sumsq = torch.zeros(1, dtype=torch.float32, device=g0.device)
                ops.zero_(self.merged_sumsq)
                ops.load_ext().lane_merge(g0, rest, self.merged_sumsq)
                return
            self.merged_sumsq = None
            for i in range(0, len(rest), 3):
                ops.load_ext().lane_merge(g0, rest[i:i + 3])
            return
        for g in rest:
            g0.add_(g)
            g.zero_()


# ======================================================================================
# per-microbatch context
# ======================================================================================


class MBContext:
    """Activation stash of one microbatch on one stage (a dict per layer)."""

    def __init__(self, mb: int, seed: int):
        self.mb = mb
        self.seed = seed
        self.layers: Dict[int, dict] = {}
        self.misc: dict = {}


# MIPIPE_FUSE_QKV_BIAS=1: the attention backward kernels sum the QKV bias gradient
# themselves.  Off by default: measured 2 % slower end to end (same-box A/B, GPT-2 small:
# 740K vs 754K tok/s) than the separate colsum pass -- the cross-lane reductions and the
# contended per-column atomics in the attention epilogue cost more than re-reading dQKV
_FUSE_QKV_BIAS = os.environ.get("MIPIPE_FUSE_QKV_BIAS", "0") == "1"
# MIPIPE_FUSE_FC1_BIAS=0: the fc1 bias gradient in a separate pass instead of the dX GEMM's epilogue
_FUSE_FC1_BIAS = os.environ.get("MIPIPE_FUSE_FC1_BIAS", "1") != "0"
# MIPIPE_WGRAD_STREAM=0: weight-gradient GEMMs inline on the compute stream (no overlap)
_WGRAD_STREAM = os.environ.get("MIPIPE_WGRAD_STREAM", "1") != "0"
_WGRAD_SIDE: Dict[int, "torch.cuda.Stream"] = {}


class WGradOverlap:
    """Weight-gradient work of a full stage backward (``B``) on a second HIP stream.

    The dX chain of a backward is the critical path (its result goes to the previous
    stage); the dW GEMMs only feed the optimizer.  Issued on a side stream right after
    their layer's dX work, they fill the CUs the dX GEMMs leave idle (an N = 768 output
    is 192 256x256 tiles on 256 CUs) and overlap the memory-bound norm / attention
    backward kernels.  Every job list stays referenced until the compute stream has
    waited for it, so neither the caching allocator nor a HIP-graph capture's private
    pool can hand its input blocks to a concurrent writer; at most ``depth`` layers are
    in flight (bounded extra activation lifetime).  :meth:`join` closes the fork, so a
    captured backward graph is self-contained.
    """

    def __init__(self, device: torch.device, depth: int = 2):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        side = _WGRAD_SIDE.get(idx)
        if side is None:
            # Which stream (hence which hardware queue: HIP maps streams onto
            # GPU_MAX_HW_QUEUES=4 queues per priority) carries the dW work matters a lot.
            # Measured, GPT-2 small bench on one MI355X (profiles/r2_wgrad_stream_ab.txt):
            # torch's normal-priority pool stream 831K tok/s; a private stream (normal or
            # high priority) or the high-priority pool 725K; dW inline 800K.  Default: the
            # pool stream; MIPIPE_WGRAD_POOL=high|0 selects the alternatives for A/B runs.
            pool = os.environ.get("MIPIPE_WGRAD_POOL", "1")
            if pool in ("1", "high"):
                side = torch.cuda.Stream(device=idx, priority=-1 if pool == "high" else 0)
            else:
                side = torch.cuda.ExternalStream(ops.load_ext().create_stream(idx, 0),
                                                 device=torch.device("cuda", idx))
            _WGRAD_SIDE[idx] = side
            from ..parallel.graphs import register_side_stream
            register_side_stream(side)     # joined back if a capture fails mid-fork
        self.side = side
        self.main = torch.cuda.current_stream(idx)
        if self.side.cuda_stream == self.main.cuda_stream:
            raise RuntimeError("weight-gradient side stream is the compute stream: no overlap possible")
        self.depth = depth
        self.inflight: List[tuple] = []   # (completion event, job list)

    @staticmethod
    def make(device: torch.device, weight_grads: bool = True) -> Optional["WGradOverlap"]:
        if not (_WGRAD_STREAM and weight_grads and device.type == "cuda"):
            return None
        return WGradOverlap(device)

    def run(self, jobs: List[Callable[[], None]]) -> None:
        if not jobs:
            return
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            ops.run_wjobs(jobs)
        ev = torch.cuda.Event()
        ev.record(self.side)
        self.inflight.append((ev, jobs))
        while len(self.inflight) > self.depth:
            self.main.wait_event(self.inflight.pop(0)[0])

    def join(self) -> None:
        if self.inflight:
            self.main.wait_stream(self.side)
            self.inflight.clear()


def _seed(base: int, *parts: int) -> int:
    x = base & 0xFFFFFFFFFFFF
    for p in parts:
        x = (x * 0x100000001B3 + (p + 0x9E37)) & 0x7FFFFFFFFFFFFFFF
    return x


# ======================================================================================
# blocks
# ======================================================================================


def block_param_specs(cfg: NativeConfig, i: int) -> List[ParamSpec]:
    d, f = cfg.d_model, cfg.d_ff
    std, rstd = cfg.init_std, cfg.init_std / math.sqrt(2 * cfg.n_layers)
    nb = "ones"
    out: List[ParamSpec] = []
    P = f"layers.{i}."
    if cfg.cross_attn:  # reference nn.TransformerDecoderLayer names
        for att in ("self_attn", "multihead_attn"):
            out += [ParamSpec(P + f"{att}.in_proj_weight", (3 * d, d), "normal", True, std, True),
                    ParamSpec(P + f"{att}.in_proj_bias", (3 * d,), "zeros", False),
                    ParamSpec(P + f"{att}.out_proj.weight", (d, d), "normal", True, std, True),
                    ParamSpec(P + f"{att}.out_proj.bias", (d,), "zeros", False)]
        out += [ParamSpec(P + "linear1.weight", (f, d), "normal", True, std, True),
                ParamSpec(P + "linear1.bias", (f,), "zeros", False),
                ParamSpec(P + "linear2.weight", (d, f), "normal", True, std, True),
                ParamSpec(P + "linear2.bias", (d,), "zeros", False)]
        for k in (1, 2, 3):
            out += [ParamSpec(P + f"norm{k}.weight", (d,), nb, False), ParamSpec(P + f"norm{k}.bias", (d,), "zeros", False)]
        return out
    out += [ParamSpec(P + "attn_norm.weight", (d,), nb, False)]
    if cfg.norm == "layernorm":
        out += [ParamSpec(P + "attn_norm.bias", (d,), "zeros", False)]
    out += [ParamSpec(P + "attn.wqkv.weight", (cfg.qkv_dim, d), "normal", True, std, True),
            ParamSpec(P + "attn.wo.weight", (d, d), "normal", True, rstd, True)]
    if cfg.bias:
        out += [ParamSpec(P + "attn.wqkv.bias", (cfg.qkv_dim,), "zeros", False),
                ParamSpec(P + "attn.wo.bias", (d,), "zeros", False)]
    out += [ParamSpec(P + "ffn_norm.weight", (d,), nb, False)]
    if cfg.norm == "layernorm":
        out += [ParamSpec(P + "ffn_norm.bias", (d,), "zeros", False)]
    if cfg.activation == "swiglu":
        out += [ParamSpec(P + "ffn.w13.weight", (2 * f, d), "normal", True, std, True),
                ParamSpec(P + "ffn.w2.weight", (d, f), "normal", True, rstd, True)]
    else:
        out += [ParamSpec(P + "ffn.w1.weight", (f, d), "normal", True, std, True),
                ParamSpec(P + "ffn.w2.weight", (d, f), "normal", True, rstd, True)]
        if cfg.bias:
            out += [ParamSpec(P + "ffn.w1.bias", (f,), "zeros", False),
                    ParamSpec(P + "ffn.w2.bias", (d,), "zeros", False)]
    return out


class Block:
    """One transformer layer with explicit forward / backward (pre-norm GPT-2/Llama or
    the reference post-norm self+cross-attention block)."""

    def __init__(self, cfg: NativeConfig, idx: int, arena: ParamArena, rope=None):
        self.cfg = cfg
        self.i = idx
        self.A = arena
        self.P = f"layers.{idx}."
        self.rope = rope  # (cos, sin) tables

    def w(self, n):
        return self.A.w(self.P + n)

    def g(self, n):
        return self.A.g(self.P + n)

    def wb(self, n):
        return self.A.w(self.P + n) if self.A.has(self.P + n) else None

    def wt(self, n):
        return self.A.wt(self.P + n)

    def gb(self, n):
        return self.A.g(self.P + n) if self.A.has(self.P + n) else None

    # ------------------------------------------------------------------ pre-norm
    def _attn_fwd(self, h, B, S, st, seed):
        cfg = self.cfg
        H, KV, Dh = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
        qkv, _ = ops.linear(h, self.w("attn.wqkv.weight"), self.wb("attn.wqkv.bias"))
        if cfg.pos == "rope":
            ops.rope_(qkv, self.rope[0], self.rope[1], S, H, KV, Dh)
        q, k, v = qkv[:, : H * Dh], qkv[:, H * Dh:(H + KV) * Dh], qkv[:, (H + KV) * Dh:]
        o = torch.empty(h.shape[0], H * Dh, device=h.device, dtype=h.dtype)
        lse = torch.empty(B * H * S, device=h.device, dtype=torch.float32)
        ops.attn_fwd(q, k, v, o, lse, B, S, S, H, KV, Dh, cfg.causal, p_drop=cfg.dropout, seed=seed)
        st["qkv"], st["o"], st["lse"] = qkv, o, lse
        return o

    def forward(self, x: torch.Tensor, B: int, S: int, ctx: MBContext, recompute: bool = False):
        cfg = self.cfg
        st: dict = {}
        sd = _seed(ctx.seed, self.i)
        if cfg.cross_attn:
            y = self._ref_forward(x, B, S, st, sd)
        else:
            kind = cfg.norm
            h1, _, mu1, rs1 = ops.norm_fwd(x, self.w("attn_norm.weight"), self.wb("attn_norm.bias"), kind=kind,
                                           eps=cfg.norm_eps)
            o = self._attn_fwd(h1, B, S, st, _seed(sd, 1))
            x2, _ = ops.linear(o, self.w("attn.wo.weight"), self.wb("attn.wo.bias"), residual=x)
            h2, _, mu2, rs2 = ops.norm_fwd(x2, self.w("ffn_norm.weight"), self.wb("ffn_norm.bias"), kind=kind,
                                           eps=cfg.norm_eps)
            if cfg.activation == "swiglu":
                gu, _ = ops.linear(h2, self.w("ffn.w13.weight"))
                gact = ops.swiglu_fwd(gu)
                y, _ = ops.linear(gact, self.w("ffn.w2.weight"), residual=x2)
                st.update(gu=gu, g=gact)
            else:
                gact, a = ops.linear(h2, self.w("ffn.w1.weight"), self.wb("ffn.w1.bias"), act=cfg.activation)
                y, _ = ops.linear(gact, self.w("ffn.w2.weight"), self.wb("ffn.w2.bias"), residual=x2)
                st.update(a=a, g=gact)
            st.update(x=x, h1=h1, mu1=mu1, rs1=rs1, x2=x2, h2=h2, mu2=mu2, rs2=rs2)
        if recompute:
            st = {"x": x}  # full recompute: keep only the layer input
        ctx.layers[self.i] = st
        return y

    def _ensure(self, B, S, ctx):
        st = ctx.layers[self.i]
        if len(st) == 1 and "x" in st:  # recompute the stash
            tmp = MBContext(ctx.mb, ctx.seed)
            self.forward(st["x"], B, S, tmp, recompute=False)
            ctx.layers[self.i] = tmp.layers[self.i]
        return ctx.layers[self.i]

    def backward(self, dy: torch.Tensor, B: int, S: int, ctx: MBContext, weight_grads: bool = True,
                 defer: Optional[list] = None, ov: Optional[WGradOverlap] = None):
        """Returns dx.  If ``weight_grads`` is False the dW GEMMs are appended to ``defer``
        (zero-bubble split: I now, W later); with an ``ov`` they run on its side stream."""
        st = self._ensure(B, S, ctx)
        cfg = self.cfg
        sd = _seed(ctx.seed, self.i)
        wjobs: List[Callable[[], None]] = []
        if cfg.cross_attn:
            dx = self._ref_backward(dy, B, S, st, sd, wjobs)
        else:
            kind = cfg.norm
            H, KV, Dh = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
            # ---------------- FFN
            if cfg.activation == "swiglu":
                dgact = ops.linear_dx(dy, self.w("ffn.w2.weight"), wt=self.wt("ffn.w2.weight"))
                gact, h2, gu = st["g"], st["h2"], st["gu"]
                wjobs.append(ops.DW(dy, gact, self.g("ffn.w2.weight")))
                dgu = ops.swiglu_bwd(gu, dgact)
                wjobs.append(ops.DW(dgu, h2, self.g("ffn.w13.weight")))
                dh2 = ops.linear_dx(dgu, self.w("ffn.w13.weight"), wt=self.wt("ffn.w13.weight"))
            else:
                gact, a, h2 = st["g"], st["a"], st["h2"]
                # the fc1 bias gradient (column sums of da) is accumulated by the dX GEMM's
                # epilogue instead of a second pass over da
                fuse_b1 = cfg.bias and _FUSE_FC1_BIAS
                da = ops.linear_dx(dy, self.w("ffn.w2.weight"), act_input=a, act=cfg.activation,
                                   wt=self.wt("ffn.w2.weight"), colsum=self.g("ffn.w1.bias") if fuse_b1 else None)
                wjobs.append(ops.DW(dy, gact, self.g("ffn.w2.weight")))
                if cfg.bias and not fuse_b1:
                    wjobs.append(lambda da=da: ops.colsum(da, self.g("ffn.w1.bias")))
                wjobs.append(ops.DW(da, h2, self.g("ffn.w1.weight")))
                dh2 = ops.linear_dx(da, self.w("ffn.w1.weight"), wt=self.wt("ffn.w1.weight"))
            fuse_cs = cfg.bias and kind == "layernorm"
            dx2, _ = ops.norm_bwd(dh2, st["x2"], self.w("ffn_norm.weight"), st["mu2"], st["rs2"], kind=kind,
                                  dres=dy, dw=self.g("ffn_norm.weight"), dbias=self.gb("ffn_norm.bias"),
                                  colsum_dres=self.g("ffn.w2.bias") if fuse_cs else None,
                                  colsum_ds=self.g("attn.wo.bias") if fuse_cs else None)
            if cfg.bias and not fuse_cs:
                wjobs.append(lambda dy=dy: ops.colsum(dy, self.g("ffn.w2.bias")))
            # ---------------- attention
            o = st["o"]
            do = ops.linear_dx(dx2, self.w("attn.wo.weight"), wt=self.wt("attn.wo.weight"))
            wjobs.append(ops.DW(dx2, o, self.g("attn.wo.weight")))
            if cfg.bias and not fuse_cs:
                wjobs.append(lambda dx2=dx2: ops.colsum(dx2, self.g("attn.wo.bias")))
            qkv = st["qkv"]
            q, k, v = qkv[:, : H * Dh], qkv[:, H * Dh:(H + KV) * Dh], qkv[:, (H + KV) * Dh:]
            dqkv = torch.empty_like(qkv)
            dq, dk, dv = dqkv[:, : H * Dh], dqkv[:, H * Dh:(H + KV) * Dh], dqkv[:, (H + KV) * Dh:]
            # the QKV bias gradient is summed by the attention backward kernels themselves
            # (no second pass over dQKV), unless RoPE still has to rotate dQ/dK afterwards
            fuse_qkv_bias = cfg.bias and cfg.pos != "rope" and _FUSE_QKV_BIAS
            ops.attn_bwd(q, k, v, o, do, st["lse"], dq, dk, dv, B, S, S, H, KV, Dh, cfg.causal,
                         p_drop=cfg.dropout, seed=_seed(sd, 1),
                         dbias=self.g("attn.wqkv.bias") if fuse_qkv_bias else None)
            if cfg.pos == "rope":
                ops.rope_(dqkv, self.rope[0], self.rope[1], S, H, KV, Dh, inverse=True)
            h1 = st["h1"]
            wjobs.append(ops.DW(dqkv, h1, self.g("attn.wqkv.weight")))
            if cfg.bias and not fuse_qkv_bias:
                wjobs.append(lambda dqkv=dqkv: ops.colsum(dqkv, self.g("attn.wqkv.bias")))
            dh1 = ops.linear_dx(dqkv, self.w("attn.wqkv.weight"), wt=self.wt("attn.wqkv.weight"))
            dx, _ = ops.norm_bwd(dh1, st["x"], self.w("attn_norm.weight"), st["mu1"], st["rs1"], kind=kind,
                                 dres=dx2, dw=self.g("attn_norm.weight"), dbias=self.gb("attn_norm.bias"))
        if ov is not None:
            ov.run(wjobs)
        elif weight_grads:
            ops.run_wjobs(wjobs)
        else:
            defer.extend(wjobs)
        del ctx.layers[self.i]
        return dx

    # ------------------------------------------------------------------ reference post-norm block
    def _mha(self, prefix, xq, xkv, B, S, seed, st, key, self_attn: bool):
        cfg = self.cfg
        H, Dh, d = cfg.n_heads, cfg.head_dim, cfg.d_model
        W, b = self.w(prefix + ".in_proj_weight"), self.w(prefix + ".in_proj_bias")
        if self_attn:
            qkv, _ = ops.linear(xq, W, b)
            q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
            st[key + "qkv"] = qkv
        else:
            q, _ = ops.linear(xq, W[:d], b[:d])
            kv, _ = ops.linear(xkv, W[d:], b[d:])
            k, v = kv[:, :d], kv[:, d:]
            st[key + "q"], st[key + "kv"] = q, kv
        o = torch.empty(xq.shape[0], d, device=xq.device, dtype=xq.dtype)
        lse = torch.empty(B * H * S, device=xq.device, dtype=torch.float32)
        ops.attn_fwd(q, k, v, o, lse, B, S, S, H, H, Dh, False, p_drop=cfg.dropout, seed=seed)
        st[key + "o"], st[key + "lse"] = o, lse
        out, _ = ops.linear(o, self.w(prefix + ".out_proj.weight"), self.w(prefix + ".out_proj.bias"))
        return out

    def _ref_forward(self, h, B, S, st, sd):
        cfg = self.cfg
        p = cfg.dropout
        sa = self._mha("self_attn", h, h, B, S, _seed(sd, 1), st, "sa_", True)
        x1, s1, mu1, rs1 = ops.norm_fwd(h, self.w("norm1.weight"), self.w("norm1.bias"), branch=sa, eps=cfg.norm_eps,
                                        p_drop=p, seed=_seed(sd, 2))
        ca = self._mha("multihead_attn", x1, h, B, S, _seed(sd, 3), st, "ca_", False)
        x2, s2, mu2, rs2 = ops.norm_fwd(x1, self.w("norm2.weight"), self.w("norm2.bias"), branch=ca,
                                        eps=cfg.norm_eps, p_drop=p, seed=_seed(sd, 4))
        # linear1 + bias + ReLU + dropout in one GEMM epilogue (pre-activation kept in a)
        gact, a = ops.linear(x2, self.w("linear1.weight"), self.w("linear1.bias"), act="relu", p_drop=p,
                             seed=_seed(sd, 5))
        f, _ = ops.linear(gact, self.w("linear2.weight"), self.w("linear2.bias"))
        y, s3, mu3, rs3 = ops.norm_fwd(x2, self.w("norm3.weight"), self.w("norm3.bias"), branch=f, eps=cfg.norm_eps,
                                       p_drop=p, seed=_seed(sd, 6))
        st.update(x=h, x1=x1, s1=s1, mu1=mu1, rs1=rs1, x2=x2, s2=s2, mu2=mu2, rs2=rs2, a=a, g=gact, s3=s3, mu3=mu3,
                  rs3=rs3)
        return y

    def _mha_bwd(self, prefix, dout, xq, xkv, B, S, seed, st, key, self_attn, wjobs, dres_q, dres_kv):
        """Self-attention: returns (dx, None), the residual grad folded in.  Cross-attention:
        returns (dxq, dkv) -- the K/V projections' input gradient is left to the caller,
        which folds it into the block input's gradient as a residual GEMM epilogue (no
        separate add).  The out_proj bias grad was accumulated by the norm backward that
        produced ``dout``."""
        cfg = self.cfg
        H, Dh, d = cfg.n_heads, cfg.head_dim, cfg.d_model
        W = self.w(prefix + ".in_proj_weight")
        gW, gb = self.g(prefix + ".in_proj_weight"), self.g(prefix + ".in_proj_bias")
        o = st[key + "o"]
        wjobs.append(ops.DW(dout, o, self.g(prefix + ".out_proj.weight")))
        do = ops.linear_dx(dout, self.w(prefix + ".out_proj.weight"), wt=self.wt(prefix + ".out_proj.weight"))
        if self_attn:
            qkv = st[key + "qkv"]
            q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
            dqkv = torch.empty_like(qkv)
            dq, dk, dv = dqkv[:, :d], dqkv[:, d:2 * d], dqkv[:, 2 * d:]
        else:
            q, kv = st[key + "q"], st[key + "kv"]
            k, v = kv[:, :d], kv[:, d:]
            dq = torch.empty_like(q)
            dkv = torch.empty_like(kv)
            dk, dv = dkv[:, :d], dkv[:, d:]
        # the in_proj bias grads stay weight-gradient jobs (colsum kernels off the critical
        # path): the attention kernels' fused column sums (dbias=) cost 5 % of the reference
        # step here (tools/runs/archive/ab_ref_dbias.sh: 574-579K vs 609-610K tok/s, L8H8)
        ops.attn_bwd(q, k, v, o, do, st[key + "lse"], dq, dk, dv, B, S, S, H, H, Dh, False, p_drop=cfg.dropout,
                     seed=seed)
        if self_attn:
            wjobs.append(lambda dqkv=dqkv: ops.colsum(dqkv, gb))
        else:
            wjobs.append(lambda dq=dq: ops.colsum(dq, gb[:d]))
            wjobs.append(lambda dkv=dkv: ops.colsum(dkv, gb[d:]))
        if self_attn:
            wjobs.append(ops.DW(dqkv, xq, gW))
            dx = ops.linear_dx(dqkv, W, residual=dres_q, wt=self.wt(prefix + ".in_proj_weight"))
            return dx, None
        wjobs.append(ops.DW(dq, xq, gW[:d]))
        wjobs.append(ops.DW(dkv, xkv, gW[d:]))
        WT = self.wt(prefix + ".in_proj_weight")
        dxq = ops.linear_dx(dq, W[:d], residual=dres_q, wt=None if WT is None else WT[:, :d])
        return dxq, dkv

    def _ref_backward(self, dy, B, S, st, sd, wjobs):
        cfg = self.cfg
        p = cfg.dropout
        # norm3(x2 + drop(f)); the linear2 bias grad (column sums of the branch gradient)
        # accumulates in the same pass
        ds3, df = ops.norm_bwd(dy, st["s3"], self.w("norm3.weight"), st["mu3"], st["rs3"], dw=self.g("norm3.weight"),
                               dbias=self.g("norm3.bias"), p_drop=p, seed=_seed(sd, 6), want_branch=True,
                               colsum_branch=self.g("linear2.bias"))
        gact, a, x2 = st["g"], st["a"], st["x2"]
        wjobs.append(ops.DW(df, gact, self.g("linear2.weight")))
        # linear2 dX GEMM with dReLU x dropout mask in its epilogue and the linear1 bias
        # grad (column sums of the result) accumulated there too
        da = ops.linear_dx(df, self.w("linear2.weight"), act_input=a, act="relu", wt=self.wt("linear2.weight"),
                           colsum=self.g("linear1.bias"), p_drop=p, seed=_seed(sd, 5))
        wjobs.append(ops.DW(da, x2, self.g("linear1.weight")))
        dx2 = ops.linear_dx(da, self.w("linear1.weight"), residual=ds3, wt=self.wt("linear1.weight"))
        # norm2(x1 + drop(ca))
        ds2, dca = ops.norm_bwd(dx2, st["s2"], self.w("norm2.weight"), st["mu2"], st["rs2"], dw=self.g("norm2.weight"),
                                dbias=self.g("norm2.bias"), p_drop=p, seed=_seed(sd, 4), want_branch=True,
                                colsum_branch=self.g("multihead_attn.out_proj.bias"))
        h, x1 = st["x"], st["x1"]
        dx1, dkv_mem = self._mha_bwd("multihead_attn", dca, x1, h, B, S, _seed(sd, 3), st, "ca_", False, wjobs,
                                     dres_q=ds2, dres_kv=None)
        # norm1(h + drop(sa))
        ds1, dsa = ops.norm_bwd(dx1, st["s1"], self.w("norm1.weight"), st["mu1"], st["rs1"], dw=self.g("norm1.weight"),
                                dbias=self.g("norm1.bias"), p_drop=p, seed=_seed(sd, 2), want_branch=True,
                                colsum_branch=self.g("self_attn.out_proj.bias"))
        dh, _ = self._mha_bwd("self_attn", dsa, h, h, B, S, _seed(sd, 1), st, "sa_", True, wjobs, dres_q=ds1,
                              dres_kv=None)
        # memory = h (helper:52): the cross-attention K/V projections' input gradient
        # accumulates into dh through the residual epilogue of their dX GEMM, in place
        d = cfg.d_model
        W, WT = self.w("multihead_attn.in_proj_weight"), self.wt("multihead_attn.in_proj_weight")
        ops.linear_dx(dkv_mem, W[d:], residual=dh, out=dh, wt=None if WT is None else WT[:, d:])
        return dh


# ======================================================================================
# stage model
# ======================================================================================


# Sustained rates of this engine's kernels on MI355X (profiles/r1_v2_*, r1_v1_kernel_microbench):
# Sustained rates measured on MI355X (profiles/): a layer's projection GEMMs ~900 TF/s,
# the big-N head GEMMs ~1000 (fwd 950, dX 1230, dW 870), causal flash attention at
# D = 64 ~456 fwd / ~359 bwd (in the half-FLOP causal count below), the fused CE ~5.2 TB/s;
# norms / residual / elementwise add ~20 % to a layer.  GPT-2 small, 16K-token microbatch:
# model 3.65 head units vs 3.55 measured (head 4.37 ms, layer 1.23 ms).
_E_GEMM, _E_HEAD, _E_ATTN_F, _E_ATTN_B, _BW_CE = 900e12, 1000e12, 456e12, 359e12, 5.2e12
_LAYER_OVERHEAD = 1.2


def stage_cost_model(cfg: NativeConfig, seq_len: int = 1024) -> Tuple[float, float, float]:
    """(layer, head, embedding) costs in forward-layer units: the pipeline simulator
    prices F = 1, B = 2 per layer unit and a head chunk at 3 x its share of the head.

    Costs are *time* estimates from per-kernel sustained rates, not FLOP ratios: the
    LM head is one large, efficient GEMM family while a layer mixes smaller GEMMs with
    attention, so FLOPs alone overprice the head (GPT-2 small: 5.2 vs ~3.3 measured)."""
    d = cfg.d_model
    mm = d * cfg.qkv_dim + d * d + (3 if cfg.activation == "swiglu" else 2) * d * cfg.d_ff
    attn = 2.0 * seq_len * d * (0.5 if cfg.causal else 1.0)
    if cfg.cross_attn:
        mm += 4 * d * d
        attn *= 2
    t_layer = _LAYER_OVERHEAD * (3 * 2 * mm / _E_GEMM + 2 * attn / _E_ATTN_F + 2.5 * 2 * attn / _E_ATTN_B)
    t_head = 3 * 2 * d * cfg.vocab_padded / _E_HEAD + 2 * 2 * cfg.vocab_padded / _BW_CE
    head_units = t_head / t_layer
    return 1.0, head_units + 0.1, 0.1


def comm_units(cfg: NativeConfig, seq_len: int = 1024, link_gbps: Optional[float] = None,
               latency_us: float = 15.0, tokens: int = 32768) -> float:
    """Transfer time of one microbatch's stage-boundary activation (bf16 [T, d]) in the
    forward-layer units of :func:`stage_cost_model` -- the simulator's p2p latency for the
    head-aware schedule planner.  ``link_gbps``: effective one-direction p2p bandwidth of an
    xGMI link (MIPIPE_LINK_GBPS, default 60: MI355X's 153.6 GB/s link figure counts both
    directions; RCCL p2p reaches ~80 % of a direction).  GPT-2 small: ~1.0 unit, i.e. a
    hop costs about one layer forward."""
    if link_gbps is None:
        link_gbps = float(os.environ.get("MIPIPE_LINK_GBPS", "60"))
    d = cfg.d_model
    mm = d * cfg.qkv_dim + d * d + (3 if cfg.activation == "swiglu" else 2) * d * cfg.d_ff
    attn = 2.0 * seq_len * d * (0.5 if cfg.causal else 1.0)
    if cfg.cross_attn:
        mm += 4 * d * d
        attn *= 2
    t_layer = _LAYER_OVERHEAD * (3 * 2 * mm / _E_GEMM + 2 * attn / _E_ATTN_F + 2.5 * 2 * attn / _E_ATTN_B)
    unit = tokens * t_layer / 3.0                 # one layer forward of the microbatch
    msg = tokens * d * 2 / (link_gbps * 1e9) + latency_us * 1e-6
    return msg / unit


def balanced_layer_ranges(cfg: NativeConfig, num_stages: int, seq_len: int = 1024,
                          reference_rule: bool = False, head_on_last: bool = True,
                          ranks: Optional[int] = None) -> List[Tuple[int, int]]:
    """Layer ranges per stage.

    ``reference_rule``: ``L // num_stages`` per stage, remainder on the last stage
    (reference helper:70-75).  Otherwise a cost-balanced split: the embedding and the
    LM head (+ loss) are priced in layer-equivalents from their FLOPs and the layers are
    distributed so the max stage cost is minimal (the head of a 50k-vocab GPT-2 costs
    ~4.5 layers; leaving it out of the balance is what makes naive PP=8 splits slow).

    ``ranks`` (virtual stages, ``num_stages = ranks x v`` in loop placement, stage s on
    rank s % ranks): what bounds the pipeline is a RANK's summed work, so the one-layer
    remainders go to the stages of the least-loaded ranks and the split minimises the
    max rank load first, then the max stage cost, and prefers no empty stage (GPT-2
    small, P = 4, v = 2: [1,1,1,2,2,2,2,1] -- every rank 3 layers -- instead of
    [1,1,2,2,2,2,2,0], which leaves one rank 2 and another 4)."""
    L = cfg.n_layers
    if reference_rule or num_stages == 1:
        per = L // num_stages
        return [(s * per, (s + 1) * per if s < num_stages - 1 else L) for s in range(num_stages)]
    _, head_cost, emb_cost = stage_cost_model(cfg, seq_len)
    if not head_on_last:  # distributed head (parallel/headsplit.py): only the final norm stays
        head_cost = 0.1
    P = num_stages
    multi = ranks is not None and 1 < ranks < P
    best = None
    for k_last in range(0, L + 1):
        rest = L - k_last
        base, extra = divmod(rest, P - 1)
        if not multi:
            # give the remainder to the later non-head stages (stage 0 also holds the embedding)
            counts = [base + (1 if s >= P - 1 - extra else 0) for s in range(P - 1)] + [k_last]
        else:
            counts = [base] * (P - 1) + [k_last]
            load = [0.0] * ranks
            for s, c in enumerate(counts):
                load[s % ranks] += c + (emb_cost if s == 0 else 0.0) + (head_cost if s == P - 1 else 0.0)
            for _ in range(extra):
                # the +1 goes to the least-loaded rank's latest stage without one yet
                cand = [s for s in range(P - 1) if counts[s] == base]
                s = min(cand, key=lambda t: (load[t % ranks], -t))
                counts[s] += 1
                load[s % ranks] += 1
        costs = [c + (emb_cost if s == 0 else 0.0) + (head_cost if s == P - 1 else 0.0)
                 for s, c in enumerate(counts)]
        if multi:
            rload = [sum(costs[s] for s in range(P) if s % ranks == r) for r in range(ranks)]
            key = (round(max(rload), 6), round(max(costs), 6), -min(counts))
        else:
            key = (round(max(costs), 6), -min(counts[:-1]) if P > 1 else 0)
        if best is None or key < best[0]:
            best = (key, counts)
    out, start = [], 0
    for k in best[1]:
        out.append((start, start + k))
        start += k
    return out


def head_param_specs(cfg: NativeConfig) -> List[ParamSpec]:
    d = cfg.d_model
    if cfg.tie_embeddings:
        return [ParamSpec("tok_embeddings.weight", (cfg.vocab_padded, d), "normal", False, cfg.init_std, True)]
    out = [ParamSpec("output.weight", (cfg.vocab_padded, d), "normal", True, cfg.init_std, True)]
    if cfg.bias and cfg.cross_attn:
        out.append(ParamSpec("output.bias", (cfg.vocab_padded,), "zeros", False))
    return out


# MIPIPE_FUSED_MERGE_NORM=0: merge the lane gradients without the fused sum of squares (the
# optimizer then makes its own pass for the clipping norm) -- the A/B switch of the fusion.
_FUSED_MERGE_NORM = os.environ.get("MIPIPE_FUSED_MERGE_NORM", "1") != "0"

# MIPIPE_HEAD_CHUNK: how the last stage runs its LM head + CE.
#   -1 (default): logits GEMM + fused CE in the forward, the dX / dW GEMMs in the backward
#       (the [T, Vp] dlogits live from F to B);
#    0: head forward AND backward inside the forward action, one chunk: only dL/dh
#       ([T, D]) is stashed, the logits are transient;
#    N: the same in token chunks of N (a chunk's logits fit the 256 MB Infinity Cache).
# Measured, GPT-2 small bench, 1 GPU (profiles/r2_head_chunk_ab.txt): -1 834K tok/s,
# 8192 810K, 4096 793K, 2048 788K -- the smaller dX / dW GEMMs cost more than the
# logits traffic saves, and 288 GB of HBM holds the stash; chunking is for memory-bound
# configurations (long sequences, large vocabularies, deep 1F1B stashes).
_HEAD_CHUNK = int(os.environ.get("MIPIPE_HEAD_CHUNK", "-1"))


def head_fwd_bwd(h: torch.Tensor, target: torch.Tensor, W: torch.Tensor, Wt: Optional[torch.Tensor],
                 hb: Optional[torch.Tensor], gW: torch.Tensor, gb: Optional[torch.Tensor], dh_out: torch.Tensor,
                 vocab: int, grad_scale: float, loss_out: torch.Tensor, chunk: int = 0,
                 ov: Optional["WGradOverlap"] = None) -> None:
    """LM head + softmax-CE forward AND backward for the rows of ``h`` [T, D]: per token
    chunk, logits = h W^T (+ hb) -> fused CE (row losses into ``loss_out``, dlogits in
    place) -> dh = dlogits W into ``dh_out`` and gW (+= dlogits^T h), gb (+= colsum).
    With ``ov`` the weight-gradient GEMMs run on its side stream (the caller joins)."""
    T = h.shape[0]
    step = T if chunk <= 0 else min(chunk, T)
    for c0 in range(0, T, step):
        r = slice(c0, min(T, c0 + step))
        hc = h[r]
        logits, _ = ops.linear(hc, W, hb)
        ops.xent_fwd_bwd(logits, target[r], vocab, grad_scale=grad_scale, loss=loss_out[r])
        jobs = [ops.DW(logits, hc, gW)]
        if gb is not None:
            jobs.append(lambda lg=logits: ops.colsum(lg, gb))
        if ov is not None:
            ov.run(jobs)
        ops.linear_dx(logits, W, out=dh_out[r], wt=Wt)
        if ov is None:
            for j in jobs:
                j()


class HeadShard:
    """LM head + loss replicated on every pipeline rank (distributed head,
    parallel/headsplit.py).  Runs one token chunk of a microbatch: logits, fused
    softmax-CE fwd+bwd, input grad (returned to the last stage) and weight grad
    (accumulated locally, all-reduced once per step).  With tied embeddings the
    first stage's embedding reads/updates this same arena."""

    def __init__(self, cfg: NativeConfig, device, seed: int = 0, dtype=torch.bfloat16, init: bool = True,
                 shards: int = 1):
        self.cfg = cfg
        self.device = torch.device(device)
        # numel divisible by 8 x shards: equal, 16-byte aligned blocks for the ZeRO-1
        # reduce-scatter / all-gather over the pipeline group (engine.py)
        self.arena = ParamArena(head_param_specs(cfg), self.device, dtype=dtype, seed=seed, init=init,
                                numel_multiple=8 * max(1, shards))
        self.wname = "tok_embeddings.weight" if cfg.tie_embeddings else "output.weight"

    def weight(self):
        return self.arena.w(self.wname)

    def run(self, h: torch.Tensor, target: torch.Tensor, dh_out: torch.Tensor, grad_scale: float) -> torch.Tensor:
        """h [Tc, D] final-norm output rows, target [Tc] ids; writes dL/dh into
        ``dh_out`` and returns the chunk's summed token loss (f32 scalar tensor)."""
        A = self.arena
        hb = A.w("output.bias") if A.has("output.bias") else None
        row_loss = torch.empty(h.shape[0], device=h.device, dtype=torch.float32)
        head_fwd_bwd(h, target.reshape(-1), self.weight(), A.wt(self.wname), hb, A.g(self.wname),
                     A.g("output.bias") if hb is not None else None, dh_out, self.cfg.vocab_size, grad_scale,
                     row_loss, chunk=_HEAD_CHUNK)
        return row_loss.sum()


class NativeModel:
    """The part of a model that one pipeline stage owns (embedding on stage 0, head +
    loss on the last stage), with explicit fwd/bwd per microbatch."""

    def __init__(self, cfg: NativeConfig, stage_index: int, num_stages: int, device, layer_range=None,
                 seed: int = 0, recompute: bool = False, mbs: int = 1, seq_len: int = 1024, init: bool = True,
                 dtype=torch.bfloat16, head: Optional[HeadShard] = None, arena_multiple: int = 8):
        self.cfg = cfg
        self.stage_index = stage_index
        self.num_stages = num_stages
        self.first = stage_index == 0
        self.last = stage_index == num_stages - 1
        # distributed head: the last stage stops at the final norm, the (tied) vocab
        # matrix lives in the shared HeadShard arena
        self.head = head
        self.split_head = head is not None
        # dW GEMMs of a backward on the side stream (WGradOverlap); off with microbatch
        # lanes, where a second microbatch fills the CUs instead and a graph that forks onto
        # a side stream measured no concurrency with the other lane's graphs
        self.wgrad_side = True
        self.device = torch.device(device)
        if layer_range is None:
            layer_range = balanced_layer_ranges(cfg, num_stages, seq_len)[stage_index]
        self.layer_range = layer_range
        # activation recompute: True / False (every layer / none), or an int k -- the first k
        # local layers keep only their input and rebuild their stash in the backward
        # (selective, engine.plan_recompute picks k from the HBM plan)
        n_local = layer_range[1] - layer_range[0]
        self.recompute_layers = (n_local if recompute is True else 0) if isinstance(recompute, bool) or \
            recompute is None else max(0, int(recompute))
        self.recompute = self.recompute_layers > 0
        specs: List[ParamSpec] = []
        d = cfg.d_model
        if self.first:
            if not (self.split_head and cfg.tie_embeddings):
                specs.append(ParamSpec("tok_embeddings.weight", (cfg.vocab_padded, d), "normal", False,
                                       cfg.init_std, cfg.tie_embeddings and self.last))
            if cfg.pos == "learned":
                specs.append(ParamSpec("pos_embeddings.weight", (cfg.max_seq_len, d), "normal", False, 0.01))
        for i in range(*layer_range):
            specs += block_param_specs(cfg, i)
        if self.last:
            if cfg.final_norm:
                specs.append(ParamSpec("norm.weight", (d,), "ones", False))
                if cfg.norm == "layernorm":
                    specs.append(ParamSpec("norm.bias", (d,), "zeros", False))
            if self.split_head:
                pass
            elif cfg.tie_embeddings:
                if not self.first:  # tied copy on the last stage, kept in sync by the embed group
                    specs.append(ParamSpec("tok_embeddings.weight", (cfg.vocab_padded, d), "normal", False,
                                           cfg.init_std, True))
            else:
                specs.append(ParamSpec("output.weight", (cfg.vocab_padded, d), "normal", True, cfg.init_std, True))
                if cfg.bias and cfg.cross_attn:
                    specs.append(ParamSpec("output.bias", (cfg.vocab_padded,), "zeros", False))
        # arena_multiple: 8 x DP when the arena is ZeRO-1-sharded over DP replicas (equal,
        # 16-byte aligned blocks for the reduce-scatter / all-gather, engine.py)
        self.arena = ParamArena(specs, self.device, dtype=dtype, seed=seed, init=init, numel_multiple=arena_multiple)
        rope = None
        if cfg.pos == "rope":
            rope = ops.rope_tables(cfg.max_seq_len, cfg.head_dim, cfg.rope_theta, self.device)
        self.blocks = [Block(cfg, i, self.arena, rope) for i in range(*layer_range)]
        self.defer_w: Dict[int, list] = {}

    # ------------------------------------------------------------------ helpers
    def _emb_arena(self) -> ParamArena:
        if self.split_head and self.cfg.tie_embeddings:
            return self.head.arena
        return self.arena

    def head_weight(self):
        return self.arena.w("tok_embeddings.weight" if self.cfg.tie_embeddings else "output.weight")

    def head_weight_t(self):
        return self.arena.wt("tok_embeddings.weight" if self.cfg.tie_embeddings else "output.weight")

    def head_grad(self):
        return self.arena.g("tok_embeddings.weight" if self.cfg.tie_embeddings else "output.weight")

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, ctx: MBContext, B: int, S: int, target: Optional[torch.Tensor] = None,
                loss_scale: float = 1.0, keep_logits: bool = False):
        """x: tokens [B,S] (stage 0) or hidden [B*S, D].  Last stage: returns the mean
        loss (f32 scalar tensor) and keeps dlogits for the backward (the fused CE writes
        the gradient over the logits; ``keep_logits`` saves a copy first, in
        ``ctx.misc['logits_out']``, for callers that want the outputs too)."""
        cfg = self.cfg
        if self.first:
            tokens = x.reshape(-1)
            h = ops.embed_fwd(tokens, self._emb_arena().w("tok_embeddings.weight"),
                              self.arena.w("pos_embeddings.weight") if cfg.pos == "learned" else None, S)
            ctx.misc["tokens"] = tokens
        else:
            h = x
        for li, blk in enumerate(self.blocks):
            h = blk.forward(h, B, S, ctx, recompute=li < self.recompute_layers)
        if not self.last:
            return h
        # final norm + head + fused CE (grad computed now, consumed by the backward)
        if cfg.final_norm:
            hn, _, mu, rs = ops.norm_fwd(h, self.arena.w("norm.weight"),
                                         self.arena.w("norm.bias") if self.arena.has("norm.bias") else None,
                                         kind=cfg.norm, eps=cfg.norm_eps)
            ctx.misc.update(hpre=h, mu=mu, rs=rs)
        else:
            hn = h
        if self.split_head:  # the head runs as distributed chunks (HeadShard.run)
            return hn
        hb = self.arena.w("output.bias") if self.arena.has("output.bias") else None
        T = hn.shape[0]
        if target is not None and not keep_logits and _HEAD_CHUNK >= 0:
            # fused head: forward + backward of the LM head and CE now, chunk by chunk; the
            # backward starts from dhn (no [T, V] logits kept)
            dhn = torch.empty_like(hn)
            row_loss = torch.empty(T, device=hn.device, dtype=torch.float32)
            ov = WGradOverlap.make(self.device, self.wgrad_side)
            head_fwd_bwd(hn, target.reshape(-1), self.head_weight(), self.head_weight_t(), hb, self.head_grad(),
                         self.arena.g("output.bias") if hb is not None else None, dhn, cfg.vocab_size,
                         loss_scale / T, row_loss, chunk=_HEAD_CHUNK, ov=ov)
            if ov is not None:
                ov.join()
            ctx.misc.update(dhn=dhn)
            return ops.mean(row_loss)
        logits, _ = ops.linear(hn, self.head_weight(), hb)
        if target is None:
            ctx.misc.update(hn=hn, logits=logits)
            return logits
        if keep_logits:   # (into the caller's persistent buffer when it gives one: a plain device copy)
            dst = ctx.misc.pop("logits_dst", None)
            ctx.misc["logits_out"] = dst.copy_(logits) if dst is not None else logits.clone()
        row_loss = ops.xent_fwd_bwd(logits, target.reshape(-1), cfg.vocab_size, grad_scale=loss_scale / T)
        ctx.misc.update(hn=hn, dlogits=logits)
        return ops.mean(row_loss)

    # ------------------------------------------------------------------ backward
    def backward(self, dy: Optional[torch.Tensor], ctx: MBContext, B: int, S: int, weight_grads: bool = True):
        cfg = self.cfg
        defer: List = []
        ov = WGradOverlap.make(self.device, weight_grads and self.wgrad_side)   # dW GEMMs on a side stream
        if self.last and self.split_head:
            # dy = dL/d(final-norm output), gathered from the head chunks
            if cfg.final_norm:
                dy, _ = ops.norm_bwd(dy, ctx.misc.pop("hpre"), self.arena.w("norm.weight"), ctx.misc.pop("mu"),
                                     ctx.misc.pop("rs"), kind=cfg.norm, dw=self.arena.g("norm.weight"),
                                     dbias=self.arena.g("norm.bias") if self.arena.has("norm.bias") else None)
        elif self.last and "dhn" in ctx.misc:
            # the fused head already produced dL/d(final-norm output) in the forward
            dhn = ctx.misc.pop("dhn")
            if cfg.final_norm:
                dy, _ = ops.norm_bwd(dhn, ctx.misc.pop("hpre"), self.arena.w("norm.weight"), ctx.misc.pop("mu"),
                                     ctx.misc.pop("rs"), kind=cfg.norm, dw=self.arena.g("norm.weight"),
                                     dbias=self.arena.g("norm.bias") if self.arena.has("norm.bias") else None)
            else:
                dy = dhn
        elif self.last:
            dl = ctx.misc.pop("dlogits")
            hn = ctx.misc.pop("hn")
            W = self.head_weight()
            jobs = [ops.DW(dl, hn, self.head_grad())]
            if self.arena.has("output.bias"):
                jobs.append(lambda dl=dl: ops.colsum(dl, self.arena.g("output.bias")))
            if ov is not None:
                ov.run(jobs)    # the head dW runs beside the head dX GEMM
            dhn = ops.linear_dx(dl, W, wt=self.head_weight_t())
            if ov is not None:
                pass    # already issued
            elif weight_grads:
                for j in jobs:
                    j()
            else:
                defer.extend(jobs)
            if cfg.final_norm:
                dy, _ = ops.norm_bwd(dhn, ctx.misc.pop("hpre"), self.arena.w("norm.weight"), ctx.misc.pop("mu"),
                                     ctx.misc.pop("rs"), kind=cfg.norm, dw=self.arena.g("norm.weight"),
                                     dbias=self.arena.g("norm.bias") if self.arena.has("norm.bias") else None)
            else:
                dy = dhn
        for blk in reversed(self.blocks):
            dy = blk.backward(dy, B, S, ctx, weight_grads=weight_grads, defer=defer, ov=ov)
        if ov is not None:
            # close the fork before the embedding gradient: with tied weights it
            # accumulates into the head's dW buffer
            ov.join()
        if self.first:
            tokens = ctx.misc.pop("tokens")
            ea = self._emb_arena()
            jobs = [lambda dy=dy, tokens=tokens: ops.embed_bwd(
                tokens, dy, ea.g("tok_embeddings.weight"),
                self.arena.g("pos_embeddings.weight") if cfg.pos == "learned" else None, S)]
            if weight_grads:
                jobs[0]()
            else:
                defer.extend(jobs)
            dy = None
        if not weight_grads:
            self.defer_w[ctx.mb] = defer
        return dy

    def backward_weight(self, mb: int):
        ops.run_wjobs(self.defer_w.pop(mb, []))
