"""Typed run configuration: model / parallel / train sections as
dataclasses, loadable from YAML or JSON, overridable from the command line.

The reference hard-codes everything (m=4 at helper:214, 2 warmup iterations at
helper:113, batch 32 / seq 128 at nb:306, sweep lists at nb:346-349, port 29500 at
helper:169).  Here every one of those is a field; ``RunConfig.reference_compat()``
reproduces the reference defaults.

    cfg = RunConfig.load("configs/gpt2_small_pp4.yaml", overrides=["parallel.pp=8", "train.steps=20"])
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field, fields, is_dataclass
from typing import Any, Dict, List, Optional, Sequence, Union


@dataclass
class ModelSection:
    name: str = "gpt2-small"            # NativeConfig.by_name: gpt2-{tiny,small,medium,large,xl}, llama3-{...}, ref
    overrides: Dict[str, Any] = field(default_factory=dict)   # NativeConfig field overrides


@dataclass
class ParallelSection:
    pp: int = 1
    dp: int = 1
    schedule: str = "1F1B"              # GPipe | 1F1B | Interleaved1F1B | LoopedBFS | ZBH1 | ZBV | auto (engine.pick_schedule)
    microbatches: Optional[int] = None  # default 2*pp
    v: Optional[int] = None             # virtual stages per rank (interleaved)
    style: str = "loop"                 # stage placement: loop | v
    split_head: Optional[bool] = None   # distributed LM head (default on for pp > 1)
    layer_ranges: Optional[List[List[int]]] = None


@dataclass
class TrainSection:
    micro_batch: int = 8
    seq_len: int = 1024
    steps: int = 100
    lr: float = 3e-4
    min_lr: float = 3e-5
    warmup_steps: int = 10
    lr_schedule: str = "cosine"         # cosine | constant
    weight_decay: float = 0.1
    max_grad_norm: float = 1.0
    # True (every layer), False, "auto" (selective: the fewest recomputed layers per stage the
    # HBM plan needs, engine.plan_recompute) or an int k (the first k layers of every stage)
    recompute: Union[bool, str, int] = False
    graphs: Optional[bool] = None       # HIP-graph replay + native stage runner (None: on for GPU)
    seed: int = 0
    data: str = "synthetic"             # synthetic | pattern[:K] (learnable permutation walk) | path to a uint16/int32 token file (memory-mapped)
    log_every: int = 10
    metrics_file: Optional[str] = None  # JSONL, one record per logged step
    ckpt_dir: Optional[str] = None
    ckpt_every: int = 0
    resume: Optional[str] = None
    watchdog_s: float = 0.0             # abort the job if a step takes longer (0 = off)


@dataclass
class RunConfig:
    model: ModelSection = field(default_factory=ModelSection)
    parallel: ParallelSection = field(default_factory=ParallelSection)
    train: TrainSection = field(default_factory=TrainSection)

    # ------------------------------------------------------------------ presets
    @staticmethod
    def reference_compat(n_layers: int = 8, n_heads: int = 8, pp: int = 2, schedule: str = "1F1B") -> "RunConfig":
        """The reference's hard-coded experiment (helper:98-235, nb:306-372): post-LN
        decoder layers with layer(h, h), vocab 10000, batch 32 = 4 microbatches x 8,
        seq 128, dropout 0.1."""
        return RunConfig(
            model=ModelSection("ref", dict(n_layers=n_layers, n_heads=n_heads, dim=768, vocab_size=10000)),
            parallel=ParallelSection(pp=pp, schedule=schedule, microbatches=4, split_head=False),
            train=TrainSection(micro_batch=8, seq_len=128, steps=5, lr_schedule="constant", warmup_steps=0))

    # ------------------------------------------------------------------ io
    def to_dict(self) -> dict:
        return asdict(self)

    @staticmethod
    def from_dict(d: dict) -> "RunConfig":
        cfg = RunConfig()
        for sec in ("model", "parallel", "train"):
            if sec in d and d[sec] is not None:
                _assign(getattr(cfg, sec), d[sec], sec)
        unknown = set(d) - {"model", "parallel", "train"}
        if unknown:
            raise KeyError(f"unknown config sections {sorted(unknown)}")
        return cfg

    @staticmethod
    def load(path: Optional[str] = None, overrides: Sequence[str] = ()) -> "RunConfig":
        d: dict = {}
        if path:
            with open(path) as f:
                text = f.read()
            if path.endswith((".yaml", ".yml")):
                import yaml
                d = yaml.safe_load(text) or {}
            else:
                d = json.loads(text)
        cfg = RunConfig.from_dict(d)
        for ov in overrides:
            cfg.set(ov)
        return cfg

    def save(self, path: str) -> None:
        with open(path, "w") as f:
            if path.endswith((".yaml", ".yml")):
                import yaml
                yaml.safe_dump(self.to_dict(), f, sort_keys=False)
            else:
                json.dump(self.to_dict(), f, indent=1)

    def set(self, assignment: str) -> None:
        """``section.field=value`` (value parsed as YAML: ints, floats, bools, lists, null);
        ``model.overrides.<key>=value`` sets a model-config override."""
        import yaml
        key, _, raw = assignment.partition("=")
        if not _:
            raise ValueError(f"override {assignment!r} is not key=value")
        val = yaml.safe_load(raw)
        if isinstance(val, str):  # YAML 1.1 reads "1e-3" as a string
            try:
                val = float(val)
            except ValueError:
                pass
        parts = key.strip().split(".")
        if parts[:2] == ["model", "overrides"] and len(parts) == 3:
            self.model.overrides[parts[2]] = val
            return
        if len(parts) != 2 or parts[0] not in ("model", "parallel", "train"):
            raise KeyError(f"bad override key {key!r} (use section.field)")
        _assign(getattr(self, parts[0]), {parts[1]: val}, parts[0])

    # ------------------------------------------------------------------ derived
    def native_config(self):
        from .models.config import NativeConfig
        return NativeConfig.by_name(self.model.name, **self.model.overrides)

    @property
    def microbatches(self) -> int:
        p = self.parallel
        return p.microbatches if p.microbatches is not None else max(2, 2 * p.pp)


def _assign(obj, values: dict, where: str) -> None:
    names = {f.name for f in fields(obj)}
    for k, v in values.items():
        if k not in names:
            raise KeyError(f"unknown field {where}.{k}")
        setattr(obj, k, v)


def lr_at(step: int, t: TrainSection) -> float:
    """Linear warmup then cosine decay to ``min_lr`` (or constant)."""
    import math
    if t.warmup_steps and step < t.warmup_steps:
        return t.lr * (step + 1) / t.warmup_steps
    if t.lr_schedule == "constant":
        return t.lr
    span = max(1, t.steps - t.warmup_steps)
    frac = min(1.0, (step - t.warmup_steps) / span)
    return t.min_lr + 0.5 * (t.lr - t.min_lr) * (1.0 + math.cos(math.pi * frac))
