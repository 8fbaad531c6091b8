"""Model configurations for the native (HIP-kernel, explicit-backward) model family.

One transformer description covers the three architectures the framework targets:

* ``reference(L, H)`` -- the reference's toy model (helper:23-55): post-LN
  ``nn.TransformerDecoderLayer`` blocks (self-attn, cross-attn with memory = the
  block input, ReLU FFN 2048, dropout 0.1), vocab 10000, untied head.
* ``gpt2(size)`` -- GPT-2 small/medium/large/xl: pre-LN, causal, GELU(tanh), learned
  positions, tied embeddings, vocab 50257 padded to 50304 for the GEMMs.
* ``llama3(size)`` -- Llama-3 (8B, and a 1B-class config): pre-RMSNorm, causal GQA,
  RoPE (theta 500000), SwiGLU, no biases, untied head, vocab 128256.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field
from typing import Optional


def _pad(n: int, m: int = 64) -> int:
    return (n + m - 1) // m * m


@dataclass
class NativeConfig:
    name: str = "custom"
    vocab_size: int = 50257
    d_model: int = 768
    n_layers: int = 12
    n_heads: int = 12
    n_kv_heads: Optional[int] = None
    d_ff: int = 3072
    max_seq_len: int = 1024
    norm: str = "layernorm"          # layernorm | rmsnorm
    norm_eps: float = 1e-5
    pre_norm: bool = True
    activation: str = "gelu_tanh"    # gelu_tanh | relu | swiglu
    pos: str = "learned"             # learned | rope | none
    rope_theta: float = 10000.0
    causal: bool = True
    cross_attn: bool = False         # reference block: cross-attention over the block input
    dropout: float = 0.0
    bias: bool = True
    tie_embeddings: bool = True
    final_norm: bool = True
    init_std: float = 0.02
    vocab_padded: int = field(default=0)

    def __post_init__(self):
        if self.n_kv_heads is None:
            self.n_kv_heads = self.n_heads
        if not self.vocab_padded:
            self.vocab_padded = _pad(self.vocab_size)
        if self.d_model % self.n_heads:
            raise ValueError("d_model must be divisible by n_heads")
        if self.n_heads % self.n_kv_heads:
            raise ValueError("n_heads must be divisible by n_kv_heads")

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    @property
    def qkv_dim(self) -> int:
        return (self.n_heads + 2 * self.n_kv_heads) * self.head_dim

    def to_dict(self):
        return asdict(self)

    # ------------------------------------------------------------------ presets
    @staticmethod
    def reference(n_layers: int = 8, n_heads: int = 8, dim: int = 768, vocab_size: int = 10000,
                  dropout: float = 0.1, dim_feedforward: int = 2048) -> "NativeConfig":
        return NativeConfig(name=f"reference-L{n_layers}-H{n_heads}", vocab_size=vocab_size, d_model=dim,
                            n_layers=n_layers, n_heads=n_heads, d_ff=dim_feedforward, max_seq_len=4096,
                            norm="layernorm", pre_norm=False, activation="relu", pos="none", causal=False,
                            cross_attn=True, dropout=dropout, bias=True, tie_embeddings=False, final_norm=True,
                            vocab_padded=_pad(vocab_size))

    @staticmethod
    def gpt2(size: str = "small", **kw) -> "NativeConfig":
        dims = {"small": (768, 12, 12), "medium": (1024, 24, 16), "large": (1280, 36, 20), "xl": (1600, 48, 25),
                "tiny": (128, 4, 4)}
        d, L, H = dims[size]
        base = dict(name=f"gpt2-{size}", vocab_size=50257, d_model=d, n_layers=L, n_heads=H, d_ff=4 * d,
                    max_seq_len=1024, norm="layernorm", pre_norm=True, activation="gelu_tanh", pos="learned",
                    causal=True, bias=True, tie_embeddings=True)
        base.update(kw)
        return NativeConfig(**base)

    @staticmethod
    def llama3(size: str = "8b", **kw) -> "NativeConfig":
        dims = {"8b": (4096, 32, 32, 8, 14336), "1b": (2048, 16, 32, 8, 8192), "tiny": (256, 4, 8, 2, 512)}
        d, L, H, KV, F = dims[size]
        base = dict(name=f"llama3-{size}", vocab_size=128256, d_model=d, n_layers=L, n_heads=H, n_kv_heads=KV,
                    d_ff=F, max_seq_len=8192, norm="rmsnorm", pre_norm=True, activation="swiglu", pos="rope",
                    rope_theta=500000.0, causal=True, bias=False, tie_embeddings=False)
        base.update(kw)
        return NativeConfig(**base)

    @staticmethod
    def by_name(name: str, **kw) -> "NativeConfig":
        n = name.lower()
        if n.startswith("gpt2"):
            size = n.split("-", 1)[1] if "-" in n else "small"
            return NativeConfig.gpt2(size, **kw)
        if n.startswith("llama"):
            size = n.split("-", 1)[1] if "-" in n else "8b"
            return NativeConfig.llama3(size, **kw)
        if n.startswith("ref"):
            return NativeConfig.reference(**kw)
        raise ValueError(f"unknown model {name!r}")

    # ------------------------------------------------------------------ accounting
    def layer_params(self) -> int:
        d, f = self.d_model, self.d_ff
        b = 1 if self.bias else 0
        p = d * self.qkv_dim + b * self.qkv_dim + d * d + b * d
        if self.cross_attn:
            p += 3 * d * d + 3 * b * d + d * d + b * d
        if self.activation == "swiglu":
            p += 3 * d * f
        else:
            p += 2 * d * f + b * (f + d)
        nn = 3 if self.cross_attn else 2
        p += nn * d * (2 if self.norm == "layernorm" else 1)
        return p

    def n_params(self) -> int:
        d = self.d_model
        p = self.vocab_size * d + self.n_layers * self.layer_params()
        if self.pos == "learned":
            p += self.max_seq_len * d
        if self.final_norm:
            p += d * (2 if self.norm == "layernorm" else 1)
        if not self.tie_embeddings:
            p += self.vocab_size * d + (self.vocab_size if self.bias and self.cross_attn else 0)
        return p

    def stash_bytes_per_layer(self, tokens: int, recompute: bool = False) -> int:
        """bf16 activations one layer keeps for its backward, per microbatch of ``tokens``
        (models/native.py Block.forward stash): layer input, norm outputs, QKV, attention
        output, FFN pre-activation / gate tensors.  With full recompute only the input."""
        d, f = self.d_model, self.d_ff
        if recompute:
            return 2 * tokens * d
        if self.activation == "swiglu":
            ffn = 3 * f                    # gate|up (2f) + activated (f)
        else:
            ffn = 2 * f                    # pre-activation + activated
        per_tok = 5 * d + self.qkv_dim + ffn
        if self.cross_attn:                # second attention block: q/kv projections, output, norm
            per_tok += 3 * d + 2 * d
        return 2 * tokens * per_tok

    def wgrad_stash_bytes_per_layer(self, tokens: int) -> int:
        """bf16 output gradients one layer keeps from its input-gradient half (I) to its
        weight-gradient half (W) of a split backward (ZBH1 / ZBV; models/native.py deferred
        ``wjobs``): the GEMMs' dY -- QKV, attention output, FFN in (2 for SwiGLU) and out."""
        d, f = self.d_model, self.d_ff
        per_tok = self.qkv_dim + d + (2 * f if self.activation == "swiglu" else f) + d
        if self.cross_attn:
            per_tok += 3 * d + d
        return 2 * tokens * per_tok

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token (fwd+bwd = 3x fwd), incl. attention and the LM head."""
        d = self.d_model
        mm = d * self.qkv_dim + d * d + (3 if self.activation == "swiglu" else 2) * d * self.d_ff
        attn = 2 * seq_len * d * (0.5 if self.causal else 1.0)  # QK^T + PV per token, /2 causal
        if self.cross_attn:
            mm += 4 * d * d
            attn *= 2
        fwd = self.n_layers * (2 * mm + 2 * attn) + 2 * d * self.vocab_size
        return 3.0 * fwd
