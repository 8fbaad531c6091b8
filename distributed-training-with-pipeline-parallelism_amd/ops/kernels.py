"""Op wrappers: GPU -> HIP kernels in ``_C.so``; CPU -> PyTorch f32 reference math."""
from __future__ import annotations

import importlib.util
import math
import os
from typing import Optional, Tuple

import torch

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_EXT = None
_EXT_ERR: Optional[str] = None

ACT = {"none": 0, "gelu_tanh": 1, "gelu": 1, "relu": 2}
EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RELU, EPI_BIAS_RES, EPI_RES, EPI_DGELU, EPI_DRELU = range(8)
LOG2E = 1.4426950408889634

# GEMM backend for plain (epilogue-free) GEMMs on GPU: "hip" (default: our MFMA engines),
# "blas" (hipBLASLt through torch, also for the dW GEMMs) or "auto": each plain forward /
# dX GEMM shape is timed once on both (outside graph capture) and keeps the faster.
# hipBLASLt wins some isolated K = 768 - 3072 NT shapes by 5-12 %
# (profiles/r2_kernel_microbench.json) but not inside the GPT-2 / reference steps
# (tools/runs/archive/ab_plain_gemm.sh: 883.6K / 889.4K tok/s auto vs 889.9K / 888.1K hip), so "auto"
# stays opt-in.  Fused-epilogue GEMMs always use the HIP kernels.
GEMM_BACKEND = os.environ.get("MIPIPE_GEMM", "hip")
_PLAIN_BEST: dict = {}


def _plain_pick(key, run_hip, run_lib) -> str:
    """Backend of one plain GEMM shape: decided by timing both (3 runs each after a warm
    run, CUDA events) the first time the shape is seen outside graph capture."""
    if GEMM_BACKEND != "auto":
        return GEMM_BACKEND
    d = _PLAIN_BEST.get(key)
    if d is not None:
        return d
    if torch.cuda.is_current_stream_capturing():
        return "hip"
    t = {}
    for name, fn in (("hip", run_hip), ("blas", run_lib)):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            fn()
        e.record()
        e.synchronize()
        t[name] = s.elapsed_time(e)
    d = "blas" if t["blas"] < 0.97 * t["hip"] else "hip"
    _PLAIN_BEST[key] = d
    return d


def plain_gemm_choices() -> dict:
    """{"fwd|dx MxNxK": backend} of the plain GEMM shapes decided so far (bench JSON)."""
    return {f"{k[0]} {k[1]}x{k[2]}x{k[3]}": v for k, v in sorted(_PLAIN_BEST.items())}
# GEMM engine: 2 = 8-wave glds engine (gemm2.hip) with fallback to 1 (gemm.hip) for
# combinations v2 does not instantiate; 1 = always gemm.hip.
GEMM_V = int(os.environ.get("MIPIPE_GEMM_V", "2"))


def load_ext():
    global _EXT, _EXT_ERR
    if _EXT is not None or _EXT_ERR is not None:
        return _EXT
    # MIPIPE_EXT_VARIANT=name loads _C_<name>.so: a build of the same sources with extra
    # compile-time defines (tools/build_ext.py --variant), for in-process A/B of kernel variants
    variant = os.environ.get("MIPIPE_EXT_VARIANT", "")
    path = os.path.join(_PKG_DIR, f"_C_{variant}.so" if variant else "_C.so")
    if not os.path.exists(path):
        _EXT_ERR = f"{path} not found (build it with: python tools/build_ext.py)"
        return None
    try:
        import torch  # noqa: F401  (libtorch must be loaded first)
        spec = importlib.util.spec_from_file_location("mipipe._C", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _EXT = mod
    except Exception as e:  # pragma: no cover - depends on build
        _EXT_ERR = f"failed to load {path}: {e}"
    return _EXT


def ext_available() -> bool:
    return load_ext() is not None


def _ext():
    e = load_ext()
    if e is None:
        raise RuntimeError(f"mipipe HIP extension unavailable on a GPU tensor: {_EXT_ERR}")
    return e


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ======================================================================================
# normalisation (+ fused residual add / dropout)
# ======================================================================================
def _cpu_dropout_mask(shape, p, seed, device):
    g = torch.Generator(device="cpu").manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
    keep = (torch.rand(shape, generator=g) >= p).float() / (1.0 - p)
    return keep.to(device)


def norm_fwd(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
             branch: Optional[torch.Tensor] = None, kind: str = "layernorm", eps: float = 1e-5,
             p_drop: float = 0.0, seed: int = 0, y=None, s=None, mean=None, rstd=None):
    """s = x + dropout(branch) (if branch given); y = norm(s) * w (+ bias).  Returns (y, s, mean, rstd)."""
    rms = kind == "rmsnorm"
    D = x.shape[-1]
    rows = x.numel() // D
    if y is None:
        y = torch.empty_like(x)
    if branch is not None and s is None:
        s = torch.empty_like(x)
    if rstd is None:
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    if mean is None and not rms:
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    if _gpu(x):
        _ext().norm_fwd(rms, x, branch, w, bias, s if branch is not None else None, y, mean, rstd, float(eps),
                        float(p_drop), int(seed))
        return y, (s if branch is not None else x), mean, rstd
    xf = x.float()
    if branch is not None:
        bf = branch.float()
        if p_drop > 0:
            bf = bf * _cpu_dropout_mask(bf.shape, p_drop, seed, x.device)
        xf = (xf + bf).to(x.dtype).float()
        s.copy_(xf.to(x.dtype))
    src = xf.reshape(rows, D)
    mu = torch.zeros(rows) if rms else src.mean(-1)
    var = (src - mu[:, None]).pow(2).mean(-1)
    r = torch.rsqrt(var + eps)
    out = (src - mu[:, None]) * r[:, None] * w.float()
    if bias is not None:
        out = out + bias.float()
    y.copy_(out.reshape(x.shape).to(y.dtype))
    rstd.copy_(r)
    if not rms:
        mean.copy_(mu)
    return y, (s if branch is not None else x), mean, rstd


def norm_bwd(dy: torch.Tensor, s: torch.Tensor, w: torch.Tensor, mean, rstd, kind: str = "layernorm",
             dres: Optional[torch.Tensor] = None, dw: Optional[torch.Tensor] = None,
             dbias: Optional[torch.Tensor] = None, p_drop: float = 0.0, seed: int = 0, ds=None, dbranch=None,
             want_branch: bool = False, colsum_dres: Optional[torch.Tensor] = None,
             colsum_ds: Optional[torch.Tensor] = None, colsum_branch: Optional[torch.Tensor] = None):
    """ds = d(norm input) (+ dres); dw/dbias (f32) accumulate.  Optionally also accumulates
    the column sums of ``dres`` and of ``ds`` (f32) -- the bias grads of the projections
    around this residual point -- in the same pass; ``colsum_branch`` (needs
    ``want_branch``): the column sums of the returned branch gradient (= ds without
    dropout, ds * mask with it).  Returns (ds, dbranch)."""
    rms = kind == "rmsnorm"
    D = dy.shape[-1]
    rows = dy.numel() // D
    if ds is None:
        ds = torch.empty_like(dy)
    need_branch = want_branch and p_drop > 0
    if need_branch and dbranch is None:
        dbranch = torch.empty_like(dy)
    if colsum_branch is not None:
        if not want_branch or colsum_ds is not None:
            raise ValueError("colsum_branch needs want_branch and excludes colsum_ds")
    if _gpu(dy):
        cs_ds = colsum_branch if colsum_branch is not None else colsum_ds
        rc = _ext().norm_bwd(rms, dy, s, w, mean, rstd, dres, ds, dbranch if need_branch else None, dw, dbias,
                             float(p_drop), int(seed), colsum_dres, cs_ds)
        out_branch = dbranch if need_branch else (ds if want_branch else None)
        if rc == -3:     # no fused column sums for this shape: separate passes
            if colsum_dres is not None:
                _ext().colsum(dres, colsum_dres)
            if cs_ds is not None:
                _ext().colsum(out_branch if colsum_branch is not None else ds, cs_ds)
        return ds, out_branch
    d = dy.float().reshape(rows, D)
    x = s.float().reshape(rows, D)
    mu = torch.zeros(rows) if rms else mean.float()
    xh = (x - mu[:, None]) * rstd[:, None]
    g = d * w.float()
    s1 = torch.zeros(rows, 1) if rms else g.mean(-1, keepdim=True)
    s2 = (g * xh).mean(-1, keepdim=True)
    v = rstd[:, None] * (g - s1 - xh * s2)
    if dres is not None:
        v = v + dres.float().reshape(rows, D)
    ds.copy_(v.reshape(dy.shape).to(ds.dtype))
    if colsum_dres is not None:
        colsum_dres += dres.float().reshape(rows, D).sum(0)
    if colsum_ds is not None:
        colsum_ds += ds.float().reshape(rows, D).sum(0)
    if dw is not None:
        dw += (d * xh).sum(0)
    if dbias is not None:
        dbias += d.sum(0)
    if need_branch:
        m = _cpu_dropout_mask(dy.shape, p_drop, seed, dy.device)
        dbranch.copy_((v.reshape(dy.shape) * m).to(dbranch.dtype))
        if colsum_branch is not None:
            colsum_branch += dbranch.float().reshape(rows, D).sum(0)
        return ds, dbranch
    if colsum_branch is not None:
        colsum_branch += ds.float().reshape(rows, D).sum(0)
    return ds, (ds if want_branch else None)


# ======================================================================================
# fused softmax cross-entropy
# ======================================================================================
def xent_fwd_bwd(logits: torch.Tensor, target: torch.Tensor, vocab: int, grad_scale: float,
                 ignore_index: int = -100, write_grad: bool = True, loss: Optional[torch.Tensor] = None):
    """Per-row CE loss (f32 [T]); if write_grad, logits are overwritten IN PLACE by
    (softmax - onehot) * grad_scale (padded vocab columns -> 0)."""
    Vp = logits.shape[-1]
    T = logits.numel() // Vp
    if loss is None:
        loss = torch.empty(T, device=logits.device, dtype=torch.float32)
    if _gpu(logits):
        _ext().xent(logits, target, loss, int(vocab), float(grad_scale), int(ignore_index), bool(write_grad))
        return loss
    lg = logits.float().reshape(T, Vp)[:, :vocab]
    tg = target.reshape(T)
    lse = torch.logsumexp(lg, -1)
    valid = tg != ignore_index
    tsafe = torch.where(valid, tg, torch.zeros_like(tg))
    l = lse - lg.gather(1, tsafe[:, None])[:, 0]
    loss.copy_(torch.where(valid, l, torch.zeros_like(l)))
    if write_grad:
        p = torch.softmax(lg, -1)
        p[torch.arange(T), tsafe] -= 1.0
        p = p * grad_scale * valid[:, None].float()
        out = torch.zeros(T, Vp)
        out[:, :vocab] = p
        logits.copy_(out.reshape(logits.shape).to(logits.dtype))
    return loss


# ======================================================================================
# embeddings
# ======================================================================================
def embed_fwd(idx: torch.Tensor, wte: torch.Tensor, wpe: Optional[torch.Tensor], S: int, pos_offset: int = 0,
              out: Optional[torch.Tensor] = None):
    T = idx.numel()
    D = wte.shape[1]
    if out is None:
        out = torch.empty(T, D, device=wte.device, dtype=wte.dtype)
    if _gpu(wte):
        _ext().embed_fwd(idx.reshape(-1), wte, wpe, out, int(S), int(pos_offset))
        return out
    e = wte.float()[idx.reshape(-1)]
    if wpe is not None:
        pos = torch.arange(T) % S + pos_offset
        e = e + wpe.float()[pos]
    out.copy_(e.to(out.dtype))
    return out


def embed_bwd(idx: torch.Tensor, dout: torch.Tensor, dwte: torch.Tensor, dwpe: Optional[torch.Tensor], S: int,
              pos_offset: int = 0):
    if _gpu(dout):
        _ext().embed_bwd(idx.reshape(-1), dout, dwte, dwpe, int(S), int(pos_offset))
        return
    T = idx.numel()
    d = dout.float().reshape(T, -1)
    dwte.index_add_(0, idx.reshape(-1), d)
    if dwpe is not None:
        pos = torch.arange(T) % S + pos_offset
        dwpe.index_add_(0, pos, d)


# ======================================================================================
# GEMMs (linear layers)
# ======================================================================================
def _gemm(A, B, C, bias=None, residual=None, aux=None, transA=False, transB=False, epi=EPI_NONE, accum=False,
          alpha=1.0, cfg: int = -1, colsum=None, p_drop: float = 0.0, seed: int = 0):
    """``colsum`` (f32 [N]): also accumulate the column sums of the bf16 output (fused in
    the GEMM epilogue where the engine supports it, else one extra pass).  ``p_drop``
    (EPI_BIAS_RELU / EPI_DRELU, contiguous output): dropout after the activation / the
    dropout mask times the activation derivative, regenerated from (seed, element index)
    exactly as act_fwd / act_bwd do."""
    e = _ext()
    if GEMM_V >= 2:
        rc = e.gemm2(A, B, C, bias, residual, aux, bool(transA), bool(transB), int(epi), bool(accum), float(alpha),
                     int(cfg), colsum, float(p_drop), int(seed))
        if rc:
            if rc == 2 and colsum is not None:
                e.colsum(C, colsum)
            return C
    if p_drop > 0:
        raise RuntimeError("GEMM dropout epilogue needs the v2 engine for this shape")
    e.gemm(A, B, C, bias, residual, aux, bool(transA), bool(transB), int(epi), bool(accum), float(alpha))
    if colsum is not None:
        e.colsum(C, colsum)
    return C


# f32 GEMM epilogues (csrc/kernels/gemm_f32.hip mp_gemm_f32_ex)
F32_NONE, F32_BIAS, F32_BIAS_RELU, F32_RES, F32_BIAS_RES, F32_DRELU = range(6)


def _gemm_f32(A, B, C, bias=None, R=None, X=None, epi=F32_NONE, alpha=1.0, accumulate=False, p_drop=0.0, seed=0):
    """C = epi(alpha * A @ B (+ C)) on the f32 MFMA engine; A [M,K], B [K,N] views with a unit
    stride in either dimension.  Raises if the layout is not supported (the f32 GPU path has
    no ATen fallback: the reference-precision numbers must come from our kernels)."""
    if not _ext().gemm_f32_ex(A, B, C, bias, R, X, int(epi), float(alpha), bool(accumulate), float(p_drop), int(seed), 0):
        raise RuntimeError(f"gemm_f32_ex: unsupported layout A{tuple(A.shape)}/{A.stride()} B{tuple(B.shape)}/{B.stride()}")
    return C


def transpose(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = x^T for a 2-D bf16 matrix (row-contiguous views allowed)."""
    if out is None:
        out = torch.empty(x.shape[1], x.shape[0], device=x.device, dtype=x.dtype)
    if _gpu(x):
        _ext().transpose(x, out)
    else:
        out.copy_(x.t())
    return out


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: str = "none",
           residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           aux: Optional[torch.Tensor] = None, p_drop: float = 0.0, seed: int = 0):
    """y = drop(act(x @ w^T + bias)) (+ residual).  x [T,K], w [N,K].  With an activation
    ``aux`` receives what the backward's dX epilogue needs (``linear_dx(act_input=aux)``):
    the pre-activation for ReLU, GELU's derivative at the pre-activation for GELU (one
    sigmoid serves both here; the backward then multiplies).  Unfused, a GELU aux goes to
    ``act_bwd(..., saved="grad")``, a ReLU aux to ``act_bwd(..., saved="pre")``.  ``p_drop``
    (ReLU only) applies the fused dropout of the reference FFN.  Returns (y, aux)."""
    if p_drop > 0 and act != "relu":
        raise ValueError("the fused GEMM dropout follows a ReLU epilogue")
    T, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(T, N, device=x.device, dtype=x.dtype)
    if act != "none" and aux is None:
        aux = torch.empty(T, N, device=x.device, dtype=x.dtype)
    if _gpu(x) and x.dtype == torch.float32:
        # the reference-precision path: f32 MFMA GEMM with the same fused epilogues
        if act not in ("none", "relu"):
            raise ValueError("f32 GEMM epilogues: ReLU only")
        if act == "relu":
            if bias is None or residual is not None:
                raise ValueError("activation epilogue needs a bias and no residual")
            _gemm_f32(x, w.t(), out, bias=bias, X=aux, epi=F32_BIAS_RELU, p_drop=p_drop, seed=seed)
        elif residual is not None:
            _gemm_f32(x, w.t(), out, bias=bias, R=residual, epi=F32_BIAS_RES if bias is not None else F32_RES)
        else:
            _gemm_f32(x, w.t(), out, bias=bias, epi=F32_BIAS if bias is not None else F32_NONE)
        return out, aux
    if _gpu(x):
        if act != "none":
            if bias is None or residual is not None:
                raise ValueError("activation epilogue needs a bias and no residual")
            _gemm(x, w, out, bias=bias, aux=aux, epi=EPI_BIAS_GELU if ACT[act] == 1 else EPI_BIAS_RELU,
                  p_drop=p_drop, seed=seed)
        elif residual is not None:
            _gemm(x, w, out, bias=bias, residual=residual, epi=EPI_BIAS_RES if bias is not None else EPI_RES)
        elif bias is not None:
            _gemm(x, w, out, bias=bias, epi=EPI_BIAS)
        else:
            run_hip = lambda: _gemm(x, w, out)
            run_lib = lambda: torch.mm(x, w.t(), out=out)
            (run_lib if _plain_pick(("fwd", T, N, K), run_hip, run_lib) == "blas" else run_hip)()
        return out, aux
    y = x.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if act != "none":
        pre = y.to(x.dtype)
        aux.copy_(_act_grad_cpu(pre.float(), act) if ACT[act] == 1 else pre)
        y = _act_cpu(pre.float(), act)
        if p_drop > 0:
            y = y * _cpu_dropout_mask(y.shape, p_drop, seed, y.device)
    if residual is not None:
        y = y + residual.float()
    out.copy_(y.to(out.dtype))
    return out, aux


def _act_cpu(x, act):
    if ACT[act] == 1:
        return torch.nn.functional.gelu(x, approximate="tanh")
    if ACT[act] == 2:
        return torch.relu(x)
    return x


def _act_grad_cpu(x, act):
    if ACT[act] == 1:
        k0, k1 = 0.7978845608028654, 0.044715
        u = k0 * (x + k1 * x ** 3)
        t = torch.tanh(u)
        return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)
    if ACT[act] == 2:
        return (x > 0).float()
    return torch.ones_like(x)


def _plain_dx_hip(dy, wt, out):
    T, K = out.shape
    N = dy.shape[1]
    if (T // 256) * (K // 192) < 128 and N >= 4096:
        acc = torch.zeros(T, K, device=dy.device, dtype=torch.float32)
        _gemm(dy, wt, acc, accum=True)
        out.copy_(acc)
    else:
        _gemm(dy, wt, out)
    return out


def linear_dx(dy: torch.Tensor, w: torch.Tensor, act_input: Optional[torch.Tensor] = None, act: str = "none",
              out: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
              wt: Optional[torch.Tensor] = None, colsum: Optional[torch.Tensor] = None, p_drop: float = 0.0,
              seed: int = 0):
    """dx = dy @ w  (w [N,K]), optionally times act'(.) given by ``act_input`` -- what
    ``linear(act=...)`` saved in ``aux``: ReLU's pre-activation, or GELU's derivative itself
    -- and plus ``residual``.  With ``wt`` (= w^T, [K,N], kept by the param arena) the GEMM
    runs in the both-K-contiguous form on the v2 engine."""
    T, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(T, K, device=dy.device, dtype=dy.dtype)
    if _gpu(dy) and dy.dtype == torch.float32:
        if act not in ("none", "relu"):
            raise ValueError("f32 GEMM epilogues: dReLU only")
        if act == "relu":
            if residual is not None:
                raise ValueError("dReLU epilogue takes no residual")
            _gemm_f32(dy, w, out, R=act_input, epi=F32_DRELU, p_drop=p_drop, seed=seed)
        elif residual is not None:
            _gemm_f32(dy, w, out, R=residual, epi=F32_RES)
        else:
            _gemm_f32(dy, w, out)
        if colsum is not None:
            _ext().colsum(out, colsum)
        return out
    if (_gpu(dy) and wt is not None and act == "none" and residual is None and colsum is None and
            _plain_pick(("dx", T, K, N), lambda: _plain_dx_hip(dy, wt, out), lambda: torch.mm(dy, w, out=out)) == "blas"):
        torch.mm(dy, w, out=out)
        return out
    if _gpu(dy) and wt is not None and GEMM_BACKEND != "blas":
        if act == "none" and residual is None and (T // 256) * (K // 192) < 128 and N >= 4096:
            # few output tiles, long reduction (a distributed-head chunk: [Tc, D] = dl[Tc, V] W):
            # split-K into an f32 buffer fills the chip; one cast pass at the end
            acc = torch.zeros(T, K, device=dy.device, dtype=torch.float32)
            _gemm(dy, wt, acc, accum=True)
            out.copy_(acc)
            return out
        if act != "none":
            _gemm(dy, wt, out, aux=act_input, epi=EPI_DGELU if ACT[act] == 1 else EPI_DRELU, colsum=colsum,
                  p_drop=p_drop, seed=seed)
        elif residual is not None:
            _gemm(dy, wt, out, residual=residual, epi=EPI_RES, colsum=colsum)
        else:
            _gemm(dy, wt, out, colsum=colsum)
        return out
    if _gpu(dy):
        if act != "none":
            _gemm(dy, w, out, aux=act_input, transB=True, epi=EPI_DGELU if ACT[act] == 1 else EPI_DRELU,
                  p_drop=p_drop, seed=seed)
        elif residual is not None:
            _gemm(dy, w, out, residual=residual, transB=True, epi=EPI_RES)
        elif GEMM_BACKEND == "blas":
            torch.mm(dy, w, out=out)
        else:
            _gemm(dy, w, out, transB=True)
        if colsum is not None:
            _ext().colsum(out, colsum)
        return out
    g = dy.float() @ w.float()
    if act != "none":
        g = g * (act_input.float() if ACT[act] == 1 else _act_grad_cpu(act_input.float(), act))
        if p_drop > 0:
            g = g * _cpu_dropout_mask(g.shape, p_drop, seed, g.device)
    if residual is not None:
        g = g + residual.float()
    out.copy_(g.to(out.dtype))
    if colsum is not None:
        colsum += out.float().sum(0)
    return out


def linear_dw(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, alpha: float = 1.0):
    """dw (f32 [N,K]) += alpha * dy^T @ x   (dy [T,N], x [T,K])."""
    if _gpu(dy) and dy.dtype == torch.float32:
        return _gemm_f32(dy.t(), x, dw, alpha=alpha, accumulate=True)
    if _gpu(dy):
        if GEMM_BACKEND == "blas":
            dw.add_(torch.mm(dy.t(), x, out_dtype=torch.float32), alpha=alpha)
        else:
            _gemm(dy, x, dw, transA=True, transB=True, accum=True, alpha=alpha)
        return dw
    dw += alpha * (dy.float().t() @ x.float())
    return dw


# ======================================================================================
# f32 linears on the f32-input MFMA (csrc/kernels/gemm_f32.hip) -- the reference-precision
# path for autograd modules (the reference's own f32 model, helper:36-46)
# ======================================================================================
class _LinearF32(torch.autograd.Function):
    """y = x W^T + b with the forward and both backward GEMMs on gemm_f32 (exact f32
    products, f32 accumulate); any layout the kernel does not take falls back to ATen."""

    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        out = torch.empty(x2.shape[0], w.shape[0], device=x.device, dtype=torch.float32)
        if not _ext().gemm_f32(x2, w.t(), out, b, 1.0, False):
            out = torch.addmm(b, x2, w.t()) if b is not None else torch.mm(x2, w.t())
        ctx.save_for_backward(x2, w)
        ctx.has_b = b is not None
        ctx.in_shape = x.shape
        return out.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1])
        if g2.stride(1) != 1:
            g2 = g2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(g2.shape[0], w.shape[1], device=gy.device, dtype=torch.float32)
            if not _ext().gemm_f32(g2, w, dx, None, 1.0, False):
                dx = torch.mm(g2, w)
            dx = dx.view(ctx.in_shape)
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w)
            if not _ext().gemm_f32(g2.t(), x2, dw, None, 1.0, False):
                dw = torch.mm(g2.t(), x2)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = g2.sum(0)
        return dx, dw, db


def linear_f32(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """F.linear for f32 CUDA tensors on the f32 MFMA GEMM (autograd-aware)."""
    return _LinearF32.apply(x, w, b)


class F32Linear(torch.nn.Linear):
    """``nn.Linear`` whose f32 GPU forward/backward run on :func:`linear_f32` (other dtypes
    and CPU: ATen).  Installed by class swap (:func:`use_f32_kernels`): same parameters,
    same state_dict keys."""

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.float32 and self.weight.dtype == torch.float32:
            return _LinearF32.apply(x, self.weight, self.bias)
        return super().forward(x)


def _mha_projected(mod: torch.nn.MultiheadAttention, query, key, value, is_causal: bool, linear):
    """``nn.MultiheadAttention`` forward without attention weights: packed / k-v-shared /
    separate input projections through ``linear``, SDPA core, output projection."""
    same_qkv, same_kv = query is key and key is value, key is value
    if not mod.batch_first:
        query, key, value = (t.transpose(0, 1) for t in (query, key, value))
    B, L, E = query.shape
    H = mod.num_heads
    w, b = mod.in_proj_weight, mod.in_proj_bias

    def part(lo, hi):
        return w[lo:hi], (b[lo:hi] if b is not None else None)
    if same_qkv:
        q, k, v = linear(query, w, b).chunk(3, dim=-1)
    elif same_kv:
        q = linear(query, *part(0, E))
        k, v = linear(key, *part(E, 3 * E)).chunk(2, dim=-1)
    else:
        q = linear(query, *part(0, E))
        k = linear(key, *part(E, 2 * E))
        v = linear(value, *part(2 * E, 3 * E))

    def heads(t):
        return t.reshape(B, t.shape[1], H, E // H).transpose(1, 2)
    o = torch.nn.functional.scaled_dot_product_attention(
        heads(q), heads(k), heads(v), dropout_p=mod.dropout if mod.training else 0.0, is_causal=is_causal)
    o = o.transpose(1, 2).reshape(B, L, E)
    o = linear(o, mod.out_proj.weight, mod.out_proj.bias)
    return o.transpose(0, 1) if not mod.batch_first else o


class F32MultiheadAttention(torch.nn.MultiheadAttention):
    """``nn.MultiheadAttention`` whose input / output projections run on :func:`linear_f32`
    and whose core is SDPA -- the path torch's own ``multi_head_attention_forward`` takes
    with ``need_weights=False`` (what ``nn.TransformerDecoderLayer`` passes, helper:40-44).
    Anything else (weights requested, masks, separate k/v dims, bias_k, add_zero_attn, CPU,
    non-f32) runs the stock module."""

    def forward(self, query, key, value, key_padding_mask=None, need_weights=True, attn_mask=None,
                average_attn_weights=True, is_causal=False):
        stock = (need_weights or key_padding_mask is not None or attn_mask is not None or not query.is_cuda
                 or query.dtype != torch.float32 or not self._qkv_same_embed_dim or self.bias_k is not None
                 or self.add_zero_attn or query.dim() != 3)
        if stock:
            return super().forward(query, key, value, key_padding_mask=key_padding_mask, need_weights=need_weights,
                                   attn_mask=attn_mask, average_attn_weights=average_attn_weights, is_causal=is_causal)
        return _mha_projected(self, query, key, value, is_causal, _LinearF32.apply), None


_F32_SWAP = {torch.nn.Linear: F32Linear, torch.nn.modules.linear.NonDynamicallyQuantizableLinear: F32Linear,
             torch.nn.MultiheadAttention: F32MultiheadAttention}


def use_f32_kernels(module: torch.nn.Module, on: bool = True) -> int:
    """Route an f32 module's linears and attention projections to the f32 MFMA GEMM by
    swapping the class of its ``nn.Linear`` / ``nn.MultiheadAttention`` submodules (and back
    with ``on=False``).  Parameters, buffers and state_dict keys are untouched, and nothing
    outside ``module`` changes (no global patch of ``torch.nn.functional``).  Returns the
    number of submodules switched."""
    n = 0
    for mod in module.modules():
        if on:
            cls = _F32_SWAP.get(type(mod))
            if cls is not None:
                mod._mipipe_f32_orig_cls = type(mod)
                mod.__class__ = cls
                n += 1
        elif type(mod) in (F32Linear, F32MultiheadAttention):
            mod.__class__ = mod.__dict__.pop("_mipipe_f32_orig_cls")
            n += 1
    return n


# MIPIPE_WGRAD_GROUP=0: every weight-gradient GEMM of a job list in its own launch
_WGRAD_GROUP = os.environ.get("MIPIPE_WGRAD_GROUP", "1") != "0"
_GROUP_MAX = 8


class DW:
    """A weight-gradient job ``dw (f32) += alpha * dy^T x`` kept as data, so that
    :func:`run_wjobs` can issue the short-token ones of a job list as ONE grouped launch
    (csrc/kernels/gemm2.hip ``gemms_tt_grouped_kernel``).  Calling it runs it alone."""
    __slots__ = ("dy", "x", "dw", "alpha")

    def __init__(self, dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, alpha: float = 1.0):
        self.dy, self.x, self.dw, self.alpha = dy, x, dw, alpha

    def __call__(self):
        linear_dw(self.dy, self.x, self.dw, self.alpha)

    def groupable(self) -> bool:
        """Short reductions (<= 4096 tokens) over few 256x256 output tiles: the shapes the
        planner sends to the small 64x64 TT engine (gemm2.hip mp_gemm2_plan, cfg 13)."""
        dy, x, dw = self.dy, self.x, self.dw
        if not (_gpu(dy) and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dw.dtype == torch.float32):
            return False
        if dy.stride(1) != 1 or x.stride(1) != 1 or dw.stride(1) != 1:
            return False
        T, N = dy.shape
        K = x.shape[1]
        if T % 64 or N % 8 or K % 8 or T > 4096:
            return False
        return ((N + 255) // 256) * ((K + 255) // 256) < 64


def run_wjobs(jobs) -> None:
    """Run a list of weight-gradient jobs (:class:`DW` objects and plain callables such as
    bias column sums).  The groupable DW jobs with the same alpha go out as grouped
    launches of up to 8 GEMMs; everything else runs in list order.  Jobs of one list
    write distinct gradient buffers, so the reordering is exact."""
    if not jobs:
        return
    rest, groups = [], {}
    if _WGRAD_GROUP and GEMM_BACKEND != "blas":
        for j in jobs:
            if isinstance(j, DW) and j.groupable():
                groups.setdefault(j.alpha, []).append(j)
            else:
                rest.append(j)
    else:
        rest = list(jobs)
    for alpha, g in groups.items():
        if len(g) == 1:
            g[0]()
            continue
        for i in range(0, len(g), _GROUP_MAX):
            part = g[i:i + _GROUP_MAX]
            _ext().gemm_tt_grouped([j.dy for j in part], [j.x for j in part], [j.dw for j in part], float(alpha))
    for j in rest:
        j()


# ======================================================================================
# elementwise
# ======================================================================================
def act_fwd(a: torch.Tensor, act: str, p_drop: float = 0.0, seed: int = 0, out=None):
    if out is None:
        out = torch.empty_like(a)
    if _gpu(a):
        _ext().act_fwd(a, out, ACT[act], float(p_drop), int(seed))
        return out
    y = _act_cpu(a.float(), act)
    if p_drop > 0:
        y = y * _cpu_dropout_mask(a.shape, p_drop, seed, a.device)
    out.copy_(y.to(out.dtype))
    return out


def act_bwd(dg: torch.Tensor, a: torch.Tensor, act: str, dbias: Optional[torch.Tensor] = None,
            p_drop: float = 0.0, seed: int = 0, out=None, saved: str = "pre"):
    """dA = dG * act'(.) (dropout mask regenerated from (seed, element index)), plus the
    column sums into ``dbias``.  ``saved`` says what ``a`` holds: "pre" -- the pre-activation
    (act_fwd's input; ReLU's aux from :func:`linear`) -- or "grad" -- act' itself, which is
    what ``linear(act="gelu_tanh")`` stores in its aux (the two forms are not
    interchangeable; passing a GELU aux as "pre" would silently give wrong gradients)."""
    if saved not in ("pre", "grad"):
        raise ValueError(f"saved must be 'pre' or 'grad', not {saved!r}")
    if out is None:
        out = torch.empty_like(dg)
    if saved == "grad":
        d = dg.float() * a.float()
        if p_drop > 0:
            if _gpu(dg):
                raise ValueError("the dropout mask with a saved derivative is fused into linear_dx's epilogue")
            d = d * _cpu_dropout_mask(a.shape, p_drop, seed, a.device)
        out.copy_(d.to(out.dtype))
        if dbias is not None:
            if _gpu(dg):
                _ext().colsum(out, dbias)
            else:
                dbias += out.float().reshape(-1, out.shape[-1]).sum(0)
        return out
    if _gpu(dg):
        _ext().act_bwd(dg, a, out, dbias, ACT[act], float(p_drop), int(seed))
        return out
    d = dg.float() * _act_grad_cpu(a.float(), act)
    if p_drop > 0:
        d = d * _cpu_dropout_mask(a.shape, p_drop, seed, a.device)
    out.copy_(d.to(out.dtype))
    if dbias is not None:
        dbias += out.float().reshape(-1, out.shape[-1]).sum(0)
    return out


def colsum(x: torch.Tensor, dbias: torch.Tensor):
    if _gpu(x):
        _ext().colsum(x, dbias)
        return dbias
    dbias += x.float().reshape(-1, x.shape[-1]).sum(0)
    return dbias


def swiglu_fwd(gu: torch.Tensor, out=None):
    T, F2 = gu.shape
    F = F2 // 2
    if out is None:
        out = torch.empty(T, F, device=gu.device, dtype=gu.dtype)
    if _gpu(gu):
        _ext().swiglu_fwd(gu, out)
        return out
    g, u = gu.float()[:, :F], gu.float()[:, F:]
    out.copy_((torch.nn.functional.silu(g) * u).to(out.dtype))
    return out


def swiglu_bwd(gu: torch.Tensor, dy: torch.Tensor, out=None):
    if out is None:
        out = torch.empty_like(gu)
    if _gpu(gu):
        _ext().swiglu_bwd(gu, dy, out)
        return out
    F = dy.shape[-1]
    g, u, d = gu.float()[:, :F], gu.float()[:, F:], dy.float()
    sg = torch.sigmoid(g)
    out[:, F:] = (d * g * sg).to(out.dtype)
    out[:, :F] = (d * u * sg * (1 + g * (1 - sg))).to(out.dtype)
    return out


def rope_tables(S: int, Dh: int, theta: float, device) -> Tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, Dh, 2, dtype=torch.float64) / Dh))
    ang = torch.arange(S, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cos(ang).float().to(device), torch.sin(ang).float().to(device)


def rope_(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, S: int, H: int, Hkv: int, Dh: int,
          pos_offset: int = 0, inverse: bool = False):
    """In-place rotate-half RoPE on the q and k heads of a packed [T, (H+2Hkv)*Dh] buffer."""
    if _gpu(qkv):
        _ext().rope(qkv, cos, sin, int(S), int(H), int(Hkv), int(Dh), int(pos_offset), bool(inverse))
        return qkv
    T = qkv.shape[0]
    x = qkv.float().reshape(T, H + 2 * Hkv, Dh)
    pos = torch.arange(T) % S + pos_offset
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    if inverse:
        s = -s
    half = Dh // 2
    rot = x[:, : H + Hkv]
    a, b = rot[..., :half], rot[..., half:]
    new = torch.cat([a * c - b * s, b * c + a * s], -1)
    x[:, : H + Hkv] = new
    qkv.copy_(x.reshape(T, -1).to(qkv.dtype))
    return qkv


# ======================================================================================
# attention
# ======================================================================================
def _heads(t: torch.Tensor, B: int, S: int, nh: int, D: int):
    """token-major [B*S, stride] view (first nh*D cols) -> [B, nh, S, D] f32"""
    return t[:, : nh * D].float().reshape(B, S, nh, D).permute(0, 2, 1, 3)


def _cpu_attn_mask(B, H, Sq, Sk, causal, device):
    if not causal:
        return None
    shift = Sk - Sq
    q = torch.arange(Sq)[:, None]
    k = torch.arange(Sk)[None, :]
    return (k > q + shift).to(device)


def _cpu_attn_drop(B, H, Sq, Sk, p, seed, device):
    if p <= 0:
        return None
    return _cpu_dropout_mask((B, H, Sq, Sk), p, seed, device)


def attn_fwd(q, k, v, o, lse, B: int, Sq: int, Sk: int, H: int, Hkv: int, D: int, causal: bool,
             scale: Optional[float] = None, p_drop: float = 0.0, seed: int = 0):
    """q/k/v/o: token-major 2-D views ([B*S, row_stride], head h at cols h*D).  lse: f32
    [B*H*Sq] (log2 units).  Writes o and lse."""
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if _gpu(q):
        _ext().attn_fwd(q, k, v, o, lse, B, Sq, Sk, H, Hkv, D, bool(causal), float(scale), float(p_drop), int(seed))
        return o
    Q, K, V = _heads(q, B, Sq, H, D), _heads(k, B, Sk, Hkv, D), _heads(v, B, Sk, Hkv, D)
    rep = H // Hkv
    K, V = K.repeat_interleave(rep, 1), V.repeat_interleave(rep, 1)
    s = (Q @ K.transpose(-1, -2)) * scale
    mask = _cpu_attn_mask(B, H, Sq, Sk, causal, q.device)
    if mask is not None:
        s = s.masked_fill(mask, float("-inf"))
    l2 = torch.logsumexp(s, -1) * LOG2E
    p = torch.softmax(s, -1)
    dm = _cpu_attn_drop(B, H, Sq, Sk, p_drop, seed, q.device)
    if dm is not None:
        p = p * dm
    out = (p @ V).permute(0, 2, 1, 3).reshape(B * Sq, H * D)
    o[:, : H * D].copy_(out.to(o.dtype))
    lse.view(-1)[: B * H * Sq].copy_(l2.reshape(-1))
    return o


def attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B: int, Sq: int, Sk: int, H: int, Hkv: int, D: int, causal: bool,
             scale: Optional[float] = None, p_drop: float = 0.0, seed: int = 0, delta=None,
             dbias: Optional[torch.Tensor] = None):
    """Writes dq, dk, dv (token-major views like the inputs).  ``dbias`` (f32
    [(H + 2 Hkv) D]): also accumulate the QKV bias gradient (column sums of dq | dk | dv)."""
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if _gpu(q):
        if delta is None:
            delta = torch.empty(B * H * Sq, device=q.device, dtype=torch.float32)
        _ext().attn_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, B, Sq, Sk, H, Hkv, D, bool(causal),
                        float(scale), float(p_drop), int(seed), dbias)
        return dq, dk, dv
    rep = H // Hkv
    Q, K, V = _heads(q, B, Sq, H, D), _heads(k, B, Sk, Hkv, D), _heads(v, B, Sk, Hkv, D)
    dO, O = _heads(do, B, Sq, H, D), _heads(o, B, Sq, H, D)
    Kr, Vr = K.repeat_interleave(rep, 1), V.repeat_interleave(rep, 1)
    s = (Q @ Kr.transpose(-1, -2)) * scale
    mask = _cpu_attn_mask(B, H, Sq, Sk, causal, q.device)
    if mask is not None:
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, -1)
    dm = _cpu_attn_drop(B, H, Sq, Sk, p_drop, seed, q.device)
    pd = p * dm if dm is not None else p
    dV = pd.transpose(-1, -2) @ dO
    dP = dO @ Vr.transpose(-1, -2)
    if dm is not None:
        dP = dP * dm
    delta_ = (dO * O).sum(-1, keepdim=True)
    dS = p * (dP - delta_)
    dQ = (dS @ Kr) * scale
    dK = (dS.transpose(-1, -2) @ Q) * scale
    dK = dK.reshape(B, Hkv, rep, Sk, D).sum(2)
    dV = dV.reshape(B, Hkv, rep, Sk, D).sum(2)
    dq[:, : H * D].copy_(dQ.permute(0, 2, 1, 3).reshape(B * Sq, H * D).to(dq.dtype))
    dk[:, : Hkv * D].copy_(dK.permute(0, 2, 1, 3).reshape(B * Sk, Hkv * D).to(dk.dtype))
    dv[:, : Hkv * D].copy_(dV.permute(0, 2, 1, 3).reshape(B * Sk, Hkv * D).to(dv.dtype))
    if dbias is not None:
        dbias[: H * D] += dq[:, : H * D].float().sum(0)
        dbias[H * D:(H + Hkv) * D] += dk[:, : Hkv * D].float().sum(0)
        dbias[(H + Hkv) * D:] += dv[:, : Hkv * D].float().sum(0)
    return dq, dk, dv


# ======================================================================================
# optimizer
# ======================================================================================
def set_dropout_step(step: int, device: Optional[torch.device] = None) -> None:
    """Set the training-step counter every dropout kernel mixes into its seed (device
    memory, stream-ordered on the current stream).  Issued once per step outside any
    captured graph, it lets HIP-graph replays draw a fresh mask each step.  No-op on CPU."""
    if device is not None and device.type != "cuda":
        return
    _ext().set_dropout_step(int(step))


def zero_(t: torch.Tensor) -> torch.Tensor:
    """t <- 0 (GPU: hipMemsetAsync on the current stream instead of an ATen fill kernel)."""
    if _gpu(t) and t.is_contiguous():
        _ext().zero_(t)
        return t
    return t.zero_()


def mean(x: torch.Tensor) -> torch.Tensor:
    """Mean of an f32 tensor as a 0-dim f32 tensor (GPU: one deterministic workgroup,
    optim.hip scaled_sum_kernel -- e.g. the microbatch's mean token loss)."""
    if _gpu(x) and x.dtype == torch.float32 and x.is_contiguous():
        out = torch.empty((), device=x.device, dtype=torch.float32)
        _ext().scaled_sum(x, 1.0 / max(1, x.numel()), out)
        return out
    return x.mean()


def sumsq(g: torch.Tensor, out: torch.Tensor):
    if _gpu(g):
        _ext().sumsq(g, out)
        return out
    out += (g.float() ** 2).sum()
    return out


def adamw_(p, g, m, v, w16, n_decay: int, lr: float, b1: float, b2: float, eps: float, wd: float, step: int,
           sumsq_buf=None, max_norm: float = 0.0, grad_scale: float = 1.0, zero_grad: bool = True):
    """Fused AdamW over flat f32 buffers; also refreshes the bf16 copy ``w16`` and zeroes g."""
    if _gpu(p):
        _ext().adamw(p, g, m, v, w16, int(n_decay), float(lr), float(b1), float(b2), float(eps), float(wd), int(step),
                     sumsq_buf, float(max_norm), float(grad_scale), bool(zero_grad))
        return
    coef = grad_scale
    if max_norm > 0 and sumsq_buf is not None:
        nrm = math.sqrt(float(sumsq_buf.item())) * grad_scale
        coef *= min(1.0, max_norm / (nrm + 1e-6))
    gr = g * coef
    m.mul_(b1).add_(gr, alpha=1 - b1)
    v.mul_(b2).addcmul_(gr, gr, value=1 - b2)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    upd = (m / bc1) / ((v / bc2).sqrt() + eps)
    decay = torch.zeros_like(p)
    decay[:n_decay] = wd
    p.sub_(lr * (upd + decay * p))
    if zero_grad:
        g.zero_()
    if w16 is not None:
        w16.copy_(p.to(w16.dtype))


def cast_f32_bf16(src: torch.Tensor, dst: torch.Tensor):
    if _gpu(src):
        _ext().cast_f32_bf16(src, dst)
    else:
        dst.copy_(src.to(dst.dtype))
    return dst
