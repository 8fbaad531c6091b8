"""One-off environment probe: device props, hipBLASLt GEMM rates, SDPA, eager GPT-2 step.
Used to establish the library baselines our HIP kernels must beat."""
import time, json, torch, torch.nn.functional as F

def t(fn, iters=20, warm=5):
    for _ in range(warm): fn()
    torch.cuda.synchronize(); s = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - s) / iters

out = {}
p = torch.cuda.get_device_properties(0)
out["device"] = dict(name=p.name, cus=p.multi_processor_count, mem_gb=p.total_memory / 2**30, arch=getattr(p, "gcnArchName", "?"))
dev = "cuda"
res = {}
for (M, K, N) in [(8192, 768, 2304), (8192, 768, 768), (8192, 768, 3072), (8192, 3072, 768), (8192, 768, 50304),
                  (8192, 4096, 4096), (8192, 4096, 14336), (8192, 14336, 4096), (4096, 4096, 4096), (8192, 8192, 8192)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16); b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    dt = t(lambda: a @ b)
    res[f"{M}x{K}x{N}"] = round(2 * M * N * K / dt / 1e12, 1)
out["hipblaslt_bf16_tflops"] = res
for (B, H, S, D, causal) in [(8, 12, 1024, 64, True), (4, 32, 2048, 128, True), (8, 8, 128, 96, False)]:
    q = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn_like(q, requires_grad=True); v = torch.randn_like(q, requires_grad=True)
    fw = t(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=causal))
    o = F.scaled_dot_product_attention(q, k, v, is_causal=causal); g = torch.randn_like(o)
    def fb():
        o = F.scaled_dot_product_attention(q, k, v, is_causal=causal); o.backward(g)
    tb = t(fb)
    fl = 4 * B * H * S * S * D * (0.5 if causal else 1)
    out[f"sdpa_B{B}H{H}S{S}D{D}c{int(causal)}"] = dict(fwd_ms=fw * 1e3, fwdbwd_ms=tb * 1e3, fwd_tflops=fl / fw / 1e12, fb_tflops=3.5 * fl / tb / 1e12)
# eager GPT-2 small training step (bf16 weights, torch ops) as a library baseline
import torch.nn as nn
class Blk(nn.Module):
    def __init__(s, d, h):
        super().__init__(); s.h = h; s.ln1 = nn.LayerNorm(d); s.qkv = nn.Linear(d, 3 * d); s.o = nn.Linear(d, d)
        s.ln2 = nn.LayerNorm(d); s.f1 = nn.Linear(d, 4 * d); s.f2 = nn.Linear(4 * d, d)
    def forward(s, x):
        B, T, C = x.shape
        q, k, v = s.qkv(s.ln1(x)).split(C, 2)
        q, k, v = [z.view(B, T, s.h, C // s.h).transpose(1, 2) for z in (q, k, v)]
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, C)
        x = x + s.o(y)
        return x + s.f2(F.gelu(s.f1(s.ln2(x)), approximate="tanh"))
class G(nn.Module):
    def __init__(s):
        super().__init__(); s.wte = nn.Embedding(50257, 768); s.wpe = nn.Embedding(1024, 768)
        s.blocks = nn.ModuleList([Blk(768, 12) for _ in range(12)]); s.lnf = nn.LayerNorm(768)
    def forward(s, idx, tgt):
        x = s.wte(idx) + s.wpe(torch.arange(idx.shape[1], device=idx.device))
        for b in s.blocks: x = b(x)
        logits = F.linear(s.lnf(x), s.wte.weight)
        return F.cross_entropy(logits.float().view(-1, logits.shape[-1]), tgt.view(-1))
m = G().to(dev)
opt = torch.optim.AdamW(m.parameters(), lr=1e-4, fused=True)
B, S, mbs = 8, 1024, 8
idx = torch.randint(0, 50257, (B, S), device=dev); tgt = torch.randint(0, 50257, (B, S), device=dev)
def step():
    for _ in range(mbs):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m(idx, tgt)
        loss.backward()
    opt.step(); opt.zero_grad(set_to_none=True)
dt = t(step, iters=5, warm=2)
out["torch_eager_gpt2s_autocast_tok_s"] = B * S * mbs / dt
out["torch_eager_gpt2s_step_ms"] = dt * 1e3
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/probe.json", "w"), indent=1)
