"""Time the fused CE kernel on the GPT-2 head shape (T x 50304 bf16 logits, grad in place)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402

T, V, Vp = int(sys.argv[1]) if len(sys.argv) > 1 else 16384, int(sys.argv[2]) if len(sys.argv) > 2 else 50257, int(sys.argv[3]) if len(sys.argv) > 3 else 50304
x = torch.randn(T, Vp, device="cuda").to(torch.bfloat16)
tgt = torch.randint(0, V, (T,), device="cuda")
for _ in range(3):
    ops.xent_fwd_bwd(x, tgt, V, 1.0 / T)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    ops.xent_fwd_bwd(x, tgt, V, 1.0 / T)
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) / 20 * 1e3
print(f"xent {T}x{Vp}: {us:.1f} us, {2 * T * Vp * 2 / us / 1e6:.2f} TB/s")
