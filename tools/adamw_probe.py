"""AdamW kernel bandwidth on one MI355X: GPT-2 small (124M) and Llama-3 8B-layer-sized
(1.75B) flat arenas; bytes = 30 per element (p, g, m, v read; p, m, v, g written; bf16
copy).  MIPIPE_EXT_VARIANT selects an A/B build (tools/build_ext.py --variant)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mipipe  # noqa: F401
from mipipe import ops

for n in (124_439_808, 1_750_000_000):
    p, g, m, v = (torch.randn(n, device="cuda") for _ in range(4))
    w = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    ss = torch.ones(1, device="cuda")
    for _ in range(3):
        ops.adamw_(p, g, m, v, w, n // 2, 1e-4, 0.9, 0.95, 1e-8, 0.1, 5, ss, 1.0, 1.0, zero_grad=True)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 10
    s.record()
    for _ in range(it):
        ops.adamw_(p, g, m, v, w, n // 2, 1e-4, 0.9, 0.95, 1e-8, 0.1, 5, ss, 1.0, 1.0, zero_grad=True)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / it * 1e3
    print(f"variant={os.environ.get('MIPIPE_EXT_VARIANT', '') or 'default'} n={n}: {us:.1f} us = "
          f"{30 * n / us / 1e6:.2f} TB/s", flush=True)
    del p, g, m, v, w
    torch.cuda.empty_cache()
