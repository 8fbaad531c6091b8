"""Time one distributed-head chunk (HeadShard.run: logits GEMM + fused CE + dX + dW) for
several chunk sizes vs the full-microbatch head, GPT-2 small."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.models.config import NativeConfig  # noqa: E402
from mipipe.models.native import HeadShard  # noqa: E402


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


cfg = NativeConfig.by_name(sys.argv[1] if len(sys.argv) > 1 else "gpt2-small")
head = HeadShard(cfg, "cuda")
res = {}
for Tc in (256, 512, 1024, 2048, 3584, 4096, 8192, 16384):
    h = torch.randn(Tc, cfg.d_model, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, cfg.vocab_size, (Tc,), device="cuda")
    dh = torch.empty_like(h)
    ms = t(lambda: head.run(h, y, dh, 1.0 / 16384))
    res[Tc] = dict(ms=round(ms, 3), us_per_token=round(ms * 1e3 / Tc, 4))
    print(Tc, res[Tc], flush=True)
print(json.dumps(res))
