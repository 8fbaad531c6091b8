"""Weight-gradient batching probe (reference model shapes, 1024-token microbatches, m = 4):
the dW GEMMs + bias column sums of one layer run per microbatch (4 x K = 1024, today's
path) vs once over the 4 microbatches (K = 4096, operands contiguous).

    python tools/wbatch_probe.py      (GPU; one JSON line per shape + a total line)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


m, T, d, f = 4, 1024, 768, 2048
# (name, N = dy width, K = x width, bias?)  -- the 7 dW GEMMs of one reference layer
SHAPES = [("sa_qkv", 3 * d, d, True), ("sa_out", d, d, False), ("ca_q", d, d, True), ("ca_kv", 2 * d, d, True),
          ("ca_out", d, d, False), ("lin1", f, d, False), ("lin2", d, f, False)]
tot = {"per_mb_us": 0.0, "batched_us": 0.0}
for name, N, K, has_b in SHAPES:
    dy = (torch.randn(m * T, N, device="cuda") * 0.1).to(torch.bfloat16)
    x = (torch.randn(m * T, K, device="cuda") * 0.1).to(torch.bfloat16)
    g = torch.zeros(N, K, device="cuda")
    gb = torch.zeros(N, device="cuda")

    def per_mb():
        for i in range(m):
            ops.linear_dw(dy[i * T:(i + 1) * T], x[i * T:(i + 1) * T], g)
            if has_b:
                ops.colsum(dy[i * T:(i + 1) * T], gb)

    def batched():
        ops.linear_dw(dy, x, g)
        if has_b:
            ops.colsum(dy, gb)
    a, b = timeit(per_mb), timeit(batched)
    tot["per_mb_us"] += a
    tot["batched_us"] += b
    fl = 2.0 * m * T * N * K
    print(json.dumps({"shape": name, "N": N, "K": K, "per_mb_us": round(a, 2), "batched_us": round(b, 2),
                      "per_mb_tf": round(fl / a / 1e6, 1), "batched_tf": round(fl / b / 1e6, 1)}), flush=True)
tot = {k: round(v, 2) for k, v in tot.items()}
tot["speedup"] = round(tot["per_mb_us"] / tot["batched_us"], 3)
print(json.dumps({"layer_total": tot}), flush=True)
