"""Attention forward / backward time at the headline shape (GPT-2 small microbatch: B 64,
S 1024, H 12, D 64, causal), 20 launches replayed from one HIP graph.
    python tools/attn_time.py [B S H D]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402
from tools.gemm_epi_probe import timed  # noqa: E402

B, S, H, D = (int(x) for x in sys.argv[1:5]) if len(sys.argv) > 4 else (64, 1024, 12, 64)
T = B * S
qkv = torch.randn(T, 3 * H * D, device="cuda").to(torch.bfloat16)
q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
o = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B * H * S, device="cuda")
do = torch.randn_like(o)
d = torch.empty_like(qkv)
fwd = lambda: ops.attn_fwd(q, k, v, o, lse, B, S, S, H, H, D, True)  # noqa: E731
bwd = lambda: ops.attn_bwd(q, k, v, o, do, lse, d[:, :H * D], d[:, H * D:2 * H * D], d[:, 2 * H * D:],  # noqa: E731
                           B, S, S, H, H, D, True)
fwd()
tf, tb = timed(fwd, True), timed(bwd, True)
fl = 4 * B * H * S * S * D / 2          # causal: QK^T + PV over half the scores
print(json.dumps({"shape": [B, S, H, D], "fwd_us": round(tf, 1), "bwd_us": round(tb, 1),
                  "fwd_tf": round(fl / tf / 1e6, 1), "bwd_tf": round(2.5 * fl / tb / 1e6, 1)}))
