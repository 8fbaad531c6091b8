"""Run attention fwd+bwd a few times (for rocprofv3 --pmc): python tools/attn_probe.py B S H KV D [causal]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402

B, S, H, KV, D = (int(x) for x in sys.argv[1:6])
causal = bool(int(sys.argv[6])) if len(sys.argv) > 6 else True
T = B * S
qkv = torch.randn(T, (H + 2 * KV) * D, device="cuda").to(torch.bfloat16)
q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
o = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B * H * S, device="cuda")
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
dq, dk, dv = dqkv[:, :H * D], dqkv[:, H * D:(H + KV) * D], dqkv[:, (H + KV) * D:]
for _ in range(3):
    ops.attn_fwd(q, k, v, o, lse, B, S, S, H, KV, D, causal)
    ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, S, H, KV, D, causal)
torch.cuda.synchronize()
print("ok")
