import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))
import torch
from test_learning import _fit
from mipipe.models.config import NativeConfig
dev = torch.device("cuda", 0)
cfg = NativeConfig.reference(n_layers=2, n_heads=4, vocab_size=512, dim=256, dim_feedforward=1024)
for rep in range(2):
    losses = _fit(cfg, 1, dev, torch.bfloat16, 200, 2e-3, graphs=True, pattern=256, mbs=8, seq=128, m=4)
    print(rep, [round(l, 4) for l in losses[::10]], "last10", [round(l, 3) for l in losses[-10:]], flush=True)
