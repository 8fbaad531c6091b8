"""One reference-config (L, H) training loop on one GPU, for rocprofv3 kernel stats.
    python tools/ref_step_probe.py --L 4 --H 12 [--steps 5]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--graphs", type=int, default=1)
    a = ap.parse_args()
    import torch
    import mipipe  # noqa: F401
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig
    cfg = NativeConfig.reference(n_layers=a.L, n_heads=a.H)
    dev = torch.device("cuda", 0)
    tr = PipelineTrainer(cfg, pp=1, n_microbatches=4, mbs=8, seq_len=128, device=dev, graphs=bool(a.graphs))
    x = torch.randint(0, cfg.vocab_size, (32, 128), device=dev)
    y = torch.randint(0, cfg.vocab_size, (32, 128), device=dev)
    if a.graphs:
        tr.capture_graphs(x, y)
    for _ in range(a.steps):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
