"""Reference fp32 workload at P = 1: throughput per lane count, and how long the host takes
to issue one replayed step (runtime.step without a sync) vs the step's GPU time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.bench.compat import native_reference_schedule, run_train_iterations  # noqa: E402
from mipipe.models.ref_transformer import ModelArgs  # noqa: E402

args = ModelArgs(n_layers=8, n_heads=8)
dev = torch.device("cuda", 0)
x = torch.randint(0, args.vocab_size, (32, 128), device=dev)
y = torch.randint(0, args.vocab_size, (32, 128), device=dev)
for lanes in [int(v) for v in os.environ.get("LANES", "1,2,4").split(",")]:
    s = native_reference_schedule(args, "1F1B", 0, 1, 32, 128, 4, dev, precision="fp32", lanes=lanes)
    met = run_train_iterations(s, x, y, 0, 1, num_iterations=20, warmup=5, device=dev, measure_bubble=False)
    torch.cuda.synchronize()
    host = []
    for _ in range(5):
        t0 = time.perf_counter()
        s.step(x, target=y, losses=[])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((round((t1 - t0) * 1e3, 2), round((t2 - t0) * 1e3, 2)))
    print(f"lanes {s.runtime.lanes}: {met['throughput']:.0f} tok/s  host-issue / total ms {host}", flush=True)
