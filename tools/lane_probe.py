"""Would two microbatches' stage compute run faster concurrently on two HIP streams?

Captures a training step's per-microbatch graphs (PP=1), then replays pairs of forward
graphs (F0 || F1) and backward graphs (B0 || B1) on two streams vs back to back on one,
and reports the time ratio.  The concurrent replays race on the shared gradient arena:
results are meaningless, only the timing is read (all addresses stay valid).

    python tools/lane_probe.py --model reference|gpt2-small"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.engine import PipelineTrainer  # noqa: E402
from mipipe.models.config import NativeConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="reference")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.model == "reference":
        cfg, mbs, S, m = NativeConfig.reference(n_layers=8, n_heads=8), 8, 128, 4
    else:
        cfg, mbs, S, m = NativeConfig.gpt2("small"), 16, 1024, 2
    tr = PipelineTrainer(cfg, pp=1, schedule="1F1B", n_microbatches=m, mbs=mbs, seq_len=S, device=dev, seed=0,
                         graphs=True)
    x = torch.randint(0, cfg.vocab_size, (m * mbs, S), device=dev)
    tr.capture_graphs(x, x)
    for _ in range(3):
        tr.train_step(x, x)
    torch.cuda.synchronize()
    st = tr.stages[0]
    gs = {k: v[0] for k, v in st.graphs.graphs.items()}
    print("graphs:", sorted(map(str, gs)), flush=True)
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(a.iters):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / a.iters

    out = {}
    for kind in ("F", "B", "FB"):
        g0, g1 = (gs.get((kind, 0)), gs.get((kind, 1))) if kind != "FB" else (gs.get(("B", 0)), gs.get(("F", 1)))
        if g0 is None or g1 is None:
            continue
        cur = torch.cuda.current_stream()

        def serial():
            g0.replay()
            g1.replay()

        def pair():
            sA.wait_stream(cur)
            sB.wait_stream(cur)
            with torch.cuda.stream(sA):
                g0.replay()
            with torch.cuda.stream(sB):
                g1.replay()
            cur.wait_stream(sA)
            cur.wait_stream(sB)

        ts, tp = timed(serial), timed(pair)
        out[kind] = {"serial_ms": round(ts, 3), "two_streams_ms": round(tp, 3), "speedup": round(ts / tp, 3)}
        print(json.dumps({kind: out[kind]}), flush=True)
    print(json.dumps({"model": a.model, "mbs": mbs, "seq": S, **out}))


if __name__ == "__main__":
    main()
