"""Which HIP streams actually run concurrently on this box (hardware-queue mapping probe).

HIP maps streams onto a small set of hardware queues per priority (GPU_MAX_HW_QUEUES, 4 on
the pool's boxes); two streams on one queue serialise, and a stream wait on one blocks the
other.  For each candidate stream X this launches a bounded spin kernel
(``torch.cuda._sleep``) on the compute stream, then a tiny kernel on X, and reports whether
X's kernel finished before the spin did (= a separate hardware queue).

    python tools/stream_probe.py          (GPU; prints one JSON line)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def concurrent(main, other, cycles=int(2e8)) -> dict:
    a = torch.zeros(1024, device="cuda")
    torch.cuda.synchronize()
    t0, t_main, t_x = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    with torch.cuda.stream(main):
        t0.record(main)
        torch.cuda._sleep(cycles)
        t_main.record(main)
    with torch.cuda.stream(other):
        a.add_(1.0)
        t_x.record(other)
    torch.cuda.synchronize()
    return dict(spin_ms=round(t0.elapsed_time(t_main), 3), other_done_ms=round(t0.elapsed_time(t_x), 3),
                concurrent=t0.elapsed_time(t_x) < 0.5 * t0.elapsed_time(t_main))


def main():
    import mipipe  # noqa: F401
    from mipipe import ops
    ext = ops.load_ext()
    dev = torch.cuda.current_device()
    main_s = torch.cuda.current_stream()
    cands = {
        "pool_low": torch.cuda.Stream(),
        "pool_low_2": torch.cuda.Stream(),
        "pool_high": torch.cuda.Stream(priority=-1),
        "raw_normal": torch.cuda.ExternalStream(ext.create_stream(dev, 0)),
        "raw_high": torch.cuda.ExternalStream(ext.create_stream(dev, -1)),
        "raw_high_2": torch.cuda.ExternalStream(ext.create_stream(dev, -1)),
    }
    out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
    for k, s in cands.items():
        out[f"main|{k}"] = concurrent(main_s, s)
    for a_, b_ in (("raw_high", "raw_high_2"), ("pool_low", "raw_high"), ("pool_low", "pool_high"),
                   ("raw_normal", "pool_low")):
        out[f"{a_}|{b_}"] = concurrent(cands[a_], cands[b_])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
