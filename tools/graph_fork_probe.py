import json, os, sys
sys.path.insert(0, "/root/repo")
import torch
import mipipe
from mipipe import ops

def graph_fork_time(side, cycles=int(5e7)):
    main = torch.cuda.current_stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        side.wait_stream(cap)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cycles)
        torch.cuda._sleep(cycles)
        cap.wait_stream(side)
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    one = torch.cuda.Event(enable_timing=True); two = torch.cuda.Event(enable_timing=True)
    one.record(); torch.cuda._sleep(cycles); two.record(); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / one.elapsed_time(two), 2)   # ~1 concurrent, ~2 serial

mode = sys.argv[1]
ext = ops.load_ext()
dev = torch.cuda.current_device()
res = {}
if mode == "pool":
    s = torch.cuda.Stream()
elif mode == "raw":
    s = torch.cuda.ExternalStream(ext.create_stream(dev, 0))
elif mode == "rawhigh":
    s = torch.cuda.ExternalStream(ext.create_stream(dev, -1))
for i in range(4):
    res[f"fork_ratio_{i}"] = graph_fork_time(s)
# eager fork as well
main = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize(); e0.record()
s.wait_stream(main)
with torch.cuda.stream(s):
    torch.cuda._sleep(int(5e7))
torch.cuda._sleep(int(5e7))
main.wait_stream(s); e1.record(); torch.cuda.synchronize()
res["eager_ms"] = round(e0.elapsed_time(e1), 2)
print(mode, json.dumps(res))
