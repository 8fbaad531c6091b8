"""Print the recorded native tape of the reference fp32 workload (P = 1, 1F1B, lanes) --
which stream each graph runs on and every cross-stream sync."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.bench.compat import native_reference_schedule, run_train_iterations  # noqa: E402
from mipipe.models.ref_transformer import ModelArgs  # noqa: E402
from mipipe.parallel import native_runner as NR  # noqa: E402

log = []
names = {}


def sname(s):
    return names.setdefault(int(s), f"S{len(names)}") if s else "main"


og, osy, oc, ocall = NR.TapeRecorder.graph, NR.TapeRecorder.sync, NR.TapeRecorder.copy, NR.TapeRecorder.call


def g(self, gr, label=""):
    log.append(f"GRAPH {label} on {sname(self._stream())}")
    return og(self, gr, label)


def sy(self, w, s):
    log.append(f"SYNC {sname(0 if int(w.cuda_stream) == self.main_stream else w.cuda_stream)} waits "
               f"{sname(0 if int(s.cuda_stream) == self.main_stream else s.cuda_stream)}")
    return osy(self, w, s)


def cp(self, d, s):
    log.append(f"COPY {d.numel() * d.element_size()} B on {sname(self._stream())}")
    return oc(self, d, s)


def ca(self, fn):
    log.append(f"CALL {getattr(fn, '__qualname__', fn)}")
    return ocall(self, fn)


NR.TapeRecorder.graph, NR.TapeRecorder.sync, NR.TapeRecorder.copy, NR.TapeRecorder.call = g, sy, cp, ca
sched = os.environ.get("SCHED", "1F1B")
args = ModelArgs(n_layers=8, n_heads=8)
dev = torch.device("cuda", 0)
x = torch.randint(0, args.vocab_size, (32, 128), device=dev)
y = torch.randint(0, args.vocab_size, (32, 128), device=dev)
s = native_reference_schedule(args, sched, 0, 1, 32, 128, 4, dev, precision="fp32")
met = run_train_iterations(s, x, y, 0, 1, num_iterations=5, warmup=2, device=dev, measure_bubble=False)
print("lanes", s.runtime.lanes, "tok/s", met["throughput"], "native", met.get("native_runner"))
for line in log:
    print(line)
