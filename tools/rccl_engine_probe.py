"""Step-by-step probe of the native RCCL P2P engine (csrc/comm/rccl_engine.cpp) on one GPU.

Prints a line before each stage so a failure points at the exact call.  GPU only: run it
through gpurun.
"""
import faulthandler
import os
import sys

faulthandler.enable(all_threads=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402
from mipipe.parallel.comm import load_native_rccl  # noqa: E402


def say(*a):
    print("[probe]", *a, flush=True)


say("torch", torch.__version__, "hip", torch.version.hip)
ext = _k.load_ext()
say("ext", ext.__file__)
with open("/proc/self/maps") as f:
    say("rccl maps", sorted({ln.split()[-1] for ln in f if "librccl" in ln}))
load_native_rccl(ext)
say("loaded")
torch.cuda.init()
dev = torch.cuda.current_device()
say("device", dev)
uid = b"".join(ext.RcclEngine.unique_id() for _ in range(3))
say("uid", len(uid))
eng = ext.RcclEngine(uid, 1, 0, dev, [0, 1, 2])
say("comm up")
src = torch.randn(1 << 20, device="cuda").to(torch.bfloat16)
dst = torch.empty_like(src)
h = eng.post(0, [(src, 0)], [(dst, 0)])
say("posted", h)
eng.wait(h)
torch.cuda.synchronize()
say("equal", torch.equal(dst, src))
eng.close()
say("closed")
