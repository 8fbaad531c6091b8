"""The full multi-process pipeline stack on the GPU: 2 and 4 ranks sharing one device
(gloo carries the traffic through host memory, MIPIPE_DIST_BACKEND=gloo) must train
exactly like one process -- HIP kernels, distributed head, schedules and HIP graphs in
the real multi-rank runtime.  RCCL itself needs one GPU per rank and is exercised by
the 8-GPU scaling bench."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, *args, port):
    env = dict(os.environ, MIPIPE_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "mp_gpu_check.py")] + list(args)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


@pytest.fixture(scope="module")
def reference():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _run(1, port=29771)["losses"]


@pytest.mark.parametrize("n,schedule,graphs,split,dp", [(2, "1F1B", 0, 1, 1), (2, "ZBH1", 1, 1, 1),
                                                        (4, "1F1B", 1, 1, 1), (4, "GPipe", 0, 0, 1),
                                                        (2, "ZBV", 0, 1, 1), (4, "1F1B", 1, 1, 2)])
def test_multirank_gpu_matches_single(reference, n, schedule, graphs, split, dp):
    """dp=2: DP x PP (2 x 2) with HIP graphs -- the stages' DP all-reduce replays as a
    recorded CALL on the native runner's tape."""
    res = _run(n, "--schedule", schedule, "--graphs", str(graphs), "--split-head", str(split), "--dp", str(dp),
               port=29772 + n + 10 * graphs + 20 * split + 40 * dp)
    # bf16 kernels + split-K atomics: equal up to reduction-order rounding
    assert res["losses"] == pytest.approx(reference, rel=2e-3)
    # with graphs, steps after the first replay run from the native stage runner's tape
    # (gloo transfers recorded as CALLs)
    assert res["native_runner"] == bool(graphs), res["native_reason"]
