"""Measured pipeline bubble on CPU/gloo: PP=4 with uniform stages must
measure within 5 points of the analytic (P-1)/(m+P-1) for GPipe and 1F1B.

The stages are fixed-duration stand-ins (``SleepStage``: a forward "costs" 30 ms, a
backward 60 ms, tiny tensors cross the real gloo transport), so the test exercises the
runtime's schedule execution and its busy/step accounting -- the same numbers bench.py
reports (from the native tape on GPUs, from the Python executor's timer here) -- without
CPU-load noise from real kernels.  A second case uses a real native GPT-2 stage stack."""
import time

import pytest
import torch

from dist_utils import run_world


def _sleep_worker(rank, world, m, sched, tf, tb):
    import torch.distributed as dist
    import mipipe  # noqa: F401
    from mipipe.parallel.comm import P2P
    from mipipe.parallel.runtime import PipelineRuntime
    from mipipe.parallel.stage import StageBase

    class SleepStage(StageBase):
        def __init__(self, idx, n):
            self.stage_index, self.num_stages, self.device = idx, n, torch.device("cpu")
            self.input_specs = [((4,), torch.float32)]
            self.output_specs = [((4,), torch.float32)]

        def forward_mb(self, mb, args, target, loss_fn, loss_scale):
            time.sleep(tf)
            x = args[0].float() + 1.0
            if self.is_last:
                return (x,), x.sum() * loss_scale
            return (x,), None

        def backward_mb(self, mb, grad_outputs):
            time.sleep(tb)
            return (torch.ones(4),) if self.stage_index > 0 else ()

        def infer_output_specs(self, args):
            return self.output_specs

    st = SleepStage(rank, world)
    rt = PipelineRuntime([st], sched, m, rank, world, P2P(None, list(range(world)), torch.device("cpu")))
    inputs = [(torch.zeros(4),) for _ in range(m)] if rank == 0 else None
    targets = [torch.zeros(4) for _ in range(m)] if rank == world - 1 else None
    rt.step(inputs, targets, [], return_outputs=False)
    out = []
    for _ in range(3):   # min over 3: a loaded machine (parallel test workers) only adds time
        dist.barrier()
        rt.profile = True
        rt.step(inputs, targets, [], return_outputs=False)
        rt.profile = False
        t = torch.tensor([rt.busy_ms(), rt.last_step_ms], dtype=torch.float64)
        allv = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        out.append(1.0 - sum(float(v[0]) for v in allv) / (world * max(float(v[1]) for v in allv)))
    return min(out)


@pytest.mark.parametrize("sched,m", [("1F1B", 4), ("1F1B", 8), ("GPipe", 8)])
def test_measured_bubble_matches_analytic_pp4(sched, m):
    measured = run_world(_sleep_worker, 4, m, sched, 0.03, 0.06)[0]
    analytic = 3 / (m + 3)
    assert abs(measured - analytic) < 0.05, (measured, analytic)


def _native_worker(rank, world, m):
    import torch.distributed as dist
    import mipipe  # noqa: F401
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig
    torch.set_num_threads(1)
    cfg = NativeConfig.gpt2("tiny", vocab_size=64, d_model=256, n_layers=8, n_heads=4, d_ff=1024, max_seq_len=64)
    tr = PipelineTrainer(cfg, pp=world, schedule="1F1B", n_microbatches=m, mbs=4, seq_len=64,
                         device=torch.device("cpu"), dtype=torch.float32, split_head=False,
                         layer_ranges=[(2 * i, 2 * i + 2) for i in range(world)])
    x = torch.randint(0, 64, (m * 4, 64), generator=torch.Generator().manual_seed(0))
    tr.train_step(x, x)
    dist.barrier()
    tr.runtime.profile = True
    tr.train_step(x, x)
    return tr.runtime.busy_ms(), tr.runtime.last_step_ms, [n for n, _, _ in tr.runtime.last_timeline]


def test_native_stages_profiled_step_timeline():
    """Real native stages: every compute action of the rank's program is timed once and
    the busy time never exceeds the step."""
    res = run_world(_native_worker, 4, 4)
    for r in range(4):
        busy, step, names = res[r]
        assert 0 < busy <= step
        assert sorted(names) == sorted([f"{r}F{i}" for i in range(4)] + [f"{r}B{i}" for i in range(4)])
